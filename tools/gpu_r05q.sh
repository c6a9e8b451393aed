# Round-5: per-launch K3 durations in the step with the q_sqrt side job (default) and
# without it (k1_in_k3_qside): kernel traces of short bench runs.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/new -o t -- python3 bench.py --no-cpu-baseline --no-modes --no-train --steps 60 > $O/new.log 2>&1 || { tail -5 $O/new.log; exit 1; }
MGP_STEP_SCHEDULE=k1_in_k3_qside timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/qside -o t -- python3 bench.py --no-cpu-baseline --no-modes --no-train --steps 60 > $O/qside.log 2>&1 || { tail -5 $O/qside.log; exit 1; }
echo r05q-ok
