# Round-5: where K3's in-step time goes now.  Kernel traces of (a) K3 alone, (b) K3 with
# the K1 side job, both standalone (bench_kernels), and (c) the bench step; per-launch
# timelines of the step launches from each.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/k3 -o k3 -- python3 tools/bench_kernels.py --only kuu_chol_x2,kuu_chol_kuf_x2 --reps 20 > $O/k3.log 2>&1 || { tail -5 $O/k3.log; exit 1; }
tail -3 $O/k3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --no-modes --no-train --steps 100 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
tail -1 $O/prof.log
echo r05g-ok
