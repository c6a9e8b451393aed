# Round-5 closing call 2/2 (final tree): the default bench line (with the CPU baseline),
# a rocprofv3 kernel trace + stats of the bench command, and a fresh K3 PMC pass.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zz
mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --no-modes --steps 50 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
K3PMC_OUT=$O/k3pmc bash tools/k3_pmc.sh || exit 1
echo r05zz-bench-ok
