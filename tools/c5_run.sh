# BASELINE config 5 on one GPU on the current tree: the c5 bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python bench.py --config c5 --steps 10 --warmup 2 > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err; rc=$?; tail -c 600 gpurun_out/c5_bench.json; exit $rc
