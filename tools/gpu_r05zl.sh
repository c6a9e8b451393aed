# Multi-rank bench rehearsal on the final round-5 tree, one GPU (gloo, every rank on
# cuda:0): the driver's --gpus N path (rank spawn, barrier + max-over-ranks timing, the
# data-term all-reduce, the training leg's gradient buckets after the batched tail),
# N = 2 and 4.  Timings are not scaling figures (the ranks share one GPU).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05zl
export MGP_BENCH_SHARE_GPU=1 MGP_BENCH_BACKEND=gloo
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-modes > gpurun_out/r05zl/bench_n2.json 2> gpurun_out/r05zl/bench_n2.err || { tail -20 gpurun_out/r05zl/bench_n2.err; exit 1; }
tail -c 300 gpurun_out/r05zl/bench_n2.json
timeout -k 10 500 python bench.py --gpus 4 --steps 6 --warmup 1 --no-cpu-baseline --no-modes > gpurun_out/r05zl/bench_n4.json 2> gpurun_out/r05zl/bench_n4.err || { tail -20 gpurun_out/r05zl/bench_n4.err; exit 1; }
tail -c 300 gpurun_out/r05zl/bench_n4.json
echo r05zl-ok
