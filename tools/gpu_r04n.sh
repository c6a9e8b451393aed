# Multi-rank bench rehearsal on one GPU (gloo, every rank on cuda:0): the driver's
# --gpus N path (rank spawn, barrier + max-over-ranks timing, data-term all-reduce,
# gradient buckets), N = 2 and 8; timings are not scaling figures (ranks share a GPU).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MGP_BENCH_SHARE_GPU=1 MGP_BENCH_BACKEND=gloo
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-modes > gpurun_out/r04n_bench_n2.json 2> gpurun_out/r04n_bench_n2.err || { tail -20 gpurun_out/r04n_bench_n2.err; exit 1; }
tail -c 400 gpurun_out/r04n_bench_n2.json
timeout -k 10 500 python bench.py --gpus 8 --steps 5 --warmup 1 --no-cpu-baseline --no-modes > gpurun_out/r04n_bench_n8.json 2> gpurun_out/r04n_bench_n8.err || { tail -20 gpurun_out/r04n_bench_n8.err; exit 1; }
tail -c 400 gpurun_out/r04n_bench_n8.json
echo round-ok
