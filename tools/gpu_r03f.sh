# Final-tree bench line and its rocprofv3 kernel-trace summary (round 3, last session).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_f.json 2> gpurun_out/bench_f.err
tail -c 300 gpurun_out/bench_f.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proff -o bench -- python3 bench.py > gpurun_out/bench_proff.json 2> gpurun_out/bench_proff.err
echo round-ok
