# Round-3 closing measurement on the final tree (run from the repo root via gpurun):
# the GPU test suite, the default bench line and its rocprofv3 kernel-trace summary.
# PMC passes: tools/gpu_r03.sh's last two steps.  Every GPU step has its own limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
tail -c 400 gpurun_out/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
timeout -k 10 60 tools/f64_mfma_probe > gpurun_out/f64_mfma_probe.log 2>&1 && cat gpurun_out/f64_mfma_probe.log
echo round-ok
