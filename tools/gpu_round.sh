# Round-end measurement on the GPU box (run from the repo root via gpurun):
#   GPU tests, the bench line (with CPU baseline), the rocprofv3 kernel-trace
#   summary of the same bench command, per-kernel micro-benchmarks and the PMC
#   passes for HBM traffic.  SKIP_TESTS=1 skips the pytest step.
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  tail -2 gpurun_out/pytest_gpu.log
fi
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
tail -c 300 gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels.json 2> gpurun_out/bench_kernels.err
ONLY=${ONLY:-} bash tools/pmc_pass.sh
python tools/pmc_summary.py gpurun_out gpurun_out/pmc_traffic.json > /dev/null
echo round-ok
