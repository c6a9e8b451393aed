# Round-3 closing measurement on the GPU box (run from the repo root via gpurun): the
# default bench line, its rocprofv3 kernel-trace summary and the PMC passes of the
# split-f16 K4 / K5 kernels that run by default (trsm_stats16_kernel, expert_cond16_kernel).
# Every GPU step has its own limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
tail -c 400 gpurun_out/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
ONLY=${ONLY:-expert_cond_f16,trsm_stats_f16} bash tools/pmc_pass.sh
python tools/pmc_summary.py gpurun_out gpurun_out/pmc_traffic.json > /dev/null
echo round-ok
