# Round-3 measurement on the GPU box (run from the repo root via gpurun): the default
# bench line, its rocprofv3 kernel-trace summary, a dedicated K1 trace, and the PMC
# passes for the kernels the bench line reports.  Every GPU step has its own limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
tail -c 400 gpurun_out/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k1 -o k1 -- python3 tools/bench_kernels.py --only rbf_kuf_f16 --reps 10 > gpurun_out/k1_bench.json 2> gpurun_out/k1.err
ONLY=${ONLY:-expert_cond_f16,expert_cond_f16x8,rbf_kuf_f16,kuu_chol_x2,trsm_stats_f16} bash tools/pmc_pass.sh
python tools/pmc_summary.py gpurun_out gpurun_out/pmc_traffic.json > /dev/null
echo round-ok
