# Round-4 closing measurement on the layer-batched tree: GPU suite, smoke, PMC passes of
# the batched K4 / K5 (merged into profiles/pmc_traffic.json for the bench's traffic),
# bench line, rocprof kernel trace of the bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04z_pytest.txt 2>&1 || { tail -30 gpurun_out/r04z_pytest.txt; exit 1; }
tail -3 gpurun_out/r04z_pytest.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04z_smoke.txt 2>&1 || { tail -20 gpurun_out/r04z_smoke.txt; exit 1; }
tail -2 gpurun_out/r04z_smoke.txt
mkdir -p gpurun_out/r04z_pmc
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r04z_pmc/pmc_$n -o p -- python3 tools/bench_kernels.py --reps 2 --only trsm_f16_pair,expert_cond_f16_pair > gpurun_out/r04z_pmc/pmc_$n.log 2>&1 || { echo "pmc fail $n"; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/r04z_pmc gpurun_out/r04z_pmc/summary.json SQ_WAVE_CYCLES FETCH_SIZE WRITE_SIZE TCC_HIT_sum > gpurun_out/r04z_pmc/summary.log 2>&1 || { echo "summary fail"; exit 1; }
python3 tools/pmc_merge.py gpurun_out/r04z_pmc/summary.json
timeout -k 10 400 python bench.py > gpurun_out/r04z_bench.json 2> gpurun_out/r04z_bench.err || { tail -5 gpurun_out/r04z_bench.err; exit 1; }
tail -c 400 gpurun_out/r04z_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04z_prof -o bench -- python3 bench.py --no-cpu-baseline --no-modes --steps 50 > gpurun_out/r04z_prof.log 2>&1 || { tail -5 gpurun_out/r04z_prof.log; exit 1; }
echo round-ok
