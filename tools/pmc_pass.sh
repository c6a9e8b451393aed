# Separate rocprofv3 --pmc passes (one counter group per run, kernel-trace only)
# over tools/bench_kernels.py.  Usage on the GPU box:
#   ONLY=expert_cond_x6,trsm_stats_x6 bash tools/pmc_pass.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ONLY=${ONLY:-}
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$n -o p -- python3 tools/bench_kernels.py --reps 2 --only "$ONLY" > gpurun_out/pmc_$n.log 2>&1 || { echo "fail $n"; exit 1; }
done
echo ok
