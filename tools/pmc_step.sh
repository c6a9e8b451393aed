# PMC passes over the shipped step itself (round 6): bench.py's c3 ELBO step and training
# step (few steps, no CPU baseline / modes), one counter group per rocprofv3 run
# (kernel-trace only), into $OUT/pmc_<group>/; summarise with tools/pmc_summary.py.
#   OUT=gpurun_out/pmcstep bash tools/pmc_step.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/pmcstep}
mkdir -p $OUT
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$n -o p -- python3 bench.py --no-cpu-baseline --no-modes --steps 3 --repeats 1 --warmup 1 > $OUT/pmc_$n.log 2>&1 || { echo "fail $n"; exit 1; }
done
echo ok
