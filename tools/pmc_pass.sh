cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$n -o p -- python tools/bench_kernels.py --reps 2 > gpurun_out/pmc_$n.log 2>&1 || { echo "fail $n"; exit 1; }
done
echo ok
