# K3 counters on the c3 micro-benchmark (both layers' Kuu, M = 1024): kernel trace for
# durations, then one PMC pass per counter group (kernel-trace only), summarised by
# tools/pmc_summary.py (clock-free MFMA busy + the f64 MFMA count) and the analytic count.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=${K3PMC_OUT:-gpurun_out/k3pmc}
CASE=${K3PMC_CASE:-kuu_chol_x2}   # kuu_chol_kuf_x2: with the Kuf side job (the ELBO step's form)
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o k3 -- python3 tools/bench_kernels.py --reps 3 --only $CASE > $OUT/trace.log 2>&1 || { echo "trace fail"; exit 1; }
for c in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$n -o p -- python3 tools/bench_kernels.py --reps 2 --only $CASE > $OUT/pmc_$n.log 2>&1 || { echo "pmc fail $n"; exit 1; }
done
python3 tools/pmc_summary.py $OUT $OUT/k3_pmc.json SQ_VALU_MFMA_BUSY_CYCLES FETCH_SIZE WRITE_SIZE > $OUT/summary.log 2>&1 || { echo "summary fail"; exit 1; }
python3 tools/k3_mfma_count.py 1024 2 > $OUT/analytic.json
echo k3-pmc-ok
