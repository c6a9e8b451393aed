# Round-5 opening call: bench line on the round-4 tree (this box's baseline), the
# K5 stall breakdown (SQ wait/active buckets of expert_cond16_pair_kernel<false>) and
# a fresh K3 PMC pass (replaces profiles/pmc_traffic.json's K3 rows).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || { echo "counter list failed"; tail -5 $O/counters.txt; }
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$n -o p -- python3 tools/bench_kernels.py --reps 2 --only expert_cond_f16_pair,trsm_f16_pair > $O/pmc_$n.log 2>&1 || { echo "pmc fail $n"; tail -5 $O/pmc_$n.log; exit 1; }
done
K3PMC_OUT=$O/k3pmc bash tools/k3_pmc.sh || exit 1
echo r05a-ok
