# PMC of the training step's P_k gram (gram_rows2_kernel) and grad_a_c: issue / wait /
# LDS counters, one pass per counter group (kernel-trace only, kernels filtered).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04p
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/r04p/avail.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" gpurun_out/r04p/avail.txt | sort -u > gpurun_out/r04p/sq_names.txt || true
i=0
for c in "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "gram_rows2|grad_a_c" --output-format csv -d gpurun_out/r04p/p$i -o p -- python3 tools/train_steps.py 2 > gpurun_out/r04p/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/r04p/p$i.log; }
done
echo round-ok
