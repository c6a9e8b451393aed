# K3 launch structures on the GPU box: parity tests (all three paths), the standalone
# probe (tools/chol_probe.py), the c3 ELBO step with and without tile pairs, and one
# SQ counter pass per structure over the K3 micro-benchmark (MFMA busy).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "potrf or kuu" > gpurun_out/k3_tests.log 2>&1; rc=$?; tail -3 gpurun_out/k3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/chol_probe.py > gpurun_out/k3_probe.log 2>&1 && cat gpurun_out/k3_probe.log || exit 1
timeout -k 10 300 python -u tools/env_ab_probe.py '{"tiles": {"MGP_CHOL_PAIR": "0"}, "pairs": {"MGP_CHOL_PAIR": "1"}}' > gpurun_out/k3_ab.log 2>&1 && tail -1 gpurun_out/k3_ab.log || exit 1
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES"
for v in 1 0; do
  MGP_CHOL_PAIR=$v timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/k3pmc$v/pmc_SQ_WAVE_CYCLES -o p -- python3 tools/bench_kernels.py --reps 2 --only kuu_chol_x2 > gpurun_out/k3pmc$v.log 2>&1 || { echo "pmc fail $v"; exit 1; }
done
echo k3-ok
