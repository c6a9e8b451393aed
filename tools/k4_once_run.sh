# K4 single-split epilogue on the GPU box: bit-identity + timing probe, the K4/K5 and
# full-size parity tests, and the c3 ELBO step with either epilogue.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 180 python -u tools/k4_once_probe.py > gpurun_out/k4_once_probe.log 2>&1; rc=$?; cat gpurun_out/k4_once_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_f16.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/k4_tests.log 2>&1; rc=$?; tail -3 gpurun_out/k4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/env_ab_probe.py '{"twice": {"MGP_K4_SPLIT_ONCE": "0"}, "once": {"MGP_K4_SPLIT_ONCE": "1"}}' > gpurun_out/k4_ab.log 2>&1 && tail -1 gpurun_out/k4_ab.log
