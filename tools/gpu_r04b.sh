# Step-schedule A/B (tools/schedule_probe.py) + the tests touched this session.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_f16.py tests/test_gpu_model.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b_pytest.txt 2>&1
tail -2 gpurun_out/r04b_pytest.txt
timeout -k 10 300 python -u tools/schedule_probe.py 3 > gpurun_out/r04b_sched.log 2>&1
tail -1 gpurun_out/r04b_sched.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04b_trace -o t -- python3 tools/schedule_probe.py 1 overlap,k1a_late > gpurun_out/r04b_trace.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -q -k c4 --timeout 900 --timeout-method thread > gpurun_out/r04b_c4.txt 2>&1
tail -2 gpurun_out/r04b_c4.txt
echo round-ok
