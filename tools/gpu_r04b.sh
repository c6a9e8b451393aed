# Round-4 measurement call: tests touched this round, step-schedule A/B, K3 stamps
# (debug build) and PMC counters (release build), then one bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_f16.py tests/test_gpu_model.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b_pytest.txt 2>&1 || { tail -30 gpurun_out/r04b_pytest.txt; exit 1; }
tail -2 gpurun_out/r04b_pytest.txt
timeout -k 10 300 python -u tools/schedule_probe.py 3 > gpurun_out/r04b_sched.log 2>&1 || { tail -5 gpurun_out/r04b_sched.log; exit 1; }
tail -1 gpurun_out/r04b_sched.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04b_trace -o t -- python3 tools/schedule_probe.py 1 overlap,k1a_late,k1a_k5 > gpurun_out/r04b_trace.log 2>&1 || { echo "trace fail"; exit 1; }
bash tools/k3_pmc.sh || exit 1
cp modulatedgps_amd/libmgp_hip.so /tmp/libmgp_release.so
timeout -k 10 240 python -u tools/chol_stamps.py 1024 > gpurun_out/r04b_stamps.log 2>&1 || { echo "stamps fail"; tail -5 gpurun_out/r04b_stamps.log; exit 1; }
timeout -k 10 240 python -u tools/chol_stamps.py 1024 --with-k1 > gpurun_out/r04b_stamps_k1.log 2>&1 || { echo "stamps k1 fail"; exit 1; }
cp /tmp/libmgp_release.so modulatedgps_amd/libmgp_hip.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -q -k c4 --timeout 900 --timeout-method thread > gpurun_out/r04b_c4.txt 2>&1 || { tail -20 gpurun_out/r04b_c4.txt; exit 1; }
tail -2 gpurun_out/r04b_c4.txt
echo round-ok
