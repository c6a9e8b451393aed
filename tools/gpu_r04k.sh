# K4 on a two-per-CU strided grid (+ permlane epilogues): tests, ELBO and training A/B against
# against the previous library (abvar/head.so), K4 stamps, kernel trace of the bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_f16.py tests/test_gpu_training.py > gpurun_out/r04k_pytest.txt 2>&1 || { tail -30 gpurun_out/r04k_pytest.txt; exit 1; }
tail -2 gpurun_out/r04k_pytest.txt
for r in 1 2; do
  timeout -k 10 200 python -u tools/elbo_ab.py 3 50 new >> gpurun_out/r04k_ab.log 2>&1 || exit 1
  MGP_HIP_LIB=$PWD/abvar/head.so timeout -k 10 200 python -u tools/elbo_ab.py 3 50 old >> gpurun_out/r04k_ab.log 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 200 python -u tools/train_ab.py 3 30 new >> gpurun_out/r04k_ab.log 2>&1 || exit 1
  MGP_HIP_LIB=$PWD/abvar/head.so timeout -k 10 200 python -u tools/train_ab.py 3 30 old >> gpurun_out/r04k_ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r04k_ab.log
timeout -k 10 300 python -u tools/k4_stamps.py > gpurun_out/r04k_k4_stamps.log 2>&1 || { tail -30 gpurun_out/r04k_k4_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04k_k4_stamps.log
echo round-ok
