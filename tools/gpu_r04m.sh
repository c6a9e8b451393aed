# K5 on expert pairs (two experts per workgroup sharing A's fragments): f16 / full-size
# parity, ELBO-step A/B against the previous library (abvar/head.so), kernel trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_f16.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py > gpurun_out/r04m_pytest.txt 2>&1 || { tail -30 gpurun_out/r04m_pytest.txt; exit 1; }
tail -2 gpurun_out/r04m_pytest.txt
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/elbo_ab.py 3 50 new >> gpurun_out/r04m_ab.log 2>&1 || exit 1
  MGP_HIP_LIB=$PWD/abvar/head.so timeout -k 10 200 python -u tools/elbo_ab.py 3 50 old >> gpurun_out/r04m_ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r04m_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04m_prof -o new -- python3 tools/elbo_ab.py 1 50 new > gpurun_out/r04m_prof.log 2>&1 || { echo "prof fail"; exit 1; }
MGP_HIP_LIB=$PWD/abvar/head.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04m_prof -o old -- python3 tools/elbo_ab.py 1 50 old >> gpurun_out/r04m_prof.log 2>&1 || { echo "prof fail"; exit 1; }
grep -h expert_cond gpurun_out/r04m_prof/*kernel_stats.csv | cut -c1-60,200-320
echo round-ok
