# cond_finalize with its tile loads issued eight at a time: parity (f16 / model suites),
# standalone finalize timing via the ELBO A/B (new vs abvar/finold.so), kernel trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_f16.py tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04zc_pytest.txt 2>&1 || { tail -30 gpurun_out/r04zc_pytest.txt; exit 1; }
tail -2 gpurun_out/r04zc_pytest.txt
for r in 1 2; do
  for v in finnew finold; do
    MGP_HIP_LIB=$PWD/abvar/$v.so timeout -k 10 200 python -u tools/elbo_ab.py 3 50 $v >> gpurun_out/r04zc_elbo_ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/r04zc_elbo_ab.log
for v in finnew finold; do
  MGP_HIP_LIB=$PWD/abvar/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04zc_prof_$v -o t -- python3 tools/elbo_ab.py 1 30 $v > gpurun_out/r04zc_prof_$v.log 2>&1 || { echo "prof fail"; exit 1; }
  grep cond_finalize gpurun_out/r04zc_prof_$v/t_kernel_stats.csv | cut -d, -f1-4
done
echo round-ok
