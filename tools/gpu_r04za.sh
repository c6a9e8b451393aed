# Both layers' cond_finalize in one launch (after the batched K5): parity suites, ELBO A/B.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_f16.py tests/test_gpu_model.py tests/test_gpu_training.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04za_pytest.txt 2>&1 || { tail -30 gpurun_out/r04za_pytest.txt; exit 1; }
tail -2 gpurun_out/r04za_pytest.txt
for r in 1 2; do
  timeout -k 10 200 python -u tools/elbo_ab.py 3 50 batched >> gpurun_out/r04za_elbo_ab.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/elbo_ab.py 3 50 single k4single >> gpurun_out/r04za_elbo_ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r04za_elbo_ab.log
echo round-ok
