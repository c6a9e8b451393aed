# K3 step launches: + the two light tiles of a row in one pair:
# K3 tests, K3 PMC (MFMA busy on the active CUs), ELBO-step A/B against the previous
# K3 (abvar/lib_old.so), then the stamps of the debug build.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04q_pytest.txt 2>&1 || { tail -30 gpurun_out/r04q_pytest.txt; exit 1; }
tail -2 gpurun_out/r04q_pytest.txt
MGP_HIP_LIB=$PWD/abvar/lib_new.so K3PMC_OUT=gpurun_out/k3pmc bash tools/k3_pmc.sh || exit 1
MGP_HIP_LIB=$PWD/abvar/lib_old.so K3PMC_OUT=gpurun_out/k3pmc_old bash tools/k3_pmc.sh || exit 1
grep -A8 '"chol_step_pair"' gpurun_out/k3pmc/k3_pmc.json gpurun_out/k3pmc_old/k3_pmc.json
for r in 1 2; do
  MGP_HIP_LIB=$PWD/abvar/lib_new.so timeout -k 10 200 python -u tools/elbo_ab.py 3 50 new >> gpurun_out/r04q_elbo_ab.log 2>&1 || exit 1
  MGP_HIP_LIB=$PWD/abvar/lib_old.so timeout -k 10 200 python -u tools/elbo_ab.py 3 50 old >> gpurun_out/r04q_elbo_ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r04q_elbo_ab.log
timeout -k 10 240 python -u tools/chol_stamps.py 1024 > gpurun_out/r04q_stamps.log 2>&1 || { echo "stamps fail"; tail -5 gpurun_out/r04q_stamps.log; exit 1; }
cat gpurun_out/r04q_stamps.log
echo round-ok
