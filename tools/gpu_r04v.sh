# K3 panel sweep with the chain's gaps filled (FMAs + next broadcasts between the
# rsqrt chain's ops): K3 tests, standalone K3 and ELBO-step A/B against the previous
# sweep (abvar/k3old.so, -DMGP_PANEL_OLD), then the look-ahead stamps of the new sweep.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04v_pytest.txt 2>&1 || { tail -30 gpurun_out/r04v_pytest.txt; exit 1; }
tail -2 gpurun_out/r04v_pytest.txt
for r in 1 2; do
  for v in k3new k3old; do
    MGP_HIP_LIB=$PWD/abvar/$v.so timeout -k 10 120 python -u tools/bench_kernels.py --reps 5 --only kuu_chol_x2 > gpurun_out/r04v_k3_$v.json 2>/dev/null || { echo "k3 $v fail"; exit 1; }
    echo "$v $(tail -c 120 gpurun_out/r04v_k3_$v.json)" >> gpurun_out/r04v_k3_ab.log
    MGP_HIP_LIB=$PWD/abvar/$v.so timeout -k 10 200 python -u tools/elbo_ab.py 3 50 $v >> gpurun_out/r04v_elbo_ab.log 2>&1 || exit 1
  done
done
cat gpurun_out/r04v_k3_ab.log; grep -v amdgpu.ids gpurun_out/r04v_elbo_ab.log
timeout -k 10 240 python -u tools/chol_stamps.py 1024 > gpurun_out/r04v_stamps.log 2>&1 || { echo "stamps fail"; tail -5 gpurun_out/r04v_stamps.log; exit 1; }
head -24 gpurun_out/r04v_stamps.log
echo round-ok
