# Training forward's colnorm_max on the side stream: training / backward parity, train-step A/B.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_backward.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04zg_pytest.txt 2>&1 || { tail -30 gpurun_out/r04zg_pytest.txt; exit 1; }
tail -2 gpurun_out/r04zg_pytest.txt
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/train_ab.py 3 30 side >> gpurun_out/r04zg_train_ab.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/train_ab.py 3 30 main colmaxmain >> gpurun_out/r04zg_train_ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r04zg_train_ab.log
echo round-ok
