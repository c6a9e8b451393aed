# Gram consumers pipelined across the chunk barrier: gradient / gram tests, training
# A/B against the previous library (abvar/head.so), kernel trace of the training step.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_backward.py > gpurun_out/r04o_pytest.txt 2>&1 || { tail -30 gpurun_out/r04o_pytest.txt; exit 1; }
tail -2 gpurun_out/r04o_pytest.txt
for r in 1 2; do
  timeout -k 10 200 python -u tools/train_ab.py 3 30 new >> gpurun_out/r04o_train_ab.log 2>&1 || exit 1
  MGP_HIP_LIB=$PWD/abvar/head.so timeout -k 10 200 python -u tools/train_ab.py 3 30 old >> gpurun_out/r04o_train_ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r04o_train_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04o_train -o tr -- python3 tools/train_steps.py 10 > gpurun_out/r04o_train.log 2>&1 || { echo "train trace fail"; exit 1; }
echo round-ok
