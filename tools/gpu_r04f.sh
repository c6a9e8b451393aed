# Training-step layer concurrency: bit-identity test, A/B timing, kernel trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_training.py -k "backward_streams or (test_elbo_and_grad and f16-)" > gpurun_out/r04f_pytest.txt 2>&1 || { tail -30 gpurun_out/r04f_pytest.txt; exit 1; }
tail -3 gpurun_out/r04f_pytest.txt
timeout -k 10 300 python -u tools/train_ab.py 3 30 > gpurun_out/r04f_train_ab.log 2>&1 || { tail -20 gpurun_out/r04f_train_ab.log; exit 1; }
cat gpurun_out/r04f_train_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f_train -o tr -- python3 tools/train_steps.py 10 > gpurun_out/r04f_train.log 2>&1 || { echo "train trace fail"; exit 1; }
echo round-ok
