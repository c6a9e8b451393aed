# Round-5: the new GPU tests (step-schedule bit-identity, tiled= opt-in, empty samples,
# full-c3 ELBO through the C-ABI alone, full-c3 gradient vs float64 autograd).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -s tests/test_gpu_schedules.py tests/test_gpu_api.py tests/test_gpu_c_abi.py "tests/test_gpu_training.py::test_elbo_and_grad_c3_full" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
grep -E "passed|failed|C-ABI|e-0" $O/pytest.txt | tail -20
echo r05b-ok
