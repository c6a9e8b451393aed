# Round-5 fix: the K6 backward's gradient rows addressed with G's true row stride
# (a K = 1 [4, K, N] view reported torch's contiguous placeholder N as stride(1), so
# var_f / mu_a / var_a's rows landed off by (ld - N) when N % 4 != 0).  The tiny-N
# debug, the regression cases, the hypothesis properties (incl. the gradient), and
# the backward / training suites.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zi
mkdir -p $O
timeout -k 10 200 python3 tools/dbg_small_k6.py > $O/dbg_small_k6.log 2>&1 || { tail -20 $O/dbg_small_k6.log; exit 1; }
grep -v amdgpu.ids $O/dbg_small_k6.log
timeout -k 10 200 python3 tools/dbg_small_grad.py > $O/dbg_small_grad.log 2>&1 || { tail -20 $O/dbg_small_grad.log; exit 1; }
grep "bad:" $O/dbg_small_grad.log | cut -c1-160
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -s tests/test_gpu_properties.py > $O/pytest_props.txt 2>&1 || { tail -60 $O/pytest_props.txt; exit 1; }
tail -2 $O/pytest_props.txt
echo r05zi-ok
