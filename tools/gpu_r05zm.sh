# Round-5: the C-images backward's q_sqrt-only launches (L_k's image, L_k^T) as a prep
# on the side stream beside K3 (mgp_conditional_backward_prep_f16c).  Tests (prepped
# outputs bit-identical; training gradients), training A/B x3 on the same library
# (flag noprep = inside the backward), a trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zm
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_training.py tests/test_gpu_properties.py -k "conditional_backward or elbo_and_grad or gradient or adam" > $O/pytest_prep.txt 2>&1 || { tail -40 $O/pytest_prep.txt; exit 1; }
tail -1 $O/pytest_prep.txt
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/train_ab.py 3 30 noprep noprep > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  timeout -k 10 300 python3 tools/train_ab.py 3 30 prep > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o t -- python3 tools/train_ab.py 1 10 trace > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
echo r05zm-ok
