# Round-5: the training step's per-layer tail launches batched -- both layers'
# Cholesky backward (5 launches instead of 16), RBF backward (3 instead of 10) and
# Adam over every parameter block in one launch (instead of 11).  Bit-identity
# tests, the backward / training suites, A/B against the per-layer launches (same
# library, tools/train_ab.py tailper adamper), the bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_training.py -k "batch or set or chol or rbf or adam" > $O/pytest_bit.txt 2>&1 || { tail -40 $O/pytest_bit.txt; exit 1; }
tail -1 $O/pytest_bit.txt
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_training.py > $O/pytest_train.txt 2>&1 || { tail -40 $O/pytest_train.txt; exit 1; }
tail -1 $O/pytest_train.txt
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/train_ab.py 3 30 batched > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
  timeout -k 10 300 python3 tools/train_ab.py 3 30 per-layer tailper adamper > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train -o t -- python3 tools/train_ab.py 1 15 trace > $O/train_trace.log 2>&1 || { tail -5 $O/train_trace.log; exit 1; }
echo r05y-ok
