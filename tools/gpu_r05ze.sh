# Round-5: the x6 grams (gram_x6_kernel: the training step's g_q_sqrt and g_Lm products) with
# 8 consumer waves (64 x 32 of the tile each, 1024 threads) instead of 4: _ab/cw8.so against
# the tree's library.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ze
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
MGP_HIP_LIB=$AB/cw8.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_training.py -k "gram or conditional_backward or elbo_and_grad or chol" > $O/pytest_pw8.txt 2>&1 || { tail -40 $O/pytest_pw8.txt; exit 1; }
tail -1 $O/pytest_pw8.txt
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/train_ab.py 3 30 cw4 > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  MGP_HIP_LIB=$AB/cw8.so timeout -k 10 300 python3 tools/train_ab.py 3 30 cw8 > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
MGP_HIP_LIB=$AB/cw8.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cw8 -o t -- python3 tools/train_ab.py 1 10 trace > $O/cw8_trace.log 2>&1 || { tail -5 $O/cw8_trace.log; exit 1; }
grep -h "gram_x6_kernel" $O/cw8/*kernel_stats.csv | cut -c1-40,200-
echo r05ze-ok
