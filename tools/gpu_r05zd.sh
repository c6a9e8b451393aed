# Round-5: the P_k gram (gram_rows2_kernel) with 8 producer waves (1024 threads, each
# producer thread half the row groups of a chunk) instead of 4: _ab/pw8.so against the
# tree's library (4).  Gram / backward tests on the variant, standalone gram, training A/B x3.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zd
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
MGP_HIP_LIB=$AB/pw8.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_training.py -k "gram or conditional_backward or elbo_and_grad" > $O/pytest_pw8.txt 2>&1 || { tail -40 $O/pytest_pw8.txt; exit 1; }
tail -1 $O/pytest_pw8.txt
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/train_ab.py 3 30 pw4 > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  MGP_HIP_LIB=$AB/pw8.so timeout -k 10 300 python3 tools/train_ab.py 3 30 pw8 > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
MGP_HIP_LIB=$AB/pw8.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pw8 -o t -- python3 tools/train_ab.py 1 10 trace > $O/pw8_trace.log 2>&1 || { tail -5 $O/pw8_trace.log; exit 1; }
grep -h "gram_rows2" $O/pw8/*kernel_stats.csv | cut -c1-40,200-
echo r05zd-ok
