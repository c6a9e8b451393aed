# Round-5: training-step small launches: sum_parts (g_var) staged through LDS (the
# single-thread loop took 16 us), the batched RBF backward overwriting gZ / g_ls
# (accumulate 2: four zero fills fewer).  Tests, A/B against _ab/base.so with zero fills.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zg
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_training.py tests/test_gpu_schedules.py -k "not c3_full" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
  MGP_HIP_LIB=$AB/base.so timeout -k 10 300 python3 tools/train_ab.py 3 30 base fill > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  timeout -k 10 300 python3 tools/train_ab.py 3 30 new > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o t -- python3 tools/train_ab.py 1 10 trace > $O/new_trace.log 2>&1 || { tail -5 $O/new_trace.log; exit 1; }
echo r05zg-ok
