# Round-5: the conditional-backward prep launched on the side stream after K3 (beside
# K4 / K5, default) vs beside K3 (flag prepearly); same library: training tests,
# training A/B x3, a trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zz5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_properties.py -k "elbo_and_grad or gradient or train" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/train_ab.py 3 30 early prepearly > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  timeout -k 10 300 python3 tools/train_ab.py 3 30 late > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o t -- python3 tools/train_ab.py 1 10 trace > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r05zz5/tr/t_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('chol_step_pair','trsm_stats16','expert_cond16')): print(r['Name'][:50], r['AverageNs'])"
echo r05zz5-ok
