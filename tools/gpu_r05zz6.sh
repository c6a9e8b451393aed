# Round-5: the conditional-backward prep as one fixed-grid (256 workgroups) launch (default)
# vs its two full-size launches (_ab/pf0.so, -DMGP_PREP_FUSED=0): c_images + training tests,
# training A/B x3, a trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zz6
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_training.py -k "c_images or elbo_and_grad" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
  MGP_HIP_LIB=$PWD/modulatedgps_amd/_ab/pf0.so timeout -k 10 300 python3 tools/train_ab.py 3 30 pf0 > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  timeout -k 10 300 python3 tools/train_ab.py 3 30 fused > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o t -- python3 tools/train_ab.py 1 10 trace > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r05zz6/tr/t_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('chol_step_pair','cond_prep','split_tri','tril_transpose')): print(r['Name'][:50], r['AverageNs'])"
echo r05zz6-ok
