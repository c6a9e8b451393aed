# Round-5: the grams' split-K partial stores non-temporal (default) vs write-back
# (_ab/gnt0.so, -DMGP_GRAM_NT=0): c_images / training tests, training A/B x3, traces.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zz4
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_training.py tests/test_gpu_kernels.py -k "gram or c_images or elbo_and_grad" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
  MGP_HIP_LIB=$AB/gnt0.so timeout -k 10 300 python3 tools/train_ab.py 3 30 cwb > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  timeout -k 10 300 python3 tools/train_ab.py 3 30 cnt > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o t -- python3 tools/train_ab.py 1 10 trace > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
MGP_HIP_LIB=$AB/gnt0.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr0 -o t -- python3 tools/train_ab.py 1 10 trace > $O/trace0.log 2>&1 || { tail -5 $O/trace0.log; exit 1; }
python3 -c "
import csv
for d in ('tr0','tr'):
    for r in csv.DictReader(open('gpurun_out/r05zz4/'+d+'/t_kernel_stats.csv')):
        if any(k in r['Name'] for k in ('gram_rows2','gram_x6')): print(d, r['Name'][:50], r['AverageNs'])"
echo r05zz4-ok
