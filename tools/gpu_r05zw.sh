# Round-5: cond_finalize2 with four experts per thread (Σ_t stats[t][0][n] read once per
# point and four experts instead of once per expert; same sums, bit-identical) vs HEAD
# (_ab/fin1.so): the batched-vs-per-layer bit-identity tests, ELBO A/B x3, a trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zw
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_f16.py tests/test_gpu_properties.py tests/test_gpu_kernels.py -k "batch or identical or finalize or elbo" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
  MGP_HIP_LIB=$AB/fin1.so timeout -k 10 300 python3 tools/elbo_ab.py 3 100 fin1 > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  timeout -k 10 300 python3 tools/elbo_ab.py 3 100 fin4 > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o t -- python3 tools/elbo_ab.py 1 50 trace > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
MGP_HIP_LIB=$AB/fin1.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr0 -o t -- python3 tools/elbo_ab.py 1 50 trace > $O/trace0.log 2>&1 || { tail -5 $O/trace0.log; exit 1; }
python3 -c "
import csv
for d in ('tr0','tr'):
    for r in csv.DictReader(open('gpurun_out/r05zw/'+d+'/t_kernel_stats.csv')):
        if 'finalize' in r['Name']: print(d, r['Name'][:50], r['AverageNs'])"
echo r05zw-ok
