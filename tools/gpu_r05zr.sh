# Round-5: g_Lm = -tril(g_Kuf A^T) on f16 products with exact per-row scales, the row
# maxima as per-workgroup partials + one fold launch (no atomics), vs x6 (_ab/glmx6.so).
# Tests on the default (c_images incl. "tiny", training gradients), A/Bs, a trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zr
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_training.py tests/test_gpu_properties.py -k "conditional_backward or elbo_and_grad or gradient or adam" > $O/pytest.txt 2>&1; st=$?
tail -4 $O/pytest.txt
[ $st -le 1 ] || exit 1
MGP_HIP_LIB=$AB/glmx6.so timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py -k "c_images and tiny" > $O/pytest_x6.txt 2>&1; st=$?
tail -2 $O/pytest_x6.txt
[ $st -le 1 ] || exit 1
for r in 1 2 3; do
  MGP_HIP_LIB=$AB/glmx6.so timeout -k 10 300 python3 tools/train_ab.py 3 30 glmx6 > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  timeout -k 10 300 python3 tools/train_ab.py 3 30 glm16 > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o t -- python3 tools/train_ab.py 1 10 trace > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 -c "import csv; [print(r[\"Name\"][:50], r[\"AverageNs\"], r[\"Calls\"]) for r in csv.DictReader(open(\"gpurun_out/r05zr/tr/t_kernel_stats.csv\")) if \"trsm_bwd\" in r[\"Name\"] or \"gram_x6\" in r[\"Name\"] or \"prep_kernel\" in r[\"Name\"]]"
echo r05zr-ok
