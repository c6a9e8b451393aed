# Round-5: trsm_bwd16's per-tile rescale hook before its k-step's MFMAs (default) vs
# after the previous k-step's MFMAs (_ab/bhearly.so, -DMGP_BH_EARLY=1); the c_images
# tests (new "tiny" pattern) on both and on the x6 B-d library; training A/B x3.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zp
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py -k "c_images" > $O/pytest.txt 2>&1; st=$?
tail -3 $O/pytest.txt
[ $st -le 1 ] || exit 1
MGP_HIP_LIB=$AB/x6bwd.so timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py -k "c_images and tiny" > $O/pytest_x6.txt 2>&1; st=$?
tail -3 $O/pytest_x6.txt
[ $st -le 1 ] || exit 1
MGP_HIP_LIB=$AB/bhearly.so timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py -k "c_images" > $O/pytest_early.txt 2>&1; st=$?
tail -3 $O/pytest_early.txt
[ $st -le 1 ] || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/train_ab.py 3 30 late > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  MGP_HIP_LIB=$AB/bhearly.so timeout -k 10 300 python3 tools/train_ab.py 3 30 early > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
MGP_HIP_LIB=$AB/bhearly.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o t -- python3 tools/train_ab.py 1 10 trace > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 -c "import csv; [print(r[\"Name\"][:40], r[\"AverageNs\"]) for r in csv.DictReader(open(\"gpurun_out/r05zp/tr/t_kernel_stats.csv\")) if \"trsm_bwd\" in r[\"Name\"]]"
echo r05zp-ok
