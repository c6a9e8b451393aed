# Round-5: grad_a_prep_kernel with one A-tile LDS buffer (29.7 KB, four workgroups per CU
# instead of three, one more barrier per row block): _ab/prep1.so against the tree (two
# buffers).  Tests on the variant, training A/B x3, a trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zk
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
MGP_HIP_LIB=$AB/prep1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_training.py -k "conditional_backward or elbo_and_grad or prep" > $O/pytest_prep1.txt 2>&1 || { tail -40 $O/pytest_prep1.txt; exit 1; }
tail -1 $O/pytest_prep1.txt
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/train_ab.py 3 30 prep2 > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  MGP_HIP_LIB=$AB/prep1.so timeout -k 10 300 python3 tools/train_ab.py 3 30 prep1 > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
MGP_HIP_LIB=$AB/prep1.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prep1 -o t -- python3 tools/train_ab.py 1 10 trace > $O/prep1_trace.log 2>&1 || { tail -5 $O/prep1_trace.log; exit 1; }
python3 -c "import csv; [print(r[\"Name\"][:40], r[\"AverageNs\"]) for r in csv.DictReader(open(\"gpurun_out/r05zk/prep1/t_kernel_stats.csv\")) if \"prep\" in r[\"Name\"]]"
echo r05zk-ok
