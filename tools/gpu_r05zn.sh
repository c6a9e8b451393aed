# Round-5: B-d (gKuf = Linv^T gA) on split-f16 images -- grad_a_c writes gA's image
# per (128-row tile, column) exactly scaled, trsm_bwd16_kernel rescales the tiles to
# the column's largest in f16 before its MFMAs (3 f16 products instead of 6 bf16).
# Tests, training A/B x3 against _ab/x6bwd.so (-DMGP_TRSM_BWD16=0), a trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zn
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py tests/test_gpu_training.py tests/test_gpu_properties.py -k "conditional_backward or elbo_and_grad or gradient or adam" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
  MGP_HIP_LIB=$AB/x6bwd.so timeout -k 10 300 python3 tools/train_ab.py 3 30 x6bwd > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  timeout -k 10 300 python3 tools/train_ab.py 3 30 bwd16 > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o t -- python3 tools/train_ab.py 1 10 trace > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 -c "import csv; [print(r[\"Name\"][:40], r[\"AverageNs\"]) for r in csv.DictReader(open(\"gpurun_out/r05zn/tr/t_kernel_stats.csv\")) if \"trsm_bwd\" in r[\"Name\"] or \"grad_a_c\" in r[\"Name\"]]"
echo r05zn-ok
