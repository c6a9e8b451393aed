# Round-5: the row-max fold on 1024 threads and max |LinvT| handed from K3's bounded
# L^-T images to the C-images backward (t_bound) vs HEAD (_ab/prev.so, flag notb: the
# backward reduces it itself).  Full GPU suite first (many changes this round), A/B x3.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zt
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
for r in 1 2 3; do
  MGP_HIP_LIB=$AB/prev.so timeout -k 10 300 python3 tools/train_ab.py 3 30 prev notb > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
  timeout -k 10 300 python3 tools/train_ab.py 3 30 new > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o t -- python3 tools/train_ab.py 1 10 trace > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 -c "import csv; [print(r[\"Name\"][:50], r[\"AverageNs\"], r[\"Calls\"]) for r in csv.DictReader(open(\"gpurun_out/r05zt/tr/t_kernel_stats.csv\")) if \"rowmax\" in r[\"Name\"] or \"absmax\" in r[\"Name\"] or \"fill\" in r[\"Name\"]]"
echo r05zt-ok
