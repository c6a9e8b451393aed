# Round-5: clean A/B of the K1-in-K3 schedule on one library (k1_in_k3 vs overlap) and
# of the side job's image-store policy (_ab/kufpol1.so non-temporal, _ab/kufpol2.so
# write-through sc1) -- the dirty-L2-at-launch-boundary hypothesis.  Interleaved x3.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05e
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
for v in kufpol1 kufpol2; do
  MGP_HIP_LIB=$AB/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "kuf_side_job" > $O/pytest_$v.txt 2>&1 || { tail -30 $O/pytest_$v.txt; exit 1; }
  tail -1 $O/pytest_$v.txt
done
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_k1k3_$r.json 2> $O/bench_k1k3_$r.err || { tail -5 $O/bench_k1k3_$r.err; exit 1; }
  MGP_STEP_SCHEDULE=overlap timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_overlap_$r.json 2> $O/bench_overlap_$r.err || { tail -5 $O/bench_overlap_$r.err; exit 1; }
  MGP_HIP_LIB=$AB/kufpol1.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_pol1_$r.json 2> $O/bench_pol1_$r.err || { tail -5 $O/bench_pol1_$r.err; exit 1; }
  MGP_HIP_LIB=$AB/kufpol2.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_pol2_$r.json 2> $O/bench_pol2_$r.err || { tail -5 $O/bench_pol2_$r.err; exit 1; }
done
python - <<'PY'
import json
for r in (1, 2, 3):
    for a in ("k1k3", "overlap", "pol1", "pol2"):
        d = json.load(open(f"gpurun_out/r05e/bench_{a}_{r}.json"))
        k = d["kernels"]
        print(f"{a}_{r}", round(d["value"], 1), "kuu_chol", round(k["kuu_chol"]["avg_us"], 1), "K4", round(k["trsm_stats"]["avg_us"], 1),
              "K5", round(k["expert_cond"]["avg_us"], 1), "train", round(d["train"]["value"], 2))
PY
echo r05e-ok
