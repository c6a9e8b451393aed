# Round-5: K4 pair workgroups staggered (every other workgroup of an XCD runs its short
# row tile first): _ab/k4stag.so against the tree's library (long tile first).  K4 /
# model tests on the variant (bit-identical images and statistics), standalone K4 pair
# and the ELBO bench line, interleaved x3.  Also the tree's fresh-ELBO-tensor change.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zf
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_api.py tests/test_gpu_training.py -k "not c3_full" > $O/pytest_tree.txt 2>&1 || { tail -40 $O/pytest_tree.txt; exit 1; }
tail -1 $O/pytest_tree.txt
MGP_HIP_LIB=$AB/k4stag.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f16.py tests/test_gpu_kernels.py -k "trsm or batch" > $O/pytest_k4stag.txt 2>&1 || { tail -40 $O/pytest_k4stag.txt; exit 1; }
tail -1 $O/pytest_k4stag.txt
for r in 1 2 3; do
  for v in base k4stag; do
    L=$PWD/modulatedgps_amd/libmgp_hip.so; [ $v = k4stag ] && L=$AB/k4stag.so
    MGP_HIP_LIB=$L timeout -k 10 300 python3 tools/bench_kernels.py --only trsm_f16_pair > $O/k4_${v}_$r.log 2>&1 || { tail -5 $O/k4_${v}_$r.log; exit 1; }
    MGP_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes --no-train > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -5 $O/bench_${v}_$r.err; exit 1; }
  done
done
python - <<'PY'
import json
for r in (1, 2, 3):
    for a in ("base", "k4stag"):
        d = json.load(open(f"gpurun_out/r05zf/bench_{a}_{r}.json"))
        k = d["kernels"]
        j = json.loads([l for l in open(f"gpurun_out/r05zf/k4_{a}_{r}.log") if "trsm_f16_pair" in l][0])
        print(f"{a}_{r}", round(d["value"], 1), "ELBO/s", round(d["ms_per_step"], 4), "ms | in-step K4", round(k["trsm_stats"]["avg_us"], 1), "K3", round(k["kuu_chol"]["avg_us"], 1), "K5", round(k["expert_cond"]["avg_us"], 1), "| standalone K4 pair", round(j["trsm_f16_pair"]["median_ms"] * 1e3, 1), "us")
PY
echo r05zf-ok
