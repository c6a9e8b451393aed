# Round-5: K3's pivot chain with one Newton step after v_rsq_f64 instead of two (accuracy
# probe tools/rsq_probe.hip first).  K3, model, backward and full-size tests, A/B against
# _ab/base.so (HEAD f799873: two Newton steps),
# standalone K3 and the ELBO bench line, interleaved x3 on one box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zb
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
timeout -k 10 60 tools/rsq_probe > $O/rsq_probe.log 2>&1 || { cat $O/rsq_probe.log; exit 1; }
cat $O/rsq_probe.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "potrf or kuu or chol or non_spd or ill" > $O/pytest_k3.txt 2>&1 || { tail -40 $O/pytest_k3.txt; exit 1; }
tail -1 $O/pytest_k3.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_backward.py tests/test_gpu_f16.py tests/test_gpu_fullsize.py > $O/pytest_model.txt 2>&1 || { tail -40 $O/pytest_model.txt; exit 1; }
tail -1 $O/pytest_model.txt
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/bench_kernels.py --only kuu_chol_x2,kuu_chol_kuf_x2 > $O/k3_new_$r.log 2>&1 || { tail -5 $O/k3_new_$r.log; exit 1; }
  MGP_HIP_LIB=$AB/base.so timeout -k 10 300 python3 tools/bench_kernels.py --only kuu_chol_x2,kuu_chol_kuf_x2 > $O/k3_base_$r.log 2>&1 || { tail -5 $O/k3_base_$r.log; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes --no-train > $O/bench_new_$r.json 2> $O/bench_new_$r.err || { tail -5 $O/bench_new_$r.err; exit 1; }
  MGP_HIP_LIB=$AB/base.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes --no-train > $O/bench_base_$r.json 2> $O/bench_base_$r.err || { tail -5 $O/bench_base_$r.err; exit 1; }
done
python - <<'PY'
import json
for r in (1, 2, 3):
    for a in ("new", "base"):
        d = json.load(open(f"gpurun_out/r05zb/bench_{a}_{r}.json"))
        k = d["kernels"]
        k3 = open(f"gpurun_out/r05zb/k3_{a}_{r}.log").read().split("\n")
        k3 = " | ".join(l.strip() for l in k3 if "kuu_chol" in l)
        print(f"{a}_{r}", round(d["value"], 1), "ms", round(d["ms_per_step"], 4), "kuu_chol", round(k["kuu_chol"]["avg_us"], 1), "K4", round(k["trsm_stats"]["avg_us"], 1),
              "K5", round(k["expert_cond"]["avg_us"], 1), "| standalone:", k3)
PY
echo r05zb-ok
