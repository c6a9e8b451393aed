# Round-5: the K3 panel sweep with its pivot check after the sweep (no per-column branch).
# Panel probe, K3 tests, A/B against the previous library (_ab/base.so, x3), stamps last.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 60 tools/panel_probe > $O/panel_probe.log 2>&1 || { tail -5 $O/panel_probe.log; exit 1; }
tail -13 $O/panel_probe.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "kuf_side_job or potrf or kuu" > $O/pytest_k3.txt 2>&1 || { tail -40 $O/pytest_k3.txt; exit 1; }
tail -1 $O/pytest_k3.txt
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_new_$r.json 2> $O/bench_new_$r.err || { tail -5 $O/bench_new_$r.err; exit 1; }
  MGP_HIP_LIB=$PWD/modulatedgps_amd/_ab/base.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_base_$r.json 2> $O/bench_base_$r.err || { tail -5 $O/bench_base_$r.err; exit 1; }
done
python - <<'PY'
import json
for r in (1, 2, 3):
    for a in ("new", "base"):
        d = json.load(open(f"gpurun_out/r05l/bench_{a}_{r}.json"))
        k = d["kernels"]
        print(f"{a}_{r}", round(d["value"], 1), "kuu_chol", round(k["kuu_chol"]["avg_us"], 1), "K4", round(k["trsm_stats"]["avg_us"], 1),
              "K5", round(k["expert_cond"]["avg_us"], 1), "train", round(d["train"]["value"], 2))
PY
timeout -k 10 400 python3 tools/chol_stamps.py > $O/stamps_alone.log 2>&1 || { tail -20 $O/stamps_alone.log; exit 1; }
timeout -k 10 300 python3 tools/chol_stamps.py --elbo > $O/stamps_elbo.log 2>&1 || { tail -20 $O/stamps_elbo.log; exit 1; }
echo r05l-ok
