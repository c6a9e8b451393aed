# Round-5: the tril(q_sqrt) images and KL terms as a side job of K3's step launches
# (mgp_kuu_potrf_trtri_kuf's q_sqrt job).  K3/side-job tests, model tests, A/B against the
# schedule k1_in_k3_qside (the same library, the q_sqrt work on the side stream), then the GPU suite.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "q_side_job or kuf_side_job or potrf or kuu or kl" > $O/pytest_k3.txt 2>&1 || { tail -40 $O/pytest_k3.txt; exit 1; }
tail -1 $O/pytest_k3.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_schedules.py tests/test_gpu_f16.py tests/test_gpu_api.py > $O/pytest_model.txt 2>&1 || { tail -40 $O/pytest_model.txt; exit 1; }

for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_new_$r.json 2> $O/bench_new_$r.err || { tail -5 $O/bench_new_$r.err; exit 1; }
  MGP_STEP_SCHEDULE=k1_in_k3_qside timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_base_$r.json 2> $O/bench_base_$r.err || { tail -5 $O/bench_base_$r.err; exit 1; }
done
python - <<'PY'
import json
for r in (1, 2, 3):
    for a in ("new", "base"):
        d = json.load(open(f"gpurun_out/r05r/bench_{a}_{r}.json"))
        k = d["kernels"]
        print(f"{a}_{r}", round(d["value"], 1), "kuu_chol", round(k["kuu_chol"]["avg_us"], 1), "K4", round(k["trsm_stats"]["avg_us"], 1),
              "K5", round(k["expert_cond"]["avg_us"], 1), "train", round(d["train"]["value"], 2))
PY


echo r05r-ok
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/new -o t -- python3 bench.py --no-cpu-baseline --no-modes --no-train --steps 60 > $O/new.log 2>&1 || { tail -5 $O/new.log; exit 1; }
