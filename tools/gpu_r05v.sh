# Round-5: K4 with its q_mu staging after the main loop.  K4 tests (bit-identity of the
# layer batch, f16 parity), kernel timings and the bench A/B against the kept library.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f16.py tests/test_gpu_kernels.py -k "trsm or f16 or conditional" > $O/pytest_k4.txt 2>&1 || { tail -40 $O/pytest_k4.txt; exit 1; }
tail -1 $O/pytest_k4.txt
for r in 1 2; do
  for v in new base; do
    lib=$PWD/modulatedgps_amd/libmgp_hip.so; [ $v = base ] && lib=$PWD/modulatedgps_amd/_ab/base.so
    MGP_HIP_LIB=$lib timeout -k 10 200 python3 tools/bench_kernels.py --reps 10 --only trsm_f16_pair,trsm_stats_f16 > $O/k_${v}_$r.json 2> $O/k_${v}_$r.err || { tail -5 $O/k_${v}_$r.err; exit 1; }
    echo "$v $r $(tail -1 $O/k_${v}_$r.json | cut -c1-260)"
  done
done
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_new_$r.json 2> $O/bench_new_$r.err || { tail -5 $O/bench_new_$r.err; exit 1; }
  MGP_HIP_LIB=$PWD/modulatedgps_amd/_ab/base.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_base_$r.json 2> $O/bench_base_$r.err || { tail -5 $O/bench_base_$r.err; exit 1; }
done
python - <<'PY'
import json
for r in (1, 2, 3):
    for a in ("new", "base"):
        d = json.load(open(f"gpurun_out/r05v/bench_{a}_{r}.json"))
        k = d["kernels"]
        print(f"{a}_{r}", round(d["value"], 1), "kuu_chol", round(k["kuu_chol"]["avg_us"], 1), "K4", round(k["trsm_stats"]["avg_us"], 1),
              "K5", round(k["expert_cond"]["avg_us"], 1), "train", round(d["train"]["value"], 2))
PY
echo r05v-ok
