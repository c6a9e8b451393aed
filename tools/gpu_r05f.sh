# Round-5: non-temporal stores at kernel boundaries.  Default tree = the K1 side job's
# image stores non-temporal; A/B against _ab/kufpol0.so (plain side-job stores),
# _ab/k3nt.so (+ K3's L / L^-T / workspace tile stores non-temporal) and _ab/k4nt.so
# (+ K4's A-image stores non-temporal).  Interleaved x3 on one box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05f
mkdir -p $O
AB=$PWD/modulatedgps_amd/_ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "kuf_side_job or potrf or kuu" > $O/pytest_default.txt 2>&1 || { tail -30 $O/pytest_default.txt; exit 1; }
tail -1 $O/pytest_default.txt
MGP_HIP_LIB=$AB/k3nt.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "kuf_side_job or potrf or kuu" > $O/pytest_k3nt.txt 2>&1 || { tail -30 $O/pytest_k3nt.txt; exit 1; }
tail -1 $O/pytest_k3nt.txt
MGP_HIP_LIB=$AB/k4nt.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_f16.py -k "trsm or elbo" > $O/pytest_k4nt.txt 2>&1 || { tail -30 $O/pytest_k4nt.txt; exit 1; }
tail -1 $O/pytest_k4nt.txt
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_default_$r.json 2> $O/bench_default_$r.err || { tail -5 $O/bench_default_$r.err; exit 1; }
  for v in kufpol0 k3nt k4nt; do
    MGP_HIP_LIB=$AB/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -5 $O/bench_${v}_$r.err; exit 1; }
  done
done
python - <<'PY'
import json
for r in (1, 2, 3):
    for a in ("default", "kufpol0", "k3nt", "k4nt"):
        d = json.load(open(f"gpurun_out/r05f/bench_{a}_{r}.json"))
        k = d["kernels"]
        print(f"{a}_{r}", round(d["value"], 1), "kuu_chol", round(k["kuu_chol"]["avg_us"], 1), "K4", round(k["trsm_stats"]["avg_us"], 1),
              "K5", round(k["expert_cond"]["avg_us"], 1), "train", round(d["train"]["value"], 2))
PY
echo r05f-ok
