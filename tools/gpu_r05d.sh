# Round-5: K3 look-ahead row preparation (RowPrep) + K1 inside K3's step launches.
# K3 / K1-side-job tests first, the SIMD-sharing probe, the GPU suite, then the bench
# A/B on one box: this tree, the K1-only library (_ab/libmgp_hip_phase2.so), and the
# round-4 schedule (overlap), a K3 PMC pass and a kernel trace of the bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "kuf_side_job or potrf or kuu" > $O/pytest_k3.txt 2>&1 || { tail -40 $O/pytest_k3.txt; exit 1; }
tail -2 $O/pytest_k3.txt
timeout -k 10 60 tools/simd_share_probe > $O/simd_share_probe.log 2>&1 || { tail -5 $O/simd_share_probe.log; exit 1; }
cat $O/simd_share_probe.log
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -s tests -m gpu > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
grep -E "passed|failed|C-ABI" $O/pytest_gpu.txt | tail -4
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_new_$r.json 2> $O/bench_new_$r.err || { tail -5 $O/bench_new_$r.err; exit 1; }
  MGP_HIP_LIB=$PWD/modulatedgps_amd/_ab/libmgp_hip_phase2.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_p2_$r.json 2> $O/bench_p2_$r.err || { tail -5 $O/bench_p2_$r.err; exit 1; }
  MGP_STEP_SCHEDULE=overlap timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_overlap_$r.json 2> $O/bench_overlap_$r.err || { tail -5 $O/bench_overlap_$r.err; exit 1; }
done
python - <<'PY'
import json
for n in ("new_1", "p2_1", "overlap_1", "new_2", "p2_2", "overlap_2"):
    d = json.load(open(f"gpurun_out/r05d/bench_{n}.json"))
    k = d["kernels"]
    print(n, round(d["value"], 1), "kuu_chol", round(k["kuu_chol"]["avg_us"], 1), "K4", round(k["trsm_stats"]["avg_us"], 1),
          "K5", round(k["expert_cond"]["avg_us"], 1), "train", round(d["train"]["value"], 2))
PY
K3PMC_OUT=$O/k3pmc bash tools/k3_pmc.sh || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --no-modes --steps 50 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
echo r05d-ok
