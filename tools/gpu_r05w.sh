# Round-5: both layers' tril(q_sqrt) images and KL terms in three launches on the side
# stream (mgp_qsqrt_images_kl_f16_batch) instead of ten.  Bit-identity test, model tests,
# A/B against the per-layer launches (same library, tools/elbo_ab.py qsper), a kernel trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "qsqrt or kl or split" > $O/pytest_q.txt 2>&1 || { tail -40 $O/pytest_q.txt; exit 1; }
tail -1 $O/pytest_q.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_schedules.py tests/test_gpu_f16.py tests/test_gpu_api.py > $O/pytest_model.txt 2>&1 || { tail -40 $O/pytest_model.txt; exit 1; }
tail -1 $O/pytest_model.txt
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/elbo_ab.py 3 50 batched > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
  timeout -k 10 300 python3 tools/elbo_ab.py 3 50 per-layer qsper > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_new.json 2> $O/bench_new.err || { tail -5 $O/bench_new.err; exit 1; }
python3 -c "import json; d = json.load(open('gpurun_out/r05w/bench_new.json')); k = d['kernels']; print('bench', round(d['value'], 1), 'kuu_chol', round(k['kuu_chol']['avg_us'], 1), 'train', round(d['train']['value'], 2))"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/new -o t -- python3 bench.py --no-cpu-baseline --no-modes --no-train --steps 60 > $O/new.log 2>&1 || { tail -5 $O/new.log; exit 1; }
echo r05w-ok
