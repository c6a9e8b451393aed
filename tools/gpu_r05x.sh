# Round-5: the side stream's tril(q_sqrt) work started with the step (beside K3's Kuu build)
# instead of after it.  Model/schedule/training tests, A/B (tools/elbo_ab.py sidelate), trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_schedules.py tests/test_gpu_f16.py tests/test_gpu_training.py -k "not c3_full" > $O/pytest_model.txt 2>&1 || { tail -40 $O/pytest_model.txt; exit 1; }
tail -1 $O/pytest_model.txt
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/elbo_ab.py 3 50 early > $O/ab_new_$r.log 2>&1 || { tail -5 $O/ab_new_$r.log; exit 1; }
  tail -1 $O/ab_new_$r.log
  timeout -k 10 300 python3 tools/elbo_ab.py 3 50 late sidelate > $O/ab_base_$r.log 2>&1 || { tail -5 $O/ab_base_$r.log; exit 1; }
  tail -1 $O/ab_base_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/new -o t -- python3 bench.py --no-cpu-baseline --no-modes --no-train --steps 60 > $O/new.log 2>&1 || { tail -5 $O/new.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes > $O/bench_new.json 2> $O/bench_new.err || { tail -5 $O/bench_new.err; exit 1; }
python3 -c "import json; d = json.load(open('gpurun_out/r05x/bench_new.json')); k = d['kernels']; print('bench', round(d['value'], 1), 'kuu_chol', round(k['kuu_chol']['avg_us'], 1), 'train', round(d['train']['value'], 2))"
echo r05x-ok
