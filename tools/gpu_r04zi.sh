# Final tree with the two-layer L^-T split: GPU suite, smoke, bench line, rocprof kernel trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04zi_pytest.txt 2>&1 || { tail -30 gpurun_out/r04zi_pytest.txt; exit 1; }
tail -3 gpurun_out/r04zi_pytest.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04zi_smoke.txt 2>&1 || { tail -20 gpurun_out/r04zi_smoke.txt; exit 1; }
tail -2 gpurun_out/r04zi_smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/r04zi_bench.json 2> gpurun_out/r04zi_bench.err || { tail -5 gpurun_out/r04zi_bench.err; exit 1; }
tail -c 300 gpurun_out/r04zi_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04zi_prof -o bench -- python3 bench.py --no-cpu-baseline --no-modes --steps 50 > gpurun_out/r04zi_prof.log 2>&1 || { tail -5 gpurun_out/r04zi_prof.log; exit 1; }
echo round-ok
