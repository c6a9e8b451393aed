# Round-4 baseline on a fresh box: the GPU suite, then one bench line.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04a_pytest.txt 2>&1
tail -3 gpurun_out/r04a_pytest.txt
timeout -k 10 300 python bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err
tail -c 400 gpurun_out/r04a_bench.json
echo round-ok
