# Round-5: hypothesis-driven shape properties (tests/test_gpu_properties.py).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zc
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -s tests/test_gpu_properties.py > $O/pytest_props.txt 2>&1 || { tail -60 $O/pytest_props.txt; exit 1; }
tail -3 $O/pytest_props.txt
echo r05zc-ok
