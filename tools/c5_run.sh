# BASELINE config 5 on one GPU on the current tree: K3 launch structures at M = 2048
# (tools/chol_probe.py), then the c5 bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
PROBE_M=2048 timeout -k 10 240 python -u tools/chol_probe.py > gpurun_out/k3_c5_probe.log 2>&1 && cat gpurun_out/k3_c5_probe.log || exit 1
timeout -k 10 600 python bench.py --config c5 --steps 10 --warmup 2 > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err; rc=$?; tail -c 600 gpurun_out/c5_bench.json; exit $rc
