# K4 batching probe: two launches at N = 65536 vs one at N = 131072.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/k4_batch_probe.py > gpurun_out/r04w_k4_batch_probe.log 2>&1 || { tail -20 gpurun_out/r04w_k4_batch_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04w_k4_batch_probe.log
echo round-ok
