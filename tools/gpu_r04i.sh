# K4 phase stamps (debug build in the scratch tree).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/k4_stamps.py > gpurun_out/r04i_k4_stamps.log 2>&1 || { tail -30 gpurun_out/r04i_k4_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04i_k4_stamps.log
echo round-ok
