# K3 pair-workgroup stamps with the entry and load-issue times (debug build).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/chol_stamps.py 1024 > gpurun_out/r04r_stamps.log 2>&1 || { echo "stamps fail"; tail -5 gpurun_out/r04r_stamps.log; exit 1; }
grep -A16 "pair workgroup" gpurun_out/r04r_stamps.log; head -18 gpurun_out/r04r_stamps.log
echo round-ok
