# Round-5: K3's per-step wall, shader clock and phases from in-kernel stamps (debug
# build in the box's scratch tree): standalone vs inside the c3 ELBO step.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 400 python3 tools/chol_stamps.py > $O/stamps_alone.log 2>&1 || { tail -20 $O/stamps_alone.log; exit 1; }
timeout -k 10 300 python3 tools/chol_stamps.py --elbo > $O/stamps_elbo.log 2>&1 || { tail -20 $O/stamps_elbo.log; exit 1; }
echo r05h-ok
