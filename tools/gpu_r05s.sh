# Round-5: kernel trace of the c3 training step (timeline per step with tools/timeline.py).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train -o t -- python3 tools/train_steps.py 12 > $O/train.log 2>&1 || { tail -5 $O/train.log; exit 1; }
echo r05s-ok
