# Training-step kernel profile (c3) and a full bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04d_train -o tr -- python3 tools/train_steps.py 10 > gpurun_out/r04d_train.log 2>&1 || { echo "train trace fail"; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r04d_bench.json 2> gpurun_out/r04d_bench.err || { tail -5 gpurun_out/r04d_bench.err; exit 1; }
tail -c 300 gpurun_out/r04d_bench.json
echo round-ok
