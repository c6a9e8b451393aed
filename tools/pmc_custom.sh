# Ad-hoc counter passes (one group per rocprofv3 run, kernel-trace only) over
# tools/bench_kernels.py.  Usage on the GPU box:
#   ONLY=gram_x6_P PMC_GROUPS="SQ_INSTS_VALU SQ_INSTS_LDS;SQ_WAVE_CYCLES" bash tools/pmc_custom.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ONLY=${ONLY:-}
i=0
IFS=';' read -ra GS <<< "$PMC_GROUPS"
for c in "${GS[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmcc_$i -o p -- python3 tools/bench_kernels.py --reps 1 --only "$ONLY" > gpurun_out/pmcc_$i.log 2>&1 || { echo "fail $c"; exit 1; }
done
echo ok
