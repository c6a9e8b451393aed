# K4 item order A/B: in half of the workgroups the small row tile of the pair first
# (k4o1: by dispatch round on a CU, k4o2: alternate workgroups on an XCD) vs k4o0 (the kept order).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for v in k4o0 k4o1 k4o2; do
    MGP_HIP_LIB=$PWD/abvar/$v.so timeout -k 10 120 python -u tools/bench_kernels.py --reps 5 --only trsm_stats_f16 > gpurun_out/r04u_k4_$v.json 2>/dev/null || { echo "k4 $v fail"; exit 1; }
    echo "$v $(tail -c 200 gpurun_out/r04u_k4_$v.json)" >> gpurun_out/r04u_k4_ab.log
    MGP_HIP_LIB=$PWD/abvar/$v.so timeout -k 10 200 python -u tools/elbo_ab.py 3 50 $v >> gpurun_out/r04u_elbo_ab.log 2>&1 || exit 1
  done
done
cat gpurun_out/r04u_k4_ab.log; grep -v amdgpu.ids gpurun_out/r04u_elbo_ab.log
echo round-ok
