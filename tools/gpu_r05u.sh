# Round-5: K4 timing probes (results wrong in the probe arms): _ab/k4nostore.so (no A-image
# stores), _ab/k4loop.so (main loop only, no epilogue), against the kept library.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05u
mkdir -p $O
for r in 1 2; do
  for v in base k4loop; do
    lib=$PWD/modulatedgps_amd/_ab/$v.so
    MGP_HIP_LIB=$lib timeout -k 10 200 python3 tools/bench_kernels.py --reps 10 --only trsm_f16_pair,trsm_stats_f16,trsm_f16_nostats > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    echo "$v $r $(tail -1 $O/${v}_$r.json)"
  done
done
echo r05u-ok
