# K3 diagnostics: look-ahead and pair-workgroup stamps (debug build in the box's tree),
# then the PMC counters of the release build.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cp modulatedgps_amd/libmgp_hip.so /tmp/libmgp_release.so
timeout -k 10 240 python -u tools/chol_stamps.py 1024 > gpurun_out/r04c_stamps.log 2>&1 || { echo "stamps fail"; exit 1; }
timeout -k 10 240 python -u tools/chol_stamps.py 1024 --with-k1 > gpurun_out/r04c_stamps_k1.log 2>&1 || { echo "stamps k1 fail"; exit 1; }
cp /tmp/libmgp_release.so modulatedgps_amd/libmgp_hip.so
touch modulatedgps_amd/libmgp_hip.so
bash tools/k3_pmc.sh
echo round-ok
