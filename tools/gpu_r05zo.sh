# Round-5: trsm_bwd16 with two-factor scales (tiles of tiny gA values): the c_images
# backward tests incl. the new "tiny" pattern, run on the x6 B-d library too.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zo
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py -k "c_images" > $O/pytest.txt 2>&1; st=$?
tail -5 $O/pytest.txt
[ $st -eq 0 ] || [ $st -eq 1 ] || exit 1
MGP_HIP_LIB=$PWD/modulatedgps_amd/_ab/x6bwd.so timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_backward.py -k "c_images and tiny" > $O/pytest_x6.txt 2>&1; tail -3 $O/pytest_x6.txt
echo r05zo-done
