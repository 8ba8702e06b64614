# tile engine iteration: stage statistics + timings at the bench density, then the ICP tests
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-tileiter}; mkdir -p $O
for ab in 16 0; do PCP_ICP_ABLATE=$ab timeout -k 10 200 python3 -u tools/dbg_tile_perf.py > $O/perf_$ab.log 2>&1; done
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_icp.py tests/test_gpu_cloud.py -k "icp or rot or tile or registration" > $O/icp_tests.log 2>&1
echo done
