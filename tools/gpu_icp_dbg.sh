# ICP accounting debug: the registration-exactness test with accumulator checks
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-icpdbg}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_icp.py -k "verify_pass_exact or device_loop_matches or correspondence_bit" > $O/icp_tests.log 2>&1 || true
echo done
