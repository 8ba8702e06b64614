# the ICP tests against an A/B build (variants/$VAR): a variant that changes results must still pass
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-x12}; mkdir -p $O
PCP_AB=1 PCP_LIB=variants/${VAR:-xyz12}/libpcp.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_icp.py tests/test_gpu_c4_scale.py -x -q --timeout 500 --timeout-method thread > $O/icp_tests_${VAR:-xyz12}.log 2>&1
echo tests-ok
