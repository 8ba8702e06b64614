# G-lane ring pass A/B: ICP GPU tests on the default build, then one traced bench registration per variant
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ring}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_icp.py tests/test_gpu_c4_scale.py -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
TAG=${TAG:-ring} ORDER="${ORDER:-rg1 default}" bash tools/gpu_variant_trace.sh
