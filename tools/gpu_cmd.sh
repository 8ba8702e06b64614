set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/rpca1; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_rpca.py tests/test_shim.py tests/test_gpu_c4_scale.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo done
