# a subset of the GPU tests (TESTS="tests/a.py tests/b.py")
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-sub}; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest ${TESTS} -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
echo done
