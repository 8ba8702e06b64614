set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-nrm}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_knn.py tests/test_gpu_rpca.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_knn.log 2>&1
timeout -k 10 400 python3 -u tools/normals_ab.py > $O/normals_ab.log 2>&1
echo done
