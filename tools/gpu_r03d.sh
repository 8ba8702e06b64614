#!/bin/bash
# Round 3d: the tiled normals' far pass with a workgroup per deferred query (default) against one
# wave per query (variants/far1), interleaved, after the kNN / normals GPU tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03d}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_knn.py tests/test_gpu_rpca.py tests/test_gpu_bruteforce.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_knn.log 2>&1
for v in ${ORDER:-default}; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  echo "== $v" >> $O/normals_ab.log
  timeout -k 10 300 python3 -u tools/normals_ab.py --ks ${KS:-32} --tiles 2,0 >> $O/normals_ab.log 2>&1
done
echo done
