#!/bin/bash
# Normals A/B by library variant (ORDER, interleaved), with the kNN / normals / RPCA GPU tests
# run on the variant named in TESTLIB (default build when unset).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03k}; mkdir -p $O
if [ -n "$TESTLIB" ]; then export PCP_LIB=$GRAFT_REPO_ROOT/variants/$TESTLIB/libpcp.so; fi
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_knn.py tests/test_gpu_rpca.py tests/test_segments.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_knn.log 2>&1
unset PCP_LIB
for v in ${ORDER:-default}; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  echo "== $v" >> $O/normals_ab.log
  timeout -k 10 300 python3 -u tools/normals_ab.py --ks ${KS:-32} --tiles ${TILES:-2,0} >> $O/normals_ab.log 2>&1
done
echo done
