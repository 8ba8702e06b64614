#!/bin/bash
# Round 3b: buffered tile insertion and the flat far pass, A/B by library variant
# (ORDER: default | variant names under variants/; "default:near0" = PCP_NORMALS_NEAR=0),
# after the kNN/normals GPU tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-nrm3b}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_knn.py tests/test_gpu_rpca.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_knn.log 2>&1
for spec in ${ORDER:-default}; do
  v=${spec%%:*}
  unset PCP_NORMALS_NEAR
  if [ "$spec" != "$v" ]; then export PCP_NORMALS_NEAR=0; fi
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  echo "== $spec" >> $O/normals_ab.log
  timeout -k 10 300 python3 -u tools/normals_ab.py --ks ${KS:-32} --tiles ${TILES:-2,0} >> $O/normals_ab.log 2>&1
done
echo done
