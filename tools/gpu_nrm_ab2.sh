# normals k=32 (C3 centroids): tests on the default build, then the A/B timing + debug counters
# of the default and base libraries, then the C3 line per library
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-nrm2}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_knn.py tests/test_gpu_bruteforce.py tests/test_gpu_rpca.py -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
for v in default base default base; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  timeout -k 10 300 python3 -u tools/normals_ab.py --ks 32 --tiles 2,0 > $O/ab_$v.log 2>&1
  echo "== $v" >> $O/summary.txt; grep -v amdgpu $O/ab_$v.log | grep "tile_R\|coop: queries" >> $O/summary.txt
done
echo done
