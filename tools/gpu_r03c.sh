#!/bin/bash
# Round 3c: far-pass row prefetch (normals A/B by library, ORDER) and the C2 sign-bit filter
# (bench --config C2 per library, C2ORDER), after the kNN / brute-force GPU tests (default
# build, and the brute-force tests again on the c2sign build).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03c}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_knn.py tests/test_gpu_rpca.py tests/test_gpu_bruteforce.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_knn.log 2>&1
PCP_LIB=$GRAFT_REPO_ROOT/variants/c2sign/libpcp.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bruteforce.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_c2sign.log 2>&1
for v in ${ORDER:-default}; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  echo "== $v" >> $O/normals_ab.log
  timeout -k 10 300 python3 -u tools/normals_ab.py --ks 32 --tiles 2,0 >> $O/normals_ab.log 2>&1
done
for v in ${C2ORDER:-default}; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  timeout -k 10 300 python3 bench.py --config C2 --no-cpu > $O/bench_C2_$v.json 2> $O/bench_C2_$v.err
  python3 -c "import json; d=json.load(open('$O/bench_C2_$v.json')); print('$v', d['value'], d['unit'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))" >> $O/c2_summary.txt
done
echo done
