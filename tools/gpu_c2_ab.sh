#!/bin/bash
# C2 A/B by library variant (C2ORDER, interleaved) with the brute-force tests on each variant.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-c2ab}; mkdir -p $O
for v in ${C2ORDER:-default}; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_AB=1 PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  if [ ! -f $O/tests_$v.log ]; then
    timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bruteforce.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1
  fi
  timeout -k 10 300 python3 bench.py --config C2 --no-cpu > $O/bench_C2_$v.json 2> $O/bench_C2_$v.err
  python3 -c "import json; d=json.load(open('$O/bench_C2_$v.json')); print('$v', d['value'], d['unit'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))" >> $O/c2_summary.txt
done
echo done
