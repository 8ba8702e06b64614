# bench.py --config $CFG per library variant (ORDER: default | variant names, repeat to
# interleave), after the tests in $TESTS on the default build; runs -> $O/all.jsonl
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-cfgab}; mkdir -p $O
if [ -n "$TESTS" ]; then
timeout -k 10 600 python3 -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
for v in $ORDER; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_AB=1 PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  timeout -k 10 300 python3 bench.py --config $CFG --no-cpu > $O/bench_$v.json 2> $O/bench_$v.err
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['unit'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))" >> $O/summary.txt
done
echo done
