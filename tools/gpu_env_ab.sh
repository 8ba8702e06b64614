# bench.py (no CPU leg) per environment setting of one variable, interleaved; every run is
# appended to $O/all.jsonl with label = the value.  VAR=name VALS="a b c" ROUNDS=2
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-envab}; mkdir -p $O
if [ -n "$TESTS" ]; then
timeout -k 10 600 python3 -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
for r in $(seq ${ROUNDS:-2}); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python3 bench.py --no-cpu --steps ${STEPS:-3} > $O/bench_$v.json 2> $O/bench_$v.err
    python3 -c "import json,sys; d=json.load(open('$O/bench_$v.json')); d['label']='$VAR=$v'; print(json.dumps(d))" >> $O/all.jsonl
  done
done
echo done
