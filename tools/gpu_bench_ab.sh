# bench.py (no CPU leg) per library variant, plus the GPU tests on the default build.
# ORDER lists variants (repeat names to interleave); every run is appended to $O/all.jsonl.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-benchab}; mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
for v in ${ORDER:-default ${VARIANTS}}; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_AB=1 PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  timeout -k 10 300 python3 bench.py --no-cpu --steps ${STEPS:-3} ${CELL:+--cell $CELL} > $O/bench_$v.json 2> $O/bench_$v.err
  python3 -c "import json,sys; d=json.load(open('$O/bench_$v.json')); d['label']='$v'; print(json.dumps(d))" >> $O/all.jsonl
done
echo done
