# Octant pass lanes-per-query A/B (PCP_OCT_G="first,list"): ICP GPU tests under each setting
# in GS, then interleaved bench runs (every run appended to $O/all.jsonl) and one kernel trace
# per setting (per-iteration octant times via tools/trace_iters.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-octg}; mkdir -p $O
GS=${GS:-"1,1 1,4"}
for gs in $GS; do
  PCP_OCT_G=$gs timeout -k 10 400 python3 -u -m pytest tests/test_gpu_icp.py ${SCALE:+tests/test_gpu_c4_scale.py} -x -q \
    --timeout 200 --timeout-method thread > $O/tests_${gs/,/_}.log 2>&1
done
for rep in 1 2; do
  for gs in $GS; do
    PCP_OCT_G=$gs timeout -k 10 300 python3 bench.py --no-cpu --steps 3 > $O/bench_${gs/,/_}_$rep.json 2> $O/bench.err
    python3 -c "import json; d=json.load(open('$O/bench_${gs/,/_}_$rep.json')); d['label']='$gs'; print(json.dumps(d))" >> $O/all.jsonl
  done
done
for gs in $GS; do
  PCP_OCT_G=$gs timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_${gs/,/_} -o run -- \
    python3 bench.py --no-cpu --steps 1 --warmup 1 > $O/trace.log 2>&1
done
echo done
