# bench.py (no CPU leg) at several ICP grid cell sizes, default library (run under gpurun).
# Cells below ~0.095 m turn the C4 grid sparse (cell table > 16 n), i.e. the slow general path.
# Repeat sizes in CELLS to interleave; every run is appended to $O/all.jsonl.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-cellsweep}; mkdir -p $O
for c in ${CELLS:-0.1 0.11 0.12}; do
  timeout -k 10 300 python3 bench.py --no-cpu --steps ${STEPS:-3} --cell $c > $O/bench_$c.json 2> $O/bench_$c.err
  python3 -c "import json,sys; d=json.load(open('$O/bench_$c.json')); d['label']='cell$c'; print(json.dumps(d))" >> $O/all.jsonl
done
echo done
