# bench.py --config lines (C1, C2, C3, C5) with a rocprofv3 kernel-stats pass each
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-cfg}; mkdir -p $O
for c in ${CONFIGS:-C1 C2 C3 C5}; do
  timeout -k 10 300 python3 bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o run -- python3 bench.py --config $c --no-cpu --steps 2 > $O/trace_$c.log 2>&1
done
echo done
