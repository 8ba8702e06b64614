# Round-3 record: full GPU suite, smoke, PMC traffic of the C4 iteration kernels (FETCH_SIZE and
# WRITE_SIZE in separate passes), the bench line (reads the sha-matched pmc_traffic.json written
# here), a kernel trace of the bench, and the other config lines.  Output under $O (merged back)
# and, for the bench's traffic lookup on this box, $P/pmc_traffic.json.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-final}; mkdir -p $O
P=profiles/${PTAG:-r03_final}; mkdir -p $P
if [ -z "$NOTEST" ]; then
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/pmc_write.log 2>&1
python3 tools/pmc_summary.py $O/fetch $O/write > $O/pmc_traffic.json
cp $O/pmc_traffic.json $P/pmc_traffic.json
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/trace_bench.log 2>&1
python3 tools/trace_iters.py $O/trace > $O/per_iteration.txt 2>&1 || true
if [ -z "$NOCFG" ]; then
for c in C1 C2 C3 C5; do
  timeout -k 10 600 python3 -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err
done
fi
echo done
