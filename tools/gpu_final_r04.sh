# Round-4 record: the GPU suite, smoke, PMC traffic of the C4 iteration kernels and of the C5 row
# kernels (FETCH_SIZE and WRITE_SIZE in separate passes; written into profiles/ on the box so the
# bench lines find them sha-matched), the C4 bench line (CPU baseline included), a kernel trace of
# it, and the C1/C2/C3/C5 lines.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-final}; mkdir -p $O
P=profiles/${PTAG:-r04_final}; mkdir -p $P
if [ -z "$NOTEST" ]; then
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/pmc_write.log 2>&1
python3 tools/pmc_summary.py $O/fetch $O/write > $O/pmc_traffic.json
cp $O/pmc_traffic.json $P/pmc_traffic.json
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/C5fetch -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/C5write -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5write.log 2>&1
python3 tools/pmc_summary.py --src=h16.hip $O/C5fetch $O/C5write k_h16_radius k_h16_tile k_h16_rows_to_caller tile_scan k_h16_ids k_h16_plane_default k_h16_sorted_counts k_h16_overflow k_h16_cw k_h16_cw_planes > $O/pmc_traffic_C5.json
cp $O/pmc_traffic_C5.json $P/pmc_traffic_C5.json
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/trace_bench.log 2>&1
python3 tools/trace_iters.py $O/trace > $O/per_iteration.txt 2>&1 || true
if [ -z "$NOCFG" ]; then
for c in C1 C2 C3 C5; do
  timeout -k 10 600 python3 -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err
done
fi
echo done
