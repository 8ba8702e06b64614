# Round-4 GPU call X (final record): the C5 planes pass with the fp32 closed form (7 waves/SIMD),
# h16 tests, the C5 full-size test, interleaved C5 A/B against the fp64 form
# (variants/p64), the C5 traffic + line for this h16.hip, then the whole GPU suite and smoke.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04x}; mkdir -p $O
P=profiles/${PTAG:-r04_final6}; mkdir -p $P
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_h16.py -x -v -s --timeout 300 --timeout-method thread > $O/h16_tests.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py -x -v -s --timeout 800 --timeout-method thread -k c5 > $O/c5_full.log 2>&1
for i in 1 2; do
  for v in new p64; do
    L=""; [ $v = p64 ] && L=$GRAFT_REPO_ROOT/variants/p64/libpcp.so
    PCP_LIB=$L timeout -k 10 200 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_$v.jsonl 2>> $O/c5_ab.err
  done
done
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/C5fetch -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/C5write -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5write.log 2>&1
python3 tools/pmc_summary.py --src=h16.hip $O/C5fetch $O/C5write k_h16_radius k_h16_tile k_h16_rows_to_caller tile_scan k_h16_ids k_h16_plane_default k_h16_sorted_counts k_h16_overflow k_h16_cw k_h16_cw_planes > $O/pmc_traffic_C5.json
cp $O/pmc_traffic_C5.json $P/pmc_traffic_C5.json
timeout -k 10 600 python3 -u bench.py --config C5 > $O/bench_C5.json 2> $O/bench_C5.err
mkdir -p $O/C5
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5/trace -o run -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 > $O/C5/trace.log 2>&1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo done
