# Round-4 GPU call P: C3 FETCH/WRITE traffic (knn.hip changed since r04e) and the C3 line; the C5
# cell-wave kernels with fp64-reciprocal cell coordinates and a row dy/dz table (h16 tests, C5 A/B
# against the record-2 build variants/c5head), then the C5 traffic and line for this h16.hip.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04p}; mkdir -p $O
P=profiles/${PTAG:-r04_final3}; mkdir -p $P
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/C3fetch -o run -- python3 bench.py --config C3 --no-cpu --steps 1 --warmup 0 > $O/C3fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/C3write -o run -- python3 bench.py --config C3 --no-cpu --steps 1 --warmup 0 > $O/C3write.log 2>&1
python3 tools/pmc_summary.py --src=knn.hip $O/C3fetch $O/C3write k_normals_tile k_normals k_normals_coop k_brick_keys k_plane_default > $O/pmc_traffic_C3.json
cp $O/pmc_traffic_C3.json $P/pmc_traffic_C3.json
timeout -k 10 600 python3 -u bench.py --config C3 > $O/bench_C3.json 2> $O/bench_C3.err
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_h16.py -x -v -s --timeout 300 --timeout-method thread > $O/h16_tests.log 2>&1
for i in 1 2; do
  for v in new c5head; do
    L=""; [ $v = c5head ] && L=$GRAFT_REPO_ROOT/variants/c5head/libpcp.so
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
echo done
