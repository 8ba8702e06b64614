# Round-6 records, in parts (each call stays well inside gpurun's limit):
#   PART=tests  the GPU suite + smoke
#   PART=pmc    FETCH_SIZE / WRITE_SIZE passes (separate runs) of the C4, C5, C3 and C2 lines,
#               summarised into profiles/$PTAG/pmc_traffic*.json keyed on the sources' sha1 and the
#               workload (written under gpurun_out/; copy them into profiles/$PTAG/ before the
#               bench part, whose lines then quote them)
#   PART=pmc5   the C5 passes only
#   PART=bench  the C4 line (CPU baseline included), its kernel trace + per-iteration table, and
#               the C1 / C2 / C3 / C5 lines
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-final}; mkdir -p $O
P=profiles/${PTAG:-r06_final}; mkdir -p $P
case ${PART} in
tests)
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1
  timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
pmc)
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/pmc_fetch.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/pmc_write.log 2>&1
  python3 tools/pmc_summary.py --key=n=50000000 --key=world=1 --key=mode=slab $O/fetch $O/write > $O/pmc_traffic.json && cp $O/pmc_traffic.json $P/pmc_traffic.json
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/C5fetch -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5fetch.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/C5write -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5write.log 2>&1
  python3 tools/pmc_summary.py --src=h16.hip --key=n=200000000 --key=world=1 $O/C5fetch $O/C5write k_h16_mx k_h16_mx_planes k_h16_mx_planes_fb tile_scan k_h16_ids k_h16_plane_default > $O/pmc_traffic_C5.json && cp $O/pmc_traffic_C5.json $P/pmc_traffic_C5.json
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/C3fetch -o run -- python3 bench.py --config C3 --no-cpu --steps 1 --warmup 0 > $O/C3fetch.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/C3write -o run -- python3 bench.py --config C3 --no-cpu --steps 1 --warmup 0 > $O/C3write.log 2>&1
  python3 tools/pmc_summary.py --src=knn.hip --key=n=10000000 --key=world=1 $O/C3fetch $O/C3write k_normals_tile k_normals k_normals_coop k_brick_keys k_plane_default > $O/pmc_traffic_C3.json && cp $O/pmc_traffic_C3.json $P/pmc_traffic_C3.json
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/C2fetch -o run -- python3 bench.py --config C2 --no-cpu --steps 1 --warmup 0 > $O/C2fetch.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/C2write -o run -- python3 bench.py --config C2 --no-cpu --steps 1 --warmup 0 > $O/C2write.log 2>&1
  python3 tools/pmc_summary.py --src=knn_bf.hip --key=n=1000000 --key=world=1 $O/C2fetch $O/C2write k_bf_mfma k_bf_fallback k_bf_targets k_bf_pad > $O/pmc_traffic_C2.json && cp $O/pmc_traffic_C2.json $P/pmc_traffic_C2.json ;;
pmc5)  # the C5 passes only (after an h16.hip change)
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/C5fetch -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5fetch.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/C5write -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5write.log 2>&1
  python3 tools/pmc_summary.py --src=h16.hip --key=n=200000000 --key=world=1 $O/C5fetch $O/C5write k_h16_mx k_h16_mx_planes k_h16_mx_planes_fb tile_scan k_h16_ids k_h16_plane_default > $O/pmc_traffic_C5.json ;;
bench)
  timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/trace_bench.log 2>&1
  python3 tools/trace_iters.py $O/trace > $O/per_iteration.txt 2>&1 || true
  for c in ${CFGS:-C1 C2 C3 C5}; do
    timeout -k 10 600 python3 -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err
  done ;;
esac
echo done
