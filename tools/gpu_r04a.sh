# Round-4 GPU call: the whole GPU suite (incl. the full-size C2/C3/C5 parity tests), a C3 A/B of the
# per-lane window scan (PCP_TILE_LANE 1 vs 0, interleaved) with its debug counters, the C4 bench
# line and kernel trace, and counters of the C2/C3/C5 lines: HBM traffic (FETCH_SIZE / WRITE_SIZE
# passes) and the SQ instruction / cycle set (two passes) per kernel.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04a}; mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread ${TESTS:-} > $O/gpu_tests.log 2>&1
fi
if [ -z "$NOAB" ]; then
PCP_KNN_DEBUG=1 timeout -k 10 200 python3 -u bench.py --config C3 --no-cpu --steps 1 --warmup 0 > $O/c3_debug.json 2> $O/c3_debug.err
for i in 1 2; do
  for l in 1 0; do
    PCP_TILE_LANE=$l timeout -k 10 200 python3 -u bench.py --config C3 --no-cpu --steps 5 >> $O/c3_ab_lane$l.jsonl 2>> $O/c3_ab.err
  done
done
for i in 1 2; do
  for t in 1 0; do
    PCP_H16_TILE=$t timeout -k 10 200 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_tile$t.jsonl 2>> $O/c5_ab.err
  done
done
fi
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 5 > $O/bench_C4.json 2> $O/bench_C4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/trace_bench.log 2>&1
python3 tools/trace_iters.py $O/trace > $O/per_iteration.txt 2>&1 || true
if [ -z "$NOPMC" ]; then
sq1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU"
sq2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_F32 SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
for cfg in ${CFGS:-C3 C5 C2}; do
  mkdir -p $O/$cfg
  extra=""; [ $cfg = C5 ] && extra="--c5-points ${C5N:-200000000}"
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$cfg/trace -o run -- python3 bench.py --config $cfg --no-cpu --steps 2 --warmup 1 $extra > $O/$cfg/trace.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$cfg/fetch -o run -- python3 bench.py --config $cfg --no-cpu --steps 1 --warmup 0 $extra > $O/$cfg/fetch.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$cfg/write -o run -- python3 bench.py --config $cfg --no-cpu --steps 1 --warmup 0 $extra > $O/$cfg/write.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc $sq1 --output-format csv -d $O/$cfg/p0 -o run -- python3 bench.py --config $cfg --no-cpu --steps 1 --warmup 0 $extra > $O/$cfg/p0.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc $sq2 --output-format csv -d $O/$cfg/p1 -o run -- python3 bench.py --config $cfg --no-cpu --steps 1 --warmup 0 $extra > $O/$cfg/p1.log 2>&1
done
fi
echo done
