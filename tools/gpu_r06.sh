# Round-6 GPU call wrapper: STEPS selects what runs (space separated), each step under its own
# time limit, the first failure ends the call.
#   h16tests   the C5 tests (tests/test_gpu_h16.py) and the 200M full-size C5 test
#   icptests   the ICP tests and the 50M-scale C4 check
#   bftests    the brute-force kNN tests and the 1M x 1M full-size C2 check
#   c5ab       interleaved A/B of the C5 bench line: this tree vs variants/$VAR (PCP_LIB)
#   c5trace    rocprofv3 kernel trace + stats of one C5 bench run
#   tests      the whole GPU suite + smoke
#   c4ab       interleaved A/B of the C4 bench line: this tree vs variants/$V for V in $VARS (or $VAR)
#   c4trace    kernel trace of the C4 bench (per-iteration table)
#   c3ab       interleaved A/B of the C3 bench line vs variants/$V for V in $VARS
#   knntests   the kNN / normals tests and the full-size C3 check
#   c2ab       interleaved A/B of the C2 bench line vs variants/$VAR
#   octg       per-launch octant times at fixed search-list lanes per query (kernel traces)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06}; mkdir -p $O
for st in ${STEPS}; do
case $st in
micro)
  timeout -k 10 120 tools/sort_micro > $O/sort_micro.log 2>&1 ;;
c4bench)
  timeout -k 10 300 python3 -u bench.py --no-cpu --steps ${NSTEPS:-5} --warmup 2 >> $O/c4_bench.jsonl 2>> $O/c4_bench.err ;;
c5bench)
  timeout -k 10 300 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_bench.jsonl 2>> $O/c5_bench.err ;;
h16tests)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_h16.py "tests/test_gpu_fullsize.py::test_c5_fullsize_200m" -x -v -s --timeout 500 --timeout-method thread > $O/h16_tests.log 2>&1 ;;
bftests)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bruteforce.py "tests/test_gpu_fullsize.py::test_c2_fullsize_bit_exact" -x -v -s --timeout 500 --timeout-method thread > $O/bf_tests.log 2>&1 ;;
icptests)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_icp.py tests/test_gpu_c4_scale.py -x -v -s --timeout 500 --timeout-method thread > $O/icp_tests.log 2>&1 ;;
c5ab)
  for rep in 1 2; do
    timeout -k 10 300 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_new.jsonl 2>> $O/c5_ab.err
    for V in ${VARS:-$VAR}; do
      PCP_AB=1 PCP_LIB=variants/$V/libpcp.so timeout -k 10 300 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_$V.jsonl 2>> $O/c5_ab.err
    done
  done ;;
c5trace)
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5trace -o run -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 > $O/c5trace.log 2>&1 ;;
tests)
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1
  timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
c4ab)
  for rep in 1 2 3; do
    timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 --warmup 2 >> $O/c4_ab_new.jsonl 2>> $O/c4_ab.err
    for V in ${VARS:-$VAR}; do
      PCP_AB=1 PCP_LIB=variants/$V/libpcp.so timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 --warmup 2 >> $O/c4_ab_$V.jsonl 2>> $O/c4_ab.err
    done
  done ;;
c4trace)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4trace -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/c4trace.log 2>&1
  python3 tools/trace_iters.py $O/c4trace > $O/per_iteration.txt 2>&1 || true ;;
c3ab)
  for rep in 1 2 3; do
    timeout -k 10 300 python3 -u bench.py --config C3 --no-cpu --steps 5 >> $O/c3_ab_new.jsonl 2>> $O/c3_ab.err
    for V in ${VARS:-$VAR}; do
      PCP_AB=1 PCP_LIB=variants/$V/libpcp.so timeout -k 10 300 python3 -u bench.py --config C3 --no-cpu --steps 5 >> $O/c3_ab_$V.jsonl 2>> $O/c3_ab.err
    done
  done ;;
knntests)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_knn.py "tests/test_gpu_fullsize.py::test_c3_fullsize_voxel_and_normals" -x -v -s --timeout 500 --timeout-method thread > $O/knn_tests.log 2>&1 ;;
c2ab)
  for rep in 1 2; do
    timeout -k 10 300 python3 -u bench.py --config C2 --no-cpu --steps 3 >> $O/c2_ab_new.jsonl 2>> $O/c2_ab.err
    for V in ${VARS:-$VAR}; do
      PCP_AB=1 PCP_LIB=variants/$V/libpcp.so timeout -k 10 300 python3 -u bench.py --config C2 --no-cpu --steps 3 >> $O/c2_ab_$V.jsonl 2>> $O/c2_ab.err
    done
  done ;;
c5pmc)
  sq1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU"
  sq2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
  sq3="SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"
  mkdir -p $O/c5pmc
  timeout -k 10 60 rocprofv3 -L > $O/c5pmc/counters_list.txt 2>&1
  i=0
  for c in "$sq1" "$sq2" "$sq3" "WRITE_SIZE" "FETCH_SIZE"; do
    timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/c5pmc/p$i -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 --c5-points ${C5N:-50000000} > $O/c5pmc/p$i.log 2>&1
    i=$((i+1))
  done
  python3 tools/pmc_table.py $O/c5pmc k_h16 > $O/c5pmc/table.txt 2>&1 ;;
c5order)
  for rep in 1 2; do
    timeout -k 10 300 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_native.jsonl 2>> $O/c5_ab.err
    timeout -k 10 300 python3 -u bench.py --config C5 --no-cpu --steps 3 --c5-order cells >> $O/c5_ab_cells.jsonl 2>> $O/c5_ab.err
  done ;;
pmc)
  # SQ / traffic counters of one bench config: CFG (C2, C3, C5 ...), KEYS = kernel substrings
  sq1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU"
  sq2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
  sq3="SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE"
  ta1="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
  P=$O/pmc_$CFG; mkdir -p $P
  i=0
  for c in "$sq1" "$sq2" "$sq3" "$ta1" "WRITE_SIZE" "FETCH_SIZE"; do
    timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $P/p$i -o run -- python3 bench.py --config $CFG --no-cpu --steps 1 --warmup 0 $ARGS > $P/p$i.log 2>&1
    i=$((i+1))
  done
  python3 tools/pmc_table.py $P $KEYS > $P/table.txt 2>&1 ;;
trace)
  # kernel trace + stats of one bench config: CFG, ARGS
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$CFG -o run -- python3 bench.py --config $CFG --no-cpu --steps 3 --warmup 1 $ARGS > $O/trace_$CFG.log 2>&1 ;;
octg)
  # per-launch octant times with fixed lanes per query on the search lists (G = 1 2 4 8) and the
  # default density rule (0): one registration each under a kernel trace
  for G in 0 1 2 4 8; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/octg$G -o run -- python3 bench.py --no-cpu --steps 1 --warmup 0 --icp-lanes 0,$G,0 > $O/octg$G.log 2>&1
    python3 tools/trace_iters.py $O/octg$G > $O/octg$G.txt 2>&1 || true
  done ;;
rehearsal)
  # N = 2 on ONE GPU over gloo (the driver owns the 8-GPU runs): the C4 line and a 50M C5 line
  # with the slab-vs-single-process row check
  PCP_BENCH_DEVICE=0 PCP_BENCH_BACKEND=gloo timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu > $O/rehearsal_c4_2rank.json 2> $O/rehearsal_c4.err
  PCP_BENCH_DEVICE=0 PCP_BENCH_BACKEND=gloo timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --config C5 --c5-points 50000000 --c5-check 20000 > $O/rehearsal_c5_2rank.json 2> $O/rehearsal_c5.err ;;
esac
echo "step $st done" >> $O/steps.log
done
echo done
