# Round-4 GPU call B: the 2-rank one-GPU rehearsal (per-rank pre-iteration / iterations spans in the
# line), a C2 A/B of the grouped hit test (variants/bfg4, PCP_BF_GROUP=4, interleaved, with the
# brute-force tests on the variant), then the PMC passes of the C3/C5/C2 lines (HBM traffic and the
# SQ instruction / cycle set per kernel).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04b}; mkdir -p $O
if [ -z "$NOREH" ]; then
PCP_BENCH_DEVICE=0 PCP_BENCH_BACKEND=gloo timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --points 5000000 --no-cpu > $O/rehearsal_2rank.json 2> $O/rehearsal_2rank.err
fi
if [ -z "$NOC2" ]; then
for v in ${C2V:-bfglds bfglds2 bfglds4}; do
  [ -f variants/$v/libpcp.so ] || continue
  PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bruteforce.py -x -q --timeout 120 --timeout-method thread > $O/c2_${v}_tests.log 2>&1
done
for i in 1 2; do
  for v in default ${C2V:-bfglds bfglds2 bfglds4}; do
    if [ $v = default ]; then L=""; else L=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
    PCP_LIB=$L timeout -k 10 200 python3 -u bench.py --config C2 --no-cpu --steps 5 >> $O/c2_ab_$v.jsonl 2>> $O/c2_ab.err
  done
done
fi
if [ -z "$NOSORT" ]; then
PCP_QSORT_IDX=1 PCP_TSORT_IDX=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_icp.py tests/test_gpu_c4_scale.py -x -q --timeout 300 --timeout-method thread > $O/sortidx_tests.log 2>&1
for i in 1 2 3; do
  for v in 00 11 10 01; do
    PCP_QSORT_IDX=${v:0:1} PCP_TSORT_IDX=${v:1:1} timeout -k 10 200 python3 -u bench.py --no-cpu --steps 5 >> $O/c4_sort_ab_$v.jsonl 2>> $O/c4_sort_ab.err
  done
done
fi
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
