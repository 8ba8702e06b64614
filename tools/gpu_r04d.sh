# Round-4 GPU call D: the GPU suite on the current defaults (C2 LDS-DMA tiles, C3 one-pass lane
# windows), a C3 A/B (default / PCP_TILE_ROWTAB variant / union-box scan), the C2 and C3 lines, and
# one SQ counter pass of the C3 line.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04d}; mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
for i in 1 2; do
  for v in default rowtab lane0; do
    L=""; LM=1
    [ $v = rowtab ] && L=$GRAFT_REPO_ROOT/variants/rowtab/libpcp.so
    [ $v = lane0 ] && LM=0
    PCP_LIB=$L PCP_TILE_LANE=$LM timeout -k 10 200 python3 -u bench.py --config C3 --no-cpu --steps 5 >> $O/c3_ab_$v.jsonl 2>> $O/c3_ab.err
  done
done
timeout -k 10 300 python3 -u bench.py --config C2 --no-cpu --steps 5 > $O/bench_C2.json 2> $O/bench_C2.err
sq1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU"
sq2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_F32 SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
for c in C3 C2; do
  mkdir -p $O/$c
  timeout -s KILL 300 rocprofv3 --pmc $sq1 --output-format csv -d $O/$c/p0 -o run -- python3 bench.py --config $c --no-cpu --steps 1 --warmup 0 > $O/$c/p0.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc $sq2 --output-format csv -d $O/$c/p1 -o run -- python3 bench.py --config $c --no-cpu --steps 1 --warmup 0 > $O/$c/p1.log 2>&1
done
echo done
