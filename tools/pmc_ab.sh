# PMC A/B of the ICP micro per variant (profiling aid); one rocprofv3 run per counter pass.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-pmcab}; mkdir -p $O
passes=(
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
  "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD"
  "FETCH_SIZE"
  "WRITE_SIZE TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
)
for v in ${VARIANTS:-default}; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_AB=1 PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  mkdir -p $O/$v; i=0
  for p in "${passes[@]}"; do
    timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $O/$v/p$i -o run -- python3 tools/icp_micro.py --reps 1 --iters ${ITERS:-8} > $O/$v/p$i.log 2>&1
    i=$((i+1))
  done
done
echo done
