# FETCH_SIZE / WRITE_SIZE / TA / SQ counters of the ICP micro (one rocprofv3 --pmc run per pass)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-pmc}; mkdir -p $O
i=0
for p in "FETCH_SIZE" "WRITE_SIZE" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $O/p$i -o run -- python3 tools/icp_micro.py --reps 1 --iters ${ITERS:-12} > $O/p$i.log 2>&1
  i=$((i+1))
done
echo done
