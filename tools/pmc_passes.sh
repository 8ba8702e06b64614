#!/bin/bash
# Collect a set of PMC passes (one rocprofv3 run each) over a command; profiling aid.
#   tools/pmc_passes.sh <outdir> -- <program> [args...]
# Writes <outdir>/pN/run_counter_collection.csv per pass.  Each pass runs under its own
# time limit; the script stops at the first failing pass.
set -e
out=$1; shift; [ "$1" = "--" ] && shift
passes=(  # at most 2 counters per TA/TCP/TCC block per pass (hardware limit)
  "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum"
  "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
  "TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum"
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum"
  "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES"
  "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum"
  "SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD"
)
mkdir -p "$out"
i=0
for p in "${passes[@]}"; do
  timeout -k 10 ${PASS_TIMEOUT:-150} rocprofv3 --pmc $p --output-format csv -d "$out/p$i" -o run -- "$@" > "$out/p$i.log" 2>&1
  i=$((i+1))
done
