# ICP per-pass timings + octant list statistics per iteration (PCP_ICP_ABLATE=16: counters only)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-dbg}; mkdir -p $O
PCP_ICP_ABLATE=16 timeout -k 10 300 python3 tools/icp_micro.py --reps 1 > $O/micro_dbg16.log 2>&1
echo done
