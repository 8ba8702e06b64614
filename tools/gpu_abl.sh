# ICP micro under several PCP_ICP_ABLATE values (profiling aid; ablated results are meaningless)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abl}; mkdir -p $O
for ab in ${ABL:-32}; do
  PCP_ICP_ABLATE=$ab timeout -k 10 200 python3 tools/icp_micro.py --reps 1 > $O/micro_$ab.log 2>&1
done
echo done
