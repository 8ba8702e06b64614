# Per-kernel durations (rocprofv3 --kernel-trace --stats) of the ICP micro under PCP_ICP_ABLATE values
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-kt}; mkdir -p $O
for ab in ${ABL:-0}; do
  export PCP_ICP_ABLATE=$ab
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$ab -o run -- python3 tools/icp_micro.py --reps 1 ${MICRO_ARGS} > $O/kt_$ab.log 2>&1
done
echo done
