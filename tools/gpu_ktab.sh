# kernel-trace A/B: the ICP micro under rocprofv3 --kernel-trace --stats per library variant
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ktab}; mkdir -p $O
for v in default ${VARIANTS}; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  export PCP_ICP_ABLATE=${ABL:-32}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 tools/icp_micro.py --reps 1 ${MICRO_ARGS} > $O/kt_$v.log 2>&1
done
echo done
