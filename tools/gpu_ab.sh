# A/B: GPU tests on the default build, then the ICP micro per variant (profiling aid)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab}; mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
for v in default ${VARIANTS}; do
  if [ $v = default ]; then L=""; else L=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  PCP_LIB=$L PCP_ICP_ABLATE=${ABL:-32} timeout -k 10 200 python3 tools/icp_micro.py --reps 1 > $O/micro_$v.log 2>&1
done
echo done
