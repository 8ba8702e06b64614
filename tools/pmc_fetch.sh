# FETCH_SIZE (+ TCC hit/miss) of the ICP micro kernels: one rocprofv3 --pmc run per pass
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-pmcf}; mkdir -p $O
for v in default ${VARIANTS}; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_AB=1 PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  mkdir -p $O/$v
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$v/p0 -o run -- python3 tools/icp_micro.py --reps 1 --iters ${ITERS:-6} > $O/$v/p0.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/$v/p1 -o run -- python3 tools/icp_micro.py --reps 1 --iters ${ITERS:-6} > $O/$v/p1.log 2>&1
done
echo done
