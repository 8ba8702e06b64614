# Kernel traces (one bench registration each) of library variants in ORDER (variants/NAME/libpcp.so)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-vtrace}; mkdir -p $O
for v in ${ORDER:-default}; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$v -o run -- python3 bench.py --no-cpu --steps 1 --warmup 1 > $O/trace_$v.log 2>&1
done
echo done
