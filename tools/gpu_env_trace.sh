# Kernel traces (one bench registration each) under each PCP_OCT_G setting in GS, then of the
# library variants in ORDER (variants/NAME/libpcp.so); per-iteration times via trace_iters.py
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-etrace}; mkdir -p $O
for gs in ${GS:-}; do
  PCP_OCT_G=$gs timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_g${gs/,/_} -o run -- \
    python3 bench.py --no-cpu --steps 1 --warmup 1 > $O/trace.log 2>&1
done
for v in ${ORDER:-}; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$v -o run -- python3 bench.py --no-cpu --steps 1 --warmup 1 > $O/trace_$v.log 2>&1
done
echo done
