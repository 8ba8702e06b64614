# C5 kernel A/B: kernel traces of the C5 line (200M) for this tree and variants/$V for V in $VARS (or $VAR)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-c5planes}; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new$rep -o run -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 > $O/new$rep.log 2>&1
  for V in ${VARS:-${VAR:-trig0}}; do
    PCP_AB=1 PCP_LIB=variants/$V/libpcp.so timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${V}_$rep -o run -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 > $O/${V}_$rep.log 2>&1
  done
done
echo done
