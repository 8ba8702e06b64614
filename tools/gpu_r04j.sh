# Round-4 GPU call J: the cell-wave C5 kernels (PCP_H16_CW, default 1): the h16 tests (incl. the
# cell-wave vs per-lane byte test), the C5 full-size sampled band test, an interleaved C5 bench
# A/B (cw 1 vs 0), then the C5 kernel trace.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04j}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_h16.py -x -v -s --timeout 300 --timeout-method thread > $O/h16_tests.log 2>&1
if [ -z "$NOFULL" ]; then
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py -x -v -s --timeout 800 --timeout-method thread -k c5 > $O/c5_full.log 2>&1
fi
for i in 1 2; do
  for v in cw1 cwpk cwpkminb1 cw0; do
    L=""; F=1
    case $v in cwminb1|cwpk|cwpkminb1) L=$GRAFT_REPO_ROOT/variants/$v/libpcp.so;; esac
    [ $v = cw0 ] && F=0
    PCP_LIB=$L PCP_H16_CW=$F timeout -k 10 200 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_$v.jsonl 2>> $O/c5_ab.err
  done
done
mkdir -p $O/C5
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5/trace -o run -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 > $O/C5/trace.log 2>&1
echo done
