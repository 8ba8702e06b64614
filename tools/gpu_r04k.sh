# Round-4 GPU call K: the cell-wave C5 kernels after the padding-lane NaN fix: h16 tests, the ICP
# tests on the default build (cache memset change), the C5 full-size test, a C5 bench A/B over
# cw1 / cwpk / cwpkminb1 / cw0, then the C5 kernel trace.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04k}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_h16.py -x -v -s --timeout 300 --timeout-method thread > $O/h16_tests.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_icp.py tests/test_gpu_c4_scale.py -x -q --timeout 300 --timeout-method thread > $O/icp_tests.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py -x -v -s --timeout 800 --timeout-method thread -k c5 > $O/c5_full.log 2>&1
for i in 1 2; do
  for v in cw1 cwpk cwpkminb1 cw0; do
    L=""; F=1
    case $v in cwpk|cwpkminb1) L=$GRAFT_REPO_ROOT/variants/$v/libpcp.so;; esac
    [ $v = cw0 ] && F=0
    PCP_LIB=$L PCP_H16_CW=$F timeout -k 10 200 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_$v.jsonl 2>> $O/c5_ab.err
  done
done
mkdir -p $O/C5
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5/trace -o run -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 > $O/C5/trace.log 2>&1
echo done
