# Round-4 GPU call Y: the C5 planes pass with the fp32 closed form (variants/p32: 72 VGPRs, 7
# waves/SIMD; rows of fewer than 16 points and near-degenerate rows keep fp64) against the default
# fp64 form: h16 tests and the C5 full-size test on the variant, interleaved C5 A/B, variant trace.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04y}; mkdir -p $O
V=$GRAFT_REPO_ROOT/variants/p32/libpcp.so
PCP_LIB=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_h16.py -x -v -s --timeout 300 --timeout-method thread > $O/h16_tests_p32.log 2>&1
PCP_LIB=$V timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py -x -v -s --timeout 800 --timeout-method thread -k c5 > $O/c5_full_p32.log 2>&1
for i in 1 2; do
  for v in default p32; do
    L=""; [ $v = p32 ] && L=$V
    PCP_LIB=$L timeout -k 10 200 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_$v.jsonl 2>> $O/c5_ab.err
  done
done
mkdir -p $O/C5
PCP_LIB=$V timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5/trace -o run -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 > $O/C5/trace.log 2>&1
echo done
