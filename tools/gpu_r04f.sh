# Round-4 GPU call F: the C5 fill's late id gather (variants/lateid) and two C2 occupancy variants
# (variants/bfq2w2: two query blocks per wave at 2 waves/SIMD; variants/bfw3: 3 waves/SIMD), each
# with its parity tests, interleaved A/B against the default.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04f}; mkdir -p $O
PCP_LIB=$GRAFT_REPO_ROOT/variants/lateid/libpcp.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_h16.py tests/test_gpu_fullsize.py -x -v -s --timeout 500 --timeout-method thread -k "h16 or c5" > $O/lateid_tests.log 2>&1
for v in bfq2w2 bfw3; do
  PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bruteforce.py -x -q --timeout 120 --timeout-method thread > $O/${v}_tests.log 2>&1
done
for i in 1 2; do
  for v in default lateid; do
    L=""; [ $v = lateid ] && L=$GRAFT_REPO_ROOT/variants/lateid/libpcp.so
    PCP_LIB=$L timeout -k 10 200 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_$v.jsonl 2>> $O/ab.err
  done
  for v in default bfq2w2 bfw3; do
    L=""; [ $v != default ] && L=$GRAFT_REPO_ROOT/variants/$v/libpcp.so
    PCP_LIB=$L timeout -k 10 200 python3 -u bench.py --config C2 --no-cpu --steps 5 >> $O/c2_ab_$v.jsonl 2>> $O/ab.err
  done
done
echo done
