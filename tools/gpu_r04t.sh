# Round-4 GPU call T: the octant list launches with 2-record load batches at 5 / 6 waves per SIMD
# (variants/lu2w5, lu2w6; default 4-record batches at 4 waves): ICP tests on both variants, an
# interleaved C4 A/B and kernel traces (per-launch octant times).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04t}; mkdir -p $O
for v in lu2w5 lu2w6; do
  PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_icp.py tests/test_gpu_c4_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/icp_tests_$v.log 2>&1
done
for i in 1 2; do
  for v in default lu2w5 lu2w6; do
    L=""; [ $v != default ] && L=$GRAFT_REPO_ROOT/variants/$v/libpcp.so
    PCP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --steps 5 >> $O/c4_ab_$v.jsonl 2>> $O/c4_ab.err
  done
done
for v in default lu2w5 lu2w6; do
  L=""; [ $v != default ] && L=$GRAFT_REPO_ROOT/variants/$v/libpcp.so
  PCP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$v -o run -- python3 bench.py --no-cpu --steps 1 --warmup 1 > $O/trace_$v.log 2>&1
done
echo done
