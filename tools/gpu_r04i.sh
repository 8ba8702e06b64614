# Round-4 GPU call I: the octant list launches with chunk-pipelined row starts (PCP_OCT_PF,
# variants/octpf): ICP parity tests on the variant, an interleaved C4 bench A/B, kernel traces.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04i}; mkdir -p $O
PCP_LIB=$GRAFT_REPO_ROOT/variants/octpf/libpcp.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_icp.py tests/test_gpu_c4_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/icp_tests_octpf.log 2>&1
for i in 1 2; do
  for v in default octpf; do
    if [ $v = default ]; then export PCP_LIB=""; else export PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
    timeout -k 10 300 python3 bench.py --no-cpu --steps 5 >> $O/c4_ab_$v.jsonl 2>> $O/c4_ab.err
  done
done
for v in default octpf; do
  if [ $v = default ]; then export PCP_LIB=""; else export PCP_LIB=$GRAFT_REPO_ROOT/variants/$v/libpcp.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$v -o run -- python3 bench.py --no-cpu --steps 1 --warmup 1 > $O/trace_$v.log 2>&1
done
echo done
