# Round-4 GPU call Q: planes formed in place by the cell-wave fill (fp64 covariance, fp32 closed
# form; PCP_H16_CW_PLANES=1, default) against the separate planes pass (0): h16 tests, C5 full-size,
# interleaved C5 A/B, trace.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04q}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_h16.py -x -v -s --timeout 300 --timeout-method thread > $O/h16_tests.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py -x -v -s --timeout 800 --timeout-method thread -k c5 > $O/c5_full.log 2>&1
for i in 1 2; do
  for f in 1 0; do
    PCP_H16_CW_PLANES=$f timeout -k 10 200 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_pl$f.jsonl 2>> $O/c5_ab.err
  done
done
mkdir -p $O/C5
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5/trace -o run -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 > $O/C5/trace.log 2>&1
echo done
