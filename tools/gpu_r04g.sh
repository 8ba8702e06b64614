# Round-4 GPU call G: the fused C5 count (PCP_H16_FUSED, default 1): the h16 tests (incl. the
# fused-vs-two-pass byte test at the default and a 16-entry stride), the C5 full-size sampled band
# test, an interleaved C5 bench A/B (fused 1 vs 0), then the C5 trace and FETCH/WRITE passes.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04g}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_h16.py -x -v -s --timeout 300 --timeout-method thread > $O/h16_tests.log 2>&1
if [ -z "$NOFULL" ]; then
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py -x -v -s --timeout 800 --timeout-method thread -k c5 > $O/c5_full.log 2>&1
fi
for i in 1 2; do
  for f in 1 0; do
    PCP_H16_FUSED=$f timeout -k 10 200 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_fused$f.jsonl 2>> $O/c5_ab.err
  done
done
mkdir -p $O/C5
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5/trace -o run -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 > $O/C5/trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/C5/fetch -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/C5/write -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5/write.log 2>&1
echo done
