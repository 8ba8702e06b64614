# Round-4 GPU call C: kernel traces of the C5 row kernels (per-lane, LDS-staged, LDS-staged with the
# direct caller-order fill) at 25M points and of C3 (lane windows on / off), then the C4 pre-iteration
# sort A/B ((key, index) pairs + gather vs record payloads) with the ICP tests on the variant.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04c}; mkdir -p $O
for t in 0 1 D; do
  if [ $t = D ]; then T=1; DI=1; else T=$t; DI=0; fi
  PCP_H16_TILE=$T PCP_H16_DIRECT=$DI timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_$t -o run -- python3 bench.py --config C5 --c5-points 25000000 --no-cpu --steps 2 --warmup 1 > $O/c5_$t.log 2>&1
done
for l in 1 0; do
  PCP_TILE_LANE=$l timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3_$l -o run -- python3 bench.py --config C3 --no-cpu --steps 2 --warmup 1 > $O/c3_$l.log 2>&1
done
PCP_QSORT_IDX=1 PCP_TSORT_IDX=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_icp.py tests/test_gpu_c4_scale.py -x -q --timeout 300 --timeout-method thread > $O/sortidx_tests.log 2>&1
for i in 1 2; do
  for v in 00 11; do
    PCP_QSORT_IDX=${v:0:1} PCP_TSORT_IDX=${v:1:1} timeout -k 10 200 python3 -u bench.py --no-cpu --steps 5 >> $O/c4_sort_ab_$v.jsonl 2>> $O/c4_sort_ab.err
  done
done
PCP_QSORT_IDX=1 PCP_TSORT_IDX=1 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4_trace11 -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/c4_trace11.log 2>&1
echo done
