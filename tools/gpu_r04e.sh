# Round-4 GPU call E: the C5 fill's 64-byte flushes (default) against 16-byte ones (variants/flush4):
# tests, interleaved A/B at 200M points, FETCH/WRITE traffic of both; FETCH/WRITE of the C2/C3 lines.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04e}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_h16.py tests/test_gpu_fullsize.py tests/test_gpu_knn.py -x -v -s --timeout 500 --timeout-method thread -k "h16 or c5 or c3 or normals" > $O/h16_tests.log 2>&1
for i in 1 2; do
  for v in default flush4; do
    L=""; [ $v = flush4 ] && L=$GRAFT_REPO_ROOT/variants/flush4/libpcp.so
    PCP_LIB=$L timeout -k 10 200 python3 -u bench.py --config C5 --no-cpu --steps 3 >> $O/c5_ab_$v.jsonl 2>> $O/c5_ab.err
  done
done
for v in default flush4; do
  L=""; [ $v = flush4 ] && L=$GRAFT_REPO_ROOT/variants/flush4/libpcp.so
  mkdir -p $O/C5_$v
  PCP_LIB=$L timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/C5_$v/fetch -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5_$v/fetch.log 2>&1
  PCP_LIB=$L timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/C5_$v/write -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0 > $O/C5_$v/write.log 2>&1
done
PCP_LIB="" timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5_trace -o run -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 > $O/C5_trace.log 2>&1
for c in C3 C2; do
  mkdir -p $O/$c
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$c/fetch -o run -- python3 bench.py --config $c --no-cpu --steps 1 --warmup 0 > $O/$c/fetch.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$c/write -o run -- python3 bench.py --config $c --no-cpu --steps 1 --warmup 0 > $O/$c/write.log 2>&1
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${c}_trace -o run -- python3 bench.py --config $c --no-cpu --steps 2 --warmup 1 > $O/${c}_trace.log 2>&1
done
echo done
