# 2-rank rehearsal of the multi-GPU bench on one GPU (gloo, both ranks on device 0), then a
# traced single-GPU bench whose exit status is recorded (exit-time fault check), the shim
# driver (concurrent per-point searches) and its host-ASan/UBSan build
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-rehearsal}; mkdir -p $O
PCP_BENCH_DEVICE=0 PCP_BENCH_BACKEND=gloo timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --points 5000000 --no-cpu > $O/rehearsal_2rank.json 2> $O/rehearsal_2rank.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/trace_bench.log 2>&1
echo "traced bench exit status $?" > $O/trace_rc.txt
timeout -k 10 600 tests/cpp/_build/shim_test > $O/shim_test.log 2>&1
ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 900 tests/cpp/_build/shim_test_asan > $O/shim_test_asan.log 2>&1
echo done
