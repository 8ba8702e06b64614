# ICP iteration: the ICP GPU tests, smoke, a bench line + kernel trace, c4 scale
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-icp}; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_icp.py tests/test_gpu_cloud.py -k "icp or rot or tile or registration" > $O/icp_tests.log 2>&1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/trace_bench.log 2>&1
python3 tools/trace_iters.py $O/trace > $O/per_iteration.txt 2>&1 || true
if [ -n "$SCALE" ]; then timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_c4_scale.py > $O/c4_scale.log 2>&1; fi
echo done
