# ICP iteration: the ICP GPU tests, smoke, a bench line and the per-pass counters (PCP_ICP_ABLATE=16)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-icp}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_icp.py tests/test_gpu_cloud.py -k "icp or rot" > $O/icp_tests.log 2>&1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err
PCP_ICP_ABLATE=16 timeout -k 10 300 python3 -u tools/icp_micro.py --reps 1 > $O/micro_dbg16.log 2>&1
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_c4_scale.py > $O/c4_scale.log 2>&1
echo done
