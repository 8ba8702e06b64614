# ICP GPU tests + a bench line (quick check of an ICP kernel change)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-icpchk}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_icp.py tests/test_gpu_c4_scale.py -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 2 > $O/trace_bench.log 2>&1
echo done
