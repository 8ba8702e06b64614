# Round profile: GPU tests, PMC FETCH/WRITE passes and a kernel trace of bench.py (run under gpurun)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-round}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu > $O/trace_bench.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
echo done
