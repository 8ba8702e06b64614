# kernel trace of one bench registration (+ per-iteration pass table)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-tb}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/trace_bench.log 2>&1
python3 tools/trace_iters.py $O/trace > $O/per_iteration.txt 2>&1
echo done
