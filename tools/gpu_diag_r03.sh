# Round-3 diagnostics: per-iteration verify reasons (PCP_ICP_ABLATE=16 counters) + baseline bench line
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-diag}; mkdir -p $O
PCP_ICP_ABLATE=16 timeout -k 10 300 python3 -u tools/icp_micro.py --reps 1 > $O/micro_dbg16.log 2>&1
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err
echo done
