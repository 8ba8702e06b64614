set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-dbgperf}; mkdir -p $O
for ab in ${ABS:-16 272 0}; do PCP_ICP_ABLATE=$ab timeout -k 10 200 python3 -u tools/dbg_tile_perf.py > $O/perf_$ab.log 2>&1; done
PCP_ICP_ENGINE=cache PCP_ICP_ABLATE=16 timeout -k 10 200 python3 -u tools/dbg_tile_perf.py > $O/perf_cache.log 2>&1
echo done
