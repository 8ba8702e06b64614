set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-dbgtile}; mkdir -p $O
for ab in 0 128 256; do PCP_ICP_ABLATE=$ab timeout -k 10 300 python3 -u tools/dbg_tile.py > $O/dbg_$ab.log 2>&1; done
PCP_ICP_ENGINE=cache timeout -k 10 300 python3 -u tools/dbg_tile.py > $O/dbg_cache.log 2>&1
echo done
