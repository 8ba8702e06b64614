# Round-4 GPU call R: the whole GPU suite (incl. the new cell-wave edge-case tests) and smoke on
# the final tree.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04r}; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo done
