set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/fold3; mkdir -p $O
timeout -k 10 200 python3 tools/fold_micro.py > $O/fold_micro.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo done
