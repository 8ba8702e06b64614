set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/b3; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --steps 4 > $O/bench.json 2> $O/bench.err
echo done
