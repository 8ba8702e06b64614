set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/mg2; mkdir -p $O

timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
PCP_BENCH_DEVICE=0 PCP_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 2 --no-cpu > $O/bench_g2.json 2> $O/bench_g2.err
echo done
