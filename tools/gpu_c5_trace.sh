# C5 kernel traces at 25M and 200M points per GPU
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-c5trace}; mkdir -p $O
for n in 25000000 200000000; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$n -o run -- python3 bench.py --config C5 --no-cpu --steps 1 --warmup 1 --c5-points $n > $O/t$n.log 2>&1
done
echo done
