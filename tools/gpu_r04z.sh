# Round-4 GPU call Z: the 2-rank one-GPU rehearsal of the C4 line on the final tree (gloo, 5M-vs-5M
# per rank's slab; per-rank pre-iteration / iterations spans).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04z}; mkdir -p $O
PCP_BENCH_DEVICE=0 PCP_BENCH_BACKEND=gloo timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --points 5000000 --no-cpu > $O/rehearsal_2rank.json 2> $O/rehearsal_2rank.err
echo done
