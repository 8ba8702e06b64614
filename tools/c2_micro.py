"""C2 micro-run for profiling: one 1M x 1M brute-force kNN (k=8)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloudprocess_amd import ops, synth  # noqa: E402
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ctx = ops.Context(0)
t = synth.uniform_cube(n, 2001, device=ctx.device)
q = synth.uniform_cube(n, 2002, device=ctx.device)
ops.knn_bruteforce(ctx, t, q, 8)
torch.cuda.synchronize()
print("fallback", ops.knn_bruteforce_last_fallback(ctx))
