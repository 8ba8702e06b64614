"""Debug: per-iteration verify statistics (PCP_ICP_ABLATE=16 counters) over a 20-iteration
registration at the bench density (N points over the C4 scene's density)."""
import math, os, sys
import numpy as np
os.environ.setdefault("PCP_ICP_ABLATE", "16")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pointcloudprocess_amd import ops, synth

n = int(os.environ.get("DBG_N", "12500000"))
ext = 200.0 * math.sqrt(n / 50e6)
ctx = ops.Context(0)
T_true = synth.rigid()
tgt, q = synth.icp_pair(n, n, 1, 2, T_true, extent=(ext, ext), device=ctx.device)
index = ops.GridIndex(ctx, tgt, cell_size=0.12)
icp = ops.ICP(index, q)
T = np.eye(4)
for it in range(20):
    acc = icp.step(T, 0.25)
    print(f"iter {it}: searched {icp.last_searched()} fallback {icp.last_fallback()}", file=sys.stderr, flush=True)
    rc, dT = ops.icp_solve(acc.cpu().numpy())
    T = dT @ T
print("final T err", np.abs(T - T_true).max(), file=sys.stderr)
icp.close(); index.close(); ctx.close()
