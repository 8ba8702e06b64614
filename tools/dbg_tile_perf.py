"""Debug: tile-engine stage statistics and split timings at the bench's density (C4 street
scene, 50M points over 200 m x 200 m -> here N points over the same density)."""
import math, os, sys
import numpy as np
os.environ.setdefault("PCP_ICP_ENGINE", "tile")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pointcloudprocess_amd import ops, synth

n = int(os.environ.get("DBG_N", "12500000"))
ext = 200.0 * math.sqrt(n / 50e6)
ctx = ops.Context(0)
T_true = synth.rigid()
tgt, q = synth.icp_pair(n, n, 1, 2, T_true, extent=(ext, ext), device=ctx.device)
index = ops.GridIndex(ctx, tgt, cell_size=float(os.environ.get("DBG_CELL", "0.12")))
icp = ops.ICP(index, q)
for pi, T in enumerate((np.eye(4), T_true, T_true)):
    acc = icp.step(T, 0.25)
    print(f"pose {pi}: fallback {icp.last_fallback()} kernel ms {icp.last_kernel_ms()}", flush=True)
icp.close(); index.close(); ctx.close()
