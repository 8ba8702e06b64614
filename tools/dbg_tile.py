"""Debug: tile-engine correspondences vs the oracle on test_correspondence_bit_exact's data."""
import os, sys
import numpy as np
os.environ.setdefault("PCP_ICP_ENGINE", "tile")
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ctypes as ora
from pointcloudprocess_amd import ops, synth

ctx = ops.Context(0)
T_true = synth.rigid()
tgt, q = synth.icp_pair(200_000, 200_000, 11, 12, T_true, extent=(40.0, 40.0))
tg = tgt.numpy()
o = tg.min(0)
print("target min", o, "max", tg.max(0), flush=True)
mode = os.environ.get("PCP_ICP_ABLATE", "0")
for cell in (0.3,):
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=cell)
    icp = ops.ICP(index, q.to(ctx.device))
    oi = ora.F32Index(tg)
    h = index.cell_size
    for pi, T in enumerate((np.eye(4), T_true, synth.rigid(0.2, 0.1, 0.1, (0.1, 0.1, -0.05)))):
        acc, ci, cd = icp.step(T, 0.25, corr=True)
        R = T[:3, :3].astype(np.float32)
        t = T[:3, 3].astype(np.float32)
        ei, ed = oi.correspond(q.numpy(), R, t, 0.25)
        gi, gd = ci.cpu().numpy(), cd.cpu().numpy()
        bad = np.nonzero(gi != ei)[0]
        print(f"[ablate {mode}] cell {cell} (h {h:.4f}) pose {pi}: {len(bad)} mismatches; fallback {icp.last_fallback()}", flush=True)
        for b in bad[:6]:
            qq = q.numpy()[b]
            qt = np.array([np.fma if False else 0 for _ in range(3)], np.float32)
            for r in range(3):
                x = np.float32(np.float32(R[r, 0]) * qq[0] + t[r])
                x = np.float32(np.float32(R[r, 1]) * qq[1] + x)
                x = np.float32(np.float32(R[r, 2]) * qq[2] + x)
                qt[r] = x
            f = (qt - o) / np.float32(h)
            fg = (tg[gi[b]] - o) / h if gi[b] >= 0 else None
            fe = (tg[ei[b]] - o) / h if ei[b] >= 0 else None
            print(f"  q {b}: got {gi[b]} d2 {gd[b]!r}, oracle {ei[b]} d2 {ed[b]!r}; f {f} got-cell {np.floor(fg) if fg is not None else None} oracle-cell {np.floor(fe) if fe is not None else None}", flush=True)
    icp.close(); index.close()
ctx.close()
