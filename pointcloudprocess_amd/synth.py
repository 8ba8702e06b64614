"""Synthetic LiDAR-like clouds for benchmarks and parity tests.

The reference's data (HD-map PCD slices) is not available; BASELINE.json's configs are
quoted on synthetic clouds of these shapes.  torch is used only as a seeded RNG that runs
on the host or on the device (identical algorithm, device-specific random streams).
"""
import math

import numpy as np
import torch


def _u(g, n, lo, hi, device):
    return torch.rand(n, generator=g, device=device, dtype=torch.float64) * (hi - lo) + lo


def street_scene(n, seed, extent=(200.0, 200.0), noise=0.01, device="cpu", dtype=torch.float32):
    """Street scene: undulating ground + building facades + poles (C3/C4/C5 generator).

    Returns an (n, 3) tensor centred near the origin.  Points are allocated to the three
    surface kinds in proportion to their area, so the surface density is about uniform
    (as in the reference's inputs, which remove_duplicate(0.04) caps at ~625 pts/m^2;
    point_cloud_helper.cpp:42-63, main_blend.cpp:276,462).
    """
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    X, Y = float(extent[0]), float(extent[1])
    n_sx = len(np.arange(-X / 2 + 25, X / 2, 50.0))
    n_sy = len(np.arange(-Y / 2 + 25, Y / 2, 50.0))
    n_poles = 2 * n_sy * len(np.arange(-X / 2 + 7.5, X / 2, 15.0))
    a_ground = X * Y
    a_fac = 11.5 * (2 * n_sx * Y + 2 * n_sy * X)     # mean facade height 11.5 m
    a_pole = n_poles * 2 * math.pi * 0.15 * 6.0
    a_tot = a_ground + a_fac + a_pole
    n_ground = int(n * a_ground / a_tot)
    n_fac = int(n * a_fac / a_tot)
    n_pole = n - n_ground - n_fac

    def gnoise(m):
        return torch.randn(m, generator=g, device=device, dtype=torch.float64) * noise

    def ground_z(x, y):
        return 0.3 * torch.sin(x / 15.0) + 0.2 * torch.cos(y / 20.0)

    # ground
    gx = _u(g, n_ground, -X / 2, X / 2, device)
    gy = _u(g, n_ground, -Y / 2, Y / 2, device)
    gz = ground_z(gx, gy) + gnoise(n_ground)

    # facades: streets every 50 m along both axes, facade planes at +-9 m of each centreline
    sx = torch.tensor([c for c in np.arange(-X / 2 + 25, X / 2, 50.0)], dtype=torch.float64, device=device)
    sy = torch.tensor([c for c in np.arange(-Y / 2 + 25, Y / 2, 50.0)], dtype=torch.float64, device=device)
    planes_x = torch.cat([sx - 9.0, sx + 9.0])  # planes x = const (span y)
    planes_y = torch.cat([sy - 9.0, sy + 9.0])  # planes y = const (span x)
    npl = planes_x.numel() + planes_y.numel()
    k = torch.randint(0, npl, (n_fac,), generator=g, device=device)
    along_is_x = k >= planes_x.numel()
    u = torch.where(along_is_x, _u(g, n_fac, -X / 2, X / 2, device), _u(g, n_fac, -Y / 2, Y / 2, device))
    seg = torch.floor(u / 12.0) + k.to(torch.float64) * 101.0
    hgt = 8.0 + 7.0 * torch.frac(torch.abs(torch.sin(seg * 12.9898) * 43758.5453))
    v = torch.rand(n_fac, generator=g, device=device, dtype=torch.float64) * hgt
    off = torch.where(along_is_x, planes_y[(k - planes_x.numel()).clamp(min=0)],
                      planes_x[k.clamp(max=planes_x.numel() - 1)])
    relief = 0.05 * torch.sin(u * 2.0) * torch.sin(v * 1.3)
    w = off + relief + gnoise(n_fac)
    fx = torch.where(along_is_x, u, w)
    fy = torch.where(along_is_x, w, u)
    fz = ground_z(fx, fy) + v

    # poles: every 15 m along the streets at +-6 m
    px_list, py_list = [], []
    for c in np.arange(-Y / 2 + 25, Y / 2, 50.0):
        for a in np.arange(-X / 2 + 7.5, X / 2, 15.0):
            px_list += [a, a]
            py_list += [c - 6.0, c + 6.0]
    ppx = torch.tensor(px_list, dtype=torch.float64, device=device)
    ppy = torch.tensor(py_list, dtype=torch.float64, device=device)
    j = torch.randint(0, ppx.numel(), (n_pole,), generator=g, device=device)
    th = _u(g, n_pole, 0.0, 2 * math.pi, device)
    rr = 0.15 + gnoise(n_pole)
    qx = ppx[j] + rr * torch.cos(th)
    qy = ppy[j] + rr * torch.sin(th)
    qz = ground_z(qx, qy) + _u(g, n_pole, 0.0, 6.0, device)

    x = torch.cat([gx, fx, qx])
    y = torch.cat([gy, fy, qy])
    z = torch.cat([gz, fz, qz])
    pts = torch.stack([x, y, z], dim=1)
    # shuffle so that the input order carries no spatial structure
    perm = torch.randperm(n, generator=g, device=device)
    return pts[perm].to(dtype)


def rigid(deg_z=0.05, deg_x=0.02, deg_y=-0.015, t=(0.05, -0.04, 0.02)):
    """Row-major 4x4 double: R = Rz Ry Rx, translation t."""
    a, b, c = (math.radians(v) for v in (deg_z, deg_y, deg_x))
    Rz = np.array([[math.cos(a), -math.sin(a), 0], [math.sin(a), math.cos(a), 0], [0, 0, 1]])
    Ry = np.array([[math.cos(b), 0, math.sin(b)], [0, 1, 0], [-math.sin(b), 0, math.cos(b)]])
    Rx = np.array([[1, 0, 0], [0, math.cos(c), -math.sin(c)], [0, math.sin(c), math.cos(c)]])
    T = np.eye(4)
    T[:3, :3] = Rz @ Ry @ Rx
    T[:3, 3] = t
    return T


def apply_inverse(pts, T):
    """q = R^T (p - t) computed in float64, returned in pts' dtype (query = target frame
    moved by T^-1, so ICP(query -> target) should recover T)."""
    R = torch.as_tensor(T[:3, :3], dtype=torch.float64, device=pts.device)
    t = torch.as_tensor(T[:3, 3], dtype=torch.float64, device=pts.device)
    return ((pts.to(torch.float64) - t) @ R).to(pts.dtype)


def icp_pair(n_target, n_query, seed_t, seed_q, T_true, extent=(200.0, 200.0), device="cpu"):
    tgt = street_scene(n_target, seed_t, extent=extent, device=device)
    src = street_scene(n_query, seed_q, extent=extent, device=device)
    return tgt, apply_inverse(src, T_true)


def uniform_cube(n, seed, half=50.0, device="cpu"):
    """C2: uniform in [-half, half]^3, fp32-representable, as float64."""
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    p = (torch.rand((n, 3), generator=g, device=device, dtype=torch.float64) * 2 - 1) * half
    return p.to(torch.float32).to(torch.float64)
