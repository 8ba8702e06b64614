"""Generate the known-answer fixtures pinned by the reference's own smoke tests.

The reference ships no fixtures and cannot be built here; its two
hot-path smoke tests print answers that follow from the reference semantics alone:

* main_test.cpp:156-188 ``test_kd_tree``: 100 points (0.1 i, 0.1 i, 0.1 i), query at the
  origin, KdTreeFLANN::nearestKSearch k=10.
* main_test.cpp:126-154 ``test_voxel_grid``: (i,i,i) for i<10 then (0.1 i,...) for i<100,
  VoxelGrid leaf (1,1,1).

This script recomputes both answers in plain Python (independently of oracle/ and of the
HIP code), following kd_tree.h:814-845 (+ FLANN L2_Simple accumulation) and
voxel_grid.h:811-1056 (+ concatenate.h:153 float cast), and writes JSON fixtures.
Floats are stored with repr() so they round-trip bit-exactly.

Run: python tests/golden/make_golden.py
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def kat_kd_tree():
    cloud = [(0.1 * i, 0.1 * i, 0.1 * i) for i in range(100)]  # main_test.cpp:159-164
    q = (0.0, 0.0, 0.0)
    res = []
    for j, p in enumerate(cloud):
        r = 0.0  # flann::L2_Simple<double>: result += diff*diff, left to right
        for a in range(3):
            d = q[a] - p[a]
            r += d * d
        res.append((r, j))
    res.sort()
    k = 10
    return {
        "source": "main_test.cpp:156-188 test_kd_tree",
        "cloud_xyz": cloud,
        "query": q,
        "k": k,
        "expected_indices": [j for _, j in res[:k]],
        "expected_sqr_distances": [r for r, _ in res[:k]],
    }


def f32(v):
    return float(np.float32(v))


def kat_voxel_grid():
    pts = [(float(i), float(i), float(i)) for i in range(10)]          # main_test.cpp:129-135
    pts += [(0.1 * i, 0.1 * i, 0.1 * i) for i in range(100)]           # :136-142
    leaf = 1.0
    inv = 1.0 / leaf
    mn = [min(p[a] for p in pts) for a in range(3)]
    mx = [max(max(p[a] for p in pts), 2.2250738585072014e-308) for a in range(3)]
    min_b = [int(mn[a] * inv) for a in range(3)]
    max_b = [int(mx[a] * inv) for a in range(3)]
    div_b = [max_b[a] - min_b[a] + 1 for a in range(3)]
    mul = [1, div_b[0], div_b[0] * div_b[1]]
    keyed = []
    for cp, p in enumerate(pts):
        ijk = [int(p[a] * inv - min_b[a]) for a in range(3)]
        keyed.append((ijk[0] * mul[0] + ijk[1] * mul[1] + ijk[2] * mul[2], cp))
    keyed.sort()
    out = []
    i0 = 0
    while i0 < len(keyed):
        i1 = i0
        while i1 < len(keyed) and keyed[i1][0] == keyed[i0][0]:
            i1 += 1
        c = [0.0, 0.0, 0.0]
        for s in range(i0, i1):
            p = pts[keyed[s][1]]
            for a in range(3):
                c[a] += f32(p[a])  # NdCopyPointEigenFunctor static_cast<float>
        n = i1 - i0
        out.append({"voxel_idx": keyed[i0][0], "count": n,
                    "xyz": [c[a] / n for a in range(3)]})
        i0 = i1
    return {
        "source": "main_test.cpp:126-154 test_voxel_grid",
        "cloud_xyz": pts,
        "leaf": [leaf, leaf, leaf],
        "expected": out,
    }


def main():
    for name, fn in (("kat_kd_tree.json", kat_kd_tree), ("kat_voxel_grid.json", kat_voxel_grid)):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(fn(), f, indent=1)
        print("wrote", name)


if __name__ == "__main__":
    main()
