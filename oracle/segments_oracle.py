"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's region growing, the checker
for pcp_region_growing (pointcloudprocess_amd/csrc/segments.hip).  Never imported by the
product path.

Follows TreeExtration::region_growning (extraction_tree.cpp:177-271) step by step: UnSegment
as a walk over indices in ascending order, one nearestKSearch(cloud[PointID[p]], 50) per
popped point (the oracle kd-tree, issued lazily in pop order as the reference does), the
float tests of compute_included_angle_between_vector (:36-44) and
compute_distance_from_point_to_plane (:47-64) in float32 numpy arithmetic, the > 5 size rule
and the reset of a dropped segment's SegmentID.  The filters follow static.cpp:24-79.

Parity: the walk and the float tests are restated from the source; the reference ships no
fixture for this path, so the oracle is pinned only through its kd-tree (itself pinned by
tests/golden/kat_kd_tree.json) -- "parity unpinned" for the segmentation rules themselves.
One assumption is recorded: sqrt of a float argument resolves to cmath's float overload
(MSVC's <cmath> and libstdc++ with `using namespace std` both pick it).
"""
import numpy as np

F = np.float32
K = 50


def plane_dis(a, b, c, d, x, y, z):
    """compute_distance_from_point_to_plane, vectorised over points (float32 inputs)."""
    a, b, c, d = F(a), F(b), F(c), F(d)
    x1, y1, z1 = x.astype(F), y.astype(F), z.astype(F)
    g = np.float64(np.sqrt(F(F(a * a) + F(b * b)) + F(c * c)).astype(F))
    f = np.abs((((a * x1).astype(np.float64) + (b * y1).astype(np.float64)) + (c * z1).astype(np.float64))
               + np.float64(d))
    return (f / g).astype(F)


def included_cos(nx, ny, nz, vx, vy, vz):
    """compute_included_angle_between_vector with a fixed first vector, vectorised."""
    nx, ny, nz = F(nx), F(ny), F(nz)
    n_n1 = ((nx * vx).astype(F) + (ny * vy).astype(F)).astype(F) + (nz * vz).astype(F)
    n_n = np.sqrt(F(F(nx * nx) + F(ny * ny)) + F(nz * nz)).astype(F)
    n1 = np.sqrt(((vx * vx).astype(F) + (vy * vy).astype(F)).astype(F) + (vz * vz).astype(F)).astype(F)
    return np.abs((n_n1.astype(F) / (n_n * n1).astype(F)).astype(F))


def region_growing(xyz, props, tree, distance_t, cosfa_t):
    """xyz (n, 3) float64; props: structured LAS_POINT_PROPERTY array (modified: segment_id);
    tree: an oracle KdTree over xyz.  Returns [(seed, [point ids in push order])]."""
    n = len(xyz)
    nxs, nys, nzs = props["normal_x"], props["normal_y"], props["normal_z"]
    seg = np.full(n, -1, np.int64)
    walked = np.zeros(n, bool)
    out = []
    label = 0
    for m0 in range(n):
        if walked[m0]:
            continue
        walked[m0] = True
        if not props["curvature"][m0] < 0.005:
            continue
        nx, ny, nz = nxs[m0], nys[m0], nzs[m0]
        seg[m0] = label
        members = [m0]
        fifo = [m0]
        head = 0
        while head < len(fifo):
            p = fifo[head]
            head += 1
            row, _ = tree.knn(xyz[props["point_id"][p]][None, :], K)
            row = row[0]
            row = row[row >= 0]
            q = row[seg[row] == -1]
            if not len(q):
                continue
            cs = included_cos(nx, ny, nz, nxs[q], nys[q], nzs[q])
            dis = plane_dis(nxs[p], nys[p], nzs[p], F(props["distance"][p]), xyz[q, 0], xyz[q, 1], xyz[q, 2])
            for j in q[(cs.astype(np.float64) > cosfa_t) & (dis.astype(np.float64) < distance_t)]:
                seg[j] = label
                members.append(int(j))
                walked[j] = True
                fifo.append(int(j))
        if len(members) > 5:
            out.append((m0, members))
            label += 1
        else:
            seg[members] = -1
    props["segment_id"] = seg
    return out


def filters(segments, props, n):
    """tree / shaft / ground filter point lists (static.cpp:24-79) from region_growing's output."""
    tree = [j for _, m in segments if len(m) > 50 for j in m]
    shaft = [j for s, m in segments if abs(float(props["normal_z"][s])) < 0.30 for j in m]
    ground = set(j for s, m in segments if abs(float(props["normal_z"][s])) > 0.9 for j in m)
    return tree, shaft, [i for i in range(n) if i not in ground]
