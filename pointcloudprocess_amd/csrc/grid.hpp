// Device-side view of the uniform-grid index and the exact ring search shared by the
// kNN / radius / normals / ICP kernels.
//
// Cells: c_a = floor((v_a - o_a) * inv_h) in the index precision (float for the fp32
// ICP index, double for the fp64 FLANN-contract index), identical in build and search.
// Bricks of 4x4x4 cells; brick table -> slot; cell (slot, local) owns sorted points
// [cstart[64*slot+local], cstart[64*slot+local+1]).
#pragma once
#include <functional>

#include "common.hpp"

namespace pcp {

// the fp32 build with a callback once the grid geometry is final (before the cell sort is
// enqueued on the context's stream): pcp_icp_create_with_target starts the query sort there
using GeomHook = std::function<int(const GridDesc&)>;
int index_build_f32_hooked(pcp_ctx* ctx, const float* xyz, size_t stride, int64_t n, double cell_size,
                           pcp_index** out, const GeomHook& on_geom);

template <typename T> struct Real;
template <> struct Real<float> {
    using V4 = float4;
    __device__ static float floor_(float x) { return floorf(x); }
};
template <> struct Real<double> {
    using V4 = double4;
    __device__ static double floor_(double x) { return floor(x); }
};

template <typename T> __device__ __forceinline__ T g_o(const GridDesc& g, int a);
template <> __device__ __forceinline__ float g_o<float>(const GridDesc& g, int a) { return g.of[a]; }
template <> __device__ __forceinline__ double g_o<double>(const GridDesc& g, int a) { return g.o[a]; }
template <typename T> __device__ __forceinline__ T g_inv(const GridDesc& g);
template <> __device__ __forceinline__ float g_inv<float>(const GridDesc& g) { return g.inv_hf; }
template <> __device__ __forceinline__ double g_inv<double>(const GridDesc& g) { return g.inv_h; }

// continuous cell coordinate (unclamped, saturated to +-2^30 to keep int conversion safe)
template <typename T>
__device__ __forceinline__ T cell_f(const GridDesc& g, T v, int a) {
    T f = (v - g_o<T>(g, a)) * g_inv<T>(g);
    f = f < (T)-1073741824.0 ? (T)-1073741824.0 : f;
    f = f > (T)1073741824.0 ? (T)1073741824.0 : f;
    return f;
}

template <typename T>
__device__ __forceinline__ int cell_i(const GridDesc& g, T v, int a) {
    return (int)Real<T>::floor_(cell_f<T>(g, v, a));
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ int64_t brick_of(const GridDesc& g, int cx, int cy, int cz) {
    return ((int64_t)(cz >> 2) * g.nb[1] + (cy >> 2)) * g.nb[0] + (cx >> 2);
}
__device__ __forceinline__ int local_of(int cx, int cy, int cz) {
    return (cx & 3) | ((cy & 3) << 2) | ((cz & 3) << 4);
}

__device__ __forceinline__ int64_t dense_id(const GridDesc& g, int cx, int cy, int cz) {
    return ((int64_t)cz * g.n[1] + cy) * g.n[0] + cx;
}

// cstart index of an in-range cell, or -1 when its brick is empty (sparse mode)
__device__ __forceinline__ int64_t cell_id(const GridDesc& g, int cx, int cy, int cz) {
    if (g.dense) return dense_id(g, cx, cy, cz);
    const int32_t slot = g.brick[brick_of(g, cx, cy, cz)];
    return slot < 0 ? -1 : (int64_t)slot * 64 + local_of(cx, cy, cz);
}

// point range of an in-range cell; returns false when the cell is empty
__device__ __forceinline__ bool cell_range(const GridDesc& g, int cx, int cy, int cz,
                                           uint32_t& s, uint32_t& e) {
    const int64_t c = cell_id(g, cx, cy, cz);
    if (c < 0) return false;
    s = g.cstart[c];
    e = g.cstart[c + 1];
    return e > s;
}

// Exact two-level ring search.  Phase 1 visits cells in order of Chebyshev distance from
// the query's cell up to kCellRings; phase 2 (only when the visitor's bound still reaches
// further) walks rings of 4x4x4-cell bricks, skipping empty bricks through the brick
// occupancy table and the cells phase 1 already covered -- so an isolated query costs
// O((r/4h)^3) brick probes instead of O((r/h)^3) cell probes.
//   V::bound()       current pruning radius^2 (in the index precision's units), may shrink
//   V::visit(s, e)   scan sorted points [s,e)
// Cells, bricks and whole rings whose box distance exceeds bound() (with a conservative
// margin `mc` in cell units covering floor() rounding of both the cells and the query) are
// skipped without touching their points.  Visiting order never changes the result:
// visitors keep a lexicographic (d2, index) order.
constexpr int kCellRings = 3;

template <typename T>
__device__ __forceinline__ T axis_gap(int c, int cq, T l) {
    // cells between the query (cell cq, offset l in it) and cell c along one axis
    return c < cq ? (l + (T)(cq - c - 1)) : (c > cq ? ((T)1 - l + (T)(c - cq - 1)) : (T)0);
}

template <typename T>
__device__ __forceinline__ T sq_gap(T gcell, T mc) {
    return gcell > mc ? (gcell - mc) * (gcell - mc) : (T)0;
}

template <typename T, typename Vis>
__device__ void brick_search(const GridDesc& g, T fx, T fy, T fz, int cx, int cy, int cz, T lx, T ly, T lz,
                             T mc, Vis& vis) {
    const T h2 = (T)g.h * (T)g.h;
    const int bx = cx >> 2, by = cy >> 2, bz = cz >> 2;  // floor division
    // query offset inside its brick (cells) and the distance to the nearest brick face
    const T ox = fx - (T)(4 * bx), oy = fy - (T)(4 * by), oz = fz - (T)(4 * bz);
    const T bdmin = fmin(fmin(fmin(ox, (T)4 - ox), fmin(oy, (T)4 - oy)), fmin(oz, (T)4 - oz));
    int far = 0;
    far = max(far, max(bx - (g.nb[0] - 1), -bx));
    far = max(far, max(by - (g.nb[1] - 1), -by));
    far = max(far, max(bz - (g.nb[2] - 1), -bz));
    const int sbmax = far + max(g.nb[0], max(g.nb[1], g.nb[2]));
    for (int sb = 0; sb <= sbmax; sb++) {
        if (sb > 0) {
            const T rmin = (T)(4 * (sb - 1)) + bdmin - mc;
            if (rmin > (T)0 && rmin * rmin * h2 > vis.bound()) return;
        }
        const int z0 = max(bz - sb, 0), z1 = min(bz + sb, g.nb[2] - 1);
        const int y0 = max(by - sb, 0), y1 = min(by + sb, g.nb[1] - 1);
        const int x0 = max(bx - sb, 0), x1 = min(bx + sb, g.nb[0] - 1);
        if (z0 > z1 || y0 > y1 || x0 > x1) continue;
        for (int zb = z0; zb <= z1; zb++) {
            const bool zface = (zb == bz - sb) || (zb == bz + sb);
            // brick box gap along z (cells)
            const T gz = zb < bz ? (oz + (T)(4 * (bz - zb - 1))) : (zb > bz ? ((T)4 - oz + (T)(4 * (zb - bz - 1))) : (T)0);
            const T gz2 = sq_gap(gz, mc);
            if (gz2 * h2 > vis.bound()) continue;
            for (int yb = y0; yb <= y1; yb++) {
                const bool yface = zface || (yb == by - sb) || (yb == by + sb);
                const T gy = yb < by ? (oy + (T)(4 * (by - yb - 1))) : (yb > by ? ((T)4 - oy + (T)(4 * (yb - by - 1))) : (T)0);
                const T gyz2 = gz2 + sq_gap(gy, mc);
                if (gyz2 * h2 > vis.bound()) continue;
                const int step = yface ? 1 : 2 * sb;
                for (int xb = yface ? x0 : bx - sb; xb <= x1; xb += (step > 0 ? step : 1)) {
                    if (xb < x0) continue;
                    const T gx = xb < bx ? (ox + (T)(4 * (bx - xb - 1))) : (xb > bx ? ((T)4 - ox + (T)(4 * (xb - bx - 1))) : (T)0);
                    if ((gyz2 + sq_gap(gx, mc)) * h2 > vis.bound()) continue;
                    if (g.brick[((int64_t)zb * g.nb[1] + yb) * g.nb[0] + xb] < 0) continue;  // empty brick
                    // the brick's cells not covered by phase 1
                    for (int z = 4 * zb; z < min(4 * zb + 4, g.n[2]); z++) {
                        const T cz2 = sq_gap(axis_gap<T>(z, cz, lz), mc);
                        const bool zin = abs(z - cz) <= kCellRings;
                        for (int y = 4 * yb; y < min(4 * yb + 4, g.n[1]); y++) {
                            const T cyz2 = cz2 + sq_gap(axis_gap<T>(y, cy, ly), mc);
                            if (cyz2 * h2 > vis.bound()) continue;
                            const bool yzin = zin && abs(y - cy) <= kCellRings;
                            for (int x = 4 * xb; x < min(4 * xb + 4, g.n[0]); x++) {
                                if (yzin && abs(x - cx) <= kCellRings) continue;
                                if ((cyz2 + sq_gap(axis_gap<T>(x, cx, lx), mc)) * h2 > vis.bound()) continue;
                                uint32_t st, en;
                                if (cell_range(g, x, y, z, st, en)) vis.visit(st, en);
                            }
                        }
                    }
                }
            }
        }
    }
}

// kFar = false: cell rings only; returns false when the bound still reaches past them (the
// caller then re-runs the query with kFar = true).  kFar = true: complete two-level search.
template <typename T, typename Vis, bool kFar = true>
__device__ __forceinline__ bool ring_search(const GridDesc& g, T qx, T qy, T qz, T mc, Vis& vis) {
    const T fx = cell_f<T>(g, qx, 0), fy = cell_f<T>(g, qy, 1), fz = cell_f<T>(g, qz, 2);
    const int cx = (int)Real<T>::floor_(fx), cy = (int)Real<T>::floor_(fy), cz = (int)Real<T>::floor_(fz);
    // offsets inside the query's own cell
    const T lx = fx - (T)cx, ly = fy - (T)cy, lz = fz - (T)cz;
    const T h2 = (T)g.h * (T)g.h;
    const T dmin = fmin(fmin(fmin(lx, (T)1 - lx), fmin(ly, (T)1 - ly)), fmin(lz, (T)1 - lz));
    // the furthest ring that can still intersect the grid
    int far = 0;
    far = max(far, max(cx - (g.n[0] - 1), -cx));
    far = max(far, max(cy - (g.n[1] - 1), -cy));
    far = max(far, max(cz - (g.n[2] - 1), -cz));
    const int rmax = far + max(g.n[0], max(g.n[1], g.n[2]));
    const int smax = min(rmax, kCellRings);
    for (int s = 0; s <= smax + 1; s++) {
        if (s > 0) {
            const T rmin = ((T)(s - 1) + dmin - mc);
            if (rmin > (T)0 && rmin * rmin * h2 > vis.bound()) return true;
        }
        if (s > smax) break;
        const int z0 = max(cz - s, 0), z1 = min(cz + s, g.n[2] - 1);
        const int y0 = max(cy - s, 0), y1 = min(cy + s, g.n[1] - 1);
        const int x0 = max(cx - s, 0), x1 = min(cx + s, g.n[0] - 1);
        if (z0 > z1 || y0 > y1 || x0 > x1) continue;
        for (int z = z0; z <= z1; z++) {
            const bool zface = (z == cz - s) || (z == cz + s);
            const T gz2 = sq_gap(axis_gap<T>(z, cz, lz), mc);
            if (gz2 * h2 > vis.bound()) continue;
            for (int y = y0; y <= y1; y++) {
                const bool yface = zface || (y == cy - s) || (y == cy + s);
                const T gyz2 = gz2 + sq_gap(axis_gap<T>(y, cy, ly), mc);
                if (gyz2 * h2 > vis.bound()) continue;
                const int step = yface ? 1 : 2 * s;
                for (int x = yface ? x0 : cx - s; x <= x1; x += (step > 0 ? step : 1)) {
                    if (x < x0) continue;
                    if ((gyz2 + sq_gap(axis_gap<T>(x, cx, lx), mc)) * h2 > vis.bound()) continue;
                    uint32_t st, en;
                    if (cell_range(g, x, y, z, st, en)) vis.visit(st, en);
                }
            }
        }
    }
    if (rmax <= kCellRings) return true;
    if (!kFar) return false;
    brick_search<T>(g, fx, fy, fz, cx, cy, cz, lx, ly, lz, mc, vis);
    return true;
}

// Dense grids, queries inside the grid: the cell window of ring_search's phase 1 (Chebyshev
// radius kCellRings) walked by (y, z) rows instead of cells -- each row's cells within the
// bound are one contiguous point range, so a row costs one cstart round trip where the cell
// walk pays one per cell.  Rows go nearest plane first (0, -1, +1, ...), so the bound falls
// early.  Returns false when the bound still reaches past the window (the caller defers the
// query to the far pass), exactly ring_search's FAR = false contract.
template <typename Vis>
__device__ __forceinline__ bool row_window_search(const GridDesc& g, double qx, double qy, double qz, double mc,
                                                  Vis& vis) {
    constexpr int R = kCellRings;
    const double fx = cell_f<double>(g, qx, 0), fy = cell_f<double>(g, qy, 1), fz = cell_f<double>(g, qz, 2);
    const int cx = (int)floor(fx), cy = (int)floor(fy), cz = (int)floor(fz);
    const double lx = fx - cx, ly = fy - cy, lz = fz - cz;
    const double h2 = g.h * g.h, inv_h2 = 1.0 / h2;
    for (int oz = 0; oz <= 2 * R; oz++) {
        const int dz = (oz & 1) ? -((oz + 1) >> 1) : (oz >> 1);
        const int z = cz + dz;
        if (z < 0 || z >= g.n[2]) continue;
        const double gz2 = sq_gap(axis_gap<double>(z, cz, lz), mc);
        if (gz2 * h2 > vis.bound()) continue;
        for (int oy = 0; oy <= 2 * R; oy++) {
            const int dy = (oy & 1) ? -((oy + 1) >> 1) : (oy >> 1);
            const int y = cy + dy;
            if (y < 0 || y >= g.n[1]) continue;
            const double gyz2 = gz2 + sq_gap(axis_gap<double>(y, cy, ly), mc);
            const double lim = vis.bound() * inv_h2 - gyz2;  // remaining x extent^2 (cells)
            if (lim < 0.0) continue;
            int xa = cx - R, xb = cx + R;  // the whole window row while the bound is that wide
            if (lim < (double)((R + 2) * (R + 2))) {
                const double rx = sqrt(lim) * (1.0 + 1e-12) + mc;
                xa = max((int)floor(fx - rx), xa);
                xb = min((int)floor(fx + rx), xb);
            }
            xa = max(xa, 0);
            xb = min(xb, g.n[0] - 1);
            if (xa > xb) continue;
            const int64_t c = dense_id(g, xa, y, z);
            const uint32_t s = g.cstart[c], e = g.cstart[c + (xb - xa + 1)];
            if (e > s) vis.visit(s, e);
        }
    }
    // the window covers the grid: nothing lies outside it
    if (cx - R <= 0 && cx + R >= g.n[0] - 1 && cy - R <= 0 && cy + R >= g.n[1] - 1 && cz - R <= 0 &&
        cz + R >= g.n[2] - 1)
        return true;
    // every point outside the window lies at least R + dmin - mc cells away
    const double dmin = fmin(fmin(fmin(lx, 1 - lx), fmin(ly, 1 - ly)), fmin(lz, 1 - lz));
    const double rmin = (double)R + dmin - mc;
    return rmin > 0.0 && rmin * rmin * h2 > vis.bound();
}

}  // namespace pcp
