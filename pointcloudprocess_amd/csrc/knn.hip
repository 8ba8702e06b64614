// Exact fp64 neighbour queries over the uniform-grid index: the FLANN contract of
// KdTreeFLANN::nearestKSearch / radiusSearch (kd_tree.h:814-845, 863-903), the per-point
// PCA normals of calculate_feature.cpp:119-206 over kNN neighbourhoods, and the
// kd_tree_lod KdTree (kd_tree_lod/kd_tree.cpp:29-117).
//
// One lane per query.  The k best (d2, internal j) pairs live in registers (compile-time
// K, unrolled branch-free insertion) and the ring search (grid.hpp) visits cells nearest
// first, pruning with the current k-th distance.  d2 is FLANN L2_Simple<double>
// ((0 + d0^2) + d1^2) + d2^2 with contraction off (the build compiles -ffp-contract=off),
// so distances are bit-identical to the reference's and ties break on internal j exactly
// like FLANN's "first found in index order" result set after sorting.
#include <cfloat>
#include <cstdlib>
#include <climits>
#include <cmath>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

#include "grid.hpp"
#include "topk.hpp"
#include "pca.hpp"

#ifndef PCP_NORMALS_STATS
#define PCP_NORMALS_STATS 0  // profiling builds: per-phase counters of pcp_normals_knn on stderr
#endif
namespace pcp {
namespace {

constexpr int kB = 256;

// pruning margin in cell units: floor() rounding of query and point cell coordinates
__host__ __device__ inline double cell_margin64(const GridDesc& g) {
    const int nmax = g.n[0] > g.n[1] ? (g.n[0] > g.n[2] ? g.n[0] : g.n[2]) : (g.n[1] > g.n[2] ? g.n[1] : g.n[2]);
    return 1e-9 + 8e-16 * (double)nmax;
}

// Candidates of a cell are loaded PCP_KNN_BATCH (or 2 for the wide top-k) at a time before
// they are pushed, so the loads of a batch are in flight together instead of one dependent
// round trip per candidate.  Push order is unchanged (and irrelevant: (d2, j) order).
#ifndef PCP_KNN_BATCH
#define PCP_KNN_BATCH 4
#endif
#ifndef PCP_COOP_KTH_BISECT  // far pass: shared bound by counting bisection (1) or the exact k-th merge (0)
#define PCP_COOP_KTH_BISECT 1
#endif
#ifndef PCP_COOP_VISIT_BATCH  // far pass: point loads in flight per visit step
#define PCP_COOP_VISIT_BATCH 1
#endif
#ifndef PCP_TILE_MORTON  // tiled normals: queries in Morton order inside each brick (1) or index order (0)
#define PCP_TILE_MORTON 1
#endif
#ifndef PCP_T_MX  // tiled normals: keys kept per lane beyond k (the re-rank's slack)
#define PCP_T_MX 1
#endif
#ifndef PCP_T_PF  // tiled normals: the next chunk's positions loaded a chunk ahead
#define PCP_T_PF 1
#endif
#ifndef PCP_T_SB  // staged points per lane per load batch (tiled normals)
#define PCP_T_SB 4
#endif
#ifndef PCP_T_RB  // fp64 records per gather batch of the tiled normals' re-rank and PCA
#define PCP_T_RB 8
#endif
#ifndef PCP_T_WB  // window rows per batch of cell-start loads (tiled normals)
#define PCP_T_WB 5
#endif
#ifndef PCP_TILE_ROWTAB  // tiled normals: per-point row bytes in LDS (1) or binary searches of the row table (0)
#define PCP_TILE_ROWTAB 1
#endif
#ifndef PCP_TILE_LANE_DEFAULT  // tiled normals: each lane scans its own window (1) or the union box (0)
#define PCP_TILE_LANE_DEFAULT 1
#endif
#ifndef PCP_NEAR_ROWS  // normals near pass on dense grids: 1 = row walk of the cell window, 0 = cell rings
#define PCP_NEAR_ROWS 1
#endif
#ifndef PCP_COOP_FLAT  // far pass: 1 = a batch's occupied-brick rows dealt over the lanes
#define PCP_COOP_FLAT 1
#endif
#ifndef PCP_NORMALS_NEAR_DEFAULT  // tiled normals: 1 = the lane-per-query near pass before the far pass
#define PCP_NORMALS_NEAR_DEFAULT 1
#endif
#ifndef PCP_T_NOPCA  // profiling builds only: the tile skips its mean/covariance passes (planes wrong)
#define PCP_T_NOPCA 0
#endif
template <int K>
struct KnnVisitor {
    static constexpr int U = K <= 16 ? PCP_KNN_BATCH : 2;
    const double4* pts;
    double qx, qy, qz;
    TopK<K> top;
    // a known upper bound on the query's k-th d2 (the tile's: k points it already holds), or inf
    double cap = INFINITY;
    // pruning radius^2 (1e-12 covers the rounding of the cell-box bound and of d2)
    __device__ double bound() const { return fmin(top.kth(), cap) * (1.0 + 1e-12); }
    __device__ __forceinline__ void take(double d, int j) {
        if (d <= cap * (1.0 + 1e-12)) top.push(d, j);
    }
    __device__ void visit(uint32_t s, uint32_t e) {
        uint32_t t = s;
        for (; t + U <= e; t += U) {
            double4 p[U];
#pragma unroll
            for (int u = 0; u < U; u++) p[u] = pts[t + u];
#pragma unroll
            for (int u = 0; u < U; u++) take(l2_simple(qx, qy, qz, p[u]), (int)p[u].w);
        }
        for (; t < e; t++) {
            const double4 p = pts[t];
            take(l2_simple(qx, qy, qz, p), (int)p.w);
        }
    }
};

__device__ __forceinline__ const double* qptr(const double* q, size_t stride, int64_t i) {
    return (const double*)((const char*)q + (size_t)i * stride);
}

// Two-pass scheduling of the ring search (grid.hpp): the near pass (FAR = false) runs the
// cell rings only and appends queries whose bound reaches past them to `far_list`; the far
// pass (FAR = true) re-runs exactly those (or every query when far_list is null) with the
// brick-level search.  Keeps the common path's register footprint small.
struct FarList {
    int32_t* list;
    uint32_t* count;
    // optional, per entry: an upper bound on the query's exact k-th d2 (the k-th exact d2 of a
    // set of k points the earlier pass already holds), so the next pass prunes from the start
    double* ub = nullptr;
};

// Deferred queries are few but each is expensive, so the far pass gives every one its own
// wave (lane 0) to spread them over all CUs instead of packing them into a few waves.
template <bool FAR>
__device__ __forceinline__ int64_t work_count(const FarList& f, int64_t n) {
    if (FAR && f.list) return (threadIdx.x & 63) ? 0 : (int64_t)*f.count * 64;
    return n;
}
template <bool FAR>
__device__ __forceinline__ int64_t work_item(const FarList& f, int64_t w) {
    return (FAR && f.list) ? (int64_t)f.list[w >> 6] : w;
}
__device__ __forceinline__ void defer(const FarList& f, int64_t i, double ub = INFINITY) {
    const uint32_t at = atomicAdd(f.count, 1u);
    f.list[at] = (int32_t)i;
    if (f.ub) f.ub[at] = ub;
}

// K3: batch nearestKSearch.  Rows ascending by (d2, internal j), indices mapped through
// index_mapping_ (kd_tree.h:837-842); entries past min(k, size) are -1 / +inf.
template <int K, bool FAR>
__global__ __launch_bounds__(kB) void k_knn(GridDesc g, const double4* pts, const int32_t* mapping, int identity,
                                            const double* q, size_t qstride, int64_t nq, int k, int kk,
                                            double mc, int32_t* oidx, double* od2, FarList far) {
    const int64_t nw = work_count<FAR>(far, nq);
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = work_item<FAR>(far, w);
        const double* qp = qptr(q, qstride, i);
        KnnVisitor<K> v;
        v.pts = pts;
        v.qx = qp[0]; v.qy = qp[1]; v.qz = qp[2];
        v.top.init(kk);
        if (kk > 0 && finite3(v.qx, v.qy, v.qz) &&
            !ring_search<double, KnnVisitor<K>, FAR>(g, v.qx, v.qy, v.qz, mc, v)) {
            defer(far, i);
            continue;
        }
        int32_t* ri = oidx + i * k;
        double* rd = od2 + i * k;
        v.top.for_each_ascending(kk, [&](int r, double d, int j) {
            const bool ok = j != INT_MAX;
            ri[r] = ok ? (identity ? j : mapping[j]) : -1;
            if (od2) rd[r] = ok ? d : INFINITY;
        });
        for (int r = kk; r < k; r++) {
            ri[r] = -1;
            if (od2) rd[r] = INFINITY;
        }
    }
}

// ---- the far pass, wave-cooperative: one query per wave.  The deferred queries are the few
// whose k-th neighbour lies beyond the near pass's cell rings -- isolated points, where one lane
// walking rings of bricks alone took milliseconds.  Here the cells of each Chebyshev ring (then
// the bricks of each brick ring) are dealt round-robin over the 64 lanes; every lane keeps its
// own exact top-k of what it scanned, pruned by min(own k-th, the wave's shared bound), where
// the shared bound -- the minimum over lanes of their k-th -- is an upper bound on the global
// k-th (a superset has a smaller k-th), refreshed at each ring.  Every point within the final
// global k-th distance was scanned by some lane, so merging the lanes' lists (k rounds of a
// wave-wide lexicographic argmin) gives the exact FLANN (d2, j) order.
template <int K>
struct CoopVisitor {
    const double4* pts;
    double qx, qy, qz;
    double shared = INFINITY;  // wave-uniform
    TopK<K> top;
    __device__ double bound() const { return fmin(top.kth(), shared) * (1.0 + 1e-12); }
    __device__ double ubound() const { return shared * (1.0 + 1e-12); }
    // a point beyond the wave's shared bound (an upper bound on the global k-th) cannot be in
    // the result: only the cheap compare, not the K-slot insertion (which a lane's own list,
    // empty until it has seen k points, would otherwise take for every point)
    __device__ __forceinline__ void take(double d, int j) {
        if (d <= shared * (1.0 + 1e-12)) top.push(d, j);
    }
    __device__ void visit(uint32_t s, uint32_t e) {
        constexpr int U = PCP_COOP_VISIT_BATCH;
        uint32_t t = s;
        if (U > 1) {
            for (; t + U <= e; t += U) {
                double4 p[U];
#pragma unroll
                for (int u = 0; u < U; u++) p[u] = pts[t + u];
#pragma unroll
                for (int u = 0; u < U; u++) take(l2_simple(qx, qy, qz, p[u]), (int)p[u].w);
            }
        }
        for (; t < e; t++) {
            const double4 p = pts[t];
            take(l2_simple(qx, qy, qz, p), (int)p.w);
        }
    }
};
// the exact k-th (d2, j) of the union of the lanes' lists (wave-uniform; every lane calls):
// k rounds of a wave-wide lexicographic argmin on a copy of the lists
template <int K>
__device__ double global_kth(const TopK<K>& top, int kk, int lane) {
    TopK<K> c = top;
    c.normalize(kk);
    double kth = INFINITY;
    for (int r = 0; r < kk; r++) {
        double bd = c.best_d();
        int bj = c.best_j(), bl = lane;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double od = __shfl_xor(bd, o, 64);
            const int oj = __shfl_xor(bj, o, 64), ol = __shfl_xor(bl, o, 64);
            const bool take = lex_less(od, oj, bd, bj);
            bd = take ? od : bd;
            bj = take ? oj : bj;
            bl = take ? ol : bl;
        }
        if (bj == INT_MAX) return INFINITY;  // fewer than kk points scanned
        if (lane == bl) c.pop_best();
        kth = bd;
    }
    return kth;
}

// An upper bound on the wave's exact k-th d2 within 2^-20 of it, without copying the lists:
// the smallest tau (a double whose low word is all ones) with at least kk list entries <= tau,
// by bisection on tau's high word; each step counts the entries with one compare per slot into
// a lane mask and popcounts (SALU), no cross-lane moves.  +inf when fewer than kk are finite.
template <int K>
__device__ double kth_bound(const TopK<K>& top, int kk) {
    auto count = [&](double t) {
        int c = 0;
#pragma unroll
        for (int i = 0; i < K; i++) c += __popcll(__ballot(i < kk && top.d[i] <= t));
        return c;
    };
    if (count(DBL_MAX) < kk) return INFINITY;
    uint32_t lo = 0, hi = 0x7fefffffu;  // DBL_MAX's high word
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (count(__hiloint2double((int)mid, (int)0xffffffffu)) >= kk) hi = mid;
        else lo = mid + 1;
    }
    return __hiloint2double((int)hi, (int)0xffffffffu);
}

// An upper bound on the wave's exact k-th d2, cheap enough to refresh inside a shell: the
// kk-th smallest of the lanes' own best d2 (a subset of the union, so its kk-th smallest is at
// least the union's), by a 64-lane bitonic sort; +inf until kk lanes hold a point.
template <int K>
__device__ double wave_kth_of_bests(const TopK<K>& top, int kk, int lane) {
    double x = INFINITY;
#pragma unroll
    for (int i = 0; i < K; i++)
        if (i == kk - 1) x = top.d[i];
#pragma unroll
    for (int k2 = 2; k2 <= 64; k2 <<= 1)
#pragma unroll
        for (int j = k2 >> 1; j > 0; j >>= 1) {
            const double y = __shfl_xor(x, j, 64);
            const bool up = (lane & k2) == 0, lower = (lane & j) == 0;
            x = (lower == up) ? fmin(x, y) : fmax(x, y);
        }
    return __shfl(x, kk - 1, 64);
}

// bricks per lane per batch of the far pass's shells (8 spilled the K = 32 lists to scratch:
// ~700 bytes per lane, every list update a round trip to memory)
constexpr int kCoopBB = 4;

template <int K>
__device__ void coop_search(const GridDesc& g, double mc, CoopVisitor<K>& v, int lane, int kk,
                            int* shells = nullptr, long long* tk = nullptr) {
    const double fx = cell_f<double>(g, v.qx, 0), fy = cell_f<double>(g, v.qy, 1), fz = cell_f<double>(g, v.qz, 2);
    const int cx = (int)floor(fx), cy = (int)floor(fy), cz = (int)floor(fz);
    const double lx = fx - cx, ly = fy - cy, lz = fz - cz;
    const double h2 = g.h * g.h;
    const double dmin = fmin(fmin(fmin(lx, 1 - lx), fmin(ly, 1 - ly)), fmin(lz, 1 - lz));
    int far = 0;
    far = max(far, max(cx - (g.n[0] - 1), -cx));
    far = max(far, max(cy - (g.n[1] - 1), -cy));
    far = max(far, max(cz - (g.n[2] - 1), -cz));
    const int rmax = far + max(g.n[0], max(g.n[1], g.n[2]));
    const int smax = min(rmax, kCellRings);
    // Point ranges gathered one per lane (a cell, or a row's one or two runs), then their points
    // dealt flat over the lanes -- point p to lane p % 64, its range found by a binary search of
    // the ranges' prefix in LDS -- so no lane runs a long range as a serial chain of loads while
    // the others wait.  Wave-uniform call.
    __shared__ uint32_t s_fr[kB / 64][4][64];  // per wave: the ranges' prefix, starts, lengths
    uint32_t* const f_pre = s_fr[threadIdx.x >> 6][0];
    uint32_t* const f_s1 = s_fr[threadIdx.x >> 6][1];
    uint32_t* const f_l1 = s_fr[threadIdx.x >> 6][2];
    uint32_t* const f_s2 = s_fr[threadIdx.x >> 6][3];
    constexpr int kFlatU = 2;  // points per lane in flight (4 spilled the K = 32 lists to scratch)
    auto flat_visit = [&](uint32_t s1, uint32_t l1, uint32_t s2, uint32_t l2) {
        const uint32_t cnt = l1 + l2;
        uint32_t inc = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t tv = (uint32_t)__shfl_up((int)inc, o, 64);
            if (lane >= o) inc += tv;
        }
        const uint32_t tot = (uint32_t)__shfl((int)inc, 63, 64);
        if (tot == 0) return;
        f_pre[lane] = inc - cnt;
        f_s1[lane] = s1;
        f_l1[lane] = l1;
        f_s2[lane] = s2;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t p0 = 0; p0 < tot; p0 += 64u * kFlatU) {  // wave-uniform
            uint32_t idx[kFlatU];
#pragma unroll
            for (int u = 0; u < kFlatU; u++) {
                const uint32_t pp = p0 + (uint32_t)lane + 64u * u;
                // the owner: the last lane whose prefix is <= pp (an empty lane shares its prefix
                // with the next, so the last one is the non-empty owner)
                int o = 0;
#pragma unroll
                for (int b = 32; b >= 1; b >>= 1) o += f_pre[o + b] <= pp ? b : 0;
                const uint32_t off = pp - f_pre[o], a1 = f_l1[o];
                idx[u] = pp < tot ? (off < a1 ? f_s1[o] + off : f_s2[o] + (off - a1)) : ~0u;
            }
            double4 q4[kFlatU];
#pragma unroll
            for (int u = 0; u < kFlatU; u++) q4[u] = v.pts[idx[u] != ~0u ? idx[u] : 0u];
#pragma unroll
            for (int u = 0; u < kFlatU; u++)
                if (idx[u] != ~0u) v.take(l2_simple(v.qx, v.qy, v.qz, q4[u]), (int)q4[u].w);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the next call rewrites f_*
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    uint32_t t = 0;  // the wave's cell / brick counter: item t belongs to lane t % 64
    uint32_t rs = 0, rl = 0;  // this lane's pending cell range (flushed every 64 items)
    for (int s = 0; s <= smax + 1; s++) {
        if (s > 0) {
            v.shared = fmin(v.shared, PCP_COOP_KTH_BISECT ? kth_bound<K>(v.top, kk) : global_kth<K>(v.top, kk, lane));
            const double rmin = (double)(s - 1) + dmin - mc;
            if (rmin > 0 && rmin * rmin * h2 > v.ubound()) return;
        }
        if (s > smax) break;
        const int z0 = max(cz - s, 0), z1 = min(cz + s, g.n[2] - 1);
        const int y0 = max(cy - s, 0), y1 = min(cy + s, g.n[1] - 1);
        const int x0 = max(cx - s, 0), x1 = min(cx + s, g.n[0] - 1);
        if (z0 > z1 || y0 > y1 || x0 > x1) continue;
        for (int z = z0; z <= z1; z++) {
            const bool zface = (z == cz - s) || (z == cz + s);
            const double gz2 = sq_gap(axis_gap<double>(z, cz, lz), mc);
            if (gz2 * h2 > v.ubound()) continue;
            for (int y = y0; y <= y1; y++) {
                const bool yface = zface || (y == cy - s) || (y == cy + s);
                const double gyz2 = gz2 + sq_gap(axis_gap<double>(y, cy, ly), mc);
                if (gyz2 * h2 > v.ubound()) continue;
                const int step = yface ? 1 : 2 * s;
                for (int x = yface ? x0 : cx - s; x <= x1; x += (step > 0 ? step : 1)) {
                    if (x < x0) continue;
                    const bool mine = (t & 63u) == (uint32_t)lane;
                    t++;
                    if (mine && (gyz2 + sq_gap(axis_gap<double>(x, cx, lx), mc)) * h2 <= v.bound()) {
                        uint32_t st, en;
                        if (cell_range(g, x, y, z, st, en)) {
                            rs = st;
                            rl = en - st;
                        }
                    }
                    if ((t & 63u) == 0u) {  // (uniform) a chunk of 64 cells: its points, flat
                        flat_visit(rs, rl, 0u, 0u);
                        rl = 0u;
                    }
                }
            }
        }
        flat_visit(rs, rl, 0u, 0u);  // the ring's last partial chunk
        rl = 0u;
    }
    if (rmax <= kCellRings) return;
    // bricks of 4x4x4 cells, rings outward, the cells phase 1 covered skipped
    const int bx = cx >> 2, by = cy >> 2, bz = cz >> 2;
    const double ox = fx - 4 * bx, oy = fy - 4 * by, oz = fz - 4 * bz;
    const double bdmin = fmin(fmin(fmin(ox, 4 - ox), fmin(oy, 4 - oy)), fmin(oz, 4 - oz));
    int farb = 0;
    farb = max(farb, max(bx - (g.nb[0] - 1), -bx));
    farb = max(farb, max(by - (g.nb[1] - 1), -by));
    farb = max(farb, max(bz - (g.nb[2] - 1), -bz));
    const int sbmax = farb + max(g.nb[0], max(g.nb[1], g.nb[2]));
#if PCP_COOP_FLAT
    __shared__ int4 s_flat[kB / 64][64 * kCoopBB];  // per wave: a batch's occupied bricks {x, y, z, word}
    __shared__ uint16_t s_rows[kB / 64][64 * kCoopBB * 16];  // per wave: their non-empty rows (brick << 4 | row)
    int4* const flat = s_flat[threadIdx.x >> 6];
    uint16_t* const rows = s_rows[threadIdx.x >> 6];
#endif
    // rings closer than `farb` lie wholly outside the grid (a query far away from it)
    if (tk) tk[0] = clock64();
    for (int sb = farb; sb <= sbmax; sb++) {
        if (shells) (*shells)++;
        const long long c0 = tk ? (long long)clock64() : 0;
        v.shared = fmin(v.shared, PCP_COOP_KTH_BISECT ? kth_bound<K>(v.top, kk) : global_kth<K>(v.top, kk, lane));
        if (tk) tk[1] += (long long)clock64() - c0;
        if (sb > 0) {
            const double rmin = (double)(4 * (sb - 1)) + bdmin - mc;
            if (rmin > 0 && rmin * rmin * h2 > v.ubound()) return;
        }
        // the shell's bricks inside the grid: two z-faces, two y-faces (z strictly inside), two
        // x-faces (y and z strictly inside), each a rectangle clipped to the grid; brick t of the
        // shell goes to lane t % 64
        const int X0 = max(bx - sb, 0), X1 = min(bx + sb, g.nb[0] - 1);
        const int Y0 = max(by - sb, 0), Y1 = min(by + sb, g.nb[1] - 1);
        const int Z0 = max(bz - sb, 0), Z1 = min(bz + sb, g.nb[2] - 1);
        if (X0 > X1 || Y0 > Y1 || Z0 > Z1) continue;
        const int Yi0 = max(by - sb + 1, 0), Yi1 = min(by + sb - 1, g.nb[1] - 1);
        const int Zi0 = max(bz - sb + 1, 0), Zi1 = min(bz + sb - 1, g.nb[2] - 1);
        int64_t area[6];
        int fixc[6];
        const int nx = X1 - X0 + 1, ny = Y1 - Y0 + 1, nyi = max(Yi1 - Yi0 + 1, 0), nzi = max(Zi1 - Zi0 + 1, 0);
        for (int f = 0; f < 6; f++) {
            const int sgn = (f & 1) ? 1 : -1;
            if (f < 2) {  // z = bz -+ sb
                fixc[f] = bz + sgn * sb;
                area[f] = (fixc[f] >= 0 && fixc[f] < g.nb[2] && (sb > 0 || f == 0)) ? (int64_t)nx * ny : 0;
            } else if (f < 4) {  // y = by -+ sb, z inside
                fixc[f] = by + sgn * sb;
                area[f] = (sb > 0 && fixc[f] >= 0 && fixc[f] < g.nb[1]) ? (int64_t)nx * nzi : 0;
            } else {  // x = bx -+ sb, y and z inside
                fixc[f] = bx + sgn * sb;
                area[f] = (sb > 0 && fixc[f] >= 0 && fixc[f] < g.nb[0]) ? (int64_t)nyi * nzi : 0;
            }
        }
        const int64_t total = area[0] + area[1] + area[2] + area[3] + area[4] + area[5];
        // bricks t = lane + 64 u: the occupancy words of a batch are loaded together (mostly
        // empty bricks around isolated queries: one dependent load each would serialise)
        constexpr int kBB = kCoopBB;
        for (int64_t base = 0; base < total; base += 64 * kBB) {  // wave-uniform trip count
            const long long cb0 = tk ? (long long)clock64() : 0;
            const int64_t t0 = base + lane;
            int bxs[kBB], bys[kBB], bzs[kBB];
            int32_t occ[kBB];
#if PCP_COOP_FLAT
            uint32_t msk[kBB], bat[kBB];  // row masks and flat[] positions of this lane's bricks
#endif
#pragma unroll
            for (int u = 0; u < kBB; u++) {
                const int64_t t = t0 + 64 * u;
                int xb = 0, yb = 0, zb = 0;
                bool live = t < total;
                if (live) {
                    int f = 0;
                    int64_t r = t;
                    while (r >= area[f]) { r -= area[f]; f++; }
                    if (f < 2) {
                        xb = X0 + (int)(r % nx); yb = Y0 + (int)(r / nx); zb = fixc[f];
                    } else if (f < 4) {
                        xb = X0 + (int)(r % nx); zb = Zi0 + (int)(r / nx); yb = fixc[f];
                    } else {
                        yb = Yi0 + (int)(r % nyi); zb = Zi0 + (int)(r / nyi); xb = fixc[f];
                    }
                    const double gz = zb < bz ? (oz + 4.0 * (bz - zb - 1)) : (zb > bz ? (4.0 - oz + 4.0 * (zb - bz - 1)) : 0.0);
                    const double gy = yb < by ? (oy + 4.0 * (by - yb - 1)) : (yb > by ? (4.0 - oy + 4.0 * (yb - by - 1)) : 0.0);
                    const double gx = xb < bx ? (ox + 4.0 * (bx - xb - 1)) : (xb > bx ? (4.0 - ox + 4.0 * (xb - bx - 1)) : 0.0);
                    live = (sq_gap(gz, mc) + sq_gap(gy, mc) + sq_gap(gx, mc)) * h2 <= v.bound();
                }
                bxs[u] = xb; bys[u] = yb; bzs[u] = zb;
                occ[u] = live ? g.brick[((int64_t)zb * g.nb[1] + yb) * g.nb[0] + xb] : -1;
            }
            const long long cb1 = tk ? (long long)clock64() : 0;
            if (tk) tk[2] += cb1 - cb0;  // brick coordinates, pruning and occupancy loads
#if PCP_COOP_FLAT
            // The batch's occupied bricks are listed in LDS, then their rows that hold points
            // (the brick word's row mask on dense fp64 grids; all 16 rows otherwise) as one flat
            // item list dealt round-robin over the lanes: every lane's round is one row's
            // cstart round trip, and empty rows cost none.
            uint32_t nocc = 0, nrow = 0;
            uint32_t myrows = 0;
#pragma unroll
            for (int u = 0; u < kBB; u++) {
                const uint64_t m = __ballot(occ[u] >= 0);
                if (occ[u] >= 0) {
                    const uint32_t at = nocc + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    flat[at] = make_int4(bxs[u], bys[u], bzs[u], occ[u]);
                    bat[u] = at;
                    const uint32_t rm = (g.dense && occ[u] > 0) ? (uint32_t)occ[u] & 0xffffu : 0xffffu;
                    msk[u] = rm;
                    myrows += (uint32_t)__popc(rm);
                } else {
                    msk[u] = 0u;
                }
                nocc += (uint32_t)__popcll(m);
            }
            // exclusive scan of the lanes' row counts -> this lane's first row slot
            uint32_t incl = myrows;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t tv = (uint32_t)__shfl_up((int)incl, o, 64);
                if (lane >= o) incl += tv;
            }
            nrow = (uint32_t)__shfl((int)incl, 63, 64);
            uint32_t slot = incl - myrows;
#pragma unroll
            for (int u = 0; u < kBB; u++) {
                uint32_t rm = msk[u];
                while (rm) {
                    const uint32_t r = (uint32_t)__builtin_ctz(rm);
                    rm &= rm - 1u;
                    rows[slot++] = (uint16_t)((bat[u] << 4) | r);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // Rows in chunks of 64, one per lane: the lane resolves its row to at most two point
            // ranges (one cstart round trip for the whole chunk), then the chunk's points are
            // dealt flat over the lanes -- point p to lane p % 64, its range found by a binary
            // search of the ranges' prefix in LDS -- so a long row no longer runs as one lane's
            // serial chain of loads while the others wait.
            for (uint32_t r0 = 0; r0 < nrow; r0 += 64) {
                const uint32_t ir = r0 + (uint32_t)lane;
                uint32_t s1 = 0, l1 = 0, s2 = 0, l2 = 0;
                do {
                    if (ir >= nrow) break;
                    const uint32_t it = rows[ir];
                    const int4 bk = flat[it >> 4];
                    const int y = 4 * bk.y + (int)(it & 3), z = 4 * bk.z + (int)((it >> 2) & 3);
                    if (y >= g.n[1] || z >= g.n[2]) break;
                    const double cyz2 = sq_gap(axis_gap<double>(z, cz, lz), mc) + sq_gap(axis_gap<double>(y, cy, ly), mc);
                    if (cyz2 * h2 > v.bound()) break;
                    const bool yzin = abs(z - cz) <= kCellRings && abs(y - cy) <= kCellRings;
                    int xa = 4 * bk.x, xe = min(4 * bk.x + 3, g.n[0] - 1);
                    while (xa <= xe && (cyz2 + sq_gap(axis_gap<double>(xa, cx, lx), mc)) * h2 > v.bound()) xa++;
                    while (xe >= xa && (cyz2 + sq_gap(axis_gap<double>(xe, cx, lx), mc)) * h2 > v.bound()) xe--;
                    if (xa > xe) break;
                    const int64_t rb = g.dense ? dense_id(g, 0, y, z) : (int64_t)bk.w * 64 + local_of(0, y, z);
                    auto range = [&](int x0, int x1, uint32_t& st, uint32_t& len) {  // cells [x0, x1]
                        if (x0 > x1) return;
                        const int64_t c0 = g.dense ? rb + x0 : rb + (x0 & 3);
                        st = g.cstart[c0];
                        len = g.cstart[c0 + (x1 - x0) + 1] - st;
                    };
                    if (yzin) {
                        range(xa, min(xe, cx - kCellRings - 1), s1, l1);
                        range(max(xa, cx + kCellRings + 1), xe, s2, l2);
                    } else {
                        range(xa, xe, s1, l1);
                    }
                } while (false);
                flat_visit(s1, l1, s2, l2);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the next batch rewrites flat[]
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#else
#pragma unroll 1
            for (int u = 0; u < kBB; u++) {
                if (occ[u] < 0) continue;  // empty or pruned brick
                const int xb = bxs[u], yb = bys[u], zb = bzs[u];
                // the brick's rows of 4 cells are contiguous point ranges (x fastest, dense or
                // brick-slot layout): one range per row run instead of one per cell
                const int xc0 = 4 * xb, xc1 = min(4 * xb + 3, g.n[0] - 1);
                const int64_t rowbase = g.dense ? 0 : (int64_t)occ[u] * 64;
                for (int z = 4 * zb; z < min(4 * zb + 4, g.n[2]); z++) {
                    const double cz2 = sq_gap(axis_gap<double>(z, cz, lz), mc);
                    const bool zin = abs(z - cz) <= kCellRings;
                    for (int y = 4 * yb; y < min(4 * yb + 4, g.n[1]); y++) {
                        const double cyz2 = cz2 + sq_gap(axis_gap<double>(y, cy, ly), mc);
                        if (cyz2 * h2 > v.bound()) continue;
                        const bool yzin = zin && abs(y - cy) <= kCellRings;
                        // cells within the bound form an interval around cx; phase 1's cells
                        // (|x - cx| <= kCellRings on this row) are cut out of it
                        int xa = xc0, xe = xc1;
                        while (xa <= xe && (cyz2 + sq_gap(axis_gap<double>(xa, cx, lx), mc)) * h2 > v.bound()) xa++;
                        while (xe >= xa && (cyz2 + sq_gap(axis_gap<double>(xe, cx, lx), mc)) * h2 > v.bound()) xe--;
                        if (xa > xe) continue;
                        const int64_t r0 = g.dense ? dense_id(g, 0, y, z) : rowbase + local_of(0, y, z);
                        auto run = [&](int x0, int x1) {  // cells [x0, x1] of this row
                            if (x0 > x1) return;
                            const int64_t c0 = g.dense ? r0 + x0 : r0 + (x0 & 3);
                            const uint32_t st = g.cstart[c0], en = g.cstart[c0 + (x1 - x0) + 1];
                            if (en > st) v.visit(st, en);
                        };
                        if (yzin) {
                            run(xa, min(xe, cx - kCellRings - 1));
                            run(max(xa, cx + kCellRings + 1), xe);
                        } else {
                            run(xa, xe);
                        }
                    }
                }
            }
#endif
            const long long cb2 = tk ? (long long)clock64() : 0;
            if (tk) tk[3] += cb2 - cb1;  // the occupied bricks' rows and points
            // tighten the shared bound mid-shell (the exact k-th is refreshed per shell)
            if (kk <= 64) v.shared = fmin(v.shared, wave_kth_of_bests<K>(v.top, kk, lane));
            if (tk) tk[4] += (long long)clock64() - cb2;
        }
    }
}

// merge the lanes' top-k lists: round r leaves the r-th (d2, j) of the query in lane r's
// (md, mj) (r < kk); every lane must call it
template <int K>
__device__ __forceinline__ void coop_merge(CoopVisitor<K>& v, int kk, int lane, double& md, int& mj) {
    v.top.normalize(kk);
    md = INFINITY;
    mj = INT_MAX;
    for (int r = 0; r < kk; r++) {
        double bd = v.top.best_d();
        int bj = v.top.best_j(), bl = lane;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double od = __shfl_xor(bd, o, 64);
            const int oj = __shfl_xor(bj, o, 64), ol = __shfl_xor(bl, o, 64);
            const bool take = lex_less(od, oj, bd, bj);
            bd = take ? od : bd;
            bj = take ? oj : bj;
            bl = take ? ol : bl;
        }
        if (lane == bl && bj != INT_MAX) v.top.pop_best();
        if (lane == r) { md = bd; mj = bj; }
    }
}

template <int K>
__global__ __launch_bounds__(kB) void k_knn_coop(GridDesc g, const double4* pts, const int32_t* mapping, int identity,
                                                 const double* q, size_t qstride, int k, int kk, double mc,
                                                 int32_t* oidx, double* od2, FarList far) {
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64), cnt = *far.count;
    for (int64_t w = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6); w < cnt; w += nwaves) {
        const int64_t i = far.list[w];
        const double* qp = qptr(q, qstride, i);
        CoopVisitor<K> v;
        v.pts = pts;
        v.qx = qp[0]; v.qy = qp[1]; v.qz = qp[2];
        v.top.init(kk);
        coop_search<K>(g, mc, v, lane, kk);
        double md;
        int mj;
        coop_merge<K>(v, kk, lane, md, mj);
        if (lane < k) {
            const bool ok = lane < kk && mj != INT_MAX;
            oidx[i * k + lane] = ok ? (identity ? mj : mapping[mj]) : -1;
            if (od2) od2[i * k + lane] = ok ? md : INFINITY;
        }
    }
}

template <int K>
__global__ __launch_bounds__(kB, 2) void k_normals_coop(GridDesc g, const double4* pts, const int32_t* mapping,
                                                     int identity, const int32_t* pos_of_j, int kk, double mc,
                                                     pcp_plane* out, int64_t n_out, FarList far,
                                                     unsigned long long* dbg = nullptr) {
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64), cnt = *far.count;
    for (int64_t w = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6); w < cnt; w += nwaves) {
        const int64_t s = far.list[w];
        const double4 qp = pts[s];
        CoopVisitor<K> v;
        v.pts = pts;
        v.qx = qp.x; v.qy = qp.y; v.qz = qp.z;
        v.top.init(kk);
        if (far.ub) v.shared = far.ub[w];  // the earlier passes' k-th: pruning from the first ring
        int shells = 0;
        const long long t0 = dbg ? (long long)clock64() : 0;
        long long tk[5] = {t0, 0, 0, 0, 0};
        coop_search<K>(g, mc, v, lane, kk, dbg ? &shells : nullptr, dbg ? tk : nullptr);
        if (dbg && lane == 0) {  // PCP_KNN_DEBUG: shells walked and cycles per deferred query
            const unsigned long long dt = (unsigned long long)((long long)clock64() - t0);
            atomicAdd(dbg + 0, 1ull);
            atomicAdd(dbg + 1, (unsigned long long)shells);
            atomicMax(dbg + 2, (unsigned long long)shells);
            atomicAdd(dbg + 3, dt);
            atomicMax(dbg + 4, dt);
            atomicAdd(dbg + 9, (unsigned long long)(tk[0] - t0));  // ring phase
            atomicAdd(dbg + 10, (unsigned long long)tk[1]);        // global_kth in the shells
            if (dt >= dbg[4]) {  // the slowest query's coordinates and phases (racy, debugging only)
                dbg[11] = (unsigned long long)(tk[0] - t0);
                dbg[12] = (unsigned long long)tk[1];
                dbg[13] = (unsigned long long)tk[2];
                dbg[14] = (unsigned long long)tk[3];
                dbg[15] = (unsigned long long)tk[4];
                dbg[5] = (unsigned long long)__double_as_longlong(qp.x);
                dbg[6] = (unsigned long long)__double_as_longlong(qp.y);
                dbg[7] = (unsigned long long)__double_as_longlong(qp.z);
                dbg[8] = (unsigned long long)__double_as_longlong(v.shared);
            }
        }
        double md;
        int mj;
        coop_merge<K>(v, kk, lane, md, mj);
        const int jq = (int)qp.w;
        const int64_t oi = identity ? jq : mapping[jq];
        if (oi >= n_out) continue;
        // mean and X X^T, sequential in kNN order (calculate_feature.cpp:131-164), wave-uniform;
        // lane r fetches the r-th neighbour once (all loads in flight together), the sums then
        // walk the lanes in order through shuffles
        double4 pr = make_double4(0.0, 0.0, 0.0, 0.0);
        if (lane < kk && mj != INT_MAX) pr = pts[pos_of_j[mj]];
        double xa = 0, ya = 0, za = 0;
        for (int r = 0; r < kk; r++) {
            xa += __shfl(pr.x, r, 64); ya += __shfl(pr.y, r, 64); za += __shfl(pr.z, r, 64);
        }
        xa /= kk; ya /= kk; za /= kk;
        double c00 = 0, c01 = 0, c02 = 0, c11 = 0, c12 = 0, c22 = 0;
        for (int r = 0; r < kk; r++) {
            const double4 p = make_double4(__shfl(pr.x, r, 64), __shfl(pr.y, r, 64), __shfl(pr.z, r, 64), 0.0);
            const double x0 = p.x - xa, x1 = p.y - ya, x2 = p.z - za;
            c00 += x0 * x0; c01 += x0 * x1; c02 += x0 * x2;
            c11 += x1 * x1; c12 += x1 * x2; c22 += x2 * x2;
        }
        if (lane == 0) {
            const double C[9] = {c00, c01, c02, c01, c11, c12, c02, c12, c22};
            pcp_plane pl;
            plane_from_cov(C, xa, ya, za, pl);
            out[oi] = pl;
        }
    }
}

// K4 count pass: #points with d2 < r2 (strict, FLANN RadiusResultSet), truncated to max_nn
struct CountVisitor {
    const double4* pts;
    double qx, qy, qz, r2, b;
    uint32_t cnt;
    __device__ double bound() const { return b; }
    __device__ void visit(uint32_t s, uint32_t e) {
        uint32_t t = s;
        for (; t + 4 <= e; t += 4) {
            const double4 p0 = pts[t], p1 = pts[t + 1], p2 = pts[t + 2], p3 = pts[t + 3];
            cnt += (l2_simple(qx, qy, qz, p0) < r2 ? 1u : 0u) + (l2_simple(qx, qy, qz, p1) < r2 ? 1u : 0u) +
                   (l2_simple(qx, qy, qz, p2) < r2 ? 1u : 0u) + (l2_simple(qx, qy, qz, p3) < r2 ? 1u : 0u);
        }
        for (; t < e; t++) cnt += l2_simple(qx, qy, qz, pts[t]) < r2 ? 1u : 0u;
    }
};

template <bool FAR>
__global__ __launch_bounds__(kB) void k_radius_count(GridDesc g, const double4* pts, const double* q, size_t qstride,
                                                     int64_t nq, double r2, uint32_t cap, double mc, int32_t* ocnt,
                                                     FarList far) {
    const int64_t nw = work_count<FAR>(far, nq);
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = work_item<FAR>(far, w);
        const double* qp = qptr(q, qstride, i);
        CountVisitor v{pts, qp[0], qp[1], qp[2], r2, r2 * (1.0 + 1e-12), 0u};
        if (finite3(v.qx, v.qy, v.qz) && !ring_search<double, CountVisitor, FAR>(g, v.qx, v.qy, v.qz, mc, v)) {
            defer(far, i);
            continue;
        }
        ocnt[i] = (int32_t)(v.cnt < cap ? v.cnt : cap);
    }
}

// K4 fill pass.  A row that max_nn does not truncate (m < cap) receives its points in
// visiting order (k_sort_rows orders it afterwards); a possibly truncated row (m == cap)
// keeps the m best found so far sorted by (d2, j) by insertion.
struct FillVisitor {
    const double4* pts;
    double qx, qy, qz, r2, b;
    int32_t* ri;
    double* rd;
    int64_t m, filled;
    bool append;
    __device__ double bound() const { return b; }
    __device__ void visit(uint32_t s, uint32_t e) {
        if (append) {  // batched loads; entries appended in visiting order
            uint32_t t = s;
            for (; t + 4 <= e; t += 4) {
                double4 p[4];
#pragma unroll
                for (int u = 0; u < 4; u++) p[u] = pts[t + u];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const double d = l2_simple(qx, qy, qz, p[u]);
                    if (d < r2 && filled < m) { rd[filled] = d; ri[filled] = (int)p[u].w; filled++; }
                }
            }
            for (; t < e; t++) {
                const double4 p = pts[t];
                const double d = l2_simple(qx, qy, qz, p);
                if (d < r2 && filled < m) { rd[filled] = d; ri[filled] = (int)p.w; filled++; }
            }
            return;
        }
        for (uint32_t t = s; t < e; t++) {
            const double4 p = pts[t];
            const double d = l2_simple(qx, qy, qz, p);
            if (!(d < r2)) continue;
            const int j = (int)p.w;
            int64_t pos;
            if (filled < m) pos = filled++;
            else if (lex_less(d, j, rd[m - 1], ri[m - 1])) pos = m - 1;
            else continue;
            while (pos > 0 && lex_less(d, j, rd[pos - 1], ri[pos - 1])) {
                rd[pos] = rd[pos - 1];
                ri[pos] = ri[pos - 1];
                pos--;
            }
            rd[pos] = d;
            ri[pos] = j;
        }
    }
};

// Orders each appended CSR row by (d2, j) and maps j -> caller index.  One wave per row:
// rows up to kSortMax elements are bitonic-sorted in the wave's LDS slice; longer rows
// (rare) are insertion-sorted by lane 0 in place.
constexpr int kSortMax = 1024;
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(256) void k_sort_rows(const int64_t* off, int64_t nq, uint32_t cap, int32_t* ri,
                                                   double* rd, const int32_t* mapping, int identity) {
    __shared__ double sd[4][kSortMax];
    __shared__ int sj[4][kSortMax];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t row = (int64_t)blockIdx.x * 4 + w; row < nq; row += nw) {
        const int64_t o = off[row], m = off[row + 1] - o;
        if (m <= 0 || (uint64_t)m >= cap) {  // empty, or an insertion-sorted (truncatable) row
            if (!identity)
                for (int64_t t = lane; t < m; t += 64) ri[o + t] = mapping[ri[o + t]];
            continue;
        }
        if (m > kSortMax) {
            if (lane == 0) {
                for (int64_t a = 1; a < m; a++) {
                    const double d = rd[o + a];
                    const int j = ri[o + a];
                    int64_t p = a;
                    while (p > 0 && lex_less(d, j, rd[o + p - 1], ri[o + p - 1])) {
                        rd[o + p] = rd[o + p - 1];
                        ri[o + p] = ri[o + p - 1];
                        p--;
                    }
                    rd[o + p] = d;
                    ri[o + p] = j;
                }
            }
            wave_lds_sync();
            if (!identity)
                for (int64_t t = lane; t < m; t += 64) ri[o + t] = mapping[ri[o + t]];
            continue;
        }
        int N = 1;
        while (N < m) N <<= 1;
        for (int t = lane; t < N; t += 64) {
            sd[w][t] = t < m ? rd[o + t] : INFINITY;
            sj[w][t] = t < m ? ri[o + t] : INT_MAX;
        }
        wave_lds_sync();
        for (int k = 2; k <= N; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int t = lane; t < N; t += 64) {
                    const int u = t ^ j;
                    if (u > t) {
                        const double a = sd[w][t], b = sd[w][u];
                        const int ja = sj[w][t], jb = sj[w][u];
                        const bool up = (t & k) == 0;
                        if (up == lex_less(b, jb, a, ja)) {
                            sd[w][t] = b; sd[w][u] = a;
                            sj[w][t] = jb; sj[w][u] = ja;
                        }
                    }
                }
                wave_lds_sync();
            }
        for (int t = lane; t < m; t += 64) {
            rd[o + t] = sd[w][t];
            ri[o + t] = identity ? sj[w][t] : mapping[sj[w][t]];
        }
        wave_lds_sync();
    }
}

template <bool FAR>
__global__ __launch_bounds__(kB) void k_radius_fill(GridDesc g, const double4* pts, const double* q, size_t qstride,
                                                    int64_t nq, double r2, uint32_t cap, double mc,
                                                    const int64_t* off, int32_t* oidx, double* od2, FarList far) {
    const int64_t nw = work_count<FAR>(far, nq);
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = work_item<FAR>(far, w);
        const int64_t o = off[i], m = off[i + 1] - o;
        if (m <= 0) continue;
        const double* qp = qptr(q, qstride, i);
        FillVisitor v{pts, qp[0], qp[1], qp[2], r2, r2 * (1.0 + 1e-12), oidx + o, od2 + o, m, 0,
                      (uint64_t)m < cap};
        if (!ring_search<double, FillVisitor, FAR>(g, v.qx, v.qy, v.qz, mc, v))
            defer(far, i);  // the far pass rebuilds the row from scratch
    }
}

// F1 PCA core (eigen_sym3, plane_from_cov): pca.hpp

__global__ void k_plane_default(pcp_plane* out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = pcp_plane{0.f, 0.f, 0.f, 0.f, 1.f, 0.f};  // rpca's N <= 3 branch (:353-361)
}

// queries = the indexed points themselves, walked in the index's spatial order
// `in` (near pass only): the sorted positions to process (the tiled kernel's uncertified
// queries), or every point when in.list is null
// ROWS (the near pass over the tiled kernel's uncertified queries): the row walk below; its
// own instantiation, so the all-points ring path does not carry its registers
template <int K, bool FAR, bool ROWS = false>
__global__ __launch_bounds__(kB) void k_normals(GridDesc g, const double4* pts, const int32_t* mapping, int identity,
                                                const int32_t* pos_of_j, int64_t n, int kk, double mc,
                                                pcp_plane* out, int64_t n_out, FarList far,
                                                FarList in = FarList{nullptr, nullptr}) {
    const int64_t nw = (!FAR && in.list) ? (int64_t)*in.count : work_count<FAR>(far, n);
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = (!FAR && in.list) ? (int64_t)in.list[w] : work_item<FAR>(far, w);
        const double4 qp = pts[s];
        KnnVisitor<K> v;
        v.pts = pts;
        v.qx = qp.x; v.qy = qp.y; v.qz = qp.z;
        v.top.init(kk);
        // the tile's k-th: its kk points lie within its window (+-2 cells), inside this pass's
        // window, so the walk below still finds kk points under the cap
        if (ROWS && !FAR && in.ub) v.cap = in.ub[w];
        // the near pass over the tiled kernel's uncertified queries, on dense grids, walks the
        // window by rows (the queries are indexed points, so they lie inside the grid).  Not for
        // every point: a large k over a dense neighbourhood fills its list faster cell by cell
        // (measured: k = 32 over all 8.86M C3 points 32.7 -> 67.0 ms by rows; the tile's 10.9K
        // uncertified rows 0.3 ms faster, k = 8 0.3 ms)
        const bool done = (ROWS && !FAR && g.dense)
                              ? row_window_search<KnnVisitor<K>>(g, v.qx, v.qy, v.qz, mc, v)
                              : ring_search<double, KnnVisitor<K>, FAR>(g, v.qx, v.qy, v.qz, mc, v);
        if (!done) {
            // the tile's bound or the window's own k-th, whichever is smaller
            defer(far, s, fmin((!FAR && in.ub) ? in.ub[w] : INFINITY, v.top.kth()));
            continue;
        }
        const int jq = (int)qp.w;
        const int64_t oi = identity ? jq : mapping[jq];
        if (oi >= n_out) continue;
        // mean, sequential in kNN order (:131-142)
        double xa = 0, ya = 0, za = 0;
        v.top.for_each_ascending(kk, [&](int, double, int j) {
            const double4 p = pts[pos_of_j[j]];
            xa += p.x; ya += p.y; za += p.z;
        });
        xa /= kk; ya /= kk; za /= kk;
        double c00 = 0, c01 = 0, c02 = 0, c11 = 0, c12 = 0, c22 = 0;
        v.top.for_each_ascending(kk, [&](int, double, int j) {
            const double4 p = pts[pos_of_j[j]];
            const double x0 = p.x - xa, x1 = p.y - ya, x2 = p.z - za;
            c00 += x0 * x0; c01 += x0 * x1; c02 += x0 * x2;
            c11 += x1 * x1; c12 += x1 * x2; c22 += x2 * x2;
        });
        const double C[9] = {c00, c01, c02, c01, c11, c12, c02, c12, c22};
        pcp_plane pl;
        plane_from_cov(C, xa, ya, za, pl);
        out[oi] = pl;
    }
}

// F1 over kNN, tiled (dense grids, k <= 32): one wave per 64 consecutive sorted points.
// The wave copies the union of its queries' neighbourhoods -- the box of their cells grown by
// R cells, one contiguous point run per (y, z) row -- into LDS as fp32 coordinates relative to
// the box corner plus the sorted position.  Every lane then scans the whole list (uniform trip
// count, broadcast LDS reads, no divergence) keeping its M = K + PCP_T_MX (1) smallest packed keys
// (bits(fp32 d2) & ~1023 | list index) and the (M+1)-th as a bound with a v_med3_u32 network
// (M + 1 VALU ops per candidate instead of the fp64 register top-k's divergent shifts).  The
// kept candidates are re-ranked by the exact FLANN fp64 (d2, j) and sorted; the lane's result
// is certified when its k-th exact d2 lies strictly below both the bound on every uncached
// list point (the (M+1)-th key less the fp32 error) and the squared distance to the box faces
// (points outside the box).  Uncertified lanes go to the exact two-level search (the far pass
// of k_normals), so the output is that of the exact path bit for bit.
constexpr int kTileCap = 2048;   // union points per wave (11-bit list index)
constexpr int kTileRows = 255;   // (y, z) rows per wave (255: the wave's LDS fits 8 waves per CU)
constexpr int kTileQ = 16383;    // 14-bit fixed-point coordinates: squared distances fit in int32
constexpr int kTileExt = 96;     // box extent (cells) cap: keeps the fixed-point step fine
constexpr int kLaneR = 2;        // largest window half-width of the per-lane window scan
// (dy, dz) of row i of a 5 x 5 (y, z) window, rows by squared distance (the first 9 are the 3 x 3
// window): (dy + 2) | (dz + 2) << 3 in 6-bit fields, 10 to a word (i is wave-uniform: scalar ops)
__device__ __forceinline__ void window_row(int i, int& dy, int& dz) {
    const uint64_t w = i < 10 ? 0x50964b6ca6914d2ull : (i < 20 ? 0x8438c860c702890ull : 0x804901ull);
    const uint32_t v = (uint32_t)(w >> (6 * (i % 10))) & 63u;
    dy = (int)(v & 7u) - 2;
    dz = (int)(v >> 3) - 2;
}
__device__ __forceinline__ uint32_t umed3_(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// squared distance of two packed 14-bit points: (x | y << 16, z) -- v_pk_sub_i16 + v_dot2_i32_i16
__device__ __forceinline__ uint32_t qd2(uint32_t qxy, int qz, uint32_t pxy, int pz) {
    uint32_t dxy;
    asm("v_pk_sub_i16 %0, %1, %2" : "=v"(dxy) : "v"(qxy), "v"(pxy));
    const int dz = qz - pz;
    int r;
    asm("v_dot2_i32_i16 %0, %1, %1, %2" : "=v"(r) : "v"(dxy), "v"(__mul24(dz, dz)));  // |dz| < 2^14: v_mul_i32_i24, full rate
    return (uint32_t)r;
}
__device__ __forceinline__ int wmin_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wmax_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// keeps a loaded value live on every lane: a load whose result is only used under a per-lane
// condition is otherwise sunk into a branch with its own wait, one round trip per load
__device__ __forceinline__ void pin(uint32_t& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(double& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ int quant14(double v, double inv) {
    const double t = rint(v * inv);
    return (int)(t < 0.0 ? 0.0 : (t > (double)kTileQ ? (double)kTileQ : t));
}

// the union box of the lanes with `in` set, grown by R cells; its rows' point runs are listed
// (start and exclusive prefix in s_rs / s_rb) when `write` is set
struct TileBox {
    int x0, x1, y0, y1, z0, z1, ny, nrow;
    uint32_t total;  // points in the box (0xffffffff: too many rows / too wide)
};
__device__ __forceinline__ TileBox tile_box(const GridDesc& g, int cx, int cy, int cz, bool in, int R, int lane,
                                            uint32_t* s_rs, uint32_t* s_rb, bool write) {
    TileBox b;
    b.x0 = max(wmin_i(in ? cx : INT_MAX) - R, 0), b.x1 = min(wmax_i(in ? cx : INT_MIN) + R, g.n[0] - 1);
    b.y0 = max(wmin_i(in ? cy : INT_MAX) - R, 0), b.y1 = min(wmax_i(in ? cy : INT_MIN) + R, g.n[1] - 1);
    b.z0 = max(wmin_i(in ? cz : INT_MAX) - R, 0), b.z1 = min(wmax_i(in ? cz : INT_MIN) + R, g.n[2] - 1);
    b.ny = b.y1 - b.y0 + 1;
    b.nrow = b.ny * (b.z1 - b.z0 + 1);
    b.total = 0xffffffffu;
    const int ext = max(max(b.x1 - b.x0, b.y1 - b.y0), b.z1 - b.z0) + 1;
    if (b.nrow > kTileRows || ext > kTileExt) return b;
    // every row's cell starts first (unconditional loads of a clamped row: one round trip for
    // the whole box), then the prefix sums
    constexpr int kRowIt = (kTileRows + 63) / 64;
    uint32_t st_[kRowIt], en_[kRowIt];
#pragma unroll
    for (int it = 0; it < kRowIt; it++) {
        const int r = it * 64 + lane;
        const int rc = r < b.nrow ? r : 0;
        const int y = b.y0 + rc % b.ny, z = b.z0 + rc / b.ny;
        st_[it] = g.cstart[dense_id(g, b.x0, y, z)];
        en_[it] = g.cstart[dense_id(g, b.x1, y, z) + 1];
    }
#pragma unroll
    for (int it = 0; it < kRowIt; it++) pin(st_[it]), pin(en_[it]);
    uint32_t carry = 0;
#pragma unroll
    for (int it = 0; it < kRowIt; it++) {
        const int r0 = it * 64;
        if (r0 >= b.nrow) break;
        const int r = r0 + lane;
        const uint32_t st = r < b.nrow ? st_[it] : 0u;
        const uint32_t cnt = r < b.nrow ? en_[it] - st_[it] : 0u;
        uint32_t inc = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(inc, o, 64);
            if (lane >= o) inc += t;
        }
        if (write && r < b.nrow) {
            s_rs[r] = st;
            s_rb[r] = carry + inc - cnt;
        }
        carry += __shfl(inc, 63, 64);
    }
    if (write && lane == 0) s_rb[b.nrow] = carry;
    b.total = carry;
    return b;
}

// query order of the tiled kernel: sorted positions by 8x8x8-cell brick (stable, so row-major
// inside a brick), so that a wave's 64 queries are neighbours in all three axes -- in the index's
// row-major order the points of one x-row of a facade are metres apart
constexpr int kTileBrick = 3;  // log2 brick edge (cells)
// Inside a brick the key continues with `lb` bits of a Morton code of the point's position
// (cell and sub-cell: 2^(lb/3) steps per brick edge), so a wave's 64 queries form a compact
// patch instead of a run along one x-row of cells (lb = 0: index order inside the brick).
__device__ __forceinline__ uint32_t spread3(uint32_t v) {  // bits b -> 3b
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x30000ffu;
    v = (v | (v << 8)) & 0x300f00fu;
    v = (v | (v << 4)) & 0x30c30c3u;
    v = (v | (v << 2)) & 0x9249249u;
    return v;
}
__global__ void k_brick_keys(GridDesc g, const double4* pts, int64_t n, int lb, uint32_t* key, uint32_t* pos) {
    const int nbx = (g.n[0] + 7) >> kTileBrick, nby = (g.n[1] + 7) >> kTileBrick;
    const int sub = lb / 3 - kTileBrick;  // sub-cell bits per axis (>= 0 when lb > 0)
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < n; s += (int64_t)gridDim.x * blockDim.x) {
        const double4 p = pts[s];
        const double fx = cell_f<double>(g, p.x, 0), fy = cell_f<double>(g, p.y, 1), fz = cell_f<double>(g, p.z, 2);
        const int cx = clampi((int)floor(fx), 0, g.n[0] - 1), cy = clampi((int)floor(fy), 0, g.n[1] - 1),
                  cz = clampi((int)floor(fz), 0, g.n[2] - 1);
        uint32_t k = (uint32_t)(((int64_t)(cz >> kTileBrick) * nby + (cy >> kTileBrick)) * nbx + (cx >> kTileBrick));
        if (lb > 0) {
            const double sc = (double)(1 << sub);
            auto loc = [&](double f, int c) {  // position in the brick, 2^(3 + sub) steps
                const int q = (c & ((1 << kTileBrick) - 1)) << sub;
                const int t = (int)((f - (double)c) * sc);
                return (uint32_t)(q + (t < 0 ? 0 : (t >= (1 << sub) ? (1 << sub) - 1 : t)));
            };
            k = (k << lb) | spread3(loc(fx, cx)) | (spread3(loc(fy, cy)) << 1) | (spread3(loc(fz, cz)) << 2);
        }
        key[s] = k;
        pos[s] = (uint32_t)s;
    }
}

template <int K>
__global__ __launch_bounds__(64, 2) void k_normals_tile(GridDesc g, const double4* pts, const int32_t* mapping,
                                                     int identity, int64_t n, int kk, int R, double mc,
                                                     pcp_plane* out, int64_t n_out, FarList far,
                                                     unsigned long long* stats, const uint32_t* order,
                                                     int lane_mode) {
    constexpr int M = K + PCP_T_MX;
    constexpr uint32_t kMax = 0xffffffffu;
    __shared__ uint2 s_u[kTileCap];
    __shared__ uint32_t s_rs[kTileRows], s_rb[kTileRows + 1];
#if PCP_TILE_ROWTAB
    __shared__ uint8_t s_row[kTileCap];  // the (y, z) row of each staged point
#endif
    const int lane = threadIdx.x;
#if PCP_T_PF
    // the next chunk's sorted positions are loaded a chunk ahead (the chain order -> point ->
    // cells -> rows -> staging starts one round trip shorter)
    uint32_t s_next = blockIdx.x * 64 < n ? order[min((int64_t)blockIdx.x * 64 + lane, n - 1)] : 0u;
#endif
    for (int64_t c = blockIdx.x; c * 64 < n; c += gridDim.x) {
        const bool valid = c * 64 + lane < n;
#if PCP_T_PF
        const int64_t s = s_next;  // a sorted position
        {
            const int64_t cn = c + gridDim.x;
            if (cn * 64 < n) s_next = order[min(cn * 64 + lane, n - 1)];
        }
#else
        const int64_t s = order[valid ? c * 64 + lane : c * 64];  // a sorted position
#endif
        const double4 q = pts[s];
        const int cx = cell_i<double>(g, q.x, 0), cy = cell_i<double>(g, q.y, 1), cz = cell_i<double>(g, q.z, 2);
        // Groups of lanes, each staged and scanned on its own: the whole wave when its box fits
        // the LDS list; else the runs of lanes in one query brick (the wave's queries are in
        // brick order, so a wave that crosses into a distant brick -- the next row of bricks --
        // splits there), cut to at most 16 lanes if a run still does not fit.  A group whose box
        // does not fit even then takes the exact search.
        int grp = 0, G = 1;
        bool over = false;  // this lane's group does not fit: deferred
        // the whole wave's box, listed at once (the common case: no second pass of row starts)
        wave_lds_fence();  // the previous chunk's readers are done with the lists
        const TileBox bw = tile_box(g, cx, cy, cz, valid, R, lane, s_rs, s_rb, true);
        const bool whole = bw.total <= (uint32_t)kTileCap;
        if (!whole) {
            const int nbx = (g.n[0] + 7) >> kTileBrick, nby = (g.n[1] + 7) >> kTileBrick;
            const int bxq = clampi(cx, 0, g.n[0] - 1) >> kTileBrick, byq = clampi(cy, 0, g.n[1] - 1) >> kTileBrick,
                      bzq = clampi(cz, 0, g.n[2] - 1) >> kTileBrick;
            const uint32_t bid = (uint32_t)(((int64_t)bzq * nby + byq) * nbx + bxq);
            const uint32_t prev = (uint32_t)__shfl_up((int)bid, 1, 64);
            const uint64_t below = lane == 63 ? ~0ull : ((2ull << lane) - 1);  // lanes <= this one
            const uint64_t heads = __ballot(lane == 0 || bid != prev);
            const int run = __popcll(heads & below) - 1;
            const int rstart = 63 - __clzll(heads & below);
            const int nruns = __popcll(heads);
            for (int pass = 0; pass < 2; pass++) {
                G = pass == 0 ? nruns : nruns * 4;
                grp = pass == 0 ? run : run * 4 + (lane - rstart) / 16;
                bool bad = false;
                for (int gi = 0; gi < G; gi++) {
                    const bool in = valid && grp == gi;
                    if (!__ballot(in)) continue;
                    const TileBox b = tile_box(g, cx, cy, cz, in, R, lane, s_rs, s_rb, false);
                    if (b.total > (uint32_t)kTileCap) {
                        bad = true;
                        over = over || grp == gi;
                    }
                }
                if (!bad) break;
                if (pass == 0) over = false;
            }
        }
        if (over) {  // this lane's group takes the exact search
            if (valid) defer(far, s);
            if (stats) atomicAdd(stats + 1, 1ull);
        }
        if (stats && lane == 0 && G > 1) atomicAdd(stats + 3, (unsigned long long)G);
        for (int gi = 0; gi < G; gi++) {
            const bool mine = grp == gi && !over;
            if (!__ballot(mine && valid)) continue;  // an empty or deferred group
            TileBox b = bw;
            if (!whole) {
                wave_lds_fence();  // the previous group's readers are done with the lists
                b = tile_box(g, cx, cy, cz, mine && valid, R, lane, s_rs, s_rb, true);
            }
            const uint32_t total = b.total;
            wave_lds_fence();
            // 14-bit fixed point relative to the box corner, one step for all three axes
            const double ox = g.o[0] + (double)b.x0 * g.h, oy = g.o[1] + (double)b.y0 * g.h,
                         oz = g.o[2] + (double)b.z0 * g.h;
            const int ext = max(max(b.x1 - b.x0, b.y1 - b.y0), b.z1 - b.z0) + 1;
            const double step = (double)ext * g.h / (double)kTileQ, inv = 1.0 / step;
#if !PCP_TILE_ROWTAB
            const int nrow = b.nrow;
            auto row_of = [&](uint32_t e) {
                int r = 0;
#pragma unroll
                for (int stp = (kTileRows + 1) / 2; stp > 0; stp >>= 1)
                    r = (r + stp < nrow && s_rb[r + stp] <= e) ? r + stp : r;
                return r;
            };
#endif
#if PCP_TILE_ROWTAB
            // e advances by 64 per step, so each lane's row only moves forward: a short walk
            // instead of a binary search, and the row of every staged point is kept (one byte)
            // for the re-rank's list index -> position lookups.  kSB entries per lane per step:
            // their rows first, then kSB unconditional loads (a lane past the list reads position
            // 0), so a step waits on one round trip, not kSB
            int rw = 0;
            constexpr int kSB = PCP_T_SB;
            for (uint32_t e0 = lane; e0 < total; e0 += 64 * kSB) {
                uint32_t pi[kSB];
#pragma unroll
                for (int u = 0; u < kSB; u++) {
                    const uint32_t e = e0 + 64u * u;
                    const bool on = e < total;
                    while (on && s_rb[rw + 1] <= e) rw++;
                    if (on) s_row[e] = (uint8_t)rw;
                    pi[u] = on ? s_rs[rw] + (e - s_rb[rw]) : 0u;
                }
                double px[kSB], py[kSB], pz[kSB];
#pragma unroll
                for (int u = 0; u < kSB; u++) {
                    const double4* pp = pts + pi[u];
                    px[u] = pp->x;
                    py[u] = pp->y;
                    pz[u] = pp->z;
                }
#pragma unroll
                for (int u = 0; u < kSB; u++) {
                    pin(px[u]), pin(py[u]), pin(pz[u]);
                }
#pragma unroll
                for (int u = 0; u < kSB; u++) {
                    const uint32_t e = e0 + 64u * u;
                    if (e < total)
                        s_u[e] = make_uint2((uint32_t)quant14(px[u] - ox, inv) | ((uint32_t)quant14(py[u] - oy, inv) << 16),
                                            (uint32_t)quant14(pz[u] - oz, inv));
                }
            }
#else
            for (uint32_t e = lane; e < total; e += 64) {
                const int r = row_of(e);
                const double4 p = pts[s_rs[r] + (e - s_rb[r])];
                s_u[e] = make_uint2((uint32_t)quant14(p.x - ox, inv) | ((uint32_t)quant14(p.y - oy, inv) << 16),
                                    (uint32_t)quant14(p.z - oz, inv));
            }
#endif
            wave_lds_fence();
            const uint32_t qxy = (uint32_t)quant14(q.x - ox, inv) | ((uint32_t)quant14(q.y - oy, inv) << 16);
            const int qz = quant14(q.z - oz, inv);
            uint32_t t[M + 1];
#pragma unroll
            for (int i = 0; i <= M; i++) t[i] = kMax;
            // keys: the float bits of the integer d2 (relative precision 2^-12 after the index
            // bits, whatever the step) | list index
            auto key = [&](uint32_t d, uint32_t e) {
                return (__float_as_uint((float)d) & ~(uint32_t)(kTileCap - 1)) | e;
            };
            auto insert = [&](uint32_t x) {
#pragma unroll
                for (int i = M; i >= 1; i--) t[i] = umed3_(t[i - 1], t[i], x);
                t[0] = min(t[0], x);
            };
            // Per-lane windows (lane_mode, R <= kLaneR): each lane scans only the rows of ITS OWN
            // (2R+1)^2 (y, z) window -- the x-range of its +-R cells, nearest rows first -- from
            // the staged list, instead of every point of the wave's union box (a compact patch's
            // union box holds 4-10x a lane's window).  The lanes walk their own row lists (kept in
            // LDS after the staged points) in lockstep with per-lane LDS addresses, and the
            // insertion network runs only when some lane's key is below its current (M+1)-th
            // (insertion of a larger key is a no-op on every slot).  Every window point not kept
            // has a key >= the final (M+1)-th, so the list bound below is unchanged; the box-face
            // bound becomes the lane's window faces.
            bool lane_path = false;
            const bool act = mine && valid;
            const int wx0 = max(cx - R, b.x0), wx1 = min(cx + R, b.x1);
            if (lane_mode && R <= kLaneR) {
                constexpr int kW = (2 * kLaneR + 1) * (2 * kLaneR + 1);
                const int nwin = R >= 2 ? 25 : (R == 1 ? 9 : 1);
                // the LDS run [a, e) of every window row as a | e << 16 (0: empty / outside the
                // box).  The cell-start loads of all kW rows are unconditional (cell 0 for a row
                // outside) and issued before any is used: one round trip, not one per row
                // row (dy, dz) of the window: cell (wx0, cy + dy, cz + dz) = the lane's base cell
                // plus a uniform offset (scalar: dy, dz are constants of the unrolled loop)
                const int64_t cbase = act ? dense_id(g, wx0, cy, cz) : 0;
                const int64_t sy = g.n[0], sz = (int64_t)g.n[0] * g.n[1];
                const uint32_t xw = (uint32_t)(wx1 - wx0 + 1);
                const int rbase = (cy - b.y0) + (cz - b.z0) * b.ny;
                uint32_t run[kW];
                constexpr int kWB = PCP_T_WB;  // rows per batch of cell-start loads
#pragma unroll
                for (int i0 = 0; i0 < kW; i0 += kWB) {
                    uint32_t ca[kWB], cb[kWB], okm = 0;
#pragma unroll
                    for (int u = 0; u < kWB && i0 + u < kW; u++) {
                        int dy, dz;
                        window_row(i0 + u, dy, dz);
                        const int y = cy + dy, z = cz + dz;
                        const bool ok = act && i0 + u < nwin && y >= b.y0 && y <= b.y1 && z >= b.z0 && z <= b.z1;
                        okm |= ok ? 1u << u : 0u;
                        const int64_t c0 = ok ? cbase + dy * sy + dz * sz : 0;
                        ca[u] = g.cstart[c0];
                        cb[u] = g.cstart[ok ? c0 + xw : 0];
                    }
#pragma unroll
                    for (int u = 0; u < kWB && i0 + u < kW; u++) pin(ca[u]), pin(cb[u]);
#pragma unroll
                    for (int u = 0; u < kWB && i0 + u < kW; u++) {
                        int dy, dz;
                        window_row(i0 + u, dy, dz);
                        const bool ok = (okm >> u) & 1u;
                        const int r = ok ? rbase + dy + dz * b.ny : 0;
                        const uint32_t a0 = s_rb[r] + (ca[u] - s_rs[r]);
                        run[i0 + u] = ok && cb[u] > ca[u] ? a0 | ((a0 + (cb[u] - ca[u])) << 16) : 0u;
                    }
                }
                uint32_t* s_w = reinterpret_cast<uint32_t*>(s_u);
                int nr = 0, excl = 0;
                if (2 * total + 64u * kW <= 2u * kTileCap) {
                    // room for a fixed kW-word region per lane at the end of the list (odd stride:
                    // the lanes' reads of one slot fall in distinct banks)
                    lane_path = true;
                    excl = 2 * kTileCap - 64 * kW + lane * kW;
#pragma unroll
                    for (int i = 0; i < kW; i++)
                        if (run[i]) s_w[excl + nr++] = run[i];
                } else {
#pragma unroll
                    for (int i = 0; i < kW; i++) nr += run[i] ? 1 : 0;  // this lane's non-empty rows
                    excl = nr;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const int t2 = __shfl_up(excl, o, 64);
                        if (lane >= o) excl += t2;
                    }
                    const int tot_rows = __shfl(excl, 63, 64);
                    excl -= nr;
                    lane_path = 2 * total + (uint32_t)tot_rows <= 2u * kTileCap;
                    if (lane_path) {  // compacted after the staged points
                        excl += 2 * (int)total;
                        int j = excl;
#pragma unroll
                        for (int i = 0; i < kW; i++)
                            if (run[i]) s_w[j++] = run[i];
                    }
                }
                if (lane_path) {
                    wave_lds_fence();
                    uint32_t rp = (uint32_t)excl, rend = (uint32_t)(excl + nr);
                    uint32_t e = 0, ee = 0;
                    for (;;) {
                        if (e >= ee && rp < rend) {
                            const uint32_t wr = s_w[rp++];
                            e = wr & 0xffffu;
                            ee = wr >> 16;
                        }
                        const bool on = e < ee;
                        if (__ballot(on) == 0) break;
                        const uint2 pp = s_u[on ? e : 0u];
                        const uint32_t x = on ? key(qd2(qxy, qz, pp.x, (int)pp.y), e) : kMax;
                        e += on ? 1u : 0u;
                        if (__ballot(x < t[M]) != 0) insert(x);
                    }
                    if (stats && lane == 0) atomicAdd(stats + 20, 1ull);
                }
            }
            if (!lane_path) {
                uint32_t e = 0;
                for (; e + 4 <= total; e += 4) {
                    uint2 p[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) p[u] = s_u[e + u];
#pragma unroll
                    for (int u = 0; u < 4; u++) insert(key(qd2(qxy, qz, p[u].x, (int)p[u].y), e + u));
                }
                for (; e < total; e++) {
                    const uint2 pp = s_u[e];
                    insert(key(qd2(qxy, qz, pp.x, (int)pp.y), e));
                }
                if (stats && lane == 0) atomicAdd(stats + 21, 1ull);
            }
            if (!mine) continue;  // (no wave-wide operation follows)
            // the faces of the scanned region (the box, or the lane's window) that have grid cells
            // beyond them bound every point outside the list (taken before the re-rank, so that
            // only b2 stays live across it)
            int fx0 = b.x0, fx1 = b.x1, fy0 = b.y0, fy1 = b.y1, fz0 = b.z0, fz1 = b.z1;
            if (lane_path) {
                fx0 = wx0; fx1 = wx1;
                fy0 = max(cy - R, b.y0); fy1 = min(cy + R, b.y1);
                fz0 = max(cz - R, b.z0); fz1 = min(cz + R, b.z1);
            }
            double bd = INFINITY;
            if (fx0 > 0) bd = fmin(bd, q.x - (g.o[0] + (double)fx0 * g.h));
            if (fx1 < g.n[0] - 1) bd = fmin(bd, g.o[0] + (double)(fx1 + 1) * g.h - q.x);
            if (fy0 > 0) bd = fmin(bd, q.y - (g.o[1] + (double)fy0 * g.h));
            if (fy1 < g.n[1] - 1) bd = fmin(bd, g.o[1] + (double)(fy1 + 1) * g.h - q.y);
            if (fz0 > 0) bd = fmin(bd, q.z - (g.o[2] + (double)fz0 * g.h));
            if (fz1 < g.n[2] - 1) bd = fmin(bd, g.o[2] + (double)(fz1 + 1) * g.h - q.z);
            bd -= mc * g.h + 1e-12 * (fabs(q.x) + fabs(q.y) + fabs(q.z) + 1.0);
            const double b2 = bd > 0.0 ? bd * bd * (1.0 - 1e-12) : (bd == INFINITY ? INFINITY : 0.0);
            // exact FLANN re-rank of the kept candidates.  The fp64 records are gathered in
            // batches of kRB unconditional loads (a slot without a candidate reads position 0 and
            // is discarded), so a wave waits on M / kRB round trips instead of one per candidate
            // (a load under a per-lane condition is a branch with its own wait).
            constexpr int kRB = PCP_T_RB;
            double D[M];
            uint32_t P[M];
#pragma unroll
            for (int i = 0; i < M; i++) {
                const bool has = t[i] != kMax;
                const uint32_t ei = t[i] & (uint32_t)(kTileCap - 1);
#if PCP_TILE_ROWTAB
                const int r = s_row[has ? ei : 0u];
#else
                const int r = row_of(has ? ei : 0u);
#endif
                P[i] = has ? s_rs[r] + (ei - s_rb[r]) : 0u;
            }
#pragma unroll
            for (int i0 = 0; i0 < M; i0 += kRB) {
                double px[kRB], py[kRB], pz[kRB];
#pragma unroll
                for (int u = 0; u < kRB && i0 + u < M; u++) {
                    const double4* pp = pts + P[i0 + u];
                    px[u] = pp->x;
                    py[u] = pp->y;
                    pz[u] = pp->z;
                }
#pragma unroll
                for (int u = 0; u < kRB && i0 + u < M; u++) {
                    pin(px[u]), pin(py[u]), pin(pz[u]);
                }
#pragma unroll
                for (int u = 0; u < kRB && i0 + u < M; u++)
                    D[i0 + u] = t[i0 + u] != kMax ? l2_simple(q.x, q.y, q.z, make_double4(px[u], py[u], pz[u], 0.0))
                                                  : INFINITY;
            }
            // every list point not kept: its quantised distance is >= sqrt(float(t[M] & ~2047))
            // steps (the int -> float rounding is covered by the 2^-20), and quantisation moves
            // each coordinate of both points by <= step / 2
            double lb = INFINITY;
            if (t[M] != kMax) {
                const double v =
                    (sqrt((double)__uint_as_float(t[M] & ~(uint32_t)(kTileCap - 1))) * (1.0 - 0x1p-20) -
                     1.7320508075688772 - 1e-3) * step;
                lb = v > 0.0 ? v * v * (1.0 - 1e-12) : 0.0;
            }
            // sort (d2, j) ascending: odd-even transposition rounds until no swap (the approximate
            // order is almost exact, so this ends after one or two rounds)
            bool any = true;
            while (any) {
                any = false;
#pragma unroll
                for (int par = 0; par < 2; par++) {
#pragma unroll
                    for (int i = par; i + 1 < M; i += 2) {
                        bool gt = D[i] > D[i + 1];
                        if (D[i] == D[i + 1] && D[i] != INFINITY)
                            gt = (int)pts[P[i]].w > (int)pts[P[i + 1]].w;
                        const double dl = gt ? D[i + 1] : D[i], dh = gt ? D[i] : D[i + 1];
                        const uint32_t pl = gt ? P[i + 1] : P[i], ph = gt ? P[i] : P[i + 1];
                        D[i] = dl; D[i + 1] = dh; P[i] = pl; P[i + 1] = ph;
                        any = any || gt;
                    }
                }
            }
            double dk = INFINITY;
#pragma unroll
            for (int i = 0; i < M; i++)
                if (i == kk - 1) dk = D[i];
            if (!valid) continue;
            if (!(dk < lb && dk < b2)) {
                defer(far, s, dk);  // dk: the k-th exact d2 of the kept points, an upper bound
                if (stats) atomicAdd(stats + (dk < lb ? 2 : 0), 1ull);
                continue;
            }
            const int jq = (int)q.w;
            const int64_t oi = identity ? jq : mapping[jq];
            if (oi >= n_out) continue;
#if PCP_T_NOPCA
            {
                pcp_plane pl{};
                pl.normal_x = (float)D[0]; pl.normal_y = (float)D[1]; pl.distance = (float)P[K - 1];
                out[oi] = pl;
                continue;
            }
#endif
            // mean, sequential in kNN order (calculate_feature.cpp:131-142); the records again in
            // batches of unconditional loads (P[i] is a valid position for every i)
            double xa = 0, ya = 0, za = 0;
#pragma unroll
            for (int i0 = 0; i0 < K; i0 += kRB) {
                double px[kRB], py[kRB], pz[kRB];
#pragma unroll
                for (int u = 0; u < kRB && i0 + u < K; u++) {
                    const double4* pp = pts + P[i0 + u];
                    px[u] = pp->x;
                    py[u] = pp->y;
                    pz[u] = pp->z;
                }
#pragma unroll
                for (int u = 0; u < kRB && i0 + u < K; u++) {
                    pin(px[u]), pin(py[u]), pin(pz[u]);
                }
#pragma unroll
                for (int u = 0; u < kRB && i0 + u < K; u++) {
                    if (i0 + u < kk) {
                        xa += px[u]; ya += py[u]; za += pz[u];
                    }
                }
            }
            xa /= kk; ya /= kk; za /= kk;
            double c00 = 0, c01 = 0, c02 = 0, c11 = 0, c12 = 0, c22 = 0;
#pragma unroll
            for (int i0 = 0; i0 < K; i0 += kRB) {
                double px[kRB], py[kRB], pz[kRB];
#pragma unroll
                for (int u = 0; u < kRB && i0 + u < K; u++) {
                    const double4* pp = pts + P[i0 + u];
                    px[u] = pp->x;
                    py[u] = pp->y;
                    pz[u] = pp->z;
                }
#pragma unroll
                for (int u = 0; u < kRB && i0 + u < K; u++) {
                    pin(px[u]), pin(py[u]), pin(pz[u]);
                }
#pragma unroll
                for (int u = 0; u < kRB && i0 + u < K; u++) {
                    if (i0 + u < kk) {
                        const double a0 = px[u] - xa, a1 = py[u] - ya, a2 = pz[u] - za;
                        c00 += a0 * a0; c01 += a0 * a1; c02 += a0 * a2;
                        c11 += a1 * a1; c12 += a1 * a2; c22 += a2 * a2;
                    }
                }
            }
            const double C[9] = {c00, c01, c02, c01, c11, c12, c02, c12, c22};
            pcp_plane pl;
            plane_from_cov(C, xa, ya, za, pl);
            out[oi] = pl;
        }
    }
}

// F1 batch: one plane per CSR segment, points xyz[idx[t]] (or xyz[t]) for t in
// [off[s], off[s+1]), accumulated sequentially in segment order (calculate_feature.cpp:
// 131-164) -- calculate_plan_parameter_h_points per segment, and the radius variant
// (calculate_feature.h:15, F4) when the segments are radiusSearch rows.
__global__ __launch_bounds__(kB) void k_plane_segments(const double* xyz, size_t stride, const int64_t* off,
                                                       const int32_t* idx, int64_t nseg, pcp_plane* out) {
    for (int64_t sg = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; sg < nseg;
         sg += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = off[sg], e = off[sg + 1];
        const int64_t h = e - s;
        if (h <= 0) {
            out[sg] = pcp_plane{0.f, 0.f, 0.f, 0.f, 1.f, 0.f};
            continue;
        }
        auto P = [&](int64_t t) { return qptr(xyz, stride, idx ? (int64_t)idx[t] : t); };
        double xa = 0, ya = 0, za = 0;
        for (int64_t t = s; t < e; t++) {
            const double* p = P(t);
            xa += p[0]; ya += p[1]; za += p[2];
        }
        xa /= h; ya /= h; za /= h;
        double c00 = 0, c01 = 0, c02 = 0, c11 = 0, c12 = 0, c22 = 0;
        for (int64_t t = s; t < e; t++) {
            const double* p = P(t);
            const double x0 = p[0] - xa, x1 = p[1] - ya, x2 = p[2] - za;
            c00 += x0 * x0; c01 += x0 * x1; c02 += x0 * x2;
            c11 += x1 * x1; c12 += x1 * x2; c22 += x2 * x2;
        }
        const double C[9] = {c00, c01, c02, c01, c11, c12, c02, c12, c22};
        pcp_plane pl;
        plane_from_cov(C, xa, ya, za, pl);
        out[sg] = pl;
    }
}

// K7 (main_blend.cpp:306-325): argmin over queries of the 1-NN d2, strict '<' from an
// initial bound, so the first query wins ties.  Per-block lexicographic (d2, i) minimum.
__global__ __launch_bounds__(kB) void k_argmin_d2(const double* d2, int64_t n, double* pd, int64_t* pi) {
    double bd = INFINITY;
    int64_t bi = INT64_MAX;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double d = d2[i];
        if (d < bd || (d == bd && i < bi)) { bd = d; bi = i; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o, 64);
        const int64_t oi = __shfl_xor(bi, o, 64);
        if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
    }
    __shared__ double sd[kB / 64];
    __shared__ int64_t si[kB / 64];
    if ((threadIdx.x & 63) == 0) { sd[threadIdx.x >> 6] = bd; si[threadIdx.x >> 6] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kB / 64; w++)
            if (sd[w] < bd || (sd[w] == bd && si[w] < bi)) { bd = sd[w]; bi = si[w]; }
        pd[blockIdx.x] = bd;
        pi[blockIdx.x] = bi;
    }
}

// ------------------------------------------------------------------ K6: kd_tree_lod
// fp32 kNN over the float vertices float(p - c) (kd_tree_lod/kd_tree.cpp:39-43, 62-68;
// the trimesh2 search is external: exact k nearest, ties by vertex index).
template <int K>
struct LodVisitor {
    const float4* pts;
    float qx, qy, qz;
    TopK<K, float> top;
    __device__ float bound() const { return top.kth() * (1.0f + 1e-5f); }
    __device__ void visit(uint32_t s, uint32_t e) {
        for (uint32_t t = s; t < e; t++) {
            const float4 p = pts[t];
            const float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
            float d = dx * dx;
            d = d + dy * dy;
            d = d + dz * dz;
            top.push(d, __float_as_int(p.w));
        }
    }
};

// first original j with point_dis2(k_point, cloud[j]) <= FLT_EPSILON (kd_tree.cpp:91-105)
struct MatchVisitor {
    const double4* pts;
    const int32_t* mapping;
    int identity;
    double kx, ky, kz;
    int best;
    double bestd;
    __device__ double bound() const { return (double)FLT_EPSILON * (1.0 + 1e-9); }
    __device__ void visit(uint32_t s, uint32_t e) {
        for (uint32_t t = s; t < e; t++) {
            const double4 p = pts[t];
            const double dx = kx - p.x, dy = ky - p.y, dz = kz - p.z;
            double d = dx * dx + dy * dy;  // pow(.,2) + pow(.,2) + pow(.,2)
            d = d + dz * dz;
            if (d <= (double)FLT_EPSILON) {
                const int jo = identity ? (int)p.w : mapping[(int)p.w];
                if (jo < best) { best = jo; bestd = d; }
            }
        }
    }
};

template <int K>
__global__ __launch_bounds__(kB) void k_lod(GridDesc gf, const float4* fpts, GridDesc gd, const double4* dpts,
                                            const int32_t* dmap, int didentity, const char* cloud, int64_t n,
                                            const char* q, int64_t nq, int k, int kk, float mcf, double mcd,
                                            int ci0, int ci1, int ci2, int32_t* oidx, double* od2) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nq; i += (int64_t)gridDim.x * blockDim.x) {
        const double* qp = (const double*)(q + i * PCP_AOS48_STRIDE);
        LodVisitor<K> v;
        v.pts = fpts;
        v.qx = (float)(qp[0] - ci0); v.qy = (float)(qp[1] - ci1); v.qz = (float)(qp[2] - ci2);
        v.top.init(kk);
        ring_search<float>(gf, v.qx, v.qy, v.qz, mcf, v);
        const double* last = (const double*)(cloud + (n - 1) * PCP_AOS48_STRIDE);
        v.top.for_each_ascending(kk, [&](int r, float, int jv) {
            int index = -1;
            double d2 = INFINITY;
            if (jv != INT_MAX) {
                const double* vp = (const double*)(cloud + (int64_t)jv * PCP_AOS48_STRIDE);
                // vertex float(p - c), neighbour rebuilt as double(float + float(c)) (:71-73)
                const float fx = (float)(vp[0] - ci0), fy = (float)(vp[1] - ci1), fz = (float)(vp[2] - ci2);
                MatchVisitor m{dpts, dmap, didentity, (double)(float)(fx + (float)ci0),
                               (double)(float)(fy + (float)ci1), (double)(float)(fz + (float)ci2), INT_MAX, 0.0};
                ring_search<double>(gd, m.kx, m.ky, m.kz, mcd, m);
                if (m.best != INT_MAX) {
                    index = m.best;
                    d2 = m.bestd;
                } else {  // no match: k_dis2 = residual to the last scanned point (:100)
                    const double dx = m.kx - last[0], dy = m.ky - last[1], dz = m.kz - last[2];
                    double dd = dx * dx + dy * dy;
                    d2 = dd + dz * dz;
                }
            }
            oidx[i * k + r] = index;
            od2[i * k + r] = d2;
        });
        for (int r = kk; r < k; r++) {
            oidx[i * k + r] = -1;
            od2[i * k + r] = INFINITY;
        }
    }
}

__global__ void k_lod_vertices(const char* cloud, int64_t n, int ci0, int ci1, int ci2, float* v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double* p = (const double*)(cloud + i * PCP_AOS48_STRIDE);
        v[3 * i + 0] = (float)(p[0] - ci0);
        v[3 * i + 1] = (float)(p[1] - ci1);
        v[3 * i + 2] = (float)(p[2] - ci2);
    }
}

int pick_k(int k) {
    if (k <= 1) return 1;
    if (k <= 4) return 4;
    if (k <= 8) return 8;
    if (k <= 16) return 16;
    if (k <= 32) return 32;
    if (k <= 64) return 64;
    return 0;
}

unsigned blocks_for(int64_t n) { return grid_for(n, kB, 1 << 22); }

int check_f64_index(pcp_ctx* ctx, const pcp_index* ix) {
    if (!ctx || !ix) return PCP_ERR_ARG;
    if (!ix->is_f64) return set_error(ctx, PCP_ERR_ARG, "fp64 (FLANN-contract) index required");
    return PCP_OK;
}

}  // namespace

int centroid_aos48_dev(pcp_ctx* ctx, const void* in, int64_t n, int is_dense, double c[4], uint32_t* count);

// deferred-query list of one call (returned to the context's cache on scope exit)
struct FarBuf {
    FarList f{nullptr, nullptr};
    pcp_ctx* ctx = nullptr;
    ~FarBuf() { dfree(ctx, f.list); dfree(ctx, f.count); dfree(ctx, f.ub); }
    int alloc(pcp_ctx* c, int64_t n, bool with_ub = false) {
        ctx = c;
        PCP_TRY(dmalloc(ctx, &f.list, n));
        PCP_TRY(dmalloc(ctx, &f.count, 1));
        if (with_ub) PCP_TRY(dmalloc(ctx, &f.ub, n));
        PCP_HIP(ctx, hipMemsetAsync(f.count, 0, sizeof(uint32_t), ctx->stream));
        return PCP_OK;
    }
};
constexpr unsigned kFarBlocks = 2048;

// a fixed radius that reaches past the near pass's cell rings goes straight to the far pass
bool radius_needs_far(const pcp_index* ix, double radius) { return radius * ix->g.inv_h >= (double)kCellRings; }

}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_knn(pcp_ctx* ctx, const pcp_index* ix, const double* q, size_t qstride, int64_t nq, int k,
            int32_t* oidx, double* od2) {
    PCP_TRY(check_f64_index(ctx, ix));
    if (nq < 0 || k <= 0 || (nq > 0 && (!q || !oidx))) return set_error(ctx, PCP_ERR_ARG, "pcp_knn: bad arguments");
    if (qstride == 0) qstride = 3 * sizeof(double);
    if (nq == 0) return PCP_OK;
    const int kk = (int)(k < ix->n ? k : ix->n);  // kd_tree.h:820-821
    const int K = pick_k(kk);
    if (!K) return set_error(ctx, PCP_ERR_UNSUPPORTED, "pcp_knn: k=%d > 64 not supported yet", k);
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    const double mc = cell_margin64(ix->g);
    const double4* pts = (const double4*)ix->pts;
    FarBuf fb;
    PCP_TRY(fb.alloc(ctx, nq));
#define LAUNCH_KNN(KV)                                                                                          \
    hipLaunchKernelGGL((k_knn<KV, false>), dim3(blocks_for(nq)), dim3(kB), 0, ctx->stream, ix->g, pts, ix->mapping,  \
                       ix->identity, q, qstride, nq, k, kk, mc, oidx, od2, fb.f);                                  \
    hipLaunchKernelGGL((k_knn_coop<KV>), dim3(kFarBlocks), dim3(kB), 0, ctx->stream, ix->g, pts, ix->mapping,         \
                       ix->identity, q, qstride, k, kk, mc, oidx, od2, fb.f)
    switch (K) {
        case 1: LAUNCH_KNN(1); break;
        case 4: LAUNCH_KNN(4); break;
        case 8: LAUNCH_KNN(8); break;
        case 16: LAUNCH_KNN(16); break;
        case 32: LAUNCH_KNN(32); break;
        default: LAUNCH_KNN(64); break;
    }
#undef LAUNCH_KNN
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

static uint32_t radius_cap(const pcp_index* ix, uint32_t max_nn) {
    // max_nn == 0 or > total => unlimited (kd_tree.h:873-883)
    if (max_nn == 0 || (int64_t)max_nn >= ix->n) return UINT32_MAX;
    return max_nn;
}

int pcp_radius_count(pcp_ctx* ctx, const pcp_index* ix, const double* q, size_t qstride, int64_t nq, double radius,
                     uint32_t max_nn, int32_t* ocnt) {
    PCP_TRY(check_f64_index(ctx, ix));
    if (nq < 0 || (nq > 0 && (!q || !ocnt)) || !(radius >= 0))
        return set_error(ctx, PCP_ERR_ARG, "pcp_radius_count: bad arguments");
    if (qstride == 0) qstride = 3 * sizeof(double);
    if (nq == 0) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    const double4* pts = (const double4*)ix->pts;
    const uint32_t cap = radius_cap(ix, max_nn);
    const double mc = cell_margin64(ix->g);
    if (radius_needs_far(ix, radius)) {
        hipLaunchKernelGGL(k_radius_count<true>, dim3(blocks_for(nq)), dim3(kB), 0, ctx->stream, ix->g, pts, q, qstride,
                           nq, radius * radius, cap, mc, ocnt, FarList{nullptr, nullptr});
    } else {
        FarBuf fb;
        PCP_TRY(fb.alloc(ctx, nq));
        hipLaunchKernelGGL(k_radius_count<false>, dim3(blocks_for(nq)), dim3(kB), 0, ctx->stream, ix->g, pts, q,
                           qstride, nq, radius * radius, cap, mc, ocnt, fb.f);
        hipLaunchKernelGGL(k_radius_count<true>, dim3(kFarBlocks), dim3(kB), 0, ctx->stream, ix->g, pts, q, qstride,
                           nq, radius * radius, cap, mc, ocnt, fb.f);
    }
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_radius_fill(pcp_ctx* ctx, const pcp_index* ix, const double* q, size_t qstride, int64_t nq, double radius,
                    uint32_t max_nn, const int64_t* off, int32_t* oidx, double* od2) {
    PCP_TRY(check_f64_index(ctx, ix));
    if (nq < 0 || (nq > 0 && (!q || !off || !oidx || !od2)) || !(radius >= 0))
        return set_error(ctx, PCP_ERR_ARG, "pcp_radius_fill: bad arguments");
    (void)max_nn;  // row lengths were fixed by the count pass
    if (qstride == 0) qstride = 3 * sizeof(double);
    if (nq == 0) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    const double4* pts = (const double4*)ix->pts;
    const double mc = cell_margin64(ix->g);
    const uint32_t cap = radius_cap(ix, max_nn);
    if (radius_needs_far(ix, radius)) {
        hipLaunchKernelGGL(k_radius_fill<true>, dim3(blocks_for(nq)), dim3(kB), 0, ctx->stream, ix->g, pts, q, qstride,
                           nq, radius * radius, cap, mc, off, oidx, od2, FarList{nullptr, nullptr});
    } else {
        FarBuf fb;
        PCP_TRY(fb.alloc(ctx, nq));
        hipLaunchKernelGGL(k_radius_fill<false>, dim3(blocks_for(nq)), dim3(kB), 0, ctx->stream, ix->g, pts, q,
                           qstride, nq, radius * radius, cap, mc, off, oidx, od2, fb.f);
        hipLaunchKernelGGL(k_radius_fill<true>, dim3(kFarBlocks), dim3(kB), 0, ctx->stream, ix->g, pts, q, qstride,
                           nq, radius * radius, cap, mc, off, oidx, od2, fb.f);
    }
    hipLaunchKernelGGL(k_sort_rows, dim3(grid_for((nq + 3) / 4, 1, 1 << 16)), dim3(256), 0, ctx->stream, off, nq, cap,
                       oidx, od2, ix->mapping, ix->identity);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_normals_knn(pcp_ctx* ctx, const pcp_index* ix, int k, pcp_plane* out, int64_t n_out) {
    PCP_TRY(check_f64_index(ctx, ix));
    if (k <= 0 || n_out < 0 || (n_out > 0 && !out)) return set_error(ctx, PCP_ERR_ARG, "pcp_normals_knn: bad arguments");
    if (n_out < ix->n_in) return set_error(ctx, PCP_ERR_CAPACITY, "pcp_normals_knn: n_out < cloud size");
    const int kk = (int)(k < ix->n ? k : ix->n);
    const int K = pick_k(kk);
    if (!K || K > 32) return set_error(ctx, PCP_ERR_UNSUPPORTED, "pcp_normals_knn: k=%d > 32 not supported yet", k);
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    if (n_out > 0) hipLaunchKernelGGL(k_plane_default, dim3(blocks_for(n_out)), dim3(kB), 0, ctx->stream, out, n_out);
    if (ix->n == 0 || kk <= 3) return PCP_OK;  // rpca's N > 3 guard (calculate_feature.cpp:237)
    const double mc = cell_margin64(ix->g);
    const double4* pts = (const double4*)ix->pts;
    FarBuf fb;
    PCP_TRY(fb.alloc(ctx, ix->n, true));
    const int tile_R = kk <= 8 ? 1 : 2;  // the tile's window half-width in cells
    if (ix->g.dense) {
        unsigned long long* st = nullptr;  // per-phase counters of profiling builds (PCP_NORMALS_STATS)
#if PCP_NORMALS_STATS
        PCP_TRY(dmalloc(ctx, &st, 24));
        PCP_HIP(ctx, hipMemsetAsync(st, 0, 24 * sizeof(unsigned long long), ctx->stream));
#endif
        const unsigned nbt = (unsigned)std::min<int64_t>((ix->n + 63) / 64, 1 << 20);
        // brick order of the queries: (brick key, sorted position) radix-sorted
        uint32_t *k0 = nullptr, *k1 = nullptr, *v0 = nullptr, *order = nullptr;
        void* tmp = nullptr;
        size_t tb = 0;
        struct Free {
            pcp_ctx* c;
            uint32_t **a, **b, **d, **e;
            void** t;
            ~Free() { dfree(c, *a); dfree(c, *b); dfree(c, *d); dfree(c, *e); dfree(c, (char*)*t); }
        } fr{ctx, &k0, &k1, &v0, &order, &tmp};
        PCP_TRY(dmalloc(ctx, &k0, ix->n));
        PCP_TRY(dmalloc(ctx, &k1, ix->n));
        PCP_TRY(dmalloc(ctx, &v0, ix->n));
        PCP_TRY(dmalloc(ctx, &order, ix->n));
        const int64_t nbr = (int64_t)((ix->g.n[0] + 7) >> kTileBrick) * ((ix->g.n[1] + 7) >> kTileBrick) *
                            ((ix->g.n[2] + 7) >> kTileBrick);
        unsigned bits = 1;
        while (bits < 32 && ((int64_t)1 << bits) < nbr) bits++;
        // Morton bits inside the brick: cell + sub-cell (12) when the key still fits 32 bits
        int lb = 0;
        if (PCP_TILE_MORTON) lb = bits + 12 <= 32 ? 12 : (bits + 9 <= 32 ? 9 : 0);
        hipLaunchKernelGGL(k_brick_keys, dim3(blocks_for(ix->n)), dim3(kB), 0, ctx->stream, ix->g, pts, ix->n, lb, k0,
                           v0);
        bits += (unsigned)lb;
        PCP_HIP(ctx, rocprim::radix_sort_pairs(nullptr, tb, k0, k1, v0, order, (size_t)ix->n, 0u, bits, ctx->stream));
        PCP_TRY(dmalloc(ctx, (char**)&tmp, tb));
        PCP_HIP(ctx, rocprim::radix_sort_pairs(tmp, tb, k0, k1, v0, order, (size_t)ix->n, 0u, bits, ctx->stream));
        FarBuf fb2;  // the near pass's own deferred queries
        PCP_TRY(fb2.alloc(ctx, ix->n, true));
        // the tile's uncertified queries: the lane-per-query near pass (cell rings), its own
        // deferrals then the wave-per-query pass (PCP_NORMALS_NEAR_DEFAULT; 0: all of them straight
        // to the wave-per-query pass, measured slower)
        const bool near_pass = PCP_NORMALS_NEAR_DEFAULT;
        const int lane_mode = PCP_TILE_LANE_DEFAULT;  // 0: every lane scans the union box (slower)
#define LAUNCH_TILE(KV)                                                                                          \
        hipLaunchKernelGGL((k_normals_tile<KV>), dim3(nbt), dim3(64), 0, ctx->stream, ix->g, pts, ix->mapping,      \
                           ix->identity, ix->n, kk, tile_R, mc, out, n_out, fb.f, st, order, lane_mode);          \
        if (near_pass)                                                                                            \
            hipLaunchKernelGGL((k_normals<KV, false, PCP_NEAR_ROWS != 0>), dim3(blocks_for(ix->n)), dim3(kB), 0,     \
                               ctx->stream, ix->g,                                                              \
                               pts, ix->mapping, ix->identity, ix->pos_of_j, ix->n, kk, mc, out, n_out, fb2.f, fb.f); \
        hipLaunchKernelGGL((k_normals_coop<KV>), dim3(kFarBlocks), dim3(kB), 0, ctx->stream, ix->g, pts,            \
                           ix->mapping, ix->identity, ix->pos_of_j, kk, mc, out, n_out, near_pass ? fb2.f : fb.f,  \
                           st ? st + 4 : nullptr)
        switch (K) {
            case 1: case 4: LAUNCH_TILE(4); break;
            case 8: LAUNCH_TILE(8); break;
            case 16: LAUNCH_TILE(16); break;
            default: LAUNCH_TILE(32); break;
        }
#undef LAUNCH_TILE
        PCP_LAUNCH_CHECK(ctx);
#if PCP_NORMALS_STATS
        {
            unsigned long long h[24];
            unsigned c1 = 0, c2 = 0;
            PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
            PCP_HIP(ctx, hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
            PCP_HIP(ctx, hipMemcpy(&c1, fb.f.count, 4, hipMemcpyDeviceToHost));
            PCP_HIP(ctx, hipMemcpy(&c2, fb2.f.count, 4, hipMemcpyDeviceToHost));
            const unsigned long long* d = h + 4;
            fprintf(stderr, "normals stats: n=%lld k=%d tile deferred %u (list bound %llu, box %llu, oversize %llu), "
                    "near deferred %u; far pass: %llu queries, shells mean %.1f max %llu, cycles mean %.0f max %llu "
                    "(slowest: ring %llu, kth %llu, bricks %llu, rows+points %llu, mid-shell %llu; at %.2f %.2f %.2f)\n",
                    (long long)ix->n, k, c1, h[0], h[2], h[1], c2, d[0], d[0] ? (double)d[1] / d[0] : 0.0, d[2],
                    d[0] ? (double)d[3] / d[0] : 0.0, d[4], d[11], d[12], d[13], d[14], d[15],
                    __builtin_bit_cast(double, d[5]), __builtin_bit_cast(double, d[6]), __builtin_bit_cast(double, d[7]));
            dfree(ctx, st);
        }
#endif
        return PCP_OK;
    }
#define LAUNCH_NRM(KV)                                                                                              \
    hipLaunchKernelGGL((k_normals<KV, false>), dim3(blocks_for(ix->n)), dim3(kB), 0, ctx->stream, ix->g, pts,          \
                       ix->mapping, ix->identity, ix->pos_of_j, ix->n, kk, mc, out, n_out, fb.f);                      \
    hipLaunchKernelGGL((k_normals_coop<KV>), dim3(kFarBlocks), dim3(kB), 0, ctx->stream, ix->g, pts, ix->mapping,       \
                       ix->identity, ix->pos_of_j, kk, mc, out, n_out, fb.f)
    switch (K) {
        case 1: LAUNCH_NRM(1); break;
        case 4: LAUNCH_NRM(4); break;
        case 8: LAUNCH_NRM(8); break;
        case 16: LAUNCH_NRM(16); break;
        default: LAUNCH_NRM(32); break;
    }
#undef LAUNCH_NRM
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_plane_fit_segments(pcp_ctx* ctx, const double* xyz, size_t stride, const int64_t* off, const int32_t* idx,
                           int64_t nseg, pcp_plane* out) {
    if (!ctx || nseg < 0 || (nseg > 0 && (!xyz || !off || !out)))
        return set_error(ctx, PCP_ERR_ARG, "pcp_plane_fit_segments: bad arguments");
    if (stride == 0) stride = 3 * sizeof(double);
    if (nseg == 0) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_plane_segments, dim3(blocks_for(nseg)), dim3(kB), 0, ctx->stream, xyz, stride, off, idx, nseg,
                       out);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_nearest_query(pcp_ctx* ctx, const pcp_index* ix, const double* q, size_t qstride, int64_t nq,
                      double init_bound, int64_t* best_q, double* best_d2) {
    PCP_TRY(check_f64_index(ctx, ix));
    if (nq < 0 || (nq > 0 && !q) || !best_q || !best_d2)
        return set_error(ctx, PCP_ERR_ARG, "pcp_nearest_query: bad arguments");
    *best_q = -1;
    *best_d2 = init_bound;
    if (nq == 0 || ix->n == 0) return PCP_OK;
    int32_t* idx = nullptr;
    double* d2 = nullptr;
    double* pd = nullptr;
    int64_t* pi = nullptr;
    const unsigned nb = grid_for(nq, kB, 1024);
    int rc = dmalloc(ctx, &idx, nq);
    if (!rc) rc = dmalloc(ctx, &d2, nq);
    if (!rc) rc = dmalloc(ctx, &pd, nb);
    if (!rc) rc = dmalloc(ctx, &pi, nb);
    if (!rc) rc = pcp_knn(ctx, ix, q, qstride, nq, 1, idx, d2);
    if (!rc) {
        hipLaunchKernelGGL(k_argmin_d2, dim3(nb), dim3(kB), 0, ctx->stream, d2, nq, pd, pi);
        std::vector<double> hd(nb);
        std::vector<int64_t> hi(nb);
        hipError_t e = hipMemcpyAsync(hd.data(), pd, nb * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(hi.data(), pi, nb * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) rc = hip_fail(ctx, e, "nearest_query", __FILE__, __LINE__);
        // lexicographic (d2, query) minimum == the sequential strict-'<' scan's winner
        double bd = INFINITY;
        int64_t bi = INT64_MAX;
        for (unsigned b = 0; b < nb && !rc; b++)
            if (hd[b] < bd || (hd[b] == bd && hi[b] < bi)) { bd = hd[b]; bi = hi[b]; }
        if (!rc && bd < init_bound) { *best_d2 = bd; *best_q = bi; }
    }
    dfree(ctx, idx); dfree(ctx, d2); dfree(ctx, pd); dfree(ctx, pi);
    return rc;
}

int pcp_knn_lod(pcp_ctx* ctx, const void* cloud, int64_t n, const void* q, int64_t nq, int k, int32_t* oidx,
                double* od2) {
    if (!ctx || n < 0 || nq < 0 || k <= 0 || (n > 0 && !cloud) || (nq > 0 && (!q || !oidx || !od2)))
        return set_error(ctx, PCP_ERR_ARG, "pcp_knn_lod: bad arguments");
    if (n == 0 || nq == 0) return PCP_OK;
    const int kk = (int)(k < n ? k : n);
    const int K = pick_k(kk);
    if (!K || K > 32) return set_error(ctx, PCP_ERR_UNSUPPORTED, "pcp_knn_lod: k=%d > 32 not supported yet", k);
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    // c = Vector3i truncation of the centroid (kd_tree_lod/kd_tree.cpp:33-37)
    double c[4];
    uint32_t cnt = 0;
    PCP_TRY(centroid_aos48_dev(ctx, cloud, n, 1, c, &cnt));
    const int ci0 = (int)c[0], ci1 = (int)c[1], ci2 = (int)c[2];
    float* v = nullptr;
    PCP_TRY(dmalloc(ctx, &v, 3 * (size_t)n));
    hipLaunchKernelGGL(k_lod_vertices, dim3(blocks_for(n)), dim3(kB), 0, ctx->stream, (const char*)cloud, n, ci0, ci1,
                       ci2, v);
    pcp_index* fi = nullptr;
    pcp_index* di = nullptr;
    int rc = pcp_index_build_f32(ctx, v, 3 * sizeof(float), n, 0.0, &fi);
    if (rc == PCP_OK) rc = pcp_index_build_f64(ctx, (const double*)cloud, PCP_AOS48_STRIDE, n, nullptr, 0, 0.0, &di);
    if (rc == PCP_OK) {
        const GridDesc& gf = fi->g;
        const int nmax = std::max(gf.n[0], std::max(gf.n[1], gf.n[2]));
        const float mcf = 1e-5f + 8e-7f * (float)nmax;
#define LAUNCH_LOD(KV)                                                                                     \
    hipLaunchKernelGGL(k_lod<KV>, dim3(blocks_for(nq)), dim3(kB), 0, ctx->stream, fi->g, (const float4*)fi->pts, \
                       di->g, (const double4*)di->pts, di->mapping, di->identity, (const char*)cloud, n,           \
                       (const char*)q, nq, k, kk, mcf, cell_margin64(di->g), ci0, ci1, ci2, oidx, od2)
        switch (K) {
            case 1: LAUNCH_LOD(1); break;
            case 4: LAUNCH_LOD(4); break;
            case 8: LAUNCH_LOD(8); break;
            case 16: LAUNCH_LOD(16); break;
            default: LAUNCH_LOD(32); break;
        }
#undef LAUNCH_LOD
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) rc = hip_fail(ctx, e, "k_lod", __FILE__, __LINE__);
    }
    if (fi) pcp_index_destroy(fi);
    if (di) pcp_index_destroy(di);
    dfree(ctx, v);
    return rc;
}

}  // extern "C"
