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

#include "grid.hpp"
#include "topk.hpp"
#include "pca.hpp"

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
template <int K>
struct KnnVisitor {
    static constexpr int U = K <= 16 ? PCP_KNN_BATCH : 2;
    const double4* pts;
    double qx, qy, qz;
    TopK<K> top;
    // pruning radius^2 (1e-12 covers the rounding of the cell-box bound and of d2)
    __device__ double bound() const { return top.kth() * (1.0 + 1e-12); }
    __device__ void visit(uint32_t s, uint32_t e) {
        uint32_t t = s;
        for (; t + U <= e; t += U) {
            double4 p[U];
#pragma unroll
            for (int u = 0; u < U; u++) p[u] = pts[t + u];
#pragma unroll
            for (int u = 0; u < U; u++) top.push(l2_simple(qx, qy, qz, p[u]), (int)p[u].w);
        }
        for (; t < e; t++) {
            const double4 p = pts[t];
            top.push(l2_simple(qx, qy, qz, p), (int)p.w);
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
__device__ __forceinline__ void defer(const FarList& f, int64_t i) { f.list[atomicAdd(f.count, 1u)] = (int32_t)i; }

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
template <int K, bool FAR>
__global__ __launch_bounds__(kB) void k_normals(GridDesc g, const double4* pts, const int32_t* mapping, int identity,
                                                const int32_t* pos_of_j, int64_t n, int kk, double mc,
                                                pcp_plane* out, int64_t n_out, FarList far) {
    const int64_t nw = work_count<FAR>(far, n);
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = work_item<FAR>(far, w);
        const double4 qp = pts[s];
        KnnVisitor<K> v;
        v.pts = pts;
        v.qx = qp.x; v.qy = qp.y; v.qz = qp.z;
        v.top.init(kk);
        if (!ring_search<double, KnnVisitor<K>, FAR>(g, v.qx, v.qy, v.qz, mc, v)) {
            defer(far, s);
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
    ~FarBuf() { dfree(ctx, f.list); dfree(ctx, f.count); }
    int alloc(pcp_ctx* c, int64_t n) {
        ctx = c;
        PCP_TRY(dmalloc(ctx, &f.list, n));
        PCP_TRY(dmalloc(ctx, &f.count, 1));
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
    hipLaunchKernelGGL((k_knn<KV, true>), dim3(kFarBlocks), dim3(kB), 0, ctx->stream, ix->g, pts, ix->mapping,        \
                       ix->identity, q, qstride, nq, k, kk, mc, oidx, od2, fb.f)
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
    if (getenv("PCP_KNN_DEBUG")) {
        uint32_t c = 0;
        hipMemcpy(&c, fb.f.count, 4, hipMemcpyDeviceToHost);
        fprintf(stderr, "pcp_knn: k=%d nq=%lld deferred to the far pass: %u\n", k, (long long)nq, c);
    }
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
    PCP_TRY(fb.alloc(ctx, ix->n));
#define LAUNCH_NRM(KV)                                                                                              \
    hipLaunchKernelGGL((k_normals<KV, false>), dim3(blocks_for(ix->n)), dim3(kB), 0, ctx->stream, ix->g, pts,          \
                       ix->mapping, ix->identity, ix->pos_of_j, ix->n, kk, mc, out, n_out, fb.f);                      \
    hipLaunchKernelGGL((k_normals<KV, true>), dim3(kFarBlocks), dim3(kB), 0, ctx->stream, ix->g, pts, ix->mapping,      \
                       ix->identity, ix->pos_of_j, ix->n, kk, mc, out, n_out, fb.f)
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
