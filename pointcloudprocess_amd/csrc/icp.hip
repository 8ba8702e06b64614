// ICP correspondence/transform loop (replaces the trimesh2 ICP() call inside
// PointCloudHelper::get_rot_icp, point_cloud_helper.cpp:75-166; callers main_blend.cpp:106,
// 818, 887 and point_cloud_closure via main_blend).
//
// Per iteration one fused kernel: transform-on-load of each (spatially sorted) query by
// the current pose (fp32 fmaf chain, the contract in DESIGN.md §ICP), exact 1-NN within
// rmax over the fp32 grid index (ring search, lexicographic (d2, target index)), and the
// 24 double accumulators reduced per wavefront (shuffles) -> per workgroup (LDS) -> one
// fixed-order pass over the workgroup partials.  The host solves the 3x3 Kabsch/Umeyama
// problem (pcp_icp_solve) and composes the pose.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include "sortcfg.hpp"

#include "grid.hpp"
#include "wave_acc.hpp"

namespace pcp {
// a sorted query's coordinates: 12 bytes (one global_load_dwordx3 per lane)
struct QXyz {
    float x, y, z;
};
}  // namespace pcp

struct pcp_icp {
    pcp_ctx* ctx = nullptr;       // the context of the last call (launches go to its stream)
    pcp_ctx* owner = nullptr;     // the creating context: owns the buffers (a lifetime reference)
    const pcp_index* target = nullptr;
    int64_t nq = 0;               // finite queries
    int64_t nq_in = 0;            // queries passed to pcp_icp_create
    pcp::QXyz* q = nullptr;       // sorted queries, 12-byte xyz (the verify stream reads 12 B, not 16)
    int32_t* qidx = nullptr;      // their original indices (read only for caller-order outputs)
    uint32_t* cand = nullptr;     // per sorted query: its cache record (cache_load / cache_store): the
                                  // sorted-target positions of its 3 nearest targets at its last search
                                  // (the winner is always among them), the launch slot s of that search
                                  // and D, a lower bound on the distance from the query, at that launch's
                                  // pose, to every target NOT cached.  12 bytes when the target has fewer
                                  // than 2^26 - 2 points (narrow), else 16
    bool narrow = false;
    float* pose_hist = nullptr;   // 256 x 12 floats: the pose of launch t at slot t & hist_mask
    int64_t launches = 0;         // correspondence launches so far (the first has nothing to verify)
    bool last_verified = false;   // the last launch ran the verify pass
    int32_t* sv = nullptr;        // verify pass: per-wave segments of uncertified queries (sv_seg each)
    uint32_t* sv_count = nullptr;
    uint32_t* sv_off = nullptr;   // [nseg_v]: the search list's length (k_list_compact)
    int32_t* svc = nullptr;       // compacted search list
    int64_t sv_seg = 0;
    int64_t nseg_v = 0;           // verify list segments: one per wave, or one per chunk (XCD split)
    int nb_ver = 0;
    int32_t* fb = nullptr;        // fallback lists: one segment of fb_seg entries per octant WG
    uint32_t* fb_count = nullptr; // per octant wave: entries in its segment
    uint32_t* fb_off = nullptr;   // [nseg]: the fallback list's length (k_list_compact)
    int32_t* fbc = nullptr;       // compacted fallback list
    int64_t fb_seg = 0;
    double* partials = nullptr;   // (nb_ver + nb_fast + nb_ring) * 24
    double* acc = nullptr;        // 24 (scratch for pcp_icp_run)
    int nb_fast = 0, nb_ring = 0;
    int nb_fast_l = 0;            // octant grid of the list launches (<= nb_fast)
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_mid = nullptr, ev_ver = nullptr;
    float* pose_dev = nullptr;    // 24 floats: this launch's pose (R row-major, t), then the previous one
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;  // per-launch timing events (device loop)
    size_t ntev = 0;              // pairs recorded since the last pcp_icp_kernel_ms
    int dbg = 0;                  // ablation flags (pcp_icp_set_options; profiling only: results are wrong)
    int oct_g_first = 1;          // lanes per query of the octant pass: first launch (all queries)
    int oct_g_list = 0;           // ... and the verify pass's search lists (0: by the list's density)
    int ring_g = 0;               // lanes per query of the fallback pass, 0 = by the list's length
    double last_ms = 0.0;
    int last_launches = 0;
    uint32_t last_fallback = 0;
    uint32_t last_searched = 0;   // queries the verify pass could not certify (searched)
    hipGraphExec_t gexec = nullptr;  // the verify .. fallback section of a device-pose launch (icp_launch)
    float graph_r2 = 0.f;            // the rmax^2 it was captured with
    bool graph_off = false;          // capture failed: plain launches
    bool graph = false;              // PCP_ICP_OPT_GRAPH
};

namespace pcp {
namespace {

constexpr int kIcpBlock = 256;
#ifndef PCP_OCT_WAVES_LIST  // the octant pass over the verify pass's lists: more registers, fewer waves
#define PCP_OCT_WAVES_LIST 4
#endif
#ifndef PCP_OCT_WAVES
#define PCP_OCT_WAVES 6
#endif
#ifndef PCP_VER_WAVES   // verify (per-lane accumulators: ~100 VGPRs)
#define PCP_VER_WAVES 4
#endif

#ifndef PCP_RING_WAVES
#define PCP_RING_WAVES 6
#endif
constexpr int kAcc = 24;

struct IcpArgs {
    GridDesc g;
    const float4* tp;   // sorted target points
    const QXyz* q;      // sorted queries (xyz)
    const int32_t* qidx;  // their original indices
    int64_t nq;
    int64_t nchunks;
    float R[9], t[3];
    float Rp[9], tq[3]; // the previous launch's pose (verify pass)
    float r2;
    float cert2;        // certified radius^2 of the 2x2x2 octant search
    float rho;          // octant half-width in cell units (0.5 - margin)
    float mc;           // cell-unit margin for pruning
    double* partials;
    uint32_t* cand;     // cache records (cache_load / cache_store)
    int narrow;         // 12-byte records
    uint32_t hist_mask; // pose history slot of a launch: launch & hist_mask (63 narrow, 255 wide)
    uint32_t max_age;   // older caches are searched again (so their slot is never reused)
    float dunit, inv_dunit;  // narrow D code unit (cell size / 1024)
    const float* pose_hist;
    uint32_t launch;    // this launch's index (mod 2^32)
    uint32_t ntp;       // target points (tp[ntp] is the far sentinel)
    int32_t* sv;        // verify pass output segments (sv_seg entries per wave)
    uint32_t* sv_count;
    uint32_t* sv_off;
    int64_t sv_seg;
    int64_t nseg_v;     // verify-pass waves
    int32_t* fb;
    uint32_t* fb_count;
    uint32_t* fb_off;   // [nseg]: the compacted fallback list's length
    int64_t fb_seg;
    int nb_fast;
    int64_t nseg;       // fallback segments (= waves of the octant kernel)
    int ring_all;       // ring kernel: process every query (sparse grid) instead of the list
    int dbg;            // ablation flags (pcp_icp_set_options; profiling only)
    int oct_g;          // octant pass lanes per query: 1, 2, 4, 8, or 0 = by the list's density
    int ring_g;         // fallback pass lanes per query: 1, 2, 4, 8, or 0 = PCP_RING_G / by length
    const float* pose;  // device poses (current, previous: 24 floats) overriding R/t, Rp/tq, or null
    const uint32_t* launch_dev;  // device copy of `launch` (k_pose_set), so a captured launch graph replays
};

// sorted query i as {x, y, z, 0}
__device__ __forceinline__ float4 ldq(const IcpArgs& a, int64_t i) {
    const QXyz v = a.q[i];
    return make_float4(v.x, v.y, v.z, 0.f);
}

// the pose as the kernels use it: from the device copy when the loop is device-resident
__device__ __forceinline__ void load_pose(IcpArgs& a) {
    if (a.launch_dev) a.launch = *a.launch_dev;
    if (a.pose) {
#pragma unroll
        for (int k = 0; k < 9; k++) a.R[k] = a.pose[k];
#pragma unroll
        for (int k = 0; k < 3; k++) a.t[k] = a.pose[9 + k];
    }
}
__device__ __forceinline__ void load_prev_pose(IcpArgs& a) {
#pragma unroll
    for (int k = 0; k < 9; k++) a.Rp[k] = a.pose[12 + k];
#pragma unroll
    for (int k = 0; k < 3; k++) a.tq[k] = a.pose[21 + k];
}

// Ablation switches for profiling (pcp_icp_set_options, PCP_ICP_ABLATE_*); results are wrong
// when any is set.
constexpr int kDbgNoScan = PCP_ICP_ABLATE_NO_SCAN, kDbgNoAccum = PCP_ICP_ABLATE_NO_ACCUM,
              kDbgNoFallback = PCP_ICP_ABLATE_NO_FALLBACK, kDbgNoVerify = PCP_ICP_ABLATE_NO_VERIFY;

__device__ __forceinline__ void xform(const IcpArgs& a, const float4 q, float& x, float& y, float& z) {
    // q' = R q + t: x' = fmaf(R02,z,fmaf(R01,y,fmaf(R00,x,t0)))
    x = __fmaf_rn(a.R[2], q.z, __fmaf_rn(a.R[1], q.y, __fmaf_rn(a.R[0], q.x, a.t[0])));
    y = __fmaf_rn(a.R[5], q.z, __fmaf_rn(a.R[4], q.y, __fmaf_rn(a.R[3], q.x, a.t[1])));
    z = __fmaf_rn(a.R[8], q.z, __fmaf_rn(a.R[7], q.y, __fmaf_rn(a.R[6], q.x, a.t[2])));
}
// the same expression under the previous launch's pose
__device__ __forceinline__ void xform_prev(const IcpArgs& a, const float4 q, float& x, float& y, float& z) {
    x = __fmaf_rn(a.Rp[2], q.z, __fmaf_rn(a.Rp[1], q.y, __fmaf_rn(a.Rp[0], q.x, a.tq[0])));
    y = __fmaf_rn(a.Rp[5], q.z, __fmaf_rn(a.Rp[4], q.y, __fmaf_rn(a.Rp[3], q.x, a.tq[1])));
    z = __fmaf_rn(a.Rp[8], q.z, __fmaf_rn(a.Rp[7], q.y, __fmaf_rn(a.Rp[6], q.x, a.tq[2])));
}

// running 1-NN: best d2, its target index (tie order) and its position in the scanned array
#ifndef PCP_SCAN_UNROLL
#define PCP_SCAN_UNROLL 4
#endif
#ifndef PCP_TRACK_BEST
#define PCP_TRACK_BEST 0
#endif
// the contract's fp32 d2: fmaf(dz,dz,fmaf(dy,dy,dx*dx))
__device__ __forceinline__ float icp_d2(float qx, float qy, float qz, const float4 p) {
    const float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
    return __fmaf_rn(dz, dz, __fmaf_rn(dy, dy, dx * dx));
}

// min / max of non-NaN floats as one v_med3_f32 (fminf/fmaxf add canonicalizing v_max ops)
__device__ __forceinline__ float fmin_nn(float a, float b) { return __builtin_amdgcn_fmed3f(a, b, -INFINITY); }
__device__ __forceinline__ float fmax_nn(float a, float b) { return __builtin_amdgcn_fmed3f(a, b, INFINITY); }

// position of candidate v of four concatenated rows (row prefixes c1 <= c2 <= c3, per-row
// offsets o0..o3): register selects only (an indexed form was lowered to an LDS table of
// pointers plus a scratch load per candidate)
__device__ __forceinline__ uint32_t cat_addr(uint32_t v, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t o0,
                                             uint32_t o1, uint32_t o2, uint32_t o3) {
    const uint32_t a = v < c3 ? o2 : o3;
    const uint32_t b = v < c2 ? o1 : a;
    return v + (v < c1 ? o0 : b);
}

struct Best {
    float bd;
    int bj;
    uint32_t bk;
    float px, py, pz;  // filled by fetch() once the scan is over (or tracked, PCP_TRACK_BEST)
    __device__ __forceinline__ void consider(float qx, float qy, float qz, const float4 p, uint32_t k) {
        const float d2 = icp_d2(qx, qy, qz, p);
        const int id = __float_as_int(p.w);
        // "<=" on the index: re-visiting the current winner (a provisional bound) refreshes bk
        const bool take = d2 < bd || (d2 == bd && id <= bj);
        bd = take ? d2 : bd;
        bj = take ? id : bj;
        bk = take ? k : bk;
#if PCP_TRACK_BEST
        px = take ? p.x : px;
        py = take ? p.y : py;
        pz = take ? p.z : pz;
#endif
    }
    // candidates [s, e) of `pts` (LDS or global); loads issued 4 at a time so the memory
    // latency of a candidate is not serialised behind the previous update
    template <typename P>
    __device__ __forceinline__ void scan(const P* pts, uint32_t s, uint32_t e, float qx, float qy, float qz) {
        uint32_t k = s;
        for (; k + 4 <= e; k += 4) {
            const float4 p0 = pts[k], p1 = pts[k + 1], p2 = pts[k + 2], p3 = pts[k + 3];
            consider(qx, qy, qz, p0, k);
            consider(qx, qy, qz, p1, k + 1);
            consider(qx, qy, qz, p2, k + 2);
            consider(qx, qy, qz, p3, k + 3);
        }
        for (; k < e; k++) consider(qx, qy, qz, pts[k], k);
    }
    // rows r = 0..3 ([rs[r], rs[r] + rn[r])) scanned as one concatenated list, 4 loads in flight
    template <typename P, int NR>
    __device__ __forceinline__ void scan_rows(const P* pts, const uint32_t (&rs)[NR], const uint32_t (&rn)[NR],
                                              float qx, float qy, float qz) {
        static_assert(NR == 3 || NR == 4, "3 or 4 rows");
        const uint32_t c1 = rn[0], c2 = c1 + rn[1], c3 = c2 + rn[2], L = NR == 4 ? c3 + rn[NR - 1] : c3;
        const uint32_t o0 = rs[0], o1 = rs[1] - c1, o2 = rs[2] - c2, o3 = rs[NR - 1] - c3;
        const uint32_t c3e = NR == 4 ? c3 : 0xffffffffu;  // 3 rows: never past the third
        auto addr = [=](uint32_t v) { return cat_addr(v, c1, c2, c3e, o0, o1, o2, o3); };
        uint32_t v = 0;
        constexpr int U = PCP_SCAN_UNROLL;
        for (; v + U <= L; v += U) {
            uint32_t k[U];
            float4 p[U];
#pragma unroll
            for (int u = 0; u < U; u++) k[u] = addr(v + u);
#pragma unroll
            for (int u = 0; u < U; u++) p[u] = pts[k[u]];
#pragma unroll
            for (int u = 0; u < U; u++) consider(qx, qy, qz, p[u], k[u]);
        }
        for (; v < L; v++) {
            const uint32_t k = addr(v);
            consider(qx, qy, qz, pts[k], k);
        }
    }
    // G lanes per query: lane `sub` of the group takes entries sub, sub + G, ... of the same
    // ranges (strided scan / scan_rows), then merge_group() gives every lane of the group the
    // group's (d2, index) winner.  A lane prunes with its own bound, which is never below the
    // group's, so nothing the group's winner needs is skipped.
    template <int G, typename P>
    __device__ __forceinline__ void scan_g(const P* pts, uint32_t s, uint32_t e, float qx, float qy, float qz,
                                           uint32_t sub) {
        if (G == 1) {
            scan(pts, s, e, qx, qy, qz);
            return;
        }
        uint32_t k = s + sub;
        for (; k + 3 * G < e; k += 4 * G) {
            const float4 p0 = pts[k], p1 = pts[k + G], p2 = pts[k + 2 * G], p3 = pts[k + 3 * G];
            consider(qx, qy, qz, p0, k);
            consider(qx, qy, qz, p1, k + G);
            consider(qx, qy, qz, p2, k + 2 * G);
            consider(qx, qy, qz, p3, k + 3 * G);
        }
        for (; k < e; k += G) consider(qx, qy, qz, pts[k], k);
    }
    template <int G, typename P, int NR>
    __device__ __forceinline__ void scan_rows_g(const P* pts, const uint32_t (&rs)[NR], const uint32_t (&rn)[NR],
                                                float qx, float qy, float qz, uint32_t sub) {
        if (G == 1) {
            scan_rows(pts, rs, rn, qx, qy, qz);
            return;
        }
        static_assert(NR == 3 || NR == 4, "3 or 4 rows");
        const uint32_t c1 = rn[0], c2 = c1 + rn[1], c3 = c2 + rn[2], L = NR == 4 ? c3 + rn[NR - 1] : c3;
        const uint32_t o0 = rs[0], o1 = rs[1] - c1, o2 = rs[2] - c2, o3 = rs[NR - 1] - c3;
        const uint32_t c3e = NR == 4 ? c3 : 0xffffffffu;
        auto addr = [=](uint32_t v) { return cat_addr(v, c1, c2, c3e, o0, o1, o2, o3); };
        uint32_t v = sub;
        constexpr int U = PCP_SCAN_UNROLL;
        for (; v + (U - 1) * G < L; v += U * G) {
            uint32_t k[U];
            float4 p[U];
#pragma unroll
            for (int u = 0; u < U; u++) k[u] = addr(v + u * G);
#pragma unroll
            for (int u = 0; u < U; u++) p[u] = pts[k[u]];
#pragma unroll
            for (int u = 0; u < U; u++) consider(qx, qy, qz, p[u], k[u]);
        }
        for (; v < L; v += G) {
            const uint32_t k = addr(v);
            consider(qx, qy, qz, pts[k], k);
        }
    }
    template <int G>
    __device__ __forceinline__ void merge_group() {
#pragma unroll
        for (int s = 1; s < G; s <<= 1) {
            const float od = __shfl_xor(bd, s, 64);
            const int oj = __shfl_xor(bj, s, 64);
            const uint32_t ok = (uint32_t)__shfl_xor((int)bk, s, 64);
#if PCP_TRACK_BEST
            const float ox = __shfl_xor(px, s, 64), oy = __shfl_xor(py, s, 64), oz = __shfl_xor(pz, s, 64);
#endif
            const bool t = od < bd || (od == bd && oj < bj);
            bd = t ? od : bd;
            bj = t ? oj : bj;
            bk = t ? ok : bk;
#if PCP_TRACK_BEST
            px = t ? ox : px;
            py = t ? oy : py;
            pz = t ? oz : pz;
#endif
        }
    }
    template <typename P>
    __device__ __forceinline__ void fetch(const P* pts) {
        const float4 p = pts[bk];
        px = p.x; py = p.y; pz = p.z;
    }
};

// Exact 1-NN within sqrt(b.bd) by rows of cells: the rows (y,z) that intersect the sphere's
// bounding box are visited nearest-first, and each row is scanned over the x-range of cells
// still within the (shrinking) bound -- one contiguous point range per row on a dense grid.
// Rows and cells are pruned conservatively (margin mc cells, 2e-5 relative on d2), so the
// winner equals an exhaustive lexicographic (d2, index) search.
template <int G = 1>
__device__ __forceinline__ void box_search(const GridDesc& g, const float4* tp, float qx, float qy,
                                           float qz, float mc, Best& b, uint32_t sub = 0) {
    const float fx = cell_f<float>(g, qx, 0), fy = cell_f<float>(g, qy, 1), fz = cell_f<float>(g, qz, 2);
    const int cy = (int)floorf(fy), cz = (int)floorf(fz);
    const float ly = fy - (float)cy, lz = fz - (float)cz;
    const float inv_h2 = g.inv_hf * g.inv_hf;
    const float rc = sqrtf(b.bd * 1.00002f * inv_h2) + mc;  // initial radius in cells
    // G > 1: rows are pruned by the group's bound as of its last merge (every lane of the group
    // then cuts the same x-range, so the strided entries still partition it)
    float gb = b.bd;
    const int ry = (int)ceilf(rc) + 1, rz = ry;
    for (int oz = 0; oz <= 2 * rz; oz++) {
        const int dz = (oz & 1) ? -((oz + 1) >> 1) : (oz >> 1);  // 0, -1, +1, -2, +2, ...
        const int z = cz + dz;
        if (z < 0 || z >= g.n[2]) continue;
        const float gz = dz < 0 ? (lz + (float)(-dz - 1)) : (dz > 0 ? (1.f - lz + (float)(dz - 1)) : 0.f);
        const float gz2 = gz > mc ? (gz - mc) * (gz - mc) : 0.f;
        for (int oy = 0; oy <= 2 * ry; oy++) {
            const int dy = (oy & 1) ? -((oy + 1) >> 1) : (oy >> 1);
            const int y = cy + dy;
            if (y < 0 || y >= g.n[1]) continue;
            const float gy = dy < 0 ? (ly + (float)(-dy - 1)) : (dy > 0 ? (1.f - ly + (float)(dy - 1)) : 0.f);
            const float gyz2 = gz2 + (gy > mc ? (gy - mc) * (gy - mc) : 0.f);
            const float lim = (G == 1 ? b.bd : gb) * 1.00002f * inv_h2 - gyz2;  // remaining x extent^2 (cells)
            if (lim < 0.f) continue;
            const float rx = sqrtf(lim) + mc;
            const int xa = max((int)floorf(fx - rx), 0), xb = min((int)floorf(fx + rx), g.n[0] - 1);
            if (xa > xb) continue;
            if (g.dense) {
                const int64_t c = dense_id(g, xa, y, z);
                b.scan_g<G>(tp, g.cstart[c], g.cstart[c + (xb - xa + 1)], qx, qy, qz, sub);
            } else {
                for (int x = xa; x <= xb; x++) {
                    uint32_t s, e;
                    if (cell_range(g, x, y, z, s, e)) b.scan_g<G>(tp, s, e, qx, qy, qz, sub);
                }
            }
        }
        b.merge_group<G>();  // the group's bound prunes the next plane
        gb = b.bd;
    }
    b.merge_group<G>();
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ int wave_min_i(int v) {
    for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
    return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
    for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
    return v;
}

// Main pass (dense grid).  Wave-autonomous, one query per lane: waves take 64-query chunks
// of the spatially sorted query set (grid-stride, so the 4 waves of a workgroup work on
// adjacent chunks and share L1), transform each query, and scan its 2x2x2 "octant" block
// of cells straight from the x-rows of the dense table.  The octant holds every target
// within (0.5 - mc) cells of the query: a winner with d2 <= cert2 is the exact 1-NN, and
// "nothing within rmax" is certified when rmax^2 <= cert2.  Other queries keep their
// provisional octant winner (a valid upper bound for the exact fallback search) and go to
// the wave's fallback segment (ballot + mbcnt, no atomics).
// Accumulators: per chunk, fp32 products centred on the chunk's first query are summed
// across the wave with DPP adds (no LDS permutes), un-centred in fp64 by one lane and kept
// in LDS -- no accumulator registers, so the kernel fits 8 waves per SIMD.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_add(float v) {
    const int t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWMASK, 0xf, false);
    return v + __int_as_float(t);
}
// full-wave fp32 sum (every lane must be active); the total ends in lane 63
__device__ __forceinline__ float wave_sum_f32(float v) {
    v = dpp_add<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
    v = dpp_add<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
    v = dpp_add<0x141, 0xf>(v);  // row_half_mirror
    v = dpp_add<0x140, 0xf>(v);  // row_mirror
    v = dpp_add<0x142, 0xa>(v);  // row_bcast:15
    v = dpp_add<0x143, 0xc>(v);  // row_bcast:31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Add one chunk's accepted pairs (lanes with ok) to the wave's fp64 accumulators S (LDS):
// fp32 products centred on lane 0's query, summed across the wave and un-centred in fp64
// (wave_acc.hpp: reduce-scatter butterfly, one lane per accumulator; PCP_WAVE_ACC=0 keeps
// the former 23 DPP reductions with lane 0 un-centring).  Every lane of the wave must call
// it (full EXEC).
#ifndef PCP_WAVE_ACC
#define PCP_WAVE_ACC 1
#endif
__device__ __forceinline__ void chunk_accumulate(bool ok, float qx, float qy, float qz, const Best& b,
                                                 double* S, int lane) {
    if (!__ballot(ok)) return;
    const float ccx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qx), 0));
    const float ccy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qy), 0));
    const float ccz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qz), 0));
    const float x0 = ok ? qx - ccx : 0.f, x1 = ok ? qy - ccy : 0.f, x2 = ok ? qz - ccz : 0.f;
    const float p0 = ok ? b.px - ccx : 0.f, p1 = ok ? b.py - ccy : 0.f, p2 = ok ? b.pz - ccz : 0.f;
#if PCP_WAVE_ACC
    const float v[23] = {ok ? 1.f : 0.f, x0, x1, x2, p0, p1, p2,
                         x0 * p0, x0 * p1, x0 * p2, x1 * p0, x1 * p1, x1 * p2, x2 * p0, x2 * p1, x2 * p2,
                         x0 * x0, x0 * x1, x0 * x2, x1 * x1, x1 * x2, x2 * x2, ok ? b.bd : 0.f};
    wave_accumulate(v, S, lane, ccx, ccy, ccz);
#else
    const float nn = wave_sum_f32(ok ? 1.f : 0.f);
    const float A0 = wave_sum_f32(x0), A1 = wave_sum_f32(x1), A2 = wave_sum_f32(x2);
    const float B0 = wave_sum_f32(p0), B1 = wave_sum_f32(p1), B2 = wave_sum_f32(p2);
    const float AB[9] = {wave_sum_f32(x0 * p0), wave_sum_f32(x0 * p1), wave_sum_f32(x0 * p2),
                         wave_sum_f32(x1 * p0), wave_sum_f32(x1 * p1), wave_sum_f32(x1 * p2),
                         wave_sum_f32(x2 * p0), wave_sum_f32(x2 * p1), wave_sum_f32(x2 * p2)};
    const float AA[6] = {wave_sum_f32(x0 * x0), wave_sum_f32(x0 * x1), wave_sum_f32(x0 * x2),
                         wave_sum_f32(x1 * x1), wave_sum_f32(x1 * x2), wave_sum_f32(x2 * x2)};
    const float DD = wave_sum_f32(ok ? b.bd : 0.f);
    if (lane == 0) {  // un-centre in fp64: q = a + c, p = b + c
        const double n = nn, C[3] = {ccx, ccy, ccz}, A[3] = {A0, A1, A2}, B[3] = {B0, B1, B2};
        S[0] += n;
        for (int k = 0; k < 3; k++) { S[1 + k] += A[k] + n * C[k]; S[4 + k] += B[k] + n * C[k]; }
        for (int r = 0; r < 3; r++)
            for (int k = 0; k < 3; k++)
                S[7 + 3 * r + k] += (double)AB[3 * r + k] + A[r] * C[k] + C[r] * B[k] + n * C[r] * C[k];
        const int ir[6] = {0, 0, 0, 1, 1, 2}, ik[6] = {0, 1, 2, 1, 2, 2};
        for (int m = 0; m < 6; m++)
            S[16 + m] += (double)AA[m] + A[ir[m]] * C[ik[m]] + C[ir[m]] * A[ik[m]] + n * C[ir[m]] * C[ik[m]];
        S[22] += DD;
    }
#endif
}

// XCD-blocked work split: workgroups are dealt round-robin over the 8 XCDs, so workgroup b
// runs on XCD b % 8.  The 64-query chunks [0, nch) are cut into np = min(8, grid) contiguous
// parts, one per XCD, and each part is handed out grid-stride to that XCD's waves: spatially
// adjacent chunks then share one L2 (their cell rows and target points) instead of being
// fetched once per XCD.
struct XcdSplit {
    int64_t c0, c1, w, nw;  // this wave's part [c0, c1), its index and the part's wave count
};
__device__ __forceinline__ XcdSplit xcd_split(int64_t nch, int kW) {
    const int np = min(8, (int)gridDim.x);
    const int part = (int)(blockIdx.x % np);
    const int64_t nblk = ((int64_t)gridDim.x - part + np - 1) / np;  // workgroups of this part
    XcdSplit x;
    x.c0 = part * nch / np;
    x.c1 = (part + 1) * nch / np;
    x.w = (int64_t)(blockIdx.x / np) * kW + (threadIdx.x >> 6);
    x.nw = nblk * kW;
    return x;
}

__device__ __forceinline__ void write_wave_partials(double (*s_acc)[kAcc], double* out) {
    __syncthreads();
    if (threadIdx.x < kAcc) {
        double s = 0.0;
        if (threadIdx.x < kAcc - 1)
            for (int w = 0; w < kIcpBlock / 64; w++) s += s_acc[w][threadIdx.x];
        out[threadIdx.x] = s;
    }
}

// Per-lane accumulation: each lane sums its accepted pairs in fp32, centred on the
// (transformed) first query of the wave's current stretch of chunks, into 23 registers; every
// kFlush chunks (and at the end) the wave reduces them with DPP adds and lane 0 un-centres the
// totals in fp64 into the wave's LDS accumulators.  A stretch is at most kFlush * 64
// consecutive sorted queries (a few metres), so the centred fp32 products stay small.
#ifndef PCP_KFLUSH  // chunks per accumulator stretch
#define PCP_KFLUSH 32
#endif
constexpr int kFlush = PCP_KFLUSH;
#ifndef PCP_FLUSH_INLINE  // 1: inline the stretch flush (no call frame spilled to scratch)
#define PCP_FLUSH_INLINE 1
#endif
#if PCP_FLUSH_INLINE
#define PCP_FLUSH_ATTR __attribute__((always_inline))
#else
#define PCP_FLUSH_ATTR __attribute__((noinline))
#endif
struct LaneAcc {
    float v[kAcc - 1];  // n, A(3), B(3), AB(9), AA(6), D  (centred on c)
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int k = 0; k < kAcc - 1; k++) v[k] = 0.f;
    }
    __device__ __forceinline__ void add(float qx, float qy, float qz, float px, float py, float pz, float d2,
                                        float cx, float cy, float cz) {
        const float x[3] = {qx - cx, qy - cy, qz - cz}, p[3] = {px - cx, py - cy, pz - cz};
        v[0] += 1.f;
#pragma unroll
        for (int k = 0; k < 3; k++) { v[1 + k] += x[k]; v[4 + k] += p[k]; }
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int k = 0; k < 3; k++) v[7 + 3 * r + k] = __fmaf_rn(x[r], p[k], v[7 + 3 * r + k]);
        v[16] = __fmaf_rn(x[0], x[0], v[16]);
        v[17] = __fmaf_rn(x[0], x[1], v[17]);
        v[18] = __fmaf_rn(x[0], x[2], v[18]);
        v[19] = __fmaf_rn(x[1], x[1], v[19]);
        v[20] = __fmaf_rn(x[1], x[2], v[20]);
        v[21] = __fmaf_rn(x[2], x[2], v[21]);
        v[22] += d2;
    }
    // whole wave (full EXEC): totals -> S (fp64, un-centred by lane 0).  Not inlined: it runs once
    // per kFlush chunks, and its fp64 temporaries would otherwise raise the loop's register count.
    __device__ PCP_FLUSH_ATTR void flush(double* S, int lane, float cx, float cy, float cz) {
#if PCP_WAVE_ACC
        wave_accumulate(v, S, lane, cx, cy, cz);
#else
        float t[kAcc - 1];
#pragma unroll
        for (int k = 0; k < kAcc - 1; k++) t[k] = wave_sum_f32(v[k]);
        if (lane == 0) {
            const double n = t[0], C[3] = {cx, cy, cz}, A[3] = {t[1], t[2], t[3]}, B[3] = {t[4], t[5], t[6]};
            S[0] += n;
            for (int k = 0; k < 3; k++) { S[1 + k] += A[k] + n * C[k]; S[4 + k] += B[k] + n * C[k]; }
            for (int r = 0; r < 3; r++)
                for (int k = 0; k < 3; k++)
                    S[7 + 3 * r + k] += (double)t[7 + 3 * r + k] + A[r] * C[k] + C[r] * B[k] + n * C[r] * C[k];
            const int ir[6] = {0, 0, 0, 1, 1, 2}, ik[6] = {0, 1, 2, 1, 2, 2};
            for (int m = 0; m < 6; m++)
                S[16 + m] += (double)t[16 + m] + A[ir[m]] * C[ik[m]] + C[ir[m]] * A[ik[m]] + n * C[ir[m]] * C[ik[m]];
            S[22] += t[22];
        }
#endif
        zero();
    }
};

// ---- candidate cache (a Verlet-style neighbour list per query)
// The search that last settled query i left its record: the positions of its kCache nearest
// targets (or fewer) and D, a lower bound on the distance from the query, at that launch's pose
// q_s, to every target point NOT cached.  With q_t the query at the
// current pose and Delta = |q_t - q_s|, every uncached point p has |q_t - p| >= D - Delta
// (triangle inequality).  So if the nearest cached point is closer than D - Delta (with
// relative margins far above the fp32 rounding of d2), it is the exact 1-NN under the
// contract -- the same (d2, index) winner an exhaustive search returns, cached ties included
// -- and the query is settled without a search; the bound moves to D - Delta.
constexpr int kCache = 3;

// The record (per sorted query; the verify pass streams it every launch):
//   wide   (16 B): {c0, c1, c2, dlb}, dlb = bits(D) & ~0xff | (launch & 255) -- D rounded down to
//                  15 mantissa bits (still a lower bound), the slot of the pose history;
//   narrow (12 B, targets < 2^26 - 2): c0 | x0 << 26, c1 | x1 << 26, c2 | x2 << 26 with the 18-bit
//                  word x = (launch & 63) | code(D) << 6, code(D) = D in units of cell / 1024 as a
//                  4-bit exponent and 8-bit mantissa, rounded down (0: D < 1 unit; 0xfff caps D at
//                  ~32 cells).  An empty slot is 2^26 - 1 (above every position and the sentinel).
// A smaller D only sends more queries to the search, so every rounding is down.
struct CacheRec {
    uint32_t c0, c1, c2;  // positions, ~0u = empty slot
    uint32_t slot;        // launch of the search & hist_mask
    float D;
};
constexpr uint32_t kPos26 = (1u << 26) - 1;
constexpr int kHist = 256;  // pose history slots allocated (narrow records use 64 of them)
__device__ __forceinline__ uint32_t dcode12(float D, float inv_unit) {
    const float x = D * inv_unit;
    if (!(x >= 1.f)) return 0u;
    const uint32_t b = __float_as_uint(x);
    const uint32_t e = (b >> 23) - 127u;
    return e >= 15u ? 0xfffu : ((e + 1u) << 8) | ((b >> 15) & 0xffu);
}
__device__ __forceinline__ float ddecode12(uint32_t c, float unit) {
    return c ? __uint_as_float((((c >> 8) + 126u) << 23) | ((c & 0xffu) << 15)) * unit : 0.f;
}
// the raw words of record i (narrow: .w unused)
__device__ __forceinline__ uint4 cache_raw(const IcpArgs& a, int64_t i) {
    if (a.narrow) {
        const uint3 w = *(const uint3*)(a.cand + 3 * i);
        return make_uint4(w.x, w.y, w.z, 0u);
    }
    return ((const uint4*)a.cand)[i];
}
__device__ __forceinline__ CacheRec cache_dec(const IcpArgs& a, const uint4 w) {
    CacheRec r;
    if (a.narrow) {
        auto pos = [](uint32_t v) { const uint32_t c = v & kPos26; return c == kPos26 ? ~0u : c; };
        r.c0 = pos(w.x);
        r.c1 = pos(w.y);
        r.c2 = pos(w.z);
        const uint32_t x = (w.x >> 26) | ((w.y >> 26) << 6) | ((w.z >> 26) << 12);
        r.slot = x & 63u;
        r.D = ddecode12(x >> 6, a.dunit);
    } else {
        r.c0 = w.x;
        r.c1 = w.y;
        r.c2 = w.z;
        r.slot = w.w & 0xffu;
        r.D = __uint_as_float(w.w & ~0xffu);
    }
    return r;
}
__device__ __forceinline__ CacheRec cache_load(const IcpArgs& a, int64_t i) { return cache_dec(a, cache_raw(a, i)); }
__device__ __forceinline__ void cache_store(const IcpArgs& a, int64_t i, uint32_t c0, uint32_t c1, uint32_t c2, float D,
                                            uint32_t launch) {
    if (a.narrow) {
        auto pos = [](uint32_t c) { return c == ~0u ? kPos26 : c; };
        const uint32_t x = (launch & 63u) | (dcode12(D, a.inv_dunit) << 6);
        *(uint3*)(a.cand + 3 * i) =
            make_uint3(pos(c0) | ((x & 63u) << 26), pos(c1) | (((x >> 6) & 63u) << 26), pos(c2) | ((x >> 12) << 26));
    } else {
        ((uint4*)a.cand)[i] = make_uint4(c0, c1, c2, (__float_as_uint(fmaxf(D, 0.f)) & ~0xffu) | (launch & 0xffu));
    }
}

// the cached candidates' winner under the current pose, by (d2, target index)
struct CacheBest {
    float bd = INFINITY;
    int bj = 0x7fffffff;
    uint32_t bk = ~0u;
    float4 P = make_float4(0.f, 0.f, 0.f, 0.f);
};
__device__ __forceinline__ CacheBest cache_best(const float4* tp, const CacheRec& cd, float qx, float qy, float qz) {
    const uint32_t c[3] = {cd.c0, cd.c1, cd.c2};
    float4 p[kCache];
#pragma unroll
    for (int s = 0; s < kCache; s++) p[s] = c[s] != ~0u ? tp[c[s]] : make_float4(0.f, 0.f, 0.f, 0.f);
    CacheBest r;
#pragma unroll
    for (int s = 0; s < kCache; s++) {
        if (c[s] == ~0u) continue;
        const float d2 = icp_d2(qx, qy, qz, p[s]);
        const int id = __float_as_int(p[s].w);
        if (d2 < r.bd || (d2 == r.bd && id < r.bj)) {
            r.bd = d2;
            r.bj = id;
            r.bk = c[s];
            r.P = p[s];
        }
    }
    return r;
}

// 16-byte record of a table by element index.  The byte offset is 32-bit (so the load can use
// the saddr + 32-bit VGPR offset form): pcp_icp_check_sizes() keeps every table this reads
// (the fp32 target incl. its far sentinel) below 2^28 records = 4 GB.
template <typename V>
__device__ __forceinline__ V ld16(const V* base, uint32_t idx) {
    return *(const V*)((const char*)base + (size_t)(idx * 16u));
}

// ---- verify pass (every query, every launch after the first)
// Settles a query from its cache (above): q_s is recomputed exactly from the pose of the
// launch s that searched it (pose history in LDS), so the bound is |q_t - q_s| (not a sum of
// steps) and nothing is written for a settled query.  "No correspondence" is settled the same
// way when the nearest cached point is beyond rmax.  Everything else goes to the search list
// (per-wave segments, compacted afterwards).  Wave w owns the contiguous chunk range
// [w*nch/nwaves, (w+1)*nch/nwaves) of the sorted queries; accumulation is per lane (fp32,
// centred on the stretch's first query).
__global__ void __launch_bounds__(kIcpBlock, PCP_VER_WAVES) k_icp_verify(IcpArgs a) {
    __shared__ float4 s_pose[kHist][3];
    constexpr int kW = kIcpBlock / 64;
    __shared__ double s_acc[kW][kAcc];
    for (int k = threadIdx.x; k < kHist * 3; k += blockDim.x)
        s_pose[k / 3][k % 3] = ((const float4*)a.pose_hist)[k];
    load_pose(a);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * kW + wid;
    const int64_t nch = (a.nq + 63) / 64;
    // contiguous ranges: wave w owns chunks [w*nch/nwaves, (w+1)*nch/nwaves)
    const int64_t nwaves = (int64_t)gridDim.x * kW;
    const int64_t cstart_ = gw * nch / nwaves;
    const int64_t nsteps = (gw + 1) * nch / nwaves - cstart_;
    if (lane < kAcc) s_acc[wid][lane] = 0.0;
    __syncthreads();
    uint32_t svn = 0;
    LaneAcc acc;
    acc.zero();
    const float r2m = a.r2 * 1.0003f;
    // software pipeline: the query, cache and bound words two chunks ahead, the cached points'
    // gathers one chunk ahead (this chunk's were issued during the previous one)
    const uint4 none = make_uint4(~0u, ~0u, ~0u, ~0u);
    auto raw = [&](int64_t k, float4& q, uint4& cd) {
        const int64_t i = (cstart_ + k) * 64 + lane;
        if (k < nsteps && i < a.nq) {
            q = ldq(a, i);
            cd = cache_raw(a, i);
        } else {
            q = make_float4(0.f, 0.f, 0.f, 0.f);
            cd = none;
            cd.w = 0u;
        }
    };
    auto gather = [&](const uint4 cd, float4& p0, float4& p1, float4& p2) {
        // an empty slot reads the far sentinel tp[ntp]: d2 = inf
        const CacheRec r = cache_dec(a, cd);
        p0 = ld16(a.tp, min(r.c0, a.ntp));
        p1 = ld16(a.tp, min(r.c1, a.ntp));
        p2 = ld16(a.tp, min(r.c2, a.ntp));
    };
    float4 q1, q2;
    uint4 c1_, c2_;
    float4 g0, g1, g2;
    raw(0, q1, c1_);
    raw(1, q2, c2_);
    gather(c1_, g0, g1, g2);
    for (int64_t k0 = 0; k0 < nsteps; k0 += kFlush) {  // stretches of kFlush chunks
        const int64_t k1 = min(k0 + (int64_t)kFlush, nsteps);
        // centre: the stretch's first query under the current pose (wave-uniform)
        float ccx, ccy, ccz;
        xform(a, ldq(a, (cstart_ + k0) * 64), ccx, ccy, ccz);
        ccx = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(ccx)));
        ccy = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(ccy)));
        ccz = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(ccz)));
        for (int64_t k = k0; k < k1; k++) {
            const int64_t i = (cstart_ + k) * 64 + lane;
            const bool valid = i < a.nq;
            const float4 qq = q1;
            const CacheRec rec = cache_dec(a, c1_);
            const float4 p0 = g0, p1 = g1, p2 = g2;
            // issue chunk c+1's gathers and chunk c+2's words before using chunk c's
            gather(c2_, g0, g1, g2);
            q1 = q2;
            c1_ = c2_;
            raw(k + 2, q2, c2_);
            float qx, qy, qz;
            xform(a, qq, qx, qy, qz);
            // winner among the cached points by (d2, target index); an empty slot never wins
            float m = INFINITY, px = 0.f, py = 0.f, pz = 0.f;
            int mj = 0x7fffffff;
            auto take = [&](const float4 p) {
                const float e = icp_d2(qx, qy, qz, p);
                const int id = __float_as_int(p.w);
                const bool t = e < m || (e == m && id < mj);
                m = t ? e : m;
                mj = t ? id : mj;
                px = t ? p.x : px;
                py = t ? p.y : py;
                pz = t ? p.z : pz;
            };
            take(p0);
            take(p1);
            take(p2);
            // the query at the pose of its last search
            const uint32_t sl = rec.slot;
            const float4 A = s_pose[sl][0], B = s_pose[sl][1], C = s_pose[sl][2];
            const float ex = qx - __fmaf_rn(A.z, qq.z, __fmaf_rn(A.y, qq.y, __fmaf_rn(A.x, qq.x, C.y)));
            const float ey = qy - __fmaf_rn(B.y, qq.z, __fmaf_rn(B.x, qq.y, __fmaf_rn(A.w, qq.x, C.z)));
            const float ez = qz - __fmaf_rn(C.x, qq.z, __fmaf_rn(B.w, qq.y, __fmaf_rn(B.z, qq.x, C.w)));
            const float delta = sqrtf(__fmaf_rn(ez, ez, __fmaf_rn(ey, ey, ex * ex))) * 1.00001f + 1e-7f;
            const float lb = rec.D * 0.99998f - delta;  // every uncached point is >= lb
            // the nearest cached point is the exact 1-NN (it beats lb), or nothing is within rmax
            const float thr = fminf(m * 1.0003f, r2m);
            bool ok = valid && ((a.launch - sl) & a.hist_mask) < a.max_age && lb > 0.f && thr + 1e-12f < lb * lb;
            ok = ok && !(a.dbg & kDbgNoVerify);
            const bool srch = valid && !ok;
            const uint64_t msk = __ballot(srch);
            if (srch) {
                const uint32_t pos = svn + __builtin_amdgcn_mbcnt_hi((uint32_t)(msk >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)msk, 0u));
                a.sv[gw * a.sv_seg + pos] = (int32_t)i;
            }
            svn += (uint32_t)__popcll(msk);
            if (ok && m <= a.r2 && !(a.dbg & kDbgNoAccum)) acc.add(qx, qy, qz, px, py, pz, m, ccx, ccy, ccz);
        }
        acc.flush(s_acc[wid], lane, ccx, ccy, ccz);
    }
    if (lane == 0) {
        a.sv_count[gw] = svn;
    }
    write_wave_partials(s_acc, a.partials + (int64_t)blockIdx.x * kAcc);
}

// running 3-NN (kCache = 3): d0 <= d1 <= d2 with positions, d3 = the 4th smallest d2 scanned
struct Top3 {
    float d0 = INFINITY, d1 = INFINITY, d2 = INFINITY, d3 = INFINITY;
    uint32_t p0 = ~0u, p1 = ~0u, p2 = ~0u;
    // insertion as three independent compare-swaps from the bottom (flat selects: a nested
    // select form was lowered to branches and register moves)
    __device__ __forceinline__ void consider(float qx, float qy, float qz, const float4 p, uint32_t k) {
        float x = icp_d2(qx, qy, qz, p);
        uint32_t kx = k;
        cswap(d2, p2, x, kx);
        d3 = fmin_nn(d3, x);  // what fell out of the top 3
        cswap(d1, p1, d2, p2);
        cswap(d0, p0, d1, p1);
    }
    // (a, pa) <- the smaller of (a, pa), (b, pb) by d2; (b, pb) <- the larger (ties keep a)
    __device__ __forceinline__ static void cswap(float& a, uint32_t& pa, float& b, uint32_t& pb) {
        const bool t = b < a;
        const float lo = fmin_nn(a, b), hi = fmax_nn(a, b);
        const uint32_t ql = t ? pb : pa, qh = t ? pa : pb;
        a = lo;
        b = hi;
        pa = ql;
        pb = qh;
    }
    __device__ __forceinline__ void scan4(const float4* pts, const uint32_t (&rs)[4], const uint32_t (&rn)[4],
                                          float qx, float qy, float qz) {
        const uint32_t c1 = rn[0], c2 = c1 + rn[1], c3 = c2 + rn[2], L = c3 + rn[3];
        const uint32_t o0 = rs[0], o1 = rs[1] - c1, o2 = rs[2] - c2, o3 = rs[3] - c3;
        auto addr = [=](uint32_t v) { return cat_addr(v, c1, c2, c3, o0, o1, o2, o3); };
        constexpr int U = PCP_SCAN_UNROLL;
        uint32_t v = 0;
        for (; v + U <= L; v += U) {
            uint32_t k[U];
            float4 p[U];
#pragma unroll
            for (int u = 0; u < U; u++) k[u] = addr(v + u);
#pragma unroll
            for (int u = 0; u < U; u++) p[u] = pts[k[u]];
#pragma unroll
            for (int u = 0; u < U; u++) consider(qx, qy, qz, p[u], k[u]);
        }
        for (; v < L; v++) {
            const uint32_t k = addr(v);
            consider(qx, qy, qz, pts[k], k);
        }
    }
};

// running 3-NN on packed keys: key = (bits(d2) & ~255) | v, v the candidate's index in the
// concatenated octant list (< 256).  Non-negative floats order like their bits, so a
// v_med3_u32 network keeps the 4 smallest keys -- values and list indices together -- in 4 VALU
// ops per candidate (the compare-swap form, Top3, needs 16).  The truncated d2 only chooses
// WHICH points are cached: the winner among them is decided on the exact d2 afterwards, and
// the 4th key with its low byte cleared bounds the d2 of every scanned point not kept (an
// uncached point's key is >= t3, so its d2 bits are >= t3 & ~255).
constexpr uint32_t kKeyMax = 0x7f7fffffu;  // FLT_MAX: above every real key
constexpr uint32_t kMaxOctList = 256;       // list indices that fit the key's low byte
// median of three u32 (one v_med3_u32; the float form adds canonicalizing ops on bit-cast keys)
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// position of candidate v of the concatenated rows, or the far sentinel `sent` past the list
__device__ __forceinline__ uint32_t cat_addr_l(uint32_t v, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t L,
                                               uint32_t o0, uint32_t o1, uint32_t o2, uint32_t o3, uint32_t sent) {
    const uint32_t d = v < L ? o3 : sent - v;
    const uint32_t c = v < c3 ? o2 : d;
    const uint32_t b = v < c2 ? o1 : c;
    return v + (v < c1 ? o0 : b);
}
__device__ __forceinline__ int wave_max_u(int v) {
    v = max(v, __shfl_xor(v, 1, 64));
    v = max(v, __shfl_xor(v, 2, 64));
    v = max(v, __shfl_xor(v, 4, 64));
    v = max(v, __shfl_xor(v, 8, 64));
    v = max(v, __shfl_xor(v, 16, 64));
    v = max(v, __shfl_xor(v, 32, 64));
    return v;
}
struct Top3P {
    uint32_t t0 = kKeyMax, t1 = kKeyMax, t2 = kKeyMax, t3 = kKeyMax;
    __device__ __forceinline__ void consider(float qx, float qy, float qz, const float4 p, uint32_t v) {
        const float d = icp_d2(qx, qy, qz, p);
        const uint32_t x = (__float_as_uint(d) & ~0xffu) | v;
        t3 = umed3(t2, t3, x);
        t2 = umed3(t1, t2, x);
        t1 = umed3(t0, t1, x);
        t0 = min(t0, x);
    }
    // the wave's lists with a uniform trip count (lanes past their own list read the far
    // sentinel: d2 = inf, never kept), U loads per step, the next step's loads issued before
    // this step's keys are formed (software pipeline: two batches in flight).  With G lanes per
    // query, lane `sub` of the group takes list entries sub, sub + G, sub + 2G, ...: the group's
    // loads of one step are G consecutive records of a row (one or two cache lines), so a wave
    // instruction touches ~64 / G lines instead of 64 (what bounds the sparse search lists).
    template <int G>
    __device__ __forceinline__ void scan4(const float4* pts, uint32_t sent, const uint32_t (&rs)[4],
                                          const uint32_t (&rn)[4], uint32_t Lw, float qx, float qy, float qz,
                                          uint32_t sub) {
        const uint32_t c1 = rn[0], c2 = c1 + rn[1], c3 = c2 + rn[2], L = c3 + rn[3];
        const uint32_t o0 = rs[0], o1 = rs[1] - c1, o2 = rs[2] - c2, o3 = rs[3] - c3;
        auto lv = [=](uint32_t v) { return v * G + sub; };  // this lane's v-th list entry
        auto addr = [=](uint32_t v) { return cat_addr_l(lv(v), c1, c2, c3, L, o0, o1, o2, o3, sent); };
        const uint32_t Lg = (Lw + G - 1) / G;
        constexpr int U = 4;
        float4 A[U], B[U];
#pragma unroll
        for (int u = 0; u < U; u++) A[u] = ld16(pts, addr(u));
        for (uint32_t v = 0; v < Lg; v += 2 * U) {
            // two register sets, no copies: B's loads are in flight while A's keys are formed
#pragma unroll
            for (int u = 0; u < U; u++) B[u] = ld16(pts, addr(v + U + u));
            __builtin_amdgcn_sched_barrier(0);  // keep B's loads ahead of A's keys
#pragma unroll
            for (int u = 0; u < U; u++) consider(qx, qy, qz, A[u], lv(v + u));
            if (v + U >= Lg) break;
#pragma unroll
            for (int u = 0; u < U; u++) A[u] = ld16(pts, addr(v + 2 * U + u));
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; u++) consider(qx, qy, qz, B[u], lv(v + U + u));
        }
    }
    // the G lanes of a query merge their 4 smallest keys: per butterfly step the 4 smallest of
    // two ascending lists are min(t_i, u_{3-i}) (a bitonic sequence), sorted by two stages of
    // compare-exchange.  Keys of one query are distinct (the list index is in the low byte)
    // except kKeyMax.  Afterwards every lane of the group holds the group's t0..t3.
    template <int G>
    __device__ __forceinline__ void merge_group() {
#pragma unroll
        for (int s = 1; s < G; s <<= 1) {
            const uint32_t u0 = xor_lane(t0, s), u1 = xor_lane(t1, s), u2 = xor_lane(t2, s), u3 = xor_lane(t3, s);
            const uint32_t c0 = min(t0, u3), c1 = min(t1, u2), c2 = min(t2, u1), c3 = min(t3, u0);
            const uint32_t l02 = min(c0, c2), h02 = max(c0, c2), l13 = min(c1, c3), h13 = max(c1, c3);
            t0 = min(l02, l13);
            t1 = max(l02, l13);
            t2 = min(h02, h13);
            t3 = max(h02, h13);
        }
    }
    // lane ^ s inside a quad by DPP quad_perm (s = 1, 2), else a bpermute
    __device__ __forceinline__ static uint32_t xor_lane(uint32_t v, int s) {
        if (s == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);  // [1,0,3,2]
        if (s == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);  // [2,3,0,1]
        return (uint32_t)__shfl_xor((int)v, s, 64);
    }
};

// ---- search pass (the verify pass's list; every query at the first launch)
// One query per lane, 64-query chunks grid-stride over the list.  Each query scans its whole
// 2x2x2 "octant" block of cells (the four x-rows [floor(f - 1/2), +1]) keeping its 3 nearest.
// The octant holds every target within m = the query's distance to its faces (>= 1/2 cell,
// less the margin).  The nearest is the exact 1-NN when d0 <= m^2 and d0 < d3 (every point
// tied with it is cached, and the cache order by index decides); "nothing within rmax" is
// certified when rmax <= m.  The cache is refreshed either way (D = min(d3, m) bounds every
// uncached point); unsettled queries go to the fallback list.
//
// The scan keeps packed (d2, list index) keys (Top3P, 4 VALU ops per candidate) with a
// wave-uniform trip count; a chunk with a list longer than 256 candidates (the key's low byte)
// uses the compare-swap form (Top3).  Both end in the same OctResult: the exact (d2, index)
// winner among the 3 kept, its coordinates, the 3 cached positions and the first-uncached bound.
struct OctResult {
    float d0 = INFINITY;       // exact d2 of the winner among the kept points
    uint32_t win = ~0u;        // its sorted position (~0u: nothing scanned)
    float wx = 0.f, wy = 0.f, wz = 0.f;
    uint32_t c0 = ~0u, c1 = ~0u, c2 = ~0u;  // the cache: positions of the 3 kept points
    float dnext = INFINITY;    // lower bound on the d2 of every scanned point not kept
};

__device__ __forceinline__ void take_exact(OctResult& o, const float4 p, uint32_t pos, float qx, float qy, float qz,
                                           int& wj) {
    const float e = icp_d2(qx, qy, qz, p);
    const int id = __float_as_int(p.w);
    const bool t = pos != ~0u && (e < o.d0 || (e == o.d0 && id < wj));
    o.d0 = t ? e : o.d0;
    wj = t ? id : wj;
    o.win = t ? pos : o.win;
    o.wx = t ? p.x : o.wx;
    o.wy = t ? p.y : o.wy;
    o.wz = t ? p.z : o.wz;
}

// v of lane (group base + src) of this lane's G-lane group (groups of G consecutive lanes; G = 2
// and 4 by DPP quad permutes, inside the quad, no LDS)
template <int G>
__device__ __forceinline__ uint32_t grp_bcast(uint32_t v, int src) {
    if constexpr (G == 1) return v;
    if constexpr (G == 2) {  // quad_perm [s, s, 2 + s, 2 + s]
        return src == 0 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0 | 0 << 2 | 2 << 4 | 2 << 6, 0xf, 0xf, false)
                        : (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 1 | 1 << 2 | 3 << 4 | 3 << 6, 0xf, 0xf, false);
    }
    if constexpr (G == 4) {  // quad_perm [s, s, s, s]
        switch (src) {
            case 0: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xf, 0xf, false);
            case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x55, 0xf, 0xf, false);
            case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xAA, 0xf, 0xf, false);
            default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xFF, 0xf, 0xf, false);
        }
    }
    const int lane = (int)(threadIdx.x & 63);
    return (uint32_t)__shfl((int)v, (lane & ~(G - 1)) | src, 64);
}
template <int G>
__device__ __forceinline__ uint32_t grp_xor(uint32_t v, int s) {
    if (s == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);  // [1,0,3,2]
    if (s == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);  // [2,3,0,1]
    return (uint32_t)__shfl_xor((int)v, s, 64);
}

// The octant's 4 x-rows (y = by + (r & 1), z = bz + (r >> 1), cells [xa, xb], xb - xa + 1 = 1 or
// 2): each row's point range [rs, rs + rn) from the cell starts.  A row's start and end are two
// of the three consecutive words at its first cell, loaded as one 12-byte vector (the cell table
// carries a pad word past its end for that).  With G lanes per query the group's lanes load
// different rows (lane sub: rows sub, sub + G, ...) and exchange them inside the group, so a wave
// issues 4 / G row loads instead of 8 (the loads of a sparse search list each touch a line per
// query: what bounds those launches, TA busy ~75 %).
template <int G>
__device__ __forceinline__ void octant_rows(const GridDesc& g, bool scanq, int bx, int by, int bz, uint32_t sub,
                                            uint32_t (&rs)[4], uint32_t (&rn)[4]) {
    const int xa = max(bx, 0), xb = min(bx + 1, g.n[0] - 1);
    constexpr int PER = G >= 4 ? 1 : 4 / G;  // rows this lane loads
    uint32_t ls[PER], le[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int r = (int)sub + k * G;
        const int y = by + (r & 1), z = bz + (r >> 1);
        const bool in = scanq && r < 4 && xa <= xb && y >= 0 && y < g.n[1] && z >= 0 && z < g.n[2];
        uint3 t = make_uint3(0u, 0u, 0u);
        if (in) t = *(const uint3*)(g.cstart + dense_id(g, xa, y, z));
        ls[k] = t.x;
        le[k] = xb > xa ? t.z : t.y;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint32_t s0 = G == 1 ? ls[r] : grp_bcast<G>(ls[(r / G) % PER], r % G);
        const uint32_t e0 = G == 1 ? le[r] : grp_bcast<G>(le[(r / G) % PER], r % G);
        rs[r] = s0;
        rn[r] = e0 - s0;
    }
}

// packed-key scan (every lane's list < 256 candidates); G lanes per query share its list.  The
// exact re-rank of the 3 kept points: with G > 1 the group's lanes gather different kept points
// and reduce the exact (d2, index) winner inside the group (1 or 2 gathers per lane, not 3).
template <int G>
__device__ __forceinline__ OctResult octant_packed(const IcpArgs& a, const uint32_t (&rs)[4], const uint32_t (&rn)[4],
                                                   uint32_t Lw, float qx, float qy, float qz, uint32_t sub) {
    Top3P k;
    k.scan4<G>(a.tp, a.ntp, rs, rn, Lw, qx, qy, qz, sub);
    k.merge_group<G>();
    const uint32_t c1 = rn[0], c2 = c1 + rn[1], c3 = c2 + rn[2], L = c3 + rn[3];
    const uint32_t o0 = rs[0], o1 = rs[1] - c1, o2 = rs[2] - c2, o3 = rs[3] - c3;
    OctResult o;
    o.c0 = k.t0 != kKeyMax ? cat_addr_l(k.t0 & 0xffu, c1, c2, c3, L, o0, o1, o2, o3, a.ntp) : ~0u;
    o.c1 = k.t1 != kKeyMax ? cat_addr_l(k.t1 & 0xffu, c1, c2, c3, L, o0, o1, o2, o3, a.ntp) : ~0u;
    o.c2 = k.t2 != kKeyMax ? cat_addr_l(k.t2 & 0xffu, c1, c2, c3, L, o0, o1, o2, o3, a.ntp) : ~0u;
    int wj = 0x7fffffff;
    if constexpr (G == 1) {
        const float4 p0 = ld16(a.tp, min(o.c0, a.ntp)), p1 = ld16(a.tp, min(o.c1, a.ntp)),
                     p2 = ld16(a.tp, min(o.c2, a.ntp));
        take_exact(o, p0, o.c0, qx, qy, qz, wj);
        take_exact(o, p1, o.c1, qx, qy, qz, wj);
        take_exact(o, p2, o.c2, qx, qy, qz, wj);
    } else {
        constexpr int PER = G >= 3 ? 1 : 2;  // kept points per lane: G = 2: lane 0 {c0, c2}, lane 1 {c1}
#pragma unroll
        for (int s = 0; s < PER; s++) {
            const uint32_t kslot = sub + (uint32_t)(s * G);
            const uint32_t c = kslot == 0 ? o.c0 : (kslot == 1 ? o.c1 : (kslot == 2 ? o.c2 : ~0u));
            take_exact(o, ld16(a.tp, min(c, a.ntp)), c, qx, qy, qz, wj);
        }
        // the group's winner by (d2, index): butterfly over the group (every lane ends with it)
#pragma unroll
        for (int m = 1; m < G; m <<= 1) {
            const float od = __uint_as_float(grp_xor<G>(__float_as_uint(o.d0), m));
            const int oj = (int)grp_xor<G>((uint32_t)wj, m);
            const uint32_t ow = grp_xor<G>(o.win, m);
            const float ox = __uint_as_float(grp_xor<G>(__float_as_uint(o.wx), m));
            const float oy = __uint_as_float(grp_xor<G>(__float_as_uint(o.wy), m));
            const float oz = __uint_as_float(grp_xor<G>(__float_as_uint(o.wz), m));
            const bool t = ow != ~0u && (o.win == ~0u || od < o.d0 || (od == o.d0 && oj < wj));
            o.d0 = t ? od : o.d0;
            wj = t ? oj : wj;
            o.win = t ? ow : o.win;
            o.wx = t ? ox : o.wx;
            o.wy = t ? oy : o.wy;
            o.wz = t ? oz : o.wz;
        }
    }
    o.dnext = k.t3 == kKeyMax ? INFINITY : __uint_as_float(k.t3 & ~0xffu);
    return o;
}

// compare-swap scan (a chunk with a list of 256 or more candidates)
__device__ __noinline__ OctResult octant_exact(const IcpArgs& a, uint32_t rs0, uint32_t rs1, uint32_t rs2, uint32_t rs3,
                                               uint32_t rn0, uint32_t rn1, uint32_t rn2, uint32_t rn3, float qx, float qy,
                                               float qz) {
    const uint32_t rs[4] = {rs0, rs1, rs2, rs3}, rn[4] = {rn0, rn1, rn2, rn3};
    Top3 b;
    b.scan4(a.tp, rs, rn, qx, qy, qz);
    OctResult o;
    o.c0 = b.p0;
    o.c1 = b.p1;
    o.c2 = b.p2;
    const float4 p0 = ld16(a.tp, min(b.p0, a.ntp)), p1 = ld16(a.tp, min(b.p1, a.ntp)), p2 = ld16(a.tp, min(b.p2, a.ntp));
    int wj = 0x7fffffff;
    take_exact(o, p0, o.c0, qx, qy, qz, wj);
    take_exact(o, p1, o.c1, qx, qy, qz, wj);
    take_exact(o, p2, o.c2, qx, qy, qz, wj);
    o.dnext = b.d3;
    return o;
}

// G lanes per query (G = 1: one query per lane; G > 1: the G lanes of a group split the query's
// list, merge their keys, and only the group's first lane writes, accumulates and lists).  A
// chunk is 64 / G queries.  G > 1 serves the sparse search lists of later launches, whose
// lanes no longer share candidate lines.
constexpr int kOctW = kIcpBlock / 64;
template <int G>
__device__ __forceinline__ void octant_run(const IcpArgs& a, const int32_t* list, int64_t n,
                                           double (*s_acc)[kAcc]) {
    constexpr int kW = kOctW;
    constexpr int QPC = 64 / G;  // queries per chunk
    const GridDesc& g = a.g;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int slot = lane / G;
    const uint32_t sub = (uint32_t)(lane % G);
    const bool lead = sub == 0;
    const int64_t gw = (int64_t)blockIdx.x * kW + wid;  // global wave id = fallback segment
    uint32_t fbn = 0;  // wave-uniform count of this wave's fallback entries
    const int64_t nwaves = (int64_t)gridDim.x * kW;
    int64_t in_ = 0;
    float4 qn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gw * QPC + slot < n) {
        in_ = list ? (int64_t)list[gw * QPC + slot] : gw * QPC + slot;
        qn = ldq(a, in_);
    }
    for (int64_t c = gw; c * QPC < n; c += nwaves) {  // grid-stride (an XCD split measured slower here)
        const int64_t j = c * QPC + slot;
        const bool valid = j < n;
        const int64_t i = in_;
        const float4 qraw = qn;
        if (j + QPC * nwaves < n) {  // prefetch the next chunk's query
            in_ = list ? (int64_t)list[j + QPC * nwaves] : j + QPC * nwaves;
            qn = ldq(a, in_);
        }
        float qx = 0.f, qy = 0.f, qz = 0.f, fx = 0.f, fy = 0.f, fz = 0.f, dout = 0.f;
        int bx = 0, by = 0, bz = 0;
        bool outside = true;
        if (valid) {
            xform(a, qraw, qx, qy, qz);
            fx = cell_f<float>(g, qx, 0), fy = cell_f<float>(g, qy, 1), fz = cell_f<float>(g, qz, 2);
            bx = (int)floorf(fx - a.rho), by = (int)floorf(fy - a.rho), bz = (int)floorf(fz - a.rho);
            // a query farther than rmax from the grid's box (a target-sharded rank: the queries
            // of the other shards) is settled "no correspondence" without a scan, with D = that
            // distance (every target lies inside the box)
            const float ox = fmaxf(fmaxf(-fx, fx - (float)g.n[0]), 0.f);
            const float oy = fmaxf(fmaxf(-fy, fy - (float)g.n[1]), 0.f);
            const float oz = fmaxf(fmaxf(-fz, fz - (float)g.n[2]), 0.f);
            dout = fmaxf(sqrtf(__fmaf_rn(oz, oz, __fmaf_rn(oy, oy, ox * ox))) - a.mc, 0.f) * g.hf;
            outside = dout * dout > a.r2 * 1.0001f;
        }
        const bool scanq = !outside;
        uint32_t rs[4], rn[4];
        octant_rows<G>(g, scanq, bx, by, bz, sub, rs, rn);
        const uint32_t len = rn[0] + rn[1] + rn[2] + rn[3];
        const uint32_t Lw = (uint32_t)__builtin_amdgcn_readfirstlane(wave_max_u((int)len));  // wave-uniform
        OctResult o;
        if (!(a.dbg & kDbgNoScan)) {
            if (Lw <= kMaxOctList)
                o = octant_packed<G>(a, rs, rn, Lw, qx, qy, qz, sub);
            else
                o = octant_exact(a, rs[0], rs[1], rs[2], rs[3], rn[0], rn[1], rn[2], rn[3], qx, qy, qz);
        }
        bool settled = false, found = false;
        if (valid) {
            // this query's certified radius (cells): its distance to the nearest face of the
            // 2x2x2 block (>= 0.5 cell), less the margin
            const float m = fminf(fminf(fminf(fx - (float)bx, (float)(bx + 2) - fx),
                                        fminf(fy - (float)by, (float)(by + 2) - fy)),
                                  fminf(fz - (float)bz, (float)(bz + 2) - fz)) - a.mc;
            const float rr = m * g.hf;
            const float cert2 = fmaxf(a.cert2, rr * rr * (1.f - 2e-5f));
            found = o.d0 <= a.r2;
            settled = (found ? (o.d0 < o.dnext && o.d0 <= cert2) : a.r2 <= cert2) || outside ||
                      (a.dbg & kDbgNoFallback);
            // the cache: the 3 nearest; settled: D bounds every uncached point for the verify
            // pass.  Unsettled: the fallback pass (which overwrites the cache) gets the
            // octant's first uncached d2 instead.
            // (unsettled: the message is the octant's first uncached distance, rounded down)
            const float D = outside ? dout * 0.9999f
                                    : (settled ? fminf(sqrtf(o.dnext), (m > 0.f ? m : 0.f) * g.hf) * 0.9999f
                                               : sqrtf(o.dnext) * 0.99999f);
            if (lead) cache_store(a, i, o.c0, o.c1, o.c2, D, a.launch);
        }
        // ---- fallback list (ballot + mbcnt, no atomics) and accumulators
        const bool fb = valid && lead && !settled;
        const uint64_t fbm = __ballot(fb);
        if (fb) {
            const uint32_t pos = fbn + __builtin_amdgcn_mbcnt_hi((uint32_t)(fbm >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)fbm, 0u));
            a.fb[gw * a.fb_seg + pos] = (int32_t)i;
        }
        fbn += (uint32_t)__popcll(fbm);
        const bool acc_ok = valid && lead && settled && found && !(a.dbg & kDbgNoAccum);
        const Best w{o.d0, 0, o.win, o.wx, o.wy, o.wz};
        chunk_accumulate(acc_ok, qx, qy, qz, w, s_acc[wid], lane);
    }
    if (lane == 0) {  // every wave of the grid writes its count: no zeroing pass needed
        a.fb_count[gw] = fbn;
    }
}

// Lanes per query by the list's density (measured per launch on the C4 bench registration,
// tools/gpu_octg_ab.sh): dense lists share candidate lines between neighbouring queries and
// want one lane each; sparse ones want the group form.
__device__ __forceinline__ int octant_lanes(int64_t n, int64_t nq) {
    if (n * 100 > nq * 36) return 1;
    if (n * 100 > nq * 8) return 2;
    return 4;
}

// MINW: the first (dense) launch runs at PCP_OCT_WAVES waves/SIMD; the search lists of later
// launches at PCP_OCT_WAVES_LIST, whose larger register budget measured faster on them.  A grid
// smaller than the partial rows / list segments sized for the first launch zeroes the rest.
template <int MINW>
__global__ void __launch_bounds__(kIcpBlock, MINW) k_icp_octant(IcpArgs a, const int32_t* list,
                                                                 const uint32_t* list_n) {
    load_pose(a);
    __shared__ double s_acc[kOctW][kAcc];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t n = list ? (int64_t)*list_n : a.nq;
    if (lane < kAcc) s_acc[wid][lane] = 0.0;
    const int G = a.oct_g ? a.oct_g : octant_lanes(n, a.nq);  // uniform over the grid
    if (G == 1)
        octant_run<1>(a, list, n, s_acc);
    else if (G == 2)
        octant_run<2>(a, list, n, s_acc);
    else if (G == 4)
        octant_run<4>(a, list, n, s_acc);
    else
        octant_run<8>(a, list, n, s_acc);
    write_wave_partials(s_acc, a.partials + (int64_t)blockIdx.x * kAcc);
    for (int64_t r = gridDim.x + blockIdx.x; r < a.nb_fast; r += gridDim.x)
        if (threadIdx.x < kAcc) a.partials[r * kAcc + threadIdx.x] = 0.0;
    if (lane == 0) {
        const int64_t nw = (int64_t)gridDim.x * kOctW;
        for (int64_t sg = nw + (int64_t)blockIdx.x * kOctW + wid; sg < a.nseg; sg += nw) {
            a.fb_count[sg] = 0u;
        }
    }
}

// Fallback / general pass: exact box search (dense or sparse grid), starting from the
// octant pass's provisional winner when it has one.  Queries come from the compacted
// fallback list (or are all queries when ring_all is set, i.e. on a sparse grid); waves
// take 64-entry chunks grid-stride and accumulate like the octant pass.
// G lanes per query: the lanes of a query split its rows (Best::scan_rows_g / scan_g) and
// merge after each plane; the group's first lane writes and accumulates.  Measured per launch
// (profiles/r02_ring): the short fallback lists of later launches are latency-bound and run
// ~35 % faster with G = 4, while the long early lists (wide "nothing within rmax" boxes of
// short rows, whose per-row bookkeeping G lanes would repeat) want one lane per query.
// PCP_RING_G = 0 picks G on the device from the list's length (ring_lanes), else fixes it.
#ifndef PCP_RING_G
#define PCP_RING_G 0
#endif
__device__ __forceinline__ int ring_lanes(int64_t n, int64_t nq) {
    if (n * 1000 > nq) return 1;
    if (n * 8000 > nq) return 2;
    return 4;
}
template <int G>
__device__ __forceinline__ void ring_run(IcpArgs& a, double (*s_acc)[kAcc], const int32_t* list, const uint32_t* list_n) {
    constexpr int kW = kIcpBlock / 64;
    constexpr int QPC = 64 / G;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t sub = (uint32_t)(lane % G);
    const bool lead = sub == 0;
    const int64_t n = a.ring_all ? a.nq : (int64_t)*list_n;
    const XcdSplit xs = xcd_split((n + QPC - 1) / QPC, kW);
    for (int64_t c = xs.c0 + xs.w; c < xs.c1; c += xs.nw) {
        const int64_t j = c * QPC + lane / G;
        const bool valid = j < n;
        Best b{a.r2, 0x7fffffff, 0u, 0.f, 0.f, 0.f};
        float qx = 0.f, qy = 0.f, qz = 0.f;
        int64_t i = 0;
        if (valid) {
            i = a.ring_all ? j : list[j];
            xform(a, ldq(a, i), qx, qy, qz);
            // provisional: the cache's best (refreshed by the search pass), an upper bound
            const CacheRec cd = cache_load(a, i);
            const CacheBest cbst = cache_best(a.tp, cd, qx, qy, qz);
            if (cbst.bd <= b.bd) {
                b.bd = cbst.bd;
                b.bj = cbst.bj;
                b.bk = cbst.bk;
            }
            // the search pass left this launch's octant message: the 4th smallest distance of
            // its octant (rounded down).  Above the cached best, every octant point tied with
            // that best is cached, so the cached best IS the octant's (d2, index) winner and its
            // cells need no rescan.
            const bool skip_oct = !a.ring_all && cd.slot == (a.launch & a.hist_mask) && cd.D * cd.D > cbst.bd;
            bool done = false;
            if (!a.ring_all) {
                // stage 2: the 3x3x3 cells around the query (less the octant's when it was
                // searched completely), rows and end cells pruned by the bound, as 3 planes of 3
                // x-rows scanned like the octant pass; certifies any winner within the distance
                // to the block's faces (>= 1 cell).  Only what is left goes to the general search.
                const GridDesc& g = a.g;
                const float fx = cell_f<float>(g, qx, 0), fy = cell_f<float>(g, qy, 1), fz = cell_f<float>(g, qz, 2);
                const int cx = (int)floorf(fx), cy = (int)floorf(fy), cz = (int)floorf(fz);
                const float lx = fx - (float)cx, ly = fy - (float)cy, lz = fz - (float)cz;
                const int bxo = (int)floorf(fx - a.rho), byo = (int)floorf(fy - a.rho), bzo = (int)floorf(fz - a.rho);
                const float inv_h2 = g.inv_hf * g.inv_hf;
                const float gxl = sq_gap(lx, a.mc), gxr = sq_gap(1.f - lx, a.mc);
                for (int dz = -1; dz <= 1; dz++) {
                    const int z = cz + dz;
                    const float lim = b.bd * 1.00002f * inv_h2;  // the bound in cells^2 (shrinks)
                    const float gz2 = sq_gap(axis_gap<float>(z, cz, lz), a.mc);
                    uint32_t rs[3], rn[3];
#pragma unroll
                    for (int r = 0; r < 3; r++) {
                        const int y = cy - 1 + r;
                        const float gyz = gz2 + sq_gap(axis_gap<float>(y, cy, ly), a.mc);
                        int xlo = max(cx - 1, 0), xhi = min(cx + 1, g.n[0] - 1);
                        if (skip_oct && y >= byo && y <= byo + 1 && z >= bzo && z <= bzo + 1) {
                            if (bxo == cx - 1) xlo = max(xlo, cx + 1);
                            else xhi = min(xhi, cx - 1);
                        }
                        if (xlo == cx - 1 && gyz + gxl > lim) xlo = cx;
                        if (xhi == cx + 1 && gyz + gxr > lim) xhi = cx;
                        const bool in = y >= 0 && y < g.n[1] && z >= 0 && z < g.n[2] && gyz <= lim && xlo <= xhi;
                        const int64_t cc = in ? dense_id(g, xlo, y, z) : 0;
                        rs[r] = in ? g.cstart[cc] : 0u;
                        rn[r] = in ? g.cstart[cc + (xhi - xlo + 1)] - rs[r] : 0u;
                    }
                    b.scan_rows_g<G>(a.tp, rs, rn, qx, qy, qz, sub);
                    b.merge_group<G>();
                }
                const float m = fminf(fminf(fminf(fx - (float)(cx - 1), (float)(cx + 2) - fx),
                                            fminf(fy - (float)(cy - 1), (float)(cy + 2) - fy)),
                                      fminf(fz - (float)(cz - 1), (float)(cz + 2) - fz)) - a.mc;
                const float rr = m * g.hf;
                const float c2 = rr * rr * (1.f - 2e-5f);
                const bool found = b.bj != 0x7fffffff;
                done = (found && b.bd <= c2) || (!found && a.r2 <= c2);
            }
            if (!done) box_search<G>(a.g, a.tp, qx, qy, qz, a.mc, b, sub);
            const bool ok = b.bj != 0x7fffffff;
            // no bound kept: the next launch searches it again
            if (lead) {
                cache_store(a, i, ok ? b.bk : ~0u, ~0u, ~0u, 0.f, a.launch);
            }
        }
        const bool acc_ok = valid && lead && b.bj != 0x7fffffff && !(a.dbg & kDbgNoAccum);
        if (acc_ok) b.fetch(a.tp);
        chunk_accumulate(acc_ok, qx, qy, qz, b, s_acc[wid], lane);
    }
}

__global__ void __launch_bounds__(kIcpBlock, PCP_RING_WAVES) k_icp_ring(IcpArgs a, double* partials,
                                                                        const int32_t* list, const uint32_t* list_n) {
    load_pose(a);
    constexpr int kW = kIcpBlock / 64;
    __shared__ double s_acc[kW][kAcc];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane < kAcc) s_acc[wid][lane] = 0.0;
    const int64_t n = a.ring_all ? a.nq : (int64_t)*list_n;
    const int G = a.ring_g ? a.ring_g : PCP_RING_G ? PCP_RING_G : (a.ring_all ? 1 : ring_lanes(n, a.nq));  // uniform
    if (G == 1)
        ring_run<1>(a, s_acc, list, list_n);
    else if (G == 2)
        ring_run<2>(a, s_acc, list, list_n);
    else if (G == 4)
        ring_run<4>(a, s_acc, list, list_n);
    else
        ring_run<8>(a, s_acc, list, list_n);
    write_wave_partials(s_acc, partials + (int64_t)blockIdx.x * kAcc);
}

// Concatenate per-wave list segments (segment s holds cnt[s] entries at s * seg_cap) into one
// list, in one launch with no separate scan: block b (4 waves: segments 4b .. 4b + 3) finds the
// exclusive prefix of the counts before its first segment by summing them itself (at most nseg
// counts, L2-resident), and the block holding the last segment writes the total to *total (where
// the consumers read the list length).  The list keeps segment order, entry for entry.
__global__ void __launch_bounds__(256) k_list_compact(const int32_t* __restrict__ seg, const uint32_t* __restrict__ cnt,
                                                      int64_t nseg, int64_t seg_cap, int32_t* __restrict__ out,
                                                      uint32_t* __restrict__ total) {
    __shared__ uint32_t s_part[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t s0 = (int64_t)blockIdx.x * 4;
    uint32_t acc = 0;
    for (int64_t i = threadIdx.x; i < s0; i += 256) acc += cnt[i];
    for (int o = 32; o > 0; o >>= 1) acc += (uint32_t)__shfl_xor((int)acc, o, 64);
    if (lane == 0) s_part[w] = acc;
    __syncthreads();
    const uint32_t base = s_part[0] + s_part[1] + s_part[2] + s_part[3];
    uint32_t c[4];
#pragma unroll
    for (int k = 0; k < 4; k++) c[k] = s0 + k < nseg ? cnt[s0 + k] : 0u;
    uint32_t off = base;
#pragma unroll
    for (int k = 0; k < 3; k++) off += k < w ? c[k] : 0u;
    const int64_t sg = s0 + w;
    if (sg < nseg)
        for (uint32_t k = (uint32_t)lane; k < c[w]; k += 64) out[off + k] = seg[sg * seg_cap + k];
    if (s0 + 4 >= nseg && threadIdx.x == 0) *total = base + c[0] + c[1] + c[2] + c[3];
}

// fixed-order reduction of nb partial rows of 24 doubles -> out[24]: thread t sums column
// t % 24 over the rows b = t / 24 (mod 32) -- coalesced row reads, no barrier per column --
// then 24 threads add the 32 group sums in order.  Slot 23 (unused by the solve) carries the
// number of fallback queries of the iteration (*fb_total, or 0 without a fallback list).
constexpr int kRedGroups = 32;
__global__ void __launch_bounds__(kAcc * kRedGroups) k_reduce_partials(const double* __restrict__ part, int nb,
                                                                       double* out, const uint32_t* fb_total) {
    __shared__ double s[kRedGroups][kAcc];
    const int k = threadIdx.x % kAcc, grp = threadIdx.x / kAcc;
    double v = 0.0;
    int b = grp;
    for (; b + 7 * kRedGroups < nb; b += 8 * kRedGroups) {  // 8 loads in flight, summed in order
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; u++) x[u] = part[(int64_t)(b + u * kRedGroups) * kAcc + k];
#pragma unroll
        for (int u = 0; u < 8; u++) v += x[u];
    }
    for (; b < nb; b += kRedGroups) v += part[(int64_t)b * kAcc + k];
    s[grp][k] = v;
    __syncthreads();
    if (threadIdx.x < kAcc) {
        double t = 0.0;
        for (int j = 0; j < kRedGroups; j++) t += s[j][threadIdx.x];
        out[threadIdx.x] = threadIdx.x == kAcc - 1 ? (fb_total ? (double)*fb_total : 0.0) : t;
    }
}

// sorted-order winners -> caller (original query) order; d2 recomputed from the winner's
// position under the same pose (the same fp32 expression, so bit-identical)
__global__ void k_scatter_corr(IcpArgs a, int32_t* idx, float* d2) {
    load_pose(a);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float4 qq = ldq(a, i);
        const int oq = a.qidx[i];
        float x, y, z;
        xform(a, qq, x, y, z);
        const CacheBest w = cache_best(a.tp, cache_load(a, i), x, y, z);  // the settled winner is cached
        const bool ok = w.bd <= a.r2;
        idx[oq] = ok ? w.bj : -1;
        d2[oq] = ok ? w.bd : INFINITY;
    }
}

__global__ void k_fill_corr(int32_t* idx, float* d2, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        idx[i] = -1;
        d2[i] = INFINITY;
    }
}

// ---- target-sharded mode: per-query u64 key = (fp32 bits of d2) << 32 |
// global target index, so a MIN over ranks is the lexicographic (d2, index) winner (non-
// negative fp32 bit patterns order like the values).  No correspondence = INT64_MAX.
constexpr uint64_t kNoKey = 0x7fffffffffffffffull;

__global__ void k_fill_keys(uint64_t* keys, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        keys[i] = kNoKey;
}

__global__ void k_make_keys(IcpArgs a, uint32_t offset, uint64_t* keys) {
    load_pose(a);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.nq; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 qq = ldq(a, i);
        const int oq = a.qidx[i];
        float x, y, z;
        xform(a, qq, x, y, z);
        const CacheBest w = cache_best(a.tp, cache_load(a, i), x, y, z);
        keys[oq] = w.bd <= a.r2 ? (((uint64_t)__float_as_uint(w.bd) << 32) | (uint64_t)(uint32_t)((uint32_t)w.bj + offset))
                                : kNoKey;
    }
}

// accumulators over the queries whose global winner lies in [lo, hi) (this rank's shard);
// float products are exact in fp64, so only the summation order differs from the oracle
__global__ void __launch_bounds__(256) k_acc_keys(const QXyz* q, const int32_t* qidx, int64_t n, const uint64_t* keys,
                                                  uint64_t lo,
                                                  uint64_t hi, const float* shard, size_t stride_f, IcpArgs a,
                                                  double* partials) {
    double acc[kAcc - 1];
#pragma unroll
    for (int k = 0; k < kAcc - 1; k++) acc[k] = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 qq = make_float4(q[i].x, q[i].y, q[i].z, 0.f);
        const uint64_t key = keys[qidx[i]];
        if (key == kNoKey) continue;
        const uint64_t g = key & 0xffffffffull;
        if (g < lo || g >= hi) continue;
        const float* p = shard + (size_t)(g - lo) * stride_f;
        float x, y, z;
        xform(a, qq, x, y, z);
        const double qv[3] = {x, y, z}, pv[3] = {p[0], p[1], p[2]};
        acc[0] += 1.0;
#pragma unroll
        for (int c = 0; c < 3; c++) { acc[1 + c] += qv[c]; acc[4 + c] += pv[c]; }
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int c = 0; c < 3; c++) acc[7 + 3 * r + c] += qv[r] * pv[c];
        acc[16] += qv[0] * qv[0]; acc[17] += qv[0] * qv[1]; acc[18] += qv[0] * qv[2];
        acc[19] += qv[1] * qv[1]; acc[20] += qv[1] * qv[2]; acc[21] += qv[2] * qv[2];
        acc[22] += (double)__uint_as_float((uint32_t)(key >> 32));
    }
    __shared__ double sm[4][kAcc];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < kAcc - 1; k++) {
        double v = acc[k];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) sm[wv][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < kAcc) {
        double v = 0.0;
        if (threadIdx.x < kAcc - 1)
            for (int w = 0; w < 4; w++) v += sm[w][threadIdx.x];
        partials[(int64_t)blockIdx.x * kAcc + threadIdx.x] = v;
    }
}

__global__ void __launch_bounds__(256) k_sum_partials(const double* part, int nb, double* out) {
    __shared__ double s[256];
    for (int k = 0; k < kAcc; k++) {
        double v = 0.0;
        for (int b = threadIdx.x; b < nb; b += 256) v += part[(int64_t)b * kAcc + k];
        s[threadIdx.x] = v;
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if ((int)threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
            __syncthreads();
        }
        if (threadIdx.x == 0) out[k] = s[0];
        __syncthreads();
    }
}

// Target-sharded mode, device-resident form: after a ReduceScatter(MIN) of
// the per-query keys, each rank knows the global winners of its slice of the queries; the shard
// that owns each winner (by its global target index) is all-gathered as one byte per query, and
// every rank accumulates exactly the queries whose winner lies in its own shard, reading the
// winner from its LOCAL shard -- no rank ever holds the full target.  A SUM over ranks gives the
// accumulators of every query.
// owner[i] = s with bounds[s] <= global index < bounds[s + 1], or 255 (no correspondence)
__global__ void k_keys_owner(const uint64_t* keys, int64_t n, const int64_t* bounds, int nshards, uint8_t* owner) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        uint8_t o = 255;
        if (k != kNoKey) {
            const int64_t g = (int64_t)(k & 0xffffffffull);
            int lo = 0, hi = nshards;  // the last s with bounds[s] <= g
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (bounds[mid] <= g) lo = mid;
                else hi = mid;
            }
            o = (uint8_t)lo;
        }
        owner[i] = o;
    }
}

// accumulators of the queries (original order, q) whose winner this rank owns: the winner is
// the rank's local key's target (its global index less lo) -- for an owned query the local key
// IS the global MIN.  The pose is the device 4x4 cast to fp32 as k_pose_set does; products of
// fp32 values are exact in fp64, so only the summation order differs from the oracle.
__global__ void __launch_bounds__(256) k_acc_owned(const double* T, const float* q, size_t qs, int64_t n,
                                                   const uint64_t* keys, const uint8_t* owner, int rank, int64_t lo,
                                                   int64_t hi, const float* shard, size_t ss, double* partials) {
    float R[9], t[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
#pragma unroll
        for (int c = 0; c < 3; c++) R[3 * r + c] = (float)T[4 * r + c];
        t[r] = (float)T[4 * r + 3];
    }
    double acc[kAcc - 1];
#pragma unroll
    for (int k = 0; k < kAcc - 1; k++) acc[k] = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (owner[i] != (uint8_t)rank) continue;
        const uint64_t key = keys[i];
        const int64_t g = (int64_t)(key & 0xffffffffull);
        if (key == kNoKey || g < lo || g >= hi) continue;
        const float* qp = q + (size_t)i * qs;
        const float* p = shard + (size_t)(g - lo) * ss;
        const float x = __fmaf_rn(R[2], qp[2], __fmaf_rn(R[1], qp[1], __fmaf_rn(R[0], qp[0], t[0])));
        const float y = __fmaf_rn(R[5], qp[2], __fmaf_rn(R[4], qp[1], __fmaf_rn(R[3], qp[0], t[1])));
        const float z = __fmaf_rn(R[8], qp[2], __fmaf_rn(R[7], qp[1], __fmaf_rn(R[6], qp[0], t[2])));
        const double qv[3] = {x, y, z}, pv[3] = {p[0], p[1], p[2]};
        acc[0] += 1.0;
#pragma unroll
        for (int c = 0; c < 3; c++) { acc[1 + c] += qv[c]; acc[4 + c] += pv[c]; }
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int c = 0; c < 3; c++) acc[7 + 3 * r + c] += qv[r] * pv[c];
        acc[16] += qv[0] * qv[0]; acc[17] += qv[0] * qv[1]; acc[18] += qv[0] * qv[2];
        acc[19] += qv[1] * qv[1]; acc[20] += qv[1] * qv[2]; acc[21] += qv[2] * qv[2];
        acc[22] += (double)__uint_as_float((uint32_t)(key >> 32));
    }
    __shared__ double sm[4][kAcc];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < kAcc - 1; k++) {
        double v = acc[k];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) sm[wv][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < kAcc) {
        double v = 0.0;
        if (threadIdx.x < kAcc - 1)
            for (int w = 0; w < 4; w++) v += sm[w][threadIdx.x];
        partials[(int64_t)blockIdx.x * kAcc + threadIdx.x] = v;
    }
}

// co-partitioned slab guard (one thread): the owned queries' box [b0..b5] = {x0,x1,y0,y1,z0,z1}
// under the device pose must keep x within [lo, hi] (the slab core widened by the target halo
// less rmax); the x-extreme of an affine image of a box is at a corner.  Latches flag = 1.
__global__ void k_slab_guard(const double* T, double b0, double b1, double b2, double b3, double b4, double b5,
                             double lo, double hi, int* flag) {
    const double bx[2] = {b0, b1}, by[2] = {b2, b3}, bz[2] = {b4, b5};
    double mn = INFINITY, mx = -INFINITY;
    for (int c = 0; c < 8; c++) {
        const double x = T[0] * bx[c & 1] + T[1] * by[(c >> 1) & 1] + T[2] * bz[c >> 2] + T[3];
        mn = fmin(mn, x);
        mx = fmax(mx, x);
    }
    if (!(mn >= lo && mx <= hi)) *flag = 1;
}

// ---- query order (pcp_icp_create): queries sorted once by target-grid cell in brick-major
// order (4x4x4-cell bricks; stable, so input order inside a cell), carried as float4
// {x, y, z, bits(index)}
// through the radix sort; non-finite queries get key 64 * nbricks (after every cell) and
// are dropped.
#ifndef PCP_QKEY_LOCAL  // 0: brick order only (one radix pass less; measured 5 % slower searches)
#define PCP_QKEY_LOCAL 1
#endif
#ifndef PCP_QBRICK  // edge (cells) of the query-order bricks: 4 = the index's bricks
#define PCP_QBRICK 8
#endif
__host__ __device__ inline int64_t qbricks(const GridDesc& g, int a) { return (g.n[a] + PCP_QBRICK - 1) / PCP_QBRICK; }
__host__ __device__ inline uint32_t query_key_end(const GridDesc& g) {
    if (PCP_QBRICK != 4)
        return (uint32_t)(qbricks(g, 0) * qbricks(g, 1) * qbricks(g, 2) * PCP_QBRICK * PCP_QBRICK * PCP_QBRICK);
    return (uint32_t)(PCP_QKEY_LOCAL ? g.nbricks * 64 : g.nbricks);
}
__global__ void k_query_keys(GridDesc g, const float* q, size_t stride_f, int64_t n, uint32_t* key, float4* rec) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float* p = q + (size_t)i * stride_f;
        const float x = p[0], y = p[1], z = p[2];
        const bool fin = isfinite(x) && isfinite(y) && isfinite(z);
        uint32_t k = query_key_end(g);  // past every brick: non-finite queries sort last
        if (fin) {
            // the brick (4x4x4 cells) of the octant block origin floor(f - 1/2) the search pass
            // uses: a 64-query chunk then scans the target rows of about one brick
            const int cx = clampi((int)floorf(cell_f<float>(g, x, 0) - 0.5f), 0, g.n[0] - 1);
            const int cy = clampi((int)floorf(cell_f<float>(g, y, 1) - 0.5f), 0, g.n[1] - 1);
            const int cz = clampi((int)floorf(cell_f<float>(g, z, 2) - 0.5f), 0, g.n[2] - 1);
            if (PCP_QBRICK != 4) {
                constexpr int B = PCP_QBRICK;
                const int64_t b = ((int64_t)(cz / B) * qbricks(g, 1) + cy / B) * qbricks(g, 0) + cx / B;
                k = (uint32_t)(b * B * B * B + ((cz % B) * B + cy % B) * B + cx % B);
            } else {
                k = PCP_QKEY_LOCAL ? (uint32_t)(brick_of(g, cx, cy, cz) * 64 + local_of(cx, cy, cz))
                                   : (uint32_t)brick_of(g, cx, cy, cz);
            }
        }
        key[i] = k;
        rec[i] = make_float4(x, y, z, __int_as_float((int)i));
    }
}

// the sorted {x, y, z, bits(index)} records -> 12-byte xyz + index arrays
__global__ void k_split_queries(const float4* qs, int64_t n, QXyz* q, int32_t* qi) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = qs[i];
        q[i] = QXyz{v.x, v.y, v.z};
        qi[i] = __float_as_int(v.w);
    }
}

// number of finite queries = first position of the sentinel key in the sorted keys
// (a single-address atomic per wave costs ~9 ms at 50M queries; this costs nothing)
__global__ void k_first_at_least(const uint32_t* sorted, int64_t n, uint32_t key, unsigned long long* out) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (sorted[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    *out = (unsigned long long)lo;
}

// ------------------------------------------------------------------ host 3x3 solve
// One-sided Jacobi SVD of a 3x3 matrix: A = U diag(s) V^T (columns of U, V).
// (host and device: the device-resident loop solves on the GPU with the same code)
__host__ __device__ void svd3(const double Ain[9], double U[9], double s[3], double V[9]) {
    double A[9];
    for (int i = 0; i < 9; i++) A[i] = Ain[i];
    for (int i = 0; i < 9; i++) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; sweep++) {
        double off = 0.0;
        for (int p = 0; p < 2; p++)
            for (int q = p + 1; q < 3; q++) {
                double al = 0, be = 0, ga = 0;
                for (int r = 0; r < 3; r++) {
                    al += A[3 * r + p] * A[3 * r + p];
                    be += A[3 * r + q] * A[3 * r + q];
                    ga += A[3 * r + p] * A[3 * r + q];
                }
                if (ga == 0.0 || fabs(ga) <= 1e-300) continue;
                double conv = fabs(ga) / sqrt(al * be);
                if (!(conv > 1e-15)) continue;
                off = fmax(off, conv);
                double zeta = (be - al) / (2.0 * ga);
                double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                double c = 1.0 / sqrt(1.0 + t * t), sn = c * t;
                for (int r = 0; r < 3; r++) {
                    double ap = A[3 * r + p], aq = A[3 * r + q];
                    A[3 * r + p] = c * ap - sn * aq;
                    A[3 * r + q] = sn * ap + c * aq;
                    double vp = V[3 * r + p], vq = V[3 * r + q];
                    V[3 * r + p] = c * vp - sn * vq;
                    V[3 * r + q] = sn * vp + c * vq;
                }
            }
        if (off < 1e-15) break;
    }
    for (int c = 0; c < 3; c++) {
        double n = 0;
        for (int r = 0; r < 3; r++) n += A[3 * r + c] * A[3 * r + c];
        s[c] = sqrt(n);
    }
    // order singular values descending (permute U/V columns consistently)
    int ord[3] = {0, 1, 2};
    for (int i = 0; i < 3; i++)
        for (int j = i + 1; j < 3; j++)
            if (s[ord[j]] > s[ord[i]]) { const int tmp = ord[i]; ord[i] = ord[j]; ord[j] = tmp; }
    double A2[9], V2[9], s2[3];
    for (int c = 0; c < 3; c++) {
        s2[c] = s[ord[c]];
        for (int r = 0; r < 3; r++) { A2[3 * r + c] = A[3 * r + ord[c]]; V2[3 * r + c] = V[3 * r + ord[c]]; }
    }
    for (int i = 0; i < 9; i++) V[i] = V2[i];
    for (int c = 0; c < 3; c++) s[c] = s2[c];
    const double tiny = 1e-14 * (s[0] > 0 ? s[0] : 1.0);
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) U[3 * r + c] = s[c] > tiny ? A2[3 * r + c] / s[c] : 0.0;
    // complete a rank-deficient basis: u2 = u0 x u1 (planar clouds have rank 2)
    if (!(s[2] > tiny)) {
        double u0[3] = {U[0], U[3], U[6]}, u1[3] = {U[1], U[4], U[7]};
        if (!(s[1] > tiny)) {  // rank 1: any unit vector orthogonal to u0
            double a[3] = {fabs(u0[0]) < 0.9 ? 1.0 : 0.0, fabs(u0[0]) < 0.9 ? 0.0 : 1.0, 0.0};
            double d = a[0] * u0[0] + a[1] * u0[1] + a[2] * u0[2];
            for (int r = 0; r < 3; r++) u1[r] = a[r] - d * u0[r];
            double nn = sqrt(u1[0] * u1[0] + u1[1] * u1[1] + u1[2] * u1[2]);
            for (int r = 0; r < 3; r++) { u1[r] /= nn; U[3 * r + 1] = u1[r]; }
        }
        double u2[3] = {u0[1] * u1[2] - u0[2] * u1[1], u0[2] * u1[0] - u0[0] * u1[2], u0[0] * u1[1] - u0[1] * u1[0]};
        for (int r = 0; r < 3; r++) U[3 * r + 2] = u2[r];
    }
}

__host__ __device__ double det3(const double M[9]) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

}  // namespace

// device poses for the kernels: pose[12..23] <- pose[0..11] (the previous launch's), then
// pose[0..11] <- R, t of T_dev (row-major 4x4 doubles cast to fp32, as on the host) or of the
// host-cast Rh/th when T_dev is null
struct HostPose {
    float R[9], t[3];
};
__global__ void k_pose_set(const double* T, HostPose hp, float* pose, float* hist, uint32_t launch) {
    *(uint32_t*)(pose + 24) = launch;
    for (int k = 0; k < 12; k++) pose[12 + k] = pose[k];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) pose[3 * r + c] = T ? (float)T[4 * r + c] : hp.R[3 * r + c];
        pose[9 + r] = T ? (float)T[4 * r + 3] : hp.t[r];
    }
    for (int k = 0; k < 12; k++) hist[k] = pose[k];
}

__host__ __device__ int icp_solve(const double acc[24], int do_scale, double dT[16]);

// One thread: solve the 3x3 problem of acc, T <- dT * T (device pose), stats as in pcp.h
// (the host loop of pcp_icp_run, minus the convergence test).  A failed solve latches
// stats[0] = -1 and freezes T.
__global__ void k_icp_solve_dev(const double* acc, int do_scale, double* T, double* stats) {
    if (stats[0] < 0) return;
    double a[24], dT[16], Tn[16];
    for (int k = 0; k < 24; k++) a[k] = acc[k];
    stats[2] += a[23];
    if (icp_solve(a, do_scale, dT) != PCP_OK) {
        stats[0] = -1.0;
        return;
    }
    stats[1] = sqrt(a[22] / a[0]);
    stats[3] += 1.0;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double v = 0;
            for (int k = 0; k < 4; k++) v += dT[4 * i + k] * T[4 * k + j];
            Tn[4 * i + j] = v;
        }
    for (int k = 0; k < 16; k++) T[k] = Tn[k];
}

// T (host) or T_dev (device pose, read by k_pose_from_T) -- exactly one is non-null
int icp_launch(pcp_icp* icp, const double T[16], float rmax, double* acc_dev, int32_t* corr_idx,
               float* corr_d2, const double* T_dev = nullptr, IcpArgs* args_out = nullptr) {
    pcp_ctx* ctx = icp->ctx;
    const pcp_index* tg = icp->target;
    IcpArgs a{};
    a.g = tg->g;
    a.tp = (const float4*)tg->pts;
    a.q = icp->q;
    a.qidx = icp->qidx;
    a.nq = icp->nq;
    a.nchunks = (icp->nq + kIcpBlock - 1) / kIcpBlock;
    HostPose hp{};
    if (!T_dev) {
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) hp.R[3 * r + c] = (float)T[4 * r + c];
            hp.t[r] = (float)T[4 * r + 3];
        }
    }
    hipLaunchKernelGGL(k_pose_set, dim3(1), dim3(1), 0, ctx->stream, T_dev, hp, icp->pose_dev,
                       icp->pose_hist + (icp->launches & (icp->narrow ? 63 : kHist - 1)) * 12,
                       (uint32_t)icp->launches);
    a.pose = icp->pose_dev;  // every kernel reads the pose (and the previous one) from HBM
    a.launch_dev = (const uint32_t*)(icp->pose_dev + 24);  // ... and the launch index
    for (int k = 0; k < 9; k++) a.R[k] = hp.R[k];
    for (int k = 0; k < 3; k++) a.t[k] = hp.t[k];
    a.r2 = rmax * rmax;
    const int nmax = std::max(a.g.n[0], std::max(a.g.n[1], a.g.n[2]));
    a.mc = 1e-5f + 8e-7f * (float)nmax;  // >> fp32 rounding of the cell coordinates
    a.rho = 0.5f;
    // exact radius of the octant block: (0.5 - mc) cells, shrunk for fp32 d2 rounding
    const double rr = (0.5 - (double)a.mc) * a.g.h;
    a.cert2 = (float)(rr * rr * (1.0 - 1e-5));
    a.cand = icp->cand;
    a.narrow = icp->narrow ? 1 : 0;
    a.hist_mask = icp->narrow ? 63u : (uint32_t)(kHist - 1);
    a.max_age = icp->narrow ? 32u : 128u;
    a.dunit = (float)(a.g.h / 1024.0);
    a.inv_dunit = (float)(1024.0 / a.g.h);
    a.pose_hist = icp->pose_hist;
    a.launch = (uint32_t)icp->launches;
    a.ntp = (uint32_t)tg->n;
    a.sv = icp->sv;
    a.sv_count = icp->sv_count;
    a.sv_off = icp->sv_off;
    a.sv_seg = icp->sv_seg;
    a.nseg_v = icp->nseg_v;
    a.fb = icp->fb;
    a.fb_count = icp->fb_count;
    a.fb_off = icp->fb_off;
    a.fb_seg = icp->fb_seg;
    a.nb_fast = icp->nb_fast;
    a.nseg = (int64_t)icp->nb_fast * (kIcpBlock / 64);
    a.ring_all = a.g.dense ? 0 : 1;
    a.dbg = icp->dbg;
    double* part_v = icp->partials;
    double* part_o = part_v + (int64_t)icp->nb_ver * kAcc;
    double* part_r = part_o + (int64_t)icp->nb_fast * kAcc;
    hipEvent_t e0 = icp->ev0, e1 = icp->ev1;
    if (T_dev) {  // device-resident loop: one event pair per launch, read by pcp_icp_kernel_ms
        if (icp->ntev == icp->tev.size()) {
            std::pair<hipEvent_t, hipEvent_t> pr{nullptr, nullptr};
            PCP_HIP(ctx, pcp::event_get(ctx, &pr.first));
            if (pcp::event_get(ctx, &pr.second) != hipSuccess) {
                pcp::event_put(ctx, pr.first);
                return set_error(ctx, PCP_ERR_HIP, "hipEventCreate");
            }
            icp->tev.push_back(pr);
        }
        e0 = icp->tev[icp->ntev].first;
        e1 = icp->tev[icp->ntev].second;
        icp->ntev++;
    }
    PCP_HIP(ctx, hipEventRecord(e0, ctx->stream));
    const bool verify = a.g.dense && icp->launches > 0;  // the first launch has nothing cached
    icp->last_verified = verify;
    // A device-pose launch after the first is the same five kernels every time (verify, list
    // concatenation, octant search, list concatenation, fallback) with the same arguments: the
    // launch index is read from the device (k_pose_set) and the pose was already.  With
    // PCP_ICP_OPT_GRAPH the section is captured once per handle into a HIP graph and replayed --
    // one launch instead of five (measured: host enqueue is not what the loop waits for, and the
    // replayed section ran 0.5 % slower, so it is off by default).
    if (icp->graph && T_dev && verify && !icp->dbg && !corr_idx && !args_out && !icp->graph_off) {
        a.oct_g = icp->oct_g_list;
        a.ring_g = icp->ring_g;
        auto section = [&](hipStream_t st) {
            IcpArgs b = a;
            b.partials = part_v;
            hipLaunchKernelGGL(k_icp_verify, dim3(icp->nb_ver), dim3(kIcpBlock), 0, st, b);
            hipLaunchKernelGGL(k_list_compact, dim3((unsigned)((b.nseg_v + 3) / 4)), dim3(256), 0, st,
                               (const int32_t*)icp->sv, (const uint32_t*)icp->sv_count, b.nseg_v, b.sv_seg, icp->svc,
                               icp->sv_off + b.nseg_v);
            b.partials = part_o;
            hipLaunchKernelGGL(k_icp_octant<PCP_OCT_WAVES_LIST>, dim3(icp->nb_fast_l), dim3(kIcpBlock), 0, st, b,
                               (const int32_t*)icp->svc, (const uint32_t*)(icp->sv_off + b.nseg_v));
            hipLaunchKernelGGL(k_list_compact, dim3((unsigned)((b.nseg + 3) / 4)), dim3(256), 0, st,
                               (const int32_t*)icp->fb, (const uint32_t*)icp->fb_count, b.nseg, b.fb_seg, icp->fbc,
                               icp->fb_off + b.nseg);
            b.partials = part_r;
            hipLaunchKernelGGL(k_icp_ring, dim3(icp->nb_ring), dim3(kIcpBlock), 0, st, b, part_r,
                               (const int32_t*)icp->fbc, (const uint32_t*)(icp->fb_off + b.nseg));
        };
        if (icp->gexec && icp->graph_r2 != a.r2) {  // captured for another rmax (replays are stream-ordered)
            (void)hipStreamSynchronize(ctx->stream);
            (void)hipGraphExecDestroy(icp->gexec);
            icp->gexec = nullptr;
        }
        if (!icp->gexec) {  // captured on the context's side stream (capture enqueues nothing)
            hipStream_t cap = nullptr;
            hipError_t e = side_stream(ctx, &cap) == PCP_OK ? hipSuccess : hipErrorInvalidValue;
            hipGraph_t gr = nullptr;
            if (e == hipSuccess) e = hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
            if (e == hipSuccess) {
                section(cap);
                e = hipStreamEndCapture(cap, &gr);
            }
            if (e == hipSuccess) e = hipGraphInstantiate(&icp->gexec, gr, nullptr, nullptr, 0);
            if (gr) (void)hipGraphDestroy(gr);
            if (e != hipSuccess) {  // launch the kernels one by one from now on
                icp->gexec = nullptr;
                icp->graph_off = true;
                (void)hipGetLastError();
            }
            icp->graph_r2 = a.r2;
        }
        if (icp->gexec) PCP_HIP(ctx, hipGraphLaunch(icp->gexec, ctx->stream));
        else section(ctx->stream);
        PCP_HIP(ctx, hipEventRecord(e1, ctx->stream));
        hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(kAcc * kRedGroups), 0, ctx->stream, icp->partials,
                           icp->nb_ver + icp->nb_fast + icp->nb_ring, acc_dev, (const uint32_t*)(icp->fb_off + a.nseg));
        icp->launches++;
        PCP_LAUNCH_CHECK(ctx);
        return PCP_OK;
    }
    if (a.g.dense) {
        // 1. settle what the candidate caches can; the rest -> search list
        if (verify) {
            a.partials = part_v;
            hipLaunchKernelGGL(k_icp_verify, dim3(icp->nb_ver), dim3(kIcpBlock), 0, ctx->stream, a);
            hipLaunchKernelGGL(k_list_compact, dim3((unsigned)((a.nseg_v + 3) / 4)), dim3(256), 0, ctx->stream,
                               (const int32_t*)icp->sv, (const uint32_t*)icp->sv_count, a.nseg_v, a.sv_seg, icp->svc,
                               icp->sv_off + a.nseg_v);
        } else {
            PCP_HIP(ctx, hipMemsetAsync(part_v, 0, (size_t)icp->nb_ver * kAcc * sizeof(double), ctx->stream));
        }
        if (icp->dbg) PCP_HIP(ctx, hipEventRecord(icp->ev_ver, ctx->stream));
        // 2. octant search of the list (every query at the first launch); unsettled -> fallback list
        a.partials = part_o;
        {
            const int32_t* lst = verify ? (const int32_t*)icp->svc : nullptr;
            const uint32_t* lst_n = verify ? (const uint32_t*)(icp->sv_off + a.nseg_v) : nullptr;
            a.oct_g = verify ? icp->oct_g_list : icp->oct_g_first;
            if (verify)
                hipLaunchKernelGGL(k_icp_octant<PCP_OCT_WAVES_LIST>, dim3(icp->nb_fast_l), dim3(kIcpBlock), 0,
                                   ctx->stream, a, lst, lst_n);
            else
                hipLaunchKernelGGL(k_icp_octant<PCP_OCT_WAVES>, dim3(icp->nb_fast), dim3(kIcpBlock), 0, ctx->stream,
                                   a, lst, lst_n);
        }
    } else {
        PCP_HIP(ctx, hipMemsetAsync(part_v, 0, (size_t)(icp->nb_ver + icp->nb_fast) * kAcc * sizeof(double),
                                    ctx->stream));
    }
    if (icp->dbg) PCP_HIP(ctx, hipEventRecord(icp->ev_mid, ctx->stream));
    if (a.g.dense) {  // compact the per-wave fallback segments into one list
        hipLaunchKernelGGL(k_list_compact, dim3((unsigned)((a.nseg + 3) / 4)), dim3(256), 0, ctx->stream,
                           (const int32_t*)icp->fb, (const uint32_t*)icp->fb_count, a.nseg, a.fb_seg, icp->fbc,
                           icp->fb_off + a.nseg);
    }
    // 3. exact fallback (or every query on a sparse grid)
    a.partials = part_r;
    a.ring_g = icp->ring_g;
    hipLaunchKernelGGL(k_icp_ring, dim3(icp->nb_ring), dim3(kIcpBlock), 0, ctx->stream, a, part_r,
                       (const int32_t*)icp->fbc, (const uint32_t*)(icp->fb_off + a.nseg));
    PCP_HIP(ctx, hipEventRecord(e1, ctx->stream));
    hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(kAcc * kRedGroups), 0, ctx->stream, icp->partials,
                       icp->nb_ver + icp->nb_fast + icp->nb_ring, acc_dev,
                       a.g.dense ? (const uint32_t*)(icp->fb_off + a.nseg) : nullptr);
    if (corr_idx) {
        if (icp->nq_in > icp->nq)  // non-finite queries were dropped at create time
            hipLaunchKernelGGL(k_fill_corr, dim3(grid_for(icp->nq_in, 256)), dim3(256), 0, ctx->stream, corr_idx,
                               corr_d2, icp->nq_in);
        if (icp->nq > 0)
            hipLaunchKernelGGL(k_scatter_corr, dim3(grid_for(icp->nq, 256)), dim3(256), 0, ctx->stream, a,
                               corr_idx, corr_d2);
    }
    if (args_out) *args_out = a;
    icp->launches++;
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

__host__ __device__ int icp_solve(const double acc[24], int do_scale, double dT[16]) {
    const double n = acc[0];
    if (!(n >= 3.0)) return PCP_ERR_ICP;
    double qm[3], pm[3], S[9];
    for (int k = 0; k < 3; k++) { qm[k] = acc[1 + k] / n; pm[k] = acc[4 + k] / n; }
    // S = sum (q - qm)(p - pm)^T ; optimal R maximises trace(R S): S = U s V^T, R = V D U^T
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) S[3 * a + b] = acc[7 + 3 * a + b] - n * qm[a] * pm[b];
    double U[9], s[3], V[9];
    svd3(S, U, s, V);
    double R[9];
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) {
            double v = 0;
            for (int k = 0; k < 3; k++) v += V[3 * a + k] * U[3 * b + k];
            R[3 * a + b] = v;
        }
    double d = det3(R) < 0 ? -1.0 : 1.0;
    if (d < 0) {  // flip the axis of the smallest singular value
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) R[3 * a + b] -= 2.0 * V[3 * a + 2] * U[3 * b + 2];
    }
    double sc = 1.0;
    if (do_scale) {
        const double var = (acc[16] + acc[19] + acc[21]) - n * (qm[0] * qm[0] + qm[1] * qm[1] + qm[2] * qm[2]);
        if (var > 0) sc = (s[0] + s[1] + d * s[2]) / var;
    }
    for (int a = 0; a < 3; a++) {
        double t = pm[a];
        for (int b = 0; b < 3; b++) {
            dT[4 * a + b] = sc * R[3 * a + b];
            t -= sc * R[3 * a + b] * qm[b];
        }
        dT[4 * a + 3] = t;
    }
    dT[12] = dT[13] = dT[14] = 0.0;
    dT[15] = 1.0;
    return PCP_OK;
}

}  // namespace pcp

extern "C" {

int pcp_icp_check_sizes(int64_t n_target, int64_t nq) {
    if (n_target < 0 || nq < 0) return PCP_ERR_ARG;
    if (nq >= ((int64_t)1 << 31)) return PCP_ERR_ARG;
    // ld16(): 32-bit byte offsets into the fp32 target (n_target records + the far sentinel)
    if (n_target + 1 >= ((int64_t)1 << 28)) return PCP_ERR_CAPACITY;
    return PCP_OK;
}

}  // extern "C"

namespace pcp {
namespace {

// the query sort of an ICP handle between its launch and its completion: keys of the octant-block
// bricks of the target grid, a stable radix sort with the 16-byte records as payload, the count
// of finite queries
struct QuerySort {
    uint32_t *k0 = nullptr, *k1 = nullptr;
    float4 *r0 = nullptr, *qs = nullptr;
    unsigned long long* d_cnt = nullptr;
    void* tmp = nullptr;
    hipEvent_t done = nullptr;
    int64_t nq = 0;
    void release(pcp_ctx* ctx) {  // stream-ordered on ctx->stream (after it waited for `done`)
        dfree(ctx, k0); dfree(ctx, k1); dfree(ctx, r0); dfree(ctx, qs); dfree(ctx, d_cnt); dfree(ctx, tmp);
        k0 = k1 = nullptr; r0 = qs = nullptr; d_cnt = nullptr; tmp = nullptr;
        if (done) event_put(ctx, done);
        done = nullptr;
    }
};

int icp_check_grid(pcp_ctx* ctx, const GridDesc& g, int64_t n_target, int64_t nq) {
    if (int rc = pcp_icp_check_sizes(n_target, nq))
        return set_error(ctx, rc, rc == PCP_ERR_CAPACITY ? "ICP target must have < 2^28 - 1 points (32-bit record offsets)"
                                                         : "ICP supports < 2^31 queries");
    if (g.nbricks * 64 >= ((int64_t)1 << 32) ||
        qbricks(g, 0) * qbricks(g, 1) * qbricks(g, 2) * PCP_QBRICK * PCP_QBRICK * PCP_QBRICK >= ((int64_t)1 << 32))
        return set_error(ctx, PCP_ERR_UNSUPPORTED, "ICP target grid too large for 32-bit cell keys");
    return PCP_OK;
}

// enqueue the query sort on `st` (after everything enqueued so far on ctx->stream); `s.done` is
// recorded on `st` when it is complete
int qsort_launch(pcp_ctx* ctx, hipStream_t st, const GridDesc& g, const float* q, size_t q_stride, int64_t nq,
                 QuerySort& s) {
    s.nq = nq;
    int rc = PCP_OK;
    if ((rc = dmalloc(ctx, &s.k0, nq)) || (rc = dmalloc(ctx, &s.k1, nq)) || (rc = dmalloc(ctx, &s.r0, nq)) ||
        (rc = dmalloc(ctx, &s.qs, nq + 1)) || (rc = dmalloc(ctx, &s.d_cnt, 1)))
        return rc;
    PCP_HIP(ctx, event_get(ctx, &s.done));
    unsigned bits = 1;  // keys are in [0, query_key_end]
    while (bits < 32 && ((uint64_t)1 << bits) <= (uint64_t)query_key_end(g)) bits++;
    size_t tb = 0;
    if (nq > 0) {
        PCP_HIP(ctx, rocprim::radix_sort_pairs<RecSortConfig>(nullptr, tb, s.k0, s.k1, s.r0, s.qs, (size_t)nq, 0u, bits, st));
        if ((rc = dmalloc(ctx, (char**)&s.tmp, tb))) return rc;
    }
    // Every block the side stream uses is allocated above, before `go` is recorded: a block the
    // context cache hands out after that point could still be in use by main-stream work the side
    // stream does not wait for.
    if (st != ctx->stream) {  // the side stream starts after the main stream's work so far
        hipEvent_t go = nullptr;
        PCP_HIP(ctx, event_get(ctx, &go));
        hipError_t e = hipEventRecord(go, ctx->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(st, go, 0);
        event_put(ctx, go);  // (reused only by a later record on ctx->stream: stream-ordered)
        if (e != hipSuccess) return hip_fail(ctx, e, "query sort stream order", __FILE__, __LINE__);
    }
    PCP_HIP(ctx, hipMemsetAsync(s.d_cnt, 0, sizeof(unsigned long long), st));
    if (nq > 0) {
        hipLaunchKernelGGL(k_query_keys, dim3(grid_for(nq, 256)), dim3(256), 0, st, g, q, q_stride / sizeof(float), nq,
                           s.k0, s.r0);
        PCP_HIP(ctx, rocprim::radix_sort_pairs<RecSortConfig>(s.tmp, tb, s.k0, s.k1, s.r0, s.qs, (size_t)nq, 0u, bits, st));
        hipLaunchKernelGGL(k_first_at_least, dim3(1), dim3(1), 0, st, s.k1, nq, query_key_end(g), s.d_cnt);
    }
    PCP_HIP(ctx, hipGetLastError());
    PCP_HIP(ctx, hipEventRecord(s.done, st));
    return PCP_OK;
}

// the sorted records -> 12-byte xyz + original indices, on ctx->stream after the sort
int qsort_finish(pcp_ctx* ctx, QuerySort& s, QXyz** q3, int32_t** qi, int64_t* nfin) {
    PCP_HIP(ctx, hipStreamWaitEvent(ctx->stream, s.done, 0));
    unsigned long long hc = 0;
    PCP_HIP(ctx, hipMemcpyAsync(&hc, s.d_cnt, sizeof(hc), hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *nfin = (int64_t)hc;
    int rc = PCP_OK;
    if ((rc = dmalloc(ctx, q3, s.nq + 1)) || (rc = dmalloc(ctx, qi, s.nq + 1))) return rc;
    if (*nfin > 0)
        hipLaunchKernelGGL(k_split_queries, dim3(grid_for(*nfin, 256)), dim3(256), 0, ctx->stream,
                           (const float4*)s.qs, *nfin, *q3, *qi);
    PCP_HIP(ctx, hipGetLastError());
    return PCP_OK;
}

// the handle over sorted queries (q3, qi: owned by the handle from here on)
int icp_make(pcp_ctx* ctx, const pcp_index* target, QXyz* q3, int32_t* qi, int64_t nfin, int64_t nq, pcp_icp** out) {
    pcp_icp* icp = new pcp_icp();
    icp->ctx = ctx;
    icp->owner = ctx;
    ctx_retain(ctx);
    icp->target = target;
    icp->nq = nfin;
    icp->nq_in = nq;
    icp->q = q3;
    icp->qidx = qi;
    int dev_cus = 256;  // one attribute query (the whole hipDeviceProp_t costs ~0.1 ms per create)
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) == hipSuccess && cus > 0)
        dev_cus = cus;
    const int64_t want = (icp->nq + kIcpBlock - 1) / kIcpBlock;
    icp->nb_fast = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)dev_cus * PCP_OCT_WAVES));
    icp->nb_fast_l = (int)std::max<int64_t>(1, std::min<int64_t>(icp->nb_fast, (int64_t)dev_cus * PCP_OCT_WAVES_LIST));
    icp->nb_ring = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)dev_cus * PCP_RING_WAVES));
    const int64_t nwaves = (int64_t)icp->nb_fast * (kIcpBlock / 64);
    const int64_t nwaves_l = (int64_t)icp->nb_fast_l * (kIcpBlock / 64);  // the smaller grid: larger segments
    const int64_t nchunks64 = (icp->nq + 63) / 64;
    icp->fb_seg = ((nchunks64 + nwaves_l - 1) / nwaves_l) * 64;
    icp->nb_ver = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)dev_cus * PCP_VER_WAVES));
    const int64_t nwaves_v = (int64_t)icp->nb_ver * (kIcpBlock / 64);
    icp->sv_seg = ((nchunks64 + nwaves_v - 1) / nwaves_v) * 64;  // contiguous ranges: <= this per wave
    icp->nseg_v = nwaves_v;
    int rc = dmalloc(ctx, &icp->partials, (size_t)(icp->nb_ver + icp->nb_fast + icp->nb_ring) * kAcc);
    if (!rc) rc = dmalloc(ctx, &icp->acc, kAcc);
    if (!rc) rc = dmalloc(ctx, &icp->pose_dev, 32);  // 24 pose floats + the launch index
    // 12-byte cache records when every position (and the far sentinel) fits 26 bits
    icp->narrow = target->n + 1 < (int64_t)kPos26;
    const int rw = icp->narrow ? 3 : 4;  // words per record
    if (!rc) rc = dmalloc(ctx, &icp->cand, (size_t)(icp->nq + 1) * rw);
    if (!rc) rc = dmalloc(ctx, &icp->pose_hist, kHist * 12);
    // the first launch over a dense grid (the octant pass over every query) writes every cache
    // record before any pass reads one: only the sentinel record needs its value then (an 800 MB
    // memset at 50M queries, ~0.1 ms of the pre-iteration span, otherwise).  An empty record has
    // no positions and D = 0 (wide: NaN), so it is never settled from.
    const bool cand_all = !target->g.dense;
    const int64_t r0 = cand_all ? 0 : icp->nq, nr = cand_all ? icp->nq + 1 : 1;
    hipError_t me = hipSuccess;
    if (!rc)
        me = icp->narrow ? hipMemsetD32Async((hipDeviceptr_t)(icp->cand + r0 * rw), (int)kPos26, (size_t)(nr * rw),
                                             ctx->stream)
                         : hipMemsetAsync(icp->cand + r0 * rw, 0xff, (size_t)nr * 16, ctx->stream);
    if (!rc && (me != hipSuccess ||
                hipMemsetAsync(icp->pose_hist, 0, kHist * 12 * sizeof(float), ctx->stream) != hipSuccess ||
                hipMemsetAsync(icp->pose_dev, 0, 32 * sizeof(float), ctx->stream) != hipSuccess))
        rc = set_error(ctx, PCP_ERR_HIP, "memset");
    if (!rc) rc = dmalloc(ctx, &icp->sv, (size_t)icp->nseg_v * icp->sv_seg + 1);
    if (!rc) rc = dmalloc(ctx, &icp->sv_count, (size_t)icp->nseg_v);
    if (!rc) rc = dmalloc(ctx, &icp->sv_off, (size_t)icp->nseg_v + 1);
    if (!rc) rc = dmalloc(ctx, &icp->svc, icp->nq + 1);
    const int64_t fb_cap = std::max<int64_t>(nwaves * icp->fb_seg, icp->nq);
    if (!rc) rc = dmalloc(ctx, &icp->fb, (size_t)fb_cap + 1);
    if (!rc) rc = dmalloc(ctx, &icp->fb_count, (size_t)nwaves);
    if (!rc) rc = dmalloc(ctx, &icp->fb_off, (size_t)nwaves + 1);
    if (!rc) rc = dmalloc(ctx, &icp->fbc, icp->nq + 1);
    if (!rc && (event_get(ctx, &icp->ev0) != hipSuccess || event_get(ctx, &icp->ev1) != hipSuccess ||
                event_get(ctx, &icp->ev_mid) != hipSuccess || event_get(ctx, &icp->ev_ver) != hipSuccess))
        rc = set_error(ctx, PCP_ERR_HIP, "hipEventCreate failed");
    if (rc) {
        pcp_icp_destroy(icp);
        return rc;
    }
    *out = icp;
    return PCP_OK;
}

}  // namespace
}  // namespace pcp

extern "C" {

int pcp_icp_create(pcp_ctx* ctx, const pcp_index* target, const float* q, size_t q_stride, int64_t nq,
                   pcp_icp** out) {
    if (!ctx || !target || !out || nq < 0 || (nq > 0 && !q)) return PCP_ERR_ARG;
    if (target->is_f64) return pcp::set_error(ctx, PCP_ERR_ARG, "ICP target must be an fp32 index");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    *out = nullptr;
    if (q_stride == 0) q_stride = 3 * sizeof(float);
    if (q_stride % sizeof(float)) return pcp::set_error(ctx, PCP_ERR_ARG, "query stride must be whole floats");
    PCP_TRY(pcp::icp_check_grid(ctx, target->g, target->n, nq));
    pcp::QuerySort s;
    pcp::QXyz* q3 = nullptr;
    int32_t* qi = nullptr;
    int64_t nfin = 0;
    int rc = pcp::qsort_launch(ctx, ctx->stream, target->g, q, q_stride, nq, s);
    if (!rc) rc = pcp::qsort_finish(ctx, s, &q3, &qi, &nfin);
    s.release(ctx);
    if (rc) {
        pcp::dfree(ctx, q3);
        pcp::dfree(ctx, qi);
        return rc;
    }
    return pcp::icp_make(ctx, target, q3, qi, nfin, nq, out);
}

int pcp_icp_create_with_target(pcp_ctx* ctx, const float* target_xyz, size_t t_stride, int64_t n_target,
                               double cell_size, const float* q, size_t q_stride, int64_t nq, pcp_index** index_out,
                               pcp_icp** icp_out) {
    if (!ctx || !index_out || !icp_out || nq < 0 || (nq > 0 && !q) || n_target < 0 || (n_target > 0 && !target_xyz))
        return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    *index_out = nullptr;
    *icp_out = nullptr;
    if (q_stride == 0) q_stride = 3 * sizeof(float);
    if (q_stride % sizeof(float)) return pcp::set_error(ctx, PCP_ERR_ARG, "query stride must be whole floats");
    // the query sort needs only the target grid's geometry: it runs on the side stream while the
    // target's cell sort runs on the main stream (two independent radix sorts overlapped)
    pcp::QuerySort s;
    bool launched = false;
    const pcp::GeomHook hook = [&](const pcp::GridDesc& g) -> int {
        PCP_TRY(pcp::icp_check_grid(ctx, g, n_target, nq));
        hipStream_t side = nullptr;
        PCP_TRY(pcp::side_stream(ctx, &side));
        launched = true;
        return pcp::qsort_launch(ctx, side, g, q, q_stride, nq, s);
    };
    pcp_index* ix = nullptr;
    int rc = pcp::index_build_f32_hooked(ctx, target_xyz, t_stride, n_target, cell_size, &ix, hook);
    pcp::QXyz* q3 = nullptr;
    int32_t* qi = nullptr;
    int64_t nfin = 0;
    if (!rc && !launched) rc = pcp::qsort_launch(ctx, ctx->stream, ix->g, q, q_stride, nq, s);
    if (!rc) rc = pcp::qsort_finish(ctx, s, &q3, &qi, &nfin);
    if (rc && launched) (void)hipStreamSynchronize(ctx->side);  // the side stream's work is over
    s.release(ctx);
    if (!rc) rc = pcp::icp_make(ctx, ix, q3, qi, nfin, nq, icp_out);
    else {
        pcp::dfree(ctx, q3);
        pcp::dfree(ctx, qi);
    }
    if (rc) {
        if (ix) pcp_index_destroy(ix);
        return rc;
    }
    *index_out = ix;
    return PCP_OK;
}

int pcp_icp_set_options(pcp_icp* icp, int oct_lanes_first, int oct_lanes_list, int ring_lanes, int ablate) {
    if (!icp) return PCP_ERR_ARG;
    auto lanes = [](int v) { return v == 0 || v == 1 || v == 2 || v == 4 || v == 8; };
    pcp_ctx* ctx = icp->owner;
    // every check and allocation first: a failed call leaves the handle as it was
    if (!lanes(oct_lanes_first) || !lanes(oct_lanes_list) || !lanes(ring_lanes) || ablate < 0)
        return pcp::set_error(ctx, PCP_ERR_ARG, "pcp_icp_set_options: lanes must be 0, 1, 2, 4 or 8; ablate >= 0");
    const bool widen = (ablate & PCP_ICP_OPT_WIDE_CACHE) && icp->narrow;
    if (widen && icp->launches > 0)
        return pcp::set_error(ctx, PCP_ERR_ARG, "PCP_ICP_OPT_WIDE_CACHE only before the handle's first launch");
    if (widen) {  // re-create the records in the 16-byte form
        uint32_t* w = nullptr;
        if (int rc = pcp::dmalloc(ctx, &w, (size_t)(icp->nq + 1) * 4)) return rc;
        if (hipMemsetAsync(w, 0xff, (size_t)(icp->nq + 1) * 16, ctx->stream) != hipSuccess) {
            pcp::dfree(ctx, w);
            return pcp::set_error(ctx, PCP_ERR_HIP, "pcp_icp_set_options: memset");
        }
        pcp::dfree(ctx, icp->cand);
        icp->cand = w;
        icp->narrow = false;
    }
    if (icp->gexec) {  // captured with the old lanes / flags
        (void)hipStreamSynchronize(icp->ctx->stream);
        (void)hipGraphExecDestroy(icp->gexec);
        icp->gexec = nullptr;
    }
    icp->oct_g_first = oct_lanes_first ? oct_lanes_first : 1;
    icp->oct_g_list = oct_lanes_list;
    icp->ring_g = ring_lanes;
    icp->dbg = ablate & ~(PCP_ICP_OPT_WIDE_CACHE | PCP_ICP_OPT_GRAPH);
    icp->graph = (ablate & PCP_ICP_OPT_GRAPH) != 0;
    return PCP_OK;
}

int pcp_icp_destroy(pcp_icp* icp) {
    if (!icp) return PCP_ERR_ARG;
    (void)hipSetDevice(icp->owner->device);
    if (icp->gexec) {  // (after its last replay has run)
        (void)hipStreamSynchronize(icp->ctx->stream);
        (void)hipGraphExecDestroy(icp->gexec);
    }
    pcp::dfree(icp->owner, icp->q);
    pcp::dfree(icp->owner, icp->qidx);
    pcp::dfree(icp->owner, icp->partials);
    pcp::dfree(icp->owner, icp->acc);
    pcp::dfree(icp->owner, icp->cand);
    pcp::dfree(icp->owner, icp->pose_hist);
    pcp::dfree(icp->owner, icp->sv);
    pcp::dfree(icp->owner, icp->sv_count);
    pcp::dfree(icp->owner, icp->sv_off);
    pcp::dfree(icp->owner, icp->svc);

    pcp::dfree(icp->owner, icp->fb);
    pcp::dfree(icp->owner, icp->fb_count);
    pcp::dfree(icp->owner, icp->fb_off);
    pcp::dfree(icp->owner, icp->fbc);
    pcp::dfree(icp->owner, icp->pose_dev);
    pcp::event_put(icp->owner, icp->ev0);
    pcp::event_put(icp->owner, icp->ev1);
    pcp::event_put(icp->owner, icp->ev_mid);
    pcp::event_put(icp->owner, icp->ev_ver);
    for (auto& pr : icp->tev) {
        pcp::event_put(icp->owner, pr.first);
        pcp::event_put(icp->owner, pr.second);
    }
    pcp_ctx* owner = icp->owner;
    delete icp;
    pcp::ctx_release(owner);
    return PCP_OK;
}

int pcp_icp_step(pcp_ctx* ctx, pcp_icp* icp, const double T[16], float rmax, double* acc_dev,
                 int32_t* corr_idx, float* corr_d2) {
    if (!ctx || !icp || !T || !acc_dev || (corr_idx && !corr_d2) || !(rmax >= 0.f)) return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    icp->ctx = ctx;
    PCP_TRY(pcp::icp_launch(icp, T, rmax, acc_dev, corr_idx, corr_d2));
    double fbn = 0.0;
    PCP_HIP(ctx, hipMemcpyAsync(&fbn, acc_dev + 23, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    uint32_t nsv = (uint32_t)icp->nq;  // sparse grid / first launch: every query is searched
    if (icp->last_verified)
        PCP_HIP(ctx, hipMemcpyAsync(&nsv, icp->sv_off + icp->nseg_v, sizeof(nsv),
                                    hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    icp->last_fallback = (uint32_t)fbn;
    icp->last_searched = nsv;
    float ms = 0.f;
    PCP_HIP(ctx, hipEventElapsedTime(&ms, icp->ev0, icp->ev1));
    icp->last_ms = ms;
    icp->last_launches = 1;
    if (icp->dbg) {
        float m1 = 0.f, mv = 0.f;
        (void)hipEventElapsedTime(&m1, icp->ev0, icp->ev_mid);
        (void)hipEventElapsedTime(&mv, icp->ev0, icp->ev_ver);
        std::fprintf(stderr, "[pcp icp dbg=%d] verify %.4f ms  octant %.4f ms  fallback %.4f ms  searched %u  "
                     "n_fallback %u\n", icp->dbg, mv, m1 - mv, ms - m1, nsv, icp->last_fallback);
    }
    return PCP_OK;
}

int pcp_icp_keys(pcp_ctx* ctx, pcp_icp* icp, const double T[16], float rmax, int64_t target_offset,
                 uint64_t* keys_dev) {
    if (!ctx || !icp || !T || !keys_dev || !(rmax >= 0.f) || target_offset < 0 ||
        target_offset + pcp_index_size(icp->target) > ((int64_t)1 << 32))
        return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    icp->ctx = ctx;
    const int saved = icp->dbg;
    icp->dbg |= pcp::kDbgNoAccum;  // correspondences only
    pcp::IcpArgs a{};
    const int rc = pcp::icp_launch(icp, T, rmax, icp->acc, nullptr, nullptr, nullptr, &a);
    icp->dbg = saved;
    PCP_TRY(rc);
    if (icp->nq_in > icp->nq)
        hipLaunchKernelGGL(pcp::k_fill_keys, dim3(pcp::grid_for(icp->nq_in, 256)), dim3(256), 0, ctx->stream, keys_dev,
                           icp->nq_in);
    if (icp->nq > 0)
        hipLaunchKernelGGL(pcp::k_make_keys, dim3(pcp::grid_for(icp->nq, 256)), dim3(256), 0, ctx->stream, a,
                           (uint32_t)target_offset, keys_dev);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_icp_keys_dev(pcp_ctx* ctx, pcp_icp* icp, const double* T_dev, float rmax, int64_t target_offset,
                     uint64_t* keys_dev) {
    if (!ctx || !icp || !T_dev || !keys_dev || !(rmax >= 0.f) || target_offset < 0 ||
        target_offset + pcp_index_size(icp->target) > ((int64_t)1 << 32))
        return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    icp->ctx = ctx;
    const int saved = icp->dbg;
    icp->dbg |= pcp::kDbgNoAccum;  // correspondences only
    pcp::IcpArgs a{};
    const int rc = pcp::icp_launch(icp, nullptr, rmax, icp->acc, nullptr, nullptr, T_dev, &a);
    icp->dbg = saved;
    PCP_TRY(rc);
    if (icp->nq_in > icp->nq)
        hipLaunchKernelGGL(pcp::k_fill_keys, dim3(pcp::grid_for(icp->nq_in, 256)), dim3(256), 0, ctx->stream, keys_dev,
                           icp->nq_in);
    if (icp->nq > 0)
        hipLaunchKernelGGL(pcp::k_make_keys, dim3(pcp::grid_for(icp->nq, 256)), dim3(256), 0, ctx->stream, a,
                           (uint32_t)target_offset, keys_dev);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_keys_owner(pcp_ctx* ctx, const uint64_t* keys_dev, int64_t n, const int64_t* bounds_dev, int nshards,
                   uint8_t* owner_dev) {
    if (!ctx || n < 0 || (n > 0 && (!keys_dev || !owner_dev)) || !bounds_dev || nshards < 1 || nshards > 255)
        return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    if (n == 0) return PCP_OK;
    hipLaunchKernelGGL(pcp::k_keys_owner, dim3(pcp::grid_for(n, 256, 8192)), dim3(256), 0, ctx->stream, keys_dev, n,
                       bounds_dev, nshards, owner_dev);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_icp_accumulate_owned(pcp_ctx* ctx, const double* T_dev, const float* q_dev, size_t q_stride, int64_t nq,
                             const uint64_t* keys_dev, const uint8_t* owner_dev, int rank, int64_t lo, int64_t hi,
                             const float* shard_xyz_dev, size_t shard_stride, double* acc_dev) {
    if (!ctx || !T_dev || nq < 0 || (nq > 0 && (!q_dev || !keys_dev || !owner_dev)) || !acc_dev || rank < 0 ||
        rank > 254 || lo < 0 || hi < lo || (hi > lo && !shard_xyz_dev))
        return PCP_ERR_ARG;
    if (q_stride == 0) q_stride = 3 * sizeof(float);
    if (shard_stride == 0) shard_stride = 3 * sizeof(float);
    if (q_stride % sizeof(float) || shard_stride % sizeof(float))
        return pcp::set_error(ctx, PCP_ERR_ARG, "strides must be whole floats");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    const int nb = (int)std::min<int64_t>(std::max<int64_t>(1, (nq + 255) / 256), 2048);
    double* part = nullptr;
    PCP_TRY(pcp::dmalloc(ctx, &part, (size_t)nb * pcp::kAcc));
    hipLaunchKernelGGL(pcp::k_acc_owned, dim3(nb), dim3(256), 0, ctx->stream, T_dev, q_dev, q_stride / sizeof(float),
                       nq, keys_dev, owner_dev, rank, lo, hi, shard_xyz_dev, shard_stride / sizeof(float), part);
    hipLaunchKernelGGL(pcp::k_sum_partials, dim3(1), dim3(256), 0, ctx->stream, (const double*)part, nb, acc_dev);
    pcp::dfree(ctx, part);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_slab_guard(pcp_ctx* ctx, const double* T_dev, const double box[6], double lo, double hi, int* flag_dev) {
    if (!ctx || !T_dev || !box || !flag_dev) return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(pcp::k_slab_guard, dim3(1), dim3(1), 0, ctx->stream, T_dev, box[0], box[1], box[2], box[3],
                       box[4], box[5], lo, hi, flag_dev);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_icp_accumulate_keys(pcp_ctx* ctx, pcp_icp* icp, const double T[16], const uint64_t* keys_dev,
                            int64_t lo, int64_t hi, const float* shard_xyz_dev, size_t shard_stride_bytes,
                            double* acc_dev) {
    if (!ctx || !icp || !T || !keys_dev || !acc_dev || lo < 0 || hi < lo || (hi > lo && !shard_xyz_dev))
        return PCP_ERR_ARG;
    if (shard_stride_bytes == 0) shard_stride_bytes = 3 * sizeof(float);
    if (shard_stride_bytes % sizeof(float)) return pcp::set_error(ctx, PCP_ERR_ARG, "shard stride must be whole floats");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    pcp::IcpArgs a{};
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) a.R[3 * r + c] = (float)T[4 * r + c];
        a.t[r] = (float)T[4 * r + 3];
    }
    const int nb = (int)std::min<int64_t>(std::max<int64_t>(1, (icp->nq + 255) / 256), icp->nb_fast + icp->nb_ring);
    hipLaunchKernelGGL(pcp::k_acc_keys, dim3(nb), dim3(256), 0, ctx->stream, icp->q, icp->qidx, icp->nq, keys_dev,
                       (uint64_t)lo, (uint64_t)hi, shard_xyz_dev, shard_stride_bytes / sizeof(float), a,
                       icp->partials);
    hipLaunchKernelGGL(pcp::k_sum_partials, dim3(1), dim3(256), 0, ctx->stream, (const double*)icp->partials, nb,
                       acc_dev);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_icp_solve(const double acc[24], int do_scale, double dT[16]) {
    if (!acc || !dT) return PCP_ERR_ARG;
    return pcp::icp_solve(acc, do_scale, dT);
}

int pcp_icp_run(pcp_ctx* ctx, pcp_icp* icp, double T[16], float rmax, int iters, int do_scale, double eps,
                float* err) {
    if (!ctx || !icp || !T || iters < 0) return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    icp->ctx = ctx;
    double e = -1.0, ms_total = 0.0;
    int launches = 0;
    for (int it = 0; it < iters; it++) {
        PCP_TRY(pcp::icp_launch(icp, T, rmax, icp->acc, nullptr, nullptr));
        double acc[24];
        PCP_HIP(ctx, hipMemcpyAsync(acc, icp->acc, sizeof(acc), hipMemcpyDeviceToHost, ctx->stream));
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
        float ms = 0.f;
        PCP_HIP(ctx, hipEventElapsedTime(&ms, icp->ev0, icp->ev1));
        ms_total += ms;
        launches++;
        double dT[16];
        if (pcp::icp_solve(acc, do_scale, dT) != PCP_OK) {
            e = -1.0;
            break;
        }
        e = std::sqrt(acc[22] / acc[0]);
        double Tn[16];
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) {
                double s = 0;
                for (int k = 0; k < 4; k++) s += dT[4 * i + k] * T[4 * k + j];
                Tn[4 * i + j] = s;
            }
        std::memcpy(T, Tn, sizeof(Tn));
        if (eps > 0) {
            double rot = std::fabs(dT[0] - 1) + std::fabs(dT[5] - 1) + std::fabs(dT[10] - 1) +
                         std::fabs(dT[1]) + std::fabs(dT[2]) + std::fabs(dT[6]);
            double tr = std::fabs(dT[3]) + std::fabs(dT[7]) + std::fabs(dT[11]);
            if (rot < eps && tr < eps) break;
        }
    }
    icp->last_ms = ms_total;
    icp->last_launches = launches;
    if (err) *err = (float)e;
    return e < 0 ? PCP_ERR_ICP : PCP_OK;
}

int pcp_icp_step_dev(pcp_ctx* ctx, pcp_icp* icp, const double* T_dev, float rmax, double* acc_dev) {
    if (!ctx || !icp || !T_dev || !acc_dev || !(rmax >= 0.f)) return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    icp->ctx = ctx;
    return pcp::icp_launch(icp, nullptr, rmax, acc_dev, nullptr, nullptr, T_dev);
}

int pcp_icp_solve_dev(pcp_ctx* ctx, const double* acc_dev, int do_scale, double* T_dev, double* stats_dev) {
    if (!ctx || !acc_dev || !T_dev || !stats_dev) return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(pcp::k_icp_solve_dev, dim3(1), dim3(1), 0, ctx->stream, acc_dev, do_scale, T_dev, stats_dev);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_icp_run_dev(pcp_ctx* ctx, pcp_icp* icp, double* T_dev, float rmax, int iters, int do_scale,
                    double* stats_dev) {
    if (!ctx || !icp || !T_dev || !stats_dev || iters < 0 || !(rmax >= 0.f)) return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    icp->ctx = ctx;
    for (int it = 0; it < iters; it++) {
        PCP_TRY(pcp::icp_launch(icp, nullptr, rmax, icp->acc, nullptr, nullptr, T_dev));
        hipLaunchKernelGGL(pcp::k_icp_solve_dev, dim3(1), dim3(1), 0, ctx->stream, (const double*)icp->acc, do_scale,
                           T_dev, stats_dev);
    }
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_icp_kernel_ms(pcp_ctx* ctx, pcp_icp* icp, double* ms, int* launches) {
    if (!ctx || !icp) return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    double tot = 0.0;
    for (size_t i = 0; i < icp->ntev; i++) {
        PCP_HIP(ctx, hipEventSynchronize(icp->tev[i].second));
        float m = 0.f;
        PCP_HIP(ctx, hipEventElapsedTime(&m, icp->tev[i].first, icp->tev[i].second));
        tot += m;
    }
    if (ms) *ms = tot;
    if (launches) *launches = (int)icp->ntev;
    icp->ntev = 0;
    return PCP_OK;
}

int pcp_icp_last_fallback(const pcp_icp* icp, int64_t* n) {
    if (!icp || !n) return PCP_ERR_ARG;
    *n = icp->last_fallback;
    return PCP_OK;
}

int pcp_icp_last_searched(const pcp_icp* icp, int64_t* n) {
    if (!icp || !n) return PCP_ERR_ARG;
    *n = icp->last_searched;
    return PCP_OK;
}

int pcp_icp_last_kernel_ms(const pcp_icp* icp, double* ms, int* launches) {
    if (!icp) return PCP_ERR_ARG;
    if (ms) *ms = icp->last_ms;
    if (launches) *launches = icp->last_launches;
    return PCP_OK;
}

}  // extern "C"
