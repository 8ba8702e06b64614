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

#include "grid.hpp"

struct pcp_icp {
    pcp_ctx* ctx = nullptr;
    const pcp_index* target = nullptr;
    int64_t nq = 0;               // finite queries
    int64_t nq_in = 0;            // queries passed to pcp_icp_create
    float4* q = nullptr;          // sorted queries {x,y,z,bits(original index)}
    int32_t* win = nullptr;       // per sorted query: winning target index (-1 = rejected)
    float* wd2 = nullptr;         // per sorted query: winning d2 (+inf = rejected)
    int32_t* fb = nullptr;        // fallback lists: one segment of fb_seg entries per octant WG
    uint32_t* fb_count = nullptr; // per octant wave: entries in its segment
    uint32_t* fb_off = nullptr;   // exclusive scan of fb_count (+ total)
    int32_t* fbc = nullptr;       // compacted fallback list
    int64_t fb_seg = 0;
    double* partials = nullptr;   // (nb_fast + nb_ring) * 24
    double* acc = nullptr;        // 24 (scratch for pcp_icp_run)
    int nb_fast = 0, nb_ring = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_mid = nullptr;
    float* pose_dev = nullptr;    // 12 floats (R row-major, t) for the device-resident loop
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;  // per-launch timing events (device loop)
    size_t ntev = 0;              // pairs recorded since the last pcp_icp_kernel_ms
    int dbg = 0;                  // PCP_ICP_ABLATE flags (profiling only)
    double last_ms = 0.0;
    int last_launches = 0;
    uint32_t last_fallback = 0;
};

namespace pcp {
namespace {

constexpr int kIcpBlock = 256;
#ifndef PCP_OCT_WAVES
#define PCP_OCT_WAVES 8
#endif
constexpr int kAcc = 24;

struct IcpArgs {
    GridDesc g;
    const float4* tp;   // sorted target points
    const float4* q;    // sorted queries
    int64_t nq;
    int64_t nchunks;
    float R[9], t[3];
    float r2;
    float cert2;        // certified radius^2 of the 2x2x2 octant search
    float rho;          // octant half-width in cell units (0.5 - margin)
    float mc;           // cell-unit margin for pruning
    double* partials;
    int32_t* win;
    float* wd2;
    int32_t* fb;
    uint32_t* fb_count;
    uint32_t* fb_off;   // nseg + 1: the counts again, scanned in place after the pass
    int64_t fb_seg;
    int nb_fast;
    int64_t nseg;       // fallback segments (= waves of the octant kernel)
    int ring_all;       // ring kernel: process every query (sparse grid) instead of the list
    int dbg;            // ablation flags (PCP_ICP_ABLATE, profiling builds of the bench only)
    const float* pose;  // device pose (R row-major, t) overriding R/t, or null
};

// the pose as the kernels use it: from the device copy when the loop is device-resident
__device__ __forceinline__ void load_pose(IcpArgs& a) {
    if (a.pose) {
#pragma unroll
        for (int k = 0; k < 9; k++) a.R[k] = a.pose[k];
#pragma unroll
        for (int k = 0; k < 3; k++) a.t[k] = a.pose[9 + k];
    }
}

// Ablation switches for profiling (env PCP_ICP_ABLATE); results are wrong when any is set.
constexpr int kDbgNoScan = 1, kDbgNoAccum = 4, kDbgNoFallback = 8;

__device__ __forceinline__ void xform(const IcpArgs& a, const float4 q, float& x, float& y, float& z) {
    // q' = R q + t: x' = fmaf(R02,z,fmaf(R01,y,fmaf(R00,x,t0)))
    x = __fmaf_rn(a.R[2], q.z, __fmaf_rn(a.R[1], q.y, __fmaf_rn(a.R[0], q.x, a.t[0])));
    y = __fmaf_rn(a.R[5], q.z, __fmaf_rn(a.R[4], q.y, __fmaf_rn(a.R[3], q.x, a.t[1])));
    z = __fmaf_rn(a.R[8], q.z, __fmaf_rn(a.R[7], q.y, __fmaf_rn(a.R[6], q.x, a.t[2])));
}

// running 1-NN: best d2, its target index (tie order) and its position in the scanned array
#ifndef PCP_SCAN_UNROLL
#define PCP_SCAN_UNROLL 4
#endif
#ifndef PCP_TRACK_BEST
#define PCP_TRACK_BEST 0
#endif
struct Best {
    float bd;
    int bj;
    uint32_t bk;
    float px, py, pz;  // filled by fetch() once the scan is over (or tracked, PCP_TRACK_BEST)
    __device__ __forceinline__ void consider(float qx, float qy, float qz, const float4 p, uint32_t k) {
        const float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
        const float d2 = __fmaf_rn(dz, dz, __fmaf_rn(dy, dy, dx * dx));
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
        auto addr = [&](uint32_t v) {
            return v < c1 ? rs[0] + v
                          : (v < c2 ? rs[1] + (v - c1) : ((NR == 3 || v < c3) ? rs[2] + (v - c2) : rs[NR - 1] + (v - c3)));
        };
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
__device__ __forceinline__ void box_search(const GridDesc& g, const float4* tp, float qx, float qy,
                                           float qz, float mc, Best& b) {
    const float fx = cell_f<float>(g, qx, 0), fy = cell_f<float>(g, qy, 1), fz = cell_f<float>(g, qz, 2);
    const int cy = (int)floorf(fy), cz = (int)floorf(fz);
    const float ly = fy - (float)cy, lz = fz - (float)cz;
    const float inv_h2 = g.inv_hf * g.inv_hf;
    const float rc = sqrtf(b.bd * 1.00002f * inv_h2) + mc;  // initial radius in cells
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
            const float lim = b.bd * 1.00002f * inv_h2 - gyz2;  // remaining x extent^2 (cells)
            if (lim < 0.f) continue;
            const float rx = sqrtf(lim) + mc;
            const int xa = max((int)floorf(fx - rx), 0), xb = min((int)floorf(fx + rx), g.n[0] - 1);
            if (xa > xb) continue;
            if (g.dense) {
                const int64_t c = dense_id(g, xa, y, z);
                b.scan(tp, g.cstart[c], g.cstart[c + (xb - xa + 1)], qx, qy, qz);
            } else {
                for (int x = xa; x <= xb; x++) {
                    uint32_t s, e;
                    if (cell_range(g, x, y, z, s, e)) b.scan(tp, s, e, qx, qy, qz);
                }
            }
        }
    }
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
// fp32 products centred on lane 0's query, summed across the wave with DPP adds, then
// un-centred in fp64 by lane 0.  Every lane of the wave must call it (full EXEC).
__device__ __forceinline__ void chunk_accumulate(bool ok, float qx, float qy, float qz, const Best& b,
                                                 double* S, int lane) {
    if (!__ballot(ok)) return;
    const float ccx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qx), 0));
    const float ccy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qy), 0));
    const float ccz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qz), 0));
    const float x0 = ok ? qx - ccx : 0.f, x1 = ok ? qy - ccy : 0.f, x2 = ok ? qz - ccz : 0.f;
    const float p0 = ok ? b.px - ccx : 0.f, p1 = ok ? b.py - ccy : 0.f, p2 = ok ? b.pz - ccz : 0.f;
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

__global__ void __launch_bounds__(kIcpBlock, PCP_OCT_WAVES) k_icp_octant(IcpArgs a) {
    load_pose(a);
    constexpr int kW = kIcpBlock / 64;
    __shared__ double s_acc[kW][kAcc];
    const GridDesc& g = a.g;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * kW + wid;  // global wave id = fallback segment
    const int64_t nwaves = (int64_t)gridDim.x * kW;
    const int64_t nch = (a.nq + 63) / 64;
    if (lane < kAcc) s_acc[wid][lane] = 0.0;
    uint32_t fbn = 0;  // wave-uniform count of this wave's fallback entries

    float4 qn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gw < nch && gw * 64 + lane < a.nq) qn = a.q[gw * 64 + lane];
    for (int64_t c = gw; c < nch; c += nwaves) {
        const int64_t i = c * 64 + lane;
        const bool valid = i < a.nq;
        const float4 qraw = qn;
        if (c + nwaves < nch && i + 64 * nwaves < a.nq) qn = a.q[i + 64 * nwaves];  // prefetch
        Best b{a.r2, 0x7fffffff, ~0u, 0.f, 0.f, 0.f};
        float qx = 0.f, qy = 0.f, qz = 0.f;
        int bx = 0, by = 0, bz = 0;
        float cert2 = a.cert2;
        if (valid) {
            xform(a, qraw, qx, qy, qz);
            const float fx = cell_f<float>(g, qx, 0), fy = cell_f<float>(g, qy, 1), fz = cell_f<float>(g, qz, 2);
            bx = (int)floorf(fx - a.rho);
            by = (int)floorf(fy - a.rho);
            bz = (int)floorf(fz - a.rho);
            // this query's certified radius: its distance to the nearest face of the 2x2x2
            // block (>= 0.5 cell, the worst case a.cert2 is built from), less the margin
            const float m = fminf(fminf(fminf(fx - (float)bx, (float)(bx + 2) - fx),
                                        fminf(fy - (float)by, (float)(by + 2) - fy)),
                                  fminf(fz - (float)bz, (float)(bz + 2) - fz)) - a.mc;
            const float rr = m * g.hf;
            cert2 = fmaxf(a.cert2, rr * rr * (1.f - 2e-5f));
        }
        if (valid && !(a.dbg & kDbgNoScan)) {
            // the 4 x-rows of the octant: all 8 row bounds are loaded at once, then the rows
            // are scanned as one concatenated candidate list with 4 loads in flight, so a
            // chunk costs ~1 + L/4 memory round trips instead of 4 x (1 + len/4)
            const int xa = max(bx, 0), xb = min(bx + 1, g.n[0] - 1);
            uint32_t rs[4], rn[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int y = by + (r & 1), z = bz + (r >> 1);
                const bool in = xa <= xb && y >= 0 && y < g.n[1] && z >= 0 && z < g.n[2];
                const int64_t cc = in ? dense_id(g, xa, y, z) : 0;
                rs[r] = in ? g.cstart[cc] : 0u;
                rn[r] = in ? g.cstart[cc + (xb - xa + 1)] : 0u;
            }
#pragma unroll
            for (int r = 0; r < 4; r++) rn[r] -= rs[r];
            b.scan_rows(a.tp, rs, rn, qx, qy, qz);
        }
        // ---- epilogue: results, fallback list, accumulators
        const bool found = b.bj != 0x7fffffff;
        const bool done = valid && ((found && b.bd <= cert2) || (!found && a.r2 <= cert2) ||
                                    (a.dbg & kDbgNoFallback));
        if (valid) {  // provisional for fallback queries (an upper bound), final otherwise
            a.win[i] = found ? b.bj : -1;
            a.wd2[i] = found ? b.bd : INFINITY;
        }
        const bool fb = valid && !done;
        const uint64_t fbm = __ballot(fb);
        if (fb) {
            const uint32_t pos = fbn + __builtin_amdgcn_mbcnt_hi((uint32_t)(fbm >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)fbm, 0u));
            a.fb[gw * a.fb_seg + pos] = (int32_t)i;
        }
        fbn += (uint32_t)__popcll(fbm);
        const bool acc_ok = done && found && !(a.dbg & kDbgNoAccum);
#if !PCP_TRACK_BEST
        if (acc_ok) b.fetch(a.tp);
#endif
        chunk_accumulate(acc_ok, qx, qy, qz, b, s_acc[wid], lane);
    }
    if (lane == 0) {  // every wave of the grid writes its count: no zeroing pass needed
        a.fb_count[gw] = fbn;
        a.fb_off[gw] = fbn;  // scanned in place into the segment offsets
        if (gw == 0) a.fb_off[a.nseg] = 0u;
    }
    write_wave_partials(s_acc, a.partials + (int64_t)blockIdx.x * kAcc);
}

// Fallback / general pass: exact box search (dense or sparse grid), starting from the
// octant pass's provisional winner when it has one.  Queries come from the compacted
// fallback list (or are all queries when ring_all is set, i.e. on a sparse grid); waves
// take 64-entry chunks grid-stride and accumulate like the octant pass.
__global__ void __launch_bounds__(kIcpBlock, PCP_OCT_WAVES) k_icp_ring(IcpArgs a, double* partials,
                                                                        const int32_t* list, const uint32_t* list_n) {
    load_pose(a);
    constexpr int kW = kIcpBlock / 64;
    __shared__ double s_acc[kW][kAcc];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane < kAcc) s_acc[wid][lane] = 0.0;
    const int64_t n = a.ring_all ? a.nq : (int64_t)*list_n;
    const int64_t gw = (int64_t)blockIdx.x * kW + wid, nwaves = (int64_t)gridDim.x * kW;
    for (int64_t c = gw; c * 64 < n; c += nwaves) {
        const int64_t j = c * 64 + lane;
        const bool valid = j < n;
        Best b{a.r2, 0x7fffffff, 0u, 0.f, 0.f, 0.f};
        float qx = 0.f, qy = 0.f, qz = 0.f;
        int64_t i = 0;
        if (valid) {
            i = a.ring_all ? j : list[j];
            xform(a, a.q[i], qx, qy, qz);
            if (!a.ring_all && a.win[i] >= 0) {  // provisional octant winner: a valid upper bound
                b.bd = a.wd2[i];
                b.bj = a.win[i];
            }
            bool done = false;
            if (!a.ring_all) {
                // stage 2: the 3x3x3 cells around the query, as 3 planes of 3 x-rows scanned
                // like the octant pass; certifies any winner within the distance to the
                // block's faces (>= 1 cell).  Only what is left goes to the general search.
                const GridDesc& g = a.g;
                const float fx = cell_f<float>(g, qx, 0), fy = cell_f<float>(g, qy, 1), fz = cell_f<float>(g, qz, 2);
                const int cx = (int)floorf(fx), cy = (int)floorf(fy), cz = (int)floorf(fz);
                const int xa = max(cx - 1, 0), xb = min(cx + 1, g.n[0] - 1);
                if (xa <= xb) {
                    for (int dz = -1; dz <= 1; dz++) {
                        const int z = cz + dz;
                        uint32_t rs[3], rn[3];
#pragma unroll
                        for (int r = 0; r < 3; r++) {
                            const int y = cy - 1 + r;
                            const bool in = y >= 0 && y < g.n[1] && z >= 0 && z < g.n[2];
                            const int64_t cc = in ? dense_id(g, xa, y, z) : 0;
                            rs[r] = in ? g.cstart[cc] : 0u;
                            rn[r] = in ? g.cstart[cc + (xb - xa + 1)] - rs[r] : 0u;
                        }
                        b.scan_rows(a.tp, rs, rn, qx, qy, qz);
                    }
                }
                const float m = fminf(fminf(fminf(fx - (float)(cx - 1), (float)(cx + 2) - fx),
                                            fminf(fy - (float)(cy - 1), (float)(cy + 2) - fy)),
                                      fminf(fz - (float)(cz - 1), (float)(cz + 2) - fz)) - a.mc;
                const float rr = m * g.hf;
                const float c2 = rr * rr * (1.f - 2e-5f);
                const bool found = b.bj != 0x7fffffff;
                done = (found && b.bd <= c2) || (!found && a.r2 <= c2);
            }
            if (!done) box_search(a.g, a.tp, qx, qy, qz, a.mc, b);
            const bool ok = b.bj != 0x7fffffff;
            a.win[i] = ok ? b.bj : -1;
            a.wd2[i] = ok ? b.bd : INFINITY;
        }
        const bool acc_ok = valid && b.bj != 0x7fffffff && !(a.dbg & kDbgNoAccum);
        if (acc_ok) b.fetch(a.tp);
        chunk_accumulate(acc_ok, qx, qy, qz, b, s_acc[wid], lane);
    }
    write_wave_partials(s_acc, partials + (int64_t)blockIdx.x * kAcc);
}

// concatenate the per-wave fallback segments (one wave per segment)
__global__ void k_fb_compact(const int32_t* fb, const uint32_t* cnt, const uint32_t* off, int64_t nseg,
                             int64_t seg_cap, int32_t* out) {
    const int64_t seg = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (seg >= nseg) return;
    const uint32_t n = cnt[seg], o = off[seg];
    for (uint32_t k = threadIdx.x & 63; k < n; k += 64) out[o + k] = fb[seg * seg_cap + k];
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

// sorted-order winners -> caller (original query) order
__global__ void k_scatter_corr(const float4* q, const int32_t* win, const float* wd2, int64_t n,
                               int32_t* idx, float* d2) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int oq = __float_as_int(q[i].w);
        idx[oq] = win[i];
        d2[oq] = wd2[i];
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

__global__ void k_make_keys(const float4* q, const int32_t* win, const float* wd2, int64_t n, uint32_t offset,
                            uint64_t* keys) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int oq = __float_as_int(q[i].w);
        const int w = win[i];
        keys[oq] = w < 0 ? kNoKey
                         : (((uint64_t)__float_as_uint(wd2[i]) << 32) | (uint64_t)(uint32_t)((uint32_t)w + offset));
    }
}

// accumulators over the queries whose global winner lies in [lo, hi) (this rank's shard);
// float products are exact in fp64, so only the summation order differs from the oracle
__global__ void __launch_bounds__(256) k_acc_keys(const float4* q, int64_t n, const uint64_t* keys, uint64_t lo,
                                                  uint64_t hi, const float* shard, size_t stride_f, IcpArgs a,
                                                  double* partials) {
    double acc[kAcc - 1];
#pragma unroll
    for (int k = 0; k < kAcc - 1; k++) acc[k] = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 qq = q[i];
        const uint64_t key = keys[__float_as_int(qq.w)];
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

// ---- query order (pcp_icp_create): queries sorted once by target-grid cell in brick-major
// order (4x4x4-cell bricks; stable, so input order inside a cell), carried as float4
// {x, y, z, bits(index)}
// through the radix sort; non-finite queries get key 64 * nbricks (after every cell) and
// are dropped.
__global__ void k_query_keys(GridDesc g, const float* q, size_t stride_f, int64_t n, uint32_t* key, float4* rec) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float* p = q + (size_t)i * stride_f;
        const float x = p[0], y = p[1], z = p[2];
        const bool fin = isfinite(x) && isfinite(y) && isfinite(z);
        uint32_t k = (uint32_t)(g.nbricks * 64);  // past every cell: non-finite queries sort last
        if (fin) {
            // dual cell = the octant block origin floor(f - 1/2) the main pass will use: lanes
            // with the same block scan the same target rows, so their loads coalesce
            const int cx = clampi((int)floorf(cell_f<float>(g, x, 0) - 0.5f), 0, g.n[0] - 1);
            const int cy = clampi((int)floorf(cell_f<float>(g, y, 1) - 0.5f), 0, g.n[1] - 1);
            const int cz = clampi((int)floorf(cell_f<float>(g, z, 2) - 0.5f), 0, g.n[2] - 1);
            k = (uint32_t)(brick_of(g, cx, cy, cz) * 64 + local_of(cx, cy, cz));  // brick-major block order
        }
        key[i] = k;
        rec[i] = make_float4(x, y, z, __int_as_float((int)i));
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

// device pose for the kernels: R, t of T (row-major 4x4 doubles) cast to fp32 as on the host
__global__ void k_pose_from_T(const double* T, float* pose) {
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) pose[3 * r + c] = (float)T[4 * r + c];
        pose[9 + r] = (float)T[4 * r + 3];
    }
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
               float* corr_d2, const double* T_dev = nullptr) {
    pcp_ctx* ctx = icp->ctx;
    const pcp_index* tg = icp->target;
    IcpArgs a;
    a.g = tg->g;
    a.tp = (const float4*)tg->pts;
    a.q = icp->q;
    a.nq = icp->nq;
    a.nchunks = (icp->nq + kIcpBlock - 1) / kIcpBlock;
    a.pose = nullptr;
    if (T_dev) {
        hipLaunchKernelGGL(k_pose_from_T, dim3(1), dim3(1), 0, ctx->stream, T_dev, icp->pose_dev);
        a.pose = icp->pose_dev;
        for (int k = 0; k < 9; k++) a.R[k] = 0.f;
        for (int k = 0; k < 3; k++) a.t[k] = 0.f;
    } else {
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) a.R[3 * r + c] = (float)T[4 * r + c];
            a.t[r] = (float)T[4 * r + 3];
        }
    }
    a.r2 = rmax * rmax;
    const int nmax = std::max(a.g.n[0], std::max(a.g.n[1], a.g.n[2]));
    a.mc = 1e-5f + 8e-7f * (float)nmax;  // >> fp32 rounding of the cell coordinates
    a.rho = 0.5f;
    // exact radius of the octant block: (0.5 - mc) cells, shrunk for fp32 d2 rounding
    const double rr = (0.5 - (double)a.mc) * a.g.h;
    a.cert2 = (float)(rr * rr * (1.0 - 1e-5));
    a.partials = icp->partials;
    a.win = icp->win;
    a.wd2 = icp->wd2;
    a.fb = icp->fb;
    a.fb_count = icp->fb_count;
    a.fb_off = icp->fb_off;
    a.fb_seg = icp->fb_seg;
    a.nb_fast = icp->nb_fast;
    a.nseg = (int64_t)icp->nb_fast * (kIcpBlock / 64);
    a.ring_all = a.g.dense ? 0 : 1;
    a.dbg = icp->dbg;
    hipEvent_t e0 = icp->ev0, e1 = icp->ev1;
    if (T_dev) {  // device-resident loop: one event pair per launch, read by pcp_icp_kernel_ms
        if (icp->ntev == icp->tev.size()) {
            std::pair<hipEvent_t, hipEvent_t> pr{nullptr, nullptr};
            PCP_HIP(ctx, hipEventCreate(&pr.first));
            if (hipEventCreate(&pr.second) != hipSuccess) {
                (void)hipEventDestroy(pr.first);
                return set_error(ctx, PCP_ERR_HIP, "hipEventCreate");
            }
            icp->tev.push_back(pr);
        }
        e0 = icp->tev[icp->ntev].first;
        e1 = icp->tev[icp->ntev].second;
        icp->ntev++;
    }
    PCP_HIP(ctx, hipEventRecord(e0, ctx->stream));
    if (a.g.dense) {
        hipLaunchKernelGGL(k_icp_octant, dim3(icp->nb_fast), dim3(kIcpBlock), 0, ctx->stream, a);
    } else {
        PCP_HIP(ctx, hipMemsetAsync(icp->partials, 0, (size_t)icp->nb_fast * kAcc * sizeof(double), ctx->stream));
    }
    if (icp->dbg) PCP_HIP(ctx, hipEventRecord(icp->ev_mid, ctx->stream));
    if (a.g.dense) {  // compact the per-wave fallback segments into one list
        PCP_TRY(scan_u32_inplace(ctx, icp->fb_off, a.nseg + 1, nullptr));
        hipLaunchKernelGGL(k_fb_compact, dim3((unsigned)((a.nseg + 3) / 4)), dim3(256), 0, ctx->stream, icp->fb,
                           (const uint32_t*)icp->fb_count, (const uint32_t*)icp->fb_off, a.nseg, a.fb_seg, icp->fbc);
    }
    hipLaunchKernelGGL(k_icp_ring, dim3(icp->nb_ring), dim3(kIcpBlock), 0, ctx->stream, a,
                       icp->partials + (int64_t)icp->nb_fast * kAcc, (const int32_t*)icp->fbc,
                       (const uint32_t*)(icp->fb_off + a.nseg));
    PCP_HIP(ctx, hipEventRecord(e1, ctx->stream));
    hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(kAcc * kRedGroups), 0, ctx->stream, icp->partials,
                       icp->nb_fast + icp->nb_ring, acc_dev,
                       a.g.dense ? (const uint32_t*)(icp->fb_off + a.nseg) : nullptr);
    if (corr_idx) {
        if (icp->nq_in > icp->nq)  // non-finite queries were dropped at create time
            hipLaunchKernelGGL(k_fill_corr, dim3(grid_for(icp->nq_in, 256)), dim3(256), 0, ctx->stream, corr_idx,
                               corr_d2, icp->nq_in);
        if (icp->nq > 0)
            hipLaunchKernelGGL(k_scatter_corr, dim3(grid_for(icp->nq, 256)), dim3(256), 0, ctx->stream, icp->q,
                               icp->win, icp->wd2, icp->nq, corr_idx, corr_d2);
    }
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

int pcp_icp_create(pcp_ctx* ctx, const pcp_index* target, const float* q, size_t q_stride, int64_t nq,
                   pcp_icp** out) {
    if (!ctx || !target || !out || nq < 0 || (nq > 0 && !q)) return PCP_ERR_ARG;
    if (target->is_f64) return pcp::set_error(ctx, PCP_ERR_ARG, "ICP target must be an fp32 index");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    *out = nullptr;
    if (q_stride == 0) q_stride = 3 * sizeof(float);
    if (q_stride % sizeof(float)) return pcp::set_error(ctx, PCP_ERR_ARG, "query stride must be whole floats");
    if (nq >= ((int64_t)1 << 31)) return pcp::set_error(ctx, PCP_ERR_ARG, "ICP supports < 2^31 queries");
    if (target->g.nbricks * 64 >= ((int64_t)1 << 32))
        return pcp::set_error(ctx, PCP_ERR_UNSUPPORTED, "ICP target grid too large for 32-bit cell keys");
    // sort the query set once by target-grid brick (stable radix sort, record as payload)
    hipStream_t st = ctx->stream;
    float4* qs = nullptr;
    int64_t nfin = 0;
    {
        uint32_t *k0 = nullptr, *k1 = nullptr;
        float4* r0 = nullptr;
        unsigned long long* d_cnt = nullptr;
        void* tmp = nullptr;
        int rc = pcp::dmalloc(ctx, &k0, nq);
        if (!rc) rc = pcp::dmalloc(ctx, &k1, nq);
        if (!rc) rc = pcp::dmalloc(ctx, &r0, nq);
        if (!rc) rc = pcp::dmalloc(ctx, &qs, nq + 1);
        if (!rc) rc = pcp::dmalloc(ctx, &d_cnt, 1);
        if (!rc && hipMemsetAsync(d_cnt, 0, sizeof(unsigned long long), st) != hipSuccess)
            rc = pcp::set_error(ctx, PCP_ERR_HIP, "memset");
        if (!rc && nq > 0) {
            hipLaunchKernelGGL(pcp::k_query_keys, dim3(pcp::grid_for(nq, 256)), dim3(256), 0, st, target->g, q,
                               q_stride / sizeof(float), nq, k0, r0);
            unsigned bits = 1;  // keys are in [0, 64 * nbricks]
            while (bits < 32 && ((uint64_t)1 << bits) <= (uint64_t)target->g.nbricks * 64) bits++;
            size_t tb = 0;
            hipError_t e = rocprim::radix_sort_pairs(nullptr, tb, k0, k1, r0, qs, (size_t)nq, 0u, bits, st);
            if (e == hipSuccess && !(rc = pcp::dmalloc(ctx, (char**)&tmp, tb)))
                e = rocprim::radix_sort_pairs(tmp, tb, k0, k1, r0, qs, (size_t)nq, 0u, bits, st);
            if (!rc && e == hipSuccess)
                hipLaunchKernelGGL(pcp::k_first_at_least, dim3(1), dim3(1), 0, st, k1, nq,
                                   (uint32_t)(target->g.nbricks * 64), d_cnt);
            unsigned long long hc = 0;
            if (!rc && e == hipSuccess) e = hipMemcpyAsync(&hc, d_cnt, sizeof(hc), hipMemcpyDeviceToHost, st);
            if (!rc && e == hipSuccess) e = hipStreamSynchronize(st);
            if (!rc && e != hipSuccess) rc = pcp::hip_fail(ctx, e, "query sort", __FILE__, __LINE__);
            nfin = (int64_t)hc;
        }
        pcp::dfree(ctx, k0);
        pcp::dfree(ctx, k1);
        pcp::dfree(ctx, r0);
        pcp::dfree(ctx, d_cnt);
        pcp::dfree(ctx, tmp);
        if (rc) {
            pcp::dfree(ctx, qs);
            return rc;
        }
    }
    pcp_icp* icp = new pcp_icp();
    icp->ctx = ctx;
    icp->target = target;
    icp->nq = nfin;
    icp->nq_in = nq;
    icp->q = qs;
    int dev_cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, ctx->device) == hipSuccess && prop.multiProcessorCount > 0)
        dev_cus = prop.multiProcessorCount;
    const int64_t want = (icp->nq + pcp::kIcpBlock - 1) / pcp::kIcpBlock;
    icp->nb_fast = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)dev_cus * 8));
    icp->nb_ring = icp->nb_fast;
    const int64_t nwaves = (int64_t)icp->nb_fast * (pcp::kIcpBlock / 64);
    const int64_t nchunks64 = (icp->nq + 63) / 64;
    icp->fb_seg = ((nchunks64 + nwaves - 1) / nwaves) * 64;
    int rc = pcp::dmalloc(ctx, &icp->partials, (size_t)(icp->nb_fast + icp->nb_ring) * pcp::kAcc);
    if (!rc) rc = pcp::dmalloc(ctx, &icp->acc, pcp::kAcc);
    if (!rc) rc = pcp::dmalloc(ctx, &icp->pose_dev, 12);
    if (!rc) rc = pcp::dmalloc(ctx, &icp->win, icp->nq + 1);
    if (!rc) rc = pcp::dmalloc(ctx, &icp->wd2, icp->nq + 1);
    if (!rc) rc = pcp::dmalloc(ctx, &icp->fb, (size_t)nwaves * icp->fb_seg + 1);
    if (!rc) rc = pcp::dmalloc(ctx, &icp->fb_count, (size_t)nwaves);
    if (!rc) rc = pcp::dmalloc(ctx, &icp->fb_off, (size_t)nwaves + 1);
    if (!rc) rc = pcp::dmalloc(ctx, &icp->fbc, icp->nq + 1);
    if (!rc && (hipEventCreate(&icp->ev0) != hipSuccess || hipEventCreate(&icp->ev1) != hipSuccess ||
                hipEventCreate(&icp->ev_mid) != hipSuccess))
        rc = pcp::set_error(ctx, PCP_ERR_HIP, "hipEventCreate failed");
    if (const char* ab = std::getenv("PCP_ICP_ABLATE")) icp->dbg = std::atoi(ab);
    if (rc) {
        pcp_icp_destroy(icp);
        return rc;
    }
    *out = icp;
    return PCP_OK;
}

int pcp_icp_destroy(pcp_icp* icp) {
    if (!icp) return PCP_ERR_ARG;
    (void)hipSetDevice(icp->ctx->device);
    pcp::dfree(icp->ctx, icp->q);
    pcp::dfree(icp->ctx, icp->partials);
    pcp::dfree(icp->ctx, icp->acc);
    pcp::dfree(icp->ctx, icp->win);
    pcp::dfree(icp->ctx, icp->wd2);
    pcp::dfree(icp->ctx, icp->fb);
    pcp::dfree(icp->ctx, icp->fb_count);
    pcp::dfree(icp->ctx, icp->fb_off);
    pcp::dfree(icp->ctx, icp->fbc);
    pcp::dfree(icp->ctx, icp->pose_dev);
    if (icp->ev0) (void)hipEventDestroy(icp->ev0);
    if (icp->ev1) (void)hipEventDestroy(icp->ev1);
    if (icp->ev_mid) (void)hipEventDestroy(icp->ev_mid);
    for (auto& pr : icp->tev) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    delete icp;
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
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    icp->last_fallback = (uint32_t)fbn;
    float ms = 0.f;
    PCP_HIP(ctx, hipEventElapsedTime(&ms, icp->ev0, icp->ev1));
    icp->last_ms = ms;
    icp->last_launches = 1;
    if (icp->dbg) {
        float m1 = 0.f;
        (void)hipEventElapsedTime(&m1, icp->ev0, icp->ev_mid);
        std::fprintf(stderr, "[pcp icp dbg=%d] octant %.4f ms  fallback %.4f ms  n_fallback %u\n", icp->dbg, m1,
                     ms - m1, icp->last_fallback);
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
    const int rc = pcp::icp_launch(icp, T, rmax, icp->acc, nullptr, nullptr);
    icp->dbg = saved;
    PCP_TRY(rc);
    if (icp->nq_in > icp->nq)
        hipLaunchKernelGGL(pcp::k_fill_keys, dim3(pcp::grid_for(icp->nq_in, 256)), dim3(256), 0, ctx->stream, keys_dev,
                           icp->nq_in);
    if (icp->nq > 0)
        hipLaunchKernelGGL(pcp::k_make_keys, dim3(pcp::grid_for(icp->nq, 256)), dim3(256), 0, ctx->stream, icp->q,
                           (const int32_t*)icp->win, (const float*)icp->wd2, icp->nq, (uint32_t)target_offset,
                           keys_dev);
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
    hipLaunchKernelGGL(pcp::k_acc_keys, dim3(nb), dim3(256), 0, ctx->stream, icp->q, icp->nq, keys_dev,
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

int pcp_icp_last_kernel_ms(const pcp_icp* icp, double* ms, int* launches) {
    if (!icp) return PCP_ERR_ARG;
    if (ms) *ms = icp->last_ms;
    if (launches) *launches = icp->last_launches;
    return PCP_OK;
}

}  // extern "C"
