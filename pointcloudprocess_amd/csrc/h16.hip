// C5 (BASELINE.json configs[4]): radius search r + per-point normals over a cloud stored as
// fp16 offsets relative to each point's grid cell, accumulated in fp32
// (KdTreeFLANN::radiusSearch kd_tree.h:863-903 with setSortedResults(false) :739-753, and the
// declared-only calculate_plan_parameter(cloud, radius), calculate_feature.h:15 = F1 over
// each radius neighbourhood, calculate_feature.cpp:119-206).
//
// Layout (HBM): the points in cell order (the fp32 grid build's radix sort), each as 8 bytes
// {fp16 x, y, z offset from its cell origin o + c h, pad} (absolute fp16 would resolve only
// ~6 cm at 100 m; offsets within a cell of h <= 0.4 m resolve <= 1.2e-4 m), its dense cell id
// (4 B) and its caller index (4 B), plus the dense cell-start table.  Cell size h >= r, so a
// query's neighbours lie in its 3x3x3 cells; rows of cells are pruned by the query's distance
// to the cell faces.
//
// Numerics: d = (dc * h + (o_p - o_q)) per axis in fp32 (the fp16 difference is exact in
// fp32), d2 = fmaf chain, neighbour iff d2 < r^2 (strict, as FLANN's RadiusResultSet).  Against
// the exact fp64 search a pair can differ only when | |p - q| - r | < 3e-4 m (the fp16
// quantisation bound); tests exclude that band.  Rows are in index (scan) order, the
// reference's unsorted mode.  Normals: fp32 sums of the neighbours' offsets from the query
// (n, S, S S^T), the covariance formed in fp64, then the F1 eigen core (pca.hpp).
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>

#include "grid.hpp"
#include "pca.hpp"

namespace pcp {
namespace {

constexpr int kB = 256;
#ifndef PCP_H16_BATCH  // candidate records loaded per batch in the row passes
#define PCP_H16_BATCH 4
#endif
#ifndef PCP_H16_TILE_DEFAULT  // 1: the LDS-staged row kernels (k_h16_tile); 0: one lane per point, global loads
#define PCP_H16_TILE_DEFAULT 0
#endif
#ifndef PCP_H16_DIRECT_DEFAULT  // tile fill: rows straight to caller order through an LDS row buffer
#define PCP_H16_DIRECT_DEFAULT 0
#endif
#ifndef PCP_H16_FLUSH16  // fill: hits gathered 16 to a 64-byte store through a per-lane LDS slot buffer (1) or 4 to a 16-byte store from registers (0)
#define PCP_H16_FLUSH16 1
#endif
#ifndef PCP_H16_LATEID  // fill (per-lane kernel): ids gathered per 16-hit flush (1) or loaded with every candidate (0)
#define PCP_H16_LATEID 0
#endif
#ifndef PCP_H16_FUSED_DEFAULT  // 1: the count pass also writes the rows and planes (fixed-stride staging); the fill moves them
#define PCP_H16_FUSED_DEFAULT 1
#endif
#ifndef PCP_H16_FUSED_STRIDE  // fused staging row capacity (a multiple of 16); longer rows spill into a pool
#define PCP_H16_FUSED_STRIDE 96
#endif
#ifndef PCP_H16_NOSTORE  // profiling variant: the fill pass without its row stores
#define PCP_H16_NOSTORE 0
#endif

__device__ __forceinline__ uint32_t pack_h2(float a, float b) {
    const _Float16 ha = (_Float16)a, hb = (_Float16)b;
    return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}
__device__ __forceinline__ float h_lo(uint32_t v) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(v & 0xffffu)); }
__device__ __forceinline__ float h_hi(uint32_t v) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(v >> 16)); }

// sorted fp32 records -> fp16 cell offsets, cell ids, caller indices
__global__ void k_h16_convert(GridDesc g, const float4* pts, int64_t n, uint2* rec, uint32_t* cell, int32_t* mapping) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 p = pts[i];
        // the build's own cell of the point (grid.hip cell_of_point, fp32)
        const int cx = clampi(cell_i<float>(g, p.x, 0), 0, g.n[0] - 1);
        const int cy = clampi(cell_i<float>(g, p.y, 1), 0, g.n[1] - 1);
        const int cz = clampi(cell_i<float>(g, p.z, 2), 0, g.n[2] - 1);
        const float ox = (float)((double)p.x - (g.o[0] + (double)cx * g.h));
        const float oy = (float)((double)p.y - (g.o[1] + (double)cy * g.h));
        const float oz = (float)((double)p.z - (g.o[2] + (double)cz * g.h));
        rec[i] = make_uint2(pack_h2(ox, oy), pack_h2(oz, 0.f));
        cell[i] = (uint32_t)dense_id(g, cx, cy, cz);
        mapping[i] = __float_as_int(p.w);
    }
}

// staging rows are padded to whole stores: 16 ids (64 B) with the LDS slot buffer, else 4 (16 B)
constexpr uint32_t kRowPad = PCP_H16_FLUSH16 ? 16u : 4u;

struct H16Args {
    GridDesc g;
    const uint2* rec;
    const uint32_t* cell;
    const int32_t* mapping;
    int64_t n, n_owned;
    float hf, r2, rcut2;  // cell size, r^2 (the test), (r + margin)^2 (cell pruning)
    // fused count: staging rows `cap` entries apart (0: rows at offsets[s]); a row that reaches cap
    // continues in a spill row of the pool at spill_base (taken from *nspill, recorded in
    // spill_of[caller]); the sorted positions of rows longer than that go to ovf, counted in *novf
    uint32_t cap;
    int32_t* ovf;
    uint32_t* novf;
    int32_t* spill_of;
    uint32_t* nspill;
    uint32_t spill_rows;
    int64_t spill_base;
    double inv_nx, inv_nxy;  // 1 / n[0], 1 / (n[0] n[1]): cell coordinates without integer division
};

// (cx, cy, cz) of dense cell id c: fp64 reciprocal products, each corrected by one step (the
// product of a 32-bit id and a rounded reciprocal is off by < 2^-20, so the floor by at most one)
__device__ __forceinline__ void cell_xyz(const GridDesc& g, const H16Args& a, uint32_t c, int& cx, int& cy, int& cz) {
    const uint32_t nx = (uint32_t)g.n[0], nxy = nx * (uint32_t)g.n[1];
    uint32_t z = (uint32_t)((double)c * a.inv_nxy);
    z -= (uint64_t)z * nxy > c ? 1u : 0u;
    z += (uint64_t)(z + 1u) * nxy <= c ? 1u : 0u;
    const uint32_t rxy = c - z * nxy;
    uint32_t y = (uint32_t)((double)rxy * a.inv_nx);
    y -= y * nx > rxy ? 1u : 0u;
    y += (y + 1u) * nx <= rxy ? 1u : 0u;
    cx = (int)(rxy - y * nx);
    cy = (int)y;
    cz = (int)z;
}

// one lane per sorted point; halo points (caller index >= n_owned) are not queries
// the id each sorted point is reported under (the global id of its caller index, or that index):
// gathered once per point here instead of once per neighbour in the fill pass
__global__ void k_h16_ids(const int32_t* mapping, const int32_t* gid, int64_t n, int32_t* out) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t m = mapping[k];
        out[k] = gid ? gid[m] : m;
    }
}

// Row staging for the fill pass.  Lanes are sorted points, whose caller rows lie far apart: a
// lane-per-row store stream touches 64 lines per instruction and leaves lines half-written
// in L2 (measured: the stores were 13 of the fill pass's 22 ms at 25M points).  So the fill
// writes the rows in sorted order (adjacent lanes, adjacent rows), and one copy pass moves them
// to caller order with full-line writes.
__global__ void k_h16_sorted_counts(const int32_t* mapping, int64_t n, int64_t n_owned, const int64_t* offsets,
                                    int32_t* cnt_s, int32_t* inv) {
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < n; s += (int64_t)gridDim.x * blockDim.x) {
        const int32_t c = mapping[s];
        const bool own = c < n_owned;
        cnt_s[s] = own ? (int32_t)((offsets[c + 1] - offsets[c] + (kRowPad - 1)) & ~(int64_t)(kRowPad - 1)) : 0;
        if (own) inv[c] = (int32_t)s;
    }
}
// one wave per 64 consecutive caller rows.  Their destination is one contiguous span of the
// caller CSR, so the wave walks it flat: lane t copies span elements t, t + 64, ... (full-line
// writes every instruction), each finding its row from the 64 row starts staged in LDS (rows
// are ~n-bar long, so a lane advances about one row per step).  The per-row form (the wave
// copying one row after another) left a dependent load->store per row and lanes idle past
// each row's end.
// Fused form (fstride > 0): the staged rows are fstride entries apart and hold caller indices,
// translated through gid when the fill reports global ids; a row longer than fstride continues
// in its spill row (spill_of), and one longer than two strides, or without a spill row, is
// rewritten whole by k_h16_overflow after this pass; the staged planes (caller order) ride along,
// one per row.
__global__ __launch_bounds__(kB) void k_h16_rows_to_caller(const int32_t* inv, int64_t n_owned, const int64_t* soff,
                                                           const int64_t* offsets, const int32_t* __restrict__ tmp,
                                                           int32_t* __restrict__ out, int64_t fstride = 0,
                                                           const int32_t* __restrict__ gid = nullptr,
                                                           const pcp_plane* __restrict__ pl_src = nullptr,
                                                           pcp_plane* __restrict__ pl_dst = nullptr,
                                                           const int32_t* __restrict__ spill_of = nullptr,
                                                           int64_t spill_base = 0) {
    constexpr int kW = kB / 64;
    __shared__ int64_t s_dst[kW][65];
    __shared__ int64_t s_src[kW][64];
    __shared__ int64_t s_spl[kW][64];  // fused: the spill row's start - fstride, or -1
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t nw = (int64_t)gridDim.x * kW;
    for (int64_t w = blockIdx.x * (int64_t)kW + wid; w * 64 < n_owned; w += nw) {
        const int rows = (int)min((int64_t)64, n_owned - w * 64);
        const int64_t c = w * 64 + lane;
        if (lane < rows) {
            if (pl_dst) pl_dst[c] = pl_src[c];
            s_dst[wid][lane] = offsets[c];
            // an empty row (e.g. a caller point the build dropped as non-finite) has no staged
            // row and no inverse entry: never read inv for it
            const int64_t len = offsets[c + 1] - offsets[c];
            s_src[wid][lane] = len > 0 ? (fstride ? (int64_t)inv[c] * fstride : soff[inv[c]]) : 0;
            // (spill_of is written for every row longer than the stride)
            const int32_t sp = fstride && len > fstride ? spill_of[c] : -1;
            s_spl[wid][lane] = sp >= 0 ? spill_base + (int64_t)sp * fstride - fstride : -1;
        }
        if (lane == 0) s_dst[wid][rows] = offsets[w * 64 + rows];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int64_t d0 = s_dst[wid][0], d1 = s_dst[wid][rows];
        int r = 0;
        int64_t rd = d0, rn = s_dst[wid][1], rs = s_src[wid][0], rp = s_spl[wid][0];
        for (int64_t p = d0 + lane; p < d1; p += 64) {
            while (p >= rn) {  // empty rows are skipped too
                r++;
                rd = rn;
                rn = s_dst[wid][r + 1];
                rs = s_src[wid][r];
                rp = s_spl[wid][r];
            }
            if (fstride == 0) {
                out[p] = tmp[rs + (p - rd)];
            } else {
                const int64_t e = p - rd;
                if (e < fstride || (rp >= 0 && e < 2 * fstride)) {
                    const int32_t v = tmp[(e < fstride ? rs : rp) + e];
                    out[p] = gid ? gid[v] : v;
                }
            }
        }
        // the LDS rows are rewritten by the wave's next group
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// A query's running row: its hit count and, in the fill pass, the hits staged four to a 16-byte
// store into its sorted-order row (rows padded to 4) and the fp32 sums of the hits' offsets
// from the query (the F1 plane's n, S, S S^T), in visiting (= index) order.
template <bool FILL, bool DIRECT = false>
struct H16Acc {
    int64_t o = 0;  // the row's start: in the staging rows, or (DIRECT) in the caller rows
    uint32_t cnt = 0;
    int32_t* slot = nullptr;  // (PCP_H16_FLUSH16 staging fill) this lane's 16 LDS slots, `stride` words apart
    int stride = 0;
    uint32_t cap = 0xffffffffu;  // fused staging: entries from cap on are not stored (the row is redone)
    uint32_t* spill_ctr = nullptr;  // fused staging: the spill pool (rows of the same stride)
    uint32_t spill_rows = 0;
    int64_t spill_base = 0;
    int32_t spill = -1;
    // the row is full: continue in a spill row (the staging offsets then address it directly)
    __device__ __forceinline__ void grow() {
        const uint32_t sp = atomicAdd(spill_ctr, 1u);
        if (sp < spill_rows) {
            spill = (int32_t)sp;
            o = spill_base + (int64_t)sp * cap - cap;
            cap *= 2u;
        }
    }
    const int32_t* late_ids = nullptr;  // set: the slots hold sorted positions, their ids gathered per flush
    int32_t sink = 0, w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    float S0 = 0.f, S1 = 0.f, S2 = 0.f, S00 = 0.f, S01 = 0.f, S02 = 0.f, S11 = 0.f, S12 = 0.f, S22 = 0.f;
    __device__ __forceinline__ void hit(float dx, float dy, float dz, int32_t id, int32_t* __restrict__ out_idx) {
        if (FILL && DIRECT) {
            out_idx[o + cnt] = id;  // caller order: one 4-byte store per hit (the tile kernel's rare path)
            S0 += dx; S1 += dy; S2 += dz;
            S00 = __fmaf_rn(dx, dx, S00); S01 = __fmaf_rn(dx, dy, S01); S02 = __fmaf_rn(dx, dz, S02);
            S11 = __fmaf_rn(dy, dy, S11); S12 = __fmaf_rn(dy, dz, S12); S22 = __fmaf_rn(dz, dz, S22);
        } else if (FILL) {
#if PCP_H16_NOSTORE
            sink ^= id;
#elif PCP_H16_FLUSH16
            // 16 hits per 64-byte store group: the row's lines are written whole by this lane in
            // one burst (16-byte pieces spread over time were written to HBM part by part: the
            // fill's WRITE_SIZE was 2.8x its row bytes)
            if (cnt == cap && spill_ctr && spill < 0) grow();
            slot[(cnt & 15u) * stride] = id;
            if ((cnt & 15u) == 15u && cnt < cap) flush(out_idx, cnt & ~15u, 16u, 16u);
#else
            if (cnt == cap && spill_ctr && spill < 0) grow();
            const uint32_t sl = cnt & 3u;
            w0 = sl == 0 ? id : w0;
            w1 = sl == 1 ? id : w1;
            w2 = sl == 2 ? id : w2;
            w3 = sl == 3 ? id : w3;
            if (sl == 3 && cnt < cap) *(int4*)(out_idx + o + (cnt & ~3u)) = make_int4(w0, w1, w2, w3);
#endif
            S0 += dx; S1 += dy; S2 += dz;
            S00 = __fmaf_rn(dx, dx, S00); S01 = __fmaf_rn(dx, dy, S01); S02 = __fmaf_rn(dx, dz, S02);
            S11 = __fmaf_rn(dy, dy, S11); S12 = __fmaf_rn(dy, dz, S12); S22 = __fmaf_rn(dz, dz, S22);
        }
        cnt++;
    }
    // the first m (a multiple of 4 up to 16) slots to row entries [at, at + m); slots from `valid`
    // on are the row's padding (stale LDS: never dereferenced)
    __device__ __forceinline__ void flush(int32_t* __restrict__ out_idx, uint32_t at, uint32_t m, uint32_t valid) {
        if (late_ids) {  // 16 independent id loads, then the stores
            int32_t v[16];
#pragma unroll
            for (uint32_t q = 0; q < 16u; q++) v[q] = q < valid ? late_ids[slot[q * stride]] : 0;
#pragma unroll
            for (uint32_t q = 0; q < 16u; q += 4u)
                if (q < m) *(int4*)(out_idx + o + at + q) = make_int4(v[q], v[q + 1], v[q + 2], v[q + 3]);
            return;
        }
#pragma unroll
        for (uint32_t q = 0; q < 16u; q += 4u)
            if (q < m)
                *(int4*)(out_idx + o + at + q) = make_int4(slot[q * stride], slot[(q + 1) * stride],
                                                           slot[(q + 2) * stride], slot[(q + 3) * stride]);
    }
    // the fill's sums and count of a hit whose id is stored elsewhere (the tile kernel's LDS rows)
    __device__ __forceinline__ void hit_sums_only(float dx, float dy, float dz) {
        S0 += dx; S1 += dy; S2 += dz;
        S00 = __fmaf_rn(dx, dx, S00); S01 = __fmaf_rn(dx, dy, S01); S02 = __fmaf_rn(dx, dz, S02);
        S11 = __fmaf_rn(dy, dy, S11); S12 = __fmaf_rn(dy, dz, S12); S22 = __fmaf_rn(dz, dz, S22);
        cnt++;
    }
    // count: the row length (caller order) and, with cnt_s, the padded length at the sorted
    // position + the inverse map; fill: the last partial store and the plane
    __device__ __forceinline__ void finish(const H16Args& a, int64_t s, int32_t caller, int cx, int cy, int cz, float qx,
                                           float qy, float qz, int32_t* count, int32_t* __restrict__ out_idx,
                                           pcp_plane* __restrict__ out_nrm, int32_t* __restrict__ cnt_s,
                                           int32_t* __restrict__ inv) {
        const GridDesc& g = a.g;
        if (PCP_H16_NOSTORE && FILL && !DIRECT && sink == 0x7fffffff) out_idx[o] = sink;
        if (!PCP_H16_NOSTORE && PCP_H16_FLUSH16 && FILL && !DIRECT && (cnt & 15u) && cnt < cap)
            flush(out_idx, cnt & ~15u, ((cnt & 15u) + 3u) & ~3u, cnt & 15u);  // the padded tail
        if (!PCP_H16_NOSTORE && !PCP_H16_FLUSH16 && FILL && !DIRECT && (cnt & 3u) && cnt < cap)
            *(int4*)(out_idx + o + (cnt & ~3u)) = make_int4(w0, w1, w2, w3);
        if (!FILL) {
            count[caller] = (int32_t)cnt;
            if (cnt_s) {
                cnt_s[s] = (int32_t)((cnt + (kRowPad - 1)) & ~(kRowPad - 1));  // whole-store staging rows
                inv[caller] = (int32_t)s;
            }
        } else if (!DIRECT && a.cap) {  // fused count: the count, the inverse map, the overflow list
            count[caller] = (int32_t)cnt;
            inv[caller] = (int32_t)s;
            if (cnt > a.cap) {
                a.spill_of[caller] = spill;
                if (cnt > cap) a.ovf[atomicAdd(a.novf, 1u)] = (int32_t)s;
            }
        }
        if (FILL && out_nrm) {
            pcp_plane pl{0.f, 0.f, 0.f, 0.f, 1.f, 0.f};
            if (cnt > 0) {
                const double nn = (double)cnt;
                const double m0 = S0 / nn, m1 = S1 / nn, m2 = S2 / nn;
                const double C[9] = {S00 - nn * m0 * m0, S01 - nn * m0 * m1, S02 - nn * m0 * m2,
                                     S01 - nn * m0 * m1, S11 - nn * m1 * m1, S12 - nn * m1 * m2,
                                     S02 - nn * m0 * m2, S12 - nn * m1 * m2, S22 - nn * m2 * m2};
                // the absolute mean = the query's position + the mean offset
                const double xa = g.o[0] + (double)cx * g.h + (double)qx + m0;
                const double ya = g.o[1] + (double)cy * g.h + (double)qy + m1;
                const double za = g.o[2] + (double)cz * g.h + (double)qz + m2;
                plane_from_cov(C, xa, ya, za, pl);
            }
            out_nrm[caller] = pl;
        }
    }
};

// count pass (FILL = false): count[caller] = the row length; with cnt_s, also the row length
// padded to 4 at the sorted position (0 for points that are not queries) and inv[caller] = s,
// which the fill pass then takes instead of gathering them back from the caller offsets.
// One query (sorted position s, an owned point) with global candidate loads: the per-lane kernel
// and the tile kernel's lanes whose neighbourhood does not fit its LDS.
template <bool FILL, bool DIRECT = false>
__device__ __forceinline__ void h16_point(const H16Args& a, int64_t s, int32_t caller, int32_t* count,
                                          const int64_t* __restrict__ offsets, const int32_t* __restrict__ ids,
                                          int32_t* __restrict__ out_idx, pcp_plane* __restrict__ out_nrm,
                                          int32_t* __restrict__ cnt_s, int32_t* __restrict__ inv, int32_t* slot,
                                          int stride) {
    const GridDesc& g = a.g;
    const uint2* __restrict__ rec = a.rec;
    const uint2 qr = a.rec[s];
    const float qx = h_lo(qr.x), qy = h_hi(qr.x), qz = h_lo(qr.y);
    const uint32_t cid = a.cell[s];
    const int cx = (int)(cid % (uint32_t)g.n[0]);
    const int cy = (int)((cid / (uint32_t)g.n[0]) % (uint32_t)g.n[1]);
    const int cz = (int)(cid / ((uint32_t)g.n[0] * (uint32_t)g.n[1]));
    // distances to the faces of the query's cell (offsets can round a hair outside [0, h])
    const float gxl = fmaxf(qx, 0.f), gxr = fmaxf(a.hf - qx, 0.f);
    const float gyl = fmaxf(qy, 0.f), gyr = fmaxf(a.hf - qy, 0.f);
    const float gzl = fmaxf(qz, 0.f), gzr = fmaxf(a.hf - qz, 0.f);
    H16Acc<FILL, DIRECT> acc;
    // the caller rows, the sorted-order staging rows, or (fused count) the fixed-stride ones
    if (FILL) acc.o = DIRECT ? offsets[caller] : (a.cap ? s * (int64_t)a.cap : offsets[s]);
    if (FILL && !DIRECT && a.cap) {
        acc.cap = a.cap;
        acc.spill_ctr = a.nspill;
        acc.spill_rows = a.spill_rows;
        acc.spill_base = a.spill_base;
    }
    acc.slot = slot;
    acc.stride = stride;
    // PCP_H16_LATEID: the candidates' ids are not loaded with their records; a hit keeps its
    // sorted position and each 16-hit flush gathers the 16 ids at once
    constexpr bool kLateId = PCP_H16_LATEID && PCP_H16_FLUSH16 && FILL && !DIRECT;
    if (kLateId) acc.late_ids = ids;
    for (int dz = -1; dz <= 1; dz++) {
        const int z = cz + dz;
        if (z < 0 || z >= g.n[2]) continue;
        const float gz = dz < 0 ? gzl : (dz > 0 ? gzr : 0.f);
        for (int dy = -1; dy <= 1; dy++) {
            const int y = cy + dy;
            if (y < 0 || y >= g.n[1]) continue;
            const float gy = dy < 0 ? gyl : (dy > 0 ? gyr : 0.f);
            const float gyz = __fmaf_rn(gy, gy, gz * gz);
            if (gyz >= a.rcut2) continue;
            const int xa = (cx > 0 && __fmaf_rn(gxl, gxl, gyz) < a.rcut2) ? cx - 1 : cx;
            const int xb = (cx + 1 < g.n[0] && __fmaf_rn(gxr, gxr, gyz) < a.rcut2) ? cx + 1 : cx;
            const int64_t c0 = dense_id(g, xa, y, z), cq = dense_id(g, cx, y, z);
            const uint32_t k0 = g.cstart[c0], k1 = g.cstart[c0 + (xb - xa + 1)];
            const uint32_t b1 = g.cstart[cq], b2 = g.cstart[cq + 1];  // the query's x column
            const float ey = (float)dy * a.hf - qy, ez = (float)dz * a.hf - qz;
            // batches of NB candidates: the loads are issued together (the hit path's stores
            // would otherwise order every later load behind them)
            constexpr int NB = PCP_H16_BATCH;
            for (uint32_t k = k0; k < k1; k += NB) {
                uint2 pr[NB];
                int32_t idv[NB];
#pragma unroll
                for (int u = 0; u < NB; u++) {
                    const uint32_t kk = min(k + (uint32_t)u, k1 - 1u);
                    pr[u] = rec[kk];
                    if (FILL && !kLateId) idv[u] = ids[kk];
                }
#pragma unroll
                for (int u = 0; u < NB; u++) {
                    const uint32_t kk = k + (uint32_t)u;
                    const float dxc = kk < b1 ? -a.hf : (kk < b2 ? 0.f : a.hf);
                    const float dx = dxc + (h_lo(pr[u].x) - qx);
                    const float dy_ = ey + h_hi(pr[u].x);
                    const float dz_ = ez + h_lo(pr[u].y);
                    const float d2 = __fmaf_rn(dz_, dz_, __fmaf_rn(dy_, dy_, dx * dx));
                    if (kk < k1 && d2 < a.r2) acc.hit(dx, dy_, dz_, FILL ? (kLateId ? (int32_t)kk : idv[u]) : 0, out_idx);
                }
            }

        }
    }
    acc.finish(a, s, caller, cx, cy, cz, qx, qy, qz, count, out_idx, out_nrm, cnt_s, inv);
}

template <bool FILL>
__global__ __launch_bounds__(kB) void k_h16_radius(H16Args a, int32_t* count, const int64_t* __restrict__ offsets,
                                                   const int32_t* __restrict__ ids, int32_t* __restrict__ out_idx,
                                                   pcp_plane* __restrict__ out_nrm, int32_t* __restrict__ cnt_s = nullptr,
                                                   int32_t* __restrict__ inv = nullptr) {
    __shared__ int32_t s_slot[(FILL && PCP_H16_FLUSH16) ? 16 * kB : 1];  // slot-major: conflict-free
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < a.n; s += (int64_t)gridDim.x * blockDim.x) {
        const int32_t caller = a.mapping[s];
        if (caller >= a.n_owned) {
            if (!FILL && cnt_s) cnt_s[s] = 0;
            continue;
        }
        h16_point<FILL>(a, s, caller, count, offsets, ids, out_idx, out_nrm, cnt_s, inv, s_slot + threadIdx.x, kB);
    }
}

// the fused fill's rows longer than two staging strides or without a spill row: each redone in
// full, straight into its caller row (a few in a million at the default stride)
__global__ __launch_bounds__(kB) void k_h16_overflow(H16Args a, const uint32_t* novf, const int32_t* __restrict__ list,
                                                     const int64_t* __restrict__ offsets, const int32_t* __restrict__ ids,
                                                     int32_t* __restrict__ out_idx) {
    const uint32_t m = *novf;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const int64_t s = list[i];
        h16_point<true, true>(a, s, a.mapping[s], (int32_t*)nullptr, offsets, ids, out_idx, (pcp_plane*)nullptr,
                              (int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr, 0);
    }
}

// ---- LDS-staged form (the default): a wave takes 64 consecutive sorted points -- cell order,
// so runs along x-rows of cells -- stages every point of the union of their 3x3x3 cell
// neighbourhoods into LDS once (coalesced row runs of the dense table, fp16 offsets widened to
// fp32 once per staged point, plus the reported id in the fill pass), and each lane then walks
// ITS OWN pruned cells of that list: a per-lane list of (LDS run, cell offset) entries in
// ascending cell order (so rows stay in index order), built after the staged points.  The
// per-candidate arithmetic is the per-lane kernel's (same formula, same visiting order): rows
// and normals are identical to it, while the candidate loads are LDS reads instead of one
// scattered global load per lane and candidate (the address path bound the per-lane form).
// A wave whose union box does not fit splits at its runs of lanes in one (y, z) row of cells;
// a run that still does not fit takes the per-lane global search.
constexpr int kH16Cap = 1024;    // staged points per wave (16 B each: fp32 offsets + id)
constexpr int kH16Rows = 192;    // (y, z) rows of a staged box
struct H16Box {
    int x0, x1, y0, y1, z0, z1, ny, nrow;
    uint32_t total;  // points in the box (0xffffffff: too many rows)
};
__device__ __forceinline__ int h16_wmin(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int h16_wmax(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ void h16_wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// the union of the 3x3x3 neighbourhoods of the lanes with `in` set; with `write`, each (y, z)
// row's run of the dense table (global start, LDS start) into s_rs / s_rb
__device__ __forceinline__ H16Box h16_box(const GridDesc& g, int cx, int cy, int cz, bool in, int lane,
                                          uint32_t* s_rs, uint32_t* s_rb, bool write) {
    H16Box b;
    b.x0 = max(h16_wmin(in ? cx : INT_MAX) - 1, 0), b.x1 = min(h16_wmax(in ? cx : INT_MIN) + 1, g.n[0] - 1);
    b.y0 = max(h16_wmin(in ? cy : INT_MAX) - 1, 0), b.y1 = min(h16_wmax(in ? cy : INT_MIN) + 1, g.n[1] - 1);
    b.z0 = max(h16_wmin(in ? cz : INT_MAX) - 1, 0), b.z1 = min(h16_wmax(in ? cz : INT_MIN) + 1, g.n[2] - 1);
    b.ny = b.y1 - b.y0 + 1;
    b.nrow = b.ny * (b.z1 - b.z0 + 1);
    b.total = 0xffffffffu;
    if (b.nrow > kH16Rows || b.x1 < b.x0) return b;
    uint32_t carry = 0;
    for (int r0 = 0; r0 < b.nrow; r0 += 64) {
        const int r = r0 + lane;
        uint32_t st = 0, cnt = 0;
        if (r < b.nrow) {
            const int y = b.y0 + r % b.ny, z = b.z0 + r / b.ny;
            st = g.cstart[dense_id(g, b.x0, y, z)];
            cnt = g.cstart[dense_id(g, b.x1, y, z) + 1] - st;
        }
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

template <bool FILL, bool DIRECT = false>
__global__ __launch_bounds__(64) void k_h16_tile(H16Args a, int32_t* count, const int64_t* __restrict__ offsets,
                                                 const int32_t* __restrict__ ids, int32_t* __restrict__ out_idx,
                                                 pcp_plane* __restrict__ out_nrm, int32_t* __restrict__ cnt_s,
                                                 int32_t* __restrict__ inv, unsigned long long* stats) {
    // staged points (<= kH16Cap), then the lanes' cell lists, then (DIRECT) the row buffer
    constexpr int kCap = DIRECT ? 3 * kH16Cap / 2 : kH16Cap;
    __shared__ float4 s_p[kCap];
    __shared__ __attribute__((aligned(16))) uint32_t s_rs[kH16Rows];  // (DIRECT: 64 int64 caller starts)
    __shared__ uint32_t s_rb[kH16Rows + 1];
    __shared__ int32_t s_slot[(FILL && PCP_H16_FLUSH16) ? 16 * 64 : 1];
    const GridDesc& g = a.g;
    const int lane = threadIdx.x;
    for (int64_t c = blockIdx.x; c * 64 < a.n; c += gridDim.x) {
        const int64_t s = c * 64 + lane;
        const bool valid = s < a.n;
        const int32_t caller = valid ? a.mapping[s] : INT_MAX;
        const bool act = valid && caller < a.n_owned;
        if (!FILL && valid && !act && cnt_s) cnt_s[s] = 0;
        uint2 qr = make_uint2(0u, 0u);
        uint32_t cid = 0;
        if (act) {
            qr = a.rec[s];
            cid = a.cell[s];
        }
        const float qx = h_lo(qr.x), qy = h_hi(qr.x), qz = h_lo(qr.y);
        const int cx = (int)(cid % (uint32_t)g.n[0]);
        const int cy = (int)((cid / (uint32_t)g.n[0]) % (uint32_t)g.n[1]);
        const int cz = (int)(cid / ((uint32_t)g.n[0] * (uint32_t)g.n[1]));
        // groups: the whole wave when its box fits, else its runs of lanes in one (y, z) row
        int grp = 0, G = 1;
        bool over = false;  // this lane's group does not fit: the global search
        if (h16_box(g, cx, cy, cz, act, lane, s_rs, s_rb, false).total > (uint32_t)kH16Cap) {
            const uint32_t row = cid / (uint32_t)g.n[0];  // (y, z) row id
            const uint32_t prev = (uint32_t)__shfl_up((int)row, 1, 64);
            const uint64_t below = lane == 63 ? ~0ull : ((2ull << lane) - 1);
            const uint64_t heads = __ballot(lane == 0 || row != prev);
            grp = __popcll(heads & below) - 1;
            G = __popcll(heads);
            for (int gi = 0; gi < G; gi++) {
                const bool in = act && grp == gi;
                if (!__ballot(in)) continue;
                if (h16_box(g, cx, cy, cz, in, lane, s_rs, s_rb, false).total > (uint32_t)kH16Cap)
                    over = over || grp == gi;
            }
        }
        if (stats && lane == 0) {
            atomicAdd(stats + 0, (unsigned long long)G);
            atomicAdd(stats + 1, (unsigned long long)__popcll(__ballot(over && act)));
        }
        for (int gi = 0; gi < G; gi++) {
            const bool mine = act && grp == gi && !over;
            if (!__ballot(mine)) continue;
            h16_wave_fence();  // the previous group's readers are done with the LDS
            const H16Box b = h16_box(g, cx, cy, cz, mine, lane, s_rs, s_rb, true);
            const uint32_t total = b.total;
            h16_wave_fence();
            const int nrow = b.nrow;
            for (uint32_t e = lane; e < total; e += 64) {
                int r = 0;
#pragma unroll
                for (int stp = 128; stp > 0; stp >>= 1)
                    r = (r + stp < nrow && s_rb[r + stp] <= e) ? r + stp : r;
                const uint32_t pos = s_rs[r] + (e - s_rb[r]);
                const uint2 pr = a.rec[pos];
                s_p[e] = make_float4(h_lo(pr.x), h_hi(pr.x), h_lo(pr.y), FILL ? __int_as_float(ids[pos]) : 0.f);
            }
            // the lane's cells: rows pruned by the query's distance to the cell faces (as the
            // per-lane form), each as (LDS run start, end, cell offset + 1 per axis) in ascending
            // cell order; pass 1 counts them, pass 2 (from the caches) writes them
            const float gxl = fmaxf(qx, 0.f), gxr = fmaxf(a.hf - qx, 0.f);
            const float gyl = fmaxf(qy, 0.f), gyr = fmaxf(a.hf - qy, 0.f);
            const float gzl = fmaxf(qz, 0.f), gzr = fmaxf(a.hf - qz, 0.f);
            uint32_t* const s_w = reinterpret_cast<uint32_t*>(s_p) + 4 * total;
            auto cells = [&](bool write, int j) {
                int m = 0;
                for (int dz = -1; dz <= 1; dz++) {
                    const int z = cz + dz;
                    const float gz = dz < 0 ? gzl : (dz > 0 ? gzr : 0.f);
                    for (int dy = -1; dy <= 1; dy++) {
                        const int y = cy + dy;
                        const float gy = dy < 0 ? gyl : (dy > 0 ? gyr : 0.f);
                        const float gyz = __fmaf_rn(gy, gy, gz * gz);
                        if (!mine || z < 0 || z >= g.n[2] || y < 0 || y >= g.n[1] || gyz >= a.rcut2) continue;
                        const bool xl = cx > 0 && __fmaf_rn(gxl, gxl, gyz) < a.rcut2;
                        const bool xr = cx + 1 < g.n[0] && __fmaf_rn(gxr, gxr, gyz) < a.rcut2;
                        const int64_t cq = dense_id(g, cx, y, z);
                        const uint32_t b1 = g.cstart[cq], b2 = g.cstart[cq + 1];
                        const uint32_t b0 = xl ? g.cstart[cq - 1] : b1, b3 = xr ? g.cstart[cq + 2] : b2;
                        const int r = (y - b.y0) + (z - b.z0) * b.ny;
                        const uint32_t base = s_rb[r] - s_rs[r];  // LDS index = global position + base
                        const uint32_t code = (uint32_t)(dy + 1) << 24 | (uint32_t)(dz + 1) << 26;
                        if (b1 > b0) { if (write) s_w[j + m] = (b0 + base) | (b1 + base) << 11 | code; m++; }
                        if (b2 > b1) { if (write) s_w[j + m] = (b1 + base) | (b2 + base) << 11 | code | 1u << 22; m++; }
                        if (b3 > b2) { if (write) s_w[j + m] = (b2 + base) | (b3 + base) << 11 | code | 2u << 22; m++; }
                    }
                }
                return m;
            };
            const int nc = cells(false, 0);
            int excl = nc;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t2 = __shfl_up(excl, o, 64);
                if (lane >= o) excl += t2;
            }
            const int tot = __shfl(excl, 63, 64);
            excl -= nc;
            if (4 * total + (uint32_t)tot > 4u * kCap) {  // no room for the cell lists
                if (mine)
                    h16_point<FILL, DIRECT>(a, s, caller, count, offsets, ids, out_idx, out_nrm, cnt_s, inv,
                                            s_slot + lane, 64);
                if (stats && lane == 0) atomicAdd(stats + 2, 1ull);
                continue;
            }
            cells(true, excl);
            // DIRECT fill: the rows go straight to their caller positions.  Each lane's hits are
            // appended (as 16-bit staged-list indices) to its run of an LDS row buffer after the
            // cell lists -- the run's length is its count, known from the count pass -- and the
            // wave then writes the 64 rows flat, lane t taking elements t, t + 64, ... (consecutive
            // lanes, consecutive addresses of one row: full-line writes), instead of staging rows
            // in sorted order and copying them to caller order in another pass.  A group whose rows
            // do not fit stores each hit at its caller position from the lane.
            int64_t dst = 0;
            uint32_t rcnt = 0, rb = 0, rtot = 0;
            bool rbuf = false;
            uint16_t* const s_h = reinterpret_cast<uint16_t*>(s_w + tot);
            if (DIRECT) {
                if (mine) {
                    dst = offsets[caller];
                    rcnt = (uint32_t)(offsets[caller + 1] - dst);
                }
                uint32_t inc = rcnt;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t t2 = __shfl_up(inc, o, 64);
                    if (lane >= o) inc += t2;
                }
                rtot = __shfl(inc, 63, 64);
                rb = inc - rcnt;
                rbuf = 4 * total + (uint32_t)tot + (rtot + 1) / 2 <= 4u * kCap;
            }
            h16_wave_fence();
            H16Acc<FILL, DIRECT> acc;
            if (FILL && mine) acc.o = DIRECT ? dst : offsets[s];
            acc.slot = s_slot + lane;
            acc.stride = 64;
            uint32_t rp = (uint32_t)excl, rend = (uint32_t)(excl + nc);
            uint32_t e = 0, ee = 0;
            float dxc = 0.f, ey = 0.f, ez = 0.f;
            for (;;) {
                if (e >= ee && rp < rend) {
                    const uint32_t w = s_w[rp++];
                    e = w & 0x7ffu;
                    ee = (w >> 11) & 0x7ffu;
                    dxc = (float)((int)((w >> 22) & 3u) - 1) * a.hf;
                    ey = (float)((int)((w >> 24) & 3u) - 1) * a.hf - qy;
                    ez = (float)((int)((w >> 26) & 3u) - 1) * a.hf - qz;
                }
                const bool on = e < ee;
                if (__ballot(on) == 0) break;
                const float4 p = s_p[on ? e : 0u];
                const float dx = dxc + (p.x - qx);
                const float dy_ = ey + p.y;
                const float dz_ = ez + p.z;
                const float d2 = __fmaf_rn(dz_, dz_, __fmaf_rn(dy_, dy_, dx * dx));
                if (on && d2 < a.r2) {
                    if (DIRECT && rbuf) {  // (the row length is the count pass's: never past it)
                        if (acc.cnt < rcnt) s_h[rb + acc.cnt] = (uint16_t)e;
                        acc.hit_sums_only(dx, dy_, dz_);
                    } else if (!DIRECT || acc.cnt < rcnt) {
                        acc.hit(dx, dy_, dz_, __float_as_int(p.w), out_idx);
                    }
                }
                e += on ? 1u : 0u;
            }
            if (DIRECT && rbuf) {
                // the wave writes its rows: per-lane (LDS start, caller start) staged, then flat
                uint32_t* const s_rb0 = s_rb;  // reuse: the box's row table is no longer read
                int64_t* const s_dst = reinterpret_cast<int64_t*>(s_rs);
                h16_wave_fence();
                s_rb0[lane] = rb;
                if (lane == 0) s_rb0[64] = rtot;
                s_dst[lane] = dst;
                h16_wave_fence();
                int r = 0;
                for (uint32_t t = lane; t < rtot; t += 64) {
                    while (s_rb0[r + 1] <= t) r++;
                    out_idx[s_dst[r] + (t - s_rb0[r])] = __float_as_int(s_p[s_h[t]].w);
                }
            }
            if (mine) acc.finish(a, s, caller, cx, cy, cz, qx, qy, qz, count, out_idx, out_nrm, cnt_s, inv);
        }
        if (over && act)
            h16_point<FILL, DIRECT>(a, s, caller, count, offsets, ids, out_idx, out_nrm, cnt_s, inv, s_slot + lane, 64);
    }
}

__global__ void k_h16_plane_default(pcp_plane* out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = pcp_plane{0.f, 0.f, 0.f, 0.f, 1.f, 0.f};  // points dropped as non-finite
}

// ---- cell-wave form (PCP_H16_CW, the default): one wave per query cell, lanes = candidates.
// The wave loads its cell's 3x3x3 neighbourhood once -- the 9 (dy, dz) rows of cells [cx - 1,
// cx + 1], concatenated in the per-lane kernel's visiting order (dz, dy, then ascending sorted
// position) -- one candidate per lane and step, into registers (fp16 offsets widened to fp32, the
// x-cell offset dxc and the row's dy h, dz h).  Each query of the cell is then a wave-uniform
// value: its test d2 < r^2 runs on every lane against that lane's candidates (the per-lane
// kernel's formula, op for op, so the hit set is identical; the per-lane kernel's row/cell
// pruning only skips cells that cannot hold a hit), the hits are compacted by ballot + mbcnt
// in candidate order, which IS the row's order, and stored as one contiguous run per step
// straight into the caller's CSR row.  No per-lane load chains, no divergent stores, no
// staging rows and no caller-order copy.  The F1 sums (n, S, S S^T of the offsets from the
// query) are accumulated per lane for 4 queries at once and reduce-scattered across the wave
// (36 values, ~25 VALU ops per query); they go out in sorted order and k_h16_cw_planes forms
// the planes (the fp64 eigen core stays out of this kernel's registers).
#ifndef PCP_H16_CW_DEFAULT
#define PCP_H16_CW_DEFAULT 1
#endif
#ifndef PCP_H16_CW_MINB  // blocks per CU the cell-wave kernels are register-budgeted for
#define PCP_H16_CW_MINB 4
#endif
constexpr int kCwWaves = kB / 64;
constexpr int kCwSteps = 6;  // candidate steps held in registers (6 x 64); larger neighbourhoods loop
constexpr int kCwQ = 4;      // queries per accumulator batch (4 x 9 sums reduce-scattered together)
typedef float f2 __attribute__((ext_vector_type(2)));

struct alignas(16) CwSums {  // one query's F1 sums (sorted order) for k_h16_cw_planes (3 x 16-byte words)
    float S0, S1, S2, S00, S01, S02, S11, S12, S22;
    int32_t n, pad0, pad1;
};

template <int CTRL>
__device__ __forceinline__ float cw_dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ float cw_bfly(float a, float b, bool s) {
    const float t = s ? b : a, u = s ? a : b;
    return t + cw_dpp<CTRL>(u);
}
__device__ __forceinline__ float cw_swap_add32(float a, float b) {  // lanes < 32: a_lo + a_hi; >= 32: b_lo + b_hi
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float cw_swap_add16(float a, float b) {  // even rows: a's row pair; odd rows: b's
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// Reduce-scatter of v[36] (value qi * 9 + k) over the wave: afterwards lane l holds the wave total
// of value 18 b5 + 9 b4 + (b0 + 2 b1 + 3 b2 + 5 b3) when cw_owner(l) (each value exactly once).
__device__ __forceinline__ float cw_reduce36(const float (&v)[36], int lane) {
    float w18[18];
#pragma unroll
    for (int i = 0; i < 18; i++) w18[i] = cw_swap_add32(v[i], v[i + 18]);
    float w9[9];
#pragma unroll
    for (int i = 0; i < 9; i++) w9[i] = cw_swap_add16(w18[i], w18[i + 9]);
    const bool s3 = lane & 8, s2 = lane & 4, s1 = lane & 2, s0 = lane & 1;
    float x5[5];
#pragma unroll
    for (int i = 0; i < 5; i++) x5[i] = cw_bfly<0x140>(w9[i], i + 5 < 9 ? w9[i + 5] : 0.f, s3);  // row mirror
    float x3[3];
#pragma unroll
    for (int i = 0; i < 3; i++) x3[i] = cw_bfly<0x141>(x5[i], i + 3 < 5 ? x5[i + 3] : 0.f, s2);  // half-row mirror
    const float y0 = cw_bfly<0x4E>(x3[0], x3[2], s1), y1 = cw_bfly<0x4E>(x3[1], 0.f, s1);  // quad [2,3,0,1]
    return cw_bfly<0xB1>(y0, y1, s0);                                                     // quad [1,0,3,2]
}
__device__ __forceinline__ int cw_slot9(int lane) {
    return (lane & 1) + 2 * ((lane >> 1) & 1) + 3 * ((lane >> 2) & 1) + 5 * ((lane >> 3) & 1);
}
__device__ __forceinline__ bool cw_owner(int lane) {
    const int i1 = (lane & 1) + 2 * ((lane >> 1) & 1), i2 = i1 + 3 * ((lane >> 2) & 1);
    return i1 < 3 && i2 < 5 && i2 + 5 * ((lane >> 3) & 1) < 9;
}

// FILL = false: count[caller] = the row length.  FILL = true: the row's ids (ids[sorted position])
// at out_idx[offsets[caller] ...] and the query's sums at sums[sorted position].
template <bool FILL>
__global__ __launch_bounds__(kB, PCP_H16_CW_MINB) void k_h16_cw(H16Args a, int32_t* __restrict__ count, const int64_t* __restrict__ offsets,
                                               const int32_t* __restrict__ ids, int32_t* __restrict__ out_idx,
                                               CwSums* __restrict__ sums) {
    __shared__ uint4 s_row[kCwWaves][9];  // per neighbour row: kk = j + off, the query column [b1, b2)
    __shared__ float2 s_rdz[kCwWaves][9];  // per neighbour row: its dy h, dz h
    __shared__ float s_sum[kCwWaves][64 * 9];
    const GridDesc& g = a.g;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t nwaves = (int64_t)gridDim.x * kCwWaves;
    const float hf = a.hf, r2 = a.r2;
    for (int64_t w = blockIdx.x * (int64_t)kCwWaves + wid; w * 64 < a.n; w += nwaves) {
        // the cells whose first point lies in this wave's 64 sorted positions
        const int64_t p = w * 64 + lane;
        const uint32_t cp = p < a.n ? a.cell[p] : 0xffffffffu;
        const uint32_t cq = (p < a.n && p > 0) ? a.cell[p - 1] : 0xfffffffeu;
        uint64_t heads = __ballot(p < a.n && (p == 0 || cp != cq));
        while (heads) {
            const int hl = __builtin_ctzll(heads);
            heads &= heads - 1;
            const uint32_t cid = (uint32_t)__builtin_amdgcn_readlane((int)cp, hl);
            const int64_t cs = w * 64 + hl;
            const int64_t ce = (int64_t)g.cstart[(int64_t)cid + 1];
            int cx, cy, cz;
            cell_xyz(g, a, cid, cx, cy, cz);
            // the 9 rows (lane r: dz = r / 3 - 1, dy = r % 3 - 1), cells [cx - 1, cx + 1] clipped
            uint32_t len = 0;
            if (lane < 9) {
                const int y = cy + lane % 3 - 1, z = cz + lane / 3 - 1;
                uint32_t k0 = 0, b1 = 0, b2 = 0;
                if (y >= 0 && y < g.n[1] && z >= 0 && z < g.n[2]) {
                    const int xa = max(cx - 1, 0), xb = min(cx + 1, g.n[0] - 1);
                    const int64_t c0 = dense_id(g, xa, y, z), cc = dense_id(g, cx, y, z);
                    k0 = g.cstart[c0];
                    len = g.cstart[c0 + (xb - xa + 1)] - k0;
                    b1 = g.cstart[cc];
                    b2 = g.cstart[cc + 1];
                }
                uint32_t pre = 0;  // exclusive prefix of the row lengths
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t lk = (uint32_t)__shfl((int)len, k, 64);
                    pre += k < lane ? lk : 0u;
                }
                s_row[wid][lane] = make_uint4(k0 - pre, b1, b2, pre);
                s_rdz[wid][lane] = make_float2((float)(lane % 3 - 1) * hf, (float)(lane / 3 - 1) * hf);
            }
            uint32_t P[9];  // wave-uniform row starts in the concatenated list, and M
            {
                uint32_t acc = 0;
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    P[k] = acc;
                    acc += (uint32_t)__builtin_amdgcn_readlane((int)len, k);
                }
                len = acc;  // M
            }
            const uint32_t M = len;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // candidates of block `blk` (kCwSteps x 64 from list entry blk) into registers
            float cox[kCwSteps], coy[kCwSteps], coz[kCwSteps], cdx[kCwSteps], cdy[kCwSteps], cdz[kCwSteps];
            int32_t cid_[kCwSteps];
            auto load_block = [&](uint32_t blk) {
#pragma unroll
                for (int s = 0; s < kCwSteps; s++) {
                    if (blk + 64u * s >= M) break;  // (uniform) the block's steps past the list are never read
                    const uint32_t j = blk + 64u * s + (uint32_t)lane;
                    const bool ok = j < M;
                    // the row of list entry j: the largest r with P[r] <= j (binary search over the
                    // uniform row starts; P[8] then settles the last row)
                    int r = j >= P[4] ? 4 : 0;
                    r += j >= (r ? P[6] : P[2]) ? 2 : 0;
                    r += j >= (r == 0 ? P[1] : r == 2 ? P[3] : r == 4 ? P[5] : P[7]) ? 1 : 0;
                    r += (r == 7 && j >= P[8]) ? 1 : 0;
                    const uint4 row = s_row[wid][r];
                    const uint32_t kk = ok ? j + row.x : 0u;
                    const uint2 pr = a.rec[kk];
                    cid_[s] = FILL && ok ? ids[kk] : 0;
                    cox[s] = h_lo(pr.x);
                    coy[s] = h_hi(pr.x);
                    coz[s] = h_lo(pr.y);
                    // past the list: a finite far offset (d2 ~ 1e38 >= r^2, never a hit)
                    cdx[s] = ok ? (kk < row.y ? -hf : (kk < row.z ? 0.f : hf)) : 1e19f;
                    const float2 rdz = s_rdz[wid][r];
                    cdy[s] = rdz.x;
                    cdz[s] = rdz.y;
                }
            };
            // the per-lane kernel's expression (h16_point), op for op: same d2, same hit set
            auto test = [&](int s, float x, float y, float z, float& dx, float& dy, float& dz) {
                dx = cdx[s] + (cox[s] - x);
                dy = (cdy[s] - y) + coy[s];
                dz = (cdz[s] - z) + coz[s];
                return __fmaf_rn(dz, dz, __fmaf_rn(dy, dy, dx * dx)) < r2;
            };
            const uint32_t nblk = (M + kCwSteps * 64 - 1) / (kCwSteps * 64);
            if (nblk == 1) load_block(0u);
            // the cell's queries, 64 at a time
            for (int64_t qs = cs; qs < ce; qs += 64) {
                const int nseg = (int)min((int64_t)64, ce - qs);
                float qx = 0.f, qy = 0.f, qz = 0.f;
                int32_t caller = 0x7fffffff;
                int64_t base = 0;
                if (lane < nseg) {
                    const uint2 qr = a.rec[qs + lane];
                    qx = h_lo(qr.x), qy = h_hi(qr.x), qz = h_lo(qr.y);
                    caller = a.mapping[qs + lane];
                    if (FILL && caller < a.n_owned) base = offsets[caller];
                }
                int32_t cntv = 0;  // lane i: the row length of query i of the segment
                const uint64_t ownm = __ballot(lane < nseg && caller < a.n_owned);  // the segment's queries
                if constexpr (!FILL) {
                    // count: two queries at a time (the tests as packed fp32: v_pk_add/mul/fma_f32
                    // round each half exactly as the scalar ops), one ballot per query and step
                    for (int qi = 0; qi < nseg; qi += 2) {
                        const int q1 = min(qi + 1, 63);
                        if (!((ownm >> qi) & 3ull)) continue;
                        const f2 sx = {__int_as_float(__builtin_amdgcn_readlane(__float_as_int(qx), qi)),
                                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qx), q1))};
                        const f2 sy = {__int_as_float(__builtin_amdgcn_readlane(__float_as_int(qy), qi)),
                                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qy), q1))};
                        const f2 sz = {__int_as_float(__builtin_amdgcn_readlane(__float_as_int(qz), qi)),
                                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qz), q1))};
                        uint32_t c0 = 0, c1 = 0;
                        for (uint32_t b = 0; b < nblk; b++) {
                            if (nblk > 1) load_block(b * (uint32_t)(kCwSteps * 64));
                            const uint32_t mb = min(M - b * (uint32_t)(kCwSteps * 64), (uint32_t)(kCwSteps * 64));
#pragma unroll
                            for (int s = 0; s < kCwSteps; s++) {
                                if (64u * s >= mb) break;
                                const f2 dx = (f2)cdx[s] + ((f2)cox[s] - sx);
                                const f2 dy = ((f2)cdy[s] - sy) + (f2)coy[s];
                                const f2 dz = ((f2)cdz[s] - sz) + (f2)coz[s];
                                const f2 d2 = __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
                                c0 += (uint32_t)__popcll(__ballot(d2[0] < r2));
                                c1 += (uint32_t)__popcll(__ballot(d2[1] < r2));
                            }
                        }
                        cntv = lane == qi ? (int32_t)c0 : cntv;
                        cntv = lane == qi + 1 ? (int32_t)c1 : cntv;
                    }
                } else {
                    for (int qb = 0; qb < nseg; qb += kCwQ) {
                        float acc[kCwQ * 9];
#pragma unroll
                        for (int v = 0; v < kCwQ * 9; v++) acc[v] = 0.f;
                        float sqx[kCwQ], sqy[kCwQ], sqz[kCwQ];
                        int64_t sbase[kCwQ];
                        bool act[kCwQ];
                        uint32_t qcnt[kCwQ];
#pragma unroll
                        for (int qi = 0; qi < kCwQ; qi++) {
                            const int q = min(qb + qi, 63);
                            sqx[qi] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qx), q));
                            sqy[qi] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qy), q));
                            sqz[qi] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qz), q));
                            act[qi] = (ownm >> q) & 1ull && qb + qi < nseg;
                            const uint64_t bq = (uint64_t)base;
                            sbase[qi] = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bq, q)) |
                                                  ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bq >> 32), q) << 32));
                            qcnt[qi] = 0u;
                        }
                        for (uint32_t b = 0; b < nblk; b++) {
                            if (nblk > 1) load_block(b * (uint32_t)(kCwSteps * 64));
                            const uint32_t mb = min(M - b * (uint32_t)(kCwSteps * 64), (uint32_t)(kCwSteps * 64));
#pragma unroll
                            for (int s = 0; s < kCwSteps; s++) {
                                if (64u * s >= mb) break;
#pragma unroll
                                for (int qi = 0; qi < kCwQ; qi++) {
                                    if (!act[qi]) continue;
                                    float dx, dy, dz;
                                    const bool hit = test(s, sqx[qi], sqy[qi], sqz[qi], dx, dy, dz);
                                    const uint64_t m = __ballot(hit);
                                    if (hit) {  // the row entry (ballot order = candidate order) and the sums
                                        const uint32_t pos = qcnt[qi] + __builtin_amdgcn_mbcnt_hi(
                                                                            (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                                        out_idx[sbase[qi] + pos] = cid_[s];
                                        float* A = acc + qi * 9;
                                        A[0] += dx;
                                        A[1] += dy;
                                        A[2] += dz;
                                        A[3] = __fmaf_rn(dx, dx, A[3]);
                                        A[4] = __fmaf_rn(dx, dy, A[4]);
                                        A[5] = __fmaf_rn(dx, dz, A[5]);
                                        A[6] = __fmaf_rn(dy, dy, A[6]);
                                        A[7] = __fmaf_rn(dy, dz, A[7]);
                                        A[8] = __fmaf_rn(dz, dz, A[8]);
                                    }
                                    qcnt[qi] += (uint32_t)__popcll(m);
                                }
                            }
                        }
#pragma unroll
                        for (int qi = 0; qi < kCwQ; qi++) cntv = lane == qb + qi ? (int32_t)qcnt[qi] : cntv;
                        const float tot = cw_reduce36(acc, lane);
                        const int qi = 2 * ((lane >> 5) & 1) + ((lane >> 4) & 1);
                        if (cw_owner(lane) && qb + qi < 64) s_sum[wid][(qb + qi) * 9 + cw_slot9(lane)] = tot;
                    }
                }
                if (!FILL) {
                    if (lane < nseg && caller < a.n_owned) count[caller] = cntv;
                } else {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    if (sums && lane < nseg && caller < a.n_owned) {
                        const float* S = &s_sum[wid][lane * 9];
                        sums[qs + lane] = CwSums{S[0], S[1], S[2], S[3], S[4], S[5], S[6], S[7], S[8], cntv, 0, 0};
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
            }
            // s_row is rewritten by the next cell
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
}

// F1's plane from the fp64 covariance by the closed-form symmetric 3x3 eigen decomposition
// (trigonometric eigenvalues, the smallest one's eigenvector as the largest cross product of two
// rows of C - l3 I): a fixed ~250 fp64 ops against the cyclic Jacobi's 4-6 data-dependent sweeps
// (the planes pass was 12.8 ms of the 200M-point step with it).  Rows whose two smallest
// eigenvalues nearly coincide (the normal is ill-conditioned in any method; fewer than 3
// neighbours, lines) keep the Jacobi core, as does everything outside C5, whose results are
// checked to tolerance (fp32 sums of fp16 offsets) rather than bit for bit.
// Returns false (out untouched) for the rows that keep the Jacobi core (k_h16_cw_planes_fb: the
// rare rows must not set the register budget of the streaming pass).
__device__ inline bool h16_plane(const double C[9], double xa, double ya, double za, pcp_plane& out) {
    const double a00 = C[0], a01 = C[1], a02 = C[2], a11 = C[4], a12 = C[5], a22 = C[8];
    const double m = (a00 + a11 + a22) / 3.0;
    const double b00 = a00 - m, b11 = a11 - m, b22 = a22 - m;
    const double p1 = a01 * a01 + a02 * a02 + a12 * a12;
    const double q = (b00 * b00 + b11 * b11 + b22 * b22 + 2.0 * p1) / 6.0;
    bool ok = q > 0.0;
    double l1 = m, l2 = m, l3 = m, n0 = 1.0, n1 = 0.0, n2 = 0.0;
    if (ok) {
        const double p = sqrt(q);
        const double det = b00 * (b11 * b22 - a12 * a12) - a01 * (a01 * b22 - a12 * a02) + a02 * (a01 * a12 - b11 * a02);
        const double r = fmin(fmax(det / (2.0 * p * p * p), -1.0), 1.0);
        const double phi = acos(r) / 3.0;
        l1 = m + 2.0 * p * cos(phi);
        l3 = m + 2.0 * p * cos(phi + 2.0943951023931954923);  // + 2 pi / 3
        l2 = 3.0 * m - l1 - l3;
        ok = (l2 - l3) > 1e-4 * (l1 - l3);
        if (ok) {
            const double r00 = a00 - l3, r11 = a11 - l3, r22 = a22 - l3;
            // cross products of the rows (r00, a01, a02), (a01, r11, a12), (a02, a12, r22)
            const double x0 = a01 * a12 - a02 * r11, y0 = a02 * a01 - r00 * a12, z0 = r00 * r11 - a01 * a01;
            const double x1 = a01 * r22 - a02 * a12, y1 = a02 * a02 - r00 * r22, z1 = r00 * a12 - a01 * a02;
            const double x2 = r11 * r22 - a12 * a12, y2 = a12 * a02 - a01 * r22, z2 = a01 * a12 - r11 * a02;
            const double s0 = x0 * x0 + y0 * y0 + z0 * z0, s1 = x1 * x1 + y1 * y1 + z1 * z1,
                         s2 = x2 * x2 + y2 * y2 + z2 * z2;
            double cx = x0, cy = y0, cz = z0, sb = s0;
            if (s1 > sb) cx = x1, cy = y1, cz = z1, sb = s1;
            if (s2 > sb) cx = x2, cy = y2, cz = z2, sb = s2;
            ok = sb > 0.0;
            const double inv = ok ? 1.0 / sqrt(sb) : 0.0;
            n0 = cx * inv, n1 = cy * inv, n2 = cz * inv;
        }
    }
    if (!ok) return false;
    // the F1 core's sign, distance and ratios (pca.hpp plane_from_cov)
    double n[3] = {n0, n1, n2};
    int big = 0;
    for (int k = 1; k < 3; k++)
        if (fabs(n[k]) > fabs(n[big])) big = k;
    if (n[big] < 0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
    out.normal_x = (float)n[0];
    out.normal_y = (float)n[1];
    out.normal_z = (float)n[2];
    const double dist = -((double)out.normal_x * xa + (double)out.normal_y * ya + (double)out.normal_z * za);
    out.distance = (float)dist;
    out.min_value = (float)l3;
    out.curvature = (float)(l3 / (l1 + l2 + l3));
    return true;
}

// the fp64 covariance and absolute mean of sorted point s from its F1 sums (H16Acc::finish)
__device__ inline void cw_cov(const H16Args& a, int64_t s, const CwSums& q, double C[9], double& xa, double& ya,
                              double& za) {
    const GridDesc& g = a.g;
    const uint2 qr = a.rec[s];
    const float qx = h_lo(qr.x), qy = h_hi(qr.x), qz = h_lo(qr.y);
    int cx, cy, cz;
    cell_xyz(g, a, a.cell[s], cx, cy, cz);
    const double nn = (double)q.n;
    const double m0 = q.S0 / nn, m1 = q.S1 / nn, m2 = q.S2 / nn;
    C[0] = q.S00 - nn * m0 * m0; C[1] = q.S01 - nn * m0 * m1; C[2] = q.S02 - nn * m0 * m2;
    C[3] = C[1];                 C[4] = q.S11 - nn * m1 * m1; C[5] = q.S12 - nn * m1 * m2;
    C[6] = C[2];                 C[7] = C[5];                 C[8] = q.S22 - nn * m2 * m2;
    xa = g.o[0] + (double)cx * g.h + (double)qx + m0;
    ya = g.o[1] + (double)cy * g.h + (double)qy + m1;
    za = g.o[2] + (double)cz * g.h + (double)qz + m2;
}

// the rows h16_plane left to the Jacobi core
__global__ __launch_bounds__(kB) void k_h16_cw_planes_fb(H16Args a, const CwSums* __restrict__ sums, const int64_t* __restrict__ list,
                                                         const uint32_t* __restrict__ nlist, pcp_plane* __restrict__ out_nrm) {
    const uint32_t m = *nlist;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const int64_t s = list[i];
        double C[9], xa, ya, za;
        cw_cov(a, s, sums[s], C, xa, ya, za);
        pcp_plane pl;
        plane_from_cov(C, xa, ya, za, pl);
        out_nrm[a.mapping[s]] = pl;
    }
}

// the planes of k_h16_cw's sums (sorted order): H16Acc::finish's fp64 covariance, then h16_plane
__global__ __launch_bounds__(kB) void k_h16_cw_planes(H16Args a, const CwSums* __restrict__ sums, pcp_plane* __restrict__ out_nrm,
                                                      int64_t* __restrict__ fb, uint32_t* __restrict__ nfb) {
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < a.n; s += (int64_t)gridDim.x * blockDim.x) {
        const int32_t caller = a.mapping[s];
        if (caller >= a.n_owned) continue;
        const CwSums q = sums[s];
        pcp_plane pl{0.f, 0.f, 0.f, 0.f, 1.f, 0.f};
        if (q.n > 0) {
            double C[9], xa, ya, za;
            cw_cov(a, s, q, C, xa, ya, za);
            if (!h16_plane(C, xa, ya, za, pl)) {
                fb[atomicAdd(nfb, 1u)] = s;
                continue;
            }
        }
        out_nrm[caller] = pl;
    }
}

H16Args make_args(const pcp_index* ix, float r, int64_t n_owned) {
    H16Args a{};
    a.g = ix->g;
    a.rec = ix->h16;
    a.cell = ix->cell;
    a.mapping = ix->mapping;
    a.n = ix->n;
    a.n_owned = n_owned;
    a.hf = (float)ix->g.h;
    a.r2 = r * r;
    a.inv_nx = 1.0 / (double)ix->g.n[0];
    a.inv_nxy = 1.0 / ((double)ix->g.n[0] * (double)ix->g.n[1]);
    const float rc = r * 1.0001f + 2e-4f;  // conservative: fp16 offsets and fp32 face gaps
    a.rcut2 = rc * rc;
    return a;
}

// the LDS-staged kernel (1, default) or the per-lane global one (PCP_H16_TILE=0, for A/B)
bool h16_tile_mode() {
    const char* e = getenv("PCP_H16_TILE");
    return e ? atoi(e) != 0 : PCP_H16_TILE_DEFAULT != 0;
}
// the tile fill writes rows straight to caller order (1) or stages them for the copy pass (0);
// PCP_H16_DIRECT for A/B
bool h16_direct_mode() {
    const char* e = getenv("PCP_H16_DIRECT");
    return e ? atoi(e) != 0 : PCP_H16_DIRECT_DEFAULT != 0;
}
// the fused count (1, default) or count-only + full fill (PCP_H16_FUSED=0); PCP_H16_FUSED_STRIDE
// overrides the staging stride (tests force overflowing rows with a small one)
// the cell-wave kernels (1, default) or the per-lane / tile forms (PCP_H16_CW=0, for A/B)
bool h16_cw_mode() {
    const char* e = getenv("PCP_H16_CW");
    return e ? atoi(e) != 0 : PCP_H16_CW_DEFAULT != 0;
}
unsigned cw_blocks(int64_t n) {
    const int64_t waves = (n + 63) / 64;
    return (unsigned)std::min<int64_t>(std::max<int64_t>((waves + kCwWaves - 1) / kCwWaves, 1), 1 << 20);
}
bool h16_fused_mode() {
    const char* e = getenv("PCP_H16_FUSED");
    return e ? atoi(e) != 0 : PCP_H16_FUSED_DEFAULT != 0;
}
uint32_t h16_fused_stride() {
    const char* e = getenv("PCP_H16_FUSED_STRIDE");
    const long v = e ? atol(e) : PCP_H16_FUSED_STRIDE;
    return (uint32_t)std::min<long>(std::max<long>((v + 15) / 16 * 16, 16), 4096);
}
unsigned tile_blocks(int64_t n) { return (unsigned)std::min<int64_t>(std::max<int64_t>((n + 63) / 64, 1), 1 << 20); }

int check_query(pcp_ctx* ctx, const pcp_index* ix, float r, int64_t n_owned) {
    if (!ix || !ix->is_h16) return set_error(ctx, PCP_ERR_ARG, "not an fp16 (pcp_index_build_h16) index");
    if (!(r > 0.f) || (double)r > ix->g.h * 1.000001)
        return set_error(ctx, PCP_ERR_UNSUPPORTED, "h16 radius must satisfy 0 < r <= cell size (3x3x3 cells)");
    if (n_owned < 0) return set_error(ctx, PCP_ERR_ARG, "n_owned < 0");
    return PCP_OK;
}

}  // namespace
}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_index_build_h16(pcp_ctx* ctx, const float* xyz, size_t stride, int64_t n, double cell_size, pcp_index** out) {
    if (!ctx || !out || !(cell_size > 0)) return set_error(ctx, PCP_ERR_ARG, "pcp_index_build_h16: bad arguments");
    if (cell_size > 0.5) return set_error(ctx, PCP_ERR_UNSUPPORTED, "h16 cells > 0.5 m lose fp16 offset precision");
    pcp_index* ix = nullptr;
    PCP_TRY(pcp_index_build_f32(ctx, xyz, stride, n, cell_size, &ix));
    if (!ix->g.dense) {
        pcp_index_destroy(ix);
        return set_error(ctx, PCP_ERR_UNSUPPORTED, "h16 index needs a dense cell table (bbox too large for the cell size)");
    }
    int rc = PCP_OK;
    if ((rc = dmalloc(ctx, &ix->h16, ix->n + 1)) || (rc = dmalloc(ctx, &ix->cell, ix->n + 1)) ||
        (!ix->mapping && (rc = dmalloc(ctx, &ix->mapping, ix->n + 1)))) {
        pcp_index_destroy(ix);
        return rc;
    }
    if (ix->n > 0)
        hipLaunchKernelGGL(k_h16_convert, dim3(grid_for(ix->n, kB)), dim3(kB), 0, ctx->stream, ix->g,
                           (const float4*)ix->pts, ix->n, ix->h16, ix->cell, ix->mapping);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        pcp_index_destroy(ix);
        return hip_fail(ctx, e, "h16 convert", __FILE__, __LINE__);
    }
    dfree(ctx, ix->pts);  // the fp32 records are not needed by the fp16 search
    ix->pts = nullptr;
    ix->is_h16 = 1;
    *out = ix;
    return PCP_OK;
}

int pcp_h16_radius_count(pcp_ctx* ctx, const pcp_index* ix, float radius, int64_t n_owned, int32_t* count_dev) {
    if (!ctx || (n_owned > 0 && !count_dev)) return set_error(ctx, PCP_ERR_ARG, "pcp_h16_radius_count: bad arguments");
    PCP_TRY(check_query(ctx, ix, radius, n_owned));
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    if (n_owned == 0) return PCP_OK;
    // rows of owned points the build dropped as non-finite stay empty (the cell-wave count writes
    // every point of the index, so with nothing dropped there is nothing to clear)
    if (!(h16_cw_mode() && ix->n == ix->n_in))
        PCP_HIP(ctx, hipMemsetAsync(count_dev, 0, (size_t)n_owned * sizeof(int32_t), ctx->stream));
    if (ix->n == 0) return PCP_OK;
    const H16Args a = make_args(ix, radius, n_owned);
    // keep the sorted-order row lengths and the inverse map for the fill of the same query set
    pcp_index* ixm = const_cast<pcp_index*>(ix);
    ixm->h16_last_r = -1.f;
    if (!ixm->h16_cnt_s) PCP_TRY(dmalloc(ix->owner, &ixm->h16_cnt_s, (size_t)ix->n));
    if (ixm->h16_inv_cap < n_owned) {
        dfree(ix->owner, ixm->h16_inv);
        ixm->h16_inv = nullptr;
        ixm->h16_inv_cap = 0;
        PCP_TRY(dmalloc(ix->owner, &ixm->h16_inv, (size_t)n_owned));
        ixm->h16_inv_cap = n_owned;
    }
    ixm->h16_fused_r = -1.f;
    if (h16_cw_mode()) {
        hipLaunchKernelGGL(k_h16_cw<false>, dim3(cw_blocks(ix->n)), dim3(kB), 0, ctx->stream, a, count_dev,
                           (const int64_t*)nullptr, (const int32_t*)nullptr, (int32_t*)nullptr, (CwSums*)nullptr);
        PCP_LAUNCH_CHECK(ctx);
        return PCP_OK;
    }
    if (!h16_tile_mode() && h16_fused_mode()) {
        // the fused count: rows, planes and the overflow list for the fill; needs ~4 x stride
        // bytes per point of staging, so it gives way to the two-pass form when that is not there
        const uint32_t stride = h16_fused_stride();
        const int64_t spill_rows = std::max<int64_t>(1024, ix->n / 32);  // ~1.4 % of the rows spill at 96
        const size_t need = ((size_t)ix->n + (size_t)spill_rows) * stride;
        bool ok = true;
        if (ixm->h16_rows_cap < (int64_t)need) {
            dfree(ix->owner, ixm->h16_rows);
            ixm->h16_rows = nullptr;
            ixm->h16_rows_cap = 0;
            ok = dmalloc(ix->owner, &ixm->h16_rows, need) == PCP_OK;
            if (ok) ixm->h16_rows_cap = (int64_t)need;
        }
        if (ok && ixm->h16_ovf_cap < n_owned) {
            dfree(ix->owner, ixm->h16_planes);
            dfree(ix->owner, ixm->h16_ovf);
            dfree(ix->owner, ixm->h16_spill_of);
            ixm->h16_planes = nullptr;
            ixm->h16_ovf = nullptr;
            ixm->h16_spill_of = nullptr;
            ixm->h16_ovf_cap = 0;
            ok = dmalloc(ix->owner, &ixm->h16_planes, (size_t)n_owned) == PCP_OK &&
                 dmalloc(ix->owner, &ixm->h16_ovf, (size_t)n_owned + 2) == PCP_OK &&
                 dmalloc(ix->owner, &ixm->h16_spill_of, (size_t)n_owned) == PCP_OK;
            if (ok) ixm->h16_ovf_cap = n_owned;
        }
        if (ok) {
            H16Args af = a;
            af.cap = stride;
            af.ovf = ixm->h16_ovf;
            af.novf = (uint32_t*)(ixm->h16_ovf + ixm->h16_ovf_cap);
            af.nspill = af.novf + 1;
            af.spill_of = ixm->h16_spill_of;
            af.spill_rows = (uint32_t)spill_rows;
            af.spill_base = (int64_t)ix->n * stride;
            PCP_HIP(ctx, hipMemsetAsync(af.novf, 0, 2 * sizeof(uint32_t), ctx->stream));
            hipLaunchKernelGGL(k_h16_plane_default, dim3(grid_for(n_owned, kB)), dim3(kB), 0, ctx->stream,
                               ixm->h16_planes, n_owned);
            hipLaunchKernelGGL(k_h16_radius<true>, dim3(grid_for(ix->n, kB)), dim3(kB), 0, ctx->stream, af, count_dev,
                               (const int64_t*)nullptr, (const int32_t*)ix->mapping, ixm->h16_rows, ixm->h16_planes,
                               (int32_t*)nullptr, ixm->h16_inv);
            PCP_LAUNCH_CHECK(ctx);
            ixm->h16_fused_r = radius;
            ixm->h16_fused_owned = n_owned;
            ixm->h16_fused_stride = stride;
            return PCP_OK;
        }
        // not enough device memory for the staging: release what was taken, count only
        dfree(ix->owner, ixm->h16_rows);
        ixm->h16_rows = nullptr;
        ixm->h16_rows_cap = 0;
    }
    if (h16_tile_mode())
        hipLaunchKernelGGL(k_h16_tile<false>, dim3(tile_blocks(ix->n)), dim3(64), 0, ctx->stream, a, count_dev,
                           (const int64_t*)nullptr, (const int32_t*)nullptr, (int32_t*)nullptr, (pcp_plane*)nullptr,
                           ixm->h16_cnt_s, ixm->h16_inv, (unsigned long long*)nullptr);
    else
        hipLaunchKernelGGL(k_h16_radius<false>, dim3(grid_for(ix->n, kB)), dim3(kB), 0, ctx->stream, a, count_dev,
                           (const int64_t*)nullptr, (const int32_t*)nullptr, (int32_t*)nullptr, (pcp_plane*)nullptr,
                           ixm->h16_cnt_s, ixm->h16_inv);
    PCP_LAUNCH_CHECK(ctx);
    ixm->h16_last_r = radius;
    ixm->h16_last_owned = n_owned;
    return PCP_OK;
}

int pcp_h16_radius_fill(pcp_ctx* ctx, const pcp_index* ix, float radius, int64_t n_owned, const int64_t* offsets_dev,
                        const int32_t* global_id_dev, int32_t* idx_dev, pcp_plane* normals_dev) {
    if (!ctx || (n_owned > 0 && (!offsets_dev || !idx_dev)))
        return set_error(ctx, PCP_ERR_ARG, "pcp_h16_radius_fill: bad arguments");
    PCP_TRY(check_query(ctx, ix, radius, n_owned));
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    if (n_owned == 0) return PCP_OK;
    if (ix->n > 0 && ix->h16_rows && ix->h16_fused_r == radius && ix->h16_fused_owned == n_owned) {
        // the fused count of this radius and query set staged the rows and planes: move them
        const H16Args a = make_args(ix, radius, n_owned);
        const uint32_t* novf_dev = (const uint32_t*)(ix->h16_ovf + ix->h16_ovf_cap);
        uint32_t novf = 0;
        PCP_HIP(ctx, hipMemcpyAsync(&novf, novf_dev, sizeof(novf), hipMemcpyDeviceToHost, ctx->stream));
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
        hipLaunchKernelGGL(k_h16_rows_to_caller, dim3(grid_for(n_owned, kB, 1 << 16)), dim3(kB), 0, ctx->stream,
                           (const int32_t*)ix->h16_inv, n_owned, (const int64_t*)nullptr, offsets_dev,
                           (const int32_t*)ix->h16_rows, idx_dev, (int64_t)ix->h16_fused_stride, global_id_dev,
                           (const pcp_plane*)ix->h16_planes, normals_dev, (const int32_t*)ix->h16_spill_of,
                           (int64_t)ix->n * ix->h16_fused_stride);
        PCP_LAUNCH_CHECK(ctx);
        if (novf == 0) return PCP_OK;
        int32_t* ids = nullptr;
        struct Free {
            pcp_ctx* c; int32_t** a;
            ~Free() { dfree(c, *a); }
        } fr{ctx, &ids};
        const int32_t* rep_ids = ix->mapping;  // the reported ids: the caller indices, or their global ids
        if (global_id_dev) {
            PCP_TRY(dmalloc(ctx, &ids, (size_t)ix->n));
            hipLaunchKernelGGL(k_h16_ids, dim3(grid_for(ix->n, kB)), dim3(kB), 0, ctx->stream, (const int32_t*)ix->mapping,
                               global_id_dev, ix->n, ids);
            rep_ids = ids;
        }
        hipLaunchKernelGGL(k_h16_overflow, dim3(grid_for(novf, kB)), dim3(kB), 0, ctx->stream, a, novf_dev,
                           (const int32_t*)ix->h16_ovf, offsets_dev, rep_ids, idx_dev);
        PCP_LAUNCH_CHECK(ctx);
        return PCP_OK;
    }
    // planes of points the build dropped; the cell-wave fill writes every point of the index
    if (normals_dev && !(h16_cw_mode() && ix->n == ix->n_in))
        hipLaunchKernelGGL(k_h16_plane_default, dim3(grid_for(n_owned, kB)), dim3(kB), 0, ctx->stream, normals_dev,
                           n_owned);
    if (ix->n == 0) return PCP_OK;
    const H16Args a = make_args(ix, radius, n_owned);
    if (h16_cw_mode()) {  // rows straight into the caller's CSR, sums in sorted order, then the planes
        int32_t* ids = nullptr;
        CwSums* sm = nullptr;
        struct Free {
            pcp_ctx* c; int32_t** a; CwSums** b;
            ~Free() { dfree(c, *a); dfree(c, *b); }
        } fr{ctx, &ids, &sm};
        if (normals_dev) PCP_TRY(dmalloc(ctx, &sm, (size_t)ix->n));
        // the reported ids: the caller indices (the index's own mapping), or their global ids
        const int32_t* rep_ids = ix->mapping;
        if (global_id_dev) {
            PCP_TRY(dmalloc(ctx, &ids, (size_t)ix->n));
            hipLaunchKernelGGL(k_h16_ids, dim3(grid_for(ix->n, kB)), dim3(kB), 0, ctx->stream,
                               (const int32_t*)ix->mapping, global_id_dev, ix->n, ids);
            rep_ids = ids;
        }
        hipLaunchKernelGGL(k_h16_cw<true>, dim3(cw_blocks(ix->n)), dim3(kB), 0, ctx->stream, a, (int32_t*)nullptr,
                           offsets_dev, rep_ids, idx_dev, sm);
        if (normals_dev) {
            int64_t* fb = nullptr;
            struct FreeFb {
                pcp_ctx* c; int64_t** a;
                ~FreeFb() { dfree(c, *a); }
            } ffb{ctx, &fb};
            PCP_TRY(dmalloc(ctx, &fb, (size_t)ix->n + 1));
            uint32_t* nfb = (uint32_t*)(fb + ix->n);
            PCP_HIP(ctx, hipMemsetAsync(nfb, 0, sizeof(uint32_t), ctx->stream));
            hipLaunchKernelGGL(k_h16_cw_planes, dim3(grid_for(ix->n, kB)), dim3(kB), 0, ctx->stream, a,
                               (const CwSums*)sm, normals_dev, fb, nfb);
            hipLaunchKernelGGL(k_h16_cw_planes_fb, dim3(256), dim3(kB), 0, ctx->stream, a, (const CwSums*)sm,
                               (const int64_t*)fb, (const uint32_t*)nfb, normals_dev);
        }
        PCP_LAUNCH_CHECK(ctx);
        return PCP_OK;
    }
    int64_t total = 0;
    PCP_HIP(ctx, hipMemcpyAsync(&total, offsets_dev + n_owned, sizeof(total), hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    int32_t *ids = nullptr, *cnt_s = nullptr, *inv = nullptr, *tmp = nullptr;
    int64_t* soff = nullptr;
    struct Free {
        pcp_ctx* c; int32_t **a, **b, **d, **e; int64_t** f;
        ~Free() { dfree(c, *a); dfree(c, *b); dfree(c, *d); dfree(c, *e); dfree(c, *f); }
    } fr{ctx, &ids, &cnt_s, &inv, &tmp, &soff};
    PCP_TRY(dmalloc(ctx, &ids, (size_t)ix->n));
    hipLaunchKernelGGL(k_h16_ids, dim3(grid_for(ix->n, kB)), dim3(kB), 0, ctx->stream, (const int32_t*)ix->mapping,
                       global_id_dev, ix->n, ids);
    if (h16_tile_mode() && h16_direct_mode()) {  // rows straight into the caller's CSR (no staging, no copy)
        hipLaunchKernelGGL((k_h16_tile<true, true>), dim3(tile_blocks(ix->n)), dim3(64), 0, ctx->stream, a,
                           (int32_t*)nullptr, offsets_dev, (const int32_t*)ids, idx_dev, normals_dev, (int32_t*)nullptr,
                           (int32_t*)nullptr, (unsigned long long*)nullptr);
        PCP_LAUNCH_CHECK(ctx);
        return PCP_OK;
    }
    PCP_TRY(dmalloc(ctx, &soff, (size_t)ix->n + 1));
    PCP_TRY(dmalloc(ctx, &tmp, (size_t)total + (kRowPad - 1) * (size_t)n_owned + kRowPad));  // padded rows
    // the sorted-order row lengths and the inverse map: kept by the count pass of this radius and
    // query set, else gathered back from the caller offsets
    const int32_t *cnt_use = ix->h16_cnt_s, *inv_use = ix->h16_inv;
    if (!(ix->h16_cnt_s && ix->h16_last_r == radius && ix->h16_last_owned == n_owned)) {
        PCP_TRY(dmalloc(ctx, &cnt_s, (size_t)ix->n));
        PCP_TRY(dmalloc(ctx, &inv, (size_t)n_owned));
        hipLaunchKernelGGL(k_h16_sorted_counts, dim3(grid_for(ix->n, kB)), dim3(kB), 0, ctx->stream,
                           (const int32_t*)ix->mapping, ix->n, n_owned, offsets_dev, cnt_s, inv);
        cnt_use = cnt_s;
        inv_use = inv;
    }
    PCP_LAUNCH_CHECK(ctx);
    PCP_TRY(scan_i32_to_i64(ctx, cnt_use, ix->n, soff, nullptr));
    if (h16_tile_mode())
        hipLaunchKernelGGL((k_h16_tile<true, false>), dim3(tile_blocks(ix->n)), dim3(64), 0, ctx->stream, a, (int32_t*)nullptr,
                           (const int64_t*)soff, (const int32_t*)ids, tmp, normals_dev, (int32_t*)nullptr,
                           (int32_t*)nullptr, (unsigned long long*)nullptr);
    else
        hipLaunchKernelGGL(k_h16_radius<true>, dim3(grid_for(ix->n, kB)), dim3(kB), 0, ctx->stream, a,
                           (int32_t*)nullptr, (const int64_t*)soff, (const int32_t*)ids, tmp, normals_dev);
    hipLaunchKernelGGL(k_h16_rows_to_caller, dim3(grid_for(n_owned, kB, 1 << 16)), dim3(kB), 0, ctx->stream,
                       inv_use, n_owned, (const int64_t*)soff, offsets_dev, (const int32_t*)tmp, idx_dev);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

}  // extern "C"
