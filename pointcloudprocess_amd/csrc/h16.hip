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
// query's neighbours lie in its 3x3x3 cells.
//
// The search is a matrix contraction on the matrix cores (k_h16_mx): one wave per query cell
// holds the cell's 3x3x3 neighbourhood (the candidates, one per lane and step), and for 16
// queries at a time
//   * the hit test d^2 - r^2 = |P|^2 - 2 P.Q + (|Q|^2 - r^2) < 0 is a K = 4 product of the
//     candidates' [P, |P|^2] with the queries' [-2 Q, 1] on fp32 MFMA (v_mfma_f32_4x4x1_16b_f32:
//     rows = 4 queries broadcast to every lane block, columns = the 64 candidates, so one compare
//     gives a query's hit mask over the wave in candidate = row order);
//   * the F1 sums (S P, S P P^T of the hits) are the product of the 0/1 hit matrix with the
//     candidates' moment features, on f16 MFMA with fp32 accumulation
//     (v_mfma_f32_16x16x32_f16; each moment, in cell units, as an f16 hi + lo pair, ~22
//     significant bits at any cell size).  The hit
//     matrix comes from the same contraction evaluated in the transposed layout
//     (v_mfma_f32_16x16x4_f32: rows = candidates, columns = queries), which is the f16 MFMA's B
//     operand with no lane movement; both layouts run the same k-ordered fp32 fma chain on the
//     same operands, so the sums see exactly the row's hit set (tools/mfma_probe.hip checks the
//     bit identity on the hardware).
// Coordinates are relative to the query cell's centre (|P| <= 1.5 h per axis), in fp32.
//
// Numerics: neighbour iff d^2 < r^2 (strict, as FLANN's RadiusResultSet) with d^2 from the
// expansion above; against the exact fp64 search a pair can differ only when | |p - q| - r | <
// 3e-4 m (the fp16 quantisation bound of the stored offsets; the expansion's own fp32 error is
// ~1e-7 m); tests exclude that band.  Rows are in index (scan) order, the reference's unsorted
// mode.  Normals: the covariance S P P^T - n mu mu^T formed in fp64 from the fp32 sums, then the
// F1 eigen core (closed form, Jacobi for near-degenerate rows; pca.hpp).
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "grid.hpp"
#include "pca.hpp"

namespace pcp {
namespace {

constexpr int kB = 256;

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

struct H16Args {
    GridDesc g;
    const uint2* rec;
    const uint32_t* cell;
    const int32_t* mapping;
    int64_t n, n_owned;
    float hf, r2;             // cell size, r^2
    double inv_nx, inv_nxy;   // 1 / n[0], 1 / (n[0] n[1]): cell coordinates without integer division
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

// the id each sorted point is reported under (the global id of its caller index): gathered once
// per point here instead of once per neighbour in the fill pass
__global__ void k_h16_ids(const int32_t* mapping, const int32_t* gid, int64_t n, int32_t* out) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t m = mapping[k];
        out[k] = gid ? gid[m] : m;
    }
}

__global__ void k_h16_plane_default(pcp_plane* out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = pcp_plane{0.f, 0.f, 0.f, 0.f, 1.f, 0.f};  // points dropped as non-finite
}

// ---- the MFMA cell-wave kernels (count and fill)
// One wave (one 64-thread workgroup) per query cell: the cells whose first sorted point falls in
// the wave's 64 sorted positions.  The cell's 3x3x3 neighbourhood -- the 9 (dy, dz) rows of cells
// [cx - 1, cx + 1], concatenated in visiting order (dz, dy, then ascending sorted position) --
// is loaded one candidate per lane and step, in blocks of kMxSteps steps (larger neighbourhoods,
// ~2 % of the queries of the C5 scene, loop over blocks).  The cell's queries then run 16 at a
// time (a "query tile": lane l serves query l & 15):
//   rows  per step and query group g (4 queries): 4 chained v_mfma_f32_4x4x1_16b_f32 with
//         cbsz = 4, abid = g (the group's 4 query coefficients broadcast to all 16 lane blocks)
//         from C = |Q|^2 - r^2 give D[query 4g + i][candidate = lane] in register i; one compare
//         is the query's hit mask, ballot order = candidate order = the row's order, stored as
//         one contiguous run per step straight into the caller's CSR row;
//   sums  (fill) per step and 32-candidate chunk: two v_mfma_f32_16x16x4_f32 give the same
//         D[candidate 16 h + 4 (l >> 4) + i][query l & 15] in register i of lane l, clamped to
//         0/1 as the f16 B operand of v_mfma_f32_16x16x32_f16 whose A operand is the moment
//         features (staged in LDS once per block): D[moment row][query] accumulates S P and
//         S P P^T over the row's hits.
// Per query and 64-candidate step this is ~8 VALU ops (compare, row-store addressing, the mask
// conversion) against ~34 for the per-lane-FMA form it replaces (round 4: the test, the 9 sum
// FMAs on every lane and the sums' 36-value reduce-scatter).
// candidate steps per block (2 x 64): a smaller block is more blocks per neighbourhood but less
// LDS per wave -- 5 waves/SIMD at 128 candidates against 3 at 256 (measured: 256 / 192 / 128 / 64
// candidates 2030 / 2165 / 2240 / 2257 Mpts/s, profiles/r05_c5/)
#ifndef PCP_H16_TRIG32  // planes: the eigen angle in fp32 + fp64 Newton polish of l3 (0: fp64 acos / cos)
#define PCP_H16_TRIG32 1
#endif
#ifndef PCP_MX_STEPS
#define PCP_MX_STEPS 2
#endif
constexpr int kMxSteps = PCP_MX_STEPS;
#ifndef PCP_MX_COUNT_STEPS  // the count pass's steps per block (it stages nothing in LDS)
#define PCP_MX_COUNT_STEPS 4
#endif
constexpr int kMxCountSteps = PCP_MX_COUNT_STEPS;
constexpr int kMxC = kMxSteps * 64;      // candidates per block
constexpr int kMxF = 9;                  // moment feature rows: x y z xx xy xz yy yz zz, each word = (hi, lo) f16
constexpr int kMxFS = kMxC + 4;          // feature row stride (words)
constexpr int kMxPS = kMxC + 16;         // P row stride (floats)
constexpr float kMxFar = 1e30f;          // |P|^2 of a padding candidate, C of a non-query: never a hit
constexpr int kMxWaves = 5;              // waves per SIMD (~7.3 KB of LDS per fill wave)

typedef float mx_f4 __attribute__((ext_vector_type(4)));
typedef _Float16 mx_h8 __attribute__((ext_vector_type(8)));

// one query's F1 sums for k_h16_mx_planes, by caller index: S P (3), S P P^T (xx xy xz yy yz zz) in cell units,
// the hit count and the query's cell (P relative to its centre).  64 bytes: the fill writes each
// record whole with one store instruction (a 64-byte-aligned random write, no partial line), so
// the planes pass reads the sums and writes the planes both in caller order -- a plane written at
// a random caller position (24 B, straddling lines) cost ~8 ms of the 200M step (profiles/r05_c5).
struct alignas(64) MxSums {
    float S[9];
    int32_t n;
    uint32_t cell;
    float pad[5];
};

// D[query 4G + i][candidate lane] += the K = 3 + 1 product of the step (C: the group's |Q|^2 - r^2)
template <int G>
__device__ __forceinline__ mx_f4 mx_rows(float ax, float ay, float az, float bx, float by, float bz, float bp, mx_f4 c) {
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(ax, bx, c, 4, G, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(ay, by, c, 4, G, 0);
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(az, bz, c, 4, G, 0);
    return __builtin_amdgcn_mfma_f32_4x4x1f32(1.f, bp, c, 4, G, 0);
}
template <int G>
__device__ __forceinline__ mx_f4 mx_c(float qc) {  // register i = query 4G + i's |Q|^2 - r^2, exact
    const mx_f4 z = {0.f, 0.f, 0.f, 0.f};
    return __builtin_amdgcn_mfma_f32_4x4x1f32(qc, 1.f, z, 4, G, 0);
}
// 0/1 of a hit (d^2 - r^2 < 0; -0 and +0 are not hits, like the rows' compare): a nonzero D is
// at least ~2^-60 in magnitude (a fma of fp32 operands ~0.1), so the scaled clamp is exact
__device__ __forceinline__ float mx_hit(float d) { return __builtin_amdgcn_fmed3f(d * -0x1p64f, 0.f, 1.f); }

template <bool FILL>
__global__ __launch_bounds__(64, kMxWaves) void k_h16_mx(H16Args a, int32_t* __restrict__ count,
                                                             const int64_t* __restrict__ offsets,
                                                             const int32_t* __restrict__ ids,
                                                             int32_t* __restrict__ out_idx, MxSums* __restrict__ sums) {
    __shared__ uint4 s_row[9];   // per neighbour row: kk = j + off, the query column [b1, b2)
    __shared__ float2 s_rdz[9];  // per neighbour row: its dy h, dz h
    __shared__ float s_p[FILL ? 4 : 1][FILL ? kMxPS : 1];                          // P x y z, |P|^2
    __shared__ __attribute__((aligned(16))) uint32_t s_f[FILL ? kMxF : 1][FILL ? kMxFS : 1];  // moments
    // candidate steps per block: the fill's LDS-sized blocks, the count's own (no LDS staging)
    constexpr int kS = FILL ? kMxSteps : kMxCountSteps;
    constexpr int kC = kS * 64;
    const GridDesc& g = a.g;
    const int lane = threadIdx.x;
    const float hf = a.hf, hh = 0.5f * a.hf, r2 = a.r2;
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    for (int64_t w = blockIdx.x; w * 64 < a.n; w += gridDim.x) {
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
                s_row[lane] = make_uint4(k0 - pre, b1, b2, pre);
                s_rdz[lane] = make_float2((float)(lane % 3 - 1) * hf, (float)(lane / 3 - 1) * hf);
            }
            uint32_t P[9];  // wave-uniform row starts in the concatenated list
            uint32_t M = 0;
#pragma unroll
            for (int k = 0; k < 9; k++) {
                P[k] = M;
                M += (uint32_t)__builtin_amdgcn_readlane((int)len, k);
            }
            wave_sync();
            // the block's candidates: P (query-cell-centre frame) in registers (the rows' B
            // operands) and, for the fill, P and the moment features in LDS
            float bx[kS], by[kS], bz[kS], bp[kS];
            int32_t cidv[kS];
            auto load_block = [&](uint32_t blk) {
#pragma unroll
                for (int s = 0; s < kS; s++) {
                    if (blk + 64u * s >= M) break;  // (uniform) steps past the list are never read
                    const uint32_t j = blk + 64u * s + (uint32_t)lane;
                    const bool ok = j < M;
                    // the row of list entry j: the largest r with P[r] <= j = the number of row
                    // starts P[1..8] at or below j (compares against uniform values, summed: no
                    // divergent branches; a binary search over selects of P compiled to ~40
                    // exec-mask branch instructions per step)
                    int r = 0;
#pragma unroll
                    for (int k = 1; k < 9; k++) r += j >= P[k] ? 1 : 0;
                    const uint4 row = s_row[r];
                    const uint32_t kk = ok ? j + row.x : 0u;
                    const uint2 pr = a.rec[kk];
                    cidv[s] = FILL && ok ? ids[kk] : 0;
                    const float2 rdz = s_rdz[r];
                    const float cdx = kk < row.y ? -hf : (kk < row.z ? 0.f : hf);
                    const float px = ok ? (cdx + h_lo(pr.x)) - hh : 0.f;
                    const float py = ok ? (rdz.x + h_hi(pr.x)) - hh : 0.f;
                    const float pz = ok ? (rdz.y + h_lo(pr.y)) - hh : 0.f;
                    const float p2 = ok ? __fmaf_rn(pz, pz, __fmaf_rn(py, py, px * px)) : kMxFar;
                    bx[s] = px;
                    by[s] = py;
                    bz[s] = pz;
                    bp[s] = p2;
                    if constexpr (FILL) {
                        const int c = 64 * s + lane;
                        s_p[0][c] = px;
                        s_p[1][c] = py;
                        s_p[2][c] = pz;
                        s_p[3][c] = p2;
                        // the moments in cell units (|u| <= 1.5), not metres: split into f16 (hi, lo)
                        // pairs they keep ~22 significant bits at any cell size, where metre-sized
                        // moments of a mm-scale cell would fall into f16's subnormal range
                        const float ux = px * g.inv_hf, uy = py * g.inv_hf, uz = pz * g.inv_hf;
                        const float mo[9] = {ux, uy, uz, ux * ux, ux * uy, ux * uz, uy * uy, uy * uz, uz * uz};
#pragma unroll
                        for (int k = 0; k < 9; k++) {
                            const _Float16 hi = (_Float16)mo[k];
                            const _Float16 lo = (_Float16)(mo[k] - (float)hi);
                            s_f[k][c] = (uint32_t)__builtin_bit_cast(uint16_t, hi) |
                                        ((uint32_t)__builtin_bit_cast(uint16_t, lo) << 16);
                        }
                    }
                }
            };
            const uint32_t nblk = (M + kC - 1) / kC;
            if (nblk == 1) {
                load_block(0u);
                wave_sync();
            }
            // the cell's queries, 16 at a time
            for (int64_t qs = cs; qs < ce; qs += 16) {
                const int nq = (int)min((int64_t)16, ce - qs);
                const int t = lane & 15, kq = lane >> 4;
                float Qx = 0.f, Qy = 0.f, Qz = 0.f;
                int32_t caller = 0x7fffffff;
                int64_t base = 0;
                if (t < nq) {
                    const uint2 qr = a.rec[qs + t];
                    Qx = h_lo(qr.x) - hh, Qy = h_hi(qr.x) - hh, Qz = h_lo(qr.y) - hh;
                    caller = a.mapping[qs + t];
                    if (FILL && caller < a.n_owned) base = offsets[caller];
                }
                const bool own = t < nq && caller < a.n_owned;
                const uint32_t ownm = (uint32_t)__ballot(own && lane < 16);  // the tile's queries (bits 0..15)
                const float qc = own ? __fmaf_rn(Qz, Qz, __fmaf_rn(Qy, Qy, Qx * Qx)) - r2 : kMxFar;
                const float ax = own ? -2.f * Qx : 0.f, ay = own ? -2.f * Qy : 0.f, az = own ? -2.f * Qz : 0.f;
                const mx_f4 C0 = mx_c<0>(qc), C1 = mx_c<1>(qc), C2 = mx_c<2>(qc), C3 = mx_c<3>(qc);
                // the transposed form's B operand (k = lane >> 4 of query lane & 15) and C
                const float b16 = kq == 0 ? ax : (kq == 1 ? ay : (kq == 2 ? az : 1.f));
                const mx_f4 c16 = {qc, qc, qc, qc};
                int32_t cntv = 0;  // lane t: query t's row length so far
                mx_f4 acc1 = {0.f, 0.f, 0.f, 0.f};
                // rows of query group G (queries 4G .. 4G + 3) over the block's steps: the group's
                // row starts and lengths live in scalar registers for the pass
                auto group_rows = [&](auto gtag, const mx_f4& Cg, uint32_t mb) {
                    constexpr int G = decltype(gtag)::value;
                    if (!((ownm >> (4 * G)) & 0xfu)) return;
                    int64_t rb[4];
                    uint32_t rc[4];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        rc[i] = (uint32_t)__builtin_amdgcn_readlane(cntv, 4 * G + i);
                        if constexpr (FILL) {
                            const uint64_t bq = (uint64_t)base;
                            rb[i] = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bq, 4 * G + i)) |
                                              ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bq >> 32), 4 * G + i) << 32));
                        }
                    }
                    // the block's products first (independent chains in flight), then the rows
                    mx_f4 Ds[kS];
#pragma unroll
                    for (int s = 0; s < kS; s++)
                        if (64u * s < mb) Ds[s] = mx_rows<G>(ax, ay, az, bx[s], by[s], bz[s], bp[s], Cg);
#pragma unroll
                    for (int s = 0; s < kS; s++) {
                        if (64u * s >= mb) break;
                        const mx_f4 D = Ds[s];
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            // (a query outside the tile has C = far: never a hit)
                            const bool hit = D[i] < 0.f;
                            const uint64_t m = __ballot(hit);
                            if constexpr (FILL) {
                                if (hit) {  // the row entries of this step: one contiguous run
                                    int32_t* row = out_idx + (rb[i] + (int64_t)rc[i]);  // uniform
                                    row[__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = cidv[s];
                                }
                            }
                            rc[i] += (uint32_t)__popcll(m);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < 4; i++) cntv = lane == 4 * G + i ? (int32_t)rc[i] : cntv;
                };
                for (uint32_t b = 0; b < nblk; b++) {
                    if (nblk > 1) {  // (uniform) a neighbourhood larger than one block
                        wave_sync();
                        load_block(b * (uint32_t)kC);
                        wave_sync();
                    }
                    const uint32_t mb = min(M - b * (uint32_t)kC, (uint32_t)kC);
                    group_rows(std::integral_constant<int, 0>{}, C0, mb);
                    group_rows(std::integral_constant<int, 1>{}, C1, mb);
                    group_rows(std::integral_constant<int, 2>{}, C2, mb);
                    group_rows(std::integral_constant<int, 3>{}, C3, mb);
                    if constexpr (FILL) {
#pragma unroll
                        for (int s = 0; s < kS; s++) {
                            if (64u * s >= mb) break;
                            // sums: the hit matrix in the transposed layout, then moments x hits,
                            // 16 candidates per product: K = 32 runs over (candidate, hi / lo)
                            // pairs, so each moment's two f16 halves meet the same hit and add
#pragma unroll
                            for (int ch = 0; ch < 4; ch++) {
                                if (64u * s + 16u * ch >= mb) break;
                                const int c0 = 64 * s + 16 * ch;
                                const mx_f4 S = __builtin_amdgcn_mfma_f32_16x16x4f32(s_p[kq][c0 + t], b16, c16, 0, 0, 0);
                                mx_h8 mk;
#pragma unroll
                                for (int i = 0; i < 4; i++) {
                                    const _Float16 h = (_Float16)mx_hit(S[i]);
                                    mk[2 * i] = h;
                                    mk[2 * i + 1] = h;
                                }
                                // A: moment t (rows past the 9 moments repeat the last; their
                                // sums are never read) of candidates c0 + 4 kq + 0..3, (hi, lo) each
                                const mx_h8 fa = __builtin_bit_cast(mx_h8, *(const uint4*)&s_f[min(t, kMxF - 1)][c0 + 4 * kq]);
                                acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa, mk, acc1, 0, 0, 0);
                            }
                        }
                    }
                }
                if constexpr (!FILL) {
                    if (own && lane < 16) count[caller] = cntv;
                } else if (sums) {
                    // lane l: 16 bytes of query t's record -- moments 4 kq + i (kq = 2: the ninth, zz,
                    // the count and the cell; kq = 3: padding), the four lanes one whole record
                    const int32_t n_t = __shfl(cntv, t, 64);
                    float4 v = make_float4(acc1[0], acc1[1], acc1[2], acc1[3]);
                    if (kq == 2) v = make_float4(acc1[0], __int_as_float(n_t), __uint_as_float(cid), 0.f);
                    if (kq == 3) v = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (own) *((float4*)(sums + caller) + kq) = v;
                }
            }
            wave_sync();  // s_row and the block's LDS are rewritten by the next cell
        }
    }
}

// F1's plane from the fp64 covariance by the closed-form symmetric 3x3 eigen decomposition
// (trigonometric eigenvalues, the smallest one's eigenvector as the largest cross product of two
// rows of C - l3 I): a fixed ~250 fp64 ops against the cyclic Jacobi's 4-6 data-dependent sweeps.
// Rows whose two smallest eigenvalues nearly coincide (the normal is ill-conditioned in any
// method; fewer than 3 neighbours, lines) keep the Jacobi core, as does everything outside C5,
// whose results are checked to tolerance (fp32 sums of fp16 offsets) rather than bit for bit.
// Returns false (out untouched) for the rows that keep the Jacobi core (k_h16_mx_planes_fb: the
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
#if PCP_H16_TRIG32
        // The angle and its cosines in fp32 (the fp64 acos and two cos were most of the pass's ~750
        // instructions), then l3 polished by two fp64 Newton steps on det(C - l I).  acos(r) comes
        // from 2 asin(sqrt((1 - |r|) / 2)) with 1 - |r| taken in fp64, so the fp32 angle keeps a
        // relative error ~1e-7 up to |r| -> 1: at r -> 1 (l2 -> l3) l3 then starts within ~1e-7
        // of the l2 - l3 gap from its root (Newton squares that ratio per step; l2 = l3 itself is
        // the Jacobi fallback below), and at r -> -1 (l1 -> l2, planes) l3 does not depend on the
        // angle to first order.
        const float hs = 2.f * asinf(sqrtf((float)(0.5 * (1.0 - fabs(r)))));  // acos(|r|)
        const float phif = (r >= 0.0 ? hs : 3.14159265f - hs) * (1.f / 3.f);
        l1 = m + 2.0 * p * (double)cosf(phif);
        double l = m + 2.0 * p * (double)cosf(phif + 2.0943951f);  // + 2 pi / 3
        const double tr = a00 + a11 + a22;
        const double c1 = a00 * a11 + a00 * a22 + a11 * a22 - p1;  // sum of the principal 2x2 minors
        const double dc = a00 * (a11 * a22 - a12 * a12) - a01 * (a01 * a22 - a12 * a02) + a02 * (a01 * a12 - a11 * a02);
#pragma unroll
        for (int it = 0; it < 2; it++) {
            const double f = ((tr - l) * l - c1) * l + dc;  // det(C - l I) = -l^3 + tr l^2 - c1 l + det C
            const double fp = (2.0 * tr - 3.0 * l) * l - c1;
            l = fp != 0.0 ? l - f / fp : l;
        }
        l3 = l;
#else
        const double phi = acos(r) / 3.0;
        l1 = m + 2.0 * p * cos(phi);
        l3 = m + 2.0 * p * cos(phi + 2.0943951023931954923);  // + 2 pi / 3
#endif
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

// the fp64 covariance S P P^T - n mu mu^T and the absolute mean (the query cell's centre + mu) of
// sorted point s from its sums
__device__ inline void mx_cov(const H16Args& a, uint32_t cid, const MxSums& q, double C[9], double& xa, double& ya,
                              double& za) {
    const GridDesc& g = a.g;
    int cx, cy, cz;
    cell_xyz(g, a, cid, cx, cy, cz);
    // the sums are in cell units (k_h16_mx): back to metres with the kernel's fp32 cell size
    const double nn = (double)q.n, hd = (double)a.hf, hd2 = hd * hd;
    const double m0 = q.S[0] * hd / nn, m1 = q.S[1] * hd / nn, m2 = q.S[2] * hd / nn;
    C[0] = q.S[3] * hd2 - nn * m0 * m0; C[1] = q.S[4] * hd2 - nn * m0 * m1; C[2] = q.S[5] * hd2 - nn * m0 * m2;
    C[3] = C[1];                        C[4] = q.S[6] * hd2 - nn * m1 * m1; C[5] = q.S[7] * hd2 - nn * m1 * m2;
    C[6] = C[2];                        C[7] = C[5];                        C[8] = q.S[8] * hd2 - nn * m2 * m2;
    const double hh = (double)(0.5f * a.hf);  // the kernel's fp32 half cell
    xa = g.o[0] + (double)cx * g.h + hh + m0;
    ya = g.o[1] + (double)cy * g.h + hh + m1;
    za = g.o[2] + (double)cz * g.h + hh + m2;
}

// the rows h16_plane left to the Jacobi core (caller indices)
__global__ __launch_bounds__(kB) void k_h16_mx_planes_fb(H16Args a, const MxSums* __restrict__ sums,
                                                         const int64_t* __restrict__ list,
                                                         const uint32_t* __restrict__ nlist, pcp_plane* __restrict__ out_nrm) {
    const uint32_t m = *nlist;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const int64_t c = list[i];
        const MxSums q = sums[c];
        double C[9], xa, ya, za;
        mx_cov(a, q.cell, q, C, xa, ya, za);
        pcp_plane pl;
        plane_from_cov(C, xa, ya, za, pl);
        out_nrm[c] = pl;
    }
}

// the planes of k_h16_mx's sums, in caller order (sequential reads and writes)
__global__ __launch_bounds__(kB) void k_h16_mx_planes(H16Args a, const MxSums* __restrict__ sums,
                                                      const int64_t* __restrict__ offsets,
                                                      pcp_plane* __restrict__ out_nrm, int64_t* __restrict__ fb,
                                                      uint32_t* __restrict__ nfb) {
    for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < a.n_owned;
         c += (int64_t)gridDim.x * blockDim.x) {
        // the reads issued together (one memory round trip per point; the compiler otherwise sinks
        // the record's loads into the branch below)
        const int64_t o0 = offsets[c], o1 = offsets[c + 1];
        const MxSums q = sums[c];
        asm volatile("" ::"v"(o0), "v"(o1), "v"(q.n));
        if (o1 == o0) continue;  // a point the build dropped: no record, the default plane is set
        pcp_plane pl{0.f, 0.f, 0.f, 0.f, 1.f, 0.f};
        if (q.n > 3) {  // rows of 3 points or fewer keep the default plane (the F1 guard, N > 3)
            double C[9], xa, ya, za;
            mx_cov(a, q.cell, q, C, xa, ya, za);
            if (!h16_plane(C, xa, ya, za, pl)) {
                fb[atomicAdd(nfb, 1u)] = c;
                continue;
            }
        }
        out_nrm[c] = pl;
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
    return a;
}

// one 64-thread workgroup per 64 sorted positions, grid-stride past ~8 resident rounds
unsigned mx_blocks(int64_t n) {
    const int64_t chunks = (n + 63) / 64;
    return (unsigned)std::min<int64_t>(std::max<int64_t>(chunks, 1), 1 << 20);
}

int check_query(pcp_ctx* ctx, const pcp_index* ix, float r, int64_t n_owned) {
    if (!ix || !ix->is_h16) return set_error(ctx, PCP_ERR_ARG, "not an fp16 (pcp_index_build_h16) index");
    if (!(r > 0.f) || (double)r > ix->g.h * 1.000001)
        return set_error(ctx, PCP_ERR_UNSUPPORTED, "h16 radius must satisfy 0 < r <= cell size (3x3x3 cells)");
    if (n_owned < 0) return set_error(ctx, PCP_ERR_ARG, "n_owned < 0");
    // the owned points are a prefix of the cloud the index was built on
    if (n_owned > ix->n_in) return set_error(ctx, PCP_ERR_ARG, "n_owned exceeds the indexed cloud's size");
    return PCP_OK;
}

}  // namespace
}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_index_build_h16(pcp_ctx* ctx, const float* xyz, size_t stride, int64_t n, double cell_size, pcp_index** out) {
    if (!ctx || !out || !(cell_size > 0)) return set_error(ctx, PCP_ERR_ARG, "pcp_index_build_h16: bad arguments");
    if (cell_size > 0.5) return set_error(ctx, PCP_ERR_UNSUPPORTED, "h16 cells > 0.5 m lose fp16 offset precision");
    if (cell_size < 1e-3)  // offsets below ~6e-5 m are f16 subnormals (absolute spacing 6e-8 m)
        return set_error(ctx, PCP_ERR_UNSUPPORTED, "h16 cells < 1 mm put the fp16 offsets in the subnormal range");
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
    // rows of owned points the build dropped as non-finite stay empty (the count writes every
    // owned point of the index, so with nothing dropped there is nothing to clear)
    if (ix->n != ix->n_in) PCP_HIP(ctx, hipMemsetAsync(count_dev, 0, (size_t)n_owned * sizeof(int32_t), ctx->stream));
    if (ix->n == 0) return PCP_OK;
    const H16Args a = make_args(ix, radius, n_owned);
    hipLaunchKernelGGL(k_h16_mx<false>, dim3(mx_blocks(ix->n)), dim3(64), 0, ctx->stream, a, count_dev,
                       (const int64_t*)nullptr, (const int32_t*)nullptr, (int32_t*)nullptr, (MxSums*)nullptr);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_h16_radius_fill(pcp_ctx* ctx, const pcp_index* ix, float radius, int64_t n_owned, const int64_t* offsets_dev,
                        const int32_t* global_id_dev, int32_t* idx_dev, pcp_plane* normals_dev) {
    if (!ctx || (n_owned > 0 && (!offsets_dev || !idx_dev)))
        return set_error(ctx, PCP_ERR_ARG, "pcp_h16_radius_fill: bad arguments");
    PCP_TRY(check_query(ctx, ix, radius, n_owned));
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    if (n_owned == 0) return PCP_OK;
    // planes of points the build dropped (the fill writes every owned point of the index)
    if (normals_dev && ix->n != ix->n_in)
        hipLaunchKernelGGL(k_h16_plane_default, dim3(grid_for(n_owned, kB)), dim3(kB), 0, ctx->stream, normals_dev,
                           n_owned);
    if (ix->n == 0) return PCP_OK;
    const H16Args a = make_args(ix, radius, n_owned);
    int32_t* ids = nullptr;
    MxSums* sm = nullptr;
    int64_t* fb = nullptr;
    struct Free {
        pcp_ctx* c; int32_t** a; MxSums** b; int64_t** d;
        ~Free() { dfree(c, *a); dfree(c, *b); dfree(c, *d); }
    } fr{ctx, &ids, &sm, &fb};
    if (normals_dev) PCP_TRY(dmalloc(ctx, &sm, (size_t)n_owned));
    // the reported ids: the caller indices (the index's own mapping), or their global ids
    const int32_t* rep_ids = ix->mapping;
    if (global_id_dev) {
        PCP_TRY(dmalloc(ctx, &ids, (size_t)ix->n));
        hipLaunchKernelGGL(k_h16_ids, dim3(grid_for(ix->n, kB)), dim3(kB), 0, ctx->stream, (const int32_t*)ix->mapping,
                           global_id_dev, ix->n, ids);
        rep_ids = ids;
    }
    hipLaunchKernelGGL(k_h16_mx<true>, dim3(mx_blocks(ix->n)), dim3(64), 0, ctx->stream, a, (int32_t*)nullptr,
                       offsets_dev, rep_ids, idx_dev, sm);
    if (normals_dev) {
        PCP_TRY(dmalloc(ctx, &fb, (size_t)n_owned + 1));
        uint32_t* nfb = (uint32_t*)(fb + n_owned);
        PCP_HIP(ctx, hipMemsetAsync(nfb, 0, sizeof(uint32_t), ctx->stream));
        hipLaunchKernelGGL(k_h16_mx_planes, dim3(grid_for(n_owned, kB)), dim3(kB), 0, ctx->stream, a,
                           (const MxSums*)sm, offsets_dev, normals_dev, fb, nfb);
        hipLaunchKernelGGL(k_h16_mx_planes_fb, dim3(256), dim3(kB), 0, ctx->stream, a, (const MxSums*)sm,
                           (const int64_t*)fb, (const uint32_t*)nfb, normals_dev);
    }
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

}  // extern "C"
