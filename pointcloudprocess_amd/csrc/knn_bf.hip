// Brute-force exact kNN (BASELINE config C2) on the fp32 matrix cores of gfx950.
//
// Contract: pcp_knn (KdTreeFLANN::nearestKSearch, kd_tree.h:814-845) without an index --
// rows ascending by the FLANN L2_Simple<double> d2 with ties on the target index, d2
// bit-identical to the reference's.  The all-pairs ranking is the one dense contraction
// of the path: score(q, p) = |p|^2 - 2 q.p, a K=4 product
//   A (16 queries x 4) = [-2qx, -2qy, -2qz, 1],  B (4 x 16 targets) = [px; py; pz; |p|^2]
// done by v_mfma_f32_16x16x4_f32 (exact fp32 fma chain).  Lane l of a wave owns target
// column class c = l & 15 and query rows 4*(l>>4)+r (the MFMA C layout), and keeps the L
// best fp32 scores of each (row, class) in registers.  The union of the 16 class lists is
// then re-ranked with the exact fp64 d2 and CERTIFIED: every target outside it has
// score >= tau = min_c(L-th best of class c), so d2 >= |q|^2 + tau - E (E bounds the fp32
// rounding).  A query whose k-th exact d2 is not below that bound is re-done by an exact
// fp64 scan (k_bf_fallback) -- the result is exact either way.
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <vector>

#include "common.hpp"
#include "topk.hpp"

namespace pcp {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4;              // waves per block
// k <= 8 configuration: list length per (row, class), query blocks per wave, waves/SIMD
#ifndef PCP_BF_L8
#define PCP_BF_L8 5
#endif
#ifndef PCP_BF_QB8
#define PCP_BF_QB8 1
#endif
#ifndef PCP_BF_W8
#define PCP_BF_W8 4
#endif
constexpr int kBlock = 64 * kWaves;
#ifndef PCP_BF_TILE
#define PCP_BF_TILE 1024
#endif
#ifndef PCP_BF_DEPTH  // MFMA sub-tiles in flight ahead of the hit test (software pipeline depth)
#define PCP_BF_DEPTH 1
#endif
#ifndef PCP_BF_UNROLL  // sub-tile steps per unrolled loop body
#define PCP_BF_UNROLL 4
#endif
constexpr int kTile = PCP_BF_TILE;     // targets staged in LDS per step
constexpr int kBfUnroll = PCP_BF_UNROLL;
// s_waitcnt immediate for vmcnt(0) with expcnt / lgkmcnt left at their maxima (gfx9 encoding:
// vmcnt [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8])
constexpr int kWaitVm0 = 0x0F70;
constexpr int kPerThread = kTile / kBlock;

__device__ __forceinline__ const double* dptr(const double* base, size_t stride, int64_t i) {
    return (const double*)((const char*)base + (size_t)i * stride);
}

// targets -> {x, y, z, |p|^2} in k-major groups of 16 (group g = targets 16g..16g+15 as x[16],
// y[16], z[16], |p|^2[16]: the B fragment of a 16-target sub-tile, read by lane l as word
// 16 (l >> 4) + (l & 15), is 64 consecutive LDS words, no bank conflicts); non-finite ->
// |p|^2 = +inf (never ranked).  Per-block max of |p|^2 (fp64) and finite count for the host.
__device__ __forceinline__ void bf_put(float* t4, int64_t i, float4 v) {
    float* g = t4 + (i >> 4) * 64 + (i & 15);
    g[0] = v.x;
    g[16] = v.y;
    g[32] = v.z;
    g[48] = v.w;
}
__global__ __launch_bounds__(256) void k_bf_targets(const double* t, size_t stride, int64_t n, float* t4,
                                                    double* part) {
    double pmax = 0.0, cnt = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double* p = dptr(t, stride, i);
        const double x = p[0], y = p[1], z = p[2];
        float4 v;
        if (finite3(x, y, z)) {
            v.x = (float)x; v.y = (float)y; v.z = (float)z;
            v.w = v.x * v.x + v.y * v.y + v.z * v.z;
            pmax = fmax(pmax, x * x + y * y + z * z);
            cnt += 1.0;
        } else {
            v.x = 0.f; v.y = 0.f; v.z = 0.f; v.w = INFINITY;
        }
        bf_put(t4, i, v);
    }
    for (int o = 32; o > 0; o >>= 1) {
        pmax = fmax(pmax, __shfl_xor(pmax, o, 64));
        cnt += __shfl_xor(cnt, o, 64);
    }
    __shared__ double sm[4][2];
    if ((threadIdx.x & 63) == 0) { sm[threadIdx.x >> 6][0] = pmax; sm[threadIdx.x >> 6][1] = cnt; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = sm[0][0], c = sm[0][1];
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) { a = fmax(a, sm[w][0]); c += sm[w][1]; }
        part[2 * blockIdx.x] = a;
        part[2 * blockIdx.x + 1] = c;
    }
}

// the padding [from, to) of the last target tile: never ranked (|p|^2 = +inf)
__global__ void k_bf_pad(float* t4, int64_t from, int64_t to) {
    for (int64_t i = from + threadIdx.x; i < to; i += blockDim.x) bf_put(t4, i, make_float4(0.f, 0.f, 0.f, INFINITY));
}

struct BfArgs {
    const float* t4;   // k-major groups of 16 targets (k_bf_targets)
    const double* t;
    size_t tstride;
    int64_t nt;
    const double* q;
    size_t qstride;
    int64_t nq;
    int k;       // row length of the outputs
    int kk;      // min(k, finite targets)
    double E2;   // fp32 score error bound coefficient: E = E2 * (sqrt(Pmax2) + |q|)^2
    double pmax; // max |p| over finite targets
    int32_t* oidx;
    double* od2;
    int32_t* fb;      // queries to redo exactly
    uint32_t* fb_count;
};

template <int L>
__device__ __forceinline__ void list_insert(float (&s)[L], int (&t)[L], float x, int tx) {
#pragma unroll
    for (int i = L - 1; i >= 1; i--) {
        if (x < s[i - 1]) { s[i] = s[i - 1]; t[i] = t[i - 1]; }
        else if (x < s[i]) { s[i] = x; t[i] = tx; }
    }
    if (x < s[0]) { s[0] = x; t[0] = tx; }
}

// group-of-16 lexicographic min of (d, j)
__device__ __forceinline__ void group_min(double& d, int& j) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
        const double od = __shfl_xor(d, o, 64);
        const int oj = __shfl_xor(j, o, 64);
        if (lex_less(od, oj, d, j)) { d = od; j = oj; }
    }
}

// QB blocks of 16 queries per wave; L = per-(row, class) list length.
template <int L, int QB, int W>
__global__ __launch_bounds__(kBlock, W) void k_bf_mfma(BfArgs a) {
    __shared__ float tiles[2][4 * kTile];  // LDS-DMA double buffer of k-major target groups
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int cls = lane & 15, grp = lane >> 4;
    const int64_t qbase = ((int64_t)blockIdx.x * kWaves + wave) * (16 * QB);

    // A fragments: lane holds A[row = lane&15][k = lane>>4] of each query block
    float afrag[QB];
#pragma unroll
    for (int b = 0; b < QB; b++) {
        const int64_t qi = qbase + b * 16 + cls;
        float v = 0.f;
        if (qi < a.nq) {
            if (grp == 3) v = 1.f;
            else {
                const double c = dptr(a.q, a.qstride, qi)[grp];
                v = isfinite(c) ? -2.f * (float)c : 0.f;
            }
        }
        afrag[b] = v;
    }
    float ls[QB][4][L];
    int lt[QB][4][L];
    // thr = min(class L-th score, th): the score filter.  th = theta + 2E is a row-global
    // bound: theta = k-th smallest of the 16 class bests (k distinct targets score <= theta),
    // so a target scoring above theta + 2E has an exact d2 above theirs -- and above the
    // k-th candidate's -- and can be dropped without weakening the certification.
    // Both bounds only decrease, so thr is maintained as a running min without storing th.
    float thr[QB][4];
#pragma unroll
    for (int b = 0; b < QB; b++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            thr[b][r] = INFINITY;
#pragma unroll
            for (int i = 0; i < L; i++) { ls[b][r][i] = INFINITY; lt[b][r][i] = -1; }
        }
    // The filter rides in the MFMA: C = -thr per row, so an output is negative exactly when the
    // score is below the row's threshold (as of the MFMA's issue; thresholds only fall, so a
    // stale one lets more through), and the common path's hit test is two ORs of the sign bits
    // instead of four compares.  A hit re-scores its target on the VALU from the staged record
    // and this lane's rows' -2q (the same fp32 fma chain as the MFMA's K = 4 product), so the
    // lists never hold a score that passed through the threshold subtraction.
    f32x4 nthr[QB];
    float qm[QB][4][3];
#pragma unroll
    for (int b = 0; b < QB; b++) {
        nthr[b] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int64_t qi = qbase + b * 16 + grp * 4 + r;
#pragma unroll
            for (int c3 = 0; c3 < 3; c3++) {
                float v = 0.f;
                if (qi < a.nq) {
                    const double c = dptr(a.q, a.qstride, qi)[c3];
                    v = isfinite(c) ? -2.f * (float)c : 0.f;
                }
                qm[b][r][c3] = v;
            }
        }
    }
    // wave-uniform fp32 score error bound E (largest |q| of the wave's queries)
    float ew;
    {
        double q2 = 0.0;
#pragma unroll
        for (int b = 0; b < QB; b++) {
            const int64_t qi = qbase + b * 16 + cls;
            if (qi < a.nq && grp == 0) {
                const double* qp = dptr(a.q, a.qstride, qi);
                if (finite3(qp[0], qp[1], qp[2])) q2 = fmax(q2, qp[0] * qp[0] + qp[1] * qp[1] + qp[2] * qp[2]);
            }
        }
        for (int o = 32; o > 0; o >>= 1) q2 = fmax(q2, __shfl_xor(q2, o, 64));
        const double qn = sqrt(q2);
        ew = (float)(a.E2 * (a.pmax + qn) * (a.pmax + qn) * 1.001);
    }
    const bool use_theta = a.kk <= 16;

    const int64_t ntiles = (a.nt + kTile - 1) / kTile;
    // global -> LDS directly (global_load_lds_dwordx4: wave-uniform LDS base + lane * 16 B), one
    // tile ahead into the other buffer; the target array is padded to whole tiles with
    // never-ranked records, so every lane's source address is valid
    auto fetch = [&](int64_t tb, int buf) {
#pragma unroll
        for (int u = 0; u < kPerThread; u++) {
            const float* src = a.t4 + (tb + u * kBlock + threadIdx.x) * 4;  // 16 B per thread, in layout order
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)(&tiles[buf][(u * kBlock) * 4] +
                                                                                       (threadIdx.x & ~63u) * 4),
                                             16, 0, 0);
        }
    };
    fetch(0, 0);
    for (int64_t tt = 0; tt < ntiles; tt++) {
        // tile tt has landed: this wave's LDS-DMA loads are complete (an explicit vmcnt(0): a
        // workgroup barrier's release fence waits only on lgkmcnt on gfx9), then every wave's are,
        // and every wave is done with tile tt - 1
        __builtin_amdgcn_s_waitcnt(kWaitVm0);
        __syncthreads();
        if (tt + 1 < ntiles) fetch((tt + 1) * kTile, (int)((tt + 1) & 1));
        const float* const tf = tiles[tt & 1];
        const int tb = (int)(tt * kTile);
        // B fragment of sub-tile s: word 64 s + 16 grp + cls (k-major group: conflict-free)
        auto bfrag_at = [&](int sub) { return tf[sub * 64 + grp * 16 + cls]; };
        // software pipeline, PCP_BF_DEPTH deep: the MFMAs of sub-tiles s+1 .. s+DEPTH are in flight
        // while the scores of sub-tile s are tested, so the hit test never waits on the result of
        // the MFMA issued just before it (at depth 1 the compiler pads every step with s_nop wait
        // states for that MFMA -> VALU dependency, and the matrix pipe idles meanwhile).  The C
        // operand (-threshold) is taken at issue: deeper means staler, which only lets more
        // candidates through to the exact re-score.
        constexpr int DEPTH = PCP_BF_DEPTH;
        constexpr int NS = kTile / 16;
        f32x4 cq[DEPTH][QB];  // cq[d]: the MFMA results of sub-tile s + 1 + d
        float bnext;          // B fragment of sub-tile s + DEPTH + 1, read from LDS a step ahead
        {
#pragma unroll
            for (int d = 0; d < DEPTH; d++) {
                const float bf = bfrag_at(d);
#pragma unroll
                for (int b = 0; b < QB; b++) cq[d][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(afrag[b], bf, nthr[b], 0, 0, 0);
            }
            bnext = bfrag_at(DEPTH);
        }
#pragma unroll kBfUnroll
        for (int sub = 0; sub < NS; sub++) {
            f32x4 c[QB];
#pragma unroll
            for (int b = 0; b < QB; b++) c[b] = cq[0][b];
#pragma unroll
            for (int d = 0; d + 1 < DEPTH; d++)
#pragma unroll
                for (int b = 0; b < QB; b++) cq[d][b] = cq[d + 1][b];
            if (sub + DEPTH < NS) {
                const float bfrag = bnext;
                if (sub + DEPTH + 1 < NS) bnext = bfrag_at(sub + DEPTH + 1);
#pragma unroll
                for (int b = 0; b < QB; b++)
                    cq[DEPTH - 1][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(afrag[b], bfrag, nthr[b], 0, 0, 0);
            }
            // one combined test per step; the insertion path runs only when a lane has a hit
            uint32_t sg = 0;
#pragma unroll
            for (int b = 0; b < QB; b++)
                sg |= __float_as_uint(c[b][0]) | __float_as_uint(c[b][1]) | __float_as_uint(c[b][2]) |
                      __float_as_uint(c[b][3]);
            if ((int32_t)sg < 0) {
                const int tidx = tb + sub * 16 + cls;
                const float* g = tf + sub * 64 + cls;
                const float4 p = make_float4(g[0], g[16], g[32], g[48]);
#pragma unroll
                for (int b = 0; b < QB; b++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        if ((int32_t)__float_as_uint(c[b][r]) >= 0) continue;
                        const float x = __fmaf_rn(qm[b][r][2], p.z, __fmaf_rn(qm[b][r][1], p.y,
                                                  __fmaf_rn(qm[b][r][0], p.x, p.w)));
                        if (x < thr[b][r]) {
                            list_insert<L>(ls[b][r], lt[b][r], x, tidx);
                            thr[b][r] = fminf(ls[b][r][L - 1], thr[b][r]);
                            nthr[b][r] = -thr[b][r];
                        }
                    }
            }
        }
        // refresh theta after tiles 1, 2, 4, 8, ... (rank of each class best in its group)
        if (use_theta && ((tt + 1) & tt) == 0) {
#pragma unroll
            for (int b = 0; b < QB; b++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const float v = ls[b][r][0];
                    int rank = 0;
#pragma unroll
                    for (int j = 0; j < 16; j++) {
                        const float vj = __shfl(v, (lane & ~15) | j, 64);
                        rank += (vj < v || (vj == v && j < cls)) ? 1 : 0;
                    }
                    float cand = rank == a.kk - 1 ? v : INFINITY;
#pragma unroll
                    for (int o = 1; o < 16; o <<= 1) cand = fminf(cand, __shfl_xor(cand, o, 64));
                    const float t2 = cand + 2.f * ew;
                    if (cand != INFINITY) thr[b][r] = fminf(thr[b][r], t2 + fabsf(t2) * 1e-6f);
                    nthr[b][r] = -thr[b][r];
                }
        }
    }

    // ---- exact fp64 re-rank + certification, row by row
#pragma unroll
    for (int b = 0; b < QB; b++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int64_t qi = qbase + b * 16 + grp * 4 + r;  // C row = 4*(lane>>4) + r
            const bool qok = qi < a.nq;
            double qx = 0, qy = 0, qz = 0;
            if (qok) {
                const double* qp = dptr(a.q, a.qstride, qi);
                qx = qp[0]; qy = qp[1]; qz = qp[2];
            }
            const bool qfin = qok && finite3(qx, qy, qz);
            double d[L];
            int j[L];
#pragma unroll
            for (int i = 0; i < L; i++) {
                j[i] = lt[b][r][i];
                d[i] = INFINITY;
                if (qfin && j[i] >= 0) {
                    const double* p = dptr(a.t, a.tstride, j[i]);
                    d[i] = l2_simple(qx, qy, qz, make_double4(p[0], p[1], p[2], 0.0));
                } else {
                    j[i] = INT_MAX;
                }
            }
            // sort the lane's list by (d, j)
#pragma unroll
            for (int x = 1; x < L; x++)
#pragma unroll
                for (int y = x; y > 0; y--)
                    if (lex_less(d[y], j[y], d[y - 1], j[y - 1])) {
                        const double td = d[y]; d[y] = d[y - 1]; d[y - 1] = td;
                        const int tj = j[y]; j[y] = j[y - 1]; j[y - 1] = tj;
                    }
            // tau: smallest L-th score over the 16 classes (inf if a class list is short)
            float tau = ls[b][r][L - 1];
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) tau = fminf(tau, __shfl_xor(tau, o, 64));
            double kth = INFINITY;
            for (int rr = 0; rr < a.kk; rr++) {
                double md = d[0];
                int mj = j[0];
                group_min(md, mj);
                if (j[0] == mj && mj != INT_MAX) {  // this lane owned the head: pop it
#pragma unroll
                    for (int i = 0; i < L - 1; i++) { d[i] = d[i + 1]; j[i] = j[i + 1]; }
                    d[L - 1] = INFINITY;
                    j[L - 1] = INT_MAX;
                }
                if (qok && cls == 0) {
                    a.oidx[qi * a.k + rr] = mj == INT_MAX ? -1 : mj;
                    a.od2[qi * a.k + rr] = mj == INT_MAX ? INFINITY : md;
                }
                kth = md;
            }
            if (qok && cls == 0) {
                for (int rr = a.kk; rr < a.k; rr++) {
                    a.oidx[qi * a.k + rr] = -1;
                    a.od2[qi * a.k + rr] = INFINITY;
                }
                if (qfin && a.kk > 0) {
                    const double qn = sqrt(qx * qx + qy * qy + qz * qz);
                    const double e = a.E2 * (a.pmax + qn) * (a.pmax + qn);
                    const double lb = (qx * qx + qy * qy + qz * qz) + (double)tau - e;
                    if (!(kth < lb)) a.fb[atomicAdd(a.fb_count, 1u)] = (int32_t)qi;
                }
            }
        }
}

// exact fp64 scan for uncertified queries: one 256-thread block per query, per-lane
// register top-k, then a block merge (k rounds: wave minimum, then across the 4 waves)
template <int K>
__global__ __launch_bounds__(256) void k_bf_fallback(BfArgs a, const int32_t* fb, const uint32_t* fb_count) {
    __shared__ double sd[4];
    __shared__ int sj[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t nfb = *fb_count;
    for (uint32_t w = blockIdx.x; w < nfb; w += gridDim.x) {
        const int64_t qi = fb[w];
        const double* qp = dptr(a.q, a.qstride, qi);
        const double qx = qp[0], qy = qp[1], qz = qp[2];
        TopK<K> top;
        top.init(a.kk);
        for (int64_t t = threadIdx.x; t < a.nt; t += 256) {
            const double* p = dptr(a.t, a.tstride, t);
            if (!finite3(p[0], p[1], p[2])) continue;
            top.push(l2_simple(qx, qy, qz, make_double4(p[0], p[1], p[2], 0.0)), (int)t);
        }
        top.normalize(a.kk);
        for (int rr = 0; rr < a.kk; rr++) {
            double md = top.best_d();
            int mj = top.best_j();
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const double od = __shfl_xor(md, o, 64);
                const int oj = __shfl_xor(mj, o, 64);
                if (lex_less(od, oj, md, mj)) { md = od; mj = oj; }
            }
            if (lane == 0) { sd[wid] = md; sj[wid] = mj; }
            __syncthreads();
            md = sd[0];
            mj = sj[0];
#pragma unroll
            for (int v = 1; v < 4; v++)
                if (lex_less(sd[v], sj[v], md, mj)) { md = sd[v]; mj = sj[v]; }
            __syncthreads();
            if (top.best_j() == mj && mj != INT_MAX) top.pop_best();
            if (threadIdx.x == 0) {
                a.oidx[qi * a.k + rr] = mj == INT_MAX ? -1 : mj;
                a.od2[qi * a.k + rr] = mj == INT_MAX ? INFINITY : md;
            }
        }
    }
}

}  // namespace
}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_knn_bruteforce(pcp_ctx* ctx, const double* t, size_t tstride, int64_t nt, const double* q, size_t qstride,
                       int64_t nq, int k, int32_t* oidx, double* od2) {
    if (!ctx || nt < 0 || nq < 0 || k <= 0 || (nt > 0 && !t) || (nq > 0 && (!q || !oidx || !od2)))
        return set_error(ctx, PCP_ERR_ARG, "pcp_knn_bruteforce: bad arguments");
    if (k > 32) return set_error(ctx, PCP_ERR_UNSUPPORTED, "pcp_knn_bruteforce: k=%d > 32 not supported yet", k);
    if (nt >= ((int64_t)1 << 31)) return set_error(ctx, PCP_ERR_ARG, "pcp_knn_bruteforce: < 2^31 targets");
    if (tstride == 0) tstride = 3 * sizeof(double);
    if (qstride == 0) qstride = 3 * sizeof(double);
    ctx->bf_fallback = 0;
    if (nq == 0) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    float* t4 = nullptr;
    double* part = nullptr;
    int32_t* fb = nullptr;
    uint32_t* fbc = nullptr;
    const unsigned npb = grid_for(nt > 0 ? nt : 1, 256, 1024);
    const int64_t ntpad = std::max<int64_t>((nt + kTile - 1) / kTile * kTile, 1);  // whole tiles (LDS-DMA)
    int rc = dmalloc(ctx, &t4, 4 * (size_t)ntpad);
    if (!rc) rc = dmalloc(ctx, &part, 2 * (size_t)npb);
    if (!rc) rc = dmalloc(ctx, &fb, nq);
    if (!rc) rc = dmalloc(ctx, &fbc, 1);
    double pmax2 = 0.0, nfin = 0.0;
    if (!rc && nt > 0) {
        hipLaunchKernelGGL(k_bf_targets, dim3(npb), dim3(256), 0, st, t, tstride, nt, t4, part);
        if (ntpad > nt)
            hipLaunchKernelGGL(k_bf_pad, dim3(1), dim3(256), 0, st, t4, nt, ntpad);
        std::vector<double> h(2 * npb);
        hipError_t e = hipMemcpyAsync(h.data(), part, h.size() * sizeof(double), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = hip_fail(ctx, e, "bf targets", __FILE__, __LINE__);
        for (unsigned b = 0; b < npb; b++) { pmax2 = std::fmax(pmax2, h[2 * b]); nfin += h[2 * b + 1]; }
    }
    if (!rc) {
        BfArgs a;
        a.t4 = t4; a.t = t; a.tstride = tstride; a.nt = nt;
        a.q = q; a.qstride = qstride; a.nq = nq;
        a.k = k;
        a.kk = (int)std::min<double>((double)k, nfin);
        // 32 unit roundoffs of (|p| + |q|)^2: casts to fp32, |p|^2 in fp32 and the 4-term
        // fma chain each contribute a few
        // (and 8 more for the threshold subtraction inside the filter's MFMA)
        a.E2 = 40.0 * std::ldexp(1.0, -24);
        a.pmax = std::sqrt(pmax2);
        a.oidx = oidx; a.od2 = od2; a.fb = fb; a.fb_count = fbc;
        if (hipMemsetAsync(fbc, 0, sizeof(uint32_t), st) != hipSuccess) rc = set_error(ctx, PCP_ERR_HIP, "memset");
        if (!rc) {
            if (k <= 8) {
                const int64_t per = kWaves * 16 * PCP_BF_QB8;
                hipLaunchKernelGGL((k_bf_mfma<PCP_BF_L8, PCP_BF_QB8, PCP_BF_W8>), dim3((unsigned)((nq + per - 1) / per)),
                                   dim3(kBlock), 0, st, a);
            } else if (k <= 16) {
                const int64_t per = kWaves * 16;
                hipLaunchKernelGGL((k_bf_mfma<10, 1, 3>), dim3((unsigned)((nq + per - 1) / per)), dim3(kBlock), 0, st, a);
            } else {
                const int64_t per = kWaves * 16;
                hipLaunchKernelGGL((k_bf_mfma<16, 1, 2>), dim3((unsigned)((nq + per - 1) / per)), dim3(kBlock), 0, st, a);
            }
            const unsigned fbg = 1024;
            if (k <= 8) hipLaunchKernelGGL(k_bf_fallback<8>, dim3(fbg), dim3(256), 0, st, a, fb, fbc);
            else if (k <= 16) hipLaunchKernelGGL(k_bf_fallback<16>, dim3(fbg), dim3(256), 0, st, a, fb, fbc);
            else hipLaunchKernelGGL(k_bf_fallback<32>, dim3(fbg), dim3(256), 0, st, a, fb, fbc);
            hipError_t e = hipGetLastError();
            if (e == hipSuccess) e = hipMemcpyAsync(&ctx->bf_fallback, fbc, sizeof(uint32_t), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) rc = hip_fail(ctx, e, "k_bf_mfma", __FILE__, __LINE__);
        }
    }
    dfree(ctx, t4);
    dfree(ctx, part);
    dfree(ctx, fb);
    dfree(ctx, fbc);
    return rc;
}

int pcp_knn_bruteforce_last_fallback(const pcp_ctx* ctx, int64_t* n) {
    if (!ctx || !n) return PCP_ERR_ARG;
    *n = ctx->bf_fallback;
    return PCP_OK;
}

}  // extern "C"
