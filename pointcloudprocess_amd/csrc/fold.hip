// compute3DCentroid's sequential left fold, bit-exact, evaluated in parallel.
//
// The reference sums a cloud as  s = ((0 + x_0) + x_1) + ... + x_{n-1}  in fp64, one point after
// the other (point_cloud_helper.h:193-230; get_rot_icp folds src then temp, :78-83).  A tree sum
// is not bit-identical to that, and remove_duplicate's voxel bins and output coordinates depend
// on the centroid's last bit (point_cloud_helper.cpp:42-63).  A single lane folding 100M points
// takes ~0.2 s, so the fold is evaluated as a scan over chunk transfer maps instead:
//
// * Within one binade: if every partial sum of a chunk stays in [2^e + u, 2^(e+1) - u] (u =
//   2^(e-52), one sign), each add is  RN(s + x) = s + u * d  with d = x/u rounded to an
//   integer, ties to the d that makes (s/u + d) even.  d depends on s only through the parity
//   of s/u, so a chunk's effect is a map  parity -> (total D, lowest/highest partial D)  for the
//   two parities: 2-state automata that compose associatively (one wave scan per chunk).
// * The binade e of a chunk is predicted from an approximate prefix of chunk sums.
// * A one-wave pass then walks the chunks in order, carrying the exact s: a chunk whose map
//   was built for s's binade and whose partials provably stay inside it advances s by u*D;
//   any other chunk (the first one, sums near 0, binade crossings, non-finite values) is
//   folded point by point from s.  Every step is exact, so the result equals the sequential
//   fold bit for bit, whatever the data.
//
// Only +0/-0 subtlety: a skipped (non-finite, !is_dense) point contributes -0.0, the additive
// identity of RN arithmetic (s + -0.0 == s for s = +0.0 too).
#include <cmath>
#include <cstring>

#include "common.hpp"

namespace pcp {
namespace {

constexpr int kChunk = 2048;  // points per chunk: one wave, 32 sub-tiles of 64
constexpr int kSub = kChunk / 64;

struct FoldSrc {
    const char* p0;  // AoS48 records: x, y, z doubles at byte 0/8/16
    int64_t n0;
    const char* p1;  // optional second segment (get_rot_icp: cloud_all = src ++ temp)
    int64_t n1;
    int is_dense;
};

// transfer map of one chunk and one coordinate (built for binade e and sign of the predicted s)
struct alignas(64) FoldMap {
    double d[2];   // total advance (units of u) for start parity 0 / 1
    double lo[2];  // lowest partial advance (incl. 0) for start parity 0 / 1
    double hi[2];  // highest partial advance (incl. 0)
    int be;        // biased exponent of the binade; 0 = no map (chunk is folded point by point)
    int neg;
};
static_assert(sizeof(FoldMap) == 64, "one 64-byte record per chunk and coordinate");

__device__ __forceinline__ bool load_xyz(const FoldSrc& s, int64_t i, double v[3]) {
    const char* p = i < s.n0 ? s.p0 + (size_t)i * 48 : s.p1 + (size_t)(i - s.n0) * 48;
    const double2 xy = *(const double2*)p;
    v[0] = xy.x; v[1] = xy.y; v[2] = *(const double*)(p + 16);
    return s.is_dense || (isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2]));
}

__device__ __forceinline__ double pow2(int be) { return __longlong_as_double((long long)be << 52); }
// parity of an integer-valued double of magnitude < 2^53
__device__ __forceinline__ int par(double v) { return v != 2.0 * floor(0.5 * v) ? 1 : 0; }

// element map: d_p = x/u rounded to nearest, ties to (p + d) even; q = x/u exactly
struct Map2 {
    double a, b;  // advance for start parity 0, 1
};
__device__ __forceinline__ Map2 elem_map(double q) {
    if (!(fabs(q) < 4503599627370496.0)) return {q, q};  // |q| >= 2^52: q is an integer
    const double m = floor(q), h = m + 0.5;                 // both exact
    if (q > h) return {m + 1.0, m + 1.0};
    if (q < h) return {m, m};
    const int pm = par(m);  // tie: d = m if (p + m) even, else m + 1
    return {pm == 0 ? m : m + 1.0, pm == 1 ? m : m + 1.0};
}
// A then B
__device__ __forceinline__ Map2 compose(Map2 A, Map2 B) {
    const double b0 = par(A.a) ? B.b : B.a;        // start parity 0: after A, parity = par(A.a)
    const double b1 = par(A.b) ? B.a : B.b;        // start parity 1: parity = 1 ^ par(A.b)
    return {A.a + b0, A.b + b1};
}

// pass 1: approximate per-chunk sums (binade prediction only) and exact finite counts
__global__ __launch_bounds__(256) void k_fold_sums(FoldSrc s, int64_t nchunks, double4* sums) {
    const int64_t c = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= nchunks) return;
    const int64_t n = s.n0 + s.n1;
    double a0 = 0, a1 = 0, a2 = 0, cnt = 0;
    for (int j = 0; j < kSub; j++) {
        const int64_t i = c * kChunk + j * 64 + lane;
        if (i >= n) break;
        double v[3];
        if (load_xyz(s, i, v)) { a0 += v[0]; a1 += v[1]; a2 += v[2]; cnt += 1.0; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        a0 += __shfl_xor(a0, o, 64); a1 += __shfl_xor(a1, o, 64);
        a2 += __shfl_xor(a2, o, 64); cnt += __shfl_xor(cnt, o, 64);
    }
    if (lane == 0) sums[c] = make_double4(a0, a1, a2, cnt);
}

// pass 2 (one block): exclusive prefix of the approximate sums -> predicted s at each chunk start
constexpr int kPfxThreads = 1024;
__global__ __launch_bounds__(kPfxThreads) void k_fold_prefix(const double4* sums, int64_t nchunks, double4* est) {
    __shared__ double sh[3][kPfxThreads];
    const int t = threadIdx.x;
    const int64_t per = (nchunks + kPfxThreads - 1) / kPfxThreads;
    const int64_t b = t * per, e = min(nchunks, b + per);
    double l0 = 0, l1 = 0, l2 = 0;
    for (int64_t c = b; c < e; c++) { l0 += sums[c].x; l1 += sums[c].y; l2 += sums[c].z; }
    sh[0][t] = l0; sh[1][t] = l1; sh[2][t] = l2;
    __syncthreads();
    for (int o = 1; o < kPfxThreads; o <<= 1) {
        double v0 = 0, v1 = 0, v2 = 0;
        if (t >= o) { v0 = sh[0][t - o]; v1 = sh[1][t - o]; v2 = sh[2][t - o]; }
        __syncthreads();
        sh[0][t] += v0; sh[1][t] += v1; sh[2][t] += v2;
        __syncthreads();
    }
    double r0 = sh[0][t] - l0, r1 = sh[1][t] - l1, r2 = sh[2][t] - l2;  // exclusive (approximate)
    for (int64_t c = b; c < e; c++) {
        est[c] = make_double4(r0, r1, r2, 0.0);
        r0 += sums[c].x; r1 += sums[c].y; r2 += sums[c].z;
    }
}

// pass 3: one wave per chunk builds the chunk's transfer map per coordinate (wave scan of the
// element automata, carried across the 32 sub-tiles)
__global__ __launch_bounds__(256) void k_fold_maps(FoldSrc s, int64_t nchunks, const double4* est, FoldMap* maps) {
    const int64_t c = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= nchunks) return;
    const int64_t n = s.n0 + s.n1;
    const double4 e4 = est[c];
    const double se[3] = {e4.x, e4.y, e4.z};
    int be[3];
    double scale[3], lim[3];
    bool ok[3];
    Map2 carry[3];
    double lo0[3], lo1[3], hi0[3], hi1[3];
#pragma unroll
    for (int a = 0; a < 3; a++) {
        be[a] = (int)((__double_as_longlong(se[a]) >> 52) & 0x7ff);
        ok[a] = be[a] >= 53 && be[a] < 0x7fe;  // u = 2^(e-52) normal, 2^(e+1) finite
        scale[a] = ok[a] ? pow2(1023 + 52 - (be[a] - 1023)) : 0.0;  // 1/u
        lim[a] = ok[a] ? pow2(be[a] + 1) : 0.0;                     // |x| < 2^(e+1)
        carry[a] = {0.0, 0.0};
        lo0[a] = lo1[a] = hi0[a] = hi1[a] = 0.0;
    }
    for (int j = 0; j < kSub; j++) {
        const int64_t i = c * kChunk + j * 64 + lane;
        double v[3] = {0.0, 0.0, 0.0};
        bool use = false;
        if (i < n) use = load_xyz(s, i, v);
#pragma unroll
        for (int a = 0; a < 3; a++) {
            if (use && !(fabs(v[a]) < lim[a])) ok[a] = false;  // also catches NaN/Inf (dense)
            Map2 m = use && ok[a] ? elem_map(v[a] * scale[a]) : Map2{0.0, 0.0};
            if (__all(m.a == m.b)) {
                // no half-ulp tie in this sub-tile (the common case): the advances do not
                // depend on the parity, so the automaton scan is a plain prefix sum
                double t = m.a;
                for (int o = 1; o < 64; o <<= 1) {
                    const double p = __shfl_up(t, o, 64);
                    if (lane >= o) t += p;
                }
                m = {t, t};
                const Map2 D{carry[a].a + t, carry[a].b + t};
                lo0[a] = fmin(lo0[a], D.a); hi0[a] = fmax(hi0[a], D.a);
                lo1[a] = fmin(lo1[a], D.b); hi1[a] = fmax(hi1[a], D.b);
                carry[a] = {__shfl(D.a, 63, 64), __shfl(D.b, 63, 64)};
                continue;
            }
            // inclusive wave scan of the automata (lane order = fold order)
            for (int o = 1; o < 64; o <<= 1) {
                Map2 p{__shfl_up(m.a, o, 64), __shfl_up(m.b, o, 64)};
                if (lane >= o) m = compose(p, m);
            }
            const Map2 D = compose(carry[a], m);  // advance after this lane's point
            lo0[a] = fmin(lo0[a], D.a); hi0[a] = fmax(hi0[a], D.a);
            lo1[a] = fmin(lo1[a], D.b); hi1[a] = fmax(hi1[a], D.b);
            carry[a] = {__shfl(D.a, 63, 64), __shfl(D.b, 63, 64)};
        }
    }
#pragma unroll
    for (int a = 0; a < 3; a++) {
        double l0 = lo0[a], l1 = lo1[a], h0 = hi0[a], h1 = hi1[a];
        for (int o = 32; o > 0; o >>= 1) {
            l0 = fmin(l0, __shfl_xor(l0, o, 64)); l1 = fmin(l1, __shfl_xor(l1, o, 64));
            h0 = fmax(h0, __shfl_xor(h0, o, 64)); h1 = fmax(h1, __shfl_xor(h1, o, 64));
        }
        const bool all_ok = __all(ok[a]);
        if (lane == 0) {
            FoldMap f;
            f.d[0] = carry[a].a; f.d[1] = carry[a].b;
            f.lo[0] = l0; f.lo[1] = l1; f.hi[0] = h0; f.hi[1] = h1;
            f.be = all_ok ? be[a] : 0;
            f.neg = se[a] < 0.0;
            maps[c * 3 + a] = f;
        }
    }
}

// pass 4 (one wave): the exact scan.  Lanes 0..2 carry s_x, s_y, s_z; lane 3 the finite count.
// The maps of 64 chunks at a time are staged in LDS (the next batch's loads are in flight in
// registers while this batch is walked), so the dependent chain per chunk is ~15 ALU ops.
constexpr int kBatch = 64;
__global__ __launch_bounds__(64) void k_fold_scan(FoldSrc s, int64_t nchunks, const FoldMap* maps,
                                                   const double4* sums, double* out) {
    __shared__ FoldMap smap[kBatch * 3];
    __shared__ double scount[kBatch];
    __shared__ double tile[3][64];
    __shared__ int fin[64];
    const int lane = threadIdx.x;
    const int64_t n = s.n0 + s.n1;
    double acc = 0.0;  // centroid.setZero() (point_cloud_helper.h:200)
    // register stage of one batch: 3 maps per lane-triple = 12 x 16 B per lane... as 3 x 64 B
    // records per lane (192 records / 64 lanes), plus one count per lane
    FoldMap r[3];
    double rc = 0.0;
    auto fetch = [&](int64_t c0) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const int64_t rec = c0 * 3 + k * 64 + lane;
            if (rec < nchunks * 3) r[k] = maps[rec];
        }
        rc = c0 + lane < nchunks ? sums[c0 + lane].w : 0.0;
    };
    if (nchunks > 0) fetch(0);
    for (int64_t c0 = 0; c0 < nchunks; c0 += kBatch) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 3; k++) smap[k * 64 + lane] = r[k];
        scount[lane] = rc;
        __syncthreads();
        if (c0 + kBatch < nchunks) fetch(c0 + kBatch);  // next batch in flight during this walk
        const int nb = (int)min((int64_t)kBatch, nchunks - c0);
        for (int b = 0; b < nb; b++) {
            const int64_t c = c0 + b;
            bool fb = false;
            if (lane < 3) {
                const FoldMap& m = smap[b * 3 + lane];
                const long long bits = __double_as_longlong(acc);
                const int be = (int)((bits >> 52) & 0x7ff);
                const bool neg = bits < 0;
                fb = true;
                if (m.be != 0 && be == m.be && neg == (bool)m.neg) {
                    const double u = pow2(be - 52), lo_b = pow2(be) + u, hi_b = pow2(be + 1) - u;
                    const int p = (int)(bits & 1);  // parity of s/u = last mantissa bit
                    // every partial s + D u (lo <= D <= hi) inside the binade, with a one-ulp
                    // margin so the exact sums (not only the rounded ones) are on the u-grid;
                    // out-of-range values cannot round back into range (the bounds are representable)
                    const double lo_v = acc + (p ? m.lo[1] : m.lo[0]) * u, hi_v = acc + (p ? m.hi[1] : m.hi[0]) * u;
                    if (neg ? (hi_v <= -lo_b && lo_v >= -hi_b) : (lo_v >= lo_b && hi_v <= hi_b)) {
                        acc = acc + (p ? m.d[1] : m.d[0]) * u;  // exact: stays on the binade's u-grid
                        fb = false;
                    }
                }
            } else if (lane == 3) {
                acc += scount[b];  // exact integer count
            }
            if (__any(fb)) {  // fold this chunk point by point from the exact s
                for (int j = 0; j < kSub; j++) {
                    const int64_t i = c * kChunk + j * 64 + lane;
                    double v[3] = {-0.0, -0.0, -0.0};
                    int f = 0;
                    if (i < n) f = load_xyz(s, i, v) ? 1 : 0;
                    __syncthreads();
                    tile[0][lane] = v[0]; tile[1][lane] = v[1]; tile[2][lane] = v[2];
                    fin[lane] = f;
                    __syncthreads();
                    if (fb) {
                        for (int k = 0; k < 64; k++) {
                            const double x = tile[lane][k];
                            acc = fin[k] ? acc + x : acc;
                        }
                    }
                }
            }
        }
    }
    if (lane < 4) out[lane] = acc;
}

}  // namespace

// Sequential fold of x/y/z over the records of seg0 ++ seg1 (skipping non-finite points when
// !is_dense): s_host[0..2] = the sums exactly as the reference's loop forms them, s_host[3] = the
// number of points summed.
int seqfold_aos48(pcp_ctx* ctx, const void* p0, int64_t n0, const void* p1, int64_t n1, int is_dense,
                  double s_host[4]) {
    for (int a = 0; a < 4; a++) s_host[a] = 0.0;
    const int64_t n = n0 + n1;
    if (n <= 0) return PCP_OK;
    const FoldSrc src{(const char*)p0, n0, (const char*)p1, n1, is_dense};
    const int64_t nchunks = (n + kChunk - 1) / kChunk;
    double4 *sums = nullptr, *est = nullptr;
    FoldMap* maps = nullptr;
    double* out = nullptr;
    int rc = dmalloc(ctx, &sums, nchunks);
    if (!rc) rc = dmalloc(ctx, &est, nchunks);
    if (!rc) rc = dmalloc(ctx, &maps, 3 * nchunks);
    if (!rc) rc = dmalloc(ctx, &out, 4);
    if (!rc) {
        hipStream_t st = ctx->stream;
        const unsigned nb = (unsigned)((nchunks + 3) / 4);
        hipLaunchKernelGGL(k_fold_sums, dim3(nb), dim3(256), 0, st, src, nchunks, sums);
        hipLaunchKernelGGL(k_fold_prefix, dim3(1), dim3(kPfxThreads), 0, st, sums, nchunks, est);
        hipLaunchKernelGGL(k_fold_maps, dim3(nb), dim3(256), 0, st, src, nchunks, est, maps);
        hipLaunchKernelGGL(k_fold_scan, dim3(1), dim3(64), 0, st, src, nchunks, maps, sums, out);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(s_host, out, 4 * sizeof(double), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = hip_fail(ctx, e, "sequential fold", __FILE__, __LINE__);
    }
    dfree(ctx, sums);
    dfree(ctx, est);
    dfree(ctx, maps);
    dfree(ctx, out);
    return rc;
}

}  // namespace pcp
