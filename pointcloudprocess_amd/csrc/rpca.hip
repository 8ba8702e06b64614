// F3: robust per-point normals, CalculateFeature::calculate_plan_parameter_rpca
// (calculate_feature.cpp:208-368) -- the normals entry the reference's pipeline calls
// (static.cpp:17).  Per point j over its kNN(20) neighbourhood (N points):
//   IterationNumber (34 at Pr 0.99, epi 0.5) draws of 3 distinct neighbours -> 3-point plane ->
//   distances of the N neighbours (float, extraction_tree.cpp:47-64) -> the h = floor(2N/3)
//   nearest (float coordinates, LAS_POINT_PROPERTY_sim) -> h-point PCA; the plane of smallest
//   lambda3 wins; MAD = 1.4826 * median |d - median d|; points with |d - median| / MAD < 2.5
//   (all when MAD == 0) -> final PCA if more than 3 remain, else {0, 0, 0, 0, curvature 1}.
// Deterministic by construction: the draws are a counter-based hash of (seed, j, iteration,
// slot) where the reference calls rand() after srand(time); sorts are stable (the reference's
// std::sort is not); min_value ties keep the earlier iteration.  oracle/pcp_oracle.c ora_rpca
// restates the same contract; results are bit-identical.
//
// GPU mapping: one wave per point.  The neighbourhood lives in LDS (double and float copies);
// lane i runs iteration i (3-point plane, distances, a 20-entry sorting network in registers,
// 13-point PCA with a 3x3 Jacobi eigen); a wave arg-min picks the plane; the median / MAD are
// rank counts over LDS; one lane sums the final PCA in neighbour order.
#include <cmath>

#include "pca.hpp"

namespace pcp {
namespace {

constexpr int kB = 256;
constexpr int kK = 20;  // the reference's nearestKSearch(searchPoint, 20, ...) (:233)

__device__ __forceinline__ uint32_t rpca_draw(uint64_t seed, uint32_t j, uint32_t it, uint32_t slot) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (((uint64_t)j << 32) | ((uint64_t)it << 2) | slot) +
                 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 32);
}

// extraction_tree.cpp:47-64 (float coordinates and coefficients, double sums)
__device__ __forceinline__ float plane_dist(float x1, float y1, float z1, float a, float b, float c, float d) {
    const float aa = a * a, bb = b * b, cc = c * c;
    const double g = (double)sqrtf((aa + bb) + cc);
    const double f1 = (double)(a * x1), f2 = (double)(b * y1), f3 = (double)(c * z1), f4 = (double)d;
    const double f = fabs(((f1 + f2) + f3) + f4);
    return (float)(f / g);
}

// h-point plane (calculate_plan_parameter_h_points) of points fetched by `at(t)`, t = 0..h-1
template <typename At>
__device__ __forceinline__ void plane_h(int h, At at, pcp_plane& out) {
    double xa = 0, ya = 0, za = 0;
    for (int t = 0; t < h; t++) {
        double p[3];
        at(t, p);
        xa += p[0]; ya += p[1]; za += p[2];
    }
    xa /= h; ya /= h; za /= h;
    double c00 = 0, c01 = 0, c02 = 0, c11 = 0, c12 = 0, c22 = 0;
    for (int t = 0; t < h; t++) {
        double p[3];
        at(t, p);
        const double x0 = p[0] - xa, x1 = p[1] - ya, x2 = p[2] - za;
        c00 += x0 * x0; c01 += x0 * x1; c02 += x0 * x2;
        c11 += x1 * x1; c12 += x1 * x2; c22 += x2 * x2;
    }
    const double C[9] = {c00, c01, c02, c01, c11, c12, c02, c12, c22};
    plane_from_cov(C, xa, ya, za, out);
}

struct alignas(8) RpcaOut {  // LAS_POINT_PROPERTY (data_struct.h:161-172)
    float nx, ny, nz;
    double distance, curvature;
    int32_t point_id, segment_id;
    float dis;
};
static_assert(sizeof(RpcaOut) == sizeof(pcp_point_property), "LAS_POINT_PROPERTY layout");

__global__ __launch_bounds__(kB) void k_rpca(const double* xyz, size_t stride_d, int64_t n, const int32_t* knn,
                                             int k, int iters, uint64_t seed, RpcaOut* out) {
    constexpr int kW = kB / 64;
    __shared__ double sP[kW][kK][3];
    __shared__ float sF[kW][kK][3];
    __shared__ float sD[kW][kK];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t nwaves = (int64_t)gridDim.x * kW;
    for (int64_t j = (int64_t)blockIdx.x * kW + w; j < n; j += nwaves) {
        const int32_t nb = lane < k ? knn[j * k + lane] : -1;
        const uint64_t have = __ballot(lane < kK && nb >= 0);
        const int N = __popcll(have);  // rows are -1 padded after the found neighbours
        if (lane < N) {
            const double* p = xyz + (size_t)nb * stride_d;
            for (int a = 0; a < 3; a++) {
                sP[w][lane][a] = p[a];
                sF[w][lane][a] = (float)p[a];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        RpcaOut o{0.f, 0.f, 0.f, 0.0, 1.0, (int32_t)j, 0, 0.f};
        if (N > 3) {
            const int hf = (int)(2.0 / 3 * N);  // :238-239
            // ---- iterations (:244-282): lane it (+ 64 r), best plane per lane
            float bmin = INFINITY;
            int bit = INT_MAX;
            pcp_plane bpl{0.f, 0.f, 0.f, 0.f, 1.f, 0.f};
            for (int it = lane; it < iters; it += 64) {
                int num[3];
#pragma unroll
                for (int s = 0; s < 3; s++) num[s] = (int)(rpca_draw(seed, (uint32_t)j, (uint32_t)it, (uint32_t)s) % (uint32_t)N);
                if (num[0] == num[1] || num[0] == num[2] || num[1] == num[2]) continue;
                pcp_plane p3;
                plane_h(3, [&](int t, double p[3]) {
                    const int m = t == 0 ? num[0] : (t == 1 ? num[1] : num[2]);
                    p[0] = sP[w][m][0]; p[1] = sP[w][m][1]; p[2] = sP[w][m][2];
                }, p3);
                // distances + stable sort of (d, m): an insertion network over kK registers
                float d[kK];
                int id[kK];
#pragma unroll
                for (int m = 0; m < kK; m++) {
                    d[m] = m < N ? plane_dist(sF[w][m][0], sF[w][m][1], sF[w][m][2], p3.normal_x, p3.normal_y,
                                              p3.normal_z, p3.distance)
                                 : INFINITY;
                    id[m] = m;
                }
#pragma unroll
                for (int a = 1; a < kK; a++)
#pragma unroll
                    for (int b = a; b > 0; b--) {
                        const bool sw = d[b - 1] > d[b];  // strict: equal keys keep their order
                        const float lo = sw ? d[b] : d[b - 1], hi = sw ? d[b - 1] : d[b];
                        const int il = sw ? id[b] : id[b - 1], ih = sw ? id[b - 1] : id[b];
                        d[b - 1] = lo; d[b] = hi; id[b - 1] = il; id[b] = ih;
                    }
                pcp_plane ph;
                plane_h(hf, [&](int t, double p[3]) {
                    int m = id[0];
#pragma unroll
                    for (int u = 1; u < kK; u++) m = t == u ? id[u] : m;
                    p[0] = (double)sF[w][m][0]; p[1] = (double)sF[w][m][1]; p[2] = (double)sF[w][m][2];
                }, ph);
                if (ph.min_value < bmin || (ph.min_value == bmin && it < bit)) {
                    bmin = ph.min_value;
                    bit = it;
                    bpl = ph;
                }
            }
            // ---- the plane of smallest min_value, earliest iteration on ties (:283-286)
            float vm = bmin;
            int vi = bit;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const float om = __shfl_xor(vm, off, 64);
                const int oi = __shfl_xor(vi, off, 64);
                if (om < vm || (om == vm && oi < vi)) { vm = om; vi = oi; }
            }
            if (vi != INT_MAX) {
                const int src = vi & 63;  // iteration vi ran on lane vi % 64
                const float fnx = __shfl(bpl.normal_x, src, 64), fny = __shfl(bpl.normal_y, src, 64);
                const float fnz = __shfl(bpl.normal_z, src, 64), fd = __shfl(bpl.distance, src, 64);
                // ---- median and MAD of the distances to that plane (:287-312)
                float dm = 0.f;
                if (lane < N) {
                    dm = plane_dist(sF[w][lane][0], sF[w][lane][1], sF[w][lane][2], fnx, fny, fnz, fd);
                    sD[w][lane] = dm;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                auto kth = [&](float v) {  // is this lane's value the (N/2)-th smallest?
                    int less = 0, le = 0;
                    for (int m = 0; m < N; m++) {
                        const float x = sD[w][m];
                        less += x < v;
                        le += x <= v;
                    }
                    return lane < N && less <= N / 2 && N / 2 < le;
                };
                const uint64_t mk = __ballot(kth(dm));
                const float med = __shfl(dm, __ffsll((unsigned long long)mk) - 1, 64);
                const float tm = fabsf(dm - med);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();  // every lane has read the distances
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (lane < N) sD[w][lane] = tm;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint64_t mt = __ballot(kth(tm));
                const float mad = (float)(1.4826 * (double)__shfl(tm, __ffsll((unsigned long long)mt) - 1, 64));
                // ---- inliers in neighbour order (:313-334) and the final PCA (:337-351)
                const bool keep = lane < N && (mad == 0.0f || (double)(tm / mad) < 2.5);
                const uint64_t km = __ballot(keep);
                const int cnt = __popcll(km);
                if (cnt > 3 && lane == 0) {
                    pcp_plane f;
                    plane_h(cnt, [&](int t, double p[3]) {
                        uint64_t m = km;  // the t-th set bit of km
                        for (int u = 0; u < t; u++) m &= m - 1;
                        const int r = __ffsll((unsigned long long)m) - 1;
                        p[0] = sP[w][r][0]; p[1] = sP[w][r][1]; p[2] = sP[w][r][2];
                    }, f);
                    o.nx = f.normal_x; o.ny = f.normal_y; o.nz = f.normal_z;
                    o.distance = (double)f.distance;
                    o.curvature = (double)f.curvature;
                }
            }
        }
        if (lane == 0) out[j] = o;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the next point overwrites the LDS rows
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

}  // namespace
}  // namespace pcp

extern "C" int pcp_normals_rpca(pcp_ctx* ctx, const double* xyz, size_t stride, int64_t n, const int32_t* knn_idx,
                                int k, float pr, float epi, uint64_t seed, pcp_point_property* out) {
    if (!ctx || n < 0 || (n > 0 && (!xyz || !knn_idx || !out)) || k <= 0)
        return pcp::set_error(ctx, PCP_ERR_ARG, "pcp_normals_rpca: bad arguments");
    if (k > pcp::kK) return pcp::set_error(ctx, PCP_ERR_UNSUPPORTED, "pcp_normals_rpca: k <= 20 (the reference's kNN(20))");
    if (stride == 0) stride = 3 * sizeof(double);
    if (stride % sizeof(double)) return pcp::set_error(ctx, PCP_ERR_ARG, "pcp_normals_rpca: stride must be whole doubles");
    if (n == 0) return PCP_OK;
    // compute_iteration_number (calculate_feature.cpp:28-33)
    const double num = (double)std::log10(1.0f - pr), den = std::log10(1.0 - std::pow((double)(1.0f - epi), 3));
    const double itf = num / den;
    if (!(itf >= 0.0 && itf < 65536.0)) return pcp::set_error(ctx, PCP_ERR_ARG, "pcp_normals_rpca: Pr/epi out of range");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    const unsigned nb = pcp::grid_for((n + 3) / 4, 1, 1 << 20);
    hipLaunchKernelGGL(pcp::k_rpca, dim3(nb), dim3(pcp::kB), 0, ctx->stream, xyz, stride / sizeof(double), n, knn_idx,
                       k, (int)itf, seed, (pcp::RpcaOut*)out);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}
