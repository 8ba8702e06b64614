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
#include <cstring>
#include <vector>

#include "grid.hpp"

struct pcp_icp {
    pcp_ctx* ctx = nullptr;
    const pcp_index* target = nullptr;
    int64_t nq = 0;
    float4* q = nullptr;          // sorted queries {x,y,z,bits(original index)}
    double* partials = nullptr;   // nblocks * 24
    double* acc = nullptr;        // 24 (scratch for pcp_icp_run)
    int nblocks = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0.0;
    int last_launches = 0;
};

namespace pcp {
namespace {

constexpr int kIcpBlock = 256;
constexpr int kAcc = 24;

struct IcpArgs {
    GridDesc g;
    const float4* tp;   // sorted target points
    const float4* q;    // sorted queries
    int64_t nq;
    float R[9], t[3];
    float r2;
    float mc;           // cell-unit margin for pruning
    double* partials;
    int32_t* corr_idx;  // optional, original query order
    float* corr_d2;
};

struct NN1 {
    const float4* pts;
    float qx, qy, qz;
    float bd;
    int bj;
    float px, py, pz;
    __device__ __forceinline__ float bound() const { return bd * 1.00002f + 1e-30f; }
    __device__ __forceinline__ void visit(uint32_t s, uint32_t e) {
        for (uint32_t k = s; k < e; k++) {
            const float4 p = pts[k];
            const float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
            const float d2 = __fmaf_rn(dz, dz, __fmaf_rn(dy, dy, dx * dx));
            const int id = __float_as_int(p.w);
            if (d2 < bd || (d2 == bd && id < bj)) {
                bd = d2; bj = id; px = p.x; py = p.y; pz = p.z;
            }
        }
    }
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__global__ void __launch_bounds__(kIcpBlock) k_icp_step(IcpArgs a) {
    double acc[kAcc - 1];
#pragma unroll
    for (int k = 0; k < kAcc - 1; k++) acc[k] = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kIcpBlock;
    for (int64_t i = blockIdx.x * (int64_t)kIcpBlock + threadIdx.x; i < a.nq; i += stride) {
        const float4 q = a.q[i];
        // q' = R q + t: x' = fmaf(R02,z,fmaf(R01,y,fmaf(R00,x,t0)))
        const float qx = __fmaf_rn(a.R[2], q.z, __fmaf_rn(a.R[1], q.y, __fmaf_rn(a.R[0], q.x, a.t[0])));
        const float qy = __fmaf_rn(a.R[5], q.z, __fmaf_rn(a.R[4], q.y, __fmaf_rn(a.R[3], q.x, a.t[1])));
        const float qz = __fmaf_rn(a.R[8], q.z, __fmaf_rn(a.R[7], q.y, __fmaf_rn(a.R[6], q.x, a.t[2])));
        NN1 v{a.tp, qx, qy, qz, a.r2, 0x7fffffff, 0.f, 0.f, 0.f};
        ring_search<float>(a.g, qx, qy, qz, a.mc, v);
        const bool ok = v.bj != 0x7fffffff;
        if (a.corr_idx) {
            const int oq = __float_as_int(q.w);
            a.corr_idx[oq] = ok ? v.bj : -1;
            a.corr_d2[oq] = ok ? v.bd : INFINITY;
        }
        if (ok) {
            const double x0 = qx, x1 = qy, x2 = qz, p0 = v.px, p1 = v.py, p2 = v.pz;
            acc[0] += 1.0;
            acc[1] += x0; acc[2] += x1; acc[3] += x2;
            acc[4] += p0; acc[5] += p1; acc[6] += p2;
            acc[7] += x0 * p0; acc[8] += x0 * p1; acc[9] += x0 * p2;
            acc[10] += x1 * p0; acc[11] += x1 * p1; acc[12] += x1 * p2;
            acc[13] += x2 * p0; acc[14] += x2 * p1; acc[15] += x2 * p2;
            acc[16] += x0 * x0; acc[17] += x0 * x1; acc[18] += x0 * x2;
            acc[19] += x1 * x1; acc[20] += x1 * x2; acc[21] += x2 * x2;
            acc[22] += (double)v.bd;
        }
    }
    __shared__ double red[kIcpBlock / 64][kAcc];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < kAcc - 1; k++) {
        double s = wave_sum(acc[k]);
        if (lane == 0) red[wid][k] = s;
    }
    __syncthreads();
    if (threadIdx.x < kAcc) {
        double s = 0.0;
        if (threadIdx.x < kAcc - 1)
            for (int w = 0; w < kIcpBlock / 64; w++) s += red[w][threadIdx.x];
        a.partials[(int64_t)blockIdx.x * kAcc + threadIdx.x] = s;
    }
}

// fixed-order reduction of nb partial rows of 24 doubles -> out[24]
__global__ void __launch_bounds__(256) k_reduce_partials(const double* part, int nb, double* out) {
    __shared__ double s[256];
    for (int k = 0; k < kAcc; k++) {
        double v = 0.0;
        for (int b = threadIdx.x; b < nb; b += 256) v += part[(int64_t)b * kAcc + k];
        s[threadIdx.x] = v;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) out[k] = s[0];
        __syncthreads();
    }
}

__global__ void k_fill_corr(int32_t* idx, float* d2, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        idx[i] = -1;
        d2[i] = INFINITY;
    }
}

// ------------------------------------------------------------------ host 3x3 solve
// One-sided Jacobi SVD of a 3x3 matrix: A = U diag(s) V^T (columns of U, V).
void svd3(const double Ain[9], double U[9], double s[3], double V[9]) {
    double A[9];
    std::memcpy(A, Ain, sizeof(A));
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
                if (ga == 0.0 || std::fabs(ga) <= 1e-300) continue;
                double conv = std::fabs(ga) / std::sqrt(al * be);
                if (!(conv > 1e-15)) continue;
                off = std::fmax(off, conv);
                double zeta = (be - al) / (2.0 * ga);
                double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                double c = 1.0 / std::sqrt(1.0 + t * t), sn = c * t;
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
        s[c] = std::sqrt(n);
    }
    // order singular values descending (permute U/V columns consistently)
    int ord[3] = {0, 1, 2};
    for (int i = 0; i < 3; i++)
        for (int j = i + 1; j < 3; j++)
            if (s[ord[j]] > s[ord[i]]) std::swap(ord[i], ord[j]);
    double A2[9], V2[9], s2[3];
    for (int c = 0; c < 3; c++) {
        s2[c] = s[ord[c]];
        for (int r = 0; r < 3; r++) { A2[3 * r + c] = A[3 * r + ord[c]]; V2[3 * r + c] = V[3 * r + ord[c]]; }
    }
    std::memcpy(V, V2, sizeof(V2));
    for (int c = 0; c < 3; c++) s[c] = s2[c];
    const double tiny = 1e-14 * (s[0] > 0 ? s[0] : 1.0);
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) U[3 * r + c] = s[c] > tiny ? A2[3 * r + c] / s[c] : 0.0;
    // complete a rank-deficient basis: u2 = u0 x u1 (planar clouds have rank 2)
    if (!(s[2] > tiny)) {
        double u0[3] = {U[0], U[3], U[6]}, u1[3] = {U[1], U[4], U[7]};
        if (!(s[1] > tiny)) {  // rank 1: any unit vector orthogonal to u0
            double a[3] = {std::fabs(u0[0]) < 0.9 ? 1.0 : 0.0, std::fabs(u0[0]) < 0.9 ? 0.0 : 1.0, 0.0};
            double d = a[0] * u0[0] + a[1] * u0[1] + a[2] * u0[2];
            for (int r = 0; r < 3; r++) u1[r] = a[r] - d * u0[r];
            double nn = std::sqrt(u1[0] * u1[0] + u1[1] * u1[1] + u1[2] * u1[2]);
            for (int r = 0; r < 3; r++) { u1[r] /= nn; U[3 * r + 1] = u1[r]; }
        }
        double u2[3] = {u0[1] * u1[2] - u0[2] * u1[1], u0[2] * u1[0] - u0[0] * u1[2], u0[0] * u1[1] - u0[1] * u1[0]};
        for (int r = 0; r < 3; r++) U[3 * r + 2] = u2[r];
    }
}

double det3(const double M[9]) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

}  // namespace

int icp_launch(pcp_icp* icp, const double T[16], float rmax, double* acc_dev, int32_t* corr_idx,
               float* corr_d2) {
    pcp_ctx* ctx = icp->ctx;
    const pcp_index* tg = icp->target;
    IcpArgs a;
    a.g = tg->g;
    a.tp = (const float4*)tg->pts;
    a.q = icp->q;
    a.nq = icp->nq;
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) a.R[3 * r + c] = (float)T[4 * r + c];
        a.t[r] = (float)T[4 * r + 3];
    }
    a.r2 = rmax * rmax;
    const int nmax = std::max(a.g.n[0], std::max(a.g.n[1], a.g.n[2]));
    a.mc = 1e-5f + 8e-7f * (float)nmax;  // >> fp32 rounding of the cell coordinates
    a.partials = icp->partials;
    a.corr_idx = corr_idx;
    a.corr_d2 = corr_d2;
    if (corr_idx && icp->nq > 0)
        hipLaunchKernelGGL(k_fill_corr, dim3(grid_for(icp->nq, 256)), dim3(256), 0, ctx->stream, corr_idx,
                           corr_d2, icp->nq);
    PCP_HIP(ctx, hipEventRecord(icp->ev0, ctx->stream));
    hipLaunchKernelGGL(k_icp_step, dim3(icp->nblocks), dim3(kIcpBlock), 0, ctx->stream, a);
    PCP_HIP(ctx, hipEventRecord(icp->ev1, ctx->stream));
    hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(256), 0, ctx->stream, icp->partials, icp->nblocks,
                       acc_dev);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int icp_solve(const double acc[24], int do_scale, double dT[16]) {
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
    // spatially sort the query set once (same grid machinery), keep its sorted points
    pcp_index* qi = nullptr;
    PCP_TRY(pcp_index_build_f32(ctx, q, q_stride, nq, target->g.h, &qi));
    pcp_icp* icp = new pcp_icp();
    icp->ctx = ctx;
    icp->target = target;
    icp->nq = qi->n;
    icp->q = (float4*)qi->pts;
    qi->pts = nullptr;
    pcp_index_destroy(qi);
    int dev_cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, ctx->device) == hipSuccess && prop.multiProcessorCount > 0)
        dev_cus = prop.multiProcessorCount;
    const int64_t want = (icp->nq + pcp::kIcpBlock - 1) / pcp::kIcpBlock;
    icp->nblocks = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)dev_cus * 8));
    int rc = pcp::dmalloc(ctx, &icp->partials, (size_t)icp->nblocks * pcp::kAcc);
    if (!rc) rc = pcp::dmalloc(ctx, &icp->acc, pcp::kAcc);
    if (!rc && (hipEventCreate(&icp->ev0) != hipSuccess || hipEventCreate(&icp->ev1) != hipSuccess))
        rc = pcp::set_error(ctx, PCP_ERR_HIP, "hipEventCreate failed");
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
    hipFree(icp->q);
    hipFree(icp->partials);
    hipFree(icp->acc);
    if (icp->ev0) hipEventDestroy(icp->ev0);
    if (icp->ev1) hipEventDestroy(icp->ev1);
    delete icp;
    return PCP_OK;
}

int pcp_icp_step(pcp_ctx* ctx, pcp_icp* icp, const double T[16], float rmax, double* acc_dev,
                 int32_t* corr_idx, float* corr_d2) {
    if (!ctx || !icp || !T || !acc_dev || (corr_idx && !corr_d2) || !(rmax >= 0.f)) return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    icp->ctx = ctx;
    PCP_TRY(pcp::icp_launch(icp, T, rmax, acc_dev, corr_idx, corr_d2));
    PCP_HIP(ctx, hipEventSynchronize(icp->ev1));
    float ms = 0.f;
    PCP_HIP(ctx, hipEventElapsedTime(&ms, icp->ev0, icp->ev1));
    icp->last_ms = ms;
    icp->last_launches = 1;
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

int pcp_icp_last_kernel_ms(const pcp_icp* icp, double* ms, int* launches) {
    if (!icp) return PCP_ERR_ARG;
    if (ms) *ms = icp->last_ms;
    if (launches) *launches = icp->last_launches;
    return PCP_OK;
}

}  // extern "C"
