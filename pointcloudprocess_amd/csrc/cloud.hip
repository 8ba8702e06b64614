// Cloud-level passes over AoS48 PointXYZRGBA clouds (point_type.h:9-82, 48-byte stride):
//   getMinMax3D       point_cloud_helper.h:59-90     (V2)
//   compute3DCentroid point_cloud_helper.h:193-230   (I3)
//   transformPointCloud point_cloud_helper.h:92-127  (I2)
//   VoxelGrid::applyFilter voxel_grid.h:811-1056     (V3)
//   remove_duplicate  point_cloud_helper.cpp:42-63   (V4)
//   get_rot_icp       point_cloud_helper.cpp:75-166  (I1, front-end of the ICP kernels)
//
// All passes stream the 48-byte records once (HBM-bound).  The voxel sort is rocPRIM's
// device radix sort (LSD, stable) on u32 voxel keys; keying, run detection and the
// per-voxel averaging are the kernels below.
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

#include "common.hpp"

namespace pcp {
namespace {

constexpr int kB = 256;
constexpr int kRedBlocks = 1024;

struct P48 {
    double x, y, z, w;
    uint32_t rgba, stamp_id, pad0, pad1;
};
static_assert(sizeof(P48) == PCP_AOS48_STRIDE, "AoS48 layout");

__device__ __forceinline__ double wave_min(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

// V2: per-block min/max of data[0..3] over (finite unless is_dense) points.  Eigen's
// min/max on a non-NaN running value are exact, so any reduction order gives the
// reference's result; max starts at DBL_MIN (point_cloud_helper.h:64-65).
__global__ __launch_bounds__(kB) void k_minmax48(const P48* in, int64_t n, int is_dense, double* part) {
    double mn[4] = {DBL_MAX, DBL_MAX, DBL_MAX, DBL_MAX}, mx[4] = {DBL_MIN, DBL_MIN, DBL_MIN, DBL_MIN};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const P48 p = in[i];
        if (!is_dense && !finite3(p.x, p.y, p.z)) continue;
        const double v[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
        for (int a = 0; a < 4; a++) {
            if (v[a] < mn[a]) mn[a] = v[a];
            if (mx[a] < v[a]) mx[a] = v[a];
        }
    }
    __shared__ double sm[kB / 64][8];
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
    for (int a = 0; a < 4; a++) {
        const double a0 = wave_min(mn[a]), a1 = wave_max(mx[a]);
        if (ln == 0) { sm[wv][a] = a0; sm[wv][4 + a] = a1; }
    }
    __syncthreads();
    if (threadIdx.x < 8) {
        double r = sm[0][threadIdx.x];
        for (int w = 1; w < kB / 64; w++) r = threadIdx.x < 4 ? fmin(r, sm[w][threadIdx.x]) : fmax(r, sm[w][threadIdx.x]);
        part[blockIdx.x * 8 + threadIdx.x] = r;
    }
}

// I2: p <- R p + t with Eigen's lazy product order ((r0 x + r1 y) + r2 z) + t.
struct Xf {
    double m[12];
};
__device__ __forceinline__ void xform(const Xf& T, double x, double y, double z, double o[3]) {
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double acc = T.m[4 * r + 0] * x;
        acc = acc + T.m[4 * r + 1] * y;
        acc = acc + T.m[4 * r + 2] * z;
        o[r] = acc + T.m[4 * r + 3];
    }
}

__global__ __launch_bounds__(kB) void k_transform48(const P48* in, P48* out, int64_t n, int is_dense, Xf T) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        P48 p = in[i];
        if (is_dense || finite3(p.x, p.y, p.z)) {
            double o[3];
            xform(T, p.x, p.y, p.z, o);
            p.x = o[0]; p.y = o[1]; p.z = o[2];
        }
        out[i] = p;
    }
}

// V4 step 1-2: copyPointCloud (registered fields only, data[3] = 1) fused with the
// centring transform (point_cloud_helper.cpp:46-53)
__global__ __launch_bounds__(kB) void k_copy_centre(const P48* in, P48* out, int64_t n, int is_dense, Xf T) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const P48 s = in[i];
        P48 p{s.x, s.y, s.z, 1.0, s.rgba, s.stamp_id, 0u, 0u};
        if (is_dense || finite3(p.x, p.y, p.z)) {
            double o[3];
            xform(T, p.x, p.y, p.z, o);
            p.x = o[0]; p.y = o[1]; p.z = o[2];
        }
        out[i] = p;
    }
}

// V3 keying (voxel_grid.h:928-943): ijk_a = (int)(double(p_a*inv_a) - min_b_a), linear index
// i + j*div_b0 + k*div_b0*div_b1 in wrapping int32 arithmetic, kept as u32.
struct VoxGeom {
    double inv[3];
    double min_b[3];
    uint32_t mul1, mul2;
};

__global__ __launch_bounds__(kB) void k_vox_flag(const P48* in, int64_t n, int is_dense, uint32_t* flag) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const P48 p = in[i];
        flag[i] = (is_dense || finite3(p.x, p.y, p.z)) ? 1u : 0u;
    }
}

__global__ __launch_bounds__(kB) void k_vox_key(const P48* in, int64_t n, int is_dense, VoxGeom g,
                                                const uint32_t* pos, uint32_t* keys, uint32_t* vals) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const P48 p = in[i];
        if (!is_dense && !finite3(p.x, p.y, p.z)) continue;
        const int i0 = (int)((p.x * g.inv[0]) - g.min_b[0]);
        const int i1 = (int)((p.y * g.inv[1]) - g.min_b[1]);
        const int i2 = (int)((p.z * g.inv[2]) - g.min_b[2]);
        const uint32_t idx = (uint32_t)i0 + (uint32_t)i1 * g.mul1 + (uint32_t)i2 * g.mul2;
        const uint32_t o = is_dense ? (uint32_t)i : pos[i];
        keys[o] = idx;
        vals[o] = (uint32_t)i;
    }
}

__global__ __launch_bounds__(kB) void k_run_heads(const uint32_t* keys, int64_t m, uint32_t* head) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

// head[] holds the exclusive scan of the run-head flags: run r starts at the i whose flag
// was set and whose scan value is r.
__global__ __launch_bounds__(kB) void k_run_starts(const uint32_t* keys, const uint32_t* headscan, int64_t m,
                                                   uint32_t* start) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        if (i == 0 || keys[i] != keys[i - 1]) start[headscan[i]] = (uint32_t)i;
}

// V3 averaging (voxel_grid.h:985-1054), one lane per voxel, members in input order
// (the stable restatement of the unstable std::sort).
__global__ __launch_bounds__(kB) void k_vox_reduce(const P48* in, const uint32_t* keys, const uint32_t* vals,
                                                   const uint32_t* start, int64_t nvox, int64_t m, int all_data,
                                                   P48* out, uint32_t* out_vidx) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nvox; v += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t s = start[v];
        const uint32_t e = v + 1 < nvox ? start[v + 1] : (uint32_t)m;
        P48 o{0, 0, 0, 1.0, 0u, 0u, 0u, 0u};
        const double dn = (double)(e - s);
        if (!all_data) {
            double c0 = 0, c1 = 0, c2 = 0;
            for (uint32_t t = s; t < e; t++) {
                const P48 p = in[vals[t]];
                c0 += p.x; c1 += p.y; c2 += p.z;
            }
            o.x = c0 / dn; o.y = c1 / dn; o.z = c2 / dn;
        } else {
            // x,y,z,rgba,stamp_id through static_cast<float> (concatenate.h:153), then the
            // r,g,b bytes (voxel_grid.h:995-1004); first member assigned, the rest added
            double c[8];
            for (uint32_t t = s; t < e; t++) {
                const P48 p = in[vals[t]];
                const double tv[8] = {(double)(float)p.x, (double)(float)p.y, (double)(float)p.z,
                                      (double)(float)p.rgba, (double)(float)p.stamp_id,
                                      (double)((p.rgba >> 16) & 0xFF), (double)((p.rgba >> 8) & 0xFF),
                                      (double)(p.rgba & 0xFF)};
                if (t == s) {
#pragma unroll
                    for (int f = 0; f < 8; f++) c[f] = tv[f];
                } else {
#pragma unroll
                    for (int f = 0; f < 8; f++) c[f] += tv[f];
                }
            }
#pragma unroll
            for (int f = 0; f < 8; f++) c[f] /= dn;  // :1034
            o.x = c[0]; o.y = c[1]; o.z = c[2];
            o.rgba = (uint32_t)c[3];
            o.stamp_id = (uint32_t)c[4];
            const float r = (float)c[5], gg = (float)c[6], b = (float)c[7];  // :1045-1050
            o.rgba = (uint32_t)(((int)r << 16) | ((int)gg << 8) | (int)b);
        }
        out[v] = o;
        if (out_vidx) out_vidx[v] = keys[s];
    }
}

// I1: float(p - c) vertices (point_cloud_helper.cpp:89-104)
__global__ __launch_bounds__(kB) void k_centre_f32(const P48* in, int64_t n, double c0, double c1, double c2, float* v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const P48 p = in[i];
        v[3 * i + 0] = (float)(p.x - c0);
        v[3 * i + 1] = (float)(p.y - c1);
        v[3 * i + 2] = (float)(p.z - c2);
    }
}

// device buffers of one voxel-filter call
struct VoxBufs {
    pcp_ctx* ctx;
    uint32_t* flag = nullptr;
    uint32_t* k0 = nullptr;
    uint32_t* k1 = nullptr;
    uint32_t* v0 = nullptr;
    uint32_t* v1 = nullptr;
    uint32_t* head = nullptr;
    void* tmp = nullptr;
    ~VoxBufs() {
        dfree(ctx, flag); dfree(ctx, k0); dfree(ctx, k1); dfree(ctx, v0); dfree(ctx, v1); dfree(ctx, head);
        dfree(ctx, tmp);
    }
};

}  // namespace

int minmax_aos48_dev(pcp_ctx* ctx, const void* in, int64_t n, int is_dense, double mn[4], double mx[4]) {
    for (int a = 0; a < 4; a++) { mn[a] = DBL_MAX; mx[a] = DBL_MIN; }
    if (n <= 0) return PCP_OK;
    const unsigned nb = grid_for(n, kB, kRedBlocks);
    double* part;
    PCP_TRY(dmalloc(ctx, &part, 8 * (size_t)nb));
    hipLaunchKernelGGL(k_minmax48, dim3(nb), dim3(kB), 0, ctx->stream, (const P48*)in, n, is_dense, part);
    std::vector<double> h(8 * nb);
    hipError_t e = hipMemcpyAsync(h.data(), part, h.size() * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    dfree(ctx, part);
    if (e != hipSuccess) return hip_fail(ctx, e, "minmax", __FILE__, __LINE__);
    for (unsigned b = 0; b < nb; b++)
        for (int a = 0; a < 4; a++) {
            if (h[8 * b + a] < mn[a]) mn[a] = h[8 * b + a];
            if (mx[a] < h[8 * b + 4 + a]) mx[a] = h[8 * b + 4 + a];
        }
    return PCP_OK;
}

int centroid_aos48_dev(pcp_ctx* ctx, const void* in, int64_t n, int is_dense, double c[4], uint32_t* count) {
    if (n <= 0) {  // point_cloud_helper.h:197-198: centroid untouched, 0 returned
        if (count) *count = 0;
        return PCP_OK;
    }
    // the reference's sequential left fold, bit for bit (point_cloud_helper.h:199-227)
    double s[4];
    PCP_TRY(seqfold_aos48(ctx, in, n, nullptr, 0, is_dense, s));
    const uint32_t cp = is_dense ? (uint32_t)n : (uint32_t)s[3];
    const double dn = is_dense ? (double)n : (double)cp;  // size() (size_t) or unsigned cp
    c[0] = s[0] / dn; c[1] = s[1] / dn; c[2] = s[2] / dn; c[3] = 0.0 / dn;
    if (count) *count = cp;
    return PCP_OK;
}

static Xf make_xf(const double T[16]) {
    Xf x;
    for (int i = 0; i < 12; i++) x.m[i] = T[i];
    return x;
}

// V3 on device: returns the voxel count through *n_out
static int voxel_filter_impl(pcp_ctx* ctx, const P48* in, int64_t n, int is_dense, const double leaf[3], int all_data,
                             P48* out, int64_t* n_out, uint32_t* out_vidx) {
    *n_out = 0;
    if (n <= 0) return PCP_OK;  // voxel_grid.h:815-820
    if (n >= (int64_t)1 << 32) return set_error(ctx, PCP_ERR_ARG, "voxel filter supports < 2^32 points");
    hipStream_t st = ctx->stream;
    // setLeafSize (voxel_grid.h:538-549): inverse by array division
    VoxGeom g;
    for (int a = 0; a < 3; a++) g.inv[a] = 1.0 / leaf[a];
    double mn[4], mx[4];
    PCP_TRY(minmax_aos48_dev(ctx, in, n, is_dense, mn, mx));  // :831
    int min_b[3], max_b[3], div_b[3];
    for (int a = 0; a < 3; a++) {  // :835-843, truncating casts
        min_b[a] = (int)(double)(mn[a] * g.inv[a]);
        max_b[a] = (int)(double)(mx[a] * g.inv[a]);
        div_b[a] = max_b[a] - min_b[a] + 1;
        g.min_b[a] = (double)min_b[a];
    }
    g.mul1 = (uint32_t)div_b[0];  // divb_mul_ in wrapping int32 (:847)
    g.mul2 = (uint32_t)div_b[0] * (uint32_t)div_b[1];

    VoxBufs b{ctx};
    PCP_TRY(dmalloc(ctx, &b.k0, n));
    PCP_TRY(dmalloc(ctx, &b.k1, n));
    PCP_TRY(dmalloc(ctx, &b.v0, n));
    PCP_TRY(dmalloc(ctx, &b.v1, n));
    PCP_TRY(dmalloc(ctx, &b.head, n + 1));
    int64_t m = n;
    if (!is_dense) {
        PCP_TRY(dmalloc(ctx, &b.flag, n + 1));
        hipLaunchKernelGGL(k_vox_flag, dim3(grid_for(n, kB)), dim3(kB), 0, st, in, n, is_dense, b.flag);
        uint32_t valid = 0;
        PCP_TRY(scan_u32_inplace(ctx, b.flag, n, &valid));
        m = valid;
    }
    hipLaunchKernelGGL(k_vox_key, dim3(grid_for(n, kB)), dim3(kB), 0, st, in, n, is_dense, g, b.flag, b.k0, b.v0);
    PCP_LAUNCH_CHECK(ctx);
    if (m == 0) return PCP_OK;
    // stable LSD radix sort by the u32 key (voxel_grid.h:948)
    size_t tmp_bytes = 0;
    PCP_HIP(ctx, rocprim::radix_sort_pairs(nullptr, tmp_bytes, b.k0, b.k1, b.v0, b.v1, (size_t)m, 0, 32, st));
    PCP_TRY(dmalloc(ctx, (char**)&b.tmp, tmp_bytes));
    PCP_HIP(ctx, rocprim::radix_sort_pairs(b.tmp, tmp_bytes, b.k0, b.k1, b.v0, b.v1, (size_t)m, 0, 32, st));
    // runs of equal keys = voxels (:952-960)
    hipLaunchKernelGGL(k_run_heads, dim3(grid_for(m, kB)), dim3(kB), 0, st, b.k1, m, b.head);
    uint32_t nvox = 0;
    PCP_TRY(scan_u32_inplace(ctx, b.head, m, &nvox));
    uint32_t* start = b.k0;  // reuse
    hipLaunchKernelGGL(k_run_starts, dim3(grid_for(m, kB)), dim3(kB), 0, st, b.k1, b.head, m, start);
    hipLaunchKernelGGL(k_vox_reduce, dim3(grid_for(nvox, kB)), dim3(kB), 0, st, in, b.k1, b.v1, start,
                       (int64_t)nvox, m, all_data, out, out_vidx);
    PCP_LAUNCH_CHECK(ctx);
    PCP_HIP(ctx, hipStreamSynchronize(st));
    *n_out = nvox;
    return PCP_OK;
}

}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_minmax_aos48(pcp_ctx* ctx, const void* in, int64_t n, int is_dense, double mn[4], double mx[4]) {
    if (!ctx || n < 0 || (n > 0 && !in) || !mn || !mx) return set_error(ctx, PCP_ERR_ARG, "pcp_minmax_aos48: bad arguments");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    return minmax_aos48_dev(ctx, in, n, is_dense, mn, mx);
}

int pcp_centroid_aos48(pcp_ctx* ctx, const void* in, int64_t n, int is_dense, double c[4], uint32_t* count) {
    if (!ctx || n < 0 || (n > 0 && !in) || !c) return set_error(ctx, PCP_ERR_ARG, "pcp_centroid_aos48: bad arguments");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    return centroid_aos48_dev(ctx, in, n, is_dense, c, count);
}

int pcp_centroid_concat_aos48(pcp_ctx* ctx, const void* a, int64_t na, const void* b, int64_t nb, int is_dense,
                              double c[4], uint32_t* count) {
    if (!ctx || na < 0 || nb < 0 || (na > 0 && !a) || (nb > 0 && !b) || !c)
        return set_error(ctx, PCP_ERR_ARG, "pcp_centroid_concat_aos48: bad arguments");
    if (na + nb == 0) {
        if (count) *count = 0;
        return PCP_OK;
    }
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    double s[4];
    PCP_TRY(seqfold_aos48(ctx, a, na, b, nb, is_dense, s));
    const uint32_t cp = is_dense ? (uint32_t)(na + nb) : (uint32_t)s[3];
    const double dn = is_dense ? (double)(na + nb) : (double)cp;
    c[0] = s[0] / dn; c[1] = s[1] / dn; c[2] = s[2] / dn; c[3] = 0.0 / dn;
    if (count) *count = cp;
    return PCP_OK;
}

int pcp_transform_aos48(pcp_ctx* ctx, const void* in, void* out, int64_t n, int is_dense, const double T[16]) {
    if (!ctx || n < 0 || (n > 0 && (!in || !out)) || !T) return set_error(ctx, PCP_ERR_ARG, "pcp_transform_aos48: bad arguments");
    if (n == 0) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_transform48, dim3(grid_for(n, kB)), dim3(kB), 0, ctx->stream, (const P48*)in, (P48*)out, n,
                       is_dense, make_xf(T));
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

int pcp_voxel_filter(pcp_ctx* ctx, const void* in, int64_t n, int is_dense, const double leaf[3], int all_data,
                     void* out, int64_t* n_out, uint32_t* out_vidx) {
    if (!ctx || n < 0 || (n > 0 && (!in || !out)) || !leaf || !n_out)
        return set_error(ctx, PCP_ERR_ARG, "pcp_voxel_filter: bad arguments");
    for (int a = 0; a < 3; a++)
        if (!(leaf[a] > 0)) return set_error(ctx, PCP_ERR_ARG, "pcp_voxel_filter: leaf sizes must be > 0");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    return voxel_filter_impl(ctx, (const P48*)in, n, is_dense, leaf, all_data, (P48*)out, n_out, out_vidx);
}

int pcp_remove_duplicate(pcp_ctx* ctx, const void* in, int64_t n, int is_dense, float leaf, void* out, int64_t* n_out) {
    if (!ctx || n < 0 || (n > 0 && (!in || !out)) || !n_out || !(leaf > 0))
        return set_error(ctx, PCP_ERR_ARG, "pcp_remove_duplicate: bad arguments");
    *n_out = 0;
    if (n == 0) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    double c[4] = {0, 0, 0, 0};
    PCP_TRY(centroid_aos48_dev(ctx, in, n, is_dense, c, nullptr));  // :45
    double T[16] = {1, 0, 0, -c[0], 0, 1, 0, -c[1], 0, 0, 1, -c[2], 0, 0, 0, 1};
    P48* tmp = nullptr;
    PCP_TRY(dmalloc(ctx, &tmp, n));
    hipLaunchKernelGGL(k_copy_centre, dim3(grid_for(n, kB)), dim3(kB), 0, ctx->stream, (const P48*)in, tmp, n, is_dense,
                       make_xf(T));
    const double lf = (double)leaf;  // float leaf widened (:57)
    const double l3[3] = {lf, lf, lf};
    int64_t m = 0;
    int rc = voxel_filter_impl(ctx, tmp, n, is_dense, l3, 1, (P48*)out, &m, nullptr);
    if (rc == PCP_OK && m > 0) {
        T[3] = c[0]; T[7] = c[1]; T[11] = c[2];  // :60-61
        hipLaunchKernelGGL(k_transform48, dim3(grid_for(m, kB)), dim3(kB), 0, ctx->stream, (const P48*)out, (P48*)out,
                           m, 1, make_xf(T));
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) rc = hip_fail(ctx, e, "remove_duplicate", __FILE__, __LINE__);
    }
    dfree(ctx, tmp);
    if (rc == PCP_OK) *n_out = m;
    return rc;
}

int pcp_get_rot_icp(pcp_ctx* ctx, const void* src, int64_t ns, int src_dense, const void* tmp, int64_t nt,
                    int tmp_dense, double M[16], float rmax, int iters, int do_scale, double cell_size, float* err) {
    if (!ctx || ns < 0 || nt < 0 || (ns > 0 && !src) || (nt > 0 && !tmp) || !M || iters < 0)
        return set_error(ctx, PCP_ERR_ARG, "pcp_get_rot_icp: bad arguments");
    if (err) *err = -1.0f;
    for (int i = 0; i < 16; i++) M[i] = (i % 5 == 0) ? 1.0 : 0.0;
    // the reference passes maxdist = 0 (point_cloud_helper.cpp:127), which makes trimesh2 derive
    // its own threshold from the clouds' overlap (ICP.h:17-28; library absent, not restated):
    // this build needs an explicit correspondence distance and says so instead of guessing one
    if (!(rmax > 0.f))
        return set_error(ctx, PCP_ERR_UNSUPPORTED,
                         "pcp_get_rot_icp: rmax must be > 0 (trimesh2's automatic maxdist = 0 is not provided)");
    if (ns == 0 || nt == 0) return PCP_OK;  // ICP fails: err < 0 (ICP.h:26-28)
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    // joint centroid over cloud_all = src ++ temp (point_cloud_helper.cpp:78-83): one sequential
    // fold over the concatenation; cloud_all.is_dense = src.is_dense && temp.is_dense
    // (PointCloud::operator+=), so a non-dense input skips non-finite points of both
    double s[4];
    const int joint_dense = src_dense && tmp_dense;
    PCP_TRY(seqfold_aos48(ctx, src, ns, tmp, nt, joint_dense, s));
    const double dn = joint_dense ? (double)(ns + nt) : (double)(uint32_t)s[3];  // size() / unsigned cp
    const double c[3] = {s[0] / dn, s[1] / dn, s[2] / dn};
    float* fs = nullptr;
    float* ft = nullptr;
    PCP_TRY(dmalloc(ctx, &fs, 3 * (size_t)ns));
    int rc = dmalloc(ctx, &ft, 3 * (size_t)nt);
    pcp_index* ix = nullptr;
    pcp_icp* icp = nullptr;
    if (rc == PCP_OK) {
        hipLaunchKernelGGL(k_centre_f32, dim3(grid_for(ns, kB)), dim3(kB), 0, ctx->stream, (const P48*)src, ns, c[0],
                           c[1], c[2], fs);
        hipLaunchKernelGGL(k_centre_f32, dim3(grid_for(nt, kB)), dim3(kB), 0, ctx->stream, (const P48*)tmp, nt, c[0],
                           c[1], c[2], ft);
        rc = pcp_index_build_f32(ctx, fs, 3 * sizeof(float), ns, cell_size, &ix);
    }
    if (rc == PCP_OK) rc = pcp_icp_create(ctx, ix, ft, 3 * sizeof(float), nt, &icp);
    double T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    float e = -1.0f;
    if (rc == PCP_OK) {
        rc = pcp_icp_run(ctx, icp, T, rmax, iters, do_scale, 0.0, &e);
        if (rc == PCP_ERR_ICP) rc = PCP_OK;  // failure is reported through err < 0
    }
    if (rc == PCP_OK) {
        std::memcpy(M, T, sizeof(T));
        for (int r = 0; r < 3; r++) {  // t' = (t - R c) + c (:164)
            double rcv = M[4 * r] * c[0];
            rcv = rcv + M[4 * r + 1] * c[1];
            rcv = rcv + M[4 * r + 2] * c[2];
            M[4 * r + 3] = (M[4 * r + 3] - rcv) + c[r];
        }
        if (err) *err = e;
    }
    if (icp) pcp_icp_destroy(icp);
    if (ix) pcp_index_destroy(ix);
    dfree(ctx, fs);
    dfree(ctx, ft);
    return rc;
}

}  // extern "C"
