// Region growing: TreeExtration::region_growning (extraction_tree.cpp:66-272; the live body is
// :177-271), as called by point_segment (static.cpp:8-21) with the per-point planes of
// calculate_plan_parameter_rpca (rpca.hip).
//
// The reference walks the points in index order; a point whose rpca curvature is < 0.005 seeds
// a segment, which grows breadth-first: each popped point p issues nearestKSearch(cloud
// [PointID[p]], 50) and every still-unsegmented neighbour q joins when
//   |cos(seed normal, normal q)| > cosfaT   (compute_included_angle_between_vector, :36-44)
//   dist(q, plane of p) < distanceT         (compute_distance_from_point_to_plane, :47-64)
// A segment of <= 5 points is dropped (its points go back to UNSEGMENTATION, but stay out of
// the seed walk).  Labels and the order of each segment's PointID list depend on that
// sequential walk, so it is replayed on the host exactly; everything it needs that does not
// depend on the walk runs on the GPU first:
//   1. the 50-NN graph of every point (pcp_knn: FLANN's order, exact fp64) -- the reference's
//      dominant cost, one nearestKSearch per popped point;
//   2. the plane-distance test of every (p, neighbour i) edge, folded into one 64-bit mask per
//      point (k_rg_edges): it depends on p's plane and q's position only.
// The host walk then reads the graph, the masks and the seed-normal test (which does depend on
// the segment's seed) -- about 50 int32 + 1 mask + a few floats per popped point.
#include <cmath>
#include <cstring>
#include <vector>

#include "common.hpp"

namespace pcp {
namespace {

constexpr int kRgK = 50;                 // nearestKSearch(searchPoint, 50, ...) (:222)
constexpr double kSeedCurvature = 0.005;  // PointProperty[minNum].curvature < 0.005 (:196)

// compute_distance_from_point_to_plane (:47-64): float plane coefficients (the doubles of the
// call are narrowed by the float parameters) and float point; the norm is the float sqrt of a
// float sum (cmath's float overload), widened; the products are float, summed in double.
__host__ __device__ inline float plane_dis(float a, float b, float c, float d, double px, double py, double pz) {
    const float x1 = (float)px, y1 = (float)py, z1 = (float)pz;
    const double g = (double)sqrtf(a * a + b * b + c * c);
    const double f1 = a * x1, f2 = b * y1, f3 = c * z1, f4 = d;
    const double f = fabs(f1 + f2 + f3 + f4);
    return (float)(f / g);
}

// compute_included_angle_between_vector (:36-44), all float
inline float included_cos(float vx1, float vy1, float vz1, float vx2, float vy2, float vz2) {
    const float n_n1 = vx1 * vx2 + vy1 * vy2 + vz1 * vz2;
    const float n_n = std::sqrt(vx1 * vx1 + vy1 * vy1 + vz1 * vz1);
    const float n1_n1 = std::sqrt(vx2 * vx2 + vy2 * vy2 + vz2 * vz2);
    return std::fabs(n_n1 / (n_n * n1_n1));
}

// One thread per point p: bit i of mask[p] = neighbour i of cloud[PointID[p]] lies within
// distanceT of p's plane.  Rows end at the first -1 (fewer than k valid points, or a
// non-finite query that FLANN answers with no neighbours).
__global__ void k_rg_edges(const pcp_point_property* __restrict__ props, const char* __restrict__ xyz, size_t stride,
                           int64_t n, const int32_t* __restrict__ nbr, int k, double distance_t,
                           uint64_t* __restrict__ mask) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const pcp_point_property pp = props[p];
        const float a = pp.normal_x, b = pp.normal_y, c = pp.normal_z, d = (float)pp.distance;
        const int32_t* row = nbr + (int64_t)pp.point_id * k;
        uint64_t m = 0;
        for (int i = 0; i < k; i++) {
            const int32_t j = row[i];
            if (j < 0) break;
            const double* q = (const double*)(xyz + (int64_t)j * stride);
            if ((double)plane_dis(a, b, c, d, q[0], q[1], q[2]) < distance_t) m |= 1ull << i;
        }
        mask[p] = m;
    }
}

}  // namespace
}  // namespace pcp

using namespace pcp;

extern "C" int pcp_region_growing(pcp_ctx* ctx, const pcp_index* index, const double* xyz, size_t stride, int64_t n,
                                  pcp_point_property* props, double distance_t, double cosfa_t, int64_t* seg_offsets,
                                  int32_t* seg_points, int32_t* seg_seeds, int64_t* n_seg) {
    if (!ctx || !index || !n_seg || n < 0 || (n > 0 && (!xyz || !props || !seg_offsets || !seg_points || !seg_seeds)))
        return set_error(ctx, PCP_ERR_ARG, "pcp_region_growing: bad arguments");
    if (stride == 0) stride = 3 * sizeof(double);
    *n_seg = 0;
    seg_offsets[0] = 0;
    if (n == 0) return PCP_OK;
    if (index->n_in != n)
        return set_error(ctx, PCP_ERR_ARG, "pcp_region_growing: index covers %lld points, cloud has %lld",
                         (long long)index->n_in, (long long)n);
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    std::vector<pcp_point_property> hp((size_t)n);
    PCP_HIP(ctx, hipMemcpyAsync(hp.data(), props, n * sizeof(pcp_point_property), hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    for (int64_t p = 0; p < n; p++)
        if (hp[p].point_id < 0 || hp[p].point_id >= n)
            return set_error(ctx, PCP_ERR_ARG, "pcp_region_growing: PointID %d of point %lld outside the cloud",
                             hp[p].point_id, (long long)p);

    const int k = kRgK;
    int32_t* nbr = nullptr;
    uint64_t* mask = nullptr;
    PCP_TRY(dmalloc(ctx, &nbr, (size_t)n * k));
    PCP_TRY(dmalloc(ctx, &mask, (size_t)n));
    struct Free {
        pcp_ctx* c; void* a; void* b;
        ~Free() { dfree(c, a); dfree(c, b); }
    } fr{ctx, nbr, mask};
    PCP_TRY(pcp_knn(ctx, index, xyz, stride, n, k, nbr, nullptr));
    hipLaunchKernelGGL(k_rg_edges, dim3(grid_for(n, 256, 1 << 16)), dim3(256), 0, ctx->stream, props,
                       (const char*)xyz, stride, n, nbr, k, distance_t, mask);
    PCP_LAUNCH_CHECK(ctx);
    std::vector<int32_t> hn((size_t)n * k);
    std::vector<uint64_t> hm((size_t)n);
    PCP_HIP(ctx, hipMemcpyAsync(hn.data(), nbr, hn.size() * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipMemcpyAsync(hm.data(), mask, hm.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));

    // the sequential walk (:184-269); `walked` is UnSegment's complement, seg is SegmentID
    std::vector<int32_t> seg((size_t)n, -1);
    std::vector<uint8_t> walked((size_t)n, 0);
    std::vector<int32_t> fifo((size_t)n);
    int32_t label = 0;
    int64_t npts = 0;
    for (int64_t m0 = 0; m0 < n; m0++) {
        if (walked[m0]) continue;
        walked[m0] = 1;
        if (!(hp[m0].curvature < kSeedCurvature)) continue;
        const int32_t seed = (int32_t)m0;
        const float nx = hp[seed].normal_x, ny = hp[seed].normal_y, nz = hp[seed].normal_z;
        const int64_t first = npts;
        seg[seed] = label;
        seg_points[npts++] = seed;
        int64_t head = 0, tail = 0;
        fifo[tail++] = seed;
        while (head < tail) {
            const int32_t p = fifo[head++];
            const int32_t* row = &hn[(size_t)hp[p].point_id * k];
            const uint64_t em = hm[p];
            for (int i = 0; i < k; i++) {
                const int32_t q = row[i];
                if (q < 0) break;
                if (seg[q] != -1) continue;
                const float cs = included_cos(nx, ny, nz, hp[q].normal_x, hp[q].normal_y, hp[q].normal_z);
                if ((double)cs > cosfa_t && ((em >> i) & 1)) {
                    seg[q] = label;
                    seg_points[npts++] = q;
                    walked[q] = 1;
                    fifo[tail++] = q;
                }
            }
        }
        if (npts - first > 5) {
            seg_seeds[label] = seed;
            seg_offsets[++label] = npts;
        } else {
            for (int64_t t = first; t < npts; t++) seg[seg_points[t]] = -1;
            npts = first;
        }
    }
    *n_seg = label;
    for (int64_t p = 0; p < n; p++) hp[p].segment_id = seg[p];
    PCP_HIP(ctx, hipMemcpyAsync(props, hp.data(), n * sizeof(pcp_point_property), hipMemcpyHostToDevice, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return PCP_OK;
}
