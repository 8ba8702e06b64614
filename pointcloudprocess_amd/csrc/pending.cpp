// Entry points declared in include/pcp.h whose kernels land in later commits.
// Each returns PCP_ERR_UNSUPPORTED loudly (never a CPU fallback).
#include "common.hpp"

#define PCP_PENDING(name) pcp::set_error(ctx, PCP_ERR_UNSUPPORTED, name " not implemented yet")

extern "C" {
int pcp_knn(pcp_ctx* ctx, const pcp_index*, const double*, size_t, int64_t, int, int32_t*, double*) {
    return PCP_PENDING("pcp_knn");
}
int pcp_radius_count(pcp_ctx* ctx, const pcp_index*, const double*, size_t, int64_t, double, uint32_t,
                     int32_t*) { return PCP_PENDING("pcp_radius_count"); }
int pcp_radius_fill(pcp_ctx* ctx, const pcp_index*, const double*, size_t, int64_t, double, uint32_t,
                    const int64_t*, int32_t*, double*) { return PCP_PENDING("pcp_radius_fill"); }
int pcp_knn_bruteforce(pcp_ctx* ctx, const double*, size_t, int64_t, const double*, size_t, int64_t, int,
                       int32_t*, double*) { return PCP_PENDING("pcp_knn_bruteforce"); }
int pcp_knn_lod(pcp_ctx* ctx, const void*, int64_t, const void*, int64_t, int, int32_t*, double*) {
    return PCP_PENDING("pcp_knn_lod");
}
int pcp_minmax_aos48(pcp_ctx* ctx, const void*, int64_t, int, double*, double*) { return PCP_PENDING("pcp_minmax_aos48"); }
int pcp_centroid_aos48(pcp_ctx* ctx, const void*, int64_t, int, double*, uint32_t*) { return PCP_PENDING("pcp_centroid_aos48"); }
int pcp_transform_aos48(pcp_ctx* ctx, const void*, void*, int64_t, int, const double*) { return PCP_PENDING("pcp_transform_aos48"); }
int pcp_voxel_filter(pcp_ctx* ctx, const void*, int64_t, int, const double*, int, void*, int64_t*, uint32_t*) {
    return PCP_PENDING("pcp_voxel_filter");
}
int pcp_remove_duplicate(pcp_ctx* ctx, const void*, int64_t, int, float, void*, int64_t*) { return PCP_PENDING("pcp_remove_duplicate"); }
int pcp_normals_knn(pcp_ctx* ctx, const pcp_index*, int, pcp_plane*, int64_t) { return PCP_PENDING("pcp_normals_knn"); }
int pcp_get_rot_icp(pcp_ctx* ctx, const void*, int64_t, const void*, int64_t, double*, float, int, int, double, float*) {
    return PCP_PENDING("pcp_get_rot_icp");
}
}
