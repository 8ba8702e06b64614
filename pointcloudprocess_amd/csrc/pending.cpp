// Entry points declared in include/pcp.h whose kernels land in later commits.
// Each returns PCP_ERR_UNSUPPORTED loudly (never a CPU fallback).
#include "common.hpp"

#define PCP_PENDING(name) pcp::set_error(ctx, PCP_ERR_UNSUPPORTED, name " not implemented yet")

extern "C" {
int pcp_knn_bruteforce(pcp_ctx* ctx, const double*, size_t, int64_t, const double*, size_t, int64_t, int,
                       int32_t*, double*) { return PCP_PENDING("pcp_knn_bruteforce"); }
}
