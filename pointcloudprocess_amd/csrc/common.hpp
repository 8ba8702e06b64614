// Shared internals of libpcp (HIP, gfx950).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <unordered_map>

#include <vector>

#include "../../include/pcp.h"

struct pcp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // a non-blocking stream for work that overlaps the main stream inside one call (the query
    // sort of pcp_icp_create_with_target); created on first use, ordered by events both ways
    hipStream_t side = nullptr;
    std::string last_error;
    // grow-only scratch arena (one per context; contexts are not shared across threads)
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    uint32_t bf_fallback = 0;  // queries of the last pcp_knn_bruteforce that needed the exact scan
    // look-back scan state (scan.hip): per-tile status words tagged with the call's epoch, so
    // no clearing pass is needed per call; [tiles] u64 status, then the tile counter and total
    uint64_t* scan_status = nullptr;
    // timing events returned by destroyed ICP handles, reused by the next (creating and
    // destroying ~44 events per registration cost ~0.3 ms of host time)
    std::vector<hipEvent_t> event_pool;
    int64_t scan_tiles = 0;
    uint32_t scan_epoch = 0;
    // Caching device allocator for the library's internal buffers (index builds, ICP state,
    // per-call scratch): blocks are reused in stream order on this context's stream instead
    // of paying a synchronising hipMalloc/hipFree each time.  Objects allocated through a
    // context must be destroyed before it.
    std::multimap<size_t, void*> free_blocks;
    std::unordered_map<void*, size_t> block_size;
    size_t cached_bytes = 0;
    size_t cache_cap = (size_t)16 << 30;  // set from the device size at create (a third of HBM)
    // lifetime: every index / ICP handle / CloudGrid made on the context holds a reference, so
    // the objects may be destroyed before OR after pcp_ctx_destroy (a garbage-collected host
    // language finalises them in any order): destroy marks the context closing, frees what no
    // object uses, and the last object's destroy finishes the job
    int live = 0;
    bool closing = false;
};

namespace pcp {

int set_error(pcp_ctx* ctx, int code, const char* fmt, ...);
int hip_fail(pcp_ctx* ctx, hipError_t e, const char* what, const char* file, int line);
// scratch of at least `bytes` (invalidates earlier scratch pointers)
int scratch(pcp_ctx* ctx, size_t bytes, void** out);
// the context's side stream (created on first use)
int side_stream(pcp_ctx* ctx, hipStream_t* out);

#define PCP_HIP(ctx, expr)                                                           \
    do {                                                                             \
        hipError_t _e = (expr);                                                      \
        if (_e != hipSuccess) return ::pcp::hip_fail((ctx), _e, #expr, __FILE__, __LINE__); \
    } while (0)

#define PCP_TRY(expr)                 \
    do {                              \
        int _rc = (expr);             \
        if (_rc != PCP_OK) return _rc; \
    } while (0)

#define PCP_LAUNCH_CHECK(ctx) PCP_HIP(ctx, hipGetLastError())

// cached device allocation of `bytes` (>= 1) on ctx; dfree returns it to ctx's cache
int cache_alloc(pcp_ctx* ctx, size_t bytes, void** p);
void dfree(pcp_ctx* ctx, void* p);
void cache_release(pcp_ctx* ctx);
// object lifetime references on a context (see pcp_ctx::live)
void ctx_retain(pcp_ctx* ctx);
void ctx_release(pcp_ctx* ctx);
// a timing event from ctx's pool (or a new one); event_put returns it to the pool
hipError_t event_get(pcp_ctx* ctx, hipEvent_t* ev);
void event_put(pcp_ctx* ctx, hipEvent_t ev);

template <typename T>
int dmalloc(pcp_ctx* ctx, T** p, size_t count) {
    void* v = nullptr;
    const int rc = cache_alloc(ctx, (count ? count : 1) * sizeof(T), &v);
    *p = (T*)v;
    return rc;
}
inline unsigned grid_for(int64_t n, int block, int64_t cap = 1 << 20) {
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ bool finite3(double x, double y, double z) {
    return isfinite(x) && isfinite(y) && isfinite(z);
}

// compute3DCentroid's sequential fp64 fold of x/y/z over the AoS48 records seg0 ++ seg1, bit-exact
// (fold.hip); s_host[3] = number of points summed (finite ones when !is_dense).
int seqfold_aos48(pcp_ctx* ctx, const void* p0, int64_t n0, const void* p1, int64_t n1, int is_dense,
                  double s_host[4]);

// Exclusive scan of `n` uint32 values in place (values' total must fit uint32).
// Returns the total through *total_dev (device, optional) and *total_host (optional, syncs).
int scan_u32_inplace(pcp_ctx* ctx, uint32_t* data, int64_t n, uint32_t* total_host);
// Exclusive scan of int32 counts into int64 offsets (n+1 entries).
int scan_i32_to_i64(pcp_ctx* ctx, const int32_t* in, int64_t n, int64_t* out, int64_t* total_host);

// ---------------------------------------------------------------- grid description
// Uniform grid of cubic cells.  Dense mode (the MI355X default whenever the table fits the
// HBM budget): cstart has one entry per cell of the bounding grid, linear id
// (z*ny + y)*nx + x, so a row of cells along x is one contiguous point range.  Sparse
// mode (huge sparse bounding boxes): 4x4x4 bricks, a dense brick table maps a brick to a
// slot (or -1) and each slot owns 64 consecutive cstart entries.
struct GridDesc {
    double o[3];      // origin (bbox min)
    double h, inv_h;  // cell size
    float of[3];
    float hf, inv_hf;
    int n[3];         // cells per axis
    int nb[3];        // bricks per axis
    int64_t nbricks;
    int64_t nslots;
    int dense;                // 1: cstart is indexed by the linear cell id (x fastest)
    int64_t ncells;           // dense: n[0]*n[1]*n[2]
    const int32_t* brick;     // nbricks (sparse mode only)
    const uint32_t* cstart;   // dense: ncells + 1 ; sparse: 64*nslots + 1
};


}  // namespace pcp

struct pcp_index {
    int is_f64 = 0;
    pcp::GridDesc g{};
    int64_t n_in = 0;        // size of the cloud passed in (n, or n_indices)
    int64_t n = 0;           // valid points (total_nr_points_)
    int identity = 0;
    int32_t* brick = nullptr;
    uint32_t* cstart = nullptr;
    void* pts = nullptr;        // float4[n] or double4[n], sorted by (slot, local cell)
    int32_t* mapping = nullptr; // internal j -> caller index (n)
    int32_t* sorted_j = nullptr; // sorted position -> internal j (n)
    int32_t* pos_of_j = nullptr; // internal j -> sorted position (n, fp64 index only)
    // fp16 cell-relative index (C5, h16.hip): per sorted point its offset from its cell's
    // origin as 3 x fp16 (+ 16-bit pad) and its dense cell id; pts is released after the build
    int is_h16 = 0;
    uint2* h16 = nullptr;
    uint32_t* cell = nullptr;
    pcp_ctx* owner = nullptr;
};
