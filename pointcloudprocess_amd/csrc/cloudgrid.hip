// CloudGrid (cloud_grid.h:37-88, cloud_grid.cpp) on the GPU: the map cache that builds every
// ICP target (main_blend.cpp:263, 471, 792-795, 1027).  The reference keeps a boost hash map of
// 1 m x 1 m cells keyed by ((int)x, (int)y) and, per cell, the points kept by a greedy 4 cm
// de-duplication in arrival order (add_cloud_internal, cloud_grid.cpp:34-78).
//
// Here the grid is a cell-sorted table: cell keys ascending by (ix, iy), a start offset per
// cell and the kept 48-byte records grouped by cell in kept order.
//   add_cloud  stable radix sort of (cell key, arrival order) over the old kept points and the
//              new ones (old first, so a cell's old points come first in their order); then one
//              wave per cell replays the reference's sequential de-duplication exactly -- the
//              kept points of the cell live in an LDS hash of 0.045 m sub-cells (any conflict
//              lies within one sub-cell per axis), so each arrival checks the 27 neighbouring
//              sub-cells' chains in parallel lanes instead of every kept point; a compaction
//              writes the new table.
//   box        get_cloud_with_pos: rows i of the key range, each row's cells one contiguous run.
//   match      get_grid_cloud(src, src_out, dst, dis): per source point its cell (binary
//              search), the cell's z-range test, the Chebyshev-dis matches; each grid point is
//              emitted at its first matching source point (atomicMin), ordered by (that source
//              index, position) -- the reference's push order.
#include <cfloat>
#include <climits>
#include <cmath>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

#include "common.hpp"

struct pcp_grid {
    pcp_ctx* ctx = nullptr;
    int64_t n = 0;               // kept points
    int64_t ncell = 0;           // non-empty cells
    uint8_t* pts = nullptr;      // n records (48 B), grouped by cell, kept order within a cell
    uint64_t* keys = nullptr;    // ncell cell keys, ascending
    int64_t* cstart = nullptr;   // ncell + 1 offsets into pts
};

namespace pcp {
namespace {

constexpr double kDupX = 0.04;                // MAX_DIS_2POINT_X (cloud_grid.cpp:11)
constexpr double kDup2 = kDupX * kDupX;       // MAX_DIS_2POINT (:12)
constexpr double kSub = 0.045;                // hash sub-cell (> kDupX: a conflict is within +-1 sub-cell)
constexpr int kHashSlots = 2048;              // per wave (LDS): sub-cell key + chain head

__device__ __forceinline__ uint64_t cell_key(int ix, int iy) {
    return ((uint64_t)((uint32_t)ix ^ 0x80000000u) << 32) | (uint64_t)((uint32_t)iy ^ 0x80000000u);
}
__device__ __forceinline__ const double* rec_xyz(const uint8_t* base, int64_t i) {
    return (const double*)(base + 48 * i);
}

// keys and arrival order: old kept points (already grouped by cell) first, then the new cloud
__global__ void k_grid_keys(const uint8_t* old_pts, int64_t n_old, const uint8_t* cloud, int64_t n_new,
                            uint64_t* key, uint32_t* order) {
    const int64_t m = n_old + n_new;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x) {
        const double* p = t < n_old ? rec_xyz(old_pts, t) : rec_xyz(cloud, t - n_old);
        // int irow = x; int icol = y (truncation toward zero, cloud_grid.cpp:38-39)
        key[t] = cell_key((int)p[0], (int)p[1]);
        order[t] = (uint32_t)t;
    }
}

__global__ void k_grid_gather(const uint8_t* old_pts, int64_t n_old, const uint8_t* cloud, const uint32_t* order,
                              int64_t m, uint8_t* rec) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = order[t];
        const uint4* s = (const uint4*)(o < n_old ? old_pts + 48 * o : cloud + 48 * (o - n_old));
        uint4* d = (uint4*)(rec + 48 * t);
        d[0] = s[0];
        d[1] = s[1];
        d[2] = s[2];
    }
}

// run heads of the sorted keys -> 1 at each cell's first point
__global__ void k_grid_heads(const uint64_t* key, int64_t m, uint32_t* head) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x)
        head[t] = (t == 0 || key[t] != key[t - 1]) ? 1u : 0u;
}
// head prefix (exclusive) -> cell start offsets and keys
__global__ void k_grid_cells(const uint64_t* key, const uint32_t* head_scan, const uint32_t* head, int64_t m,
                             int64_t* cstart, uint64_t* ckey) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x)
        if (head[t]) {
            cstart[head_scan[t]] = t;
            ckey[head_scan[t]] = key[t];
        }
}

__device__ __forceinline__ uint32_t sub_key(const double* p) {
    const int sx = (int)floor(p[0] / kSub), sy = (int)floor(p[1] / kSub), sz = (int)floor(p[2] / kSub);
    return ((uint32_t)sx & 0x3ffu) | (((uint32_t)sy & 0x3ffu) << 10) | (((uint32_t)sz & 0xfffu) << 20);
}
__device__ __forceinline__ uint32_t sub_key_off(uint32_t k, int dx, int dy, int dz) {
    const uint32_t x = (k + (uint32_t)dx) & 0x3ffu, y = ((k >> 10) + (uint32_t)dy) & 0x3ffu,
                   z = ((k >> 20) + (uint32_t)dz) & 0xfffu;
    return x | (y << 10) | (z << 20);
}
__device__ __forceinline__ uint32_t hslot(uint32_t k) { return (k * 2654435761u) >> 21; }  // 11 bits

// is_2point_high_x(a, b, 0.04) false and dis_two_point(a, b) < MAX_DIS_2POINT: the float-valued
// squared distance of cloud_grid.h:73-77 compared against the double constant
__device__ __forceinline__ bool is_dup(const double* a, const double* b) {
    const double dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    if (fabs(dx) > kDupX || fabs(dy) > kDupX || fabs(dz) > kDupX) return false;
    const float d = (float)(dx * dx + dy * dy + dz * dz);
    return (double)d < kDup2;
}

// one wave per cell: the reference's sequential arrival loop (cloud_grid.cpp:36-77)
__global__ __launch_bounds__(64) void k_grid_dedupe(const uint8_t* rec, const int64_t* cstart, int64_t ncell,
                                                    int64_t n_old_total, const uint32_t* order, int32_t* next,
                                                    int32_t* klist, uint32_t* keep) {
    __shared__ uint32_t s_key[kHashSlots];
    __shared__ int32_t s_head[kHashSlots];
    const int lane = threadIdx.x;
    for (int64_t c = blockIdx.x; c < ncell; c += gridDim.x) {
        const int64_t s = cstart[c], e = cstart[c + 1];
        for (int h = lane; h < kHashSlots; h += 64) {
            s_key[h] = 0xffffffffu;
            s_head[h] = -1;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        int nfill = 0;         // occupied hash slots
        bool brute = false;    // the hash filled up: scan the kept list instead
        int64_t kc = 0;        // kept so far (klist[s .. s + kc))
        for (int64_t t = s; t < e; t++) {
            const double* p = rec_xyz(rec, t);
            const bool old = order[t] < (uint32_t)n_old_total;
            bool dup = false;
            if (!old) {
                if (!brute) {
                    const uint32_t k0 = sub_key(p);
                    if (lane < 27) {
                        const uint32_t kk = sub_key_off(k0, lane % 3 - 1, (lane / 3) % 3 - 1, lane / 9 - 1);
                        uint32_t h = hslot(kk);
                        while (s_key[h] != 0xffffffffu && s_key[h] != kk) h = (h + 1) & (kHashSlots - 1);
                        for (int32_t q = s_key[h] == kk ? s_head[h] : -1; q >= 0 && !dup; q = next[q])
                            dup = is_dup(rec_xyz(rec, q), p);
                    }
                } else {
                    for (int64_t q = lane; q < kc && !dup; q += 64) dup = is_dup(rec_xyz(rec, klist[s + q]), p);
                }
                dup = __ballot(dup) != 0;
            }
            if (!dup) {  // kept: into the kept list and the sub-cell hash
                if (lane == 0) {
                    keep[t] = 1u;
                    klist[s + kc] = (int32_t)t;
                    if (!brute) {
                        const uint32_t kk = sub_key(p);
                        uint32_t h = hslot(kk);
                        while (s_key[h] != 0xffffffffu && s_key[h] != kk) h = (h + 1) & (kHashSlots - 1);
                        if (s_key[h] != kk) {
                            s_key[h] = kk;
                            nfill++;
                        }
                        next[t] = s_head[h];
                        s_head[h] = (int32_t)t;
                    }
                }
                kc++;
                nfill = __shfl(nfill, 0, 64);
                if (nfill > kHashSlots * 3 / 4) brute = true;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __syncthreads();
            } else if (lane == 0) {
                keep[t] = 0u;
            }
        }
        __syncthreads();
    }
}

__global__ void k_grid_compact(const uint8_t* rec, const uint32_t* keep, const uint32_t* pos, int64_t m, uint8_t* out) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x)
        if (keep[t]) {
            const uint4* s = (const uint4*)(rec + 48 * t);
            uint4* d = (uint4*)(out + 48 * (int64_t)pos[t]);
            d[0] = s[0];
            d[1] = s[1];
            d[2] = s[2];
        }
}
// new cell starts: the kept prefix at each old cell start
__global__ void k_grid_restart(const int64_t* cstart, const uint32_t* pos, int64_t ncell, int64_t m, uint32_t total,
                               int64_t* out) {
    for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c <= ncell; c += (int64_t)gridDim.x * blockDim.x)
        out[c] = c < ncell ? (int64_t)pos[cstart[c]] : (int64_t)total;
}

__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t* a, int64_t n, uint64_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// box: per row i of [i0, i1) the point range of the cells (i, [j0, j1))
__global__ void k_grid_rows(const uint64_t* keys, const int64_t* cstart, int64_t ncell, int i0, int nrows, int j0,
                            int j1, int64_t* rlo, int64_t* rlen) {
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += gridDim.x * blockDim.x) {
        const int i = i0 + r;
        const int64_t a = lower_bound_u64(keys, ncell, cell_key(i, j0));
        const int64_t b = lower_bound_u64(keys, ncell, cell_key(i, j1));
        rlo[r] = cstart[a];
        rlen[r] = cstart[b] - cstart[a];
    }
}
__global__ void k_grid_box_copy(const uint8_t* pts, const int64_t* rlo, const int64_t* roff, int nrows, int64_t total,
                                uint8_t* out) {
    for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < total; o += (int64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = nrows - 1;  // the row with roff[r] <= o < roff[r + 1]
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (roff[mid] <= o) lo = mid;
            else hi = mid - 1;
        }
        const uint4* s = (const uint4*)(pts + 48 * (rlo[lo] + (o - roff[lo])));
        uint4* d = (uint4*)(out + 48 * o);
        d[0] = s[0];
        d[1] = s[1];
        d[2] = s[2];
    }
}

// match: per cell its z range with the reference's initial values (max from DBL_MIN,
// cloud_grid.cpp:185-190); per source point, the cell's matches
__global__ void k_grid_zrange(const uint8_t* pts, const int64_t* cstart, int64_t ncell, uint8_t* tall) {
    for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < ncell; c += (int64_t)gridDim.x * blockDim.x) {
        double mn = DBL_MAX, mx = DBL_MIN;
        for (int64_t k = cstart[c]; k < cstart[c + 1]; k++) {
            const double z = rec_xyz(pts, k)[2];
            mn = fmin(mn, z);
            mx = fmax(mx, z);
        }
        tall[c] = !(mx - mn < 1.5);
    }
}
__global__ void k_grid_match(const uint8_t* pts, const uint64_t* keys, const int64_t* cstart, int64_t ncell,
                             const uint8_t* tall, const uint8_t* src, int64_t nsrc, double dis, uint32_t* found,
                             uint32_t* first) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nsrc; i += (int64_t)gridDim.x * blockDim.x) {
        const double* p = rec_xyz(src, i);
        const uint64_t k = cell_key((int)p[0], (int)p[1]);
        const int64_t c = lower_bound_u64(keys, ncell, k);
        uint32_t f = 0;
        if (c < ncell && keys[c] == k && tall[c]) {
            for (int64_t q = cstart[c]; q < cstart[c + 1]; q++) {
                const double* g = rec_xyz(pts, q);
                if (fabs(g[0] - p[0]) > dis || fabs(g[1] - p[1]) > dis || fabs(g[2] - p[2]) > dis) continue;
                f = 1;
                atomicMin(first + q, (uint32_t)i);
            }
        }
        found[i] = f;
    }
}
__global__ void k_grid_fill_u32(uint32_t* a, int64_t n, uint32_t v) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) a[t] = v;
}
// dst order keys: (first matching source index, position) for the matched grid points
__global__ void k_grid_dst_keys(const uint32_t* first, int64_t n, const uint32_t* pos, uint64_t* out) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
        if (first[t] != 0xffffffffu) out[pos[t]] = ((uint64_t)first[t] << 32) | (uint64_t)t;
}
__global__ void k_grid_matched(const uint32_t* first, int64_t n, uint32_t* flag) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
        flag[t] = first[t] != 0xffffffffu ? 1u : 0u;
}
__global__ void k_grid_gather_sorted(const uint8_t* pts, const uint64_t* skeys, int64_t m, uint8_t* out) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x) {
        const uint4* s = (const uint4*)(pts + 48 * (int64_t)(uint32_t)skeys[t]);
        uint4* d = (uint4*)(out + 48 * t);
        d[0] = s[0];
        d[1] = s[1];
        d[2] = s[2];
    }
}

struct Tmp {  // per-call device temporaries, returned to the context's cache on scope exit
    pcp_ctx* ctx;
    std::vector<void*> v;
    explicit Tmp(pcp_ctx* c) : ctx(c) {}
    ~Tmp() {
        for (void* p : v) dfree(ctx, p);
    }
    template <typename T>
    int get(T** p, size_t n) {
        PCP_TRY(dmalloc(ctx, p, n));
        v.push_back((void*)*p);
        return PCP_OK;
    }
    // hand an allocation over to the caller (on success): the guard no longer frees it
    void release(const void* p) {
        for (void*& q : v)
            if (q == p) q = nullptr;
    }
};

}  // namespace
}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_grid_create(pcp_ctx* ctx, pcp_grid** out) {
    if (!ctx || !out) return PCP_ERR_ARG;
    pcp_grid* g = new pcp_grid();
    g->ctx = ctx;
    ctx_retain(ctx);
    *out = g;
    return PCP_OK;
}

int pcp_grid_clear(pcp_ctx* ctx, pcp_grid* g) {
    if (!ctx || !g) return PCP_ERR_ARG;
    dfree(ctx, g->pts);
    dfree(ctx, g->keys);
    dfree(ctx, g->cstart);
    g->pts = nullptr;
    g->keys = nullptr;
    g->cstart = nullptr;
    g->n = g->ncell = 0;
    return PCP_OK;
}

int pcp_grid_destroy(pcp_grid* g) {
    if (!g) return PCP_ERR_ARG;
    pcp_grid_clear(g->ctx, g);
    pcp_ctx* owner = g->ctx;
    delete g;
    ctx_release(owner);
    return PCP_OK;
}

int64_t pcp_grid_size(const pcp_grid* g) { return g ? g->n : -1; }
int64_t pcp_grid_cells(const pcp_grid* g) { return g ? g->ncell : -1; }
int pcp_grid_points(pcp_ctx* ctx, const pcp_grid* g, void* out_dev, int64_t cap, int64_t* n_out) {
    if (!ctx || !g || !n_out) return PCP_ERR_ARG;
    *n_out = g->n;
    if (!out_dev || g->n == 0) return PCP_OK;
    if (g->n > cap) return set_error(ctx, PCP_ERR_CAPACITY, "pcp_grid_points: %lld points > cap", (long long)g->n);
    PCP_HIP(ctx, hipMemcpyAsync(out_dev, g->pts, 48 * (size_t)g->n, hipMemcpyDeviceToDevice, ctx->stream));
    return PCP_OK;
}

int pcp_grid_add_cloud(pcp_ctx* ctx, pcp_grid* g, const void* cloud_dev, int64_t n) {
    if (!ctx || !g || n < 0 || (n > 0 && !cloud_dev)) return PCP_ERR_ARG;
    if (g->n + n >= ((int64_t)1 << 31)) return set_error(ctx, PCP_ERR_CAPACITY, "CloudGrid: < 2^31 points");
    if (n == 0) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int64_t m = g->n + n;
    Tmp tmp(ctx);
    uint64_t *k0, *k1;
    uint32_t *o0, *o1, *head, *keep;
    int32_t *next, *klist;
    uint8_t* rec;
    PCP_TRY(tmp.get(&k0, m));
    PCP_TRY(tmp.get(&k1, m));
    PCP_TRY(tmp.get(&o0, m));
    PCP_TRY(tmp.get(&o1, m));
    PCP_TRY(tmp.get(&head, m + 1));
    PCP_TRY(tmp.get(&rec, 48 * m));
    hipLaunchKernelGGL(k_grid_keys, dim3(grid_for(m, 256)), dim3(256), 0, st, g->pts, g->n, (const uint8_t*)cloud_dev,
                       n, k0, o0);
    size_t tb = 0;
    PCP_HIP(ctx, rocprim::radix_sort_pairs(nullptr, tb, k0, k1, o0, o1, (size_t)m, 0, 64, st));
    void* sortmem;
    PCP_TRY(tmp.get((char**)&sortmem, tb));
    PCP_HIP(ctx, rocprim::radix_sort_pairs(sortmem, tb, k0, k1, o0, o1, (size_t)m, 0, 64, st));
    hipLaunchKernelGGL(k_grid_gather, dim3(grid_for(m, 256)), dim3(256), 0, st, g->pts, g->n,
                       (const uint8_t*)cloud_dev, o1, m, rec);
    hipLaunchKernelGGL(k_grid_heads, dim3(grid_for(m, 256)), dim3(256), 0, st, k1, m, head);
    uint32_t* hs;
    PCP_TRY(tmp.get(&hs, m + 1));
    PCP_HIP(ctx, hipMemcpyAsync(hs, head, m * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    uint32_t ncell = 0;
    PCP_TRY(scan_u32_inplace(ctx, hs, m, &ncell));
    int64_t* cst;
    uint64_t* ckey;
    PCP_TRY(tmp.get(&cst, (size_t)ncell + 1));
    PCP_TRY(tmp.get(&ckey, ncell));  // every result is guarded until the swap below
    hipLaunchKernelGGL(k_grid_cells, dim3(grid_for(m, 256)), dim3(256), 0, st, k1, hs, head, m, cst, ckey);
    const int64_t mm = m;
    PCP_HIP(ctx, hipMemcpyAsync(cst + ncell, &mm, sizeof(int64_t), hipMemcpyHostToDevice, st));
    // the sequential de-duplication, one wave per cell
    PCP_TRY(tmp.get(&next, m));
    PCP_TRY(tmp.get(&klist, m));
    PCP_TRY(tmp.get(&keep, m + 1));
    hipLaunchKernelGGL(k_grid_dedupe, dim3(grid_for(ncell, 1, 1 << 18)), dim3(64), 0, st, rec, cst, (int64_t)ncell,
                       g->n, o1, next, klist, keep);
    // compaction: kept records and the new cell starts
    PCP_HIP(ctx, hipMemcpyAsync(head, keep, m * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    uint32_t nkeep = 0;
    PCP_TRY(scan_u32_inplace(ctx, head, m, &nkeep));
    uint8_t* pts;
    int64_t* cstart;
    PCP_TRY(tmp.get(&pts, 48 * (size_t)nkeep));
    PCP_TRY(tmp.get(&cstart, (size_t)ncell + 1));
    hipLaunchKernelGGL(k_grid_compact, dim3(grid_for(m, 256)), dim3(256), 0, st, rec, keep, head, m, pts);
    hipLaunchKernelGGL(k_grid_restart, dim3(grid_for(ncell + 1, 256)), dim3(256), 0, st, cst, head, (int64_t)ncell, m,
                       nkeep, cstart);
    PCP_LAUNCH_CHECK(ctx);
    PCP_HIP(ctx, hipStreamSynchronize(st));
    tmp.release(pts);
    tmp.release(ckey);
    tmp.release(cstart);
    dfree(ctx, g->pts);
    dfree(ctx, g->keys);
    dfree(ctx, g->cstart);
    g->pts = pts;
    g->keys = ckey;
    g->cstart = cstart;
    g->n = nkeep;
    g->ncell = ncell;
    return PCP_OK;
}

int pcp_grid_box(pcp_ctx* ctx, const pcp_grid* g, int i0, int i1, int j0, int j1, void* out_dev, int64_t cap,
                 int64_t* n_out) {
    if (!ctx || !g || !n_out) return PCP_ERR_ARG;
    *n_out = 0;
    if (i1 <= i0 || j1 <= j0 || g->ncell == 0) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int nrows = i1 - i0;
    Tmp tmp(ctx);
    int64_t *rlo, *rlen, *roff;
    PCP_TRY(tmp.get(&rlo, nrows));
    PCP_TRY(tmp.get(&rlen, nrows));
    PCP_TRY(tmp.get(&roff, nrows));
    hipLaunchKernelGGL(k_grid_rows, dim3(grid_for(nrows, 256)), dim3(256), 0, st, g->keys, g->cstart, g->ncell, i0,
                       nrows, j0, j1, rlo, rlen);
    std::vector<int64_t> len(nrows), off(nrows);
    PCP_HIP(ctx, hipMemcpyAsync(len.data(), rlen, nrows * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    PCP_HIP(ctx, hipStreamSynchronize(st));
    int64_t total = 0;
    for (int r = 0; r < nrows; r++) {
        off[r] = total;
        total += len[r];
    }
    *n_out = total;
    if (!out_dev) return PCP_OK;  // count only
    if (total > cap) return set_error(ctx, PCP_ERR_CAPACITY, "pcp_grid_box: %lld points > cap", (long long)total);
    if (total == 0) return PCP_OK;
    PCP_HIP(ctx, hipMemcpyAsync(roff, off.data(), nrows * sizeof(int64_t), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_grid_box_copy, dim3(grid_for(total, 256)), dim3(256), 0, st, g->pts, rlo, roff, nrows, total,
                       (uint8_t*)out_dev);
    PCP_LAUNCH_CHECK(ctx);
    PCP_HIP(ctx, hipStreamSynchronize(st));  // off lives on the host stack
    return PCP_OK;
}

int pcp_grid_match(pcp_ctx* ctx, const pcp_grid* g, const void* src_dev, int64_t nsrc, float dis, void* src_out_dev,
                   int64_t* n_src_out, void* dst_dev, int64_t cap, int64_t* n_dst) {
    if (!ctx || !g || nsrc < 0 || (nsrc > 0 && (!src_dev || !src_out_dev)) || !n_src_out || !n_dst)
        return PCP_ERR_ARG;
    *n_src_out = *n_dst = 0;
    if (nsrc >= ((int64_t)1 << 32) - 1) return set_error(ctx, PCP_ERR_CAPACITY, "pcp_grid_match: < 2^32 - 1 sources");
    if (nsrc == 0 || g->ncell == 0) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    Tmp tmp(ctx);
    uint8_t* tall;
    uint32_t *found, *first, *pos, *fpos;
    uint64_t *dk, *dk1;
    PCP_TRY(tmp.get(&tall, g->ncell));
    PCP_TRY(tmp.get(&found, nsrc + 1));
    PCP_TRY(tmp.get(&fpos, nsrc + 1));
    PCP_TRY(tmp.get(&first, g->n));
    PCP_TRY(tmp.get(&pos, g->n + 1));
    hipLaunchKernelGGL(k_grid_zrange, dim3(grid_for(g->ncell, 256)), dim3(256), 0, st, g->pts, g->cstart, g->ncell, tall);
    hipLaunchKernelGGL(k_grid_fill_u32, dim3(grid_for(g->n, 256)), dim3(256), 0, st, first, g->n, 0xffffffffu);
    hipLaunchKernelGGL(k_grid_match, dim3(grid_for(nsrc, 256)), dim3(256), 0, st, g->pts, g->keys, g->cstart, g->ncell,
                       tall, (const uint8_t*)src_dev, nsrc, (double)dis, found, first);
    // src_out: the matched source points in order
    PCP_HIP(ctx, hipMemcpyAsync(fpos, found, nsrc * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    uint32_t ns = 0;
    PCP_TRY(scan_u32_inplace(ctx, fpos, nsrc, &ns));
    hipLaunchKernelGGL(k_grid_compact, dim3(grid_for(nsrc, 256)), dim3(256), 0, st, (const uint8_t*)src_dev, found, fpos,
                       nsrc, (uint8_t*)src_out_dev);
    *n_src_out = ns;
    // dst: matched grid points ordered by (first matching source, position)
    hipLaunchKernelGGL(k_grid_matched, dim3(grid_for(g->n, 256)), dim3(256), 0, st, first, g->n, pos);
    uint32_t nd = 0;
    PCP_TRY(scan_u32_inplace(ctx, pos, g->n, &nd));
    *n_dst = nd;
    if (nd > cap || (nd > 0 && !dst_dev)) return set_error(ctx, PCP_ERR_CAPACITY, "pcp_grid_match: %u dst > cap", nd);
    if (nd == 0) return PCP_OK;
    PCP_TRY(tmp.get(&dk, nd));
    PCP_TRY(tmp.get(&dk1, nd));
    hipLaunchKernelGGL(k_grid_dst_keys, dim3(grid_for(g->n, 256)), dim3(256), 0, st, first, g->n, pos, dk);
    size_t tb = 0;
    PCP_HIP(ctx, rocprim::radix_sort_keys(nullptr, tb, dk, dk1, (size_t)nd, 0, 64, st));
    void* sortmem;
    PCP_TRY(tmp.get((char**)&sortmem, tb));
    PCP_HIP(ctx, rocprim::radix_sort_keys(sortmem, tb, dk, dk1, (size_t)nd, 0, 64, st));
    hipLaunchKernelGGL(k_grid_gather_sorted, dim3(grid_for(nd, 256)), dim3(256), 0, st, g->pts, dk1, (int64_t)nd,
                       (uint8_t*)dst_dev);
    PCP_LAUNCH_CHECK(ctx);
    PCP_HIP(ctx, hipStreamSynchronize(st));
    return PCP_OK;
}

}  // extern "C"
