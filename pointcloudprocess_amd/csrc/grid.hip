// Uniform-grid index build (replaces KdTreeFLANN::setInputCloud, kd_tree.h:772-798,
// and the trimesh2 KDtree constructions at point_cloud_helper.cpp:110-111).
//
// Build = compaction of finite points (index_mapping_) -> bbox -> brick marking (sparse
// mode) -> per-point cell keys -> stable device radix sort of (cell, point) -> per-cell
// counts from the sorted runs -> cell-start scan -> gather into cell order.  Within a cell
// points keep input order, so the layout is deterministic.  All passes are HBM streams;
// the only host round trips are the bbox (to size the tables) and the slot count.
#include <cmath>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include "sortcfg.hpp"

#include "grid.hpp"

namespace pcp {
namespace {

constexpr int kB = 256;

template <typename T>
__device__ __forceinline__ const T* pt_ptr(const T* base, size_t stride_bytes, int64_t i) {
    return (const T*)((const char*)base + (size_t)i * stride_bytes);
}

// validity flags of the (optionally indexed) input
template <typename T>
__global__ void k_valid(const T* xyz, size_t stride, int64_t n_in, const int32_t* indices,
                        uint32_t* flag) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_in;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t ci = indices ? indices[i] : i;
        const T* p = pt_ptr(xyz, stride, ci);
        flag[i] = (isfinite((double)p[0]) && isfinite((double)p[1]) && isfinite((double)p[2])) ? 1u : 0u;
    }
}

// compaction: internal j = exclusive prefix of the flags (convertCloudToArray order)
template <typename T>
__global__ void k_compact(const T* xyz, size_t stride, int64_t n_in, const int32_t* indices,
                          const uint32_t* pos, const uint32_t* flagbits, T* cxyz, int32_t* mapping) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_in;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (!((flagbits[i >> 5] >> (i & 31)) & 1u)) continue;
        int64_t ci = indices ? indices[i] : i;
        const T* p = pt_ptr(xyz, stride, ci);
        uint32_t j = pos[i];
        cxyz[3 * (int64_t)j + 0] = p[0];
        cxyz[3 * (int64_t)j + 1] = p[1];
        cxyz[3 * (int64_t)j + 2] = p[2];
        mapping[j] = (int32_t)ci;
    }
}

// flags -> bitmask (bit i of word i/32): one coalesced flag per lane, a wave ballot per 64
__global__ void k_pack_bits(const uint32_t* flag, int64_t n, uint32_t* bits) {
    const int64_t base = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) & ~(int64_t)63;
    const int64_t i = base + (threadIdx.x & 63);
    const uint64_t m = __ballot(i < n && flag[i] != 0u);
    const int lane = threadIdx.x & 63;
    if (lane < 2 && base + 32 * lane < n) bits[(base >> 5) + lane] = (uint32_t)(m >> (32 * lane));
}

template <typename T>
__global__ void k_minmax(const T* cxyz, int64_t n, double* part) {
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        for (int a = 0; a < 3; a++) {
            double v = (double)cxyz[3 * i + a];
            mn[a] = fmin(mn[a], v);
            mx[a] = fmax(mx[a], v);
        }
    }
    __shared__ double s[6][kB];
    for (int a = 0; a < 3; a++) { s[a][threadIdx.x] = mn[a]; s[3 + a][threadIdx.x] = mx[a]; }
    __syncthreads();
    for (int w = kB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int a = 0; a < 3; a++) {
                s[a][threadIdx.x] = fmin(s[a][threadIdx.x], s[a][threadIdx.x + w]);
                s[3 + a][threadIdx.x] = fmax(s[3 + a][threadIdx.x], s[3 + a][threadIdx.x + w]);
            }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int a = 0; a < 6; a++) part[blockIdx.x * 6 + a] = s[a][0];
}

// one pass over the caller's cloud: bbox of the finite points + the number of non-finite ones
// (the fp32 build skips the compaction when that number is 0)
template <typename T>
__global__ void k_bbox_count(const T* xyz, size_t stride, int64_t n, double* part, unsigned long long* bad) {
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    unsigned nb = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const T* p = pt_ptr(xyz, stride, i);
        const double v[3] = {(double)p[0], (double)p[1], (double)p[2]};
        if (!(isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2]))) { nb++; continue; }
        for (int a = 0; a < 3; a++) {
            mn[a] = fmin(mn[a], v[a]);
            mx[a] = fmax(mx[a], v[a]);
        }
    }
    __shared__ double s[6][kB];
    for (int a = 0; a < 3; a++) { s[a][threadIdx.x] = mn[a]; s[3 + a][threadIdx.x] = mx[a]; }
    __syncthreads();
    for (int w = kB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int a = 0; a < 3; a++) {
                s[a][threadIdx.x] = fmin(s[a][threadIdx.x], s[a][threadIdx.x + w]);
                s[3 + a][threadIdx.x] = fmax(s[3 + a][threadIdx.x], s[3 + a][threadIdx.x + w]);
            }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int a = 0; a < 6; a++) part[blockIdx.x * 6 + a] = s[a][0];
    for (int o = 32; o > 0; o >>= 1) nb += __shfl_xor(nb, o, 64);
    if ((threadIdx.x & 63) == 0 && nb) atomicAdd(bad, (unsigned long long)nb);
}

template <typename T>
__device__ __forceinline__ void cell_of_point(const GridDesc& g, const T* p, int& cx, int& cy, int& cz) {
    cx = clampi(cell_i<T>(g, p[0], 0), 0, g.n[0] - 1);
    cy = clampi(cell_i<T>(g, p[1], 1), 0, g.n[1] - 1);
    cz = clampi(cell_i<T>(g, p[2], 2), 0, g.n[2] - 1);
}

// points stride_t values apart: the compacted array (3) or the caller's all-finite cloud
template <typename T>
__global__ void k_mark(GridDesc g, const T* cxyz, size_t stride_t, int64_t n, int32_t* brick) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int cx, cy, cz;
        cell_of_point<T>(g, cxyz + stride_t * i, cx, cy, cz);
        brick[brick_of(g, cx, cy, cz)] = 1;
    }
}

// dense mode: brick occupancy for the two-level ring search (0 = occupied, -1 = empty)
__global__ void k_brick_flag(int32_t* brick, int64_t nb) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nb;
         i += (int64_t)gridDim.x * blockDim.x)
        brick[i] = brick[i] ? 0 : -1;
}

// dense fp64 grids, after the cell starts: an occupied brick's word becomes the mask of its
// 16 (y, z) cell rows that hold points (bit yo | zo << 2, >= 1), so the far pass visits only
// those rows instead of one cstart round trip per row; empty bricks stay -1
__global__ void k_brick_rows(GridDesc g, int32_t* brick) {
    const int64_t nb = (int64_t)g.nb[0] * g.nb[1] * g.nb[2];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nb;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (brick[i] < 0) continue;
        const int xb = (int)(i % g.nb[0]), yb = (int)((i / g.nb[0]) % g.nb[1]), zb = (int)(i / ((int64_t)g.nb[0] * g.nb[1]));
        const int x0 = 4 * xb, x1 = min(4 * xb + 3, g.n[0] - 1);
        uint32_t st[16], en[16];
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int y = 4 * yb + (r & 3), z = 4 * zb + (r >> 2);
            const bool in = y < g.n[1] && z < g.n[2];
            st[r] = in ? g.cstart[dense_id(g, x0, y, z)] : 0u;
            en[r] = in ? g.cstart[dense_id(g, x1, y, z) + 1] : 0u;
        }
        int32_t m = 0;
#pragma unroll
        for (int r = 0; r < 16; r++) m |= en[r] > st[r] ? (1 << r) : 0;
        brick[i] = m;
    }
}

__global__ void k_brick_bits(const int32_t* brick, int64_t nb, uint32_t* bits) {
    int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (w >= (nb + 31) / 32) return;
    uint32_t v = 0;
    for (int b = 0; b < 32; b++) {
        int64_t i = w * 32 + b;
        if (i < nb && brick[i] != 0) v |= 1u << b;
    }
    bits[w] = v;
}

__global__ void k_brick_final(int32_t* brick, int64_t nb, const uint32_t* bits) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nb;
         i += (int64_t)gridDim.x * blockDim.x) {
        bool on = (bits[i >> 5] >> (i & 31)) & 1u;
        brick[i] = on ? brick[i] : -1;  // brick[] holds the exclusive prefix = slot id
    }
}

// Cell starts without a count array or a scan.  cstart[c] = first sorted position whose key
// is >= c, c in [0, ncells].  The cells are cut into chunks of kChunk; k_chunk_lo finds each
// chunk's first position from the run starts (a run start fills the chunk boundaries of the
// key gap before it; p = n is a virtual run start closing the table); k_cell_starts then resolves one chunk per
// block in LDS (run starts scattered, suffix minimum) and writes it out coalesced.
constexpr int kChunk = 4096;
// grids of the streaming passes over every point (bbox, chunk bounds): enough waves in flight per
// CU to cover the loads' latency (at 1024 blocks the 200M-point passes ran at 1-4 TB/s)
#ifndef PCP_SCAN_BLOCKS
#define PCP_SCAN_BLOCKS 16384
#endif
#ifndef PCP_BBOX_BLOCKS
#define PCP_BBOX_BLOCKS 4096
#endif
constexpr int64_t kScanBlocks = PCP_SCAN_BLOCKS;
constexpr int64_t kBboxBlocks = PCP_BBOX_BLOCKS;

__global__ void k_chunk_lo(const uint32_t* key, int64_t n, int64_t nchunk, uint32_t* lo) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p <= n; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t kc = p < n ? (int64_t)key[p] : nchunk * kChunk;
        const int64_t kp = p > 0 ? (int64_t)key[p - 1] : -1;
        if (kc == kp) continue;
        const int64_t b0 = kp < 0 ? 0 : kp / kChunk + 1;  // chunks whose first cell is in (kp, kc]
        const int64_t b1 = min(kc / kChunk, nchunk);
        for (int64_t b = b0; b <= b1; b++) lo[b] = (uint32_t)p;
    }
}

__global__ void __launch_bounds__(256) k_cell_starts(const uint32_t* __restrict__ key, const uint32_t* __restrict__ lo,
                                                     int64_t ncells1, uint32_t* __restrict__ cstart) {
    constexpr int kPer = kChunk / 256;  // 16 cells per thread
    __shared__ uint32_t s[kChunk];
    __shared__ uint32_t s_wmin[4];
    const int64_t c0 = (int64_t)blockIdx.x * kChunk;
    const uint32_t p0 = lo[blockIdx.x], p1 = lo[blockIdx.x + 1];
    for (int i = threadIdx.x; i < kChunk; i += 256) s[i] = p1;
    __syncthreads();
    for (uint32_t p = p0 + threadIdx.x; p < p1; p += 256) {
        const uint32_t k = key[p];
        if (p == p0 || k != key[p - 1]) s[k - c0] = p;
    }
    __syncthreads();
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    uint32_t v[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j += 4) {
        const uint4 u = *(const uint4*)&s[kPer * t + j];
        v[j] = u.x; v[j + 1] = u.y; v[j + 2] = u.z; v[j + 3] = u.w;
    }
#pragma unroll
    for (int j = kPer - 2; j >= 0; j--) v[j] = min(v[j], v[j + 1]);
    // minimum over the threads after this one
    uint32_t x = v[0];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_down(x, o, 64);
        if (lane + o < 64) x = min(x, y);
    }
    if (lane == 0) s_wmin[wid] = x;
    uint32_t after = __shfl_down(x, 1, 64);
    if (lane == 63) after = p1;
    __syncthreads();
    for (int w = wid + 1; w < 4; w++) after = min(after, s_wmin[w]);
    // back through LDS, so every 16-byte store instruction of a wave covers 1 KB contiguously
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPer; j += 4)
        *(uint4*)&s[kPer * t + j] = make_uint4(min(v[j], after), min(v[j + 1], after), min(v[j + 2], after),
                                               min(v[j + 3], after));
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer / 4; k++) {
        const int e = 4 * (k * 256 + t);  // element offset in the chunk
        const uint4 o = *(const uint4*)&s[e];
        const int64_t c = c0 + e;
        if (c + 3 < ncells1) {
            *(uint4*)&cstart[c] = o;
        } else {
            if (c < ncells1) cstart[c] = o.x;
            if (c + 1 < ncells1) cstart[c + 1] = o.y;
            if (c + 2 < ncells1) cstart[c + 2] = o.z;
        }
    }
}

// fp32 build: sort key + the point record {x, y, z, caller index bits} as the sort payload
// the fp32 index's pts[n]: +inf coordinates, index INT_MAX -- a gather target that never wins
__global__ void k_far_sentinel(float4* pts, int64_t n) {
    pts[n] = make_float4(INFINITY, INFINITY, INFINITY, __int_as_float(0x7fffffff));
}

// mapping == null: the points are the caller's cloud itself (all finite, stride_f floats apart)
__global__ void k_cell_keys_rec(GridDesc g, const float* cxyz, size_t stride_f, const int32_t* mapping, int64_t n,
                                uint32_t* key, float4* rec, int32_t* mark) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float* p = cxyz + stride_f * i;
        int cx, cy, cz;
        cell_of_point<float>(g, p, cx, cy, cz);
        key[i] = (uint32_t)cell_id(g, cx, cy, cz);
        rec[i] = make_float4(p[0], p[1], p[2], __int_as_float(mapping ? mapping[i] : (int32_t)i));
        if (mark) mark[brick_of(g, cx, cy, cz)] = 1;
    }
}


// Radix-sort build: key = cell id (cstart index) of each compacted point, value = its
// internal index.  A stable LSD sort then yields cell order with ties in input order
// (deterministic); dense mode also flags the point's brick for the two-level search.
template <typename T>
__global__ void k_cell_keys(GridDesc g, const T* cxyz, size_t stride_t, int64_t n, uint32_t* key, uint32_t* val,
                            int32_t* mark) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int cx, cy, cz;
        cell_of_point<T>(g, cxyz + stride_t * i, cx, cy, cz);
        key[i] = (uint32_t)cell_id(g, cx, cy, cz);
        val[i] = (uint32_t)i;
        if (mark) mark[brick_of(g, cx, cy, cz)] = 1;
    }
}

// The automatic cell size's occupancy probe: the number of non-empty cells of geometry g
// without sorting -- every point stores a 1 into its cell's byte of a flag array (plain byte
// stores: every writer stores the same value, and a bitmap's atomics serialised on the few
// words a row of cells shares; a lane whose cell equals the previous lane's skips its store),
// then k_count_flags sums the bytes.  The same count as the runs of the sorted keys.
template <typename T>
__global__ void k_cell_flags(GridDesc g, const T* cxyz, size_t stride_t, int64_t n, uint8_t* flags) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int cx, cy, cz;
        cell_of_point<T>(g, cxyz + stride_t * i, cx, cy, cz);
        const uint32_t k = (uint32_t)cell_id(g, cx, cy, cz);
        const uint32_t prev = (uint32_t)__shfl_up((int)k, 1, 64);
        if ((threadIdx.x & 63) == 0 || prev != k) flags[k] = 1;
    }
}
// nv 16-byte vectors of 0/1 bytes
__global__ void k_count_flags(const uint4* flags, int64_t nv, unsigned long long* count) {
    __shared__ unsigned long long s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    unsigned long long c = 0;
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nv; w += (int64_t)gridDim.x * blockDim.x) {
        const uint4 v = flags[w];
        c += (unsigned)(__popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w));
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&s_cnt, c);
    __syncthreads();
    if (threadIdx.x == 0 && s_cnt) atomicAdd(count, s_cnt);
}

// points in cell order: w = internal j (fp64, FLANN tie order) or caller index bits (fp32)
template <typename T>
__global__ void k_gather(const T* cxyz, size_t stride_t, const uint32_t* val, const int32_t* mapping, int64_t n,
                         typename Real<T>::V4* pts, int32_t* sorted_j, int is_f64) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t i = val[k];
        const T* p = cxyz + stride_t * i;
        typename Real<T>::V4 v;
        v.x = p[0]; v.y = p[1]; v.z = p[2];
        if (is_f64) v.w = (T)(double)i;
        else v.w = (T)__int_as_float(mapping[i]);
        pts[k] = v;
        sorted_j[k] = (int32_t)i;
    }
}

__global__ void k_inverse(const int32_t* sorted_j, int64_t n, int32_t* pos_of_j) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x)
        pos_of_j[sorted_j[k]] = (int32_t)k;
}

// Grid geometry for a cell size.  Returns false when the brick table would exceed the cap.
bool make_geometry(GridDesc& g, const double mn[3], const double mx[3], double h, int64_t cap) {
    g.h = h;
    g.inv_h = 1.0 / h;
    g.hf = (float)h;
    g.inv_hf = (float)(1.0 / h);
    int64_t nb = 1;
    for (int a = 0; a < 3; a++) {
        g.o[a] = mn[a];
        g.of[a] = (float)mn[a];
        double ext = (mx[a] - mn[a]) / h;
        if (!(ext < 4.0e8)) return false;
        int64_t na = (int64_t)std::floor(ext) + 2;  // +1 for the max point, +1 guard for rounding
        g.n[a] = (int)na;
        g.nb[a] = (int)((na + 3) / 4);
        nb *= g.nb[a];
        if (nb > cap) return false;
    }
    g.nbricks = nb;
    return true;
}

template <typename T>
int build_impl(pcp_ctx* ctx, const T* xyz, size_t stride, int64_t n_in, const int32_t* indices,
               double cell_size, int is_f64, pcp_index** out, bool force_sparse = false,
               const GeomHook* on_geom = nullptr) {
    if (!ctx || !out || n_in < 0 || (n_in > 0 && !xyz)) return PCP_ERR_ARG;
    if (n_in >= (int64_t)1 << 31) return set_error(ctx, PCP_ERR_ARG, "index supports < 2^31 points");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    pcp_index* ix = new pcp_index();
    ix->is_f64 = is_f64;
    ix->owner = ctx;
    ctx_retain(ctx);
    ix->n_in = n_in;
    auto fail = [&](int rc) { pcp_index_destroy(ix); return rc; };

    int rc;
    T* cxyz = nullptr;
    double mn[3] = {0, 0, 0}, mx[3] = {0, 0, 0};
    // ---- bbox + non-finite count in one pass; an all-finite cloud without an indices subset is
    // keyed and gathered straight from the caller's array (no compaction: the identity mapping,
    // which the compaction of an all-finite cloud would produce)
    bool direct = false, have_bbox = false;
    if (!indices && n_in > 0 && stride % sizeof(T) == 0) {
        const unsigned nbk = grid_for(n_in, kB, kBboxBlocks);
        double* part = nullptr;
        unsigned long long* d_bad = nullptr;
        if ((rc = dmalloc(ctx, &part, 6 * (size_t)nbk)) || (rc = dmalloc(ctx, &d_bad, 1))) {
            dfree(ctx, part);
            return fail(rc);
        }
        hipError_t e = hipMemsetAsync(d_bad, 0, sizeof(unsigned long long), st);
        hipLaunchKernelGGL(k_bbox_count<T>, dim3(nbk), dim3(kB), 0, st, xyz, stride, n_in, part, d_bad);
        std::vector<double> hp(6 * nbk);
        unsigned long long bad = 0;
        if (e == hipSuccess) e = hipMemcpyAsync(hp.data(), part, hp.size() * sizeof(double), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        dfree(ctx, part);
        dfree(ctx, d_bad);
        if (e != hipSuccess) return fail(hip_fail(ctx, e, "bbox", __FILE__, __LINE__));
        if (bad < (unsigned long long)n_in) {  // the bbox of the finite points = the compacted cloud's
            have_bbox = true;
            for (int a = 0; a < 3; a++) { mn[a] = INFINITY; mx[a] = -INFINITY; }
            for (unsigned b = 0; b < nbk; b++)
                for (int a = 0; a < 3; a++) {
                    mn[a] = std::fmin(mn[a], hp[6 * b + a]);
                    mx[a] = std::fmax(mx[a], hp[6 * b + 3 + a]);
                }
        }
        if (bad == 0) {
            direct = true;
            ix->n = n_in;
            ix->identity = 1;
        }
    }
    // ---- compaction (convertCloudToArray)
    uint32_t* flag = nullptr;
    uint32_t* bits = nullptr;
    const int64_t nw = (n_in + 31) / 32;
    if (!direct) {
        if ((rc = dmalloc(ctx, &flag, n_in + 1)) || (rc = dmalloc(ctx, &bits, nw + 1))) {
            dfree(ctx, flag); dfree(ctx, bits);
            return fail(rc);
        }
        uint32_t nvalid = 0;
        if (n_in > 0) {
            hipLaunchKernelGGL(k_valid<T>, dim3(grid_for(n_in, kB)), dim3(kB), 0, st, xyz, stride, n_in, indices, flag);
            hipLaunchKernelGGL(k_pack_bits, dim3((unsigned)((n_in + kB - 1) / kB)), dim3(kB), 0, st, flag, n_in, bits);
            rc = scan_u32_inplace(ctx, flag, n_in, &nvalid);
            if (rc) { dfree(ctx, flag); dfree(ctx, bits); return fail(rc); }
        }
        ix->n = nvalid;
        ix->identity = (indices == nullptr && (int64_t)nvalid == n_in) ? 1 : 0;
        if ((rc = dmalloc(ctx, &cxyz, 3 * (size_t)(nvalid + 1))) || (rc = dmalloc(ctx, &ix->mapping, nvalid + 1))) {
            dfree(ctx, flag); dfree(ctx, bits); dfree(ctx, cxyz);
            return fail(rc);
        }
        if (n_in > 0)
            hipLaunchKernelGGL(k_compact<T>, dim3(grid_for(n_in, kB)), dim3(kB), 0, st, xyz, stride, n_in,
                               indices, flag, bits, cxyz, ix->mapping);
        dfree(ctx, flag);
        dfree(ctx, bits);  // cached: reuse is stream-ordered on ctx's stream
    }
    const int64_t n = ix->n;

    // ---- bbox (of an indices subset)
    if (n > 0 && !have_bbox) {
        const unsigned nbk = grid_for(n, kB, kBboxBlocks);
        double* part;
        if ((rc = dmalloc(ctx, &part, 6 * (size_t)nbk))) { dfree(ctx, cxyz); return fail(rc); }
        hipLaunchKernelGGL(k_minmax<T>, dim3(nbk), dim3(kB), 0, st, cxyz, n, part);
        std::vector<double> hp(6 * nbk);
        hipMemcpyAsync(hp.data(), part, hp.size() * sizeof(double), hipMemcpyDeviceToHost, st);
        hipError_t e = hipStreamSynchronize(st);
        dfree(ctx, part);
        if (e != hipSuccess) { dfree(ctx, cxyz); return fail(hip_fail(ctx, e, "bbox", __FILE__, __LINE__)); }
        for (int a = 0; a < 3; a++) { mn[a] = INFINITY; mx[a] = -INFINITY; }
        for (unsigned b = 0; b < nbk; b++)
            for (int a = 0; a < 3; a++) {
                mn[a] = std::fmin(mn[a], hp[6 * b + a]);
                mx[a] = std::fmax(mx[a], hp[6 * b + 3 + a]);
            }
    }

    // ---- cell size: given, or a density estimate refined once from the measured occupancy
    const int64_t cap = std::max<int64_t>((int64_t)1 << 24, 8 * n);
    // dense cell table budget: up to 16 cells per point (<= 6.4 GB for 100M points), < 2^31
    const int64_t dense_cap = std::min<int64_t>(((int64_t)1 << 31) - 2, std::max<int64_t>((int64_t)1 << 26, 16 * n));
    double ext[3];
    for (int a = 0; a < 3; a++) ext[a] = std::max(mx[a] - mn[a], 1e-9);
    const bool auto_h = !(cell_size > 0);
    double h = cell_size;
    if (auto_h) {
        const double target = 4.0;  // points per non-empty cell
        h = std::cbrt(ext[0] * ext[1] * ext[2] * target / std::max<double>((double)n, 1.0));
        double emax = std::max(ext[0], std::max(ext[1], ext[2]));
        if (!(h > emax * 1e-7)) h = emax * 1e-7;
        if (!(h > 0)) h = 1.0;
    }
    uint32_t* count = nullptr;
    uint32_t* rank = nullptr;  // sort input values (point index)
    uint32_t* skey = nullptr;  // sort input keys (cell id)
    if ((is_f64 && (rc = dmalloc(ctx, &rank, n + 1))) || (rc = dmalloc(ctx, &skey, n + 1))) {
        dfree(ctx, rank);
        dfree(ctx, cxyz);
        return fail(rc);
    }
    if ((rc = dmalloc(ctx, (typename Real<T>::V4**)&ix->pts, n + 1))) {
        dfree(ctx, rank); dfree(ctx, skey); dfree(ctx, cxyz);
        return fail(rc);
    }
    bool hooked = false;
    for (int attempt = 0; attempt < 3; attempt++) {
        GridDesc g{};
        while (!make_geometry(g, mn, mx, h, cap)) h *= 2.0;
        dfree(ctx, ix->brick); ix->brick = nullptr;
        dfree(ctx, count); count = nullptr;
        const int64_t ncells_dense = (int64_t)g.n[0] * g.n[1] * g.n[2];
        g.dense = (!force_sparse && ncells_dense <= dense_cap) ? 1 : 0;
        g.ncells = ncells_dense;
        int64_t ncells;
        if (g.dense) {
            ncells = ncells_dense;
            g.nslots = 0;
            if ((rc = dmalloc(ctx, &ix->brick, g.nbricks))) break;
            PCP_HIP(ctx, hipMemsetAsync(ix->brick, 0, (size_t)g.nbricks * sizeof(int32_t), st));
            g.brick = ix->brick;  // marked by k_count, turned into 0 / -1 flags below
        } else {
            if ((rc = dmalloc(ctx, &ix->brick, g.nbricks))) break;
            PCP_HIP(ctx, hipMemsetAsync(ix->brick, 0, (size_t)g.nbricks * sizeof(int32_t), st));
            if (n > 0)  // the direct (uncompacted) fp32 path keys the caller's cloud in place
                hipLaunchKernelGGL(k_mark<T>, dim3(grid_for(n, kB)), dim3(kB), 0, st, g, direct ? xyz : cxyz,
                                   direct ? stride / sizeof(T) : (size_t)3, n, ix->brick);
            const int64_t nbw = (g.nbricks + 31) / 32;
            uint32_t* bbits;
            if ((rc = dmalloc(ctx, &bbits, nbw + 1))) break;
            hipLaunchKernelGGL(k_brick_bits, dim3(grid_for(nbw, kB)), dim3(kB), 0, st, ix->brick, g.nbricks, bbits);
            uint32_t nslots = 0;
            rc = scan_u32_inplace(ctx, (uint32_t*)ix->brick, g.nbricks, &nslots);
            if (rc) { dfree(ctx, bbits); break; }
            hipLaunchKernelGGL(k_brick_final, dim3(grid_for(g.nbricks, kB)), dim3(kB), 0, st, ix->brick, g.nbricks, bbits);
            dfree(ctx, bbits);
            g.nslots = nslots;
            g.brick = ix->brick;
            ncells = (int64_t)nslots * 64;
        }
        if (auto_h && attempt < 2 && n > 0) {
            // the automatic cell size, refined from this geometry's measured occupancy before
            // any sort (a count of the non-empty cells by byte flags)
            const int64_t nv = (ncells + 15) / 16;  // 16-byte vectors of cell flags
            uint4* cflag = nullptr;
            unsigned long long* d_ne = nullptr;
            if ((rc = dmalloc(ctx, &cflag, nv)) || (rc = dmalloc(ctx, &d_ne, 1))) { dfree(ctx, cflag); break; }
            hipError_t e = hipMemsetAsync(cflag, 0, (size_t)nv * sizeof(uint4), st);
            if (e == hipSuccess) e = hipMemsetAsync(d_ne, 0, sizeof(unsigned long long), st);
            hipLaunchKernelGGL(k_cell_flags<T>, dim3(grid_for(n, kB)), dim3(kB), 0, st, g, direct ? xyz : cxyz,
                               direct ? stride / sizeof(T) : (size_t)3, n, (uint8_t*)cflag);
            hipLaunchKernelGGL(k_count_flags, dim3(grid_for(nv, kB, 1024)), dim3(kB), 0, st, cflag, nv, d_ne);
            unsigned long long ne = 0;
            if (e == hipSuccess) e = hipMemcpyAsync(&ne, d_ne, sizeof(ne), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            dfree(ctx, cflag);
            dfree(ctx, d_ne);
            if (e != hipSuccess) { rc = hip_fail(ctx, e, "occupancy", __FILE__, __LINE__); break; }
            const double occ = (double)n / std::max(1.0, (double)ne);
            bool redo = false;
            if (occ > 12.0) { h *= std::sqrt(4.0 / occ); redo = true; }   // surface-like data
            else if (occ < 1.5) { h *= std::cbrt(4.0 / occ); redo = true; }  // sparser than assumed
            if (redo) continue;
        }
        if (on_geom && *on_geom && !hooked) {  // the geometry is final (a given cell size, or the
            hooked = true;                      // refinement is done): let the caller start work
            if ((rc = (*on_geom)(g))) break;    // that needs only it (overlaps the sort)
        }
        // + 1 pad entry: the ICP octant pass loads a row's starts as one 3-word vector at the row's
        // first cell, whose third word lies one past the table for a 1-cell row at the last cell
        if ((rc = dmalloc(ctx, &count, ncells + 2))) break;
        // ---- stable radix sort by cell id.  fp32: the payload is the point record itself, so
        // the sort output is the cell-ordered point array (no gather).  fp64: the payload is the
        // internal j (FLANN tie order), gathered below.
        uint32_t* key1 = nullptr;
        uint32_t* val1 = nullptr;
        using V4 = typename Real<T>::V4;
        if (n > 0) {
            if ((rc = dmalloc(ctx, &key1, n))) break;
            if (is_f64 && (rc = dmalloc(ctx, &val1, n))) { dfree(ctx, key1); break; }
            float4* rec0 = nullptr;
            if (!is_f64 && (rc = dmalloc(ctx, &rec0, n))) { dfree(ctx, key1); break; }
            unsigned bits = 1;
            while (bits < 32 && ((uint64_t)1 << bits) <= (uint64_t)ncells) bits++;
            size_t tmp_bytes = 0;
            void* tmp = nullptr;
            if (is_f64) {
                hipLaunchKernelGGL(k_cell_keys<T>, dim3(grid_for(n, kB)), dim3(kB), 0, st, g, direct ? xyz : cxyz,
                                   direct ? stride / sizeof(T) : (size_t)3, n, skey, rank, g.dense ? ix->brick : nullptr);
                PCP_HIP(ctx, rocprim::radix_sort_pairs(nullptr, tmp_bytes, skey, key1, rank, val1, (size_t)n, 0u,
                                                       bits, st));
                if (!(rc = dmalloc(ctx, (char**)&tmp, tmp_bytes)))
                    PCP_HIP(ctx, rocprim::radix_sort_pairs(tmp, tmp_bytes, skey, key1, rank, val1, (size_t)n, 0u,
                                                           bits, st));
            } else {
                // no brick marks: the fp32 index serves ICP only, whose dense-grid searches never
                // read brick occupancy (its brick table stays all-zero = "occupied")
                if (direct)
                    hipLaunchKernelGGL(k_cell_keys_rec, dim3(grid_for(n, kB)), dim3(kB), 0, st, g, (const float*)xyz,
                                       stride / sizeof(float), (const int32_t*)nullptr, n, skey, rec0, nullptr);
                else
                    hipLaunchKernelGGL(k_cell_keys_rec, dim3(grid_for(n, kB)), dim3(kB), 0, st, g, (const float*)cxyz,
                                       (size_t)3, (const int32_t*)ix->mapping, n, skey, rec0, nullptr);
                PCP_HIP(ctx, rocprim::radix_sort_pairs<RecSortConfig>(nullptr, tmp_bytes, skey, key1, rec0, (float4*)ix->pts,
                                                       (size_t)n, 0u, bits, st));
                if (!(rc = dmalloc(ctx, (char**)&tmp, tmp_bytes)))
                    PCP_HIP(ctx, rocprim::radix_sort_pairs<RecSortConfig>(tmp, tmp_bytes, skey, key1, rec0, (float4*)ix->pts,
                                                           (size_t)n, 0u, bits, st));
            }
            dfree(ctx, tmp);
            dfree(ctx, rec0);
            if (rc) { dfree(ctx, key1); dfree(ctx, val1); break; }
            if (!is_f64)  // pts[n]: a point at infinity (d2 = inf from any finite query) for gathers
                hipLaunchKernelGGL(k_far_sentinel, dim3(1), dim3(1), 0, st, (float4*)ix->pts, n);
        }
        if (g.dense && is_f64)
            hipLaunchKernelGGL(k_brick_flag, dim3(grid_for(g.nbricks, kB)), dim3(kB), 0, st, ix->brick, g.nbricks);
        // ---- chunk boundaries of the sorted keys
        const int64_t nchunk = (ncells + 1 + kChunk - 1) / kChunk;
        uint32_t* lo = nullptr;
        if ((rc = dmalloc(ctx, &lo, nchunk + 1))) {
            dfree(ctx, key1); dfree(ctx, val1);
            break;
        }
        hipLaunchKernelGGL(k_chunk_lo, dim3(grid_for(n + 1, kB, kScanBlocks)), dim3(kB), 0, st, (const uint32_t*)key1, n,
                           nchunk, lo);
        // ---- cell starts straight from the sorted keys (no count array, no scan)
        hipLaunchKernelGGL(k_cell_starts, dim3((unsigned)nchunk), dim3(kB), 0, st, (const uint32_t*)key1,
                           (const uint32_t*)lo, ncells + 1, count);
        dfree(ctx, lo);
        g.cstart = count;
        if (g.dense && is_f64 && n > 0)
            hipLaunchKernelGGL(k_brick_rows, dim3(grid_for(g.nbricks, kB)), dim3(kB), 0, st, g, ix->brick);
        ix->g = g;
        ix->cstart = count;
        count = nullptr;
        if (is_f64) {
            if ((rc = dmalloc(ctx, &ix->sorted_j, n + 1))) { dfree(ctx, key1); dfree(ctx, val1); break; }
            if (n > 0)
                hipLaunchKernelGGL(k_gather<T>, dim3(grid_for(n, kB)), dim3(kB), 0, st, direct ? xyz : cxyz,
                                   direct ? stride / sizeof(T) : (size_t)3, (const uint32_t*)val1,
                                   (const int32_t*)ix->mapping, n, (V4*)ix->pts, ix->sorted_j, is_f64);
        }
        dfree(ctx, key1);
        dfree(ctx, val1);
        if (is_f64) {
            if ((rc = dmalloc(ctx, &ix->pos_of_j, n + 1))) break;
            if (n > 0)
                hipLaunchKernelGGL(k_inverse, dim3(grid_for(n, kB)), dim3(kB), 0, st,
                                   (const int32_t*)ix->sorted_j, n, ix->pos_of_j);
        }
        break;
    }
    dfree(ctx, count);
    dfree(ctx, rank);
    dfree(ctx, skey);
    dfree(ctx, cxyz);
    if (!rc && on_geom && *on_geom && !hooked) rc = (*on_geom)(ix->g);  // (not reached: the loop hooks before its sort)
    if (rc) return fail(rc);
    PCP_HIP(ctx, hipGetLastError());
    PCP_HIP(ctx, hipStreamSynchronize(st));
    *out = ix;
    return PCP_OK;
}

}  // namespace

int index_build_f32_hooked(pcp_ctx* ctx, const float* xyz, size_t stride, int64_t n, double cell_size,
                           pcp_index** out, const GeomHook& on_geom) {
    if (stride == 0) stride = 3 * sizeof(float);
    return build_impl<float>(ctx, xyz, stride, n, nullptr, cell_size, 0, out, false, &on_geom);
}

}  // namespace pcp

extern "C" {

int pcp_index_build_f64(pcp_ctx* ctx, const double* xyz, size_t stride, int64_t n,
                        const int32_t* indices, int64_t n_indices, double cell_size, pcp_index** out) {
    if (stride == 0) stride = 3 * sizeof(double);
    return pcp::build_impl<double>(ctx, xyz, stride, indices ? n_indices : n, indices, cell_size, 1, out);
}

int pcp_index_build_f32(pcp_ctx* ctx, const float* xyz, size_t stride, int64_t n, double cell_size,
                        pcp_index** out) {
    if (stride == 0) stride = 3 * sizeof(float);
    return pcp::build_impl<float>(ctx, xyz, stride, n, nullptr, cell_size, 0, out);
}

int pcp_index_destroy(pcp_index* ix) {
    if (!ix) return PCP_ERR_ARG;
    if (ix->owner) (void)hipSetDevice(ix->owner->device);
    pcp::dfree(ix->owner, ix->brick);
    pcp::dfree(ix->owner, ix->cstart);
    pcp::dfree(ix->owner, ix->pts);
    pcp::dfree(ix->owner, ix->mapping);
    pcp::dfree(ix->owner, ix->sorted_j);
    pcp::dfree(ix->owner, ix->pos_of_j);
    pcp::dfree(ix->owner, ix->h16);
    pcp::dfree(ix->owner, ix->cell);
    pcp_ctx* owner = ix->owner;
    delete ix;
    pcp::ctx_release(owner);
    return PCP_OK;
}

int64_t pcp_index_size(const pcp_index* ix) { return ix ? ix->n : -1; }
int pcp_index_identity_mapping(const pcp_index* ix) { return ix ? ix->identity : 0; }
double pcp_index_cell_size(const pcp_index* ix) { return ix ? ix->g.h : 0.0; }
int64_t pcp_index_cells(const pcp_index* ix) { return ix ? (ix->g.dense ? ix->g.ncells : ix->g.nslots * 64) : 0; }
const void* pcp_index_sorted_points(const pcp_index* ix) { return ix ? ix->pts : nullptr; }

}  // extern "C"
