// Device exclusive scans used by the index build (brick slots, cell starts) and the
// radius-search CSR offsets.  Three-pass tile scan (reduce -> scan of tile sums -> scan +
// offset), deterministic, wave64 shuffles + LDS.
#include "common.hpp"

namespace pcp {
namespace {

constexpr int kBlock = 256;
constexpr int kItems = 8;
constexpr int kTile = kBlock * kItems;

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        T o = __shfl_up(v, off, 64);
        if (lane >= off) v += o;
    }
    return v;
}

// block-wide exclusive scan of one value per thread; returns exclusive prefix, *total = sum
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* total) {
    __shared__ T wsum[kBlock / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T incl = wave_incl_scan(v);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    T wofs = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; w++) {
        T s = wsum[w];
        if (w < wid) wofs += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return wofs + incl - v;
}

template <typename Tin, typename Tacc>
__global__ void __launch_bounds__(kBlock) tile_reduce(const Tin* __restrict__ in, int64_t n,
                                                      Tacc* __restrict__ sums) {
    const int64_t base = (int64_t)blockIdx.x * kTile;
    Tacc s = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        int64_t idx = base + (int64_t)i * kBlock + threadIdx.x;
        if (idx < n) s += (Tacc)in[idx];
    }
    Tacc tot;
    (void)block_excl_scan<Tacc>(s, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// exclusive scan of each tile (thread owns kItems consecutive elements) + tile offset
template <typename Tin, typename Tacc>
__global__ void __launch_bounds__(kBlock) tile_scan(const Tin* in, int64_t n, const Tacc* __restrict__ offs,
                                                    Tacc* out) {
    const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems;
    Tacc v[kItems];
    Tacc s = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        int64_t idx = base + i;
        v[i] = idx < n ? (Tacc)in[idx] : (Tacc)0;
        s += v[i];
    }
    Tacc tot;
    Tacc run = block_excl_scan<Tacc>(s, &tot) + (offs ? offs[blockIdx.x] : (Tacc)0);
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        int64_t idx = base + i;
        if (idx < n) out[idx] = run;
        run += v[i];
    }
}

template <typename Tacc>
__global__ void write_total(const Tacc* last_in_excl, const Tacc* last_val, Tacc* dst) {
    *dst = *last_in_excl + *last_val;
}

// recursive exclusive scan: out[i] = sum(in[0..i)) ; works in place when Tin == Tacc
template <typename Tin, typename Tacc>
int scan_rec(pcp_ctx* ctx, const Tin* in, int64_t n, Tacc* out, Tacc* tmp, int64_t tmp_cap) {
    const int64_t tiles = (n + kTile - 1) / kTile;
    if (tiles <= 1) {
        hipLaunchKernelGGL((tile_scan<Tin, Tacc>), dim3(1), dim3(kBlock), 0, ctx->stream, in, n,
                           (const Tacc*)nullptr, out);
        PCP_LAUNCH_CHECK(ctx);
        return PCP_OK;
    }
    if (tmp_cap < tiles) return set_error(ctx, PCP_ERR_ARG, "scan scratch too small");
    Tacc* sums = tmp;
    hipLaunchKernelGGL((tile_reduce<Tin, Tacc>), dim3((unsigned)tiles), dim3(kBlock), 0, ctx->stream,
                       in, n, sums);
    PCP_LAUNCH_CHECK(ctx);
    PCP_TRY((scan_rec<Tacc, Tacc>(ctx, sums, tiles, sums, tmp + tiles, tmp_cap - tiles)));
    hipLaunchKernelGGL((tile_scan<Tin, Tacc>), dim3((unsigned)tiles), dim3(kBlock), 0, ctx->stream,
                       in, n, (const Tacc*)sums, out);
    PCP_LAUNCH_CHECK(ctx);
    return PCP_OK;
}

__global__ void append_total_i64(int64_t* out, const int32_t* in, int64_t n) {
    out[n] = out[n - 1] + (int64_t)in[n - 1];
}

int64_t scan_tmp_elems(int64_t n) {
    int64_t total = 0;
    while (true) {
        int64_t tiles = (n + kTile - 1) / kTile;
        if (tiles <= 1) break;
        total += tiles;
        n = tiles;
    }
    return total + 16;
}

// ---- single-pass u32 exclusive scan with decoupled look-back (one read + one write of the
// data): tiles take ids in launch order from an atomic counter, publish their aggregate at
// once and their inclusive prefix after looking back over predecessors (64 at a time, one
// per lane of wave 0).  Status word = (2-bit state << 62) | 32-bit value.
constexpr int kLbBlock = 256;
constexpr int kLbSeg = 4;                       // segments of 1024 elements per tile
constexpr int kLbTile = kLbBlock * 4 * kLbSeg;  // 4096 elements
// status word: flag (bits 62-63) | epoch (bits 32-61) | value; a word of another epoch reads as
// "not published yet"
constexpr uint64_t kStAgg = 1ull << 62, kStPre = 2ull << 62, kStMask = 3ull << 62;
constexpr uint32_t kEpochMask = 0x3fffffffu;

__device__ __forceinline__ uint64_t st_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(kLbBlock) k_scan_lookback(uint32_t* data, int64_t n, uint64_t* status,
                                                            uint32_t* tile_ctr, uint32_t* total_out,
                                                            uint32_t epoch) {
    __shared__ uint32_t s_tile, s_prefix;
    __shared__ uint32_t s_wsum[kLbBlock / 64][kLbSeg];
    if (threadIdx.x == 0) {
        s_tile = atomicAdd(tile_ctr, 1u);
        // the last tile id is handed out last: reset the counter for the next call
        if (s_tile == gridDim.x - 1) atomicExch(tile_ctr, 0u);
    }
    __syncthreads();
    const uint32_t tile = s_tile;
    const int64_t base = (int64_t)tile * kLbTile;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t v[kLbSeg][4], sum[kLbSeg];
#pragma unroll
    for (int k = 0; k < kLbSeg; k++) {
        const int64_t idx = base + k * 1024 + 4 * threadIdx.x;
        if (idx + 3 < n) {
            const uint4 u = *(const uint4*)(data + idx);
            v[k][0] = u.x; v[k][1] = u.y; v[k][2] = u.z; v[k][3] = u.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) v[k][j] = idx + j < n ? data[idx + j] : 0u;
        }
        sum[k] = v[k][0] + v[k][1] + v[k][2] + v[k][3];
    }
    uint32_t incl[kLbSeg];
#pragma unroll
    for (int k = 0; k < kLbSeg; k++) {
        incl[k] = wave_incl_scan(sum[k]);
        if (lane == 63) s_wsum[wid][k] = incl[k];
    }
    __syncthreads();
    uint32_t excl[kLbSeg], segpre[kLbSeg], tile_total = 0;
#pragma unroll
    for (int k = 0; k < kLbSeg; k++) {
        uint32_t wofs = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kLbBlock / 64; w++) {
            const uint32_t x = s_wsum[w][k];
            wofs += w < wid ? x : 0u;
            tot += x;
        }
        excl[k] = wofs + incl[k] - sum[k];
        segpre[k] = tile_total;
        tile_total += tot;
    }
    if (wid == 0) {
        const uint64_t ep = (uint64_t)epoch << 32;
        uint32_t prefix = 0;
        if (tile == 0) {
            if (lane == 0) st_store(&status[0], kStPre | ep | tile_total);
        } else {
            if (lane == 0) st_store(&status[tile], kStAgg | ep | tile_total);
            int64_t top = (int64_t)tile - 1;
            while (true) {
                const int64_t p = top - lane;
                const uint64_t st = p >= 0 ? st_load(&status[p]) : kStPre | ep;
                const uint64_t flag = (st & ~kStMask & ~0xffffffffull) == ep ? st & kStMask : 0ull;
                const uint64_t pre = __ballot(flag == kStPre);
                const uint64_t notready = __ballot(flag == 0);
                const int first = pre ? __ffsll((long long)pre) - 1 : 64;
                const uint64_t need = first >= 63 ? ~0ull : ((1ull << (first + 1)) - 1);
                if (notready & need) continue;  // a predecessor has not published yet
                uint32_t x = lane <= first ? (uint32_t)st : 0u;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
                prefix += x;
                if (first < 64) break;
                top -= 64;
            }
            if (lane == 0) st_store(&status[tile], kStPre | ep | (prefix + tile_total));
        }
        if (lane == 0) s_prefix = prefix;
    }
    __syncthreads();
    const uint32_t pfx = s_prefix;
    if (total_out && threadIdx.x == 0 && base + kLbTile >= n) *total_out = pfx + tile_total;
#pragma unroll
    for (int k = 0; k < kLbSeg; k++) {
        const int64_t idx = base + k * 1024 + 4 * threadIdx.x;
        uint32_t run = pfx + segpre[k] + excl[k];
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; j++) { o[j] = run; run += v[k][j]; }
        if (idx + 3 < n) {
            *(uint4*)(data + idx) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (idx + j < n) data[idx + j] = o[j];
        }
    }
}

}  // namespace

int scan_u32_inplace(pcp_ctx* ctx, uint32_t* data, int64_t n, uint32_t* total_host) {
    if (n <= 0) {
        if (total_host) *total_host = 0;
        return PCP_OK;
    }
    const int64_t tiles = (n + kLbTile - 1) / kLbTile;
    // persistent state: [status (tiles u64)] [tile counter, total (u32)], cleared once when it
    // grows; each call tags its status words with a new epoch instead of clearing them
    if (tiles > ctx->scan_tiles) {
        if (ctx->scan_status) {
            PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
            PCP_HIP(ctx, hipFree(ctx->scan_status));
            ctx->scan_status = nullptr;
            ctx->scan_tiles = 0;
        }
        const int64_t want = tiles + tiles / 4 + 64;
        PCP_HIP(ctx, hipMalloc(&ctx->scan_status, (size_t)(want + 1) * sizeof(uint64_t)));
        PCP_HIP(ctx, hipMemsetAsync(ctx->scan_status, 0, (size_t)(want + 1) * sizeof(uint64_t), ctx->stream));
        ctx->scan_tiles = want;
        ctx->scan_epoch = 0;
    }
    ctx->scan_epoch = (ctx->scan_epoch + 1) & kEpochMask;
    if (ctx->scan_epoch == 0) {
        // wrapped after 2^30 - 1 calls: a status word left by an older call with fewer tiles
        // could carry the epoch about to be reused, so clear them all once (0: the cleared state)
        PCP_HIP(ctx, hipMemsetAsync(ctx->scan_status, 0, (size_t)ctx->scan_tiles * sizeof(uint64_t), ctx->stream));
        ctx->scan_epoch = 1;
    }
    uint64_t* status = ctx->scan_status;
    uint32_t* ctr = (uint32_t*)(status + ctx->scan_tiles);
    hipLaunchKernelGGL(k_scan_lookback, dim3((unsigned)tiles), dim3(kLbBlock), 0, ctx->stream, data, n, status, ctr,
                       ctr + 1, ctx->scan_epoch);
    PCP_LAUNCH_CHECK(ctx);
    if (total_host) {
        PCP_HIP(ctx, hipMemcpyAsync(total_host, ctr + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    return PCP_OK;
}

int scan_i32_to_i64(pcp_ctx* ctx, const int32_t* in, int64_t n, int64_t* out, int64_t* total_host) {
    if (n <= 0) {
        PCP_HIP(ctx, hipMemsetAsync(out, 0, sizeof(int64_t), ctx->stream));
        if (total_host) *total_host = 0;
        return PCP_OK;
    }
    int64_t tmp_elems = scan_tmp_elems(n);
    void* tmp;
    PCP_TRY(scratch(ctx, tmp_elems * sizeof(int64_t), &tmp));
    PCP_TRY((scan_rec<int32_t, int64_t>(ctx, in, n, out, (int64_t*)tmp, tmp_elems)));
    hipLaunchKernelGGL(append_total_i64, dim3(1), dim3(1), 0, ctx->stream, out, in, n);
    PCP_LAUNCH_CHECK(ctx);
    if (total_host) {
        PCP_HIP(ctx, hipMemcpyAsync(total_host, out + n, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    return PCP_OK;
}

}  // namespace pcp

extern "C" int pcp_scan_counts(pcp_ctx* ctx, const int32_t* count_dev, int64_t n,
                               int64_t* offsets_dev, int64_t* total_host) {
    if (!ctx || n < 0 || (n > 0 && !count_dev) || !offsets_dev) return PCP_ERR_ARG;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    return pcp::scan_i32_to_i64(ctx, count_dev, n, offsets_dev, total_host);
}
