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

}  // namespace

int scan_u32_inplace(pcp_ctx* ctx, uint32_t* data, int64_t n, uint32_t* total_host) {
    if (n <= 0) {
        if (total_host) *total_host = 0;
        return PCP_OK;
    }
    int64_t tmp_elems = scan_tmp_elems(n);
    void* tmp;
    // +2 for the last value and the total
    PCP_TRY(scratch(ctx, (tmp_elems + 2) * sizeof(uint32_t), &tmp));
    uint32_t* t = (uint32_t*)tmp;
    uint32_t* last = t + tmp_elems;
    if (total_host)
        PCP_HIP(ctx, hipMemcpyAsync(last, data + n - 1, sizeof(uint32_t), hipMemcpyDeviceToDevice, ctx->stream));
    PCP_TRY((scan_rec<uint32_t, uint32_t>(ctx, data, n, data, t, tmp_elems)));
    if (total_host) {
        hipLaunchKernelGGL((write_total<uint32_t>), dim3(1), dim3(1), 0, ctx->stream, data + n - 1,
                           last, last + 1);
        PCP_LAUNCH_CHECK(ctx);
        PCP_HIP(ctx, hipMemcpyAsync(total_host, last + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
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
