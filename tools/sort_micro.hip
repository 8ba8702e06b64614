// Micro-benchmark (round-6 verdict item 2): the C4 pre-iteration cell sort of 50M points into a
// dense 650M-cell table -- rocPRIM's radix sort of (cell id, 16-byte record) pairs, as the build
// runs it today, against a counting sort on the dense cell table (memset, one returning atomic
// per point for its rank in its cell, an exclusive scan of the counts = the cell starts, a
// scatter, and a per-cell pass that restores the stable caller order).  Synthetic points at the
// bench scene's density: 55 % on a ground layer, 45 % on 24 vertical facades, random order.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sort_micro.hip -o tools/sort_micro && tools/sort_micro
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int NX = 1667, NY = 1667, NZ = 250;
constexpr float H = 0.12f;

__device__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
__device__ float u01(uint32_t s) { return (hash32(s) >> 8) * (1.0f / 16777216.0f); }

__global__ void k_gen(float4* rec, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)i * 4u;
        float x, y, z;
        if (u01(s) < 0.55f) {  // ground
            x = u01(s + 1) * 199.9f; y = u01(s + 2) * 199.9f; z = 0.05f + 0.2f * u01(s + 3);
        } else {                // facades: 12 planes x = const, 12 planes y = const
            const int f = (int)(u01(s + 1) * 24.f);
            const float a = u01(s + 2) * 199.9f, b = 0.1f + 25.f * u01(s + 3);
            const float c = 8.f + 16.f * (f % 12) + 0.05f * u01(s + 5);
            x = f < 12 ? c : a; y = f < 12 ? a : c; z = b;
        }
        rec[i] = make_float4(x, y, z, __int_as_float((int)i));
    }
}

__device__ __forceinline__ uint32_t cell_key(float x, float y, float z) {
    const int cx = min(max((int)floorf(x * (1.f / H)), 0), NX - 1);
    const int cy = min(max((int)floorf(y * (1.f / H)), 0), NY - 1);
    const int cz = min(max((int)floorf(z * (1.f / H)), 0), NZ - 1);
    return (uint32_t)(((int64_t)cz * NY + cy) * NX + cx);
}

__global__ void k_keys(const float4* rec, int64_t n, uint32_t* key) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 p = rec[i];
        key[i] = cell_key(p.x, p.y, p.z);
    }
}

// count: rank of the point in its cell (arrival order) from a returning atomic
__global__ void k_count(const float4* rec, int64_t n, uint32_t* cnt, uint32_t* rank) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 p = rec[i];
        rank[i] = atomicAdd(&cnt[cell_key(p.x, p.y, p.z)], 1u);
    }
}
__global__ void k_count_nr(const float4* rec, int64_t n, uint32_t* cnt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 p = rec[i];
        atomicAdd(&cnt[cell_key(p.x, p.y, p.z)], 1u);
    }
}

__global__ void k_scatter(const float4* rec, const uint32_t* rank, const uint32_t* cstart, int64_t n, float4* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 p = rec[i];
        out[cstart[cell_key(p.x, p.y, p.z)] + rank[i]] = p;
    }
}

// the stable order inside each cell: position = cell start + the cell's points with a smaller index
__global__ void k_fix(const float4* in, const uint32_t* cstart, int64_t n, float4* out) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const float4 p = in[k];
        const uint32_t c = cell_key(p.x, p.y, p.z);
        const uint32_t s = cstart[c], e = cstart[c + 1];
        const int me = __float_as_int(p.w);
        uint32_t r = 0;
        for (uint32_t j = s; j < e; j++) r += __float_as_int(in[j].w) < me ? 1u : 0u;
        out[s + r] = p;
    }
}

int main() {
    const int64_t n = 50'000'000;
    const int64_t ncells = (int64_t)NX * NY * NZ;
    float4 *rec, *sorted, *out, *out2;
    uint32_t *key, *key2, *cnt, *rank, *cst;
    CK(hipMalloc(&rec, n * 16)); CK(hipMalloc(&sorted, n * 16)); CK(hipMalloc(&out, n * 16)); CK(hipMalloc(&out2, n * 16));
    CK(hipMalloc(&key, n * 4)); CK(hipMalloc(&key2, n * 4)); CK(hipMalloc(&rank, n * 4));
    CK(hipMalloc(&cnt, (ncells + 1) * 4)); CK(hipMalloc(&cst, (ncells + 1) * 4));
    hipStream_t st; CK(hipStreamCreate(&st));
    const dim3 G(2048), B(256);
    k_gen<<<G, B, 0, st>>>(rec, n);
    size_t tb = 0, tb2 = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tb, key, key2, rec, sorted, (size_t)n, 0u, 30u, st));
    CK(rocprim::exclusive_scan(nullptr, tb2, cnt, cst, 0u, (size_t)ncells + 1, rocprim::plus<uint32_t>(), st));
    void* tmp; CK(hipMalloc(&tmp, std::max(tb, tb2)));
    hipEvent_t ev[12];
    for (auto& e : ev) CK(hipEventCreate(&e));
    auto ms = [&](int a, int b) { float t; CK(hipEventElapsedTime(&t, ev[a], ev[b])); return t; };
    for (int rep = 0; rep < 4; rep++) {
        CK(hipEventRecord(ev[0], st));
        k_keys<<<G, B, 0, st>>>(rec, n, key);
        CK(rocprim::radix_sort_pairs(tmp, tb, key, key2, rec, sorted, (size_t)n, 0u, 30u, st));
        CK(hipEventRecord(ev[1], st));
        CK(hipMemsetAsync(cnt, 0, (ncells + 1) * 4, st));
        CK(hipEventRecord(ev[2], st));
        k_count<<<G, B, 0, st>>>(rec, n, cnt, rank);
        CK(hipEventRecord(ev[3], st));
        CK(rocprim::exclusive_scan(tmp, tb2, cnt, cst, 0u, (size_t)ncells + 1, rocprim::plus<uint32_t>(), st));
        CK(hipEventRecord(ev[4], st));
        k_scatter<<<G, B, 0, st>>>(rec, rank, cst, n, out);
        CK(hipEventRecord(ev[5], st));
        k_fix<<<G, B, 0, st>>>(out, cst, n, out2);
        CK(hipEventRecord(ev[6], st));
        CK(hipMemsetAsync(cnt, 0, (ncells + 1) * 4, st));
        CK(hipEventRecord(ev[7], st));
        k_count_nr<<<G, B, 0, st>>>(rec, n, cnt);
        CK(hipEventRecord(ev[8], st));
        CK(hipStreamSynchronize(st));
        printf("rep %d: radix (keys + sort) %.3f ms | counting: memset %.3f count(ret) %.3f scan %.3f scatter %.3f fix %.3f "
               "= %.3f ms | count(no-ret) %.3f\n", rep, ms(0, 1), ms(1, 2), ms(2, 3), ms(3, 4), ms(4, 5), ms(5, 6),
               ms(1, 6), ms(7, 8));
    }
    // the two orders must agree record for record
    std::vector<float4> a(n), b(n);
    CK(hipMemcpy(a.data(), sorted, n * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), out2, n * 16, hipMemcpyDeviceToHost));
    int64_t diff = 0;
    for (int64_t i = 0; i < n; i++) diff += memcmp(&a[i], &b[i], 16) != 0;
    printf("records differing between the radix and the counting order: %lld\n", (long long)diff);
    return 0;
}
