// MFMA layout / numerics / issue-rate probe for the C5 cell-wave kernels (gfx950).
// Checks, with exact data and against host fmaf chains:
//   1. v_mfma_f32_4x4x1_16b_f32 with cbsz=4, abid=g: D reg i, lane l = A[lane 4g+i] * B[lane l] + C
//      (rows = 4 queries broadcast from block g, columns = the 64 candidates, one per lane);
//   2. v_mfma_f32_16x16x4_f32 (A[row l&15][k l>>4], B[k l>>4][col l&15], D row 4(l>>4)+i col l&15)
//      gives bit-identical values to the 4x4x1 chain of the same products in the same k order;
//   3. v_mfma_f32_16x16x32_f16 A/B lane maps are symmetric (any k permutation shared by A and B)
//      and f16 subnormal inputs are not flushed;
//   4. issue interval of back-to-back independent MFMAs of each shape (s_memtime cycles).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o tools/mfma_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

// 1 + 2: a[5][64] query coefficients (lane = query), b[5][64] candidate values (lane = candidate)
// chain: D = fma(a4,b4, fma(a3,b3, fma(a2,b2, fma(a1,b1, fma(a0,b0, 0)))))
template <int G>
__device__ f4 chain4x4(const float* a, const float* b, int l) {
    f4 d = {0.f, 0.f, 0.f, 0.f};
    d = __builtin_amdgcn_mfma_f32_4x4x1f32(a[0 * 64 + l], b[0 * 64 + l], d, 4, G, 0);
    d = __builtin_amdgcn_mfma_f32_4x4x1f32(a[1 * 64 + l], b[1 * 64 + l], d, 4, G, 0);
    d = __builtin_amdgcn_mfma_f32_4x4x1f32(a[2 * 64 + l], b[2 * 64 + l], d, 4, G, 0);
    d = __builtin_amdgcn_mfma_f32_4x4x1f32(a[3 * 64 + l], b[3 * 64 + l], d, 4, G, 0);
    d = __builtin_amdgcn_mfma_f32_4x4x1f32(a[4 * 64 + l], b[4 * 64 + l], d, 4, G, 0);
    return d;
}
__global__ void k_chain(const float* a, const float* b, float* out /*[16 groups][4][64]*/) {
    const int l = threadIdx.x;
    f4 d[16];
    d[0] = chain4x4<0>(a, b, l);   d[1] = chain4x4<1>(a, b, l);   d[2] = chain4x4<2>(a, b, l);
    d[3] = chain4x4<3>(a, b, l);   d[4] = chain4x4<4>(a, b, l);   d[5] = chain4x4<5>(a, b, l);
    d[6] = chain4x4<6>(a, b, l);   d[7] = chain4x4<7>(a, b, l);   d[8] = chain4x4<8>(a, b, l);
    d[9] = chain4x4<9>(a, b, l);   d[10] = chain4x4<10>(a, b, l); d[11] = chain4x4<11>(a, b, l);
    d[12] = chain4x4<12>(a, b, l); d[13] = chain4x4<13>(a, b, l); d[14] = chain4x4<14>(a, b, l);
    d[15] = chain4x4<15>(a, b, l);
    for (int g = 0; g < 16; g++)
        for (int i = 0; i < 4; i++) out[(g * 4 + i) * 64 + l] = d[g][i];
}
// 16x16x4: S[c][q] for candidates c of sub-tile t (16 of the 64) and queries q of tile u (16 of 64):
// A[c][k] = b[k+1][16t + c] (x, y, z, |P|^2), B[k][q] = a[k+1][16u + q], C = a[0][16u+q] * b[0][..] (= a0 since b0 = 1)
__global__ void k_16x16(const float* a, const float* b, float* out /*[4 u][4 t][4 i][64]*/) {
    const int l = threadIdx.x;
    for (int u = 0; u < 4; u++)
        for (int t = 0; t < 4; t++) {
            const float c0 = a[0 * 64 + 16 * u + (l & 15)] * b[0];  // b0 == 1 exactly
            f4 d = {c0, c0, c0, c0};
            d = __builtin_amdgcn_mfma_f32_16x16x4f32(b[(1 + (l >> 4)) * 64 + 16 * t + (l & 15)],
                                                     a[(1 + (l >> 4)) * 64 + 16 * u + (l & 15)], d, 0, 0, 0);
            for (int i = 0; i < 4; i++) out[((u * 4 + t) * 4 + i) * 64 + l] = d[i];
        }
}
// 3: 16x16x32 f16: A[16][32], B[32][16] small integers (and subnormals), lane maps
//    A: lane l elem j = A[l&15][8(l>>4)+j], B: lane l elem j = B[8(l>>4)+j][l&15]
__global__ void k_f16(const _Float16* A, const _Float16* B, float* D) {
    const int l = threadIdx.x;
    h8 af, bf;
    for (int j = 0; j < 8; j++) {
        af[j] = A[(l & 15) * 32 + 8 * (l >> 4) + j];
        bf[j] = B[(8 * (l >> 4) + j) * 16 + (l & 15)];
    }
    f4 d = {0.f, 0.f, 0.f, 0.f};
    d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, d, 0, 0, 0);
    for (int i = 0; i < 4; i++) D[(4 * (l >> 4) + i) * 16 + (l & 15)] = d[i];
}
// 4: issue rate: N rounds of 8 independent accumulators
template <int KIND>
__global__ void k_rate(float* sink, long long* cyc, int rounds) {
    const int l = threadIdx.x;
    float av = (float)l * 1e-3f, bv = 1.f - av;
    h8 ah, bh;
    for (int j = 0; j < 8; j++) ah[j] = (_Float16)(av * j), bh[j] = (_Float16)(bv * j);
    f4 acc[8];
    for (int k = 0; k < 8; k++) acc[k] = (f4){0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    const long long t0 = __builtin_readcyclecounter();
    for (int r = 0; r < rounds; r++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (KIND == 0) acc[k] = __builtin_amdgcn_mfma_f32_4x4x1f32(av, bv, acc[k], 4, 0, 0);
            if (KIND == 1) acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[k], 0, 0, 0);
            if (KIND == 2) acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[k], 0, 0, 0);
        }
    }
    const long long t1 = __builtin_readcyclecounter();
    float s = 0.f;
    for (int k = 0; k < 8; k++) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    sink[blockIdx.x * 64 + l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

static float frand(unsigned& s) {
    s = s * 1664525u + 1013904223u;
    return ((s >> 8) & 0xffffff) / 16777216.0f;
}

int main() {
    int bad = 0;
    // ---- 1 + 2
    std::vector<float> a(5 * 64), b(5 * 64);
    unsigned seed = 12345;
    for (int l = 0; l < 64; l++) {
        const float qx = frand(seed) * 0.2f - 0.1f, qy = frand(seed) * 0.2f - 0.1f, qz = frand(seed) * 0.2f - 0.1f;
        a[0 * 64 + l] = qx * qx + qy * qy + qz * qz - 0.04f;  // |Q|^2 - r^2
        a[1 * 64 + l] = -2.f * qx;
        a[2 * 64 + l] = -2.f * qy;
        a[3 * 64 + l] = -2.f * qz;
        a[4 * 64 + l] = 1.f;
        const float px = frand(seed) * 0.6f - 0.3f, py = frand(seed) * 0.6f - 0.3f, pz = frand(seed) * 0.6f - 0.3f;
        b[0 * 64 + l] = 1.f;
        b[1 * 64 + l] = px;
        b[2 * 64 + l] = py;
        b[3 * 64 + l] = pz;
        b[4 * 64 + l] = px * px + py * py + pz * pz;
    }
    float *da, *db, *dout, *d16;
    CK(hipMalloc(&da, a.size() * 4));
    CK(hipMalloc(&db, b.size() * 4));
    CK(hipMalloc(&dout, 16 * 4 * 64 * 4));
    CK(hipMalloc(&d16, 4 * 4 * 4 * 64 * 4));
    CK(hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, da, db, dout);
    hipLaunchKernelGGL(k_16x16, dim3(1), dim3(64), 0, 0, da, db, d16);
    CK(hipDeviceSynchronize());
    std::vector<float> out(16 * 4 * 64), o16(4 * 4 * 4 * 64);
    CK(hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(o16.data(), d16, o16.size() * 4, hipMemcpyDeviceToHost));
    int bad1 = 0, bad2 = 0;
    for (int g = 0; g < 16; g++)
        for (int i = 0; i < 4; i++)
            for (int l = 0; l < 64; l++) {
                const int q = 4 * g + i;
                float d = 0.f;
                for (int k = 0; k < 5; k++) d = std::fmaf(a[k * 64 + q], b[k * 64 + l], d);
                const float got = out[(g * 4 + i) * 64 + l];
                if (memcmp(&d, &got, 4) != 0) {
                    if (bad1 < 5) printf("4x4x1 g=%d i=%d l=%d: got %.9g want %.9g\n", g, i, l, got, d);
                    bad1++;
                }
            }
    for (int u = 0; u < 4; u++)
        for (int t = 0; t < 4; t++)
            for (int i = 0; i < 4; i++)
                for (int l = 0; l < 64; l++) {
                    const int c = 16 * t + 4 * (l >> 4) + i, q = 16 * u + (l & 15);
                    const float got = o16[((u * 4 + t) * 4 + i) * 64 + l];
                    const float ref = out[(q / 4 * 4 + q % 4) * 64 + c];  // 4x4x1: group q/4, reg q%4, lane c
                    if (memcmp(&ref, &got, 4) != 0) {
                        if (bad2 < 5) printf("16x16x4 vs chain u=%d t=%d i=%d l=%d: got %.9g chain %.9g\n", u, t, i, l, got, ref);
                        bad2++;
                    }
                }
    printf("check1 4x4x1_16b cbsz4/abid layout == host fmaf chain: %s (%d bad of 4096)\n", bad1 ? "FAIL" : "ok", bad1);
    printf("check2 16x16x4 S[c][q] bit-identical to the 4x4x1 chain: %s (%d bad of 4096)\n", bad2 ? "FAIL" : "ok", bad2);
    bad += bad1 + bad2;
    // ---- 3
    std::vector<_Float16> A(16 * 32), B(32 * 16);
    std::vector<float> Af(16 * 32), Bf(32 * 16);
    for (int r = 0; r < 16; r++)
        for (int k = 0; k < 32; k++) {
            float v = (float)(((r * 7 + k * 3) % 11) - 5);
            if (k == 5 && r == 3) v = 1.1920929e-7f;  // f16 subnormal (2^-23)
            A[r * 32 + k] = (_Float16)v;
            Af[r * 32 + k] = (float)A[r * 32 + k];
        }
    for (int k = 0; k < 32; k++)
        for (int c = 0; c < 16; c++) {
            float v = (float)(((k * 5 + c * 13) % 9) - 4) + (k == 5 ? 1.f : 0.f);
            B[k * 16 + c] = (_Float16)v;
            Bf[k * 16 + c] = (float)B[k * 16 + c];
        }
    _Float16 *dA, *dB;
    float* dD;
    CK(hipMalloc(&dA, A.size() * 2));
    CK(hipMalloc(&dB, B.size() * 2));
    CK(hipMalloc(&dD, 256 * 4));
    CK(hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_f16, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    CK(hipDeviceSynchronize());
    std::vector<float> D(256);
    CK(hipMemcpy(D.data(), dD, 256 * 4, hipMemcpyDeviceToHost));
    int bad3 = 0;
    for (int r = 0; r < 16; r++)
        for (int c = 0; c < 16; c++) {
            double s = 0;
            for (int k = 0; k < 32; k++) s += (double)Af[r * 32 + k] * Bf[k * 16 + c];
            if (std::fabs(s - D[r * 16 + c]) > 1e-6 * (1 + std::fabs(s))) {
                if (bad3 < 5) printf("f16 r=%d c=%d got %.9g want %.9g\n", r, c, D[r * 16 + c], s);
                bad3++;
            }
        }
    printf("check3 16x16x32 f16 lane maps + subnormal inputs: %s (%d bad of 256; row 3 carries 2^-23 x B[5][c])\n",
           bad3 ? "FAIL" : "ok", bad3);
    bad += bad3;
    // ---- 4
    float* sink;
    long long* cyc;
    const int nb = 1024 * 4;  // 4 waves per SIMD
    CK(hipMalloc(&sink, nb * 64 * 4));
    CK(hipMalloc(&cyc, nb * 8));
    const char* names[3] = {"v_mfma_f32_4x4x1_16b_f32", "v_mfma_f32_16x16x4_f32", "v_mfma_f32_16x16x32_f16"};
    for (int kind = 0; kind < 3; kind++) {
        const int rounds = 2000;
        for (int rep = 0; rep < 2; rep++) {
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            CK(hipEventRecord(e0));
            if (kind == 0) hipLaunchKernelGGL(k_rate<0>, dim3(nb), dim3(64), 0, 0, sink, cyc, rounds);
            if (kind == 1) hipLaunchKernelGGL(k_rate<1>, dim3(nb), dim3(64), 0, 0, sink, cyc, rounds);
            if (kind == 2) hipLaunchKernelGGL(k_rate<2>, dim3(nb), dim3(64), 0, 0, sink, cyc, rounds);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::vector<long long> c(nb);
            CK(hipMemcpy(c.data(), cyc, nb * 8, hipMemcpyDeviceToHost));
            double avg = 0;
            for (long long v : c) avg += (double)v;
            avg /= nb;
            // one wave's 8 x rounds MFMAs; 4 waves share a SIMD; 1024 SIMDs
            const double per_simd_ns = ms * 1e6 / ((double)nb / 1024.0 * 8.0 * rounds);
            if (rep == 1)
                printf("rate %-26s wave cycles/MFMA %.2f (4 waves/SIMD), chip ns per MFMA per SIMD %.3f (%.1f cycles @2.4GHz)\n",
                       names[kind], avg / (8.0 * rounds), per_simd_ns, per_simd_ns * 2.4);
        }
    }
    printf(bad ? "PROBE FAIL\n" : "PROBE OK\n");
    return bad ? 1 : 0;
}
