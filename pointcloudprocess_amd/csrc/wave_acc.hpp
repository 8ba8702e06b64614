// Wave-level reduction of the 23 ICP accumulator sums and their fp64 un-centring
// (shared by the verify, search and fallback passes of icp.hip).
//
// Each lane holds 23 fp32 values centred on a wave-uniform point c: n, A = sum(q - c),
// B = sum(p - c), AB = sum((q - c)(p - c)^T) (9), AA = sum((q - c)(q - c)^T) (6, upper
// triangle) and D = sum(d2).  A reduce-scatter butterfly halves the values a lane holds at
// each step -- v_permlane32_swap / v_permlane16_swap for lane bits 5 and 4, DPP row mirror,
// half-row mirror and quad permutes for bits 3..0 -- so lane l ends with the wave total of
// value v(l) = 12 b5 + 6 b4 + 3 b3 + 2 b2 + b1 (about 55 VALU ops, against 23 full DPP
// reductions of 7 ops each).  The lanes with b0 = 0 then un-centre their own value in fp64
// and add it to the wave's LDS accumulator S[v], one lane per value in parallel (formerly one
// lane ran all 23 fp64 updates in turn).
#pragma once
#include <hip/hip_runtime.h>

namespace pcp {

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// one butterfly step on DPP partner lanes: lanes with s keep the sum of b, the others of a
template <int CTRL>
__device__ __forceinline__ float bfly(float a, float b, bool s) {
    const float t = s ? b : a, u = s ? a : b;
    return t + dpp_mov<CTRL>(u);
}
// lanes 32..63 of a <-> lanes 0..31 of b
__device__ __forceinline__ void swap32(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
// odd rows (16 lanes) of a <-> even rows of b
__device__ __forceinline__ void swap16(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
// x[i] of four uniform values by a per-lane index 0..3 (flat selects)
__device__ __forceinline__ float pick4(int i, float x0, float x1, float x2, float x3) {
    float r = x3;
    r = i == 2 ? x2 : r;
    r = i == 1 ? x1 : r;
    r = i == 0 ? x0 : r;
    return r;
}

// the accumulator index whose wave total lane l holds after the butterfly
__device__ __forceinline__ int acc_value_of_lane(int lane) {
    return 12 * ((lane >> 5) & 1) + 6 * ((lane >> 4) & 1) + 3 * ((lane >> 3) & 1) + 2 * ((lane >> 2) & 1) +
           ((lane >> 1) & 1);
}

// Whole wave (full EXEC): S[k] += the un-centred wave total of v[k], k < 23.
__device__ __forceinline__ void wave_accumulate(const float (&v)[23], double* S, int lane, float cx, float cy,
                                                float cz) {
    // bit 5: 23 (+1 pad) -> 12 values per lane
    float w12[12];
#pragma unroll
    for (int i = 0; i < 12; i++) {
        float a = v[i], b = i + 12 < 23 ? v[i + 12] : 0.f;
        swap32(a, b);  // a = {a.lo, b.lo}, b = {a.hi, b.hi}
        w12[i] = a + b;
    }
    // bit 4: 12 -> 6
    float w6[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        float a = w12[i], b = w12[i + 6];
        swap16(a, b);  // a = {a.r0, b.r0, a.r2, b.r2}, b = {a.r1, b.r1, a.r3, b.r3}
        w6[i] = a + b;
    }
    // bit 3 (row mirror, lane i <-> 15 - i): 6 -> 3
    const bool s3 = lane & 8, s2 = lane & 4, s1 = lane & 2;
    float w3[3];
#pragma unroll
    for (int i = 0; i < 3; i++) w3[i] = bfly<0x140>(w6[i], w6[i + 3], s3);
    // bit 2 (half-row mirror): 3 (+1 pad) -> 2
    const float x0 = bfly<0x141>(w3[0], w3[2], s2);
    const float x1 = bfly<0x141>(w3[1], 0.f, s2);
    // bit 1 (quad_perm [2,3,0,1]), bit 0 (quad_perm [1,0,3,2])
    float tot = bfly<0x4E>(x0, x1, s1);
    tot += dpp_mov<0xB1>(tot);
    // n, A, B (values 0..6) for every lane
    auto at = [&](int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tot), l)); };
    const float n = at(0), A0 = at(2), A1 = at(4), A2 = at(8), B0 = at(10), B1 = at(12), B2 = at(16);
    // this lane's value k and its un-centring: S[k] += t + a c + e b + (n e) c, with
    //   k = 1..3 (A), 4..6 (B):  e = 1, c = C[j]
    //   k = 7 + 3r + j (AB):     a = A[r], c = C[j], e = C[r], b = B[j]
    //   k = 16 + m (AA, r <= j): a = A[r], c = C[j], e = C[r], b = A[j]
    //   k = 0 (n), 22 (D):       t only
    const int k = acc_value_of_lane(lane);
    const bool own = !(lane & 1) && ((lane >> 1) & 3) != 3 && k < 23;
    int r = 3, j = 3;  // 3: none
    if (k >= 1 && k <= 6) j = (k - 1) % 3;
    if (k >= 7 && k <= 15) { r = (k - 7) / 3; j = (k - 7) % 3; }
    if (k >= 16 && k <= 21) {
        const int m = k - 16;
        r = m < 3 ? 0 : (m < 5 ? 1 : 2);
        j = m < 3 ? m : (m < 5 ? m - 2 : 2);
    }
    const int jb = (k >= 7 && k <= 21) ? j : 3;
    const float a = pick4(r, A0, A1, A2, 0.f);
    const float c = pick4(j, cx, cy, cz, 0.f);
    const float e = (k >= 1 && k <= 6) ? 1.f : pick4(r, cx, cy, cz, 0.f);
    const float b = k <= 15 ? pick4(jb, B0, B1, B2, 0.f) : pick4(jb, A0, A1, A2, 0.f);
    const double de = e, dc = c;
    const double val = (double)tot + (double)a * dc + de * (double)b + (double)n * de * dc;
    if (own) S[k] += val;
}

}  // namespace pcp
