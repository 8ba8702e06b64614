// fp64 (d2, index) helpers shared by the grid and brute-force kNN kernels: the FLANN
// L2_Simple<double> distance and a register-resident sorted top-k.
#pragma once
#include <climits>
#include <cmath>

namespace pcp {

template <typename T>
__device__ __forceinline__ bool lex_less(T da, int ja, T db, int jb) {
    return da < db || (da == db && ja < jb);
}

// FLANN L2_Simple<double> (external): r = 0; r += d0*d0; ...
__device__ __forceinline__ double l2_simple(double qx, double qy, double qz, const double4& p) {
    const double d0 = qx - p.x, d1 = qy - p.y, d2 = qz - p.z;
    double r = d0 * d0;
    r = r + d1 * d1;
    r = r + d2 * d2;
    return r;
}

// k best (d2, j) in registers, kept in DESCENDING order so that the current k-th best
// (the pruning bound) is always slot 0.  For a runtime k < K the tail slots hold -inf
// sentinels that nothing can displace: real entries occupy [0, k), best at k-1.
// Insertion is in place from slot 0 upward (slot i takes slot i+1 while x is better than
// it), so no per-slot flag array is kept and every index is a compile-time constant.
template <int K, typename T = double>
struct TopK {
    T d[K];
    int j[K];
    __device__ void init(int k) {
#pragma unroll
        for (int i = 0; i < K; i++) {
            const bool real = i < k;
            d[i] = real ? INFINITY : -INFINITY;
            j[i] = real ? INT_MAX : INT_MIN;
        }
    }
    __device__ T kth() const { return d[0]; }
    __device__ __forceinline__ void push(T x, int jx) {
        if (!lex_less(x, jx, d[0], j[0])) return;
        bool below = true;  // x better than the old slot i (true for i = 0)
#pragma unroll
        for (int i = 0; i < K - 1; i++) {
            const bool nb = lex_less(x, jx, d[i + 1], j[i + 1]);
            if (nb) { d[i] = d[i + 1]; j[i] = j[i + 1]; }
            else if (below) { d[i] = x; j[i] = jx; }
            below = nb;
        }
        if (below) { d[K - 1] = x; j[K - 1] = jx; }
    }
    // r-th best (ascending) lives in slot k-1-r; visit r = 0..k-1 with f(r, d, j)
    template <typename F>
    __device__ __forceinline__ void for_each_ascending(int k, F f) const {
#pragma unroll
        for (int i = K - 1; i >= 0; i--)
            if (i < k) f(k - 1 - i, d[i], j[i]);
    }
    // move the -inf sentinels to the front (best at slot K-1), for pop_best()
    __device__ void normalize(int k) {
        for (int t = k; t < K; t++) {
#pragma unroll
            for (int i = K - 1; i >= 1; i--) { d[i] = d[i - 1]; j[i] = j[i - 1]; }
            d[0] = INFINITY;
            j[0] = INT_MAX;
        }
    }
    __device__ T best_d() const { return d[K - 1]; }
    __device__ int best_j() const { return j[K - 1]; }
    __device__ void pop_best() {
#pragma unroll
        for (int i = K - 1; i >= 1; i--) { d[i] = d[i - 1]; j[i] = j[i - 1]; }
        d[0] = INFINITY;
        j[0] = INT_MAX;
    }
};

}  // namespace pcp
