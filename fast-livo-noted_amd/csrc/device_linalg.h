// device_linalg.h — one-wave dense linear algebra shared by the IEKF solve
// (livo_kernels.hip) and the VIO photometric update (vio_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace livo {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// LU factorisation runs one matrix row per lane in registers (pivot search =
// wave argmax, rows move by v_readlane); the factors go to LDS and the
// triangular solves run one right-hand side per lane with the factors read as
// LDS broadcasts.
__device__ __forceinline__ double bcast(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// PartialPivLU as the oracle (inverse18): first maximum |a_ik| over i >= k,
// f = a_ik / a_kk, a_ij -= f * a_kj.  Row `lane` of the matrix is A; on return
// LU (row-major 18x18) and the row permutation are in LDS.
template <int N>
__device__ __forceinline__ void wave_lu_to_lds(double (&A)[N], int lane, double* s_LU, int* s_piv) {
    int piv = lane;
#pragma unroll
    for (int k = 0; k < N; k++) {
        // pivot: the first maximum of |a_ik| over i >= k, scanned in row order
        // on wave-uniform copies of column k (v_readlane, no LDS round trips)
        int p = k;
        double best = fabs(bcast(A[k], k));
#pragma unroll
        for (int i = k + 1; i < N; i++) {
            const double v = fabs(bcast(A[k], i));
            if (v > best) {
                best = v;
                p = i;
            }
        }
        if (p != k) {  // wave-uniform: swap rows k and p, one element at a time
            const int pk = __builtin_amdgcn_readlane(piv, k), pp = __builtin_amdgcn_readlane(piv, p);
#pragma unroll
            for (int j = 0; j < N; j++) {
                const double ak = bcast(A[j], k), ap = bcast(A[j], p);
                A[j] = lane == k ? ap : (lane == p ? ak : A[j]);
            }
            piv = lane == k ? pp : (lane == p ? pk : piv);
        }
        // f = a_ik / a_kk, a_ij -= f * a_kj (rows below k)
        const double f = A[k] / bcast(A[k], k);
        const bool below = lane > k && lane < N;
        if (below) A[k] = f;
#pragma unroll
        for (int j = k + 1; j < N; j++) {
            const double rkj = bcast(A[j], k);
            if (below) A[j] = A[j] - f * rkj;
        }
    }
    if (lane < N) {
#pragma unroll
        for (int j = 0; j < N; j++) s_LU[lane * N + j] = A[j];
        s_piv[lane] = piv;
    }
}

// Column c of A^-1 from the LU in LDS (forward then backward substitution,
// sums in ascending index order exactly as the oracle).
template <int N>
__device__ __forceinline__ void lds_lu_column(const double* s_LU, const int* s_piv, int c, double (&y)[N]) {
#pragma unroll
    for (int i = 0; i < N; i++) {
        double sacc = (s_piv[i] == c) ? 1.0 : 0.0;
#pragma unroll
        for (int j = 0; j < i; j++) sacc = sacc - s_LU[i * N + j] * y[j];
        y[i] = sacc;
    }
#pragma unroll
    for (int i = N - 1; i >= 0; i--) {
        double sacc = y[i];
#pragma unroll
        for (int j = i + 1; j < N; j++) sacc = sacc - s_LU[i * N + j] * y[j];
        y[i] = sacc / s_LU[i * N + i];
    }
}

}  // namespace livo
