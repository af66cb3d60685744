// device_linalg.h — one-wave dense linear algebra shared by the IEKF solve
// (livo_kernels.hip) and the VIO photometric update (vio_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "livo.h"

namespace livo {

// Sum over each 16-lane row by DPP (quad_perm xor 1, xor 2, row_ror 4, 8):
// every lane of a row ends with the row's sum, in VALU latency (no LDS
// permute round trips as __shfl_xor has).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double row_sum16(double v) {
    v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_f64<0x124>(v);  // row_ror:4
    v += dpp_f64<0x128>(v);  // row_ror:8
    return v;
}

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

#define WAVE_SYNC() do { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); __builtin_amdgcn_wave_barrier(); } while (0)

// SO3 Exp / Log (so3_math.h:55-81) and 3x3 products, sums in index order.
__device__ __forceinline__ void so3_exp(double v1, double v2, double v3, double* R) {
    const double norm = sqrt(v1 * v1 + v2 * v2 + v3 * v3);
    _Pragma("unroll") for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (norm > 0.00001) {
        const double r[3] = {v1 / norm, v2 / norm, v3 / norm};
        const double K[9] = {0.0, -r[2], r[1], r[2], 0.0, -r[0], -r[1], r[0], 0.0};
        const double s = sin(norm), c1 = 1.0 - cos(norm);
        double cK[9];
        _Pragma("unroll") for (int i = 0; i < 9; i++) cK[i] = c1 * K[i];
        _Pragma("unroll") for (int i = 0; i < 3; i++)
            _Pragma("unroll") for (int j = 0; j < 3; j++) {
                const double kk = (cK[i * 3 + 0] * K[0 * 3 + j] + cK[i * 3 + 1] * K[1 * 3 + j]) + cK[i * 3 + 2] * K[2 * 3 + j];
                R[i * 3 + j] = (R[i * 3 + j] + s * K[i * 3 + j]) + kk;
            }
    }
}
__device__ __forceinline__ void so3_log(const double* R, double* o) {
    const double tr = (R[0] + R[4]) + R[8];
    const double theta = (tr > 3.0 - 1e-6) ? 0.0 : acos(0.5 * (tr - 1));
    const double K[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
    if (fabs(theta) < 0.001) {
        _Pragma("unroll") for (int i = 0; i < 3; i++) o[i] = 0.5 * K[i];
    } else {
        const double f = 0.5 * theta / sin(theta);
        _Pragma("unroll") for (int i = 0; i < 3; i++) o[i] = f * K[i];
    }
}
__device__ __forceinline__ void mat3_mul(const double* A, const double* B, double* C) {
    _Pragma("unroll") for (int i = 0; i < 3; i++)
        _Pragma("unroll") for (int j = 0; j < 3; j++)
            C[i * 3 + j] = (A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j]) + A[i * 3 + 2] * B[2 * 3 + j];
}

// The head of livo_state (everything but cov): a staged copy in LDS.
struct StateHead {
    double rot[9];
    double pos[3];
    double vel[3];
    double bias_g[3];
    double bias_a[3];
    double gravity[3];
};

// StatesGroup a - b (common_lib.h:576-587): Log(b.rot^T a.rot), then differences.
// S: livo_state or its StateHead.
template <class S>
__device__ __forceinline__ void state_minus_d(const S& a, const S& b, double* v) {
    double bt[9], ra[9], rd[9], v3[3];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) {
            bt[r * 3 + c] = b.rot[c * 3 + r];
            ra[r * 3 + c] = a.rot[r * 3 + c];
        }
    mat3_mul(bt, ra, rd);
    so3_log(rd, v3);
#pragma unroll
    for (int r = 0; r < 3; r++) {
        v[r] = v3[r];
        v[3 + r] = a.pos[r] - b.pos[r];
        v[6 + r] = a.vel[r] - b.vel[r];
        v[9 + r] = a.bias_g[r] - b.bias_g[r];
        v[12 + r] = a.bias_a[r] - b.bias_a[r];
        v[15 + r] = a.gravity[r] - b.gravity[r];
    }
}

// StatesGroup += (common_lib.h:565-574): rot * Exp(d0..2), the rest added.
template <class S>
__device__ __forceinline__ void state_boxplus_d(S& st, const double* sol) {
    double E[9], Rn[9];
    so3_exp(sol[0], sol[1], sol[2], E);
    mat3_mul(st.rot, E, Rn);
#pragma unroll
    for (int k = 0; k < 9; k++) st.rot[k] = Rn[k];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        st.pos[k] += sol[3 + k];
        st.vel[k] += sol[6 + k];
        st.bias_g[k] += sol[9 + k];
        st.bias_a[k] += sol[12 + k];
        st.gravity[k] += sol[15 + k];
    }
}

}  // namespace livo
