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
// LU (row-major N x N, rows in the swapped order) and the row permutation are
// in LDS.  Rows never move between lanes: each lane keeps its row and its
// position `pos` in the swapped order (a swap of rows k and p exchanges the two
// lanes' positions), the pivot is a wave max-reduction of (|a_k|, -pos) over
// the lanes at positions >= k (DPP within 16 lanes, one swizzle across), which
// is the sequential scan's first maximum, and the pivot row -- final once
// chosen -- is written to its place in s_LU, from where the lanes below read
// it.  Every a_ij sees the same operations in the same order as with the rows
// swapped in registers, so the factors are bit for bit those.
__device__ __forceinline__ void lu_pick(double& v, int& pos, double ov, int op) {
    // larger |a| wins; equal |a|: the smaller position (the scan's first maximum)
    const bool take = ov > v || (ov == v && op < pos);
    v = take ? ov : v;
    pos = take ? op : pos;
}
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int N>
__device__ __forceinline__ void wave_lu_to_lds(double (&A)[N], int lane, double* s_LU, int* s_piv) {
    static_assert(N <= 32, "rows on lanes 0..31");
    int pos = lane;
#pragma unroll
    for (int k = 0; k < N; k++) {
        // pivot: the first maximum of |a_ik| over positions i >= k (NaN never
        // replaces the running maximum: a NaN at position k keeps k, elsewhere it
        // is skipped)
        const bool live = lane < N && pos >= k;
        const bool nan_at_k = __ballot(lane < N && pos == k && A[k] != A[k]) != 0ull;
        double v = live && !(fabs(A[k]) != fabs(A[k])) ? fabs(A[k]) : -1.0;
        int pp = live ? pos : 0x7fffffff;
        // (only the steps the rows' lanes need: lanes 0..N-1)
        lu_pick(v, pp, dpp_f64<0xB1>(v), dpp_i32<0xB1>(pp));                      // quad_perm [1,0,3,2]
        if (N > 2) lu_pick(v, pp, dpp_f64<0x4E>(v), dpp_i32<0x4E>(pp));           // quad_perm [2,3,0,1]
        if (N > 4) lu_pick(v, pp, dpp_f64<0x141>(v), dpp_i32<0x141>(pp));         // row_half_mirror
        if (N > 8) lu_pick(v, pp, dpp_f64<0x140>(v), dpp_i32<0x140>(pp));         // row_mirror
        if (N > 16) lu_pick(v, pp, __shfl_xor(v, 16, 64), __shfl_xor(pp, 16, 64));
        int p = __builtin_amdgcn_readfirstlane(pp);
        if (nan_at_k) p = k;  // (a NaN at position k: the scan keeps k)
        // swap positions k and p (wave-uniform), then the row now at k is the pivot
        if (p != k) pos = pos == k ? p : (pos == p ? k : pos);
        if (lane < N && pos == k) {
#pragma unroll
            for (int j = 0; j < N; j++) s_LU[k * N + j] = A[j];
            s_piv[k] = lane;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // f = a_ik / a_kk, a_ij -= f * a_kj (rows below k)
        if (lane < N && pos > k) {
            const double f = A[k] / s_LU[k * N + k];
            A[k] = f;
#pragma unroll
            for (int j = k + 1; j < N; j++) A[j] = A[j] - f * s_LU[k * N + j];
        }
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

// The same column solve with the factors read from the lanes that hold them:
// after wave_lu_to_lds every lane's A is its row of the LU (row at position i
// on lane piv[i]), so L / U entries come by v_readlane from registers instead
// of as LDS broadcasts (no LDS round trip on the dependent chain).  The same
// operations in the same order: bit for bit lds_lu_column.  Every lane < N of
// the wave must hold its row (the caller keeps A from wave_lu_to_lds).
template <int N>
__device__ __forceinline__ void reg_lu_column(const double (&A)[N], const int* s_piv, int c, double (&y)[N]) {
    int pv[N];
#pragma unroll
    for (int i = 0; i < N; i++) pv[i] = __builtin_amdgcn_readfirstlane(s_piv[i]);
    // (scheduling barriers every 4 terms: the readlanes stay with their chain,
    // not hoisted ahead into more scalar registers than the kernel has)
#pragma unroll
    for (int i = 0; i < N; i++) {
        double sacc = (pv[i] == c) ? 1.0 : 0.0;
#pragma unroll
        for (int j = 0; j < i; j++) {
            sacc = sacc - bcast(A[j], pv[i]) * y[j];
            if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
        y[i] = sacc;
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = N - 1; i >= 0; i--) {
        double sacc = y[i];
#pragma unroll
        for (int j = i + 1; j < N; j++) {
            sacc = sacc - bcast(A[j], pv[i]) * y[j];
            if (((j - i) & 3) == 0) __builtin_amdgcn_sched_barrier(0);
        }
        y[i] = sacc / bcast(A[i], pv[i]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

#define WAVE_SYNC() do { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); __builtin_amdgcn_wave_barrier(); } while (0)

// Short-argument sine / cosine and arccosine near 1 for the IEKF's rotation
// increments (well under 0.5 rad, an arccosine argument near 1 for under 8
// degrees): Taylor series in nested form, within a few ulp of the library's
// (their next terms are below 1e-18 relative), and a fraction of its code.
// The solve runs once per scan per evaluation on a CU that has not run it
// recently, so its code is fetched cold (profiles/r06_tail_phases.txt): the
// library's argument reduction is in the instruction stream only for the rare
// large argument that takes it.
__device__ __forceinline__ void sincos_short(double x, double& s, double& c) {
    if (fabs(x) <= 0.5) {
        const double x2 = x * x;
        s = x * (1.0 - x2 / 6.0 * (1.0 - x2 / 20.0 * (1.0 - x2 / 42.0 * (1.0 - x2 / 72.0 *
                 (1.0 - x2 / 110.0 * (1.0 - x2 / 156.0 * (1.0 - x2 / 210.0)))))));
        c = 1.0 - x2 / 2.0 * (1.0 - x2 / 12.0 * (1.0 - x2 / 30.0 * (1.0 - x2 / 56.0 *
                 (1.0 - x2 / 90.0 * (1.0 - x2 / 132.0 * (1.0 - x2 / 182.0 * (1.0 - x2 / 240.0)))))));
    } else {
        s = sin(x);
        c = cos(x);
    }
}
__device__ __forceinline__ double acos_near1(double x) {
    if (x >= 0.99 && x <= 1.0) {  // acos(x) = 2 asin(y), y = sqrt((1 - x) / 2) <= 0.071
        const double y = sqrt((1.0 - x) * 0.5), y2 = y * y;
        const double a = y * (1.0 + y2 * (1.0 / 6.0 + y2 * (3.0 / 40.0 + y2 * (5.0 / 112.0 + y2 * (35.0 / 1152.0 +
                         y2 * (63.0 / 2816.0 + y2 * (231.0 / 13312.0 + y2 * (143.0 / 10240.0))))))));
        return 2.0 * a;
    }
    return acos(x);
}

// SO3 Exp / Log (so3_math.h:55-81) and 3x3 products, sums in index order.
__device__ __forceinline__ void so3_exp(double v1, double v2, double v3, double* R) {
    const double norm = sqrt(v1 * v1 + v2 * v2 + v3 * v3);
    _Pragma("unroll") for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (norm > 0.00001) {
        const double r[3] = {v1 / norm, v2 / norm, v3 / norm};
        const double K[9] = {0.0, -r[2], r[1], r[2], 0.0, -r[0], -r[1], r[0], 0.0};
        double s, cn;
        sincos_short(norm, s, cn);
        const double c1 = 1.0 - cn;
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
    const double theta = (tr > 3.0 - 1e-6) ? 0.0 : acos_near1(0.5 * (tr - 1));
    const double K[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
    if (fabs(theta) < 0.001) {
        _Pragma("unroll") for (int i = 0; i < 3; i++) o[i] = 0.5 * K[i];
    } else {
        double st, ct;
        sincos_short(theta, st, ct);
        const double f = 0.5 * theta / st;
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
