// vio_kernels.hip — CDNA4 (gfx950) kernels of the VIO photometric update
// (SURVEY.md §8f row 4): LidarSelector::UpdateState / ComputeJ,
// src/lidar_selection.cpp:748-978.
//
//   k_vio_begin   UpdateState's entry for one pyramid level: old_state =
//                 state, last_error = total_residual (1e10f), EKF_end = false.
//   k_vio_iter    one iteration: one visual point per thread -- projection
//                 (vikit PinholeCamera::world2cam), dpi (:90-100), the
//                 patch_size^2 bilinear residuals and their 6-wide Jacobian
//                 rows (:818-850), HᵀH / Hᵀz block partials and patch errors.
//   k_vio_solve   the iteration's update, one block: the patch errors summed
//                 in point order (float, as the reference's `error +=
//                 patch_error`) beside the partials' reduction in block order
//                 and the gain K1(:, 0:6) of (HᵀH + (cov / img_point_cov)^-1)^-1
//                 by one 6x6 LU, G, solution; then boxplus and convergence, or
//                 the revert when the error grew (:855-891).
//   k_vio_end     ComputeJ's covariance update cov -= G cov (:975-978).
// Control stays on the device (VioCtrl): every launch of a finished level
// exits at its first instruction.  Numerics as livo_kernels.hip:
// -ffp-contract=off, the reference's float / double expression order.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "device_common.h"
#include "device_linalg.h"
#include "livo_internal.h"

namespace livo {

__global__ void k_vio_begin(VioParams P, int level) {
    VioSlot* s = P.slot;
    for (int t = threadIdx.x; t < (int)(sizeof(livo_state) / sizeof(double)); t += blockDim.x)
        reinterpret_cast<double*>(&s->old_state)[t] = reinterpret_cast<const double*>(&s->state)[t];
    if (threadIdx.x == 0) {
        s->ctrl.level = level;
        s->ctrl.iteration = 0;
        s->ctrl.last_error = 1e10f;  // ComputeJ passes error = 1e10 to every level (:969-974)
        s->ctrl.end = (P.n <= 0 || P.max_iter <= 0) ? 1 : 0;
        s->ctrl.level_error[2 - level] = 1e10f;  // UpdateState returns total_residual if nothing updates
        s->ticket = 0u;
    }
}

__device__ __forceinline__ void vio_world2cam(const VioParams& P, const double* xyz, double* px) {
    const double u = xyz[0] / xyz[2], v = xyz[1] / xyz[2];  // project2d
    if (!P.distortion) {
        px[0] = P.fx * u + P.cx;
        px[1] = P.fy * v + P.cy;
        return;
    }
    const double x = u, y = v;
    const double r2 = x * x + y * y, r4 = r2 * r2, r6 = r4 * r2;
    const double a1 = 2 * x * y, a2 = r2 + 2 * x * x, a3 = r2 + 2 * y * y;
    const double cdist = 1 + P.d[0] * r2 + P.d[1] * r4 + P.d[4] * r6;
    const double xd = x * cdist + P.d[2] * a1 + P.d[3] * a2;
    const double yd = y * cdist + P.d[2] * a3 + P.d[3] * a1;
    px[0] = xd * P.fx + P.cx;
    px[1] = yd * P.fy + P.cy;
}

__device__ __forceinline__ void row3_mat(const double* r, const double* M, double* o) {
#pragma unroll
    for (int k = 0; k < 3; k++) o[k] = (r[0] * M[0 * 3 + k] + r[1] * M[1 * 3 + k]) + r[2] * M[2 * 3 + k];
}

// LDS of k_vio_solve (the patch errors are staged in dynamic LDS behind it).
struct VioSolveLds {
    double sum[32];
    double A[kDim * 6];   // (cov / img_point_cov)(:, 0:6)
    double C[36];         // H_T_H(0:6, 0:6)
    double M[36];         // I6 + C A(0:6, 0:6)
    double LU[36];
    double Minv[36];
    double K1[kDim * 6];  // K1(:, 0:6)
    double G6[kDim * 6];
    double vec[kDim];
    double sol[kDim];
    int piv[6];
    float error;
};

// The gain and the solution of one iteration (lidar_selection.cpp:855-866) on
// one wave, from the reduced sums: K1 = (H_T_H + (cov / img_point_cov)^-1)^-1
// is needed only in its columns 0..5 and H_T_H is zero outside its 6x6 block
// C, so with A = cov / img_point_cov, K1(:, 0:6) = A(:, 0:6) (I6 + C A66)^-1
// (livo_kernels.hip solve_scan's form: one 6x6 LU instead of two 18x18
// inversions); G(:, 0:6) = K1(:, 0:6) C, solution = -K1 Hᵀz + vec - G vec(0:6).
__device__ void vio_gain(const VioSlot* slot, VioSolveLds& L, const int lane) {
    if (lane < 36) {
        const int r = lane / 6, c = lane % 6;
        const int a = r < c ? r : c, b = r < c ? c : r;
        L.C[lane] = L.sum[a * 6 - (a * (a - 1)) / 2 + (b - a)];
    }
    if (lane == 0) state_minus_d(slot->prior, slot->state, L.vec);
    WAVE_SYNC();
    if (lane < 36) {
        const int r = lane / 6, c = lane % 6;
        double m = L.C[r * 6 + 0] * L.A[0 * 6 + c];
#pragma unroll
        for (int k = 1; k < 6; k++) m = m + L.C[r * 6 + k] * L.A[k * 6 + c];
        L.M[lane] = (r == c ? 1.0 : 0.0) + m;
    }
    WAVE_SYNC();
    double Ar[6];
#pragma unroll
    for (int j = 0; j < 6; j++) Ar[j] = lane < 6 ? L.M[lane * 6 + j] : 0.0;
    wave_lu_to_lds<6>(Ar, lane, L.LU, L.piv);
    WAVE_SYNC();
    {
        double y[6];
        reg_lu_column<6>(Ar, L.piv, lane, y);  // (readlanes: every lane runs it)
        if (lane < 6) {
#pragma unroll
            for (int i = 0; i < 6; i++) L.Minv[i * 6 + lane] = y[i];
        }
    }
    WAVE_SYNC();
    for (int t = lane; t < kDim * 6; t += 64) {
        const int r = t / 6, c = t % 6;
        double k1 = L.A[r * 6 + 0] * L.Minv[0 * 6 + c];
#pragma unroll
        for (int k = 1; k < 6; k++) k1 = k1 + L.A[r * 6 + k] * L.Minv[k * 6 + c];
        L.K1[t] = k1;
    }
    WAVE_SYNC();
    for (int t = lane; t < kDim * 6; t += 64) {
        const int i = t / 6, j = t % 6;
        double g = L.K1[i * 6 + 0] * L.C[0 * 6 + j];
#pragma unroll
        for (int l = 1; l < 6; l++) g = g + L.K1[i * 6 + l] * L.C[l * 6 + j];
        L.G6[t] = g;
    }
    WAVE_SYNC();
    if (lane < kDim) {
        const int i = lane;
        double kz = L.K1[i * 6 + 0] * L.sum[21 + 0];
#pragma unroll
        for (int l = 1; l < 6; l++) kz = kz + L.K1[i * 6 + l] * L.sum[21 + l];
        double g = L.G6[i * 6 + 0] * L.vec[0];
#pragma unroll
        for (int l = 1; l < 6; l++) g = g + L.G6[i * 6 + l] * L.vec[l];
        L.sol[i] = (-kz + L.vec[i]) - g;
    }
}

// One iteration's update (lidar_selection.cpp:851-891), one block after the
// iteration's k_vio_iter: the HᵀH / Hᵀz partials in block order (wave 0), the
// gain and solution (wave 1) beside the patch errors' float sum in point order
// (the reference's `error += patch_error`, serial by definition: thread 0 over
// the errors staged in LDS, `chunk` at a time), then the accept / revert.
__global__ __launch_bounds__(256) void k_vio_solve(VioParams P, int chunk) {
    __shared__ VioSolveLds L;
    extern __shared__ float s_err[];  // chunk floats
    VioSlot* slot = P.slot;
    if (slot->ctrl.end) return;  // block-uniform
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = P.n, pst = P.ps * P.ps;
    if (tid < 27) {
        // the block partials in order (the same additions as a serial loop), 16
        // loads in flight: one dependent load per block took ~1 us each (~80 us
        // per solve at 20k points)
        constexpr int kF = 16;
        double v = P.partial[tid];
        for (int b0 = 1; b0 < P.nblk; b0 += kF) {
            double x[kF];
#pragma unroll
            for (int k = 0; k < kF; k++) x[k] = b0 + k < P.nblk ? P.partial[(size_t)(b0 + k) * kVioCols + tid] : 0.0;
#pragma unroll
            for (int k = 0; k < kF; k++)
                if (b0 + k < P.nblk) v = v + x[k];
        }
        L.sum[tid] = v;
    }
    for (int t = tid; t < kDim * 6; t += 256) L.A[t] = slot->state.cov[(t / 6) * kDim + t % 6] / P.img_cov;
    float err = 0.0f;
    for (int base = 0; base < n; base += chunk) {
        const int cnt = min(chunk, n - base);
        for (int t = tid; t < cnt; t += 256) s_err[t] = P.perr[base + t];
        __syncthreads();
        if (base == 0 && w == 1) vio_gain(slot, L, lane);
        if (tid == 0) {
            // error += patch_error in point order (lidar_selection.cpp:849): one
            // dependent chain, its LDS reads 8 float4 ahead of the adds
            const float4* e4 = reinterpret_cast<const float4*>(s_err);
            int t = 0;
            for (; t + 32 <= cnt; t += 32) {
                float4 v[8];
#pragma unroll
                for (int k = 0; k < 8; k++) v[k] = e4[(t >> 2) + k];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    err += v[k].x;
                    err += v[k].y;
                    err += v[k].z;
                    err += v[k].w;
                }
            }
            for (; t + 4 <= cnt; t += 4) {
                const float4 v = e4[t >> 2];
                err += v.x;
                err += v.y;
                err += v.z;
                err += v.w;
            }
            for (; t < cnt; t++) err += s_err[t];
        }
        __syncthreads();
    }
    if (w > 0) return;
    const int n_meas = n * pst;
    const float error = __shfl(err, 0) / n_meas;
    const int li = 2 - slot->ctrl.level;
    bool end = false;
    if (error <= slot->ctrl.last_error) {
        for (int t = lane; t < (int)(sizeof(livo_state) / sizeof(double)); t += 64)
            reinterpret_cast<double*>(&slot->old_state)[t] = reinterpret_cast<const double*>(&slot->state)[t];
        for (int t = lane; t < kDim * 6; t += 64) slot->G6[t] = L.G6[t];
        WAVE_SYNC();
        if (lane == 0) {
            double sol[kDim];
#pragma unroll
            for (int k = 0; k < kDim; k++) sol[k] = L.sol[k];
            state_boxplus_d(slot->state, sol);
            const double rn = sqrt((sol[0] * sol[0] + sol[1] * sol[1]) + sol[2] * sol[2]);
            const double tn = sqrt((sol[3] * sol[3] + sol[4] * sol[4]) + sol[5] * sol[5]);
            end = (rn * 57.3f < 0.001f) && (tn * 100.0f < 0.001f);
            slot->ctrl.pinv_ready = 1;
            slot->ctrl.last_error = error;
            slot->ctrl.updates[li]++;
        }
    } else {
        for (int t = lane; t < (int)(sizeof(livo_state) / sizeof(double)); t += 64)
            reinterpret_cast<double*>(&slot->state)[t] = reinterpret_cast<const double*>(&slot->old_state)[t];
        end = true;
    }
    WAVE_SYNC();
    if (lane == 0) {
        slot->ctrl.n_meas = n_meas;
        slot->ctrl.iters[li]++;
        slot->ctrl.iteration++;
        slot->ctrl.end = (end || slot->ctrl.iteration >= P.max_iter) ? 1 : 0;
        slot->ctrl.level_error[li] = slot->ctrl.last_error;
    }
}

__global__ __launch_bounds__(256) void k_vio_iter(VioParams P) {
    VioSlot* slot = P.slot;
    if (slot->ctrl.end) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i = blockIdx.x * 256 + tid;
    const int level = P.level, ps = P.ps, pst = ps * ps, ph = ps / 2, width = P.w;
    double acc[27];
#pragma unroll
    for (int k = 0; k < 27; k++) acc[k] = 0.0;
    if (i < P.n) {
        const livo_state& st = slot->state;
        double RwiT[9], Rcw[9], Pcw[3], pf[3], pc[2];
#pragma unroll
        for (int a = 0; a < 3; a++)
#pragma unroll
            for (int b = 0; b < 3; b++) RwiT[a * 3 + b] = st.rot[b * 3 + a];
        mat3_mul(P.Rci, RwiT, Rcw);  // Rcw = Jdp_dt
#pragma unroll
        for (int k = 0; k < 3; k++) Pcw[k] = -((Rcw[k * 3 + 0] * st.pos[0] + Rcw[k * 3 + 1] * st.pos[1]) + Rcw[k * 3 + 2] * st.pos[2]) + P.Pci[k];
        const double* pw = P.pos + 3 * (size_t)i;
#pragma unroll
        for (int k = 0; k < 3; k++) pf[k] = ((Rcw[k * 3 + 0] * pw[0] + Rcw[k * 3 + 1] * pw[1]) + Rcw[k * 3 + 2] * pw[2]) + Pcw[k];
        vio_world2cam(P, pf, pc);
        const double zi = 1. / pf[2], zi2 = zi * zi;
        const double Jdpi[6] = {P.fx * zi, 0.0, -P.fx * pf[0] * zi2, 0.0, P.fy * zi, -P.fy * pf[1] * zi2};
        const double p_hat[9] = {0.0, -pf[2], pf[1], pf[2], 0.0, -pf[0], -pf[1], pf[0], 0.0};
        const int scale = 1 << (level + P.levels[i]);
        const float u_ref = (float)pc[0], v_ref = (float)pc[1];
        const int u_ref_i = (int)(floorf((float)(pc[0] / scale)) * scale);
        const int v_ref_i = (int)(floorf((float)(pc[1] / scale)) * scale);
        const float su = (u_ref - u_ref_i) / scale, sv = (v_ref - v_ref_i) / scale;
        const float w_tl = (1.0 - su) * (1.0 - sv), w_tr = su * (1.0 - sv), w_bl = (1.0 - su) * sv, w_br = su * sv;
        const float* Pt = P.patches + (size_t)i * 3 * pst;
        float patch_error = 0.0f;
        unsigned oof = 0;
        for (int x = 0; x < ps; x++) {
            const int row0 = v_ref_i + x * scale - ph * scale;
            for (int y = 0; y < ps; ++y) {
                const int col0 = u_ref_i - ph * scale + y * scale;
                const int s = scale;
                oof += (row0 - s < 0 || row0 + 2 * s >= P.h || col0 - s < 0 || col0 + 2 * s >= P.w) ? 1u : 0u;
                auto I = [&](int dr, int dc) -> float {
                    int r = row0 + dr, c = col0 + dc;
                    r = r < 0 ? 0 : (r >= P.h ? P.h - 1 : r);
                    c = c < 0 ? 0 : (c >= P.w ? P.w - 1 : c);
                    return (float)P.img[(size_t)r * width + c];
                };
                const float du = 0.5f * ((w_tl * I(0, s) + w_tr * I(0, 2 * s) + w_bl * I(s, s) + w_br * I(s, 2 * s)) -
                                         (w_tl * I(0, -s) + w_tr * I(0, 0) + w_bl * I(s, -s) + w_br * I(s, 0)));
                const float dv = 0.5f * ((w_tl * I(s, 0) + w_tr * I(s, s) + w_bl * I(2 * s, 0) + w_br * I(2 * s, s)) -
                                         (w_tl * I(-s, 0) + w_tr * I(-s, s) + w_bl * I(0, 0) + w_br * I(0, s)));
                const double j0 = (double)du * (1.0 / scale), j1 = (double)dv * (1.0 / scale);
                double t[3], Jdphi[3], Jdp[3], a[3], b[3], h[6];
#pragma unroll
                for (int k = 0; k < 3; k++) t[k] = j0 * Jdpi[k] + j1 * Jdpi[3 + k];
                row3_mat(t, p_hat, Jdphi);
#pragma unroll
                for (int k = 0; k < 3; k++) Jdp[k] = -j0 * Jdpi[k] + -j1 * Jdpi[3 + k];
                row3_mat(Jdphi, P.Jdphi_dR, a);
                row3_mat(Jdp, P.Jdp_dR, b);
#pragma unroll
                for (int k = 0; k < 3; k++) h[k] = a[k] + b[k];
                row3_mat(Jdp, Rcw, h + 3);
                const double res = (double)(w_tl * I(0, 0) + w_tr * I(0, s) + w_bl * I(s, 0) + w_br * I(s, s) -
                                            Pt[pst * level + x * ps + y]);
                patch_error += res * res;
                int q = 0;
#pragma unroll
                for (int r = 0; r < 6; r++)
#pragma unroll
                    for (int c = r; c < 6; c++) acc[q++] += h[r] * h[c];
#pragma unroll
                for (int r = 0; r < 6; r++) acc[21 + r] += h[r] * res;
            }
        }
        P.perr[i] = patch_error;
        if (oof) atomicAdd(&slot->ctrl.oof, (unsigned long long)oof);
    }
    // deterministic block partial: lanes (xor tree), then waves in order; the
    // iteration's update runs in k_vio_solve behind this launch
    __shared__ double wsum[4][32];
#pragma unroll
    for (int k = 0; k < 27; k++) {
        const double v = wave_sum(acc[k]);
        if (lane == 0) wsum[w][k] = v;
    }
    __syncthreads();
    if (tid < 27) {
        double v = wsum[0][tid];
        for (int ww = 1; ww < 4; ww++) v = v + wsum[ww][tid];
        P.partial[(size_t)blockIdx.x * kVioCols + tid] = v;
    }
}

// ComputeJ's covariance update (:975-978): if the last level's error < 1e10,
// cov -= G * cov, with G(:, 6:18) = 0.
__global__ __launch_bounds__(64) void k_vio_end(VioParams P) {
    VioSlot* slot = P.slot;
    if (P.n <= 0 || !(slot->ctrl.level_error[2] < 1e10f)) return;
    __shared__ double cov[kDim * kDim];
    for (int t = threadIdx.x; t < kDim * kDim; t += 64) cov[t] = slot->state.cov[t];
    __syncthreads();
    for (int t = threadIdx.x; t < kDim * kDim; t += 64) {
        const int i = t / kDim, j = t % kDim;
        double g = slot->G6[i * 6 + 0] * cov[0 * kDim + j];
#pragma unroll
        for (int l = 1; l < 6; l++) g = g + slot->G6[i * 6 + l] * cov[l * kDim + j];
        slot->state.cov[t] = cov[t] - g;
    }
    if (threadIdx.x == 0) slot->ctrl.cov_updated = 1;
}

int launch_vio_begin(const VioParams& p, int level, void* stream) {
    hipLaunchKernelGGL(k_vio_begin, dim3(1), dim3(64), 0, (hipStream_t)stream, p, level);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
int launch_vio_iter(const VioParams& p, void* stream) {
    if (p.n <= 0) return LIVO_OK;
    hipLaunchKernelGGL(k_vio_iter, dim3((unsigned)p.nblk), dim3(256), 0, (hipStream_t)stream, p);
    if (hipGetLastError() != hipSuccess) return LIVO_E_HIP;
    // the errors staged 24k at a time (96 KB of LDS; one workgroup may take 160 KB)
    const int chunk = (int)std::min<int64_t>(((int64_t)p.n + 3) & ~(int64_t)3, 24576);
    hipLaunchKernelGGL(k_vio_solve, dim3(1), dim3(256), (size_t)chunk * sizeof(float), (hipStream_t)stream, p, chunk);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
int launch_vio_end(const VioParams& p, void* stream) {
    hipLaunchKernelGGL(k_vio_end, dim3(1), dim3(64), 0, (hipStream_t)stream, p);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

}  // namespace livo
