// vio_kernels.hip — CDNA4 (gfx950) kernels of the VIO photometric update
// (SURVEY.md §8f row 4): LidarSelector::UpdateState / ComputeJ,
// src/lidar_selection.cpp:748-978.
//
//   k_vio_begin   UpdateState's entry for one pyramid level: old_state =
//                 state, last_error = total_residual (1e10f), EKF_end = false.
//   k_vio_iter    one iteration: one visual point per thread -- projection
//                 (vikit PinholeCamera::world2cam), dpi (:90-100), the
//                 patch_size^2 bilinear residuals and their 6-wide Jacobian
//                 rows (:818-850), HᵀH / Hᵀz block partials; the last block
//                 then sums the patch errors in point order (float, as the
//                 reference's `error += patch_error`), reduces the partials in
//                 block order and, on one wave, runs the update: (cov /
//                 img_point_cov)^-1 once, K1 = (HᵀH + that)^-1 (columns 0..5,
//                 the only ones read), G, solution, boxplus, convergence, or
//                 the revert when the error grew (:855-891).
//   k_vio_end     ComputeJ's covariance update cov -= G cov (:975-978).
// Control stays on the device (VioCtrl): every launch of a finished level
// exits at its first instruction.  Numerics as livo_kernels.hip:
// -ffp-contract=off, the reference's float / double expression order.
#include <hip/hip_runtime.h>
#include <math.h>

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

struct VioLds {
    double wsum[4][32];
    double sum[32];
    double Pinv[kDim * kDim];
    double LU[kDim * kDim];
    double K1[kDim * 6];
    double HTH[36];
    double vec[kDim];
    double sol[kDim];
    int piv[kDim];
    float error;
    int last;
};

// The update of the last block (one wave): lidar_selection.cpp:851-891.
__device__ void vio_solve(const VioParams& P, VioLds& L, const int lane) {
    VioSlot* slot = P.slot;
    const int pst = P.ps * P.ps;
    // error = sum of patch errors in point order (float), / n_meas
    if (lane == 0) {
        float err = 0.0f;
        for (int i = 0; i < P.n; i++) err += P.perr[i];
        const int n_meas = P.n * pst;
        L.error = err / n_meas;
        slot->ctrl.n_meas = n_meas;
    }
    // HᵀH / Hᵀz: the block partials summed in block order
    if (lane < 27) {
        double v = P.partial[lane];
        for (int b = 1; b < P.nblk; b++) v = v + P.partial[(size_t)b * kVioCols + lane];
        L.sum[lane] = v;
    }
    WAVE_SYNC();
    const int li = 2 - slot->ctrl.level;
    const float error = L.error;
    bool end = false;
    if (error <= slot->ctrl.last_error) {
        for (int t = lane; t < (int)(sizeof(livo_state) / sizeof(double)); t += 64)
            reinterpret_cast<double*>(&slot->old_state)[t] = reinterpret_cast<const double*>(&slot->state)[t];
        for (int t = lane; t < 36; t += 64) {
            const int r = t / 6, c = t % 6;
            const int a = r < c ? r : c, b = r < c ? c : r;
            L.HTH[t] = L.sum[a * 6 - (a * (a - 1)) / 2 + (b - a)];
        }
        const bool row = lane < kDim;
        // (cov / img_point_cov)^-1, once: the covariance is fixed inside ComputeJ
        if (!slot->ctrl.pinv_ready) {
            double A[kDim];
#pragma unroll
            for (int j = 0; j < kDim; j++) A[j] = row ? slot->state.cov[lane * kDim + j] / P.img_cov : 0.0;
            wave_lu_to_lds<kDim>(A, lane, L.LU, L.piv);
            WAVE_SYNC();
            if (lane < kDim) {
                double y[kDim];
                lds_lu_column<kDim>(L.LU, L.piv, lane, y);
#pragma unroll
                for (int i = 0; i < kDim; i++) L.Pinv[i * kDim + lane] = y[i];
            }
            WAVE_SYNC();
            for (int t = lane; t < kDim * kDim; t += 64) slot->Pinv[t] = L.Pinv[t];
        } else {
            for (int t = lane; t < kDim * kDim; t += 64) L.Pinv[t] = slot->Pinv[t];
        }
        WAVE_SYNC();
        // K1 = (H_T_H + Pinv)^-1, columns 0..5
        {
            double A[kDim];
#pragma unroll
            for (int j = 0; j < kDim; j++)
                A[j] = row ? (((lane < 6 && j < 6) ? L.HTH[lane * 6 + j] : 0.0) + L.Pinv[lane * kDim + j]) : 0.0;
            if (lane < 6) {
                // HTH6 + Pinv in the oracle's order: A = Pinv, then the 6x6 block = HTH + Pinv
#pragma unroll
                for (int j = 0; j < 6; j++) A[j] = L.HTH[lane * 6 + j] + L.Pinv[lane * kDim + j];
            }
            wave_lu_to_lds<kDim>(A, lane, L.LU, L.piv);
            WAVE_SYNC();
            if (lane < 6) {
                double y[kDim];
                lds_lu_column<kDim>(L.LU, L.piv, lane, y);
#pragma unroll
                for (int i = 0; i < kDim; i++) L.K1[i * 6 + lane] = y[i];
            }
            WAVE_SYNC();
        }
        // G(:, 0:6) = K1(:, 0:6) HTH6
        for (int t = lane; t < kDim * 6; t += 64) {
            const int i = t / 6, j = t % 6;
            double g = L.K1[i * 6 + 0] * L.HTH[0 * 6 + j];
#pragma unroll
            for (int l = 1; l < 6; l++) g = g + L.K1[i * 6 + l] * L.HTH[l * 6 + j];
            slot->G6[t] = g;
        }
        if (lane == 0) state_minus_d(slot->prior, slot->state, L.vec);
        WAVE_SYNC();
        // solution = -K1(:,0:6) Hᵀz + vec - G(:,0:6) vec(0:6)
        if (row) {
            const int i = lane;
            double kz = L.K1[i * 6 + 0] * L.sum[21 + 0];
#pragma unroll
            for (int l = 1; l < 6; l++) kz = kz + L.K1[i * 6 + l] * L.sum[21 + l];
            double g = slot->G6[i * 6 + 0] * L.vec[0];
#pragma unroll
            for (int l = 1; l < 6; l++) g = g + slot->G6[i * 6 + l] * L.vec[l];
            L.sol[i] = (-kz + L.vec[i]) - g;
        }
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
        slot->ctrl.iters[li]++;
        slot->ctrl.iteration++;
        slot->ctrl.end = (end || slot->ctrl.iteration >= P.max_iter) ? 1 : 0;
        slot->ctrl.level_error[li] = slot->ctrl.last_error;
    }
}

__global__ __launch_bounds__(256) void k_vio_iter(VioParams P) {
    __shared__ VioLds L;
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
    // deterministic block partial: lanes (xor tree), then waves in order
#pragma unroll
    for (int k = 0; k < 27; k++) {
        const double v = wave_sum(acc[k]);
        if (lane == 0) L.wsum[w][k] = v;
    }
    __syncthreads();
    if (tid < 27) {
        double v = L.wsum[0][tid];
        for (int ww = 1; ww < 4; ww++) v = v + L.wsum[ww][tid];
        P.partial[(size_t)blockIdx.x * kVioCols + tid] = v;
    }
    // the last block to finish runs the update
    __threadfence();
    __syncthreads();
    if (tid == 0)
        L.last = __hip_atomic_fetch_add(&slot->ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                 (unsigned)(P.nblk - 1);
    __syncthreads();
    if (!L.last) return;
    __threadfence();
    if (w == 0) vio_solve(P, L, lane);
    if (tid == 0) slot->ticket = 0u;
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
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
int launch_vio_end(const VioParams& p, void* stream) {
    hipLaunchKernelGGL(k_vio_end, dim3(1), dim3(64), 0, (hipStream_t)stream, p);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

}  // namespace livo
