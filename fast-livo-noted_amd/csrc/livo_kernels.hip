// livo_kernels.hip — CDNA4 (gfx950) kernels of the LIO scan-to-map IEKF path.
//
//   k_knn_pass<SEEDED> exact k=5 NN of every scan point (ikd_Tree.cpp:350-380,
//                      843-986) after pointBodyToWorld (laser_mapping.cpp:662-671),
//                      one point per thread, writing one 128-B neighbour record per
//                      point (the Nearest_Points cache, laser_mapping.h:165).
//                      !SEEDED = the first evaluation of an update (every point);
//                      SEEDED = rematch evaluations (where the device-side
//                      nearest_search_en of a scan is set), bounded by the
//                      previous neighbours.  k_knn_replay recomputes the rare
//                      queries whose answer could depend on tie order with the
//                      exact reference heap and visiting order.
//   k_hshare<FIRST>    one thread per point, coalesced: plane fit (esti_plane,
//                      common_lib.h:670-702), residual and gates
//                      (laser_mapping.cpp:518,532-543,552), Jacobian row and the
//                      HᵀH / HᵀL block partials (laser_mapping.cpp:564-593).
//   k_solve            one wave per scan: deterministic reduction of the block
//                      partials, the 18x18 solve (rows on lanes, in registers),
//                      boxplus, convergence and rematch control, covariance update
//                      (laser_mapping.cpp:171-238, common_lib.h:565-587).
//
// Numerics: compiled with -ffp-contract=off and correctly rounded f32
// division/sqrt, and every expression keeps the reference's operation order,
// so the float plane fit and the float k-NN distances are bit-identical to
// the CPU restatement (oracle/livo_oracle.cpp).  Doubles are summed in a
// fixed order (wave shuffle tree -> LDS -> block order) so results are
// reproducible run to run.
#include <hip/hip_runtime.h>
#include <math.h>

#include <utility>

#include "livo_internal.h"
#include "device_common.h"
#include "device_linalg.h"

#if defined(LIVO_EVAL_PROF) && !defined(LIVO_TAIL_PROF)
#define LIVO_TAIL_PROF  // the tail / solve phase marks alone: no per-block atomics (tools/tail_prof.py)
#endif

namespace livo {

// Global addressing for the sc1 accessors' pointers (struct fields copied from
// the job tables arrive generic): a generic (flat) access also counts against
// the 4-bit LDS counter, so at most 15 are in flight per wave where global
// loads keep up to 63.  Atomic accesses only: a plain load through a global,
// block-uniform pointer may become a scalar load, which does not see other
// CUs' stores within a launch.
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gptr(const T* p) {
    return (const __attribute__((address_space(1))) T*)p;
}
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}
// ========================================================= IKFoM path =====
// The IKFoM formulation: state_ikfom (use-ikfom.hpp:12-21),
// the legacy h-model (origin_laserMapping.cpp:916-1048) and
// esekf::update_iterated_dyn_share_modified (esekfom.hpp:1619-1928) with the
// MTK pieces it uses.  Same operation order as oracle/livo_oracle.cpp.
constexpr double kMtkTol = 1e-11;            // MTK::tolerance<double>() (mtkmath.hpp:122)
constexpr double kS2Len = 98090.0 / 10000.0;  // S2<double, 98090, 10000, 1> (use-ikfom.hpp:9)

struct Qd {
    double w, x, y, z;
};
__device__ __forceinline__ Qd qd_mul(const Qd& a, const Qd& b) {  // Eigen generic quat_product
    return Qd{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
              a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z, a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ Qd qd_conj(const Qd& q) { return Qd{q.w, -q.x, -q.y, -q.z}; }
__device__ __forceinline__ Qd qd_load(const double* a) { return Qd{a[0], a[1], a[2], a[3]}; }
__device__ __forceinline__ void qd_store(const Qd& q, double* a) { a[0] = q.w; a[1] = q.x; a[2] = q.y; a[3] = q.z; }
__device__ __forceinline__ void cross3d(const double* a, const double* b, double* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
// Eigen::QuaternionBase::_transformVector
__device__ __forceinline__ void qd_rot(const Qd& q, const double* v, double* o) {
    const double qv[3] = {q.x, q.y, q.z};
    double uv[3], c[3];
    cross3d(qv, v, uv);
    _Pragma("unroll") for (int i = 0; i < 3; i++) uv[i] = uv[i] + uv[i];
    cross3d(qv, uv, c);
    _Pragma("unroll") for (int i = 0; i < 3; i++) o[i] = (v[i] + q.w * uv[i]) + c[i];
}
__device__ __forceinline__ void qd_mat(const Qd& q, double* R) {  // toRotationMatrix
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
__device__ __forceinline__ void hat3d(const double* v, double* H) {
    H[0] = 0; H[1] = -v[2]; H[2] = v[1];
    H[3] = v[2]; H[4] = 0; H[5] = -v[0];
    H[6] = -v[1]; H[7] = v[0]; H[8] = 0;
}
__device__ __forceinline__ void mat3d_mul(const double* A, const double* B, double* C) {
    _Pragma("unroll") for (int i = 0; i < 3; i++)
        _Pragma("unroll") for (int j = 0; j < 3; j++)
            C[i * 3 + j] = (A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j]) + A[i * 3 + 2] * B[2 * 3 + j];
}
__device__ __forceinline__ void mat3d_vec(const double* M, const double* v, double* o) {
    _Pragma("unroll") for (int r = 0; r < 3; r++) o[r] = (M[r * 3] * v[0] + M[r * 3 + 1] * v[1]) + M[r * 3 + 2] * v[2];
}
// MTK::cos_sinc_sqrt (mtkmath.hpp:142-171)
__device__ __forceinline__ void cos_sinc_sqrt_d(double x2, double& c, double& sc) {
    const double taylor_0 = 2.220446049250313e-16, taylor_2 = sqrt(taylor_0), taylor_n = sqrt(taylor_2);
    if (x2 >= taylor_n) {
        const double x = sqrt(x2);
        c = cos(x);
        sc = sin(x) / x;
        return;
    }
    const double inv[7] = {1 / 3., 1 / 4., 1 / 5., 1 / 6., 1 / 7., 1 / 8., 1 / 9.};
    double cosi = 1., sinc = 1;
    double term = -1 / 2. * x2;
    _Pragma("unroll") for (int i = 0; i < 3; ++i) {
        cosi += term;
        term *= inv[2 * i];
        sinc += term;
        term *= -inv[2 * i + 1] * x2;
    }
    c = cosi;
    sc = sinc;
}
__device__ __forceinline__ Qd mtk_exp_d(const double* v, double scale) {  // MTK::exp -> quaternion
    const double norm2 = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2];
    double c, sc;
    cos_sinc_sqrt_d(scale * scale * norm2, c, sc);
    const double mult = sc * scale;
    return Qd{c, mult * v[0], mult * v[1], mult * v[2]};
}
__device__ __forceinline__ void so3_log_qd(const Qd& q, double* o) {  // SO3::log (periodic)
    double nv = sqrt((q.x * q.x + q.y * q.y) + q.z * q.z);
    if (nv < kMtkTol) nv = kMtkTol;
    const double s = 2.0 / nv * atan(nv / q.w);
    o[0] = s * q.x;
    o[1] = s * q.y;
    o[2] = s * q.z;
}
__device__ __forceinline__ void A_matrix_d(const double* v, double* A) {  // MTK::A_matrix
    const double sq = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    const double norm = sqrt(sq);
    _Pragma("unroll") for (int i = 0; i < 9; i++) A[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (norm < kMtkTol) return;
    double H[9], HH[9];
    hat3d(v, H);
    mat3d_mul(H, H, HH);
    const double a = (1 - cos(norm)) / sq, b = (1 - sin(norm) / norm) / sq;
    _Pragma("unroll") for (int i = 0; i < 9; i++) A[i] = (A[i] + a * H[i]) + b * HH[i];
}
__device__ __forceinline__ void s2_Bx_d(const double* vec, double* B) {  // S2_Bx, S2_typ = 1
    const double L = kS2Len;
    if (vec[0] + L > kMtkTol) {
        B[0] = -vec[1];
        B[1] = -vec[2];
        B[2] = L - vec[1] * vec[1] / (L + vec[0]);
        B[3] = -vec[2] * vec[1] / (L + vec[0]);
        B[4] = -vec[2] * vec[1] / (L + vec[0]);
        B[5] = L - vec[2] * vec[2] / (L + vec[0]);
        _Pragma("unroll") for (int i = 0; i < 6; i++) B[i] /= L;
    } else {
        _Pragma("unroll") for (int i = 0; i < 6; i++) B[i] = 0.0;
        B[3] = -1;
        B[4] = 1;
    }
}
__device__ __forceinline__ void s2_boxplus_d(double* vec, const double* delta) {
    double B[6];
    s2_Bx_d(vec, B);
    const double Bu[3] = {B[0] * delta[0] + B[1] * delta[1], B[2] * delta[0] + B[3] * delta[1],
                          B[4] * delta[0] + B[5] * delta[1]};
    const Qd r = mtk_exp_d(Bu, 0.5);
    double R[9], o[3];
    qd_mat(r, R);
    mat3d_vec(R, vec, o);
    vec[0] = o[0];
    vec[1] = o[1];
    vec[2] = o[2];
}
__device__ __forceinline__ void s2_boxminus_d(const double* vec, const double* other, double* res) {
    double H[9], hv[3];
    hat3d(vec, H);
    mat3d_vec(H, other, hv);
    const double v_sin = sqrt((hv[0] * hv[0] + hv[1] * hv[1]) + hv[2] * hv[2]);
    const double v_cos = (vec[0] * other[0] + vec[1] * other[1]) + vec[2] * other[2];
    const double theta = atan2(v_sin, v_cos);
    if (v_sin < kMtkTol) {
        res[0] = fabs(theta) > kMtkTol ? 3.1415926 : 0.0;
        res[1] = 0.0;
        return;
    }
    double B[6], Ho[9], t[3];
    s2_Bx_d(other, B);
    hat3d(other, Ho);
    mat3d_vec(Ho, vec, t);
    const double f = theta / v_sin;
    _Pragma("unroll") for (int r = 0; r < 2; r++) res[r] = f * ((B[0 * 2 + r] * t[0] + B[1 * 2 + r] * t[1]) + B[2 * 2 + r] * t[2]);
}
// J = S2_Nx_yy(x.grav) * S2_Mx(xp.grav, seg)  (2x2; exp_delta in S2_Mx is the identity)
__device__ __forceinline__ void s2_J_d(const double* gx, const double* gp, const double* seg, double* J) {
    double B[6], H[9], N[6], M[6];
    s2_Bx_d(gx, B);
    hat3d(gx, H);
    const double f = 1 / kS2Len / kS2Len;
    _Pragma("unroll") for (int r = 0; r < 2; r++)
        _Pragma("unroll") for (int c = 0; c < 3; c++)
            N[r * 3 + c] = f * ((B[0 * 2 + r] * H[0 * 3 + c] + B[1 * 2 + r] * H[1 * 3 + c]) + B[2 * 2 + r] * H[2 * 3 + c]);
    s2_Bx_d(gp, B);
    hat3d(gp, H);
    const double dn = sqrt(seg[0] * seg[0] + seg[1] * seg[1]);
    if (dn < kMtkTol) {
        _Pragma("unroll") for (int r = 0; r < 3; r++)
            _Pragma("unroll") for (int c = 0; c < 2; c++)
                M[r * 2 + c] = -((H[r * 3 + 0] * B[0 * 2 + c] + H[r * 3 + 1] * B[1 * 2 + c]) + H[r * 3 + 2] * B[2 * 2 + c]);
    } else {
        const double Bu[3] = {B[0] * seg[0] + B[1] * seg[1], B[2] * seg[0] + B[3] * seg[1], B[4] * seg[0] + B[5] * seg[1]};
        double A[9], AT[9], HA[9];
        A_matrix_d(Bu, A);
        _Pragma("unroll") for (int r = 0; r < 3; r++)
            _Pragma("unroll") for (int c = 0; c < 3; c++) AT[r * 3 + c] = A[c * 3 + r];
        mat3d_mul(H, AT, HA);
        _Pragma("unroll") for (int r = 0; r < 3; r++)
            _Pragma("unroll") for (int c = 0; c < 2; c++)
                M[r * 2 + c] = -((HA[r * 3 + 0] * B[0 * 2 + c] + HA[r * 3 + 1] * B[1 * 2 + c]) + HA[r * 3 + 2] * B[2 * 2 + c]);
    }
    _Pragma("unroll") for (int r = 0; r < 2; r++)
        _Pragma("unroll") for (int c = 0; c < 2; c++)
            J[r * 2 + c] = (N[r * 3 + 0] * M[0 * 2 + c] + N[r * 3 + 1] * M[1 * 2 + c]) + N[r * 3 + 2] * M[2 * 2 + c];
}
__device__ __forceinline__ void so3_J_d(const double* seg, double* J) {  // A_matrix(seg)^T
    double A[9];
    A_matrix_d(seg, A);
    _Pragma("unroll") for (int r = 0; r < 3; r++)
        _Pragma("unroll") for (int c = 0; c < 3; c++) J[r * 3 + c] = A[c * 3 + r];
}
__device__ __forceinline__ void ik_boxplus_d(livo_ikfom_state& s, const double* dx) {
    _Pragma("unroll") for (int i = 0; i < 3; i++) s.pos[i] += dx[i];
    qd_store(qd_mul(qd_load(s.rot), mtk_exp_d(dx + 3, 0.5)), s.rot);
    qd_store(qd_mul(qd_load(s.offset_R), mtk_exp_d(dx + 6, 0.5)), s.offset_R);
    _Pragma("unroll") for (int i = 0; i < 3; i++) {
        s.offset_T[i] += dx[9 + i];
        s.vel[i] += dx[12 + i];
        s.bg[i] += dx[15 + i];
        s.ba[i] += dx[18 + i];
    }
    s2_boxplus_d(s.grav, dx + 21);
}
__device__ __forceinline__ void ik_boxminus_d(const livo_ikfom_state& a, const livo_ikfom_state& b, double* dx) {
    _Pragma("unroll") for (int i = 0; i < 3; i++) dx[i] = a.pos[i] - b.pos[i];
    so3_log_qd(qd_mul(qd_conj(qd_load(b.rot)), qd_load(a.rot)), dx + 3);
    so3_log_qd(qd_mul(qd_conj(qd_load(b.offset_R)), qd_load(a.offset_R)), dx + 6);
    _Pragma("unroll") for (int i = 0; i < 3; i++) {
        dx[9 + i] = a.offset_T[i] - b.offset_T[i];
        dx[12 + i] = a.vel[i] - b.vel[i];
        dx[15 + i] = a.bg[i] - b.bg[i];
        dx[18 + i] = a.ba[i] - b.ba[i];
    }
    s2_boxminus_d(a.grav, b.grav, dx + 21);
}
// p_global = rot * (offset_R * p_body + offset_T) + pos (origin_laserMapping.cpp:937), stored as float
__device__ __forceinline__ void ik_world_point(const livo_ikfom_state& s, float bx, float by, float bz, float& wx,
                                               float& wy, float& wz) {
    const double b[3] = {(double)bx, (double)by, (double)bz};
    double t0[3], t1[3], g[3];
    qd_rot(qd_load(s.offset_R), b, t0);
    _Pragma("unroll") for (int c = 0; c < 3; c++) t1[c] = t0[c] + s.offset_T[c];
    qd_rot(qd_load(s.rot), t1, g);
    wx = (float)(g[0] + s.pos[0]);
    wy = (float)(g[1] + s.pos[1]);
    wz = (float)(g[2] + s.pos[2]);
}


// ============================================================== k-NN ======
// PointType_CMP::operator< (ikd_Tree.h:57-60).
__device__ __forceinline__ bool cand_less(float da, float xa, float db, float xb) {
    if ((double)fabsf(da - db) < 1e-10) return xa < xb;
    return da < db;
}

// MANUAL_HEAP (ikd_Tree.cpp:1345-1411) with capacity 2k and at most k = 5
// live entries, held in registers: every slot index below is a compile-time
// constant (the runtime heap size only selects a branch), so nothing spills
// to scratch.  The same FloatUp / MoveDown steps as the reference keep even
// the order of entries that compare equal (duplicate points) identical.
struct KHeap {
    float d[kNN];
    float x[kNN];
    uint32_t node[kNN];  // heap index of the map record
    int size;
};

#define KH_CPY(h, i, j) do { (h).d[i] = (h).d[j]; (h).x[i] = (h).x[j]; (h).node[i] = (h).node[j]; } while (0)
#define KH_SET(h, i, cd, cx, cn) do { (h).d[i] = (cd); (h).x[i] = (cx); (h).node[i] = (cn); } while (0)
#define KH_LT(h, i, cd, cx) cand_less((h).d[i], (h).x[i], (cd), (cx))     /* heap[i] < c */
#define KH_GT(h, i, cd, cx) cand_less((cd), (cx), (h).d[i], (h).x[i])     /* c < heap[i] */

// push into a heap of size s < 5: FloatUp from slot s.
__device__ __forceinline__ void kh_push(KHeap& h, float cd, float cx, uint32_t cn) {
    const int s = h.size;
    if (s == 0) {
        KH_SET(h, 0, cd, cx, cn);
    } else if (s == 1) {
        if (KH_LT(h, 0, cd, cx)) { KH_CPY(h, 1, 0); KH_SET(h, 0, cd, cx, cn); } else KH_SET(h, 1, cd, cx, cn);
    } else if (s == 2) {
        if (KH_LT(h, 0, cd, cx)) { KH_CPY(h, 2, 0); KH_SET(h, 0, cd, cx, cn); } else KH_SET(h, 2, cd, cx, cn);
    } else if (s == 3) {
        if (KH_LT(h, 1, cd, cx)) {
            KH_CPY(h, 3, 1);
            if (KH_LT(h, 0, cd, cx)) { KH_CPY(h, 1, 0); KH_SET(h, 0, cd, cx, cn); } else KH_SET(h, 1, cd, cx, cn);
        } else KH_SET(h, 3, cd, cx, cn);
    } else {
        if (KH_LT(h, 1, cd, cx)) {
            KH_CPY(h, 4, 1);
            if (KH_LT(h, 0, cd, cx)) { KH_CPY(h, 1, 0); KH_SET(h, 0, cd, cx, cn); } else KH_SET(h, 1, cd, cx, cn);
        } else KH_SET(h, 4, cd, cx, cn);
    }
    h.size = s + 1;
}

// pop the top of a heap of size s >= 1: heap[0] = heap[s-1], MoveDown(0).
__device__ __forceinline__ void kh_pop(KHeap& h) {
    const int s = h.size;
    if (s <= 1) { h.size = 0; return; }
    float td, tx;
    uint32_t tn;
    if (s == 5) { td = h.d[4]; tx = h.x[4]; tn = h.node[4]; }
    else if (s == 4) { td = h.d[3]; tx = h.x[3]; tn = h.node[3]; }
    else if (s == 3) { td = h.d[2]; tx = h.x[2]; tn = h.node[2]; }
    else { td = h.d[1]; tx = h.x[1]; tn = h.node[1]; }
    const int ns = s - 1;  // heap_size after the pop (1..4)
    if (ns == 1) {
        KH_SET(h, 0, td, tx, tn);
    } else if (ns == 2) {
        if (KH_GT(h, 1, td, tx)) { KH_CPY(h, 0, 1); KH_SET(h, 1, td, tx, tn); } else KH_SET(h, 0, td, tx, tn);
    } else {
        // ns = 3 or 4: l = 1, or 2 if heap[1] < heap[2]
        const bool right = cand_less(h.d[1], h.x[1], h.d[2], h.x[2]);
        if (!right) {
            if (KH_GT(h, 1, td, tx)) {
                KH_CPY(h, 0, 1);
                if (ns == 4 && KH_GT(h, 3, td, tx)) { KH_CPY(h, 1, 3); KH_SET(h, 3, td, tx, tn); }
                else KH_SET(h, 1, td, tx, tn);
            } else KH_SET(h, 0, td, tx, tn);
        } else {
            if (KH_GT(h, 2, td, tx)) { KH_CPY(h, 0, 2); KH_SET(h, 2, td, tx, tn); } else KH_SET(h, 0, td, tx, tn);
        }
    }
    h.size = ns;
}

// The candidate list handed back by Nearest_Search (:374-378): the heap
// popped top-first and inserted at the front, i.e. ascending.
struct Cands {
    float d[kNN];
    uint32_t node[kNN];
    int n;
};

__device__ __forceinline__ void kh_extract(KHeap& h, Cands& c) {
    const int found = h.size;
    float pd[kNN];
    uint32_t pn[kNN];
#pragma unroll
    for (int i = 0; i < kNN; i++) {  // pd[i] = i-th pop (descending)
        pd[i] = h.d[0];
        pn[i] = h.node[0];
        if (i < found) kh_pop(h);
    }
#pragma unroll
    for (int j = 0; j < kNN; j++) {  // c[j] = pop number found-1-j
        float dj = INFINITY;
        uint32_t nj = 0u;
#pragma unroll
        for (int i = 0; i < kNN; i++)
            if (i == found - 1 - j) { dj = pd[i]; nj = pn[i]; }
        c.d[j] = dj;
        c.node[j] = nj;
    }
    c.n = found;
}

// calc_box_dist (ikd_Tree.cpp:1297-1307), same add order.
__device__ __forceinline__ float box_dist(float px, float py, float pz, float x0, float x1, float y0, float y1,
                                          float z0, float z1) {
    float m = 0.0f;
    float t;
    t = px - x0; if (px < x0) m = m + t * t;
    t = px - x1; if (px > x1) m = m + t * t;
    t = py - y0; if (py < y0) m = m + t * t;
    t = py - y1; if (py > y1) m = m + t * t;
    t = pz - z0; if (pz < z0) m = m + t * t;
    t = pz - z1; if (pz > z1) m = m + t * t;
    return m;
}

__device__ __forceinline__ const float4* rec_ptr(const MapNode* nodes, uint32_t h) {
    return reinterpret_cast<const float4*>(nodes + (size_t)h + 1);
}

__device__ __forceinline__ int level_of(uint32_t h) { return 31 - __clz(h + 1); }

// Reference k-NN: the visiting order of KD_TREE::Search (ikd_Tree.cpp:843-986)
// with the exact MANUAL_HEAP (ikd_Tree.cpp:1345-1411), without a stack.  At
// each node the point is offered to the heap; then the sons are taken
// near-first (left on a tie, :869), each only if the heap is not full or its
// box distance is below the current top at the moment it is reached.  With
// heap-ordered records the pending far son of every level fits in one bit of
// `trail`; when a subtree is finished the traversal jumps to the deepest
// ancestor with a pending far son, re-reads that (already visited, cached)
// record for the son's box distance and re-checks it, which is exactly the
// check a stack pop makes.  Same visits, same candidates, same order, ties
// included.  Used for the rare queries the fast pass flags (k_knn_replay).
// The record fetch is a parameter: one lane's loads (knn_exact) or a wave's
// subtree cache (knn_exact_wave); the traversal is the same code.
struct NodeRec {
    float4 a, b, c, d;
};
template <class Fetch>
__device__ __forceinline__ void knn_exact_t(Fetch&& fetch, int has_map, float qx, float qy, float qz, Cands& c) {
    KHeap h;
#pragma unroll
    for (int j = 0; j < kNN; j++) { h.d[j] = INFINITY; h.x[j] = 0.0f; h.node[j] = 0u; }
    h.size = 0;
    uint32_t cur = 0, trail = 0;
    bool down = true;
    while (has_map) {
        const NodeRec r = fetch(cur);
        const float4 a = r.a, b = r.b, cc = r.c, dd = r.d;
        const uint32_t meta = __float_as_uint(a.w);
        const bool hl = (meta & kLeftBit) != 0u, hr = (meta & kRightBit) != 0u;
        const float dl = hl ? box_dist(qx, qy, qz, b.x, b.y, b.z, b.w, cc.x, cc.y) : INFINITY;
        const float dr = hr ? box_dist(qx, qy, qz, cc.z, cc.w, dd.x, dd.y, dd.z, dd.w) : INFINITY;
        const bool lf = dl <= dr;
        const uint32_t nnear = 2u * cur + (lf ? 1u : 2u), nfar = 2u * cur + (lf ? 2u : 1u);
        const float dnear = lf ? dl : dr, dfar = lf ? dr : dl;
        const bool enear = lf ? hl : hr, efar = lf ? hr : hl;
        const int lev = level_of(cur);
        if (down) {
            const float dx = qx - a.x, dy = qy - a.y, dz = qz - a.z;
            const float dist = (dx * dx + dy * dy) + dz * dz;  // calc_dist (:1291-1295)
            if (dist <= INFINITY && (h.size < kNN || dist < h.d[0])) {
                if (h.size >= kNN) kh_pop(h);  // q.pop(); q.push(current_point)  (:861-863)
                kh_push(h, dist, a.x, cur);
            }
            const bool full = h.size >= kNN;
            const float top = h.d[0];
            const bool far_ok = efar && (!full || dfar < top);
            if (enear && (!full || dnear < top)) {
                if (far_ok) trail |= (1u << lev);
                cur = nnear;
                continue;
            }
            if (far_ok) { cur = nfar; continue; }
        } else {
            const bool full = h.size >= kNN;
            const float top = h.d[0];
            trail &= ~(1u << lev);
            if (efar && (!full || dfar < top)) { cur = nfar; down = true; continue; }
        }
        const uint32_t pend = trail & ((lev > 0) ? ((1u << lev) - 1u) : 0u);
        if (pend == 0u) break;
        const int al = 31 - __clz(pend);
        cur = ((cur + 1u) >> (lev - al)) - 1u;
        down = false;
    }
    kh_extract(h, c);
}
__device__ __forceinline__ void knn_exact(const MapNode* __restrict__ nodes, int has_map, float qx, float qy, float qz,
                                          Cands& c) {
    knn_exact_t(
        [&](uint32_t hn) {
            const float4* rp = rec_ptr(nodes, hn);
            return NodeRec{rp[0], rp[1], rp[2], rp[3]};
        },
        has_map, qx, qy, qz, c);
}

// knn_exact for one query by a whole wave (every lane active, the query
// wave-uniform): the traversal is a chain of dependent record loads (~50 per
// query on a 1M-point tree), so the wave loads the 63 records of the K = 6
// levels below the current node in one round trip (heap order: the
// descendants of h at depth d are (h + 1) 2^d - 1 + 0 .. 2^d - 1) into its 4 KB
// of LDS, walks them from there, and reloads only when the walk leaves that
// subtree.  Every lane runs the same walk on the same LDS words, so every lane
// ends with the same candidates as knn_exact.
constexpr int kReplayLevels = 6;
__device__ __forceinline__ void knn_exact_wave(const MapNode* __restrict__ nodes, int64_t n_nodes, int has_map, float qx,
                                               float qy, float qz, float4* __restrict__ cache, Cands& c) {
    const unsigned lane = threadIdx.x & 63u;
    uint32_t root = 0xFFFFFFFFu;
    int root_lev = 0;
    auto reload = [&](uint32_t hn) {
        root = hn;
        root_lev = level_of(hn);
        if (lane < (1u << kReplayLevels) - 1u) {
            const int lv = 31 - __clz(lane + 1u);
            const uint64_t node = ((uint64_t)(hn + 1u) << lv) - 1u + (lane - ((1u << lv) - 1u));
            if (node < (uint64_t)n_nodes) {
                const float4* rp = rec_ptr(nodes, (uint32_t)node);
#pragma unroll
                for (int k = 0; k < 4; k++) cache[lane * 4u + k] = rp[k];
            }
        }
        WAVE_SYNC();
    };
    knn_exact_t(
        [&](uint32_t hn) {
            const int d = level_of(hn) - root_lev;
            if (root == 0xFFFFFFFFu || d < 0 || d >= kReplayLevels || ((hn + 1u) >> d) != root + 1u) reload(hn);
            const int dd = level_of(hn) - root_lev;
            const uint32_t loc = (1u << dd) - 1u + ((hn + 1u) - ((root + 1u) << dd));
            const float4* rp = cache + loc * 4u;
            return NodeRec{rp[0], rp[1], rp[2], rp[3]};
        },
        has_map, qx, qy, qz, c);
    WAVE_SYNC();  // every lane has read the cache before the next query reloads it
}

// ------------------------------------------------------- fast candidates --
// The hot loop keeps the 5 best candidates as a list sorted by distance
// (compare-and-swap insertion) and searches the same tree exactly, so it
// returns the exact 5 nearest points.  The reference's MANUAL_HEAP ordered by
// PointType_CMP (distance, x within |Δd| < 1e-10) gives the same points in the
// same order unless two inserted candidates are fuzz-close (CMP then looks at
// x, and stops being transitive across chains) or a point ties exactly with
// the 5th (the reference resolves that by visiting order).  Both are flagged
// (fuzz-close pairs need |Δd| <= 1e-10, i.e. equal or near-duplicate
// distances) and recomputed by the exact heap (k_knn_replay); boxes at exactly
// the 5th distance are searched rather than pruned, so no tied point is missed.
constexpr float kFuzz = 0x1.b7cdfcp-34f;  // largest float < 1e-10: |d| < 1e-10 <=> |d| <= kFuzz

struct SList {
    float d[kNN];
    uint32_t node[kNN];
    int n;
    bool fuzz;  // two inserted candidates were fuzz-close: exact replay
};

__device__ __forceinline__ void sl_init(SList& s) {
#pragma unroll
    for (int j = 0; j < kNN; j++) {
        s.d[j] = INFINITY;
        s.node[j] = 0u;
    }
    s.n = 0;
    s.fuzz = false;
}

__device__ __forceinline__ void sl_insert(SList& s, float d, uint32_t node) {
    bool close = false;
#pragma unroll
    for (int j = 0; j < kNN; j++) close |= fabsf(d - s.d[j]) <= kFuzz;  // empty slots are +inf
    s.fuzz |= close;
    s.d[kNN - 1] = d;
    s.node[kNN - 1] = node;
#pragma unroll
    for (int j = kNN - 1; j > 0; j--) {
        const bool sw = s.d[j] < s.d[j - 1];
        const float td = s.d[j];
        const uint32_t tn = s.node[j];
        s.d[j] = sw ? s.d[j - 1] : td;
        s.node[j] = sw ? s.node[j - 1] : tn;
        s.d[j - 1] = sw ? td : s.d[j - 1];
        s.node[j - 1] = sw ? tn : s.node[j - 1];
    }
    s.n = s.n < kNN ? s.n + 1 : kNN;
}

// One neighbour record per point (Nearest_Points[i] + pointSearchSqDis);
// flag = 1 if the query goes to the exact replay; node[] = heap ids (seeds of the next search).
__device__ __forceinline__ void write_nnrec(NNRec* __restrict__ out, const MapNode* __restrict__ nodes, int cnt,
                                            const float (&d)[kNN], const uint32_t (&node)[kNN], int flag) {
    float4* o4 = reinterpret_cast<float4*>(out);
    int32_t idx[kNN];
#pragma unroll
    for (int k = 0; k < kNN; k++) {
        float4 v = make_float4(0.f, 0.f, 0.f, INFINITY);
        idx[k] = -1;
        if (k < cnt) {
            const float4 a = rec_ptr(nodes, node[k])[0];
            v = make_float4(a.x, a.y, a.z, d[k]);
            idx[k] = (int32_t)(__float_as_uint(a.w) & kIdxMask);
        }
        o4[k] = v;
    }
    int4* oi = reinterpret_cast<int4*>(out) + 5;
    oi[0] = make_int4(idx[0], idx[1], idx[2], idx[3]);
    oi[1] = make_int4(idx[4], cnt, flag, (int)node[0]);
    oi[2] = make_int4((int)node[1], (int)node[2], (int)node[3], (int)node[4]);
}

// The state an evaluation transforms its points with, wherever it is held
// (k_iekf_eval: in LDS, solved by the launch's own blocks).
struct PoseRef {
    const double* rot;
    const double* pos;
};
__device__ __forceinline__ void query_point(const KnnParams& P, const PoseRef& S, const float4 b, float& qx, float& qy,
                                            float& qz) {
    if (P.identity) {
        qx = b.x; qy = b.y; qz = b.z;
    } else {
        world_point(S.rot, S.pos, P.R_LI, P.t_LI, b.x, b.y, b.z, qx, qy, qz);
    }
}
__device__ __forceinline__ void query_point(const KnnParams& P, const IekfSlot* slot, const float4 b, float& qx,
                                            float& qy, float& qz) {
    if (P.identity) {
        qx = b.x; qy = b.y; qz = b.z;
    } else if (slot->model == kModelIkfom) {
        ik_world_point(slot->ik.x, b.x, b.y, b.z, qx, qy, qz);  // origin_laserMapping.cpp:937
    } else {
        world_point(slot->state.rot, slot->state.pos, P.R_LI, P.t_LI, b.x, b.y, b.z, qx, qy, qz);
    }
}

__device__ __forceinline__ void count_visits(const KnnParams& P, IekfSlot* slot, unsigned visits,
                                             unsigned points = 0u) {
    unsigned long long wv = visits, wp = points;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        wv += __shfl_xor(wv, off, 64);
        wp += __shfl_xor(wp, off, 64);
    }
    if ((threadIdx.x & 63) == 0 && (wv || wp)) {
        int e = P.force >= 0 ? 0 : slot->ctrl.n_evals;
        e = e < LIVO_MAX_EVALS ? e : LIVO_MAX_EVALS - 1;
        if (wv) atomicAdd(&slot->visits[e], wv);
        if (wp) atomicAdd(&slot->scanned[e], wp);
    }
}

__device__ __forceinline__ void flag_for_replay(const KnnParams& P, unsigned job, int i) {
    const unsigned slot_i = atomicAdd(P.replay_count, 1u);
    P.replay_list[slot_i] = ((unsigned long long)job << 32) | (unsigned)i;
}

// ------------------------------------------------ reference-order k-NN ----
// livo_knn / livo_h_share: one query per thread, the near-first DFS of
// KD_TREE::Search on the ikd-Tree records, so the nodes it visits (counted)
// are exactly the reference's V_ref.  Sorted-list candidates.  The pending
// far sons lie on the current root-to-node path, at most one per level, so
// the "stack" is a trail bit mask plus one box distance per level in LDS
// ([level][lane], conflict-free, 4 B per entry): popping takes the deepest
// pending level and rebuilds the son's heap id from the current node id.
__global__ __launch_bounds__(kKnnBlock, 8) void k_knn_pass(KnnParams P) {  // 8 waves/SIMD: <= 64 VGPRs
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned bjob, bx;
    xcd_block(P.nb, bjob, bx);
    const HsJob job = P.jobs[bjob];
    IekfSlot* slot = job.slot;
    if (P.force >= 0) {
        if (!P.force) return;
    } else if (slot->ctrl.stop) {
        return;
    }
    const int i = (int)bx * kKnnBlock + threadIdx.x;
    if (i >= job.n) return;
    float* dstack = reinterpret_cast<float*>(smem) + threadIdx.x;
    const MapNode* __restrict__ nodes = P.nodes;
    float qx, qy, qz;
    query_point(P, slot, reinterpret_cast<const float4*>(job.pts)[i], qx, qy, qz);
    SList s;
    sl_init(s);
    unsigned flag = 0;  // reason bits: 1 CMP fuzz / equivalence, 2 point tied with the 5th, 8 overrun
    unsigned visits = 0;
    const unsigned max_visits = (2u << P.depth) + 64u;  // exit every wave reaches (see k_knn_leaf)
    uint32_t node = 0, cur = 0;
    uint32_t trail = 0;  // bit L: a far son at level L is pending (its box distance in dstack[L-1])
    bool has = P.has_map != 0;
    while (true) {
        if (visits > max_visits) {
            flag |= 8u;
            break;
        }
        if (!has) {
            if (trail == 0u) break;
            const int L = 31 - __clz(trail);
            trail &= ~(1u << L);
            const float de = dstack[(L - 1) * kKnnBlock];
            // boxes at exactly the current 5th distance are searched too (a point
            // tied with the 5th may hide there): the answer is exact either way
            if (!(s.n < kNN || de <= s.d[kNN - 1])) continue;
            // the pending son is the sibling of cur's ancestor at level L
            const uint32_t a = ((cur + 1u) >> (level_of(cur) - L)) - 1u;
            node = ((a - 1u) ^ 1u) + 1u;
        }
        cur = node;
        const float4* rp = rec_ptr(nodes, node);
        const float4 a = rp[0];
        const float4 b = rp[1];
        const float4 cc = rp[2];
        const float4 dd = rp[3];
        visits++;
        const uint32_t meta = __float_as_uint(a.w);
        {
            const float dx = qx - a.x, dy = qy - a.y, dz = qz - a.z;
            const float dist = (dx * dx + dy * dy) + dz * dz;  // calc_dist (:1291-1295)
            const bool full = s.n >= kNN;
            const float top = s.d[kNN - 1];
            if (!full || dist < top) sl_insert(s, dist, node);
            flag |= (full && dist == top) ? 2u : 0u;
        }
        const bool hl = (meta & kLeftBit) != 0u;
        const bool hr = (meta & kRightBit) != 0u;
        const float dl = hl ? box_dist(qx, qy, qz, b.x, b.y, b.z, b.w, cc.x, cc.y) : INFINITY;
        const float dr = hr ? box_dist(qx, qy, qz, cc.z, cc.w, dd.x, dd.y, dd.z, dd.w) : INFINITY;
        const bool left_first = dl <= dr;
        const float dnear = left_first ? dl : dr;
        const float dfar = left_first ? dr : dl;
        const bool enear = left_first ? hl : hr;
        const bool efar = left_first ? hr : hl;
        const bool full = s.n >= kNN;
        const float top = s.d[kNN - 1];
        if (efar && (!full || dfar <= top)) {
            const int Lc = level_of(node) + 1;  // level of the sons
            dstack[(Lc - 1) * kKnnBlock] = dfar;
            trail |= 1u << Lc;
        }
        has = enear && (!full || dnear <= top);
        node = 2u * node + (left_first ? 1u : 2u);
    }
    flag |= s.fuzz ? 1u : 0u;
#ifdef LIVO_LAB_NOFLAGS
    flag = 0;
#endif
    float od[kNN];
    uint32_t on[kNN];
#pragma unroll
    for (int k = 0; k < kNN; k++) { od[k] = s.d[k]; on[k] = s.node[k]; }
    write_nnrec(job.nn + i, nodes, s.n, od, on, (int)flag);
    if (flag) flag_for_replay(P, bjob, i);
    count_visits(P, slot, visits);
}

// ------------------------------------------------------- leaf-map k-NN ----
// The batched IEKF search (k_knn_leaf<SEEDED>): one query per thread on the
// leaf map (livo_internal.h), the same trail/LDS distance stack over the
// internal levels, and a leaf scan with independent loads at the bottom.
//
// Equivalence with the reference (ikd_Tree.cpp:843-986, MANUAL_HEAP
// :1345-1411, PointType_CMP ikd_Tree.h:50-61).  Let S5 be the 5 nearest map
// points by squared distance, d5 the 5th distance and d6 the next one.  If
//   (C1) d6 - d5 > 1e-10 (float subtraction, as PointType_CMP computes it), and
//   (C2) no two members of S5 are within 1e-10 of each other,
// then every S5 member compares below every other point under PointType_CMP,
// so no heap operation can place an S5 member above a non-member, a full heap
// always pops a non-member, every S5 member passes the push test when
// visited, and Nearest_Search returns exactly S5 in ascending distance --
// whatever the visiting order.  The search below finds S5 exactly, and also
// every point within 1e-10 of d5: a box is skipped only if its distance
// exceeds min(5th candidate, seed bound B) by more than 1e-10 (both are
// >= d5 and float subtraction is monotone; box distances never exceed the
// distance of a point inside, as in calc_box_dist).  It tracks e6, the
// smallest distance rejected or evicted from the 5 candidates, and flags the
// query (exact replay on the ikd-Tree) if C1 or C2 fails.
// One query of the leaf-map search: its world point, seed bound, sorted
// 5-candidate list and e6 (smallest distance rejected or evicted).
// A candidate's position in the cell runs (vrun_search) rather than a grid /
// leaf-map slot: lq_finish reads it from P.vpts.
constexpr uint32_t kRunPos = 0x80000000u;
struct LeafQuery {
    float qx, qy, qz, B, e6;
    float d[kNN];
    uint32_t nd[kNN];
};

template <bool SEEDED, class Src>
__device__ __forceinline__ void lq_init(LeafQuery& q, const KnnParams& P, const Src& slot, const HsJob& job, int i,
                                        bool valid) {
#pragma unroll
    for (int k = 0; k < kNN; k++) { q.d[k] = INFINITY; q.nd[k] = 0u; }
    q.e6 = INFINITY;
    q.B = INFINITY;
    q.qx = q.qy = q.qz = 0.0f;
    if (!valid) {
        q.B = -INFINITY;  // threshold -inf: never asks for a box
        return;
    }
    query_point(P, slot, reinterpret_cast<const float4*>(job.pts)[i], q.qx, q.qy, q.qz);
    if (SEEDED) {
        // the point's 5 previous neighbours, re-measured: 5 distinct map points
        // at distance <= B, so B >= d5
        const NNRec* sr = job.nn + i;
        if (sr->cnt == kNN) {
            float bmax = 0.0f;
#pragma unroll
            for (int k = 0; k < kNN; k++) {
                const float4 a = reinterpret_cast<const float4*>(sr->p)[k];
                const float dx = q.qx - a.x, dy = q.qy - a.y, dz = q.qz - a.z;
                bmax = fmaxf(bmax, (dx * dx + dy * dy) + dz * dz);
            }
            q.B = bmax;
        }
    }
}

__device__ __forceinline__ float lq_thr(const LeafQuery& q) { return fminf(q.d[kNN - 1], q.B); }
// an empty list (the query point kept)
__device__ __forceinline__ void lq_reset(LeafQuery& q) {
#pragma unroll
    for (int k = 0; k < kNN; k++) { q.d[k] = INFINITY; q.nd[k] = 0u; }
    q.e6 = INFINITY;
    q.B = INFINITY;
}

// One scanned point: inserted into the sorted list if below the 5th (the
// evicted 5th, +inf while the list is not full, becomes a candidate for e6),
// else a candidate for e6 itself.
__device__ __forceinline__ void lq_offer(LeafQuery& q, float dist, uint32_t slot) {
    if (dist < q.d[kNN - 1]) {
        q.e6 = fminf(q.e6, q.d[kNN - 1]);
        q.d[kNN - 1] = dist;
        q.nd[kNN - 1] = slot;
#pragma unroll
        for (int k = kNN - 1; k > 0; k--) {
            const bool sw = q.d[k] < q.d[k - 1];
            const float td = q.d[k];
            const uint32_t tn = q.nd[k];
            q.d[k] = sw ? q.d[k - 1] : td;
            q.nd[k] = sw ? q.nd[k - 1] : tn;
            q.d[k - 1] = sw ? td : q.d[k - 1];
            q.nd[k - 1] = sw ? tn : q.nd[k - 1];
        }
    } else {
        q.e6 = fminf(q.e6, dist);
    }
}
__device__ __forceinline__ void lq_point(LeafQuery& q, const float4 v, uint32_t slot) {
    const float dx = q.qx - v.x, dy = q.qy - v.y, dz = q.qz - v.z;
    lq_offer(q, (dx * dx + dy * dy) + dz * dz, slot);  // calc_dist (:1291-1295)
}

// C1/C2 check, neighbour record, replay flag.
//
// Exact ties inside the list are resolved here rather than replayed.  The
// reference inserts a point only when dist < top (ikd_Tree.cpp:860), so every
// point nearer than the final 5th distance D is in its heap whatever the
// visiting order; only a point AT D competing for the last place (C1:
// e6 - d5 <= fuzz) depends on the order.  Its output order is the heap's pop
// order under PointType_CMP (ikd_Tree.h:57-60): equal distances compare by x.
// When every adjacent gap of the list is either 0 or > 1e-10 that comparison
// is a strict total order on the 5 points, so sorting by (dist, x) gives the
// reference's order.  A gap in (0, 1e-10] (CMP not transitive) or an exact tie
// with equal x (neither point "less") still goes to the exact replay.
// RUNS: candidates may be cell-run positions (kRunPos, vrun_search) besides slots of lpts
template <bool RUNS>
__device__ __forceinline__ float4 cand_point(const float4* __restrict__ lpts, const float4* __restrict__ vpts,
                                             uint32_t nd) {
    if constexpr (RUNS) return (nd & kRunPos) ? vpts[nd & ~kRunPos] : lpts[nd];
    return lpts[nd];
}
#ifdef LIVO_EVAL_PROF
// why queries were flagged for the exact replay: [uncertified, C1 (e6 - d5 <= 1e-10),
// C2 gap in (0, 1e-10], C2 exact tie with equal x, C1 with e6 == d5 exactly]
__device__ unsigned long long g_amb_reason[8];
#endif
template <bool RUNS = false>
// stage: the wave's LDS record buffer (64 x 8 float4, part k of lane l's record at
// l * 8 + ((k + l) & 7): 8 distinct 16-B slots per row, so the lanes' writes spread
// over the banks); nullptr: the record goes straight to job.nn.
__device__ __forceinline__ bool lq_finish(LeafQuery& q, const KnnParams& P, const HsJob& job, unsigned bjob,
                                          int i, const float4* __restrict__ lpts, bool overrun, bool enqueue = true,
                                          const float4* __restrict__ vpts = nullptr, float4* nbr = nullptr,
                                          float4* stage = nullptr) {
    const int cnt = (int)min<int64_t>(P.lM, (int64_t)kNN);
    float4 a[kNN];
#pragma unroll
    for (int k = 0; k < kNN; k++) a[k] = k < cnt ? cand_point<RUNS>(lpts, vpts, q.nd[k]) : make_float4(0.f, 0.f, 0.f, 0.f);
    bool amb = overrun || q.e6 - q.d[kNN - 1] <= kFuzz;  // C1 (false while e6 = +inf)
    bool tie = false;
#pragma unroll
    for (int k = 0; k + 1 < kNN; k++) {
        if (k + 1 < cnt && q.d[k + 1] - q.d[k] <= kFuzz) {  // C2
            if (q.d[k + 1] == q.d[k] && a[k + 1].x != a[k].x) tie = true;
            else amb = true;
        }
    }
#ifdef LIVO_EVAL_PROF
    if (amb || tie) {
        bool gap = false, eqx = false;
        for (int k = 0; k + 1 < kNN; k++)
            if (k + 1 < cnt && q.d[k + 1] - q.d[k] <= kFuzz) {
                if (q.d[k + 1] == q.d[k] && a[k + 1].x == a[k].x) eqx = true;
                else if (q.d[k + 1] != q.d[k]) gap = true;
            }
        if (overrun) atomicAdd(&g_amb_reason[0], 1ull);
        else if (q.e6 - q.d[kNN - 1] <= kFuzz) atomicAdd(&g_amb_reason[q.e6 == q.d[kNN - 1] ? 4 : 1], 1ull);
        if (gap) atomicAdd(&g_amb_reason[2], 1ull);
        if (eqx) atomicAdd(&g_amb_reason[3], 1ull);
    }
#endif
    if (tie && !amb) {
        // (dist, x) order; the list is already sorted by dist
        float ax[kNN];
#pragma unroll
        for (int k = 0; k < kNN; k++) ax[k] = a[k].x;
#pragma unroll
        for (int pass = 0; pass + 1 < kNN; pass++) {
#pragma unroll
            for (int k = 0; k + 1 < kNN; k++) {
                const bool sw = k + 1 < cnt && q.d[k + 1] == q.d[k] && ax[k + 1] < ax[k];
                const float tx = ax[k];
                const uint32_t tn = q.nd[k];
                ax[k] = sw ? ax[k + 1] : tx;
                q.nd[k] = sw ? q.nd[k + 1] : tn;
                ax[k + 1] = sw ? tx : ax[k + 1];
                q.nd[k + 1] = sw ? tn : q.nd[k + 1];
            }
        }
#pragma unroll
        for (int k = 0; k < kNN; k++)
            if (k < cnt) a[k] = cand_point<RUNS>(lpts, vpts, q.nd[k]);
    }
    // neighbour record: points, distances, original indices; node[] = leaf-map slots
    float4* o4 = reinterpret_cast<float4*>(job.nn + i);
    const int sl = threadIdx.x & 63;
    auto put = [&](int k, float4 v) {
        if (stage) stage[sl * 8 + ((k + sl) & 7)] = v;
        else o4[k] = v;
    };
    int32_t idx[kNN];
#pragma unroll
    for (int k = 0; k < kNN; k++) {
        float4 v = make_float4(0.f, 0.f, 0.f, INFINITY);
        idx[k] = -1;
        if (k < cnt) {
            v = make_float4(a[k].x, a[k].y, a[k].z, q.d[k]);
            idx[k] = (int32_t)__float_as_uint(a[k].w);
        }
        put(k, v);
        if (nbr) nbr[k] = v;  // (x, y, z, sqdist) as the record holds them
    }
    const int flag = amb ? 4 : (tie ? 16 : 0);
    auto i4 = [](int x, int y, int z, int w) {
        return make_float4(__int_as_float(x), __int_as_float(y), __int_as_float(z), __int_as_float(w));
    };
    put(5, i4(idx[0], idx[1], idx[2], idx[3]));
    put(6, i4(idx[4], cnt, flag, (int)q.nd[0]));
    put(7, i4((int)q.nd[1], (int)q.nd[2], (int)q.nd[3], (int)q.nd[4]));
    if (amb && enqueue) flag_for_replay(P, bjob, i);
    return amb;
}

// Q queries per thread walk the tree together (a box is entered if any of them
// may need it; a pending far son keeps the smallest of their box distances and
// is re-checked against the largest threshold, which may visit a box no query
// needs, never skip one).  Only Q = 1 is launched: measured on MI355X, Q = 2
// (Morton-adjacent pairs sharing each load) was 1.4x slower at 8 scans.
template <bool SEEDED, int Q>
__global__ __launch_bounds__(kKnnBlock, Q == 1 ? 8 : 6) void k_knn_leaf(KnnParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned bjob, bx;
    xcd_block(P.nb, bjob, bx);
    const HsJob job = P.jobs[bjob];
    IekfSlot* slot = job.slot;
    if (P.force >= 0) {
        if (!P.force) return;
    } else {
        if (slot->ctrl.stop) return;
        if (SEEDED && !slot->ctrl.search_en) return;
    }
    const int i0 = ((int)bx * kKnnBlock + threadIdx.x) * Q;
    if (i0 >= job.n) return;
    float* dstack = reinterpret_cast<float*>(smem) + threadIdx.x;
    const float4* __restrict__ lnodes = reinterpret_cast<const float4*>(P.lnodes);
    const float4* __restrict__ lpts = reinterpret_cast<const float4*>(P.lpts);
    LeafQuery q[Q];
#pragma unroll
    for (int u = 0; u < Q; u++) lq_init<SEEDED>(q[u], P, slot, job, i0 + u, i0 + u < job.n);
    const int D = P.ldepth;
    const uint32_t first_leaf = (1u << D) - 1u;
    const int64_t M = P.lM;
    unsigned visits = 0;
    // a correct search visits each node at most once: past that, stop and let
    // the exact replay answer (every wave reaches an exit)
    const unsigned max_visits = (2u << D) + 64u;
    bool overrun = false;
    uint32_t node = 0, cur = 0, trail = 0;
    bool has = M > 0;
    while (true) {
        if (visits > max_visits) {
            overrun = true;
            break;
        }
        if (!has) {
            if (trail == 0u) break;
            const int L = 31 - __clz(trail);
            trail &= ~(1u << L);
            const float de = dstack[(L - 1) * kKnnBlock];
            float thr = lq_thr(q[0]);
#pragma unroll
            for (int u = 1; u < Q; u++) thr = fmaxf(thr, lq_thr(q[u]));
            if (de - thr > kFuzz) continue;
            const uint32_t a = ((cur + 1u) >> (level_of(cur) - L)) - 1u;
            node = ((a - 1u) ^ 1u) + 1u;
        }
        cur = node;
        visits++;
        if (node >= first_leaf) {
            // leaf: its points, 4 independent loads at a time
            const int64_t j = node - first_leaf;
            const int lo = (int)((j * M) >> D), hi = (int)(((j + 1) * M) >> D);
            for (int k0 = lo; k0 < hi; k0 += 4) {
                float4 v[4];
#pragma unroll
                for (int w = 0; w < 4; w++) v[w] = lpts[k0 + w];  // padded by 3 points
#pragma unroll
                for (int w = 0; w < 4; w++)
                    if (k0 + w < hi) {
#pragma unroll
                        for (int u = 0; u < Q; u++) lq_point(q[u], v[w], (uint32_t)(k0 + w));
                    }
            }
            has = false;
            continue;
        }
        const float4* rp = lnodes + 4 * (size_t)node;
        const float4 b = rp[0];
        const float4 cc = rp[1];
        const float4 dd = rp[2];
        bool want_l = false, want_r = false;
        float ml = INFINITY, mr = INFINITY;
#pragma unroll
        for (int u = 0; u < Q; u++) {
            const float dl = box_dist(q[u].qx, q[u].qy, q[u].qz, b.x, b.y, b.z, b.w, cc.x, cc.y);
            const float dr = box_dist(q[u].qx, q[u].qy, q[u].qz, cc.z, cc.w, dd.x, dd.y, dd.z, dd.w);
            const float thr = lq_thr(q[u]);
            want_l |= dl - thr <= kFuzz;
            want_r |= dr - thr <= kFuzz;
            ml = fminf(ml, dl);
            mr = fminf(mr, dr);
        }
        const bool left_first = ml <= mr;
        const bool want_near = left_first ? want_l : want_r, want_far = left_first ? want_r : want_l;
        // the far son waits on the stack only while the near son is searched
        // first (a pop must find cur at or below the pending level); if only
        // the far son is wanted, go there directly
        if (want_near && want_far) {
            const int Lc = level_of(node) + 1;
            dstack[(Lc - 1) * kKnnBlock] = left_first ? mr : ml;
            trail |= 1u << Lc;
        }
        has = want_near || want_far;
        node = 2u * node + ((left_first == want_near) ? 1u : 2u);
    }
#pragma unroll
    for (int u = 0; u < Q; u++)
        if (i0 + u < job.n) lq_finish(q[u], P, job, bjob, i0 + u, lpts, overrun);
    count_visits(P, slot, visits);
}

// ------------------------------------------------------- cell-grid k-NN ----
// The cell-grid search (LIVO_KNN_KIND=grid).  Stage 0 scans the 2x2x2 block of
// cells around the query (its own cell first, then the neighbours on the side
// of the cell the query lies in).  Stage 1 scans, within the 3x3x3 cube of
// cells, those the current bound min(5th candidate, seed bound) still reaches
// (the whole cube while fewer than 5 points are known), so the bound shrinks
// before stage 2 scans every remaining cell overlapping the cube of half-edge
// sqrt(bound) around the query: every point that can still enter the list lies
// there, so the list is exact.  A query whose list is not full by then, or whose
// stage-2 box exceeds kGridMaxCells cells, goes to the exact replay.  Cells are found by hashing (a 16-B slot holds the cell's
// point range: one load, then the points), cells farther than
// min(5th candidate, seed bound) + 1e-10 are skipped.  Same candidate list, e6
// and C1/C2 flags as k_knn_leaf, so the same equivalence argument holds.
__device__ __forceinline__ unsigned long long grid_key_d(int cx, int cy, int cz) {
    return (unsigned long long)(cx + kGridBias) | ((unsigned long long)(cy + kGridBias) << 21) |
           ((unsigned long long)(cz + kGridBias) << 42);
}

#ifndef LIVO_GRID_WAVES
#define LIVO_GRID_WAVES 5  // waves per SIMD (VGPR budget 96: no spills)
#endif

// --- LDS tiles ---------------------------------------------------------------
// The scan is Morton-ordered, so the queries of a block lie a few cells
// apart.  The block takes the box of cells within one cell of any of its
// queries (at most CELLS cells), resolves every cell of the box through the
// hash at once (threads probe in parallel), and copies the box's points into
// LDS in cell order in one pass of independent loads.  Each thread then runs
// exactly the stages of grid_search -- same cells, same order, same pruning,
// so the same list, e6 and flags -- reading its cells from LDS instead of
// chasing hash probe -> cell run -> points through L2.  Stage-2 or sparse-map
// cells outside the box, and blocks whose box or points do not fit, take the
// global path.
template <int CELLS, int PTS>
struct TileLds {
    static constexpr int kChunk = 8;  // points per chunked read of a cell (grid_search)
    float4 pts[PTS + kChunk];  // the box's points (x, y, z, gpts index bits); padded for the chunked reads
    uint32_t off[CELLS + 1];  // LDS start of each cell's run
    uint32_t start[CELLS];    // its start in gpts
    uint32_t wred[16];        // per-wave partials of the block scans
    int box[6 * 16];          // per-wave cell bounds
};
struct TileView {
    bool on = false;
    int lo0 = 0, lo1 = 0, lo2 = 0, hi0 = -1, hi1 = -1, hi2 = -1, d0 = 0, d1 = 0;
    const float4* pts = nullptr;
    const uint32_t* off = nullptr;
};
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
// Block-wide inclusive scan (sum or max) of one value per thread; NT threads.
template <int NT, bool MAX>
__device__ __forceinline__ uint32_t block_incl_scan(uint32_t v, uint32_t* wred, uint32_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(v, o, 64);
        if (lane >= o) v = MAX ? (y > v ? y : v) : v + y;
    }
    if constexpr (NT == 64) {
        total = __shfl(v, 63, 64);
        return v;
    } else {
        if (lane == 63) wred[wave] = v;
        __syncthreads();
        uint32_t before = 0u, all = 0u;
#pragma unroll
        for (int w = 0; w < NT / 64; w++) {
            const uint32_t t = wred[w];
            if (w < wave) before = MAX ? (t > before ? t : before) : before + t;
            all = MAX ? (t > all ? t : all) : all + t;
        }
        __syncthreads();
        total = all;
        return MAX ? (before > v ? before : v) : before + v;
    }
}

// Builds the block's tile for the cells (c0, c1, c2) of its valid threads.
// Every thread of the block calls it (NT threads).
template <int NT, int CELLS, int PTS>
__device__ __forceinline__ TileView build_tile(TileLds<CELLS, PTS>& L, const KnnParams& P, bool valid, int c0, int c1,
                                               int c2, unsigned& visits, unsigned& npts) {
    static_assert(CELLS % NT == 0 && PTS % NT == 0, "tile sizes");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    TileView tv;
    int b[6] = {wave_min_i(valid ? c0 : INT_MAX), wave_min_i(valid ? c1 : INT_MAX), wave_min_i(valid ? c2 : INT_MAX),
                wave_max_i(valid ? c0 : INT_MIN), wave_max_i(valid ? c1 : INT_MIN), wave_max_i(valid ? c2 : INT_MIN)};
    if constexpr (NT > 64) {
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < 6; k++) L.box[6 * wave + k] = b[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 6; k++) {
            int v = L.box[k];
#pragma unroll
            for (int w = 1; w < NT / 64; w++) v = k < 3 ? min(v, L.box[6 * w + k]) : max(v, L.box[6 * w + k]);
            b[k] = v;
        }
        __syncthreads();
    }
    if (b[0] > b[3]) return tv;  // no valid thread
    tv.lo0 = b[0] - 1; tv.lo1 = b[1] - 1; tv.lo2 = b[2] - 1;
    tv.hi0 = b[3] + 1; tv.hi1 = b[4] + 1; tv.hi2 = b[5] + 1;
    tv.d0 = tv.hi0 - tv.lo0 + 1;
    tv.d1 = tv.hi1 - tv.lo1 + 1;
    const long long vol = (long long)tv.d0 * tv.d1 * (long long)(tv.hi2 - tv.lo2 + 1);
    if (!(P.lM > 0 && vol <= CELLS)) return tv;
    const int V = (int)vol;
    const GridSlot* __restrict__ slots = P.gslots;
    const float4* __restrict__ gpts = reinterpret_cast<const float4*>(P.gpts);
    const uint64_t mask = (1ull << P.glog2) - 1ull;
    constexpr int kPer = CELLS / NT;
    // 1. directory: every cell of the box through the hash, first probes in flight together
    unsigned long long key[kPer];
    uint64_t sl[kPer];
    GridSlot gs[kPer];
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const int t = tid + NT * u;
        if (t < V) {
            key[u] = grid_key_d(tv.lo0 + t % tv.d0, tv.lo1 + (t / tv.d0) % tv.d1, tv.lo2 + t / (tv.d0 * tv.d1));
            sl[u] = (uint64_t)((key[u] * 0x9E3779B97F4A7C15ull) >> (64 - P.glog2));
            gs[u] = slots[sl[u]];
            visits++;
        }
    }
    uint32_t cnt_u[kPer];
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const int t = tid + NT * u;
        cnt_u[u] = 0u;
        if (t < V) {
            while (gs[u].key != key[u] && gs[u].key != kGridEmpty) {  // linear probing
                sl[u] = (sl[u] + 1) & mask;
                gs[u] = slots[sl[u]];
                visits++;
            }
            const bool hit = gs[u].key == key[u];
            L.start[t] = hit ? gs[u].start : 0u;
            cnt_u[u] = hit ? gs[u].count : 0u;
            L.off[t] = cnt_u[u];
        }
    }
    __syncthreads();
    // 2. exclusive scan of the counts (thread: cells kPer*tid .. kPer*tid + kPer - 1)
    uint32_t cc[kPer], loc = 0;
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const int t = kPer * tid + u;
        cc[u] = t < V ? L.off[t] : 0u;
        loc += cc[u];
    }
    uint32_t total;
    const uint32_t incl = block_incl_scan<NT, false>(loc, L.wred, total);
    __syncthreads();  // every count read before the offsets overwrite them
    uint32_t run = incl - loc;
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const int t = kPer * tid + u;
        if (t < V) L.off[t] = run;
        run += cc[u];
    }
    if (tid == 0) L.off[V] = total;
    if (total > (uint32_t)PTS) return tv;  // (block-uniform)
    const int npt = (int)total;
    for (int p = tid; p < npt; p += NT) L.pts[p].w = __uint_as_float(0u);
    __syncthreads();
    // 3. owner cell of every LDS point: each non-empty cell marks its first
    // point, then an inclusive max-scan over the points
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const int t = tid + NT * u;
        if (t < V && cnt_u[u] > 0u) L.pts[L.off[t]].w = __uint_as_float((uint32_t)t);
    }
    __syncthreads();
    constexpr int kPP = PTS / NT;
    uint32_t ow[kPP], mx = 0u;
#pragma unroll
    for (int k = 0; k < kPP; k++) {
        const int p = kPP * tid + k;
        const uint32_t o = p < npt ? __float_as_uint(L.pts[p].w) : 0u;
        mx = o > mx ? o : mx;
        ow[k] = mx;
    }
    uint32_t all;
    const uint32_t mi = block_incl_scan<NT, true>(mx, L.wred, all);
    uint32_t carry = NT == 64 ? __shfl_up(mi, 1, 64) : 0u;
    if constexpr (NT > 64) {
        // exclusive max = the inclusive max of the previous thread
        if (lane == 63) L.wred[wave] = mi;  // (block_incl_scan's own barriers are done)
        const uint32_t up = __shfl_up(mi, 1, 64);
        __syncthreads();
        carry = lane > 0 ? up : (wave > 0 ? L.wred[wave - 1] : 0u);
        __syncthreads();
    } else if (lane == 0) {
        carry = 0u;
    }
#pragma unroll
    for (int k = 0; k < kPP; k++) {
        const int p = kPP * tid + k;
        if (p < npt) L.pts[p].w = __uint_as_float(ow[k] > carry ? ow[k] : carry);
    }
    __syncthreads();
    // 4. copy: LDS point p = gpts[start[cell] + p - off[cell]], 8 loads in flight per thread
    for (int p0 = 0; p0 < npt; p0 += NT * 8) {
        uint32_t src[8];
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int p = p0 + NT * u + tid;
            src[u] = 0u;
            if (p < npt) {
                const uint32_t t = __float_as_uint(L.pts[p].w);
                src[u] = L.start[t] + (uint32_t)p - L.off[t];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (p0 + NT * u + tid < npt) v[u] = gpts[src[u]];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int p = p0 + NT * u + tid;
            if (p < npt) L.pts[p] = make_float4(v[u].x, v[u].y, v[u].z, __uint_as_float(src[u]));
        }
    }
    if (tid == 0) npts += total;
    __syncthreads();
    tv.on = true;
    tv.pts = L.pts;
    tv.off = L.off;
    return tv;
}

// Query cell and the side of it the query lies in (dir = -1 / +1 per axis).
__device__ __forceinline__ void grid_cell(const KnnParams& P, const LeafQuery& q, int& c0, int& c1, int& c2, int& s0,
                                          int& s1, int& s2) {
    const float inv = 1.0f / P.gh;
    auto cell_of = [&](float v, float o, int& c, int& dir) {
        const float t = (v - o) * inv;
        float f = floorf(t);
        f = fminf(fmaxf(f, (float)(8 - kGridBias)), (float)(kGridBias - 8));  // NaN -> 8 - bias
        c = (int)f;
        dir = (t - f < 0.5f) ? -1 : 1;
    };
    cell_of(q.qx, P.gorg[0], c0, s0);
    cell_of(q.qy, P.gorg[1], c1, s1);
    cell_of(q.qz, P.gorg[2], c2, s2);
}

// The exact 5-NN of one query on the cell grid (stages 0-2 above); cells of an
// active tile come from LDS.  Returns whether the list is certified exact.
// cube_done: every cell of the 3x3x3 cube was already scanned or pruned (the
// wave search below), so only the rings and stage 2 outside it remain.
// stage0_done: the 2x2x2 block was already scanned (vrun_search).
__device__ __forceinline__ bool grid_search(LeafQuery& q, const KnnParams& P, int c0, int c1, int c2, int s0, int s1,
                                            int s2, const TileView& tv, unsigned& visits, unsigned& npts,
                                            unsigned long long* prof = nullptr, bool cube_done = false,
                                            bool stage0_done = false) {
    // (prof: profiling builds, thread 0's stage cycles)
    unsigned long long pt = prof ? __builtin_amdgcn_s_memtime() : 0ull;
    auto mark = [&](int k) {
        if (prof) {
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            atomicAdd(prof + k, now - pt);
            pt = now;
        }
    };
    const float4* __restrict__ gpts = reinterpret_cast<const float4*>(P.gpts);
    const GridSlot* __restrict__ slots = P.gslots;
    const float h = P.gh, eps = P.geps;
    const uint64_t mask = (1ull << P.glog2) - 1ull;
    auto visit = [&](int cx, int cy, int cz) __attribute__((always_inline)) {
        const float x0 = P.gorg[0] + (float)cx * h - eps, y0 = P.gorg[1] + (float)cy * h - eps;
        const float z0 = P.gorg[2] + (float)cz * h - eps;
        const float w = h + 2 * eps;
        const float bd = box_dist(q.qx, q.qy, q.qz, x0, x0 + w, y0, y0 + w, z0, z0 + w);
        if (bd - lq_thr(q) > kFuzz) return;
        if (tv.on && cx >= tv.lo0 && cx <= tv.hi0 && cy >= tv.lo1 && cy <= tv.hi1 && cz >= tv.lo2 && cz <= tv.hi2) {
            const int t = ((cz - tv.lo2) * tv.d1 + (cy - tv.lo1)) * tv.d0 + (cx - tv.lo0);
            const int lo = (int)tv.off[t], hi = (int)tv.off[t + 1];
            constexpr int CH = TileLds<8, 8>::kChunk;  // every tile is padded by CH points
            for (int k0 = lo; k0 < hi; k0 += CH) {
                float4 v[CH];
#pragma unroll
                for (int u = 0; u < CH; u++) v[u] = tv.pts[k0 + u];  // padded by CH points
#pragma unroll
                for (int u = 0; u < CH; u++)
                    if (k0 + u < hi) lq_point(q, v[u], __float_as_uint(v[u].w));
            }
            return;
        }
        const unsigned long long key = grid_key_d(cx, cy, cz);
        uint64_t sl = (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - P.glog2));
        GridSlot gs = slots[sl];
        visits++;
        while (gs.key != key && gs.key != kGridEmpty) {  // linear probing (load factor <= 1/4)
            sl = (sl + 1) & mask;
            gs = slots[sl];
            visits++;
        }
        if (gs.key != key) return;
        const int lo = (int)gs.start, hi = (int)(gs.start + gs.count);
        npts += gs.count;
        for (int k0 = lo; k0 < hi; k0 += 4) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = gpts[k0 + u];  // padded by 3 points
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (k0 + u < hi) lq_point(q, v[u], (uint32_t)(k0 + u));
        }
    };
    // Cell boxes are int3 ranges [lo, hi]; a box with lo > hi is empty.
    // scan_box visits the cells of `r` outside the skip box.
    struct CBox { int l0, h0, l1, h1, l2, h2; };
    auto inside = [](const CBox& b, int x, int y, int z) {
        return x >= b.l0 && x <= b.h0 && y >= b.l1 && y <= b.h1 && z >= b.l2 && z <= b.h2;
    };
    auto scan_box = [&](const CBox& r, const CBox& skip) __attribute__((always_inline)) {
#pragma unroll 1
        for (int cz = r.l2; cz <= r.h2; cz++)
#pragma unroll 1
            for (int cy = r.l1; cy <= r.h1; cy++)
#pragma unroll 1
                for (int cx = r.l0; cx <= r.h0; cx++)
                    if (!inside(skip, cx, cy, cz)) visit(cx, cy, cz);
    };
    // the cells that can hold a point within sqrt(t) (+ the fuzz, + the float
    // slack of the cell assignment); false if that box is too large
    auto range_of = [&](float t, CBox& r) {
        const double rad = sqrt((double)t + 1e-9) * (1.0 + 1e-5) + (double)eps;
        const double ih = 1.0 / (double)h;
        const double lim = (double)(kGridBias - 8);
        const double l0 = floor(((double)q.qx - rad - (double)P.gorg[0]) * ih), h0 = floor(((double)q.qx + rad - (double)P.gorg[0]) * ih);
        const double l1 = floor(((double)q.qy - rad - (double)P.gorg[1]) * ih), h1 = floor(((double)q.qy + rad - (double)P.gorg[1]) * ih);
        const double l2 = floor(((double)q.qz - rad - (double)P.gorg[2]) * ih), h2 = floor(((double)q.qz + rad - (double)P.gorg[2]) * ih);
        if (!(fmax(fmax(fabs(l0), fabs(h0)), fmax(fmax(fabs(l1), fabs(h1)), fmax(fabs(l2), fabs(h2)))) < lim)) return false;
        r = CBox{(int)l0, (int)h0, (int)l1, (int)h1, (int)l2, (int)h2};
        return true;
    };
    if (!(P.lM > 0)) return false;
    const CBox cube{c0 - 1, c0 + 1, c1 - 1, c1 + 1, c2 - 1, c2 + 1};
    if (!cube_done) {
        // stage 0: the 2x2x2 block, own cell first
        if (!stage0_done) {
#pragma unroll 1
            for (int b = 0; b < 8; b++)
                visit(c0 + ((b & 1) ? s0 : 0), c1 + ((b & 2) ? s1 : 0), c2 + ((b & 4) ? s2 : 0));
        }
        mark(0);
        const CBox blk{c0 + min(s0, 0), c0 + max(s0, 0), c1 + min(s1, 0), c1 + max(s1, 0), c2 + min(s2, 0),
                       c2 + max(s2, 0)};
        // stage 1: within the 3x3x3 cube, the cells the current bound still
        // reaches (all of them while fewer than 5 points are known)
        CBox r1 = cube;
        if (lq_thr(q) < INFINITY && range_of(lq_thr(q), r1)) {
            r1.l0 = max(r1.l0, cube.l0); r1.h0 = min(r1.h0, cube.h0);
            r1.l1 = max(r1.l1, cube.l1); r1.h1 = min(r1.h1, cube.h1);
            r1.l2 = max(r1.l2, cube.l2); r1.h2 = min(r1.h2, cube.h2);
        } else {
            r1 = cube;
        }
        scan_box(r1, blk);
        mark(1);
    }
    // still fewer than 5 points (sparse map): cubes of radius 2, 3, ...
    CBox vis = cube;
#pragma unroll 1
    for (int rr = 2; rr <= kGridMaxRing && !(lq_thr(q) < INFINITY); rr++) {
        const CBox nb{c0 - rr, c0 + rr, c1 - rr, c1 + rr, c2 - rr, c2 + rr};
        scan_box(nb, vis);
        vis = nb;
    }
    // stage 2: every cell the final bound reaches; the list is then exact.
    // The bound only shrank, so the cells of `vis` it reaches are scanned
    // (r1 / the block / the cubes; a cell skipped there was beyond the bound)
    CBox r2;
    const float t = lq_thr(q);
    if (t < INFINITY && range_of(t, r2)) {
        const double span = (double)(r2.h0 - r2.l0 + 1) * (double)(r2.h1 - r2.l1 + 1) * (double)(r2.h2 - r2.l2 + 1);
        if (span <= (double)kGridMaxCells) {
            scan_box(r2, vis);
            mark(2);
            return true;
        }
    }
    mark(2);
    return false;
}

// ------------------------------------------------------------ run scan ----
// One query's scan of a run sorted by rho2 (the squared distance of each entry
// to the run's centre (cx, cy, cz); dqv >= |q - centre|): chunks of 8 entries,
// a chunk's 8 distances offered to the list only when one of them is below e6,
// and the scan stops at the first chunk whose first entry has rho > b = dqv +
// sqrt(bound) (+ margins), every later entry being farther than the bound.
// Returns the entries read.  The run array is padded by kRunPad entries.
//
// LIVO_RUN_PIPE = 1: two chunks in flight (A / B ping-pong): the loads of
// chunk k+2 are issued as soon as chunk k is consumed, so a lane waits for one
// load round trip per two chunks.  Chunk k+2 is not loaded when the run ends
// before it or when chunk k's last entry is already beyond b (the entries are
// sorted, so the scan stops at chunk k+1 at the latest).
#ifndef LIVO_RUN_PIPE
#define LIVO_RUN_PIPE 0
#endif
__device__ __forceinline__ float run_bound(const LeafQuery& q, float dqv) {
    const float thr = lq_thr(q);
    return thr < INFINITY ? dqv + __builtin_amdgcn_sqrtf(thr) * (1.0f + 1e-6f) + 1e-4f : INFINITY;
}
// slot(u): the candidate tag of entry k0 + u (a run position or a grid position)
template <class Slot>
__device__ __forceinline__ void run_chunk(LeafQuery& q, const float4 (&v)[8], uint32_t k0, uint32_t cnt, Slot&& slot) {
    float dist[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const float dx = q.qx - v[u].x, dy = q.qy - v[u].y, dz = q.qz - v[u].z;
        const float d = (dx * dx + dy * dy) + dz * dz;  // calc_dist (:1291-1295)
        dist[u] = k0 + u < cnt ? d : INFINITY;
    }
    const float m = fminf(fminf(fminf(dist[0], dist[1]), fminf(dist[2], dist[3])),
                          fminf(fminf(dist[4], dist[5]), fminf(dist[6], dist[7])));
    if (m < q.e6) {
#pragma unroll
        for (int u = 0; u < 8; u++) lq_offer(q, dist[u], slot(u));
    }
}
#if LIVO_IDX_RUNS
// Index runs: the run holds grid positions (4-aligned run start); a chunk's 8
// positions are two aligned 16-B loads, its points are gathered from the cell
// grid (pts), and the next chunk's positions are loaded with this chunk's
// points, so a chunk costs one gather round trip.  Candidates are grid
// positions (lq_finish reads them from pts like the cell walk's).
// On the incremental map's base set a point deleted after the runs were built
// keeps its place with x = NaN (k_dyn_tomb): its distance is NaN, which no
// comparison of the list admits (lq_offer: NaN < d is false, fminf drops it),
// and as a chunk's first entry it never stops the scan (NaN > b is false).
__device__ __forceinline__ uint32_t scan_run(LeafQuery& q, const uint32_t* __restrict__ run, uint32_t cnt,
                                             const float4* __restrict__ pts, float cx, float cy, float cz, float dqv,
                                             uint32_t tag = 0u) {
    if (cnt == 0) return 0;
    const uint4* __restrict__ r4 = reinterpret_cast<const uint4*>(run);  // (run start: a multiple of 4 words)
    uint4 ia = r4[0], ib = r4[1];  // (padded: kRunPad words behind the last run)
    uint32_t k0 = 0;
#pragma unroll 1
    for (; k0 < cnt; k0 += 8) {
        const uint32_t id[8] = {ia.x, ia.y, ia.z, ia.w, ib.x, ib.y, ib.z, ib.w};
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = pts[id[u]];  // (positions past the run: other runs' or 0, masked)
        if (k0 + 8 < cnt) {
            ia = r4[(k0 >> 2) + 2];
            ib = r4[(k0 >> 2) + 3];
        }
        const float b = run_bound(q, dqv);
        if (centre_d2(cx, cy, cz, v[0].x, v[0].y, v[0].z) > b * b) break;  // rho of every later entry > b
        run_chunk(q, v, k0, cnt, [&](int u) { return id[u] | tag; });
    }
    return min(k0, cnt);
}
#else
__device__ __forceinline__ uint32_t scan_run(LeafQuery& q, const float4* __restrict__ run, uint32_t cnt, uint32_t lo,
                                             float cx, float cy, float cz, float dqv) {
    auto slot = [&](uint32_t k0) { return [=](int u) { return kRunPos | (lo + k0 + (uint32_t)u); }; };
    uint32_t k0 = 0;
#if LIVO_RUN_PIPE
    if (cnt == 0) return 0;
    float4 A[8], B[8];
#pragma unroll
    for (int u = 0; u < 8; u++) A[u] = run[u];
    if (cnt > 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) B[u] = run[8 + u];
    }
    // one chunk: stop test, distances, then the loads two chunks ahead into the same registers
    auto step = [&](float4 (&v)[8]) __attribute__((always_inline)) -> bool {
        const float b = run_bound(q, dqv);
        if (centre_d2(cx, cy, cz, v[0].x, v[0].y, v[0].z) > b * b) return false;  // rho of every later entry > b
        run_chunk(q, v, k0, cnt, slot(k0));
        const float b2 = run_bound(q, dqv);
        const bool more = k0 + 16 < cnt && !(centre_d2(cx, cy, cz, v[7].x, v[7].y, v[7].z) > b2 * b2);
        if (more) {
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = run[k0 + 16 + u];
        }
        k0 += 8;
        return k0 < cnt;
    };
#pragma unroll 1
    while (true) {
        if (!step(A)) break;
        if (!step(B)) break;
    }
#else
#pragma unroll 1
    for (; k0 < cnt; k0 += 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = run[k0 + u];  // padded by kRunPad entries
        const float b = run_bound(q, dqv);
        if (centre_d2(cx, cy, cz, v[0].x, v[0].y, v[0].z) > b * b) break;  // rho of every later entry > b
        run_chunk(q, v, k0, cnt, slot(k0));
    }
#endif
    return min(k0, cnt);
}
#endif

// ------------------------------------------------------------ cell-run search ----
// The batched IEKF search on the cell runs (livo_internal.h): the run of the
// query's own cell c holds every map point of the 3x3x3 cells around c (the
// cube grid_search's stages 0-1 walk), sorted by rho2, the squared distance to
// c's centre.  One hash probe, then one contiguous scan.  By the triangle
// inequality a point with rho > |q - centre| + sqrt(bound) is farther than the
// bound min(5th candidate, seed bound), so the scan stops at the first chunk
// whose first entry is such a point (with a 1e-4 m margin over every float
// rounding involved, the approximate square root included: a point left out
// is farther than bound + 1e-10, so it could neither enter the list nor make
// e6 - d5 <= 1e-10, exactly as a pruned cell of grid_search).  Within a chunk
// of 8 entries a lane takes the per-point insertion path only when one of
// them is below its e6.  Candidates carry their run position (kRunPos bit
// set); lq_finish reads coordinates and map index from the run entry.  If the
// ball of the final bound lies in the cube the list is certified (every point
// within the bound was scanned); else the lane continues with grid_search's
// stage 2 outside the cube (candidates there are cell-grid slots).
// DYN (runs on the incremental map): the runs index P.rpts with deletion marks,
// and a list the cube does not certify is left uncertified (the caller's
// canonical resolution), since the cell walk's grid positions index another array.
template <bool DYN = false>
__device__ __forceinline__ bool vrun_search(LeafQuery& q, const KnnParams& P, bool valid, int c0, int c1, int c2,
                                            int s0, int s1, int s2, unsigned& visits, unsigned& npts) {
    if (!valid || !(P.lM > 0)) return false;
    const unsigned long long key = grid_key_d(c0, c1, c2);
    const uint64_t mask = (1ull << P.vlog2) - 1ull;
    uint64_t sl = (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - P.vlog2));
    GridSlot g = P.vslots[sl];
    visits++;
    while (g.key != key && g.key != kGridEmpty) {  // linear probing (load factor <= 1/4)
        sl = (sl + 1) & mask;
        g = P.vslots[sl];
        visits++;
    }
    const uint32_t lo = g.key == key ? g.start : 0u, cnt = g.key == key ? g.count : 0u;
    const float h = P.gh;
    const float cx = cell_centre(P.gorg[0], h, c0), cy = cell_centre(P.gorg[1], h, c1);
    const float cz = cell_centre(P.gorg[2], h, c2);
    const float dqv = __builtin_amdgcn_sqrtf(centre_d2(cx, cy, cz, q.qx, q.qy, q.qz)) * (1.0f + 1e-6f);
#if LIVO_IDX_RUNS
    npts += scan_run(q, P.vpts + lo, cnt, reinterpret_cast<const float4*>(P.rpts), cx, cy, cz, dqv);
#else
    const float4* __restrict__ run = reinterpret_cast<const float4*>(P.vpts) + lo;
    npts += scan_run(q, run, cnt, lo, cx, cy, cz, dqv);
#endif
    // certified when the ball of the final bound lies in the cube [c - 1, c + 1]
    const float t = lq_thr(q);
    if (t < INFINITY) {
        const double rad = sqrt((double)t + 1e-9) * (1.0 + 1e-5) + (double)P.geps;
        const double ih = 1.0 / (double)P.gh;
        const double q3[3] = {(double)q.qx, (double)q.qy, (double)q.qz};
        const int cc[3] = {c0, c1, c2};
        bool inside = true;
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const double l = floor((q3[a] - rad - (double)P.gorg[a]) * ih);
            const double hh = floor((q3[a] + rad - (double)P.gorg[a]) * ih);
            inside = inside && l >= (double)(cc[a] - 1) && hh <= (double)(cc[a] + 1);
        }
        if (inside) return true;
    }
    if constexpr (DYN) return false;
    TileView none;
    return grid_search(q, P, c0, c1, c2, s0, s1, s2, none, visits, npts, nullptr, true);
}

// ------------------------------------------------------------ ball-run search ----
// The batched IEKF search on the ball runs (livo_internal.h KnnParams::bslots):
// the run of the query's anchor cell a (edge P.bh) holds every map point within
// brmax of a's centre, sorted by rho2 (cr_rho2, the build's float operations).
// One hash probe, then one contiguous scan with vrun_search's stop rule: the
// scan stops at the first chunk whose first entry has rho > b = |q - a| +
// sqrt(bound) (+ the same margins), every later entry being farther than the
// bound.  The anchor is nearer the query than a cell-run centre (anchors are
// smaller than grid cells), so the scan reads fewer entries.  The list is
// certified when the final b satisfies b^2 <= P.bcert2 (brmax^2 less a relative
// 1e-5): every point within the bound (+ 1e-10) then lies in the ball, so it is
// in the run and was scanned.  Points outside the ball are farther than b, so,
// as a pruned cell of grid_search, they could neither enter the list nor make
// e6 - d5 <= 1e-10.  Not certified (or no run): the caller searches the cell
// runs from scratch.  Candidates carry their position in P.bpts (kRunPos set).
template <bool DYN = false>
__device__ __forceinline__ bool brun_search(LeafQuery& q, const KnnParams& P, bool valid, unsigned& visits,
                                            unsigned& npts) {
    if (!valid || !(P.lM > 0)) return false;
    const float inv = 1.0f / P.bh;
    int a[3];
    const float qq[3] = {q.qx, q.qy, q.qz};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        float f = floorf((qq[k] - P.gorg[k]) * inv);
        f = fminf(fmaxf(f, (float)(8 - kGridBias)), (float)(kGridBias - 8));  // NaN -> 8 - bias
        a[k] = (int)f;
    }
    const unsigned long long key = grid_key_d(a[0], a[1], a[2]);
    const uint64_t mask = (1ull << P.blog2) - 1ull;
    uint64_t sl = (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - P.blog2));
    GridSlot g = P.bslots[sl];
    visits++;
    while (g.key != key && g.key != kGridEmpty) {  // linear probing (load factor <= 1/4)
        sl = (sl + 1) & mask;
        g = P.bslots[sl];
        visits++;
    }
    if (g.key != key) return false;
#if LIVO_IDX_RUNS
    const size_t lo = (size_t)g.start << 2;  // (ball-run starts are stored / 4: 2^34 words addressable)
#else
    const uint32_t lo = g.start;
#endif
    const uint32_t cnt = g.count;
    const float cx = cell_centre(P.gorg[0], P.bh, a[0]), cy = cell_centre(P.gorg[1], P.bh, a[1]);
    const float cz = cell_centre(P.gorg[2], P.bh, a[2]);
    const float dqv = __builtin_amdgcn_sqrtf(centre_d2(cx, cy, cz, q.qx, q.qy, q.qz)) * (1.0f + 1e-6f);
#if LIVO_IDX_RUNS
    npts += scan_run(q, P.bpts + lo, cnt, reinterpret_cast<const float4*>(P.rpts), cx, cy, cz, dqv);
#else
    const float4* __restrict__ run = reinterpret_cast<const float4*>(P.bpts) + lo;
    npts += scan_run(q, run, cnt, lo, cx, cy, cz, dqv);
#endif
    const float t = lq_thr(q);
    if (!(t < INFINITY)) return false;
    const float b = dqv + __builtin_amdgcn_sqrtf(t) * (1.0f + 1e-6f) + 1e-4f;
    return b * b <= P.bcert2;
}

#if LIVO_IDX_RUNS
// The incremental map's delta (points added since its runs were built) has
// cell runs of its own over the delta grid: the query's cell's run (its
// 3x3x3 cube's delta points, sorted by rho2) scanned like the base's, its
// candidates tagged kRunPos | position in P.dpts.  Together with the base's
// run the cube's points are then all scanned: a list whose bound ball lies in
// the cube (cube_inside) is exact over both sets.
__device__ __forceinline__ void dvrun_scan(LeafQuery& q, const KnnParams& P, int c0, int c1, int c2, unsigned& visits,
                                           unsigned& npts) {
    const unsigned long long key = grid_key_d(c0, c1, c2);
    const uint64_t mask = (1ull << P.dvlog2) - 1ull;
    uint64_t sl = (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - P.dvlog2));
    GridSlot g = P.dvslots[sl];
    visits++;
    while (g.key != key && g.key != kGridEmpty) {
        sl = (sl + 1) & mask;
        g = P.dvslots[sl];
        visits++;
    }
    if (g.key != key) return;
    const float h = P.gh;
    const float cx = cell_centre(P.gorg[0], h, c0), cy = cell_centre(P.gorg[1], h, c1);
    const float cz = cell_centre(P.gorg[2], h, c2);
    const float dqv = __builtin_amdgcn_sqrtf(centre_d2(cx, cy, cz, q.qx, q.qy, q.qz)) * (1.0f + 1e-6f);
    npts += scan_run(q, P.dvidx + g.start, g.count, reinterpret_cast<const float4*>(P.dpts), cx, cy, cz, dqv, kRunPos);
}
#endif
// true when the ball of the list's bound (+ grid_search's margins) lies in the cube [c - 1, c + 1]
__device__ __forceinline__ bool cube_inside(const LeafQuery& q, const KnnParams& P, int c0, int c1, int c2) {
    const float t = lq_thr(q);
    if (!(t < INFINITY)) return false;
    const double rad = sqrt((double)t + 1e-9) * (1.0 + 1e-5) + (double)P.geps;
    const double ih = 1.0 / (double)P.gh;
    const double q3[3] = {(double)q.qx, (double)q.qy, (double)q.qz};
    const int cc[3] = {c0, c1, c2};
    bool inside = true;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const double l = floor((q3[a] - rad - (double)P.gorg[a]) * ih);
        const double hh = floor((q3[a] + rad - (double)P.gorg[a]) * ih);
        inside = inside && l >= (double)(cc[a] - 1) && hh <= (double)(cc[a] + 1);
    }
    return inside;
}

// The delta grid of the incremental map (points added since its runs were
// built; the cell grid's layout in P.dslots / P.dpts): every point of the
// cells the ball of the current bound reaches (with grid_search's margins) is
// offered, tagged kRunPos | its position in P.dpts.  The run search before it
// certified the base points within the bound, so the list is then exact over
// both sets (the bound only shrinks).  False when the ball spans more than
// kDeltaMaxCells cells: the caller's canonical resolution takes the query.
constexpr int kDeltaMaxCells = 64;
__device__ __forceinline__ bool delta_search(LeafQuery& q, const KnnParams& P, unsigned& visits, unsigned& npts) {
    const float t = lq_thr(q);
    if (!(t < INFINITY)) return false;
    const double rad = sqrt((double)t + 1e-9) * (1.0 + 1e-5) + (double)P.geps;
    const double ih = 1.0 / (double)P.gh, lim = (double)(kGridBias - 8);
    const double q3[3] = {(double)q.qx, (double)q.qy, (double)q.qz};
    int l[3], h[3];
    double span = 1.0;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const double lo = floor((q3[a] - rad - (double)P.gorg[a]) * ih), hi = floor((q3[a] + rad - (double)P.gorg[a]) * ih);
        if (!(fabs(lo) < lim && fabs(hi) < lim)) return false;
        l[a] = (int)lo;
        h[a] = (int)hi;
        span *= hi - lo + 1.0;
    }
    if (span > (double)kDeltaMaxCells) return false;
    const float4* __restrict__ dp = reinterpret_cast<const float4*>(P.dpts);
    const uint64_t mask = (1ull << P.dlog2) - 1ull;
#pragma unroll 1
    for (int cz = l[2]; cz <= h[2]; cz++)
#pragma unroll 1
        for (int cy = l[1]; cy <= h[1]; cy++)
#pragma unroll 1
            for (int cx = l[0]; cx <= h[0]; cx++) {
                const unsigned long long key = grid_key_d(cx, cy, cz);
                uint64_t sl = (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - P.dlog2));
                GridSlot g = P.dslots[sl];
                visits++;
                while (g.key != key && g.key != kGridEmpty) {
                    sl = (sl + 1) & mask;
                    g = P.dslots[sl];
                    visits++;
                }
                if (g.key != key) continue;
                npts += g.count;
#pragma unroll 1
                for (uint32_t k = g.start; k < g.start + g.count; k++) lq_point(q, dp[k], kRunPos | k);
            }
    return true;
}

// 512 points / 128 cells per wave (10.5 KB): 4 waves per SIMD (VGPR-bound);
// on MI355X 1024 / 256 (18.5 KB, 2 waves per SIMD) was 12 % slower at config 2
#ifndef LIVO_TILE_CELLS
#define LIVO_TILE_CELLS 128
#endif
#ifndef LIVO_TILE_PTS
#define LIVO_TILE_PTS 512
#endif
using WaveTile = TileLds<LIVO_TILE_CELLS, LIVO_TILE_PTS>;
// the block's tile (instantiated only by the TILE kernels)
__device__ __forceinline__ WaveTile& wave_tile_lds() {
    __shared__ WaveTile t;
    return t;
}

template <bool SEEDED, bool TILE>
__global__ __launch_bounds__(TILE ? 64 : kKnnBlock, TILE ? 4 : LIVO_GRID_WAVES) void k_knn_grid(KnnParams P) {
    constexpr int kB = TILE ? 64 : kKnnBlock;
    unsigned bjob, bx;
    xcd_block(P.nb, bjob, bx);
    const HsJob job = P.jobs[bjob];
    IekfSlot* slot = job.slot;
    if (P.force >= 0) {
        if (!P.force) return;
    } else {
        if (slot->ctrl.stop) return;
        if (SEEDED && !slot->ctrl.search_en) return;
    }
    const int i = (int)bx * kB + threadIdx.x;
    // the tile is built by the whole block: threads past the scan's end stay
    if (TILE ? (int)bx * kB >= job.n : i >= job.n) return;
    const bool valid = i < job.n;
    LeafQuery q;
    lq_init<SEEDED>(q, P, slot, job, i, valid);
    int c0 = 0, c1 = 0, c2 = 0, s0 = 1, s1 = 1, s2 = 1;
    if (valid) grid_cell(P, q, c0, c1, c2, s0, s1, s2);
    unsigned visits = 0, npts = 0;  // hash slots and map points read from global memory
    TileView tv;
    if constexpr (TILE) tv = build_tile<64>(wave_tile_lds(), P, valid, c0, c1, c2, visits, npts);
    if (valid) {
        const bool certified = grid_search(q, P, c0, c1, c2, s0, s1, s2, tv, visits, npts);
        lq_finish(q, P, job, bjob, i, reinterpret_cast<const float4*>(P.gpts), !certified);
    }
    count_visits(P, slot, visits, npts);
}

#if LIVO_IDX_RUNS
// The runs' search as a pass of its own (the unfused paths: the IKFoM update,
// LIVO_FUSED=0): k_iekf_eval's search stage -- ball run, cell run, the cell
// walk past the cube -- for every point of the batch, the neighbour record
// written, flagged queries queued for k_knn_replay.  LATER: a later
// evaluation, run only for scans whose last solve asked for a search (the
// search itself unseeded, as the fused kernel's).
template <bool LATER>
__global__ __launch_bounds__(kEvalBlock) void k_knn_runs(KnnParams P) {
    unsigned bjob, bx;
    xcd_block(P.nb, bjob, bx);
    const HsJob job = P.jobs[bjob];
    IekfSlot* slot = job.slot;
    if (P.force >= 0) {
        if (!P.force) return;
    } else {
        if (slot->ctrl.stop) return;
        if (LATER && !slot->ctrl.search_en) return;
    }
    if ((int)bx * kEvalBlock >= job.n) return;  // (block-uniform)
    const int i = (int)bx * kEvalBlock + threadIdx.x;
    const bool valid = i < job.n;
    LeafQuery q;
    lq_init<false>(q, P, slot, job, i, valid);
    int c0 = 0, c1 = 0, c2 = 0, s0 = 1, s1 = 1, s2 = 1;
    if (valid) grid_cell(P, q, c0, c1, c2, s0, s1, s2);
    unsigned visits = 0, npts = 0;
    bool certified = false;
    if (P.bslots) {
        certified = brun_search(q, P, valid, visits, npts);
        if (valid && !certified) lq_init<false>(q, P, slot, job, i, valid);
    }
    if (!certified) certified = vrun_search(q, P, valid, c0, c1, c2, s0, s1, s2, visits, npts);
    if (valid) lq_finish<false>(q, P, job, bjob, i, reinterpret_cast<const float4*>(P.gpts), !certified, true);
    count_visits(P, slot, visits, npts);
}
#endif

// Exact reference-order recomputation of the queries the fast pass flagged:
// KD_TREE::Search's visiting order with the far sons on an LDS stack and the
// exact MANUAL_HEAP (rare: ties / duplicates; one query per thread).
__global__ __launch_bounds__(64) void k_knn_replay(KnnParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char replay_smem[];  // (tree depth) x 64 stack entries
    uint2* const st_lds = reinterpret_cast<uint2*>(replay_smem);
    const unsigned n = *P.replay_count;
    if (blockIdx.x == 0 && threadIdx.x == 0 && n) atomicAdd(P.replay_total, (unsigned long long)n);
    uint2* stack = st_lds + threadIdx.x;
    for (unsigned t = blockIdx.x * 64 + threadIdx.x; t < n; t += gridDim.x * 64) {
        const unsigned long long e = P.replay_list[t];
        const HsJob job = P.jobs[(unsigned)(e >> 32)];
        const int i = (int)(unsigned)(e & 0xffffffffu);
        float qx, qy, qz;
        query_point(P, job.slot, reinterpret_cast<const float4*>(job.pts)[i], qx, qy, qz);
        KHeap h;
#pragma unroll
        for (int j = 0; j < kNN; j++) { h.d[j] = INFINITY; h.x[j] = 0.0f; h.node[j] = 0u; }
        h.size = 0;
        uint32_t node = 0;
        bool has = P.has_map != 0;
        int sp = 0;
        while (true) {
            if (!has) {
                if (sp == 0) break;
                sp--;
                const uint2 se = stack[sp * 64];
                if (h.size < kNN || __uint_as_float(se.y) < h.d[0]) { node = se.x; has = true; }
                else continue;
            }
            const float4* rp = rec_ptr(P.nodes, node);
            const float4 a = rp[0], b = rp[1], cc = rp[2], dd = rp[3];
            const uint32_t meta = __float_as_uint(a.w);
            const float dx = qx - a.x, dy = qy - a.y, dz = qz - a.z;
            const float dist = (dx * dx + dy * dy) + dz * dz;  // calc_dist (:1291-1295)
            if (dist <= INFINITY && (h.size < kNN || dist < h.d[0])) {
                if (h.size >= kNN) kh_pop(h);  // q.pop(); q.push(current_point)  (:861-863)
                kh_push(h, dist, a.x, node);
            }
            const bool hl = (meta & kLeftBit) != 0u, hr = (meta & kRightBit) != 0u;
            const float dl = hl ? box_dist(qx, qy, qz, b.x, b.y, b.z, b.w, cc.x, cc.y) : INFINITY;
            const float dr = hr ? box_dist(qx, qy, qz, cc.z, cc.w, dd.x, dd.y, dd.z, dd.w) : INFINITY;
            const bool lf = dl <= dr;
            const bool full = h.size >= kNN;
            const float top = h.d[0];
            if ((lf ? hr : hl) && (!full || (lf ? dr : dl) < top)) {
                stack[sp * 64] = make_uint2(2u * node + (lf ? 2u : 1u), __float_as_uint(lf ? dr : dl));
                sp++;
            }
            has = (lf ? hl : hr) && (!full || (lf ? dl : dr) < top);
            node = 2u * node + (lf ? 1u : 2u);
        }
        Cands c;
        kh_extract(h, c);
        float od[kNN];
        uint32_t on[kNN];
#pragma unroll
        for (int k = 0; k < kNN; k++) { od[k] = c.d[k]; on[k] = c.node[k]; }
        write_nnrec(job.nn + i, P.nodes, c.n, od, on, job.nn[i].flag | 0x100);
    }
}

// Canonical recomputation on the incremental map (livo_map_add_points, the
// ikd-Tree map_incremental, livo_map_delete_boxes).  After those the map is a
// point set whose ikd-Tree shape (Add_by_point, Rebuild and the background
// rebuild thread, ikd_Tree.cpp:158-300, 604-624) has no deterministic
// restatement, so the queries k_knn_grid flags (C1/C2) take the 5 nearest
// alive points in (distance, x, id) order -- PointType_CMP's order
// (ikd_Tree.h:50-61) wherever that is a strict order.  One query per thread:
// every cell within the grid's 5th distance, or every point if that bound is
// infinite or spans too many cells.
constexpr int kCanonMaxCells = 1 << 15;
__device__ __forceinline__ bool canon_less(float d1, float x1, uint32_t i1, float d2, float x2, uint32_t i2) {
    return d1 < d2 || (d1 == d2 && (x1 < x2 || (x1 == x2 && i1 < i2)));
}
template <class Src>
__device__ __forceinline__ void canon_query(const KnnParams& P, const HsJob& job, int i, const Src& src) {
    const float4* __restrict__ gpts = reinterpret_cast<const float4*>(P.gpts);
    const uint64_t mask = (1ull << P.glog2) - 1ull;
    {
        float qx, qy, qz;
        query_point(P, src, reinterpret_cast<const float4*>(job.pts)[i], qx, qy, qz);
        NNRec* rec = job.nn + i;
        const float T = rec->cnt == kNN ? rec->p[kNN - 1][3] : INFINITY;
        const int flag = rec->flag | 0x100;
        float bd[kNN], bx[kNN];
        uint32_t bi[kNN], bs[kNN];
#pragma unroll
        for (int k = 0; k < kNN; k++) { bd[k] = INFINITY; bx[k] = 0.f; bi[k] = 0xFFFFFFFFu; bs[k] = 0u; }
        auto offer = [&](uint32_t s) {
            const float4 v = gpts[s];
            const float dx = qx - v.x, dy = qy - v.y, dz = qz - v.z;
            const float d = (dx * dx + dy * dy) + dz * dz;  // calc_dist (:1291-1295)
            const uint32_t id = __float_as_uint(v.w);
            if (!canon_less(d, v.x, id, bd[kNN - 1], bx[kNN - 1], bi[kNN - 1])) return;
            bd[kNN - 1] = d; bx[kNN - 1] = v.x; bi[kNN - 1] = id; bs[kNN - 1] = s;
#pragma unroll
            for (int k = kNN - 1; k > 0; k--) {
                const bool sw = canon_less(bd[k], bx[k], bi[k], bd[k - 1], bx[k - 1], bi[k - 1]);
                const float td = bd[k], tx = bx[k];
                const uint32_t ti = bi[k], ts = bs[k];
                bd[k] = sw ? bd[k - 1] : td; bx[k] = sw ? bx[k - 1] : tx;
                bi[k] = sw ? bi[k - 1] : ti; bs[k] = sw ? bs[k - 1] : ts;
                bd[k - 1] = sw ? td : bd[k - 1]; bx[k - 1] = sw ? tx : bx[k - 1];
                bi[k - 1] = sw ? ti : bi[k - 1]; bs[k - 1] = sw ? ts : bs[k - 1];
            }
        };
        bool scanned = false;
        if (T < INFINITY && P.lM > 0) {
            const double rad = sqrt((double)T + 1e-9) * (1.0 + 1e-5) + (double)P.geps;
            const double ih = 1.0 / (double)P.gh, lim = (double)(kGridBias - 8);
            const double q3[3] = {qx, qy, qz};
            int l[3], h[3];
            bool ok = true;
            double span = 1.0;
#pragma unroll
            for (int a = 0; a < 3; a++) {
                const double lo = floor((q3[a] - rad - (double)P.gorg[a]) * ih);
                const double hi = floor((q3[a] + rad - (double)P.gorg[a]) * ih);
                ok = ok && fabs(lo) < lim && fabs(hi) < lim;
                l[a] = ok ? (int)lo : 0;
                h[a] = ok ? (int)hi : -1;
                span *= hi - lo + 1.0;
            }
            if (ok && span <= (double)kCanonMaxCells) {
                const float eps = P.geps, w = P.gh + 2 * eps;
                for (int cz = l[2]; cz <= h[2]; cz++)
                    for (int cy = l[1]; cy <= h[1]; cy++)
                        for (int cx = l[0]; cx <= h[0]; cx++) {
                            const float x0 = P.gorg[0] + (float)cx * P.gh - eps, y0 = P.gorg[1] + (float)cy * P.gh - eps;
                            const float z0 = P.gorg[2] + (float)cz * P.gh - eps;
                            if (box_dist(qx, qy, qz, x0, x0 + w, y0, y0 + w, z0, z0 + w) - T > kFuzz) continue;
                            const unsigned long long key = grid_key_d(cx, cy, cz);
                            uint64_t sl = (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - P.glog2));
                            GridSlot gs = P.gslots[sl];
                            while (gs.key != key && gs.key != kGridEmpty) {
                                sl = (sl + 1) & mask;
                                gs = P.gslots[sl];
                            }
                            if (gs.key != key) continue;
                            for (uint32_t s = gs.start; s < gs.start + gs.count; s++) offer(s);
                        }
                scanned = true;
            }
        }
        if (!scanned)
            for (int64_t s = 0; s < P.lM; s++) offer((uint32_t)s);
        const int cnt = (int)min<int64_t>(P.lM, (int64_t)kNN);
        float4* o4 = reinterpret_cast<float4*>(rec);
        int32_t idx[kNN];
#pragma unroll
        for (int k = 0; k < kNN; k++) {
            float4 v = make_float4(0.f, 0.f, 0.f, INFINITY);
            idx[k] = -1;
            if (k < cnt) {
                const float4 a = gpts[bs[k]];
                v = make_float4(a.x, a.y, a.z, bd[k]);
                idx[k] = (int32_t)bi[k];
            }
            o4[k] = v;
        }
        int4* oi = reinterpret_cast<int4*>(rec) + 5;
        oi[0] = make_int4(idx[0], idx[1], idx[2], idx[3]);
        oi[1] = make_int4(idx[4], cnt, flag, (int)bs[0]);
        oi[2] = make_int4((int)bs[1], (int)bs[2], (int)bs[3], (int)bs[4]);
    }
}
__global__ __launch_bounds__(64) void k_knn_canon(KnnParams P) {
    const unsigned n = *P.replay_count;
    if (blockIdx.x == 0 && threadIdx.x == 0 && n) atomicAdd(P.replay_total, (unsigned long long)n);
    for (unsigned t = blockIdx.x * 64 + threadIdx.x; t < n; t += gridDim.x * 64) {
        const unsigned long long e = P.replay_list[t];
        const HsJob& job = P.jobs[(unsigned)(e >> 32)];
        canon_query(P, job, (int)(unsigned)(e & 0xffffffffu), job.slot);
    }
}

// ======================================================== esti_plane ======
// Eigen 3.3 ColPivHouseholderQR<Matrix<float,5,3>> + solve(-1), restated with
// the SSE2 reduction orders documented in oracle/livo_oracle.cpp.  Columns of
// A live in registers as q[col][row] with compile-time indices only.
__device__ __forceinline__ float dot_tail(const float (&a)[5], const float (&b)[5], int k) {
    // sum_{i=k+1..4} a[i]*b[i]; length 4 uses the Packet4f predux order
    if (k == 0) return ((a[1] * b[1]) + (a[3] * b[3])) + ((a[2] * b[2]) + (a[4] * b[4]));
    if (k == 1) return (a[2] * b[2] + a[3] * b[3]) + a[4] * b[4];
    return a[3] * b[3] + a[4] * b[4];
}
__device__ __forceinline__ float sqn_tail(const float (&a)[5], int k) {
    if (k == 0) return ((a[1] * a[1] + a[2] * a[2]) + a[3] * a[3]) + a[4] * a[4];
    if (k == 1) return (a[2] * a[2] + a[3] * a[3]) + a[4] * a[4];
    return a[3] * a[3] + a[4] * a[4];
}

__device__ __forceinline__ void swap_cols(float (&u)[5], float (&v)[5]) {
#pragma unroll
    for (int r = 0; r < 5; r++) {
        float t = u[r]; u[r] = v[r]; v[r] = t;
    }
}

__device__ __forceinline__ bool esti_plane(const float (&px)[5], const float (&py)[5], const float (&pz)[5],
                                           float thr, float (&pabcd)[4]) {
    float q0[5], q1[5], q2[5];
#pragma unroll
    for (int r = 0; r < 5; r++) { q0[r] = px[r]; q1[r] = py[r]; q2[r] = pz[r]; }
    float nu[3], nd[3], hc[3];
    int tr[3];
    {
        float s0 = ((q0[0] * q0[0] + q0[2] * q0[2]) + (q0[1] * q0[1] + q0[3] * q0[3])) + q0[4] * q0[4];
        float s1 = ((q1[0] * q1[0] + q1[2] * q1[2]) + (q1[1] * q1[1] + q1[3] * q1[3])) + q1[4] * q1[4];
        float s2 = ((q2[0] * q2[0] + q2[2] * q2[2]) + (q2[1] * q2[1] + q2[3] * q2[3])) + q2[4] * q2[4];
        nd[0] = sqrtf(s0); nd[1] = sqrtf(s1); nd[2] = sqrtf(s2);
        nu[0] = nd[0]; nu[1] = nd[1]; nu[2] = nd[2];
    }
    const float eps = 1.1920928955078125e-07f;  // FLT_EPSILON
    float mxn = nu[0];
    if (nu[1] > mxn) mxn = nu[1];
    if (nu[2] > mxn) mxn = nu[2];
    const float th_help = (mxn * eps) * (mxn * eps) / 5.0f;
    const float ndt = sqrtf(eps);
    int nonzero = 3;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        // pivot: first maximum of the updated norms over columns k..2
        int big = k;
        float bigv = nu[k];
#pragma unroll
        for (int j = k + 1; j < 3; j++)
            if (nu[j] > bigv) { bigv = nu[j]; big = j; }
        const float big_sq = bigv * bigv;
        if (nonzero == 3 && big_sq < th_help * (float)(5 - k)) nonzero = k;
        tr[k] = big;
        if (big != k) {
            if (k == 0) {
                if (big == 1) { swap_cols(q0, q1); float t = nu[0]; nu[0] = nu[1]; nu[1] = t; t = nd[0]; nd[0] = nd[1]; nd[1] = t; }
                else { swap_cols(q0, q2); float t = nu[0]; nu[0] = nu[2]; nu[2] = t; t = nd[0]; nd[0] = nd[2]; nd[2] = t; }
            } else {
                swap_cols(q1, q2); float t = nu[1]; nu[1] = nu[2]; nu[2] = t; t = nd[1]; nd[1] = nd[2]; nd[2] = t;
            }
        }
        float (&col)[5] = (k == 0) ? q0 : (k == 1 ? q1 : q2);
        // makeHouseholderInPlace
        const float c0 = col[k];
        const float tailSq = sqn_tail(col, k);
        float tau, beta;
        if (tailSq <= 1.17549435082228750797e-38f) {  // FLT_MIN
            tau = 0.0f;
            beta = c0;
#pragma unroll
            for (int i = k + 1; i < 5; i++) col[i] = 0.0f;
        } else {
            beta = sqrtf(c0 * c0 + tailSq);
            if (c0 >= 0.0f) beta = -beta;
            const float den = c0 - beta;
#pragma unroll
            for (int i = k + 1; i < 5; i++) col[i] = col[i] / den;
            tau = (beta - c0) / beta;
        }
        hc[k] = tau;
        col[k] = beta;
        // applyHouseholderOnTheLeft on columns k+1..2
        if (tau != 0.0f) {
#pragma unroll
            for (int j = k + 1; j < 3; j++) {
                float (&cj)[5] = (j == 1) ? q1 : q2;
                float tmp = dot_tail(col, cj, k);
                tmp = tmp + cj[k];
                cj[k] = cj[k] - tau * tmp;
#pragma unroll
                for (int i = k + 1; i < 5; i++) cj[i] = cj[i] - (tau * col[i]) * tmp;
            }
        }
        // norm downdate
#pragma unroll
        for (int j = k + 1; j < 3; j++) {
            const float (&cj)[5] = (j == 1) ? q1 : q2;
            if (nu[j] != 0.0f) {
                float temp = fabsf(cj[k]) / nu[j];
                temp = (1.0f + temp) * (1.0f - temp);
                temp = temp < 0.0f ? 0.0f : temp;
                const float ratio = nu[j] / nd[j];
                const float temp2 = temp * (ratio * ratio);
                if (temp2 <= ndt) {
                    nd[j] = sqrtf(sqn_tail(cj, k));
                    nu[j] = nd[j];
                } else {
                    nu[j] = nu[j] * sqrtf(temp);
                }
            }
        }
    }
    int perm[3] = {0, 1, 2};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        // swap(perm[k], perm[tr[k]]) with compile-time indices
        const int t = tr[k];
        int pk = perm[k];
        int pt = (t == 0) ? perm[0] : (t == 1 ? perm[1] : perm[2]);
        if (t != k) {
            if (t == 1) perm[1] = pk; else if (t == 2) perm[2] = pk; else perm[0] = pk;
            perm[k] = pt;
        }
    }
    float x0 = 0.0f, x1 = 0.0f, x2 = 0.0f;
    if (nonzero > 0) {
        float c[5] = {-1.0f, -1.0f, -1.0f, -1.0f, -1.0f};
#pragma unroll
        for (int k = 0; k < 3; k++) {
            if (k < nonzero) {
                const float tau = hc[k];
                if (tau != 0.0f) {
                    const float (&ess)[5] = (k == 0) ? q0 : (k == 1 ? q1 : q2);
                    float tmp = dot_tail(ess, c, k);
                    tmp = tmp + c[k];
                    c[k] = c[k] - tau * tmp;
#pragma unroll
                    for (int i = k + 1; i < 5; i++) c[i] = c[i] - (tau * ess[i]) * tmp;
                }
            }
        }
        // back substitution with R = upper triangle of q (R(s,i) = q_i[s])
#pragma unroll
        for (int i = 2; i >= 0; i--) {
            if (i < nonzero && c[i] != 0.0f) {
                const float (&qi)[5] = (i == 0) ? q0 : (i == 1 ? q1 : q2);
                c[i] = c[i] / qi[i];
#pragma unroll
                for (int s = 0; s < i; s++) c[s] = c[s] - c[i] * qi[s];
            }
        }
        float xs[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int i = 0; i < 3; i++) {
            if (i < nonzero) {
                const int pi = perm[i];
                if (pi == 0) xs[0] = c[i]; else if (pi == 1) xs[1] = c[i]; else xs[2] = c[i];
            }
        }
        x0 = xs[0]; x1 = xs[1]; x2 = xs[2];
    }
    const float n = sqrtf((x0 * x0 + x1 * x1) + x2 * x2);
    pabcd[0] = x0 / n;
    pabcd[1] = x1 / n;
    pabcd[2] = x2 / n;
    pabcd[3] = (float)(1.0 / (double)n);
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const float r = ((pabcd[0] * px[j] + pabcd[1] * py[j]) + pabcd[2] * pz[j]) + pabcd[3];
        if (fabsf(r) > thr) ok = false;
    }
    return ok;
}

// ========================================================== solve =========
// One wave per scan (laser_mapping.cpp:187-193).  The reference forms
//   K1 = (H_T_H + P^-1)^-1,  G(:,0:9) = K1(:,0:9) HTH,
//   solution = K1(:,0:9) HTL + vec - G(:,0:9) vec(0:9)
// with two 18x18 PartialPivLU inversions.  H_T_H is non-zero only in its 6x6
// block C (rows/cols 6..8 of HTH are zero without GNSS, :580-590), so with
// U = [I6; 0]:  (P^-1 + U C U^T) K1 U = U  gives
//   K1(:,0:6) = P(:,0:6) (I6 + C P66)^-1          (P66 = P(0:6,0:6))
// and K1(:,6:9) only ever multiplies zeros.  Hence
//   G(:,0:6) = K1(:,0:6) C,  solution = K1(:,0:6) (HTL6 - C vec6) + vec,
//   state.cov = (I - G) P = P - G(:,0:6) P(0:6,:)
// -- one 6x6 LU instead of two 18x18 ones and no P^-1 at all.  Same quantities
// as the oracle's LU path to ~1e-13 relative (tests/test_gpu_parity.py bars:
// state delta 1e-5, covariance 1e-9).
#ifdef LIVO_SOLVE_PROF  // phase timestamps for tools/solve_lab (compiled out of the product)
__device__ unsigned long long g_solve_prof[256][16];
#define SOLVE_MARK(k) do { if ((threadIdx.x & 63) == 0) g_solve_prof[blockIdx.x][k] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define SOLVE_MARK(k) do { } while (0)
#endif
#ifdef LIVO_TAIL_PROF  // solve_scan's phases summed per evaluation kind (tools/eval_prof.py)
__device__ unsigned long long g_solve_ph[3][16];
#define SPH_MARK(k)                                                                                     \
    do {                                                                                               \
        if (pk >= 0 && lane == 0) {                                                                    \
            const unsigned long long now_ = __builtin_amdgcn_s_memtime();                             \
            atomicAdd(&g_solve_ph[pk][(k)], now_ - sph_t);                                             \
            sph_t = now_;                                                                              \
        }                                                                                              \
    } while (0)
#else
#define SPH_MARK(k) do { } while (0)
#endif
// LDS of one scan's solve.  The slot fields it reads are staged here by the
// calling block (solve_stage) in one round trip, so the solve itself reads no
// global memory and its stores go out behind it.
struct alignas(16) SolveLds {
    double sum[kRedCols];
    double P[kDim * kDim];      // state.cov
    StateHead st;               // state (rot, pos, vel, biases, gravity)
    StateHead pr;               // prior (state_propagat)
    double C[36];               // H_T_H(0:6, 0:6)
    double M[36];               // I6 + C P66
    double LU[36];
    double Minv[36];
    double K6[kDim * 6];        // K1(:, 0:6)
    double G6[kDim * 6];        // G(:, 0:6)
    double w[6];                // HTL6 - C vec6
    double vec[kDim];
    double sol[kDim];
    // the factored path (slot->cov_ok): S = L L^T and B = P(:, 0:6) L^-T staged
    // from the slot (covL, covB contiguous, as in IekfSlot), Q = I6 + L^T C L
    double covL[36];
    double covB[(kDim - 6) * 6];
    double T[36];               // C L
    double Q[36];               // I6 + L^T C L
    double F[28];               // LDL^T of Q: 21 packed lower entries (D on the diagonal), then 6 x 1/D
    double u[6];                // L^T w
    double Qi[36];              // Q^-1 (stopping solve)
    double V[kDim * 6];         // B (I6 - Q^-1) (stopping solve)
    int piv[6];
    alignas(16) IekfCtrl ctrl;
    int knn_passes;             // stats.knn_passes so far
    int cov_ok;                 // slot->cov_ok
};
static_assert(offsetof(SolveLds, covB) == offsetof(SolveLds, covL) + 36 * sizeof(double) &&
                  offsetof(IekfSlot, covB) == offsetof(IekfSlot, covL) + 36 * sizeof(double),
              "covL, covB contiguous in the slot and in LDS");
constexpr int kStHead = (int)(sizeof(StateHead) / sizeof(double));  // 24
static_assert(sizeof(StateHead) == 24 * sizeof(double) && offsetof(livo_state, cov) == sizeof(StateHead),
              "StateHead is the head of livo_state");

// sc1 (agent-coherent) loads and write-through stores of slot / partial words
// (global addressing: gptr, top of the file).
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __hip_atomic_load(gptr(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_sc1(const int* p) {
    return __hip_atomic_load(gptr(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_sc1(const unsigned long long* p) {
    return __hip_atomic_load(gptr(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Write-through (sc1) stores of slot / partial words read by other CUs inside
// one launch (the reduction's hand-offs).  INVARIANT: every in-launch read of a
// word another workgroup stored goes through ld_sc1 (an agent-scope atomic load
// of a global address): a plain or scalar load may be served by this CU's L1 or
// by the scalar cache, which other CUs' stores do not refresh (round 5: job
// pointers laundered into scalar loads faulted).
template <class T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
    __hip_atomic_store(gptr(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Stage the solve's inputs (cov, state and prior heads, control, knn_passes)
// into L: thread t of nt, two loads in flight per thread before any LDS store.
// sc1 loads: the slot may have been written by another CU of this launch.
__device__ __forceinline__ void solve_stage(const IekfSlot* slot, SolveLds& L, int t, int nt) {
    // doubles: cov, state head, prior head, covariance factors (covL, covB)
    constexpr int nP = kDim * kDim, nH = nP + 2 * kStHead, nD = nH + 36 + (kDim - 6) * 6;
    auto src = [&](int k) -> const double* {
        return k < nP ? slot->state.cov + k
                      : (k < nP + kStHead ? slot->state.rot + (k - nP)
                                          : (k < nH ? slot->prior.rot + (k - nP - kStHead) : slot->covL + (k - nH)));
    };
    auto dst = [&](int k) -> double* {
        return k < nP ? L.P + k
                      : (k < nP + kStHead ? L.st.rot + (k - nP) : (k < nH ? L.pr.rot + (k - nP - kStHead) : L.covL + (k - nH)));
    };
    for (int k0 = t; k0 < nD; k0 += 2 * nt) {
        const int k1 = k0 + nt;
        const double v0 = ld_sc1(src(k0));
        const double v1 = k1 < nD ? ld_sc1(src(k1)) : 0.0;
        *dst(k0) = v0;
        if (k1 < nD) *dst(k1) = v1;
    }
    if (t == nt - 1) {
        const unsigned long long* c = reinterpret_cast<const unsigned long long*>(&slot->ctrl);
        const unsigned long long c0 = ld_sc1(c), c1 = ld_sc1(c + 1), c2 = ld_sc1(c + 2), c3 = ld_sc1(c + 3);
        const int kp = ld_sc1(&slot->stats.knn_passes);
        const int ok = ld_sc1(&slot->cov_ok);
        unsigned long long* d = reinterpret_cast<unsigned long long*>(&L.ctrl);
        d[0] = c0;
        d[1] = c1;
        d[2] = c2;
        d[3] = c3;
        L.knn_passes = kp;
        L.cov_ok = ok;
    }
}
static_assert(sizeof(IekfCtrl) == 8 * sizeof(int) && alignof(IekfSlot) >= 16 && offsetof(IekfSlot, ctrl) % 16 == 0,
              "IekfCtrl is two aligned int4");

// One wave (lanes 0..63 of the calling block), from the reduced h_share sums
// in L.sum and the staged inputs.  vec = state_propagat - state is computed by
// lane 0 first (SPLIT_VEC = false) or, beside M and its LU, by another wave of
// the block that then meets this wave at one block barrier (SPLIT_VEC = true).
// Only this wave touches L otherwise, so LDS hand-offs between its lanes need
// a wave-level fence, not a block barrier.  Returns EKF_stop_flg (uniform).
template <bool SPLIT_VEC = false>
__device__ __forceinline__ int solve_scan(IekfSlot* slot, SolveLds& L, const int lane, int pk = -1) {
#ifdef LIVO_TAIL_PROF
    unsigned long long sph_t = __builtin_amdgcn_s_memtime();
#else
    (void)pk;
#endif
    const double* const s_sum = L.sum;
    const double* const s_P = L.P;
    if (!SPLIT_VEC && lane == 0) state_minus_d(L.pr, L.st, L.vec);  // vec = state_propagat - state
    if (lane < 36) {
        const int r = lane / 6, c = lane % 6;
        const int a = r < c ? r : c, b = r < c ? c : r;
        L.C[lane] = s_sum[a * 6 - (a * (a - 1)) / 2 + (b - a)];  // upper-tri packed index
    }
    const IekfCtrl ctrl0 = L.ctrl;
    const int e = ctrl0.n_evals;
    WAVE_SYNC();
    SOLVE_MARK(2);
    SPH_MARK(0);
    const bool fac = L.cov_ok != 0;  // (LDS: uniform)
    if (fac) {
        // The factored form (slot covL / covB, made by the host from the covariance):
        // with S = P66 = L L^T, M = I6 + C S = L^-T Q L^T for Q = I6 + L^T C L, so
        //   K1(:, 0:6) = P(:, 0:6) M^-1 = B Q^-1 L^T,  B = P(:, 0:6) L^-T,
        //   solution = B Q^-1 (L^T w) + vec.
        // Q is SPD with eigenvalues >= 1: an LDL^T without pivoting is stable, and
        // every lane factors it in registers (the same values, no cross-lane steps):
        // the pivoted 6x6 LU's argmax / row broadcasts are off the chain.
        const double* const Lf = L.covL;
#ifdef LIVO_TAIL_TWICE  // I-cache probe (tools/tail_prof.py): T and Q formed twice, the first pass timed into marks 8, 9
#pragma unroll 1
        for (int rep = 0; rep < 2; rep++) {
#endif
        // T = C L (lanes 0..35): T(r, c) = sum_{k >= c} C(r, k) L(k, c)
        if (lane < 36) {
            const int r = lane / 6, c = lane % 6;
            double t = 0.0;
#pragma unroll
            for (int k = 0; k < 6; k++)
                if (k >= c) t = t + L.C[r * 6 + k] * Lf[k * 6 + c];
            L.T[lane] = t;
        }
        WAVE_SYNC();
#ifdef LIVO_TAIL_TWICE
        SPH_MARK(rep == 0 ? 8 : 1);
#else
        SPH_MARK(1);
#endif
        // Q = I6 + L^T T (lanes 0..35): Q(r, c) = [r == c] + sum_{k >= r} L(k, r) T(k, c)
        if (lane < 36) {
            const int r = lane / 6, c = lane % 6;
            double q = 0.0;
#pragma unroll
            for (int k = 0; k < 6; k++)
                if (k >= r) q = q + Lf[k * 6 + r] * L.T[k * 6 + c];
            L.Q[lane] = (r == c ? 1.0 : 0.0) + q;
        }
        WAVE_SYNC();
#ifdef LIVO_TAIL_TWICE
        if (rep == 0) SPH_MARK(9);
        }
#endif
        // LDL^T of Q in place (f: packed lower, D on the diagonal), every lane
        double f[21], di[6];
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
            for (int j = 0; j <= i; j++) f[i * (i + 1) / 2 + j] = 0.5 * (L.Q[i * 6 + j] + L.Q[j * 6 + i]);
#pragma unroll
        for (int j = 0; j < 6; j++) {
            double wv[6];
            double d = f[j * (j + 1) / 2 + j];
#pragma unroll
            for (int k = 0; k < j; k++) {
                wv[k] = f[j * (j + 1) / 2 + k] * f[k * (k + 1) / 2 + k];  // L(j, k) D(k)
                d = d - f[j * (j + 1) / 2 + k] * wv[k];
            }
            f[j * (j + 1) / 2 + j] = d;
            di[j] = 1.0 / d;
#pragma unroll
            for (int i = j + 1; i < 6; i++) {
                double v = f[i * (i + 1) / 2 + j];
#pragma unroll
                for (int k = 0; k < j; k++) v = v - f[i * (i + 1) / 2 + k] * wv[k];
                f[i * (i + 1) / 2 + j] = v * di[j];
            }
        }
        if (lane == 0) {  // for a stopping solve's Q^-1
#pragma unroll
            for (int k = 0; k < 21; k++) L.F[k] = f[k];
#pragma unroll
            for (int k = 0; k < 6; k++) L.F[21 + k] = di[k];
        }
        SPH_MARK(2);
        if (SPLIT_VEC) __syncthreads();  // L.vec from the other wave (it waits here too)
        // w = HTL6 - C vec6, u = L^T w (lanes 0..5)
        if (lane < 6) {
            double wv = s_sum[21 + lane];
#pragma unroll
            for (int k = 0; k < 6; k++) wv = wv - L.C[lane * 6 + k] * L.vec[k];
            L.w[lane] = wv;
        }
        WAVE_SYNC();
        if (lane < 6) {
            double uu = 0.0;
#pragma unroll
            for (int k = 0; k < 6; k++)
                if (k >= lane) uu = uu + Lf[k * 6 + lane] * L.w[k];
            L.u[lane] = uu;
        }
        WAVE_SYNC();
        SPH_MARK(3);
        // y = Q^-1 u (every lane), solution = B y + vec (lanes 0..17)
        double y[6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            double z = L.u[i];
#pragma unroll
            for (int k = 0; k < i; k++) z = z - f[i * (i + 1) / 2 + k] * y[k];
            y[i] = z;
        }
#pragma unroll
        for (int i = 0; i < 6; i++) y[i] = y[i] * di[i];
#pragma unroll
        for (int i = 4; i >= 0; i--) {
            double z = y[i];
#pragma unroll
            for (int k = i + 1; k < 6; k++) z = z - f[k * (k + 1) / 2 + i] * y[k];
            y[i] = z;
        }
        SPH_MARK(4);
        if (lane < kDim) {
            const double* b = lane < 6 ? Lf + lane * 6 : L.covB + (lane - 6) * 6;
            double a = b[0] * y[0];
#pragma unroll
            for (int k = 1; k < 6; k++) a = a + b[k] * y[k];
            L.sol[lane] = a + L.vec[lane];
        }
        WAVE_SYNC();
        SPH_MARK(5);
    } else {
        // M = I6 + C P66
        if (lane < 36) {
            const int r = lane / 6, c = lane % 6;
            double m = L.C[r * 6 + 0] * s_P[0 * kDim + c];
#pragma unroll
            for (int k = 1; k < 6; k++) m = m + L.C[r * 6 + k] * s_P[k * kDim + c];
            L.M[lane] = (r == c ? 1.0 : 0.0) + m;
        }
        WAVE_SYNC();
        SPH_MARK(1);
        double A6[6];
#pragma unroll
        for (int j = 0; j < 6; j++) A6[j] = lane < 6 ? L.M[lane * 6 + j] : 0.0;
        wave_lu_to_lds<6>(A6, lane, L.LU, L.piv);
        WAVE_SYNC();
        SPH_MARK(2);
        {
            double y[6];
            reg_lu_column<6>(A6, L.piv, lane, y);  // (readlanes: every lane runs it)
            if (lane < 6) {
#pragma unroll
                for (int i = 0; i < 6; i++) L.Minv[i * 6 + lane] = y[i];
            }
        }
        if (SPLIT_VEC) __syncthreads();  // L.vec from the other wave (it waits here too)
        if (lane < 6) {
            double wv = s_sum[21 + lane];
#pragma unroll
            for (int k = 0; k < 6; k++) wv = wv - L.C[lane * 6 + k] * L.vec[k];
            L.w[lane] = wv;
        }
        WAVE_SYNC();
        SOLVE_MARK(4);
        SPH_MARK(3);
        // K1(:, 0:6) = P(:, 0:6) M^-1
        for (int t = lane; t < kDim * 6; t += 64) {
            const int r = t / 6, c = t % 6;
            double k6 = s_P[r * kDim + 0] * L.Minv[0 * 6 + c];
#pragma unroll
            for (int k = 1; k < 6; k++) k6 = k6 + s_P[r * kDim + k] * L.Minv[k * 6 + c];
            L.K6[t] = k6;
        }
        WAVE_SYNC();
        SPH_MARK(4);
        // G(:, 0:6) = K1(:, 0:6) C ;  solution = K1(:, 0:6) w + vec
        for (int t = lane; t < kDim * 6; t += 64) {
            const int r = t / 6, c = t % 6;
            double g = L.K6[r * 6 + 0] * L.C[0 * 6 + c];
#pragma unroll
            for (int k = 1; k < 6; k++) g = g + L.K6[r * 6 + k] * L.C[k * 6 + c];
            L.G6[t] = g;
        }
        if (lane < kDim) {
            double a = L.K6[lane * 6 + 0] * L.w[0];
#pragma unroll
            for (int k = 1; k < 6; k++) a = a + L.K6[lane * 6 + k] * L.w[k];
            L.sol[lane] = a + L.vec[lane];
        }
        WAVE_SYNC();
        SPH_MARK(5);
        SOLVE_MARK(7);
    }
    // 8. boxplus, convergence, rematch control (laser_mapping.cpp:204-237) on the
    // staged state, the whole wave: every lane forms Exp(sol(0:3)) and the control
    // from the same values (one SIMT pass of the sin / cos chain instead of lane 0
    // alone walking the state), lanes 0..8 the new rotation, 9..23 the additive
    // parts; the stores below go out behind the solve (nothing waits for them)
    int stop_now = 0;
    {
        IekfCtrl ctrl = ctrl0;
        const double v0 = L.sol[0], v1 = L.sol[1], v2 = L.sol[2];
        const double t0 = L.sol[3], t1 = L.sol[4], t2 = L.sol[5];
        double rot[9], E[9];
#pragma unroll
        for (int k = 0; k < 9; k++) rot[k] = L.st.rot[k];
        so3_exp(v0, v1, v2, E);  // StatesGroup += (common_lib.h:565-574): rot * Exp(sol(0:3))
        const double rn = sqrt((v0 * v0 + v1 * v1) + v2 * v2);
        const double tn = sqrt((t0 * t0 + t1 * t1) + t2 * t2);
        const bool converged = (rn * 180 / (3.14159265358) < 0.01) && (tn * 100 < 0.015);
        const int searched = ctrl.search_en;
        bool next_search = false;
        if (converged || ((ctrl.rematch_num == 0) && (ctrl.iter_count == (ctrl.max_iter - 2)))) {
            next_search = true;
            ctrl.rematch_num++;
        }
        const bool stop = (ctrl.rematch_num >= 2 || (ctrl.iter_count == ctrl.max_iter - 1));
        ctrl.converged = converged ? 1 : 0;
        ctrl.last_search = searched;
        ctrl.search_en = next_search ? 1 : 0;
        ctrl.iter_count++;
        ctrl.n_evals = e + 1;
        // the loop condition iterCount < NUM_MAX_ITERATIONS (:178) also ends it
        ctrl.stop = (stop || ctrl.iter_count >= ctrl.max_iter || ctrl.n_evals >= LIVO_MAX_EVALS) ? 1 : 0;
        stop_now = stop ? 1 : 0;
        if (lane < 9) {  // mat3_mul(rot, E) entry (r, c), sums in index order
            const int r = lane / 3, c = lane % 3;
            double a0 = 0.0, a1 = 0.0, a2 = 0.0, e0 = 0.0, e1 = 0.0, e2 = 0.0;
#pragma unroll
            for (int k = 0; k < 3; k++) {
                if (r == k) { a0 = rot[k * 3 + 0]; a1 = rot[k * 3 + 1]; a2 = rot[k * 3 + 2]; }
                if (c == k) { e0 = E[0 * 3 + k]; e1 = E[1 * 3 + k]; e2 = E[2 * 3 + k]; }
            }
            L.st.rot[lane] = (a0 * e0 + a1 * e1) + a2 * e2;
        } else if (lane < kStHead) {  // pos, vel, bias_g, bias_a, gravity += sol(3:18)
            L.st.rot[lane] = L.st.rot[lane] + L.sol[lane - 6];
        }
        if (lane == 0) L.ctrl = ctrl;
    }
    stop_now = __builtin_amdgcn_readfirstlane(stop_now);
    WAVE_SYNC();
    SOLVE_MARK(8);
    SPH_MARK(6);
    // stores: state head, statistics, control (write-through: the stopping scan's
    // host slot copy reads them back inside this launch)
    if (lane < kStHead) st_sc1(slot->state.rot + lane, L.st.rot[lane]);
    livo_iter_stats& S = slot->stats;
    if (e < LIVO_MAX_EVALS) {
        if (lane < kDim) S.solution[e][lane] = L.sol[lane];
        if (lane == 0) {
            S.effct_feat_num[e] = (int64_t)s_sum[28];
            S.res_mean[e] = s_sum[27] / s_sum[28];
            slot->eval_search[e] = ctrl0.search_en;
        }
    }
    if (lane == 0) {
        S.iterations = e + 1;
        st_sc1(&S.knn_passes, L.knn_passes + (ctrl0.search_en ? 1 : 0));
        S.converged = L.ctrl.converged;
        S.rematch_num = L.ctrl.rematch_num;
    }
    if (lane < 4) {  // the control block as four 8-B stores
        const unsigned long long c = reinterpret_cast<const unsigned long long*>(&L.ctrl)[lane];
        st_sc1(reinterpret_cast<unsigned long long*>(&slot->ctrl) + lane, c);
    }
    // 9. covariance update state.cov = (I - G) * state.cov (:224-227) = P - G(:,0:6) P(0:6,:)
    if (stop_now && fac) {
        // factored: G(:, 0:6) P(0:6, :) = B Q^-1 (L^T C L) B^T = B (I6 - Q^-1) B^T
        if (lane < 6) {  // column `lane` of Q^-1 from the LDL^T factors
            double x[6];
#pragma unroll
            for (int i = 0; i < 6; i++) {
                double z = i == lane ? 1.0 : 0.0;
#pragma unroll
                for (int k = 0; k < i; k++) z = z - L.F[i * (i + 1) / 2 + k] * x[k];
                x[i] = z;
            }
#pragma unroll
            for (int i = 0; i < 6; i++) x[i] = x[i] * L.F[21 + i];
#pragma unroll
            for (int i = 4; i >= 0; i--) {
                double z = x[i];
#pragma unroll
                for (int k = i + 1; k < 6; k++) z = z - L.F[k * (k + 1) / 2 + i] * x[k];
                x[i] = z;
            }
#pragma unroll
            for (int i = 0; i < 6; i++) L.Qi[i * 6 + lane] = x[i];
        }
        WAVE_SYNC();
        auto brow = [&](int r) -> const double* { return r < 6 ? L.covL + r * 6 : L.covB + (r - 6) * 6; };
        for (int t = lane; t < kDim * 6; t += 64) {  // V = B (I6 - Q^-1)
            const int r = t / 6, c = t % 6;
            const double* b = brow(r);
            double v = b[0] * L.Qi[0 * 6 + c];
#pragma unroll
            for (int k = 1; k < 6; k++) v = v + b[k] * L.Qi[k * 6 + c];
            L.V[t] = b[c] - v;
        }
        WAVE_SYNC();
        for (int t = lane; t < kDim * kDim; t += 64) {  // cov = P - V B^T
            const int i = t / kDim, j = t % kDim;
            const double* b = brow(j);
            double gp = L.V[i * 6 + 0] * b[0];
#pragma unroll
            for (int l = 1; l < 6; l++) gp = gp + L.V[i * 6 + l] * b[l];
            st_sc1(slot->state.cov + t, s_P[t] - gp);
        }
    } else if (stop_now) {
        for (int t = lane; t < kDim * kDim; t += 64) {
            const int i = t / kDim, j = t % kDim;
            double gp = L.G6[i * 6 + 0] * s_P[0 * kDim + j];
#pragma unroll
            for (int l = 1; l < 6; l++) gp = gp + L.G6[i * 6 + l] * s_P[l * kDim + j];
            st_sc1(slot->state.cov + t, s_P[t] - gp);
        }
    }
    SOLVE_MARK(9);
#ifdef LIVO_TAIL_PROF
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    SPH_MARK(7);
    return stop_now;
}

// ===================================================== per-point pass =====
// One point of h_share_model (laser_mapping.cpp:503-593): world point, gate,
// plane (esti_plane, or the plane cached since the last search), residual
// gates, Jacobian row and its HᵀH / HᵀL terms added to acc.
// Point i's loads, issued together (one memory round trip): the body point and,
// for an evaluation without a search, the cached plane state and plane.
struct HsPointIn {
    float4 pb, plane;
    uint8_t ps;
};
__device__ __forceinline__ HsPointIn hshare_load(const HsJob& job, int i, bool cached) {
    HsPointIn in;
    in.pb = reinterpret_cast<const float4*>(job.pts)[i];
    in.ps = cached ? job.pstate[i] : 0;
    in.plane = cached ? reinterpret_cast<const float4*>(job.plane)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    return in;
}
// One point's contribution to the h_share sums: its Jacobian row H, the
// residual term err = -pd2 and |pd2|; all zero unless the point is kept.  The
// sums' columns are formed from it where they are reduced (hs_col), so the 29
// double terms are never live in registers at once.
struct HsRow {
    double H[6];
    double err;
    float apd;
    bool keep;
};
__device__ __forceinline__ void hs_row_clear(HsRow& w) {
#pragma unroll
    for (int k = 0; k < 6; k++) w.H[k] = 0.0;
    w.err = 0.0;
    w.apd = 0.0f;
    w.keep = false;
}
// Column j (0..kRedUsed-1) of the sums for one point: 21 HTH upper-triangle
// terms (H[r] / R) * H[c], 6 HTL terms (H[r] / R) * err, |pd2|, 1.  Each is
// 0.0 + term, the value a zeroed accumulator holds after one point.
template <int J>
__device__ __forceinline__ double hs_col(const HsRow& w, double inv_r) {
    if constexpr (J < 21) {
        constexpr int r = J < 6 ? 0 : J < 11 ? 1 : J < 15 ? 2 : J < 18 ? 3 : J < 20 ? 4 : 5;
        constexpr int base = r * 6 - (r * (r - 1)) / 2;
        constexpr int c = r + (J - base);
        return w.keep ? 0.0 + (w.H[r] * inv_r) * w.H[c] : 0.0;
    } else if constexpr (J < 27) {
        return w.keep ? 0.0 + (w.H[J - 21] * inv_r) * w.err : 0.0;
    } else if constexpr (J == 27) {
        return w.keep ? 0.0 + (double)w.apd : 0.0;
    } else {
        return w.keep ? 0.0 + 1.0 : 0.0;
    }
}
// acc[j] += column j (the unfused plane pass: several points per thread)
template <int J = 0>
__device__ __forceinline__ void hs_accumulate(double (&acc)[kRedUsed], const HsRow& w, double inv_r) {
    if constexpr (J < kRedUsed) {
        if constexpr (J < 21) {
            constexpr int r = J < 6 ? 0 : J < 11 ? 1 : J < 15 ? 2 : J < 18 ? 3 : J < 20 ? 4 : 5;
            constexpr int base = r * 6 - (r * (r - 1)) / 2;
            constexpr int c = r + (J - base);
            if (w.keep) acc[J] += (w.H[r] * inv_r) * w.H[c];
        } else if constexpr (J < 27) {
            if (w.keep) acc[J] += (w.H[J - 21] * inv_r) * w.err;
        } else if constexpr (J == 27) {
            if (w.keep) acc[J] += (double)w.apd;
        } else {
            if (w.keep) acc[J] += 1.0;
        }
        hs_accumulate<J + 1>(acc, w, inv_r);
    }
}
// The plane of point i from its 5 neighbours (x, y, z, sqdist) and their
// count, after a search or (search = 0) from the cached neighbours:
// point_selected_surf, esti_plane, and the plane state / plane cache stores.
// Returns the plane state: 0 not selected (a searched point beyond the sqdist
// gate: the next evaluation without a search fits it, as the reference does),
// 1 no plane (fewer than 5 neighbours, :525, or esti_plane false), 2 plane.
__device__ __forceinline__ uint8_t fit_plane(const HsParams& P, const HsJob& job, int i, int search,
                                             const float4 (&nb)[kNN], int cnt, float4& plane) {
    float nx[kNN], ny[kNN], nz[kNN];
#pragma unroll
    for (int k = 0; k < kNN; k++) { nx[k] = nb[k].x; ny[k] = nb[k].y; nz[k] = nb[k].z; }
    const float d4 = nb[kNN - 1].w;
    // point_selected_surf: sqdis[4] > 5 => false after a search (:518); true otherwise (:490)
    const bool sel = search ? ((cnt == kNN) && !(d4 > P.max_sqd)) : true;
    uint8_t ps = 0;
    float pa[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    bool plane_ok = false;
    if (cnt < kNN) {
        ps = 1;  // points_near.size() < 5 (:525) until the next search
    } else if (sel) {
        plane_ok = esti_plane(nx, ny, nz, P.plane_thr, pa);
        ps = plane_ok ? 2 : 1;
    }
    job.pstate[i] = ps;
    plane = make_float4(pa[0], pa[1], pa[2], pa[3]);
    if (plane_ok) reinterpret_cast<float4*>(job.plane)[i] = plane;
    return ps;
}

// St: livo_state or a staged StateHead (only rot and pos are read).  A plane
// fitted here (plane state 0) also updates `in`, the caller's copy of the cache.
template <class St, bool NOFIT = false>
__device__ __forceinline__ void hshare_point(const HsParams& P, const HsJob& job, const St& S, int i,
                                             int search, HsRow& w, HsPointIn& in, bool prefit = false) {
            const float4 pb = in.pb;
            const double* R = S.rot;
            float wx, wy, wz;
            world_point(R, S.pos, P.R_LI, P.t_LI, pb.x, pb.y, pb.z, wx, wy, wz);
            if (P.dbg.world) {
                P.dbg.world[3 * i + 0] = wx;
                P.dbg.world[3 * i + 1] = wy;
                P.dbg.world[3 * i + 2] = wz;
            }
            // esti_plane depends only on the 5 cached neighbours (Nearest_Points),
            // so an evaluation without a search refits exactly the plane of the
            // last one: the plane is kept per point (job.plane / job.pstate:
            // 0 not fitted yet, 1 no plane, 2 plane) and reused bit for bit.
            bool plane_ok = false;
            float pa[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            // prefit: the fused search already fitted this evaluation's plane
            // from its neighbours in registers (in.ps / in.plane, fit_plane)
            uint8_t ps = (search && !prefit) ? 0 : in.ps;
            if (!NOFIT && ps == 0 && !prefit) {  // (NOFIT: the caller fitted every plane state 0 beforehand)
                const float4* rec = reinterpret_cast<const float4*>(job.nn + i);
                float4 nb[kNN];
    #pragma unroll
                for (int k = 0; k < kNN; k++) nb[k] = rec[k];
                const int cnt = reinterpret_cast<const int4*>(job.nn + i)[6].y;
                float4 pl;
                ps = fit_plane(P, job, i, search, nb, cnt, pl);
                plane_ok = ps == 2;
                pa[0] = pl.x; pa[1] = pl.y; pa[2] = pl.z; pa[3] = pl.w;
                in.ps = ps;
                in.plane = pl;
            } else if (ps == 2) {
                const float4 v = in.plane;
                pa[0] = v.x; pa[1] = v.y; pa[2] = v.z; pa[3] = v.w;
                plane_ok = true;
            }
            bool accepted = false, keep = false;
            float pd2 = 0.0f;
            if (plane_ok) {
                pd2 = ((pa[0] * wx + pa[1] * wy) + pa[2] * wz) + pa[3];
                const double bx = pb.x, by = pb.y, bz = pb.z;
                const double bn = sqrt((bx * bx + by * by) + bz * bz);
                const float s = (float)(1 - 0.9 * (double)fabsf(pd2) / sqrt(bn));
                accepted = (double)s > 0.9;                          // :535-542
                keep = accepted && (double)fabsf(pd2) <= P.max_res;  // :552
            }
            if (P.dbg.normvec)
                reinterpret_cast<float4*>(P.dbg.normvec)[i] =
                    accepted ? make_float4(pa[0], pa[1], pa[2], pd2) : make_float4(0.f, 0.f, 0.f, 0.f);
            if (P.dbg.sel) P.dbg.sel[i] = keep ? 1 : 0;
            if (keep) {
                // Jacobian row (laser_mapping.cpp:564-593): p_I = R_LI p_b + t_LI;
                // A = [p_I]x * rot^T * n;  Hsub = [A, n]
                const double bx = pb.x, by = pb.y, bz = pb.z;
                const double* RL = P.R_LI;
                const double ix = ((RL[0] * bx + RL[1] * by) + RL[2] * bz) + P.t_LI[0];
                const double iy = ((RL[3] * bx + RL[4] * by) + RL[5] * bz) + P.t_LI[1];
                const double iz = ((RL[6] * bx + RL[7] * by) + RL[8] * bz) + P.t_LI[2];
                const double cr[9] = {0.0, -iz, iy, iz, 0.0, -ix, -iy, ix, 0.0};
                double M[9];
    #pragma unroll
                for (int r = 0; r < 3; r++)
    #pragma unroll
                    for (int cI = 0; cI < 3; cI++)
                        M[r * 3 + cI] = (cr[r * 3 + 0] * R[cI * 3 + 0] + cr[r * 3 + 1] * R[cI * 3 + 1]) +
                                        cr[r * 3 + 2] * R[cI * 3 + 2];
                const double n0 = pa[0], n1 = pa[1], n2 = pa[2];
                double H[6];
                H[0] = (M[0] * n0 + M[1] * n1) + M[2] * n2;
                H[1] = (M[3] * n0 + M[4] * n1) + M[5] * n2;
                H[2] = (M[6] * n0 + M[7] * n1) + M[8] * n2;
                H[3] = n0; H[4] = n1; H[5] = n2;
#pragma unroll
                for (int r = 0; r < 6; r++) w.H[r] = H[r];
                w.err = -(double)pd2;
                w.apd = fabsf(pd2);
                w.keep = true;
            }
}

// Block partials of a scan's h_share sums -> the last block of the scan
// reduces every partial in a fixed order and (P.solve) its wave 0 runs the
// scan's solve.  nblk = blocks of the scan in this launch, NT threads.
constexpr int kRedRows = kEvalBlock > 256 ? kEvalBlock / 16 : 16;  // 16-lane rows of the largest block
struct HsReduceLds {
    double red[kRedRows * kRedCols];      // one partial per 16-lane row
    double fin[kRedRows / 2 * kRedCols];  // the last block: one sum per 32-thread group
    int last, last2;                      // this block completed its shard / the scan
};
// NU = kRedUsed + 2 (the fused evaluation): columns 29 / 30 carry the search's
// hash-slot and map-point counts (integers, exact in double), reduced with the
// sums instead of per-wave device atomics on two addresses per scan (those
// serialise across the XCDs); the last block adds them to slot->visits /
// scanned of this evaluation.
// col(std::integral_constant<int, j>) gives this thread's value of column j;
// the block partials per 16-lane row:
// a reduce-scatter butterfly over the 16 lanes of a row: each of 4 DPP exchange stages (row_mirror, row_half_mirror, two quad
// permutations: symmetric pairings of lanes that hold the same columns) halves
// the columns a lane holds and adds its partner's half, so a row's 32 columns
// cost 16 + 8 + 4 + 2 exchanges and adds instead of 4 per column; lane l of a
// row ends with columns base(l) + {0, 1}.
template <int CTRL>
__device__ __forceinline__ void bfly_stage(double* x, int m, bool low) {
    // x[0..2m): a low lane keeps x[0..m) and sends x[m..2m); a high lane the other way
#pragma unroll
    for (int j = 0; j < m; j++) {
        const double send = low ? x[m + j] : x[j];
        const double keep = low ? x[j] : x[m + j];
        x[j] = keep + dpp_f64<CTRL>(send);
    }
}
template <int NU, class Col, int... J>
__device__ __forceinline__ void hs_row_sums_bfly(const Col& col, HsReduceLds& R, int tid,
                                                 std::integer_sequence<int, J...>) {
    static_assert(NU <= 32, "32 columns per row");
    double x[32];
    auto get = [&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        if constexpr (j < NU) x[j] = col(jc);
        else x[j] = 0.0;
    };
    (get(std::integral_constant<int, J>{}), ...);
    const int l = tid & 15;
    // partners hold the same columns at every stage: l <-> 15 - l, then 7 - l within
    // each half-row, 3 - l within each quad, l ^ 1; the halves split by bits 3, 2, 1, 0
    bfly_stage<0x140>(x, 16, (l & 8) == 0);  // row_mirror
    bfly_stage<0x141>(x, 8, (l & 4) == 0);   // row_half_mirror
    bfly_stage<0x1B>(x, 4, (l & 2) == 0);    // quad_perm [3,2,1,0]
    bfly_stage<0xB1>(x, 2, (l & 1) == 0);    // quad_perm [1,0,3,2]
    const int base = ((l & 8) ? 16 : 0) + ((l & 4) ? 8 : 0) + ((l & 2) ? 4 : 0) + ((l & 1) ? 2 : 0);
    if (base < NU) R.red[(tid >> 4) * kRedCols + base] = x[0];
    if (base + 1 < NU) R.red[(tid >> 4) * kRedCols + base + 1] = x[1];
}

#ifdef LIVO_TAIL_PROF  // the reduction's phases (tools/eval_prof.py; compiled out of the product)
// [kind][k]: 0 blocks, 1 butterfly + partial store + ticket (every block), 2 last block: the
// partials' reduction, 3 solve, 4 host slot write, 5 last blocks
__device__ unsigned long long g_tail_prof[3][8];
#define TAIL_MARK(k, t)                                                                                 \
    do {                                                                                               \
        if (pk >= 0 && threadIdx.x == 0) {                                                             \
            const unsigned long long now_ = __builtin_amdgcn_s_memtime();                             \
            atomicAdd(&g_tail_prof[pk][(k)], now_ - (t));                                              \
            (t) = now_;                                                                                \
        }                                                                                              \
    } while (0)
#else
#define TAIL_MARK(k, t) do { } while (0)
#endif
#ifndef LIVO_SOLVE_PRIO
#define LIVO_SOLVE_PRIO 1
#endif
#ifndef LIVO_RED_INFLIGHT
#define LIVO_RED_INFLIGHT 32
#endif
constexpr int kRedInFlight = LIVO_RED_INFLIGHT;  // partial loads in flight per thread of the last block
// The scan's slot into the host-mapped staging copy, by threads t of nt: read
// back past the L1 (sc1: this CU's other waves stored it, drained to L2).
__device__ __forceinline__ void hs_host_slot(const HsJob& job, const IekfSlot* slot, int t, int nt) {
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(slot);
    for (int w = t; w < (int)((kSlotWbBytes + 15) / 16); w += nt) {
        const unsigned long long lo = __hip_atomic_load(gptr(src + 2 * w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long hi = __hip_atomic_load(gptr(src + 2 * w + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        job.host_slot[w] = make_uint4((unsigned)lo, (unsigned)(lo >> 32), (unsigned)hi, (unsigned)(hi >> 32));
    }
}

// The block partial of one 256-point chunk (blk): the row butterflies into R.red,
// then wave 0's fixed pairwise tree over the rows, stored write-through (sc1).
// Ends with wave 0's stores issued; a caller that reuses R.red must barrier first.
template <int NT, int NU, class Col>
__device__ __forceinline__ void hs_block_partial(const HsJob& job, const Col& col, unsigned blk, HsReduceLds& R) {
    const int tid = threadIdx.x;
    constexpr int NR = NT / 16;  // 16-lane rows of the block
    static_assert(NR <= kRedRows, "HsReduceLds row partials");
    constexpr int NRM = NR > 16 ? NR : 16;  // rows of the fixed pairwise tree (16 for NT <= 256)
    // (21.0k vs 20.2k updates/s over row_sum16 per column, evaluations without a
    // search 0.107 vs 0.116 ms per step: profiles/r03_ab_bfly.txt)
    hs_row_sums_bfly<NU>(col, R, tid, std::make_integer_sequence<int, 32>{});
    __syncthreads();
    if (tid < NU) {
        double r[NRM];
#pragma unroll
        for (int w = 0; w < NRM; w++) r[w] = w < NR ? R.red[w * kRedCols + tid] : 0.0;
#pragma unroll
        for (int h = NRM / 2; h >= 1; h >>= 1)  // fixed pairwise tree
#pragma unroll
            for (int w = 0; w < h; w++) r[w] = r[w] + r[w + h];
        const double v = r[0];
        __hip_atomic_store(gptr(job.partial + (size_t)blk * kRedCols + tid), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int NT, int NU>
__device__ __forceinline__ void hs_scan_tail(const HsParams& P, const HsJob& job, IekfSlot* slot, int nblk,
                                             HsReduceLds& R, SolveLds& L, int pk
#ifdef LIVO_TAIL_PROF
                                             , unsigned long long tp
#endif
);

// Block partials of a scan's h_share sums -> a two-level fixed-order reduction
// -> (P.solve) the scan's solve.  nblk = partials (256-point chunks) of the scan
// in this launch; this block has stored partial `blk` (hs_block_partial).
//
// Level 1: partial b belongs to shard b % K (K = min(kRedShards, nblk)); each
// shard has a ticket of its own (a 128-B line of the slot), so ~nblk / K blocks
// contend per counter instead of every block of the scan on one (a device-scope
// atomic serialises per line: ~12 ns each, 391 arrivals ~4.7 us,
// MI355X_MICROARCH.md fan-in).  The block that completes a shard sums its
// partials (~nblk / K rows, all loads in flight at once: ~6 per thread) in a
// fixed order into row s of the partial buffer.  Level 2: that block takes the
// scan's ticket; the last of the K reduces rows 0..K-1 and solves (hs_scan_tail).
// The scan's last block thus reads K rows instead of every partial (~97 KB at
// 100k points), and the per-shard work runs on K CUs at once.  Every hand-off
// is sc1 stores drained by s_waitcnt vmcnt(0) before an agent-scope atomic, and
// sc1 loads after it (MI355X_MICROARCH.md, Workgroup dispatch: sc1 hand-off).
// The sums' order depends only on nblk, not on arrival order: deterministic.
// Level 1 of the reduction: the shard ticket, and in the block that completes
// the shard the sum of its partials into row sh (drained before return, the
// shard's ticket reset).  Returns true in that block only (block-uniform).
template <int NT, int NU = kRedUsed>
__device__ __forceinline__ bool hs_shard_level(const HsJob& job, IekfSlot* slot, int nblk, unsigned blk,
                                               HsReduceLds& R) {
    static_assert(NU == kRedUsed || NU == kRedUsed + 2, "h_share sums (+ search counts)");
    static_assert(NT / 32 <= kRedRows / 2, "R.fin holds one row per 32-thread group");
    const int tid = threadIdx.x;
    const int K = nblk < kRedShards ? nblk : kRedShards;
    const int sh = (int)(blk % (unsigned)K);
    const int cnt = (nblk - sh + K - 1) / K;  // partials of shard sh: sh, sh + K, ...
    unsigned* const sh_ticket = slot->sh_ticket + 32 * sh;
    // wave 0 stored the partial write-through; once drained, the shard's ticket
    if (tid < 64) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0)
            R.last = __hip_atomic_fetch_add(gptr(sh_ticket), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                     (unsigned)cnt - 1u;
    }
    __syncthreads();
    if (!R.last) return false;
    if (cnt > 1) {
        // thread (g, c) sums rows sh + K (g + G t), t = 0, 1, ... of column c in that
        // order, every load in flight at once (G = NT / 32 groups)
        constexpr int G = NT / 32;
        constexpr int kMaxPer = 8;  // loads per thread per round (nblk <= 8 G K in one round)
        const int c = tid & 31, g = tid >> 5;
        double acc = 0.0;
        if (c < NU) {
            const double* src = job.partial + c;
            for (int j0 = g; j0 < cnt; j0 += kMaxPer * G) {
                double v[kMaxPer];
#pragma unroll
                for (int k = 0; k < kMaxPer; k++) {
                    const int j = j0 + G * k;
                    v[k] = j < cnt ? ld_sc1(src + (size_t)(sh + K * j) * kRedCols) : 0.0;
                }
#pragma unroll
                for (int k = 0; k < kMaxPer; k++) acc += v[k];
            }
        }
        R.fin[g * kRedCols + c] = acc;
        __syncthreads();
        if (tid < NU) {
            constexpr int NG = G > 8 ? G : 8;
            double f[NG];
#pragma unroll
            for (int q = 0; q < NG; q++) f[q] = q < G ? R.fin[q * kRedCols + tid] : 0.0;
#pragma unroll
            for (int h = NG / 2; h >= 1; h >>= 1)  // ((f0 + f1) + (f2 + f3)) + ...
#pragma unroll
                for (int q = 0; q < h; q++) f[q] = f[2 * q] + f[2 * q + 1];
            st_sc1(job.partial + (size_t)sh * kRedCols + tid, f[0]);  // row sh: the shard's sum
        }
    }
    if (tid < 64) {
        if (tid == 0) st_sc1(sh_ticket, 0u);  // ready for the next pass
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the shard's row drained
    }
    return true;
}

template <int NT, int NU = kRedUsed>
__device__ __forceinline__ void hs_ticket_tail(const HsParams& P, const HsJob& job, IekfSlot* slot, int nblk,
                                               unsigned blk, HsReduceLds& R, SolveLds& L, int pk = -1) {
    const int tid = threadIdx.x;
#ifdef LIVO_TAIL_PROF
    unsigned long long tp = __builtin_amdgcn_s_memtime();
    if (pk >= 0 && tid == 0) atomicAdd(&g_tail_prof[pk][0], 1ull);
#else
    (void)pk;
#endif
    if (!hs_shard_level<NT, NU>(job, slot, nblk, blk, R)) return;
    TAIL_MARK(1, tp);
    const int K = nblk < kRedShards ? nblk : kRedShards;
    // the shard's row drained: the scan's ticket
    if (tid == 0)
        R.last2 = __hip_atomic_fetch_add(gptr(&slot->hs_ticket), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                  (unsigned)K - 1u;
    __syncthreads();
    if (!R.last2) return;
#ifdef LIVO_TAIL_PROF
    hs_scan_tail<NT, NU>(P, job, slot, K, R, L, pk, tp);
#else
    hs_scan_tail<NT, NU>(P, job, slot, K, R, L, pk);
#endif
}

// The scan's tail once every partial of it is stored: the fixed-order reduction,
// then (P.solve) wave 0's solve and the host slot copy of a stopping solve.
template <int NT, int NU>
__device__ __forceinline__ void hs_scan_tail(const HsParams& P, const HsJob& job, IekfSlot* slot, int nblk,
                                             HsReduceLds& R, SolveLds& L, int pk
#ifdef LIVO_TAIL_PROF
                                             , unsigned long long tp
#endif
) {
    const int tid = threadIdx.x;
#if LIVO_SOLVE_PRIO
    // the scan's serial tail (reduction, solve) ahead of the other waves on its SIMDs
    __builtin_amdgcn_s_setprio(3);
#endif
#ifdef LIVO_TAIL_PROF
    if (pk >= 0 && tid == 0) atomicAdd(&g_tail_prof[pk][5], 1ull);
#endif
    const bool solve = P.solve != 0;  // (kernel parameter: uniform)
    // the solve's inputs go out first, in the same round trip as the partials
    if (solve) solve_stage(slot, L, tid, NT);
    {
        // thread (g, c) sums blocks g, g+G, ... of column c in that order, kRedInFlight
        // loads in flight (G = NT / 32 groups)
        constexpr int G = NT / 32;
        const int c = tid & 31, g = tid >> 5;
        double acc = 0.0;
        if (c < NU) {
            double* src = job.partial + c;
            for (int b0 = g; b0 < nblk; b0 += kRedInFlight * G) {
                double v[kRedInFlight];
#pragma unroll
                for (int k = 0; k < kRedInFlight; k++) {
                    const int b = b0 + G * k;
                    v[k] = b < nblk ? ld_sc1(src + (size_t)b * kRedCols) : 0.0;
                }
#pragma unroll
                for (int k = 0; k < kRedInFlight; k++) acc += v[k];
            }
        }
        R.fin[g * kRedCols + c] = acc;
    }
    __syncthreads();  // the block partials' sums and the staged inputs
    const bool wb = solve && job.host_slot != nullptr;  // (uniform) the stopping solve writes the host's slot
    if (tid >= 64) {
        // vec = state_propagat - state beside wave 0's M and LU; then the one barrier
        // solve_scan<true> waits at before it uses vec
        if (solve && tid == 64) state_minus_d(L.pr, L.st, L.vec);
        if (solve) __syncthreads();
        if (wb) {
            __syncthreads();  // wave 0's solve and its slot stores are done
            if (L.ctrl.stop) hs_host_slot(job, slot, tid, NT);
        }
        return;
    }
    TAIL_MARK(2, tp);
    if (tid < kRedCols) {
        double v = 0.0;
        if (tid < NU) {
            constexpr int NG = NT / 32 > 8 ? NT / 32 : 8;
            double f[NG];
#pragma unroll
            for (int g = 0; g < NG; g++) f[g] = g < NT / 32 ? R.fin[g * kRedCols + tid] : 0.0;
#pragma unroll
            for (int h = NG / 2; h >= 1; h >>= 1)  // ((f0 + f1) + (f2 + f3)) + ... for NG = 8
#pragma unroll
                for (int g = 0; g < h; g++) f[g] = f[2 * g] + f[2 * g + 1];
            v = f[0];
        }
        if (NU > kRedUsed && tid >= kRedUsed) {
            if (tid < NU && v > 0.0) {
                int e = solve ? L.ctrl.n_evals : slot->ctrl.n_evals;
                e = e < LIVO_MAX_EVALS ? e : LIVO_MAX_EVALS - 1;
                // (no return value: the wave does not wait for it)
                atomicAdd((tid == kRedUsed ? slot->visits : slot->scanned) + e, (unsigned long long)v);
            }
            v = 0.0;
        }
        L.sum[tid] = v;
        slot->red[tid] = v;
    }
    if (tid == 0) st_sc1(&slot->hs_ticket, 0u);  // ready for the next pass (atomics see it)
    if (!solve) return;  // livo_h_share: the sums only
    WAVE_SYNC();
    solve_scan<true>(slot, L, tid, pk);
    TAIL_MARK(3, tp);
    if (wb) {
        // the solve that stops the scan writes its slot straight into the host's
        // staging copy (no copy back after the batch's last evaluation), the
        // whole block sharing it: wave 0's slot stores drained to L2 first
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (L.ctrl.stop) hs_host_slot(job, slot, tid, NT);
    }
#ifdef LIVO_TAIL_PROF
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    TAIL_MARK(4, tp);
}

// One chunk per block: its partial, then the ticket and the tail.
template <int NT, int NU = kRedUsed, class Col>
__device__ __forceinline__ void hshare_reduce_solve(const HsParams& P, const HsJob& job, IekfSlot* slot,
                                                    const Col& col, int nblk, unsigned blk, HsReduceLds& R,
                                                    SolveLds& L, int pk = -1) {
    hs_block_partial<NT, NU>(job, col, blk, R);
    hs_ticket_tail<NT, NU>(P, job, slot, nblk, blk, R, L, pk);
}

template <bool FIRST>
__global__ __launch_bounds__(kBlock) void k_hshare(HsParams P) {
    __shared__ HsReduceLds R;
    __shared__ SolveLds L;
    const HsJob job = P.jobs[blockIdx.y];
    // the k-NN replay of this evaluation has run (stream order): reset its count
    if (P.replay_count && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *P.replay_count = 0u;
    if (P.replay_count2 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *P.replay_count2 = 0u;
    if ((int)blockIdx.x >= job.nblk) return;
    IekfSlot* slot = job.slot;
    int search;
    if (P.force >= 0) {
        search = P.force;
    } else {
        if (slot->ctrl.stop) return;  // block-uniform
        search = FIRST ? 1 : slot->ctrl.search_en;
    }
    const livo_state& S = slot->state;
    double acc[kRedUsed];
#pragma unroll
    for (int j = 0; j < kRedUsed; j++) acc[j] = 0.0;
    for (int rep = 0; rep < kPtsPerThread; rep++) {  // points of this block: strided for coalescing
        const int i = (blockIdx.x * kPtsPerThread + rep) * kBlock + threadIdx.x;
        if (i < job.n) {
            HsRow w;
            hs_row_clear(w);
            HsPointIn in = hshare_load(job, i, !search);
            hshare_point(P, job, S, i, search, w, in);
            hs_accumulate(acc, w, P.inv_r);
        }
    }
    hshare_reduce_solve<kBlock>(P, job, slot, [&](auto jc) { return acc[decltype(jc)::value]; }, job.nblk,
                                blockIdx.x, R, L);
}

// ================================================ fused evaluation =======
// k_iekf_eval<FIRST>: one evaluation of the IEKF loop (laser_mapping.cpp:
// 178-237) for every point of a batch of scans in ONE launch per stream group.
// Each 256-thread block takes 256 Morton-consecutive points of one scan:
//   - if the evaluation searches (the first one, or nearest_search_en set by
//     the previous solve): the LDS-tiled cell-grid k-NN of its points (one
//     block-wide tile of the box of cells within one cell of any of them),
//     seeded by the previous neighbours after the first evaluation; the rare
//     queries whose answer depends on the reference's tie order are recomputed
//     in place by the same thread (knn_exact on the ikd-Tree records, or the
//     canonical order on an incremental map);
//   - the plane fit / residual / Jacobian of each point (hshare_point);
//   - block partials, and the scan's last block reduces them and runs the solve.
// Evaluations of a stopped scan exit at the first instruction.  Replaces the
// k-NN launch, the replay launch and the plane-pass launch of each
// evaluation; answers identical to those kernels.
#ifndef LIVO_EVAL_TILE_CELLS
#define LIVO_EVAL_TILE_CELLS 256
#endif
#ifndef LIVO_EVAL_TILE_PTS
#define LIVO_EVAL_TILE_PTS 1024
#endif
using BlockTile = TileLds<LIVO_EVAL_TILE_CELLS, LIVO_EVAL_TILE_PTS>;

// The flagged queries of one wave (amb), each replayed by the whole wave
// (knn_exact_wave) with `cache` (4 KB of LDS) as its subtree cache.
__device__ __forceinline__ void replay_wave(const KnnParams& P, const HsJob& job, int i, bool amb, float4* cache,
                                            const PoseRef& pose) {
    unsigned long long m = __ballot(amb);
    const int lane = (int)(threadIdx.x & 63u);
    while (m) {  // wave-uniform
        const int l = __ffsll((long long)m) - 1;
        m &= m - 1ull;
        const int il = __shfl(i, l);
        float qx, qy, qz;
        query_point(P, pose, reinterpret_cast<const float4*>(job.pts)[il], qx, qy, qz);
        Cands c;
        knn_exact_wave(P.nodes, P.n_nodes, P.has_map, qx, qy, qz, cache, c);
        if (lane == l) {
            float od[kNN];
            uint32_t on[kNN];
#pragma unroll
            for (int k = 0; k < kNN; k++) { od[k] = c.d[k]; on[k] = c.node[k]; }
            write_nnrec(job.nn + il, P.nodes, c.n, od, on, job.nn[il].flag | 0x100);
        }
    }
}

struct EvalParams {
    KnnParams k;
    HsParams h;
};

#ifdef LIVO_EVAL_PROF  // per-phase block time of k_iekf_eval (tools/eval_prof.py; compiled out of the product)
// [search][phase]: cycles summed over blocks (thread 0's s_memtime deltas) and block counts
__device__ unsigned long long g_eval_prof[3][8];  // [no search / rematch / first search][phase]
// [kind][stat]: lanes, ball-certified, cell-run lanes, ball entries (sum, wave max), cell entries (sum, wave max), waves
__device__ unsigned long long g_eval_stats[3][8];
#define EVAL_MARK(k)                                                                                   \
    do {                                                                                               \
        if (threadIdx.x == 0) {                                                                        \
            const unsigned long long now = __builtin_amdgcn_s_memtime();                              \
            if ((k) > 0) atomicAdd(&g_eval_prof[FIRST ? 2 : (search ? 1 : 0)][(k)], now - prof_t);     \
            else atomicAdd(&g_eval_prof[FIRST ? 2 : (search ? 1 : 0)][0], 1ull);       \
            prof_t = now;                                                                              \
        }                                                                                              \
    } while (0)
#define EVAL_MARK_SYNC(k) do { __syncthreads(); EVAL_MARK(k); } while (0)
// block timeline of the last batch: [evaluation][block] = (start, end) s_memtime of thread 0
constexpr int kTlBlocks = 4096;
__device__ unsigned long long g_eval_tl[LIVO_MAX_EVALS][kTlBlocks][2];
#define EVAL_PROF_DECL unsigned long long prof_t = 0
#else
#define EVAL_MARK(k) do { } while (0)
#define EVAL_MARK_SYNC(k) do { } while (0)
#define EVAL_PROF_DECL do { } while (0)
#endif
#ifndef LIVO_EVAL_WAVES
#define LIVO_EVAL_WAVES 4  // waves per SIMD the VGPR budget must allow (<= 128 VGPRs)
#endif
template <bool FIRST>
__global__ __launch_bounds__(kEvalBlock, LIVO_EVAL_WAVES) void k_iekf_eval(EvalParams E) {
    const KnnParams& P = E.k;
    EVAL_PROF_DECL;
#ifdef LIVO_EVAL_PROF
    const unsigned long long tl_start = __builtin_amdgcn_s_memtime();
#endif
    // the search's LDS is dead (block barrier) before the reduction and solve use theirs
    __shared__ union {
        BlockTile tile;  // the cell walk's block tile (no vertex runs: an incremental map)
        struct {
            HsReduceLds R;
            SolveLds solve;  // the scan's last block solves after its search is done
        } rs;
        float4 nnstage[kEvalBlock / 64][64 * 8];  // each wave's 64 neighbour records (the run searches)
    } U;
    unsigned bjob, bx;
    // the same block order in every evaluation: the plane caches stay in the L2 that wrote them
    xcd_chunk_block(P.nb, P.xcd_chunk, bjob, bx);
    const HsJob job = P.jobs[bjob];
    IekfSlot* slot = job.slot;
    if (bx > 0 && (int)bx * kEvalBlock >= job.n) return;  // (an empty scan keeps one block: it solves)
    const int i = (int)bx * kEvalBlock + threadIdx.x;
    const bool valid = i < job.n;
    // the point's loads go out with the slot's control reads (after the first
    // evaluation the plane cache too: used unless this evaluation searches)
    HsPointIn pin = valid ? hshare_load(job, i, !FIRST) : HsPointIn{};
    bool prefit = false;  // the plane of this evaluation fitted in the search branch
    if (slot->ctrl.stop) return;  // block-uniform
    const int search = FIRST ? 1 : slot->ctrl.search_en;
    const PoseRef pose{slot->state.rot, slot->state.pos};
#ifdef LIVO_EVAL_PROF
    const int tl_e = min(slot->ctrl.n_evals, LIVO_MAX_EVALS - 1);
#endif
    EVAL_MARK(0);
    unsigned n_slots = 0u, n_pts = 0u;  // hash slots and map points this thread's search read
    if (search) {
        // Later searches start unseeded too: the previous neighbours' bound saved
        // less than reading their record cost (rematch 0.156 vs 0.159 ms, 18991 vs
        // 18643 updates/s, profiles/r03_ab_prefit_seed.txt); the answer is the
        // same exact list either way
        LeafQuery q;
        lq_init<false>(q, P, pose, job, i, valid);
        int c0 = 0, c1 = 0, c2 = 0, s0 = 1, s1 = 1, s2 = 1;
        if (valid) grid_cell(P, q, c0, c1, c2, s0, s1, s2);
        unsigned visits = 0, npts = 0;
        bool amb = false;
        if (P.vslots) {  // (kernel parameter: uniform)
            EVAL_MARK(1);
            bool certified = false;
            const float4* runs = reinterpret_cast<const float4*>(P.vpts);  // (float4 run entries only)
#ifdef LIVO_EVAL_PROF
            const unsigned np0 = npts;
            bool ball_ok = false;
#endif
#if LIVO_IDX_RUNS
            const bool dyn = P.dyn_runs != 0;  // (uniform) runs on the incremental map
#else
            constexpr bool dyn = false;
#endif
            if (P.bslots) {  // (uniform) the ball runs first; the cell runs for a query they do not certify
                certified = dyn ? brun_search<true>(q, P, valid, visits, npts) : brun_search<false>(q, P, valid, visits, npts);
                if (certified) runs = reinterpret_cast<const float4*>(P.bpts);  // (float4 run entries only)
                if (valid && !certified) lq_init<false>(q, P, pose, job, i, valid);
#ifdef LIVO_EVAL_PROF
                ball_ok = certified;
#endif
            }
#ifdef LIVO_EVAL_PROF
            const unsigned np1 = npts;
#endif
            if (!certified)
                certified = dyn ? vrun_search<true>(q, P, valid, c0, c1, c2, s0, s1, s2, visits, npts)
                                : vrun_search<false>(q, P, valid, c0, c1, c2, s0, s1, s2, visits, npts);
            // the incremental map's points added since its runs (none: no delta grid): the
            // cube's delta run; the list is exact if the base was and its ball lies in the cube
#if LIVO_IDX_RUNS
            if (dyn && valid && P.dvslots) {
                dvrun_scan(q, P, c0, c1, c2, visits, npts);
                certified = certified && cube_inside(q, P, c0, c1, c2);
            } else if (dyn && valid && certified && P.dslots) {
                certified = delta_search(q, P, visits, npts);
            }
#endif
            // (a query the runs leave uncertified: vrun_search's serial walk beyond the cube; a
            // wave-parallel walk of one query's cells was slower)
            bool walked = false;
            if (dyn && valid && !certified) {  // the incremental map: the current grid's serial walk
                lq_init<false>(q, P, pose, job, i, valid);
                TileView none;
                certified = grid_search(q, P, c0, c1, c2, s0, s1, s2, none, visits, npts);
                walked = true;
            }
#ifdef LIVO_EVAL_PROF
            {  // block totals: lanes past the 2x2x2 block, run entries scanned, ambiguous
                const unsigned long long nf = __ballot(valid && !certified);
                if ((threadIdx.x & 63) == 0) {
                    atomicAdd(&g_eval_prof[FIRST ? 2 : 1][7], (unsigned long long)__popcll(nf));
                }
                // search statistics per evaluation kind: lanes, ball-certified lanes,
                // entries scanned in the ball / cell stage (sum over lanes and the
                // per-wave maximum: the wave runs its slowest lane's chunks)
                const unsigned nb = valid ? np1 - np0 : 0u, nc = valid ? npts - np1 : 0u;
                unsigned mb = nb, mc = nc, sb = nb, sc = nc;
                for (int o = 1; o < 64; o <<= 1) {
                    mb = max(mb, (unsigned)__shfl_xor((int)mb, o));
                    mc = max(mc, (unsigned)__shfl_xor((int)mc, o));
                    sb += (unsigned)__shfl_xor((int)sb, o);
                    sc += (unsigned)__shfl_xor((int)sc, o);
                }
                const unsigned long long nv = __ballot(valid), nbo = __ballot(valid && ball_ok);
                const unsigned long long ncr = __ballot(valid && !ball_ok && nc > 0);
                if ((threadIdx.x & 63) == 0) {
                    unsigned long long* g = g_eval_stats[FIRST ? 2 : (search ? 1 : 0)];
                    atomicAdd(g + 0, (unsigned long long)__popcll(nv));
                    atomicAdd(g + 1, (unsigned long long)__popcll(nbo));
                    atomicAdd(g + 2, (unsigned long long)__popcll(ncr));
                    atomicAdd(g + 3, (unsigned long long)sb);
                    atomicAdd(g + 4, (unsigned long long)mb);
                    atomicAdd(g + 5, (unsigned long long)sc);
                    atomicAdd(g + 6, (unsigned long long)mc);
                    atomicAdd(g + 7, 1ull);
                }
            }
            EVAL_MARK(5);
#endif
            if (valid) {
                float4 nb[kNN];
                // candidates: grid positions (index runs, the cell walk), or run positions (float4 runs);
                // on the incremental map positions in its base set rpts, or kRunPos | delta positions
                float4* stage = U.nnstage[threadIdx.x >> 6];
                if (dyn)
                    amb = lq_finish<true>(q, P, job, bjob, i, reinterpret_cast<const float4*>(walked ? P.gpts : P.rpts),
                                          !certified, false, reinterpret_cast<const float4*>(P.dpts), nb, stage);
                else
                    amb = lq_finish<!LIVO_IDX_RUNS>(q, P, job, bjob, i, reinterpret_cast<const float4*>(P.gpts),
                                                    !certified, false, walked ? nullptr : runs, nb, stage);
                // the plane from the neighbours in registers (18643 vs 18011 updates/s
                // re-reading the record just written, profiles/r03_ab_prefit_seed.txt)
                if (!amb && (!P.canon || dyn)) {  // (a replayed query's plane is fitted from its record below)
                    float4 pl;
                    pin.ps = fit_plane(E.h, job, i, 1, nb, (int)min<int64_t>(P.lM, (int64_t)kNN), pl);
                    pin.plane = pl;
                    prefit = true;
                }
            }
            {
                // the wave's 64 records leave as one coalesced 8-KB run (the AoS
                // record stores put each lane's 16 B in its own 128-B line: 64
                // lines per store instruction, 8 instructions per wave)
                const int lane = threadIdx.x & 63;
                const float4* st = U.nnstage[threadIdx.x >> 6];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                const int base = i - lane;
                float4* dst = reinterpret_cast<float4*>(job.nn + base);
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int u = j * 64 + lane, rec = u >> 3;
#ifdef LIVO_AB_REC_KNOCKOUT  // A/B only (wrong records): 64 of each record's 128 B stored, to price the writes
                    if ((u & 7) >= 4) continue;
#endif
                    if (base + rec < job.n) dst[u] = st[rec * 8 + (((u & 7) + rec) & 7)];
                }
                // a flagged query's replay (same wave) reads its record back
                if (__ballot(amb)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            EVAL_MARK(6);
        } else {
            const TileView tv = build_tile<kEvalBlock>(U.tile, P, valid, c0, c1, c2, visits, npts);
            EVAL_MARK(1);
            if (valid) {
#ifdef LIVO_EVAL_PROF
                unsigned long long* sp = threadIdx.x == 0 ? g_eval_prof[FIRST ? 2 : 1] + 5 : nullptr;  // (stage slots 5-7)
#else
                unsigned long long* sp = nullptr;
#endif
                const bool certified = grid_search(q, P, c0, c1, c2, s0, s1, s2, tv, visits, npts, sp);
                amb = lq_finish(q, P, job, bjob, i, reinterpret_cast<const float4*>(P.gpts), !certified, false);
            }
        }
        n_slots = visits;
        n_pts = npts;
        if (amb) atomicAdd(P.replay_total, 1ull);
        if (P.canon) {  // (kernel parameter: uniform) the incremental map's exact resolution
            if (amb) canon_query(P, job, i, pose);
            __syncthreads();  // the tile's LDS is reused by the solve
        } else if (__syncthreads_or(amb)) {  // block-uniform: some query of this block is flagged
            // the tile's LDS is free after the barrier: 4 KB per wave of subtree cache
            static_assert(sizeof(U) >= (size_t)(kEvalBlock / 64) * (4u << kReplayLevels) * sizeof(float4),
                          "replay caches do not fit the evaluation's LDS");
            float4* cache = reinterpret_cast<float4*>(&U) + (threadIdx.x >> 6) * (4u << kReplayLevels);
            replay_wave(P, job, i, amb, cache, pose);
            __syncthreads();  // the caches' LDS is reused by the solve
        }
        EVAL_MARK(2);
    }
    HsRow w;
    hs_row_clear(w);
    const int nblk = max(1, (job.n + kEvalBlock - 1) / kEvalBlock);
    if (valid) {
        hshare_point(E.h, job, pose, i, search, w, pin, prefit);
    }
    EVAL_MARK_SYNC(3);
    const double inv_r = E.h.inv_r;
    // the sums' columns, then the search's counts (they ride in the block partials)
    auto col = [&](auto jc) -> double {
        constexpr int j = decltype(jc)::value;
        if constexpr (j < kRedUsed) return hs_col<j>(w, inv_r);
        else if constexpr (j == kRedUsed) return (double)n_slots;
        else return (double)n_pts;
    };
#ifdef LIVO_TAIL_PROF
    const int pk = FIRST ? 2 : (search ? 1 : 0);
#else
    const int pk = -1;
#endif
    hshare_reduce_solve<kEvalBlock, kRedUsed + 2>(E.h, job, slot, col, nblk, bx, U.rs.R, U.rs.solve, pk);
    EVAL_MARK(4);
#ifdef LIVO_EVAL_PROF
    if (threadIdx.x == 0 && blockIdx.x < (unsigned)kTlBlocks) {
        g_eval_tl[tl_e][blockIdx.x][0] = tl_start;
        g_eval_tl[tl_e][blockIdx.x][1] = __builtin_amdgcn_s_memtime();
    }
#endif
}

// Per-point persistent selection of the IKFoM h-model: point_selected_surf is a
// global array there (origin_laserMapping.cpp:155), so a point dropped by the
// plane test stays dropped until the next search.  NNRec.flag bit:
constexpr int kIkDrop = 0x1000;

// LDS of the IKFoM plane pass: per-rep point rows, then (last block) the solve.
struct IkSolveLds {
    double P[kIkDim * kIkDim];
    double Pinv[kIkDim * kIkDim];
    double LU[kIkDim * kIkDim];
    double L[kIkDim * kIkDim];
    double Kx[kIkDim * 12];
    double sum[kIkCols];
    double dx[kIkDim], dxn[kIkDim], dxu[kIkDim], Kh[kIkDim];
    double J[9];
    double Hm[kIkFewRows * 13];   // measurement-space branch: the m < 23 effective rows (h_x row, h)
    double Km[kIkDim * kIkFewRows];
    int piv[kIkDim];
    int m;                        // effective rows; < 23: measurement-space gain
    int stop;
};
constexpr int kIkRow = 15;  // 12 row + h + |pd2| + keep

// One wave, the part of esekfom.hpp:1638-1787 that does not depend on this
// evaluation's measurements: dx = x_ boxminus x_propagated, P_ = P_propagated
// with the SO3 / S2 corrections of dx_new and P_ (:1638-1697), and (P_ / R)^-1
// of the information-form gain (:1775-1777).  k_solve_ik runs it on its last
// wave beside the other waves' reduction of the block partials.
__device__ void ik_prep(const IekfSlot* slot, IkSolveLds& S, const int lane, const double R) {
    const IkBlock& K = slot->ik;
    constexpr int N = kIkDim;
    if (lane == 0) {
        double dx[N];
        ik_boxminus_d(K.x, K.xp, dx);  // x_.boxminus(dx, x_propagated)
        for (int k = 0; k < N; k++) S.dx[k] = S.dxn[k] = dx[k];
    }
    for (int t = lane; t < N * N; t += 64) S.P[t] = K.xp.cov[t];  // P_ = P_propagated
    WAVE_SYNC();
    SOLVE_MARK(3);
    // SO3 (idx 3, 6) and S2 (idx 21) corrections of dx_new and P_ (:1659-1697)
#pragma unroll
    for (int b = 0; b < 3; b++) {
        const int idx = b == 0 ? 3 : (b == 1 ? 6 : 21), d = b == 2 ? 2 : 3;
        if (lane == 0) {
            double J[9], o[3];
            if (b < 2) so3_J_d(S.dx + idx, J);
            else s2_J_d(K.x.grav, K.xp.grav, S.dx + 21, J);
            for (int r = 0; r < d; r++) {
                double acc = J[r * d] * S.dxn[idx];
                for (int k = 1; k < d; k++) acc = acc + J[r * d + k] * S.dxn[idx + k];
                o[r] = acc;
            }
            for (int r = 0; r < d; r++) S.dxn[idx + r] = o[r];
            for (int k = 0; k < d * d; k++) S.J[k] = J[k];
        }
        WAVE_SYNC();
        if (lane < N) {  // rows idx.. of column `lane`: J * P
            double o[3];
            for (int r = 0; r < d; r++) {
                double acc = S.J[r * d] * S.P[idx * N + lane];
                for (int k = 1; k < d; k++) acc = acc + S.J[r * d + k] * S.P[(idx + k) * N + lane];
                o[r] = acc;
            }
            for (int r = 0; r < d; r++) S.P[(idx + r) * N + lane] = o[r];
        }
        WAVE_SYNC();
        if (lane < N) {  // columns idx.. of row `lane`: P * J^T
            double o[3];
            for (int c = 0; c < d; c++) {
                double acc = S.P[lane * N + idx] * S.J[c * d];
                for (int k = 1; k < d; k++) acc = acc + S.P[lane * N + idx + k] * S.J[c * d + k];
                o[c] = acc;
            }
            for (int c = 0; c < d; c++) S.P[lane * N + idx + c] = o[c];
        }
        WAVE_SYNC();
    }
    SOLVE_MARK(4);
    {
        double A[N];
        for (int j = 0; j < N; j++) A[j] = lane < N ? S.P[lane * N + j] / R : 0.0;
        wave_lu_to_lds<N>(A, lane, S.LU, S.piv);
        WAVE_SYNC();
        if (lane < N) {
            double y[N];
            lds_lu_column<N>(S.LU, S.piv, lane, y);
            for (int i = 0; i < N; i++) S.Pinv[i * N + lane] = y[i];
        }
        WAVE_SYNC();
    }
    SOLVE_MARK(5);
}

// One wave: esekfom.hpp:1701-1921 from the reduced sums in S.sum and the
// evaluation's prep (ik_prep: S.dx, S.dxn, S.P, S.Pinv = (P_ / R)^-1).
__device__ void ik_solve(IekfSlot* slot, const HsJob& job, IkSolveLds& S, const int lane, const double R) {
    IkBlock& K = slot->ik;
    const IekfCtrl ctrl0 = slot->ctrl;
    const int e = ctrl0.n_evals;
    const int it = ctrl0.iter_count;  // i of the reference loop (starts at -1)
    constexpr int N = kIkDim;
    auto hth = [&](int r, int c) {
        const int a = r < c ? r : c, bb = r < c ? c : r;
        return S.sum[a * 12 - (a * (a - 1)) / 2 + (bb - a)];
    };
    if (S.m < kIkDim) {
        // measurement-space gain (:1701-1736) for m < 23 effective points:
        // K = P Hc^T (Hc P Hc^T / R + I)^-1 / R, K_h = K h, K_x = K Hc
        const int m = S.m;
        double* PHt = S.L;  // 23 x m (S.L is rebuilt from S.P for the covariance)
        for (int t = lane; t < N * m; t += 64) {
            const int r = t / m, j = t % m;
            double acc = S.P[r * N + 0] * S.Hm[j * 13 + 0];
            for (int k = 1; k < 12; k++) acc = acc + S.P[r * N + k] * S.Hm[j * 13 + k];
            PHt[r * m + j] = acc;
        }
        WAVE_SYNC();
        {
            // S = Hc PHt / R + I, padded with the identity to 22 x 22 (the
            // padding neither pivots nor eliminates: the m x m LU and inverse)
            double A[kIkFewRows];
            for (int bcol = 0; bcol < kIkFewRows; bcol++) {
                double v = lane == bcol ? 1.0 : 0.0;
                if (lane < m && bcol < m) {
                    double acc = S.Hm[lane * 13 + 0] * PHt[0 * m + bcol];
                    for (int k = 1; k < 12; k++) acc = acc + S.Hm[lane * 13 + k] * PHt[k * m + bcol];
                    v = acc / R + (lane == bcol ? 1.0 : 0.0);
                }
                A[bcol] = lane < kIkFewRows ? v : 0.0;
            }
            wave_lu_to_lds<kIkFewRows>(A, lane, S.LU, S.piv);
            WAVE_SYNC();
            if (lane < m) {
                double y[kIkFewRows];
                lds_lu_column<kIkFewRows>(S.LU, S.piv, lane, y);
                for (int i = 0; i < kIkFewRows; i++) S.Pinv[i * kIkFewRows + lane] = y[i];  // Sinv(i, lane)
            }
            WAVE_SYNC();
        }
        for (int t = lane; t < N * m; t += 64) {  // K = PHt Sinv / R
            const int r = t / m, j = t % m;
            double acc = PHt[r * m + 0] * S.Pinv[0 * kIkFewRows + j];
            for (int k = 1; k < m; k++) acc = acc + PHt[r * m + k] * S.Pinv[k * kIkFewRows + j];
            S.Km[r * kIkFewRows + j] = acc / R;
        }
        WAVE_SYNC();
        if (lane < N) {
            const int r = lane;
            double kh = 0.0;
            for (int j = 0; j < m; j++) kh = (j == 0) ? S.Km[r * kIkFewRows] * S.Hm[12] : kh + S.Km[r * kIkFewRows + j] * S.Hm[j * 13 + 12];
            S.Kh[r] = kh;
            for (int c = 0; c < 12; c++) {
                double acc = 0.0;
                for (int j = 0; j < m; j++) acc = (j == 0) ? S.Km[r * kIkFewRows] * S.Hm[c] : acc + S.Km[r * kIkFewRows + j] * S.Hm[j * 13 + c];
                S.Kx[r * 12 + c] = acc;
            }
        }
        WAVE_SYNC();
    } else {
    // gain, information form (:1775-1787): P_temp = (P_/R)^-1 + HTH, P_inv = P_temp^-1.
    // (The Woodbury form K(:, 0:12) = A(:, 0:12) (I12 + C A11)^-1 with A = P_ / R
    // needs one 12x12 LU instead of two 23x23 inversions, but at converged steps
    // dx = K_h + (K_x - I) dx_new cancels ~1e5-fold and shows its different
    // rounding at 4e-5 of |dx| against the reference's inversions: kept exact.)
    {
        double A[N];
        for (int t = lane; t < 144; t += 64) {
            const int r = t / 12, c = t % 12;
            const int a = r < c ? r : c, bb = r < c ? c : r;
            S.Pinv[r * N + c] += S.sum[a * 12 - (a * (a - 1)) / 2 + (bb - a)];
        }
        WAVE_SYNC();
        for (int j = 0; j < N; j++) A[j] = lane < N ? S.Pinv[lane * N + j] : 0.0;
        wave_lu_to_lds<N>(A, lane, S.LU, S.piv);
        WAVE_SYNC();
        if (lane < N) {
            double y[N];
            lds_lu_column<N>(S.LU, S.piv, lane, y);
            for (int i = 0; i < N; i++) S.Pinv[i * N + lane] = y[i];
        }
        WAVE_SYNC();
    }
    SOLVE_MARK(6);
    if (lane < N) {
        const int r = lane;
        double kh = S.Pinv[r * N] * S.sum[78];
        for (int c = 1; c < 12; c++) kh = kh + S.Pinv[r * N + c] * S.sum[78 + c];
        S.Kh[r] = kh;
        for (int c = 0; c < 12; c++) {
            double a2 = S.Pinv[r * N] * hth(0, c);
            for (int k = 1; k < 12; k++) a2 = a2 + S.Pinv[r * N + k] * hth(k, c);
            S.Kx[r * 12 + c] = a2;
        }
    }
    WAVE_SYNC();
    }
    SOLVE_MARK(7);
    if (lane < N) {  // dx_ = K_h + (K_x - I) dx_new
        const int r = lane;
        double acc = 0.0;
        for (int c = 0; c < N; c++) {
            const double kxi = (c < 12 ? S.Kx[r * 12 + c] : 0.0) - (r == c ? 1.0 : 0.0);
            acc = (c == 0) ? kxi * S.dxn[0] : acc + kxi * S.dxn[c];
        }
        S.dxu[r] = S.Kh[r] + acc;
    }
    WAVE_SYNC();
    if (lane == 0) {
        double dxu[N];
        for (int k = 0; k < N; k++) dxu[k] = S.dxu[k];
        ik_boxplus_d(K.x, dxu);
        bool converge = true;
        for (int k = 0; k < N; k++)
            if (fabs(dxu[k]) > 0.001) {
                converge = false;
                break;
            }
        int t = K.t + (converge ? 1 : 0);
        if (!t && it == ctrl0.max_iter - 2) converge = true;
        const bool stop = t > 1 || it == ctrl0.max_iter - 1;
        livo_ikfom_stats& st = K.stats;
        if (e < LIVO_MAX_EVALS) {
            st.effct_feat_num[e] = (int64_t)S.sum[91];
            st.res_mean[e] = S.sum[90] / S.sum[91];
            for (int k = 0; k < N; k++) st.dx[e][k] = dxu[k];
        }
        st.iterations = e + 1;
        st.knn_passes += ctrl0.search_en ? 1 : 0;
        st.converged = converge ? 1 : 0;
        st.t = t;
        K.t = t;
        IekfCtrl ctrl = ctrl0;
        ctrl.last_search = ctrl0.search_en;
        ctrl.search_en = converge ? 1 : 0;  // dyn_share.converge: search at the next h_dyn_share
        ctrl.converged = converge ? 1 : 0;
        ctrl.iter_count = it + 1;
        ctrl.n_evals = e + 1;
        ctrl.stop = (stop || ctrl.iter_count >= ctrl.max_iter || ctrl.n_evals >= LIVO_MAX_EVALS) ? 1 : 0;
        slot->ctrl = ctrl;
        S.stop = stop ? 1 : 0;
    }
    WAVE_SYNC();
    SOLVE_MARK(8);
    if (!S.stop) return;
    // covariance (:1838-1921): L_ = P_ with the corrections at dx_, P_ = L_ - K_x(:,0:12) P_(0:12,:)
    for (int t = lane; t < N * N; t += 64) S.L[t] = S.P[t];
    WAVE_SYNC();
#pragma unroll
    for (int b = 0; b < 3; b++) {
        const int idx = b == 0 ? 3 : (b == 1 ? 6 : 21), d = b == 2 ? 2 : 3;
        if (lane == 0) {
            double J[9];
            if (b < 2) so3_J_d(S.dxu + idx, J);
            else s2_J_d(K.x.grav, K.xp.grav, S.dxu + 21, J);
            for (int k = 0; k < d * d; k++) S.J[k] = J[k];
        }
        WAVE_SYNC();
        if (lane < N) {  // L rows idx.. = J * P rows, column `lane`
            for (int r = 0; r < d; r++) {
                double acc = S.J[r * d] * S.P[idx * N + lane];
                for (int k = 1; k < d; k++) acc = acc + S.J[r * d + k] * S.P[(idx + k) * N + lane];
                S.L[(idx + r) * N + lane] = acc;
            }
        }
        if (lane < 12) {  // K_x rows idx.. (first 12 columns), column `lane`
            double o[3];
            for (int r = 0; r < d; r++) {
                double acc = S.J[r * d] * S.Kx[idx * 12 + lane];
                for (int k = 1; k < d; k++) acc = acc + S.J[r * d + k] * S.Kx[(idx + k) * 12 + lane];
                o[r] = acc;
            }
            for (int r = 0; r < d; r++) S.Kx[(idx + r) * 12 + lane] = o[r];
        }
        WAVE_SYNC();
        if (lane < N) {  // L and P columns idx.. of row `lane`: * J^T
            double lo[3], po[3];
            for (int c = 0; c < d; c++) {
                double al = S.L[lane * N + idx] * S.J[c * d], ap = S.P[lane * N + idx] * S.J[c * d];
                for (int k = 1; k < d; k++) {
                    al = al + S.L[lane * N + idx + k] * S.J[c * d + k];
                    ap = ap + S.P[lane * N + idx + k] * S.J[c * d + k];
                }
                lo[c] = al;
                po[c] = ap;
            }
            for (int c = 0; c < d; c++) {
                S.L[lane * N + idx + c] = lo[c];
                S.P[lane * N + idx + c] = po[c];
            }
        }
        WAVE_SYNC();
    }
    for (int t = lane; t < N * N; t += 64) {
        const int r = t / N, c = t % N;
        double acc = S.Kx[r * 12] * S.P[c];
        for (int k = 1; k < 12; k++) acc = acc + S.Kx[r * 12 + k] * S.P[k * N + c];
        K.x.cov[t] = S.L[t] - acc;
    }
    SOLVE_MARK(9);
}

// Compensated (Neumaier) sum, as oracle/livo_oracle.cpp's CompSum: s + c is
// the sum to ~1e-27 relative in any order, so the block partials merged here
// round to the same doubles as the oracle's serial sum.  The IKFoM update's
// converged steps cancel ~1e5-fold (dx = K_h + (K_x - I) dx_new), which would
// show summation-order rounding of h_x^T h_x.
__device__ __forceinline__ void comp_add(double& s, double& c, double x) {
    const double t = s + x;
    c += (fabs(s) >= fabs(x)) ? (s - t) + x : (x - t) + s;
    s = t;
}

// IKFoM plane pass (origin_laserMapping.cpp:916-1048): 4 points per thread as
// k_hshare; each point's 12-wide row [n, A, B, C], h = -pd2 goes to LDS and the
// block's 92 sums (h_x^T h_x upper triangle, h_x^T h, residual sum, count) are
// formed by 92 threads over the rows in point order (k_solve_ik reduces them).
template <bool FIRST>
__global__ __launch_bounds__(kBlock) void k_hshare_ik(HsParams P) {
    __shared__ double rows[kBlock * kIkRow];
    const HsJob job = P.jobs[blockIdx.y];
    if ((int)blockIdx.x >= job.nblk) return;
    IekfSlot* slot = job.slot;
    if (slot->ctrl.stop) return;  // block-uniform
    const int search = FIRST ? 1 : slot->ctrl.search_en;
    const int tid = threadIdx.x;
    const livo_ikfom_state& X = slot->ik.x;
    // Each wave sums the rows of its own 64 points: lane l forms output l and
    // (l < 28) output l + 64 of the block's 92 sums -- (a, b) of the upper
    // triangle, or HTh / res / count -- over them, the four waves' compensated
    // sums are merged at the end (order-free to ~1e-27, comp_add).
    const int lane = tid & 63, wv = tid >> 6;
    const int o1 = lane, o2 = lane + 64;
    auto tri = [](int o, int& a, int& b) {
        int t = o, r = 0;
        while (t >= 12 - r) { t -= 12 - r; r++; }
        a = r;
        b = r + t;
    };
    int a1 = 0, b1 = 0, a2 = 0, b2 = 0;
    tri(o1, a1, b1);
    if (o2 < 78) tri(o2, a2, b2);
    double acc1 = 0.0, acc1_c = 0.0, acc2 = 0.0, acc2_c = 0.0;  // compensated
    __shared__ double wpart[kBlock / 64][2][kIkUsed];
    __shared__ uint32_t wcnt[kBlock / 64];
    uint32_t bcnt = 0;  // effective rows of this block so far (point order)
    for (int rep = 0; rep < kPtsPerThread; rep++) {
        const int i = (blockIdx.x * kPtsPerThread + rep) * kBlock + tid;
        double row[kIkRow];
        for (int k = 0; k < kIkRow; k++) row[k] = 0.0;
        if (i < job.n) {
            const float4 pb = reinterpret_cast<const float4*>(job.pts)[i];
            float wx, wy, wz;
            ik_world_point(X, pb.x, pb.y, pb.z, wx, wy, wz);
            const float4* rec = reinterpret_cast<const float4*>(job.nn + i);
            int* flagp = reinterpret_cast<int*>(job.nn + i) + 26;  // NNRec::flag
            const int cnt = reinterpret_cast<const int4*>(job.nn + i)[6].y;
            const int flag = *flagp;
            // Without a search a point is processed only if the last evaluation
            // kept it, and that evaluation fitted its plane from the same five
            // neighbours: the plane cache (pstate 2) holds that fit, so the
            // neighbours are not read and esti_plane not rerun.  A search (or a
            // point not fitted since one, pstate 0) fits and caches it.
#ifndef LIVO_IK_PLANE_CACHE
#define LIVO_IK_PLANE_CACHE 1
#endif
            const uint8_t ps = (search || !LIVO_IK_PLANE_CACHE) ? (uint8_t)0 : job.pstate[i];
            const bool sel = search ? ((cnt == kNN) && !(rec[kNN - 1].w > P.max_sqd)) : !(flag & kIkDrop);
            bool fin = false;
            float pa[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            float pd2 = 0.0f;
            bool planed = false;
            if (sel && cnt >= kNN) {
                if (ps == 2) {
                    const float4 c4 = reinterpret_cast<const float4*>(job.plane)[i];
                    pa[0] = c4.x; pa[1] = c4.y; pa[2] = c4.z; pa[3] = c4.w;
                    planed = true;
                } else if (ps == 0) {
                    float nx[kNN], ny[kNN], nz[kNN];
#pragma unroll
                    for (int k = 0; k < kNN; k++) {
                        const float4 v = rec[k];
                        nx[k] = v.x; ny[k] = v.y; nz[k] = v.z;
                    }
                    planed = esti_plane(nx, ny, nz, P.plane_thr, pa);
                    if (planed) reinterpret_cast<float4*>(job.plane)[i] = make_float4(pa[0], pa[1], pa[2], pa[3]);
                    job.pstate[i] = planed ? 2 : 1;
                }
                if (planed) {
                    pd2 = ((pa[0] * wx + pa[1] * wy) + pa[2] * wz) + pa[3];
                    const double bx = pb.x, by = pb.y, bz = pb.z;
                    const double bn = sqrt((bx * bx + by * by) + bz * bz);
                    const float s = (float)(1 - 0.9 * (double)fabsf(pd2) / sqrt(bn));
                    fin = (double)s > 0.9;
                }
            }
            const int nflag = fin ? (flag & ~kIkDrop) : (flag | kIkDrop);
            if (nflag != flag) *flagp = nflag;
            if (P.dbg.sel) P.dbg.sel[i] = (fin && (double)fabsf(pd2) <= P.max_res) ? 1 : 0;
            if (fin && (double)fabsf(pd2) <= P.max_res) {
                const double be[3] = {(double)pb.x, (double)pb.y, (double)pb.z};
                const Qd qo = qd_load(X.offset_R);
                double t0[3], pt[3];
                qd_rot(qo, be, t0);
                for (int c = 0; c < 3; c++) pt[c] = t0[c] + X.offset_T[c];
                const double n[3] = {(double)pa[0], (double)pa[1], (double)pa[2]};
                double C[3], A[3], Bv[3], Hp[9], Hb[9], Rt[9], HbR[9];
                qd_rot(qd_conj(qd_load(X.rot)), n, C);
                hat3d(pt, Hp);
                mat3d_vec(Hp, C, A);
                hat3d(be, Hb);
                qd_mat(qd_conj(qo), Rt);
                mat3d_mul(Hb, Rt, HbR);
                mat3d_vec(HbR, C, Bv);
                row[0] = n[0]; row[1] = n[1]; row[2] = n[2];
                row[3] = A[0]; row[4] = A[1]; row[5] = A[2];
                row[6] = Bv[0]; row[7] = Bv[1]; row[8] = Bv[2];
                row[9] = C[0]; row[10] = C[1]; row[11] = C[2];
                row[12] = -(double)pd2;
                row[13] = (double)fabsf(pd2);
                row[14] = 1.0;
            }
        }
        for (int k = 0; k < kIkRow; k++) rows[tid * kIkRow + k] = row[k];
        // the block's first kIkFewRows effective rows in point order: with fewer
        // than 23 effective points in the whole scan every block has fewer, and
        // the solve forms the reference's measurement-space gain from them
        const bool eff = row[14] != 0.0;
        const unsigned long long bal = __ballot(eff);
        if (lane == 0) wcnt[tid >> 6] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t pos = bcnt + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        uint32_t tot = 0;
        for (int w = 0; w < kBlock / 64; w++) {
            if (w < (tid >> 6)) pos += wcnt[w];
            tot += wcnt[w];
        }
        if (eff && pos < (uint32_t)kIkFewRows) {
            double* dst = job.ikrows + ((size_t)blockIdx.x * kIkFewRows + pos) * 13;
            for (int k = 0; k < 13; k++) dst[k] = row[k];
        }
        bcnt += tot;
        // (the rows were written before the __syncthreads above)
        const double* wrows = rows + (wv * 64) * kIkRow;
        for (int r = 0; r < 64; r++) {
            const double* q = wrows + r * kIkRow;
            comp_add(acc1, acc1_c, q[a1] * q[b1]);
            if (o2 < kIkUsed) {
                double v;
                if (o2 < 78) v = q[a2] * q[b2];
                else if (o2 < 90) v = q[o2 - 78] * q[12];
                else v = q[o2 == 90 ? 13 : 14];
                comp_add(acc2, acc2_c, v);
            }
        }
        __syncthreads();
    }
    wpart[wv][0][o1] = acc1;
    wpart[wv][1][o1] = acc1_c;
    if (o2 < kIkUsed) {
        wpart[wv][0][o2] = acc2;
        wpart[wv][1][o2] = acc2_c;
    }
    __syncthreads();
    if (tid < kIkUsed) {
        double sc = 0.0, cc = 0.0;
        for (int w = 0; w < kBlock / 64; w++) {
            comp_add(sc, cc, wpart[w][0][tid]);
            cc += wpart[w][1][tid];
        }
        job.partial[(size_t)blockIdx.x * kIkCols + tid] = sc;
        job.partial[(size_t)blockIdx.x * kIkCols + kIkCompOff + tid] = cc;
    }
    if (tid == 0) job.ikcnt[blockIdx.x] = bcnt < (uint32_t)kIkFewRows ? bcnt : (uint32_t)kIkFewRows + 1u;
}

// One block of kIkSolveWaves waves per scan: the IKFoM partials merged by every
// wave over its share of the blocks (wave w: blocks w, w + W, ...; 8 loads in
// flight per column), the waves' compensated sums then merged in wave order by
// wave 0 (order-free to ~1e-27: the same doubles as one serial compensated
// sum), and wave 0 runs ik_solve (kept out of the plane pass: the 23-wide solve
// needs far more registers than the per-point work).  Measured before on one
// wave: 149.5 us per call, the serial chain of 49 dependent rounds of loads.
constexpr int kIkSolveWaves = 8;
__global__ __launch_bounds__(64 * kIkSolveWaves) void k_solve_ik(HsParams P) {
    __shared__ IkSolveLds S;
    constexpr int kG = (64 * kIkSolveWaves) / kIkUsed;  // threads per column (5)
    __shared__ double wsum[kG][2][kIkUsed];
    const HsJob job = P.jobs[blockIdx.x];
    IekfSlot* slot = job.slot;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (P.replay_count && blockIdx.x == 0 && threadIdx.x == 0) *P.replay_count = 0u;
    if (slot->ctrl.stop) return;  // block-uniform
    SOLVE_MARK(0);
    // thread t < kG * 92: column t % 92 over blocks g, g + kG, ... (g = t / 92),
    // 10 blocks' loads in flight, so a 98-block scan is two rounds of loads
    if ((int)threadIdx.x < kG * kIkUsed) {
        const int c = threadIdx.x % kIkUsed, g = threadIdx.x / kIkUsed;
        double sc = 0.0, cc = 0.0;
        const double* src = job.partial + c;
        for (int b = g; b < job.nblk; b += 10 * kG) {
            double v[10], w[10];
#pragma unroll
            for (int k = 0; k < 10; k++) {
                const int bb = b + k * kG;
                const bool in = bb < job.nblk;
                v[k] = in ? src[(size_t)bb * kIkCols] : 0.0;
                w[k] = in ? src[(size_t)bb * kIkCols + kIkCompOff] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < 10; k++) {
                comp_add(sc, cc, v[k]);
                cc += w[k];
            }
        }
        wsum[g][0][c] = sc;
        wsum[g][1][c] = cc;
    }
    // the evaluation's measurement-free part (boxminus, SO3 / S2 corrections) on
    // the last wave, beside the others' reduction
    if (wave == kIkSolveWaves - 1) ik_prep(slot, S, lane, P.lpc);
    __syncthreads();
    SOLVE_MARK(1);
    if (wave > 0) return;
    for (int c = lane; c < kIkCols; c += 64) {
        double sc = 0.0, cc = 0.0;
        if (c < kIkUsed)
            for (int g = 0; g < kG; g++) {
                comp_add(sc, cc, wsum[g][0][c]);
                cc += wsum[g][1][c];
            }
        S.sum[c] = sc + cc;
    }
    WAVE_SYNC();
    if (lane == 0) {
        // fewer than 23 effective points: their rows, in point order (blocks in order)
        const int m = (int)S.sum[91];
        S.m = m;
        if (m < kIkDim) {
            int k = 0;
            for (int b = 0; b < job.nblk && k < m; b++) {
                const int cb = (int)job.ikcnt[b];
                for (int r = 0; r < cb && k < m; r++, k++)
                    for (int c = 0; c < 13; c++) S.Hm[k * 13 + c] = job.ikrows[((size_t)b * kIkFewRows + r) * 13 + c];
            }
        }
    }
    WAVE_SYNC();
    SOLVE_MARK(2);
    ik_solve(slot, job, S, lane, P.lpc);
}

__global__ __launch_bounds__(64) void k_solve(SolveParams P) {
    __shared__ SolveLds L;
    const HsJob job = P.jobs[blockIdx.x];
    IekfSlot* slot = job.slot;
    const int lane = threadIdx.x;
    // the k-NN replay of this evaluation has run (stream order): reset its count
    if (P.replay_count && blockIdx.x == 0 && lane == 0) *P.replay_count = 0u;
    if (P.mode == 0 && slot->ctrl.stop) return;
    SOLVE_MARK(0);
    // deterministic reduction of the block partials: lane (c, h) sums the
    // blocks b = h, h+2, ... of column c with 8 loads in flight, in a fixed
    // association; then the two halves.
    {
        const int col = lane & 31, half = lane >> 5;
        const double* src = job.partial + col;
        double acc8[8];
#pragma unroll
        for (int k = 0; k < 8; k++) acc8[k] = 0.0;
        int b = half;
        for (; b + 14 < job.nblk; b += 16) {
#pragma unroll
            for (int k = 0; k < 8; k++) acc8[k] += src[(size_t)(b + 2 * k) * kRedCols];
        }
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (b + 2 * k < job.nblk) acc8[k] += src[(size_t)(b + 2 * k) * kRedCols];
        double sum = ((acc8[0] + acc8[1]) + (acc8[2] + acc8[3])) + ((acc8[4] + acc8[5]) + (acc8[6] + acc8[7]));
        sum += __shfl_xor(sum, 32, 64);
        if (col >= kRedUsed) sum = 0.0;
        if (lane < kRedCols) {
            L.sum[lane] = sum;
            slot->red[lane] = sum;
        }
    }
    SOLVE_MARK(1);
    if (P.mode == 1) return;
    solve_stage(slot, L, lane, 64);
    WAVE_SYNC();
    solve_scan(slot, L, lane);
}

// ======================================================== launchers =======
// The replay follows every search but usually has 0-5 queries: a few small
// blocks (a 64-block grid waited ~10 us for LDS behind the concurrent stream
// groups' searches), stack LDS sized to the tree's depth.
constexpr int kReplayBlocks = 8;
static size_t replay_lds_bytes(int depth) {
    return (size_t)std::max(1, std::min(depth, kMaxDepth)) * 64 * sizeof(uint2);
}

size_t knn_lds_bytes(int depth) {
    const int entries = depth > 1 ? depth - 1 : 1;  // son levels 1 .. depth-1
    return (size_t)entries * kKnnBlock * sizeof(float);
}

int launch_knn_pass(const KnnParams& p, int n_jobs, int64_t max_n, void* stream) {
    if (n_jobs <= 0 || max_n <= 0) return LIVO_OK;
    KnnParams q = p;
    q.nb = (int32_t)((max_n + kKnnBlock - 1) / kKnnBlock);
    if ((int64_t)q.nb * n_jobs >= (1ll << 31)) return LIVO_E_RANGE;
    hipLaunchKernelGGL(k_knn_pass, dim3((unsigned)(q.nb * n_jobs)), dim3(kKnnBlock), knn_lds_bytes(p.depth),
                       (hipStream_t)stream, q);
    if (hipGetLastError() != hipSuccess) return LIVO_E_HIP;
    hipLaunchKernelGGL(k_knn_replay, dim3(kReplayBlocks), dim3(64), replay_lds_bytes(q.depth), (hipStream_t)stream, q);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

int launch_knn_leaf(const KnnParams& p, int n_jobs, int64_t max_n, bool seeded, void* stream) {
    if (n_jobs <= 0 || max_n <= 0) return LIVO_OK;
    KnnParams q = p;
    q.nb = (int32_t)((max_n + kKnnBlock - 1) / kKnnBlock);
    if ((int64_t)q.nb * n_jobs >= (1ll << 31)) return LIVO_E_RANGE;
    const dim3 grid((unsigned)(q.nb * n_jobs)), block(kKnnBlock);
    const size_t lds = knn_lds_bytes(p.ldepth + 1);
    if (seeded)
        hipLaunchKernelGGL((k_knn_leaf<true, 1>), grid, block, lds, (hipStream_t)stream, q);
    else
        hipLaunchKernelGGL((k_knn_leaf<false, 1>), grid, block, lds, (hipStream_t)stream, q);
    if (hipGetLastError() != hipSuccess) return LIVO_E_HIP;
    hipLaunchKernelGGL(k_knn_replay, dim3(kReplayBlocks), dim3(64), replay_lds_bytes(q.depth), (hipStream_t)stream, q);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

int launch_knn_grid(const KnnParams& p, int n_jobs, int64_t max_n, bool seeded, bool tile, void* stream) {
    if (n_jobs <= 0 || max_n <= 0) return LIVO_OK;
    KnnParams q = p;
    const int B = tile ? 64 : kKnnBlock;
    q.nb = (int32_t)((max_n + B - 1) / B);
    if ((int64_t)q.nb * n_jobs >= (1ll << 31)) return LIVO_E_RANGE;
    const dim3 grid((unsigned)(q.nb * n_jobs)), block(B);
#if LIVO_IDX_RUNS
    if (q.vslots && !q.canon && !q.dyn_runs) {  // the runs of a static map: their search pass
        q.nb = (int32_t)((max_n + kEvalBlock - 1) / kEvalBlock);
        if ((int64_t)q.nb * n_jobs >= (1ll << 31)) return LIVO_E_RANGE;  // (the grid actually launched)
        const dim3 rgrid((unsigned)(q.nb * n_jobs)), rblock(kEvalBlock);
        if (seeded)
            hipLaunchKernelGGL(k_knn_runs<true>, rgrid, rblock, 0, (hipStream_t)stream, q);
        else
            hipLaunchKernelGGL(k_knn_runs<false>, rgrid, rblock, 0, (hipStream_t)stream, q);
    } else
#endif
    if (tile) {
        if (seeded)
            hipLaunchKernelGGL((k_knn_grid<true, true>), grid, block, 0, (hipStream_t)stream, q);
        else
            hipLaunchKernelGGL((k_knn_grid<false, true>), grid, block, 0, (hipStream_t)stream, q);
    } else if (seeded) {
        hipLaunchKernelGGL((k_knn_grid<true, false>), grid, block, 0, (hipStream_t)stream, q);
    } else {
        hipLaunchKernelGGL((k_knn_grid<false, false>), grid, block, 0, (hipStream_t)stream, q);
    }
    if (hipGetLastError() != hipSuccess) return LIVO_E_HIP;
    if (q.canon)
        hipLaunchKernelGGL(k_knn_canon, dim3(kReplayBlocks), dim3(64), 0, (hipStream_t)stream, q);
    else
        hipLaunchKernelGGL(k_knn_replay, dim3(kReplayBlocks), dim3(64), replay_lds_bytes(q.depth), (hipStream_t)stream, q);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

#ifdef LIVO_TAIL_PROF
// s_memtime ticks per s_memrealtime tick (100 MHz): the phase marks' clock
__global__ void k_clock_cal(unsigned long long* out, int iters) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float x = (float)threadIdx.x;
    for (int k = 0; k < iters; k++) x = x * 0.999f + 1.0f;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; out[2] = (unsigned long long)x; }
}
extern "C" int livo_debug_clock(double* mhz) {
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 32) != hipSuccess) return LIVO_E_HIP;
    unsigned long long h[3] = {};
    hipLaunchKernelGGL(k_clock_cal, dim3(1), dim3(64), 0, 0, d, 4 << 20);
    const bool ok = hipMemcpy(h, d, 24, hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipFree(d);
    if (!ok || h[1] == 0) return LIVO_E_HIP;
    *mhz = 100.0 * (double)h[0] / (double)h[1];
    return LIVO_OK;
}
extern "C" int livo_debug_tail_prof(unsigned long long* out) {  // [3][8] tail, then [3][16] solve phases; reset
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tail_prof), sizeof(g_tail_prof)) != hipSuccess) return LIVO_E_HIP;
    if (hipMemcpyFromSymbol(out + 24, HIP_SYMBOL(g_solve_ph), sizeof(g_solve_ph)) != hipSuccess) return LIVO_E_HIP;
    unsigned long long zero[3][16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_solve_ph), zero, sizeof(g_solve_ph)) != hipSuccess) return LIVO_E_HIP;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_tail_prof), zero, sizeof(g_tail_prof)) == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
#endif

// per-phase profile of k_iekf_eval (LIVO_EVAL_PROF builds only): out[24], reset after reading
#ifdef LIVO_EVAL_PROF
// Profiling builds only (not part of livo.h): per-phase block cycles of the
// fused evaluation since the last call (tools/eval_prof.py).
extern "C" int livo_debug_eval_timeline(unsigned long long* out, int64_t bytes) {  // LIVO_MAX_EVALS x kTlBlocks x 2
    if (bytes != (int64_t)sizeof(g_eval_tl)) return LIVO_E_INVALID;
    if (hipDeviceSynchronize() != hipSuccess) return LIVO_E_HIP;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_eval_tl), sizeof(g_eval_tl)) == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
extern "C" int livo_debug_eval_prof(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return LIVO_E_HIP;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_eval_prof), sizeof(g_eval_prof)) != hipSuccess) return LIVO_E_HIP;
    static const unsigned long long zero[24] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_eval_prof), zero, sizeof(zero)) == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
extern "C" int livo_debug_amb_reason(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return LIVO_E_HIP;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_amb_reason), sizeof(g_amb_reason)) != hipSuccess) return LIVO_E_HIP;
    static const unsigned long long zero[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_amb_reason), zero, sizeof(zero)) == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
extern "C" int livo_debug_eval_stats(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return LIVO_E_HIP;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_eval_stats), sizeof(g_eval_stats)) != hipSuccess) return LIVO_E_HIP;
    static const unsigned long long zero[24] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_eval_stats), zero, sizeof(zero)) == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
#endif

#ifdef LIVO_SOLVE_PROF
// k_solve_ik phase marks of the last launch, [block][mark] (the profiling build only)
extern "C" int livo_debug_solve_prof(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return LIVO_E_HIP;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_solve_prof), sizeof(g_solve_prof)) == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
#endif

// Word copy by a kernel, for a batch lane's staging transfers between host-mapped
// pinned memory and HBM (livo_capi.cpp batch_enqueue): on the compute queue
// with the evaluations, so a batch queued behind another waits on no DMA-engine
// hand-off.  Plain vector loads / stores, 16 B per lane.
__global__ __launch_bounds__(256) void k_copy_words(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                    int64_t n16) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

int launch_copy_words(const void* src, void* dst, size_t bytes, void* stream) {
    if (bytes == 0) return LIVO_OK;
    if (bytes % 16 || (reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) % 16) return LIVO_E_INVALID;
    const int64_t n16 = (int64_t)(bytes / 16);
    const unsigned blocks = (unsigned)std::min<int64_t>((n16 + 255) / 256, 64);
    hipLaunchKernelGGL(k_copy_words, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), n16);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

// Two ranges of 16-B words in one launch (a stream group's slots and its jobs).
__global__ __launch_bounds__(256) void k_copy_ranges(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                     int64_t a0, int64_t n0, int64_t a1, int64_t n1) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n0 + n1; i += (int64_t)gridDim.x * 256) {
        const int64_t w = i < n0 ? a0 + i : a1 + (i - n0);
        dst[w] = src[w];
    }
}

int launch_copy_ranges(const void* src, void* dst, size_t o0, size_t n0, size_t o1, size_t n1, void* stream) {
    if (n0 + n1 == 0) return LIVO_OK;
    if ((o0 | n0 | o1 | n1) % 16 || (reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) % 16)
        return LIVO_E_INVALID;
    const int64_t w0 = (int64_t)(n0 / 16), w1 = (int64_t)(n1 / 16);
    const unsigned blocks = (unsigned)std::min<int64_t>((w0 + w1 + 255) / 256, 64);
    hipLaunchKernelGGL(k_copy_ranges, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), (int64_t)(o0 / 16), w0,
                       (int64_t)(o1 / 16), w1);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

int launch_iekf_eval(const KnnParams& kp, const HsParams& hp, int n_jobs, int64_t max_n, bool first, void* stream) {
    if (n_jobs <= 0 || max_n <= 0) return LIVO_OK;
    EvalParams E;
    E.k = kp;
    E.h = hp;
    E.k.nb = (int32_t)((max_n + kEvalBlock - 1) / kEvalBlock);
    if ((int64_t)E.k.nb * n_jobs >= (1ll << 31)) return LIVO_E_RANGE;
    const dim3 grid((unsigned)(E.k.nb * n_jobs)), block(kEvalBlock);
    if (first)
        hipLaunchKernelGGL(k_iekf_eval<true>, grid, block, 0, (hipStream_t)stream, E);
    else
        hipLaunchKernelGGL(k_iekf_eval<false>, grid, block, 0, (hipStream_t)stream, E);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

int launch_hshare(const HsParams& p, int n_jobs, int max_nblk, bool first, void* stream) {
    if (n_jobs <= 0 || max_nblk <= 0) return LIVO_OK;
    dim3 grid(max_nblk, n_jobs), block(kBlock);
    if (first)
        hipLaunchKernelGGL(k_hshare<true>, grid, block, 0, (hipStream_t)stream, p);
    else
        hipLaunchKernelGGL(k_hshare<false>, grid, block, 0, (hipStream_t)stream, p);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

int launch_hshare_ik(const HsParams& p, int n_jobs, int max_nblk, bool first, void* stream) {
    if (n_jobs <= 0 || max_nblk <= 0) return LIVO_OK;
    dim3 grid(max_nblk, n_jobs), block(kBlock);
    if (first)
        hipLaunchKernelGGL(k_hshare_ik<true>, grid, block, 0, (hipStream_t)stream, p);
    else
        hipLaunchKernelGGL(k_hshare_ik<false>, grid, block, 0, (hipStream_t)stream, p);
    if (hipGetLastError() != hipSuccess) return LIVO_E_HIP;
    if (!p.solve) return LIVO_OK;
    return launch_solve_ik(p, n_jobs, stream);
}

int launch_solve_ik(const HsParams& p, int n_jobs, void* stream) {
    if (n_jobs <= 0) return LIVO_OK;
    hipLaunchKernelGGL(k_solve_ik, dim3(n_jobs), dim3(64 * kIkSolveWaves), 0, (hipStream_t)stream, p);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

int launch_solve(const SolveParams& p, int n_jobs, void* stream) {
    if (n_jobs <= 0) return LIVO_OK;
    hipLaunchKernelGGL(k_solve, dim3(n_jobs), dim3(64), 0, (hipStream_t)stream, p);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

}  // namespace livo
