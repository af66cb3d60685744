// frontend_kernels.hip — CDNA4 (gfx950) kernels of the scan front-end
// (SURVEY.md §8f row 3): the per-point work between the raw LiDAR frame and
// the resident scan the IEKF reads (feats_down_body).
//
//   k_fe_segment / k_fe_undistort   ImuProcess::UndistortPcl's backward
//       propagation (IMU_Processing.cpp:340-378).  The reference walks points
//       and IMU segments backwards together; with non-decreasing segment
//       times a point's segment is the suffix minimum over later points of
//       "last segment starting before me" (k_fe_segment + a min-scan), so
//       every point is moved independently.  The first point is moved once
//       per remaining segment, as the reference's walk does (its inner loop
//       breaks at begin() without stepping): one thread chains those moves.
//   k_fe_minmax / k_fe_leaf / k_fe_runs / k_fe_centroid   PCL VoxelGrid::
//       applyFilter (downSizeFilterSurf, laser_mapping.cpp:129-130): bounds,
//       32-bit leaf index per point, a stable radix sort by leaf, one centroid
//       per run (one wave each) in ascending leaf order.  (PCL sums a voxel in
//       std::sort's unstable order; here a fixed lane-strided tree: centroids
//       agree to float rounding, voxels and counts exactly.)
//   k_fe_morton / k_fe_gather        the resident scan's Morton order, the
//       same keys and stable order as livo_scan_upload's host sort.
//
// Numerics: -ffp-contract=off; doubles in the reference's expression order.
#include <hip/hip_runtime.h>
#include <math.h>

#include "device_common.h"
#include "livo_internal.h"

namespace livo {

// Pose6D (msg/Pose6D.msg): offset_time, acc[3], gyr[3], vel[3], pos[3], rot[9]
constexpr int kPoseD = 22;

__global__ void k_fe_segment(const float* __restrict__ raw, int64_t n, const double* __restrict__ poses, int np,
                             int32_t* __restrict__ seg_rev) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double t = (double)raw[5 * i + 4] / double(1000);
    // last head h in [0, np-2] with offset(h) < t, else -1 (offsets non-decreasing)
    int lo = 0, hi = np - 1;  // answer in [lo - 1, hi - 1]
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (poses[(int64_t)mid * kPoseD] < t)
            lo = mid + 1;
        else
            hi = mid;
    }
    seg_rev[n - 1 - i] = lo - 1;  // reversed: a prefix min-scan gives the suffix minimum
}

// Exp(ang_vel, dt) (so3_math.h:31-52)
__device__ __forceinline__ void so3_exp_dt(const double* g, double dt, double* R) {
    const double nrm = sqrt((g[0] * g[0] + g[1] * g[1]) + g[2] * g[2]);
#pragma unroll
    for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (nrm > 0.0000001) {
        const double r[3] = {g[0] / nrm, g[1] / nrm, g[2] / nrm};
        const double K[9] = {0.0, -r[2], r[1], r[2], 0.0, -r[0], -r[1], r[0], 0.0};
        const double ang = nrm * dt;
        const double s = sin(ang), c1 = 1.0 - cos(ang);
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const double kk = ((c1 * K[i * 3 + 0]) * K[0 * 3 + j] + (c1 * K[i * 3 + 1]) * K[1 * 3 + j]) +
                                  (c1 * K[i * 3 + 2]) * K[2 * 3 + j];
                R[i * 3 + j] = (R[i * 3 + j] + s * K[i * 3 + j]) + kk;
            }
    }
}

__device__ __forceinline__ void m3v(const double* M, const double* v, double* o) {
#pragma unroll
    for (int i = 0; i < 3; i++) o[i] = (M[i * 3 + 0] * v[0] + M[i * 3 + 1] * v[1]) + M[i * 3 + 2] * v[2];
}

// P_compensate = extR_Ri * (R_i * (R_LI * P_i + t_LI) + T_ei) - exrR_extT (IMU_Processing.cpp:356-370)
__device__ void fe_compensate(float* p, const double* __restrict__ head, const FrontParams& F) {
    const double dt = (double)p[4] / double(1000) - head[0];
    double Re[9], Ri[9];
    so3_exp_dt(head + 4, dt, Re);
    const double* Rh = head + 13;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            Ri[i * 3 + j] = (Rh[i * 3 + 0] * Re[0 * 3 + j] + Rh[i * 3 + 1] * Re[1 * 3 + j]) + Rh[i * 3 + 2] * Re[2 * 3 + j];
    double T[3];
#pragma unroll
    for (int k = 0; k < 3; k++)
        T[k] = ((head[10 + k] + head[7 + k] * dt) + ((0.5 * head[1 + k]) * dt) * dt) - F.pos_end[k];
    const double Pi[3] = {(double)p[0], (double)p[1], (double)p[2]};
    double a[3], b[3], c[3];
    m3v(F.R_LI, Pi, a);
#pragma unroll
    for (int k = 0; k < 3; k++) a[k] = a[k] + F.t_LI[k];
    m3v(Ri, a, b);
#pragma unroll
    for (int k = 0; k < 3; k++) b[k] = b[k] + T[k];
    m3v(F.extR_Ri, b, c);
    p[0] = (float)(c[0] - F.exrR_extT[0]);
    p[1] = (float)(c[1] - F.exrR_extT[1]);
    p[2] = (float)(c[2] - F.exrR_extT[2]);
}

// seg_rev holds the prefix minimum of the reversed segments: point i's
// segment is seg_rev[n-1-i] (-1: untouched).
__global__ void k_fe_undistort(FrontParams F) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= F.n) return;
    const int h = F.seg_rev[F.n - 1 - i];
    if (h < 0) return;
    float p[5];
#pragma unroll
    for (int k = 0; k < 5; k++) p[k] = F.raw[5 * i + k];
    if (i == 0) {
        // the walk's inner loop breaks at begin() without stepping, so every
        // earlier segment moves the first point again
        for (int hh = h; hh >= 0; hh--) fe_compensate(p, F.poses + (int64_t)hh * kPoseD, F);
    } else {
        fe_compensate(p, F.poses + (int64_t)h * kPoseD, F);
    }
#pragma unroll
    for (int k = 0; k < 3; k++) F.raw[5 * i + k] = p[k];
}

// Order-preserving float <-> uint mapping for atomic min / max.
__device__ __forceinline__ unsigned f2o(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// minmax[0..2] = ordered min of x, y, z; [3..5] = ordered max (initialised to
// 0xFFFFFFFF / 0 by the caller).  stride: floats per point.  256 threads; the
// block reduces in LDS and issues 6 device atomics (the launcher caps the grid
// at kMinmaxBlocks): per-wave atomics from ~1.6k waves on 6 addresses
// serialised across the XCDs and took 110-220 us per 100k-point scan.
constexpr int kMinmaxBlocks = 64;
__global__ __launch_bounds__(256) void k_fe_minmax(const float* __restrict__ pts, int64_t n, int stride,
                                                   unsigned* minmax) {
    __shared__ unsigned red[4][6];
    unsigned mn[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, mx[3] = {0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const unsigned o = f2o(pts[stride * i + k]);
            mn[k] = min(mn[k], o);
            mx[k] = max(mx[k], o);
        }
#pragma unroll
    for (int k = 0; k < 3; k++)
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            mn[k] = min(mn[k], (unsigned)__shfl_xor((int)mn[k], off, 64));
            mx[k] = max(mx[k], (unsigned)__shfl_xor((int)mx[k], off, 64));
        }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int k = 0; k < 3; k++) {
            red[wave][k] = mn[k];
            red[wave][3 + k] = mx[k];
        }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        unsigned v = red[0][k];
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) v = k < 3 ? min(v, red[w][k]) : max(v, red[w][k]);
        if (k < 3) atomicMin(minmax + k, v);
        else atomicMax(minmax + k, v);
    }
}

// PCL leaf index (voxel_grid.hpp): ijk = int(floor(p * inv) - float(min_b)), idx = ijk . divb_mul
__global__ void k_fe_leaf(FrontParams F) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= F.n) return;
    const float inv = F.inv_leaf;
    const int ijk0 = (int)(floorf(F.raw[5 * i + 0] * inv) - (float)F.min_b[0]);
    const int ijk1 = (int)(floorf(F.raw[5 * i + 1] * inv) - (float)F.min_b[1]);
    const int ijk2 = (int)(floorf(F.raw[5 * i + 2] * inv) - (float)F.min_b[2]);
    F.keys[i] = (uint32_t)(ijk0 * F.divb_mul[0] + ijk1 * F.divb_mul[1] + ijk2 * F.divb_mul[2]);
    F.iota[i] = (uint32_t)i;
}

// flags[k] = 1 where a new leaf starts in the sorted order
__global__ void k_fe_runs(FrontParams F) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= F.n) return;
    F.flags[k] = (k == 0 || F.skeys[k] != F.skeys[k - 1]) ? 1u : 0u;
}

__global__ void k_fe_starts(FrontParams F) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= F.n) return;
    if (F.flags[k]) F.starts[F.vid[k]] = (uint32_t)k;
    if (k == F.n - 1) F.starts[F.vid[k] + F.flags[k]] = (uint32_t)F.n;
}

// CentroidPoint of one leaf (AccumulatorXYZ / Intensity / Curvature: float
// sums / n), one wave per leaf: lanes sum strided members in input order, a
// fixed xor-tree combines them (PCL's own order is std::sort's, unspecified).
__global__ void k_fe_centroid(FrontParams F, int64_t n_vox) {
    const int64_t v = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const int lane = threadIdx.x & 63;
    if (v >= n_vox) return;
    const uint32_t a = F.starts[v], b = F.starts[v + 1];
    float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (uint32_t k = a + lane; k < b; k += 64) {
        const float* p = F.raw + 5 * (int64_t)F.svals[k];
#pragma unroll
        for (int c = 0; c < 5; c++) s[c] += p[c];
    }
#pragma unroll
    for (int c = 0; c < 5; c++)
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s[c] += __shfl_xor(s[c], off, 64);
    if (lane < 5) {
        const float cnt = (float)(b - a);
        float val = s[0];
#pragma unroll
        for (int c = 1; c < 5; c++) val = lane == c ? s[c] : val;
        F.down[5 * v + lane] = val / cnt;
    }
}

// livo_scan_upload's Morton key: 9 bits per axis (27 bits) over the scan's
// bounding box, cells of 1/scale m (0.25 m by default) or, for a box wider than
// 512 cells, the box's widest extent / 512 (every scan keeps 512 cells per axis
// at most, so one 32-bit radix sort orders it; 20 bits per axis and a 64-bit
// sort took twice the passes).  lo / hi: the order-preserving encodings.
__device__ __forceinline__ float fe_decode(unsigned o) { return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o); }
__device__ __forceinline__ float fe_key_scale(const unsigned* lo, const unsigned* hi, float scale) {
    float ext = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; a++) ext = fmaxf(ext, fe_decode(hi[a]) - fe_decode(lo[a]));
    return (ext * scale > 511.0f) ? 511.0f / ext : scale;
}
__device__ __forceinline__ uint32_t fe_key(const float* p, const unsigned* lo, float s) {
    uint32_t code = 0;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        float f = (p[a] - fe_decode(lo[a])) * s;
        if (!(f >= 0.0f)) f = 0.0f;
        const uint32_t q = (uint32_t)fminf(f, 511.0f);
#pragma unroll
        for (int b = 0; b < 9; b++) code |= ((q >> b) & 1u) << (3 * b + a);
    }
    return code;
}
__global__ void k_fe_morton(const float* __restrict__ pts, int64_t n, int stride, const unsigned* minmax,
                            float scale, uint32_t* codes, uint32_t* iota) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float s = fe_key_scale(minmax, minmax + 3, scale);
    codes[i] = fe_key(pts + stride * i, minmax, s);
    iota[i] = (uint32_t)i;
}

// the scan in stored order: pts4[k] = point perm[k]; iperm[perm[k]] = k
__global__ void k_fe_gather(const float* __restrict__ pts, int64_t n, int stride, const uint32_t* __restrict__ perm,
                            float* __restrict__ pts4, int32_t* __restrict__ iperm) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t j = perm[k];
    reinterpret_cast<float4*>(pts4)[k] =
        make_float4(pts[stride * (int64_t)j], pts[stride * (int64_t)j + 1], pts[stride * (int64_t)j + 2], 0.f);
    iperm[j] = (int32_t)k;
}

// ---- a batch of scans built in one pass (livo_scan_upload_batch_async) ----
// Every scan's points lie packed (x, y, z) in one device array at seg.off[b];
// blockIdx.y = the scan; its bounds at minmax[6b..6b+5] (mins, then the maxes
// inverted, all initialised to 0xFFFFFFFF).  Per scan the same bounds, keys and stable order as
// k_fe_minmax / k_fe_morton / k_fe_gather on that scan alone: the key carries
// the scan in its top bits, so one stable sort of the batch orders each scan's
// points as its own sort would (ties by input position in both).
__global__ __launch_bounds__(256) void k_fe_minmax_seg(const float* __restrict__ pts, FeSegs S, unsigned* minmax) {
    const int b = blockIdx.y;
    const float* p = pts + 3 * S.off[b];
    const int64_t n = S.n[b];
    __shared__ unsigned red[4][6];
    unsigned mn[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, mx[3] = {0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const unsigned o = f2o(p[3 * i + k]);
            mn[k] = min(mn[k], o);
            mx[k] = max(mx[k], o);
        }
#pragma unroll
    for (int k = 0; k < 3; k++)
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            mn[k] = min(mn[k], (unsigned)__shfl_xor((int)mn[k], off, 64));
            mx[k] = max(mx[k], (unsigned)__shfl_xor((int)mx[k], off, 64));
        }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int k = 0; k < 3; k++) {
            red[wave][k] = mn[k];
            red[wave][3 + k] = mx[k];
        }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        unsigned v = red[0][k];
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) v = k < 3 ? min(v, red[w][k]) : max(v, red[w][k]);
        atomicMin(minmax + 6 * b + k, k < 3 ? v : ~v);  // (maxes stored inverted: one 0xFF.. initialisation)
    }
}

__global__ void k_fe_morton_seg(const float* __restrict__ pts, FeSegs S, const unsigned* minmax, float scale,
                                uint32_t* codes, uint32_t* iota) {
    const int b = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S.n[b]) return;
    const int64_t g = S.off[b] + i;
    const unsigned* lo = minmax + 6 * b;
    const unsigned hi[3] = {~lo[3], ~lo[4], ~lo[5]};  // (the maxes are stored inverted)
    const float s = fe_key_scale(lo, hi, scale);
    codes[g] = ((uint32_t)b << 27) | fe_key(pts + 3 * g, lo, s);
    iota[g] = (uint32_t)g;
}

// scan b in stored order: pts4[k] = its point perm[k]; iperm[perm[k]] = k; the
// stored position -> input index map (ScanBuf::d_perm) and cleared neighbour
// records / plane states
__global__ void k_fe_gather_seg(const float* __restrict__ pts, FeSegs S, const uint32_t* __restrict__ sorted) {
    const int b = blockIdx.y;
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= S.n[b]) return;
    const int64_t o = S.off[b];
    const uint32_t jg = sorted[o + k];
    const int32_t j = (int32_t)(jg - (uint32_t)o);
    reinterpret_cast<float4*>(S.pts4[b])[k] =
        make_float4(pts[3 * (int64_t)jg], pts[3 * (int64_t)jg + 1], pts[3 * (int64_t)jg + 2], 0.f);
    S.iperm[b][j] = (int32_t)k;
    S.perm[b][k] = j;
    float4* rec = reinterpret_cast<float4*>(S.nn[b]) + 8 * k;  // (128-B NNRec)
#pragma unroll
    for (int w = 0; w < 8; w++) rec[w] = make_float4(0.f, 0.f, 0.f, 0.f);
    S.pstate[b][k] = 0;
}

// RGBpointBodyToWorld (laser_mapping.cpp:647-660) over laserCloudFullRes
// (:258-265): p_w = rot (R_LI p_b + t_LI) + pos in double, stored as float;
// intensity copied (column 3 of a 5-float source, 0 for a 4-float scan),
// curvature 0 (a fresh PointType).  perm: source position -> output index.
__global__ void k_to_world(const float* __restrict__ src, int64_t n, int stride, const int32_t* __restrict__ perm,
                           WorldParams W, float* __restrict__ out5) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const float* p = src + stride * k;
    float wx, wy, wz;
    world_point(W.rot, W.pos, W.R_LI, W.t_LI, p[0], p[1], p[2], wx, wy, wz);
    const int64_t o = perm ? (int64_t)perm[k] : k;
    float* q = out5 + 5 * o;
    q[0] = wx;
    q[1] = wy;
    q[2] = wz;
    q[3] = stride >= 5 ? p[3] : 0.0f;
    q[4] = 0.0f;
}

// laserCloudOri / corr_normvect (laser_mapping.cpp:547-561): the effective
// points in the caller's point order.  flags[caller index] = effective; an
// exclusive scan gives each its place; then body point and normvec scattered.
__global__ void k_ori_flags(const uint8_t* __restrict__ sel, const int32_t* __restrict__ perm, int64_t n,
                            uint32_t* __restrict__ flags) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    flags[perm[k]] = sel[k] ? 1u : 0u;
}
__global__ void k_ori_scatter(const float* __restrict__ pts4, const float* __restrict__ normvec,
                              const uint8_t* __restrict__ sel, const int32_t* __restrict__ perm,
                              const uint32_t* __restrict__ pos, int64_t n, float* __restrict__ ori3,
                              float* __restrict__ corr4) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n || !sel[k]) return;
    const int64_t o = pos[perm[k]];
    const float4 p = reinterpret_cast<const float4*>(pts4)[k];
    ori3[3 * o + 0] = p.x;
    ori3[3 * o + 1] = p.y;
    ori3[3 * o + 2] = p.z;
    reinterpret_cast<float4*>(corr4)[o] = reinterpret_cast<const float4*>(normvec)[k];
}

static inline dim3 fe_blocks(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }
#define FE_LAUNCH(kernel, n, ...)                                                                   \
    do {                                                                                            \
        if ((n) <= 0) return LIVO_OK;                                                               \
        hipLaunchKernelGGL(kernel, fe_blocks(n), dim3(256), 0, (hipStream_t)stream, __VA_ARGS__); \
        return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;                              \
    } while (0)

int launch_fe_segment(const FrontParams& F, void* stream) {
    FE_LAUNCH(k_fe_segment, F.n, F.raw, F.n, F.poses, F.np, F.seg);
}
int launch_fe_undistort(const FrontParams& F, void* stream) { FE_LAUNCH(k_fe_undistort, F.n, F); }
int launch_fe_minmax(const float* pts, int64_t n, int stride, unsigned* minmax, void* stream) {
    if (n <= 0) return LIVO_OK;
    const unsigned blocks = (unsigned)std::min<int64_t>(kMinmaxBlocks, (n + 255) / 256);
    hipLaunchKernelGGL(k_fe_minmax, dim3(blocks), dim3(256), 0, (hipStream_t)stream, pts, n, stride, minmax);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
int launch_fe_leaf(const FrontParams& F, void* stream) { FE_LAUNCH(k_fe_leaf, F.n, F); }
int launch_fe_runs(const FrontParams& F, void* stream) { FE_LAUNCH(k_fe_runs, F.n, F); }
int launch_fe_starts(const FrontParams& F, void* stream) { FE_LAUNCH(k_fe_starts, F.n, F); }
int launch_fe_centroid(const FrontParams& F, int64_t n_vox, void* stream) {
    if (n_vox <= 0) return LIVO_OK;
    hipLaunchKernelGGL(k_fe_centroid, dim3((unsigned)((n_vox + 3) / 4)), dim3(256), 0, (hipStream_t)stream, F, n_vox);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
int launch_fe_morton(const float* pts, int64_t n, int stride, const unsigned* minmax, float scale,
                     uint32_t* codes, uint32_t* iota, void* stream) {
    FE_LAUNCH(k_fe_morton, n, pts, n, stride, minmax, scale, codes, iota);
}
int launch_fe_gather(const float* pts, int64_t n, int stride, const uint32_t* perm, float* pts4, int32_t* iperm,
                     void* stream) {
    FE_LAUNCH(k_fe_gather, n, pts, n, stride, perm, pts4, iperm);
}
// Scan b's 3 n floats from its mapped host array: 16-B reads when the source is
// 16-B aligned (then 12 n / 16 words and a tail), else 4-B reads; blockIdx.y = b.
__global__ __launch_bounds__(256) void k_fe_copy_seg(FeSrc S, float* __restrict__ dst) {
    const int b = blockIdx.y;
    const float* src = S.src[b];
    float* d = dst + 3 * S.off[b];
    const int64_t nf = 3 * S.n[b];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((((uintptr_t)src | (uintptr_t)d) & 15u) == 0u) {
        const int64_t nw = nf >> 2;
        const float4* s4 = reinterpret_cast<const float4*>(src);
        float4* d4 = reinterpret_cast<float4*>(d);
        // 4 reads in flight per thread: the PCIe round trip, not the CU count, sets the rate
        int64_t w = t;
        for (; w + 3 * stride < nw; w += 4 * stride) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = s4[w + u * stride];
#pragma unroll
            for (int u = 0; u < 4; u++) d4[w + u * stride] = v[u];
        }
        for (; w < nw; w += stride) d4[w] = s4[w];
        for (int64_t k = 4 * nw + t; k < nf; k += stride) d[k] = src[k];
    } else {
        for (int64_t k = t; k < nf; k += stride) d[k] = src[k];
    }
}
int launch_fe_copy_seg(const FeSrc& S, int n_scans, int64_t max_n, float* dst, void* stream) {
    if (n_scans <= 0 || n_scans > kFeSegMax || max_n <= 0) return n_scans == 0 ? LIVO_OK : LIVO_E_RANGE;
    // 16 blocks a scan (4 x 16 B in flight per thread, ~256 KB per batch in flight):
    // enough outstanding reads for the link without holding the CUs the batches run on
    const unsigned bx = (unsigned)std::min<int64_t>(16, (3 * max_n / 4 + 255) / 256);
    hipLaunchKernelGGL(k_fe_copy_seg, dim3(bx, (unsigned)n_scans), dim3(256), 0, (hipStream_t)stream, S, dst);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
int launch_fe_build_seg(const float* pts, const FeSegs& S, int n_scans, int64_t max_n, unsigned* minmax, float scale,
                        uint32_t* codes, uint32_t* iota, void* stream) {
    if (n_scans <= 0 || n_scans > kFeSegMax || max_n <= 0) return n_scans == 0 ? LIVO_OK : LIVO_E_RANGE;
    const unsigned bx = (unsigned)((max_n + 255) / 256);
    const dim3 mm((unsigned)std::min<int64_t>(kMinmaxBlocks, bx), (unsigned)n_scans), g(bx, (unsigned)n_scans);
    hipLaunchKernelGGL(k_fe_minmax_seg, mm, dim3(256), 0, (hipStream_t)stream, pts, S, minmax);
    hipLaunchKernelGGL(k_fe_morton_seg, g, dim3(256), 0, (hipStream_t)stream, pts, S, minmax, scale, codes, iota);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
int launch_fe_gather_seg(const float* pts, const FeSegs& S, int n_scans, int64_t max_n, const uint32_t* sorted,
                         void* stream) {
    if (n_scans <= 0 || n_scans > kFeSegMax || max_n <= 0) return n_scans == 0 ? LIVO_OK : LIVO_E_RANGE;
    hipLaunchKernelGGL(k_fe_gather_seg, dim3((unsigned)((max_n + 255) / 256), (unsigned)n_scans), dim3(256), 0,
                       (hipStream_t)stream, pts, S, sorted);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
int launch_to_world(const float* src, int64_t n, int stride, const int32_t* perm, const WorldParams& W, float* out5,
                    void* stream) {
    FE_LAUNCH(k_to_world, n, src, n, stride, perm, W, out5);
}
int launch_ori_flags(const uint8_t* sel, const int32_t* perm, int64_t n, uint32_t* flags, void* stream) {
    FE_LAUNCH(k_ori_flags, n, sel, perm, n, flags);
}
int launch_ori_scatter(const float* pts4, const float* normvec, const uint8_t* sel, const int32_t* perm,
                       const uint32_t* pos, int64_t n, float* ori3, float* corr4, void* stream) {
    FE_LAUNCH(k_ori_scatter, n, pts4, normvec, sel, perm, pos, n, ori3, corr4);
}
}  // namespace livo
