// vrun_lab.hip -- A/B harness for the vertex-run k-NN (development tool, not
// part of the product).  Search only (no plane pass), on the product's map
// layout: the same 5-NN list and e6 per query in every variant, timed with HIP
// events over `reps` launches.  Variants:
//   0  one query per lane, the lane's run read from global memory
//   1  one query per lane, the wave's distinct runs staged in LDS first
//      (coalesced cooperative copy), then each lane scans its run from LDS
//   2  as 0 with two queries per lane
#include "../../fast-livo-noted_amd/csrc/livo_kernels.hip"

#include <cstdio>
#include <vector>

using namespace livo;

namespace {
HostGridMap g_gm;
GridSlot* d_vslots = nullptr;
float4* d_vpts = nullptr;
uint32_t* d_vidx = nullptr;
float4* d_gpts = nullptr;
int g_vlog2 = 0;
int g_mode = 0;
float4* d_q = nullptr;
int64_t g_n = 0;
int32_t* d_idx = nullptr;  // 5 x n (SoA)
float* d_d = nullptr;
int32_t* d_flag = nullptr;
uint32_t* d_scn = nullptr;
unsigned long long* d_stat = nullptr;
hipStream_t g_st = nullptr;

struct LabP {
    const GridSlot* vslots;
    const float4* vpts;
    const uint32_t* vidx;
    const float4* gpts;
    const float4* q;
    int64_t n;
    float org[3], h;
    int vlog2;
    int mode;
    int32_t* idx;
    float* d;
    int32_t* flag;
    unsigned long long* stat;
    uint32_t* scn;  // run entries scanned per query
};

__device__ __forceinline__ void vr_cell(const LabP& P, float x, float y, float z, int v[3], float& dqv) {
    const float inv = 1.0f / P.h;
    const float q[3] = {x, y, z};
    float e[3];
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float t = (q[a] - P.org[a]) * inv;
        const float f = floorf(t);
        if (P.mode == 1) {
            v[a] = (int)f;
            e[a] = q[a] - (P.org[a] + ((float)v[a] + 0.5f) * P.h);
        } else {
            v[a] = (int)f + ((t - f < 0.5f) ? 0 : 1);
            e[a] = q[a] - (P.org[a] + (float)v[a] * P.h);
        }
    }
    dqv = sqrtf((e[0] * e[0] + e[1] * e[1]) + e[2] * e[2]);
}

__device__ __forceinline__ void vr_probe(const LabP& P, const int v[3], uint32_t& lo, uint32_t& cnt) {
    const unsigned long long key = grid_key_d(v[0], v[1], v[2]);
    const uint64_t mask = (1ull << P.vlog2) - 1ull;
    uint64_t sl = (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - P.vlog2));
    GridSlot g = P.vslots[sl];
    while (g.key != key && g.key != kGridEmpty) {
        sl = (sl + 1) & mask;
        g = P.vslots[sl];
    }
    lo = g.key == key ? g.start : 0u;
    cnt = g.key == key ? g.count : 0u;
}

__device__ __forceinline__ bool vr_cert(const LabP& P, const LeafQuery& q, const int v[3]) {
    const float t = lq_thr(q);
    if (!(t < INFINITY)) return false;
    const double rad = sqrt((double)t + 1e-9) * (1.0 + 1e-5) + 1e-6;
    const double ih = 1.0 / (double)P.h;
    const double q3[3] = {(double)q.qx, (double)q.qy, (double)q.qz};
    bool in = true;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const double l = floor((q3[a] - rad - (double)P.org[a]) * ih);
        const double hh = floor((q3[a] + rad - (double)P.org[a]) * ih);
        in = in && l >= (double)(v[a] - 1) && hh <= (double)(P.mode == 1 ? v[a] + 1 : v[a]);
    }
    return in;
}

__device__ __forceinline__ void vr_out(const LabP& P, int64_t i, const LeafQuery& q, bool cert) {
#pragma unroll
    for (int k = 0; k < kNN; k++) {
        P.idx[k * P.n + i] = (int32_t)__float_as_uint(P.gpts[q.nd[k]].w);
        P.d[k * P.n + i] = q.d[k];
    }
    P.flag[i] = cert ? 0 : 1;
}

// the run scan of one query (entries from `run`: global or LDS), as vrun_search
template <typename RunPtr>
__device__ __forceinline__ uint32_t vr_scan(LeafQuery& q, RunPtr run, const uint32_t* __restrict__ rid, uint32_t cnt,
                                            float dqv) {
    uint32_t k0 = 0;
#pragma unroll 1
    for (; k0 < cnt; k0 += 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = run[k0 + u];
        const float thr = lq_thr(q);
        if (thr < INFINITY && v[0].w > dqv + sqrtf(thr) * (1.0f + 1e-6f) + 1e-4f) break;
        float dist[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const float dx = q.qx - v[u].x, dy = q.qy - v[u].y, dz = q.qz - v[u].z;
            const float d = (dx * dx + dy * dy) + dz * dz;
            dist[u] = k0 + u < cnt ? d : INFINITY;
        }
        const float m = fminf(fminf(fminf(dist[0], dist[1]), fminf(dist[2], dist[3])),
                              fminf(fminf(dist[4], dist[5]), fminf(dist[6], dist[7])));
        if (m < q.e6) {
#pragma unroll
            for (int u = 0; u < 8; u++) lq_offer(q, dist[u], rid[k0 + u]);
        }
    }
    return min(k0, cnt);
}

__device__ __forceinline__ void lq_clear(LeafQuery& q, float4 p) {
#pragma unroll
    for (int k = 0; k < kNN; k++) { q.d[k] = INFINITY; q.nd[k] = 0u; }
    q.e6 = INFINITY;
    q.B = INFINITY;
    q.qx = p.x; q.qy = p.y; q.qz = p.z;
}

// variant 3/4: floors -- probe + output only (LIM 0) / at most LIM entries of the run
template <int LIM>
__global__ __launch_bounds__(256) void k_floor(LabP P) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= P.n) return;
    LeafQuery q;
    lq_clear(q, P.q[i]);
    int v[3];
    float dqv;
    vr_cell(P, q.qx, q.qy, q.qz, v, dqv);
    uint32_t lo, cnt;
    vr_probe(P, v, lo, cnt);
    uint32_t sc = 0;
    if (LIM > 0) sc = vr_scan(q, P.vpts + lo, P.vidx + lo, min(cnt, (uint32_t)LIM), dqv);
    else q.d[0] = (float)(lo + cnt);  // keep the probe live; nd stays 0 (a valid grid index)
    vr_out(P, i, q, true);
    P.scn[i] = sc;
}

__global__ __launch_bounds__(256) void k_v0(LabP P) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= P.n) return;
    LeafQuery q;
    lq_clear(q, P.q[i]);
    int v[3];
    float dqv;
    vr_cell(P, q.qx, q.qy, q.qz, v, dqv);
    uint32_t lo, cnt;
    vr_probe(P, v, lo, cnt);
    const uint32_t sc = vr_scan(q, P.vpts + lo, P.vidx + lo, cnt, dqv);
    const bool cert = vr_cert(P, q, v);
    vr_out(P, i, q, cert);
    P.scn[i] = sc;
}

template <int Q>
__global__ __launch_bounds__(256) void k_v2(LabP P) {
    const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * Q;
    if (i0 >= P.n) return;
    LeafQuery q[Q];
    int v[Q][3];
    float dqv[Q];
    uint32_t lo[Q], cnt[Q], k0[Q];
#pragma unroll
    for (int u = 0; u < Q; u++) {
        const int64_t i = min(i0 + u, P.n - 1);
        lq_clear(q[u], P.q[i]);
        vr_cell(P, q[u].qx, q[u].qy, q[u].qz, v[u], dqv[u]);
        vr_probe(P, v[u], lo[u], cnt[u]);
        k0[u] = 0;
    }
    // interleaved chunks of the Q runs
#pragma unroll 1
    while (true) {
        bool any = false;
#pragma unroll
        for (int u = 0; u < Q; u++) {
            if (k0[u] >= cnt[u]) continue;
            const float4* run = P.vpts + lo[u];
            float4 w[8];
#pragma unroll
            for (int r = 0; r < 8; r++) w[r] = run[k0[u] + r];
            const float thr = lq_thr(q[u]);
            if (thr < INFINITY && w[0].w > dqv[u] + sqrtf(thr) * (1.0f + 1e-6f) + 1e-4f) {
                k0[u] = cnt[u] + 8;  // done
                continue;
            }
            any = true;
            float dist[8];
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const float dx = q[u].qx - w[r].x, dy = q[u].qy - w[r].y, dz = q[u].qz - w[r].z;
                const float d = (dx * dx + dy * dy) + dz * dz;
                dist[r] = k0[u] + r < cnt[u] ? d : INFINITY;
            }
            const float m = fminf(fminf(fminf(dist[0], dist[1]), fminf(dist[2], dist[3])),
                                  fminf(fminf(dist[4], dist[5]), fminf(dist[6], dist[7])));
            if (m < q[u].e6) {
#pragma unroll
                for (int r = 0; r < 8; r++) lq_offer(q[u], dist[r], P.vidx[lo[u] + k0[u] + r]);
            }
            k0[u] += 8;
        }
        if (!any) break;
    }
#pragma unroll
    for (int u = 0; u < Q; u++) {
        if (i0 + u >= P.n) break;
        const bool cert = vr_cert(P, q[u], v[u]);
        vr_out(P, i0 + u, q[u], cert);
        P.scn[i0 + u] = min(k0[u], cnt[u]);
    }
}

// variant 1: the wave's distinct runs staged in LDS (up to kCap entries; runs
// that do not fit are scanned from global memory)
constexpr int kCap = 640;
__global__ __launch_bounds__(64) void k_v1(LabP P) {
    __shared__ float4 S[kCap + 8];
    __shared__ uint32_t SI[kCap + 8];
    __shared__ unsigned long long K[64];
    const int lane = threadIdx.x;
    const int64_t i = (int64_t)blockIdx.x * 64 + lane;
    const bool valid = i < P.n;
    LeafQuery q;
    lq_clear(q, P.q[valid ? i : 0]);
    int v[3];
    float dqv;
    vr_cell(P, q.qx, q.qy, q.qz, v, dqv);
    const unsigned long long key = grid_key_d(v[0], v[1], v[2]);
    // distinct vertices of the wave
    int my = -1, nd = 0;
    unsigned long long pend = __ballot(valid);
    while (pend) {
        const int L = __builtin_ctzll(pend);
        const unsigned long long k = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(key >> 32), L) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, L);
        const bool mine = ((pend >> lane) & 1ull) && key == k;
        if (mine) my = nd;
        if (lane == L) K[nd] = k;
        pend &= ~__ballot(mine);
        nd++;
    }
    __builtin_amdgcn_wave_barrier();
    // lane j resolves distinct vertex j
    uint32_t lo = 0, cnt = 0;
    if (lane < nd) {
        const unsigned long long kk = K[lane];
        const uint64_t mask = (1ull << P.vlog2) - 1ull;
        uint64_t sl = (uint64_t)((kk * 0x9E3779B97F4A7C15ull) >> (64 - P.vlog2));
        GridSlot g = P.vslots[sl];
        while (g.key != kk && g.key != kGridEmpty) {
            sl = (sl + 1) & mask;
            g = P.vslots[sl];
        }
        if (g.key == kk) { lo = g.start; cnt = g.count; }
    }
    uint32_t inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    const uint32_t exc = inc - cnt;
    const bool fits = inc <= (uint32_t)kCap;
    const unsigned long long fm = __ballot(fits && lane < nd);
    const int nf = fm == ~0ull ? 64 : __builtin_ctzll(~fm);
    const uint32_t total = nf > 0 ? __shfl(inc, nf - 1, 64) : 0u;
    // copy, every load in flight (binary search of the owner run)
#pragma unroll 1
    for (uint32_t p0 = 0; p0 < total; p0 += 4 * 64) {
        float4 w[4];
        uint32_t wi[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t p = p0 + (uint32_t)(64 * r + lane);
            int a = 0, b = nf - 1;
#pragma unroll
            for (int it = 0; it < 6; it++) {
                const int mid = (a + b + 1) >> 1;
                if (__shfl(exc, mid, 64) <= p) a = mid; else b = mid - 1;
            }
            const uint32_t src = __shfl(lo, a, 64) + (p - __shfl(exc, a, 64));
            if (p < total) { w[r] = P.vpts[src]; wi[r] = P.vidx[src]; }
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t p = p0 + (uint32_t)(64 * r + lane);
            if (p < total) { S[p] = w[r]; SI[p] = wi[r]; }
        }
    }
    __syncthreads();
    if (!valid) return;
    const uint32_t mlo = __shfl(lo, my, 64), mcnt = __shfl(cnt, my, 64), mexc = __shfl(exc, my, 64);
    const bool staged = my < nf;
    uint32_t sc;
    if (staged) sc = vr_scan(q, S + mexc, SI + mexc, mcnt, dqv);
    else sc = vr_scan(q, P.vpts + mlo, P.vidx + mlo, mcnt, dqv);
    const bool cert = vr_cert(P, q, v);
    vr_out(P, i, q, cert);
    P.scn[i] = sc;
}

LabP params() {
    LabP P{};
    P.vslots = d_vslots; P.vpts = d_vpts; P.vidx = d_vidx; P.gpts = d_gpts; P.q = d_q; P.n = g_n;
    for (int a = 0; a < 3; a++) P.org[a] = g_gm.org[a];
    P.h = g_gm.h; P.vlog2 = g_vlog2; P.mode = g_mode;
    P.idx = d_idx; P.d = d_d; P.flag = d_flag; P.stat = d_stat; P.scn = d_scn;
    return P;
}
}  // namespace

extern "C" {
int lab_build(const float* xyz, int64_t M, float ppc, int mode) {
    g_mode = mode;
    (void)hipFree(d_vslots); (void)hipFree(d_vpts); (void)hipFree(d_vidx); (void)hipFree(d_gpts);
    if (!g_st && hipStreamCreate(&g_st) != hipSuccess) return -1;
    free_grid_map(&g_gm);
    if (build_grid_map(xyz, M, 12, 0.f, &g_gm, ppc)) return -2;
    HostVertexRuns vr;
    if (build_vertex_runs(g_gm, &vr, mode)) return -3;
    const size_t vsb = ((size_t)1 << vr.log2_slots) * sizeof(GridSlot);
    (void)hipMalloc(&d_vslots, vsb);
    (void)hipMalloc(&d_vpts, (size_t)(vr.n + 8) * 16);
    (void)hipMalloc(&d_vidx, (size_t)(vr.n + 8) * 4);
    (void)hipMalloc(&d_gpts, (size_t)(M + 3) * 16);
    (void)hipMemcpy(d_vslots, vr.slots, vsb, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_vpts, vr.pts, (size_t)(vr.n + 8) * 16, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_vidx, vr.idx, (size_t)(vr.n + 8) * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_gpts, g_gm.pts, (size_t)(M + 3) * 16, hipMemcpyHostToDevice);
    g_vlog2 = vr.log2_slots;
    printf("grid h %.4f, vertex entries %lld, slots 2^%d\n", g_gm.h, (long long)vr.n, vr.log2_slots);
    free_vertex_runs(&vr);
    return 0;
}

int lab_queries(const float* q3, int64_t n) {
    std::vector<float> q((size_t)n * 4, 0.f);
    for (int64_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) q[4 * i + k] = q3[3 * i + k];
    (void)hipFree(d_q); (void)hipFree(d_idx); (void)hipFree(d_d); (void)hipFree(d_flag);
    (void)hipMalloc(&d_q, (size_t)n * 16);
    (void)hipMalloc(&d_idx, (size_t)n * 20);
    (void)hipMalloc(&d_d, (size_t)n * 20);
    (void)hipMalloc(&d_flag, (size_t)n * 4);
    (void)hipFree(d_scn);
    (void)hipMalloc(&d_scn, (size_t)n * 4);
    if (!d_stat) (void)hipMalloc(&d_stat, 16);
    (void)hipMemcpy(d_q, q.data(), (size_t)n * 16, hipMemcpyHostToDevice);
    g_n = n;
    return 0;
}

double lab_run(int variant, int reps, int32_t* idx, float* d, int32_t* flag, long long* stat) {
    LabP P = params();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    auto launch = [&]() {
        if (variant == 0) hipLaunchKernelGGL(k_v0, dim3((unsigned)((g_n + 255) / 256)), dim3(256), 0, g_st, P);
        else if (variant == 1) hipLaunchKernelGGL(k_v1, dim3((unsigned)((g_n + 63) / 64)), dim3(64), 0, g_st, P);
        else if (variant == 2) hipLaunchKernelGGL(k_v2<2>, dim3((unsigned)((g_n + 511) / 512)), dim3(256), 0, g_st, P);
        else if (variant == 3) hipLaunchKernelGGL(k_floor<0>, dim3((unsigned)((g_n + 255) / 256)), dim3(256), 0, g_st, P);
        else if (variant == 4) hipLaunchKernelGGL(k_floor<8>, dim3((unsigned)((g_n + 255) / 256)), dim3(256), 0, g_st, P);
        else hipLaunchKernelGGL(k_floor<16>, dim3((unsigned)((g_n + 255) / 256)), dim3(256), 0, g_st, P);
    };
    launch();
    (void)hipStreamSynchronize(g_st);
    (void)hipMemsetAsync(d_stat, 0, 16, g_st);
    (void)hipEventRecord(e0, g_st);
    for (int r = 0; r < reps; r++) launch();
    (void)hipEventRecord(e1, g_st);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(idx, d_idx, (size_t)g_n * 20, hipMemcpyDeviceToHost);
    (void)hipMemcpy(d, d_d, (size_t)g_n * 20, hipMemcpyDeviceToHost);
    (void)hipMemcpy(flag, d_flag, (size_t)g_n * 4, hipMemcpyDeviceToHost);
    std::vector<uint32_t> sc((size_t)g_n);
    (void)hipMemcpy(sc.data(), d_scn, (size_t)g_n * 4, hipMemcpyDeviceToHost);
    stat[0] = 0;
    for (auto x : sc) stat[0] += x;
    stat[1] = 0;
    for (int64_t k = 0; k < g_n; k++) stat[1] += flag[k] != 0;
    return ms / reps;
}
}
