// ivox_kernels.hip — CDNA4 (gfx950) kernels of the iVox backend and of
// map_incremental.
//
//   k_ivox_knn<LATER, BIG>  IVox::GetClosestPoint(pt, closest, max_num,
//                           max_range) (include/ivox3d/ivox3d.h:132-204) with
//                           IVoxNode::KNNPointByCondition (ivox3d_node.hpp:
//                           141-205) for every point of every scan: body->world
//                           (laser_mapping.cpp:662-671), the nearby grids in
//                           the reference's order, each grid's in-range points
//                           in insertion order, libstdc++'s nth_element
//                           restated (stl_select.h) so the survivors come out
//                           in the reference's order, one 128-B NNRec per point.
//                           One query per thread with a private candidate
//                           array; a query that outgrows it (a grid with more
//                           in-range points than kIvCap allows) is flagged and
//                           recomputed by the BIG pass on a global-memory slice.
//   k_iv_*                  IVox::AddPoints (ivox3d.h:256-281): grid keys
//                           (Pos2Grid, :283-286) inserted into the hash, then
//                           the CSR of grid runs rebuilt with the new points
//                           appended to their grid in input order.
//   k_map_incr              LaserMapping::map_incremental's per-point decision
//                           (laser_mapping.cpp:343-380).
//
// Numerics as livo_kernels.hip: -ffp-contract=off, correctly rounded f32
// division / sqrt, the reference's operation order (distance2 = Eigen's
// unrolled squaredNorm of a Vector3f: d0^2 + (d1^2 + d2^2)).
#include <hip/hip_runtime.h>
#include <math.h>

#include <cstdlib>
#include <cstring>

#include "device_common.h"
#include "livo_internal.h"
#include "wave_select.h"

namespace livo {

// NearbyType grids (ivox3d.h:211-235): NEARBY6 / 18 / 26 extend each other.
__constant__ int c_nearby[kIvMaxNearby][3] = {
    {0, 0, 0},   {-1, 0, 0}, {1, 0, 0},   {0, 1, 0},  {0, -1, 0},  {0, 0, -1}, {0, 0, 1},
    {1, 1, 0},   {-1, 1, 0}, {1, -1, 0},  {-1, -1, 0}, {1, 0, 1},  {-1, 0, 1}, {1, 0, -1},
    {-1, 0, -1}, {0, 1, 1},  {0, -1, 1},  {0, 1, -1}, {0, -1, -1}, {1, 1, 1},  {-1, 1, 1},
    {1, -1, 1},  {1, 1, -1}, {-1, -1, 1}, {-1, 1, -1}, {1, -1, -1}, {-1, -1, -1}};

__device__ __forceinline__ unsigned long long iv_key(int cx, int cy, int cz) {
    return (unsigned long long)(cx + kIvBias) | ((unsigned long long)(cy + kIvBias) << 21) |
           ((unsigned long long)(cz + kIvBias) << 42);
}
__device__ __forceinline__ uint64_t iv_hash(unsigned long long key, int log2) {
    return (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - log2));
}
// Pos2Grid on one axis: round(v * inv_resolution) (float product, half away
// from zero); false beyond `lim` cells (and for NaN).
__device__ __forceinline__ bool iv_cell(float v, float inv, float lim, int& c) {
    const float t = roundf(v * inv);
    if (!(fabsf(t) <= lim)) return false;
    c = (int)t;
    return true;
}
// The grid's run {start, count} or count = 0.
__device__ __forceinline__ uint2 iv_lookup(const GridSlot* __restrict__ slots, int log2, unsigned long long key) {
    const uint64_t mask = (1ull << log2) - 1ull;
    uint64_t sl = iv_hash(key, log2);
    GridSlot gs = slots[sl];
    while (gs.key != key && gs.key != kGridEmpty) {
        sl = (sl + 1) & mask;
        gs = slots[sl];
    }
    return gs.key == key ? make_uint2(gs.start, gs.count) : make_uint2(0u, 0u);
}

// ------------------------------------------------------------ search ----
// GetClosestPoint into a[0..n): false with n = 0 when no candidate (the
// caller's Nearest_Points entry then stays as it was, ivox3d.h:165-167);
// overflow when a grid's in-range points do not fit in `cap`.
template <class Arr>
__device__ __forceinline__ int iv_query(const IvoxParams& V, float qx, float qy, float qz, Arr& a, int cap,
                                        bool& overflow) {
    overflow = false;
    int kx, ky, kz;
    const float qlim = (float)(kIvMaxKey + 8);  // beyond: no stored grid within one cell
    if (!iv_cell(qx, V.inv_res, qlim, kx) || !iv_cell(qy, V.inv_res, qlim, ky) || !iv_cell(qz, V.inv_res, qlim, kz))
        return 0;
    const float4* __restrict__ pts = reinterpret_cast<const float4*>(V.pts);
    const int K = V.max_num;
    // the next grid's first hash slot is loaded while the current grid is
    // processed (probe chains are short: load factor <= 1/2)
    const uint64_t mask = (1ull << V.log2) - 1ull;
    auto key_of = [&](int t) {
        return iv_key(kx + c_nearby[t][0], ky + c_nearby[t][1], kz + c_nearby[t][2]);
    };
    unsigned long long nkey = key_of(0);
    uint64_t nsl = iv_hash(nkey, V.log2);
    GridSlot ngs = V.slots[nsl];
    int n = 0;
#pragma unroll 1
    for (int t = 0; t < V.nearby; t++) {
        const unsigned long long key = nkey;
        uint64_t sl = nsl;
        GridSlot gs = ngs;
        if (t + 1 < V.nearby) {
            nkey = key_of(t + 1);
            nsl = iv_hash(nkey, V.log2);
            ngs = V.slots[nsl];
        }
        while (gs.key != key && gs.key != kGridEmpty) {
            sl = (sl + 1) & mask;
            gs = V.slots[sl];
        }
        if (gs.key != key) continue;
        const uint2 run = make_uint2(gs.start, gs.count);
        const int old = n;
        // the grid's points 4 at a time (the CSR array is padded by 3 points):
        // four loads in flight instead of one dependent load per point
#pragma unroll 1
        for (uint32_t k0 = 0; k0 < run.y; k0 += 4) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = pts[run.x + k0 + u];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (k0 + u >= run.y) break;
                const float dx = v[u].x - qx, dy = v[u].y - qy, dz = v[u].z - qz;
                const float d = dx * dx + (dy * dy + dz * dz);  // distance2, ivox3d_node.hpp:12-16
                if ((double)d < V.range2) {
                    if (n >= cap) {
                        overflow = true;
                        return 0;
                    }
                    a[n] = SelElem{d, run.x + k0 + u};
                    n++;
                }
            }
        }
        // KNNPointByCondition (ivox3d_node.hpp:179-183)
        if (!(old + K >= n)) {
            sel_nth_element(a, old, old + K - 1, n);
            n = old + K;
        }
    }
    if (n == 0) return 0;
    if (n > K) {  // ivox3d.h:173-177
        sel_nth_element(a, 0, K - 1, n);
        n = K;
    }
    sel_nth_element(a, 0, 0, n);  // ivox3d.h:178
    return n;
}

template <class Arr>
__device__ __forceinline__ void iv_write(NNRec* __restrict__ out, const float4* __restrict__ pts, const Arr& a,
                                         int n) {
    float4* o4 = reinterpret_cast<float4*>(out);
    int32_t idx[kNN], node[kNN];
#pragma unroll
    for (int k = 0; k < kNN; k++) {
        float4 v = make_float4(0.f, 0.f, 0.f, INFINITY);
        idx[k] = -1;
        node[k] = -1;
        if (k < n) {
            const float4 p = pts[a[k].id];
            v = make_float4(p.x, p.y, p.z, a[k].d);
            idx[k] = __float_as_int(p.w);
            node[k] = (int32_t)a[k].id;
        }
        o4[k] = v;
    }
    int4* oi = reinterpret_cast<int4*>(out) + 5;
    oi[0] = make_int4(idx[0], idx[1], idx[2], idx[3]);
    oi[1] = make_int4(idx[4], n, 0, node[0]);
    oi[2] = make_int4(node[1], node[2], node[3], node[4]);
}

__device__ __forceinline__ void iv_world(const KnnParams& P, const IekfSlot* slot, const float4 b, float& qx,
                                         float& qy, float& qz) {
    if (P.identity) {
        qx = b.x; qy = b.y; qz = b.z;
    } else {
        world_point(slot->state.rot, slot->state.pos, P.R_LI, P.t_LI, b.x, b.y, b.z, qx, qy, qz);
    }
}

// LATER: an evaluation after the first (searches only where the scan's
// device-side nearest_search_en is set).  BIG: the overflow pass over the
// flagged queries (grid-stride, one global-memory slice per thread).
template <bool LATER>
__global__ __launch_bounds__(kKnnBlock) void k_ivox_knn(KnnParams P) {
    unsigned bjob, bx;
    xcd_block(P.nb, bjob, bx);
    const HsJob job = P.jobs[bjob];
    const IekfSlot* slot = job.slot;
    if (P.force >= 0) {
        if (!P.force) return;
    } else {
        if (slot->ctrl.stop) return;
        if (LATER && !slot->ctrl.search_en) return;
    }
    const int i = (int)bx * kKnnBlock + threadIdx.x;
    if (i >= job.n) return;
    const float4 b = reinterpret_cast<const float4*>(job.pts)[i];
    float qx, qy, qz;
    iv_world(P, slot, b, qx, qy, qz);
    SelElem a[kIvCap];
    bool overflow;
    const int n = iv_query(P.iv, qx, qy, qz, a, kIvCap, overflow);
    if (overflow) {
        const unsigned r = atomicAdd(P.replay_count2, 1u);
        P.replay_list2[r] = ((unsigned long long)bjob << 32) | (unsigned)i;
        return;
    }
    if (n > 0) iv_write(job.nn + i, reinterpret_cast<const float4*>(P.iv.pts), a, n);
}

// The queries no other search could hold (replay_list2: a grid of more points
// than the wave search can stage, which map_incremental builds near the sensor),
// one wave each: the streaming form of the wave search (grid by grid, each
// grid's in-range points staged after the survivors so far and cut to K by
// KNNPointByCondition's nth_element, ivox3d_node.hpp:179-183), with the list and
// the partition tables in LDS sized for the largest grid (nearby x K + that
// grid) and the looped wave-parallel nth_element (wave_nth_big).  A selection
// that exhausts introselect's depth limit (libstdc++ then heap-selects) redoes
// the query with the per-thread search in the wave's global-memory slice.
// Used when the list fits in 64 KB of LDS (12 B an entry).
constexpr int kBigEntryBytes = 12;  // float + uint32 + two uint16 table entries
__global__ __launch_bounds__(64) void k_ivox_knn_big_wave(KnnParams P) {
    extern __shared__ uint32_t big_lds[];
    const int lane = threadIdx.x;
    const IvoxParams& V = P.iv;
    const int cap = (int)V.slice;
    const BigList L{reinterpret_cast<float*>(big_lds), big_lds + cap, reinterpret_cast<uint16_t*>(big_lds + 2 * cap),
                    reinterpret_cast<uint16_t*>(big_lds + 2 * cap) + cap};
    const float4* __restrict__ pts = reinterpret_cast<const float4*>(V.pts);
    const int K = V.max_num;
    const unsigned cnt = *P.replay_count2;
    for (unsigned r = blockIdx.x; r < cnt; r += gridDim.x) {  // (wave-uniform)
        const unsigned long long e = P.replay_list2[r];
        const unsigned bjob = (unsigned)(e >> 32);
        const int i = (int)(e & 0xFFFFFFFFu);
        const HsJob job = P.jobs[bjob];
        const float4 b = reinterpret_cast<const float4*>(job.pts)[i];
        float qx, qy, qz;
        iv_world(P, job.slot, b, qx, qy, qz);
        int kx, ky, kz;
        const float qlim = (float)(kIvMaxKey + 8);
        if (!iv_cell(qx, V.inv_res, qlim, kx) || !iv_cell(qy, V.inv_res, qlim, ky) || !iv_cell(qz, V.inv_res, qlim, kz))
            continue;  // no grid within reach: the cache stays
        uint2 run = make_uint2(0u, 0u);
        if (lane < V.nearby)
            run = iv_lookup(V.slots, V.log2, iv_key(kx + c_nearby[lane][0], ky + c_nearby[lane][1], kz + c_nearby[lane][2]));
        int n = 0;
        bool ok = true;
#pragma unroll 1
        for (int t = 0; t < V.nearby && ok; t++) {
            const uint32_t c = __shfl(run.y, t, 64), st = __shfl(run.x, t, 64);
            const int old = n;
#pragma unroll 1
            for (uint32_t k0 = 0; k0 < c && ok; k0 += 64) {
                const uint32_t k = k0 + lane;
                bool in = false;
                float d = 0.f;
                if (k < c) {
                    const float4 v = pts[st + k];
                    const float dx = v.x - qx, dy = v.y - qy, dz = v.z - qz;
                    d = dx * dx + (dy * dy + dz * dz);  // distance2, ivox3d_node.hpp:12-16
                    in = (double)d < V.range2;
                }
                const unsigned long long m = __ballot(in);
                if (n + __popcll(m) > cap) {
                    ok = false;  // (cannot happen: cap >= nearby x K + the largest grid)
                } else {
                    if (in) {
                        const int pos = n + lanes_below(m, lane);
                        L.d[pos] = d;
                        L.id[pos] = st + k;
                    }
                    n += __popcll(m);
                }
            }
            wave_sync();
            if (ok && n - old > K) {
                ok = wave_nth_big(L, old, old + K - 1, n, lane);
                n = old + K;
            }
        }
        if (ok && n == 0) continue;  // no candidate: the cache stays
        if (ok && n > K) {  // ivox3d.h:173-177
            ok = wave_nth_big(L, 0, K - 1, n, lane);
            n = K;
        }
        if (ok) ok = wave_nth_big(L, 0, 0, n, lane);  // ivox3d.h:178
        if (ok) {
            // the record: lanes 0..4 the points, lane 0 the indices (as wave_write)
            NNRec* out = job.nn + i;
            const uint32_t myid = lane < n ? L.id[lane] : 0u;
            const float myd = lane < n ? L.d[lane] : INFINITY;
            int32_t pidx = -1;
            if (lane < kNN) {
                float4 v = make_float4(0.f, 0.f, 0.f, INFINITY);
                if (lane < n) {
                    const float4 pp = pts[myid];
                    v = make_float4(pp.x, pp.y, pp.z, myd);
                    pidx = __float_as_int(pp.w);
                }
                reinterpret_cast<float4*>(out)[lane] = v;
            }
            const int32_t node = lane < n ? (int32_t)myid : -1;
            int32_t ix[kNN], nd[kNN];
#pragma unroll
            for (int q = 0; q < kNN; q++) {
                ix[q] = __shfl(pidx, q, 64);
                nd[q] = __shfl(node, q, 64);
            }
            if (lane == 0) {
                int4* oi = reinterpret_cast<int4*>(out) + 5;
                oi[0] = make_int4(ix[0], ix[1], ix[2], ix[3]);
                oi[1] = make_int4(ix[4], n, 0, nd[0]);
                oi[2] = make_int4(nd[1], nd[2], nd[3], nd[4]);
            }
        } else if (lane == 0) {  // the depth limit ran out: the exact per-thread search in global memory
            SelElem* a = V.scratch + (int64_t)blockIdx.x * V.slice;
            bool overflow;
            const int nn = iv_query(V, qx, qy, qz, a, cap, overflow);
            if (overflow) atomicOr(V.ctr, 2ull);
            else if (nn > 0) iv_write(job.nn + i, pts, a, nn);
        }
        wave_sync();  // (the list is reused by the next query)
    }
}

// The exact global-memory pass over the queries no other search could hold
// (replay_list2): one query per thread, its candidates in a private slice.
__global__ __launch_bounds__(64) void k_ivox_knn_big(KnnParams P) {
    const unsigned cnt = *P.replay_count2;
    const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
    SelElem* a = P.iv.scratch + (int64_t)tid * P.iv.slice;
    for (unsigned r = tid; r < cnt; r += gridDim.x * blockDim.x) {
        const unsigned long long e = P.replay_list2[r];
        const unsigned bjob = (unsigned)(e >> 32);
        const int i = (int)(e & 0xFFFFFFFFu);
        const HsJob job = P.jobs[bjob];
        const float4 b = reinterpret_cast<const float4*>(job.pts)[i];
        float qx, qy, qz;
        iv_world(P, job.slot, b, qx, qy, qz);
        bool overflow;
        const int n = iv_query(P.iv, qx, qy, qz, a, (int)P.iv.slice, overflow);
        if (overflow) {  // cannot happen: slice >= nearby * max_num + the largest grid
            atomicOr(P.iv.ctr, 2ull);
            continue;
        }
        if (n > 0) iv_write(job.nn + i, reinterpret_cast<const float4*>(P.iv.pts), a, n);
    }
}


// ------------------------------------------------- wave-cooperative search --
// One query per wave.  The nearby grids are probed by one lane each, their
// points loaded at once (<= kWRaw per query, 8 per lane), the in-range ones
// staged in LDS in the reference's push order (grid by grid, insertion order),
// and every std::nth_element of GetClosestPoint is run by the whole wave:
// libstdc++'s unguarded Hoare partition computed in parallel (grp_nth,
// wave_select.h: the swap pairs Lo[k] <-> Ro[k], k < k*, from two LDS tables of
// ballot ranks; the final insertion sort of <= 3 elements on lane 0).  A query with
// more than kWRaw raw points streams grid by grid instead (each grid truncated
// right away, as the reference does); one whose grids are too large even for
// that, or whose introselect exhausts its depth limit (libstdc++ then switches
// to a heap select), goes to the global-memory pass.
// NNRec from the wave's first n (<= 5) list entries: lanes 0..4 the points, lane 0 the indices.
__device__ __forceinline__ void wave_write(NNRec* __restrict__ out, const float4* __restrict__ pts, const WaveLds& L,
                                           int n, int lane) {
    float4* o4 = reinterpret_cast<float4*>(out);
    const uint32_t myid = lane < n ? L.id[lane] : 0u;
    const float myd = lane < n ? L.d[lane] : INFINITY;
    int32_t pidx = -1;
    if (lane < kNN) {
        float4 v = make_float4(0.f, 0.f, 0.f, INFINITY);
        if (lane < n) {
            const float4 pp = pts[myid];
            v = make_float4(pp.x, pp.y, pp.z, myd);
            pidx = __float_as_int(pp.w);
        }
        o4[lane] = v;
    }
    const int32_t node = lane < n ? (int32_t)myid : -1;
    const int32_t i0 = __shfl(pidx, 0, 64), i1 = __shfl(pidx, 1, 64), i2 = __shfl(pidx, 2, 64),
                  i3 = __shfl(pidx, 3, 64), i4 = __shfl(pidx, 4, 64);
    const int32_t n0 = __shfl(node, 0, 64), n1 = __shfl(node, 1, 64), n2 = __shfl(node, 2, 64),
                  n3 = __shfl(node, 3, 64), n4 = __shfl(node, 4, 64);
    if (lane == 0) {
        int4* oi = reinterpret_cast<int4*>(out) + 5;
        oi[0] = make_int4(i0, i1, i2, i3);
        oi[1] = make_int4(i4, n, 0, n0);
        oi[2] = make_int4(n1, n2, n3, n4);
    }
}

// One query (point i of job) by the whole wave: the record written (or the
// cache left as it is when no candidate is in range); true when it needs the
// exact global-memory pass (a grid too large even for streaming, or an
// introselect that exhausted its depth limit).
__device__ __forceinline__ bool ivox_wave_query(const KnnParams& P, const HsJob& job, const IekfSlot* slot, int i,
                                                WaveLds& L, int lane) {
    const IvoxParams& V = P.iv;
    const float4 b = reinterpret_cast<const float4*>(job.pts)[i];
    float qx, qy, qz;
    iv_world(P, slot, b, qx, qy, qz);
    int kx, ky, kz;
    const float qlim = (float)(kIvMaxKey + 8);
    if (!iv_cell(qx, V.inv_res, qlim, kx) || !iv_cell(qy, V.inv_res, qlim, ky) || !iv_cell(qz, V.inv_res, qlim, kz))
        return false;  // no grid within reach: nothing found, the cache stays
    // one nearby grid per lane
    uint2 run = make_uint2(0u, 0u);
    if (lane < V.nearby)
        run = iv_lookup(V.slots, V.log2, iv_key(kx + c_nearby[lane][0], ky + c_nearby[lane][1], kz + c_nearby[lane][2]));
    uint32_t incl = run.y;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
    }
    const uint32_t R = __shfl(incl, 63, 64);
    const uint32_t excl = incl - run.y;
    const int K = V.max_num;
    const float4* __restrict__ pts = reinterpret_cast<const float4*>(V.pts);
    if (R > (uint32_t)kWRaw) {
        // streaming: grid by grid, each truncated to K right away as the
        // reference does, so only 5 per grid + one grid's points are staged
        int n = 0;
        bool ok = true;
#pragma unroll 1
        for (int tt = 0; tt < V.nearby && ok; tt++) {
            const uint32_t c = __shfl(run.y, tt, 64), st = __shfl(run.x, tt, 64);
            const int old = n;
#pragma unroll 1
            for (uint32_t k0 = 0; k0 < c && ok; k0 += 64) {
                const uint32_t k = k0 + lane;
                bool in = false;
                float d = 0.f;
                if (k < c) {
                    const float4 v = pts[st + k];
                    const float dx = v.x - qx, dy = v.y - qy, dz = v.z - qz;
                    d = dx * dx + (dy * dy + dz * dz);
                    in = (double)d < V.range2;
                }
                const unsigned long long m = __ballot(in);
                if (n + __popcll(m) > kWRaw) {
                    ok = false;
                } else {
                    if (in) {
                        const int pos = n + lanes_below(m, lane);
                        L.d[pos] = d;
                        L.id[pos] = st + k;
                    }
                    n += __popcll(m);
                }
            }
            wave_sync();
            if (ok && n - old > K) {
                ok = wave_nth(L, old, old + K - 1, n, lane);
                n = old + K;
            }
        }
        if (ok && n == 0) return false;  // no candidate: the cache stays
        if (ok && n > K) {
            ok = wave_nth(L, 0, K - 1, n, lane);
            n = K;
        }
        if (ok) ok = wave_nth(L, 0, 0, n, lane);
        if (ok) {
            wave_write(job.nn + i, pts, L, n, lane);
            return false;
        }
        return true;  // a grid too large even for streaming, or a heap select
    }
    if (lane <= kIvMaxNearby) L.m[lane] = 0u;
    // every raw point at once (raw index g = 64 r + lane, in grid order)
    float dist[kWRounds];
    uint32_t pid[kWRounds];
    int gnode[kWRounds];
    bool inr[kWRounds];
#pragma unroll
    for (int r = 0; r < kWRounds; r++) {
        const uint32_t g = 64u * r + lane;
        int t = 0;
#pragma unroll 1
        for (int tt = 0; tt < V.nearby; tt++) {
            const uint32_t e = __shfl(excl, tt, 64), c = __shfl(run.y, tt, 64);
            if (g >= e && g < e + c) t = tt;
        }
        const uint32_t st = __shfl(run.x, t, 64), e = __shfl(excl, t, 64);
        gnode[r] = t;
        pid[r] = st + (g - e);
        inr[r] = false;
        dist[r] = 0.f;
        if (g < R) {
            const float4 v = pts[pid[r]];
            const float dx = v.x - qx, dy = v.y - qy, dz = v.z - qz;
            dist[r] = dx * dx + (dy * dy + dz * dz);  // distance2, ivox3d_node.hpp:12-16
            inr[r] = (double)dist[r] < V.range2;
        }
    }
    wave_sync();
    // stage the in-range points in push order (ivox3d_node.hpp:154-164)
    int base = 0;
#pragma unroll
    for (int r = 0; r < kWRounds; r++) {
        const unsigned long long m = __ballot(inr[r]);
        if (inr[r]) {
            const int pos = base + lanes_below(m, lane);
            L.d[pos] = dist[r];
            L.id[pos] = pid[r];
            L.node[pos] = (uint8_t)gnode[r];
            atomicAdd(&L.m[gnode[r]], 1u);
        }
        base += __popcll(m);
    }
    wave_sync();
#ifdef LIVO_IV_DEBUG_Q
#define IVDBG(tag, cnt)                                                                        \
    if (i == LIVO_IV_DEBUG_Q && lane == 0) {                                                   \
        printf("%s n=%d:", tag, (int)(cnt));                                                   \
        for (int z = 0; z < (int)(cnt); z++) printf(" (%.8f,%u,%d)", L.d[z], L.id[z], (int)L.node[z]); \
        printf("\n");                                                                           \
    }
#else
#define IVDBG(tag, cnt)
#endif
    IVDBG("staged", base);
    if (base == 0) return false;  // no candidate: the reference returns false, the cache stays
    // per grid: KNNPointByCondition's nth_element on its own run (ivox3d_node.hpp:179-183)
    const uint32_t mt = lane < V.nearby ? L.m[lane] : 0u;
    uint32_t s_incl = mt;
    uint32_t k_incl = min(mt, (uint32_t)K);
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(s_incl, off, 64), u = __shfl_up(k_incl, off, 64);
        if (lane >= off) {
            s_incl += v;
            k_incl += u;
        }
    }
    const uint32_t S = s_incl - mt;                      // the grid's staged segment start
    const uint32_t O = k_incl - min(mt, (uint32_t)K);    // its survivors' start in the final list
    const int n_final = (int)__shfl(k_incl, 63, 64);
    bool ok = true;
#pragma unroll 1
    for (int tt = 0; tt < V.nearby && ok; tt++) {
        const int m = (int)__shfl(mt, tt, 64);
        if (m > K) {
            const int s0 = (int)__shfl(S, tt, 64);
            ok = wave_nth(L, s0, s0 + K - 1, s0 + m, lane);
            IVDBG("pernode", base);
        }
    }
    if (ok) {
        // survivors: the first min(m, K) of each grid's segment, in grid order
        float cd[kWRounds];
        uint32_t cid[kWRounds];
        int dst[kWRounds];
#pragma unroll
        for (int r = 0; r < kWRounds; r++) {
            const int p = 64 * r + lane;
            // shuffles outside the branch: ds_bpermute reads 0 from inactive lanes
            const int t = p < base ? L.node[p] : 0;
            const int s0 = (int)__shfl(S, t, 64), o0 = (int)__shfl(O, t, 64);
            dst[r] = -1;
            if (p < base) {
                cd[r] = L.d[p];
                cid[r] = L.id[p];
                if (p - s0 < K) dst[r] = o0 + (p - s0);
            }
        }
        wave_sync();
#pragma unroll
        for (int r = 0; r < kWRounds; r++)
            if (dst[r] >= 0) {
                L.d[dst[r]] = cd[r];
                L.id[dst[r]] = cid[r];
            }
        wave_sync();
        IVDBG("compact", n_final);
        int n = n_final;
        if (n > K) {  // ivox3d.h:173-177
            ok = wave_nth(L, 0, K - 1, n, lane);
            n = K;
        }
        IVDBG("nth4", n);
        if (ok) ok = wave_nth(L, 0, 0, n, lane);  // ivox3d.h:178
        IVDBG("final", n);
        if (ok) {
            wave_write(job.nn + i, pts, L, n, lane);
            return false;
        }
    }
    // the depth limit ran out (libstdc++ would heap-select): the exact global-memory pass
    return true;
}

template <bool LATER>
__global__ __launch_bounds__(64 * kWaves) void k_ivox_knn_wave(KnnParams P) {
    __shared__ WaveLds lds[kWaves];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    WaveLds& L = lds[w];
    unsigned bjob, bx;
    xcd_block(P.nb, bjob, bx);
    const HsJob job = P.jobs[bjob];
    const IekfSlot* slot = job.slot;
    if (P.force >= 0) {
        if (!P.force) return;
    } else {
        if (slot->ctrl.stop) return;
        if (LATER && !slot->ctrl.search_en) return;
    }
    const int i = (int)bx * kWaves + w;
    if (i >= job.n) return;
    if (ivox_wave_query(P, job, slot, i, L, lane) && lane == 0) {
        const unsigned r = atomicAdd(P.replay_count2, 1u);
        P.replay_list2[r] = ((unsigned long long)bjob << 32) | (unsigned)i;
    }
}

// The team search's overflow (replay_list: a list past kIvTeamCap entries), one
// query per wave, grid-stride: a single 16-lane team cannot hold it, the wave's
// LDS list (kWRaw raw points, streaming past that) can; what it cannot either
// goes on to the global-memory pass.  (Before this pass every overflow query ran
// on one thread of k_ivox_knn_big: ~0.6 ms per launch on a grown map, the long
// pole of a single-scan iVox update.)
__global__ __launch_bounds__(64 * kWaves) void k_ivox_knn_wave_list(KnnParams P) {
    __shared__ WaveLds lds[kWaves];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    WaveLds& L = lds[w];
    const unsigned cnt = *P.replay_count;
    for (unsigned r = blockIdx.x * kWaves + w; r < cnt; r += gridDim.x * kWaves) {  // (wave-uniform)
        const unsigned long long e = P.replay_list[r];
        const unsigned bjob = (unsigned)(e >> 32);
        const int i = (int)(e & 0xFFFFFFFFu);
        const HsJob job = P.jobs[bjob];
        if (ivox_wave_query(P, job, job.slot, i, L, lane) && lane == 0) {
            const unsigned q = atomicAdd(P.replay_count2, 1u);
            P.replay_list2[q] = e;
        }
        wave_sync();  // (L reused by the next entry)
    }
}

// ------------------------------------------------------- team search ----
// One query per 16-lane team (4 per wave, 16 per 256-thread block), the list
// in LDS (kIvTeamCap SelElems = 1 KB per team): the team probes the nearby
// grids (a lane each) and loads each grid's points together (16 at a time);
// the in-range ones are appended to the list in push order (ivox3d_node.hpp:
// 154-164), and the team's lane 0 runs every std::nth_element exactly as the
// per-thread search does (stl_select.h) on the LDS list.  No private
// candidate array (k_ivox_knn's lives in scratch: ~1 KB a thread), and 16x
// fewer lanes per query than the wave search.  A query whose list would
// outgrow the capacity goes to the global-memory pass (k_ivox_knn_big).
constexpr int kIvTeam = 16;
// list capacity per team: a query's list holds <= K survivors of every grid before
// the current one plus all of the current grid's in-range points, so 18 x 5 + the
// largest grid; 128 overflowed (to the wave pass) once map_incremental had grown
// grids past ~38 points (32 KB of LDS per block: 5 blocks per CU)
#ifndef LIVO_IV_TEAM_CAP
#define LIVO_IV_TEAM_CAP 128
#endif
constexpr int kIvTeamCap = LIVO_IV_TEAM_CAP;
__device__ __forceinline__ uint32_t team_bits(unsigned long long m, int lane) {
    return (uint32_t)(m >> (lane & 48)) & 0xFFFFu;
}
// LIVO_IV_TEAM_NTH=1: the selections by the whole team (team_nth, wave_select.h);
// 0: by the team's lane 0 (sel_nth_element), as round 6 first did.
#ifndef LIVO_IV_TEAM_NTH
#define LIVO_IV_TEAM_NTH 1
#endif
// segments shorter than this stay on lane 0 (sel_nth_element)
#ifndef LIVO_IV_TEAM_NTH_MIN
#define LIVO_IV_TEAM_NTH_MIN 0
#endif
static_assert(kIvTeam == kTeamLanes && kIvTeamCap <= 256, "team_nth runs on the search team, byte tables");
template <bool LATER>
__global__ __launch_bounds__(256) void k_ivox_knn_team(KnnParams P) {
    __shared__ SelElem lst[256 / kIvTeam][kIvTeamCap];
#if LIVO_IV_TEAM_NTH
    __shared__ uint8_t tabs[256 / kIvTeam][2][kIvTeamCap];
#endif
    const int lane = threadIdx.x & 63, tl = threadIdx.x & (kIvTeam - 1), team = threadIdx.x / kIvTeam;
    SelElem* L = lst[team];
#if LIVO_IV_TEAM_NTH
    uint8_t* const lt = tabs[team][0];
    uint8_t* const rt = tabs[team][1];
#define IV_TEAM_NTH(f, k, l)                                      \
    do {                                                          \
        if ((l) - (f) >= LIVO_IV_TEAM_NTH_MIN)                    \
            team_nth(L, lt, rt, f, k, l, tl, lane);               \
        else if (tl == 0)                                         \
            sel_nth_element(L, f, k, l);                          \
    } while (0)
#else
#define IV_TEAM_NTH(f, k, l) \
    do {                     \
        if (tl == 0) sel_nth_element(L, f, k, l); \
    } while (0)
#endif
    unsigned bjob, bx;
    xcd_block(P.nb, bjob, bx);
    const HsJob job = P.jobs[bjob];
    const IekfSlot* slot = job.slot;
    if (P.force >= 0) {
        if (!P.force) return;
    } else {
        if (slot->ctrl.stop) return;  // block-uniform
        if (LATER && !slot->ctrl.search_en) return;
    }
    const int i = (int)bx * (256 / kIvTeam) + team;
    if (i >= job.n) return;  // team-uniform
    const IvoxParams& V = P.iv;
    const float4 b = reinterpret_cast<const float4*>(job.pts)[i];
    float qx, qy, qz;
    iv_world(P, slot, b, qx, qy, qz);
    int kx, ky, kz;
    const float qlim = (float)(kIvMaxKey + 8);
    if (!iv_cell(qx, V.inv_res, qlim, kx) || !iv_cell(qy, V.inv_res, qlim, ky) || !iv_cell(qz, V.inv_res, qlim, kz))
        return;  // no grid within reach: nothing found, the cache stays
    // the nearby grids' runs: grid t on lane t % 16 (two per lane for t >= 16)
    uint2 r0 = make_uint2(0u, 0u), r1 = make_uint2(0u, 0u);
    if (tl < V.nearby)
        r0 = iv_lookup(V.slots, V.log2, iv_key(kx + c_nearby[tl][0], ky + c_nearby[tl][1], kz + c_nearby[tl][2]));
    if (tl + kIvTeam < V.nearby) {
        const int t = tl + kIvTeam;
        r1 = iv_lookup(V.slots, V.log2, iv_key(kx + c_nearby[t][0], ky + c_nearby[t][1], kz + c_nearby[t][2]));
    }
    const float4* __restrict__ pts = reinterpret_cast<const float4*>(V.pts);
    const int K = V.max_num;
    const int tb = lane & 48;  // the team's first lane in the wave
    int n = 0;
    bool ok = true;
#pragma unroll 1
    for (int t = 0; t < V.nearby; t++) {
        const int src = tb + (t & (kIvTeam - 1));
        const uint32_t st = (uint32_t)__shfl((int)(t < kIvTeam ? r0.x : r1.x), src, 64);
        const uint32_t c = (uint32_t)__shfl((int)(t < kIvTeam ? r0.y : r1.y), src, 64);
        if (c == 0u) continue;  // team-uniform
        const int old = n;
#pragma unroll 1
        for (uint32_t k0 = 0; k0 < c; k0 += kIvTeam) {
            const uint32_t k = k0 + (uint32_t)tl;
            bool in = false;
            float d = 0.f;
            if (k < c) {
                const float4 v = pts[st + k];
                const float dx = v.x - qx, dy = v.y - qy, dz = v.z - qz;
                d = dx * dx + (dy * dy + dz * dz);  // distance2, ivox3d_node.hpp:12-16
                in = (double)d < V.range2;
            }
            const uint32_t m = team_bits(__ballot(in), lane);
            if (n + __popc(m) > kIvTeamCap) {
                ok = false;
                break;
            }
            if (in) L[n + __popc(m & ((1u << tl) - 1u))] = SelElem{d, st + k};
            n += __popc(m);
        }
        if (!ok) break;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // KNNPointByCondition (ivox3d_node.hpp:179-183) on the grid's segment
        if (n - old > K) {  // (team-uniform)
            IV_TEAM_NTH(old, old + K - 1, n);
            n = old + K;
        }
    }
    if (!ok) {  // a list beyond the team's capacity: the exact global-memory pass
        if (tl == 0) {
            const unsigned r = atomicAdd(P.replay_count, 1u);
            P.replay_list[r] = ((unsigned long long)bjob << 32) | (unsigned)i;
        }
        return;
    }
    if (n == 0) return;  // no candidate: the reference returns false, the cache stays
    if (n > K) IV_TEAM_NTH(0, K - 1, n);  // ivox3d.h:173-177
    n = n > K ? K : n;
    IV_TEAM_NTH(0, 0, n);  // ivox3d.h:178
#undef IV_TEAM_NTH
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // the record: lanes 0..4 of the team the points, lane 0 the indices
    NNRec* out = job.nn + i;
    SelElem e = tl < n ? L[tl] : SelElem{INFINITY, 0u};
    float4 pv = make_float4(0.f, 0.f, 0.f, INFINITY);
    int32_t pidx = -1, node = -1;
    if (tl < n) {
        const float4 p = pts[e.id];
        pv = make_float4(p.x, p.y, p.z, e.d);
        pidx = __float_as_int(p.w);
        node = (int32_t)e.id;
    }
    if (tl < kNN) reinterpret_cast<float4*>(out)[tl] = pv;
    int32_t ix[kNN], nd[kNN];
#pragma unroll
    for (int k = 0; k < kNN; k++) {
        ix[k] = __shfl(pidx, tb + k, 64);
        nd[k] = __shfl(node, tb + k, 64);
    }
    if (tl == 0) {
        int4* oi = reinterpret_cast<int4*>(out) + 5;
        oi[0] = make_int4(ix[0], ix[1], ix[2], ix[3]);
        oi[1] = make_int4(ix[4], n, 0, nd[0]);
        oi[2] = make_int4(nd[1], nd[2], nd[3], nd[4]);
    }
}

#ifndef LIVO_IV_WLIST_BLOCKS
#define LIVO_IV_WLIST_BLOCKS 4096
#endif
// Kernel choice per launch: the team search (16 lanes a query, list in LDS) by
// default; the wave-cooperative search (a query per wave) for launches of at
// most LIVO_IVOX_WAVE_MAX queries (default 0: never; a 100k-point scan alone
// is throughput-bound too); the one-query-per-thread search (private candidate
// array, in scratch) is kept as a reference.  IvoxParams::kind >= 0 (LIVO_IVOX_KIND
// = thread | wave | team at livo_ivox_init) forces one.
static int ivox_kind(const IvoxParams& V, int64_t queries) {
    static const int64_t wave_max = [] {
        const char* e = std::getenv("LIVO_IVOX_WAVE_MAX");
        return e ? (int64_t)std::atoll(e) : (int64_t)0;
    }();
    if (V.kind >= 0) return V.kind;
    return queries <= wave_max ? 1 : 2;
}

int launch_ivox_knn(const KnnParams& p, int n_jobs, int64_t max_n, bool later, int64_t overflow_threads,
                    void* stream) {
    if (n_jobs <= 0 || max_n <= 0) return LIVO_OK;
    KnnParams q = p;
    const int kind = ivox_kind(p.iv, (int64_t)n_jobs * max_n);
    if (kind == 2) {
        q.nb = (int32_t)((max_n + (256 / kIvTeam) - 1) / (256 / kIvTeam));
        if ((int64_t)q.nb * n_jobs >= (1ll << 31)) return LIVO_E_RANGE;
        const dim3 grid((unsigned)(q.nb * n_jobs)), block(256);
        if (later)
            hipLaunchKernelGGL((k_ivox_knn_team<true>), grid, block, 0, (hipStream_t)stream, q);
        else
            hipLaunchKernelGGL((k_ivox_knn_team<false>), grid, block, 0, (hipStream_t)stream, q);
    } else if (kind == 0) {
        q.nb = (int32_t)((max_n + kKnnBlock - 1) / kKnnBlock);
        if ((int64_t)q.nb * n_jobs >= (1ll << 31)) return LIVO_E_RANGE;
        const dim3 grid((unsigned)(q.nb * n_jobs)), block(kKnnBlock);
        if (later)
            hipLaunchKernelGGL((k_ivox_knn<true>), grid, block, 0, (hipStream_t)stream, q);
        else
            hipLaunchKernelGGL((k_ivox_knn<false>), grid, block, 0, (hipStream_t)stream, q);
    } else {
        q.nb = (int32_t)((max_n + kWaves - 1) / kWaves);
        if ((int64_t)q.nb * n_jobs >= (1ll << 31)) return LIVO_E_RANGE;
        const dim3 grid((unsigned)(q.nb * n_jobs)), block(64 * kWaves);
        if (later)
            hipLaunchKernelGGL((k_ivox_knn_wave<true>), grid, block, 0, (hipStream_t)stream, q);
        else
            hipLaunchKernelGGL((k_ivox_knn_wave<false>), grid, block, 0, (hipStream_t)stream, q);
    }
    if (hipGetLastError() != hipSuccess) return LIVO_E_HIP;
    // A list holds at most (nearby - 1) x K survivors + one grid's points <= slice - 8
    // (slice: nearby x K + the largest grid + 8, grown with the map, never shrunk):
    // when that fits the team's capacity no team search overflows, and the team
    // search resolves its own depth-limit cases, so the overflow passes have no work.
    if (kind == 2 && q.iv.slice - 8 <= kIvTeamCap) return LIVO_OK;
    if (kind == 2)  // the team search's overflow, one query per wave (grid-stride; blocks past the list exit)
        hipLaunchKernelGGL(k_ivox_knn_wave_list, dim3(LIVO_IV_WLIST_BLOCKS), dim3(64 * kWaves), 0, (hipStream_t)stream, q);
    const size_t lds = (size_t)q.iv.slice * kBigEntryBytes;
    // (the global slices of the depth-limit fallback: one per block, within the
    // group's big_threads slices)
    const unsigned wblocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, overflow_threads));
    if (lds <= 65536) {
        hipLaunchKernelGGL(k_ivox_knn_big_wave, dim3(wblocks), dim3(64), lds, (hipStream_t)stream, q);
    } else {
        const unsigned blocks = (unsigned)std::max<int64_t>(1, overflow_threads / 64);
        hipLaunchKernelGGL(k_ivox_knn_big, dim3(blocks), dim3(64), 0, (hipStream_t)stream, q);
    }
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

// --------------------------------------------------------- AddPoints ----
__global__ void k_iv_clear(GridSlot* slots, int64_t table) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s < table) slots[s] = GridSlot{kGridEmpty, 0u, 0u};
}

// Each point's grid key found or inserted (CAS on the key); new grids counted.
__global__ void k_iv_insert(IvoxParams P) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n_src) return;
    P.iota[i] = (uint32_t)i;
    const float4 p = reinterpret_cast<const float4*>(P.src)[i];
    int cx, cy, cz;
    const float lim = (float)kIvMaxKey;
    if (!iv_cell(p.x, P.inv_res, lim, cx) || !iv_cell(p.y, P.inv_res, lim, cy) || !iv_cell(p.z, P.inv_res, lim, cz)) {
        P.slot_of[i] = (uint32_t)P.table;  // sorts last, never placed
        atomicOr(P.ctr, 1ull);
        return;
    }
    const unsigned long long key = iv_key(cx, cy, cz);
    const uint64_t mask = (uint64_t)P.table - 1ull;
    uint64_t sl = iv_hash(key, P.log2);
    while (true) {
        unsigned long long cur = __hip_atomic_load(&P.slots[sl].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == kGridEmpty) {
            cur = atomicCAS(&P.slots[sl].key, kGridEmpty, key);
            if (cur == kGridEmpty) {
                // new grids counted: one atomic per wave's group of creators (the
                // lanes that leave the probe loop here together)
                const unsigned long long made = __ballot(true);
                if ((threadIdx.x & 63) == __ffsll((long long)made) - 1) atomicAdd(P.ctr + 1, (unsigned long long)__popcll(made));
                break;
            }
        }
        if (cur == key) break;
        sl = (sl + 1) & mask;
    }
    P.slot_of[i] = (uint32_t)sl;
    atomicAdd(P.addcnt + sl, 1u);
    atomicMin(P.first + sl, (uint32_t)i);
    atomicMax(P.lastp1 + sl, (uint32_t)i + 1u);
}

// The batch's new grids removed again (capacity reached): a new grid is a
// used slot with no points yet; every slot it could shadow was filled before.
__global__ void k_iv_rollback(IvoxParams P) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.table) return;
    if (P.slots[s].key != kGridEmpty && P.slots[s].count == 0u) P.slots[s] = GridSlot{kGridEmpty, 0u, 0u};
    P.addcnt[s] = 0u;
    P.first[s] = 0xFFFFFFFFu;
    P.lastp1[s] = 0u;
    P.evict[s] = 0u;
}

__global__ void k_iv_prepare(IvoxParams P) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.table) return;
    // an evicted grid leaves with every point it held, this batch's included
    P.tot[s] = P.evict[s] ? 0u : (P.slots[s].key != kGridEmpty ? P.slots[s].count : 0u) + P.addcnt[s];
}

// Old runs moved to their new start: the wave's 64 slots in turn, each run
// copied by the whole wave (coalesced; a grid of 1,000+ points next to the
// sensor no longer copies on one thread).
__global__ void k_iv_move(IvoxParams P) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    uint32_t st = 0u, cnt = 0u, dst = 0u;
    bool act = false;
    if (s < P.table) {
        const GridSlot g = P.slots[s];
        act = g.key != kGridEmpty && g.count != 0u && !P.evict[s];
        if (act) {
            st = g.start;
            cnt = g.count;
            dst = P.newstart[s];
        }
    }
    const float4* __restrict__ src = reinterpret_cast<const float4*>(P.pts);
    float4* __restrict__ out = reinterpret_cast<float4*>(P.npts);
    unsigned long long m = __ballot(act);
    while (m) {  // (wave-uniform)
        const int l = __ffsll((long long)m) - 1;
        m &= m - 1ull;
        const uint32_t s0 = (uint32_t)__shfl((int)st, l, 64), c0 = (uint32_t)__shfl((int)cnt, l, 64),
                       d0 = (uint32_t)__shfl((int)dst, l, 64);
        for (uint32_t k = (uint32_t)lane; k < c0; k += 64) out[(size_t)d0 + k] = src[(size_t)s0 + k];
    }
}

// New points appended to their grid's run in input order: the batch sorted by
// slot (stable) gives each point its rank inside its grid.
__global__ void k_iv_place(IvoxParams P) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= P.n_src) return;
    const uint32_t sl = P.skeys[k];
    if ((int64_t)sl >= P.table || P.evict[sl]) return;
    const uint32_t i = P.svals[k];
    const uint32_t rank = (uint32_t)k - P.addstart[sl];
    const float4 p = reinterpret_cast<const float4*>(P.src)[i];
    const uint32_t id = (uint32_t)(P.base_id + (int64_t)i);
    reinterpret_cast<float4*>(P.npts)[P.newstart[sl] + P.slots[sl].count + rank] =
        make_float4(p.x, p.y, p.z, __uint_as_float(id));
}

// Slots take their new run; the largest grid by a grid-stride pass of at most
// kFixBlocks blocks and one atomic per block (an atomic or an agent-scope load
// of the one counter per wave serialised on its line: ~88 us per 1M-slot table).
constexpr int kFixBlocks = 1024;
__global__ __launch_bounds__(256) void k_iv_fix(IvoxParams P) {
    __shared__ unsigned wmax[4];
    unsigned cnt = 0;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < P.table; s += (int64_t)gridDim.x * blockDim.x) {
        GridSlot g = P.slots[s];
        if (P.evict[s]) {
            P.addcnt[s] = 0u;  // (k_iv_drop empties the slot)
        } else if (g.key != kGridEmpty) {
            g.start = P.newstart[s];
            g.count += P.addcnt[s];
            P.slots[s] = g;
            P.addcnt[s] = 0u;
            cnt = max(cnt, g.count);
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) cnt = max(cnt, (unsigned)__shfl_xor((int)cnt, off, 64));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned b = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        if (b) atomicMax(P.ctr + 2, (unsigned long long)b);
    }
}

__global__ void k_iv_rehash(const GridSlot* __restrict__ old_slots, const unsigned long long* __restrict__ old_t,
                            int64_t old_table, GridSlot* slots, unsigned long long* tlast, int log2) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= old_table) return;
    const GridSlot g = old_slots[s];
    if (g.key == kGridEmpty) return;
    const uint64_t mask = (1ull << log2) - 1ull;
    uint64_t sl = iv_hash(g.key, log2);
    while (atomicCAS(&slots[sl].key, kGridEmpty, g.key) != kGridEmpty) sl = (sl + 1) & mask;
    slots[sl].start = g.start;
    slots[sl].count = g.count;
    tlast[sl] = old_t[s];
}

// ---- LRU eviction (ivox3d.h:263-275): when a batch takes the grid count to
// the capacity, each new grid past that point evicts grids_cache_.back(), the
// grid whose last added point is the oldest.  Grids the batch touches before
// an eviction are no longer the oldest; the fast path applies when every
// victim is a grid the batch never touches (the host splits the batch
// otherwise, see ivox_add_dev).
__global__ void k_iv_newfirst(IvoxParams P, uint32_t* out, unsigned long long* n) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.table) return;
    if (P.slots[s].key != kGridEmpty && P.slots[s].count == 0u)  // created by this batch
        out[atomicAdd(n, 1ull)] = P.first[s];
}
__global__ void k_iv_oldkeys(IvoxParams P, unsigned long long* keys, uint32_t* slot, unsigned long long* n) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.table) return;
    if (P.slots[s].key != kGridEmpty && P.slots[s].count > 0u) {
        const unsigned long long k = atomicAdd(n, 1ull);
        keys[k] = P.tlast[s];
        slot[k] = (uint32_t)s;
    }
}
__global__ void k_iv_untouched(IvoxParams P, const uint32_t* sorted_slot, int64_t n, uint32_t* flags) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) flags[k] = P.lastp1[sorted_slot[k]] == 0u ? 1u : 0u;
}
// Per old grid (oldest first) the batch's first touch (0xFFFFFFFF: untouched),
// for the host's run-of-evictions scan (ivox_evict_prefix).
__global__ void k_iv_oldfirst(IvoxParams P, const uint32_t* sorted_slot, int64_t n, uint32_t* out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) out[k] = P.first[sorted_slot[k]];
}
// Oldest first: the first ev untouched grids are the victims, unless a grid the
// batch touches only at or after the first eviction is older than the last of
// them (it would be evicted and re-created): that is flagged (ctr[0] bit 2).
__global__ void k_iv_victims(IvoxParams P, const uint32_t* sorted_slot, const uint32_t* rank, int64_t n, int64_t ev,
                             uint32_t j_first) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t s = sorted_slot[k];
    if (P.lastp1[s] == 0u) {
        if ((int64_t)rank[k] < ev) P.evict[s] = 1u;
        if ((int64_t)rank[k] == ev - 1) P.ctr[3] = (unsigned long long)k;
    }
}
__global__ void k_iv_conflict(IvoxParams P, const uint32_t* sorted_slot, int64_t n, uint32_t j_first) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n || (unsigned long long)k >= P.ctr[3]) return;
    const uint32_t s = sorted_slot[k];
    if (P.lastp1[s] != 0u && P.first[s] >= j_first) atomicOr(P.ctr, 2ull);
}
// Single eviction at the batch's last point: grids_cache_.back() among every
// grid then in the map, new ones included (their last touch this batch).
__device__ __forceinline__ unsigned long long iv_tcur(const IvoxParams& P, int64_t s) {
    return P.lastp1[s] ? (unsigned long long)P.base_id + P.lastp1[s] - 1ull : P.tlast[s];
}
__global__ void k_iv_tcur_min(IvoxParams P) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long t = ~0ull;
    if (s < P.table && P.slots[s].key != kGridEmpty) t = iv_tcur(P, s);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(t, off, 64);
        t = o < t ? o : t;
    }
    if ((threadIdx.x & 63) == 0 && t != ~0ull) atomicMin(P.ctr + 4, t);
}
__global__ void k_iv_mark_min(IvoxParams P) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s < P.table && P.slots[s].key != kGridEmpty && iv_tcur(P, s) == P.ctr[4]) P.evict[s] = 1u;
}
// After the CSR rebuild: evicted grids leave the table (the host rehashes to
// mend the probe chains).  A grid evicted by its own creation (capacity 1)
// got no points either.
__global__ void k_iv_drop(IvoxParams P) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.table || !P.evict[s]) return;
    P.slots[s] = GridSlot{kGridEmpty, 0u, 0u};
    P.evict[s] = 0u;
}
// The batch's touches become each grid's last-use id; per-batch marks reset.
__global__ void k_iv_commit(IvoxParams P) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.table) return;
    if (P.lastp1[s]) P.tlast[s] = (unsigned long long)P.base_id + P.lastp1[s] - 1ull;
    P.first[s] = 0xFFFFFFFFu;
    P.lastp1[s] = 0u;
}

static inline dim3 blocks_for(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

#define LAUNCH_CHECKED(kernel, n, ...)                                                         \
    do {                                                                                       \
        if ((n) <= 0) return LIVO_OK;                                                          \
        hipLaunchKernelGGL(kernel, blocks_for(n), dim3(256), 0, (hipStream_t)stream, __VA_ARGS__); \
        return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;                         \
    } while (0)

int launch_ivox_clear(GridSlot* slots, int64_t table, void* stream) { LAUNCH_CHECKED(k_iv_clear, table, slots, table); }
int launch_ivox_insert(const IvoxParams& p, void* stream) { LAUNCH_CHECKED(k_iv_insert, p.n_src, p); }
int launch_ivox_rollback(const IvoxParams& p, void* stream) { LAUNCH_CHECKED(k_iv_rollback, p.table, p); }
int launch_ivox_prepare(const IvoxParams& p, void* stream) { LAUNCH_CHECKED(k_iv_prepare, p.table, p); }
int launch_ivox_move(const IvoxParams& p, void* stream) { LAUNCH_CHECKED(k_iv_move, p.table, p); }
int launch_ivox_place(const IvoxParams& p, void* stream) { LAUNCH_CHECKED(k_iv_place, p.n_src, p); }
int launch_ivox_fix(const IvoxParams& p, void* stream) {
    if (p.table <= 0) return LIVO_OK;
    const unsigned blocks = (unsigned)std::min<int64_t>(kFixBlocks, (p.table + 255) / 256);
    hipLaunchKernelGGL(k_iv_fix, dim3(blocks), dim3(256), 0, (hipStream_t)stream, p);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
int launch_ivox_rehash(const GridSlot* old_slots, const unsigned long long* old_t, int64_t old_table, GridSlot* slots,
                       unsigned long long* tlast, int log2, void* stream) {
    LAUNCH_CHECKED(k_iv_rehash, old_table, old_slots, old_t, old_table, slots, tlast, log2);
}
int launch_ivox_newfirst(const IvoxParams& p, uint32_t* out, unsigned long long* n, void* stream) {
    LAUNCH_CHECKED(k_iv_newfirst, p.table, p, out, n);
}
int launch_ivox_oldkeys(const IvoxParams& p, unsigned long long* keys, uint32_t* slot, unsigned long long* n,
                        void* stream) {
    LAUNCH_CHECKED(k_iv_oldkeys, p.table, p, keys, slot, n);
}
int launch_ivox_untouched(const IvoxParams& p, const uint32_t* sorted_slot, int64_t n, uint32_t* flags, void* stream) {
    LAUNCH_CHECKED(k_iv_untouched, n, p, sorted_slot, n, flags);
}
int launch_ivox_oldfirst(const IvoxParams& p, const uint32_t* sorted_slot, int64_t n, uint32_t* out, void* stream) {
    LAUNCH_CHECKED(k_iv_oldfirst, n, p, sorted_slot, n, out);
}
int launch_ivox_victims(const IvoxParams& p, const uint32_t* sorted_slot, const uint32_t* rank, int64_t n, int64_t ev,
                        uint32_t j_first, void* stream) {
    if (n <= 0) return LIVO_OK;
    hipLaunchKernelGGL(k_iv_victims, blocks_for(n), dim3(256), 0, (hipStream_t)stream, p, sorted_slot, rank, n, ev,
                       j_first);
    if (hipGetLastError() != hipSuccess) return LIVO_E_HIP;
    LAUNCH_CHECKED(k_iv_conflict, n, p, sorted_slot, n, j_first);
}
int launch_ivox_tcur_min(const IvoxParams& p, void* stream) { LAUNCH_CHECKED(k_iv_tcur_min, p.table, p); }
int launch_ivox_mark_min(const IvoxParams& p, void* stream) { LAUNCH_CHECKED(k_iv_mark_min, p.table, p); }
int launch_ivox_drop(const IvoxParams& p, void* stream) { LAUNCH_CHECKED(k_iv_drop, p.table, p); }
int launch_ivox_commit(const IvoxParams& p, void* stream) { LAUNCH_CHECKED(k_iv_commit, p.table, p); }

// ---------------------------------------------------- map_incremental ----
// laser_mapping.cpp:343-380 for one point (stored position j).
__global__ void k_map_incr(MapIncrParams P) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= P.n) return;
    const float4 b = reinterpret_cast<const float4*>(P.pts)[j];
    float pw[3];
    world_point(P.slot->state.rot, P.slot->state.pos, P.R_LI, P.t_LI, b.x, b.y, b.z, pw[0], pw[1], pw[2]);
    const NNRec& r = P.nn[j];
    const int cnt = r.cnt;
    int cat = 1;
    if (cnt > 0 && P.ekf_inited) {
        const float fs = (float)P.fs;  // Eigen promotes the double scalar to float
        float c[3];
#pragma unroll
        for (int a = 0; a < 3; a++) c[a] = (floorf(pw[a] / fs) + 0.5f) * fs;
        const double half = 0.5 * P.fs;
        if ((double)fabsf(r.p[0][0] - c[0]) > half && (double)fabsf(r.p[0][1] - c[1]) > half &&
            (double)fabsf(r.p[0][2] - c[2]) > half) {
            cat = 2;
        } else {
            // common::calc_dist(Vector3f, Vector3f) = (p1 - p2).norm() (common_lib.h:85)
            auto norm3 = [&](float x, float y, float z) {
                const float u = x - c[0], v = y - c[1], w = z - c[2];
                return sqrtf(u * u + (v * v + w * w));
            };
            const float dist = norm3(pw[0], pw[1], pw[2]);
            bool need_add = true;
            if (cnt >= kNN)
#pragma unroll
                for (int k = 0; k < kNN; k++)
                    if (need_add && (double)norm3(r.p[k][0], r.p[k][1], r.p[k][2]) < (double)dist + 1e-6)
                        need_add = false;
            cat = need_add ? 1 : 0;
        }
    }
    if (P.cat) P.cat[j] = (uint8_t)cat;
    if (cat) {
        const int64_t pos = (cat == 1 ? 0 : (int64_t)P.n) + P.perm[j];
        reinterpret_cast<float4*>(P.ordered)[pos] = make_float4(pw[0], pw[1], pw[2], 0.f);
        P.flags[pos] = 1u;
    }
}

int launch_map_incr(const MapIncrParams& p, void* stream) {
    if (p.n <= 0) return LIVO_OK;
    hipLaunchKernelGGL(k_map_incr, blocks_for(p.n), dim3(256), 0, (hipStream_t)stream, p);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

__global__ void k_compact(const float4* __restrict__ ordered, const uint32_t* __restrict__ flags,
                          const uint32_t* __restrict__ pos, int64_t n, float4* __restrict__ dense) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n && flags[k]) dense[pos[k]] = ordered[k];
}

int launch_compact(const float* ordered, const uint32_t* flags, const uint32_t* pos, int64_t n, float* dense,
                   void* stream) {
    LAUNCH_CHECKED(k_compact, n, reinterpret_cast<const float4*>(ordered), flags, pos, n,
                   reinterpret_cast<float4*>(dense));
}

__global__ void k_inherit_nn(NNRec* dst, const int32_t* dst_perm, int64_t n_dst, const NNRec* src,
                             const int32_t* src_iperm, int64_t n_src) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_dst) return;
    const int64_t o = dst_perm[j];
    const int4* s = o < n_src ? reinterpret_cast<const int4*>(src + src_iperm[o]) : nullptr;
    int4* d = reinterpret_cast<int4*>(dst + j);
#pragma unroll
    for (int k = 0; k < 8; k++) d[k] = s ? s[k] : make_int4(0, 0, 0, 0);
}

int launch_inherit_nn(NNRec* dst, const int32_t* dst_perm, int64_t n_dst, const NNRec* src,
                      const int32_t* src_iperm, int64_t n_src, void* stream) {
    LAUNCH_CHECKED(k_inherit_nn, n_dst, dst, dst_perm, n_dst, src, src_iperm, n_src);
}

}  // namespace livo
