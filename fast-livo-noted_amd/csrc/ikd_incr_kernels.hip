// ikd_incr_kernels.hip — CDNA4 (gfx950) kernels of the ikd-Tree incremental
// map (the USE_ikdtree branch of
// LaserMapping::map_incremental, src/laser_mapping.cpp:383-384).
//
//   KD_TREE::Add_Points(points, downsample_on) (include/ikd-Tree/ikd_Tree.cpp:
//   382-457) with downsample_size = filter_size_map_min (laser_mapping.cpp:138):
//   per point, in order, the box floor(p / ds) * ds .. + ds and its centre
//   (:392-400); the box's stored points (Search_by_range, :988-1016, half open
//   vmin <= p < vmax); the nearest of them replaces the new point only if
//   strictly nearer the centre (:403-411); if the box held more than one point
//   or the new point won (same_point, :1287-1289), the box is emptied
//   (Delete_by_range, :626-688) and the winner added (:413-416).
//
//   k_add_prep    box key per point; a point within a rounding step of a box
//                 face (neighbouring float boxes overlap or leave a gap) marks
//                 the boxes it touches dirty
//   (stable radix sort by box key: a box's points in input order)
//   k_add_box     a group of lanes per box: its stored points from the cell grid,
//                 then the box's whole sequence of new points.  Boxes are
//                 independent, except dirty boxes and boxes holding a stored
//                 point that lies in two boxes: those are deferred
//   k_add_finish  one workgroup: the deferred points in input order on one
//                 thread with the reference's sequential rule, then the kept
//                 points appended with the next ids (input order)
//   k_dyn_*       the cell grid of k_knn_grid rebuilt from the surviving
//                 points (keys -> radix sort -> runs -> hash), and
//                 Delete_Point_Boxes (:501-521)
//
// Stored points at exactly the same distance from the centre are taken in id
// (insertion) order where the reference takes Search_by_range's tree order
// (its tree shape depends on Rebuild and the background rebuild thread); the
// boxes where that decides are counted (`ambiguous`).  Numerics as
// livo_kernels.hip: -ffp-contract=off, the reference's float expressions.
#include <hip/hip_runtime.h>
#include <math.h>

#include "device_common.h"
#include "livo_internal.h"

namespace livo {

__device__ __forceinline__ unsigned long long pack_key(int x, int y, int z) {  // = grid_key_d (livo_kernels.hip)
    return (unsigned long long)(x + kGridBias) | ((unsigned long long)(y + kGridBias) << 21) |
           ((unsigned long long)(z + kGridBias) << 42);
}
__device__ __forceinline__ int key_axis(unsigned long long k, int a) {
    return (int)((k >> (21 * a)) & 0x1FFFFFull) - kGridBias;
}
// One axis of Box_of_Point (:392-397): [j * ds, j * ds + ds) in floats.
__device__ __forceinline__ bool ax_in(float v, int j, float ds) {
    const float lo = (float)j * ds, hi = lo + ds;
    return lo <= v && hi > v;
}
struct DBox {
    float lo[3], hi[3], mid[3];
};
__device__ __forceinline__ DBox dbox(unsigned long long k, float ds) {
    DBox b;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        b.lo[a] = (float)key_axis(k, a) * ds;
        b.hi[a] = b.lo[a] + ds;
        b.mid[a] = (float)((double)b.lo[a] + (double)(b.hi[a] - b.lo[a]) / 2.0);  // mid_point (:398-400)
    }
    return b;
}
__device__ __forceinline__ bool in_dbox(const DBox& b, float x, float y, float z) {
    return b.lo[0] <= x && b.hi[0] > x && b.lo[1] <= y && b.hi[1] > y && b.lo[2] <= z && b.hi[2] > z;
}
__device__ __forceinline__ float mid_dist(const DBox& b, float x, float y, float z) {  // calc_dist (:1291-1295)
    const float dx = x - b.mid[0], dy = y - b.mid[1], dz = z - b.mid[2];
    return (dx * dx + dy * dy) + dz * dz;
}
__device__ __forceinline__ bool same_pt(float ax, float ay, float az, float bx, float by, float bz) {  // :1287-1289
    return (double)fabsf(ax - bx) < 1e-6 && (double)fabsf(ay - by) < 1e-6 && (double)fabsf(az - bz) < 1e-6;
}
// A point of box k that also lies in a neighbouring box (within a rounding step of a face).
__device__ __forceinline__ bool in_two(unsigned long long k, float ds, float x, float y, float z) {
    const float v[3] = {x, y, z};
    bool m = false;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const int j = key_axis(k, a);
        m = m || ax_in(v[a], j - 1, ds) || ax_in(v[a], j + 1, ds);
    }
    return m;
}
// Run {start, count} of grid cell (x, y, z); count 0 if empty.
__device__ __forceinline__ uint2 cell_run(const GridSlot* __restrict__ slots, int log2, int x, int y, int z) {
    const unsigned long long key = pack_key(x, y, z);
    const uint64_t mask = (1ull << log2) - 1ull;
    uint64_t sl = (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - log2));
    GridSlot g = slots[sl];
    while (g.key != key && g.key != kGridEmpty) {
        sl = (sl + 1) & mask;
        g = slots[sl];
    }
    return g.key == key ? make_uint2(g.start, g.count) : make_uint2(0u, 0u);
}
// Grid cells that can hold a point of the box (with the grid's rounding slack).
__device__ __forceinline__ bool box_cells(const DynAddParams& P, const DBox& b, int (&l)[3], int (&h)[3]) {
    const double ih = 1.0 / (double)P.gh;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const double lo = floor(((double)b.lo[a] - (double)P.geps - (double)P.gorg[a]) * ih);
        const double hi = floor(((double)b.hi[a] + (double)P.geps - (double)P.gorg[a]) * ih);
        if (!(fabs(lo) < (double)(kGridBias - 8) && fabs(hi) < (double)(kGridBias - 8))) return false;
        l[a] = (int)lo;
        h[a] = (int)hi;
    }
    return true;
}

// ------------------------------------------------------------ Add_Points ----
__device__ __forceinline__ uint32_t dirty_slot(unsigned long long key, uint32_t cap) {
    return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 40) & (cap - 1u);
}
// Box `key` into the dirty set (count in ctr[kDynDirty]; a full probe marks overflow).
__device__ __forceinline__ void dirty_insert(const DynAddParams& P, unsigned long long key) {
    uint32_t sl = dirty_slot(key, P.dirty_cap);
    for (uint32_t probe = 0; probe < P.dirty_cap; probe++) {
        const unsigned long long prev = atomicCAS(P.dirty + sl, 0ull, key);
        if (prev == 0ull) {
            atomicAdd(P.ctr + kDynDirty, 1ull);
            return;
        }
        if (prev == key) return;
        sl = (sl + 1u) & (P.dirty_cap - 1u);
    }
    atomicAdd(P.ctr + kDynDirty, (unsigned long long)P.dirty_cap);
}
// Whether box `key` is dirty (every box is, once the set is past half full).
__device__ __forceinline__ bool dirty_has(const DynAddParams& P, unsigned long long key) {
    if (P.ctr[kDynDirty] > (unsigned long long)(P.dirty_cap / 2)) return true;
    uint32_t sl = dirty_slot(key, P.dirty_cap);
    for (uint32_t probe = 0; probe < P.dirty_cap; probe++) {
        const unsigned long long v = P.dirty[sl];
        if (v == key) return true;
        if (v == 0ull) return false;
        sl = (sl + 1u) & (P.dirty_cap - 1u);
    }
    return true;
}

__global__ void k_add_prep(DynAddParams P) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t i = g;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g < P.n) {
        if (P.wpts) {  // map_incremental: the stored point g is caller point perm[g], to the world frame
            const float4 b = reinterpret_cast<const float4*>(P.wpts)[g];
            float wx, wy, wz;
            world_point(P.wrot, P.wpos, P.R_LI, P.t_LI, b.x, b.y, b.z, wx, wy, wz);
            i = P.wperm[g];
            p = make_float4(wx, wy, wz, 0.f);
            reinterpret_cast<float4*>(const_cast<float*>(P.W))[i] = p;
        } else {
            p = reinterpret_cast<const float4*>(P.W)[i];
        }
    }
    const float v[3] = {p.x, p.y, p.z};
    const float am = fmaxf(fmaxf(fabsf(p.x), fabsf(p.y)), fabsf(p.z));
    bool ok = am <= 1e30f;  // false for NaN / inf
    // the point's cell of the map grid must be addressable (k_knn_grid's key range)
#pragma unroll
    for (int a = 0; a < 3; a++) ok = ok && fabsf(floorf((v[a] - P.gorg[a]) * P.ginv)) < (float)(kGridBias - 8);
    {  // the batch's largest |coordinate|: one global atomic per block (one address: they serialise)
        __shared__ uint32_t bmax;
        if (threadIdx.x == 0) bmax = 0u;
        __syncthreads();
        uint32_t m = (g < P.n && ok) ? __float_as_uint(am) : 0u;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
        if ((threadIdx.x & 63) == 0 && m) atomicMax(&bmax, m);
        __syncthreads();
        if (threadIdx.x == 0 && bmax) atomicMax(P.ctr + kDynAbsMax, (unsigned long long)bmax);
    }
    if (g >= P.n) return;
    P.iota[i] = (uint32_t)i;
    P.keep[i] = P.downsample ? 0u : 1u;  // without downsampling every point is added (:438-454)
    P.defer[i] = 0u;
    P.keys[i] = 0ull;
    if (P.keys32) P.keys32[i] = 0u;
    if (!P.downsample) {
        if (!ok) atomicOr(P.ctr + kDynError, 1ull);
        return;
    }
    int j[3] = {0, 0, 0};
    bool mem[3][3];
    bool clean = true;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float f = floorf(v[a] / P.ds);
        ok = ok && fabsf(f) < (float)(kGridBias - 8);
        j[a] = ok ? (int)f : 0;
#pragma unroll
        for (int o = 0; o < 3; o++) mem[a][o] = ax_in(v[a], j[a] + o - 1, P.ds);
        clean = clean && mem[a][1] && !mem[a][0] && !mem[a][2];
    }
    if (!ok) {
        atomicOr(P.ctr + kDynError, 1ull);
        return;
    }
    const unsigned long long k = pack_key(j[0], j[1], j[2]);
    // every later pass reads the grid cells of this point's box: check their
    // range here, so that an out-of-range batch is refused before anything changes
    {
        int l[3], h[3];
        if (!box_cells(P, dbox(k, P.ds), l, h)) {
            atomicOr(P.ctr + kDynError, 1ull);
            return;
        }
    }
    P.keys[i] = k;
    if (P.keys32) P.keys32[i] = (uint32_t)(j[0] & 1023) | ((uint32_t)(j[1] & 1023) << 10) | ((uint32_t)(j[2] & 1023) << 20);
    if (clean) return;
    // processed in box k, lying inside the boxes of `mem`: all of them go to the sequential pass
    dirty_insert(P, k);
    for (int o0 = 0; o0 < 3; o0++)
        for (int o1 = 0; o1 < 3; o1++)
            for (int o2 = 0; o2 < 3; o2++)
                if (mem[0][o0] && mem[1][o1] && mem[2][o2] && !(o0 == 1 && o1 == 1 && o2 == 1))
                    dirty_insert(P, pack_key(j[0] + o0 - 1, j[1] + o1 - 1, j[2] + o2 - 1));
}

constexpr int kBoxWaves = 4;       // k_add_box: waves per block
constexpr uint32_t kBoxSmall = 64;  // boxes with at most this many new points: 16-lane groups
constexpr int kBigBlocks = 128;     // k_add_box's first blocks: a wave per crowded box

// A box's stored points (Search_by_range) by a group of G lanes (16: most
// boxes hold a few stored points and new points; 64: the crowded boxes): the
// lanes take the grid cells the box overlaps (one hash probe each), then the
// cells' points spread over the lanes (a point's cell by a binary search of the
// cells' exclusive counts in LDS).  `f(q)` per stored point.
template <int G>
struct GroupCells {
    uint32_t exc[G], start[G];
};
template <int G>
__device__ __forceinline__ bool group_any(bool x) {
    const unsigned long long b = __ballot(x);
    if constexpr (G == 64) return b != 0ull;
    else return ((b >> ((threadIdx.x & 63) & ~(G - 1))) & ((1ull << G) - 1ull)) != 0ull;
}
template <int G, class F>
__device__ __forceinline__ void group_box_points(const DynAddParams& P, const int (&l)[3], const int (&h)[3], int gl,
                                                 GroupCells<G>& W, F&& f) {
    const int ex = h[0] - l[0] + 1, ey = h[1] - l[1] + 1, ez = h[2] - l[2] + 1;
    const int ncell = (ex > 0 && ey > 0 && ez > 0) ? ex * ey * ez : 0;
    const float4* __restrict__ gp = reinterpret_cast<const float4*>(P.gpts);
    for (int c0 = 0; c0 < ncell; c0 += G) {  // group-uniform
        const int c = c0 + gl;
        uint2 r = make_uint2(0u, 0u);
        if (c < ncell) r = cell_run(P.gslots, P.glog2, l[0] + c % ex, l[1] + (c / ex) % ey, l[2] + c / (ex * ey));
        uint32_t inc = r.y;
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            const uint32_t v = __shfl_up(inc, off, G);
            if (gl >= off) inc += v;
        }
        const uint32_t total = __shfl(inc, G - 1, G);
        W.exc[gl] = inc - r.y;
        W.start[gl] = r.x;
        __builtin_amdgcn_wave_barrier();
        for (uint32_t t = gl; t < total; t += G) {
            int j = 0;  // the last cell whose exclusive count is <= t (it holds point t)
#pragma unroll
            for (int step = G / 2; step >= 1; step >>= 1)
                if (W.exc[j + step] <= t) j += step;
            f(gp[W.start[j] + (t - W.exc[j])]);
        }
        __builtin_amdgcn_wave_barrier();
    }
}
// A box's stored points: count, the first nearest in id order, whether points
// of two different positions share the nearest distance (the reference's tie,
// decided by its tree order); `defer` if the box is dirty or holds a point that
// also lies in a neighbouring box.  The lanes' partial results merge in any
// order to the same (group-uniform) result.
struct BoxStore {
    int cnt;
    float bd, bx, by, bz;
    uint32_t bid;
    bool tie, defer;
    int l[3], h[3];
};
__device__ __forceinline__ void store_merge(BoxStore& S, float d, uint32_t id, float x, float y, float z, bool tie) {
    if (d < S.bd) {
        S.bd = d; S.bid = id; S.bx = x; S.by = y; S.bz = z; S.tie = tie;
    } else if (d == S.bd) {
        S.tie = S.tie || tie || x != S.bx || y != S.by || z != S.bz;
        if (id < S.bid) { S.bid = id; S.bx = x; S.by = y; S.bz = z; }
    }
}
template <int G>
__device__ __forceinline__ void group_box_store(const DynAddParams& P, unsigned long long key, const DBox& b, int gl,
                                                GroupCells<G>& W, BoxStore& S) {
    S.cnt = 0; S.bd = INFINITY; S.bx = S.by = S.bz = 0.f; S.bid = 0xFFFFFFFFu; S.tie = false;
    S.l[0] = S.l[1] = S.l[2] = 0; S.h[0] = S.h[1] = S.h[2] = -1;
    bool defer = dirty_has(P, key);
    if (!defer && !box_cells(P, b, S.l, S.h)) defer = true;
    if (defer) {
        S.defer = true;
        return;
    }
    bool two = false;
    group_box_points<G>(P, S.l, S.h, gl, W, [&](const float4 q) {
        if (!in_dbox(b, q.x, q.y, q.z)) return;
        if (in_two(key, P.ds, q.x, q.y, q.z)) two = true;
        S.cnt++;
        store_merge(S, mid_dist(b, q.x, q.y, q.z), __float_as_uint(q.w), q.x, q.y, q.z, false);
    });
    S.defer = group_any<G>(two);
    if (S.defer) return;
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) {
        S.cnt += __shfl_xor(S.cnt, off, G);
        const float d = __shfl_xor(S.bd, off, G);
        const uint32_t id = __shfl_xor(S.bid, off, G);
        const float x = __shfl_xor(S.bx, off, G), y = __shfl_xor(S.by, off, G), z = __shfl_xor(S.bz, off, G);
        const bool t = __shfl_xor((int)S.tie, off, G) != 0;
        store_merge(S, d, id, x, y, z, t);
    }
}

// The running winner of a box's new points is a scan: (distance, position) with
// the smaller distance, the later position on ties ("d <= dc" lets the later
// point win), the winner's coordinates carried along.

// Add_Points' loop body for the box's points (:390-437) by one group of G
// lanes: the stored points (group_box_store), then the box's new points in
// input order as a prefix scan of the running winner, G points per step (after
// the first point the box holds one point), then Delete_by_range of the box
// with the lanes over its stored points (a stored winner is deleted and added
// again: it stays).
template <int G>
__device__ __forceinline__ void add_box(const DynAddParams& P, int64_t g, int gl, GroupCells<G>& W) {
    const float4* __restrict__ Ws = reinterpret_cast<const float4*>(P.Ws);
    const uint32_t s0 = P.starts[g], s1 = P.starts[g + 1];
    const unsigned long long key = P.skeys[s0];
    const DBox b = dbox(key, P.ds);
    BoxStore S;
    group_box_store<G>(P, key, b, gl, W, S);
    if (S.defer) {  // flagged, and listed (unordered) for k_add_finish
        unsigned long long at = 0;
        if (gl == 0) at = atomicAdd(P.ctr + kDynDeferred, (unsigned long long)(s1 - s0));
        at = __shfl(at, 0, G);
        for (uint32_t k = s0 + gl; k < s1; k += G) {
            const uint32_t i = P.svals[k];
            P.defer[i] = 1u;
            P.dlist_u[at + (k - s0)] = i;
        }
        return;
    }
    // the first new point against the stored ones, the carry of the scan
    const float4 p0 = Ws[s0];
    float cd = mid_dist(b, p0.x, p0.y, p0.z);  // running winner: distance, position (-1: the stored point)
    int ck = (int)s0;
    float cx = p0.x, cy = p0.y, cz = p0.z;
    if (S.cnt > 0 && S.bd < cd) { cd = S.bd; ck = -1; cx = S.bx; cy = S.by; cz = S.bz; }
    const unsigned long long amb = (S.cnt > 1 && ck < 0 && S.tie) ? 1ull : 0ull;
    unsigned long long events = 0;
    if (gl == 0 && (S.cnt > 1 || ck >= 0 || same_pt(p0.x, p0.y, p0.z, cx, cy, cz))) events = 1;
    if constexpr (G == 64) {
        // a crowded box (up to thousands of new points): each lane a segment of
        // consecutive points -- its winner, a scan of the segments' winners, then
        // the segment replayed from the winner before it to count the events
        const uint32_t cnt = s1 - (s0 + 1), L = (cnt + 63u) / 64u;
        const uint32_t a0 = min(s1, s0 + 1 + (uint32_t)gl * L), a1 = min(s1, a0 + L);
        float sd = INFINITY, sx = 0.f, sy = 0.f, sz = 0.f;
        int sk = -2;
#pragma unroll 4
        for (uint32_t k = a0; k < a1; k++) {
            const float4 p = Ws[k];
            const float d = mid_dist(b, p.x, p.y, p.z);
            if (d <= sd) { sd = d; sk = (int)k; sx = p.x; sy = p.y; sz = p.z; }
        }
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {  // inclusive: the later segment wins ties
            const float od = __shfl_up(sd, off, 64);
            const int okk = __shfl_up(sk, off, 64);
            const float ox = __shfl_up(sx, off, 64), oy = __shfl_up(sy, off, 64), oz = __shfl_up(sz, off, 64);
            if (gl >= off && !(sd <= od)) { sd = od; sk = okk; sx = ox; sy = oy; sz = oz; }
        }
        float rd = cd, rx = cx, ry = cy, rz = cz;  // the winner before the segment
        {
            const float xd = __shfl_up(sd, 1, 64);
            const float xx = __shfl_up(sx, 1, 64), xy = __shfl_up(sy, 1, 64), xz = __shfl_up(sz, 1, 64);
            if (gl > 0 && xd <= rd) { rd = xd; rx = xx; ry = xy; rz = xz; }
        }
#pragma unroll 4
        for (uint32_t k = a0; k < a1; k++) {
            const float4 p = Ws[k];
            const float d = mid_dist(b, p.x, p.y, p.z);
            if (d <= rd) {
                events++;
                rd = d; rx = p.x; ry = p.y; rz = p.z;
            } else if (same_pt(p.x, p.y, p.z, rx, ry, rz)) {
                events++;
            }
        }
        const float ld = __shfl(sd, 63, 64);
        const int lk = __shfl(sk, 63, 64);
        const float lx = __shfl(sx, 63, 64), ly = __shfl(sy, 63, 64), lz = __shfl(sz, 63, 64);
        if (lk >= 0 && ld <= cd) { cd = ld; ck = lk; cx = lx; cy = ly; cz = lz; }
    } else
    for (uint32_t k0 = s0 + 1; k0 < s1; k0 += G) {
        const uint32_t k = k0 + gl;
        const bool valid = k < s1;
        float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
        float d = INFINITY;
        int pk = -2;  // loses every comparison
        if (valid) {
            p = Ws[k];
            d = mid_dist(b, p.x, p.y, p.z);
            pk = (int)k;
        }
        // inclusive scan of the running winner over lanes 0..gl, its coordinates carried along
        float sd = d, sx = p.x, sy = p.y, sz = p.z;
        int sk = pk;
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            const float od = __shfl_up(sd, off, G);
            const int okk = __shfl_up(sk, off, G);
            const float ox = __shfl_up(sx, off, G), oy = __shfl_up(sy, off, G), oz = __shfl_up(sz, off, G);
            if (gl >= off && (od < sd || (od == sd && okk > sk))) {
                sd = od; sk = okk; sx = ox; sy = oy; sz = oz;
            }
        }
        // the winner before this point: the carry (every earlier point), then the
        // chunk's exclusive prefix -- later on equal distance, so the chunk wins ties
        float pd = cd, qx = cx, qy = cy, qz = cz;
        int pkk = ck;
        {
            const float xd = __shfl_up(sd, 1, G);
            const int xk = __shfl_up(sk, 1, G);
            const float xx = __shfl_up(sx, 1, G), xy = __shfl_up(sy, 1, G), xz = __shfl_up(sz, 1, G);
            if (gl > 0 && (xd < pd || (xd == pd && xk > pkk))) {
                pd = xd; pkk = xk; qx = xx; qy = xy; qz = xz;
            }
        }
        if (valid && (d <= pd || same_pt(p.x, p.y, p.z, qx, qy, qz))) events++;
        // new carry: the inclusive winner of the last valid lane against the carry
        const int last = (int)min<uint32_t>((uint32_t)(G - 1), s1 - 1 - k0);
        const float ld = __shfl(sd, last, G);
        const int lk = __shfl(sk, last, G);
        const float lx = __shfl(sx, last, G), ly = __shfl(sy, last, G), lz = __shfl(sz, last, G);
        if (ld < cd || (ld == cd && lk > ck)) {
            cd = ld; ck = lk; cx = lx; cy = ly; cz = lz;
        }
    }
    const bool newer = ck >= 0;
    if (newer && gl == 0) {
        const uint32_t win = __float_as_uint(Ws[ck].w);
        P.keep[win] = 1u;
        P.klist[atomicAdd(P.ctr + kDynKept, 1ull)] = win;
    }
    unsigned long long deleted = 0;
    if (S.cnt > 0 && (newer || S.cnt > 1)) {
        group_box_points<G>(P, S.l, S.h, gl, W, [&](const float4 q) {
            if (!in_dbox(b, q.x, q.y, q.z)) return;
            const uint32_t id = __float_as_uint(q.w);
            if (!newer && id == S.bid) return;
            P.alive[id] = 0;
            deleted++;
        });
    }
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) {
        events += __shfl_xor(events, off, G);
        deleted += __shfl_xor(deleted, off, G);
    }
    if (gl == 0) {
        if (events) atomicAdd(P.ctr + kDynEvents, events);
        if (deleted) atomicAdd(P.ctr + kDynDeleted, deleted);
        if (amb) atomicAdd(P.ctr + kDynAmbig, amb);
    }
}
// One launch: the first kBigBlocks blocks take the crowded boxes (listed by
// k_scan_boxes), a wave each; the others the rest, a 16-lane group each.
__global__ __launch_bounds__(64 * kBoxWaves) void k_add_box(DynAddParams P) {
    constexpr int G = 16, kGroups = 64 * kBoxWaves / G;
    __shared__ GroupCells<G> cells[kGroups];
    if (P.ctr[kDynError]) return;  // k_add_prep refused the batch: nothing changes
    if (blockIdx.x < kBigBlocks) {
        GroupCells<64>& W = reinterpret_cast<GroupCells<64>*>(cells)[threadIdx.x >> 6];
        const int64_t nb = (int64_t)P.ctr[kDynBig];
        for (int64_t b = (int64_t)blockIdx.x * kBoxWaves + (threadIdx.x >> 6); b < nb; b += kBigBlocks * kBoxWaves)
            add_box<64>(P, P.bigs[b], threadIdx.x & 63, W);
        return;
    }
    const int gl = threadIdx.x & (G - 1);
    GroupCells<G>& W = cells[threadIdx.x / G];
    const int64_t runs = (int64_t)P.ctr[kDynRuns];
    for (int64_t g = (int64_t)(blockIdx.x - kBigBlocks) * kGroups + threadIdx.x / G; g < runs;
         g += (int64_t)(gridDim.x - kBigBlocks) * kGroups) {
        if (P.starts[g + 1] - P.starts[g] > kBoxSmall) continue;  // (group-uniform) a crowded box
        add_box<G>(P, g, gl, W);
    }
}
static_assert(sizeof(GroupCells<64>) * kBoxWaves <= sizeof(GroupCells<16>) * (64 * kBoxWaves / 16), "LDS");

// The deferred points in input order on one thread: exactly Add_Points' loop.
// Returns the count of this pass's kept points (seq[0, ns), w = ~0 once deleted).
__device__ uint32_t add_seq(const DynAddParams& P, const uint32_t* list, uint32_t D) {
    const float4* __restrict__ gp = reinterpret_cast<const float4*>(P.gpts);
    const float4* __restrict__ W = reinterpret_cast<const float4*>(P.W);
    float4* seq = reinterpret_cast<float4*>(P.seq);  // this pass's kept points (x, y, z, input index)
    uint32_t ns = 0;
    unsigned long long events = 0, deleted = 0, amb = 0;
    for (uint32_t t = 0; t < D; t++) {
        const uint32_t i = list[t];
        const float4 p = W[i];
        const DBox b = dbox(P.keys[i], P.ds);
        int l[3] = {0, 0, 0}, h[3] = {-1, -1, -1};
        if (!box_cells(P, b, l, h)) {
            atomicOr(P.ctr + kDynError, 2ull);
            continue;
        }
        // Search_by_range: alive stored points (ord = id), this pass's kept points (ord = base + index)
        int cnt = 0;
        float bd = INFINITY, bx = 0.f, by = 0.f, bz = 0.f;
        unsigned long long bo = ~0ull;
        bool tie = false;
        auto consider = [&](float qx, float qy, float qz, unsigned long long ord) {
            cnt++;
            const float d = mid_dist(b, qx, qy, qz);
            if (d < bd) {
                bd = d; bo = ord; bx = qx; by = qy; bz = qz;
                tie = false;
            } else if (d == bd) {
                if (qx != bx || qy != by || qz != bz) tie = true;
                if (ord < bo) { bo = ord; bx = qx; by = qy; bz = qz; }
            }
        };
        for (int z = l[2]; z <= h[2]; z++)
            for (int y = l[1]; y <= h[1]; y++)
                for (int x = l[0]; x <= h[0]; x++) {
                    const uint2 r = cell_run(P.gslots, P.glog2, x, y, z);
                    for (uint32_t k = r.x; k < r.x + r.y; k++) {
                        const float4 q = gp[k];
                        const uint32_t id = __float_as_uint(q.w);
                        if (P.alive[id] && in_dbox(b, q.x, q.y, q.z)) consider(q.x, q.y, q.z, id);
                    }
                }
        for (uint32_t s = 0; s < ns; s++) {
            const float4 q = seq[s];
            const uint32_t qi = __float_as_uint(q.w);
            if (qi != 0xFFFFFFFFu && in_dbox(b, q.x, q.y, q.z)) consider(q.x, q.y, q.z, (unsigned long long)P.base + qi);
        }
        const bool newer = !(cnt > 0 && bd < mid_dist(b, p.x, p.y, p.z));
        if (cnt > 1 && !newer && tie) amb++;
        if (!(cnt > 1 || newer || same_pt(p.x, p.y, p.z, bx, by, bz))) continue;
        events++;
        for (int z = l[2]; z <= h[2]; z++)
            for (int y = l[1]; y <= h[1]; y++)
                for (int x = l[0]; x <= h[0]; x++) {
                    const uint2 r = cell_run(P.gslots, P.glog2, x, y, z);
                    for (uint32_t k = r.x; k < r.x + r.y; k++) {
                        const float4 q = gp[k];
                        const uint32_t id = __float_as_uint(q.w);
                        if (!P.alive[id] || !in_dbox(b, q.x, q.y, q.z) || (!newer && id == bo)) continue;
                        P.alive[id] = 0;
                        deleted++;
                    }
                }
        for (uint32_t s = 0; s < ns; s++) {
            const float4 q = seq[s];
            const uint32_t qi = __float_as_uint(q.w);
            if (qi == 0xFFFFFFFFu || !in_dbox(b, q.x, q.y, q.z) || (!newer && (unsigned long long)P.base + qi == bo))
                continue;
            P.keep[qi] = 0u;
            seq[s].w = __uint_as_float(0xFFFFFFFFu);
        }
        if (newer) {
            P.keep[i] = 1u;
            seq[ns++] = make_float4(p.x, p.y, p.z, __uint_as_float(i));
        }
    }
    if (events) atomicAdd(P.ctr + kDynEvents, events);
    if (deleted) atomicAdd(P.ctr + kDynDeleted, deleted);
    if (amb) atomicAdd(P.ctr + kDynAmbig, amb);
    return ns;
}

constexpr int kFinishThreads = 1024;
constexpr uint32_t kFinishList = 2048;  // lists up to this long are ordered by rank counts in LDS
// The positions i < n with flags[i] != 0 in input order: emit(i, rank); one
// workgroup, four flags per thread per step.  Returns the count.
template <class F>
__device__ uint32_t block_compact(const uint32_t* __restrict__ flags, int64_t n, F&& emit) {
    __shared__ uint32_t wsum[kFinishThreads / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t carry = 0;
    for (int64_t c0 = 0; c0 < n; c0 += 4 * kFinishThreads) {
        const int64_t i0 = c0 + 4 * (int64_t)threadIdx.x;
        uint32_t f[4];
#pragma unroll
        for (int u = 0; u < 4; u++) f[u] = (i0 + u < n && flags[i0 + u]) ? 1u : 0u;
        const uint32_t mine = f[0] + f[1] + f[2] + f[3];
        uint32_t inc = mine;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t v = __shfl_up(inc, off, 64);
            if (lane >= off) inc += v;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        uint32_t woff = 0, tot = 0;
        for (int w = 0; w < kFinishThreads / 64; w++) {
            const uint32_t v = wsum[w];
            woff += w < wave ? v : 0u;
            tot += v;
        }
        uint32_t r = carry + woff + inc - mine;
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (f[u]) emit(i0 + u, r++);
        carry += tot;
        __syncthreads();
    }
    return carry;
}
// The input indices in `src` (m distinct values) in increasing order into dst (LDS ranks).
__device__ __forceinline__ void block_rank_sort(const uint32_t* src, uint32_t m, uint32_t* dst) {
    for (uint32_t t = threadIdx.x; t < m; t += kFinishThreads) {
        const uint32_t v = src[t];
        uint32_t r = 0;
        for (uint32_t j = 0; j < m; j++) r += src[j] < v ? 1u : 0u;
        dst[r] = v;
    }
}

// After k_add_box, one workgroup: the deferred points in input order (ranked
// in LDS, or compacted from the flags past kFinishList), Add_Points' loop over
// them on one thread (add_seq), then the kept points in input order get the
// next ids (k_add_box's box winners + the loop's), their coordinates and
// alive flags; ctr[kDynAdded] the count.  Without downsampling every point is
// kept in input order.
__global__ __launch_bounds__(kFinishThreads) void k_add_finish(DynAddParams P, float4* all, uint8_t* alive) {
    __shared__ uint32_t A[kFinishList], B[kFinishList];
    __shared__ uint32_t ns_s, nk_s;
    if (P.ctr[kDynError]) return;  // a refused batch changes nothing (block-uniform)
    const float4* __restrict__ W = reinterpret_cast<const float4*>(P.W);
    auto put = [&](uint32_t i, uint32_t r) {
        const uint32_t id = (uint32_t)(P.base + (int64_t)r);
        const float4 p = W[i];
        all[id] = make_float4(p.x, p.y, p.z, __uint_as_float(id));
        alive[id] = 1;
    };
    if (!P.downsample) {
        for (int64_t i = threadIdx.x; i < P.n; i += kFinishThreads) put((uint32_t)i, (uint32_t)i);
        if (threadIdx.x == 0) P.ctr[kDynAdded] = (unsigned long long)P.n;
        return;
    }
    // the deferred points in input order
    const uint32_t D = (uint32_t)P.ctr[kDynDeferred];
    const uint32_t* list = B;
    if (D <= kFinishList) {
        for (uint32_t t = threadIdx.x; t < D; t += kFinishThreads) A[t] = P.dlist_u[t];
        __syncthreads();
        block_rank_sort(A, D, B);
    } else {
        block_compact(P.defer, P.n, [&](int64_t i, uint32_t r) { P.dlist[r] = (uint32_t)i; });
        list = P.dlist;
    }
    __syncthreads();
    if (threadIdx.x == 0) ns_s = D ? add_seq(P, list, D) : 0u;
    __syncthreads();
    // the kept points in input order: the box winners, then the loop's survivors
    const uint32_t nb = (uint32_t)P.ctr[kDynKept], ns = ns_s;
    if (threadIdx.x == 0) nk_s = nb;
    __syncthreads();
    const float4* seq = reinterpret_cast<const float4*>(P.seq);
    bool fits = nb + ns <= kFinishList;
    if (fits) {
        for (uint32_t t = threadIdx.x; t < nb; t += kFinishThreads) A[t] = P.klist[t];
        for (uint32_t t = threadIdx.x; t < ns; t += kFinishThreads) {
            const uint32_t qi = __float_as_uint(seq[t].w);
            if (qi != 0xFFFFFFFFu) A[atomicAdd(&nk_s, 1u)] = qi;
        }
        __syncthreads();
        const uint32_t K = nk_s;
        block_rank_sort(A, K, B);
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < K; t += kFinishThreads) put(B[t], t);
        if (threadIdx.x == 0) P.ctr[kDynAdded] = K;
    } else {
        const uint32_t K = block_compact(P.keep, P.n, [&](int64_t i, uint32_t r) { put((uint32_t)i, r); });
        if (threadIdx.x == 0) P.ctr[kDynAdded] = K;
    }
}

// ------------------------------------------------------ grid rebuild ------
__global__ void k_dyn_seed(const float4* __restrict__ gpts, int64_t M, float4* all, uint8_t* alive) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= M) return;
    const float4 q = gpts[k];
    const uint32_t id = __float_as_uint(q.w);
    all[id] = q;
    alive[id] = 1;
}


// Cell key of a point (k_knn_grid's cell_of: floor((p - org) * inv) in float);
// `bad` if outside the grid's key range (clamped).
__device__ __forceinline__ unsigned long long cell_key_of(const float4 p, float ox, float oy, float oz, float inv,
                                                          bool& bad) {
    const float lim = (float)(kGridBias - 8);
    float c[3] = {floorf((p.x - ox) * inv), floorf((p.y - oy) * inv), floorf((p.z - oz) * inv)};
#pragma unroll
    for (int a = 0; a < 3; a++) {
        if (!(fabsf(c[a]) < lim)) bad = true;
        c[a] = fminf(fmaxf(c[a], -lim), lim);
    }
    return pack_key((int)c[0], (int)c[1], (int)c[2]);
}
// Cell key of every alive point.
__global__ void k_dyn_cellkeys(const float4* __restrict__ all, const uint8_t* __restrict__ alive, int64_t n_ids,
                               float ox, float oy, float oz, float inv, unsigned long long* keys, uint32_t* vals,
                               unsigned long long* ctr) {
    const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n_ids) return;
    vals[id] = (uint32_t)id;
    if (!alive[id]) {
        keys[id] = ~0ull;
        return;
    }
    bool bad = false;
    keys[id] = cell_key_of(all[id], ox, oy, oz, inv, bad);
    if (bad) atomicOr(ctr + kDynError, 4ull);
}

// ---- one-launch exclusive scan (decoupled look-back) with fused input / output ----
// Tiles of kScanTile values; a tile takes its number from a ticket counter
// (tiles are claimed in the order they run, so a tile only waits on tiles
// that are running or done), publishes its aggregate, looks back over the
// tiles before it (64 at a time, one wave) for their aggregates up to the
// nearest published prefix, then publishes its own prefix.  Status words:
// value (bits 0-31), flag (32-33: 1 aggregate, 2 prefix), the call's epoch
// (34-63), so the status array is never cleared.  A look-back that waits
// ~seconds gives up and sets ctr bit 64 (the caller fails the call).
constexpr int kScanThreads = 256, kScanItems = 8, kScanTile = kScanThreads * kScanItems;
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr_i(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}
struct ScanState {
    unsigned long long* ticket;  // tickets issued so far (device)
    unsigned long long base;     // the tickets issued before this call
    unsigned long long* status;  // per tile
    unsigned long long epoch;    // this call's (30 bits)
    unsigned long long* err;     // ctr + kDynError
};
__device__ __forceinline__ unsigned long long scan_word(unsigned long long epoch, unsigned flag, uint32_t v) {
    return (epoch << 34) | ((unsigned long long)flag << 32) | v;
}
template <int ITEMS = kScanItems, class In, class Out>
__device__ __forceinline__ void block_scan_lookback(int64_t n, const ScanState& S, In&& in, Out&& out) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    __shared__ uint32_t s_tile, s_prefix;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        const unsigned long long t = atomicAdd(S.ticket, 1ull) - S.base;
        s_tile = t < gridDim.x ? (uint32_t)t : 0xFFFFFFFFu;
        if (t >= gridDim.x) atomicOr(S.err, 64ull);  // (tickets out of step: never expected)
    }
    __syncthreads();
    if (s_tile == 0xFFFFFFFFu) return;
    const int64_t tile = s_tile;
    const int64_t i0 = tile * (kScanThreads * ITEMS) + (int64_t)threadIdx.x * ITEMS;
    uint32_t v[ITEMS], mine = 0;
#pragma unroll
    for (int u = 0; u < ITEMS; u++) {
        v[u] = i0 + u < n ? in(i0 + u) : 0u;
        mine += v[u];
    }
    uint32_t inc = mine;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(inc, off, 64);
        if (lane >= off) inc += t;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t woff = 0, agg = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; w++) {
        woff += w < wave ? wsum[w] : 0u;
        agg += wsum[w];
    }
    if (wave == 0) {
        auto* st = gptr_i(S.status);
        if (tile == 0) {
            if (lane == 0) {
                __hip_atomic_store(st, scan_word(S.epoch, 2, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_prefix = 0u;
            }
        } else {
            if (lane == 0)
                __hip_atomic_store(st + tile, scan_word(S.epoch, 1, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint32_t prefix = 0;
            int64_t hi = tile - 1;  // look at tiles hi, hi-1, ... (lane j: hi - j)
            int spins = 0;
            for (;;) {
                const int64_t t = hi - lane;
                unsigned long long w = scan_word(S.epoch, 2, 0);  // (before tile 0: a zero prefix)
                if (t >= 0) w = __hip_atomic_load(st + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const bool ready = (w >> 34) == S.epoch && ((w >> 32) & 3ull) != 0;
                if (__ballot(!ready)) {  // some tile of the window has not published: wait
                    if (++spins > (1 << 22)) {
                        if (lane == 0) atomicOr(S.err, 64ull);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                const unsigned long long pref = __ballot(((w >> 32) & 3ull) == 2);
                const int stop = pref ? __builtin_ctzll(pref) : 64;  // the nearest tile with a prefix
                uint32_t x = lane <= stop ? (uint32_t)w : 0u;
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
                prefix += x;
                if (pref) break;
                hi -= 64;
                spins = 0;
            }
            if (lane == 0) {
                __hip_atomic_store(st + tile, scan_word(S.epoch, 2, prefix + agg), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                s_prefix = prefix;
            }
        }
    }
    __syncthreads();
    uint32_t r = s_prefix + woff + inc - mine;
#pragma unroll
    for (int u = 0; u < ITEMS; u++) {
        if (i0 + u < n) out(i0 + u, r, v[u]);
        r += v[u];
    }
}
// rank[i] = survivors of the old grid before i (i <= na_old; flag = alive[id of gpts[i]]).
__global__ __launch_bounds__(kScanThreads) void k_scan_flags(const float4* __restrict__ gpts, int64_t na_old,
                                                             const uint8_t* __restrict__ alive, uint32_t* rank,
                                                             ScanState S, GridSlot* clr, int64_t clr_n) {
    // (optional: the hash table the rebuild fills next, cleared here -- k_iv_clear's work)
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < clr_n; t += (int64_t)gridDim.x * blockDim.x)
        clr[t] = GridSlot{kGridEmpty, 0u, 0u};
    block_scan_lookback(
        na_old + 1, S,
        [&](int64_t i) { return i < na_old ? (uint32_t)alive[__float_as_uint(gpts[i].w)] : 0u; },
        [&](int64_t i, uint32_t r, uint32_t) { rank[i] = r; });
}
// Runs of equal keys: starts[run] = first position, starts[runs] = n, *nruns = runs.
__global__ __launch_bounds__(kScanThreads) void k_scan_runs(const unsigned long long* __restrict__ keys, int64_t n,
                                                            uint32_t* starts, unsigned long long* nruns, ScanState S,
                                                            const unsigned long long* dn) {
    if (dn) n = (int64_t)*dn;  // the count on the device (n: the bound the tiles were sized for)
    block_scan_lookback(
        n, S, [&](int64_t i) { return (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u; },
        [&](int64_t i, uint32_t r, uint32_t h) {
            if (h) starts[r] = (uint32_t)i;
            if (i == n - 1) {
                starts[r + h] = (uint32_t)n;
                *nruns = r + h;
            }
        });
}

// Add_Points' box runs in one launch: the sorted points' run heads in (with the
// points in box order into Ws, the 64-bit keys, the wrapped-key clash check of
// the old k_add_heads), starts[run] / the run count / the crowded-box list out (a run
// is crowded when the key kBoxSmall positions on is still its own).
constexpr int kBoxScanItems = 2;  // (the input gathers a point per item: fewer in sequence per thread)
__global__ __launch_bounds__(kScanThreads) void k_scan_boxes(DynAddParams P, ScanState S) {
    const float4* __restrict__ W = reinterpret_cast<const float4*>(P.W);
    block_scan_lookback<kBoxScanItems>(
        P.n, S,
        [&](int64_t k) {
            const uint32_t i = P.svals[k];
            bool head;
            if (P.skeys32) {
                const unsigned long long key = P.keys[i];
                head = k == 0 || P.skeys32[k] != P.skeys32[k - 1];
                if (!head && P.keys[P.svals[k - 1]] != key) atomicOr(P.ctr + kDynError, 32ull);
                P.skeys_w[k] = key;
            } else {
                head = k == 0 || P.skeys[k] != P.skeys[k - 1];
            }
            const float4 p = W[i];
            reinterpret_cast<float4*>(P.Ws)[k] = make_float4(p.x, p.y, p.z, __uint_as_float(i));
            return head ? 1u : 0u;
        },
        [&](int64_t k, uint32_t r, uint32_t h) {
            if (h) {
                P.starts[r] = (uint32_t)k;
                const int64_t e = k + kBoxSmall;
                if (e < P.n && (P.skeys32 ? P.skeys32[e] == P.skeys32[k] : P.skeys[e] == P.skeys[k]))
                    P.bigs[atomicAdd(P.ctr + kDynBig, 1ull)] = r;
            }
            if (k == P.n - 1) {
                P.starts[r + h] = (uint32_t)P.n;
                P.ctr[kDynRuns] = r + h;
            }
        });
}

// ---- the grid merged instead of re-sorted (dyn_rebuild's incremental path) ----
// The new ids' cell keys sorted by (key, index), m <= kNewSortMax: every
// workgroup keys all of them into LDS, then kNewSortSplit lanes count one key's rank, each
// over its share of the keys (broadcast reads), summed by shuffles.
constexpr int kNewSortSplit = 16;
__global__ __launch_bounds__(256) void k_dyn_newsort(const float4* __restrict__ all, const uint8_t* __restrict__ alive,
                                                     int64_t m, float ox, float oy, float oz, float inv,
                                                     unsigned long long* skeys, uint32_t* svals,
                                                     unsigned long long* ctr, const unsigned long long* dm,
                                                     unsigned long long* rerr) {
    __shared__ unsigned long long K[kNewSortMax];
    if (dm) {  // the count on the device (Add_Points' kept points), m the grid's bound
        const unsigned long long md = *dm;
        if (md > (unsigned long long)kNewSortMax) {  // too many for one workgroup: the caller sorts instead
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(rerr, 1ull);
            return;
        }
        if ((int64_t)blockIdx.x * (256 / kNewSortSplit) >= (int64_t)md) return;
        m = (int64_t)md;
    }
    const int mm = (int)m;
    bool bad = false;
    for (int i = threadIdx.x; i < mm; i += blockDim.x)
        K[i] = alive[i] ? cell_key_of(all[i], ox, oy, oz, inv, bad) : ~0ull;
    if (bad && blockIdx.x == 0) atomicOr(ctr + kDynError, 4ull);
    __syncthreads();
    const int i = (blockIdx.x * blockDim.x + threadIdx.x) / kNewSortSplit;  // (the lanes of i: one wave)
    const int q = threadIdx.x % kNewSortSplit;
    const int ii = i < mm ? i : mm - 1;
    const unsigned long long key = K[ii];
    const int per = (mm + kNewSortSplit - 1) / kNewSortSplit, j1 = min(mm, (q + 1) * per);
    int r = 0;
    for (int j = q * per; j < j1; j++) {
        const unsigned long long kj = K[j];
        r += (int)(kj < key) | ((int)(kj == key) & (int)(j < ii));
    }
#pragma unroll
    for (int off = 1; off < kNewSortSplit; off <<= 1) r += __shfl_xor(r, off, kNewSortSplit);
    if (q == 0 && i < mm) {
        skeys[r] = key;
        svals[r] = (uint32_t)i;
    }
}
// The merged grid in (cell key, id) order: the old grid's survivors keep their
// order and go before the new points of the same cell (their ids are smaller);
// the new points come sorted by (key, id).  A survivor's position = survivors
// before it + new keys below its key; a new point's = new points before it +
// survivors with key <= its key (a binary search of the old grid, keys from the
// points as k_dyn_cellkeys computes them).
__global__ void k_dyn_merge(DynMergeParams P) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float4* out = reinterpret_cast<float4*>(P.out);
    const float4* __restrict__ gp = reinterpret_cast<const float4*>(P.gpts);
    bool bad = false;
    const int64_t m_grid = P.m;  // threads for the new points (the bound when the count is on the device)
    if (P.dm) {  // the counts on the device: m = Add_Points' kept points, na = survivors + m
        P.m = (int64_t)*P.dm;
        P.na = (int64_t)P.rank[P.na_old] + P.m;
        if (t == 0) *P.dna = (unsigned long long)P.na;
        if (P.m > m_grid) {
            if (t == 0) atomicOr(P.ctr + kDynError, 16ull);
            return;
        }
    }
    if (t < P.na_old) {
        const float4 q = gp[t];
        if (!P.alive[__float_as_uint(q.w)]) return;
        const unsigned long long key = cell_key_of(q, P.org[0], P.org[1], P.org[2], P.inv, bad);
        int64_t lo = 0, hi = P.m;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (P.nkeys[mid] < key) lo = mid + 1; else hi = mid;
        }
        const int64_t pos = (int64_t)P.rank[t] + lo;
        if (pos >= P.na) {
            atomicOr(P.ctr + kDynError, 16ull);
            return;
        }
        out[pos] = q;
        P.okeys[pos] = key;
    } else if (t < P.na_old + m_grid) {
        const int64_t j = t - P.na_old;
        if (j >= P.m) return;
        const unsigned long long key = P.nkeys[j];
        if (key == ~0ull) return;  // (a dead new id sorts last)
        int64_t lo = 0, hi = P.na_old;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (cell_key_of(gp[mid], P.org[0], P.org[1], P.org[2], P.inv, bad) <= key) lo = mid + 1; else hi = mid;
        }
        const int64_t pos = j + (int64_t)P.rank[lo];
        if (pos >= P.na) {
            atomicOr(P.ctr + kDynError, 16ull);
            return;
        }
        out[pos] = reinterpret_cast<const float4*>(P.all)[P.g0 + P.nidx[j]];
        P.okeys[pos] = key;
    } else if (t < P.na_old + m_grid + 3) {  // chunk padding of k_knn_grid
        out[P.na + (t - P.na_old - m_grid)] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

__global__ void k_dyn_gather(const unsigned long long* __restrict__ skeys, const uint32_t* __restrict__ sids,
                             int64_t na, const float4* __restrict__ all, float4* gpts, uint32_t* heads) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= na + 3) return;
    if (k >= na) {  // chunk padding of k_knn_grid
        gpts[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    gpts[k] = all[sids[k]];
    heads[k] = (k == 0 || skeys[k] != skeys[k - 1]) ? 1u : 0u;
}

__global__ void k_dyn_runs(const uint32_t* __restrict__ heads, const uint32_t* __restrict__ runid, int64_t na,
                           uint32_t* starts, unsigned long long* nruns) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= na) return;
    if (heads[k]) starts[runid[k]] = (uint32_t)k;
    if (k == na - 1) {
        const uint32_t r = runid[k] + heads[k];
        starts[r] = (uint32_t)na;
        *nruns = r;
    }
}

// `dcells` (optional): the count on the device, `cells` then the bound the table
// was sized for (a count above it inserts nothing and sets ctr bit 8).
__global__ void k_dyn_slots(const unsigned long long* __restrict__ skeys, const uint32_t* __restrict__ starts,
                            int64_t cells, GridSlot* slots, int log2, const unsigned long long* dcells,
                            unsigned long long* err) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (dcells) {
        const int64_t nc = (int64_t)*dcells;
        if (nc > cells) {
            if (g == 0) atomicOr(err, 8ull);
            return;
        }
        cells = nc;
    }
    if (g >= cells) return;
    const uint32_t s0 = starts[g], s1 = starts[g + 1];
    const unsigned long long key = skeys[s0];
    const uint64_t mask = (1ull << log2) - 1ull;
    uint64_t sl = (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - log2));
    while (atomicCAS(&slots[sl].key, kGridEmpty, key) != kGridEmpty) sl = (sl + 1) & mask;
    slots[sl].start = s0;
    slots[sl].count = s1 - s0;
}

// ---- cell runs (livo_internal.h), built on the device from the cell grid ----
// Entry e = 27 j + b: grid point j in the run of the b-th cell around its own
// cell (offset (b % 3, b / 3 % 3, b / 9) - 1).  The run of cell v is sorted by
// rho2, the squared distance to v's centre, then by e.  cr_rho2 is also the
// search's termination test (vrun_search): the same float operations, so the
// same bits, and the scan order is exactly the order the test assumes.
struct CrGeo {
    float org[3];
    float h, inv;
};
__device__ __forceinline__ void cr_entry(const CrGeo& G, const float4 p, uint32_t b, int v[3], float& rho2) {
    const int o[3] = {(int)(b % 3u) - 1, (int)((b / 3u) % 3u) - 1, (int)(b / 9u) - 1};
    const float q[3] = {p.x, p.y, p.z};
#pragma unroll
    for (int k = 0; k < 3; k++) v[k] = (int)floorf((q[k] - G.org[k]) * G.inv) + o[k];  // as build_grid_map's cell
    rho2 = cr_rho2(G.org, G.h, v[0], v[1], v[2], p.x, p.y, p.z);
}
__device__ __forceinline__ unsigned long long cr_key(const int v[3]) {
    return (unsigned long long)(v[0] + kGridBias) | ((unsigned long long)(v[1] + kGridBias) << 21) |
           ((unsigned long long)(v[2] + kGridBias) << 42);
}
__global__ void k_cr_rho(const float4* __restrict__ gpts, int64_t n, CrGeo G, uint32_t* rho_bits, uint32_t* iota) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    int v[3];
    float rho2;
    cr_entry(G, gpts[e / 27], (uint32_t)(e % 27), v, rho2);
    rho_bits[e] = __float_as_uint(rho2);  // non-negative: the bits sort as the values
    iota[e] = (uint32_t)e;
}
__global__ void k_cr_key(const float4* __restrict__ gpts, const uint32_t* __restrict__ e1, int64_t n, CrGeo G,
                         unsigned long long* keys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t e = e1[i];
    int v[3];
    float rho2;
    cr_entry(G, gpts[e / 27u], e % 27u, v, rho2);
    keys[i] = cr_key(v);
}
__global__ void k_cr_fill(const float4* __restrict__ gpts, const uint32_t* __restrict__ e2,
                          const unsigned long long* __restrict__ skeys, int64_t n, float4* vpts, uint32_t* heads) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n + 8) return;
    if (i >= n) {  // chunk padding of the run scan (never inside a run: masked by the run length)
        vpts[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    vpts[i] = gpts[e2[i] / 27u];  // x, y, z, map index bits
    heads[i] = (i == 0 || skeys[i] != skeys[i - 1]) ? 1u : 0u;
}

// ---- ball runs (livo_internal.h), built on the device from the cell grid ----
// The run of anchor cell a (edge G.h, same origin as the grid) holds every map
// point whose squared distance to a's centre, cr_rho2 in float, is <= G.rmax2,
// sorted by that value, then by (point, anchor) emission order.  A point emits
// one entry per such anchor: k_br_count counts them, an exclusive scan places
// them, k_br_emit writes (rho2 bits, anchor key, grid point).
struct BrGeo {
    float org[3];
    float h, inv, rmax, rmax2;
    int x0, x1;  // anchors with x index in [x0, x1) only (a chunk of the build)
};
template <class F>
__device__ __forceinline__ void br_anchors(const BrGeo& G, const float4 p, F&& f) {
    const float q[3] = {p.x, p.y, p.z};
    int lo[3], hi[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {  // a cell range that holds every centre within rmax (one cell of slack)
        lo[k] = (int)floorf((q[k] - G.org[k] - G.rmax) * G.inv) - 1;
        hi[k] = (int)floorf((q[k] - G.org[k] + G.rmax) * G.inv) + 1;
    }
    lo[0] = max(lo[0], G.x0);
    hi[0] = min(hi[0], G.x1 - 1);
    for (int z = lo[2]; z <= hi[2]; z++)
        for (int y = lo[1]; y <= hi[1]; y++)
            for (int x = lo[0]; x <= hi[0]; x++) {
                const float r2 = cr_rho2(G.org, G.h, x, y, z, p.x, p.y, p.z);
                if (r2 <= G.rmax2) {
                    const int v[3] = {x, y, z};
                    f(v, r2);
                }
            }
}
__global__ void k_br_count(const float4* __restrict__ gpts, int64_t n, BrGeo G, uint32_t* cnt,
                           unsigned long long* total) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t k = 0;
    if (i < n) {
        br_anchors(G, gpts[i], [&](const int*, float) { k++; });
        cnt[i] = k;
    }
    // block total, one atomic per block (the u32 offsets must not overflow)
    __shared__ unsigned long long part[4];
    unsigned long long v = k;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(total, part[0] + part[1] + part[2] + part[3]);
}
__global__ void k_br_emit(const float4* __restrict__ gpts, int64_t n, BrGeo G, const uint32_t* __restrict__ off,
                          uint32_t* rho_bits, unsigned long long* keys, uint32_t* pt, uint32_t* iota) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t e = off[i];
    br_anchors(G, gpts[i], [&](const int* v, float r2) {
        rho_bits[e] = __float_as_uint(r2);  // non-negative: the bits sort as the values
        keys[e] = cr_key(v);
        pt[e] = (uint32_t)i;
        iota[e] = e;
        e++;
    });
}
__global__ void k_br_gather_keys(const unsigned long long* __restrict__ keys, const uint32_t* __restrict__ e1,
                                 int64_t n, unsigned long long* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = keys[e1[i]];
}
__global__ void k_br_fill(const float4* __restrict__ gpts, const uint32_t* __restrict__ pt,
                          const uint32_t* __restrict__ e2, const unsigned long long* __restrict__ skeys, int64_t n,
                          float4* bpts, uint32_t* heads) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n + 8) return;
    if (i >= n) {  // chunk padding of the run scan
        bpts[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    bpts[i] = gpts[pt[e2[i]]];  // x, y, z, map index bits
    heads[i] = (i == 0 || skeys[i] != skeys[i - 1]) ? 1u : 0u;
}
// ---- index runs (LIVO_IDX_RUNS): a run = an aligned segment of grid positions ----
__global__ void k_run_heads(const unsigned long long* __restrict__ skeys, int64_t n, uint32_t* heads) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) heads[i] = (i == 0 || skeys[i] != skeys[i - 1]) ? 1u : 0u;
}
__global__ void k_run_plen(const uint32_t* __restrict__ starts, int64_t nruns, uint32_t* plen) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < nruns) plen[r] = (starts[r + 1] - starts[r] + 3u) & ~3u;
}
__global__ void k_run_place(const uint32_t* __restrict__ e2, const uint32_t* __restrict__ pt,
                            const uint32_t* __restrict__ heads, const uint32_t* __restrict__ runid,
                            const uint32_t* __restrict__ starts, const uint32_t* __restrict__ pstart, int64_t n,
                            uint32_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = runid[i] + heads[i] - 1u;  // runid: exclusive scan of the heads
    const uint32_t pos = pt ? pt[e2[i]] : e2[i] / 27u;
    out[pstart[r] + ((uint32_t)i - starts[r])] = pos;
}
__global__ void k_run_slots(const unsigned long long* __restrict__ skeys, const uint32_t* __restrict__ starts,
                            const uint32_t* __restrict__ pstart, int64_t nruns, GridSlot* slots, int log2) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nruns) return;
    const uint32_t s0 = starts[r], s1 = starts[r + 1];
    const unsigned long long key = skeys[s0];
    const uint64_t mask = (1ull << log2) - 1ull;
    uint64_t sl = (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - log2));
    while (atomicCAS(&slots[sl].key, kGridEmpty, key) != kGridEmpty) sl = (sl + 1) & mask;
    slots[sl].start = pstart[r];
    slots[sl].count = s1 - s0;
}
// ---- runs on the incremental map: base point positions, deletion marks ----
__global__ void k_dyn_rpos(const float4* __restrict__ rpts, int64_t base_n, uint32_t* rpos) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < base_n) rpos[__float_as_uint(rpts[k].w)] = (uint32_t)k;
}
__global__ void k_dyn_tomb(float4* rpts, uint32_t* rpos, const uint8_t* __restrict__ alive, int64_t base_ids,
                           unsigned long long* ctr) {
    const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t marked = 0;
    if (id < base_ids) {
        const uint32_t p = rpos[id];
        if (p != 0xFFFFFFFFu && !alive[id]) {
            rpts[p].x = __uint_as_float(0x7FC00000u);  // NaN: never a candidate (livo_kernels.hip scan_run)
            rpos[id] = 0xFFFFFFFFu;
            marked = 1;
        }
    }
    const unsigned long long b = __ballot(marked);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(ctr + kDynTomb, (unsigned long long)__popcll(b));
}
__global__ void k_count_alive(const uint8_t* __restrict__ alive, int64_t n, unsigned long long* ctr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long b = __ballot(i < n && alive[i]);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(ctr + kDynAliveCnt, (unsigned long long)__popcll(b));
}
__global__ void k_add_u32(uint32_t* v, int64_t n, uint32_t add) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] += add;
}

// Delete_Point_Boxes (:501-521): boxes as BoxPointType {vertex_min[3], vertex_max[3]}, half open.
__global__ void k_dyn_delete_boxes(const float4* __restrict__ all, uint8_t* alive, int64_t n_ids,
                                   const float* __restrict__ boxes, int64_t nb, unsigned long long* cnt) {
    const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n_ids || !alive[id]) return;
    const float4 p = all[id];
    for (int64_t b = 0; b < nb; b++) {
        const float* B = boxes + 6 * b;
        if (B[0] <= p.x && B[3] > p.x && B[1] <= p.y && B[4] > p.y && B[2] <= p.z && B[5] > p.z) {
            alive[id] = 0;
            atomicAdd(cnt, 1ull);
            return;
        }
    }
}

// ------------------------------------------------------------ launchers ----
static inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

#define DYN_LAUNCH(kernel, n, ...)                                                              \
    do {                                                                                        \
        if ((n) <= 0) return LIVO_OK;                                                           \
        hipLaunchKernelGGL(kernel, grid_for(n), dim3(256), 0, (hipStream_t)stream, __VA_ARGS__); \
        return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;                          \
    } while (0)

int launch_add_prep(const DynAddParams& p, void* stream) { DYN_LAUNCH(k_add_prep, p.n, p); }
int launch_add_group(const DynAddParams& p, void* stream) {
    if (p.n <= 0) return LIVO_OK;
    const int64_t per_block = 64 * kBoxWaves / 16;  // runs <= n: a 16-lane group per box, at most 64k groups
    const int64_t blocks = (p.n + per_block - 1) / per_block;
    hipLaunchKernelGGL(k_add_box, dim3((unsigned)(kBigBlocks + (blocks < 4096 ? blocks : 4096))), dim3(64 * kBoxWaves),
                       0, (hipStream_t)stream, p);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
int launch_add_finish(const DynAddParams& p, float* all, uint8_t* alive, void* stream) {
    if (p.n <= 0) return LIVO_OK;
    hipLaunchKernelGGL(k_add_finish, dim3(1), dim3(kFinishThreads), 0, (hipStream_t)stream, p,
                       reinterpret_cast<float4*>(all), alive);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
int launch_dyn_seed(const float* gpts, int64_t M, float* all, uint8_t* alive, void* stream) {
    DYN_LAUNCH(k_dyn_seed, M, reinterpret_cast<const float4*>(gpts), M, reinterpret_cast<float4*>(all), alive);
}
int launch_dyn_cellkeys(const float* all, const uint8_t* alive, int64_t n_ids, const float* org, float inv,
                        unsigned long long* keys, uint32_t* vals, unsigned long long* ctr, void* stream) {
    DYN_LAUNCH(k_dyn_cellkeys, n_ids, reinterpret_cast<const float4*>(all), alive, n_ids, org[0], org[1], org[2], inv,
               keys, vals, ctr);
}
int launch_dyn_gather(const unsigned long long* skeys, const uint32_t* sids, int64_t na, const float* all, float* gpts,
                      uint32_t* heads, void* stream) {
    DYN_LAUNCH(k_dyn_gather, na + 3, skeys, sids, na, reinterpret_cast<const float4*>(all),
               reinterpret_cast<float4*>(gpts), heads);
}
int launch_dyn_runs(const uint32_t* heads, const uint32_t* runid, int64_t na, uint32_t* starts,
                    unsigned long long* nruns, void* stream) {
    DYN_LAUNCH(k_dyn_runs, na, heads, runid, na, starts, nruns);
}
int launch_dyn_slots(const unsigned long long* skeys, const uint32_t* starts, int64_t cells, GridSlot* slots, int log2,
                     void* stream, const unsigned long long* dcells, unsigned long long* err) {
    DYN_LAUNCH(k_dyn_slots, cells, skeys, starts, cells, slots, log2, dcells, err);
}
int launch_dyn_newsort(const float* all, const uint8_t* alive, int64_t m, const float* org, float inv,
                       unsigned long long* skeys, uint32_t* svals, unsigned long long* ctr, void* stream,
                       const unsigned long long* dm, unsigned long long* rerr) {
    if (m <= 0) return LIVO_OK;
    if (m > kNewSortMax) {
        if (!dm) return LIVO_E_RANGE;
        m = kNewSortMax;  // (a device count above it is flagged in rerr)
    }
    hipLaunchKernelGGL(k_dyn_newsort, dim3((unsigned)((m * kNewSortSplit + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(all), alive, m, org[0], org[1], org[2], inv, skeys, svals, ctr,
                       dm, rerr);
    return hipGetLastError() == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}
static ScanState scan_state(const ScanCtx& sc, int64_t tiles) {
    ScanState S;
    S.ticket = sc.ticket;
    S.base = sc.issued;
    S.status = sc.status;
    S.epoch = sc.epoch & ((1ull << 30) - 1ull);
    S.err = sc.err;
    return S;
}
static int scan_launch_check(ScanCtx& sc, int64_t tiles) {
    if (hipGetLastError() != hipSuccess) return LIVO_E_HIP;  // (no tickets taken)
    sc.issued += (unsigned long long)tiles;
    sc.epoch++;
    return LIVO_OK;
}
int scan_tiles(int64_t n) { return (int)((n + kScanThreads * kBoxScanItems - 1) / (kScanThreads * kBoxScanItems)); }
int launch_scan_flags(ScanCtx& sc, const float* gpts, int64_t na_old, const uint8_t* alive, uint32_t* rank,
                      void* stream, GridSlot* clr, int64_t clr_n) {
    const int64_t tiles = (na_old + 1 + kScanTile - 1) / kScanTile;
    if (tiles > sc.status_cap) return LIVO_E_RANGE;
    hipLaunchKernelGGL(k_scan_flags, dim3((unsigned)tiles), dim3(kScanThreads), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(gpts), na_old, alive, rank, scan_state(sc, tiles), clr,
                       clr ? clr_n : (int64_t)0);
    return scan_launch_check(sc, tiles);
}
int launch_scan_runs(ScanCtx& sc, const unsigned long long* keys, int64_t n, uint32_t* starts,
                     unsigned long long* nruns, void* stream, const unsigned long long* dn) {
    if (n <= 0) return LIVO_OK;
    const int64_t tiles = (n + kScanTile - 1) / kScanTile;
    if (tiles > sc.status_cap) return LIVO_E_RANGE;
    hipLaunchKernelGGL(k_scan_runs, dim3((unsigned)tiles), dim3(kScanThreads), 0, (hipStream_t)stream, keys, n, starts,
                       nruns, scan_state(sc, tiles), dn);
    return scan_launch_check(sc, tiles);
}
int launch_scan_boxes(ScanCtx& sc, const DynAddParams& p, void* stream) {
    if (p.n <= 0) return LIVO_OK;
    const int64_t tile = kScanThreads * kBoxScanItems, tiles = (p.n + tile - 1) / tile;
    if (tiles > sc.status_cap) return LIVO_E_RANGE;
    hipLaunchKernelGGL(k_scan_boxes, dim3((unsigned)tiles), dim3(kScanThreads), 0, (hipStream_t)stream, p,
                       scan_state(sc, tiles));
    return scan_launch_check(sc, tiles);
}
int launch_dyn_merge(const DynMergeParams& p, void* stream) { DYN_LAUNCH(k_dyn_merge, p.na_old + p.m + 3, p); }
int launch_cr_rho(const float* gpts, int64_t n, const float org[3], float h, uint32_t* rho_bits, uint32_t* iota,
                  void* stream) {
    const CrGeo G{{org[0], org[1], org[2]}, h, 1.0f / h};
    DYN_LAUNCH(k_cr_rho, n, reinterpret_cast<const float4*>(gpts), n, G, rho_bits, iota);
}
int launch_cr_key(const float* gpts, const uint32_t* e1, int64_t n, const float org[3], float h,
                  unsigned long long* keys, void* stream) {
    const CrGeo G{{org[0], org[1], org[2]}, h, 1.0f / h};
    DYN_LAUNCH(k_cr_key, n, reinterpret_cast<const float4*>(gpts), e1, n, G, keys);
}
int launch_cr_fill(const float* gpts, const uint32_t* e2, const unsigned long long* skeys, int64_t n,
                   const float org[3], float h, float* vpts, uint32_t* heads, void* stream) {
    (void)org;
    (void)h;
    DYN_LAUNCH(k_cr_fill, n + 8, reinterpret_cast<const float4*>(gpts), e2, skeys, n,
               reinterpret_cast<float4*>(vpts), heads);
}
static BrGeo br_geo(const float org[3], float h, float rmax, int x0, int x1) {
    return BrGeo{{org[0], org[1], org[2]}, h, 1.0f / h, rmax, rmax * rmax, x0, x1};
}
int launch_br_count(const float* gpts, int64_t n, const float org[3], float h, float rmax, uint32_t* cnt,
                    unsigned long long* total, void* stream, int x0, int x1) {
    DYN_LAUNCH(k_br_count, n, reinterpret_cast<const float4*>(gpts), n, br_geo(org, h, rmax, x0, x1), cnt, total);
}
int launch_br_emit(const float* gpts, int64_t n, const float org[3], float h, float rmax, const uint32_t* off,
                   uint32_t* rho_bits, unsigned long long* keys, uint32_t* pt, uint32_t* iota, void* stream, int x0,
                   int x1) {
    DYN_LAUNCH(k_br_emit, n, reinterpret_cast<const float4*>(gpts), n, br_geo(org, h, rmax, x0, x1), off, rho_bits,
               keys, pt, iota);
}
// One chunk's runs as {key, start >> 2, count} records (the chunk's placed runs
// start at word base + pstart[r], a multiple of 4), for k_trip_slots.
__global__ void k_run_trip(const unsigned long long* __restrict__ skeys, const uint32_t* __restrict__ starts,
                           const uint32_t* __restrict__ pstart, int64_t nruns, unsigned long long base,
                           GridSlot* trip) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nruns) return;
    const uint32_t s0 = starts[r], s1 = starts[r + 1];
    GridSlot g;
    g.key = skeys[s0];
    g.start = (uint32_t)((base + pstart[r]) >> 2);
    g.count = s1 - s0;
    trip[r] = g;
}
__global__ void k_trip_slots(const GridSlot* __restrict__ trip, int64_t nruns, GridSlot* slots, int log2) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nruns) return;
    const GridSlot g = trip[r];
    const uint64_t mask = (1ull << log2) - 1ull;
    uint64_t sl = (uint64_t)((g.key * 0x9E3779B97F4A7C15ull) >> (64 - log2));
    while (atomicCAS(&slots[sl].key, kGridEmpty, g.key) != kGridEmpty) sl = (sl + 1) & mask;
    slots[sl].start = g.start;
    slots[sl].count = g.count;
}
int launch_run_trip(const unsigned long long* skeys, const uint32_t* starts, const uint32_t* pstart, int64_t nruns,
                    unsigned long long base, GridSlot* trip, void* stream) {
    DYN_LAUNCH(k_run_trip, nruns, skeys, starts, pstart, nruns, base, trip);
}
int launch_trip_slots(const GridSlot* trip, int64_t nruns, GridSlot* slots, int log2, void* stream) {
    DYN_LAUNCH(k_trip_slots, nruns, trip, nruns, slots, log2);
}
int launch_br_gather_keys(const unsigned long long* keys, const uint32_t* e1, int64_t n, unsigned long long* out,
                          void* stream) {
    DYN_LAUNCH(k_br_gather_keys, n, keys, e1, n, out);
}
int launch_br_fill(const float* gpts, const uint32_t* pt, const uint32_t* e2, const unsigned long long* skeys,
                   int64_t n, float* bpts, uint32_t* heads, void* stream) {
    DYN_LAUNCH(k_br_fill, n + 8, reinterpret_cast<const float4*>(gpts), pt, e2, skeys, n,
               reinterpret_cast<float4*>(bpts), heads);
}
int launch_add_u32(uint32_t* v, int64_t n, uint32_t add, void* stream) { DYN_LAUNCH(k_add_u32, n, v, n, add); }
int launch_dyn_rpos(const float* rpts, int64_t base_n, uint32_t* rpos, void* stream) {
    DYN_LAUNCH(k_dyn_rpos, base_n, reinterpret_cast<const float4*>(rpts), base_n, rpos);
}
int launch_dyn_tomb(float* rpts, uint32_t* rpos, const uint8_t* alive, int64_t base_ids, unsigned long long* ctr,
                    void* stream) {
    DYN_LAUNCH(k_dyn_tomb, base_ids, reinterpret_cast<float4*>(rpts), rpos, alive, base_ids, ctr);
}
int launch_count_alive(const uint8_t* alive, int64_t n, unsigned long long* ctr, void* stream) {
    DYN_LAUNCH(k_count_alive, n, alive, n, ctr);
}
int launch_run_heads(const unsigned long long* skeys, int64_t n, uint32_t* heads, void* stream) {
    DYN_LAUNCH(k_run_heads, n, skeys, n, heads);
}
int launch_run_plen(const uint32_t* starts, int64_t nruns, uint32_t* plen, void* stream) {
    DYN_LAUNCH(k_run_plen, nruns, starts, nruns, plen);
}
int launch_run_place(const uint32_t* e2, const uint32_t* pt, const uint32_t* heads, const uint32_t* runid,
                     const uint32_t* starts, const uint32_t* pstart, int64_t n, uint32_t* out, void* stream) {
    DYN_LAUNCH(k_run_place, n, e2, pt, heads, runid, starts, pstart, n, out);
}
int launch_run_slots(const unsigned long long* skeys, const uint32_t* starts, const uint32_t* pstart, int64_t nruns,
                     GridSlot* slots, int log2, void* stream) {
    DYN_LAUNCH(k_run_slots, nruns, skeys, starts, pstart, nruns, slots, log2);
}
int launch_dyn_delete_boxes(const float* all, uint8_t* alive, int64_t n_ids, const float* boxes, int64_t nb,
                            unsigned long long* cnt, void* stream) {
    DYN_LAUNCH(k_dyn_delete_boxes, n_ids, reinterpret_cast<const float4*>(all), alive, n_ids, boxes, nb, cnt);
}

}  // namespace livo
