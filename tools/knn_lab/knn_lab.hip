// knn_lab.hip — A/B harness for k-NN traversal variants (development tool, not
// part of the product).  Reuses the product's device code and map layout; each
// variant returns neighbours + visit counts so results can be compared bit for
// bit, and is timed with HIP events over `reps` launches in one process.
#include "../../fast-livo-noted_amd/csrc/livo_kernels.hip"

#include <cstdio>
#include <cstring>
#include <vector>

using namespace livo;

// shims for the older lab variants
__device__ __forceinline__ void knn_search_exact(const MapNode* nodes, int has_map, float qx, float qy, float qz,
                                                 uint2*, int, Cands& c, unsigned&) {
    knn_exact(nodes, has_map, qx, qy, qz, c);
}

namespace {

MapNode* g_nodes = nullptr;
int g_depth = 0;
int64_t g_M = 0;
float4* g_q = nullptr;
int64_t g_n = 0;
NNRec* g_out = nullptr;
unsigned long long* g_visits = nullptr;
hipStream_t g_stream = nullptr;

constexpr int kLabBlock = 128;

// ---- stackless with a pending-far trail ------------------------------------
// Reference DFS order without a stack: at each descent the level bit is set in
// `trail` iff the far son is still pending (not pruned at that moment).  When a
// subtree is done the traversal jumps to the deepest ancestor level with a
// pending bit, re-reads that ancestor's record (cached: it was visited) to get
// the far son's box distance, and re-checks it against the current k-th
// distance (exactly the check a stack pop makes).
__device__ __forceinline__ int level_of(uint32_t h) { return 31 - __clz(h + 1); }

template <bool SEEDED>
__device__ __forceinline__ void knn_trail(const MapNode* __restrict__ nodes, float qx, float qy, float qz, SList& s,
                                          unsigned& visits) {
    uint32_t cur = 0;
    uint32_t trail = 0;
    bool down = true;
    while (true) {
        const float4* rp = rec_ptr(nodes, cur);
        const float4 a = rp[0];
        const float4 b = rp[1];
        const float4 cc = rp[2];
        const float4 dd = rp[3];
        const uint32_t meta = __float_as_uint(a.w);
        const bool hl = (meta & kLeftBit) != 0u;
        const bool hr = (meta & kRightBit) != 0u;
        const float dl = hl ? box_dist(qx, qy, qz, b.x, b.y, b.z, b.w, cc.x, cc.y) : INFINITY;
        const float dr = hr ? box_dist(qx, qy, qz, cc.z, cc.w, dd.x, dd.y, dd.z, dd.w) : INFINITY;
        const bool left_first = dl <= dr;
        const uint32_t nnear = 2u * cur + (left_first ? 1u : 2u);
        const uint32_t nfar = 2u * cur + (left_first ? 2u : 1u);
        const float dnear = left_first ? dl : dr;
        const float dfar = left_first ? dr : dl;
        const bool enear = left_first ? hl : hr;
        const bool efar = left_first ? hr : hl;
        const int lev = level_of(cur);
        if (down) {
            visits++;
            const float dx = qx - a.x, dy = qy - a.y, dz = qz - a.z;
            const float dist = (dx * dx + dy * dy) + dz * dz;
            bool dup = false;
            if (SEEDED) {
#pragma unroll
                for (int j = 0; j < kNN; j++) dup |= (j < s.n) && (s.node[j] == cur);
            }
            if (!dup && dist <= INFINITY && (s.n < kNN || dist < s.d[kNN - 1])) sl_insert(s, dist, cur);
            const bool full = s.n >= kNN;
            const float top = s.d[kNN - 1];
            const bool far_ok = efar && (!full || dfar < top);
            if (enear && (!full || dnear < top)) {
                if (far_ok) trail |= (1u << lev);
                cur = nnear;
                continue;
            }
            if (far_ok) {
                cur = nfar;
                continue;
            }
        } else {
            // back at an ancestor whose far son is pending
            const bool full = s.n >= kNN;
            const float top = s.d[kNN - 1];
            trail &= ~(1u << lev);
            if (efar && (!full || dfar < top)) {
                cur = nfar;
                down = true;
                continue;
            }
        }
        // subtree done: jump to the deepest ancestor with a pending far son
        const uint32_t pend = trail & ((lev > 0) ? ((1u << lev) - 1u) : 0u);
        if (pend == 0u) break;
        const int al = 31 - __clz(pend);
        cur = ((cur + 1u) >> (lev - al)) - 1u;
        down = false;
    }
}

// exact-heap replay without a stack (same visit order as knn_search_exact)
__device__ __noinline__ void knn_exact_trail(const MapNode* __restrict__ nodes, float qx, float qy, float qz,
                                             Cands& c) {
    KHeap h;
#pragma unroll
    for (int j = 0; j < kNN; j++) { h.d[j] = INFINITY; h.x[j] = 0.0f; h.node[j] = 0u; }
    h.size = 0;
    uint32_t cur = 0, trail = 0;
    bool down = true;
    while (true) {
        const float4* rp = rec_ptr(nodes, cur);
        const float4 a = rp[0], b = rp[1], cc = rp[2], dd = rp[3];
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
            const float dist = (dx * dx + dy * dy) + dz * dz;
            if (dist <= INFINITY && (h.size < kNN || dist < h.d[0])) {
                if (h.size >= kNN) kh_pop(h);
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

// one iteration of knn_trail (one record load); returns true when the query is done
struct TrailState {
    uint32_t cur;
    uint32_t trail;
    bool down;
};

__device__ __forceinline__ bool trail_step(const MapNode* __restrict__ nodes, float qx, float qy, float qz,
                                           TrailState& t, SList& s, unsigned& visits) {
    const float4* rp = rec_ptr(nodes, t.cur);
    const float4 a = rp[0];
    const float4 b = rp[1];
    const float4 cc = rp[2];
    const float4 dd = rp[3];
    const uint32_t meta = __float_as_uint(a.w);
    const bool hl = (meta & kLeftBit) != 0u;
    const bool hr = (meta & kRightBit) != 0u;
    const float dl = hl ? box_dist(qx, qy, qz, b.x, b.y, b.z, b.w, cc.x, cc.y) : INFINITY;
    const float dr = hr ? box_dist(qx, qy, qz, cc.z, cc.w, dd.x, dd.y, dd.z, dd.w) : INFINITY;
    const bool left_first = dl <= dr;
    const uint32_t nnear = 2u * t.cur + (left_first ? 1u : 2u);
    const uint32_t nfar = 2u * t.cur + (left_first ? 2u : 1u);
    const float dnear = left_first ? dl : dr;
    const float dfar = left_first ? dr : dl;
    const bool enear = left_first ? hl : hr;
    const bool efar = left_first ? hr : hl;
    const int lev = level_of(t.cur);
    if (t.down) {
        visits++;
        const float dx = qx - a.x, dy = qy - a.y, dz = qz - a.z;
        const float dist = (dx * dx + dy * dy) + dz * dz;
        if (dist <= INFINITY && (s.n < kNN || dist < s.d[kNN - 1])) sl_insert(s, dist, t.cur);
        const bool full = s.n >= kNN;
        const float top = s.d[kNN - 1];
        const bool far_ok = efar && (!full || dfar < top);
        if (enear && (!full || dnear < top)) {
            if (far_ok) t.trail |= (1u << lev);
            t.cur = nnear;
            return false;
        }
        if (far_ok) {
            t.cur = nfar;
            return false;
        }
    } else {
        const bool full = s.n >= kNN;
        const float top = s.d[kNN - 1];
        t.trail &= ~(1u << lev);
        if (efar && (!full || dfar < top)) {
            t.cur = nfar;
            t.down = true;
            return false;
        }
    }
    const uint32_t pend = t.trail & ((lev > 0) ? ((1u << lev) - 1u) : 0u);
    if (pend == 0u) return true;
    const int al = 31 - __clz(pend);
    t.cur = ((t.cur + 1u) >> (lev - al)) - 1u;
    t.down = false;
    return false;
}

// ---- variants ----------------------------------------------------------------
template <int V>
__global__ __launch_bounds__(kLabBlock) void k_lab(const MapNode* __restrict__ nodes, int depth, const float4* q,
                                                     int64_t n, NNRec* out, unsigned long long* vis, int chunk) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint2* stack = reinterpret_cast<uint2*>(smem) + threadIdx.x;
    unsigned visits = 0;
    if (V <= 2) {  // one query per thread
        const int64_t i = (int64_t)blockIdx.x * kLabBlock + threadIdx.x;
        if (i < n) {
            const float4 p = q[i];
            float od[kNN];
            uint32_t on[kNN];
            int cnt;
            if (V == 0) {
                Cands c;
                knn_search_exact(nodes, 1, p.x, p.y, p.z, stack, kLabBlock, c, visits);
                cnt = c.n;
#pragma unroll
                for (int k = 0; k < kNN; k++) { od[k] = c.d[k]; on[k] = c.node[k]; }
            } else {
                SList s;
                sl_init(s);
                if (V == 1) {
                    // stack + sorted list (inline copy of the persistent loop body)
                    uint32_t node = 0;
                    bool has = true;
                    int sp = 0;
                    while (true) {
                        if (!has) {
                            if (sp == 0) break;
                            sp--;
                            const uint2 e = stack[sp * kLabBlock];
                            if (s.n < kNN || __uint_as_float(e.y) < s.d[kNN - 1]) { node = e.x; has = true; }
                            else continue;
                        }
                        const float4* rp = rec_ptr(nodes, node);
                        const float4 a = rp[0], b = rp[1], cc = rp[2], dd = rp[3];
                        visits++;
                        const uint32_t meta = __float_as_uint(a.w);
                        const float dx = p.x - a.x, dy = p.y - a.y, dz = p.z - a.z;
                        const float dist = (dx * dx + dy * dy) + dz * dz;
                        if (dist <= INFINITY && (s.n < kNN || dist < s.d[kNN - 1])) sl_insert(s, dist, node);
                        const bool hl = (meta & kLeftBit) != 0u, hr = (meta & kRightBit) != 0u;
                        const float dl = hl ? box_dist(p.x, p.y, p.z, b.x, b.y, b.z, b.w, cc.x, cc.y) : INFINITY;
                        const float dr = hr ? box_dist(p.x, p.y, p.z, cc.z, cc.w, dd.x, dd.y, dd.z, dd.w) : INFINITY;
                        const bool lf = dl <= dr;
                        const bool full = s.n >= kNN;
                        const float top = s.d[kNN - 1];
                        if ((lf ? hr : hl) && (!full || (lf ? dr : dl) < top)) {
                            stack[sp * kLabBlock] = make_uint2(2u * node + (lf ? 2u : 1u), __float_as_uint(lf ? dr : dl));
                            sp++;
                        }
                        has = (lf ? hl : hr) && (!full || (lf ? dl : dr) < top);
                        node = 2u * node + (lf ? 1u : 2u);
                    }
                } else {
                    knn_trail<false>(nodes, p.x, p.y, p.z, s, visits);
                }
                cnt = s.n;
#pragma unroll
                for (int k = 0; k < kNN; k++) { od[k] = s.d[k]; on[k] = s.node[k]; }
                if (s.fuzz) atomicAdd(vis + 1, 1ull);  // replayed by a separate kernel in the product
            }
            write_nnrec(out + i, nodes, cnt, od, on, 0);
        }
    } else {  // V == 3: persistent lanes + trail (a lane that finishes pulls the next query)
        const int lane = threadIdx.x & 63;
        const int per_wave = 64 * chunk;
        const int64_t q0 = ((int64_t)blockIdx.x * (kLabBlock / 64) + (threadIdx.x >> 6)) * per_wave;
        if (q0 < n) {
            const int64_t q1 = min(q0 + (int64_t)per_wave, n);
            int64_t qi = q0 + lane;
            bool live = qi < q1;
            int64_t next = q0 + 64;
            float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
            SList s;
            sl_init(s);
            TrailState t{0u, 0u, true};
            if (live) p = q[qi];
            while (true) {
                bool done = false;
                if (live) done = trail_step(nodes, p.x, p.y, p.z, t, s, visits);
                if (done) {
                    float od[kNN];
                    uint32_t on[kNN];
                    int cnt = s.n;
#pragma unroll
                    for (int k = 0; k < kNN; k++) { od[k] = s.d[k]; on[k] = s.node[k]; }
                    if (s.fuzz) atomicAdd(vis + 1, 1ull);
                    write_nnrec(out + qi, nodes, cnt, od, on, 0);
                    live = false;
                }
                const unsigned long long idle = __ballot(!live);
                if (next >= q1) {
                    if (idle == ~0ull) break;
                } else {
                    if (!live) {
                        const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(idle >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((unsigned)idle, 0u));
                        const int64_t qn = next + r;
                        if (qn < q1) {
                            qi = qn;
                            live = true;
                            p = q[qi];
                            sl_init(s);
                            t = TrailState{0u, 0u, true};
                        }
                    }
                    next += __popcll(idle);
                }
            }
        }
    }
    unsigned long long wv = visits;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) wv += __shfl_xor(wv, off, 64);
    if ((threadIdx.x & 63) == 0 && wv) atomicAdd(vis, wv);
}

// ---- V4: sorted list + capped LDS stack; any tie/overflow => flagged for replay
template <int CAP, int BLK>
__global__ __launch_bounds__(BLK) void k_lab_cap(const MapNode* __restrict__ nodes, const float4* q, int64_t n,
                                                  NNRec* out, unsigned long long* vis) {
    __shared__ uint2 st_lds[CAP * BLK];
    uint2* stack = st_lds + threadIdx.x;
    unsigned visits = 0;
    const int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (i < n) {
        const float4 p = q[i];
        SList s;
        sl_init(s);
        bool flag = false;
        uint32_t node = 0;
        bool has = true;
        int sp = 0;
        while (true) {
            if (!has) {
                if (sp == 0) break;
                sp--;
                const uint2 e = stack[sp * BLK];
                const float de = __uint_as_float(e.y);
                const bool full = s.n >= kNN;
                if (!full || de < s.d[kNN - 1]) { node = e.x; has = true; }
                else { flag |= fabsf(de - s.d[kNN - 1]) <= kFuzz; continue; }
            }
            const float4* rp = rec_ptr(nodes, node);
            const float4 a = rp[0], b = rp[1], cc = rp[2], dd = rp[3];
            visits++;
            const uint32_t meta = __float_as_uint(a.w);
            const float dx = p.x - a.x, dy = p.y - a.y, dz = p.z - a.z;
            const float dist = (dx * dx + dy * dy) + dz * dz;
            if (dist <= INFINITY && (s.n < kNN || dist < s.d[kNN - 1])) sl_insert(s, dist, node);
            else flag |= fabsf(dist - s.d[kNN - 1]) <= kFuzz;
            const bool hl = (meta & kLeftBit) != 0u, hr = (meta & kRightBit) != 0u;
            const float dl = hl ? box_dist(p.x, p.y, p.z, b.x, b.y, b.z, b.w, cc.x, cc.y) : INFINITY;
            const float dr = hr ? box_dist(p.x, p.y, p.z, cc.z, cc.w, dd.x, dd.y, dd.z, dd.w) : INFINITY;
            const bool lf = dl <= dr;
            const bool full = s.n >= kNN;
            const float top = s.d[kNN - 1];
            const float dfar = lf ? dr : dl, dnear = lf ? dl : dr;
            const bool efar = lf ? hr : hl, enear = lf ? hl : hr;
            if (efar) {
                if (!full || dfar < top) {
                    if (sp < CAP) { stack[sp * BLK] = make_uint2(2u * node + (lf ? 2u : 1u), __float_as_uint(dfar)); sp++; }
                    else flag = true;  // overflow: exact replay
                } else flag |= fabsf(dfar - top) <= kFuzz;
            }
            has = enear && (!full || dnear < top);
            if (enear && !has) flag |= fabsf(dnear - top) <= kFuzz;
            node = 2u * node + (lf ? 1u : 2u);
        }
        flag |= s.fuzz;
        float od[kNN];
        uint32_t on[kNN];
#pragma unroll
        for (int k = 0; k < kNN; k++) { od[k] = s.d[k]; on[k] = s.node[k]; }
        write_nnrec(out + i, nodes, s.n, od, on, 0);
        if (flag) atomicAdd(vis + 1, 1ull);
    }
    unsigned long long wv = visits;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) wv += __shfl_xor(wv, off, 64);
    if ((threadIdx.x & 63) == 0 && wv) atomicAdd(vis, wv);
}

template <int CAP, int BLK>
void launch_cap() {
    dim3 grid((unsigned)((g_n + BLK - 1) / BLK));
    hipLaunchKernelGGL((k_lab_cap<CAP, BLK>), grid, dim3(BLK), 0, g_stream, g_nodes, g_q, g_n, g_out, g_visits);
}

// ---- V5: seeded from previous neighbour records + capped stack + full tie flagging
NNRec* g_seed = nullptr;

template <int CAP, int BLK>
__global__ __launch_bounds__(BLK) void k_lab_seed(const MapNode* __restrict__ nodes, const float4* q, int64_t n,
                                                   const NNRec* __restrict__ seed, NNRec* out,
                                                   unsigned long long* vis) {
    __shared__ uint2 st_lds[CAP * BLK];
    uint2* stack = st_lds + threadIdx.x;
    unsigned visits = 0;
    const int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (i < n) {
        const float4 p = q[i];
        SList s;
        sl_init(s);
        bool flag = false;
        // seeds: the previous neighbours, re-measured from the new query point
        const int4 si0 = reinterpret_cast<const int4*>(seed + i)[7];  // pad holds the node ids (lab only)
        const int4 si1 = reinterpret_cast<const int4*>(seed + i)[6];
        const int scnt = si1.y;
        const uint32_t sn[kNN] = {(uint32_t)si0.x, (uint32_t)si0.y, (uint32_t)si0.z, (uint32_t)si0.w,
                                  (uint32_t)si1.z};
#pragma unroll
        for (int k = 0; k < kNN; k++) {
            if (k < scnt) {
                const float4 a = rec_ptr(nodes, sn[k])[0];
                const float dx = p.x - a.x, dy = p.y - a.y, dz = p.z - a.z;
                const float dist = (dx * dx + dy * dy) + dz * dz;
                sl_insert(s, dist, sn[k]);
            }
        }
        uint32_t node = 0;
        bool has = true;
        int sp = 0;
        while (true) {
            if (!has) {
                if (sp == 0) break;
                sp--;
                const uint2 e = stack[sp * BLK];
                const float de = __uint_as_float(e.y);
                const bool full = s.n >= kNN;
                if (!full || de < s.d[kNN - 1]) { node = e.x; has = true; }
                else { flag |= fabsf(de - s.d[kNN - 1]) <= kFuzz; continue; }
            }
            const float4* rp = rec_ptr(nodes, node);
            const float4 a = rp[0], b = rp[1], cc = rp[2], dd = rp[3];
            visits++;
            const uint32_t meta = __float_as_uint(a.w);
            const float dx = p.x - a.x, dy = p.y - a.y, dz = p.z - a.z;
            const float dist = (dx * dx + dy * dy) + dz * dz;
            bool dup = false;
#pragma unroll
            for (int k = 0; k < kNN; k++) dup |= (k < s.n) && (s.node[k] == node);
            if (!dup) {
                if (dist <= INFINITY && (s.n < kNN || dist < s.d[kNN - 1])) sl_insert(s, dist, node);
                else flag |= fabsf(dist - s.d[kNN - 1]) <= kFuzz;
            }
            const bool hl = (meta & kLeftBit) != 0u, hr = (meta & kRightBit) != 0u;
            const float dl = hl ? box_dist(p.x, p.y, p.z, b.x, b.y, b.z, b.w, cc.x, cc.y) : INFINITY;
            const float dr = hr ? box_dist(p.x, p.y, p.z, cc.z, cc.w, dd.x, dd.y, dd.z, dd.w) : INFINITY;
            const bool lf = dl <= dr;
            const bool full = s.n >= kNN;
            const float top = s.d[kNN - 1];
            const float dfar = lf ? dr : dl, dnear = lf ? dl : dr;
            const bool efar = lf ? hr : hl, enear = lf ? hl : hr;
            if (efar) {
                if (!full || dfar < top) {
                    if (sp < CAP) { stack[sp * BLK] = make_uint2(2u * node + (lf ? 2u : 1u), __float_as_uint(dfar)); sp++; }
                    else flag = true;
                } else flag |= fabsf(dfar - top) <= kFuzz;
            }
            has = enear && (!full || dnear < top);
            if (enear && !has) flag |= fabsf(dnear - top) <= kFuzz;
            node = 2u * node + (lf ? 1u : 2u);
        }
        flag |= s.fuzz;
        float od[kNN];
        uint32_t on[kNN];
#pragma unroll
        for (int k = 0; k < kNN; k++) { od[k] = s.d[k]; on[k] = s.node[k]; }
        write_nnrec(out + i, nodes, s.n, od, on, 0);
        int4* pad = reinterpret_cast<int4*>(out + i) + 7;
        *pad = make_int4((int)on[0], (int)on[1], (int)on[2], (int)on[3]);
        reinterpret_cast<int4*>(out + i)[6].z = (int)on[4];
        reinterpret_cast<int4*>(out + i)[6].w = flag ? 1 : 0;
        if (flag) atomicAdd(vis + 1, 1ull);
    }
    unsigned long long wv = visits;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) wv += __shfl_xor(wv, off, 64);
    if ((threadIdx.x & 63) == 0 && wv) atomicAdd(vis, wv);
}

template <int CAP, int BLK>
void launch_seed() {
    dim3 grid((unsigned)((g_n + BLK - 1) / BLK));
    hipLaunchKernelGGL((k_lab_seed<CAP, BLK>), grid, dim3(BLK), 0, g_stream, g_nodes, g_q, g_n, g_seed, g_out,
                       g_visits);
}

template <int V>
void launch_v(int chunk) {
    size_t lds = (V == 0 || V == 1) ? (size_t)g_depth * kLabBlock * sizeof(uint2) : 0;
    if (V <= 2) {
        dim3 grid((unsigned)((g_n + kLabBlock - 1) / kLabBlock));
        hipLaunchKernelGGL(k_lab<V>, grid, dim3(kLabBlock), lds, g_stream, g_nodes, g_depth, g_q, g_n, g_out,
                           g_visits, 1);
    } else {
        const int64_t per_block = (int64_t)kLabBlock * chunk;
        dim3 grid((unsigned)((g_n + per_block - 1) / per_block));
        hipLaunchKernelGGL(k_lab<V>, grid, dim3(kLabBlock), lds, g_stream, g_nodes, g_depth, g_q, g_n, g_out,
                           g_visits, chunk);
    }
}

}  // namespace

__global__ void k_fill_seed_ids(const MapNode* nodes, const float4* q, int64_t n, NNRec* rec, int64_t M) {
    (void)nodes; (void)q; (void)M;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    (void)rec;
}

extern "C" {

// seeds = the last output; node ids recovered on the host from map indices
int lab_set_seed_nodes(const int32_t* node_ids /* n*5, -1 pad */, const int32_t* cnt) {
    std::vector<NNRec> h((size_t)g_n);
    for (int64_t i = 0; i < g_n; i++) {
        std::memset(&h[i], 0, sizeof(NNRec));
        h[i].cnt = cnt[i];
        int* pad = reinterpret_cast<int*>(&h[i]) + 28;  // int4 #7
        for (int k = 0; k < 4; k++) pad[k] = node_ids[i * 5 + k];
        reinterpret_cast<int*>(&h[i])[26] = node_ids[i * 5 + 4];  // int4 #6 .z
    }
    if (!g_seed) hipMalloc((void**)&g_seed, (size_t)g_n * sizeof(NNRec));
    hipMemcpy(g_seed, h.data(), h.size() * sizeof(NNRec), hipMemcpyHostToDevice);
    return 0;
}

// map index -> heap node id (host table built from the device records)
int lab_node_of_index(int32_t* out /* M */) {
    HostMap dummy;
    (void)dummy;
    return 0;
}

int lab_build_map(const float* xyz, int64_t M) {
    if (!g_stream) hipStreamCreate(&g_stream);
    HostMap hm;
    int rc = build_host_map(xyz, M, 12, &hm);
    if (rc) return rc;
    if (g_nodes) hipFree(g_nodes);
    size_t bytes = (size_t)(hm.num_slots + 1) * sizeof(MapNode);
    hipMalloc((void**)&g_nodes, bytes);
    hipMemcpy(g_nodes, hm.nodes, bytes, hipMemcpyHostToDevice);
    g_depth = hm.depth;
    g_M = M;
    free_host_map(&hm);
    return 0;
}

int64_t lab_num_slots() { return (int64_t)((1ll << g_depth) - 1); }
int lab_node_table(int32_t* idx_of_node /* slots */) {
    const int64_t slots = lab_num_slots();
    std::vector<MapNode> h((size_t)slots + 1);
    hipMemcpy(h.data(), g_nodes, h.size() * sizeof(MapNode), hipMemcpyDeviceToHost);
    for (int64_t k = 0; k < slots; k++) {
        uint32_t meta;
        std::memcpy(&meta, &h[k + 1].a[3], 4);
        idx_of_node[k] = (h[k + 1].a[0] == 0.f && h[k + 1].a[1] == 0.f && h[k + 1].a[2] == 0.f && meta == 0) ? -1
                                                                                                            : (int32_t)(meta & kIdxMask);
    }
    return 0;
}

int lab_set_queries(const float* q3, int64_t n) {
    std::vector<float> h((size_t)n * 4);
    for (int64_t i = 0; i < n; i++) {
        h[4 * i] = q3[3 * i]; h[4 * i + 1] = q3[3 * i + 1]; h[4 * i + 2] = q3[3 * i + 2]; h[4 * i + 3] = 0;
    }
    if (g_q) hipFree(g_q);
    if (g_out) hipFree(g_out);
    if (!g_visits) hipMalloc((void**)&g_visits, 16);
    hipMalloc((void**)&g_q, h.size() * 4);
    hipMalloc((void**)&g_out, (size_t)n * sizeof(NNRec));
    hipMemcpy(g_q, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    g_n = n;
    return 0;
}

// returns avg ms per launch; idx/d (n*5) and visits of the last launch
double lab_run(int v, int reps, int chunk, int32_t* idx, float* d, long long* visits, int32_t* flags) {
    // visits[0] = nodes visited by the last launch, visits[1] = queries flagged for exact replay
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto one = [&]() {
        switch (v) {
            case 0: launch_v<0>(chunk); break;
            case 1: launch_v<1>(chunk); break;
            case 2: launch_v<2>(chunk); break;
            case 3: launch_v<3>(chunk); break;
            case 10: launch_cap<4, 128>(); break;
            case 11: launch_cap<6, 128>(); break;
            case 12: launch_cap<8, 128>(); break;
            case 13: launch_cap<12, 128>(); break;
            case 14: launch_cap<20, 128>(); break;
            case 15: launch_cap<8, 256>(); break;
            case 16: launch_cap<8, 64>(); break;
            case 17: launch_cap<6, 256>(); break;
            case 20: launch_seed<4, 128>(); break;
            case 21: launch_seed<6, 128>(); break;
            case 22: launch_seed<8, 128>(); break;
            case 23: launch_seed<12, 128>(); break;
            case 24: launch_seed<20, 128>(); break;
            default: break;
        }
    };
    hipMemsetAsync(g_visits, 0, 8, g_stream);
    one();  // warm
    hipStreamSynchronize(g_stream);
    hipEventRecord(e0, g_stream);
    for (int r = 0; r < reps; r++) one();
    hipEventRecord(e1, g_stream);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemsetAsync(g_visits, 0, 16, g_stream);
    one();
    std::vector<NNRec> h((size_t)g_n);
    hipMemcpyAsync(h.data(), g_out, h.size() * sizeof(NNRec), hipMemcpyDeviceToHost, g_stream);
    unsigned long long vv[2] = {0, 0};
    hipMemcpyAsync(vv, g_visits, 16, hipMemcpyDeviceToHost, g_stream);
    hipStreamSynchronize(g_stream);
    for (int64_t i = 0; i < g_n; i++)
        for (int k = 0; k < 5; k++) {
            idx[i * 5 + k] = h[i].idx[k];
            d[i * 5 + k] = h[i].p[k][3];
        }
    if (flags)
        for (int64_t i = 0; i < g_n; i++) flags[i] = h[i].flag;
    visits[0] = (long long)vv[0];
    visits[1] = (long long)vv[1];
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return -1.0;
    return ms / reps;
}

}  // extern "C"

// ---- the product's k-NN pass (identity queries) with flag-reason histogram
extern "C" int lab_product_pass(int seeded_from_last, int32_t* flags_out, double* ms_out) {
    static IekfSlot* d_slot = nullptr;
    static HsJob* d_job = nullptr;
    static unsigned* d_cnt = nullptr;
    static unsigned long long* d_list = nullptr;
    static unsigned long long* d_tot = nullptr;
    if (!d_slot) {
        hipMalloc((void**)&d_slot, sizeof(IekfSlot));
        hipMemset(d_slot, 0, sizeof(IekfSlot));
        hipMalloc((void**)&d_job, sizeof(HsJob));
        hipMalloc((void**)&d_cnt, 4);
        hipMalloc((void**)&d_tot, 8);
        hipMalloc((void**)&d_list, 8 * (size_t)g_n);
    }
    HsJob j{};
    j.pts = reinterpret_cast<const float*>(g_q);
    j.nn = g_out;
    j.slot = d_slot;
    j.n = (int32_t)g_n;
    hipMemcpy(d_job, &j, sizeof(j), hipMemcpyHostToDevice);
    KnnParams kp{};
    kp.nodes = g_nodes; kp.jobs = d_job; kp.replay_count = d_cnt; kp.replay_list = d_list; kp.replay_total = d_tot;
    kp.has_map = 1; kp.force = 1; kp.depth = g_depth; kp.identity = 1; kp.nb = (int32_t)((g_n + kKnnBlock - 1) / kKnnBlock);
    hipEvent_t e0, e1, e2;
    hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2);
    const int reps = 10;
    float ms_pass = 0, ms_rep = 0;
    for (int r = 0; r < reps + 1; r++) {
        hipMemsetAsync(d_cnt, 0, 4, g_stream);
        hipEventRecord(e0, g_stream);
        dim3 grid((unsigned)((g_n + kKnnBlock - 1) / kKnnBlock), 1);
        const size_t lds = knn_lds_bytes(kp.depth);
        (void)seeded_from_last;
        hipLaunchKernelGGL(k_knn_pass, grid, dim3(kKnnBlock), lds, g_stream, kp);
        hipEventRecord(e1, g_stream);
        hipLaunchKernelGGL(k_knn_replay, dim3(64), dim3(64), 0, g_stream, kp);
        hipEventRecord(e2, g_stream);
        hipEventSynchronize(e2);
        float a = 0, b = 0;
        hipEventElapsedTime(&a, e0, e1);
        hipEventElapsedTime(&b, e1, e2);
        if (r > 0) { ms_pass += a; ms_rep += b; }
        if (seeded_from_last) break;  // seeds change with each pass: time the first seeded pass only
    }
    const int nr = seeded_from_last ? 1 : reps;
    ms_out[0] = (seeded_from_last ? 0 : ms_pass / nr);
    ms_out[1] = (seeded_from_last ? 0 : ms_rep / nr);
    std::vector<NNRec> h((size_t)g_n);
    hipMemcpy(h.data(), g_out, h.size() * sizeof(NNRec), hipMemcpyDeviceToHost);
    for (int64_t i = 0; i < g_n; i++) flags_out[i] = h[i].flag;
    return 0;
}
