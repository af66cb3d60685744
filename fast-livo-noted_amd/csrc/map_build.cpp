// map_build.cpp — host construction of the device map (heap-ordered 64-B records).
//
// Same tree as KD_TREE::Build (include/ikd-Tree/ikd_Tree.cpp:337-348) on the
// same input order: BuildTree (:537-602) picks the axis of largest extent over
// Storage[l..r], nth_element-partitions at mid = (l+r)>>1 and recurses on
// [l, mid-1] and [mid+1, r]; Update (:1110-1235) derives each node's bounding
// box from its sons and its point.  We run the same std::nth_element on the
// same element sequence, so the partition of points with equal coordinates
// matches the reference as well.  Instead of 176-B pointer nodes the result is
// written as heap-ordered MapNode records (livo_internal.h), each holding its
// point and its two sons' boxes.  Disjoint subtrees are built on separate
// threads (the result does not depend on the thread count).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "livo_internal.h"

namespace livo {
namespace {

struct BPoint {
    float x, y, z;
    uint32_t idx;
};

struct Box {
    float mn[3], mx[3];
    bool valid;
};

static bool cmp_x(const BPoint& a, const BPoint& b) { return a.x < b.x; }
static bool cmp_y(const BPoint& a, const BPoint& b) { return a.y < b.y; }
static bool cmp_z(const BPoint& a, const BPoint& b) { return a.z < b.z; }

static int tree_depth(int64_t n) {
    int d = 0;
    while (n > 0) {  // larger half of [l, r] after removing mid has ceil((n-1)/2) points
        d++;
        n = n - 1 - ((n - 1) >> 1);
    }
    return d;
}

struct Builder {
    std::vector<BPoint>& st;
    MapNode* nodes;

    Box build(int64_t l, int64_t r, int64_t h, int spawn_levels) {
        Box out{};
        if (l > r) {
            out.valid = false;
            return out;
        }
        int64_t mid = (l + r) >> 1;
        float mn[3] = {INFINITY, INFINITY, INFINITY};
        float mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int64_t i = l; i <= r; i++) {
            mn[0] = std::min(mn[0], st[i].x); mn[1] = std::min(mn[1], st[i].y); mn[2] = std::min(mn[2], st[i].z);
            mx[0] = std::max(mx[0], st[i].x); mx[1] = std::max(mx[1], st[i].y); mx[2] = std::max(mx[2], st[i].z);
        }
        float ext[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
        int axis = 0;
        for (int i = 1; i < 3; i++)
            if (ext[i] > ext[axis]) axis = i;
        auto b = st.begin();
        if (axis == 1) std::nth_element(b + l, b + mid, b + r + 1, cmp_y);
        else if (axis == 2) std::nth_element(b + l, b + mid, b + r + 1, cmp_z);
        else std::nth_element(b + l, b + mid, b + r + 1, cmp_x);
        const BPoint p = st[mid];
        Box bl, br;
        if (spawn_levels > 0 && (r - l) > 65536) {
            std::thread t([&] { bl = build(l, mid - 1, 2 * h + 1, spawn_levels - 1); });
            br = build(mid + 1, r, 2 * h + 2, spawn_levels - 1);
            t.join();
        } else {
            bl = build(l, mid - 1, 2 * h + 1, 0);
            br = build(mid + 1, r, 2 * h + 2, 0);
        }
        MapNode& nd = nodes[h + 1];
        uint32_t meta = p.idx | (bl.valid ? kLeftBit : 0u) | (br.valid ? kRightBit : 0u);
        // An absent son gets an empty box; the kernel never reads it (meta bits).
        Box el = bl.valid ? bl : Box{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}, false};
        Box er = br.valid ? br : Box{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}, false};
        float mw;
        std::memcpy(&mw, &meta, 4);
        nd.a[0] = p.x; nd.a[1] = p.y; nd.a[2] = p.z; nd.a[3] = mw;
        nd.b[0] = el.mn[0]; nd.b[1] = el.mx[0]; nd.b[2] = el.mn[1]; nd.b[3] = el.mx[1];
        nd.c[0] = el.mn[2]; nd.c[1] = el.mx[2]; nd.c[2] = er.mn[0]; nd.c[3] = er.mx[0];
        nd.d[0] = er.mn[1]; nd.d[1] = er.mx[1]; nd.d[2] = er.mn[2]; nd.d[3] = er.mx[2];
        // Update(): ikd_Tree.cpp:1110-1235 for a node without deletions.
        Box o{};
        o.valid = true;
        const float pc[3] = {p.x, p.y, p.z};
        if (bl.valid && br.valid) {
            for (int k = 0; k < 3; k++) {
                o.mn[k] = std::min(std::min(bl.mn[k], br.mn[k]), pc[k]);
                o.mx[k] = std::max(std::max(bl.mx[k], br.mx[k]), pc[k]);
            }
        } else if (bl.valid || br.valid) {
            const Box& s = bl.valid ? bl : br;
            for (int k = 0; k < 3; k++) {
                o.mn[k] = std::min(s.mn[k], pc[k]);
                o.mx[k] = std::max(s.mx[k], pc[k]);
            }
        } else {
            for (int k = 0; k < 3; k++) o.mn[k] = o.mx[k] = pc[k];
        }
        return o;
    }
};

}  // namespace

int build_host_map(const float* xyz, int64_t M, int64_t stride_bytes, HostMap* out) {
    if (!out || M < 0 || (M > 0 && !xyz)) return LIVO_E_INVALID;
    if (M > kMaxMapPoints) return LIVO_E_RANGE;
    if (stride_bytes == 0) stride_bytes = 3 * sizeof(float);
    if (stride_bytes < (int64_t)(3 * sizeof(float))) return LIVO_E_INVALID;
    free_host_map(out);
    int depth = tree_depth(M);
    if (depth > kMaxDepth) return LIVO_E_RANGE;
    int64_t slots = depth > 0 ? ((int64_t)1 << depth) - 1 : 0;
    size_t bytes = (size_t)(slots + 1) * sizeof(MapNode);
    MapNode* nodes = (MapNode*)std::calloc(slots + 1, sizeof(MapNode));
    if (!nodes) return LIVO_E_OOM;
    (void)bytes;
    std::vector<BPoint> st((size_t)M);
    const char* base = (const char*)xyz;
    for (int64_t i = 0; i < M; i++) {
        const float* p = (const float*)(base + i * stride_bytes);
        st[i] = BPoint{p[0], p[1], p[2], (uint32_t)i};
    }
    if (M > 0) {
        Builder b{st, nodes};
        unsigned hw = std::thread::hardware_concurrency();
        int spawn = 0;
        while ((1u << spawn) < std::min(hw ? hw : 1u, 16u)) spawn++;
        b.build(0, M - 1, 0, spawn);
    }
    out->nodes = nodes;
    out->num_points = M;
    out->num_slots = slots;
    out->depth = depth;
    return LIVO_OK;
}

void free_host_map(HostMap* m) {
    if (m && m->nodes) {
        std::free(m->nodes);
        m->nodes = nullptr;
    }
}

}  // namespace livo

// ---------------------------------------------------------------------------
// Leaf map (livo_internal.h): balanced median kd-tree of fixed depth D with
// leaves of <= leaf_size points.  Leaf j = points [j*M >> D, (j+1)*M >> D) of
// the permuted array; node h at level L covers leaves [jl, jl + 2^(D-L)) and is
// split at the first point of its middle leaf, on its longest extent.
// ---------------------------------------------------------------------------
namespace livo {
namespace {

struct LeafBuilder {
    std::vector<BPoint>& st;
    LeafNode* nodes;
    int64_t M;
    int D;

    int64_t leaf_start(int64_t j) const { return (int64_t)(((unsigned __int128)j * (unsigned __int128)M) >> D); }

    Box build(int64_t h, int level, int64_t jl, int spawn_levels) {
        const int64_t nleaves = (int64_t)1 << (D - level);
        const int64_t lo = leaf_start(jl), hi = leaf_start(jl + nleaves);
        Box out{};
        out.valid = true;
        for (int k = 0; k < 3; k++) {
            out.mn[k] = INFINITY;
            out.mx[k] = -INFINITY;
        }
        if (level == D) {
            for (int64_t i = lo; i < hi; i++) {
                const float pc[3] = {st[i].x, st[i].y, st[i].z};
                for (int k = 0; k < 3; k++) {
                    out.mn[k] = std::min(out.mn[k], pc[k]);
                    out.mx[k] = std::max(out.mx[k], pc[k]);
                }
            }
            return out;
        }
        for (int64_t i = lo; i < hi; i++) {
            const float pc[3] = {st[i].x, st[i].y, st[i].z};
            for (int k = 0; k < 3; k++) {
                out.mn[k] = std::min(out.mn[k], pc[k]);
                out.mx[k] = std::max(out.mx[k], pc[k]);
            }
        }
        int axis = 0;
        for (int k = 1; k < 3; k++)
            if (out.mx[k] - out.mn[k] > out.mx[axis] - out.mn[axis]) axis = k;
        const int64_t jm = jl + nleaves / 2, mid = leaf_start(jm);
        auto b = st.begin();
        if (mid > lo && mid < hi) {
            if (axis == 1) std::nth_element(b + lo, b + mid, b + hi, cmp_y);
            else if (axis == 2) std::nth_element(b + lo, b + mid, b + hi, cmp_z);
            else std::nth_element(b + lo, b + mid, b + hi, cmp_x);
        }
        Box bl, br;
        if (spawn_levels > 0 && hi - lo > 65536) {
            std::thread t([&] { bl = build(2 * h + 1, level + 1, jl, spawn_levels - 1); });
            br = build(2 * h + 2, level + 1, jm, spawn_levels - 1);
            t.join();
        } else {
            bl = build(2 * h + 1, level + 1, jl, 0);
            br = build(2 * h + 2, level + 1, jm, 0);
        }
        LeafNode& nd = nodes[h];
        nd.b[0] = bl.mn[0]; nd.b[1] = bl.mx[0]; nd.b[2] = bl.mn[1]; nd.b[3] = bl.mx[1];
        nd.c[0] = bl.mn[2]; nd.c[1] = bl.mx[2]; nd.c[2] = br.mn[0]; nd.c[3] = br.mx[0];
        nd.d[0] = br.mn[1]; nd.d[1] = br.mx[1]; nd.d[2] = br.mn[2]; nd.d[3] = br.mx[2];
        return out;
    }
};

}  // namespace

int build_leaf_map(const float* xyz, int64_t M, int64_t stride_bytes, int leaf_size, HostLeafMap* out) {
    if (!out || M < 0 || (M > 0 && !xyz) || leaf_size < 1) return LIVO_E_INVALID;
    if (M > kMaxMapPoints) return LIVO_E_RANGE;
    if (stride_bytes == 0) stride_bytes = 3 * sizeof(float);
    if (stride_bytes < (int64_t)(3 * sizeof(float))) return LIVO_E_INVALID;
    free_leaf_map(out);
    int D = 0;
    while (D < kMaxDepth - 1 && ((M + ((int64_t)1 << D) - 1) >> D) > leaf_size) D++;  // ceil(M / 2^D)
    const int64_t n_int = ((int64_t)1 << D) - 1;
    LeafNode* nodes = (LeafNode*)std::calloc((size_t)std::max<int64_t>(n_int, 1), sizeof(LeafNode));
    float* pts = (float*)std::calloc((size_t)(M + 3), 4 * sizeof(float));  // +3: chunk padding
    if (!nodes || !pts) {
        std::free(nodes);
        std::free(pts);
        return LIVO_E_OOM;
    }
    std::vector<BPoint> st((size_t)M);
    const char* base = (const char*)xyz;
    for (int64_t i = 0; i < M; i++) {
        const float* p = (const float*)(base + i * stride_bytes);
        st[i] = BPoint{p[0], p[1], p[2], (uint32_t)i};
    }
    if (M > 0) {
        LeafBuilder b{st, nodes, M, D};
        unsigned hw = std::thread::hardware_concurrency();
        int spawn = 0;
        while ((1u << spawn) < std::min(hw ? hw : 1u, 16u)) spawn++;
        b.build(0, 0, 0, spawn);
    }
    for (int64_t i = 0; i < M; i++) {
        float w;
        std::memcpy(&w, &st[i].idx, 4);
        pts[4 * i + 0] = st[i].x;
        pts[4 * i + 1] = st[i].y;
        pts[4 * i + 2] = st[i].z;
        pts[4 * i + 3] = w;
    }
    out->nodes = nodes;
    out->pts = pts;
    out->num_points = M;
    out->depth = D;
    return LIVO_OK;
}

void free_leaf_map(HostLeafMap* m) {
    if (!m) return;
    std::free(m->nodes);
    std::free(m->pts);
    m->nodes = nullptr;
    m->pts = nullptr;
}

}  // namespace livo

// ---------------------------------------------------------------------------
// Cell grid (livo_internal.h): points sorted by cell (input order kept inside a
// cell), an open-addressing hash of the occupied cells.
// ---------------------------------------------------------------------------
namespace livo {

static inline unsigned long long grid_key(int64_t cx, int64_t cy, int64_t cz) {
    return (unsigned long long)(cx + kGridBias) | ((unsigned long long)(cy + kGridBias) << 21) |
           ((unsigned long long)(cz + kGridBias) << 42);
}
static inline uint64_t grid_hash(unsigned long long key, int log2) {
    return (uint64_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - log2));
}

int build_grid_map(const float* xyz, int64_t M, int64_t stride_bytes, float cell_h, HostGridMap* out, float ppc_target) {
    if (!out || M < 0 || (M > 0 && !xyz)) return LIVO_E_INVALID;
    if (M > kMaxMapPoints) return LIVO_E_RANGE;
    if (stride_bytes == 0) stride_bytes = 3 * sizeof(float);
    if (stride_bytes < (int64_t)(3 * sizeof(float))) return LIVO_E_INVALID;
    free_grid_map(out);
    const char* base = (const char*)xyz;
    auto P = [&](int64_t i) { return (const float*)(base + i * stride_bytes); };
    float mn[3] = {0.f, 0.f, 0.f}, mx[3] = {0.f, 0.f, 0.f};
    if (M > 0) {
        for (int k = 0; k < 3; k++) mn[k] = mx[k] = P(0)[k];
        for (int64_t i = 1; i < M; i++)
            for (int k = 0; k < 3; k++) {
                mn[k] = std::min(mn[k], P(i)[k]);
                mx[k] = std::max(mx[k], P(i)[k]);
            }
    }
    std::vector<unsigned long long> key((size_t)M);
    auto assign = [&](float h) {
        const float inv = 1.0f / h;
        for (int64_t i = 0; i < M; i++) {
            const float* p = P(i);
            int64_t c[3];
            for (int k = 0; k < 3; k++) c[k] = (int64_t)std::floor((p[k] - mn[k]) * inv);
            key[i] = grid_key(c[0], c[1], c[2]);
        }
    };
    auto occupied = [&]() {
        std::vector<unsigned long long> k2(key);
        std::sort(k2.begin(), k2.end());
        return (int64_t)(std::unique(k2.begin(), k2.end()) - k2.begin());
    };
    float h = cell_h;
    if (!(h > 0.f)) {
        // about 8 points per occupied cell, and never more than 2^20 cells per axis
        double ext = 1e-3;
        for (int k = 0; k < 3; k++) ext = std::max(ext, (double)mx[k] - (double)mn[k]);
        h = std::max(0.05f, (float)(ext / (double)(kGridBias - 2)));
        // points per occupied cell grows about as h^2 on surface-like maps:
        // a few multiplicative steps towards 20 (measured on MI355X: 0.35-0.4 m
        // cells, 20-27 points each, searched fastest on the config-2 map)
        // ppc_target < 0: the cell runs' rule (livo_internal.h kVrunPpc): -ppc_target
        // at 1M points, growing as M^0.3 (x2 at 10M: on the config-5 map 20 / 40 / 80
        // points per cell gave 1339 / 4079 / 3960 updates/s, profiles/r03_c5_sweep_*)
        double target = ppc_target > 0.f ? (double)ppc_target : 20.0;
        if (ppc_target < 0.f)
            target = -(double)ppc_target * std::min(4.0, std::max(1.0, std::pow((double)M / 1e6, 0.3)));
        for (int it = 0; it < 6 && M > 0; it++) {
            assign(h);
            const double ppc = (double)M / (double)std::max<int64_t>(occupied(), 1);
            if (ppc >= 0.8 * target && ppc <= 1.3 * target) break;
            const float step = (float)std::min(4.0, std::max(0.5, std::sqrt(target / ppc)));
            const float hn = std::max(h * step, (float)(ext / (double)(kGridBias - 2)));
            if (hn == h) break;
            h = hn;
        }
    } else {
        double ext = 1e-3;
        for (int k = 0; k < 3; k++) ext = std::max(ext, (double)mx[k] - (double)mn[k]);
        if (ext / h >= kGridBias - 2) return LIVO_E_RANGE;
    }
    assign(h);
    std::vector<int64_t> order((size_t)M);
    for (int64_t i = 0; i < M; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return key[a] < key[b]; });
    int64_t cells = 0;
    for (int64_t i = 0; i < M; i++)
        if (i == 0 || key[order[i]] != key[order[i - 1]]) cells++;
    int log2 = 4;
    while (((int64_t)1 << log2) < 4 * cells) log2++;  // load factor <= 1/4: short probes for empty cells
    const int64_t nslots = (int64_t)1 << log2;
    GridSlot* slots = (GridSlot*)std::malloc((size_t)nslots * sizeof(GridSlot));
    float* pts = (float*)std::calloc((size_t)(M + 3), 4 * sizeof(float));
    if (!slots || !pts) {
        std::free(slots);
        std::free(pts);
        return LIVO_E_OOM;
    }
    for (int64_t s = 0; s < nslots; s++) slots[s] = GridSlot{kGridEmpty, 0u, 0u};
    for (int64_t i = 0; i < M;) {
        int64_t j = i;
        while (j < M && key[order[j]] == key[order[i]]) j++;
        uint64_t sl = grid_hash(key[order[i]], log2);
        while (slots[sl].key != kGridEmpty) sl = (sl + 1) & (uint64_t)(nslots - 1);
        slots[sl] = GridSlot{key[order[i]], (uint32_t)i, (uint32_t)(j - i)};
        i = j;
    }
    for (int64_t i = 0; i < M; i++) {
        const float* p = P(order[i]);
        const uint32_t idx = (uint32_t)order[i];
        float w;
        std::memcpy(&w, &idx, 4);
        pts[4 * i + 0] = p[0];
        pts[4 * i + 1] = p[1];
        pts[4 * i + 2] = p[2];
        pts[4 * i + 3] = w;
    }
    out->slots = slots;
    out->pts = pts;
    out->num_points = M;
    out->log2_slots = log2;
    out->cells = cells;
    for (int k = 0; k < 3; k++) out->org[k] = mn[k];
    out->h = h;
    out->cmax = 0.f;
    out->ext = 0.0;
    for (int k = 0; k < 3; k++) out->ext = std::max(out->ext, (double)mx[k] - (double)mn[k]);
    for (int k = 0; k < 3; k++) out->cmax = std::max(out->cmax, std::max(std::fabs(mn[k]), std::fabs(mx[k])));
    return LIVO_OK;
}

// Median distance from a map point to its 5th nearest other map point, over a
// strided sample of the grid's points, searched in the 3x3x3 cells around the
// point (a sample whose 5th neighbour lies farther than one cell is skipped):
// the map's local density scale, which sizes the ball runs (livo_capi.cpp).
float sample_knn_radius(const HostGridMap& gm, int samples) {
    const int64_t M = gm.num_points;
    if (M < 6 || samples <= 0) return 0.f;
    const int64_t nslots = (int64_t)1 << gm.log2_slots;
    const double inv = 1.0 / (double)gm.h;
    std::vector<float> r;
    r.reserve((size_t)samples);
    const int64_t step = std::max<int64_t>(1, M / samples);
    for (int64_t i = 0; i < M && (int64_t)r.size() < samples; i += step) {
        const float* p = gm.pts + 4 * i;
        int64_t c[3];
        for (int k = 0; k < 3; k++) c[k] = (int64_t)std::floor(((double)p[k] - (double)gm.org[k]) * inv);
        float best[6] = {INFINITY, INFINITY, INFINITY, INFINITY, INFINITY, INFINITY};  // incl. the point itself
        for (int dz = -1; dz <= 1; dz++)
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    const unsigned long long key = grid_key(c[0] + dx, c[1] + dy, c[2] + dz);
                    uint64_t sl = grid_hash(key, gm.log2_slots);
                    while (gm.slots[sl].key != key && gm.slots[sl].key != kGridEmpty) sl = (sl + 1) & (uint64_t)(nslots - 1);
                    if (gm.slots[sl].key != key) continue;
                    const float* q = gm.pts + 4 * (int64_t)gm.slots[sl].start;
                    for (uint32_t j = 0; j < gm.slots[sl].count; j++, q += 4) {
                        const float ex = q[0] - p[0], ey = q[1] - p[1], ez = q[2] - p[2];
                        float d = ex * ex + ey * ey + ez * ez;
                        for (int k = 0; k < 6; k++)
                            if (d < best[k]) std::swap(d, best[k]);
                    }
                }
        const float r5 = std::sqrt(best[5]);
        if (r5 <= gm.h) r.push_back(r5);
    }
    if (r.empty()) return 0.f;
    std::nth_element(r.begin(), r.begin() + r.size() / 2, r.end());
    return r[r.size() / 2];
}

void free_grid_map(HostGridMap* m) {
    if (!m) return;
    std::free(m->slots);
    std::free(m->pts);
    m->slots = nullptr;
    m->pts = nullptr;
}


}  // namespace livo
