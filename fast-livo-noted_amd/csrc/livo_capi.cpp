// livo_capi.cpp — the C ABI (include/livo.h): context, device map, resident
// scans, and the host side of the batched IEKF loop.
//
// Host control is launch-only: every evaluation of the IEKF loop
// (laser_mapping.cpp:178) is one k_hshare launch + one k_solve launch on the
// context's stream, and the loop's branches (convergence, rematch, stop) are
// taken on the device (IekfCtrl), so a scan update costs one host->device
// upload of the states and one device->host read of the results, with no
// round trip per iteration.  Evaluations past a scan's stop exit at the first
// instruction.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <chrono>
#include <thread>
#include <vector>

#include "livo_internal.h"

using namespace livo;

namespace {

struct ScanBuf {
    bool used = false;
    int64_t n = 0;
    int32_t nblk = 0;
    float* pts = nullptr;  // n x 4
    NNRec* nn = nullptr;   // neighbour records (Nearest_Points cache)
    int32_t* d_perm = nullptr;  // stored (Morton) position -> caller's point index
    std::vector<int32_t> perm;  // the same on the host, fetched on first use (host_perm)
    int32_t* d_iperm = nullptr; // caller's point index -> stored position
    double* partial = nullptr;  // nblk x kIkCols (the A-path uses kRedCols of each)
    float* plane = nullptr;     // N x 4: planes of the cached neighbours (k_hshare)
    uint8_t* pstate = nullptr;  // N: plane state (0: not fitted since the neighbours changed)
    double* ikrows = nullptr;   // IKFoM few-point rows (nblk x kIkFewRows x 13)
    uint32_t* ikcnt = nullptr;  // per block
    bool searched = false;      // a search has filled the neighbour cache
    int64_t cap = 0;            // points the buffers were sized for (>= n; reused after a release)
    hipEvent_t ready = nullptr; // livo_scan_upload_async: recorded on the upload stream when the scan is built
    bool pending = false;       // an asynchronous upload may still be building it (get_scan waits)
};

template <typename T>
static int dev_alloc(T** p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    if (hipMalloc((void**)p, count * sizeof(T)) != hipSuccess) {
        *p = nullptr;
        return LIVO_E_OOM;
    }
    return LIVO_OK;
}

template <typename T>
static void dev_free(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

static void free_scan_buf(ScanBuf& s) {
    dev_free(s.pts); dev_free(s.nn); dev_free(s.partial); dev_free(s.d_perm); dev_free(s.d_iperm);
    dev_free(s.plane); dev_free(s.pstate); dev_free(s.ikrows); dev_free(s.ikcnt);
    if (s.ready) (void)hipEventDestroy(s.ready);
    s.ready = nullptr;
}

}  // namespace

// The device iVox map and its AddPoints / overflow-pass scratch.
struct IvoxDev {
    bool ready = false;
    int kind = -1;  // search kernel (IvoxParams::kind), LIVO_IVOX_KIND=thread|wave|team read by livo_ivox_init
    int64_t add_passes = 0;  // device passes AddPoints took (one per batch, more at LRU conflicts)
    livo_ivox_params prm{};
    float inv_res = 5.0f;
    int nearby = 19;
    GridSlot* slots = nullptr;
    int32_t log2 = 0;
    int64_t table = 0;
    uint32_t *addcnt = nullptr, *tot = nullptr, *newstart = nullptr, *addstart = nullptr;
    float* pts[2] = {nullptr, nullptr};  // CSR double buffer (4 floats per point)
    int64_t pts_cap[2] = {0, 0};
    int cur = 0;
    int64_t npts = 0, ngrids = 0, next_id = 0, max_grid = 0;
    unsigned long long* ctr = nullptr;   // [0] error bits, [1] new grids, [2] max grid
    // batch temporaries
    float* src = nullptr;
    uint32_t *slot_of = nullptr, *iota = nullptr, *skeys = nullptr, *svals = nullptr;
    int64_t src_cap = 0;
    // overflow pass of the search
    SelElem* big = nullptr;
    int64_t big_threads = 0, big_slice = 0;
    // LRU grid cache: per slot last-use id, per-batch first / last touch, eviction mark
    unsigned long long* tlast = nullptr;
    uint32_t *first = nullptr, *lastp1 = nullptr;
    uint8_t* evict = nullptr;
    // eviction scratch (allocated the first time the capacity is reached)
    unsigned long long *ev_k = nullptr, *ev_k2 = nullptr;
    uint32_t *ev_a = nullptr, *ev_b = nullptr, *ev_c = nullptr, *ev_d = nullptr;
    int64_t ev_cap = 0;
};

// The ikd-Tree incremental map (ikd_incr_kernels.hip): the point set by id
// and the scratch of Add_Points / the grid rebuild.
struct DynDev {
    bool active = false;
    float* all = nullptr;        // per id: x, y, z, id bits
    uint8_t* alive = nullptr;
    int64_t cap = 0, n_ids = 0, n_alive = 0;
    float cmax = 0.f;            // largest |coordinate| (the grid's rounding slack)
    unsigned long long *keys = nullptr, *skeys = nullptr;
    uint32_t *iota = nullptr, *svals = nullptr, *heads = nullptr, *runid = nullptr, *starts = nullptr;
    int64_t sort_cap = 0;
    float *W = nullptr, *seq = nullptr, *Ws = nullptr;
    uint32_t *defer = nullptr, *dpos = nullptr, *dlist = nullptr, *keep = nullptr, *apos = nullptr;
    int64_t add_cap = 0;
    float* boxes = nullptr;
    int64_t box_cap = 0;
    unsigned long long *dirty = nullptr, *ctr = nullptr;
    int64_t gslot_cap = 0, gpts_cap = 0;  // capacities of ctx->gslots / ctx->gpts
    livo_map_add_stats last{};
    // The IEKF search keeps the cell and ball runs on the incremental map
    // (LIVO_IDX_RUNS): the runs index the base point set rpts (the map's points
    // in grid order when the runs were built; ids below base_ids), a deleted
    // base point is marked in rpts (x = NaN, never a candidate of the run scans), and
    // the points added since are searched in the delta grid (dslots / dpts, the
    // cell grid's layout).  When the delta or the deleted share grows past
    // rebase_frac of the base the runs are rebuilt from the current points.
    bool runs = false;
    float* rpts = nullptr;           // base points: x, y, z, id bits (x = NaN once deleted)
    uint32_t* rpos = nullptr;        // base id -> position in rpts (~0: not in the base / marked)
    int64_t base_ids = 0, base_n = 0, rpts_cap = 0, rpos_cap = 0;
    int64_t tomb = 0;                // base points marked deleted
    GridSlot* dslots = nullptr;
    float* dpts = nullptr;
    int32_t dlog2 = 4;
    GridSlot* dvslots = nullptr;     // the delta grid's cell runs (positions in dpts)
    RunWord* dvidx = nullptr;
    int32_t dvlog2 = 4;
    int64_t d_n = 0, dslot_cap = 0, dpts_cap = 0;
    int64_t rebases = 0;
    double rebase_frac = 0.125;      // LIVO_DYN_REBASE
    float min_gh = 0.f;              // the cell-walk grid's edge range: [box_cell, box_cell_max] x the Add_Points box
    float max_gh = 0.f;
    float box_cell = 1.2f;           // LIVO_DYN_BOX_CELL
    float box_cell_max = 2.0f;       // LIVO_DYN_BOX_CELL_MAX (0: no upper bound)
    // The grid rebuild merges instead of re-sorting (dyn_rebuild_merge): the
    // grid holds every alive id below grid_ids in (key, id) order on cells of
    // edge grid_gh (-1: unknown, the next rebuild sorts), `cells` of them.
    float* gpts_alt = nullptr;       // the merge's output, swapped with ctx->gpts
    int64_t gpts_alt_cap = 0;
    int64_t grid_ids = -1, cells = -1;
    float grid_gh = 0.f;
    bool merge = true;               // LIVO_DYN_MERGE=0: always sort
    int64_t rebuilds_sorted = 0, rebuilds_merged = 0;
    int64_t wide_redos = 0;          // Add_Points batches redone with 64-bit box keys
    int64_t rebuilds_fused = 0;      // merged rebuilds run in Add_Points' pass (one read-back)
    ScanCtx scan;                    // the one-launch scans' ticket and status words
};

// One batch's staging and streams.  LaserMapping batches: slots packed at
// kLmStride (the part before the IKFoM block) followed by the jobs, one
// contiguous staging area each way.  Lane 0 borrows the context's streams;
// the other lanes own theirs (created on first use).
struct BatchLane {
    char* h_lm = nullptr;
    char* d_lm = nullptr;
    char* h_lm_dev = nullptr;  // h_lm's device address (host-mapped), for the kernel copies
    size_t lm_cap = 0;
    // IKFoM batches: whole slots (their IKFoM block included) then the jobs,
    // host pinned and device, per lane so two IKFoM batches can be in flight
    char* h_ik = nullptr;
    char* d_ik = nullptr;
    char* h_ik_dev = nullptr;  // h_ik's device address (host-mapped), for the kernel copies
    size_t ik_cap = 0;
    hipStream_t st[kMaxGroups] = {};
    hipEvent_t fork = nullptr;
    hipEvent_t done[kMaxGroups] = {};  // each group's last operation (its slot copy back)
    bool owned = false;       // streams created for this lane
    bool owned_fork = false;  // fork event created for this lane
    bool busy = false;   // submitted, not yet collected
    int32_t ticket = -1;
    int32_t n = 0;
    int model = 0;
    int ngroups = 0;
    int32_t gfirst[kMaxGroups] = {}, gcount[kMaxGroups] = {};
    std::vector<int32_t> ids;
};

// pinned staging buffers of livo_scan_upload_async (two batches of 8 ahead)
constexpr int kPinRing = 16;

struct livo_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // extra streams for the groups of a batch (overlap of latency-bound kernels)
    hipStream_t xstream[kMaxGroups - 1] = {};
    hipEvent_t xjoin[kMaxGroups - 1] = {};
    // stream groups per batch (LIVO_STREAM_GROUPS; 0: the default of
    // batch_enqueue, four for the fused and IKFoM paths, two for iVox,
    // profiles/r04_ab_groups.txt)
    int groups = 0;
    int leaf_size = kLeafSize;         // leaf-map points per leaf (LIVO_LEAF_SIZE)
    hipEvent_t fork = nullptr;
    livo_params params{};
    // map
    MapNode* nodes = nullptr;
    int64_t map_points = 0;
    int64_t map_slots = 0;
    int32_t map_depth = 0;
    LeafNode* lnodes = nullptr;        // leaf map (batched IEKF search)
    float* lpts = nullptr;
    int32_t leaf_depth = 0;
    int64_t leaf_bytes = 0;
    int knn_kind = 2;                  // batched search: 0 leaf map, 1 cell grid, 2 cell grid + LDS tiles (LIVO_KNN_KIND)
    bool fused = true;                 // kind 2: one k_iekf_eval launch per evaluation (LIVO_FUSED=0: separate passes)
    float grid_cell = 0.f;             // cell edge (LIVO_GRID_CELL; 0: from the map)
    float grid_ppc = 0.f;              // target points per occupied cell when chosen from the map (LIVO_GRID_PPC)
    bool vruns = true;                 // cell runs on a static map (LIVO_VRUNS=0: the cell walk)
    // k_iekf_eval block order (LIVO_XCD_CHUNK): XCD-interleaved chunks of 8 blocks, so
    // every XCD holds a share of every scan (distinct-scan pool: 18.6k vs 17.6k /
    // 18.3k vs 17.1k / 17.1k vs 16.4k updates/s against 0, one range per XCD, whose
    // most expensive scan's XCD was the straggler; profiles/r04_ab_block_order.txt)
    int xcd_chunk = 8;
    GridSlot* vslots = nullptr;        // vertex runs (static map only)
    RunWord* vpts = nullptr;           // run entries (LIVO_IDX_RUNS: grid positions; else x, y, z, map index bits)
    int32_t vlog2 = 0;
    // ball runs (static map only): anchor cells of edge bh, runs of radius brmax
    bool bruns = true;                 // LIVO_BRUNS=0: the cell runs only
    // bh = br_ha r5, brmax = sqrt(3)/2 bh + br_r r5 (LIVO_BR_HA / LIVO_BR_R).  R = 6
    // (round 4; 3.2 before): on distinct scans the queries a ball of 3.2 r5 left
    // uncertified (off the surfaces by the prior's pose error) certify in their
    // ball run instead of the cell run and walk: pooled 21.4k vs 18.5k updates/s,
    // first evaluation 0.157 vs 0.231 ms; R = 8 / 10 / 13 no better
    // (profiles/r04_ab_ball_radius.txt)
    float br_ha = 2.0f, br_r = 6.0f;
    GridSlot* bslots = nullptr;
    RunWord* bpts = nullptr;
    int32_t blog2 = 0;
    float bh = 0.f, brmax = 0.f, br5 = 0.f;
    int64_t bentries = 0;
    int32_t bchunks = 0;               // anchor chunks of the ball runs' build
    GridSlot* gslots = nullptr;        // cell grid
    float* gpts = nullptr;
    float gorg[3] = {0.f, 0.f, 0.f};
    float gh = 1.f, geps = 0.f, gcmax = 0.f;
    DynDev dyn;                        // the incremental map (livo_map_add_points, ...)
    int32_t glog2 = 0;
    int64_t grid_bytes = 0;
    bool has_map = false;
    int backend = LIVO_BACKEND_IKDTREE;  // search structure of h_share / the IEKF loop
    IvoxDev iv;                        // iVox map (LIVO_BACKEND_IVOX)
    void* fe_buf = nullptr;            // scan front-end scratch (livo_scan_preprocess)
    size_t fe_bytes = 0;
    const float* fe_raw = nullptr;     // the last preprocessed frame, de-skewed, full resolution (5 floats a point)
    int64_t fe_n = 0;
    void* vio_buf = nullptr;           // VIO frame (image, points, partials, slot)
    size_t vio_bytes = 0;
    void* prim_tmp = nullptr;          // rocPRIM scratch (sorts, scans)
    size_t prim_bytes = 0;
    // scans
    std::vector<ScanBuf> scans;
    // released scans' device buffers, reused by the next upload of a scan that
    // fits (a drop-in run uploads and releases one scan per frame: hipMalloc /
    // hipFree of its buffers cost more than the update itself)
    std::vector<ScanBuf> spare;
    // upload scratch: Morton keys, sort buffers, bounds and the packed source points
    void* up_tmp = nullptr;
    size_t up_tmp_bytes = 0;
    // livo_scan_upload_async: its own stream, scratch and rocPRIM scratch, and a
    // ring of pinned staging buffers (each reused once the copy out of it is done)
    hipStream_t up_stream = nullptr;
    void* aup_tmp = nullptr;
    size_t aup_tmp_bytes = 0;
    void* aup_prim = nullptr;
    size_t aup_prim_bytes = 0;
    struct PinSlot {
        float* h = nullptr;
        size_t bytes = 0;
        hipEvent_t copied = nullptr;
        bool inflight = false;
    } pin[kPinRing];
    int pin_next = 0;
    // livo_scan_upload_batch_async: the copies on a stream of their own into two
    // alternating device staging buffers, so batch k+1's copy runs beside batch
    // k's build on up_stream (bsrc_copied gates the build, bsrc_free the next
    // copy into the same buffer)
    hipStream_t cp_stream = nullptr;
    void* bsrc[2] = {nullptr, nullptr};
    size_t bsrc_bytes[2] = {0, 0};
    hipEvent_t bsrc_copied[2] = {nullptr, nullptr};
    hipEvent_t bsrc_free[2] = {nullptr, nullptr};
    bool bsrc_used[2] = {false, false};
    int bsrc_next = 0;
    // batch resources
    int32_t slot_cap = 0;
    IekfSlot* d_slots = nullptr;
    // batches in flight (livo_iekf_update_batch_submit): lane 0 also carries
    // every synchronous batch
    BatchLane lane[LIVO_MAX_INFLIGHT];
    int32_t lane_gen = 0;  // tickets: generation * LIVO_MAX_INFLIGHT + lane
    bool lane_own_streams = false;  // LIVO_LANE_STREAMS=own: lanes > 0 on streams of their own
    // LIVO_LANE_SERIAL=1: a queued batch starts only once every group of the one
    // before it is done; default 0: its group 0 starts when stream 0 frees, beside
    // the other groups' tails (20.5k vs 19.1k updates/s, profiles/r03_ab_lanes.txt)
    bool lane_serial = false;
    bool lane_zc = true;            // submitted batches: staging copies by kernel over host-mapped memory (LIVO_LANE_ZC)
    bool sync_zc = false;           // synchronous batches too (LIVO_SYNC_ZC)
    bool slot_wb = true;            // fused batches: the stopping solve writes the slot back (LIVO_SLOT_WB)
    int last_lane = -1;             // lane of the batch enqueued last
    unsigned long long last_replays = 0;  // profiled batches: the replay counter read back
    IekfSlot* h_slots = nullptr;  // pinned
    HsJob* d_jobs = nullptr;
    HsJob* h_jobs = nullptr;      // pinned
    // exact-replay list of the k-NN passes
    unsigned* d_replay_count = nullptr;
    unsigned long long* d_replay_total = nullptr;
    unsigned long long* d_replay_list = nullptr;
    int64_t replay_cap = 0;
    // iVox: the wave pass's overflow for the global-memory pass (KnnParams::replay_list2);
    // per group of lane 0 (the iVox batches are synchronous)
    unsigned* d_replay_count2 = nullptr;
    unsigned long long* d_replay_list2 = nullptr;
    // scratch for livo_knn / debug outputs
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    // profiling
    int profiling = 0;
    hipEvent_t ev[kMaxGroups][3 * LIVO_MAX_EVALS + 2] = {};
    hipEvent_t b_start = nullptr, b_end[2] = {};  // profiling level 2: batch span and the gap before it
    int b_par = 0;
    bool b_prev = false;
    bool events_ready = false;
    livo_timings last{};
};

#define HIP_TRY(x)                                  \
    do {                                            \
        if ((x) != hipSuccess) return LIVO_E_HIP;   \
    } while (0)

// Host wait for a stream: spin on hipStreamQuery (microseconds to notice
// completion), then fall back to the blocking wait after ~50 ms.
static hipError_t stream_wait(hipStream_t st) {
    for (int k = 0; k < 200000; k++) {
        const hipError_t e = hipStreamQuery(st);
        if (e != hipErrorNotReady) return e;
    }
    return hipStreamSynchronize(st);
}

// The same for an event (a batch's end when other work may queue behind it).
static hipError_t event_wait(hipEvent_t ev) {
    for (int k = 0; k < 200000; k++) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
    }
    return hipEventSynchronize(ev);
}

static int set_device(livo_ctx* c) {
    return hipSetDevice(c->device) == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

static int ensure_scratch(livo_ctx* c, size_t bytes) {
    if (bytes <= c->scratch_bytes) return LIVO_OK;
    if (c->scratch) (void)hipFree(c->scratch);
    c->scratch = nullptr;
    c->scratch_bytes = 0;
    if (hipMalloc(&c->scratch, bytes) != hipSuccess) return LIVO_E_OOM;
    c->scratch_bytes = bytes;
    return LIVO_OK;
}

static int ensure_slots(livo_ctx* c, int32_t n) {
    if (n <= c->slot_cap) return LIVO_OK;
    int32_t cap = std::max(n, 8);
    dev_free(c->d_slots);
    dev_free(c->d_jobs);
    if (c->h_slots) (void)hipHostFree(c->h_slots);
    if (c->h_jobs) (void)hipHostFree(c->h_jobs);
    c->h_slots = nullptr;
    c->h_jobs = nullptr;
    c->slot_cap = 0;
    if (dev_alloc(&c->d_slots, cap) || dev_alloc(&c->d_jobs, cap)) return LIVO_E_OOM;
    if (hipHostMalloc((void**)&c->h_slots, sizeof(IekfSlot) * cap, hipHostMallocDefault) != hipSuccess) return LIVO_E_OOM;
    if (hipHostMalloc((void**)&c->h_jobs, sizeof(HsJob) * cap, hipHostMallocDefault) != hipSuccess) return LIVO_E_OOM;
    c->slot_cap = cap;
    return LIVO_OK;
}

// kLmStride-packed LaserMapping slots + jobs of a batch of n (host pinned and device).
constexpr size_t kLmStride = (kSlotLmBytes + 255) & ~(size_t)255;
static_assert(kLmStride % alignof(HsJob) == 0 && kLmStride % alignof(IekfSlot) == 0, "packed slot alignment");
static_assert(kLmStride % 16 == 0, "kernel staging copies move 16-B words");
// bytes of a batch's packed staging area, rounded up to whole 16-B words
static size_t lm_bytes(int32_t n) { return ((size_t)n * (kLmStride + sizeof(HsJob)) + 15) & ~(size_t)15; }
static int ensure_lm(BatchLane& B, int32_t n) {
    const size_t need = lm_bytes(n);
    if (need <= B.lm_cap) return LIVO_OK;
    const size_t cap = std::max(need, lm_bytes(8));
    dev_free(B.d_lm);
    if (B.h_lm) (void)hipHostFree(B.h_lm);
    B.h_lm = nullptr;
    B.lm_cap = 0;
    if (hipMalloc((void**)&B.d_lm, cap) != hipSuccess) {
        B.d_lm = nullptr;
        return LIVO_E_OOM;
    }
    // mapped + coherent: the lane's kernel copies (launch_copy_words) read and write it
    if (hipHostMalloc((void**)&B.h_lm, cap, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        B.h_lm = nullptr;
        return LIVO_E_OOM;
    }
    B.h_lm_dev = nullptr;
    if (hipHostGetDevicePointer((void**)&B.h_lm_dev, B.h_lm, 0) != hipSuccess) {
        (void)hipGetLastError();
        B.h_lm_dev = nullptr;  // DMA copies then
    }
    B.lm_cap = cap;
    return LIVO_OK;
}

static int ensure_ik(BatchLane& B, int32_t n) {
    const size_t need = (size_t)n * (sizeof(IekfSlot) + sizeof(HsJob));
    if (need <= B.ik_cap) return LIVO_OK;
    const size_t cap = std::max(need, (size_t)8 * (sizeof(IekfSlot) + sizeof(HsJob)));
    dev_free(B.d_ik);
    if (B.h_ik) (void)hipHostFree(B.h_ik);
    B.h_ik = nullptr;
    B.ik_cap = 0;
    if (hipMalloc((void**)&B.d_ik, cap) != hipSuccess) {
        B.d_ik = nullptr;
        return LIVO_E_OOM;
    }
    // mapped + coherent: a submitted batch's staging copies are kernels (as the
    // LaserMapping lanes'); DMA copies behind another lane's kernels held the
    // submitting host 2-3 ms per batch
    if (hipHostMalloc((void**)&B.h_ik, cap, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        B.h_ik = nullptr;
        return LIVO_E_OOM;
    }
    B.h_ik_dev = nullptr;
    if (hipHostGetDevicePointer((void**)&B.h_ik_dev, B.h_ik, 0) != hipSuccess) {
        (void)hipGetLastError();
        B.h_ik_dev = nullptr;  // DMA copies then
    }
    B.ik_cap = cap;
    return LIVO_OK;
}

// A lane's group streams: lane 0 the context's, the others their own.
static int lane_streams(livo_ctx* c, int L) {
    BatchLane& B = c->lane[L];
    if (B.st[0]) return LIVO_OK;
    for (int k = 0; k < kMaxGroups; k++)
        if (!B.done[k] && hipEventCreateWithFlags(&B.done[k], hipEventDisableTiming) != hipSuccess) return LIVO_E_HIP;
    if (L == 0) {
        B.st[0] = c->stream;
        for (int k = 0; k < kMaxGroups - 1; k++) B.st[k + 1] = c->xstream[k];
        B.fork = c->fork;
        return LIVO_OK;
    }
    // By default every lane queues on the context's streams: a batch submitted
    // behind another starts the moment the device finishes the first (no host
    // round trip, copy or launch latency in between), without running beside
    // it (MI355X, 8 x 100k: two batches on their own streams, so concurrent,
    // 10-13k updates/s against 16.9k for one at a time, profiles/r03_ab_lanes.txt).
    // LIVO_LANE_STREAMS=own gives each lane its own streams.
    if (!c->lane_own_streams) {
        for (int k = 0; k < kMaxGroups; k++) B.st[k] = c->lane[0].st[k] ? c->lane[0].st[k] : (k ? c->xstream[k - 1] : c->stream);
    } else {
        B.owned = true;
        for (int k = 0; k < kMaxGroups; k++)
            if (hipStreamCreateWithFlags(&B.st[k], hipStreamNonBlocking) != hipSuccess) return LIVO_E_HIP;
    }
    if (hipEventCreateWithFlags(&B.fork, hipEventDisableTiming) != hipSuccess) return LIVO_E_HIP;
    B.owned_fork = true;
    return LIVO_OK;
}

static bool any_inflight(const livo_ctx* c) {
    for (const BatchLane& B : c->lane)
        if (B.busy) return true;
    return false;
}

static bool params_valid(const livo_params* p) {
    return p && p->laser_point_cov > 0.0 && p->max_iterations >= 0 && p->max_iterations + 1 <= LIVO_MAX_EVALS &&
           p->flags == 0;
}

// Replay counters and lists per lane (LIVO_MAX_INFLIGHT slices: lane L's
// counters at L * kMaxGroups, its list at L * replay_cap), so two unfused
// batches in flight (IKFoM) keep theirs apart.
static int ensure_replay(livo_ctx* c, int64_t total) {
    if (!c->d_replay_count && dev_alloc(&c->d_replay_count, (size_t)kMaxGroups * LIVO_MAX_INFLIGHT)) return LIVO_E_OOM;
    if (!c->d_replay_total) {
        if (dev_alloc(&c->d_replay_total, 1)) return LIVO_E_OOM;
        HIP_TRY(hipMemset(c->d_replay_total, 0, sizeof(unsigned long long)));
    }
    if (!c->d_replay_count2) {
        if (dev_alloc(&c->d_replay_count2, (size_t)kMaxGroups)) return LIVO_E_OOM;
        HIP_TRY(hipMemset(c->d_replay_count2, 0, sizeof(unsigned) * kMaxGroups));
    }
    if (total <= c->replay_cap) return LIVO_OK;
    dev_free(c->d_replay_list);  // (hipFree waits for the device: no batch is still using it)
    dev_free(c->d_replay_list2);
    c->replay_cap = 0;
    if (dev_alloc(&c->d_replay_list, (size_t)total * LIVO_MAX_INFLIGHT)) return LIVO_E_OOM;
    if (dev_alloc(&c->d_replay_list2, (size_t)total)) return LIVO_E_OOM;
    c->replay_cap = total;
    return LIVO_OK;
}

static IvoxParams ivox_params(livo_ctx* c);

static KnnParams make_knn_params(livo_ctx* c) {
    KnnParams kp{};
    kp.nodes = c->nodes;
    kp.jobs = c->d_jobs;
    kp.replay_count = c->d_replay_count;
    kp.replay_list = c->d_replay_list;
    kp.replay_count2 = c->d_replay_count2;
    kp.replay_list2 = c->d_replay_list2;
    kp.replay_total = c->d_replay_total;
    std::memcpy(kp.R_LI, c->params.R_LI, sizeof(kp.R_LI));
    std::memcpy(kp.t_LI, c->params.t_LI, sizeof(kp.t_LI));
    kp.has_map = c->has_map && c->map_points > 0 ? 1 : 0;
    kp.force = -1;
    kp.depth = c->map_depth;
    kp.n_nodes = c->has_map ? c->map_slots : 0;
    kp.lnodes = c->lnodes;
    kp.lpts = c->lpts;
    kp.ldepth = c->leaf_depth;
    kp.lM = c->has_map ? c->map_points : 0;
    kp.gslots = c->gslots;
    kp.gpts = c->gpts;
    std::memcpy(kp.gorg, c->gorg, sizeof(kp.gorg));
    kp.gh = c->gh;
    kp.geps = c->geps;
    kp.glog2 = c->glog2;
    // the incremental map keeps the runs of its base point set (+ deletion marks
    // and the delta grid, dyn_runs_update) or, without them, the cell walk
    const bool dyn_runs = c->dyn.active && c->dyn.runs;
    const bool vr = c->vslots && (!c->dyn.active || dyn_runs);
    kp.rpts = dyn_runs ? c->dyn.rpts : c->gpts;
    kp.dslots = dyn_runs && c->dyn.d_n > 0 ? c->dyn.dslots : nullptr;
    kp.dpts = dyn_runs ? c->dyn.dpts : nullptr;
    kp.dlog2 = c->dyn.dlog2;
    kp.dvslots = dyn_runs && c->dyn.d_n > 0 ? c->dyn.dvslots : nullptr;
    kp.dvidx = c->dyn.dvidx;
    kp.dvlog2 = c->dyn.dvlog2;
    kp.dyn_runs = dyn_runs ? 1 : 0;
    kp.vslots = vr ? c->vslots : nullptr;
    kp.vpts = vr ? c->vpts : nullptr;
    kp.vlog2 = c->vlog2;
    const bool br = vr && c->bslots;
    kp.bslots = br ? c->bslots : nullptr;
    kp.bpts = br ? c->bpts : nullptr;
    kp.blog2 = c->blog2;
    kp.bh = c->bh;
    // certification: every point within the final bound lies in the ball (the build
    // keeps points with cr_rho2 <= brmax^2 in float: a relative 1e-5 below covers its rounding)
    kp.bcert2 = c->brmax * c->brmax * (1.0f - 1e-5f);
    kp.xcd_chunk = c->xcd_chunk;
    kp.identity = 0;
    kp.iv = ivox_params(c);
    kp.canon = c->dyn.active ? 1 : 0;
    return kp;
}

// k-NN pass + exact replay of its flagged queries (one replay list per pass).
static int knn_pass(const KnnParams& kp, int n_jobs, int64_t max_n, hipStream_t st) {
    HIP_TRY(hipMemsetAsync(kp.replay_count, 0, sizeof(unsigned), st));
    // the incremental map has no reference-order tree: the grid search + canonical replay
    if (kp.canon) return launch_knn_grid(kp, n_jobs, max_n, false, false, st);
    return launch_knn_pass(kp, n_jobs, max_n, st);
}

static float morton_scale() {
    static const float scale = [] {  // cells per metre (LIVO_MORTON_SCALE tuning knob)
        const char* e = std::getenv("LIVO_MORTON_SCALE");
        const float v = e ? (float)std::atof(e) : 4.0f;
        return v > 0.0f ? v : 4.0f;
    }();
    return scale;
}

static HsParams make_hs_params(livo_ctx* c) {
    HsParams hp{};
    hp.jobs = c->d_jobs;
    std::memcpy(hp.R_LI, c->params.R_LI, sizeof(hp.R_LI));
    std::memcpy(hp.t_LI, c->params.t_LI, sizeof(hp.t_LI));
    hp.inv_r = 1.0 / c->params.laser_point_cov;
    hp.lpc = c->params.laser_point_cov;
    hp.max_res = c->params.max_residual;
    hp.plane_thr = c->params.plane_threshold;
    // the iVox branch has no sqdist gate (laser_mapping.cpp:519-525)
    hp.max_sqd = c->backend == LIVO_BACKEND_IVOX ? INFINITY : c->params.max_nn_sqdist;
    hp.force = -1;
    return hp;
}

// doubles of a scan's block-partial buffer: the plane pass (kIkCols per
// kBlock * kPtsPerThread points) or the fused evaluation (kRedCols per kEvalBlock)
static size_t partial_doubles(int64_t N) {
    const int64_t a = std::max<int64_t>(1, (N + kBlock * kPtsPerThread - 1) / (kBlock * kPtsPerThread)) * kIkCols;
    const int64_t b = std::max<int64_t>(1, (N + kEvalBlock - 1) / kEvalBlock) * kRedCols;
    return (size_t)std::max(a, b);
}

static void fill_job(HsJob& j, ScanBuf& s, IekfSlot* slot) {
    j.pts = s.pts;
    j.nn = s.nn;
    j.partial = s.partial;
    j.plane = s.plane;
    j.pstate = s.pstate;
    j.ikrows = s.ikrows;
    j.ikcnt = s.ikcnt;
    j.host_slot = nullptr;
    j.slot = slot;
    j.n = (int32_t)s.n;
    j.nblk = s.nblk;
}

// IKFoM: x_ = x_propagated = the input state (its cov is P_propagated); the
// first h_dyn_share searches (dyn_share.converge = true, esekfom.hpp:1623).
static void init_slot_ik(IekfSlot& s, const livo_ikfom_state& st, int max_iter) {
    std::memset(&s, 0, sizeof(IekfSlot));
    s.model = kModelIkfom;
    s.ik.x = st;
    s.ik.xp = st;
    s.ctrl.search_en = 1;
    s.ctrl.iter_count = -1;
    s.ctrl.max_iter = max_iter;
}

// The covariance factors of the device solve (IekfSlot::covL / covB): the
// state covariance is fixed for the whole IEKF loop of a scan (it changes only
// when the loop stops, laser_mapping.cpp:224-227), so the 6x6 Cholesky of its
// pose block S = P(0:6, 0:6) = L L^T and B = P(:, 0:6) L^-T are formed once, on
// the host, when the slot is staged.  cov_ok = 0 (the device then takes its
// pivoted 6x6 LU path) unless P's first six rows and columns are symmetric and
// S is numerically positive definite.
static void cov_factor(IekfSlot& s) {
    const double* P = s.state.cov;
    constexpr int D = kDim;
    s.cov_ok = 0;
    double amax = 0.0;
    for (int i = 0; i < D; i++)
        for (int j = 0; j < 6; j++) {
            const double a = P[i * D + j], b = P[j * D + i];
            if (!std::isfinite(a) || !std::isfinite(b)) return;
            amax = std::max(amax, std::fabs(a));
        }
    for (int i = 0; i < D; i++)
        for (int j = 0; j < 6; j++)
            if (std::fabs(P[i * D + j] - P[j * D + i]) > 1e-12 * amax) return;
    double Lm[36] = {};
    for (int j = 0; j < 6; j++) {
        double d = P[j * D + j];
        for (int k = 0; k < j; k++) d -= Lm[j * 6 + k] * Lm[j * 6 + k];
        if (!(d > 1e-13 * P[j * D + j]) || !(d > 0.0)) return;  // not (numerically) positive definite
        const double l = std::sqrt(d);
        Lm[j * 6 + j] = l;
        for (int i = j + 1; i < 6; i++) {
            double v = P[i * D + j];
            for (int k = 0; k < j; k++) v -= Lm[i * 6 + k] * Lm[j * 6 + k];
            Lm[i * 6 + j] = v / l;
        }
    }
    double Bm[(D - 6) * 6];
    for (int r = 6; r < D; r++)  // B(r, :) L^T = P(r, 0:6): forward substitution
        for (int j = 0; j < 6; j++) {
            double v = P[r * D + j];
            for (int k = 0; k < j; k++) v -= Bm[(r - 6) * 6 + k] * Lm[j * 6 + k];
            Bm[(r - 6) * 6 + j] = v / Lm[j * 6 + j];
        }
    for (double v : Bm)
        if (!std::isfinite(v)) return;
    std::memcpy(s.covL, Lm, sizeof(Lm));
    std::memcpy(s.covB, Bm, sizeof(Bm));
    s.cov_ok = 1;
}

// bytes: how much of the slot to clear; the batched LaserMapping update uploads
// and reads only its first kSlotLmBytes, so it clears only those
static void init_slot(IekfSlot& s, const livo_state& st, const livo_state& prior, int max_iter,
                      size_t bytes = sizeof(IekfSlot)) {
    std::memset(&s, 0, bytes);
    s.state = st;
    s.prior = prior;
    s.ctrl.stop = 0;
    s.ctrl.search_en = 1;
    s.ctrl.iter_count = -1;
    s.ctrl.rematch_num = 0;
    s.ctrl.max_iter = max_iter;
    cov_factor(s);
}

static int create_group_streams(livo_ctx* c) {
    for (int k = 0; k < kMaxGroups - 1; k++) {
        if (hipStreamCreateWithFlags(&c->xstream[k], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&c->xjoin[k], hipEventDisableTiming) != hipSuccess)
            return 1;
    }
    return 0;
}


// ------------------------------------------------------------------ iVox --
static void ivox_free(IvoxDev& v) {
    dev_free(v.slots);
    dev_free(v.addcnt); dev_free(v.tot); dev_free(v.newstart); dev_free(v.addstart);
    dev_free(v.pts[0]); dev_free(v.pts[1]);
    dev_free(v.ctr);
    dev_free(v.src); dev_free(v.slot_of); dev_free(v.iota); dev_free(v.skeys); dev_free(v.svals);
    dev_free(v.big);
    dev_free(v.tlast); dev_free(v.first); dev_free(v.lastp1); dev_free(v.evict);
    dev_free(v.ev_k); dev_free(v.ev_k2);
    dev_free(v.ev_a); dev_free(v.ev_b); dev_free(v.ev_c); dev_free(v.ev_d);
    v = IvoxDev{};
}

// Rehash into a table of 2^log2 slots (and per-slot arrays to match).
static int ivox_rehash_to(livo_ctx* c, int log2) {
    IvoxDev& v = c->iv;
    if (log2 > 31) return LIVO_E_RANGE;
    const int64_t table = (int64_t)1 << log2;
    GridSlot* slots = nullptr;
    unsigned long long* tlast = nullptr;
    if (dev_alloc(&slots, (size_t)table) || dev_alloc(&tlast, (size_t)table)) {
        dev_free(slots);
        return LIVO_E_OOM;
    }
    int rc = launch_ivox_clear(slots, table, c->stream);
    if (!rc && v.slots) rc = launch_ivox_rehash(v.slots, v.tlast, v.table, slots, tlast, log2, c->stream);
    if (rc) {
        dev_free(slots);
        dev_free(tlast);
        return rc;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    dev_free(v.slots);
    dev_free(v.tlast);
    dev_free(v.addcnt); dev_free(v.tot); dev_free(v.newstart); dev_free(v.addstart);
    dev_free(v.first); dev_free(v.lastp1); dev_free(v.evict);
    v.slots = slots;
    v.tlast = tlast;
    v.table = table;
    v.log2 = log2;
    if (dev_alloc(&v.addcnt, table) || dev_alloc(&v.tot, table) || dev_alloc(&v.newstart, table) ||
        dev_alloc(&v.addstart, table) || dev_alloc(&v.first, table) || dev_alloc(&v.lastp1, table) ||
        dev_alloc(&v.evict, table))
        return LIVO_E_OOM;
    HIP_TRY(hipMemsetAsync(v.addcnt, 0, (size_t)table * sizeof(uint32_t), c->stream));
    HIP_TRY(hipMemsetAsync(v.first, 0xFF, (size_t)table * sizeof(uint32_t), c->stream));
    HIP_TRY(hipMemsetAsync(v.lastp1, 0, (size_t)table * sizeof(uint32_t), c->stream));
    HIP_TRY(hipMemsetAsync(v.evict, 0, (size_t)table, c->stream));
    return LIVO_OK;
}

static int table_log2_for(int64_t grids) {
    int log2 = 10;
    while (((int64_t)1 << log2) < 4 * grids) log2++;
    return log2;
}

// Hash table with room for `grids` grids at load factor <= 1/2 (rehash on growth).
static int ivox_ensure_table(livo_ctx* c, int64_t grids) {
    IvoxDev& v = c->iv;
    if (v.table >= 2 * grids && v.table > 0) return LIVO_OK;
    return ivox_rehash_to(c, table_log2_for(grids));
}

// After an insert sized for its worst case (every point a new grid): shrink a
// table left below 1/16 full, so the per-slot passes of later inserts stay short.
static int ivox_trim_table(livo_ctx* c) {
    IvoxDev& v = c->iv;
    const int log2 = table_log2_for(std::max<int64_t>(v.ngrids, 256));
    return log2 + 2 <= v.log2 ? ivox_rehash_to(c, log2) : LIVO_OK;
}

static int ivox_ensure_src(livo_ctx* c, int64_t n) {
    IvoxDev& v = c->iv;
    if (n <= v.src_cap) return LIVO_OK;
    const int64_t cap = std::max<int64_t>(n, 4096);
    dev_free(v.src); dev_free(v.slot_of); dev_free(v.iota); dev_free(v.skeys); dev_free(v.svals);
    v.src_cap = 0;
    if (dev_alloc(&v.src, (size_t)cap * 4) || dev_alloc(&v.slot_of, cap) || dev_alloc(&v.iota, cap) ||
        dev_alloc(&v.skeys, cap) || dev_alloc(&v.svals, cap))
        return LIVO_E_OOM;
    v.src_cap = cap;
    return LIVO_OK;
}

static int ensure_prim(livo_ctx* c, size_t bytes) {
    if (bytes <= c->prim_bytes) return LIVO_OK;
    if (c->prim_tmp) (void)hipFree(c->prim_tmp);
    c->prim_tmp = nullptr;
    c->prim_bytes = 0;
    if (hipMalloc(&c->prim_tmp, bytes) != hipSuccess) return LIVO_E_OOM;
    c->prim_bytes = bytes;
    return LIVO_OK;
}

// Exclusive scan of n u32 through rocPRIM (out != in).
static int ivox_scan(livo_ctx* c, const uint32_t* in, uint32_t* out, int64_t n) {
    size_t tb = 0;
    int rc = prim_exclusive_scan_u32(nullptr, &tb, in, out, n, c->stream);
    if (!rc) rc = ensure_prim(c, tb);
    tb = c->prim_bytes;
    if (!rc) rc = prim_exclusive_scan_u32(c->prim_tmp, &tb, in, out, n, c->stream);
    return rc;
}

static IvoxParams ivox_params(livo_ctx* c) {
    IvoxDev& v = c->iv;
    IvoxParams P{};
    P.slots = v.slots;
    P.pts = v.pts[v.cur];
    P.npts = v.pts[1 - v.cur];
    P.src = v.src;
    P.table = v.table;
    P.addcnt = v.addcnt;
    P.tot = v.tot;
    P.newstart = v.newstart;
    P.addstart = v.addstart;
    P.slot_of = v.slot_of;
    P.iota = v.iota;
    P.skeys = v.skeys;
    P.svals = v.svals;
    P.ctr = v.ctr;
    P.base_id = v.next_id;
    P.inv_res = v.inv_res;
    P.log2 = v.log2;
    P.nearby = v.nearby;
    P.max_num = kNN;
    P.kind = v.kind;
    P.range2 = 5.0 * 5.0;  // GetClosestPoint's default max_range (ivox3d.h:79), laser_mapping.cpp:520
    P.scratch = v.big;
    P.slice = v.big_slice;
    P.tlast = v.tlast;
    P.first = v.first;
    P.lastp1 = v.lastp1;
    P.evict = v.evict;
    return P;
}

// Overflow-pass scratch: a slice holds every candidate one query can hold at once.
static int ivox_ensure_big(livo_ctx* c) {
    IvoxDev& v = c->iv;
    const int64_t slice = (int64_t)v.nearby * kNN + v.max_grid + 8;
    if (slice <= v.big_slice && v.big) return LIVO_OK;
    const int64_t budget = (int64_t)1 << 28;  // 256 MiB per stream group
    int64_t threads = budget / (slice * (int64_t)sizeof(SelElem));
    threads = std::max<int64_t>(64, std::min<int64_t>(16384, threads)) / 64 * 64;
    dev_free(v.big);
    v.big_slice = 0;
    v.big_threads = 0;
    if (dev_alloc(&v.big, (size_t)(kMaxGroups * threads * slice))) return LIVO_E_OOM;  // one set per stream group
    v.big_slice = slice;
    v.big_threads = threads;
    return LIVO_OK;
}

// IVox::AddPoints of the n points in v.src (insertion order), on the device.
static int ivox_ev_scratch(livo_ctx* c, int64_t need) {
    IvoxDev& v = c->iv;
    if (need <= v.ev_cap) return LIVO_OK;
    dev_free(v.ev_k); dev_free(v.ev_k2);
    dev_free(v.ev_a); dev_free(v.ev_b); dev_free(v.ev_c); dev_free(v.ev_d);
    v.ev_cap = 0;
    const size_t cap = (size_t)need;
    if (dev_alloc(&v.ev_k, cap) || dev_alloc(&v.ev_k2, cap) || dev_alloc(&v.ev_a, cap) || dev_alloc(&v.ev_b, cap) ||
        dev_alloc(&v.ev_c, cap) || dev_alloc(&v.ev_d, cap))
        return LIVO_E_OOM;
    v.ev_cap = need;
    return LIVO_OK;
}

// The longest prefix [0, *pend) of the batch whose evictions all take old
// grids the prefix never touches, and their count *evs (0: the first eviction
// already needs a grid the batch touched before it).  At eviction k (the point
// t_ev[k] creating a new grid) grids_cache_.back() is the oldest old grid the
// batch has not touched before t_ev[k] (touched ones moved to the front,
// ivox3d.h:263-268); a victim the batch touches again later would be
// re-created, so the prefix ends before that touch.  Victims advance
// monotonically along the LRU order: one host pass over the old grids' first
// touches.
static int ivox_evict_prefix(livo_ctx* c, const IvoxParams& P, int64_t n_old, const std::vector<uint32_t>& t_ev,
                             int64_t n, int64_t* pend, int64_t* evs) {
    IvoxDev& v = c->iv;
    std::vector<uint32_t> f((size_t)n_old);
    int rc = launch_ivox_oldfirst(P, v.ev_b, n_old, v.ev_a, c->stream);
    if (rc) return rc;
    if (n_old > 0) HIP_TRY(hipMemcpyAsync(f.data(), v.ev_a, (size_t)n_old * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    int64_t end = n, k = 0, i = 0;
    for (; k < (int64_t)t_ev.size() && (int64_t)t_ev[k] < end; k++) {
        const uint32_t t = t_ev[k];
        while (i < n_old && f[(size_t)i] < t) i++;  // touched before this eviction: not the oldest
        if (i == n_old) {                            // no untouched old grid left
            end = t;
            break;
        }
        if (f[(size_t)i] != 0xFFFFFFFFu) end = std::min<int64_t>(end, f[(size_t)i]);
        i++;
    }
    *pend = end;
    *evs = k;
    return LIVO_OK;
}

// IVox::AddPoints (ivox3d.h:256-281) of the points src[off, off + n) as one
// device batch, with the LRU eviction at capacity.  *done = points consumed:
// all of them, or (when an eviction would hit a grid the batch itself touches
// later, or every old grid is touched first) the prefix up to and including
// the first evicting point, processed with its single eviction -- AddPoints of
// a prefix then of the rest is AddPoints of the whole.
static int ivox_add_part(livo_ctx* c, int64_t off, int64_t n, int64_t* done) {
    IvoxDev& v = c->iv;
    *done = 0;
    if (v.npts + n > (int64_t)0xFFFFFFFF || v.next_id + n > (int64_t)0x7FFFFFFF) return LIVO_E_RANGE;
    int rc = ivox_ensure_table(c, v.ngrids + n);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(v.ctr, 0, 5 * sizeof(unsigned long long), c->stream));
    IvoxParams P = ivox_params(c);
    P.src = v.src + 4 * off;
    P.n_src = n;
    rc = launch_ivox_insert(P, c->stream);
    if (rc) return rc;
    unsigned long long ctr[5];
    HIP_TRY(hipMemcpyAsync(ctr, v.ctr, sizeof(ctr), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (ctr[0] & 1ull) {
        rc = launch_ivox_rollback(P, c->stream);
        if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
        return rc ? rc : LIVO_E_RANGE;
    }
    const int64_t E = v.ngrids, N_new = (int64_t)ctr[1], C = v.prm.capacity;
    int64_t ev = std::max<int64_t>(0, E + N_new - (C - 1));  // grids_map_.size() >= capacity_ after a creation
    int64_t consumed = n;
    if (ev > 0) {
        rc = ivox_ev_scratch(c, std::max<int64_t>(v.table, n));
        if (rc) return rc;
        // the point of the first eviction: the (C - 1 - E)-th new grid by creation
        unsigned long long* cnt = v.ctr + 3;  // (scratch counter; ctr[3] is set again below)
        HIP_TRY(hipMemsetAsync(cnt, 0, sizeof(unsigned long long), c->stream));
        rc = launch_ivox_newfirst(P, v.ev_a, cnt, c->stream);
        size_t tb = 0;
        if (!rc) rc = prim_sort_pairs_u32(nullptr, &tb, v.ev_a, v.ev_b, v.ev_a, v.ev_c, N_new, 32, c->stream);
        if (!rc) rc = ensure_prim(c, tb);
        tb = c->prim_bytes;
        if (!rc) rc = prim_sort_pairs_u32(c->prim_tmp, &tb, v.ev_a, v.ev_b, v.ev_a, v.ev_c, N_new, 32, c->stream);
        if (rc) return rc;
        // creation index of each new grid from the (C - 1 - E)-th: the eviction times
        const int64_t c0 = std::max<int64_t>(0, C - 1 - E);
        std::vector<uint32_t> t_ev((size_t)(N_new - c0));
        HIP_TRY(hipMemcpyAsync(t_ev.data(), v.ev_b + c0, t_ev.size() * 4, hipMemcpyDeviceToHost, c->stream));
        // the old grids from the least recently used: victims and the conflict check
        HIP_TRY(hipMemsetAsync(cnt, 0, sizeof(unsigned long long), c->stream));
        rc = launch_ivox_oldkeys(P, v.ev_k, v.ev_a, cnt, c->stream);
        if (rc) return rc;
        const int64_t n_old = E;
        tb = 0;
        rc = prim_sort_pairs_u64(nullptr, &tb, v.ev_k, v.ev_k2, v.ev_a, v.ev_b, n_old, 64, c->stream);
        if (!rc) rc = ensure_prim(c, tb);
        tb = c->prim_bytes;
        if (!rc) rc = prim_sort_pairs_u64(c->prim_tmp, &tb, v.ev_k, v.ev_k2, v.ev_a, v.ev_b, n_old, 64, c->stream);
        if (!rc) rc = launch_ivox_untouched(P, v.ev_b, n_old, v.ev_c, c->stream);
        if (!rc) rc = ivox_scan(c, v.ev_c, v.ev_d, n_old);
        if (rc) return rc;
        uint32_t tail[2] = {0u, 0u};
        if (n_old > 0) {
            HIP_TRY(hipMemcpyAsync(&tail[0], v.ev_d + n_old - 1, 4, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipMemcpyAsync(&tail[1], v.ev_c + n_old - 1, 4, hipMemcpyDeviceToHost, c->stream));
        }
        HIP_TRY(hipStreamSynchronize(c->stream));
        const uint32_t j_first = t_ev[0];
        const int64_t untouched = (int64_t)tail[0] + tail[1];
        bool conflict = ev > untouched;
        if (!conflict) {
            HIP_TRY(hipMemsetAsync(v.ctr + 3, 0, sizeof(unsigned long long), c->stream));
            rc = launch_ivox_victims(P, v.ev_b, v.ev_d, n_old, ev, j_first, c->stream);
            if (rc) return rc;
            HIP_TRY(hipMemcpyAsync(ctr, v.ctr, sizeof(ctr), hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            conflict = (ctr[0] & 2ull) != 0;
        }
        if (conflict) {
            // A run of evictions: the longest prefix whose victims are old grids
            // it leaves untouched (ivox_evict_prefix), inserted again alone.
            int64_t pend = 0, evs = 0;
            rc = ivox_evict_prefix(c, P, n_old, t_ev, n, &pend, &evs);
            if (rc) return rc;
            rc = launch_ivox_rollback(P, c->stream);
            if (rc) return rc;
            if (evs > 0) {
                P.n_src = pend;
                HIP_TRY(hipMemsetAsync(v.ctr, 0, 5 * sizeof(unsigned long long), c->stream));
                rc = launch_ivox_insert(P, c->stream);
                if (!rc) rc = launch_ivox_untouched(P, v.ev_b, n_old, v.ev_c, c->stream);
                if (!rc) rc = ivox_scan(c, v.ev_c, v.ev_d, n_old);
                // (the victims kernel's conflict flag is conservative -- it also flags
                // an older grid touched between two evictions -- the scan is exact: off)
                if (!rc) rc = launch_ivox_victims(P, v.ev_b, v.ev_d, n_old, evs, 0xFFFFFFFFu, c->stream);
                if (rc) return rc;
                HIP_TRY(hipMemcpyAsync(ctr, v.ctr, sizeof(ctr), hipMemcpyDeviceToHost, c->stream));
                HIP_TRY(hipStreamSynchronize(c->stream));
                if ((ctr[0] & 2ull) || E + (int64_t)ctr[1] - (C - 1) != evs) {  // (the scan's invariant)
                    // undo the prefix's uncommitted slots, so the table stays clean for the next AddPoints
                    rc = launch_ivox_rollback(P, c->stream);
                    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
                    return rc ? rc : LIVO_E_HIP;
                }
                consumed = pend;
                ev = evs;
                conflict = false;
            }
        }
        if (conflict) {
            // the first eviction's victim is a grid the batch touched before it:
            // the prefix [0, j_first] alone, one eviction, of the grid least
            // recently used at its last point (new grids included)
            consumed = (int64_t)j_first + 1;
            P.n_src = consumed;
            HIP_TRY(hipMemsetAsync(v.ctr, 0, 5 * sizeof(unsigned long long), c->stream));
            rc = launch_ivox_insert(P, c->stream);
            if (rc) return rc;
            HIP_TRY(hipMemsetAsync(v.ctr + 4, 0xFF, sizeof(unsigned long long), c->stream));
            rc = launch_ivox_tcur_min(P, c->stream);
            if (!rc) rc = launch_ivox_mark_min(P, c->stream);
            if (rc) return rc;
            HIP_TRY(hipMemcpyAsync(ctr, v.ctr, sizeof(ctr), hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            ev = 1;
        }
    }
    const int64_t N_new_b = (int64_t)ctr[1];
    // new CSR buffer
    const int other = 1 - v.cur;
    const int64_t need = v.npts + consumed + 3;
    if (v.pts_cap[other] < need) {
        dev_free(v.pts[other]);
        v.pts_cap[other] = 0;
        const int64_t cap = std::max<int64_t>(need + need / 2, 1 << 16);
        if (dev_alloc(&v.pts[other], (size_t)cap * 4)) return LIVO_E_OOM;
        v.pts_cap[other] = cap;
        P.npts = v.pts[other];
    }
    rc = launch_ivox_prepare(P, c->stream);
    if (!rc) rc = ivox_scan(c, v.tot, v.newstart, v.table);
    if (!rc) rc = ivox_scan(c, v.addcnt, v.addstart, v.table);
    if (!rc) {
        int bits = 1;
        while (((int64_t)1 << bits) <= v.table) bits++;  // the out-of-range key `table` included
        size_t tb = 0;
        rc = prim_sort_pairs_u32(nullptr, &tb, v.slot_of, v.skeys, v.iota, v.svals, consumed, bits, c->stream);
        if (!rc) rc = ensure_prim(c, tb);
        tb = c->prim_bytes;
        if (!rc)
            rc = prim_sort_pairs_u32(c->prim_tmp, &tb, v.slot_of, v.skeys, v.iota, v.svals, consumed, bits, c->stream);
    }
    if (!rc) rc = launch_ivox_move(P, c->stream);
    if (!rc) rc = launch_ivox_place(P, c->stream);
    if (!rc) rc = launch_ivox_fix(P, c->stream);
    if (!rc) rc = launch_ivox_commit(P, c->stream);
    if (!rc && ev > 0) rc = launch_ivox_drop(P, c->stream);
    if (rc) return rc;
    // the number of points the evicted grids held leaves the map
    unsigned long long gone = 0;
    int64_t npts_new = 0;
    {
        uint32_t tail[2];
        HIP_TRY(hipMemcpyAsync(&tail[0], v.newstart + v.table - 1, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(&tail[1], v.tot + v.table - 1, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(ctr, v.ctr, sizeof(ctr), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        npts_new = (int64_t)tail[0] + tail[1];
        (void)gone;
    }
    v.cur = other;
    v.npts = npts_new;
    v.ngrids += N_new_b - ev;
    v.next_id += consumed;
    v.max_grid = (int64_t)ctr[2];
    if (ev > 0) {
        rc = ivox_rehash_to(c, v.log2);  // evicted slots leave holes in the probe chains
        if (rc) return rc;
    }
    *done = consumed;
    v.add_passes++;
    return LIVO_OK;
}

static int ivox_add_dev(livo_ctx* c, int64_t n) {
    IvoxDev& v = c->iv;
    int64_t off = 0;
    while (off < n) {
        int64_t done = 0;
        const int rc = ivox_add_part(c, off, n - off, &done);
        if (rc) return rc;
        off += done;
    }
    (void)v;
    const int rc = ivox_trim_table(c);
    return rc ? rc : ivox_ensure_big(c);
}

static bool map_ready(const livo_ctx* c) {
    return c->backend == LIVO_BACKEND_IVOX ? c->iv.ready : c->has_map;
}

// The search of one evaluation with the context's backend (+ its exact /
// overflow pass); `later`: an evaluation after the first (seeded / gated).
static int backend_knn(livo_ctx* c, const KnnParams& kp, int n_jobs, int64_t max_n, bool later, hipStream_t st) {
    if (c->backend == LIVO_BACKEND_IVOX) return launch_ivox_knn(kp, n_jobs, max_n, later, c->iv.big_threads, st);
    return c->knn_kind >= 1 ? launch_knn_grid(kp, n_jobs, max_n, later, c->knn_kind == 2, st)
                            : launch_knn_leaf(kp, n_jobs, max_n, later, st);
}

// ---------------------------------------------- ikd-Tree incremental map --
extern "C" {
static ScanBuf* get_scan(livo_ctx* c, int32_t id);
static ScanBuf* get_scan_q(livo_ctx* c, int32_t id);
}
static int build_cell_runs(livo_ctx* c, int64_t M);
static int build_ball_runs(livo_ctx* c, int64_t M, float r5, double ext);
#if LIVO_IDX_RUNS
static int build_cell_runs_into(livo_ctx* c, const float* pts, int64_t M, GridSlot** slots, RunWord** idx,
                                int32_t* log2, int64_t* words);
#endif
static void dyn_free(DynDev& d) {
    dev_free(d.all); dev_free(d.alive);
    dev_free(d.keys); dev_free(d.skeys); dev_free(d.iota); dev_free(d.svals);
    dev_free(d.heads); dev_free(d.runid); dev_free(d.starts);
    dev_free(d.W); dev_free(d.seq); dev_free(d.Ws);
    dev_free(d.defer); dev_free(d.dpos); dev_free(d.dlist); dev_free(d.keep); dev_free(d.apos);
    dev_free(d.boxes); dev_free(d.ctr);  // (d.dirty lives in d.ctr's allocation)
    dev_free(d.rpts); dev_free(d.rpos); dev_free(d.dslots); dev_free(d.dpts);
    dev_free(d.dvslots); dev_free(d.dvidx); dev_free(d.gpts_alt);
    dev_free(d.scan.ticket); dev_free(d.scan.status);
    d = DynDev{};
}

static int dyn_grow(livo_ctx* c, int64_t need) {  // id capacity
    DynDev& d = c->dyn;
    if (need <= d.cap) return LIVO_OK;
    if (need > kMaxMapPoints) return LIVO_E_RANGE;
    const int64_t cap = std::min<int64_t>(std::max<int64_t>(need + (need >> 1), 1 << 16), kMaxMapPoints);
    float* a = nullptr;
    uint8_t* l = nullptr;
    if (dev_alloc(&a, (size_t)cap * 4) || dev_alloc(&l, (size_t)cap)) {
        dev_free(a);
        dev_free(l);
        return LIVO_E_OOM;
    }
    HIP_TRY(hipMemsetAsync(l, 0, (size_t)cap, c->stream));
    if (d.n_ids > 0) {
        HIP_TRY(hipMemcpyAsync(a, d.all, (size_t)d.n_ids * 16, hipMemcpyDeviceToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(l, d.alive, (size_t)d.n_ids, hipMemcpyDeviceToDevice, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    dev_free(d.all);
    dev_free(d.alive);
    d.all = a;
    d.alive = l;
    d.cap = cap;
    return LIVO_OK;
}

static int dyn_sort_scratch(livo_ctx* c, int64_t n) {
    DynDev& d = c->dyn;
    if (n <= d.sort_cap) return LIVO_OK;
    const int64_t cap = std::max<int64_t>(n + (n >> 2), 4096);
    dev_free(d.keys); dev_free(d.skeys); dev_free(d.iota); dev_free(d.svals);
    dev_free(d.heads); dev_free(d.runid); dev_free(d.starts);
    d.sort_cap = 0;
    if (dev_alloc(&d.keys, cap) || dev_alloc(&d.skeys, cap) || dev_alloc(&d.iota, cap) || dev_alloc(&d.svals, cap) ||
        dev_alloc(&d.heads, cap) || dev_alloc(&d.runid, cap) || dev_alloc(&d.starts, cap + 1))
        return LIVO_E_OOM;
    d.sort_cap = cap;
    return LIVO_OK;
}

static int dyn_add_scratch(livo_ctx* c, int64_t n) {
    DynDev& d = c->dyn;
    if (n <= d.add_cap) return LIVO_OK;
    const int64_t cap = std::max<int64_t>(n + (n >> 2), 4096);
    dev_free(d.W); dev_free(d.seq); dev_free(d.Ws);
    dev_free(d.defer); dev_free(d.dpos); dev_free(d.dlist); dev_free(d.keep); dev_free(d.apos);
    d.add_cap = 0;
    if (dev_alloc(&d.W, (size_t)cap * 4) || dev_alloc(&d.seq, (size_t)cap * 4) || dev_alloc(&d.Ws, (size_t)cap * 4) ||
        dev_alloc(&d.defer, cap) ||
        dev_alloc(&d.dpos, cap) || dev_alloc(&d.dlist, cap) || dev_alloc(&d.keep, cap) || dev_alloc(&d.apos, cap))
        return LIVO_E_OOM;
    d.add_cap = cap;
    return LIVO_OK;
}

// The one-launch scans' state for up to n values (status words cleared once;
// every call tags its own with a new epoch).
static int dyn_scan_ready(livo_ctx* c, int64_t n) {
    ScanCtx& sc = c->dyn.scan;
    sc.err = c->dyn.ctr + kDynError;
    if (!sc.ticket) {
        if (dev_alloc(&sc.ticket, 1)) return LIVO_E_OOM;
        HIP_TRY(hipMemsetAsync(sc.ticket, 0, 8, c->stream));
        sc.issued = 0;
    }
    const int64_t tiles = scan_tiles(n + 1) + 1;
    if (sc.status_cap < tiles) {
        const int64_t cap = tiles + (tiles >> 1) + 64;
        dev_free(sc.status);
        sc.status_cap = 0;
        if (dev_alloc(&sc.status, (size_t)cap)) return LIVO_E_OOM;
        HIP_TRY(hipMemsetAsync(sc.status, 0, (size_t)cap * 8, c->stream));
        sc.status_cap = cap;
    }
    return LIVO_OK;
}
static int sort_u32(livo_ctx* c, const uint32_t* kin, uint32_t* kout, const uint32_t* vin, uint32_t* vout, int64_t n,
                    int bits) {
    size_t tb = 0;
    int rc = prim_sort_pairs_u32(nullptr, &tb, kin, kout, vin, vout, n, bits, c->stream);
    if (!rc) rc = ensure_prim(c, tb);
    tb = c->prim_bytes;
    if (!rc) rc = prim_sort_pairs_u32(c->prim_tmp, &tb, kin, kout, vin, vout, n, bits, c->stream);
    return rc;
}
static int sort_u64(livo_ctx* c, const unsigned long long* kin, unsigned long long* kout, const uint32_t* vin,
                    uint32_t* vout, int64_t n) {
    size_t tb = 0;
    int rc = prim_sort_pairs_u64(nullptr, &tb, kin, kout, vin, vout, n, 64, c->stream);
    if (!rc) rc = ensure_prim(c, tb);
    tb = c->prim_bytes;
    if (!rc) rc = prim_sort_pairs_u64(c->prim_tmp, &tb, kin, kout, vin, vout, n, 64, c->stream);
    return rc;
}

// The runs' base point set = the current cell grid (c->gpts, c->map_points
// points in grid order; the runs were built on it): rpts a copy of it (the
// grid itself is rebuilt by every change), rpos the position of each id,
// ids below n_ids the base, no deletion marks, an empty delta.
static int dyn_base_from_grid(livo_ctx* c) {
    DynDev& d = c->dyn;
    d.runs = false;
    const int64_t na = c->map_points;
    if (d.rpts_cap < na + 3) {
        dev_free(d.rpts);
        d.rpts_cap = 0;
        const int64_t cap = (na + 3) + ((na + 3) >> 3);
        if (dev_alloc(&d.rpts, (size_t)cap * 4)) return LIVO_E_OOM;
        d.rpts_cap = cap;
    }
    if (d.rpos_cap < d.n_ids) {
        dev_free(d.rpos);
        d.rpos_cap = 0;
        const int64_t cap = std::max<int64_t>(d.n_ids + (d.n_ids >> 3), 1);
        if (dev_alloc(&d.rpos, (size_t)cap)) return LIVO_E_OOM;
        d.rpos_cap = cap;
    }
    HIP_TRY(hipMemcpyAsync(d.rpts, c->gpts, (size_t)(na + 3) * 16, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(d.rpos, 0xFF, (size_t)std::max<int64_t>(d.n_ids, 1) * 4, c->stream));
    int rc = launch_dyn_rpos(d.rpts, na, d.rpos, c->stream);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    d.base_ids = d.n_ids;
    d.base_n = na;
    d.tomb = 0;
    d.d_n = 0;
    d.runs = true;
    return LIVO_OK;
}

// The runs rebuilt from the current points (the grid just rebuilt by
// dyn_rebuild): cell runs, ball runs with the build's r5, then the new base.
static int dyn_rebase(livo_ctx* c) {
    DynDev& d = c->dyn;
    d.runs = false;
    const int64_t na = c->map_points;
    const bool balls = c->bslots != nullptr && c->br5 > 0.f;
    int rc = na > 0 && na * 27 + kRunPad < (int64_t)0xFFFFFFFFll ? build_cell_runs(c, na) : LIVO_E_RANGE;
    if (!rc && balls) {
        const int brc = build_ball_runs(c, na, c->br5, 2.0 * (double)d.cmax);
        if (brc == LIVO_E_OOM) {
            (void)hipGetLastError();
            dev_free(c->bslots);
            dev_free(c->bpts);
            c->bentries = 0;
        } else if (brc) {
            rc = brc;
        }
    }
    if (!rc) rc = dyn_base_from_grid(c);
    if (rc == LIVO_E_OOM || rc == LIVO_E_RANGE) {  // the cell walk serves the map from here on
        (void)hipGetLastError();
        dev_free(c->vslots);
        dev_free(c->vpts);
        dev_free(c->bslots);
        dev_free(c->bpts);
        c->bentries = 0;
        d.runs = false;
        return LIVO_OK;
    }
    if (!rc) d.rebases++;
    return rc;
}

// After every change of the incremental map (dyn_rebuild): mark the base points
// deleted since, count the delta, rebase when it or the marks outgrow the
// base, else build the delta grid of the points added since the base.
static int dyn_runs_update(livo_ctx* c) {
    DynDev& d = c->dyn;
    if (!d.runs) return LIVO_OK;
    HIP_TRY(hipMemsetAsync(d.ctr + kDynTomb, 0, 2 * sizeof(unsigned long long), c->stream));
    int rc = launch_dyn_tomb(d.rpts, d.rpos, d.alive, d.base_ids, d.ctr, c->stream);
    const int64_t nd_ids = d.n_ids - d.base_ids;
    if (!rc && nd_ids > 0) rc = launch_count_alive(d.alive + d.base_ids, nd_ids, d.ctr, c->stream);
    if (rc) return rc;
    unsigned long long h[2];
    HIP_TRY(hipMemcpyAsync(h, d.ctr + kDynTomb, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    d.tomb += (int64_t)h[0];
    const int64_t nd = (int64_t)h[1];
    if ((double)nd > d.rebase_frac * (double)d.base_n || (double)d.tomb > 2.0 * d.rebase_frac * (double)d.base_n)
        return dyn_rebase(c);
    d.d_n = nd;
    if (nd == 0) return LIVO_OK;
    // the delta grid: cell keys of the ids since the base, sorted, gathered (k_dyn_gather pads 3)
    rc = launch_dyn_cellkeys(d.all + 4 * d.base_ids, d.alive + d.base_ids, nd_ids, c->gorg, 1.0f / c->gh, d.keys, d.iota,
                             d.ctr, c->stream);
    if (!rc) rc = sort_u64(c, d.keys, d.skeys, d.iota, d.svals, nd_ids);
    if (rc) return rc;
    if (d.dpts_cap < nd + 3) {
        dev_free(d.dpts);
        d.dpts_cap = 0;
        const int64_t cap = (nd + 3) + ((nd + 3) >> 1);
        if (dev_alloc(&d.dpts, (size_t)cap * 4)) return LIVO_E_OOM;
        d.dpts_cap = cap;
    }
    rc = launch_dyn_gather(d.skeys, d.svals, nd, d.all + 4 * d.base_ids, d.dpts, d.heads, c->stream);
    if (!rc) rc = ivox_scan(c, d.heads, d.runid, nd);
    if (!rc) rc = launch_dyn_runs(d.heads, d.runid, nd, d.starts, d.ctr + kDynRuns, c->stream);
    if (rc) return rc;
    unsigned long long cells = 0;
    HIP_TRY(hipMemcpyAsync(&cells, d.ctr + kDynRuns, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    int log2 = 4;
    while (((int64_t)1 << log2) < 4 * (int64_t)cells) log2++;
    const int64_t table = (int64_t)1 << log2;
    if (d.dslot_cap < table) {
        dev_free(d.dslots);
        d.dslot_cap = 0;
        if (dev_alloc(&d.dslots, (size_t)table)) return LIVO_E_OOM;
        d.dslot_cap = table;
    }
    rc = launch_ivox_clear(d.dslots, table, c->stream);
    if (!rc) rc = launch_dyn_slots(d.skeys, d.starts, (int64_t)cells, d.dslots, log2, c->stream);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    d.dlog2 = log2;
#if LIVO_IDX_RUNS
    // and its cell runs: a query scans its cube's delta points in one run, as the base's
    int64_t words = 0;
    rc = build_cell_runs_into(c, d.dpts, nd, &d.dvslots, &d.dvidx, &d.dvlog2, &words);
    if (rc) {
        (void)hipGetLastError();
        dev_free(d.dvslots);
        dev_free(d.dvidx);
        return rc == LIVO_E_OOM || rc == LIVO_E_RANGE ? dyn_rebase(c) : rc;
    }
#endif
    return LIVO_OK;
}

static int dyn_rebuild(livo_ctx* c);

// The built map becomes the incremental point set (ids = build indices).
static int dyn_activate(livo_ctx* c) {
    DynDev& d = c->dyn;
    if (d.active) return LIVO_OK;
    if (!c->has_map) return LIVO_E_NOMAP;
    if (c->knn_kind == 0) return LIVO_E_INVALID;  // kept on the cell grid (not LIVO_KNN_KIND=leaf)
    if (!d.ctr) {
        if (dev_alloc(&d.ctr, kDynCtrPad + kDynDirtyCap)) return LIVO_E_OOM;
        d.dirty = d.ctr + kDynCtrPad;  // (one allocation: dyn_add clears both with one memset)
    }
    const int64_t M = c->map_points;
    d.n_ids = d.n_alive = 0;
    int rc = dyn_grow(c, M + 1);
    if (rc) return rc;
    if (M == 0) {  // an empty build chose its cell from nothing: use 0.4 m cells at the origin
        c->gh = 0.4f;
        c->gorg[0] = c->gorg[1] = c->gorg[2] = 0.f;
    }
    rc = launch_dyn_seed(c->gpts, M, d.all, d.alive, c->stream);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    d.n_ids = d.n_alive = M;
    d.cmax = c->gcmax;
    d.gslot_cap = (int64_t)1 << c->glog2;
    d.gpts_cap = M + 3;
    d.active = true;
    d.runs = false;
    d.d_n = 0;
    d.grid_ids = -1;  // (the build's grid: the first rebuild sorts)
    if (const char* env = std::getenv("LIVO_DYN_MERGE")) d.merge = std::atoi(env) != 0;
    if (const char* env = std::getenv("LIVO_DYN_BOX_CELL_MAX")) {  // tuning knob (0: off)
        const double v = std::atof(env);
        if (v >= 0.0 && v < 100.0) d.box_cell_max = (float)v;
    }
    if (const char* env = std::getenv("LIVO_DYN_BOX_CELL")) {  // tuning knob (0: off)
        const double v = std::atof(env);
        if (v >= 0.0 && v < 100.0) d.box_cell = (float)v;
    }
    if (const char* env = std::getenv("LIVO_DYN_REBASE")) {
        const double v = std::atof(env);
        if (v > 0.0 && v < 100.0) d.rebase_frac = v;
    }
    // The runs on the incremental map are opt-in (LIVO_DYN_RUNS=1): they take the
    // IEKF from 0.253 to 0.215 ms per scan on a map the scans built, but keeping
    // them (marks, delta grid and runs, rebases) takes Add_Points from 0.56 to
    // 1.34 ms, so the odometry loop runs at half the rate.
    const char* env_runs = std::getenv("LIVO_DYN_RUNS");
    if (LIVO_IDX_RUNS && c->vslots && c->vpts && M > 0 && env_runs && std::atoi(env_runs) == 1) {
        rc = dyn_base_from_grid(c);  // the built map's runs index its grid: the grid becomes the base
        if (rc == LIVO_E_OOM) {
            (void)hipGetLastError();
            rc = LIVO_OK;  // (the cell walk then serves the incremental map, as without runs)
        }
        if (rc) return rc;
    }
    return LIVO_OK;
}

constexpr int kMergeRetry = -1000;  // dyn_rebuild_merge: the counts disagree, sort instead
static int dyn_rebuild_merge(livo_ctx* c);

// The cell grid of k_knn_grid rebuilt from the alive points (same layout as
// build_grid_map: cells in key order, a cell's points in id order).
static int dyn_rebuild(livo_ctx* c) {
    DynDev& d = c->dyn;
    if (!d.runs && (c->gh < d.min_gh || (d.max_gh > 0.f && c->gh > d.max_gh))) {
        const float lo = (float)(2.0 * (double)d.cmax / (double)(kGridBias - 2));
        const float h = c->gh < d.min_gh ? d.min_gh : std::max(d.max_gh, d.min_gh);
        c->gh = std::max(h, lo * 1.01f);
    }
    if (d.merge && d.grid_ids >= 0 && d.cells >= 0 && d.grid_gh == c->gh && d.grid_ids <= d.n_ids) {
        const int rc = dyn_rebuild_merge(c);
        if (rc != kMergeRetry) return rc;
        (void)hipGetLastError();  // (the merge found an inconsistency: sort instead)
    }
    int rc = dyn_sort_scratch(c, std::max<int64_t>(d.n_ids, 1));
    if (rc) return rc;
    const int64_t na = d.n_alive;
    if (d.gpts_cap < na + 3) {
        const int64_t cap = (na + 3) + ((na + 3) >> 2);
        dev_free(c->gpts);
        if (dev_alloc(&c->gpts, (size_t)cap * 4)) return LIVO_E_OOM;
        d.gpts_cap = cap;
    }
    HIP_TRY(hipMemsetAsync(d.ctr, 0, kDynCtrN * sizeof(unsigned long long), c->stream));
    if (d.n_ids > 0) {
        rc = launch_dyn_cellkeys(d.all, d.alive, d.n_ids, c->gorg, 1.0f / c->gh, d.keys, d.iota, d.ctr, c->stream);
        if (!rc) rc = sort_u64(c, d.keys, d.skeys, d.iota, d.svals, d.n_ids);
    }
    if (!rc) rc = launch_dyn_gather(d.skeys, d.svals, na, d.all, c->gpts, d.heads, c->stream);
    if (!rc && na > 0) rc = ivox_scan(c, d.heads, d.runid, na);
    if (!rc && na > 0) rc = launch_dyn_runs(d.heads, d.runid, na, d.starts, d.ctr + kDynRuns, c->stream);
    if (rc) return rc;
    unsigned long long h[kDynCtrN];
    HIP_TRY(hipMemcpyAsync(h, d.ctr, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (h[kDynError]) return LIVO_E_RANGE;
    const int64_t cells = (int64_t)h[kDynRuns];
    int log2 = 4;
    while (((int64_t)1 << log2) < 4 * cells) log2++;  // load factor <= 1/4, as build_grid_map
    const int64_t table = (int64_t)1 << log2;
    if (d.gslot_cap < table) {  // (twice: headroom for Add_Points' fused rebuild)
        dev_free(c->gslots);
        d.gslot_cap = 0;
        if (dev_alloc(&c->gslots, (size_t)(2 * table))) return LIVO_E_OOM;
        d.gslot_cap = 2 * table;
    }
    rc = launch_ivox_clear(c->gslots, table, c->stream);
    if (!rc) rc = launch_dyn_slots(d.skeys, d.starts, cells, c->gslots, log2, c->stream);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->glog2 = log2;
    c->map_points = na;
    c->geps = (float)(32.0 * std::ldexp(1.0, -24) * (double)d.cmax + 1e-7);
    c->grid_bytes = table * (int64_t)sizeof(GridSlot) + d.gpts_cap * 16;
    for (auto& s : c->scans) s.searched = false;  // cached neighbours refer to the old map
    d.grid_ids = d.n_ids;
    d.grid_gh = c->gh;
    d.cells = cells;
    d.rebuilds_sorted++;
    return dyn_runs_update(c);
}

// The grid after a change without sorting the map again: the ids added since
// the last rebuild (a few hundred per scan) are keyed and sorted, the old
// grid's survivors are ranked by a scan, and k_dyn_merge places both (the
// same (key, id) order a sort gives, so the same grid bit for bit).  The hash
// table is sized for the old cell count + the new points (a bound: each new
// point opens at most one cell), so nothing is read back before it is filled;
// one read-back at the end.  kMergeRetry: inconsistent counts (the caller
// sorts instead).
static int dyn_rebuild_merge(livo_ctx* c) {
    DynDev& d = c->dyn;
    const int64_t na_old = c->map_points, na = d.n_alive, g0 = d.grid_ids, m = d.n_ids - g0;
    int rc = dyn_sort_scratch(c, std::max<int64_t>(std::max<int64_t>(na_old, na), m) + 1);
    if (rc) return rc;
    if (d.gpts_alt_cap < na + 3) {
        const int64_t cap = (na + 3) + ((na + 3) >> 2);
        dev_free(d.gpts_alt);
        d.gpts_alt_cap = 0;
        if (dev_alloc(&d.gpts_alt, (size_t)cap * 4)) return LIVO_E_OOM;
        d.gpts_alt_cap = cap;
    }
    const float inv = 1.0f / c->gh;
    HIP_TRY(hipMemsetAsync(d.ctr, 0, kDynCtrN * sizeof(unsigned long long), c->stream));
    if (m > 0 && m <= kNewSortMax) {  // (a scan's few hundred winners: one workgroup)
        rc = launch_dyn_newsort(d.all + 4 * g0, d.alive + g0, m, c->gorg, inv, d.skeys, d.svals, d.ctr, c->stream);
    } else if (m > 0) {
        rc = launch_dyn_cellkeys(d.all + 4 * g0, d.alive + g0, m, c->gorg, inv, d.keys, d.iota, d.ctr, c->stream);
        if (!rc) rc = sort_u64(c, d.keys, d.skeys, d.iota, d.svals, m);
    }
    if (!rc) rc = dyn_scan_ready(c, std::max(na_old, na) + 1);
    if (!rc) rc = launch_scan_flags(d.scan, c->gpts, na_old, d.alive, d.runid, c->stream);
    if (rc) return rc;
    DynMergeParams P{};
    P.gpts = c->gpts; P.na_old = na_old; P.rank = d.runid; P.alive = d.alive;
    P.nkeys = d.skeys; P.nidx = d.svals; P.m = m; P.g0 = g0; P.all = d.all;
    P.out = d.gpts_alt; P.okeys = d.keys; P.na = na;
    std::memcpy(P.org, c->gorg, sizeof(P.org));
    P.inv = inv; P.ctr = d.ctr;
    rc = launch_dyn_merge(P, c->stream);
    if (!rc && na > 0) rc = launch_scan_runs(d.scan, d.keys, na, d.starts, d.ctr + kDynRuns, c->stream);
    if (rc) return rc;
    const int64_t bound = std::max<int64_t>(std::min<int64_t>(na, d.cells + m), 1);
    int log2 = 4;
    while (((int64_t)1 << log2) < 4 * bound) log2++;  // load factor <= 1/4, as build_grid_map
    const int64_t table = (int64_t)1 << log2;
    if (d.gslot_cap < table) {  // (twice: the fused pass's bound, + kNewSortMax, fits the next calls)
        dev_free(c->gslots);
        d.gslot_cap = 0;
        if (dev_alloc(&c->gslots, (size_t)(2 * table))) return LIVO_E_OOM;
        d.gslot_cap = 2 * table;
    }
    rc = launch_ivox_clear(c->gslots, table, c->stream);
    if (!rc && na > 0) rc = launch_dyn_slots(d.keys, d.starts, bound, c->gslots, log2, c->stream, d.ctr + kDynRuns,
                                             d.ctr + kDynError);
    if (rc) return rc;
    unsigned long long h[kDynCtrN];
    HIP_TRY(hipMemcpyAsync(h, d.ctr, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (h[kDynError] & 64ull) return LIVO_E_HIP;  // a scan's look-back gave up
    if (h[kDynError] & (8ull | 16ull)) return kMergeRetry;  // (c->gpts untouched: the sort rebuilds from it)
    if (h[kDynError]) return LIVO_E_RANGE;
    std::swap(c->gpts, d.gpts_alt);
    std::swap(d.gpts_cap, d.gpts_alt_cap);
    c->glog2 = log2;
    c->map_points = na;
    c->geps = (float)(32.0 * std::ldexp(1.0, -24) * (double)d.cmax + 1e-7);
    c->grid_bytes = table * (int64_t)sizeof(GridSlot) + d.gpts_cap * 16;
    for (auto& s : c->scans) s.searched = false;  // cached neighbours refer to the old map
    d.grid_ids = d.n_ids;
    d.cells = (int64_t)h[kDynRuns];
    d.rebuilds_merged++;
    return dyn_runs_update(c);
}

// Add_Points of the n points in d.W (filled by the caller).
// world: map_incremental's scan and state (k_add_prep transforms the points into d.W), or null (d.W filled)
struct DynWorldIn {
    const float* pts;
    const int32_t* perm;
    const livo_state* state;
};
static int dyn_add(livo_ctx* c, int64_t n, float ds, bool downsample, livo_map_add_stats* out,
                   const DynWorldIn* world = nullptr) {
    DynDev& d = c->dyn;
    // Add_Points' downsampling leaves one point per box of edge ds where the
    // scans pass: the cell walk's grid (rebuilt after this change) takes cells
    // of [box_cell, box_cell_max] * ds = [0.6, 1.0] m for 0.5 m boxes, so a walk
    // through thinned regions probes a few cells, not a cube of near-empty ones
    // sized for a dense built map (IEKF 0.58 vs 0.78 ms per scan on the thinned
    // 1M map), and a map built from one sparse scan does not keep cells sized
    // for its first few thousand points (0.245 vs 0.272 ms, Add_Points 0.48 vs
    // 0.62 ms; profiles/r04_ab_dyn_box_cell.txt).  The runs, when kept, index
    // the built grid.
    if (downsample && ds > 0.f && !d.runs) {
        d.min_gh = std::max(d.min_gh, d.box_cell * ds);
        if (d.box_cell_max > 0.f) d.max_gh = std::max(d.max_gh, d.box_cell_max * ds);
    }
    livo_map_add_stats st{};
    if (n > 0) {
        if (d.n_ids + n > kMaxMapPoints || n > (int64_t)0x7FFFFFFF) return LIVO_E_RANGE;
        int rc = dyn_grow(c, d.n_ids + n);
        if (!rc) rc = dyn_sort_scratch(c, n + 1);
        if (rc) return rc;
        // The merged grid rebuild runs in the same stream pass with the counts on
        // the device (one read-back for both), when the grid covers every id, its
        // cell edge stays, and the kept points fit k_dyn_newsort's workgroup (else,
        // or on any flag, dyn_rebuild runs after the read-back as before).
        const bool gh_stays = !(c->gh < d.min_gh || (d.max_gh > 0.f && c->gh > d.max_gh));
        bool fused = downsample && d.merge && !d.runs && d.grid_ids == d.n_ids && d.cells >= 0 &&
                     d.grid_gh == c->gh && gh_stays;
        const int64_t na_old = c->map_points, g0 = d.n_ids, m_ub = std::min<int64_t>(n, kNewSortMax);
        const int64_t na_ub = na_old + m_ub, cell_bound = std::max<int64_t>(std::min(na_ub, d.cells + m_ub), 1);
        int log2 = 4;
        while (((int64_t)1 << log2) < 4 * cell_bound) log2++;  // load factor <= 1/4, as build_grid_map
        const int64_t table = (int64_t)1 << log2;
        if (fused) {
            rc = dyn_sort_scratch(c, std::max(n, na_ub) + 1);
            if (!rc) rc = dyn_scan_ready(c, std::max(n, na_ub) + 1);
            if (!rc && d.gpts_alt_cap < na_ub + 3) {
                const int64_t cap = (na_ub + 3) + ((na_ub + 3) >> 2);
                dev_free(d.gpts_alt);
                d.gpts_alt_cap = 0;
                if (dev_alloc(&d.gpts_alt, (size_t)cap * 4)) rc = LIVO_E_OOM;
                else d.gpts_alt_cap = cap;
            }
            if (rc) return rc;
            // the add reads the current table: a table that must grow takes the
            // separate rebuild this time (which leaves headroom for the next)
            if (d.gslot_cap < table) fused = false;
        }
        // The box keys sort as 30-bit keys (10 bits per axis, wrapped): k_scan_boxes
        // finds two boxes sharing a wrapped key and the batch is redone with the
        // 64-bit keys (ctr bit 32: nothing changed).  LIVO_DYN_WIDE_KEYS=1: always 64-bit.
        static const bool wide_env = [] {
            const char* e = std::getenv("LIVO_DYN_WIDE_KEYS");
            return e && std::atoi(e) == 1;
        }();
        unsigned long long h[kDynCtrN];
        for (bool wide = wide_env;; wide = true) {
            HIP_TRY(hipMemsetAsync(d.ctr, 0, (kDynCtrPad + kDynDirtyCap) * sizeof(unsigned long long), c->stream));
            DynAddParams P{};
            P.W = d.W; P.n = n; P.ds = ds; P.downsample = downsample ? 1 : 0;
            P.gslots = c->gslots; P.gpts = c->gpts; P.glog2 = c->glog2;
            std::memcpy(P.gorg, c->gorg, sizeof(P.gorg));
            P.gh = c->gh; P.ginv = 1.0f / c->gh; P.geps = c->geps;
            P.base = d.n_ids; P.alive = d.alive;
            P.keys = d.keys; P.iota = d.iota; P.skeys = d.skeys; P.svals = d.svals; P.Ws = d.Ws;
            P.heads = d.heads; P.runid = d.runid; P.starts = d.starts;
            P.defer = d.defer; P.dpos = d.dpos; P.dlist = d.dlist; P.keep = d.keep; P.seq = d.seq;
            P.dirty = d.dirty; P.dirty_cap = kDynDirtyCap; P.ctr = d.ctr;
            if (world) {
                P.wpts = world->pts; P.wperm = world->perm;
                std::memcpy(P.wrot, world->state->rot, sizeof(P.wrot));
                std::memcpy(P.wpos, world->state->pos, sizeof(P.wpos));
                std::memcpy(P.R_LI, c->params.R_LI, sizeof(P.R_LI));
                std::memcpy(P.t_LI, c->params.t_LI, sizeof(P.t_LI));
            }
            P.bigs = d.dlist;  // (dlist is free from the sort until k_add_finish)
            P.dlist_u = d.dpos; P.klist = d.apos;  // (dpos: free once k_scan_boxes has read the sorted keys)
            if (downsample && !wide) {  // (dlist / dpos are free until k_add_box)
                P.keys32 = d.dlist; P.skeys32 = d.dpos; P.skeys_w = d.skeys;
            }
            // k_add_prep refuses an out-of-range batch (ctr[kDynError] bit 0): the
            // passes that change the map (k_add_box, k_add_seq, k_add_append) then
            // do nothing, so the one read-back at the end decides
            rc = launch_add_prep(P, c->stream);
            if (rc) return rc;
            if (downsample) {
                if (P.keys32) rc = sort_u32(c, P.keys32, P.skeys32, d.iota, d.svals, n, 30);
                else rc = sort_u64(c, d.keys, d.skeys, d.iota, d.svals, n);
                if (!rc) rc = dyn_scan_ready(c, n);
                if (!rc) rc = launch_scan_boxes(d.scan, P, c->stream);
                if (!rc) rc = launch_add_group(P, c->stream);
            }
            if (!rc) rc = launch_add_finish(P, d.all, d.alive, c->stream);
            if (!rc && fused) {  // the merged rebuild on the device counts (kDynR*: its flags, runs, size)
                unsigned long long* rctr = d.ctr + (kDynRErr - kDynError);  // (rctr + kDynError = ctr + kDynRErr)
                const float inv = 1.0f / c->gh;
                rc = launch_dyn_newsort(d.all + 4 * g0, d.alive + g0, m_ub, c->gorg, inv, d.skeys, d.svals, rctr,
                                        c->stream, d.ctr + kDynAdded, d.ctr + kDynRErr);
                if (!rc) rc = launch_scan_flags(d.scan, c->gpts, na_old, d.alive, d.runid, c->stream, c->gslots, table);
                DynMergeParams M{};
                M.gpts = c->gpts; M.na_old = na_old; M.rank = d.runid; M.alive = d.alive;
                M.nkeys = d.skeys; M.nidx = d.svals; M.m = m_ub; M.g0 = g0; M.all = d.all;
                M.out = d.gpts_alt; M.okeys = d.keys; M.na = na_ub;
                std::memcpy(M.org, c->gorg, sizeof(M.org));
                M.inv = inv; M.ctr = rctr;
                M.dm = d.ctr + kDynAdded; M.dna = d.ctr + kDynRNa;
                if (!rc) rc = launch_dyn_merge(M, c->stream);
                if (!rc) rc = launch_scan_runs(d.scan, d.keys, na_ub, d.starts, d.ctr + kDynRRuns, c->stream,
                                               d.ctr + kDynRNa);
                if (!rc) rc = launch_dyn_slots(d.keys, d.starts, cell_bound, c->gslots, log2, c->stream,
                                               d.ctr + kDynRRuns, d.ctr + kDynRErr);
            }
            if (rc) return rc;
            HIP_TRY(hipMemcpyAsync(h, d.ctr, sizeof(h), hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            if (fused && (h[kDynError] & (1ull | 32ull | 64ull))) {
                // the fused pass refilled the table from an unchanged point set, hashed
                // with its bound's log2 (not c->glog2): rebuild it as the grid's own
                // before returning or before the 64-bit-key redo reads it (bit 32)
                const int rrc = dyn_rebuild(c);
                if (rrc) return rrc;
            }
            if (h[kDynError] & 1ull) return LIVO_E_RANGE;  // nothing changed
            if (h[kDynError] & 64ull) return LIVO_E_HIP;   // a scan's look-back gave up (nothing changed)
            if (!(h[kDynError] & 32ull) || wide) break;
            d.wide_redos++;
        }
        // k_add_prep checked the range of every box the later passes read, so
        // the group / sequential passes cannot fail once the map is modified
        if (h[kDynError]) {
            if (fused) (void)dyn_rebuild(c);
            return LIVO_E_HIP;
        }
        const int64_t added = (int64_t)h[kDynAdded];
        st.events = (int64_t)h[kDynEvents];
        st.deleted = (int64_t)h[kDynDeleted];
        st.ambiguous = (int64_t)h[kDynAmbig];
        st.deferred = downsample ? (int64_t)h[kDynDeferred] : 0;
        st.added = added;
        d.n_ids += added;
        d.n_alive += added - st.deleted;
        const uint32_t am = (uint32_t)h[kDynAbsMax];
        float amf;
        std::memcpy(&amf, &am, 4);
        d.cmax = std::max(d.cmax, amf);
        if (fused && h[kDynRErr] == 0 && (int64_t)h[kDynRNa] == d.n_alive && d.n_ids - g0 <= m_ub) {
            std::swap(c->gpts, d.gpts_alt);
            std::swap(d.gpts_cap, d.gpts_alt_cap);
            c->glog2 = log2;
            c->map_points = d.n_alive;
            c->geps = (float)(32.0 * std::ldexp(1.0, -24) * (double)d.cmax + 1e-7);
            c->grid_bytes = table * (int64_t)sizeof(GridSlot) + d.gpts_cap * 16;
            for (auto& sc : c->scans) sc.searched = false;  // cached neighbours refer to the old map
            d.grid_ids = d.n_ids;
            d.cells = (int64_t)h[kDynRRuns];
            d.rebuilds_merged++;
            d.rebuilds_fused++;
            rc = dyn_runs_update(c);
        } else {
            rc = dyn_rebuild(c);  // (c->gpts untouched by the fused pass)
        }
        if (rc) return rc;
    }
    st.map_points = d.n_alive;
    d.last = st;
    if (out) *out = st;
    return LIVO_OK;
}

// map_incremental with USE_ikdtree (laser_mapping.cpp:343-345, 383-384): every
// point to the world frame at the state, then Add_Points(feats_down_world, true)
// with downsample_size = filter_size_map_min (set_downsample_param, :138).
static int map_incremental_ikd(livo_ctx* c, int32_t id, const livo_state* state, double fs, uint8_t* cat,
                               int64_t counts[2]) {
    if (!c->has_map) return LIVO_E_NOMAP;
    ScanBuf* s = get_scan(c, id);
    if (!s) return LIVO_E_NOSCAN;
    if (set_device(c)) return LIVO_E_HIP;
    const int64_t N = s->n;
    if (counts) counts[0] = counts[1] = 0;
    int rc = dyn_activate(c);
    if (!rc) rc = dyn_add_scratch(c, std::max<int64_t>(N, 1));
    if (rc) return rc;
    // (feats_down_world: k_add_prep takes the points to the world frame, the state in its arguments)
    const DynWorldIn world{s->pts, s->d_perm, state};
    livo_map_add_stats st{};
    rc = dyn_add(c, N, (float)fs, true, &st, &world);
    if (rc) return rc;
    if (cat && N > 0) std::memset(cat, 1, (size_t)N);  // every point is handed to Add_Points
    if (counts) {
        counts[0] = st.events;
        counts[1] = st.deleted;
    }
    return LIVO_OK;
}

extern "C" {

int livo_abi_version(void) { return LIVO_ABI_VERSION; }

const char* livo_error_string(int code) {
    switch (code) {
        case LIVO_OK: return "ok";
        case LIVO_E_INVALID: return "invalid argument";
        case LIVO_E_HIP: return "HIP runtime error (no usable GPU or launch failure)";
        case LIVO_E_NOMAP: return "map not built";
        case LIVO_E_NOSCAN: return "unknown scan id";
        case LIVO_E_OOM: return "device allocation failed";
        case LIVO_E_RANGE: return "size out of supported range";
        case LIVO_E_CAPACITY: return "capacity exceeded";
        case LIVO_E_BUSY: return "batches in flight (collect them with livo_iekf_update_batch_wait first)";
        default: return "unknown error";
    }
}

int livo_params_default(livo_params* p) {
    if (!p) return LIVO_E_INVALID;
    std::memset(p, 0, sizeof(*p));
    p->laser_point_cov = 0.001;
    p->R_LI[0] = p->R_LI[4] = p->R_LI[8] = 1.0;
    p->max_residual = 2.0;
    p->plane_threshold = 0.1f;
    p->max_nn_sqdist = 5.0f;
    p->max_iterations = 4;
    p->flags = 0;
    return LIVO_OK;
}

int livo_ctx_create(int device, const livo_params* p, livo_ctx** out) {
    if (!out) return LIVO_E_INVALID;
    *out = nullptr;
    livo_params def;
    livo_params_default(&def);
    if (p && !params_valid(p)) return LIVO_E_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return LIVO_E_HIP;
    if (device < 0 || device >= ndev) return LIVO_E_INVALID;
    livo_ctx* c = new (std::nothrow) livo_ctx();
    if (!c) return LIVO_E_OOM;
    c->device = device;
    c->params = p ? *p : def;
    if (const char* env = std::getenv("LIVO_STREAM_GROUPS")) {  // tuning knob
        const int v = std::atoi(env);
        if (v >= 1 && v <= kMaxGroups) c->groups = v;
    }
    if (const char* env = std::getenv("LIVO_LEAF_SIZE")) {  // tuning knob
        const int v = std::atoi(env);
        if (v >= 2 && v <= 256) c->leaf_size = v;
    }
    if (const char* env = std::getenv("LIVO_FUSED")) c->fused = std::atoi(env) != 0;
    if (const char* env = std::getenv("LIVO_KNN_KIND"))
        c->knn_kind = std::strcmp(env, "leaf") == 0 ? 0 : std::strcmp(env, "grid") == 0 ? 1 : 2;
    if (const char* env = std::getenv("LIVO_VRUNS")) c->vruns = std::atoi(env) != 0;
    if (const char* env = std::getenv("LIVO_LANE_STREAMS")) c->lane_own_streams = std::strcmp(env, "own") == 0;
    if (const char* env = std::getenv("LIVO_BRUNS")) c->bruns = std::atoi(env) != 0;
    if (const char* env = std::getenv("LIVO_BR_HA")) {
        const float v = (float)std::atof(env);
        if (v > 0.2f && v < 20.f) c->br_ha = v;
    }
    if (const char* env = std::getenv("LIVO_BR_R")) {
        const float v = (float)std::atof(env);
        if (v > 0.5f && v < 20.f) c->br_r = v;
    }
    if (const char* env = std::getenv("LIVO_LANE_SERIAL")) c->lane_serial = std::atoi(env) != 0;
    if (const char* env = std::getenv("LIVO_LANE_ZC")) c->lane_zc = std::atoi(env) != 0;
    if (const char* env = std::getenv("LIVO_SYNC_ZC")) c->sync_zc = std::atoi(env) != 0;
    if (const char* env = std::getenv("LIVO_SLOT_WB")) c->slot_wb = std::atoi(env) != 0;
    if (const char* env = std::getenv("LIVO_XCD_CHUNK")) c->xcd_chunk = std::max(0, std::atoi(env));  // tuning knob
    if (const char* env = std::getenv("LIVO_GRID_PPC")) {  // tuning knob
        const float v = (float)std::atof(env);
        if (v > 0.f) c->grid_ppc = v;
    }
    if (const char* env = std::getenv("LIVO_GRID_CELL")) {
        const float v = (float)std::atof(env);
        if (v > 0.f) c->grid_cell = v;
    }
    if (set_device(c) || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) != hipSuccess || create_group_streams(c)) {
        delete c;
        return LIVO_E_HIP;
    }
    *out = c;
    return LIVO_OK;
}

int livo_ctx_destroy(livo_ctx* c) {
    if (!c) return LIVO_E_INVALID;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (BatchLane& B : c->lane) {  // batches never collected: let them finish
        for (int k = 0; k < kMaxGroups && B.owned; k++)
            if (B.st[k]) (void)hipStreamSynchronize(B.st[k]);
    }
    for (int k = 0; k < kMaxGroups - 1; k++)
        if (c->xstream[k]) (void)hipStreamSynchronize(c->xstream[k]);
    if (c->up_stream) (void)hipStreamSynchronize(c->up_stream);
    if (c->cp_stream) (void)hipStreamSynchronize(c->cp_stream);
    for (int k = 0; k < 2; k++) {
        if (c->bsrc[k]) (void)hipFree(c->bsrc[k]);
        if (c->bsrc_copied[k]) (void)hipEventDestroy(c->bsrc_copied[k]);
        if (c->bsrc_free[k]) (void)hipEventDestroy(c->bsrc_free[k]);
    }
    if (c->cp_stream) (void)hipStreamDestroy(c->cp_stream);
    for (auto& s : c->scans) free_scan_buf(s);
    for (auto& s : c->spare) free_scan_buf(s);
    if (c->up_tmp) (void)hipFree(c->up_tmp);
    if (c->aup_tmp) (void)hipFree(c->aup_tmp);
    if (c->aup_prim) (void)hipFree(c->aup_prim);
    for (auto& P : c->pin) {
        if (P.h) (void)hipHostFree(P.h);
        if (P.copied) (void)hipEventDestroy(P.copied);
    }
    if (c->up_stream) (void)hipStreamDestroy(c->up_stream);
    ivox_free(c->iv);
    dyn_free(c->dyn);
    if (c->fe_buf) (void)hipFree(c->fe_buf);
    if (c->prim_tmp) (void)hipFree(c->prim_tmp);
    if (c->vio_buf) (void)hipFree(c->vio_buf);
    dev_free(c->nodes);
    dev_free(c->lnodes);
    dev_free(c->lpts);
    dev_free(c->gslots);
    dev_free(c->gpts);
    dev_free(c->vslots);
    dev_free(c->vpts);
    dev_free(c->bslots);
    dev_free(c->bpts);
    dev_free(c->d_replay_count);
    dev_free(c->d_replay_total);
    dev_free(c->d_replay_list);
    dev_free(c->d_replay_count2);
    dev_free(c->d_replay_list2);
    dev_free(c->d_slots);
    dev_free(c->d_jobs);
    if (c->h_slots) (void)hipHostFree(c->h_slots);
    if (c->h_jobs) (void)hipHostFree(c->h_jobs);
    for (BatchLane& B : c->lane) {
        dev_free(B.d_lm);
        if (B.h_lm) (void)hipHostFree(B.h_lm);
        if (B.owned)
            for (int k = 0; k < kMaxGroups; k++)
                if (B.st[k]) (void)hipStreamDestroy(B.st[k]);
        if (B.owned_fork && B.fork) (void)hipEventDestroy(B.fork);
        dev_free(B.d_ik);
        if (B.h_ik) (void)hipHostFree(B.h_ik);
        for (hipEvent_t e : B.done)
            if (e) (void)hipEventDestroy(e);
    }
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->events_ready) {
        for (auto& g : c->ev)
            for (auto& e : g) (void)hipEventDestroy(e);
        (void)hipEventDestroy(c->b_start);
        (void)hipEventDestroy(c->b_end[0]);
        (void)hipEventDestroy(c->b_end[1]);
    }
    for (int k = 0; k < kMaxGroups - 1; k++) {
        if (c->xstream[k]) (void)hipStreamSynchronize(c->xstream[k]);
        if (c->xjoin[k]) (void)hipEventDestroy(c->xjoin[k]);
        if (c->xstream[k]) (void)hipStreamDestroy(c->xstream[k]);
    }
    if (c->fork) (void)hipEventDestroy(c->fork);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return LIVO_OK;
}

int livo_ctx_set_params(livo_ctx* c, const livo_params* p) {
    if (!c || !params_valid(p)) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    c->params = *p;
    return LIVO_OK;
}

int livo_ctx_set_profiling(livo_ctx* c, int enable) {
    if (!c) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    if (set_device(c)) return LIVO_E_HIP;
    if (enable && !c->events_ready) {
        for (auto& g : c->ev)
            for (auto& e : g) HIP_TRY(hipEventCreate(&e));
        HIP_TRY(hipEventCreate(&c->b_start));
        HIP_TRY(hipEventCreate(&c->b_end[0]));
        HIP_TRY(hipEventCreate(&c->b_end[1]));
        c->events_ready = true;
    }
    c->profiling = enable < 0 ? 0 : (enable > 2 ? 2 : enable);
    c->b_prev = false;
    return LIVO_OK;
}

int livo_last_timings(livo_ctx* c, livo_timings* out) {
    if (!c || !out) return LIVO_E_INVALID;
    *out = c->last;
    return LIVO_OK;
}

#if LIVO_IDX_RUNS
// Index runs from n key-sorted entries (skeys; e2 / pt give each entry's grid
// position, as k_run_place): heads, run ids, run starts, lengths rounded up to
// 4, their exclusive scan (pstart) and the placed positions in *out (the
// padded total + kRunPad words, zero-filled), then the runs' hash slots
// (load factor <= 1/4).  plen / pstart: scratch of n + 1 words each.
static int build_index_runs(livo_ctx* c, int64_t n, const unsigned long long* skeys, const uint32_t* e2,
                            const uint32_t* pt, uint32_t* heads, uint32_t* runid, uint32_t* starts,
                            unsigned long long* nruns_dev, uint32_t* plen, uint32_t* pstart, RunWord** out,
                            GridSlot** slots, int* log2_out, int64_t* words) {
    int rc = launch_run_heads(skeys, n, heads, c->stream);
    if (!rc) rc = ivox_scan(c, heads, runid, n);
    if (!rc) rc = launch_dyn_runs(heads, runid, n, starts, nruns_dev, c->stream);
    unsigned long long runs = 0;
    if (!rc && hipMemcpyAsync(&runs, nruns_dev, 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess) rc = LIVO_E_HIP;
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
    if (rc) return rc;
    if (runs == 0) return LIVO_E_INVALID;
    rc = launch_run_plen(starts, (int64_t)runs, plen, c->stream);
    if (!rc) rc = ivox_scan(c, plen, pstart, (int64_t)runs);
    uint32_t tail[2] = {0u, 0u};
    if (!rc && hipMemcpyAsync(&tail[0], pstart + runs - 1, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        rc = LIVO_E_HIP;
    if (!rc && hipMemcpyAsync(&tail[1], plen + runs - 1, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        rc = LIVO_E_HIP;
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
    if (rc) return rc;
    const int64_t total = (int64_t)tail[0] + tail[1];  // (u32 lengths: the scan wraps beyond 2^32 words)
    if (total < n || total + kRunPad >= (int64_t)0xFFFFFFFFll) return LIVO_E_RANGE;
    if (dev_alloc(out, (size_t)(total + kRunPad))) return LIVO_E_OOM;
    rc = hipMemsetAsync(*out, 0, (size_t)(total + kRunPad) * sizeof(RunWord), c->stream) == hipSuccess ? LIVO_OK
                                                                                                         : LIVO_E_HIP;
    if (!rc) rc = launch_run_place(e2, pt, heads, runid, starts, pstart, n, *out, c->stream);
    int log2 = 4;
    while (((int64_t)1 << log2) < 4 * (int64_t)runs) log2++;
    const int64_t table = (int64_t)1 << log2;
    if (!rc && dev_alloc(slots, (size_t)table)) rc = LIVO_E_OOM;
    if (!rc) rc = launch_ivox_clear(*slots, table, c->stream);
    if (!rc) rc = launch_run_slots(skeys, starts, pstart, (int64_t)runs, *slots, log2, c->stream);
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
    if (rc) {
        dev_free(*out);
        dev_free(*slots);
        return rc;
    }
    *log2_out = log2;
    *words = total + kRunPad;
    return LIVO_OK;
}
#endif

// The cell runs of the static map's grid (livo_internal.h), built on the
// device: two stable radix sorts (rho2, then the run key) of the 27 M entries,
// the runs' heads and starts, and their hash table (load factor <= 1/4).
#if LIVO_IDX_RUNS
static int build_cell_runs_into(livo_ctx* c, const float* pts, int64_t M, GridSlot** slots, RunWord** idx,
                                int32_t* log2, int64_t* words);
static int build_cell_runs(livo_ctx* c, int64_t M) {
    int64_t words = 0;
    const int rc = build_cell_runs_into(c, c->gpts, M, &c->vslots, &c->vpts, &c->vlog2, &words);
    if (!rc && M > 0) c->grid_bytes += (int64_t)(((int64_t)1 << c->vlog2) * sizeof(GridSlot) + words * sizeof(RunWord));
    return rc;
}
// The cell runs of M grid-ordered points pts (the map's grid; on the incremental
// map also its delta grid): *slots / *idx replaced, run entries = positions in pts.
static int build_cell_runs_into(livo_ctx* c, const float* pts, int64_t M, GridSlot** slots, RunWord** idx,
                                int32_t* log2, int64_t* words) {
    dev_free(*slots);
    dev_free(*idx);
    if (M <= 0) return LIVO_OK;
#else
static int build_cell_runs(livo_ctx* c, int64_t M) {
    const float* pts = c->gpts;
    dev_free(c->vslots);
    dev_free(c->vpts);
    if (M <= 0) return LIVO_OK;
#endif
    const int64_t n = M * 27;
    if (n + 8 >= (int64_t)kRunPosLimit) return LIVO_E_RANGE;  // 31-bit run positions (kRunPos)
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t b4 = al((size_t)n * 4), b8 = al((size_t)n * 8);
    char* scr = nullptr;
    if (hipMalloc((void**)&scr, 7 * b4 + 2 * b8 + al(((size_t)n + 1) * 4) + 256) != hipSuccess) return LIVO_E_OOM;
    char* p = scr;
    uint32_t* rho = (uint32_t*)p; p += b4;
    uint32_t* iota = (uint32_t*)p; p += b4;
    uint32_t* srho = (uint32_t*)p; p += b4;
    uint32_t* e1 = (uint32_t*)p; p += b4;
    uint32_t* e2 = (uint32_t*)p; p += b4;
    uint32_t* heads = (uint32_t*)p; p += b4;
    uint32_t* runid = (uint32_t*)p; p += b4;
    unsigned long long* keys = (unsigned long long*)p; p += b8;
    unsigned long long* skeys = (unsigned long long*)p; p += b8;
    uint32_t* starts = (uint32_t*)p; p += al(((size_t)n + 1) * 4);
    unsigned long long* nruns = (unsigned long long*)p;
    int rc = LIVO_OK;
#if !LIVO_IDX_RUNS
    if (dev_alloc(&c->vpts, (size_t)(n + kRunPad) * kRunWords)) rc = LIVO_E_OOM;
#endif
    if (!rc) rc = launch_cr_rho(pts, n, c->gorg, c->gh, rho, iota, c->stream);
    if (!rc) {
        size_t tb = 0;
        rc = prim_sort_pairs_u32(nullptr, &tb, rho, srho, iota, e1, n, 32, c->stream);
        if (!rc) rc = ensure_prim(c, tb);
        tb = c->prim_bytes;
        if (!rc) rc = prim_sort_pairs_u32(c->prim_tmp, &tb, rho, srho, iota, e1, n, 32, c->stream);
    }
    if (!rc) rc = launch_cr_key(pts, e1, n, c->gorg, c->gh, keys, c->stream);
    if (!rc) rc = sort_u64(c, keys, skeys, e1, e2, n);
#if LIVO_IDX_RUNS
    // (rho, iota: dead after the sorts) the padded run lengths and their scan
    if (!rc) rc = build_index_runs(c, n, skeys, e2, nullptr, heads, runid, starts, nruns, rho, iota, idx, slots, log2,
                                   words);
    (void)hipFree(scr);
    return rc;
#else
    if (!rc) rc = launch_cr_fill(pts, e2, skeys, n, c->gorg, c->gh, c->vpts, heads, c->stream);
    if (!rc) rc = ivox_scan(c, heads, runid, n);
    if (!rc) rc = launch_dyn_runs(heads, runid, n, starts, nruns, c->stream);
    unsigned long long runs = 0;
    if (!rc && hipMemcpyAsync(&runs, nruns, 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess) rc = LIVO_E_HIP;
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
    int log2 = 4;
    while (((int64_t)1 << log2) < 4 * (int64_t)runs) log2++;
    const int64_t table = (int64_t)1 << log2;
    if (!rc && dev_alloc(&c->vslots, (size_t)table)) rc = LIVO_E_OOM;
    if (!rc) rc = launch_ivox_clear(c->vslots, table, c->stream);
    if (!rc) rc = launch_dyn_slots(skeys, starts, (int64_t)runs, c->vslots, log2, c->stream);
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
    (void)hipFree(scr);
    if (rc) {
        dev_free(c->vslots);
        dev_free(c->vpts);
        return rc;
    }
    c->vlog2 = log2;
    c->grid_bytes += (int64_t)(table * sizeof(GridSlot) + (size_t)(n + kRunPad) * 16);
    return LIVO_OK;
#endif
}

#if LIVO_IDX_RUNS
// The index ball runs, built in chunks of anchors (their x index in [x0, x1)),
// each chunk at most `cap` entries (LIVO_BR_CHUNK, default 2^29: ~26 GB of sort
// scratch), so the 32-bit sort indices and offsets of one chunk never wrap
// however many entries the map has (config 5's 10M map with 6 r5 balls passes
// 2^31).  A chunk is counted, placed behind the runs of the chunks before it in
// one run array (every run starts on a 4-word boundary), and its runs recorded
// as {key, start / 4, count}; the hash table then takes every record, so a slot's
// start addresses 2^34 words.  The runs' contents and order are those of the
// one-pass build.
static int build_ball_runs_idx(livo_ctx* c, int64_t M, float r5, float bh, float brmax, double ext) {
    int64_t cap = (int64_t)1 << 29;
    if (const char* env = std::getenv("LIVO_BR_CHUNK")) cap = std::max<int64_t>(1 << 16, std::atoll(env));
    cap = std::min<int64_t>(cap, ((int64_t)1 << 31) - 64);
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    uint32_t* cnt = nullptr;
    uint32_t* off = nullptr;
    unsigned long long* tot = nullptr;
    if (dev_alloc(&cnt, (size_t)M) || dev_alloc(&off, (size_t)M) || dev_alloc(&tot, 1)) {
        dev_free(cnt);
        dev_free(off);
        dev_free(tot);
        return LIVO_E_OOM;
    }
    // entries of the anchors with x index in [x0, x1) (a count pass over the map)
    auto count = [&](int x0, int x1, unsigned long long* n_out) -> int {
        int rc = hipMemsetAsync(tot, 0, 8, c->stream) == hipSuccess ? LIVO_OK : LIVO_E_HIP;
        if (!rc) rc = launch_br_count(c->gpts, M, c->gorg, bh, brmax, cnt, tot, c->stream, x0, x1);
        if (!rc && hipMemcpyAsync(n_out, tot, 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess) rc = LIVO_E_HIP;
        if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
        return rc;
    };
    // the anchors' x range: the map spans [gorg, gorg + ext] on every axis (the
    // grid's origin is its minimum corner), a point's anchors lie within brmax
    const int xlo = (int)std::floor(-(double)brmax / (double)bh) - 2;
    const int xhi = (int)std::floor((ext + (double)brmax) / (double)bh) + 3;  // exclusive
    struct Chunk {
        int x0, x1;
        int64_t n;
    };
    std::vector<Chunk> chunks, todo{{xlo, xhi, -1}};
    int64_t total_entries = 0, max_n = 0;
    int rc = LIVO_OK;
    while (!todo.empty() && !rc) {  // bisect the x range until every chunk fits
        Chunk ch = todo.back();
        todo.pop_back();
        unsigned long long n64 = 0;
        rc = count(ch.x0, ch.x1, &n64);
        if (rc) break;
        if ((int64_t)n64 > cap && ch.x1 - ch.x0 > 1) {
            const int mid = ch.x0 + (ch.x1 - ch.x0) / 2;
            todo.push_back({mid, ch.x1, -1});
            todo.push_back({ch.x0, mid, -1});
            continue;
        }
        if ((int64_t)n64 > cap) rc = LIVO_E_RANGE;  // one anchor column beyond the cap
        if (n64 == 0) continue;
        ch.n = (int64_t)n64;
        chunks.push_back(ch);
        total_entries += ch.n;
        max_n = std::max(max_n, ch.n);
    }
    dev_free(tot);
    if (rc || total_entries == 0) {
        dev_free(cnt);
        dev_free(off);
        return rc;
    }
    // the run array: the entries plus the padding of every run to 4 words (grown if short)
    int64_t words_cap = total_entries + total_entries / 8 + 4096 + kRunPad;
    if (dev_alloc(&c->bpts, (size_t)words_cap) ||
        hipMemsetAsync(c->bpts, 0, (size_t)words_cap * sizeof(RunWord), c->stream) != hipSuccess) {
        dev_free(cnt);
        dev_free(off);
        dev_free(c->bpts);
        return LIVO_E_OOM;
    }
    const int64_t n = max_n;
    const size_t b4 = al((size_t)n * 4), b8 = al((size_t)n * 8);
    char* scr = nullptr;
    if (hipMalloc((void**)&scr, 7 * b4 + 3 * b8 + 2 * al(((size_t)n + 1) * 4) + 256) != hipSuccess) {
        dev_free(cnt);
        dev_free(off);
        dev_free(c->bpts);
        return LIVO_E_OOM;
    }
    char* p = scr;
    uint32_t* rho = (uint32_t*)p; p += b4;
    uint32_t* iota = (uint32_t*)p; p += b4;
    uint32_t* srho = (uint32_t*)p; p += b4;
    uint32_t* e1 = (uint32_t*)p; p += b4;
    uint32_t* e2 = (uint32_t*)p; p += b4;
    uint32_t* pt = (uint32_t*)p; p += b4;
    uint32_t* heads = (uint32_t*)p; p += b4;
    unsigned long long* keys = (unsigned long long*)p; p += b8;
    unsigned long long* key1 = (unsigned long long*)p; p += b8;
    unsigned long long* skeys = (unsigned long long*)p; p += b8;
    uint32_t* starts = (uint32_t*)p; p += al(((size_t)n + 1) * 4);
    uint32_t* plen = (uint32_t*)p; p += al(((size_t)n + 1) * 4);
    unsigned long long* nruns_dev = (unsigned long long*)p;
    uint32_t* runid = rho;    // (rho is dead after the first sort)
    uint32_t* pstart = srho;  // (srho too)
    GridSlot* trip = nullptr;
    int64_t trip_cap = 0, runs_total = 0, base = 0;
    for (const Chunk& ch : chunks) {
        const int64_t nc = ch.n;
        rc = launch_br_count(c->gpts, M, c->gorg, bh, brmax, cnt, nruns_dev, c->stream, ch.x0, ch.x1);
        if (!rc) rc = ivox_scan(c, cnt, off, M);
        if (!rc) rc = launch_br_emit(c->gpts, M, c->gorg, bh, brmax, off, rho, keys, pt, iota, c->stream, ch.x0, ch.x1);
        if (!rc) {
            size_t tb = 0;
            rc = prim_sort_pairs_u32(nullptr, &tb, rho, srho, iota, e1, nc, 32, c->stream);
            if (!rc) rc = ensure_prim(c, tb);
            tb = c->prim_bytes;
            if (!rc) rc = prim_sort_pairs_u32(c->prim_tmp, &tb, rho, srho, iota, e1, nc, 32, c->stream);
        }
        if (!rc) rc = launch_br_gather_keys(keys, e1, nc, key1, c->stream);
        if (!rc) rc = sort_u64(c, key1, skeys, e1, e2, nc);
        // runs: heads, starts, lengths padded to 4 and their scan
        if (!rc) rc = launch_run_heads(skeys, nc, heads, c->stream);
        if (!rc) rc = ivox_scan(c, heads, runid, nc);
        if (!rc && hipMemsetAsync(nruns_dev, 0, 8, c->stream) != hipSuccess) rc = LIVO_E_HIP;
        if (!rc) rc = launch_dyn_runs(heads, runid, nc, starts, nruns_dev, c->stream);
        unsigned long long runs = 0;
        if (!rc && hipMemcpyAsync(&runs, nruns_dev, 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess) rc = LIVO_E_HIP;
        if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
        if (rc) break;
        if (runs == 0) continue;
        rc = launch_run_plen(starts, (int64_t)runs, plen, c->stream);
        if (!rc) rc = ivox_scan(c, plen, pstart, (int64_t)runs);
        uint32_t tail[2] = {0u, 0u};
        if (!rc && (hipMemcpyAsync(&tail[0], pstart + runs - 1, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
                    hipMemcpyAsync(&tail[1], plen + runs - 1, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
                    hipStreamSynchronize(c->stream) != hipSuccess))
            rc = LIVO_E_HIP;
        if (rc) break;
        const int64_t words = (int64_t)tail[0] + tail[1];
        if (words < nc || words >= (int64_t)0xFFFFFFFFll) {
            rc = LIVO_E_RANGE;
            break;
        }
        if (base + words + kRunPad > words_cap) {  // more padding than reserved: grow the run array
            const int64_t ncap = (base + words + kRunPad) + (base + words) / 8;
            RunWord* nb = nullptr;
            if (dev_alloc(&nb, (size_t)ncap)) {
                rc = LIVO_E_OOM;
                break;
            }
            if (hipMemsetAsync(nb, 0, (size_t)ncap * sizeof(RunWord), c->stream) != hipSuccess ||
                hipMemcpyAsync(nb, c->bpts, (size_t)base * sizeof(RunWord), hipMemcpyDeviceToDevice, c->stream) !=
                    hipSuccess ||
                hipStreamSynchronize(c->stream) != hipSuccess)
                rc = LIVO_E_HIP;
            dev_free(c->bpts);
            c->bpts = nb;
            words_cap = ncap;
            if (rc) break;
        }
        if (runs_total + (int64_t)runs > trip_cap) {  // the run records (grown by doubling)
            const int64_t ncap = std::max<int64_t>(2 * trip_cap, runs_total + (int64_t)runs + 4096);
            GridSlot* nt = nullptr;
            if (dev_alloc(&nt, (size_t)ncap)) {
                rc = LIVO_E_OOM;
                break;
            }
            if (runs_total > 0 &&
                (hipMemcpyAsync(nt, trip, (size_t)runs_total * sizeof(GridSlot), hipMemcpyDeviceToDevice,
                                c->stream) != hipSuccess ||
                 hipStreamSynchronize(c->stream) != hipSuccess))
                rc = LIVO_E_HIP;
            dev_free(trip);
            trip = nt;
            trip_cap = ncap;
            if (rc) break;
        }
        rc = launch_run_place(e2, pt, heads, runid, starts, pstart, nc, c->bpts + base, c->stream);
        if (!rc) rc = launch_run_trip(skeys, starts, pstart, (int64_t)runs, (unsigned long long)base,
                                      trip + runs_total, c->stream);
        if (rc) break;
        base += words;
        runs_total += (int64_t)runs;
    }
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
    (void)hipFree(scr);
    dev_free(cnt);
    dev_free(off);
    if (!rc && (base >> 2) >= ((int64_t)1 << 32)) rc = LIVO_E_RANGE;  // start / 4 in 32 bits
    int log2 = 4;
    while (((int64_t)1 << log2) < 4 * runs_total) log2++;
    if (!rc && runs_total > 0) {
        const int64_t table = (int64_t)1 << log2;
        if (dev_alloc(&c->bslots, (size_t)table)) rc = LIVO_E_OOM;
        if (!rc) rc = launch_ivox_clear(c->bslots, table, c->stream);
        if (!rc) rc = launch_trip_slots(trip, runs_total, c->bslots, log2, c->stream);
        if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
    }
    dev_free(trip);
    if (rc || runs_total == 0) {
        dev_free(c->bslots);
        dev_free(c->bpts);
        return rc;
    }
    c->blog2 = log2;
    c->bh = bh;
    c->brmax = brmax;
    c->br5 = r5;
    c->bentries = total_entries;
    c->bchunks = (int32_t)chunks.size();
    c->grid_bytes += (int64_t)(((int64_t)1 << log2) * sizeof(GridSlot) + words_cap * sizeof(RunWord));
    return LIVO_OK;
}
#endif

// The ball runs of the static map (livo_internal.h KnnParams::bslots), built on
// the device: every grid point emits one entry per anchor cell (edge bh) whose
// centre lies within brmax (k_br_count, a scan, k_br_emit); a stable radix sort
// by rho2, a gather of the anchor keys and a stable sort by key leave each
// anchor's run contiguous and sorted by rho2; heads, starts and the hash table
// as for the cell runs.  r5: the map's median 5-NN distance (sample_knn_radius).
static int build_ball_runs(livo_ctx* c, int64_t M, float r5, double ext) {
    dev_free(c->bslots);
    dev_free(c->bpts);
    c->bentries = 0;
    if (M <= 0 || !(r5 > 0.f)) return LIVO_OK;
    const float bh = std::max(c->br_ha * r5, 1e-3f);
    const float brmax = 0.8660254f * bh + c->br_r * r5;
    // anchor keys are 21-bit per axis (grid_key, kGridBias = 2^20) and the device
    // clamps a query's anchor to +-(kGridBias - 8): a map whose extent (+ the
    // ball radius) spans that many anchors keeps the cell runs only, rather
    // than letting keys alias into a run not sorted about its own anchor
    if ((ext + 2.0 * (double)brmax) / (double)bh + 4.0 >= (double)(kGridBias - 8)) return LIVO_OK;
#if LIVO_IDX_RUNS
    return build_ball_runs_idx(c, M, r5, bh, brmax, ext);
#endif
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    uint32_t* cnt = nullptr;
    uint32_t* off = nullptr;
    unsigned long long* tot = nullptr;
    if (dev_alloc(&cnt, (size_t)M) || dev_alloc(&off, (size_t)M) || dev_alloc(&tot, 1)) {
        dev_free(cnt);
        dev_free(off);
        dev_free(tot);
        return LIVO_E_OOM;
    }
    int rc = hipMemsetAsync(tot, 0, 8, c->stream) == hipSuccess ? LIVO_OK : LIVO_E_HIP;
    if (!rc) rc = launch_br_count(c->gpts, M, c->gorg, bh, brmax, cnt, tot, c->stream);
    if (!rc) rc = ivox_scan(c, cnt, off, M);
    unsigned long long n64 = 0;
    if (!rc && hipMemcpyAsync(&n64, tot, 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess) rc = LIVO_E_HIP;
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
    dev_free(cnt);
    dev_free(tot);
    // 31-bit run positions (kRunPos) and u32 offsets; a map too dense for the ball keeps the cell runs
    if (rc || n64 == 0 || (int64_t)n64 + 8 >= (int64_t)kRunPosLimit) {
        dev_free(off);
        return rc;
    }
    const int64_t n = (int64_t)n64;
    const size_t b4 = al((size_t)n * 4), b8 = al((size_t)n * 8);
    char* scr = nullptr;
    if (hipMalloc((void**)&scr, 7 * b4 + 3 * b8 + al(((size_t)n + 1) * 4) + 256) != hipSuccess) {
        dev_free(off);
        return LIVO_E_OOM;
    }
    char* p = scr;
    uint32_t* rho = (uint32_t*)p; p += b4;
    uint32_t* iota = (uint32_t*)p; p += b4;
    uint32_t* srho = (uint32_t*)p; p += b4;
    uint32_t* e1 = (uint32_t*)p; p += b4;
    uint32_t* e2 = (uint32_t*)p; p += b4;
    uint32_t* pt = (uint32_t*)p; p += b4;
    uint32_t* heads = (uint32_t*)p; p += b4;
    unsigned long long* keys = (unsigned long long*)p; p += b8;
    unsigned long long* key1 = (unsigned long long*)p; p += b8;
    unsigned long long* skeys = (unsigned long long*)p; p += b8;
    uint32_t* starts = (uint32_t*)p; p += al(((size_t)n + 1) * 4);
    unsigned long long* nruns = (unsigned long long*)p;
    uint32_t* runid = rho;  // (rho is dead after the first sort)
#if !LIVO_IDX_RUNS
    if (dev_alloc(&c->bpts, (size_t)(n + kRunPad) * kRunWords)) rc = LIVO_E_OOM;
#endif
    if (!rc) rc = launch_br_emit(c->gpts, M, c->gorg, bh, brmax, off, rho, keys, pt, iota, c->stream);
    if (!rc) {
        size_t tb = 0;
        rc = prim_sort_pairs_u32(nullptr, &tb, rho, srho, iota, e1, n, 32, c->stream);
        if (!rc) rc = ensure_prim(c, tb);
        tb = c->prim_bytes;
        if (!rc) rc = prim_sort_pairs_u32(c->prim_tmp, &tb, rho, srho, iota, e1, n, 32, c->stream);
    }
    if (!rc) rc = launch_br_gather_keys(keys, e1, n, key1, c->stream);
    if (!rc) rc = sort_u64(c, key1, skeys, e1, e2, n);
#if LIVO_IDX_RUNS
    int64_t words = 0;
    // (srho, iota: dead after the sorts) the padded run lengths and their scan
    if (!rc) rc = build_index_runs(c, n, skeys, e2, pt, heads, runid, starts, nruns, srho, iota, &c->bpts,
                                   &c->bslots, &c->blog2, &words);
    (void)hipFree(scr);
    dev_free(off);
    if (rc) return rc;
    c->bh = bh;
    c->brmax = brmax;
    c->br5 = r5;
    c->bentries = n;
    c->bchunks = 1;
    c->grid_bytes += (int64_t)(((int64_t)1 << c->blog2) * sizeof(GridSlot) + words * sizeof(RunWord));
    return LIVO_OK;
#else
    if (!rc) rc = launch_br_fill(c->gpts, pt, e2, skeys, n, c->bpts, heads, c->stream);
    if (!rc) rc = ivox_scan(c, heads, runid, n);
    if (!rc) rc = launch_dyn_runs(heads, runid, n, starts, nruns, c->stream);
    unsigned long long runs = 0;
    if (!rc && hipMemcpyAsync(&runs, nruns, 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess) rc = LIVO_E_HIP;
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
    int log2 = 4;
    while (((int64_t)1 << log2) < 4 * (int64_t)runs) log2++;
    const int64_t table = (int64_t)1 << log2;
    if (!rc && dev_alloc(&c->bslots, (size_t)table)) rc = LIVO_E_OOM;
    if (!rc) rc = launch_ivox_clear(c->bslots, table, c->stream);
    if (!rc) rc = launch_dyn_slots(skeys, starts, (int64_t)runs, c->bslots, log2, c->stream);
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = LIVO_E_HIP;
    (void)hipFree(scr);
    dev_free(off);
    if (rc) {
        dev_free(c->bslots);
        dev_free(c->bpts);
        return rc;
    }
    c->blog2 = log2;
    c->bh = bh;
    c->brmax = brmax;
    c->br5 = r5;
    c->bentries = n;
    c->bchunks = 1;
    c->grid_bytes += (int64_t)(table * sizeof(GridSlot) + (size_t)(n + kRunPad) * 16);
    return LIVO_OK;
#endif
}

int livo_map_build(livo_ctx* c, const float* xyz, int64_t M, int64_t stride_bytes) {
    if (!c || M < 0 || (M > 0 && !xyz)) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    if (set_device(c)) return LIVO_E_HIP;
    HostMap hm;
    int rc = build_host_map(xyz, M, stride_bytes, &hm);
    if (rc) return rc;
    HostLeafMap lm;
    HostGridMap gm;
    // (a map of more than ~79M points keeps the cell walk: run positions are 31-bit)
    const bool vr = c->knn_kind == 2 && c->vruns && M * 27 + 8 < (int64_t)kRunPosLimit;
    rc = c->knn_kind >= 1 ? build_grid_map(xyz, M, stride_bytes, c->grid_cell, &gm, c->grid_ppc > 0.f ? c->grid_ppc
                                                                                    : (vr ? -kVrunPpc : 0.f))
                          : build_leaf_map(xyz, M, stride_bytes, c->leaf_size, &lm);
    if (rc) {
        free_host_map(&hm);
        free_grid_map(&gm);
        return rc;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int k = 0; k < kMaxGroups - 1; k++) HIP_TRY(hipStreamSynchronize(c->xstream[k]));
    dev_free(c->nodes);
    dev_free(c->lnodes);
    dev_free(c->lpts);
    dev_free(c->gslots);
    dev_free(c->gpts);
    dev_free(c->vslots);
    dev_free(c->vpts);
    dev_free(c->bslots);
    dev_free(c->bpts);
    c->nodes = nullptr;
    c->lnodes = nullptr;
    c->lpts = nullptr;
    c->gslots = nullptr;
    c->gpts = nullptr;
    c->leaf_bytes = c->grid_bytes = 0;
    c->has_map = false;
    c->dyn.active = false;  // a new static map (the incremental buffers are kept for reuse)
    c->dyn.min_gh = c->dyn.max_gh = 0.f;
    c->dyn.runs = false;
    c->dyn.d_n = 0;
    c->dyn.n_ids = c->dyn.n_alive = 0;
    c->dyn.last = livo_map_add_stats{};
    const size_t bytes = (size_t)(hm.num_slots + 1) * sizeof(MapNode);
    const size_t ppb = (size_t)(M + 3) * 4 * sizeof(float);  // chunk padding
    hipError_t e = hipSuccess;
    bool oom = hipMalloc((void**)&c->nodes, bytes) != hipSuccess;
    if (c->knn_kind >= 1) {
        const size_t gsb = ((size_t)1 << gm.log2_slots) * sizeof(GridSlot);
        oom = oom || hipMalloc((void**)&c->gslots, gsb) != hipSuccess || hipMalloc((void**)&c->gpts, ppb) != hipSuccess;
        if (!oom) e = hipMemcpy(c->gslots, gm.slots, gsb, hipMemcpyHostToDevice);
        if (!oom && e == hipSuccess) e = hipMemcpy(c->gpts, gm.pts, ppb, hipMemcpyHostToDevice);
        c->grid_bytes = (int64_t)(gsb + ppb);
        std::memcpy(c->gorg, gm.org, sizeof(c->gorg));
        c->gh = gm.h;
        c->glog2 = gm.log2_slots;
        // slack for float rounding in the cell assignment (host) and cell bounds (device)
        c->geps = (float)(32.0 * std::ldexp(1.0, -24) * (double)gm.cmax + 1e-7);
        c->gcmax = gm.cmax;
    } else {
        const size_t lnb = (size_t)std::max<int64_t>(((int64_t)1 << lm.depth) - 1, 1) * sizeof(LeafNode);
        oom = oom || hipMalloc((void**)&c->lnodes, lnb) != hipSuccess || hipMalloc((void**)&c->lpts, ppb) != hipSuccess;
        if (!oom) e = hipMemcpy(c->lnodes, lm.nodes, lnb, hipMemcpyHostToDevice);
        if (!oom && e == hipSuccess) e = hipMemcpy(c->lpts, lm.pts, ppb, hipMemcpyHostToDevice);
        c->leaf_depth = lm.depth;
        c->leaf_bytes = (int64_t)(lnb + ppb);
    }
    if (!oom && e == hipSuccess) e = hipMemcpy(c->nodes, hm.nodes, bytes, hipMemcpyHostToDevice);
    const float r5 = (vr && c->bruns && c->knn_kind >= 1) ? sample_knn_radius(gm, 8192) : 0.f;
    const double gext = gm.ext;
    free_host_map(&hm);
    free_leaf_map(&lm);
    free_grid_map(&gm);
    if (oom) return LIVO_E_OOM;
    if (e != hipSuccess) return LIVO_E_HIP;
    if (vr) {
        rc = build_cell_runs(c, M);
        if (rc) return rc;
        if (r5 > 0.f) {
            // the ball runs are a speed-up over the cell runs: a map they do not
            // fit (their scratch is ~68 B per entry, ~60 entries per point) keeps
            // the cell runs and builds; other errors still fail the build
            const int brc = build_ball_runs(c, M, r5, gext);
            if (brc == LIVO_E_OOM) {
                (void)hipGetLastError();
                dev_free(c->bslots);
                dev_free(c->bpts);
                c->bentries = 0;
            } else if (brc) {
                return brc;
            }
        }
    }
    c->map_points = M;
    c->map_slots = hm.num_slots;
    c->map_depth = hm.depth;
    c->has_map = true;
    for (auto& s : c->scans) s.searched = false;  // cached neighbours refer to the old map
    return LIVO_OK;
}

int livo_map_get_info(livo_ctx* c, livo_map_info* out) {
    if (!c || !out) return LIVO_E_INVALID;
    if (!c->has_map) return LIVO_E_NOMAP;
    out->num_points = c->map_points;
    out->depth = c->map_depth;
    out->ball_chunks = c->bslots ? c->bchunks : 0;
    out->ball_entries = c->bslots ? c->bentries : 0;
    out->num_slots = c->map_slots;
    out->device_bytes = (c->map_slots + 1) * (int64_t)sizeof(MapNode) + c->leaf_bytes + c->grid_bytes +
                        c->dyn.cap * 17;
    return LIVO_OK;
}

int livo_knn(livo_ctx* c, const float* q, int64_t n, int32_t k, int32_t* idx, float* d) {
    if (!c || n < 0 || k < 1 || k > kNN || (n > 0 && (!q || !idx || !d))) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    if (!c->has_map) return LIVO_E_NOMAP;
    if (n == 0) return LIVO_OK;
    if (n > (int64_t)0x7FFFFFFF - kBlock) return LIVO_E_RANGE;
    if (set_device(c)) return LIVO_E_HIP;
    int rc = ensure_slots(c, 1);
    if (rc) return rc;
    const size_t qb = (size_t)n * 4 * sizeof(float), rb = (size_t)n * sizeof(NNRec);
    rc = ensure_scratch(c, qb + rb + 256);
    if (rc) return rc;
    char* base = (char*)c->scratch;
    float* dq = (float*)base;
    NNRec* dr = (NNRec*)(base + ((qb + 255) & ~(size_t)255));
    std::vector<float> hq((size_t)n * 4);
    for (int64_t i = 0; i < n; i++) {
        hq[4 * i] = q[3 * i]; hq[4 * i + 1] = q[3 * i + 1]; hq[4 * i + 2] = q[3 * i + 2]; hq[4 * i + 3] = 0.f;
    }
    IekfSlot zero{};
    std::memset(&zero, 0, sizeof(zero));
    c->h_slots[0] = zero;
    HsJob& j = c->h_jobs[0];
    j = HsJob{};
    j.pts = dq; j.nn = dr; j.slot = c->d_slots; j.n = (int32_t)n; j.nblk = 0;
    HIP_TRY(hipMemcpyAsync(dq, hq.data(), qb, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_slots, c->h_slots, sizeof(IekfSlot), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_jobs, c->h_jobs, sizeof(HsJob), hipMemcpyHostToDevice, c->stream));
    rc = ensure_replay(c, n);
    if (rc) return rc;
    KnnParams kp = make_knn_params(c);
    kp.force = 1;
    kp.identity = 1;
    rc = knn_pass(kp, 1, n, c->stream);
    if (rc) return rc;
    std::vector<NNRec> hr((size_t)n);
    HIP_TRY(hipMemcpyAsync(hr.data(), dr, rb, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int64_t i = 0; i < n; i++)
        for (int t = 0; t < k; t++) {
            idx[i * k + t] = hr[i].idx[t];
            d[i * k + t] = hr[i].p[t][3];
        }
    return LIVO_OK;
}

static int32_t register_scan(livo_ctx* c, const ScanBuf& s) {
    int32_t id = -1;
    for (size_t i = 0; i < c->scans.size(); i++)
        if (!c->scans[i].used) { id = (int32_t)i; break; }
    if (id < 0) {
        id = (int32_t)c->scans.size();
        c->scans.push_back(s);
    } else {
        c->scans[id] = s;
    }
    return id;
}

// The device buffers of a scan of N points: a released scan's when one fits
// (capacity N .. 2N + 4096), else fresh allocations sized for N.
// Released scan buffers are kept for reuse up to a byte budget (LIVO_SPARE_MB,
// default 8192): a hipFree synchronises the whole device, so freeing one while
// a farm's batches and uploads are in flight stalled the pipeline (a 12.9 ms
// upload call; the farm with uploads at 5.4k instead of 12.4k updates/s).
static size_t scan_buf_bytes(int64_t cap) {
    const int64_t cblk = std::max<int64_t>(1, (cap + kBlock * kPtsPerThread - 1) / (kBlock * kPtsPerThread));
    return (size_t)cap * (16 + sizeof(NNRec) + 4 + 4 + 16 + 1) + partial_doubles(cap) * 8 +
           (size_t)cblk * (kIkFewRows * 13 * 8 + 4);
}
static size_t spare_budget() {
    static const size_t b = [] {
        const char* e = std::getenv("LIVO_SPARE_MB");
        const long long mb = e ? std::atoll(e) : 8192;
        return (size_t)std::max(0LL, mb) << 20;
    }();
    return b;
}
static int alloc_scan_buf(livo_ctx* c, ScanBuf& s, int64_t N) {
    int best = -1;
    for (size_t k = 0; k < c->spare.size(); k++) {
        const int64_t cap = c->spare[k].cap;
        if (cap >= N && cap <= 2 * N + 4096 && (best < 0 || cap < c->spare[best].cap)) best = (int)k;
    }
    if (best >= 0) {
        s = c->spare[best];
        c->spare.erase(c->spare.begin() + best);
    } else {
        const int64_t cap = N;
        const int32_t cblk = (int32_t)std::max<int64_t>(1, (cap + kBlock * kPtsPerThread - 1) / (kBlock * kPtsPerThread));
        s = ScanBuf{};
        int rc = 0;
        rc |= dev_alloc(&s.pts, (size_t)cap * 4);
        rc |= dev_alloc(&s.nn, (size_t)cap);
        rc |= dev_alloc(&s.partial, partial_doubles(cap));
        rc |= dev_alloc(&s.d_perm, (size_t)cap);
        rc |= dev_alloc(&s.d_iperm, (size_t)cap);
        rc |= dev_alloc(&s.plane, (size_t)cap * 4);
        rc |= dev_alloc(&s.pstate, (size_t)cap);
        rc |= dev_alloc(&s.ikrows, (size_t)cblk * kIkFewRows * 13);
        rc |= dev_alloc(&s.ikcnt, (size_t)cblk);
        if (rc) {
            free_scan_buf(s);
            return LIVO_E_OOM;
        }
        s.cap = cap;
    }
    s.used = true;
    s.searched = false;
    s.n = N;
    s.nblk = (int32_t)std::max<int64_t>(1, (N + kBlock * kPtsPerThread - 1) / (kBlock * kPtsPerThread));
    s.pending = false;
    s.perm.clear();
    return LIVO_OK;
}

// Back to the spare list (the caller has synchronised the context's streams).
static void release_scan_buf(livo_ctx* c, ScanBuf& s) {
    size_t kept = scan_buf_bytes(s.cap);
    for (const ScanBuf& x : c->spare) kept += scan_buf_bytes(x.cap);
    while (!c->spare.empty() && kept > spare_budget()) {  // the oldest go first
        kept -= scan_buf_bytes(c->spare.front().cap);
        free_scan_buf(c->spare.front());
        c->spare.erase(c->spare.begin());
    }
    ScanBuf r = s;
    r.used = false;
    r.pending = false;
    r.perm = std::vector<int32_t>();
    c->spare.push_back(r);
    s = ScanBuf{};
}

// Upload scratch of N points: [keys | sorted keys | iota | perm | bounds], then
// (livo_scan_upload) the packed source points.
static size_t up_tmp_bytes(int64_t N) { return (size_t)N * (4 + 4 + 4 + 4) + 256; }
static int ensure_up_tmp(livo_ctx* c, size_t bytes) {
    if (bytes <= c->up_tmp_bytes) return LIVO_OK;
    if (c->up_tmp) (void)hipFree(c->up_tmp);  // (synchronous: no upload is in flight)
    c->up_tmp = nullptr;
    c->up_tmp_bytes = 0;
    if (hipMalloc(&c->up_tmp, bytes) != hipSuccess) return LIVO_E_OOM;
    c->up_tmp_bytes = bytes;
    return LIVO_OK;
}

// Where a scan is built: the stream, the sort scratch (keys, sorted keys, iota,
// perm, bounds: up_tmp_bytes) and the rocPRIM scratch, grown on demand.
struct UpTarget {
    hipStream_t st;
    void** tmp;
    size_t* tmp_bytes;
    void** prim;
    size_t* prim_bytes;
};
static int ensure_dev_bytes(void** p, size_t* have, size_t need) {
    if (need <= *have) return LIVO_OK;
    if (*p) (void)hipFree(*p);  // (the caller has drained the stream that used it)
    *p = nullptr;
    *have = 0;
    if (hipMalloc(p, need) != hipSuccess) return LIVO_E_OOM;
    *have = need;
    return LIVO_OK;
}

// Morton-order N device points (x, y, z at d_src + stride * i floats) into the
// scan buffers s on U.st: the same keys and stable order as a host sort.  Only
// enqueues; the caller synchronises or records an event.
static int scan_build_on(const UpTarget& U, const float* d_src, int stride, int64_t N, ScanBuf& s) {
    if (N <= 0) return LIVO_OK;
    char* base = (char*)*U.tmp;
    auto* codes = (uint32_t*)base;
    auto* scodes = codes + N;
    auto* iota = scodes + N;
    auto* perm = iota + N;
    auto* mm = (unsigned*)(((uintptr_t)(perm + N) + 15) & ~(uintptr_t)15);
    int rc = LIVO_OK;
    // bounds start at (+max, -max) in the order-preserving encoding
    if (hipMemsetD32Async((hipDeviceptr_t)mm, 0xFFFFFFFFu, 3, U.st) != hipSuccess ||
        hipMemsetD32Async((hipDeviceptr_t)(mm + 3), 0u, 3, U.st) != hipSuccess)
        rc = LIVO_E_HIP;
    if (!rc) rc = launch_fe_minmax(d_src, N, stride, mm, U.st);
    if (!rc) rc = launch_fe_morton(d_src, N, stride, mm, morton_scale(), codes, iota, U.st);
    if (!rc) {
        size_t tb = 0;
        rc = prim_sort_pairs_u32(nullptr, &tb, codes, scodes, iota, perm, N, 27, U.st);
        if (!rc && tb > *U.prim_bytes) {
            if (hipStreamSynchronize(U.st) != hipSuccess) rc = LIVO_E_HIP;
            if (!rc) rc = ensure_dev_bytes(U.prim, U.prim_bytes, tb);
        }
        tb = *U.prim_bytes;
        if (!rc) rc = prim_sort_pairs_u32(*U.prim, &tb, codes, scodes, iota, perm, N, 27, U.st);
    }
    if (!rc) rc = launch_fe_gather(d_src, N, stride, perm, s.pts, s.d_iperm, U.st);
    if (!rc && (hipMemcpyAsync(s.d_perm, perm, (size_t)N * 4, hipMemcpyDeviceToDevice, U.st) != hipSuccess ||
                hipMemsetAsync(s.nn, 0, (size_t)N * sizeof(NNRec), U.st) != hipSuccess ||
                hipMemsetAsync(s.pstate, 0, (size_t)N, U.st) != hipSuccess))
        rc = LIVO_E_HIP;
    return rc;
}

// A resident scan from N device points (x, y, z at d_src + stride * i floats),
// built synchronously on the context's stream.
static int scan_create_device(livo_ctx* c, const float* d_src, int stride, int64_t N, int32_t* scan_id) {
    ScanBuf s;
    int rc = alloc_scan_buf(c, s, N);
    if (rc) return rc;
    if (N > 0) {
        rc = ensure_up_tmp(c, up_tmp_bytes(N));
        const UpTarget U{c->stream, &c->up_tmp, &c->up_tmp_bytes, &c->prim_tmp, &c->prim_bytes};
        if (!rc) rc = scan_build_on(U, d_src, stride, N, s);
        if (hipStreamSynchronize(c->stream) != hipSuccess && !rc) rc = LIVO_E_HIP;
        if (rc) {
            release_scan_buf(c, s);
            return rc;
        }
    }
    *scan_id = register_scan(c, s);
    return LIVO_OK;
}

// The caller's points packed to x, y, z (a strided PointType array is read once).
static void pack_xyz(const float* xyz, int64_t N, int64_t stride_bytes, float* out) {
    const char* base = (const char*)xyz;
    if (stride_bytes == (int64_t)(3 * sizeof(float))) {
        std::memcpy(out, xyz, (size_t)N * 3 * sizeof(float));
        return;
    }
    for (int64_t i = 0; i < N; i++) std::memcpy(out + 3 * i, base + i * stride_bytes, 3 * sizeof(float));
}

int livo_scan_upload(livo_ctx* c, const float* xyz, int64_t N, int64_t stride_bytes, int32_t* scan_id) {
    if (!c || !scan_id || N < 0 || (N > 0 && !xyz)) return LIVO_E_INVALID;
    if (N > (int64_t)0x7FFFFFFF - kBlock) return LIVO_E_RANGE;
    if (stride_bytes == 0) stride_bytes = 3 * sizeof(float);
    if (stride_bytes < (int64_t)(3 * sizeof(float))) return LIVO_E_INVALID;
    if (set_device(c)) return LIVO_E_HIP;
    // the caller's points packed to x, y, z, copied to HBM behind the upload
    // scratch, then Morton-ordered on the device (scan_create_device)
    float* d_src = nullptr;
    if (N > 0) {
        const size_t off = (up_tmp_bytes(N) + 255) & ~(size_t)255;
        int rc = ensure_up_tmp(c, off + (size_t)N * 3 * sizeof(float));
        if (rc) return rc;
        d_src = (float*)((char*)c->up_tmp + off);
        float* h = nullptr;
        const bool packed = stride_bytes == (int64_t)(3 * sizeof(float));
        if (!packed) {
            h = (float*)std::malloc((size_t)N * 3 * sizeof(float));
            if (!h) return LIVO_E_OOM;
            pack_xyz(xyz, N, stride_bytes, h);
        }
        const hipError_t e = hipMemcpyAsync(d_src, packed ? xyz : h, (size_t)N * 3 * sizeof(float),
                                            hipMemcpyHostToDevice, c->stream);
        const hipError_t e2 = hipStreamSynchronize(c->stream);
        std::free(h);
        if (e != hipSuccess || e2 != hipSuccess) return LIVO_E_HIP;
    }
    return scan_create_device(c, d_src, 3, N, scan_id);
}

// livo_scan_upload without waiting: the points go through a pinned staging
// buffer (the caller's array is free again on return) and are copied and
// Morton-ordered on the context's upload stream, beside whatever the batch
// lanes run; the scan's `ready` event gates its users (batch_enqueue waits for
// it on the device, every other call through get_scan on the host).
int livo_scan_upload_async(livo_ctx* c, const float* xyz, int64_t N, int64_t stride_bytes, int32_t* scan_id) {
    if (!c || !scan_id || N < 0 || (N > 0 && !xyz)) return LIVO_E_INVALID;
    if (N > (int64_t)0x7FFFFFFF - kBlock) return LIVO_E_RANGE;
    if (stride_bytes == 0) stride_bytes = 3 * sizeof(float);
    if (stride_bytes < (int64_t)(3 * sizeof(float))) return LIVO_E_INVALID;
    if (N == 0) return livo_scan_upload(c, xyz, N, stride_bytes, scan_id);
    if (set_device(c)) return LIVO_E_HIP;
    if (!c->up_stream && hipStreamCreateWithFlags(&c->up_stream, hipStreamNonBlocking) != hipSuccess) {
        c->up_stream = nullptr;
        return LIVO_E_HIP;
    }
    const size_t off = (up_tmp_bytes(N) + 255) & ~(size_t)255, bytes = (size_t)N * 3 * sizeof(float);
    if (off + bytes > c->aup_tmp_bytes) {  // (growing: the uploads queued on it finish first)
        if (hipStreamSynchronize(c->up_stream) != hipSuccess) return LIVO_E_HIP;
        const int rc = ensure_dev_bytes(&c->aup_tmp, &c->aup_tmp_bytes, off + bytes);
        if (rc) return rc;
    }
    // a pinned staging buffer whose last copy is done (the ring's oldest)
    livo_ctx::PinSlot& P = c->pin[c->pin_next];
    c->pin_next = (c->pin_next + 1) % kPinRing;
    if (P.inflight && hipEventSynchronize(P.copied) != hipSuccess) return LIVO_E_HIP;
    P.inflight = false;
    if (!P.copied && hipEventCreateWithFlags(&P.copied, hipEventDisableTiming) != hipSuccess) {
        P.copied = nullptr;
        return LIVO_E_HIP;
    }
    if (bytes > P.bytes) {
        if (P.h) (void)hipHostFree(P.h);
        P.h = nullptr;
        P.bytes = 0;
        if (hipHostMalloc((void**)&P.h, bytes, hipHostMallocDefault) != hipSuccess) {
            P.h = nullptr;
            return LIVO_E_OOM;
        }
        P.bytes = bytes;
    }
    pack_xyz(xyz, N, stride_bytes, P.h);
    ScanBuf s;
    int rc = alloc_scan_buf(c, s, N);
    if (rc) return rc;
    if (!s.ready && hipEventCreateWithFlags(&s.ready, hipEventDisableTiming) != hipSuccess) {
        s.ready = nullptr;
        release_scan_buf(c, s);
        return LIVO_E_HIP;
    }
    float* d_src = (float*)((char*)c->aup_tmp + off);
    if (hipMemcpyAsync(d_src, P.h, bytes, hipMemcpyHostToDevice, c->up_stream) != hipSuccess ||
        hipEventRecord(P.copied, c->up_stream) != hipSuccess)
        rc = LIVO_E_HIP;
    P.inflight = rc == LIVO_OK;
    const UpTarget U{c->up_stream, &c->aup_tmp, &c->aup_tmp_bytes, &c->aup_prim, &c->aup_prim_bytes};
    if (!rc) rc = scan_build_on(U, d_src, 3, N, s);
    if (!rc && hipEventRecord(s.ready, c->up_stream) != hipSuccess) rc = LIVO_E_HIP;
    if (rc) {
        (void)hipStreamSynchronize(c->up_stream);
        release_scan_buf(c, s);
        return rc;
    }
    s.pending = true;
    *scan_id = register_scan(c, s);
    return LIVO_OK;
}

// True if p lies in page-locked host memory (livo_host_register, hipHostMalloc):
// the copy engine reads it directly.
static bool host_pinned(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}
// Both ends of [p, p + bytes) page-locked: a caller that registered a shorter
// range than the array takes the staging path, not a device page fault.
static bool host_pinned_range(const void* p, size_t bytes) {
    return host_pinned(p) && (bytes <= 1 || host_pinned((const char*)p + bytes - 1));
}

int livo_host_register(livo_ctx* c, void* p, size_t bytes) {
    if (!c || !p || bytes == 0) return LIVO_E_INVALID;
    if (set_device(c)) return LIVO_E_HIP;
    // mapped + portable: the copy engine addresses the pages directly from any
    // stream (hipHostRegisterDefault alone left some processes copying at ~6 GB/s,
    // 1.5 ms of host time per 8 x 100k batch)
    return hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable) == hipSuccess ? LIVO_OK
                                                                                                    : LIVO_E_HIP;
}
int livo_host_unregister(livo_ctx* c, void* p) {
    if (!c || !p) return LIVO_E_INVALID;
    if (set_device(c)) return LIVO_E_HIP;
    if (hipDeviceSynchronize() != hipSuccess) return LIVO_E_HIP;  // (no copy may still read it)
    return hipHostUnregister(p) == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

// livo_scan_upload_async for a batch of scans in one pass: one staging copy
// (or, from page-locked caller memory, one DMA per scan and no host copy), then
// one bounds pass, one key pass, ONE stable sort of the whole batch (the scan
// in the key's top bits) and one gather that also clears the neighbour
// records, kFeSegMax scans at a time, on the upload stream.  Each scan is
// stored exactly as livo_scan_upload stores it.
static int upload_batch_chunks(livo_ctx* c, const float* const* xyz, const int64_t* N, int32_t n,
                               int64_t stride_bytes, int32_t* scan_ids, int32_t* registered);

// The scans are built in passes of kFeSegMax: a pass that fails releases the
// scans the earlier passes of the same call registered, so a failed call leaves
// no scan behind (scan_ids unspecified).
int livo_scan_upload_batch_async(livo_ctx* c, const float* const* xyz, const int64_t* N, int32_t n,
                                 int64_t stride_bytes, int32_t* scan_ids) {
    int32_t registered = 0;
    const int rc = upload_batch_chunks(c, xyz, N, n, stride_bytes, scan_ids, &registered);
    if (rc)
        for (int32_t b = 0; b < registered; b++) (void)livo_scan_release(c, scan_ids[b]);
    return rc;
}

static int upload_batch_chunks(livo_ctx* c, const float* const* xyz, const int64_t* N, int32_t n,
                               int64_t stride_bytes, int32_t* scan_ids, int32_t* registered) {
    if (!c || !xyz || !N || !scan_ids || n < 0) return LIVO_E_INVALID;
    if (stride_bytes == 0) stride_bytes = 3 * sizeof(float);
    if (stride_bytes < (int64_t)(3 * sizeof(float))) return LIVO_E_INVALID;
    for (int32_t b = 0; b < n; b++) {
        if (N[b] < 0 || (N[b] > 0 && !xyz[b])) return LIVO_E_INVALID;
        if (N[b] > (int64_t)0x7FFFFFFF - kBlock) return LIVO_E_RANGE;
    }
    if (set_device(c)) return LIVO_E_HIP;
    // (the builds on a high-priority stream were slower: 3.8k vs 11.8k updates/s
    // with uploads)
    if (!c->up_stream && hipStreamCreateWithFlags(&c->up_stream, hipStreamNonBlocking) != hipSuccess) {
        c->up_stream = nullptr;
        return LIVO_E_HIP;
    }
    if (!c->cp_stream && hipStreamCreateWithFlags(&c->cp_stream, hipStreamNonBlocking) != hipSuccess) {
        c->cp_stream = nullptr;
        return LIVO_E_HIP;
    }
    for (int k = 0; k < 2; k++)
        if ((!c->bsrc_copied[k] && hipEventCreateWithFlags(&c->bsrc_copied[k], hipEventDisableTiming) != hipSuccess) ||
            (!c->bsrc_free[k] && hipEventCreateWithFlags(&c->bsrc_free[k], hipEventDisableTiming) != hipSuccess))
            return LIVO_E_HIP;
    for (int32_t b0 = 0; b0 < n; b0 += kFeSegMax) {
        const int32_t m = std::min<int32_t>(kFeSegMax, n - b0);
        int64_t tot = 0, max_n = 0;
        for (int32_t b = 0; b < m; b++) {
            tot += N[b0 + b];
            max_n = std::max(max_n, N[b0 + b]);
        }
        if (tot == 0) {  // (empty scans only)
            for (int32_t b = 0; b < m; b++) {
                const int rc = livo_scan_upload(c, xyz[b0 + b], 0, stride_bytes, scan_ids + b0 + b);
                if (rc) return rc;
                *registered = b0 + b + 1;
            }
            continue;
        }
        if (tot > (int64_t)0xFFFFFFFF - kBlock) return LIVO_E_RANGE;  // (32-bit positions in the batch sort)
        // build scratch (up_stream): [keys | sorted keys | iota | sorted iota | bounds (6 per scan)];
        // the packed points in the staging buffer of this pass (cp_stream copies into it)
        const size_t kb = (size_t)tot * 4, vb = (size_t)tot * 4;
        const size_t mm_off = 2 * kb + 2 * vb;
        const size_t tmp_need = mm_off + 6 * sizeof(unsigned) * kFeSegMax;
        const size_t bytes = (size_t)tot * 3 * sizeof(float);
        const int sl = c->bsrc_next;
        c->bsrc_next ^= 1;
        if (tmp_need > c->aup_tmp_bytes || bytes > c->bsrc_bytes[sl]) {  // (growing: the uploads in flight finish first)
            if (hipStreamSynchronize(c->cp_stream) != hipSuccess || hipStreamSynchronize(c->up_stream) != hipSuccess)
                return LIVO_E_HIP;
            int rc = ensure_dev_bytes(&c->aup_tmp, &c->aup_tmp_bytes, tmp_need);
            if (!rc) rc = ensure_dev_bytes(&c->bsrc[sl], &c->bsrc_bytes[sl], bytes);
            if (rc) return rc;
        }
        char* base = (char*)c->aup_tmp;
        auto* codes = (uint32_t*)base;
        auto* scodes = (uint32_t*)(base + kb);
        auto* iota = (uint32_t*)(base + 2 * kb);
        auto* sorted = (uint32_t*)(base + 2 * kb + vb);
        auto* mm = (unsigned*)(base + mm_off);
        float* d_src = (float*)c->bsrc[sl];
        // the copy into this buffer waits for the build that last read it
        if (c->bsrc_used[sl] && hipStreamWaitEvent(c->cp_stream, c->bsrc_free[sl], 0) != hipSuccess) return LIVO_E_HIP;
        // the points: straight from page-locked caller memory, else through a
        // pinned staging buffer of the ring (the caller's arrays are free on return)
        const bool trace = std::getenv("LIVO_UPLOAD_TRACE") != nullptr;  // (development: host phases to stderr)
        auto now_us = [] {
            return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
        };
        const double t_a = trace ? now_us() : 0.0;
        bool direct = stride_bytes == (int64_t)(3 * sizeof(float));
        for (int32_t b = 0; b < m && direct; b++)
            if (N[b0 + b] > 0 && !host_pinned_range(xyz[b0 + b], (size_t)N[b0 + b] * 3 * sizeof(float))) direct = false;
        const double t_b = trace ? now_us() : 0.0;
        double t_c = t_b, t_d = t_b;
        int rc = LIVO_OK;
        livo_ctx::PinSlot* P = nullptr;
        if (!direct) {
            P = &c->pin[c->pin_next];
            c->pin_next = (c->pin_next + 1) % kPinRing;
            if (P->inflight && hipEventSynchronize(P->copied) != hipSuccess) return LIVO_E_HIP;
            P->inflight = false;
            t_c = trace ? now_us() : 0.0;
            if (bytes > P->bytes) {
                if (P->h) (void)hipHostFree(P->h);
                P->h = nullptr;
                P->bytes = 0;
                if (hipHostMalloc((void**)&P->h, bytes, hipHostMallocDefault) != hipSuccess) {
                    P->h = nullptr;
                    return LIVO_E_OOM;
                }
                P->bytes = bytes;
            }
            if (!P->copied && hipEventCreateWithFlags(&P->copied, hipEventDisableTiming) != hipSuccess) {
                P->copied = nullptr;
                return LIVO_E_HIP;
            }
            // one host thread per scan (up to 8): a single thread's copy into pinned
            // memory ran at ~9 GB/s (1.07 ms per 8 x 100k batch)
            int64_t offs[kFeSegMax];
            int64_t o = 0;
            for (int32_t b = 0; b < m; b++) {
                offs[b] = o;
                o += N[b0 + b];
            }
            auto pack = [&](int32_t b) {
                if (N[b0 + b] > 0) pack_xyz(xyz[b0 + b], N[b0 + b], stride_bytes, P->h + 3 * offs[b]);
            };
            if (bytes < ((size_t)1 << 20) || m == 1) {
                for (int32_t b = 0; b < m; b++) pack(b);
            } else {
                const int nt = std::min<int>(8, m);
                std::vector<std::thread> th;
                for (int t = 1; t < nt; t++)
                    th.emplace_back([&, t] {
                        for (int32_t b = t; b < m; b += nt) pack(b);
                    });
                for (int32_t b = 0; b < m; b += nt) pack(b);
                for (auto& x : th) x.join();
            }
            t_d = trace ? now_us() : 0.0;
            if (hipMemcpyAsync(d_src, P->h, bytes, hipMemcpyHostToDevice, c->cp_stream) != hipSuccess ||
                hipEventRecord(P->copied, c->cp_stream) != hipSuccess)
                return LIVO_E_HIP;
            P->inflight = true;
        } else {
            // page-locked caller arrays: one kernel reads them through their mapped
            // device addresses (no DMA command per scan: a hipMemcpyAsync of one
            // held the host 13-16 ms now and then inside a running farm); an
            // array without a device mapping: DMA copies
            FeSrc F{};
            bool mapped = true;
            int64_t o = 0;
            for (int32_t b = 0; b < m; b++) {
                F.off[b] = o;
                F.n[b] = N[b0 + b];
                F.src[b] = nullptr;
                if (mapped && N[b0 + b] > 0) {
                    void* dp = nullptr;
                    if (hipHostGetDevicePointer(&dp, const_cast<float*>(xyz[b0 + b]), 0) != hipSuccess || !dp) {
                        (void)hipGetLastError();
                        mapped = false;
                    }
                    F.src[b] = (const float*)dp;
                }
                o += N[b0 + b];
            }
            if (mapped) {
                const int r2 = launch_fe_copy_seg(F, m, max_n, d_src, c->cp_stream);
                if (r2) return r2;
            } else {
                o = 0;
                for (int32_t b = 0; b < m; b++) {
                    if (N[b0 + b] > 0 &&
                        hipMemcpyAsync(d_src + 3 * o, xyz[b0 + b], (size_t)N[b0 + b] * 3 * sizeof(float),
                                       hipMemcpyHostToDevice, c->cp_stream) != hipSuccess)
                        return LIVO_E_HIP;
                    o += N[b0 + b];
                }
            }
            t_d = trace ? now_us() : 0.0;  // (the copies' host time)
        }
        if (hipEventRecord(c->bsrc_copied[sl], c->cp_stream) != hipSuccess ||
            hipStreamWaitEvent(c->up_stream, c->bsrc_copied[sl], 0) != hipSuccess)
            return LIVO_E_HIP;
        // the scans' buffers
        ScanBuf sb[kFeSegMax];
        FeSegs S{};
        int64_t o = 0;
        for (int32_t b = 0; b < m && !rc; b++) {
            rc = alloc_scan_buf(c, sb[b], N[b0 + b]);
            if (!rc && !sb[b].ready && hipEventCreateWithFlags(&sb[b].ready, hipEventDisableTiming) != hipSuccess) {
                sb[b].ready = nullptr;
                rc = LIVO_E_HIP;
            }
            S.off[b] = o;
            S.n[b] = N[b0 + b];
            S.pts4[b] = sb[b].pts;
            S.iperm[b] = sb[b].d_iperm;
            S.perm[b] = sb[b].d_perm;
            S.nn[b] = sb[b].nn;
            S.pstate[b] = sb[b].pstate;
            o += N[b0 + b];
        }
        // bounds start at +max (mins) and ~(-max) (maxes, stored inverted) in the order-preserving encoding
        if (!rc && (hipMemsetD32Async((hipDeviceptr_t)mm, 0xFFFFFFFFu, 6 * kFeSegMax, c->up_stream) != hipSuccess))
            rc = LIVO_E_HIP;
        if (!rc) rc = launch_fe_build_seg(d_src, S, m, max_n, mm, morton_scale(), codes, iota, c->up_stream);
        int key_bits = 27;  // + the scan index's bits
        while ((1 << (key_bits - 27)) < m) key_bits++;
        if (!rc) {
            size_t tb = 0;
            rc = prim_sort_pairs_u32(nullptr, &tb, codes, scodes, iota, sorted, tot, key_bits, c->up_stream);
            if (!rc && tb > c->aup_prim_bytes) {
                if (hipStreamSynchronize(c->up_stream) != hipSuccess) rc = LIVO_E_HIP;
                if (!rc) rc = ensure_dev_bytes(&c->aup_prim, &c->aup_prim_bytes, tb);
            }
            tb = c->aup_prim_bytes;
            if (!rc) rc = prim_sort_pairs_u32(c->aup_prim, &tb, codes, scodes, iota, sorted, tot, key_bits, c->up_stream);
        }
        if (!rc) rc = launch_fe_gather_seg(d_src, S, m, max_n, sorted, c->up_stream);
        if (!rc && hipEventRecord(c->bsrc_free[sl], c->up_stream) != hipSuccess) rc = LIVO_E_HIP;
        c->bsrc_used[sl] = true;
        for (int32_t b = 0; b < m && !rc; b++)
            if (hipEventRecord(sb[b].ready, c->up_stream) != hipSuccess) rc = LIVO_E_HIP;
        if (rc) {
            (void)hipStreamSynchronize(c->cp_stream);
            (void)hipStreamSynchronize(c->up_stream);
            for (int32_t b = 0; b < m; b++)
                if (sb[b].used) release_scan_buf(c, sb[b]);
            return rc;
        }
        if (trace)
            std::fprintf(stderr, "[upload] %d scans %s: pinned check %.1f us, ring wait %.1f, pack / copies %.1f, build %.1f\n",
                         (int)m, direct ? "direct" : "staged", t_b - t_a, t_c - t_b, t_d - t_c, now_us() - t_d);
        for (int32_t b = 0; b < m; b++) {
            if (N[b0 + b] == 0) {  // (an empty scan has nothing to build)
                release_scan_buf(c, sb[b]);
                rc = livo_scan_upload(c, xyz[b0 + b], 0, stride_bytes, scan_ids + b0 + b);
                if (rc) {
                    for (int32_t q = b + 1; q < m; q++) release_scan_buf(c, sb[q]);  // (built, not registered)
                    return rc;
                }
                *registered = b0 + b + 1;
                continue;
            }
            sb[b].pending = true;
            scan_ids[b0 + b] = register_scan(c, sb[b]);
            *registered = b0 + b + 1;
        }
    }
    return LIVO_OK;
}

int livo_scan_release(livo_ctx* c, int32_t id) {
    if (!c) return LIVO_E_INVALID;
    if (id < 0 || id >= (int32_t)c->scans.size() || !c->scans[id].used) return LIVO_E_NOSCAN;
    // a scan of a submitted batch is released once that batch is collected; every
    // other call that reads a scan returns only when its device work is done, so
    // the buffers are idle once the scan's own upload is (no stream drain: the
    // farm releases scans while the next batches run)
    for (int l = 0; l < LIVO_MAX_INFLIGHT; l++)
        if (c->lane[l].busy)
            for (int32_t x : c->lane[l].ids)
                if (x == id) return LIVO_E_BUSY;
    (void)hipSetDevice(c->device);
    ScanBuf& s = c->scans[id];
    if (s.pending && hipEventSynchronize(s.ready) != hipSuccess) return LIVO_E_HIP;
    s.pending = false;
    release_scan_buf(c, s);
    return LIVO_OK;
}

// A resident scan, its asynchronous upload finished (host wait); get_scan_q:
// without the wait (batch_enqueue, which waits for it on the device).
static ScanBuf* get_scan_q(livo_ctx* c, int32_t id) {
    if (id < 0 || id >= (int32_t)c->scans.size() || !c->scans[id].used) return nullptr;
    return &c->scans[id];
}
static ScanBuf* get_scan(livo_ctx* c, int32_t id) {
    ScanBuf* s = get_scan_q(c, id);
    if (s && s->pending) {
        if (hipEventSynchronize(s->ready) != hipSuccess) return nullptr;
        s->pending = false;
    }
    return s;
}
// The scan's stored -> caller order on the host (the per-point outputs), copied
// from the device on first use.
static int host_perm(ScanBuf* s) {
    if ((int64_t)s->perm.size() == s->n) return LIVO_OK;
    s->perm.resize((size_t)s->n);
    if (s->n > 0 && hipMemcpy(s->perm.data(), s->d_perm, (size_t)s->n * 4, hipMemcpyDeviceToHost) != hipSuccess) {
        s->perm.clear();
        return LIVO_E_HIP;
    }
    return LIVO_OK;
}

int livo_scan_neighbors(livo_ctx* c, int32_t id, int32_t* idx, float* sqdist) {
    if (!c) return LIVO_E_INVALID;
    ScanBuf* s = get_scan(c, id);
    if (!s || !s->searched) return LIVO_E_NOSCAN;
    // a scan of a submitted batch is being searched on a group stream: its
    // records are collected with the batch (livo_iekf_update_batch_wait) first
    for (const BatchLane& B : c->lane)
        if (B.busy && std::find(B.ids.begin(), B.ids.end(), id) != B.ids.end()) return LIVO_E_BUSY;
    if (set_device(c)) return LIVO_E_HIP;
    std::vector<NNRec> rec((size_t)s->n);
    if (s->n > 0) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipMemcpy(rec.data(), s->nn, (size_t)s->n * sizeof(NNRec), hipMemcpyDeviceToHost));
    }
    if (host_perm(s)) return LIVO_E_HIP;
    for (int64_t j = 0; j < s->n; j++) {
        const int64_t o = (int64_t)s->perm[(size_t)j];  // caller's point index
        for (int k = 0; k < kNN; k++) {
            if (idx) idx[o * kNN + k] = rec[(size_t)j].idx[k];
            if (sqdist) sqdist[o * kNN + k] = rec[(size_t)j].p[k][3];
        }
    }
    return LIVO_OK;
}

int livo_h_share(livo_ctx* c, int32_t id, const livo_state* state, int search_en, double HTH[81], double HTL[9],
                 int64_t* effct, const livo_point_out* out) {
    if (!c || !state || !HTH || !HTL) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    ScanBuf* s = get_scan(c, id);
    if (!s) return LIVO_E_NOSCAN;
    if (!map_ready(c)) return LIVO_E_NOMAP;
    if (set_device(c)) return LIVO_E_HIP;
    int rc = ensure_slots(c, 1);
    if (rc) return rc;
    const int64_t N = s->n;
    // debug scratch: normvec N*4, world N*3, sel N; laserCloudOri compaction: flags N, pos N, ori N*3, corr N*4
    const bool want_ori = out && (out->ori_xyz || out->corr_normvec || out->n_ori);
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t nvb = al((size_t)N * 16), wb = al((size_t)N * 12), sb = al((size_t)N);
    const size_t fb = want_ori ? al((size_t)N * 4) : 0, ob = want_ori ? al((size_t)N * 12) : 0,
                 cb = want_ori ? al((size_t)N * 16) : 0;
    rc = ensure_scratch(c, nvb + wb + sb + 2 * fb + ob + cb + 64);
    if (rc) return rc;
    char* base = (char*)c->scratch;
    init_slot(c->h_slots[0], *state, *state, c->params.max_iterations);
    fill_job(c->h_jobs[0], *s, c->d_slots);
    HIP_TRY(hipMemcpyAsync(c->d_slots, c->h_slots, sizeof(IekfSlot), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_jobs, c->h_jobs, sizeof(HsJob), hipMemcpyHostToDevice, c->stream));
    HsParams hp = make_hs_params(c);
    hp.force = search_en ? 1 : 0;
    const bool want_nv = out && out->normvec, want_sel = out && out->selected, want_w = out && out->world_xyz;
    hp.dbg.normvec = (want_nv || want_ori) ? (float*)base : nullptr;
    hp.dbg.world = want_w ? (float*)(base + nvb) : nullptr;
    hp.dbg.sel = (want_sel || want_ori) ? (uint8_t*)(base + nvb + wb) : nullptr;
    if (search_en) {
        rc = ensure_replay(c, N);
        if (rc) return rc;
        KnnParams kp = make_knn_params(c);
        kp.force = 1;
        if (c->backend == LIVO_BACKEND_IVOX) {
            HIP_TRY(hipMemsetAsync(kp.replay_count, 0, sizeof(unsigned), c->stream));
            HIP_TRY(hipMemsetAsync(kp.replay_count2, 0, sizeof(unsigned), c->stream));
            rc = backend_knn(c, kp, 1, N, false, c->stream);
        } else {
            rc = knn_pass(kp, 1, N, c->stream);
        }
        if (rc) return rc;
    } else if (!s->searched && N > 0) {
        // no cached neighbours yet: nothing is matched (points_near.size() < 5, :525)
        HIP_TRY(hipMemsetAsync(s->nn, 0, (size_t)N * sizeof(NNRec), c->stream));
    }
    rc = launch_hshare(hp, 1, std::max(s->nblk, 1), search_en != 0, c->stream);
    if (rc) return rc;
    // laserCloudOri / corr_normvect: the effective points in the caller's order (:547-561)
    int64_t n_ori = 0;
    float *d_ori = nullptr, *d_corr = nullptr;
    if (want_ori && N > 0) {
        uint32_t* flags = (uint32_t*)(base + nvb + wb + sb);
        uint32_t* pos = (uint32_t*)(base + nvb + wb + sb + fb);
        d_ori = (float*)(base + nvb + wb + sb + 2 * fb);
        d_corr = (float*)(base + nvb + wb + sb + 2 * fb + ob);
        rc = launch_ori_flags(hp.dbg.sel, s->d_perm, N, flags, c->stream);
        if (!rc) rc = ivox_scan(c, flags, pos, N);
        if (!rc) rc = launch_ori_scatter(s->pts, hp.dbg.normvec, hp.dbg.sel, s->d_perm, pos, N, d_ori, d_corr, c->stream);
        if (rc) return rc;
        uint32_t tail[2];
        HIP_TRY(hipMemcpyAsync(&tail[0], pos + N - 1, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(&tail[1], flags + N - 1, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        n_ori = (int64_t)tail[0] + tail[1];
        if (out->ori_xyz && n_ori > 0)
            HIP_TRY(hipMemcpyAsync(out->ori_xyz, d_ori, (size_t)n_ori * 12, hipMemcpyDeviceToHost, c->stream));
        if (out->corr_normvec && n_ori > 0)
            HIP_TRY(hipMemcpyAsync(out->corr_normvec, d_corr, (size_t)n_ori * 16, hipMemcpyDeviceToHost, c->stream));
    }
    if (want_ori && out->n_ori) *out->n_ori = n_ori;
    // the last plane-pass block has reduced the sums into slot->red (hp.solve = 0)
    HIP_TRY(hipMemcpyAsync(c->h_slots, c->d_slots, sizeof(IekfSlot), hipMemcpyDeviceToHost, c->stream));
    std::vector<float> h_nv, h_w;
    std::vector<uint8_t> h_sel;
    if (N > 0 && out) {
        if (want_nv) {
            h_nv.resize((size_t)N * 4);
            HIP_TRY(hipMemcpyAsync(h_nv.data(), hp.dbg.normvec, (size_t)N * 16, hipMemcpyDeviceToHost, c->stream));
        }
        if (want_w) {
            h_w.resize((size_t)N * 3);
            HIP_TRY(hipMemcpyAsync(h_w.data(), hp.dbg.world, (size_t)N * 12, hipMemcpyDeviceToHost, c->stream));
        }
        if (want_sel) {
            h_sel.resize((size_t)N);
            HIP_TRY(hipMemcpyAsync(h_sel.data(), hp.dbg.sel, (size_t)N, hipMemcpyDeviceToHost, c->stream));
        }
    }
    std::vector<NNRec> recs;
    if (N > 0 && out && (out->nn_idx || out->nn_sqdist)) {
        recs.resize((size_t)N);
        HIP_TRY(hipMemcpyAsync(recs.data(), s->nn, (size_t)N * sizeof(NNRec), hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (search_en) s->searched = true;
    const IekfSlot& hs = c->h_slots[0];
    const double* r = hs.red;
    std::memset(HTH, 0, 81 * sizeof(double));
    std::memset(HTL, 0, 9 * sizeof(double));
    int q = 0;
    for (int a = 0; a < 6; a++)
        for (int b = a; b < 6; b++) {
            HTH[a * 9 + b] = r[q];
            HTH[b * 9 + a] = r[q];
            q++;
        }
    for (int a = 0; a < 6; a++) HTL[a] = r[21 + a];
    if (effct) *effct = (int64_t)r[28];
    if (out && out->visits) *out->visits = (int64_t)hs.visits[0];
    // per-point outputs come back in the caller's point order (stored order is Morton)
    if (host_perm(s)) return LIVO_E_HIP;
    for (int64_t k = 0; k < N; k++) {
        const int64_t i = s->perm[k];
        if (!h_nv.empty()) std::memcpy(out->normvec + 4 * i, &h_nv[4 * k], 16);
        if (!h_w.empty()) std::memcpy(out->world_xyz + 3 * i, &h_w[3 * k], 12);
        if (!h_sel.empty()) out->selected[i] = h_sel[k];
        if (!recs.empty())
            for (int j = 0; j < 5; j++) {
                if (out->nn_idx) out->nn_idx[i * 5 + j] = recs[k].idx[j];
                if (out->nn_sqdist) out->nn_sqdist[i * 5 + j] = recs[k].p[j][3];
            }
    }
    return LIVO_OK;
}

// The batched iterated update of both formulations: the LaserMapping IEKF
// (states/priors/stats, model 0) or the IKFoM update (ik_states/ik_stats, model 1),
// in two halves over one batch lane: batch_enqueue puts the whole loop, and the
// copies of the slots back, on the lane's streams; batch_collect waits for them
// and unpacks the results.  Profiling (events, timings) on synchronous batches only.
static int batch_enqueue(livo_ctx* c, int L, int32_t n, const int32_t* ids, int model, const livo_state* states,
                         const livo_state* priors, const livo_ikfom_state* ik_states, bool sync) {
    if (!c || n < 0 || (n > 0 && (!ids || (model == kModelIkfom ? !ik_states : !states)))) return LIVO_E_INVALID;
    BatchLane& B = c->lane[L];
    if (B.busy) return LIVO_E_BUSY;
    B.n = 0;
    if (n == 0) return LIVO_OK;
    if (!map_ready(c)) return LIVO_E_NOMAP;
    if (model == kModelIkfom && c->backend != LIVO_BACKEND_IKDTREE) return LIVO_E_INVALID;  // ikd-Tree h-model only
    for (int32_t b = 0; b < n; b++)
        if (!get_scan_q(c, ids[b])) return LIVO_E_NOSCAN;
    {
        // a scan's neighbour records, plane cache and partials are per scan: the
        // same id twice in one batch would have two updates write them concurrently
        std::vector<int32_t> sorted(ids, ids + n);
        std::sort(sorted.begin(), sorted.end());
        if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end()) return LIVO_E_INVALID;
        // nor may a scan be in two batches in flight
        for (int l = 0; l < LIVO_MAX_INFLIGHT; l++)
            if (l != L && c->lane[l].busy)
                for (int32_t id : c->lane[l].ids)
                    if (std::binary_search(sorted.begin(), sorted.end(), id)) return LIVO_E_INVALID;
    }
    const bool lm = model != kModelIkfom;
    // the fused evaluation: search + replay + plane pass + solve in one launch
    const bool fused = c->fused && model == kModelLaserMapping && c->backend == LIVO_BACKEND_IKDTREE &&
                       c->knn_kind == 2;
    // the unfused LaserMapping passes (iVox: per-context search scratch) run as
    // synchronous batches only; IKFoM batches keep their staging and replay
    // lists per lane (checked before any device work, so a refused submit
    // leaves nothing queued)
    if (!fused && lm && (L != 0 || !sync)) return LIVO_E_INVALID;
    if (set_device(c)) return LIVO_E_HIP;
    int rc = lane_streams(c, L);
    if (rc) return rc;
    rc = lm ? ensure_lm(B, n) : ensure_ik(B, n);
    if (rc) return rc;
    // Slots and jobs: the IKFoM model uses whole slots (c->h_slots / d_slots);
    // the LaserMapping model only the part before the IKFoM block, packed at
    // kLmStride with the jobs behind them, so the batch crosses PCIe in one
    // copy each way.  (A packed slot is addressed as an IekfSlot whose IKFoM
    // block lies outside the buffer; the LaserMapping kernels never touch it.)
    const size_t stride = lm ? kLmStride : sizeof(IekfSlot);
    char* const hbase = lm ? B.h_lm : B.h_ik;
    char* const dbase = lm ? B.d_lm : B.d_ik;
    HsJob* const hjobs = reinterpret_cast<HsJob*>(hbase + (size_t)n * stride);
    HsJob* const djobs = reinterpret_cast<HsJob*>(dbase + (size_t)n * stride);
    auto hslot = [&](int32_t b) -> IekfSlot& { return *reinterpret_cast<IekfSlot*>(hbase + (size_t)b * stride); };
    auto dslot = [&](int32_t b) { return reinterpret_cast<IekfSlot*>(dbase + (size_t)b * stride); };
    const int max_iter = c->params.max_iterations;
    // fused batches: the solve that stops a scan writes its slot into the
    // host-mapped staging copy itself (LIVO_SLOT_WB=0: copies after the batch)
    const bool wb = fused && lm && B.h_lm_dev && c->slot_wb;
    int64_t total_n = 0;
    for (int32_t b = 0; b < n; b++) {
        ScanBuf* s = get_scan_q(c, ids[b]);
        if (model == kModelIkfom) {
            init_slot_ik(hslot(b), ik_states[b], max_iter);
        } else {
            init_slot(hslot(b), states[b], priors ? priors[b] : states[b], max_iter, kSlotLmBytes);
        }
        fill_job(hjobs[b], *s, dslot(b));
        if (wb) hjobs[b].host_slot = reinterpret_cast<uint4*>(B.h_lm_dev + (size_t)b * stride);
        total_n += s->n;
    }
    rc = ensure_replay(c, total_n);
    if (rc) return rc;

    // The batch in groups on separate streams: the latency-bound kernels of
    // one group (18x18 solve, tie replay, launch gaps) overlap the
    // throughput-bound k-NN / plane passes of the others.  Each group keeps
    // its own replay list.
    struct Group {
        int32_t first, count;
        int max_nblk;
        int64_t max_n, off;
        hipStream_t st;
    };
    Group g[kMaxGroups];
    // default: four groups, one per hardware queue (round 4, 8 x 100k distinct
    // scans, pipelined: 1 / 2 / 3 / 4 groups 18675 / 21170 / 22350 / 22984
    // updates/s; 6 / 8 share the box's 4 queues and lose, profiles/r04_ab_groups.txt;
    // 8 x 200k on the 10M map: 4437 vs 3960 with two): one group's
    // latency-bound evaluations (no search: launch, reduction, solve) and its
    // replay tail overlap the other groups' searches.  IKFoM four too (5.40k vs
    // 5.13k with two); the iVox path two (1,520 vs 1,513 with four)
    const int auto_groups = (fused || model == kModelIkfom) ? 4 : 2;
    const int ngroups = std::max(1, std::min<int>(c->groups > 0 ? c->groups : auto_groups, n));
    int64_t off = 0;
    for (int gi = 0; gi < ngroups; gi++) {
        g[gi].first = (int32_t)((int64_t)n * gi / ngroups);
        g[gi].count = (int32_t)((int64_t)n * (gi + 1) / ngroups) - g[gi].first;
        g[gi].max_nblk = 1;
        g[gi].max_n = 1;
        g[gi].off = off;
        g[gi].st = B.st[gi];
        for (int32_t b = g[gi].first; b < g[gi].first + g[gi].count; b++) {
            const ScanBuf* s = get_scan_q(c, ids[b]);
            g[gi].max_nblk = std::max(g[gi].max_nblk, (int)s->nblk);
            g[gi].max_n = std::max<int64_t>(g[gi].max_n, s->n);
            off += s->n;
        }
    }
    const bool prof = sync && L == 0 && c->profiling && c->events_ready;  // 1: first-search events only
    const bool full = prof && c->profiling >= 2;         // 2: every evaluation, the batch span and the gap
    if (full) {
        HIP_TRY(hipEventRecord(c->b_start, c->stream));
        // the replay count of this batch only (every batch's replays add to it)
        HIP_TRY(hipMemsetAsync(c->d_replay_total, 0, 8, c->stream));
    }
    // queued behind another lane's batch on shared streams: with LIVO_LANE_SERIAL=1
    // start only once all of its groups are done (default: each group as soon as its
    // own stream frees)
    const BatchLane* prev = (!c->lane_own_streams && c->lane_serial && c->last_lane >= 0 && c->last_lane != L &&
                             c->lane[c->last_lane].busy) ? &c->lane[c->last_lane] : nullptr;
    c->last_lane = L;
    // kernel copies for batches queued behind another on shared streams (a DMA
    // copy there waits on an engine hand-off); LIVO_LANE_ZC=0: DMA copies always
    const bool kcopy = (lm ? B.h_lm_dev != nullptr : B.h_ik_dev != nullptr) && (sync ? c->sync_zc : c->lane_zc);
    static_assert(sizeof(HsJob) % 16 == 0 && sizeof(IekfSlot) % 16 == 0 && kLmStride % 16 == 0, "16-B word copies");
    const char* const hsrc = lm ? (kcopy ? B.h_lm_dev : B.h_lm) : (kcopy ? B.h_ik_dev : B.h_ik);
    const bool iv = c->backend == LIVO_BACKEND_IVOX && lm;  // (synchronous batches only: lane 0)
    unsigned* const rcount = c->d_replay_count + (size_t)L * kMaxGroups;  // this lane's
    unsigned long long* const rlist = c->d_replay_list + (size_t)L * c->replay_cap;
    // Each group stages its own slots and jobs on its own stream and starts from
    // there: no fork from stream 0, so a group waits only for its own scans'
    // uploads and, in a pipelined farm, for its own stream's previous batch (a
    // queued batch's group g no longer waits for the previous batch's group 0).
    for (int gi = 0; gi < ngroups; gi++) {
        const hipStream_t st = g[gi].st;
        for (int32_t b = g[gi].first; b < g[gi].first + g[gi].count; b++) {
            ScanBuf* s = get_scan_q(c, ids[b]);
            // a scan whose asynchronous upload may still run: the group waits on the device
            if (s->pending) HIP_TRY(hipStreamWaitEvent(st, s->ready, 0));
            // IKFoM: its searches rewrite the neighbours without refitting the cached planes
            if (model == kModelIkfom && s->n > 0) HIP_TRY(hipMemsetAsync(s->pstate, 0, (size_t)s->n, st));
        }
        if (prev)
            for (int q = 0; q < prev->ngroups; q++) HIP_TRY(hipStreamWaitEvent(st, prev->done[q], 0));
        const size_t s0 = (size_t)g[gi].first * stride, sb = (size_t)g[gi].count * stride;
        const size_t j0 = (size_t)n * stride + (size_t)g[gi].first * sizeof(HsJob), jb = (size_t)g[gi].count * sizeof(HsJob);
        if (kcopy) {
            rc = launch_copy_ranges(hsrc, dbase, s0, sb, j0, jb, st);
            if (rc) return rc;
        } else {
            HIP_TRY(hipMemcpyAsync(dbase + s0, hsrc + s0, sb, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(dbase + j0, hsrc + j0, jb, hipMemcpyHostToDevice, st));
        }
        if (!fused) HIP_TRY(hipMemsetAsync(rcount + gi, 0, sizeof(unsigned), st));
        if (iv) HIP_TRY(hipMemsetAsync(c->d_replay_count2 + gi, 0, sizeof(unsigned), st));
        // profiling: each group's first search starts at ev[gi][0]
        if (prof) HIP_TRY(hipEventRecord(c->ev[gi][0], st));
    }
    const int evals = max_iter + 1;
    HsParams hp[kMaxGroups];
    KnnParams kp[kMaxGroups];
    for (int gi = 0; gi < ngroups; gi++) {
        hp[gi] = make_hs_params(c);
        hp[gi].jobs = djobs + g[gi].first;
        kp[gi] = make_knn_params(c);
        kp[gi].jobs = djobs + g[gi].first;
        kp[gi].replay_count = rcount + gi;
        kp[gi].replay_list = rlist + g[gi].off;
        kp[gi].replay_count2 = iv ? c->d_replay_count2 + gi : nullptr;
        kp[gi].replay_list2 = iv ? c->d_replay_list2 + g[gi].off : nullptr;
        // the iVox overflow pass of each group has its own scratch slices (groups run concurrently)
        if (kp[gi].iv.scratch) kp[gi].iv.scratch += (int64_t)gi * c->iv.big_threads * c->iv.big_slice;
        hp[gi].solve = lm ? 1 : 0;  // the last plane-pass block of each scan runs its solve (IKFoM: k_solve_ik below)
        hp[gi].replay_count = rcount + gi;
        hp[gi].replay_count2 = kp[gi].replay_count2;
    }
    // one launch per evaluation (a launch whose scans all stopped exits at once)
    for (int e = 0; e < evals; e++) {
        for (int gi = 0; gi < ngroups && fused; gi++) {
            hipStream_t st = g[gi].st;
            // full: ev[gi][e] before evaluation e, ev[gi][evals] after the last
            if (full && e > 0) HIP_TRY(hipEventRecord(c->ev[gi][e], st));
            rc = launch_iekf_eval(kp[gi], hp[gi], g[gi].count, g[gi].max_n, e == 0, st);
            if (rc) return rc;
            if (prof && !full && e == 0) HIP_TRY(hipEventRecord(c->ev[gi][1], st));
        }
        for (int gi = 0; gi < ngroups && !fused; gi++) {
            hipStream_t st = g[gi].st;
            if (full && e > 0) HIP_TRY(hipEventRecord(c->ev[gi][3 * e], st));
            // leaf-map search; rematch passes are bounded by the previous neighbours
            // (the group's replay count was zeroed before the batch / by the last k_solve)
            rc = backend_knn(c, kp[gi], g[gi].count, g[gi].max_n, e > 0, st);
            if (rc) return rc;
            if ((prof && e == 0) || full) HIP_TRY(hipEventRecord(c->ev[gi][3 * e + 1], st));
            rc = model == kModelIkfom ? launch_hshare_ik(hp[gi], g[gi].count, g[gi].max_nblk, e == 0, st)
                                      : launch_hshare(hp[gi], g[gi].count, g[gi].max_nblk, e == 0, st);
            if (rc) return rc;
            if (!lm) {
                // IKFoM: the reduction, the measurement-free part of the update and
                // the gain (k_solve_ik)
                rc = launch_solve_ik(hp[gi], g[gi].count, st);
                if (rc) return rc;
            }
        }
    }
    for (int gi = 0; gi < ngroups; gi++)
        if (full) HIP_TRY(hipEventRecord(c->ev[gi][fused ? evals : 3 * LIVO_MAX_EVALS], g[gi].st));
    // each group copies its own slots back on its own stream (no cross-stream
    // join before the copy); the host then waits for every group's stream
    for (int gi = 0; gi < ngroups; gi++) {
        if (wb) {
            // (written by the stopping solves)
        } else if (kcopy) {
            rc = launch_copy_words(dslot(g[gi].first), (lm ? B.h_lm_dev : B.h_ik_dev) + (size_t)g[gi].first * stride,
                                   stride * g[gi].count, g[gi].st);
            if (rc) return rc;
        } else {
            HIP_TRY(hipMemcpyAsync(&hslot(g[gi].first), dslot(g[gi].first), stride * g[gi].count,
                                   hipMemcpyDeviceToHost, g[gi].st));
        }
        // this batch's end on the group's stream (another lane's batch may queue behind it)
        HIP_TRY(hipEventRecord(B.done[gi], g[gi].st));
    }
    if (full) {
        // the replay counter: every group's searches have run (joined into the main stream)
        for (int gi = 1; gi < ngroups; gi++) {
            HIP_TRY(hipEventRecord(c->xjoin[gi - 1], g[gi].st));
            HIP_TRY(hipStreamWaitEvent(c->stream, c->xjoin[gi - 1], 0));
        }
        HIP_TRY(hipMemcpyAsync(&c->last_replays, c->d_replay_total, 8, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemsetAsync(c->d_replay_total, 0, 8, c->stream));
        HIP_TRY(hipEventRecord(c->b_end[c->b_par], c->stream));
    }
    B.busy = true;
    B.n = n;
    B.model = model;
    B.ngroups = ngroups;
    B.ids.assign(ids, ids + n);
    for (int gi = 0; gi < ngroups; gi++) {
        B.gfirst[gi] = g[gi].first;
        B.gcount[gi] = g[gi].count;
    }
    return LIVO_OK;
}

static int batch_collect(livo_ctx* c, int L, livo_state* states, livo_iter_stats* stats,
                         livo_ikfom_state* ik_states, livo_ikfom_stats* ik_stats, bool sync) {
    BatchLane& B = c->lane[L];
    const int32_t n = B.n;
    if (n == 0) return LIVO_OK;
    if (!B.busy) return LIVO_E_INVALID;
    const std::vector<int32_t> idv = std::move(B.ids);
    B.ids.clear();
    const int32_t* ids = idv.data();
    const int model = B.model;
    const int ngroups = B.ngroups;
    const bool lm = model != kModelIkfom;
    const size_t stride = lm ? kLmStride : sizeof(IekfSlot);
    char* const hbase = lm ? B.h_lm : B.h_ik;
    auto hslot = [&](int32_t b) -> IekfSlot& { return *reinterpret_cast<IekfSlot*>(hbase + (size_t)b * stride); };
    const bool fused = c->fused && model == kModelLaserMapping && c->backend == LIVO_BACKEND_IKDTREE &&
                       c->knn_kind == 2;
    const int evals = c->params.max_iterations + 1;
    const bool prof = sync && L == 0 && c->profiling && c->events_ready;
    const bool full = prof && c->profiling >= 2;
    struct { hipStream_t st; } g[kMaxGroups];
    for (int gi = 0; gi < ngroups; gi++) g[gi].st = B.st[gi];
    B.busy = false;  // collected (or failed): the lane is free either way
    B.n = 0;
    // wait by polling: the batch is short, and a blocking wait's wake-up
    // latency was a visible part of the gap between two batches
    for (int gi = ngroups - 1; gi >= 0; gi--) HIP_TRY(event_wait(B.done[gi]));
    if (full) HIP_TRY(stream_wait(c->stream));  // the replay counter's read-back and the batch-end event
    const unsigned long long replays = c->last_replays;
    for (int32_t b = 0; b < n; b++) {
        const IekfSlot& s = hslot(b);
        if (model == kModelIkfom) {
            ik_states[b] = s.ik.x;
            if (ik_stats) ik_stats[b] = s.ik.stats;
        } else {
            states[b] = s.state;
            if (stats) stats[b] = s.stats;
        }
        c->scans[ids[b]].searched = true;
    }
    if (prof) {
        livo_timings t{};
        // first search of the whole batch: wall time from the earliest group's
        // start to the latest group's end (the groups start on their own streams)
        double lead = 0.0;  // how long before group 0 the earliest group started
        for (int gi = 0; gi < ngroups; gi++) {
            float ms = 0.f, m0 = 0.f;
            (void)hipEventElapsedTime(&ms, c->ev[0][0], c->ev[gi][1]);
            (void)hipEventElapsedTime(&m0, c->ev[0][0], c->ev[gi][0]);
            t.knn_ms = std::max(t.knn_ms, (double)ms);
            lead = std::max(lead, -(double)m0);
        }
        t.knn_ms += lead;
        t.knn_launches = 1;
        if (full && fused) {
            // every evaluation launch: max over the concurrent groups
            t.n_evals = std::min(evals, LIVO_MAX_EVALS);
            for (int e = 0; e < t.n_evals; e++) {
                // the evaluation's window over the concurrent groups (e = 0: the same
                // window as knn_ms above, from the earliest group's start)
                double m = 0.0;
                for (int gi = 0; gi < ngroups; gi++) {
                    float ms = 0.f;
                    (void)hipEventElapsedTime(&ms, e == 0 ? c->ev[0][0] : c->ev[gi][e], c->ev[gi][e + 1]);
                    m = std::max(m, (double)ms);
                }
                if (e == 0) m = t.knn_ms;
                t.eval_ms[e] = m;
                int searched = 0;
                for (int32_t b = 0; b < n; b++) searched += hslot(b).eval_search[e] != 0;
                t.eval_searched[e] = searched;
                if (e == 0) t.knn_ms = m;
                else if (searched) t.rematch_knn_ms += m;
                else t.plane_ms += m;
            }
        }
        if (full) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, c->b_start, c->b_end[c->b_par]);
            t.batch_ms = ms;
            if (c->b_prev) {
                (void)hipEventElapsedTime(&ms, c->b_end[c->b_par ^ 1], c->b_start);
                t.gap_ms = ms;
            }
            c->b_prev = true;
            c->b_par ^= 1;
        }
        for (int gi = 0; gi < ngroups && full && !fused; gi++)
            for (int e = 0; e < evals; e++) {
                float ms_k = 0.f, ms_h = 0.f;
                if (e > 0) (void)hipEventElapsedTime(&ms_k, c->ev[gi][3 * e], c->ev[gi][3 * e + 1]);
                const hipEvent_t end = (e + 1 < evals) ? c->ev[gi][3 * e + 3] : c->ev[gi][3 * LIVO_MAX_EVALS];
                (void)hipEventElapsedTime(&ms_h, c->ev[gi][3 * e + 1], end);
                t.rematch_knn_ms += ms_k;
                t.plane_ms += ms_h;  // plane pass + the solve run by its last block
            }
        // the first evaluation searches for every point of every scan
        for (int32_t b = 0; b < n; b++) {
            t.knn_visits += (int64_t)hslot(b).visits[0];
            t.knn_points += (int64_t)hslot(b).scanned[0];
            t.knn_queries += c->scans[ids[b]].n;
            t.effct_points += model == kModelIkfom ? hslot(b).ik.stats.effct_feat_num[0]
                                                   : hslot(b).stats.effct_feat_num[0];
        }
        t.knn_replays = (int64_t)replays;
        c->last = t;
    }
    return LIVO_OK;
}

static int batch_update(livo_ctx* c, int32_t n, const int32_t* ids, int model, livo_state* states,
                        const livo_state* priors, livo_iter_stats* stats, livo_ikfom_state* ik_states,
                        livo_ikfom_stats* ik_stats) {
    if (c && any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    int rc = batch_enqueue(c, 0, n, ids, model, states, priors, ik_states, true);
    if (rc) {
        if (c) {  // an enqueue that failed half-way: let the lane's queued work finish
            for (int k = 0; k < kMaxGroups && c->lane[0].st[k]; k++) (void)hipStreamSynchronize(c->lane[0].st[k]);
            c->lane[0].busy = false;
            c->lane[0].ids.clear();
        }
        return rc;
    }
    return batch_collect(c, 0, states, stats, ik_states, ik_stats, true);
}


int livo_iekf_update_batch(livo_ctx* c, int32_t n, const int32_t* ids, livo_state* states, const livo_state* priors,
                           livo_iter_stats* stats) {
    return batch_update(c, n, ids, kModelLaserMapping, states, priors, stats, nullptr, nullptr);
}

static int batch_submit(livo_ctx* c, int32_t n, const int32_t* ids, int model, const livo_state* states,
                        const livo_state* priors, const livo_ikfom_state* ik_states, int32_t* ticket) {
    if (!c || !ticket) return LIVO_E_INVALID;
    int L = -1;
    for (int l = 0; l < LIVO_MAX_INFLIGHT && L < 0; l++)
        if (!c->lane[l].busy) L = l;
    if (L < 0) return LIVO_E_BUSY;
    int rc = batch_enqueue(c, L, n, ids, model, states, priors, ik_states, false);
    if (rc) {
        BatchLane& B = c->lane[L];
        for (int k = 0; k < kMaxGroups && B.st[k]; k++) (void)hipStreamSynchronize(B.st[k]);
        B.busy = false;
        B.n = 0;
        B.ids.clear();
        return rc;
    }
    c->lane[L].busy = true;  // (an empty batch too: its ticket is waited for like any other)
    c->lane_gen = (c->lane_gen + 1) & 0x3fffffff;
    c->lane[L].ticket = c->lane_gen * LIVO_MAX_INFLIGHT + L;
    *ticket = c->lane[L].ticket;
    return LIVO_OK;
}

int livo_iekf_update_batch_submit(livo_ctx* c, int32_t n, const int32_t* ids, const livo_state* states,
                                  const livo_state* priors, int32_t* ticket) {
    return batch_submit(c, n, ids, kModelLaserMapping, states, priors, nullptr, ticket);
}

static int batch_wait(livo_ctx* c, int32_t ticket, int model, livo_state* states, livo_iter_stats* stats,
                      livo_ikfom_state* ik_states, livo_ikfom_stats* ik_stats) {
    if (!c || ticket < 0) return LIVO_E_INVALID;
    const int L = ticket % LIVO_MAX_INFLIGHT;
    BatchLane& B = c->lane[L];
    if (!B.busy || B.ticket != ticket) return LIVO_E_INVALID;
    if (B.n > 0 && (B.model != model || (model == kModelIkfom ? !ik_states : !states))) return LIVO_E_INVALID;
    if (set_device(c)) return LIVO_E_HIP;
    B.ticket = -1;
    if (B.n == 0) {
        B.busy = false;
        return LIVO_OK;
    }
    return batch_collect(c, L, states, stats, ik_states, ik_stats, false);
}

int livo_iekf_update_batch_wait(livo_ctx* c, int32_t ticket, livo_state* states, livo_iter_stats* stats) {
    return batch_wait(c, ticket, kModelLaserMapping, states, stats, nullptr, nullptr);
}

int livo_ikfom_update_batch_submit(livo_ctx* c, int32_t n, const int32_t* ids, const livo_ikfom_state* states,
                                   int32_t* ticket) {
    return batch_submit(c, n, ids, kModelIkfom, nullptr, nullptr, states, ticket);
}

int livo_ikfom_update_batch_wait(livo_ctx* c, int32_t ticket, livo_ikfom_state* states, livo_ikfom_stats* stats) {
    return batch_wait(c, ticket, kModelIkfom, nullptr, nullptr, states, stats);
}

int livo_iekf_update(livo_ctx* c, int32_t id, livo_state* state, const livo_state* prior, livo_iter_stats* stats) {
    if (!state) return LIVO_E_INVALID;
    return livo_iekf_update_batch(c, 1, &id, state, prior, stats);
}

int livo_ikfom_update_batch(livo_ctx* c, int32_t n, const int32_t* ids, livo_ikfom_state* states,
                            livo_ikfom_stats* stats) {
    return batch_update(c, n, ids, kModelIkfom, nullptr, nullptr, nullptr, states, stats);
}

int livo_ikfom_update(livo_ctx* c, int32_t id, livo_ikfom_state* state, livo_ikfom_stats* stats) {
    if (!state) return LIVO_E_INVALID;
    return livo_ikfom_update_batch(c, 1, &id, state, stats);
}

int livo_ctx_set_backend(livo_ctx* c, int backend) {
    if (!c || (backend != LIVO_BACKEND_IKDTREE && backend != LIVO_BACKEND_IVOX)) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    if (backend != c->backend)
        for (auto& s : c->scans) s.searched = false;  // cached neighbours belong to the other map
    c->backend = backend;
    return LIVO_OK;
}

int livo_ivox_params_default(livo_ivox_params* p) {
    if (!p) return LIVO_E_INVALID;
    p->resolution = 0.2f;   // ivox_grid_resolution default (laser_mapping.cpp:1021)
    p->nearby_type = 18;    // ivox_nearby_type default (laser_mapping.cpp:1022)
    p->capacity = 1000000;  // Options::capacity_ (ivox3d.h:57)
    return LIVO_OK;
}

int livo_ivox_init(livo_ctx* c, const livo_ivox_params* p) {
    if (!c) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    livo_ivox_params prm;
    livo_ivox_params_default(&prm);
    if (p) prm = *p;
    int nearby = 0;
    switch (prm.nearby_type) {
        case 0: nearby = 1; break;
        case 6: nearby = 7; break;
        case 18: nearby = 19; break;
        case 26: nearby = 27; break;
        default: return LIVO_E_INVALID;
    }
    if (!(prm.resolution > 0.f) || !std::isfinite(prm.resolution) || prm.capacity < 1) return LIVO_E_INVALID;
    if (set_device(c)) return LIVO_E_HIP;
    HIP_TRY(hipStreamSynchronize(c->stream));
    ivox_free(c->iv);
    IvoxDev& v = c->iv;
    v.prm = prm;
    v.inv_res = (float)(1.0 / (double)prm.resolution);  // options_.inv_resolution_ = 1.0 / resolution_
    v.nearby = nearby;
    if (const char* e = std::getenv("LIVO_IVOX_KIND"))  // (A/B and tests: force one search kernel)
        v.kind = std::strcmp(e, "thread") == 0 ? 0 : (std::strcmp(e, "wave") == 0 ? 1 : (std::strcmp(e, "team") == 0 ? 2 : -1));
    if (dev_alloc(&v.ctr, 5)) return LIVO_E_OOM;  // the counters of IvoxParams::ctr
    int rc = ivox_ensure_table(c, 1024);
    if (!rc) rc = ivox_ensure_big(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    v.ready = true;
    for (auto& s : c->scans) s.searched = false;
    return LIVO_OK;
}

int livo_ivox_add_points(livo_ctx* c, const float* xyz, int64_t n, int64_t stride_bytes) {
    if (!c || n < 0 || (n > 0 && !xyz)) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    if (stride_bytes == 0) stride_bytes = 3 * sizeof(float);
    if (stride_bytes < (int64_t)(3 * sizeof(float))) return LIVO_E_INVALID;
    if (!c->iv.ready) return LIVO_E_NOMAP;
    if (n == 0) return LIVO_OK;
    if (set_device(c)) return LIVO_E_HIP;
    int rc = ivox_ensure_src(c, n);
    if (rc) return rc;
    std::vector<float> h((size_t)n * 4);
    const char* base = (const char*)xyz;
    for (int64_t i = 0; i < n; i++) {
        const float* p = (const float*)(base + i * stride_bytes);
        h[4 * i] = p[0]; h[4 * i + 1] = p[1]; h[4 * i + 2] = p[2]; h[4 * i + 3] = 0.f;
    }
    HIP_TRY(hipMemcpyAsync(c->iv.src, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
    return ivox_add_dev(c, n);
}

int livo_ivox_knn(livo_ctx* c, const float* q, int64_t n, int32_t max_num, double max_range, int32_t* idx,
                  float* d, int32_t* cnt) {
    if (!c || n < 0 || max_num < 1 || max_num > kNN || !(max_range >= 0.0) ||
        (n > 0 && (!q || !idx || !d || !cnt)))
        return LIVO_E_INVALID;
    if (!c->iv.ready) return LIVO_E_NOMAP;
    if (n == 0) return LIVO_OK;
    if (n > (int64_t)0x7FFFFFFF - kBlock) return LIVO_E_RANGE;
    if (set_device(c)) return LIVO_E_HIP;
    int rc = ensure_slots(c, 1);
    if (rc) return rc;
    const size_t qb = (size_t)n * 4 * sizeof(float), rb = (size_t)n * sizeof(NNRec);
    rc = ensure_scratch(c, qb + rb + 256);
    if (!rc) rc = ensure_replay(c, n);
    if (rc) return rc;
    char* base = (char*)c->scratch;
    float* dq = (float*)base;
    NNRec* dr = (NNRec*)(base + ((qb + 255) & ~(size_t)255));
    std::vector<float> hq((size_t)n * 4);
    for (int64_t i = 0; i < n; i++) {
        hq[4 * i] = q[3 * i]; hq[4 * i + 1] = q[3 * i + 1]; hq[4 * i + 2] = q[3 * i + 2]; hq[4 * i + 3] = 0.f;
    }
    std::memset(&c->h_slots[0], 0, sizeof(IekfSlot));
    HsJob& j = c->h_jobs[0];
    j = HsJob{};
    j.pts = dq; j.nn = dr; j.slot = c->d_slots; j.n = (int32_t)n; j.nblk = 0;
    HIP_TRY(hipMemcpyAsync(dq, hq.data(), qb, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(dr, 0xFF, rb, c->stream));  // cnt = -1: left alone = nothing found
    HIP_TRY(hipMemcpyAsync(c->d_slots, c->h_slots, sizeof(IekfSlot), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_jobs, c->h_jobs, sizeof(HsJob), hipMemcpyHostToDevice, c->stream));
    KnnParams kp = make_knn_params(c);
    kp.force = 1;
    kp.identity = 1;
    kp.iv.max_num = max_num;
    kp.iv.range2 = max_range * max_range;
    HIP_TRY(hipMemsetAsync(kp.replay_count, 0, sizeof(unsigned), c->stream));
    HIP_TRY(hipMemsetAsync(kp.replay_count2, 0, sizeof(unsigned), c->stream));
    rc = launch_ivox_knn(kp, 1, n, false, c->iv.big_threads, c->stream);
    if (rc) return rc;
    std::vector<NNRec> hr((size_t)n);
    HIP_TRY(hipMemcpyAsync(hr.data(), dr, rb, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int64_t i = 0; i < n; i++) {
        cnt[i] = hr[i].cnt;
        for (int t = 0; t < max_num; t++) {
            const bool has = hr[i].cnt > t;
            idx[i * max_num + t] = has ? hr[i].idx[t] : -1;
            d[i * max_num + t] = has ? hr[i].p[t][3] : INFINITY;
        }
    }
    return LIVO_OK;
}

int livo_ivox_get_info(livo_ctx* c, livo_ivox_info* out) {
    if (!c || !out) return LIVO_E_INVALID;
    if (!c->iv.ready) return LIVO_E_NOMAP;
    const IvoxDev& v = c->iv;
    out->num_points = v.npts;
    out->num_grids = v.ngrids;
    out->ids_issued = v.next_id;
    out->max_grid_points = v.max_grid;
    out->add_passes = v.add_passes;
    out->device_bytes = v.table * (int64_t)(sizeof(GridSlot) + 4 * sizeof(uint32_t)) +
                        (v.pts_cap[0] + v.pts_cap[1]) * 16 +
                        kMaxGroups * v.big_threads * v.big_slice * (int64_t)sizeof(SelElem);
    return LIVO_OK;
}

int livo_ivox_dump(livo_ctx* c, float* xyz, int32_t* ids, int32_t* keys, int64_t cap, int64_t* n) {
    if (!c || !n) return LIVO_E_INVALID;
    if (!c->iv.ready) return LIVO_E_NOMAP;
    const IvoxDev& v = c->iv;
    *n = v.npts;
    if (cap < v.npts) return LIVO_E_RANGE;
    if (set_device(c)) return LIVO_E_HIP;
    std::vector<GridSlot> slots((size_t)v.table);
    std::vector<unsigned long long> tl((size_t)v.table);
    std::vector<float> pts((size_t)v.npts * 4);
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(slots.data(), v.slots, slots.size() * sizeof(GridSlot), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(tl.data(), v.tlast, tl.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    if (v.npts) HIP_TRY(hipMemcpy(pts.data(), v.pts[v.cur], pts.size() * sizeof(float), hipMemcpyDeviceToHost));
    // grids_cache_ order: most recently used first (the id of each grid's last added point)
    std::vector<int64_t> order;
    for (int64_t s2 = 0; s2 < v.table; s2++)
        if (slots[(size_t)s2].key != kGridEmpty) order.push_back(s2);
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return tl[(size_t)a] > tl[(size_t)b]; });
    int64_t k = 0;
    for (const int64_t s2 : order) {
        const GridSlot& g = slots[(size_t)s2];
        const int kx = (int)(g.key & 0x1FFFFFull) - kIvBias, ky = (int)((g.key >> 21) & 0x1FFFFFull) - kIvBias,
                  kz = (int)((g.key >> 42) & 0x1FFFFFull) - kIvBias;
        for (uint32_t t = 0; t < g.count && k < v.npts; t++, k++) {
            const float* p = &pts[4 * (size_t)(g.start + t)];
            if (xyz) { xyz[3 * k] = p[0]; xyz[3 * k + 1] = p[1]; xyz[3 * k + 2] = p[2]; }
            if (ids) std::memcpy(&ids[k], &p[3], 4);
            if (keys) { keys[3 * k] = kx; keys[3 * k + 1] = ky; keys[3 * k + 2] = kz; }
        }
    }
    return k == v.npts ? LIVO_OK : LIVO_E_HIP;
}

int livo_map_incremental(livo_ctx* c, int32_t id, const livo_state* state, double fs, int ekf_inited, uint8_t* cat,
                         int64_t counts[2]) {
    if (!c || !state || !(fs > 0.0)) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    if (c->backend != LIVO_BACKEND_IVOX) return map_incremental_ikd(c, id, state, fs, cat, counts);
    if (!c->iv.ready) return LIVO_E_NOMAP;
    ScanBuf* s = get_scan(c, id);
    if (!s) return LIVO_E_NOSCAN;
    if (set_device(c)) return LIVO_E_HIP;
    const int64_t N = s->n;
    if (counts) counts[0] = counts[1] = 0;
    if (N == 0) return LIVO_OK;
    int rc = ensure_slots(c, 1);
    if (rc) return rc;
    // scratch: ordered 2N x 16 B, flags 2N x 4, pos 2N x 4, cat N
    const size_t ob = (size_t)N * 32, fb = (size_t)N * 8, cb = (size_t)N;
    rc = ensure_scratch(c, ob + 2 * fb + cb + 1024);
    if (!rc) rc = ivox_ensure_src(c, N);
    if (rc) return rc;
    char* base = (char*)c->scratch;
    float* ordered = (float*)base;
    uint32_t* flags = (uint32_t*)(base + ob);
    uint32_t* pos = (uint32_t*)(base + ob + fb);
    uint8_t* dcat = (uint8_t*)(base + ob + 2 * fb);
    init_slot(c->h_slots[0], *state, *state, c->params.max_iterations);
    HIP_TRY(hipMemcpyAsync(c->d_slots, c->h_slots, sizeof(IekfSlot), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(flags, 0, fb, c->stream));
    MapIncrParams mp{};
    mp.pts = s->pts;
    mp.nn = s->nn;
    mp.perm = s->d_perm;
    mp.slot = c->d_slots;
    std::memcpy(mp.R_LI, c->params.R_LI, sizeof(mp.R_LI));
    std::memcpy(mp.t_LI, c->params.t_LI, sizeof(mp.t_LI));
    mp.ordered = ordered;
    mp.flags = flags;
    mp.cat = cat ? dcat : nullptr;
    mp.fs = fs;
    mp.n = (int32_t)N;
    mp.ekf_inited = ekf_inited ? 1 : 0;
    rc = launch_map_incr(mp, c->stream);
    if (!rc) rc = ivox_scan(c, flags, pos, 2 * N);
    if (!rc) rc = launch_compact(ordered, flags, pos, 2 * N, c->iv.src, c->stream);
    if (rc) return rc;
    uint32_t tail[3];  // pos[N], pos[2N-1], flags[2N-1]
    HIP_TRY(hipMemcpyAsync(&tail[0], pos + N, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(&tail[1], pos + 2 * N - 1, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(&tail[2], flags + 2 * N - 1, 4, hipMemcpyDeviceToHost, c->stream));
    std::vector<uint8_t> hcat;
    if (cat) {
        hcat.resize((size_t)N);
        HIP_TRY(hipMemcpyAsync(hcat.data(), dcat, cb, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    const int64_t total = (int64_t)tail[1] + tail[2], n_add = tail[0];
    if (cat) {
        if (host_perm(s)) return LIVO_E_HIP;
        for (int64_t k = 0; k < N; k++) cat[s->perm[(size_t)k]] = hcat[(size_t)k];
    }
    rc = ivox_add_dev(c, total);
    if (rc) return rc;
    if (counts) {
        counts[0] = n_add;
        counts[1] = total - n_add;
    }
    return LIVO_OK;
}

int livo_scan_inherit_neighbors(livo_ctx* c, int32_t dst, int32_t src) {
    if (!c) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    ScanBuf* d = get_scan(c, dst);
    ScanBuf* s = get_scan(c, src);
    if (!d || !s) return LIVO_E_NOSCAN;
    if (dst == src) return LIVO_OK;
    if (set_device(c)) return LIVO_E_HIP;
    if (d->n == 0) return LIVO_OK;
    const int rc = launch_inherit_nn(d->nn, d->d_perm, d->n, s->nn, s->d_iperm, s->searched ? s->n : 0, c->stream);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(d->pstate, 0, (size_t)d->n, c->stream));  // new neighbours: planes to refit
    HIP_TRY(hipStreamSynchronize(c->stream));
    d->searched = true;  // the cache now holds the inherited entries
    return LIVO_OK;
}

int livo_scan_preprocess(livo_ctx* c, const livo_raw_point* raw, int64_t n, const livo_imu_pose* poses,
                         int32_t n_poses, const double rot_end[9], const double pos_end[3], float leaf_size,
                         int32_t* scan_id, livo_raw_point* undistorted, livo_raw_point* down, int64_t down_cap,
                         int64_t* n_down) {
    if (!c || !scan_id || n < 0 || (n > 0 && !raw) || n_poses < 0 || (n_poses > 0 && !poses) ||
        !std::isfinite(leaf_size))
        return LIVO_E_INVALID;
    const bool deskew = n_poses >= 2 && n > 0;
    if (deskew && (!rot_end || !pos_end)) return LIVO_E_INVALID;
    for (int32_t k = 1; k < n_poses; k++)
        if (!(poses[k].offset_time >= poses[k - 1].offset_time)) return LIVO_E_INVALID;  // the walk needs sorted segments
    if (n > (int64_t)0x7FFFFFFF - kBlock) return LIVO_E_RANGE;
    if (set_device(c)) return LIVO_E_HIP;
    // the previous frame's feats_undistort is gone from here on (its buffer may be
    // freed or overwritten below): livo_frame_to_world(-1) sees no frame until this
    // one has been processed completely
    c->fe_raw = nullptr;
    c->fe_n = 0;
    // scratch: raw 20n, poses, seg 2x4n, keys/iota/skeys/svals 4x4n, flags/vid 2x4n, starts 4(n+1), down 20n
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t nb = (size_t)std::max<int64_t>(n, 1);
    const size_t b_raw = al(nb * 20), b_pose = al((size_t)std::max(n_poses, 1) * 22 * 8), b4 = al(nb * 4),
                 b_st = al((nb + 1) * 4);
    const size_t total = b_raw + b_pose + 8 * b4 + b_st + b_raw + 256;
    if (total > c->fe_bytes) {
        if (c->fe_buf) (void)hipFree(c->fe_buf);
        c->fe_buf = nullptr;
        c->fe_bytes = 0;
        if (hipMalloc(&c->fe_buf, total) != hipSuccess) return LIVO_E_OOM;
        c->fe_bytes = total;
    }
    char* p = (char*)c->fe_buf;
    FrontParams F{};
    F.raw = (float*)p; p += b_raw;
    double* d_poses = (double*)p; p += b_pose;
    int32_t* seg = (int32_t*)p; p += b4;
    F.seg = seg;
    F.seg_rev = (int32_t*)p; p += b4;
    F.keys = (uint32_t*)p; p += b4;
    F.iota = (uint32_t*)p; p += b4;
    uint32_t* skeys = (uint32_t*)p; p += b4;
    uint32_t* svals = (uint32_t*)p; p += b4;
    F.flags = (uint32_t*)p; p += b4;
    F.vid = (uint32_t*)p; p += b4;
    F.starts = (uint32_t*)p; p += b_st;
    F.down = (float*)p; p += b_raw;
    unsigned* mm = (unsigned*)p;
    F.skeys = skeys;
    F.svals = svals;
    F.n = n;
    F.poses = d_poses;
    F.np = n_poses;
    std::memcpy(F.R_LI, c->params.R_LI, sizeof(F.R_LI));
    std::memcpy(F.t_LI, c->params.t_LI, sizeof(F.t_LI));
    if (n > 0) HIP_TRY(hipMemcpyAsync(F.raw, raw, (size_t)n * 20, hipMemcpyHostToDevice, c->stream));
    int rc = LIVO_OK;
    if (deskew) {
        // extR_Ri = R_LI^T rot_end^T, exrR_extT = R_LI^T t_LI (IMU_Processing.cpp:337-338)
        const double* RL = c->params.R_LI;
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) {
                double acc = RL[0 * 3 + i] * rot_end[j * 3 + 0];
                for (int l = 1; l < 3; l++) acc = acc + RL[l * 3 + i] * rot_end[j * 3 + l];
                F.extR_Ri[i * 3 + j] = acc;
            }
            F.exrR_extT[i] = (RL[0 * 3 + i] * c->params.t_LI[0] + RL[1 * 3 + i] * c->params.t_LI[1]) +
                             RL[2 * 3 + i] * c->params.t_LI[2];
            F.pos_end[i] = pos_end[i];
        }
        static_assert(sizeof(livo_imu_pose) == 22 * sizeof(double), "Pose6D row");
        HIP_TRY(hipMemcpyAsync(d_poses, poses, (size_t)n_poses * sizeof(livo_imu_pose), hipMemcpyHostToDevice,
                               c->stream));
        rc = launch_fe_segment(F, c->stream);
        if (!rc) {
            size_t tb = 0;
            rc = prim_inclusive_min_scan_i32(nullptr, &tb, seg, F.seg_rev, n, c->stream);
            if (!rc) rc = ensure_prim(c, tb);
            tb = c->prim_bytes;
            if (!rc) rc = prim_inclusive_min_scan_i32(c->prim_tmp, &tb, seg, F.seg_rev, n, c->stream);
        }
        if (!rc) rc = launch_fe_undistort(F, c->stream);
        if (rc) return rc;
    }
    if (undistorted && n > 0)
        HIP_TRY(hipMemcpyAsync(undistorted, F.raw, (size_t)n * 20, hipMemcpyDeviceToHost, c->stream));
    // downSizeFilterSurf: PCL VoxelGrid::applyFilter
    const float* kept = F.raw;
    int64_t n_kept = n;
    if (leaf_size > 0.f && n > 0) {
        const unsigned init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
        HIP_TRY(hipMemcpyAsync(mm, init, sizeof(init), hipMemcpyHostToDevice, c->stream));
        rc = launch_fe_minmax(F.raw, n, 5, mm, c->stream);
        if (rc) return rc;
        unsigned hm[6];
        HIP_TRY(hipMemcpyAsync(hm, mm, sizeof(hm), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        float mn[3], mx[3];
        auto dec = [](unsigned o) {
            const unsigned u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
            float f;
            std::memcpy(&f, &u, 4);
            return f;
        };
        for (int k = 0; k < 3; k++) {
            mn[k] = dec(hm[k]);
            mx[k] = dec(hm[3 + k]);
        }
        const float inv = 1.0f / leaf_size;  // inverse_leaf_size_
        const int64_t dx = static_cast<int64_t>((mx[0] - mn[0]) * inv) + 1;
        const int64_t dy = static_cast<int64_t>((mx[1] - mn[1]) * inv) + 1;
        const int64_t dz = static_cast<int64_t>((mx[2] - mn[2]) * inv) + 1;
        if ((dx * dy * dz) <= static_cast<int64_t>(0x7FFFFFFF)) {  // else PCL returns the input
            int max_b[3], div_b[3];
            for (int k = 0; k < 3; k++) {
                F.min_b[k] = static_cast<int>(std::floor(mn[k] * inv));
                max_b[k] = static_cast<int>(std::floor(mx[k] * inv));
                div_b[k] = max_b[k] - F.min_b[k] + 1;
            }
            F.divb_mul[0] = 1;
            F.divb_mul[1] = div_b[0];
            F.divb_mul[2] = div_b[0] * div_b[1];
            F.inv_leaf = inv;
            const int64_t cells = (int64_t)div_b[0] * div_b[1] * div_b[2];
            int bits = 1;
            while (bits < 32 && ((int64_t)1 << bits) < cells) bits++;
            rc = launch_fe_leaf(F, c->stream);
            if (!rc) {
                size_t tb = 0;
                rc = prim_sort_pairs_u32(nullptr, &tb, F.keys, skeys, F.iota, svals, n, bits, c->stream);
                if (!rc) rc = ensure_prim(c, tb);
                tb = c->prim_bytes;
                if (!rc) rc = prim_sort_pairs_u32(c->prim_tmp, &tb, F.keys, skeys, F.iota, svals, n, bits, c->stream);
            }
            if (!rc) rc = launch_fe_runs(F, c->stream);
            if (!rc) rc = ivox_scan(c, F.flags, F.vid, n);
            if (rc) return rc;
            uint32_t tail[2];
            HIP_TRY(hipMemcpyAsync(&tail[0], F.vid + n - 1, 4, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipMemcpyAsync(&tail[1], F.flags + n - 1, 4, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            const int64_t n_vox = (int64_t)tail[0] + tail[1];
            rc = launch_fe_starts(F, c->stream);
            if (!rc) rc = launch_fe_centroid(F, n_vox, c->stream);
            if (rc) return rc;
            kept = F.down;
            n_kept = n_vox;
        }
    }
    if (n_down) *n_down = n_kept;
    if (down) {
        if (down_cap < n_kept) return LIVO_E_RANGE;
        if (n_kept > 0) HIP_TRY(hipMemcpyAsync(down, kept, (size_t)n_kept * 20, hipMemcpyDeviceToHost, c->stream));
    }
    c->fe_raw = F.raw;  // feats_undistort stays resident until the next frame (livo_frame_to_world)
    c->fe_n = n;
    return scan_create_device(c, kept, 5, n_kept, scan_id);
}

int livo_vio_params_default(livo_vio_params* p) {
    if (!p) return LIVO_E_INVALID;
    std::memset(p, 0, sizeof(*p));
    // camera_pinhole_resize.yaml
    p->cam.width = 640;
    p->cam.height = 512;
    p->cam.fx = 431.795259219;
    p->cam.fy = 431.550090267;
    p->cam.cx = 310.833037316;
    p->cam.cy = 266.985989326;
    p->cam.d[0] = -0.0944205499243979;
    p->cam.d[1] = 0.0946727677776504;
    p->cam.d[2] = -0.00807970960613932;
    p->cam.d[3] = 8.07461209775283e-05;
    p->R_ci[0] = p->R_ci[4] = p->R_ci[8] = 1.0;
    p->img_point_cov = 10.0;  // laser_mapping.cpp:976
    p->patch_size = 4;        // laser_mapping.cpp:1015
    p->max_iterations = 4;    // origin_laserMapping.cpp:1208 (NUM_MAX_ITERATIONS)
    return LIVO_OK;
}

int livo_vio_update(livo_ctx* c, const livo_vio_params* p, const uint8_t* image, int32_t width, int32_t height,
                    const double* pos, const int32_t* levels, const float* patches, int64_t n, livo_state* state,
                    const livo_state* prior, float* errors, livo_vio_stats* stats) {
    if (!c || !p || !state || n < 0 || width <= 0 || height <= 0 || !image ||
        (n > 0 && (!pos || !levels || !patches)) || p->patch_size < 1 || p->patch_size > 8 ||
        p->max_iterations < 0 || !(p->img_point_cov > 0.0))
        return LIVO_E_INVALID;
    for (int64_t i = 0; i < n; i++)
        if (levels[i] < 0 || levels[i] > 8) return LIVO_E_INVALID;
    if (n > (int64_t)0x7FFFFFFF - 256) return LIVO_E_RANGE;
    if (set_device(c)) return LIVO_E_HIP;
    const int pst = p->patch_size * p->patch_size;
    const int nblk = (int)std::max<int64_t>(1, (n + 255) / 256);
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t b_img = al((size_t)width * height), b_pos = al((size_t)std::max<int64_t>(n, 1) * 24),
                 b_lev = al((size_t)std::max<int64_t>(n, 1) * 4),
                 b_pat = al((size_t)std::max<int64_t>(n, 1) * 3 * pst * 4),
                 b_par = al((size_t)nblk * kVioCols * 8), b_err = al((size_t)std::max<int64_t>(n, 1) * 4),
                 b_slot = al(sizeof(VioSlot));
    const size_t total = b_img + b_pos + b_lev + b_pat + b_par + b_err + b_slot;
    if (total > c->vio_bytes) {
        if (c->vio_buf) (void)hipFree(c->vio_buf);
        c->vio_buf = nullptr;
        c->vio_bytes = 0;
        if (hipMalloc(&c->vio_buf, total) != hipSuccess) return LIVO_E_OOM;
        c->vio_bytes = total;
    }
    char* q = (char*)c->vio_buf;
    uint8_t* d_img = (uint8_t*)q; q += b_img;
    double* d_pos = (double*)q; q += b_pos;
    int32_t* d_lev = (int32_t*)q; q += b_lev;
    float* d_pat = (float*)q; q += b_pat;
    double* d_par = (double*)q; q += b_par;
    float* d_err = (float*)q; q += b_err;
    VioSlot* d_slot = (VioSlot*)q;
    VioSlot hs;
    std::memset(&hs, 0, sizeof(hs));
    hs.state = *state;
    hs.prior = prior ? *prior : *state;
    HIP_TRY(hipMemcpyAsync(d_img, image, (size_t)width * height, hipMemcpyHostToDevice, c->stream));
    if (n > 0) {
        HIP_TRY(hipMemcpyAsync(d_pos, pos, (size_t)n * 24, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(d_lev, levels, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(d_pat, patches, (size_t)n * 3 * pst * 4, hipMemcpyHostToDevice, c->stream));
    }
    HIP_TRY(hipMemcpyAsync(d_slot, &hs, sizeof(hs), hipMemcpyHostToDevice, c->stream));
    if (n > 0) HIP_TRY(hipMemsetAsync(d_err, 0, (size_t)n * 4, c->stream));  // errors: 0 until an iteration runs
    VioParams P{};
    P.img = d_img;
    P.w = width;
    P.h = height;
    P.fx = p->cam.fx; P.fy = p->cam.fy; P.cx = p->cam.cx; P.cy = p->cam.cy;
    std::memcpy(P.d, p->cam.d, sizeof(P.d));
    P.distortion = std::fabs(p->cam.d[0]) > 0.0000001 ? 1 : 0;  // vikit: distortion_ = |d0| > 1e-7
    P.n = (int32_t)n;
    P.ps = p->patch_size;
    P.pos = d_pos;
    P.levels = d_lev;
    P.patches = d_pat;
    std::memcpy(P.Rci, p->R_ci, sizeof(P.Rci));
    std::memcpy(P.Pci, p->P_ci, sizeof(P.Pci));
    // init() (lidar_selection.cpp:44-55): Jdphi_dR = Rci, Jdp_dR = -Rci [Pic]x, Pic = -Rci^T Pci
    std::memcpy(P.Jdphi_dR, p->R_ci, sizeof(P.Jdphi_dR));
    double Pic[3];
    for (int a = 0; a < 3; a++)
        Pic[a] = -((p->R_ci[0 * 3 + a] * p->P_ci[0] + p->R_ci[1 * 3 + a] * p->P_ci[1]) + p->R_ci[2 * 3 + a] * p->P_ci[2]);
    const double tmp[9] = {0.0, -Pic[2], Pic[1], Pic[2], 0.0, -Pic[0], -Pic[1], Pic[0], 0.0};
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++)
            P.Jdp_dR[a * 3 + b] = ((-p->R_ci[a * 3 + 0]) * tmp[0 * 3 + b] + (-p->R_ci[a * 3 + 1]) * tmp[1 * 3 + b]) +
                                  (-p->R_ci[a * 3 + 2]) * tmp[2 * 3 + b];
    P.img_cov = p->img_point_cov;
    P.max_iter = p->max_iterations;
    P.nblk = nblk;
    P.partial = d_par;
    P.perr = d_err;
    P.slot = d_slot;
    int rc = LIVO_OK;
    for (int level = 2; level >= 0 && !rc; level--) {  // ComputeJ (:970-974)
        P.level = level;
        rc = launch_vio_begin(P, level, c->stream);
        for (int it = 0; it < p->max_iterations && !rc; it++) rc = launch_vio_iter(P, c->stream);
    }
    if (!rc) rc = launch_vio_end(P, c->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(&hs, d_slot, sizeof(hs), hipMemcpyDeviceToHost, c->stream));
    if (errors && n > 0) HIP_TRY(hipMemcpyAsync(errors, d_err, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (n > 0) *state = hs.state;
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        for (int k = 0; k < 3; k++) {
            stats->iterations[k] = hs.ctrl.iters[k];
            stats->updates[k] = hs.ctrl.updates[k];
            stats->last_error[k] = hs.ctrl.level_error[k];
        }
        stats->cov_updated = hs.ctrl.cov_updated;
        stats->n_meas = hs.ctrl.n_meas;
        stats->out_of_frame = (int64_t)hs.ctrl.oof;
    }
    return LIVO_OK;
}

int livo_map_add_points(livo_ctx* c, const float* xyz, int64_t n, int64_t stride_bytes, float ds, int downsample_on,
                        livo_map_add_stats* stats) {
    if (!c || n < 0 || (n > 0 && !xyz)) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    if (downsample_on && !(ds > 0.f && std::isfinite(ds))) return LIVO_E_INVALID;
    if (stride_bytes == 0) stride_bytes = 3 * sizeof(float);
    if (stride_bytes < (int64_t)(3 * sizeof(float))) return LIVO_E_INVALID;
    if (!c->has_map) return LIVO_E_NOMAP;
    if (set_device(c)) return LIVO_E_HIP;
    int rc = dyn_activate(c);
    if (!rc) rc = dyn_add_scratch(c, std::max<int64_t>(n, 1));
    if (rc) return rc;
    if (n > 0) {
        std::vector<float> h((size_t)n * 4);
        const char* base = (const char*)xyz;
        for (int64_t i = 0; i < n; i++) {
            const float* p = (const float*)(base + i * stride_bytes);
            h[4 * i] = p[0]; h[4 * i + 1] = p[1]; h[4 * i + 2] = p[2]; h[4 * i + 3] = 0.f;
        }
        HIP_TRY(hipMemcpy(c->dyn.W, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    return dyn_add(c, n, ds, downsample_on != 0, stats);
}

int livo_map_delete_boxes(livo_ctx* c, const float* boxes, int64_t nb, int64_t* deleted) {
    if (!c || nb < 0 || (nb > 0 && !boxes)) return LIVO_E_INVALID;
    if (any_inflight(c)) return LIVO_E_BUSY;  // submitted batches are collected first
    if (!c->has_map) return LIVO_E_NOMAP;
    if (set_device(c)) return LIVO_E_HIP;
    if (deleted) *deleted = 0;
    int rc = dyn_activate(c);
    if (rc || nb == 0) return rc;
    DynDev& d = c->dyn;
    if (nb > d.box_cap) {
        dev_free(d.boxes);
        d.box_cap = 0;
        if (dev_alloc(&d.boxes, (size_t)nb * 6)) return LIVO_E_OOM;
        d.box_cap = nb;
    }
    HIP_TRY(hipMemcpyAsync(d.boxes, boxes, (size_t)nb * 6 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(d.ctr, 0, kDynCtrN * sizeof(unsigned long long), c->stream));
    rc = launch_dyn_delete_boxes(d.all, d.alive, d.n_ids, d.boxes, nb, d.ctr + kDynDeleted, c->stream);
    if (rc) return rc;
    unsigned long long cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, d.ctr + kDynDeleted, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    d.n_alive -= (int64_t)cnt;
    rc = dyn_rebuild(c);
    if (rc) return rc;
    if (deleted) *deleted = (int64_t)cnt;
    return LIVO_OK;
}

int livo_map_dump(livo_ctx* c, float* xyz, int32_t* ids, int64_t cap, int64_t* n) {
    if (!c || !n || cap < 0) return LIVO_E_INVALID;
    if (!c->has_map) return LIVO_E_NOMAP;
    if (set_device(c)) return LIVO_E_HIP;
    HIP_TRY(hipStreamSynchronize(c->stream));
    std::vector<float> p;
    std::vector<int32_t> id;
    if (c->dyn.active) {
        const DynDev& d = c->dyn;
        std::vector<float> all((size_t)d.n_ids * 4);
        std::vector<uint8_t> alive((size_t)d.n_ids);
        if (d.n_ids > 0) {
            HIP_TRY(hipMemcpy(all.data(), d.all, all.size() * sizeof(float), hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(alive.data(), d.alive, alive.size(), hipMemcpyDeviceToHost));
        }
        for (int64_t k = 0; k < d.n_ids; k++)
            if (alive[(size_t)k]) {
                p.insert(p.end(), &all[(size_t)k * 4], &all[(size_t)k * 4] + 3);
                id.push_back((int32_t)k);
            }
    } else {  // the static map: its search structure's points (x, y, z, index) by index
        const int64_t M = c->map_points;
        const float* src = c->knn_kind >= 1 ? c->gpts : c->lpts;
        std::vector<float> pts((size_t)M * 4);
        if (M > 0) HIP_TRY(hipMemcpy(pts.data(), src, pts.size() * sizeof(float), hipMemcpyDeviceToHost));
        p.resize((size_t)M * 3);
        id.resize((size_t)M);
        for (int64_t k = 0; k < M; k++) {
            uint32_t ix;
            std::memcpy(&ix, &pts[(size_t)k * 4 + 3], 4);
            ix &= kIdxMask;
            if ((int64_t)ix >= M) return LIVO_E_HIP;
            std::memcpy(&p[(size_t)ix * 3], &pts[(size_t)k * 4], 12);
            id[ix] = (int32_t)ix;
        }
    }
    *n = (int64_t)id.size();
    if (!xyz && !ids) return LIVO_OK;
    if (cap < *n) return LIVO_E_RANGE;
    if (xyz && !p.empty()) std::memcpy(xyz, p.data(), p.size() * sizeof(float));
    if (ids && !id.empty()) std::memcpy(ids, id.data(), id.size() * sizeof(int32_t));
    return LIVO_OK;
}

int livo_map_last_add_stats(livo_ctx* c, livo_map_add_stats* out) {
    if (!c || !out) return LIVO_E_INVALID;
    *out = c->dyn.last;
    return LIVO_OK;
}

int livo_frame_to_world(livo_ctx* c, int32_t scan_id, const livo_state* state, livo_raw_point* out, int64_t cap,
                        int64_t* n_out) {
    if (!c || !state || !n_out) return LIVO_E_INVALID;
    const float* src;
    int64_t n;
    int stride;
    const int32_t* perm = nullptr;
    if (scan_id < 0) {
        src = c->fe_raw;
        n = c->fe_raw ? c->fe_n : 0;
        stride = 5;
    } else {
        ScanBuf* s = get_scan(c, scan_id);
        if (!s) return LIVO_E_NOSCAN;
        src = s->pts;
        n = s->n;
        stride = 4;
        perm = s->d_perm;
    }
    *n_out = n;
    if (!out || n == 0) return LIVO_OK;
    if (cap < n) return LIVO_E_RANGE;
    if (set_device(c)) return LIVO_E_HIP;
    WorldParams W;
    std::memcpy(W.rot, state->rot, sizeof(W.rot));
    std::memcpy(W.pos, state->pos, sizeof(W.pos));
    std::memcpy(W.R_LI, c->params.R_LI, sizeof(W.R_LI));
    std::memcpy(W.t_LI, c->params.t_LI, sizeof(W.t_LI));
    int rc = ensure_scratch(c, (size_t)n * 5 * sizeof(float));
    if (rc) return rc;
    float* d_out = (float*)c->scratch;
    rc = launch_to_world(src, n, stride, perm, W, d_out, c->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, d_out, (size_t)n * 5 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return LIVO_OK;
}

int livo_sync(livo_ctx* c) {
    if (!c) return LIVO_E_INVALID;
    if (set_device(c)) return LIVO_E_HIP;
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (const BatchLane& B : c->lane)  // submitted batches run on their lanes' streams
        for (int k = 0; k < kMaxGroups && B.st[k]; k++) HIP_TRY(hipStreamSynchronize(B.st[k]));
    if (c->cp_stream) HIP_TRY(hipStreamSynchronize(c->cp_stream));  // asynchronous uploads
    if (c->up_stream) HIP_TRY(hipStreamSynchronize(c->up_stream));
    return LIVO_OK;
}

}  // extern "C"

extern "C" int livo_debug_map_rebuilds(livo_ctx* c, int64_t out[4]) {
    if (!c || !out) return LIVO_E_INVALID;
    out[0] = c->dyn.rebuilds_sorted;
    out[1] = c->dyn.rebuilds_merged;
    out[2] = c->dyn.wide_redos;
    out[3] = c->dyn.rebuilds_fused;
    return LIVO_OK;
}
