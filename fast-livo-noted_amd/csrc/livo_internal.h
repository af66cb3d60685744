// livo_internal.h — layouts shared by the host runtime (livo_capi.cpp,
// map_build.cpp) and the CDNA4 kernels (livo_kernels.hip).  Not part of the ABI.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "livo.h"
#include "stl_select.h"

#ifndef LIVO_PTS_PER_THREAD
#define LIVO_PTS_PER_THREAD 1  // plane pass: 1 point per thread (A/B on MI355X: 4 -> 1 = +7 % at config 2)
#endif

// Run entries (cell runs / ball runs, KnnParams::vpts / bpts).  1 (default):
// one 4-B grid position (an index into the cell grid's points, gpts) per
// entry, every run a 4-entry aligned segment, so a run scan reads 8 positions
// (two aligned 16-B loads) and gathers their points from the 16 B x M cell grid
// that stays cache-resident: a quarter of the bytes of 0, which stores the
// point itself (x, y, z, map index bits: 16 B) in every run it belongs to.
#ifndef LIVO_IDX_RUNS
#define LIVO_IDX_RUNS 1
#endif

namespace livo {

#if LIVO_IDX_RUNS
using RunWord = uint32_t;
constexpr int kRunWords = 1;  // words per run entry
#else
using RunWord = float;
constexpr int kRunWords = 4;
#endif
constexpr int kRunPad = 8;    // entries of padding behind the last run (chunk reads)

constexpr int kNN = LIVO_NUM_MATCH_POINTS;  // 5
constexpr int kDim = LIVO_DIM_STATE;        // 18
constexpr int kBlock = 256;                 // threads per block of the per-point kernels
#ifndef LIVO_KNN_BLOCK
#define LIVO_KNN_BLOCK 128
#endif
constexpr int kKnnBlock = LIVO_KNN_BLOCK;   // threads per block of the k-NN pass (LDS stacks)
constexpr int kPtsPerThread = LIVO_PTS_PER_THREAD;  // points per thread of the plane-fit pass
constexpr int kRedCols = 32;                // doubles per block partial (29 used)
constexpr int kRedUsed = 29;                // 21 HTH upper-tri + 6 HTL + residual sum + count
#ifndef LIVO_RED_SHARDS
#define LIVO_RED_SHARDS 8
#endif
constexpr int kRedShards = LIVO_RED_SHARDS;  // first-level shards of a scan's block partials (<= 32)
static_assert(kRedShards >= 1 && kRedShards <= 32, "one shard row per column thread group of the tail");
#ifndef LIVO_MAX_GROUPS
#define LIVO_MAX_GROUPS 4
#endif
constexpr int kMaxGroups = LIVO_MAX_GROUPS;               // stream groups of a batched IEKF update

// ---------------------------------------------------------------------------
// Device map: the ikd-Tree built exactly as KD_TREE::Build (median of the
// longest-extent axis, ikd_Tree.cpp:537-602) stored in heap order (root = 0,
// children 2h+1 / 2h+2) as one 64-B record per node.  A record carries what
// the traversal needs at that node and nothing else: the node point, and the
// bounding boxes of its two children (KD_TREE_NODE::node_range_* of the
// sons, read at ikd_Tree.cpp:867-868 through calc_box_dist).  Record h lives
// at slot h+1 so the two children of a node (2h+1, 2h+2) share one 128-B line.
//
//   a = (x, y, z, meta)      meta = orig_index | left_exists<<30 | right_exists<<31
//   b = (L.minx, L.maxx, L.miny, L.maxy)
//   c = (L.minz, L.maxz, R.minx, R.maxx)
//   d = (R.miny, R.maxy, R.minz, R.maxz)
// ---------------------------------------------------------------------------
struct alignas(16) MapNode {
    float a[4];
    float b[4];
    float c[4];
    float d[4];
};
static_assert(sizeof(MapNode) == 64, "MapNode must be 64 bytes");

constexpr uint32_t kIdxMask = 0x3FFFFFFFu;
constexpr uint32_t kLeftBit = 0x40000000u;
constexpr uint32_t kRightBit = 0x80000000u;
constexpr int64_t kMaxMapPoints = (int64_t)kIdxMask;  // 2^30 - 1
constexpr int kMaxDepth = 31;

// ---------------------------------------------------------------------------
// Leaf map: the search structure of the batched IEKF k-NN passes.  A balanced
// kd-tree over the same points, split by median on the longest extent down to
// a fixed depth D so that every leaf holds ceil/floor(M / 2^D) <= leaf_size
// points; leaf j owns points [j*M >> D, (j+1)*M >> D) of a permuted copy of
// the map stored as float4 (x, y, z, original index bits).  Internal node h
// (heap order, 0 .. 2^D-2) is one 64-B record holding its two sons' boxes in
// the MapNode b/c/d layout.  The point array is padded by 3 points so that a
// leaf chunk of 4 can always be loaded.  It finds the same exact 5 nearest points as the
// ikd-Tree with fewer dependent steps (leaves are scanned with independent
// loads); the answers the reference's heap could order or pick differently
// (ties within PointType_CMP's 1e-10) are flagged and recomputed on the
// reference tree (k_knn_replay), see k_knn_leaf.
// ---------------------------------------------------------------------------
struct alignas(16) LeafNode {
    float b[4];
    float c[4];
    float d[4];
    float pad[4];  // 64 B: one record = one leaf chunk of 4 points (uniform loads)
};
static_assert(sizeof(LeafNode) == 64, "LeafNode must be 64 bytes");
constexpr int kLeafSize = 16;  // default maximum points per leaf

struct HostLeafMap {
    LeafNode* nodes = nullptr;  // 2^depth - 1 internal records
    float* pts = nullptr;       // (M + 3) x 4 floats
    int64_t num_points = 0;
    int32_t depth = 0;          // D: leaves at level D
};
int build_leaf_map(const float* xyz, int64_t M, int64_t stride_bytes, int leaf_size, HostLeafMap* out);
void free_leaf_map(HostLeafMap* m);

// ---------------------------------------------------------------------------
// Cell grid: the other search structure of the batched IEKF (LIVO_KNN_KIND).
// The map's points sorted by cubic cell (edge h, cell c = floor((p - org) / h)),
// each cell a contiguous run, found through an open-addressing hash table of
// 16-B slots {key, start, count}.  A query scans its cell, then whole rings of
// cells around it, each pruned by box distance, until the ring boundary
// certifies the 5 nearest (k_knn_grid) -- a few independent loads per query
// instead of a chain of dependent tree visits.  Equivalence with the reference
// as for the leaf map (C1 / C2, exact replay otherwise).
// ---------------------------------------------------------------------------
struct alignas(16) GridSlot {
    unsigned long long key;  // kGridEmpty: free
    uint32_t start;
    uint32_t count;
};
constexpr unsigned long long kGridEmpty = ~0ull;
constexpr int kGridBias = 1 << 20;  // cell index bias in the key (21 bits per axis)
constexpr int kGridMaxRing = 3;     // cube radius searched for the first 5 points
constexpr int kGridMaxCells = 729;  // stage-2 boxes beyond this: exact replay on the ikd-Tree

struct HostGridMap {
    GridSlot* slots = nullptr;  // 2^log2_slots
    float* pts = nullptr;       // (M + 3) x 4 floats, sorted by cell
    int64_t num_points = 0;
    int32_t log2_slots = 0;
    int64_t cells = 0;          // occupied cells
    float org[3] = {0.f, 0.f, 0.f};
    float h = 1.f;
    float cmax = 0.f;           // largest |coordinate| (bounds the float rounding of cell bounds)
    double ext = 0.0;           // largest axis extent of the map's bounding box
};
// cell_h <= 0: chosen from the map (about ppc_target points per occupied cell, 20 if 0;
// ppc_target < 0: -ppc_target x clamp((M / 1M)^0.3, 1, 4), the cell runs' sizing)
int build_grid_map(const float* xyz, int64_t M, int64_t stride_bytes, float cell_h, HostGridMap* out,
                   float ppc_target = 0.f);
float sample_knn_radius(const HostGridMap& gm, int samples);  // median 5-NN distance of map points
constexpr int64_t kRunPosLimit = 0x7FFFFFFF;  // run entries a search can address (31-bit positions)
constexpr float kVrunPpc = 20.0f;  // cell occupancy of the cell runs at 1M points (0.35 m cells on the config-2 map)
void free_grid_map(HostGridMap* m);

// Cell runs: the search structure of the batched IEKF k-NN on a static map.
// The run of cell c holds every map point of the 3x3x3 cells around c (27x
// the points: 432 MB for a 1M map), sorted by the squared distance rho2 to
// c's centre.  Entry: (x, y, z, map index bits) -- the coordinates and index
// the neighbour record needs, so a search reads nothing else; rho2 is
// recomputed from the entry with the build's float operations (same bits).
// A query takes its own cell's run: one hash probe, one contiguous scan that
// stops at the first entry with rho > |q - centre| + the current bound.

// ---------------------------------------------------------------------------
// iVox map (faster_lio::IVox<3, DEFAULT>, include/ivox3d/ivox3d.h): the
// compiled default k-NN backend of LaserMapping.  Grids (voxels of edge
// `resolution`, key = round(p / resolution)) live in an open-addressing hash
// of 16-B GridSlots {key, start, count}; the points of all grids are one CSR
// array of float4 (x, y, z, id bits), each grid one run in insertion order
// (IVoxNode::points_).  AddPoints rebuilds the CSR in one pass (old runs
// moved, new points appended in input order): the search then reads each
// grid as one contiguous run.  id = insertion sequence number of the point.
// ---------------------------------------------------------------------------
constexpr int kIvBias = 1 << 20;            // key bias (21 bits per axis)
constexpr int kIvMaxKey = kIvBias - 64;     // |cell| limit of stored points
#ifndef LIVO_IV_CAP
#define LIVO_IV_CAP 128
#endif
constexpr int kIvCap = LIVO_IV_CAP;                 // private candidates per query (k_ivox_knn); beyond: overflow pass
constexpr int kIvMaxNearby = 27;

struct IvoxParams {
    GridSlot* slots;          // 2^log2 slots
    const float* pts;         // CSR points, 4 floats each (search) / old points (AddPoints)
    float* npts;              // AddPoints: new CSR
    const float* src;         // AddPoints: points to add (4 floats each), in insertion order
    int64_t n_src;
    int64_t table;            // 2^log2
    uint32_t* addcnt;         // per slot: points added by this batch
    uint32_t* tot;            // per slot: count + addcnt (scan input)
    uint32_t* newstart;       // per slot: start in the new CSR (scan of tot)
    uint32_t* addstart;       // per slot: start of its run in the sorted batch (scan of addcnt)
    uint32_t* slot_of;        // per src point: its slot (table: out of range)
    uint32_t* iota;           // per src point: its index
    const uint32_t* skeys;    // batch sorted by slot (stable)
    const uint32_t* svals;
    unsigned long long* ctr;  // [0] error bits (1 key range, 2 LRU conflict), [1] new grids, [2] max points
                              // per grid, [3] last victim's sorted position, [4] LRU minimum (single eviction)
    int64_t base_id;          // id of src[0]
    float inv_res;            // Options::inv_resolution_ (float of 1.0 / resolution)
    int32_t log2;
    int32_t nearby;           // 1, 7, 19 or 27 nearby grids (NearbyType)
    int32_t max_num;          // GetClosestPoint max_num (<= 5)
    int32_t kind;             // search kernel: -1 by batch size, 0 thread, 1 wave, 2 team (LIVO_IVOX_KIND at livo_ivox_init)
    double range2;            // max_range * max_range
    SelElem* scratch;         // overflow pass: one slice per thread
    int64_t slice;            // elements per slice
    // LRU grid cache (ivox3d.h:256-281): per slot the id of the last point
    // added to the grid (its place in grids_cache_), and within one AddPoints
    // batch the first / last (+1) batch index touching it
    unsigned long long* tlast;
    uint32_t* first;
    uint32_t* lastp1;
    uint8_t* evict;           // per slot: evicted by this batch
};

// IEKF control block (the loop variables of laser_mapping.cpp:166-238).
struct IekfCtrl {
    int32_t stop;         // EKF_stop_flg reached: every later launch for this scan exits
    int32_t search_en;    // nearest_search_en for the next evaluation
    int32_t iter_count;   // iterCount of the next evaluation (starts at -1)
    int32_t rematch_num;
    int32_t converged;    // flg_EKF_converged of the last evaluation
    int32_t n_evals;      // evaluations done
    int32_t max_iter;     // NUM_MAX_ITERATIONS
    int32_t last_search;  // nearest_search_en used by the last evaluation
};

constexpr int kIkDim = LIVO_IKFOM_DOF;  // 23
constexpr int kIkFewRows = kIkDim - 1;  // below 23 effective points the gain is formed in measurement space
constexpr int kIkCols = 192;            // doubles per IKFoM block partial: 92 sums, then their 92 compensations
constexpr int kIkCompOff = 96;          // offset of the compensation terms in a partial
constexpr int kIkUsed = 92;             // 78 HTH upper-tri + 12 HTh + residual sum + count

// IKFoM update state (esekfom.hpp:1619-1928): x_, x_propagated (its cov is
// P_propagated), the converged counter t.
struct alignas(16) IkBlock {
    livo_ikfom_state x;
    livo_ikfom_state xp;
    livo_ikfom_stats stats;
    int32_t t;
    int32_t pad[3];
};

enum SlotModel { kModelLaserMapping = 0, kModelIkfom = 1 };

// Everything one scan update needs on the device (one per batch entry).
struct alignas(128) IekfSlot {
    livo_state state;     // in/out
    livo_state prior;     // state_propagat
    double red[kRedCols];       // last reduced h_share sums (for livo_h_share)
    livo_iter_stats stats;
    IekfCtrl ctrl;
    unsigned long long visits[LIVO_MAX_EVALS];  // k-NN nodes visited (grid: hash slots probed) per evaluation
    unsigned long long scanned[LIVO_MAX_EVALS]; // grid k-NN: map points read per evaluation
    int32_t eval_search[LIVO_MAX_EVALS];
    unsigned hs_ticket;         // reduction shards done in the current pass (the last one solves; IKFoM: blocks)
    int32_t model;              // SlotModel
    unsigned pad_[2];
    // Factors of the state covariance, made by the host when it stages the slot
    // (init_slot; the covariance changes only when the scan's loop stops):
    // S = P(0:6, 0:6) = L L^T (Cholesky, row-major 6x6, zero above the diagonal)
    // and B = P(:, 0:6) L^-T (rows 6..17; rows 0..5 are L).  The solve forms
    // K1(:, 0:6) = B Q^-1 L^T with Q = I6 + L^T C L (SPD) -- see solve_scan.
    // cov_ok 0: S is not numerically SPD or P is not symmetric (the 6x6 LU path).
    double covL[36];
    double covB[(kDim - 6) * 6];
    int32_t cov_ok;
    int32_t pad2_[3];
    // two-level reduction of the block partials (hs_ticket_tail): one ticket per
    // shard, each on a 128-B line of its own (device-scope atomics serialise per line)
    alignas(128) unsigned sh_ticket[kRedShards * 32];
    IkBlock ik;                 // model == kModelIkfom (last: the LaserMapping model copies only the part before it)
};
constexpr size_t kSlotLmBytes = offsetof(IekfSlot, ik);  // bytes of a slot the LaserMapping model reads / writes
constexpr size_t kSlotWbBytes = offsetof(IekfSlot, covL);  // what the host reads back (no factors, no tickets)

// Nearest_Points[i] + pointSearchSqDis for one point: 128 B, written by the
// k-NN pass, read by every plane-fit pass until the next search.
struct alignas(16) NNRec {
    float p[kNN][4];   // x, y, z, squared distance (ascending); +inf pad
    int32_t idx[kNN];  // map indices (input order of livo_map_build), -1 pad
    int32_t cnt;       // neighbours found (< 5 only for maps of < 5 points)
    int32_t flag;      // why the exact replay recomputed it (bits, see k_knn_pass); 0x100: replayed
    int32_t node[kNN]; // heap node ids of the neighbours (seeds of the next search)
};
static_assert(sizeof(NNRec) == 128, "NNRec must be 128 bytes");

// One scan of a batched launch.
struct HsJob {
    const float* pts;     // N x 4 floats (x, y, z, 0), device
    NNRec* nn;            // N neighbour records
    double* partial;      // nblk x kRedCols block partial sums
    IekfSlot* slot;
    float* plane;         // N x 4: esti_plane of the cached neighbours (k_hshare)
    uint8_t* pstate;      // N: 0 not fitted since the last search, 1 no plane, 2 plane
    double* ikrows;       // IKFoM: nblk x kIkFewRows x 13 effective rows (h_x row, h) per block
    uint32_t* ikcnt;      // IKFoM: nblk: effective rows of the block (capped at kIkFewRows + 1)
    uint4* host_slot;     // fused batches: the slot's host-mapped staging copy, written by the solve that
                          // stops the scan (nullptr: the batch copies the slots back itself)
    int32_t n;
    int32_t nblk;
};

// Optional per-point debug outputs (single-scan livo_h_share only).
struct HsDebug {
    float* normvec;   // N x 4
    uint8_t* sel;     // N
    float* world;     // N x 3
};

struct HsParams {
    const HsJob* jobs;
    HsDebug dbg;
    double R_LI[9];
    double t_LI[3];
    double inv_r;           // 1.0 / LASER_POINT_COV
    double max_res;         // 2.0
    float plane_thr;        // 0.1f
    float max_sqd;          // 5.0f
    int32_t force;          // -1: follow ctrl; 0: no search; 1: search
    double lpc;             // LASER_POINT_COV (the IKFoM gain divides P by it)
    int32_t solve;          // 1: the last block of a scan also runs its solve (IEKF loop)
    unsigned* replay_count; // zeroed once per launch (the group's k-NN replay count), may be null
    unsigned* replay_count2;  // iVox: the wave pass's overflow count, zeroed with replay_count (may be null)
};

struct KnnParams {
    const MapNode* nodes;   // slot 0 unused; root at slot 1
    const HsJob* jobs;
    unsigned* replay_count;            // queries flagged for the exact replay (zeroed per pass)
    unsigned long long* replay_list;   // (job << 32) | point
    // iVox: queries the wave-cooperative search could not hold (a grid too large to
    // stream, or a heap select), for the global-memory pass (k_ivox_knn_big); the
    // team search's overflow (replay_list) goes to the wave pass first
    unsigned* replay_count2;
    unsigned long long* replay_list2;
    unsigned long long* replay_total;  // running count of replayed queries (diagnostics)
    double R_LI[9];
    double t_LI[3];
    int32_t has_map;
    int32_t force;          // -1: follow ctrl; 0: skip; 1: search
    int32_t depth;          // tree levels (LDS stack entries of the full search)
    int64_t n_nodes;        // heap slots of the ikd-Tree records (the replay's subtree loads stay below)
    int32_t identity;       // 1: pts are world points already (livo_knn)
    int32_t nb;             // blocks per scan (set by the launcher)
    int32_t xcd_chunk;      // k_iekf_eval block order: XCD-interleaved chunks of this many blocks (0: one range per XCD)
    int32_t ldepth;         // leaf map depth D
    const LeafNode* lnodes; // leaf map internal records
    const float* lpts;      // leaf map points, 4 floats each (x, y, z, index bits)
    int64_t lM;             // leaf map points
    const GridSlot* gslots; // cell grid
    const float* gpts;
    float gorg[3];
    float gh;               // cell edge
    float geps;             // cell-bound slack for float rounding of the cell assignment
    int32_t glog2;          // log2 of the hash table size
    const GridSlot* vslots; // cell runs (null: the cell walk of grid_search)
    const RunWord* vpts;    // run entries (LIVO_IDX_RUNS: grid positions; else x, y, z, map index bits)
    int32_t vlog2;
    const GridSlot* bslots; // ball runs (null: the cell runs only); entries in bpts
    const RunWord* bpts;
    int32_t blog2;
    float bh;               // anchor cell edge (origin gorg)
    float bcert2;           // certified if the final scan bound b satisfies b * b <= bcert2
    IvoxParams iv;          // iVox backend (LIVO_BACKEND_IVOX)
    int32_t canon;          // incremental map: flagged queries -> k_knn_canon instead of the ikd-Tree replay
    // the points the runs index (grid positions): the cell grid's on a static map;
    // the incremental map's base set (deleted ones with x = NaN) with its runs
    const float* rpts;
    int32_t dyn_runs;       // the incremental map searched on runs: marks skipped, delta grid, no cell walk
    int32_t dlog2;
    const GridSlot* dslots; // delta grid (null: no point added since the base); points in dpts
    const float* dpts;
    const GridSlot* dvslots;  // the delta grid's cell runs (null: none); entries = positions in dpts
    const RunWord* dvidx;
    int32_t dvlog2;
};

struct SolveParams {
    IekfSlot* slots;
    const HsJob* jobs;
    unsigned* replay_count;  // zeroed by block 0 for the next k-NN pass (may be null)
    int32_t mode;           // 0: reduce + solve + control; 1: reduce only (livo_h_share)
};

// Host-side map build (map_build.cpp).
struct HostMap {
    MapNode* nodes = nullptr;  // (num_slots + 1) records, slot 0 unused
    int64_t num_points = 0;
    int64_t num_slots = 0;
    int32_t depth = 0;
};
int build_host_map(const float* xyz, int64_t M, int64_t stride_bytes, HostMap* out);
void free_host_map(HostMap* m);

// Kernel launchers (livo_kernels.hip).  All asynchronous on `stream`.
size_t knn_lds_bytes(int depth);
// Reference-order k-NN on the ikd-Tree records (livo_knn, livo_h_share): the
// visiting order of KD_TREE::Search, so the node visits it counts are V_ref.
int launch_knn_pass(const KnnParams& p, int n_jobs, int64_t max_n, void* stream);
// Batched IEKF k-NN on the leaf map; seeded: rematch pass bounded by the
// point's previous neighbours.  Both are followed by the exact tie replay.
int launch_knn_leaf(const KnnParams& p, int n_jobs, int64_t max_n, bool seeded, void* stream);
// tile: the LDS-tiled variant (one wave per block), same answers
int launch_knn_grid(const KnnParams& p, int n_jobs, int64_t max_n, bool seeded, bool tile, void* stream);
int launch_hshare(const HsParams& p, int n_jobs, int max_nblk, bool first, void* stream);
// One whole IEKF evaluation (search if due + plane pass + reduction + solve) per launch.
#ifndef LIVO_EVAL_BLOCK
#define LIVO_EVAL_BLOCK 256
#endif
constexpr int kEvalBlock = LIVO_EVAL_BLOCK;  // threads (points) per block of k_iekf_eval
int launch_iekf_eval(const KnnParams& kp, const HsParams& hp, int n_jobs, int64_t max_n, bool first, void* stream);
int launch_solve_ik(const HsParams& p, int n_jobs, void* stream);
int launch_copy_words(const void* src, void* dst, size_t bytes, void* stream);  // 16-B aligned, bytes % 16 == 0
// bytes [o0, o0 + n0) and [o1, o1 + n1) of src to the same offsets of dst, one launch (16-B aligned)
int launch_copy_ranges(const void* src, void* dst, size_t o0, size_t n0, size_t o1, size_t n1, void* stream);
// IKFoM plane pass (12-wide rows) with the manifold update in each scan's last block.
int launch_hshare_ik(const HsParams& p, int n_jobs, int max_nblk, bool first, void* stream);
int launch_solve(const SolveParams& p, int n_jobs, void* stream);

// iVox (ivox_kernels.hip).  AddPoints in stages, so the host can check the
// new grid count against the LRU capacity before anything is moved:
// insert (keys -> slots, counts) | rollback, or prepare -> scans + stable sort
// by slot -> move (old runs) -> place (new points, input order) -> fix.
int launch_ivox_clear(GridSlot* slots, int64_t table, void* stream);
int launch_ivox_insert(const IvoxParams& p, void* stream);
int launch_ivox_rollback(const IvoxParams& p, void* stream);
int launch_ivox_prepare(const IvoxParams& p, void* stream);
int launch_ivox_move(const IvoxParams& p, void* stream);
int launch_ivox_place(const IvoxParams& p, void* stream);
int launch_ivox_fix(const IvoxParams& p, void* stream);
int launch_ivox_rehash(const GridSlot* old_slots, const unsigned long long* old_t, int64_t old_table, GridSlot* slots,
                       unsigned long long* tlast, int log2, void* stream);
// LRU eviction at capacity: the new grids' first touches and the old grids'
// (last id, slot) compacted for sorting; victims marked; slots dropped; ids committed.
int launch_ivox_newfirst(const IvoxParams& p, uint32_t* out, unsigned long long* n, void* stream);
int launch_ivox_oldkeys(const IvoxParams& p, unsigned long long* keys, uint32_t* slot, unsigned long long* n,
                        void* stream);
int launch_ivox_untouched(const IvoxParams& p, const uint32_t* sorted_slot, int64_t n, uint32_t* flags, void* stream);
int launch_ivox_oldfirst(const IvoxParams& p, const uint32_t* sorted_slot, int64_t n, uint32_t* out, void* stream);
int launch_ivox_victims(const IvoxParams& p, const uint32_t* sorted_slot, const uint32_t* rank, int64_t n, int64_t ev,
                        uint32_t j_first, void* stream);
int launch_ivox_tcur_min(const IvoxParams& p, void* stream);
int launch_ivox_mark_min(const IvoxParams& p, void* stream);
int launch_ivox_drop(const IvoxParams& p, void* stream);
int launch_ivox_commit(const IvoxParams& p, void* stream);
// GetClosestPoint of every point of every job (+ the overflow pass).
int launch_ivox_knn(const KnnParams& p, int n_jobs, int64_t max_n, bool later, int64_t overflow_threads,
                    void* stream);
// rocPRIM wrappers (prims.hip); temp == nullptr queries the scratch size.
int prim_sort_pairs_u32(void* temp, size_t* temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                        const uint32_t* vals_in, uint32_t* vals_out, int64_t n, int bits, void* stream);
int prim_exclusive_scan_u32(void* temp, size_t* temp_bytes, const uint32_t* in, uint32_t* out, int64_t n,
                            void* stream);
// map_incremental decision (laser_mapping.cpp:329-389): ordered[2N] holds the
// points_to_add at their point index and point_no_need_downsample at N + index,
// flags[2N] marks them; cat (stored order, may be null) 0 skip / 1 add / 2 no-downsample.
struct MapIncrParams {
    const float* pts;         // scan body points (stored order), N x 4
    const NNRec* nn;
    const int32_t* perm;      // stored position -> caller index
    const IekfSlot* slot;     // its state = the updated state
    double R_LI[9];
    double t_LI[3];
    float* ordered;           // 2N x 4 floats
    uint32_t* flags;          // 2N
    uint8_t* cat;             // N (stored order) or null
    double fs;                // filter_size_map_min
    int32_t n;
    int32_t ekf_inited;
};
int launch_map_incr(const MapIncrParams& p, void* stream);
int launch_compact(const float* ordered, const uint32_t* flags, const uint32_t* pos, int64_t n, float* dense,
                   void* stream);
// Scan front-end (frontend_kernels.hip).
struct FrontParams {
    float* raw;               // n x 5 floats: x, y, z, intensity, curvature (ms); xyz de-skewed in place
    int64_t n;
    const double* poses;      // np x 22 (Pose6D rows)
    int32_t np;
    int32_t* seg;             // n: last segment starting before point n-1-k (reversed)
    int32_t* seg_rev;         // n: its prefix minimum = the segment of point n-1-k
    double R_LI[9], t_LI[3];
    double extR_Ri[9];        // R_LI^T rot_end^T
    double exrR_extT[3];      // R_LI^T t_LI
    double pos_end[3];
    // VoxelGrid
    float inv_leaf;
    int32_t min_b[3];
    int32_t divb_mul[3];
    uint32_t* keys;           // leaf index per point
    uint32_t* iota;
    const uint32_t* skeys;    // sorted by leaf (stable)
    const uint32_t* svals;
    uint32_t* flags;          // run heads in sorted order
    uint32_t* vid;            // scan of flags
    uint32_t* starts;         // n_vox + 1 run starts
    float* down;              // n_vox x 5 centroids
};
int launch_fe_segment(const FrontParams& F, void* stream);
int launch_fe_undistort(const FrontParams& F, void* stream);
int launch_fe_minmax(const float* pts, int64_t n, int stride, unsigned* minmax, void* stream);
int launch_fe_leaf(const FrontParams& F, void* stream);
int launch_fe_runs(const FrontParams& F, void* stream);
int launch_fe_starts(const FrontParams& F, void* stream);
int launch_fe_centroid(const FrontParams& F, int64_t n_vox, void* stream);
int launch_fe_morton(const float* pts, int64_t n, int stride, const unsigned* minmax, float scale,
                     uint32_t* codes, uint32_t* iota, void* stream);
// A batch of at most kFeSegMax scans built in one pass (kernel argument table).
constexpr int kFeSegMax = 16;  // (the scan index rides in the 32-bit sort key's bits 27..30)
struct FeSegs {
    int64_t off[kFeSegMax];  // first point of scan b in the packed batch
    int64_t n[kFeSegMax];
    float* pts4[kFeSegMax];
    int32_t* iperm[kFeSegMax];
    int32_t* perm[kFeSegMax];
    void* nn[kFeSegMax];
    uint8_t* pstate[kFeSegMax];
};
// A batch's points copied by a kernel from host-mapped (page-locked) caller
// arrays into the packed device staging (dst + 3 * off[b]).
struct FeSrc {
    const float* src[kFeSegMax];  // device addresses of the mapped host arrays
    int64_t off[kFeSegMax];
    int64_t n[kFeSegMax];
};
int launch_fe_copy_seg(const FeSrc& S, int n_scans, int64_t max_n, float* dst, void* stream);
int launch_fe_build_seg(const float* pts, const FeSegs& S, int n_scans, int64_t max_n, unsigned* minmax, float scale,
                        uint32_t* codes, uint32_t* iota, void* stream);
int launch_fe_gather_seg(const float* pts, const FeSegs& S, int n_scans, int64_t max_n, const uint32_t* sorted,
                         void* stream);
int launch_fe_gather(const float* pts, int64_t n, int stride, const uint32_t* perm, float* pts4, int32_t* iperm,
                     void* stream);
struct WorldParams {
    double rot[9], pos[3], R_LI[9], t_LI[3];
};
// RGBpointBodyToWorld of n points (stride floats each, x y z [intensity]) -> n x 5 floats.
int launch_to_world(const float* src, int64_t n, int stride, const int32_t* perm, const WorldParams& W, float* out5,
                    void* stream);
// laserCloudOri / corr_normvect compaction in the caller's order (stored-order sel / normvec / points).
int launch_ori_flags(const uint8_t* sel, const int32_t* perm, int64_t n, uint32_t* flags, void* stream);
int launch_ori_scatter(const float* pts4, const float* normvec, const uint8_t* sel, const int32_t* perm,
                       const uint32_t* pos, int64_t n, float* ori3, float* corr4, void* stream);
int prim_inclusive_min_scan_i32(void* temp, size_t* temp_bytes, const int32_t* in, int32_t* out, int64_t n,
                                void* stream);
int prim_sort_pairs_u64(void* temp, size_t* temp_bytes, const unsigned long long* keys_in,
                        unsigned long long* keys_out, const uint32_t* vals_in, uint32_t* vals_out, int64_t n,
                        int bits, void* stream);

// VIO photometric update (vio_kernels.hip).
struct VioCtrl {
    int32_t level;          // pyramid level of the current UpdateState (2, 1, 0)
    int32_t end;            // EKF_end of the current level
    int32_t iteration;      // iterations run in the current level
    int32_t pinv_ready;     // Pinv holds (cov / img_point_cov)^-1
    float last_error;       // UpdateState's last_error
    float pad_;
    int32_t iters[3], updates[3];
    float level_error[3];   // UpdateState's return value per level (2, 1, 0)
    int32_t cov_updated;
    int64_t n_meas;
    unsigned long long oof; // patch samples outside the image
};
struct alignas(16) VioSlot {
    livo_state state;
    livo_state old_state;
    livo_state prior;       // state_propagat
    double G6[kDim * 6];    // G(:, 0:6) of the last update
    double Pinv[kDim * kDim];
    VioCtrl ctrl;
    unsigned ticket;        // blocks done in the current pass (the last one solves)
    unsigned pad_[3];
};
constexpr int kVioCols = 28;  // per-block partial: 21 HTH upper-tri + 6 HTz (+ 1 spare)
struct VioParams {
    const uint8_t* img;
    int32_t w, h;
    double fx, fy, cx, cy, d[5];
    int32_t distortion;     // vikit distortion_ = |d0| > 1e-7
    int32_t n, ps;
    const double* pos;      // n x 3
    const int32_t* levels;  // n
    const float* patches;   // n x 3 ps^2
    double Rci[9], Pci[3], Jdphi_dR[9], Jdp_dR[9];
    double img_cov;
    int32_t max_iter, level, nblk, pad_;
    double* partial;        // nblk x kVioCols
    float* perr;            // n patch errors (sub_sparse_map->errors)
    VioSlot* slot;
};
int launch_vio_begin(const VioParams& p, int level, void* stream);
int launch_vio_iter(const VioParams& p, void* stream);
int launch_vio_end(const VioParams& p, void* stream);

// ikd-Tree incremental map (ikd_incr_kernels.hip):
// KD_TREE::Add_Points / Delete_Point_Boxes on the map's point set, then the
// cell grid rebuilt from the surviving points.  Counters in DynAddParams::ctr:
enum { kDynEvents = 0, kDynDeleted = 1, kDynAmbig = 2, kDynDeferred = 3, kDynError = 4, kDynDirty = 5,
       kDynAbsMax = 6, kDynRuns = 7, kDynTomb = 8, kDynAliveCnt = 9, kDynAdded = 10, kDynBig = 11, kDynKept = 12,
       kDynRErr = 13, kDynRRuns = 14, kDynRNa = 15, kDynCtrN = 16 };  // 13-15: the merged rebuild run with Add_Points
constexpr uint32_t kDynDirtyCap = 4096;  // dirty-box set slots; past half full every point takes the sequential pass
constexpr int kDynCtrPad = 16;           // ctr, then the dirty-box set (one allocation, one clear)
static_assert(kDynCtrN <= kDynCtrPad, "ctr overlaps the dirty-box set");
struct DynAddParams {
    const float* W;             // n points to add (x, y, z, -), PointToAdd order
    int64_t n;
    float ds;                   // downsample_size
    int32_t downsample;
    const GridSlot* gslots;     // the map's cell grid before this call
    const float* gpts;
    int32_t glog2;
    float gorg[3];
    float gh, ginv, geps;
    int64_t base;               // ids issued before this call
    uint8_t* alive;             // per id
    unsigned long long* keys;   // n: box key per point
    uint32_t* iota;
    const unsigned long long* skeys;  // sorted by box key (stable)
    const uint32_t* svals;
    float* Ws;                  // n x 4: the points in sorted order (x, y, z, input index bits)
    uint32_t* heads;            // n
    uint32_t* runid;            // n: exclusive scan of heads
    uint32_t* starts;           // runs + 1
    uint32_t* defer;            // n, by point: processed by the sequential pass
    uint32_t* dpos;             // exclusive scan of defer
    uint32_t* dlist;            // deferred points, input order
    uint32_t* keep;             // n, by point: left in the map by this call
    float* seq;                 // sequential pass: its kept points (4 floats each)
    unsigned long long* dirty;  // dirty box keys: an open-addressing set of dirty_cap slots (0: empty)
    uint32_t dirty_cap;
    unsigned long long* ctr;    // kDynCtrN counters
    uint32_t* keys32;           // n: the box key wrapped to 10 bits per axis (null: sort the 64-bit keys)
    uint32_t* skeys32;          // n: sorted
    unsigned long long* skeys_w;  // = skeys (k_scan_boxes writes the 64-bit keys in sorted order)
    uint32_t* bigs;             // the crowded boxes (runs), listed by k_scan_boxes (count: ctr[kDynBig])
    uint32_t* dlist_u;          // the deferred points, unordered (k_add_box; count ctr[kDynDeferred])
    uint32_t* klist;            // the box winners, unordered (k_add_box; count ctr[kDynKept])
    // map_incremental: k_add_prep first takes the scan's stored points to the
    // world frame into W (pointBodyToWorld at rot / pos; null: W is filled)
    const float* wpts;          // scan body points, stored order (4 floats each)
    const int32_t* wperm;       // stored position -> caller index
    double wrot[9], wpos[3], R_LI[9], t_LI[3];
};
int launch_add_prep(const DynAddParams& p, void* stream);
int launch_add_group(const DynAddParams& p, void* stream);
int launch_add_finish(const DynAddParams& p, float* all, uint8_t* alive, void* stream);
int launch_dyn_seed(const float* gpts, int64_t M, float* all, uint8_t* alive, void* stream);
int launch_dyn_cellkeys(const float* all, const uint8_t* alive, int64_t n_ids, const float* org, float inv,
                        unsigned long long* keys, uint32_t* vals, unsigned long long* ctr, void* stream);
int launch_dyn_gather(const unsigned long long* skeys, const uint32_t* sids, int64_t na, const float* all, float* gpts,
                      uint32_t* heads, void* stream);
int launch_dyn_runs(const uint32_t* heads, const uint32_t* runid, int64_t na, uint32_t* starts,
                    unsigned long long* nruns, void* stream);
// dcells (optional): the cell count on the device, `cells` the bound the table was sized for
int launch_dyn_slots(const unsigned long long* skeys, const uint32_t* starts, int64_t cells, GridSlot* slots, int log2,
                     void* stream, const unsigned long long* dcells = nullptr, unsigned long long* err = nullptr);
// The incremental path of the grid rebuild (k_dyn_merge, ikd_incr_kernels.hip).
struct DynMergeParams {
    const float* gpts;                 // the old grid, na_old points (x, y, z, id bits) in (key, id) order
    int64_t na_old;
    const uint32_t* rank;              // na_old + 1: exclusive scan of its survivors
    const uint8_t* alive;
    const unsigned long long* nkeys;   // m: the new ids' cell keys, sorted (dead: ~0)
    const uint32_t* nidx;              // m: their index from g0
    int64_t m, g0;
    const float* all;
    float* out;                        // na + 3: the merged grid
    unsigned long long* okeys;         // na: its cell keys
    int64_t na;
    float org[3];
    float inv;
    unsigned long long* ctr;
    const unsigned long long* dm = nullptr;  // optional: m on the device (m above: the bound); na follows
    unsigned long long* dna = nullptr;       // with dm: na written here
};
// One-launch exclusive scans (decoupled look-back, ikd_incr_kernels.hip): the
// context's ticket counter and status words (never cleared: each call tags
// its words with a new epoch).
struct ScanCtx {
    unsigned long long* ticket = nullptr;  // device: tickets issued
    unsigned long long* status = nullptr;  // device: status_cap words
    int64_t status_cap = 0;
    unsigned long long issued = 0, epoch = 1;
    unsigned long long* err = nullptr;     // where a look-back that gives up sets bit 64
};
int scan_tiles(int64_t n);
// rank[i] = old-grid survivors before i, i <= na_old (the flags read in the scan)
int launch_scan_flags(ScanCtx& sc, const float* gpts, int64_t na_old, const uint8_t* alive, uint32_t* rank,
                      void* stream, GridSlot* clr = nullptr, int64_t clr_n = 0);
// runs of equal keys -> starts, *nruns (k_run_heads + a scan + k_dyn_runs)
int launch_scan_runs(ScanCtx& sc, const unsigned long long* keys, int64_t n, uint32_t* starts,
                     unsigned long long* nruns, void* stream, const unsigned long long* dn = nullptr);
// Add_Points' box runs: heads, a scan and starts in one launch
int launch_scan_boxes(ScanCtx& sc, const DynAddParams& p, void* stream);
constexpr int kNewSortMax = 2048;  // k_dyn_newsort: new ids keyed and sorted in one workgroup
int launch_dyn_newsort(const float* all, const uint8_t* alive, int64_t m, const float* org, float inv,
                       unsigned long long* skeys, uint32_t* svals, unsigned long long* ctr, void* stream,
                       const unsigned long long* dm = nullptr, unsigned long long* rerr = nullptr);
int launch_dyn_merge(const DynMergeParams& p, void* stream);
int launch_dyn_delete_boxes(const float* all, uint8_t* alive, int64_t n_ids, const float* boxes, int64_t nb,
                            unsigned long long* cnt, void* stream);

// Cell runs on the device from the cell grid (gpts: n / 27 points): entry e's
// rho2 (bits) and e; the run key of pass-1-sorted entries; the final runs
// (x, y, z, map index bits) and the run heads.
// ball runs (k_br_*, ikd_incr_kernels.hip)
int launch_br_count(const float* gpts, int64_t n, const float org[3], float h, float rmax, uint32_t* cnt,
                    unsigned long long* total, void* stream, int x0 = -(1 << 30), int x1 = 1 << 30);
int launch_br_emit(const float* gpts, int64_t n, const float org[3], float h, float rmax, const uint32_t* off,
                   uint32_t* rho_bits, unsigned long long* keys, uint32_t* pt, uint32_t* iota, void* stream,
                   int x0 = -(1 << 30), int x1 = 1 << 30);
// ball runs built in chunks of anchors: each chunk's runs as {key, start >> 2, count}, then the table
int launch_run_trip(const unsigned long long* skeys, const uint32_t* starts, const uint32_t* pstart, int64_t nruns,
                    unsigned long long base, GridSlot* trip, void* stream);
int launch_trip_slots(const GridSlot* trip, int64_t nruns, GridSlot* slots, int log2, void* stream);
int launch_br_gather_keys(const unsigned long long* keys, const uint32_t* e1, int64_t n, unsigned long long* out,
                          void* stream);
int launch_br_fill(const float* gpts, const uint32_t* pt, const uint32_t* e2, const unsigned long long* skeys,
                   int64_t n, float* bpts, uint32_t* heads, void* stream);
int launch_add_u32(uint32_t* v, int64_t n, uint32_t add, void* stream);
int launch_cr_rho(const float* gpts, int64_t n, const float org[3], float h, uint32_t* rho_bits, uint32_t* iota,
                  void* stream);
int launch_cr_key(const float* gpts, const uint32_t* e1, int64_t n, const float org[3], float h,
                  unsigned long long* keys, void* stream);
int launch_cr_fill(const float* gpts, const uint32_t* e2, const unsigned long long* skeys, int64_t n,
                   const float org[3], float h, float* vpts, uint32_t* heads, void* stream);
// Index runs (LIVO_IDX_RUNS): the run heads of key-sorted entries; each run's
// length rounded up to 4; every entry's grid position (pt ? pt[e2[i]] :
// e2[i] / 27) at pstart[run] + its offset in the run; the runs' hash slots
// {key, pstart, length}.
int launch_run_heads(const unsigned long long* skeys, int64_t n, uint32_t* heads, void* stream);
// Runs on the incremental map: rpos[id] = position of id in rpts (base_n points);
// k_dyn_tomb marks every base point deleted since (!alive) in rpts (x = NaN) and counts the
// marks in ctr[kDynTomb]; k_count_alive counts alive[0, n) into ctr[kDynAliveCnt].
int launch_dyn_rpos(const float* rpts, int64_t base_n, uint32_t* rpos, void* stream);
int launch_dyn_tomb(float* rpts, uint32_t* rpos, const uint8_t* alive, int64_t base_ids, unsigned long long* ctr,
                    void* stream);
int launch_count_alive(const uint8_t* alive, int64_t n, unsigned long long* ctr, void* stream);
int launch_run_plen(const uint32_t* starts, int64_t nruns, uint32_t* plen, void* stream);
int launch_run_place(const uint32_t* e2, const uint32_t* pt, const uint32_t* heads, const uint32_t* runid,
                     const uint32_t* starts, const uint32_t* pstart, int64_t n, uint32_t* out, void* stream);
int launch_run_slots(const unsigned long long* skeys, const uint32_t* starts, const uint32_t* pstart, int64_t nruns,
                     GridSlot* slots, int log2, void* stream);

// Nearest_Points carried over by point index (laser_mapping.cpp:165 resize keeps entries).
int launch_inherit_nn(NNRec* dst, const int32_t* dst_perm, int64_t n_dst, const NNRec* src,
                      const int32_t* src_iperm, int64_t n_src, void* stream);

}  // namespace livo
