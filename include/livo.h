/*
 * livo.h — C ABI of the MI355X-native LIO scan-to-map IEKF hot path.
 *
 * Drop-in boundary for FAST-LIVO's scan-to-map update.  The
 * reference has no function boundary of its own for this path: the work lives
 * in private members of LaserMapping with implicit state.  Each entry point
 * below replaces one of them (reference paths under snowflakezzz/FAST-LIVO-noted):
 *
 *   livo_map_build      ← KD_TREE::Build            include/ikd-Tree/ikd_Tree.cpp:337-348
 *                         (called at src/laser_mapping.cpp:134-142 for the first scan)
 *   livo_knn            ← KD_TREE::Nearest_Search   include/ikd-Tree/ikd_Tree.cpp:350-380
 *   livo_scan_upload    ← feats_down_body handed to h_share_model
 *                                                   src/laser_mapping.cpp:129-131
 *   livo_h_share        ← LaserMapping::h_share_model(MatrixXd&, VectorXd&)
 *                                                   include/laser_mapping.h:83,
 *                                                   src/laser_mapping.cpp:485-644
 *   livo_iekf_update    ← the IEKF loop inlined in LaserMapping::Run
 *                                                   src/laser_mapping.cpp:171-238
 *   livo_iekf_update_batch ← the same for independent scans (scan farm, §8e)
 *   livo_ivox_*         ← faster_lio::IVox, the compiled default k-NN backend
 *                                                   include/ivox3d/ivox3d.h:37-305
 *   livo_map_incremental ← LaserMapping::map_incremental (iVox and ikd-Tree branches)
 *                                                   src/laser_mapping.cpp:329-389
 *   livo_map_add_points / livo_map_delete_boxes ← KD_TREE::Add_Points / Delete_Point_Boxes
 *                                                   include/ikd-Tree/ikd_Tree.cpp:382-457, 501-521
 *   livo_vio_update     ← LidarSelector::ComputeJ / UpdateState (VIO photometric update)
 *                                                   src/lidar_selection.cpp:748-978
 *   livo_scan_preprocess ← ImuProcess::UndistortPcl (per point) + downSizeFilterSurf
 *                                                   src/IMU_Processing.cpp:340-378,
 *                                                   src/laser_mapping.cpp:129-130
 *
 * Conventions
 *   - plain pointers and sizes only; no C++ or torch types cross the ABI;
 *   - every function returns int: LIVO_OK (0) or a negative LIVO_E_* code;
 *     nothing throws across the ABI (livo_error_string() explains a code);
 *   - matrices are row-major doubles (the C++ facade in
 *     fast-livo-noted_amd/host/ converts to/from Eigen-style column-major);
 *   - host pointers are read/written synchronously before return;
 *   - a livo_ctx owns one HIP stream, the device-resident map and scans, and
 *     scratch; calls on one ctx are NOT thread-safe (use one ctx per host
 *     thread / GPU, as the reference uses one LaserMapping per process).
 *   - there is no CPU fallback: every compute entry point runs on the GPU and
 *     fails with LIVO_E_HIP if no device is usable.
 */
#ifndef LIVO_H
#define LIVO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 5: livo_ivox_info grew add_passes (round 4).
 * 4: livo_timings grew the per-evaluation fields (eval_ms ... gap_ms), LIVO_E_BUSY
 *    and the submit / wait pair were added (round 3); a binary built against 3
 *    passes a smaller livo_timings. */
#define LIVO_ABI_VERSION 6
#define LIVO_DIM_STATE 18        /* DIM_STATE, include/common_lib.h:32 */
#define LIVO_NUM_MATCH_POINTS 5  /* NUM_MATCH_POINTS, include/common_lib.h:37 */
#define LIVO_MAX_EVALS 16        /* max h_share/solve evaluations per scan update */

enum {
    LIVO_OK = 0,
    LIVO_E_INVALID = -1,   /* bad argument (null pointer, negative size, ...) */
    LIVO_E_HIP = -2,       /* HIP runtime error (no device, launch failure) */
    LIVO_E_NOMAP = -3,     /* map not built */
    LIVO_E_NOSCAN = -4,    /* unknown / released scan id */
    LIVO_E_OOM = -5,       /* device allocation failed */
    LIVO_E_RANGE = -6,     /* size beyond the supported range */
    LIVO_E_CAPACITY = -7,  /* capacity exceeded (reserved) */
    LIVO_E_BUSY = -8       /* batches in flight (livo_iekf_update_batch_submit) */
};

typedef struct livo_ctx livo_ctx;

/* Hot-path parameters (defaults = reference defaults, src/laser_mapping.cpp:945-1116). */
typedef struct livo_params {
    double laser_point_cov;  /* LASER_POINT_COV, laser_mapping.cpp:975 (0.001)          */
    double R_LI[9];          /* Lidar_rot_to_IMU (row-major), default identity          */
    double t_LI[3];          /* Lidar_offset_to_IMU, default 0                           */
    double max_residual;     /* compaction gate |pd2| <= 2.0, laser_mapping.cpp:552      */
    float plane_threshold;   /* esti_plane threshold 0.1f, laser_mapping.cpp:530         */
    float max_nn_sqdist;     /* k-NN gate sqdis[4] > 5 => reject, laser_mapping.cpp:518  */
    int32_t max_iterations;  /* NUM_MAX_ITERATIONS (max_iteration, default 4, :968)      */
    int32_t flags;           /* reserved, must be 0                                      */
} livo_params;

/* StatesGroup (include/common_lib.h:518-603), row-major. */
typedef struct livo_state {
    double rot[9];      /* rot_end (IMU->world)  */
    double pos[3];      /* pos_end               */
    double vel[3];      /* vel_end               */
    double bias_g[3];
    double bias_a[3];
    double gravity[3];
    double cov[LIVO_DIM_STATE * LIVO_DIM_STATE];
} livo_state;

/* Per-scan-update statistics (the reference logs these ad hoc, laser_mapping.cpp:164-238). */
typedef struct livo_iter_stats {
    int32_t iterations;   /* h_share + solve evaluations performed            */
    int32_t knn_passes;   /* evaluations with nearest_search_en               */
    int32_t converged;    /* flg_EKF_converged at exit                        */
    int32_t rematch_num;
    int64_t effct_feat_num[LIVO_MAX_EVALS];
    double solution[LIVO_MAX_EVALS][LIVO_DIM_STATE]; /* state delta per evaluation */
    double res_mean[LIVO_MAX_EVALS];                 /* res_mean_last per evaluation */
} livo_iter_stats;

typedef struct livo_map_info {
    int64_t num_points;   /* M                                                    */
    int32_t depth;        /* tree levels                                          */
    int32_t ball_chunks;  /* anchor chunks the ball runs were built in (0: none)  */
    int64_t num_slots;    /* heap-ordered node slots (2^depth - 1)                */
    int64_t device_bytes; /* HBM bytes held by the map                            */
    int64_t ball_entries; /* entries of the ball runs (0: the cell runs only)     */
} livo_map_info;

/* Optional per-point outputs of livo_h_share (any pointer may be NULL). */
typedef struct livo_point_out {
    float* normvec;       /* N*4: plane n.x,n.y,n.z and pd2 (normvec->points[i], :537-541)      */
    uint8_t* selected;    /* N:   point_selected_surf[i] && res_last[i] <= 2.0 (:552)            */
    int32_t* nn_idx;      /* N*5: map indices (input order of livo_map_build), -1 pad           */
    float* nn_sqdist;     /* N*5: squared distances (pointSearchSqDis), +inf pad                */
    float* world_xyz;     /* N*3: feats_down_world (pointBodyToWorld, :508)                      */
    int64_t* visits;      /* 1:   k-NN nodes visited over all points (the V_ref yardstick)       */
    /* laserCloudOri / corr_normvect (:547-561): the effective points (selected and
     * |pd2| <= 2), compacted in the caller's point order; capacity N each. */
    float* ori_xyz;       /* n_ori*3: body points (laserCloudOri)                                */
    float* corr_normvec;  /* n_ori*4: their plane normal and pd2 (corr_normvect)                 */
    int64_t* n_ori;       /* 1:   effct_feat_num                                                 */
} livo_point_out;

/* Device time of the kernels of the last livo_iekf_update* call (profiling mode only).
 * knn_* describe the first evaluation's k-NN of the whole batch (pilot pass +
 * pilot-seeded pass + their tie replays, both streams), in which every point of
 * every scan is searched: the dominant kernels.  The other times are summed
 * over the streams (they overlap). */
typedef struct livo_timings {
    double knn_ms;         /* first-evaluation k-NN of the batch, device wall time     */
    double rematch_knn_ms; /* k-NN launches of later evaluations (rematch)             */
    double plane_ms;       /* plane fit + Jacobian + reduction + 18x18 solve (fused)   */
    double solve_ms;       /* 0: the solve runs in the plane pass's last block         */
    int64_t knn_launches;  /* first-evaluation k-NN phases timed (1 per call)          */
    int64_t knn_visits;    /* tree nodes those searches visited (pilot-seeded: < V_ref) */
    int64_t knn_queries;   /* points those launches processed                          */
    int64_t effct_points;  /* effective points of the first evaluation                 */
    int64_t knn_replays;   /* queries recomputed by the exact tie-order replay (all passes) */
    int64_t knn_points;    /* map points those launches read (cell grid; 0 for tree passes) */
    /* level 2, fused evaluation: device time of each evaluation launch (max over
     * the stream groups) and the scans that searched in it; the batch from its
     * first copy to its last, and the device idle time since the previous
     * batch ended (host time between calls; 0 for the first profiled batch).
     * Then knn_ms = eval_ms[0], rematch_knn_ms = the evaluations after the
     * first that searched, plane_ms = those that did not. */
    double eval_ms[LIVO_MAX_EVALS];
    int32_t eval_searched[LIVO_MAX_EVALS];
    int32_t n_evals;
    int32_t reserved_;
    double batch_ms;
    double gap_ms;
} livo_timings;

int livo_abi_version(void);
const char* livo_error_string(int code);
int livo_params_default(livo_params* p);

int livo_ctx_create(int device, const livo_params* p, livo_ctx** out);
int livo_ctx_destroy(livo_ctx* ctx);
int livo_ctx_set_params(livo_ctx* ctx, const livo_params* p);
/* Device timing of livo_iekf_update* (livo_last_timings): 0 off; 1 the first
 * search of the batch only (two events per stream group); 2 also every
 * evaluation's k-NN / plane / solve stages (costs ~10% of throughput). */
int livo_ctx_set_profiling(livo_ctx* ctx, int level);
int livo_last_timings(livo_ctx* ctx, livo_timings* out);

/* Build the device map from M host points (x,y,z floats at xyz + i*stride_bytes).
 * Same tree as KD_TREE::Build on the same input order. Replaces any previous map. */
int livo_map_build(livo_ctx* ctx, const float* xyz, int64_t M, int64_t stride_bytes);
int livo_map_get_info(livo_ctx* ctx, livo_map_info* out);

/* Exact k-NN (k <= 5) of n host queries; idx/sqdist are n*k, ascending. */
int livo_knn(livo_ctx* ctx, const float* q_xyz, int64_t n, int32_t k, int32_t* idx, float* sqdist);

/* Copy a body-frame scan (feats_down_body) to HBM; it stays resident until released. */
int livo_scan_upload(livo_ctx* ctx, const float* xyz, int64_t N, int64_t stride_bytes, int32_t* scan_id);
/* livo_scan_upload without waiting for the device: the points are packed into a
 * pinned staging buffer (xyz is free again on return), then copied and ordered
 * on the context's upload stream beside the batches in flight.  A batch using
 * the scan waits for that on the device; any other call on it, on the host.
 * (The reference hands each frame's feats_down_body to h_share_model,
 * src/laser_mapping.cpp:129-131: the upload of frame k+1 can run under frame k.) */
int livo_scan_upload_async(livo_ctx* ctx, const float* xyz, int64_t N, int64_t stride_bytes, int32_t* scan_id);
/* livo_scan_upload_async for n scans in one pass (xyz[b]: N[b] points at
 * stride_bytes, scan_ids[b] out): one staging copy, then one bounds pass, one
 * key pass, one stable sort of the whole batch and one gather on the upload
 * stream; each scan is stored exactly as livo_scan_upload stores it.  From
 * page-locked memory (livo_host_register) with stride 12 the copy engine reads
 * the caller's arrays directly (no host copy): keep them unchanged until a batch
 * that uses the scans returns (or livo_sync); otherwise they are free on return. */
int livo_scan_upload_batch_async(livo_ctx* ctx, const float* const* xyz, const int64_t* N, int32_t n,
                                 int64_t stride_bytes, int32_t* scan_ids);
/* Page-lock (hipHostRegister) / release a caller's host buffer, e.g. the point
 * arrays a scan farm uploads from; unregister waits for the device first. */
int livo_host_register(livo_ctx* ctx, void* p, size_t bytes);
int livo_host_unregister(livo_ctx* ctx, void* p);
/* Release a resident scan: LIVO_E_BUSY while a submitted batch that holds it is
 * not collected; other batches may be in flight. */
int livo_scan_release(livo_ctx* ctx, int32_t scan_id);

/* The neighbour cache of a resident scan: the k = 5 nearest map points of each
 * point from the last search on it (Nearest_Points, laser_mapping.h:165, in
 * Nearest_Search's ascending PointType_CMP order, ikd_Tree.cpp:350-380).
 * idx: N x 5 map indices (-1 pad); sqdist: N x 5 (+inf pad); either may be NULL.
 * LIVO_E_NOSCAN if the scan was never searched. */
int livo_scan_neighbors(livo_ctx* ctx, int32_t scan_id, int32_t* idx, float* sqdist);

/* One h_share_model evaluation on a resident scan at the given state.
 * nearest_search_en != 0 runs the k-NN; otherwise the neighbours cached by the
 * last search on this scan are reused (Nearest_Points, laser_mapping.h:165).
 * HTH (9x9, row-major) and HTL (9) as HPH/HPL of the reference. */
int livo_h_share(livo_ctx* ctx, int32_t scan_id, const livo_state* state, int nearest_search_en,
                 double HTH[81], double HTL[9], int64_t* effct_feat_num, const livo_point_out* out);

/* Full iterated update of one scan (laser_mapping.cpp:171-238): state in/out,
 * prior = state_propagat (NULL: prior = input state). stats may be NULL. */
int livo_iekf_update(livo_ctx* ctx, int32_t scan_id, livo_state* state, const livo_state* prior,
                     livo_iter_stats* stats);

/* n independent scan updates in one batched pass (states/priors/stats arrays of n).
 * The ids must be distinct (LIVO_E_INVALID otherwise): a scan's neighbour cache
 * belongs to one update at a time. */
int livo_iekf_update_batch(livo_ctx* ctx, int32_t n, const int32_t* scan_ids, livo_state* states,
                           const livo_state* priors, livo_iter_stats* stats);

/* The same batched update, split into enqueue and collect, so a scan farm keeps
 * the next batch queued on the device while the host collects the last one
 * (no replacement in the reference, which updates one scan per frame in
 * LaserMapping::Run; this is the farm of SURVEY.md §8e).  submit copies
 * states / priors (NULL: prior = state) at the call and returns a ticket;
 * wait(ticket) blocks until that batch is done and writes its states and
 * stats (may be NULL).  At most LIVO_MAX_INFLIGHT batches per context are
 * submitted and not yet waited for (LIVO_E_BUSY beyond), and a scan may be in
 * one of them only (LIVO_E_INVALID).  While a batch is in flight its scans
 * may not be released, and the map may not be rebuilt or changed (LIVO_E_BUSY),
 * and livo_scan_neighbors of one of its scans returns LIVO_E_BUSY.  submit
 * needs the fused ikd-Tree path (the default: LIVO_BACKEND_IKDTREE, no
 * LIVO_FUSED=0 / LIVO_KNN_KIND override): otherwise it returns LIVO_E_INVALID
 * before queuing anything, and livo_iekf_update_batch does the same update
 * synchronously. */
#define LIVO_MAX_INFLIGHT 2
int livo_iekf_update_batch_submit(livo_ctx* ctx, int32_t n, const int32_t* scan_ids, const livo_state* states,
                                  const livo_state* priors, int32_t* ticket);
int livo_iekf_update_batch_wait(livo_ctx* ctx, int32_t ticket, livo_state* states, livo_iter_stats* stats);

/* ------------------------------------------------------------------------
 * IKFoM formulation (the "solve in use-ikfom.hpp"):
 *   state_ikfom                         include/use-ikfom.hpp:12-21 (23 DOF)
 *   h_share_model (legacy h-model)      src/origin_laserMapping.cpp:916-1048
 *   esekf::update_iterated_dyn_share_modified
 *                                       include/IKFoM_toolkit/esekfom/esekfom.hpp:1619-1928
 * The same map, scans and k-NN as above; 12-wide measurement rows [n, A, B, C]
 * (extrinsic estimation on), the manifold (SO3 / S2) Jacobian corrections,
 * per-DOF convergence |dx_i| <= 0.001 (origin_laserMapping.cpp:1231-1233),
 * R = params.laser_point_cov, maximum_iter = params.max_iterations.
 * ------------------------------------------------------------------------ */
#define LIVO_IKFOM_DOF 23

/* state_ikfom: quaternions (w, x, y, z) for rot and offset_R_L_I, the S2
 * gravity as its 3-vector (length 98090/10000), cov = P_ (23x23 row-major). */
typedef struct livo_ikfom_state {
    double pos[3];
    double rot[4];
    double offset_R[4];
    double offset_T[3];
    double vel[3];
    double bg[3];
    double ba[3];
    double grav[3];
    double cov[LIVO_IKFOM_DOF * LIVO_IKFOM_DOF];
} livo_ikfom_state;

typedef struct livo_ikfom_stats {
    int32_t iterations;   /* h_dyn_share + update evaluations                    */
    int32_t knn_passes;   /* evaluations with dyn_share.converge (k-NN search)   */
    int32_t converged;    /* dyn_share.converge at exit                          */
    int32_t t;            /* converged-iteration counter t at exit               */
    int64_t effct_feat_num[LIVO_MAX_EVALS];
    double dx[LIVO_MAX_EVALS][LIVO_IKFOM_DOF];  /* dx_ applied per evaluation */
    double res_mean[LIVO_MAX_EVALS];
} livo_ikfom_stats;

/* The IKFoM iterated update of n resident scans, each starting from its state
 * (x_propagated = the input state, P_propagated = its cov).  stats may be NULL. */
int livo_ikfom_update_batch(livo_ctx* ctx, int32_t n, const int32_t* scan_ids, livo_ikfom_state* states,
                            livo_ikfom_stats* stats);
int livo_ikfom_update(livo_ctx* ctx, int32_t scan_id, livo_ikfom_state* state, livo_ikfom_stats* stats);
/* The IKFoM batch split into enqueue and collect, as livo_iekf_update_batch_submit
 * / _wait (the same LIVO_MAX_INFLIGHT lanes and tickets; a ticket is collected
 * with the wait of its own model). */
int livo_ikfom_update_batch_submit(livo_ctx* ctx, int32_t n, const int32_t* scan_ids, const livo_ikfom_state* states,
                                   int32_t* ticket);
int livo_ikfom_update_batch_wait(livo_ctx* ctx, int32_t ticket, livo_ikfom_state* states, livo_ikfom_stats* stats);

/* ------------------------------------------------------------------------
 * iVox backend: faster_lio::IVox<3, DEFAULT, PointType>
 * (include/laser_mapping.h:65), the k-NN backend of the reference's default
 * build (CMakeLists.txt:15 leaves USE_ikdtree undefined).  With
 * livo_ctx_set_backend(ctx, LIVO_BACKEND_IVOX), livo_h_share and
 * livo_iekf_update[_batch] search the iVox map with
 * GetClosestPoint(point_world, points_near, 5) (laser_mapping.cpp:520): no
 * sqdist gate, a point is matched iff 5 neighbours within 5 m were found
 * (:525), the neighbours are in the order the reference's std::nth_element
 * leaves them, and a point with no candidate keeps its previous
 * Nearest_Points entry (ivox3d.h:165-167).
 * ------------------------------------------------------------------------ */
#define LIVO_BACKEND_IKDTREE 0  /* -DUSE_ikdtree build (CMakeLists.txt:15)            */
#define LIVO_BACKEND_IVOX 1     /* the default build: IVox (laser_mapping.cpp:519-521) */

typedef struct livo_ivox_params {
    float resolution;     /* ivox_grid_resolution (0.2, laser_mapping.cpp:1021)          */
    int32_t nearby_type;  /* ivox_nearby_type: 0 CENTER, 6, 18 (default, :1022-1035), 26 */
    int64_t capacity;     /* Options::capacity_ (1000000, ivox3d.h:57)                   */
} livo_ivox_params;

typedef struct livo_ivox_info {
    int64_t num_points;      /* points held (IVox::NumPoints)                       */
    int64_t num_grids;       /* IVox::NumValidGrids (ivox3d.h:206-209)              */
    int64_t ids_issued;      /* points ever added = the id of the next point        */
    int64_t max_grid_points; /* largest grid                                        */
    int64_t device_bytes;    /* HBM held by the iVox map                            */
    int64_t add_passes;      /* device passes AddPoints took since init: one per    */
                             /* call, more when an LRU victim is re-touched         */
} livo_ivox_info;

int livo_ctx_set_backend(livo_ctx* ctx, int backend);
int livo_ivox_params_default(livo_ivox_params* p);
/* IVox(Options) (ivox3d.h:64-67, laser_mapping.cpp:776): an empty map. */
int livo_ivox_init(livo_ctx* ctx, const livo_ivox_params* p);
/* IVox::AddPoints (ivox3d.h:256-281) of n host points, in order (the first
 * scan's feats_down_body, laser_mapping.cpp:147), with the LRU grid cache:
 * once a new grid takes the grid count to capacity, the grid whose last added
 * point is the oldest is evicted with its points (:270-274).  Point ids
 * continue from ids_issued.  LIVO_E_RANGE (a key beyond the supported cell
 * range) leaves the map unchanged. */
int livo_ivox_add_points(livo_ctx* ctx, const float* xyz, int64_t n, int64_t stride_bytes);
/* IVox::GetClosestPoint(pt, closest_pt, max_num, max_range) (ivox3d.h:132-204)
 * for n host queries: idx / sqdist n*max_num in the reference's order (the
 * nearest first), cnt[i] = neighbours found, -1 when there was no candidate
 * (the reference returns false and leaves its output vector alone). */
int livo_ivox_knn(livo_ctx* ctx, const float* q_xyz, int64_t n, int32_t max_num, double max_range, int32_t* idx,
                  float* sqdist, int32_t* cnt);
int livo_ivox_get_info(livo_ctx* ctx, livo_ivox_info* out);
/* Every point, grid by grid in grids_cache_ order (most recently used grid
 * first, insertion order inside a grid): xyz n*3, ids n, keys n*3 (the grid
 * of each point); any may be NULL.
 * *n = points; LIVO_E_RANGE if cap < *n (nothing written). */
int livo_ivox_dump(livo_ctx* ctx, float* xyz, int32_t* ids, int32_t* keys, int64_t cap, int64_t* n);

/* LaserMapping::map_incremental, iVox branch (laser_mapping.cpp:329-389): the
 * scan's points at `state` (the updated state), the add / no-downsample / skip
 * decision from the scan's neighbour cache, then AddPoints(points_to_add) and
 * AddPoints(point_no_need_downsample) on the device.  cat (may be NULL): per
 * point 0 skipped, 1 added, 2 added without downsampling; counts[2] = the two
 * batch sizes.  ekf_inited = flg_EKF_inited.  iVox backend only. */
int livo_map_incremental(livo_ctx* ctx, int32_t scan_id, const livo_state* state, double filter_size_map_min,
                         int ekf_inited, uint8_t* cat, int64_t counts[2]);
/* Nearest_Points.resize(N) between scans (laser_mapping.cpp:165) keeps the
 * entries of the previous scan's points: dst's point i starts with src's
 * point i's cache (empty for i >= src's size). */
int livo_scan_inherit_neighbors(livo_ctx* ctx, int32_t dst_scan, int32_t src_scan);

/* ------------------------------------------------------------------------
 * Scan front-end: from the raw frame to the resident
 * feats_down_body on the device.
 *   ImuProcess::UndistortPcl, per-point backward propagation
 *                                       src/IMU_Processing.cpp:340-378
 *   downSizeFilterSurf.filter (PCL VoxelGrid)  src/laser_mapping.cpp:129-130
 * ------------------------------------------------------------------------ */
/* The PointXYZINormal fields the front-end reads; curvature = the point's
 * offset time in ms (preprocess.cpp:346). */
typedef struct livo_raw_point {
    float x, y, z, intensity, curvature;
} livo_raw_point;

/* Pose6D (msg/Pose6D.msg, set_pose6d common_lib.h:618-633): one IMU sample of
 * the frame's forward propagation, offset_time in seconds from the frame start. */
typedef struct livo_imu_pose {
    double offset_time;
    double acc[3];
    double gyr[3];
    double vel[3];
    double pos[3];
    double rot[9];  /* row-major */
} livo_imu_pose;

/* Raw frame -> resident scan.  With n_poses >= 2 every point is first moved to
 * the frame-end pose (rot_end, pos_end = state after propagation) through the
 * IMU segment it falls in, exactly as UndistortPcl's backward walk (poses must
 * have non-decreasing offset_time; the first point is re-compensated by every
 * remaining segment, as in the reference); then, for leaf_size > 0, PCL
 * VoxelGrid downsampling (voxel centroids of x, y, z, intensity, curvature in
 * ascending leaf order; a leaf too small for 32-bit indices keeps the input,
 * as PCL does).  The result becomes a resident scan (*scan_id), as
 * livo_scan_upload would.  undistorted (n) and down (down_cap; *n_down = its
 * size) are optional host copies. */
int livo_scan_preprocess(livo_ctx* ctx, const livo_raw_point* raw, int64_t n, const livo_imu_pose* poses,
                         int32_t n_poses, const double rot_end[9], const double pos_end[3], float leaf_size,
                         int32_t* scan_id, livo_raw_point* undistorted, livo_raw_point* down, int64_t down_cap,
                         int64_t* n_down);

/* ------------------------------------------------------------------------
 * VIO photometric update: LidarSelector::ComputeJ and
 * UpdateState (src/lidar_selection.cpp:748-978) for the visual points of
 * sub_sparse_map: per point, patch_size^2 bilinear residuals against its
 * reference patch at pyramid levels 2, 1, 0, the 6-wide Jacobian rows, and
 * the 18-dim iterated update (K1 = (HᵀH + (P / img_point_cov)^-1)^-1), then
 * cov -= G cov.  max_iterations is explicit: the compiled build never
 * assigns LidarSelector::NUM_MAX_ITERATIONS (the legacy pipeline sets it to
 * the LiDAR value, origin_laserMapping.cpp:1208).
 * ------------------------------------------------------------------------ */
/* vikit PinholeCamera (camera yaml: cam_fx ... cam_d0..d3; d[4] = k3). */
typedef struct livo_cam {
    double fx, fy, cx, cy;
    double d[5];
    int32_t width, height;
} livo_cam;

typedef struct livo_vio_params {
    livo_cam cam;
    double R_ci[9];          /* Rci = Rcl * Rli (lidar_selection.cpp:44), row-major */
    double P_ci[3];          /* Pci = Rcl * Pli + Pcl                                */
    double img_point_cov;    /* img_point_cov (10, laser_mapping.cpp:976)             */
    int32_t patch_size;      /* patch_size (4, laser_mapping.cpp:1015), <= 8          */
    int32_t max_iterations;  /* UpdateState iterations per level                      */
} livo_vio_params;

typedef struct livo_vio_stats {
    int32_t iterations[3];   /* per level 2, 1, 0 */
    int32_t updates[3];      /* iterations that updated the state (error did not grow) */
    float last_error[3];     /* UpdateState's return value per level */
    int32_t cov_updated;
    int64_t n_meas;
    int64_t out_of_frame;    /* patch samples outside the image (clamped; the reference reads out of bounds) */
} livo_vio_stats;

int livo_vio_params_default(livo_vio_params* p);
/* image: 8-bit gray, width x height, row stride = width.  pos: n x 3 world
 * positions; search_levels: n; patches: n x 3 x patch_size^2 reference
 * patches (levels 0, 1, 2, Feature::patch_).  state in/out, prior =
 * state_propagat (NULL: the input state).  errors (n, may be NULL) =
 * sub_sparse_map->errors after the last iteration. */
int livo_vio_update(livo_ctx* ctx, const livo_vio_params* p, const uint8_t* image, int32_t width, int32_t height,
                    const double* pos, const int32_t* search_levels, const float* patches, int64_t n,
                    livo_state* state, const livo_state* prior, float* errors, livo_vio_stats* stats);

/* ------------------------------------------------------------------------
 * ikd-Tree incremental map (the USE_ikdtree branch of
 * map_incremental, src/laser_mapping.cpp:383-384, and the ikd-Tree's
 * Delete_Point_Boxes).  The first call turns the built map (cell-grid search
 * structure, the default) into an incremental point set: ids = the build's
 * indices, then the next ids in input order for the points a call leaves in
 * the map.  Later k-NN (livo_knn, livo_h_share, the IEKF loops) search the
 * updated map; queries whose order the reference's tree shape would decide
 * (PointType_CMP ties) come in (distance, x, id) order.
 * livo_map_incremental with LIVO_BACKEND_IKDTREE runs Add_Points(world, true)
 * on the scan at the given state: counts[0] = its return value, counts[1] =
 * points deleted; cat = 1 for every point.
 * ------------------------------------------------------------------------ */
typedef struct livo_map_add_stats {
    int64_t events;     /* Add_Points' return value (tmp_counter, include/ikd-Tree/ikd_Tree.cpp:416,428) */
    int64_t added;      /* points of the call left in the map (new ids, input order)            */
    int64_t deleted;    /* map points removed (Delete_by_range of a downsample box, :414)        */
    int64_t ambiguous;  /* boxes whose kept stored point Search_by_range's order picks (ties)    */
    int64_t deferred;   /* points handled by the in-order pass (box-face rounding cases)         */
    int64_t map_points; /* points in the map after the call                                      */
} livo_map_add_stats;

/* KD_TREE::Add_Points(points, downsample_on) (ikd_Tree.cpp:382-457) with
 * downsample_size (set_downsample_param, :35-40); xyz at xyz + i*stride_bytes. */
int livo_map_add_points(livo_ctx* ctx, const float* xyz, int64_t n, int64_t stride_bytes, float downsample_size,
                        int downsample_on, livo_map_add_stats* stats);
/* KD_TREE::Delete_Point_Boxes (ikd_Tree.cpp:501-521): boxes n_boxes x 6 floats
 * {vertex_min[3], vertex_max[3]} (BoxPointType), half open; *deleted = points removed. */
int livo_map_delete_boxes(livo_ctx* ctx, const float* boxes, int64_t n_boxes, int64_t* deleted);
/* The map's points in id order: *n = count; xyz (cap x 3) and ids (cap) may be
 * NULL, else cap must be >= the count (LIVO_E_RANGE otherwise, *n still set). */
int livo_map_dump(livo_ctx* ctx, float* xyz, int32_t* ids, int64_t cap, int64_t* n);
/* Statistics of the last livo_map_add_points / ikd-Tree livo_map_incremental. */
int livo_map_last_add_stats(livo_ctx* ctx, livo_map_add_stats* out);

/* RGBpointBodyToWorld (src/laser_mapping.cpp:647-660) over laserCloudFullRes
 * (:258-265) at `state`: scan_id < 0 takes the last livo_scan_preprocess frame
 * at full resolution (feats_undistort, dense_map_en; resident until the next
 * frame), scan_id >= 0 a resident scan (feats_down_body, in the caller's point
 * order; intensity 0: a resident scan keeps x, y, z only).  out: n points
 * (world x, y, z; intensity copied; curvature 0), *n = their count; out may be
 * NULL to query the count, else cap >= *n (LIVO_E_RANGE otherwise). */
int livo_frame_to_world(livo_ctx* ctx, int32_t scan_id, const livo_state* state, livo_raw_point* out, int64_t cap,
                        int64_t* n);
int livo_sync(livo_ctx* ctx);
/* Diagnostics: the incremental map's grid rebuilds since the context was made,
 * out[0] by a sort of every id, out[1] by merging the added ids into the grid;
 * out[2] the Add_Points batches redone with 64-bit box keys (a wrapped-key clash),
 * out[3] the merged rebuilds run inside Add_Points' pass (counted in out[1] too). */
int livo_debug_map_rebuilds(livo_ctx* ctx, int64_t out[4]);

#ifdef __cplusplus
}
#endif
#endif /* LIVO_H */
