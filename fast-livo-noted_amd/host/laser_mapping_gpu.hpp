// laser_mapping_gpu.hpp — C++ facade over the livo C ABI with the call shape
// of the reference's scan-to-map update (snowflakezzz/FAST-LIVO-noted).
//
// The reference keeps this path inside LaserMapping as private members with
// implicit state:
//
//   ikdtree.Build(feats_down_world->points)      src/laser_mapping.cpp:134-142
//   feats_down_body / feats_down_size            src/laser_mapping.cpp:129-131
//   void h_share_model(MatrixXd &HPH, VectorXd &HPL)
//                                                include/laser_mapping.h:83,
//                                                src/laser_mapping.cpp:485-644
//   the IEKF loop in Run()                       src/laser_mapping.cpp:166-238
//
// LaserMappingGpu holds the same state under the same names (state,
// state_propagat, nearest_search_en, effct_feat_num) and exposes the same two
// operations, so a maintainer swaps the bodies of h_share_model() and of the
// iteration loop for calls into this class.  Matrix and state
// arguments are templates: any type with Eigen's accessors works (the
// reference's MatrixXd / VectorXd / StatesGroup with rot_end(i,j),
// pos_end(i), cov(i,j), ...), and nothing here needs Eigen itself.
//
// Errors: the reference has no error path (it would divide by zero at
// laser_mapping.cpp:561 on an empty match set); the facade throws
// livo::Error carrying the LIVO_E_* code of the failing C-ABI call.
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "livo.h"

namespace livo {

class Error : public std::runtime_error {
public:
    Error(const char* what, int code)
        : std::runtime_error(std::string(what) + ": " + livo_error_string(code)), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

inline void check(int rc, const char* what) {
    if (rc != LIVO_OK) throw Error(what, rc);
}

// StatesGroup (include/common_lib.h:518-603) <-> livo_state (row-major).
template <class S>
livo_state to_livo_state(const S& s) {
    livo_state o{};
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) o.rot[3 * i + j] = s.rot_end(i, j);
        o.pos[i] = s.pos_end(i);
        o.vel[i] = s.vel_end(i);
        o.bias_g[i] = s.bias_g(i);
        o.bias_a[i] = s.bias_a(i);
        o.gravity[i] = s.gravity(i);
    }
    for (int i = 0; i < LIVO_DIM_STATE; i++)
        for (int j = 0; j < LIVO_DIM_STATE; j++) o.cov[LIVO_DIM_STATE * i + j] = s.cov(i, j);
    return o;
}

template <class S>
void from_livo_state(const livo_state& o, S& s) {
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) s.rot_end(i, j) = o.rot[3 * i + j];
        s.pos_end(i) = o.pos[i];
        s.vel_end(i) = o.vel[i];
        s.bias_g(i) = o.bias_g[i];
        s.bias_a(i) = o.bias_a[i];
        s.gravity(i) = o.gravity[i];
    }
    for (int i = 0; i < LIVO_DIM_STATE; i++)
        for (int j = 0; j < LIVO_DIM_STATE; j++) s.cov(i, j) = o.cov[LIVO_DIM_STATE * i + j];
}

class LaserMappingGpu {
public:
    // Defaults are the reference's (livo_params_default); `device` is the HIP ordinal.
    explicit LaserMappingGpu(int device = 0, const livo_params* params = nullptr) {
        livo_params p;
        if (params) {
            p = *params;
        } else {
            check(livo_params_default(&p), "livo_params_default");
        }
        check(livo_ctx_create(device, &p, &ctx_), "livo_ctx_create");
        check(livo_params_default(&params_), "livo_params_default");
        params_ = p;
    }
    ~LaserMappingGpu() {
        if (ctx_) {
            if (scan_id_ >= 0) livo_scan_release(ctx_, scan_id_);
            livo_ctx_destroy(ctx_);
        }
    }
    LaserMappingGpu(const LaserMappingGpu&) = delete;
    LaserMappingGpu& operator=(const LaserMappingGpu&) = delete;

    // ikdtree.Build(points): x,y,z floats at xyz + i*stride (PointType: stride 48).
    void build_map(const float* xyz, int64_t M, int64_t stride_bytes = 3 * sizeof(float)) {
        check(livo_map_build(ctx_, xyz, M, stride_bytes), "livo_map_build");
    }

    // The compiled default backend: ivox_ = make_shared<IVoxType>(ivox_options_)
    // (laser_mapping.cpp:776, options :1021-1035); h_share_model / iterate then
    // search the iVox map (laser_mapping.cpp:519-521).
    void use_ivox(const livo_ivox_params* options = nullptr) {
        check(livo_ivox_init(ctx_, options), "livo_ivox_init");
        check(livo_ctx_set_backend(ctx_, LIVO_BACKEND_IVOX), "livo_ctx_set_backend");
        ivox_ = true;
    }
    // ivox_->AddPoints(points) (the first scan, laser_mapping.cpp:145-150).
    void ivox_add_points(const float* xyz, int64_t n, int64_t stride_bytes = 3 * sizeof(float)) {
        check(livo_ivox_add_points(ctx_, xyz, n, stride_bytes), "livo_ivox_add_points");
    }

    // feats_down_body for the next update (laser_mapping.cpp:129-131, 164-166).
    // Nearest_Points.resize keeps the previous scan's entries, which only the
    // iVox search can leave in place (ivox3d.h:165-167): carried over then.
    void set_scan(const float* body_xyz, int64_t N, int64_t stride_bytes = 3 * sizeof(float)) {
        int32_t id = -1;
        check(livo_scan_upload(ctx_, body_xyz, N, stride_bytes, &id), "livo_scan_upload");
        adopt_scan(id, N);
    }

    // The raw frame instead: UndistortPcl's per-point de-skew with the frame's
    // IMU poses (IMU_Processing.cpp:340-378) and downSizeFilterSurf
    // (laser_mapping.cpp:129-130) on the device; `down` (optional, cap
    // down_cap) receives feats_down_body.
    void set_scan_raw(const livo_raw_point* raw, int64_t n, const livo_imu_pose* poses, int32_t n_poses,
                      float filter_size_surf, livo_raw_point* down = nullptr, int64_t down_cap = 0) {
        int32_t id = -1;
        int64_t nd = 0;
        check(livo_scan_preprocess(ctx_, raw, n, poses, n_poses, state.rot, state.pos, filter_size_surf, &id,
                                   nullptr, down, down_cap, &nd),
              "livo_scan_preprocess");
        adopt_scan(id, nd);
    }

    // map_incremental() (laser_mapping.cpp:329-389) at the updated state: the iVox branch
    // (counts = added, added without downsampling) or, on the ikd-Tree backend, Add_Points
    // of every point (:383-384; counts = Add_Points' return value, points deleted).
    void map_incremental(double filter_size_map_min, bool flg_EKF_inited = true) {
        int64_t counts[2] = {0, 0};
        check(livo_map_incremental(ctx_, scan_id_, &state, filter_size_map_min, flg_EKF_inited ? 1 : 0, nullptr,
                                   counts),
              "livo_map_incremental");
        points_added = counts[0];
        points_no_downsample = counts[1];
    }

    template <class S>
    void set_state(const S& s) { state = to_livo_state(s); }
    template <class S>
    void set_state_propagat(const S& s) { state_propagat = to_livo_state(s); }
    template <class S>
    void get_state(S& s) const { from_livo_state(state, s); }

    // h_share_model(HPH, HPL) (laser_mapping.cpp:485-644): HPH is resized to
    // 9x9 and HPL to 9 exactly as the reference does; effct_feat_num is set;
    // the k-NN runs iff nearest_search_en, else cached neighbours are reused.
    template <class MatX, class VecX>
    void h_share_model(MatX& HPH, VecX& HPL) {
        double hth[81], htl[9];
        int64_t eff = 0;
        check(livo_h_share(ctx_, scan_id_, &state, nearest_search_en ? 1 : 0, hth, htl, &eff, nullptr),
              "livo_h_share");
        HPH.resize(9, 9);
        HPL.resize(9);
        for (int i = 0; i < 9; i++) {
            for (int j = 0; j < 9; j++) HPH(i, j) = hth[9 * i + j];
            HPL(i) = htl[i];
        }
        effct_feat_num = eff;
    }

    // The iteration loop of Run() (laser_mapping.cpp:166-238) for the current
    // scan: state is updated in place from prior state_propagat; the final
    // covariance update (I - G) P is included.  Returns the loop's statistics.
    livo_iter_stats iterate() {
        livo_iter_stats st{};
        check(livo_iekf_update(ctx_, scan_id_, &state, &state_propagat, &st), "livo_iekf_update");
        flg_EKF_converged = st.converged != 0;
        if (st.iterations > 0) effct_feat_num = st.effct_feat_num[st.iterations - 1];
        return st;
    }

    livo_ctx* ctx() const { return ctx_; }
    const livo_params& params() const { return params_; }

    // Reference member names (laser_mapping.h): the implicit state of the path.
    livo_state state{};
    livo_state state_propagat{};
    bool nearest_search_en = true;
    bool flg_EKF_converged = false;
    int64_t effct_feat_num = 0;
    int64_t feats_down_size = 0;
    int64_t points_added = 0, points_no_downsample = 0;  // last map_incremental

private:
    void adopt_scan(int32_t id, int64_t N) {
        if (scan_id_ >= 0) {
            if (ivox_) check(livo_scan_inherit_neighbors(ctx_, id, scan_id_), "livo_scan_inherit_neighbors");
            check(livo_scan_release(ctx_, scan_id_), "livo_scan_release");
        }
        scan_id_ = id;
        feats_down_size = N;
        nearest_search_en = true;
    }

    livo_ctx* ctx_ = nullptr;
    livo_params params_{};
    int32_t scan_id_ = -1;
    bool ivox_ = false;
};

}  // namespace livo
