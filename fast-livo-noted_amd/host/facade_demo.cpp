// facade_demo.cpp — drives LaserMappingGpu the way LaserMapping::Run drives
// its members (laser_mapping.cpp:129-238), with minimal Eigen-shaped types,
// and prints the results for tests/test_facade.py to compare with the oracle.
//
// usage: facade_demo <map.f32> <scan.f32> <state.f64> <max_iter> [ivox]
//   map.f32 / scan.f32: raw float xyz triples; state.f64: 3x3 rot (row-major),
//   pos, vel, bias_g, bias_a, gravity, 18x18 cov (row-major) = 348 doubles.
// Output (text): "hshare <effct> <81 HPH> <9 HPL>" for the first
// h_share_model(), then "iekf <iterations> <converged> <rot 9> <pos 3> <cov 324>".
// With "ivox": the map goes in through ivox_->AddPoints (the reference's
// default backend) and a final "incr <added> <no_downsample>" line reports
// map_incremental() at the updated state.
// Exit status: 0 ok, 2 usage/IO, 3 livo::Error (code printed on stderr).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "laser_mapping_gpu.hpp"

namespace {

// Column-major dense matrix / vector with Eigen's accessor shape.
struct DenseMat {
    int r = 0, c = 0;
    std::vector<double> v;
    void resize(int rows, int cols) { r = rows; c = cols; v.assign((size_t)rows * cols, 0.0); }
    void resize(int n) { resize(n, 1); }
    double& operator()(int i, int j) { return v[(size_t)j * r + i]; }
    double operator()(int i, int j) const { return v[(size_t)j * r + i]; }
    double& operator()(int i) { return v[(size_t)i]; }
    double operator()(int i) const { return v[(size_t)i]; }
};

struct States {  // StatesGroup field names (common_lib.h:518-603)
    DenseMat rot_end, pos_end, vel_end, bias_g, bias_a, gravity, cov;
    States() {
        rot_end.resize(3, 3);
        pos_end.resize(3);
        vel_end.resize(3);
        bias_g.resize(3);
        bias_a.resize(3);
        gravity.resize(3);
        cov.resize(18, 18);
    }
};

std::vector<char> slurp(const char* path) {
    std::vector<char> b;
    FILE* f = std::fopen(path, "rb");
    if (!f) return b;
    char tmp[1 << 16];
    size_t n;
    while ((n = std::fread(tmp, 1, sizeof(tmp), f)) > 0) b.insert(b.end(), tmp, tmp + n);
    std::fclose(f);
    return b;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 5 && !(argc == 6 && std::string(argv[5]) == "ivox")) {
        std::fprintf(stderr, "usage: %s map.f32 scan.f32 state.f64 max_iter [ivox]\n", argv[0]);
        return 2;
    }
    const bool ivox = argc == 6;
    const std::vector<char> map = slurp(argv[1]), scan = slurp(argv[2]), st = slurp(argv[3]);
    if (map.empty() || scan.empty() || st.size() != 348 * sizeof(double)) {
        std::fprintf(stderr, "bad input files\n");
        return 2;
    }
    const double* sd = reinterpret_cast<const double*>(st.data());
    States s0;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) s0.rot_end(i, j) = sd[3 * i + j];
        s0.pos_end(i) = sd[9 + i];
        s0.vel_end(i) = sd[12 + i];
        s0.bias_g(i) = sd[15 + i];
        s0.bias_a(i) = sd[18 + i];
        s0.gravity(i) = sd[21 + i];
    }
    for (int i = 0; i < 18; i++)
        for (int j = 0; j < 18; j++) s0.cov(i, j) = sd[24 + 18 * i + j];
    try {
        livo_params p;
        livo::check(livo_params_default(&p), "livo_params_default");
        p.t_LI[0] = 0.04165;  // the synthetic rig's extrinsic (livo_amd.synth.T_LI)
        p.t_LI[1] = 0.02326;
        p.t_LI[2] = -0.0284;
        p.max_iterations = std::atoi(argv[4]);
        livo::LaserMappingGpu lm(0, &p);
        if (ivox) {
            lm.use_ivox();  // reference defaults: 0.2 m grids, NEARBY18, capacity 1e6
            lm.ivox_add_points(reinterpret_cast<const float*>(map.data()), (int64_t)(map.size() / 12));
        } else {
            lm.build_map(reinterpret_cast<const float*>(map.data()), (int64_t)(map.size() / 12));
        }
        lm.set_scan(reinterpret_cast<const float*>(scan.data()), (int64_t)(scan.size() / 12));
        lm.set_state(s0);
        lm.set_state_propagat(s0);

        DenseMat HPH, HPL;
        lm.h_share_model(HPH, HPL);
        std::printf("hshare %lld", (long long)lm.effct_feat_num);
        for (int i = 0; i < 9; i++)
            for (int j = 0; j < 9; j++) std::printf(" %.17g", HPH(i, j));
        for (int i = 0; i < 9; i++) std::printf(" %.17g", HPL(i));
        std::printf("\n");

        lm.set_state(s0);
        const livo_iter_stats it = lm.iterate();
        States s1;
        lm.get_state(s1);
        std::printf("iekf %d %d", it.iterations, it.converged);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) std::printf(" %.17g", s1.rot_end(i, j));
        for (int i = 0; i < 3; i++) std::printf(" %.17g", s1.pos_end(i));
        for (int i = 0; i < 18; i++)
            for (int j = 0; j < 18; j++) std::printf(" %.17g", s1.cov(i, j));
        std::printf("\n");
        if (ivox) {
            lm.map_incremental(0.5);  // filter_size_map default (laser_mapping.cpp:983)
            std::printf("incr %lld %lld\n", (long long)lm.points_added, (long long)lm.points_no_downsample);
        }
    } catch (const livo::Error& e) {
        std::fprintf(stderr, "livo::Error %d %s\n", e.code(), e.what());
        return 3;
    }
    return 0;
}
