// solve_lab — times k_solve (one wave per scan: reduction, P^-1, K1 LU, G, solution,
// boxplus, control, covariance) on synthetic slots, with per-phase s_memtime marks
// (livo_kernels.hip built with -DLIVO_SOLVE_PROF).  Development tool, not the product.
// usage: solve_lab [n_jobs] [nblk]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "livo_internal.h"

namespace livo {
extern __device__ unsigned long long g_solve_prof[256][16];
}
using namespace livo;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

int main(int argc, char** argv) {
    const int n_jobs = argc > 1 ? std::atoi(argv[1]) : 8;
    const int nblk = argc > 2 ? std::atoi(argv[2]) : 98;
    if (n_jobs < 1 || n_jobs > 256 || nblk < 1) return 2;
    std::mt19937 rng(7);
    std::normal_distribution<double> N01;
    std::vector<IekfSlot> hs(n_jobs);
    std::vector<double> hp((size_t)n_jobs * nblk * kRedCols, 0.0);
    for (int j = 0; j < n_jobs; j++) {
        IekfSlot& s = hs[j];
        std::memset(&s, 0, sizeof(s));
        for (int i = 0; i < 3; i++) s.state.rot[4 * i] = 1.0;
        for (int i = 0; i < kDim; i++) s.state.cov[i * kDim + i] = 1e-3 * (1.0 + 0.1 * i);
        s.state.gravity[2] = -9.81;
        s.prior = s.state;
        s.prior.pos[0] = 0.01;
        s.ctrl.search_en = 1;
        s.ctrl.iter_count = -1;
        s.ctrl.max_iter = 4;
        // HTH (upper-tri 21) and HTL from 1000 random unit-normal rows
        for (int r = 0; r < 1000; r++) {
            double H[6];
            for (double& h : H) h = N01(rng);
            const double err = 0.01 * N01(rng);
            double* part = hp.data() + ((size_t)j * nblk + (r % nblk)) * kRedCols;
            int q = 0;
            for (int a = 0; a < 6; a++)
                for (int b = a; b < 6; b++) part[q++] += 1000.0 * H[a] * H[b];
            for (int a = 0; a < 6; a++) part[21 + a] += 1000.0 * H[a] * err;
            part[27] += std::fabs(err);
            part[28] += 1.0;
        }
    }
    IekfSlot* ds;
    double* dp;
    HsJob* dj;
    CK(hipMalloc(&ds, sizeof(IekfSlot) * n_jobs));
    CK(hipMalloc(&dp, sizeof(double) * hp.size()));
    CK(hipMalloc(&dj, sizeof(HsJob) * n_jobs));
    CK(hipMemcpy(dp, hp.data(), sizeof(double) * hp.size(), hipMemcpyHostToDevice));
    std::vector<HsJob> hj(n_jobs);
    for (int j = 0; j < n_jobs; j++) {
        hj[j] = HsJob{};
        hj[j].partial = dp + (size_t)j * nblk * kRedCols;
        hj[j].slot = ds + j;
        hj[j].n = nblk * 1024;
        hj[j].nblk = nblk;
    }
    CK(hipMemcpy(dj, hj.data(), sizeof(HsJob) * n_jobs, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    SolveParams sp{ds, dj, nullptr, 0};
    for (int evals : {1, 2}) {  // evals = 1: the first evaluation (P^-1 too); 2: a later one
        const int reps = 20;
        double ms_sum = 0.0;
        std::vector<double> ph(10, 0.0);
        for (int r = 0; r < reps + 2; r++) {
            CK(hipMemcpy(ds, hs.data(), sizeof(IekfSlot) * n_jobs, hipMemcpyHostToDevice));
            for (int e = 0; e + 1 < evals; e++) CK(launch_solve(sp, n_jobs, st) == LIVO_OK ? hipSuccess : hipErrorUnknown);
            CK(hipEventRecord(e0, st));
            CK(launch_solve(sp, n_jobs, st) == LIVO_OK ? hipSuccess : hipErrorUnknown);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            unsigned long long hp2[256][16];
            CK(hipMemcpyFromSymbol(hp2, HIP_SYMBOL(g_solve_prof), sizeof(hp2)));
            if (r >= 2) {
                ms_sum += ms;
                for (int k = 1; k < 10; k++) ph[k] += (double)(hp2[0][k] - hp2[0][k - 1]);
            }
        }
        std::printf("evals=%d n_jobs=%d nblk=%d  k_solve %.2f us   phases (s_memtime ticks, job 0):", evals, n_jobs,
                    nblk, 1000.0 * ms_sum / reps);
        const char* names[10] = {"", "reduce", "load+HTH", "Pinv", "K1-LU", "K1-cols", "G+vec", "sol+Gout", "ctrl", "cov"};
        for (int k = 1; k < 10; k++) std::printf(" %s=%.0f", names[k], ph[k] / reps);
        std::printf("\n");
    }
    return 0;
}
