// GPU unit check (tests/test_gpu_ivox.py): wave_nth (fast-livo-noted_amd/csrc/
// wave_select.h), the wave-parallel std::nth_element of the iVox search,
// against libstdc++'s std::nth_element on the host, element for element.
// One wave per case; cases of 1..kWRaw elements with many ties.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "wave_select.h"

using namespace livo;

struct Case {
    int n, first, nth;
};

__global__ void k_check(const Case* cases, const float* d_in, float* d_out, uint32_t* id_out, int* status, int ncase) {
    __shared__ WaveLds lds[1];
    const int c = blockIdx.x, lane = threadIdx.x;
    if (c >= ncase) return;
    WaveLds& L = lds[0];
    const Case k = cases[c];
    for (int p = lane; p < k.n; p += 64) {
        L.d[p] = d_in[c * kWRaw + p];
        L.id[p] = (uint32_t)p;
    }
    wave_sync();
    const bool ok = wave_nth(L, k.first, k.nth, k.n, lane);
    for (int p = lane; p < k.n; p += 64) {
        d_out[c * kWRaw + p] = L.d[p];
        id_out[c * kWRaw + p] = L.id[p];
    }
    if (lane == 0) status[c] = ok ? 1 : 0;
}

// wave_nth_big (lists past WaveLds, k_ivox_knn_big_wave): one wave per case,
// the list and its tables in dynamic LDS of kBigCap entries.
constexpr int kBigCap = 4096;
__global__ void k_check_big(const Case* cases, const float* d_in, float* d_out, uint32_t* id_out, int* status,
                            int ncase) {
    extern __shared__ uint32_t lds[];
    const BigList L{reinterpret_cast<float*>(lds), lds + kBigCap, reinterpret_cast<uint16_t*>(lds + 2 * kBigCap),
                    reinterpret_cast<uint16_t*>(lds + 2 * kBigCap) + kBigCap};
    const int c = blockIdx.x, lane = threadIdx.x;
    if (c >= ncase) return;
    const Case k = cases[c];
    for (int p = lane; p < k.n; p += 64) {
        L.d[p] = d_in[(size_t)c * kBigCap + p];
        L.id[p] = (uint32_t)p;
    }
    wave_sync();
    const bool ok = wave_nth_big(L, k.first, k.nth, k.n, lane);
    for (int p = lane; p < k.n; p += 64) {
        d_out[(size_t)c * kBigCap + p] = L.d[p];
        id_out[(size_t)c * kBigCap + p] = L.id[p];
    }
    if (lane == 0) status[c] = ok ? 1 : 0;
}

// team_nth (k_ivox_knn_team): four teams a wave, one case each, lists of up to 128
constexpr int kTeamCap = 128;  // (k_ivox_knn_team's list capacity)
__global__ void k_check_team(const Case* cases, const float* d_in, uint32_t* id_out, int ncase) {
    __shared__ SelElem lst[4][kTeamCap];
    __shared__ uint8_t tabs[4][2][kTeamCap];
    const int lane = threadIdx.x, tl = lane & 15, team = lane >> 4;
    const int c = blockIdx.x * 4 + team;
    if (c >= ncase) return;  // (team-uniform)
    const Case k = cases[c];
    SelElem* L = lst[team];
    for (int p = tl; p < k.n; p += 16) L[p] = SelElem{d_in[(size_t)c * kTeamCap + p], (uint32_t)p};
    wave_sync();
    team_nth(L, tabs[team][0], tabs[team][1], k.first, k.nth, k.n, tl, lane);
    for (int p = tl; p < k.n; p += 16) id_out[(size_t)c * kTeamCap + p] = L[p].id;
}

struct DP {
    float d;
    uint32_t id;
    bool operator<(const DP& o) const { return d < o.d; }
};

int main(int argc, char** argv) {
    const int ncase = argc > 1 ? std::atoi(argv[1]) : 20000;
    std::mt19937 rng(99);
    std::vector<Case> cases(ncase);
    std::vector<float> din((size_t)ncase * kWRaw, 0.f);
    for (int c = 0; c < ncase; c++) {
        const int n = 1 + (int)(rng() % (c % 5 == 0 ? (unsigned)kWRaw : 140u));
        const int levels = 1 + (int)(rng() % 30u);
        for (int p = 0; p < n; p++)
            din[(size_t)c * kWRaw + p] = (c % 2) ? (float)(rng() % (unsigned)levels) * 0.25f
                                                 : std::ldexp((float)(rng() & 0xFFFFF), -20);
        const int first = (c % 4 == 0 && n > 1) ? (int)(rng() % (unsigned)n) : 0;
        const int nth = first + (int)(rng() % (unsigned)(n - first));
        cases[c] = Case{n, first, nth};
    }
    Case* dc;
    float *di, *dd;
    uint32_t* dids;
    int* dst;
    hipMalloc(&dc, sizeof(Case) * ncase);
    hipMalloc(&di, din.size() * 4);
    hipMalloc(&dd, din.size() * 4);
    hipMalloc(&dids, din.size() * 4);
    hipMalloc(&dst, 4 * ncase);
    hipMemcpy(dc, cases.data(), sizeof(Case) * ncase, hipMemcpyHostToDevice);
    hipMemcpy(di, din.data(), din.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(ncase), dim3(64), 0, 0, dc, di, dd, dids, dst, ncase);
    if (hipDeviceSynchronize() != hipSuccess) {
        std::printf("kernel failed\n");
        return 2;
    }
    std::vector<float> dout(din.size());
    std::vector<uint32_t> idout(din.size());
    std::vector<int> st(ncase);
    hipMemcpy(dout.data(), dd, din.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(idout.data(), dids, din.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(st.data(), dst, 4 * ncase, hipMemcpyDeviceToHost);
    long bad = 0, fallback = 0;
    for (int c = 0; c < ncase; c++) {
        const Case k = cases[c];
        std::vector<DP> ref(k.n);
        for (int p = 0; p < k.n; p++) ref[p] = DP{din[(size_t)c * kWRaw + p], (uint32_t)p};
        std::nth_element(ref.begin() + k.first, ref.begin() + k.nth, ref.begin() + k.n);
        if (!st[c]) {
            fallback++;
            continue;
        }
        for (int p = 0; p < k.n; p++)
            if (idout[(size_t)c * kWRaw + p] != ref[p].id) {
                if (bad < 3) std::printf("case %d n %d first %d nth %d: pos %d got %u want %u\n", c, k.n, k.first,
                                         k.nth, p, idout[(size_t)c * kWRaw + p], ref[p].id);
                bad++;
                break;
            }
    }
    // wave_nth_big: cases of 1..kBigCap elements (ties, narrow and wide value ranges)
    const int nbig = std::max(200, ncase / 10);
    std::vector<Case> bcases(nbig);
    std::vector<float> bin((size_t)nbig * kBigCap, 0.f);
    for (int c = 0; c < nbig; c++) {
        const int n = 1 + (int)(rng() % (c % 3 == 0 ? (unsigned)kBigCap : 2000u));
        const int levels = 1 + (int)(rng() % 200u);
        for (int p = 0; p < n; p++)
            bin[(size_t)c * kBigCap + p] = (c % 2) ? (float)(rng() % (unsigned)levels) * 0.25f
                                                   : std::ldexp((float)(rng() & 0xFFFFF), -20);
        const int first = (c % 4 == 0 && n > 1) ? (int)(rng() % (unsigned)n) : 0;
        const int nth = first + (int)(rng() % (unsigned)(n - first));
        bcases[c] = Case{n, first, nth};
    }
    Case* bc;
    float *bi, *bd;
    uint32_t* bids;
    int* bst;
    hipMalloc(&bc, sizeof(Case) * nbig);
    hipMalloc(&bi, bin.size() * 4);
    hipMalloc(&bd, bin.size() * 4);
    hipMalloc(&bids, bin.size() * 4);
    hipMalloc(&bst, 4 * nbig);
    hipMemcpy(bc, bcases.data(), sizeof(Case) * nbig, hipMemcpyHostToDevice);
    hipMemcpy(bi, bin.data(), bin.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check_big, dim3(nbig), dim3(64), kBigCap * 12, 0, bc, bi, bd, bids, bst, nbig);
    if (hipDeviceSynchronize() != hipSuccess) {
        std::printf("big kernel failed\n");
        return 2;
    }
    std::vector<uint32_t> bout(bin.size());
    std::vector<int> bs(nbig);
    hipMemcpy(bout.data(), bids, bin.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(bs.data(), bst, 4 * nbig, hipMemcpyDeviceToHost);
    long bbad = 0, bfall = 0;
    for (int c = 0; c < nbig; c++) {
        const Case k = bcases[c];
        std::vector<DP> ref(k.n);
        for (int p = 0; p < k.n; p++) ref[p] = DP{bin[(size_t)c * kBigCap + p], (uint32_t)p};
        std::nth_element(ref.begin() + k.first, ref.begin() + k.nth, ref.begin() + k.n);
        if (!bs[c]) {
            bfall++;
            continue;
        }
        for (int p = 0; p < k.n; p++)
            if (bout[(size_t)c * kBigCap + p] != ref[p].id) {
                if (bbad < 3) std::printf("big case %d n %d first %d nth %d: pos %d got %u want %u\n", c, k.n,
                                          k.first, k.nth, p, bout[(size_t)c * kBigCap + p], ref[p].id);
                bbad++;
                break;
            }
    }
    std::printf("wave_nth_big: %d cases of up to %d, %ld mismatched, %ld depth-limit fallbacks\n", nbig, kBigCap,
                bbad, bfall);
    // team_nth: 1..128 elements, mostly the 6..40 of an iVox grid's segment; ties
    // (few levels, incl. all equal: the heap-select path) and wide ranges
    const int nteam = std::max(4000, ncase);
    std::vector<Case> tcases(nteam);
    std::vector<float> tin((size_t)nteam * kTeamCap, 0.f);
    for (int c = 0; c < nteam; c++) {
        const int n = 1 + (int)(rng() % (c % 3 == 0 ? (unsigned)kTeamCap : 40u));
        const int levels = 1 + (int)(rng() % (c % 7 == 0 ? 2u : 30u));
        for (int p = 0; p < n; p++)
            tin[(size_t)c * kTeamCap + p] = (c % 2) ? (float)(rng() % (unsigned)levels) * 0.25f
                                                    : std::ldexp((float)(rng() & 0xFFFFF), -20);
        const int first = (c % 4 == 0 && n > 1) ? (int)(rng() % (unsigned)n) : 0;
        const int nth = (c % 5 == 0) ? first + std::min(4, n - 1 - first)
                                     : first + (int)(rng() % (unsigned)(n - first));
        tcases[c] = Case{n, first, nth};
    }
    Case* tc;
    float* ti;
    uint32_t* tids;
    hipMalloc(&tc, sizeof(Case) * nteam);
    hipMalloc(&ti, tin.size() * 4);
    hipMalloc(&tids, tin.size() * 4);
    hipMemcpy(tc, tcases.data(), sizeof(Case) * nteam, hipMemcpyHostToDevice);
    hipMemcpy(ti, tin.data(), tin.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check_team, dim3((nteam + 3) / 4), dim3(64), 0, 0, tc, ti, tids, nteam);
    if (hipDeviceSynchronize() != hipSuccess) {
        std::printf("team kernel failed\n");
        return 2;
    }
    std::vector<uint32_t> tout(tin.size());
    hipMemcpy(tout.data(), tids, tin.size() * 4, hipMemcpyDeviceToHost);
    long tbad = 0;
    for (int c = 0; c < nteam; c++) {
        const Case k = tcases[c];
        std::vector<DP> ref(k.n);
        for (int p = 0; p < k.n; p++) ref[p] = DP{tin[(size_t)c * kTeamCap + p], (uint32_t)p};
        std::nth_element(ref.begin() + k.first, ref.begin() + k.nth, ref.begin() + k.n);
        for (int p = 0; p < k.n; p++)
            if (tout[(size_t)c * kTeamCap + p] != ref[p].id) {
                if (tbad < 3) std::printf("team case %d n %d first %d nth %d: pos %d got %u want %u\n", c, k.n,
                                          k.first, k.nth, p, tout[(size_t)c * kTeamCap + p], ref[p].id);
                tbad++;
                break;
            }
    }
    std::printf("team_nth: %d cases of up to %d, %ld mismatched\n", nteam, kTeamCap, tbad);
    bad += tbad;
    std::printf("%d cases, %ld mismatches, %ld depth-limit fallbacks\n", ncase + nbig + nteam, bad + bbad,
                fallback + bfall);
    return (bad + bbad) == 0 ? 0 : 1;
}
