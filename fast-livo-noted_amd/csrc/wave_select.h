// wave_select.h — std::nth_element run by a whole wavefront on an LDS list
// (k_ivox_knn_wave, ivox_kernels.hip; checked element for element against
// libstdc++ by tests/native/wave_nth_check.hip).  See ivox_kernels.hip for
// the parallel formulation of libstdc++'s unguarded Hoare partition.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "livo_internal.h"

namespace livo {

constexpr int kWRaw = 512;
#ifndef LIVO_IV_WAVES
#define LIVO_IV_WAVES 4
#endif
constexpr int kWaves = LIVO_IV_WAVES;  // queries (waves) per block
constexpr int kWRounds = kWRaw / 64;  // positions per lane

struct WaveLds {
    float d[kWRaw];
    uint32_t id[kWRaw];
    uint16_t lt[kWRaw];  // Lo table (positions by rank)
    uint16_t rt[kWRaw];  // Ro table
    uint8_t node[kWRaw]; // staged position -> nearby grid
    uint32_t m[kIvMaxNearby + 1];  // in-range points per grid
};

// Lanes exchange data through LDS: every access before this point has
// completed before any after it is issued (workgroup-scope fences make the
// compiler wait on the LDS counter; wavefront-scope ones are no-ops).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ int lanes_below(unsigned long long mask, int lane) {
    return __popcll(mask & ((1ull << lane) - 1ull));
}
__device__ __forceinline__ void lds_swap(WaveLds& L, int i, int j) {
    const float td = L.d[i];
    const uint32_t ti = L.id[i];
    L.d[i] = L.d[j];
    L.id[i] = L.id[j];
    L.d[j] = td;
    L.id[j] = ti;
}

// std::nth_element(a + first, a + nth, a + last) on the wave's LDS list; false:
// the depth limit ran out (heap select needed: the caller falls back).
// Always inlined: an outlined call would reach the LDS list through flat
// pointers, whose accesses are not ordered with the caller's ds_* ones.
__device__ __forceinline__ bool wave_nth(WaveLds& L, int first, int nth, int last, int lane) {
    if (first == last || nth == last) return true;
    int depth = 2 * sel_lg(last - first);
    while (last - first > 3) {
        if (depth == 0) return false;
        --depth;
        const int mid = first + (last - first) / 2;
        if (lane == 0) {  // __move_median_to_first(first, first + 1, mid, last - 1)
            const float a = L.d[first + 1], b = L.d[mid], c = L.d[last - 1];
            int pick;
            if (a < b)
                pick = (b < c) ? mid : ((a < c) ? last - 1 : first + 1);
            else
                pick = (a < c) ? first + 1 : ((b < c) ? last - 1 : mid);
            lds_swap(L, first, pick);
        }
        wave_sync();
        const float pv = L.d[first];
        const int lo = first + 1;
        const int nr = (last - lo + 63) >> 6;  // rounds of 64 positions actually in range (uniform)
        bool lf[kWRounds], rf[kWRounds];
        unsigned long long lm[kWRounds], rm[kWRounds];
        int nL = 0, nR = 0;
#pragma unroll
        for (int r = 0; r < kWRounds; r++) {
            lf[r] = rf[r] = false;
            lm[r] = rm[r] = 0ull;
            if (r < nr) {
                const int p = lo + 64 * r + lane;
                const bool valid = p < last;
                const float v = valid ? L.d[p] : 0.f;
                lf[r] = valid && !(v < pv);
                rf[r] = valid && !(pv < v);
                lm[r] = __ballot(lf[r]);
                rm[r] = __ballot(rf[r]);
                nL += __popcll(lm[r]);
                nR += __popcll(rm[r]);
            }
        }
        int lrank[kWRounds], rrank[kWRounds];
        bool ok[kWRounds];
        int kstar = 0, lb = 0, rb = 0;
#pragma unroll
        for (int r = 0; r < kWRounds; r++) {
            lrank[r] = lb + lanes_below(lm[r], lane);
            const int rle = rb + lanes_below(rm[r], lane) + (rf[r] ? 1 : 0);  // rf positions <= p
            rrank[r] = nR - rle;  // rf positions > p: the rank in Ro
            ok[r] = lf[r] && (nR - rle) >= lrank[r] + 1;  // Lo[k] < Ro[k]
            if (r < nr) kstar += __popcll(__ballot(ok[r]));
            lb += __popcll(lm[r]);
            rb += __popcll(rm[r]);
        }
#pragma unroll
        for (int r = 0; r < kWRounds; r++) {
            const int p = lo + 64 * r + lane;
            if (lf[r]) L.lt[lrank[r]] = (uint16_t)p;
            if (rf[r]) L.rt[rrank[r]] = (uint16_t)p;
        }
        wave_sync();
        float nd[kWRounds];
        uint32_t nid[kWRounds];
        bool sw[kWRounds];
#pragma unroll
        for (int r = 0; r < kWRounds; r++) {
            sw[r] = (lf[r] && lrank[r] < kstar) || (rf[r] && rrank[r] < kstar);
            int partner = 0;
            if (lf[r] && lrank[r] < kstar) partner = L.rt[lrank[r]];
            if (rf[r] && rrank[r] < kstar) partner = L.lt[rrank[r]];
            nd[r] = sw[r] ? L.d[partner] : 0.f;
            nid[r] = sw[r] ? L.id[partner] : 0u;
        }
        const int cut = (kstar < nL) ? (kstar > 0 ? min((int)L.lt[kstar], (int)L.rt[kstar - 1]) : (int)L.lt[0])
                                     : (int)L.rt[kstar - 1];
        wave_sync();
#pragma unroll
        for (int r = 0; r < kWRounds; r++)
            if (sw[r]) {
                const int p = lo + 64 * r + lane;
                L.d[p] = nd[r];
                L.id[p] = nid[r];
            }
        wave_sync();
        if (cut <= nth)
            first = cut;
        else
            last = cut;
    }
    if (lane == 0) {  // __insertion_sort(first, last), <= 3 elements
        for (int i = first + 1; i < last; ++i) {
            const float vd = L.d[i];
            const uint32_t vi = L.id[i];
            int hole = i;
            if (vd < L.d[first]) {
                for (; hole > first; --hole) {
                    L.d[hole] = L.d[hole - 1];
                    L.id[hole] = L.id[hole - 1];
                }
            } else {
                while (vd < L.d[hole - 1]) {
                    L.d[hole] = L.d[hole - 1];
                    L.id[hole] = L.id[hole - 1];
                    --hole;
                }
            }
            L.d[hole] = vd;
            L.id[hole] = vi;
        }
    }
    wave_sync();
    return true;
}

// The same std::nth_element on a list of any length (< 65536) in LDS given as
// separate arrays: the rounds of 64 positions are loops instead of register
// arrays, and the swap pairs (Lo[k], Ro[k]), k < k*, are exchanged pair by pair
// (the pairs are disjoint: Lo ascends, Ro descends and Lo[k] < Ro[k], so no
// position is in two of them).  For the iVox queries whose grids are too large
// for WaveLds (k_ivox_knn_big_wave).
struct BigList {
    float* d;
    uint32_t* id;
    uint16_t* lt;
    uint16_t* rt;
};
__device__ __forceinline__ bool wave_nth_big(const BigList& L, int first, int nth, int last, int lane) {
    if (first == last || nth == last) return true;
    int depth = 2 * sel_lg(last - first);
    while (last - first > 3) {
        if (depth == 0) return false;
        --depth;
        const int mid = first + (last - first) / 2;
        if (lane == 0) {  // __move_median_to_first(first, first + 1, mid, last - 1)
            const float a = L.d[first + 1], b = L.d[mid], c = L.d[last - 1];
            int pick;
            if (a < b)
                pick = (b < c) ? mid : ((a < c) ? last - 1 : first + 1);
            else
                pick = (a < c) ? first + 1 : ((b < c) ? last - 1 : mid);
            const float td = L.d[first];
            const uint32_t ti = L.id[first];
            L.d[first] = L.d[pick];
            L.id[first] = L.id[pick];
            L.d[pick] = td;
            L.id[pick] = ti;
        }
        wave_sync();
        const float pv = L.d[first];
        const int lo = first + 1;
        const int nr = (last - lo + 63) >> 6;
        int nL = 0, nR = 0;
        for (int r = 0; r < nr; r++) {  // the Lo / Ro totals
            const int p = lo + 64 * r + lane;
            const bool valid = p < last;
            const float v = valid ? L.d[p] : 0.f;
            nL += __popcll(__ballot(valid && !(v < pv)));
            nR += __popcll(__ballot(valid && !(pv < v)));
        }
        int kstar = 0, lb = 0, rb = 0;
        for (int r = 0; r < nr; r++) {  // ranks in Lo / Ro, k* and the two tables
            const int p = lo + 64 * r + lane;
            const bool valid = p < last;
            const float v = valid ? L.d[p] : 0.f;
            const bool lf = valid && !(v < pv), rf = valid && !(pv < v);
            const unsigned long long lm = __ballot(lf), rm = __ballot(rf);
            const int lrank = lb + lanes_below(lm, lane);
            const int rle = rb + lanes_below(rm, lane) + (rf ? 1 : 0);
            const int rrank = nR - rle;
            kstar += __popcll(__ballot(lf && rrank >= lrank + 1));
            if (lf) L.lt[lrank] = (uint16_t)p;
            if (rf) L.rt[rrank] = (uint16_t)p;
            lb += __popcll(lm);
            rb += __popcll(rm);
        }
        wave_sync();
        const int cut = (kstar < nL) ? (kstar > 0 ? min((int)L.lt[kstar], (int)L.rt[kstar - 1]) : (int)L.lt[0])
                                     : (int)L.rt[kstar - 1];
        for (int k = lane; k < kstar; k += 64) {
            const int a = L.lt[k], b = L.rt[k];
            const float da = L.d[a], db = L.d[b];
            const uint32_t ia = L.id[a], ib = L.id[b];
            L.d[a] = db;
            L.id[a] = ib;
            L.d[b] = da;
            L.id[b] = ia;
        }
        wave_sync();
        if (cut <= nth)
            first = cut;
        else
            last = cut;
    }
    if (lane == 0) {  // __insertion_sort(first, last), <= 3 elements
        for (int i = first + 1; i < last; ++i) {
            const float vd = L.d[i];
            const uint32_t vi = L.id[i];
            int hole = i;
            if (vd < L.d[first]) {
                for (; hole > first; --hole) {
                    L.d[hole] = L.d[hole - 1];
                    L.id[hole] = L.id[hole - 1];
                }
            } else {
                while (vd < L.d[hole - 1]) {
                    L.d[hole] = L.d[hole - 1];
                    L.id[hole] = L.id[hole - 1];
                    --hole;
                }
            }
            L.d[hole] = vd;
            L.id[hole] = vi;
        }
    }
    wave_sync();
    return true;
}

}  // namespace livo
