// wave_select.h — std::nth_element run by a group of lanes (a 16-lane team or
// a whole wavefront) on an LDS list (the iVox searches, ivox_kernels.hip;
// checked element for element against libstdc++ by
// tests/native/wave_nth_check.hip).
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

// ---------------------------------------------------------------------------
// std::nth_element(a + first, a + nth, a + last) run by a group of G lanes (a
// 16-lane team or the whole wave) on a list in LDS, libstdc++'s introselect
// round for round (stl_select.h restates it serially):
//
//   __move_median_to_first(first, first + 1, mid, last - 1), then
//   __unguarded_partition(first + 1, last, pivot = *first).
//
// The serial partition swaps the k-th element from the left that is >= pivot
// (Lo[k], by ascending position) with the k-th from the right that is <= pivot
// (Ro[k], by descending position) for as long as Lo[k] < Ro[k], and returns the
// position where the two scans cross.  Lo ascends and Ro descends, so the swaps
// are the pairs k < k* with k* the count of k with Lo[k] < Ro[k], the pairs are
// disjoint (no position is in two), and the cut is Lo[k*] when k* < |Lo| (or
// Ro[k* - 1] before it), else Ro[k* - 1].  One pass over the round's positions
// ranks both sets into LDS tables (lt: Lo ascending; rt: Ro by ascending
// position, so Ro[k] = rt[nR - 1 - k]); the pairs are then swapped in parallel.
// The median swap is folded in: the pass reads the element at `pick` as the one
// from `first`, and lane 0 writes the swap after the pass's reads.  Returns
// false when introselect's depth limit runs out (libstdc++ then heap-selects
// [first, last) as left in first / last; the callers take that path).
// Always inlined: an outlined call would reach LDS through flat pointers, whose
// accesses are not ordered with the caller's ds_* ones.

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

// list accessors: SoA (separate key / id arrays) and AoS (SelElem)
struct SoaList {
    float* d;
    uint32_t* id;
    __device__ __forceinline__ float key(int p) const { return d[p]; }
    __device__ __forceinline__ SelElem get(int p) const { return SelElem{d[p], id[p]}; }
    __device__ __forceinline__ void put(int p, const SelElem& e) const {
        d[p] = e.d;
        id[p] = e.id;
    }
};
struct AosList {
    SelElem* a;
    __device__ __forceinline__ float key(int p) const { return a[p].d; }
    __device__ __forceinline__ SelElem get(int p) const { return a[p]; }
    __device__ __forceinline__ void put(int p, const SelElem& e) const { a[p] = e; }
};

template <int G>
__device__ __forceinline__ unsigned long long grp_mask(unsigned long long m, int lane) {
    if constexpr (G == 64)
        return m;
    else
        return (m >> (lane & (64 - G))) & ((1ull << G) - 1ull);
}

template <int G, class List, class Tab>
__device__ __forceinline__ bool grp_nth(const List& L, Tab* lt, Tab* rt, int& first, int nth, int& last, int gl,
                                        int lane) {
    if (first == last || nth == last) return true;
    int depth = 2 * sel_lg(last - first);
    const unsigned long long below = (1ull << gl) - 1ull;
    while (last - first > 3) {
        if (depth == 0) return false;
        --depth;
        const int mid = first + (last - first) / 2;
        const SelElem e0 = L.get(first), ea = L.get(first + 1), eb = L.get(mid), ec = L.get(last - 1);
        int pick;  // __move_median_to_first(first, first + 1, mid, last - 1)
        SelElem pe;
        if (ea.d < eb.d) {
            if (eb.d < ec.d) { pick = mid; pe = eb; }
            else if (ea.d < ec.d) { pick = last - 1; pe = ec; }
            else { pick = first + 1; pe = ea; }
        } else if (ea.d < ec.d) { pick = first + 1; pe = ea; }
        else if (eb.d < ec.d) { pick = last - 1; pe = ec; }
        else { pick = mid; pe = eb; }
        const float pv = pe.d;
        int nL = 0, nR = 0;
#pragma unroll 1
        for (int p0 = first + 1; p0 < last; p0 += G) {  // (group-uniform)
            const int p = p0 + gl;
            const bool valid = p < last;
            const float lv = valid ? L.key(p) : 0.f;
            const float v = p == pick ? e0.d : lv;
            const bool lf = valid && !(v < pv), rf = valid && !(pv < v);
            const unsigned long long lm = grp_mask<G>(__ballot(lf), lane), rm = grp_mask<G>(__ballot(rf), lane);
            if (lf) lt[nL + __popcll(lm & below)] = (Tab)p;
            if (rf) rt[nR + __popcll(rm & below)] = (Tab)p;
            nL += __popcll(lm);
            nR += __popcll(rm);
        }
        if (gl == 0) {  // the median swap, after every read of the pass
            L.put(first, pe);
            L.put(pick, e0);
        }
        wave_sync();
        const int np = min(nL, nR);
        int kstar = 0;
#pragma unroll 1
        for (int k0 = 0; k0 < np; k0 += G) {  // (group-uniform)
            const int k = k0 + gl;
            int a = 0, b = 0;
            if (k < np) {
                a = lt[k];
                b = rt[nR - 1 - k];
            }
            const bool sw = k < np && a < b;
            kstar += __popcll(grp_mask<G>(__ballot(sw), lane));
            if (sw) {
                const SelElem xa = L.get(a), xb = L.get(b);
                L.put(a, xb);
                L.put(b, xa);
            }
        }
        const int cut = (kstar < nL) ? (kstar > 0 ? min((int)lt[kstar], (int)rt[nR - kstar]) : (int)lt[0])
                                     : (int)rt[nR - kstar];
        wave_sync();
        if (cut <= nth)
            first = cut;
        else
            last = cut;
    }
    if (gl == 0) {  // __insertion_sort(first, last), <= 3 elements
        for (int i = first + 1; i < last; ++i) {
            const SelElem v = L.get(i);
            int hole = i;
            if (v.d < L.key(first)) {
                for (; hole > first; --hole) L.put(hole, L.get(hole - 1));
            } else {
                while (v.d < L.key(hole - 1)) {
                    L.put(hole, L.get(hole - 1));
                    --hole;
                }
            }
            L.put(hole, v);
        }
    }
    wave_sync();
    return true;
}

// the wave's list of k_ivox_knn_wave / _wave_list (<= kWRaw entries)
__device__ __forceinline__ bool wave_nth(WaveLds& L, int first, int nth, int last, int lane) {
    return grp_nth<64>(SoaList{L.d, L.id}, L.lt, L.rt, first, nth, last, lane, lane);
}

// a list of any length (< 65536) in dynamic LDS (k_ivox_knn_big_wave)
struct BigList {
    float* d;
    uint32_t* id;
    uint16_t* lt;
    uint16_t* rt;
};
__device__ __forceinline__ bool wave_nth_big(const BigList& L, int first, int nth, int last, int lane) {
    return grp_nth<64>(SoaList{L.d, L.id}, L.lt, L.rt, first, nth, last, lane, lane);
}

// a 16-lane team's list of SelElems (k_ivox_knn_team: four queries a wave, <= 256
// entries: byte tables); the teams of a wave run their rounds under their own
// exec masks.  The depth limit's heap select runs on the team's lane 0, as the
// serial restatement does (stl_select.h).
constexpr int kTeamLanes = 16;
__device__ __forceinline__ void team_nth(SelElem* L, uint8_t* lt, uint8_t* rt, int first, int nth, int last,
                                         int tl, int lane) {
    if (!grp_nth<kTeamLanes>(AosList{L}, lt, rt, first, nth, last, tl, lane)) {
        if (tl == 0) {  // std::__heap_select + iter_swap (stl_algo.h __introselect)
            sel_heap_select(L, first, nth + 1, last);
            sel_swap(L, first, nth);
        }
        wave_sync();
    }
}

}  // namespace livo
