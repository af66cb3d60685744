// device_common.h — device helpers shared by the kernel files.
#pragma once
#include <hip/hip_runtime.h>

namespace livo {

__device__ __forceinline__ void world_point(const double* R, const double* pos, const double* RL, const double* tL,
                                            float bxf, float byf, float bzf, float& wx, float& wy, float& wz) {
    // pointBodyToWorld (laser_mapping.cpp:662-671): double math, float storage
    const double bx = bxf, by = byf, bz = bzf;
    const double ix = ((RL[0] * bx + RL[1] * by) + RL[2] * bz) + tL[0];
    const double iy = ((RL[3] * bx + RL[4] * by) + RL[5] * bz) + tL[1];
    const double iz = ((RL[6] * bx + RL[7] * by) + RL[8] * bz) + tL[2];
    wx = (float)(((R[0] * ix + R[1] * iy) + R[2] * iz) + pos[0]);
    wy = (float)(((R[3] * ix + R[4] * iy) + R[5] * iz) + pos[1]);
    wz = (float)(((R[6] * ix + R[7] * iy) + R[8] * iz) + pos[2]);
}

// XCD-aware block order for a 1-D grid of nb blocks per scan: blocks are dealt
// round-robin over the 8 XCDs, so give each XCD one contiguous run of (scan,
// block) ids -- one region of Morton-ordered points -- and its L2 only the
// part of the map around that region (bijective for any grid size).
__device__ __forceinline__ void xcd_block(int nb, unsigned& job, unsigned& bx) {
    const unsigned nwg = gridDim.x, orig = blockIdx.x, xcd = orig % 8u, q = nwg / 8u, r = nwg % 8u;
    const unsigned wgid = (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + orig / 8u;
    job = wgid / (unsigned)nb;
    bx = wgid % (unsigned)nb;
}

// XCD-interleaved block order in chunks of C consecutive blocks: XCD x takes
// chunks x, x + 8, x + 16, ... of the (scan, block) ids, so every XCD holds a
// share of every scan (a batch's scans cost different amounts in a search:
// with one contiguous range per XCD the most expensive scan's XCD is the
// straggler), while a chunk of C Morton-consecutive blocks keeps its map
// region in one L2.  The order is the same in every evaluation, so a block's
// plane cache is re-read on the XCD that wrote it.  C = 0: xcd_block.
__device__ __forceinline__ void xcd_chunk_block(int nb, int C, unsigned& job, unsigned& bx) {
    if (C <= 0) {
        xcd_block(nb, job, bx);
        return;
    }
    const unsigned c = (unsigned)C, orig = blockIdx.x, span = 8u * c;
    const unsigned full = gridDim.x / span * span;
    unsigned wgid = orig;
    if (orig < full) {
        const unsigned k = orig / 8u;
        wgid = ((k / c) * 8u + orig % 8u) * c + k % c;
    }
    job = wgid / (unsigned)nb;
    bx = wgid % (unsigned)nb;
}

// Centre of grid cell v along one axis, and the squared distance of a point to
// a cell centre: the cell runs' sort key (k_cr_rho) and the search's
// termination test (vrun_search) use exactly these operations, so both see
// the same bits.
__device__ __forceinline__ float cell_centre(float org, float h, int v) { return org + ((float)v + 0.5f) * h; }
__device__ __forceinline__ float centre_d2(float cx, float cy, float cz, float x, float y, float z) {
    const float t0 = x - cx, t1 = y - cy, t2 = z - cz;
    return (t0 * t0 + t1 * t1) + t2 * t2;
}
__device__ __forceinline__ float cr_rho2(const float org[3], float h, int v0, int v1, int v2, float x, float y,
                                         float z) {
    return centre_d2(cell_centre(org[0], h, v0), cell_centre(org[1], h, v1), cell_centre(org[2], h, v2), x, y, z);
}

}  // namespace livo
