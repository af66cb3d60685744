// device_common.h — device helpers shared by livo_kernels.hip and ivox_kernels.hip.
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

}  // namespace livo
