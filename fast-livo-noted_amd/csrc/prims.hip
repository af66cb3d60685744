// prims.hip — device-wide primitives from rocPRIM (radix sort, scan) behind
// plain signatures, kept in their own translation unit (template-heavy).
// Used by the iVox AddPoints path (ivox_kernels.hip), not by the hot k-NN.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "livo_internal.h"

namespace livo {

// Stable LSD radix sort of (key, value) u32 pairs on bits [0, bits).
// temp == nullptr: *temp_bytes receives the scratch size.
int prim_sort_pairs_u32(void* temp, size_t* temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                        const uint32_t* vals_in, uint32_t* vals_out, int64_t n, int bits, void* stream) {
    size_t tb = *temp_bytes;
    const hipError_t e = rocprim::radix_sort_pairs(temp, tb, keys_in, keys_out, vals_in, vals_out, (size_t)n, 0,
                                                   bits, (hipStream_t)stream);
    *temp_bytes = tb;
    return e == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

// Exclusive prefix sum of n u32 values (in-place allowed).
int prim_exclusive_scan_u32(void* temp, size_t* temp_bytes, const uint32_t* in, uint32_t* out, int64_t n,
                            void* stream) {
    size_t tb = *temp_bytes;
    const hipError_t e = rocprim::exclusive_scan(temp, tb, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(),
                                                 (hipStream_t)stream);
    *temp_bytes = tb;
    return e == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

// Inclusive prefix minimum of n int32 (the front-end's suffix minimum on reversed data).
int prim_inclusive_min_scan_i32(void* temp, size_t* temp_bytes, const int32_t* in, int32_t* out, int64_t n,
                                void* stream) {
    size_t tb = *temp_bytes;
    const hipError_t e = rocprim::inclusive_scan(temp, tb, in, out, (size_t)n, rocprim::minimum<int32_t>(),
                                                 (hipStream_t)stream);
    *temp_bytes = tb;
    return e == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

// Stable LSD radix sort of (u64 key, u32 value) pairs on bits [0, bits).
int prim_sort_pairs_u64(void* temp, size_t* temp_bytes, const unsigned long long* keys_in,
                        unsigned long long* keys_out, const uint32_t* vals_in, uint32_t* vals_out, int64_t n,
                        int bits, void* stream) {
    size_t tb = *temp_bytes;
    const hipError_t e = rocprim::radix_sort_pairs(temp, tb, keys_in, keys_out, vals_in, vals_out, (size_t)n, 0,
                                                   bits, (hipStream_t)stream);
    *temp_bytes = tb;
    return e == hipSuccess ? LIVO_OK : LIVO_E_HIP;
}

}  // namespace livo
