// Device helpers shared by the kernel translation units (ldpc_kernels.hip, sampler.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace ldpc {
namespace {

constexpr int kWave = 64;
template <bool B> using bool_c = std::integral_constant<bool, B>;

// ---------------------------------------------------------------------------
// Philox4x32-10 (the rocRAND philox4x32_10 stream: rocrand_init(seed,
// subsequence = codeword, offset = 4*g) -> rocrand4 == philox_block(g, 0,
// cw_lo, cw_hi) under key {seed_lo, seed_hi}).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox_block(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ uint32_t pick4(uint4 r, int i) {
    return i == 0 ? r.x : (i == 1 ? r.y : (i == 2 ? r.z : r.w));
}

// Exclusive prefix sum over the workgroup (any multiple of 64 threads <= 1024);
// `total` gets the sum.  Contains two barriers.
__device__ __forceinline__ int block_excl_scan(int x, int *wsum, int &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int incl = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off, kWave);
        if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int base = 0, tot = 0;
    for (int w = 0; w < nw; ++w) {
        const int v = wsum[w];
        base += (w < wave) ? v : 0;
        tot += v;
    }
    __syncthreads();
    total = tot;
    return base + incl - x;
}

template <typename K>
hipError_t allow_lds(K kernel, size_t bytes) {
    if (bytes <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void *>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace
}  // namespace ldpc
