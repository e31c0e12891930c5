// Device helpers shared by the kernel translation units (ldpc_kernels.hip, sampler.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace ldpc {
namespace {

constexpr int kWave = 64;
template <bool B> using bool_c = std::integral_constant<bool, B>;
template <int N> using int_c = std::integral_constant<int, N>;

// ---------------------------------------------------------------------------
// Philox4x32-10 (the rocRAND philox4x32_10 stream: rocrand_init(seed,
// subsequence = codeword, offset = 4*g) -> rocrand4 == philox_block(g, 0,
// cw_lo, cw_hi) under key {seed_lo, seed_hi}).
// ---------------------------------------------------------------------------
// One round = two 32x32->64 products (v_mad_u64_u32: high and low word in one instruction)
// and two three-input XORs (v_bitop3_b32, truth table 0x96): 40 VALU per block.
__device__ __forceinline__ uint4 philox_block(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

// NBK Philox blocks that differ only in the first counter word, computed round by round (the
// blocks' dependency chains interleave: NBK independent products per step instead of one
// ten-round chain after another); bit-identical to NBK philox_block calls.
template <int NBK>
__device__ __forceinline__ void philox_blocks(const uint32_t (&c0)[NBK], uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1, uint4 (&out)[NBK]) {
    uint32_t a[NBK], b[NBK], c[NBK], d[NBK];
#pragma unroll
    for (int i = 0; i < NBK; ++i) { a[i] = c0[i]; b[i] = c1; c[i] = c2; d[i] = c3; }
#pragma unroll
    for (int r = 0; r < 10; ++r) {
#pragma unroll
        for (int i = 0; i < NBK; ++i) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * a[i], p1 = (uint64_t)0xCD9E8D57u * c[i];
            a[i] = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), b[i], k0, 0x96);
            c[i] = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), d[i], k1, 0x96);
            b[i] = (uint32_t)p1;
            d[i] = (uint32_t)p0;
        }
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
#pragma unroll
    for (int i = 0; i < NBK; ++i) out[i] = make_uint4(a[i], b[i], c[i], d[i]);
}

// Philox key schedule held in VGPRs (wave-uniform values the compiler would otherwise keep in
// 20 SGPRs for the whole kernel -- with the graph sampler's other uniform state that spills
// SGPRs to VGPR lanes, v_writelane / v_readlane + hazard s_nops in the hot loop).
struct PhiloxKeys {
    uint32_t a[10], b[10];
};
__device__ __forceinline__ PhiloxKeys philox_keys(uint32_t k0, uint32_t k1) {
    PhiloxKeys K;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        K.a[r] = k0 + (uint32_t)r * 0x9E3779B9u;
        K.b[r] = k1 + (uint32_t)r * 0xBB67AE85u;
        asm volatile("" : "+v"(K.a[r]), "+v"(K.b[r]));  // keep them in VGPRs
    }
    return K;
}
template <int NBK, int ROUNDS = 10>
__device__ __forceinline__ void philox_blocks(const uint32_t (&c0)[NBK], uint32_t c1, uint32_t c2, uint32_t c3,
                                              const PhiloxKeys &K, uint4 (&out)[NBK]) {
    uint32_t a[NBK], b[NBK], c[NBK], d[NBK];
#pragma unroll
    for (int i = 0; i < NBK; ++i) { a[i] = c0[i]; b[i] = c1; c[i] = c2; d[i] = c3; }
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
#pragma unroll
        for (int i = 0; i < NBK; ++i) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * a[i], p1 = (uint64_t)0xCD9E8D57u * c[i];
            a[i] = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), b[i], K.a[r], 0x96);
            c[i] = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), d[i], K.b[r], 0x96);
            b[i] = (uint32_t)p1;
            d[i] = (uint32_t)p0;
        }
    }
#pragma unroll
    for (int i = 0; i < NBK; ++i) out[i] = make_uint4(a[i], b[i], c[i], d[i]);
}
template <int ROUNDS = 10>
__device__ __forceinline__ uint4 philox_block(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, const PhiloxKeys &K) {
    const uint32_t cc[1] = {c0};
    uint4 o[1];
    philox_blocks<1, ROUNDS>(cc, c1, c2, c3, K, o);
    return o[0];
}

__device__ __forceinline__ uint32_t pick4(uint4 r, int i) {
    return i == 0 ? r.x : (i == 1 ? r.y : (i == 2 ? r.z : r.w));
}

// ---------------------------------------------------------------------------
// Channels: variable v of codeword cw reads word v mod 4 of Philox {v/4, 0, cw_lo, cw_hi}
// ---------------------------------------------------------------------------
__device__ __forceinline__ float u01(uint32_t x) {
    return (float)(2u * (x >> 9) + 1u) * 5.9604644775390625e-8f;
}

struct ChanArgs {
    int kind;      // LDPC_CH_*
    float p, p2;   // see oracle_channel
    uint32_t k0, k1;
};

// Channel value of variable 4g + i of a codeword from its Philox block r (all-zero codeword).
__device__ __forceinline__ float chan_soft_word(const ChanArgs &ch, const uint4 &r, int i) {
    if (ch.kind == 1) return u01(pick4(r, i)) < ch.p ? -ch.p2 : ch.p2;
    const int h = i >> 1;
    const float ua = u01(h ? r.z : r.x), ub = u01(h ? r.w : r.y);
    const float rad = sqrtf(-2.0f * logf(ua));
    const float ang = 6.28318530717958647692f * ub;
    const float g = rad * ((i & 1) ? sinf(ang) : cosf(ang));
    return (1.0f + ch.p * g) * ch.p2;
}

// Channel value of variable v of codeword cw.
__device__ __forceinline__ float chan_soft(const ChanArgs &ch, uint64_t cw, int v) {
    const uint4 r = philox_block((uint32_t)(v >> 2), 0u, (uint32_t)cw, (uint32_t)(cw >> 32), ch.k0, ch.k1);
    return chan_soft_word(ch, r, v & 3);
}

// The Philox block of variables 4g .. 4g + 3 of codeword cw (one block serves the four).
__device__ __forceinline__ uint4 chan_block(const ChanArgs &ch, uint64_t cw, int g) {
    return philox_block((uint32_t)g, 0u, (uint32_t)cw, (uint32_t)(cw >> 32), ch.k0, ch.k1);
}

__device__ __forceinline__ uint8_t chan_bec(const ChanArgs &ch, uint64_t cw, int v) {
    const uint4 r = philox_block((uint32_t)(v >> 2), 0u, (uint32_t)cw, (uint32_t)(cw >> 32), ch.k0, ch.k1);
    return u01(pick4(r, v & 3)) < ch.p ? 2 : 0;
}

// ---------------------------------------------------------------------------
// Block reductions (wave64)
// ---------------------------------------------------------------------------

// Sum over the (fully active) wave as a wave-uniform value: DPP row shifts 1, 2, 4, 8 leave
// each 16-lane row's sum in its lane 15, row_bcast:15 / :31 fold the rows into lane 63 --
// full-rate VALU, no LDS round trips or lane-index vectors (the ds_bpermute butterfly's)
__device__ __forceinline__ int wave_sum(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return __builtin_amdgcn_readlane(x, 63);
}

template <int T>
__device__ __forceinline__ int block_sum(int x, int *red) {
    x = wave_sum(x);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = x;
    __syncthreads();
    int s = 0;
#pragma unroll
    for (int w = 0; w < T / kWave; ++w) s += red[w];
    __syncthreads();
    return s;
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
