// HIP kernels for gfx950 (MI355X): BEC erasure decoding, soft flooding BP
// (sum-product / normalized min-sum), on-device channels and Monte-Carlo
// statistics.  Layout and rationale: DESIGN.md.
//
// Reference behaviour restated here:
//   message_passing.c:7-82         -> bec_kernel           (bit-exact)
//   channels.py:24-26 new_transmit -> channel_kernel / chan_* (same law, Philox)
//   parallel_simulator.py:198-244  -> mc_* (per-trial statistics + stop rule)
//   parallel_simulator.py:60-129   -> ml_kernel (ML erasure decoding, optimal_decode)
#include <rocrand/rocrand_kernel.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "device_common.hpp"
#include "ldpc_internal.hpp"
#include "ldpc_mi355x.h"

namespace ldpc {
namespace {

#ifndef LDPC_VAR_PAIRS
#define LDPC_VAR_PAIRS 1  // variable pairs per sched_barrier group in the LDS kernel's variable phase
#endif
#ifndef LDPC_CHECK_PAIRS_UNROLL
#define LDPC_CHECK_PAIRS_UNROLL 2  // check pairs per iteration of the LDS kernel's check loop (1: 1.4 % slower)
#endif
#ifndef LDPC_BEC_BITS
#define LDPC_BEC_BITS 1  // fixed-code BEC Monte-Carlo on the bit-sliced kernel when its planes fit LDS
#endif
#ifndef LDPC_LDS36_PREFETCH
#define LDPC_LDS36_PREFETCH 1  // persistent LDS kernel (decode API) prefetching the next codeword's LLRs
#endif
#ifndef LDPC_BEC_DEC_BITS
#define LDPC_BEC_DEC_BITS 1  // batch BEC decode (B >= 64) on the bit-sliced kernel when its planes fit LDS
#endif
#ifndef LDPC_LOC_VGROUP
#define LDPC_LOC_VGROUP 1  // bp_loc_kernel: variable pairs per scheduling group (0: no barriers)
#endif
#ifndef LDPC_LOC_CGROUP
#define LDPC_LOC_CGROUP 1  // bp_loc_kernel: check pairs per scheduling group (0: no barriers)
#endif
// ===========================================================================
// 1. BEC erasure decoding -- message_passing.c:7-82, bit-exact.
//
// One workgroup per codeword.  LDS: caller errors[] (int32), the ternary word
// (u8) and one byte per check.  The reference's per-slot check messages are
// never materialised: a slot addressed to an ERASED variable is known iff its
// check holds exactly one erasure, and then equals the parity of the check's
// known bits (message_passing.c:31-43); so each check publishes one byte
// cs = ne==1 ? parity : 2 and an erased variable takes the last cs != 2 over
// its checks in variable_to_check_list order (message_passing.c:55-62).
// vchk = -1 marks a (variable, check) pair where the check does not hold the
// variable exactly once: such a pair never assigns in the reference.
// ===========================================================================
struct BecArgs {
    const int32_t *cvar, *cptr, *vptr, *vchk;
    int n, m, dv, dc;  // dv, dc > 0: regular (pointers implicit)
    uint8_t *words;
    int32_t *errors, *its;
    int max_iters;
    // Monte-Carlo mode
    ChanArgs ch;
    uint64_t first_cw;
    int32_t *trial;  // [B][max_iters+1]
    // ensemble mode: codeword b decodes on its own graph (cvar / vchk + b*graph_stride)
    int64_t graph_stride;
};

template <int T, bool MC>
__global__ __launch_bounds__(T) void bec_kernel(BecArgs a) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int red[T / kWave];
    const int tid = threadIdx.x;
    const size_t b = blockIdx.x;
    const int n = a.n, m = a.m, iters = a.max_iters;
    int32_t *errs = reinterpret_cast<int32_t *>(smem);
    uint8_t *mvc = smem + ((iters * 4 + 15) & ~15);
    uint8_t *cs = mvc + ((n + 15) & ~15);
    const int32_t *cvar = a.cvar + (size_t)b * a.graph_stride;
    const int32_t *vchk = a.vchk + (size_t)b * a.graph_stride;

    int init_cnt = 0;
    if (MC) {
        const uint64_t cw = a.first_cw + b;
        for (int g4 = tid; g4 < (n + 3) >> 2; g4 += T) {  // one Philox block per four variables
            const uint4 r = chan_block(a.ch, cw, g4);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (4 * g4 + q >= n) break;
                const uint8_t x = u01(pick4(r, q)) < a.ch.p ? 2 : 0;  // chan_bec
                mvc[4 * g4 + q] = x;
                init_cnt += (x == 2);
            }
        }
        for (int i = tid; i < iters; i += T) errs[i] = 0;
    } else {
        const uint8_t *w = a.words + b * n;
        for (int v = tid; v < n; v += T) mvc[v] = w[v];
        const int32_t *e = a.errors + b * iters;
        for (int i = tid; i < iters; i += T) errs[i] = e[i];
    }
    __syncthreads();
    const int initial = MC ? block_sum<T>(init_cnt, red) : 0;

    int prev1 = 0, prev2 = 0;  // errors[it-1], errors[it-2] after accumulation
    int it;
    for (it = 0; it < iters; ++it) {
        if (it >= 2 && prev1 == prev2) {  // message_passing.c:16-19 (absorbing)
            for (int i = it + tid; i < iters; i += T) errs[i] = prev1;
            it = iters;
            break;
        }
        // check phase (reads the previous word only)
        for (int c = tid; c < m; c += T) {
            const int s0 = a.dc > 0 ? c * a.dc : a.cptr[c];
            const int s1 = a.dc > 0 ? s0 + a.dc : a.cptr[c + 1];
            int ne = 0, par = 0;
            for (int s = s0; s < s1; ++s) {
                const int x = mvc[cvar[s]];
                ne += (x == 2);
                par ^= (x & 1);
            }
            cs[c] = (uint8_t)(ne == 1 ? par : 2);
        }
        __syncthreads();
        // variable phase: erased variables take the last known check message
        int cnt = 0;
        for (int v = tid; v < n; v += T) {
            int x = mvc[v];
            if (x == 2) {
                const int e0 = a.dv > 0 ? v * a.dv : a.vptr[v];
                const int e1 = a.dv > 0 ? e0 + a.dv : a.vptr[v + 1];
                for (int e = e0; e < e1; ++e) {
                    const int c = vchk[e];
                    if (c >= 0) {
                        const int y = cs[c];
                        if (y != 2) x = y;
                    }
                }
                mvc[v] = (uint8_t)x;
                cnt += (x == 2);
            }
        }
        const int base = errs[it];  // read before block_sum's barriers, written after
        const int total = block_sum<T>(cnt, red);
        const int cur = base + total;
        if (tid == 0) errs[it] = cur;
        prev2 = prev1;
        prev1 = cur;
        if (total == 0) break;  // message_passing.c:76-78
    }
    __syncthreads();
    if (MC) {
        int32_t *tr = a.trial + b * (size_t)(iters + 1);
        for (int i = tid; i <= iters; i += T) tr[i] = i == 0 ? initial : errs[i - 1];
        if (tid == 0) a.its[b] = it;
    } else {
        uint8_t *w = a.words + b * n;
        for (int v = tid; v < n; v += T) w[v] = mvc[v];
        int32_t *e = a.errors + b * iters;
        for (int i = tid; i < iters; i += T) e[i] = errs[i];
        if (tid == 0) a.its[b] = it;
    }
}

// ---------------------------------------------------------------------------
// 1b. BEC Monte-Carlo, bit-sliced: the same decoder (message_passing.c:7-82 with
// the all-zero codeword of parallel_simulator.py:222) for 32*W codewords per
// workgroup at once.  Bit b of word w of variable v is "codeword 32w+b has v
// erased".  With the all-zero codeword every known bit is 0, so the parity of a
// check's known bits is 0 and only the erasure planes evolve:
//   check c:    One[c] = codewords where exactly one of c's slots is erased
//               (carry-save: two |= one & e; one |= e; One = one & ~two)
//   variable v: E[v] &= ~OR_{edges e of v, vchk[e] >= 0} One[vchk[e]]
// which is bec_kernel's rule (an erased variable takes any known check message;
// known messages are 0) bit for bit, Jacobi (One is built from the old planes).
// Running every codeword for all iterations in lockstep is exact: a stalled or
// finished codeword is a fixed point, so its counts repeat (message_passing.c:
// 16-19 fills errors[it] = errors[it-1]; after the break at a zero count the
// caller's zeros remain).  Per-codeword counts per iteration come from one LDS
// atomic per resolved (codeword, variable); its = the first iteration whose
// count is zero, else iters; the decode stops once no codeword changes.
// Channel: bit = chan_bec(cw, v) (the stream of bec_kernel / oracle_channel),
// 32 codewords per half-wave, one Philox block per lane per 4 variables,
// transposed into the planes by ballots.  Output: trial[b][iters+1] and its[b]
// in bec_kernel's MC layout, so mc_cutoff / mc_reduce apply unchanged.
// LDS: E[n][W], One[m][W] (u32), cnt[32W], its[32W], 3 change flags.
// ---------------------------------------------------------------------------
// Plane words: P = uint32_t (32 codewords, W words per variable) or uint8_t (8
// codewords, W = 1: planes of n + m bytes, for graphs whose u32 planes do not fit).
template <typename P, int W> struct BitsVec;
template <> struct BitsVec<uint32_t, 1> { typedef uint32_t T; };
template <> struct BitsVec<uint32_t, 2> { typedef uint2 T; };
template <> struct BitsVec<uint32_t, 4> { typedef uint4 T; };
template <> struct BitsVec<uint8_t, 1> { typedef uint8_t T; };

template <typename P, int W>
__device__ __forceinline__ void bits_load(const P *p, uint32_t (&x)[W]) {
    const typename BitsVec<P, W>::T v = *reinterpret_cast<const typename BitsVec<P, W>::T *>(p);
    if constexpr (W == 1) x[0] = v;
    if constexpr (W == 2) { x[0] = v.x; x[1] = v.y; }
    if constexpr (W == 4) { x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w; }
}
template <typename P, int W>
__device__ __forceinline__ void bits_store(P *p, const uint32_t (&x)[W]) {
    typename BitsVec<P, W>::T v;
    if constexpr (W == 1) v = (P)x[0];
    if constexpr (W == 2) v = make_uint2(x[0], x[1]);
    if constexpr (W == 4) v = make_uint4(x[0], x[1], x[2], x[3]);
    *reinterpret_cast<typename BitsVec<P, W>::T *>(p) = v;
}

template <int T, int W, typename P>
__global__ __launch_bounds__(T) void bec_mc_bits_kernel(BecArgs a, int B) {
    static_assert(T % 64 == 0, "lane groups of BITS codewords tile the waves");
    constexpr int BITS = 8 * sizeof(P);  // codewords per plane word
    constexpr int NB = BITS * W;         // codewords per workgroup
    extern __shared__ __align__(16) unsigned char smem[];
    const int tid = threadIdx.x;
    const int n = a.n, m = a.m, iters = a.max_iters;
    P *Ev = reinterpret_cast<P *>(smem);  // [n][W]
    P *On = Ev + (size_t)n * W;           // [m][W]
    int *cnt = reinterpret_cast<int *>(smem + ((((size_t)n + m) * W * sizeof(P) + 15) & ~(size_t)15));  // [NB]
    int *itsl = cnt + NB;                                                       // [NB]
    uint32_t *flag = reinterpret_cast<uint32_t *>(itsl + NB);                   // [3] "some codeword changed"
    const int64_t b0 = (int64_t)blockIdx.x * NB;
    const int nloc = (int)min((int64_t)NB, (int64_t)B - b0);  // codewords of this block with trial rows

    for (int i = tid; i < NB; i += T) {
        cnt[i] = 0;
        itsl[i] = iters;
    }
    if (tid < 3) flag[tid] = 0;
    __syncthreads();
    // ---- channel: a group of BITS lanes = one (group g of 4 variables, word w); lane = codeword bit ----
    {
        const int ngr = (n + 3) >> 2;
        const int bit = tid & (BITS - 1);
        const int shift = (tid & (kWave - 1)) & ~(BITS - 1);  // this group's bits in the wave ballot
        int local[W];
#pragma unroll
        for (int w = 0; w < W; ++w) local[w] = 0;
        for (int base = tid / BITS; base < ngr * W; base += T / BITS) {
            const int g = base / W, w = base - g * W;
            const uint64_t cw = a.first_cw + (uint64_t)(b0 + BITS * w + bit);
            const uint4 r = philox_block((uint32_t)g, 0u, (uint32_t)cw, (uint32_t)(cw >> 32), a.ch.k0, a.ch.k1);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int v = 4 * g + j;
                const bool er = v < n && u01(pick4(r, j)) < a.ch.p;
                const uint64_t bal = __ballot(er);
                local[w] += er;
                if (bit == 0 && v < n) Ev[(size_t)v * W + w] = (P)(bal >> shift);
            }
        }
#pragma unroll
        for (int w = 0; w < W; ++w)
            if (local[w]) atomicAdd(&cnt[BITS * w + bit], local[w]);
    }
    __syncthreads();
    for (int i = tid; i < nloc; i += T) a.trial[(size_t)(b0 + i) * (iters + 1)] = cnt[i];

    int it = 0;
    for (; it < iters; ++it) {
        // ---- check phase (reads the previous planes only) ----
        for (int c = tid; c < m; c += T) {
            const int s0 = a.dc > 0 ? c * a.dc : a.cptr[c];
            const int s1 = a.dc > 0 ? s0 + a.dc : a.cptr[c + 1];
            uint32_t one[W], two[W];
#pragma unroll
            for (int w = 0; w < W; ++w) one[w] = two[w] = 0u;
            for (int s = s0; s < s1; ++s) {
                uint32_t e[W];
                bits_load<P, W>(Ev + (size_t)a.cvar[s] * W, e);
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    two[w] |= one[w] & e[w];
                    one[w] |= e[w];
                }
            }
#pragma unroll
            for (int w = 0; w < W; ++w) one[w] &= ~two[w];
            bits_store<P, W>(On + (size_t)c * W, one);
        }
        __syncthreads();
        if (tid == 0) flag[(it + 1) % 3] = 0u;  // next iteration's flag (last read before this barrier)
        // ---- variable phase ----
        uint32_t changed = 0u;
        for (int v = tid; v < n; v += T) {
            uint32_t e[W], any = 0u;
            bits_load<P, W>(Ev + (size_t)v * W, e);
#pragma unroll
            for (int w = 0; w < W; ++w) any |= e[w];
            if (!any) continue;
            const int e0 = a.dv > 0 ? v * a.dv : a.vptr[v];
            const int e1 = a.dv > 0 ? e0 + a.dv : a.vptr[v + 1];
            uint32_t r[W];
#pragma unroll
            for (int w = 0; w < W; ++w) r[w] = 0u;
            for (int x = e0; x < e1; ++x) {
                const int c = a.vchk[x];
                if (c < 0) continue;
                uint32_t o[W];
                bits_load<P, W>(On + (size_t)c * W, o);
#pragma unroll
                for (int w = 0; w < W; ++w) r[w] |= o[w];
            }
            uint32_t ne[W];
#pragma unroll
            for (int w = 0; w < W; ++w) {
                r[w] &= e[w];  // resolved this iteration
                ne[w] = e[w] & ~r[w];
                changed |= r[w];
            }
            bits_store<P, W>(Ev + (size_t)v * W, ne);
#pragma unroll
            for (int w = 0; w < W; ++w) {
                uint32_t q = r[w];
                while (q) {
                    const int b = __builtin_ctz(q);
                    q &= q - 1u;
                    atomicSub(&cnt[BITS * w + b], 1);
                }
            }
        }
        if (__ballot(changed != 0u) && (tid & (kWave - 1)) == 0) atomicOr(&flag[it % 3], 1u);
        __syncthreads();
        for (int i = tid; i < NB; i += T) {
            const int c = cnt[i];
            if (c == 0 && itsl[i] == iters) itsl[i] = it;
            if (i < nloc) a.trial[(size_t)(b0 + i) * (iters + 1) + it + 1] = c;
        }
        if (!flag[it % 3]) {  // nothing changed: every codeword is at its fixed point
            for (int i = tid; i < nloc; i += T) {
                int32_t *tr = a.trial + (size_t)(b0 + i) * (iters + 1);
                const int c = cnt[i];
                for (int j = it + 2; j <= iters; ++j) tr[j] = c;
            }
            break;
        }
    }
    __syncthreads();
    for (int i = tid; i < nloc; i += T) a.its[b0 + i] = itsl[i];
}

// ---------------------------------------------------------------------------
// 1c. BEC batch decode, bit-sliced: bec_kernel's non-MC contract (arbitrary
// words, caller errors[] accumulated and steering the stall test of
// message_passing.c:16-19) for H = 4*sizeof(P) codewords per plane word.
// A variable's word holds "erased" bits (low H) and value bits (high H, the
// byte's bit 0 when not erased, 0 when erased); a check's word holds "exactly
// one slot erased" bits (low) and the parity of its known bits (high), i.e.
// bec_kernel's cs = ne==1 ? parity : 2.  Variable phase, in
// variable_to_check_list order: sel = One[c] & erased & active,
// val = (val & ~sel) | (parity & sel) -- the last known check message wins
// (message_passing.c:55-62) -- and the variable is resolved iff some sel was set.
// Codeword control (counts, stall test, zero-count break) is per codeword in
// registers of lane i < NB; codewords that have stopped are masked out of the
// variable phase ("active"), so a stalled word is frozen exactly as the
// reference's early return leaves it.  When no codeword changed in an
// iteration every active codeword is at a fixed point and its remaining
// iterations (count fixed, caller errors[] still added and tested) are
// replayed by its lane without touching the graph.
// Output rewrites only the bytes that were 2 on input (a known byte is never
// changed by the reference, whatever its value).
// LDS: X[n][W], C[m][W] plane words, cnt[NB], act[W], 2 change flags, done.
// ---------------------------------------------------------------------------
template <int T, int W, typename P>
__global__ __launch_bounds__(T) void bec_dec_bits_kernel(BecArgs a, int B) {
    constexpr int H = 4 * (int)sizeof(P);  // codewords per plane word
    constexpr uint32_t LO = (1u << H) - 1u;
    constexpr int NB = H * W;  // codewords per workgroup (<= 64: control lanes in wave 0)
    static_assert(NB <= kWave, "control lanes must sit in wave 0");
    extern __shared__ __align__(16) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & (kWave - 1);
    const int n = a.n, m = a.m, iters = a.max_iters;
    P *Xv = reinterpret_cast<P *>(smem);  // [n][W]
    P *Xc = Xv + (size_t)n * W;           // [m][W]
    int *cnt = reinterpret_cast<int *>(smem + ((((size_t)n + m) * W * sizeof(P) + 15) & ~(size_t)15));  // [NB]
    uint32_t *act = reinterpret_cast<uint32_t *>(cnt + NB);  // [W]
    uint32_t *flag = act + W;                                 // [2] changed, [2] all stopped
    const int64_t b0 = (int64_t)blockIdx.x * NB;
    const int nloc = (int)min((int64_t)NB, (int64_t)B - b0);

    for (int i = tid; i < NB; i += T) cnt[i] = 0;
    if (tid < 3) flag[tid] = 0u;
    if (tid < W) act[tid] = (1u << min(max(nloc - tid * H, 0), H)) - 1u;  // codewords with rows
    __syncthreads();
    // ---- words -> planes: thread (w, v) gathers byte v of the word's H rows (lanes = consecutive v) ----
#pragma unroll
    for (int w = 0; w < W; ++w) {
        int lc[H];
#pragma unroll
        for (int j = 0; j < H; ++j) lc[j] = 0;
        for (int v = tid; v < n; v += T) {
            uint32_t x = 0u;
#pragma unroll
            for (int j = 0; j < H; ++j) {
                const int i = w * H + j;
                const uint32_t y = i < nloc ? a.words[(size_t)(b0 + i) * n + v] : 0u;
                const bool er = y == 2u;
                x |= (uint32_t)er << j | (er ? 0u : (y & 1u)) << (H + j);
                lc[j] += er;
            }
            Xv[(size_t)v * W + w] = (P)x;
        }
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const int s = wave_sum(lc[j]);
            if (lane == 0 && s) atomicAdd(&cnt[w * H + j], s);
        }
    }
    // control state of codeword tid (tid < nloc)
    int p1 = 0, p2 = 0, its = iters;
    bool done = tid >= nloc;
    int32_t *er = a.errors + (size_t)(b0 + min(tid, max(nloc - 1, 0))) * iters;
    __syncthreads();

    for (int it = 0; it < iters; ++it) {
        // ---- check phase (reads the previous planes only) ----
        for (int c = tid; c < m; c += T) {
            const int s0 = a.dc > 0 ? c * a.dc : a.cptr[c];
            const int s1 = a.dc > 0 ? s0 + a.dc : a.cptr[c + 1];
            uint32_t one[W], two[W], par[W];
#pragma unroll
            for (int w = 0; w < W; ++w) one[w] = two[w] = par[w] = 0u;
            for (int s = s0; s < s1; ++s) {
                uint32_t x[W];
                bits_load<P, W>(Xv + (size_t)a.cvar[s] * W, x);
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    const uint32_t e = x[w] & LO;
                    two[w] |= one[w] & e;
                    one[w] |= e;
                    par[w] ^= x[w] >> H;
                }
            }
#pragma unroll
            for (int w = 0; w < W; ++w) one[w] = (one[w] & ~two[w]) | (par[w] & LO) << H;
            bits_store<P, W>(Xc + (size_t)c * W, one);
        }
        __syncthreads();
        // ---- variable phase: active erased variables take the last known check message ----
        uint32_t av[W];
#pragma unroll
        for (int w = 0; w < W; ++w) av[w] = act[w];
        uint32_t changed = 0u;
        for (int v = tid; v < n; v += T) {
            uint32_t x[W], any = 0u;
            bits_load<P, W>(Xv + (size_t)v * W, x);
#pragma unroll
            for (int w = 0; w < W; ++w) any |= x[w] & av[w];
            if (!any) continue;
            const int e0 = a.dv > 0 ? v * a.dv : a.vptr[v];
            const int e1 = a.dv > 0 ? e0 + a.dv : a.vptr[v + 1];
            uint32_t val[W], res[W];
#pragma unroll
            for (int w = 0; w < W; ++w) val[w] = res[w] = 0u;
            for (int e = e0; e < e1; ++e) {
                const int c = a.vchk[e];
                if (c < 0) continue;
                uint32_t y[W];
                bits_load<P, W>(Xc + (size_t)c * W, y);
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    const uint32_t sel = y[w] & x[w] & av[w];  // low bits only (av)
                    val[w] = (val[w] & ~sel) | ((y[w] >> H) & sel);
                    res[w] |= sel;
                }
            }
#pragma unroll
            for (int w = 0; w < W; ++w) {
                x[w] = (x[w] & ~res[w]) | val[w] << H;
                changed |= res[w];
            }
            bits_store<P, W>(Xv + (size_t)v * W, x);
#pragma unroll
            for (int w = 0; w < W; ++w) {
                uint32_t q = res[w];
                while (q) {
                    const int b = __builtin_ctz(q);
                    q &= q - 1u;
                    atomicSub(&cnt[w * H + b], 1);
                }
            }
        }
        if (__ballot(changed != 0u) && lane == 0) atomicOr(&flag[it & 1], 1u);
        __syncthreads();
        // ---- control: message_passing.c:70-78 per codeword, then the stall test of the next iteration ----
        if (tid < kWave) {
            if (!done) {
                const bool chg = flag[it & 1] != 0u;
                const int c = cnt[tid];
                int cur = er[it] + c;
                er[it] = cur;
                p2 = p1;
                p1 = cur;
                if (c == 0) {
                    done = true;
                    its = it;
                } else {
                    for (int t = it + 1; t < iters; ++t) {
                        if (t >= 2 && p1 == p2) {  // message_passing.c:16-19
                            for (int j = t; j < iters; ++j) er[j] = p1;
                            done = true;
                            break;
                        }
                        if (chg) break;
                        cur = er[t] + c;  // fixed point: replay iteration t
                        er[t] = cur;
                        p2 = p1;
                        p1 = cur;
                    }
                    if (!chg) done = true;  // its stays iters
                }
            }
            const uint64_t alive = __ballot(!done);
            if (tid == 0) {
#pragma unroll
                for (int w = 0; w < W; ++w) act[w] = (uint32_t)(alive >> (w * H)) & LO;
                flag[(it + 1) & 1] = 0u;
                flag[2] = alive == 0ull;
            }
        }
        __syncthreads();
        if (flag[2]) break;
    }
    if (tid < nloc) a.its[b0 + tid] = its;
    // ---- planes -> words: rewrite the bytes that were erased on input ----
#pragma unroll
    for (int w = 0; w < W; ++w) {
        for (int v = tid; v < n; v += T) {
            const uint32_t x = Xv[(size_t)v * W + w];
#pragma unroll
            for (int j = 0; j < H; ++j) {
                const int i = w * H + j;
                if (i < nloc) {
                    uint8_t *p = a.words + (size_t)(b0 + i) * n + v;
                    if (*p == 2u) *p = ((x >> j) & 1u) ? 2u : (uint8_t)((x >> (H + j)) & 1u);
                }
            }
        }
    }
}

// ===========================================================================
// 2. Soft flooding BP (no reference counterpart; oracle_bp_decode defines it)
// ===========================================================================
// Sum-product runs in the log2 domain (messages are LLR / ln 2) and in the
// ratio form of oracle check_update_spa: e_i = 2^-min(|x_i|, 23) is one
// v_exp_f32, the exclusive product of tanh(x_i/2) = a_i / b_i (a_i = sign*(1-e_i),
// b_i = 1+e_i) is N_j / D_j from prefix/suffix products, and 2 atanh(N/D) / ln 2 =
// log2((D+N) / (D-N)) is one v_rcp_f32 + one v_log_f32 -- three transcendentals
// per edge.  Channel LLRs are scaled by log2(e) in, posteriors by ln 2 out.
template <int ALGO> struct Domain {
    static constexpr float in = ALGO == 0 ? 1.44269504088896341f : 1.0f;   // LLR -> message units
    static constexpr float out = ALGO == 0 ? 0.693147180559945309f : 1.0f; // message units -> LLR
};
// Channel LLR -> message.  Min-sum: l + 0 turns a -0 LLR into +0 (every other value is
// unchanged), so no min-sum message is ever -0 (sums and differences of non-(-0) values
// are not -0 in round-to-nearest) and the sign BIT of every check input equals the
// oracle's (x < 0) -- which lets check_update_ms6 form signs with bit operations.
template <int ALGO> __device__ __forceinline__ float to_msg(float l) {
    if constexpr (ALGO == 0) return l * Domain<0>::in;
    else return l + 0.0f;
}

// Sum-product check rule in ratio form, restated by oracle check_update_spa: for an
// input message x (log2 units here) tanh(x/2) = (R - 1) / (R + 1) with the ratio
// R = 2^x, |x| clamped to 23 (R in [2^-23, 2^23]); the exclusive products of the
// (R - 1) and (R + 1) terms give the output 2 atanh(N_j / D_j) / ln 2 =
// log2((D_j + N_j) / (D_j - N_j)) -- formed without cancellation from elementary
// symmetric polynomials of the R (check_update_spa_pair_rwire).
//
// v->c message "on the wire" of the LDS kernels: sum-product sends the clamped ratio R
// itself (the check rule's outputs (D + N) / (D - N) are invariant to a positive scale of
// each input's (R - 1, R + 1) pair, so no reciprocal per edge in the variable phase;
// magnitudes stay below 2^23 + 1, so the exclusive products of 5 inputs stay below
// 2^116); min-sum sends x itself.
template <int ALGO>
__device__ __forceinline__ float v2c_rwire(float x) {
    if (ALGO == 0) return __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(x, -23.0f, 23.0f));
    return x;
}
// an extrinsic ratio R on the wire: clamped to [2^-23, 2^23]
__device__ __forceinline__ float ratio_wire(float R) { return __builtin_amdgcn_fmed3f(R, 0x1p-23f, 0x1p23f); }
__device__ __forceinline__ float2 ratio_wire2(float2 R) {
    return make_float2(__builtin_amdgcn_fmed3f(R.x, 0x1p-23f, 0x1p23f), __builtin_amdgcn_fmed3f(R.y, 0x1p-23f, 0x1p23f));
}

// Inline-asm helpers (v_bitop3_b32, the VCC select): the compiler's hazard
// recognizer does not look inside inline asm, so their operands must not be fresh
// transcendental (v_exp / v_log / v_rcp) results -- every use below takes LDS loads, min /
// med3 / mul / bfe results or values from an earlier phase.
// v_bitop3_b32 (gfx950) with truth table T over (S0, S1, S2) = (0xF0, 0xCC, 0xAA)
// (check_update_ms6's sign stamps stay in asm: through the builtin the fixed-count min-sum
// decode measured 1.3 % slower, profiles/r05_ab_bitop3_builtin.txt)
template <int T>
__device__ __forceinline__ uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(r) : "v"(a), "v"(b), "v"(c), "n"(T));
    return r;
}
// a ^ b ^ c in one instruction (gfx950 has no v_xor3_b32: v_bitop3_b32 with table 0x96).
// Through the builtin, as bfi_u32: the hazard recognizer sees the instruction and inserts no
// conservative s_nop around it (early stop +0.9 %, min-sum Monte-Carlo +1.2 %,
// profiles/r05_ab_xor3_bfi_builtin.txt)
__device__ __forceinline__ uint32_t xor3u(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// |x| == m ? t : f as v_cmp (into VCC) + v_cndmask: the compiler would otherwise hold one
// SGPR-pair mask per output of a check pair at once and spill SGPRs
__device__ __forceinline__ uint32_t sel_abs_eq(float x, float m, uint32_t t, uint32_t f) {
    uint32_t r;
    asm("v_cmp_eq_f32_e64 vcc, |%1|, %2\n\tv_cndmask_b32 %0, %4, %3, vcc" : "=v"(r) : "v"(x), "v"(m), "v"(t), "v"(f) : "vcc");
    return r;
}
// (m & a) | (~m & b): one v_bitop3_b32 (table 0xCA), through the builtin (see xor3u)
__device__ __forceinline__ uint32_t bfi_u32(uint32_t m, uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
}
// (r & ~1) | (d & 1): one v_bfi_b32
// (plain C: the compiler emits one v_and_or_b32 / v_bfi_b32 and, unlike for inline asm, inserts
// the wait state gfx950 needs when an operand is a fresh transcendental result -- an asm
// v_bfi_b32 right after the v_exp_f32 of the initial message read a stale register)
__device__ __forceinline__ uint32_t bfi_lsb(uint32_t r, uint32_t d) { return (r & ~1u) | (d & 1u); }

// a * b + c per lane as one v_pk_fma_f32 (the SLP vectoriser packs only some)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2 pk_fma(float2 a, float2 b, float2 c) {
    const f32x2 r = __builtin_elementwise_fma(f32x2{a.x, a.y}, f32x2{b.x, b.y}, f32x2{c.x, c.y});
    return make_float2(r.x, r.y);
}

// Check-node update over D messages in registers; entries i >= d are padding (+inf
// for min-sum; skipped by sum-product).  Min-sum is bit-exact with oracle
// check_update_ms; sum-product agrees with the oracle's exact rule to the stated
// tolerance.
template <int ALGO, int D, bool WIRE = false>
__device__ __forceinline__ void check_update(float (&x)[D], float alpha, int d = D) {
    if (ALGO == 0) {
        // elementary-symmetric form (check_update_spa_pair_rwire) on the d inputs' ratios
        // R = 2^x (WIRE: the ratios themselves), outputs log2 of the exclusive ratio; (E, O)
        // sums in float2 so both chains are packed ops.  Entries i >= d are skipped.
        float R[D];
#pragma unroll
        for (int i = 0; i < D; ++i)
            R[i] = WIRE ? x[i] : __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(x[i], -23.0f, 23.0f));
        float2 pre[D];  // (E, O) of inputs {0 .. i-1}
        pre[0] = make_float2(1.0f, 0.0f);
#pragma unroll
        for (int i = 1; i < D; ++i) {
            const float2 nx = pk_fma(make_float2(R[i - 1], R[i - 1]), make_float2(pre[i - 1].y, pre[i - 1].x), pre[i - 1]);
            pre[i] = i - 1 < d ? nx : pre[i - 1];
        }
        const bool odd = (d - 1) & 1;
        float2 suf = make_float2(1.0f, 0.0f);  // (E, O) of inputs {j+1 .. d-1}
#pragma unroll
        for (int j = D - 1; j >= 0; --j) {
            if (j < d) {
                const float E = fmaf(pre[j].x, suf.x, pre[j].y * suf.y), O = fmaf(pre[j].x, suf.y, pre[j].y * suf.x);
                const float num = odd ? O : E, den = odd ? E : O;
                const float2 ns = pk_fma(make_float2(R[j], R[j]), make_float2(suf.y, suf.x), suf);
                x[j] = __builtin_amdgcn_logf(num * __builtin_amdgcn_rcpf(den));
                suf = ns;
            }
        }
    } else {
        // branch-free: m1 = running min, m2 = running second smallest (with
        // multiplicity) = med3(m1, m2, a); an edge whose magnitude equals m1 gets
        // m2 (with a tie m2 == m1: the same values as oracle check_update_ms'
        // "first minimum gets m2")
        float m1 = __builtin_inff(), m2 = __builtin_inff();
        bool neg = false;
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const float a = fabsf(x[i]);
            neg ^= (x[i] < 0.0f);
            m2 = __builtin_amdgcn_fmed3f(m1, m2, a);
            m1 = fminf(m1, a);
        }
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const float mag = alpha * (fabsf(x[i]) == m1 ? m2 : m1);
            x[i] = (neg ^ (x[i] < 0.0f)) ? -mag : mag;
        }
    }
}

// Normalized min-sum update of one degree-6 check, branch-free: the two smallest
// magnitudes (with multiplicity) from two triples -- m1 = min of the triple minima,
// m2 = min(max of the triple minima, both triple medians) -- via v_min3 / v_med3.
// An edge whose magnitude equals m1 gets m2 (with a tie m2 == m1, so this equals
// oracle check_update_ms' "index of the first minimum gets m2"); signs as there.
__device__ __forceinline__ void check_update_ms6(float (&x)[6], float alpha) {
    float ax[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) ax[i] = fabsf(x[i]);
    const float mn1 = fminf(fminf(ax[0], ax[1]), ax[2]), md1 = __builtin_amdgcn_fmed3f(ax[0], ax[1], ax[2]);
    const float mn2 = fminf(fminf(ax[3], ax[4]), ax[5]), md2 = __builtin_amdgcn_fmed3f(ax[3], ax[4], ax[5]);
    const float m1 = fminf(mn1, mn2), m2 = fminf(fminf(fmaxf(mn1, mn2), md1), md2);
    float am1 = alpha * m1, am2 = alpha * m2;
    // keep the two products: otherwise select(alpha*m2, alpha*m1) is folded into
    // alpha*select(m2, m1), one multiply per edge instead of two per check
    asm volatile("" : "+v"(am1), "+v"(am2));
    // signs as bits (no input is -0, see to_msg, so the sign bit is the oracle's x < 0):
    // S = XOR of the six sign bits, stamped onto both scaled minima once per check; each
    // output is then the selected minimum XOR its own input's sign bit -- v_cmp, v_cndmask
    // and one v_bitop3 / v_and + v_xor per output, no scalar mask arithmetic
    const uint32_t S = xor3u(xor3u(__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2])),
                             __float_as_uint(x[3]), __float_as_uint(x[4])) ^ __float_as_uint(x[5]);
    const uint32_t M = 0x80000000u;
    const uint32_t s1 = bitop3<0xF8>(__float_as_uint(am1), S, M), s2 = bitop3<0xF8>(__float_as_uint(am2), S, M);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const uint32_t mag = sel_abs_eq(x[i], m1, s2, s1);  // a | (b & M), then a ^ (b & M)
        x[i] = __uint_as_float(bitop3<0x78>(mag, __float_as_uint(x[i]), M));
    }
}


// Sum-product update of a PAIR of checks held as float2 lanes (.x = check 2q, .y = check
// 2q + 1), every product one packed op for both checks.  The inputs are the clamped
// ratios R_i = e^{x_i} (ratio_wire), and tanh(x_i/2) = (R_i - 1) / (R_i + 1).  With
// D_j = prod_{i != j} (R_i + 1) and N_j = prod_{i != j} (R_i - 1), the output ratio
// (D_j + N_j) / (D_j - N_j) is, expanding both products in the elementary symmetric
// polynomials e_k of the d - 1 inputs i != j, O_j / E_j for d - 1 odd (E_j / O_j for
// d - 1 even), where E = sum_{k even} e_k and O = sum_{k odd} e_k.  Every term is
// positive, so there is no cancellation anywhere (the difference D - N of the ratio
// form loses ~d ulps x e^|c| near saturation): each output is good to ~10 fp32 ulps.
// (E, O) of a set grows by one input R as (E + R O, O + R E) -- two fused multiply-adds,
// the cost of the ratio form's two product chains -- and two disjoint sets combine as
// (E_a E_b + O_a O_b, E_a O_b + O_a E_b).  Magnitudes: E >= 1, O >= sum R >= 2^-23,
// e_k < 2^(23 k + 3) <= 2^118 for the 5 inputs of a degree-6 check.
// INVX: the .x check has one input less, padded with R = 0 (E, O unchanged, but the
// exclusive sets count one more input), so its outputs take the other parity's ratio.
template <int D, bool INVX = false>
__device__ __forceinline__ void check_update_spa_pair_rwire(float2 (&R)[D]) {
    const float2 one = make_float2(1.0f, 1.0f);
    auto ratio = [](float2 E, float2 O) {
        constexpr bool odd = (D - 1) % 2 == 1;
        if constexpr (INVX) {
            return odd ? make_float2(E.x * __builtin_amdgcn_rcpf(O.x), O.y * __builtin_amdgcn_rcpf(E.y))
                       : make_float2(O.x * __builtin_amdgcn_rcpf(E.x), E.y * __builtin_amdgcn_rcpf(O.y));
        }
        if constexpr (odd) return O * make_float2(__builtin_amdgcn_rcpf(E.x), __builtin_amdgcn_rcpf(E.y));
        else return E * make_float2(__builtin_amdgcn_rcpf(O.x), __builtin_amdgcn_rcpf(O.y));
    };
    float2 pE[D], pO[D];  // prefix sets {0 .. i-1}
    pE[1] = one;
    pO[1] = R[0];
#pragma unroll
    for (int i = 2; i < D; ++i) {
        pE[i] = pk_fma(R[i - 1], pO[i - 1], pE[i - 1]);
        pO[i] = pk_fma(R[i - 1], pE[i - 1], pO[i - 1]);
    }
    float2 sE = one, sO = R[D - 1];  // suffix set {i+1 .. D-1}
    R[D - 1] = ratio(pE[D - 1], pO[D - 1]);
#pragma unroll
    for (int i = D - 2; i >= 1; --i) {
        const float2 E = pk_fma(pE[i], sE, pO[i] * sO);
        const float2 O = pk_fma(pE[i], sO, pO[i] * sE);
        const float2 nE = pk_fma(R[i], sO, sE);
        const float2 nO = pk_fma(R[i], sE, sO);
        R[i] = ratio(E, O);
        sE = nE;
        sO = nO;
    }
    R[0] = ratio(sE, sO);
}

// Byte address (x4) of the low / high 16-bit LDS position packed in p: one SDWA
// shift instead of an extract and a shift-add.  volatile: re-evaluated every
// iteration, so the compiler cannot hoist VPT*DV unpacked addresses out of the
// decode loop (they would not fit the VGPR budget).
typedef __attribute__((address_space(3))) float lds_f32;  // LDS word at a byte address
typedef __attribute__((address_space(3))) unsigned char lds_u8;

__device__ __forceinline__ uint32_t pos_lo_x4(uint32_t p) {
    uint32_t r;
    asm volatile("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
                 : "=v"(r) : "v"(p));
    return r;
}
__device__ __forceinline__ uint32_t pos_hi_x4(uint32_t p) {
    uint32_t r;
    asm volatile("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
                 : "=v"(r) : "v"(p));
    return r;
}

struct BpArgs {
    const int32_t *cptr, *cvar, *vptr, *vslot;
    int n, m, E, B;
    const float *llr;
    float *post;
    uint8_t *hard;
    int32_t *its;
    int max_iters;
    float alpha;
    // Monte-Carlo mode
    ChanArgs ch;
    uint64_t first_cw;
    int32_t *trial;  // [B][max_iters+1]
    // generic kernel, messages in global scratch
    float *scratch;
    size_t scratch_bytes;  // (host) bytes at scratch: the launchers refuse a layout needing more
    // LDS kernel lane layout (ldpc_graph::lane_var / lane_slot)
    const int32_t *lane_var, *lane_slot;
    int lds_slots;  // generic GMEM kernel: message slots [0, lds_slots) kept in LDS
    // irregular kernel layout (ldpc_graph::irr_*)
    const int32_t *irr_lane, *irr_cdeg;
    int irr_KC, irr_S, irr_P;
    // local-edge kernel layout (ldpc_graph::loc_*)
    const int32_t *loc_var, *loc_pos, *loc_info;
    int loc_P, loc_ncls, loc_words;
    int loc_cls_q[5], loc_cls_d[4], loc_cls_w[5];
    uint32_t *work;  // bp_loc_kernel early stop (persistent grid): next-codeword counter (zeroed per launch)
};

// ---------------------------------------------------------------------------
// 2a. Regular fast path: whole codeword resident in LDS.
//   LDS  msg[S + dummies] fp32, S = lds_pair_span(m, DC): check pairs (2q, 2q+1)
//        interleaved edge by edge ([q][edge][2], lds_pair_pos), hs[...] u8 hard
//        decision per position (ET only), curve (MC only).
//   Thread t owns check pairs t, t+T, ... and the variables of lane positions
//   p = t + i*T (i < VPT) of the host-built conflict-aware layout: every 32
//   consecutive positions (one half-wave LDS access) hit 32 distinct banks as far
//   as the graph allows; padding positions address private dummy positions.
//   Positions (packed 2 x 16 bit) and channel LLRs stay in VGPRs for the whole
//   decode.  Iteration = check phase (one conflict-free ds_read_b64 /
//   ds_write_b64 per edge of a pair; the update runs on float2, both checks in
//   every packed op) | barrier | variable phase (variables in pairs on float2:
//   DV gathers, posterior, extrinsic write-back) | barrier.  Channel LLRs in and
//   posteriors out are staged through LDS so their HBM traffic stays coalesced.
// ---------------------------------------------------------------------------
template <int DV, int DC, int T, int VPT, int ALGO, bool ET, bool MC>
__global__ __launch_bounds__(T) void bp_lds_kernel(BpArgs a) {
    static_assert(DC % 2 == 0, "pair layout: the ET parity reads whole words");
    static_assert(!ET || VPT <= 32, "early stop keeps one decision bit per lane in a 32-bit mask");
    extern __shared__ __align__(16) unsigned char smem[];
    float *msg = reinterpret_cast<float *>(smem);
    const int Ep = a.E + kLdsDummy;  // a.E = lds_pair_span(m, DC)
    uint8_t *hs = smem + (size_t)Ep * 4;
    int *curve = reinterpret_cast<int *>(smem + (((size_t)Ep * 5 + 15) & ~(size_t)15));
    const int tid = threadIdx.x;
    const int n = a.n, m = a.m, E = a.E, iters = a.max_iters;
    const int npairs = (m + 1) >> 1;
    constexpr int NS = VPT * DV;  // positions reached through my variables
    // The packed positions carry the dynamic LDS base (in words; not 0 when the
    // kernel also holds static LDS -- __syncthreads_or reduces through LDS), so
    // one SDWA shift yields the absolute address of a message.
    const int lpos0 = (int)((uint32_t)(size_t)(lds_u8 *)smem >> 2);
    uint8_t *hsb = hs - lpos0;  // hsb[address >> 2] = hs[position]

    // packed positions: codeword-independent, built once per workgroup
    uint32_t sp[(NS + 1) / 2];
#pragma unroll
    for (int q = 0; q < (NS + 1) / 2; ++q) sp[q] = 0;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
#pragma unroll
        for (int j = 0; j < DV; ++j) {
            const int q = i * DV + j;
            sp[q >> 1] |= (uint32_t)(a.lane_slot[(tid + i * T) * DV + j] + lpos0) << (16 * (q & 1));
        }
    }
    // PF: the next codeword's channel LLRs are loaded into registers (v = tid + k*T,
    // n <= VPT*T) while the current one writes its outputs, so a persistent
    // workgroup never waits for HBM between codewords
    constexpr bool PF = LDPC_LDS36_PREFETCH && !MC && !ET;  // (early stop: 2.6 % slower, not used)
    float nx[PF ? VPT : 1];
    if constexpr (PF) {
#pragma unroll
        for (int k = 0; k < VPT; ++k) {
            const int v = tid + k * T;
            nx[k] = v < n && (int)blockIdx.x < a.B ? a.llr[(size_t)blockIdx.x * n + v] : 0.0f;
        }
    }

    for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
        const uint64_t cw = a.first_cw + (uint64_t)b;
        // ---- stage the channel LLRs (coalesced) ----
        __syncthreads();  // previous codeword fully drained (msg, curve)
        if (MC) {
            for (int i = tid; i <= iters; i += T) curve[i] = 0;
        }
        int err0 = 0;
        if constexpr (PF) {
#pragma unroll
            for (int k = 0; k < VPT; ++k) {
                const int v = tid + k * T;
                if (v < n) msg[v] = to_msg<ALGO>(nx[k]);
            }
        } else {
            for (int v = tid; v < n; v += T) {
                const float l = MC ? chan_soft(a.ch, cw, v) : a.llr[(size_t)b * n + v];
                msg[v] = to_msg<ALGO>(l);
                err0 += (l < 0.0f);
            }
        }
        int lv[VPT];
#pragma unroll
        for (int i = 0; i < VPT; ++i) lv[i] = a.lane_var[tid + i * T];
        __syncthreads();
        float L[VPT];
#pragma unroll
        for (int i = 0; i < VPT; ++i) L[i] = lv[i] >= 0 ? msg[lv[i]] : 0.0f;
        // absolute LDS byte address of my variable i's edge j, and the word there
        auto addr = [&](int i, int j) -> uint32_t {
            const int q = i * DV + j;
            return (q & 1) ? pos_hi_x4(sp[q >> 1]) : pos_lo_x4(sp[q >> 1]);
        };
        auto at = [](uint32_t ba) -> lds_f32 & { return *(lds_f32 *)(size_t)ba; };
        __syncthreads();  // staging read before the message initialisation overwrites it
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            const float w = v2c_rwire<ALGO>(L[i]);
#pragma unroll
            for (int j = 0; j < DV; ++j) at(addr(i, j)) = w;
        }
        __syncthreads();
        if (MC) {
            const int w = wave_sum(err0);
            if ((tid & (kWave - 1)) == 0) atomicAdd(&curve[0], w);
        }

        // variable phase; FINAL (the last fixed-count iteration) keeps the
        // posteriors in registers instead of writing extrinsic messages.
        float pr[MC ? 1 : VPT];
        if constexpr (!MC) {
#pragma unroll
            for (int i = 0; i < VPT; ++i) pr[i] = L[i];
        }
        // PROD (sum-product, no early stop): L holds E = 2^channel from here on, the
        // check phase leaves ratios r = 2^c2v in LDS, and the variable phase forms
        // each edge's extrinsic ratio E * prod_{k != j} r_k by prefix / suffix
        // products -- no v_log_f32 per edge in the check phase, a v_rcp_f32 in place
        // of the v_exp_f32 here.  The posterior (FINAL) is L + sum log2 r_j in the
        // log-domain order, L = log2(E); MC tests post < 1.
        constexpr bool PROD = ALGO == 0;
        if constexpr (PROD) {
#pragma unroll
            for (int i = 0; i < VPT; ++i) L[i] = __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(L[i], -126.0f, 126.0f));
        }
        // ET: a variable's hard-decision bytes are rewritten only when its decision
        // changes (bit i of hb = the decision last written for lane i; hfirst makes
        // the first variable phase of a codeword write them all)
        uint32_t hb = 0u;
        bool hfirst = true;
        auto put_hard = [&](int i, bool h, const uint32_t(&ad)[DV]) {
            if (hfirst || ((hb >> i) & 1u) != (uint32_t)h) {
#pragma unroll
                for (int j = 0; j < DV; ++j) hsb[ad[j] >> 2] = (uint8_t)h;
            }
            hb = (hb & ~(1u << i)) | ((uint32_t)h << i);
        };
        auto llr_log2 = [&](int i) -> float {  // PROD: channel LLR of lane i, message units
            // log2(E) restores it to ~1e-7 absolute; a value clamped at staging
            // (|LLR| > 87 nats) is re-read from the input instead
            float l = __builtin_amdgcn_logf(L[i]);
            if (__builtin_expect(fabsf(l) >= 126.0f, 0)) {
                const int vv = a.lane_var[tid + i * T];
                l = vv >= 0 && !MC ? to_msg<ALGO>(a.llr[(size_t)b * n + vv]) : 0.0f;
            }
            return l;
        };
        auto var_phase_prod = [&](auto final_tag) {
            constexpr bool FINAL = decltype(final_tag)::value;
            int errs = 0;
            auto edges = [&](auto &cv, auto Ev, auto put_j) {
                // cv[j]: ratios of this variable's edges; put_j(j, wire)
                decltype(Ev) pre[DV];
                pre[0] = Ev;
#pragma unroll
                for (int j = 1; j < DV; ++j) pre[j] = pre[j - 1] * cv[j - 1];
                auto suf = cv[DV - 1];
                put_j(DV - 1, pre[DV - 1]);
#pragma unroll
                for (int j = DV - 2; j >= 0; --j) {
                    put_j(j, pre[j] * suf);
                    if (j > 0) suf = suf * cv[j];
                }
                return pre[DV - 1] * cv[DV - 1];  // posterior ratio
            };
#pragma unroll
            for (int i = 0; i + 1 < VPT; i += 2) {
                uint32_t a0[DV], a1[DV];
                float2 cv[DV];
#pragma unroll
                for (int j = 0; j < DV; ++j) {
                    a0[j] = addr(i, j);
                    a1[j] = addr(i + 1, j);
                }
#pragma unroll
                for (int j = 0; j < DV; ++j) cv[j] = make_float2(at(a0[j]), at(a1[j]));
                if constexpr (FINAL) {
                    float2 s = make_float2(llr_log2(i), llr_log2(i + 1));
#pragma unroll
                    for (int j = 0; j < DV; ++j)
                        s = s + make_float2(__builtin_amdgcn_logf(cv[j].x), __builtin_amdgcn_logf(cv[j].y));
                    if constexpr (!MC) { pr[i] = s.x; pr[i + 1] = s.y; }
                } else {
                    const float2 post = edges(cv, make_float2(L[i], L[i + 1]), [&](int j, float2 R) {
                        const float2 w = ratio_wire2(R);
                        at(a0[j]) = w.x;
                        at(a1[j]) = w.y;
                    });
                    if constexpr (ET) {
                        put_hard(i, post.x < 1.0f, a0);
                        put_hard(i + 1, post.y < 1.0f, a1);
                        if constexpr (!MC) {  // prod r_j (no E: cannot overflow); logged at the end
                            float2 pq = cv[0];
#pragma unroll
                            for (int j = 1; j < DV; ++j) pq = pq * cv[j];
                            pr[i] = pq.x;
                            pr[i + 1] = pq.y;
                        }
                    }
                    if constexpr (MC)
                        errs += ((a0[0] < 4u * (E + lpos0)) & (post.x < 1.0f)) + ((a1[0] < 4u * (E + lpos0)) & (post.y < 1.0f));
                    else (void)post;
                }
                if (LDPC_VAR_PAIRS > 0 && (i / 2) % LDPC_VAR_PAIRS == LDPC_VAR_PAIRS - 1)
                    __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (VPT % 2 == 1) {
                constexpr int i = VPT - 1;
                uint32_t a0[DV];
                float cv[DV];
#pragma unroll
                for (int j = 0; j < DV; ++j) a0[j] = addr(i, j);
#pragma unroll
                for (int j = 0; j < DV; ++j) cv[j] = at(a0[j]);
                if constexpr (FINAL) {
                    float s = llr_log2(i);
#pragma unroll
                    for (int j = 0; j < DV; ++j) s += __builtin_amdgcn_logf(cv[j]);
                    if constexpr (!MC) pr[i] = s;
                } else {
                    const float post = edges(cv, L[i], [&](int j, float R) { at(a0[j]) = ratio_wire(R); });
                    if constexpr (ET) {
                        put_hard(i, post < 1.0f, a0);
                        if constexpr (!MC) {
                            float pq = cv[0];
#pragma unroll
                            for (int j = 1; j < DV; ++j) pq *= cv[j];
                            pr[i] = pq;
                        }
                    }
                    if constexpr (MC) errs += (a0[0] < 4u * (E + lpos0)) & (post < 1.0f);
                    else (void)post;
                }
            }
            return errs;
        };
        auto var_phase = [&](auto final_tag) {
            constexpr bool FINAL = decltype(final_tag)::value;
            int errs = 0;
            // variables i, i+1 on float2 (packed sums and differences)
#pragma unroll
            for (int i = 0; i + 1 < VPT; i += 2) {
                uint32_t a0[DV], a1[DV];
                float2 cv[DV];
                float2 s = make_float2(L[i], L[i + 1]);
#pragma unroll
                for (int j = 0; j < DV; ++j) {  // all addresses first: the gathers issue back to back
                    a0[j] = addr(i, j);
                    a1[j] = addr(i + 1, j);
                }
#pragma unroll
                for (int j = 0; j < DV; ++j) cv[j] = make_float2(at(a0[j]), at(a1[j]));
#pragma unroll
                for (int j = 0; j < DV; ++j) s = s + cv[j];
                if constexpr (!FINAL) {
#pragma unroll
                    for (int j = 0; j < DV; ++j) {
                        const float2 w = s - cv[j];  // min-sum (sum-product: var_phase_prod)
                        at(a0[j]) = w.x;
                        at(a1[j]) = w.y;
                    }
                }
                if constexpr (!MC) {
                    if (FINAL || ET) { pr[i] = s.x; pr[i + 1] = s.y; }
                }
                if constexpr (ET) {
                    put_hard(i, s.x < 0.0f, a0);
                    put_hard(i + 1, s.y < 0.0f, a1);
                }
                if constexpr (MC) errs += ((a0[0] < 4u * (E + lpos0)) & (s.x < 0.0f)) + ((a1[0] < 4u * (E + lpos0)) & (s.y < 0.0f));
                // LDPC_VAR_PAIRS pairs' gathers in flight per thread (VGPR budget of
                // 4 waves/SIMD; the CU's 16 waves hide LDS latency)
                if (LDPC_VAR_PAIRS > 0 && (i / 2) % LDPC_VAR_PAIRS == LDPC_VAR_PAIRS - 1)
                    __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (VPT % 2 == 1) {
                constexpr int i = VPT - 1;
                uint32_t a0[DV];
                float cv[DV];
                float s = L[i];
#pragma unroll
                for (int j = 0; j < DV; ++j) a0[j] = addr(i, j);
#pragma unroll
                for (int j = 0; j < DV; ++j) cv[j] = at(a0[j]);
#pragma unroll
                for (int j = 0; j < DV; ++j) s += cv[j];
                if constexpr (!FINAL) {
#pragma unroll
                    for (int j = 0; j < DV; ++j) at(a0[j]) = s - cv[j];
                }
                if constexpr (!MC) {
                    if (FINAL || ET) pr[i] = s;
                }
                if constexpr (ET) {
                    put_hard(i, s < 0.0f, a0);
                }
                if constexpr (MC) errs += (a0[0] < 4u * (E + lpos0)) & (s < 0.0f);
            }
            return errs;
        };

        int it = 0;
        for (; it < iters; ++it) {
            if (it > 0) __syncthreads();  // variable phase (msg, hs) complete
            // check phase; with ET it also evaluates the syndrome of the previous
            // iteration's hard decisions, and the decoder stops before the next
            // variable phase when every check is satisfied
            int unsat = 0;
#pragma unroll LDPC_CHECK_PAIRS_UNROLL
            for (int q = tid; q < npairs; q += T) {
                float2 *pp = reinterpret_cast<float2 *>(msg) + q * DC;
                if (ET && it > 0) {
                    // the pair's 2*DC decision bytes: even bytes check 2q, odd 2q+1
                    const uint32_t *hw = reinterpret_cast<const uint32_t *>(hs + q * 2 * DC);
                    uint32_t x = 0;
#pragma unroll
                    for (int w = 0; w < DC / 2; ++w) x ^= hw[w];
                    x ^= x >> 16;
                    unsat |= (x & 1) | (2 * q + 1 < m ? (x >> 8) & 1 : 0);
                }
                float2 x2[DC];
#pragma unroll
                for (int i = 0; i < DC; ++i) x2[i] = pp[i];
                if constexpr (ALGO == 0) {
                    check_update_spa_pair_rwire<DC>(x2);
                } else {
                    float xa[DC], xb[DC];
#pragma unroll
                    for (int i = 0; i < DC; ++i) { xa[i] = x2[i].x; xb[i] = x2[i].y; }
                    if constexpr (DC == 6) {
                        check_update_ms6(xa, a.alpha);
                        check_update_ms6(xb, a.alpha);
                    } else {
                        check_update<ALGO, DC>(xa, a.alpha);
                        check_update<ALGO, DC>(xb, a.alpha);
                    }
#pragma unroll
                    for (int i = 0; i < DC; ++i) x2[i] = make_float2(xa[i], xb[i]);
                }
#pragma unroll
                for (int i = 0; i < DC; ++i) pp[i] = x2[i];
            }
            if constexpr (ET) {
                if (!__syncthreads_or(unsat | (it == 0))) break;
            } else {
                __syncthreads();
            }
            // fixed-count decode: the last variable phase runs after the loop
            if (!ET && !MC && it == iters - 1) break;
            int errs = 0;
            {
                if constexpr (PROD) errs = var_phase_prod(std::false_type{});
                else errs = var_phase(std::false_type{});
            }
            hfirst = false;
            if (MC) {
                const int w = wave_sum(errs);
                if ((tid & (kWave - 1)) == 0) atomicAdd(&curve[it + 1], w);
            }
        }
        if (!ET && !MC && iters > 0) {
            if constexpr (PROD) (void)var_phase_prod(std::true_type{});
            else (void)var_phase(std::true_type{});
            it = iters;
        }
        if constexpr (PF) {
            const int bn = b + (int)gridDim.x;
#pragma unroll
            for (int k = 0; k < VPT; ++k) {
                const int v = tid + k * T;
                if (v < n && bn < a.B) nx[k] = a.llr[(size_t)bn * n + v];
            }
        }
        if constexpr (PROD && ET && !MC) {  // early stop: posterior = L + log2(prod r_j)
            if (iters > 0) {
#pragma unroll
                for (int i = 0; i < VPT; ++i) pr[i] = llr_log2(i) + __builtin_amdgcn_logf(pr[i]);
            }
        }
        if constexpr (MC) {
            __syncthreads();
            int32_t *tr = a.trial + (size_t)b * (iters + 1);
            const int last = curve[it];
            for (int i = tid; i <= iters; i += T) tr[i] = i <= it ? curve[i] : last;
            if (tid == 0) a.its[b] = it;
        } else {
            // posteriors out through LDS (coalesced HBM writes)
            __syncthreads();
#pragma unroll
            for (int i = 0; i < VPT; ++i) {
                const int vv = a.lane_var[tid + i * T];
                if (vv >= 0) msg[vv] = pr[i];
            }
            __syncthreads();
            for (int v = tid; v < n; v += T) {
                const float s = msg[v];
                if (a.post) a.post[(size_t)b * n + v] = s * Domain<ALGO>::out;
                if (a.hard) a.hard[(size_t)b * n + v] = (uint8_t)(s < 0.0f);
            }
            if (a.its && tid == 0) a.its[b] = it;
        }
    }
}

// ---------------------------------------------------------------------------
// 2a'. Local-edge kernel (layout: loc_layout.cpp).  One codeword per workgroup of T
//   threads; thread t updates check pairs q = t + kT (k < KP) and the four variables
//   those checks hold as their local variables (var pairs 2k, 2k+1 on float2, .x = the
//   pair's first check side).  The local edge of each variable -- one per variable --
//   stays in a VGPR (loc[]) for the whole decode: the check phase reads it as input
//   slot s of check pair k and overwrites it with the check's output; the variable
//   phase reads that and overwrites it with the variable's extrinsic message.  Only the
//   other E - n messages live in LDS (rows per degree class, lane-contiguous
//   ds_read_b128 / ds_read_b64 on the check side, gathers on the variable side).
//   Sum-product in the product domain as bp_lds_kernel (R-wire, elementary-symmetric
//   check rule); min-sum in natural units, variable sums in variable_to_check_list order
//   (the local edge spliced in at its index) so it stays bit-exact with the oracle.
//   ABS: some variables have fewer than DVN+1 edges; their absent edges gather the
//   neutral value (ratio 1 / sum 0) and write to a private dummy word.
// ---------------------------------------------------------------------------
// SGN (sum-product with early stop): every non-local v->c ratio carries its variable's hard
// decision in one bit; with the decisions of the pair's two local variables (lpar, from the
// thread's own decision bits: bit 0 the .x check's, bit 1 the .y check's parity of them) the
// pair's parities are the syndrome of the previous variable phase (returned: 1 = a check of
// the pair unsatisfied).  The bit is the ratio's mantissa LSB (a relative change of at most
// 2^-23, far below the rule's ~10-ulp error), so the check rule takes the inputs as they are:
// the parity is two v_bitop3 XOR chains and one OR per pair, no input needs its sign stripped,
// and the local edges (registers) carry no stamp.
// seed ^ the words of entries 2 .. N-1 (N <= D) of one half of x
template <int N, int D>
__device__ __forceinline__ uint32_t bits_parity(const float2 (&x)[D], bool hi, uint32_t seed) {
    auto w = [&](int j) { return __float_as_uint(hi ? x[j].y : x[j].x); };
    uint32_t p = seed;
    int j = 2;
#pragma unroll
    for (; j + 1 < N; j += 2) p = xor3u(p, w(j), w(j + 1));
    if (j < N) p ^= w(j);
    return p;
}
template <int D, int ALGO, bool MIXED = false, bool SGN = false>
__device__ __forceinline__ int loc_check_pair(float *msg, int W, int Nc, int i, float2 &l0, float2 &l1, float alpha,
                                              uint32_t lpar = 0u) {
    constexpr int U = D - 2;
    float2 x[D];
    x[0] = l0;
    x[1] = l1;
#pragma unroll
    for (int r = 0; r < U / 2; ++r) {
        const float4 f = *reinterpret_cast<const float4 *>(msg + W + r * 4 * Nc + 4 * i);
        x[2 + 2 * r] = make_float2(f.x, f.y);
        x[3 + 2 * r] = make_float2(f.z, f.w);
    }
    if constexpr (U % 2) x[D - 1] = *reinterpret_cast<const float2 *>(msg + W + (U / 2) * 4 * Nc + 2 * i);
    int unsat = 0;
    if constexpr (SGN) {  // raw parity words: the caller ORs them and tests bit 0 once
        // a mixed pair's .x check has D - 1 inputs: its pad slot holds the rule's output for the
        // padding input (an arbitrary LSB), not a variable's decision
        unsat = (int)(bits_parity<MIXED ? D - 1 : D, D>(x, false, lpar) | bits_parity<D, D>(x, true, lpar >> 1));
    }
    if constexpr (ALGO == 0) {
        if constexpr (MIXED) {  // the .x check has D - 1 edges: pad input R = 0
            x[D - 1].x = 0.0f;
            check_update_spa_pair_rwire<D, true>(x);
        } else {
            check_update_spa_pair_rwire<D>(x);
        }
    } else {
        float xa[D], xb[D];
#pragma unroll
        for (int j = 0; j < D; ++j) { xa[j] = x[j].x; xb[j] = x[j].y; }
        if constexpr (MIXED) {  // pad: an infinite magnitude changes no minimum or sign
            xa[D - 1] = __builtin_inff();
            check_update<1, D>(xa, alpha);
            check_update<1, D>(xb, alpha);
        } else if constexpr (D == 6) {
            check_update_ms6(xa, alpha);
            check_update_ms6(xb, alpha);
        } else {
            check_update<1, D>(xa, alpha);
            check_update<1, D>(xb, alpha);
        }
#pragma unroll
        for (int j = 0; j < D; ++j) x[j] = make_float2(xa[j], xb[j]);
    }
#pragma unroll
    for (int r = 0; r < U / 2; ++r)
        *reinterpret_cast<float4 *>(msg + W + r * 4 * Nc + 4 * i) =
            make_float4(x[2 + 2 * r].x, x[2 + 2 * r].y, x[3 + 2 * r].x, x[3 + 2 * r].y);
    if constexpr (U % 2) *reinterpret_cast<float2 *>(msg + W + (U / 2) * 4 * Nc + 2 * i) = x[D - 1];
    l0 = x[0];
    l1 = x[1];
    return unsat;
}

// code = dy, or dy | dx << 8 for a mixed pair (dx = dy - 1 = DHI - 1 only)
template <int D, int DHI, int ALGO, bool SGN>
__device__ __forceinline__ int loc_check_dispatch(int code, float *msg, int W, int Nc, int i, float2 &l0, float2 &l1,
                                                  float alpha, uint32_t lpar) {
    if constexpr (D == DHI) {
        if (code >> 8) return loc_check_pair<D, ALGO, true, SGN>(msg, W, Nc, i, l0, l1, alpha, lpar);
        return loc_check_pair<D, ALGO, false, SGN>(msg, W, Nc, i, l0, l1, alpha, lpar);
    } else {
        if (code == D) return loc_check_pair<D, ALGO, false, SGN>(msg, W, Nc, i, l0, l1, alpha, lpar);
        return loc_check_dispatch<D + 1, DHI, ALGO, SGN>(code, msg, W, Nc, i, l0, l1, alpha, lpar);
    }
}

// a load whose index the compiler may not hoist out of the codeword loop (it would keep
// one 64-bit address per load live across the decode -- VGPRs the loop needs)
template <typename V>
__device__ __forceinline__ V ld_fresh(const V *p, int idx) {
    asm volatile("" : "+v"(idx));
    return p[idx];
}

// Workgroup-wide OR of a per-lane predicate with ONE barrier (__syncthreads_or reduces
// through a wave DPP chain, an LDS atomic and three barriers): each wave whose ballot is
// non-zero has lane 0 store 1 to flag[par]; after the barrier every thread reads it; thread 0
// then clears flag[par ^ 1] -- its previous readers are all past this barrier, and its next
// writers are behind the next one.  flag[] must be zero before the first call; alternate par.
__device__ __forceinline__ bool block_any(int pred, uint32_t *flag, int par) {
    if (__builtin_amdgcn_ballot_w64(pred != 0) != 0 && (threadIdx.x & (kWave - 1)) == 0) flag[par] = 1u;
    __syncthreads();
    const bool any = flag[par] != 0u;
    if (threadIdx.x == 0) flag[par ^ 1] = 0u;
    return any;
}
// block_any's count form: the number of waves' lanes with pred set (one LDS atomic per wave)
__device__ __forceinline__ uint32_t block_count(int pred, uint32_t *flag, int par) {
    const uint64_t bal = __builtin_amdgcn_ballot_w64(pred != 0);
    if (bal != 0 && (threadIdx.x & (kWave - 1)) == 0) atomicAdd(&flag[par], (uint32_t)__popcll(bal));
    __syncthreads();
    const uint32_t c = flag[par];
    if (threadIdx.x == 0) flag[par ^ 1] = 0u;
    return c;
}
#ifndef LDPC_LOC_EP_W0
#define LDPC_LOC_EP_W0 48  // early stop with posteriors: slab writes after syndromes with <= this many threads unsatisfied
#endif
#ifndef LDPC_LOC_PERSIST
#define LDPC_LOC_PERSIST 1  // bp_loc_kernel early stop without posteriors: persistent grid on a counter (2: every launch; fixed count +0.4 %, noise)
#endif
#ifndef LDPC_LOC_PRIO
// wave priority by phase: the variable phase (LDS-bound gathers / scatters) at s_setprio 1, the
// check phase (VALU-bound) at 0 -- two co-resident workgroups in opposite phases then share the
// SIMD in favour of the one that feeds the LDS pipe.  Headline +1.9 % (28.94 -> 28.39 ms), early
// stop and Monte-Carlo +1-3 %; the reverse assignment -2.4 %, odd workgroups at 1 neutral.
#define LDPC_LOC_PRIO 1
#endif


// DVN0 / DVN1: non-local edges per variable of local slot 0 / 1 (max); ABS0 / ABS1: some
// variable of that slot has fewer (its absent edges gather the neutral value).
// MC (sum-product): fused Philox channel, per-iteration error counts of the all-zero
// codeword into the trial curve, no posteriors; ET with MC: syndrome early stop on the
// sign-bit decisions (see loc_check_pair).  ET without MC (hard-decision decodes: the caller
// asked for no posteriors): the same stop, the decisions of the stopping iteration kept in a
// bit per variable (hbits) and written out; a frame that never stops takes the fixed-count
// epilogue.
// 512 threads with up to 5 check pairs each: two workgroups per CU (4 waves per SIMD, <= 128
// VGPRs), so one workgroup's barrier waits overlap the other's work; else one workgroup
constexpr int loc_waves_per_simd(int T, int KP) { return T == 512 && KP <= 5 ? 4 : 1; }

template <int DLO, int DHI, int DVN0, int DVN1, int KP, int T, int ALGO, bool ABS0, bool ABS1, bool ET = false,
          bool MC = false, bool EP = false>
__global__ __launch_bounds__(T, loc_waves_per_simd(T, KP)) void bp_loc_kernel(BpArgs a) {
    static_assert(!ET || ALGO == 0 || DLO == DHI, "min-sum early stop: one check class");
    static_assert(!ET || 2 * 2 * KP <= 64, "early stop keeps the thread's decisions in one 64-bit word");
    // MSET (min-sum Monte-Carlo with early stop): min-sum messages carry their own signs, so
    // the decisions cannot ride in them as in sum-product; instead every change of a
    // variable's decision XORs its checks' bits of an LDS syndrome (a few atomics once
    // decoding settles) and the next check phase tests that syndrome
    constexpr bool MSET = ET && ALGO == 1;
    constexpr bool SGN_LSB = ET && ALGO == 0;
    constexpr int VP = 2 * KP;  // variable pairs per thread
    constexpr int DVM = DVN0 > DVN1 ? DVN0 : DVN1;
    constexpr int DVA = DVM > 0 ? DVM : 1;
    constexpr int DVP = DVA;  // rows of loc_pos per var pair
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ uint32_t stop_flag[2];  // early stop: block_any's double-buffered flag
    float *msg = reinterpret_cast<float *>(smem);
    const int tid = threadIdx.x;
    const int n = a.n, iters = a.max_iters;
    const int lpos0 = (int)((uint32_t)(size_t)(lds_u8 *)smem >> 2);
    const uint32_t base2 = (uint32_t)lpos0 | ((uint32_t)lpos0 << 16);
    constexpr bool SPA = ALGO == 0;
    constexpr bool INF0 = ABS0 || ALGO == 1, INF1 = ABS1 || ALGO == 1;
    uint32_t sp[VP][DVA];
    uint32_t inf[VP];
    // packed LDS word pair of var pair v's non-local edge u (re-read per codeword and for
    // the posterior gathers: not held live outside the iteration loop, where the
    // staging and epilogue need the VGPRs)
    auto load_sp = [&](int v, int u) {
        return (uint32_t)ld_fresh(a.loc_pos, (v * DVP + u) * T + tid) + base2;
    };
    // the variable ids of the thread's var pairs (entry 2v + h; -1: none), every load issued
    // before the first use (one L2 round trip, not one per var pair; Monte-Carlo staging)
    auto load_vars = [&](int (&vv)[2 * VP]) {
#pragma unroll
        for (int i = 0; i < 2 * VP; ++i) vv[i] = ld_fresh(a.loc_var, i * T + tid);
    };
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        if constexpr (INF0) inf[2 * k] = (uint32_t)a.loc_info[(2 * k) * T + tid];
        if constexpr (INF1) inf[2 * k + 1] = (uint32_t)a.loc_info[(2 * k + 1) * T + tid];
    }
    auto at = [](uint32_t ba) -> lds_f32 & { return *(lds_f32 *)(size_t)ba; };
    const float neutral = SPA ? 1.0f : 0.0f;

    // gather the non-local c->v messages of var pair v (slot s) into cv[0 .. DN-1]
    auto gather = [&](auto dn_tag, auto abs_tag, int v, const uint32_t (&spv)[DVA], float2 (&cv)[DVA],
                      uint32_t (&a0)[DVA], uint32_t (&a1)[DVA]) {
        constexpr int DN = decltype(dn_tag)::value;
        constexpr bool AB = decltype(abs_tag)::value;
#pragma unroll
        for (int u = 0; u < DN; ++u) {
            a0[u] = pos_lo_x4(spv[u]);
            a1[u] = pos_hi_x4(spv[u]);
        }
#pragma unroll
        for (int u = 0; u < DN; ++u) cv[u] = make_float2(at(a0[u]), at(a1[u]));
        if constexpr (AB) {
#pragma unroll
            for (int u = 0; u < DN; ++u) {
                cv[u].x = (inf[v] >> u) & 1u ? cv[u].x : neutral;
                cv[u].y = (inf[v] >> (u + 4)) & 1u ? cv[u].y : neutral;
            }
        }
    };
    // min-sum posterior of var pair v: L + messages in variable_to_check_list order,
    // the local one spliced in at its index jl (the oracle's order: bit-exact)
    auto ms_sum = [&](auto dn_tag, int v, const float2 &Lv, const float2 &lv, const float2 (&cv)[DVA]) {
        constexpr int DN = decltype(dn_tag)::value;
        if constexpr (DN == 2) {
            // three terms in order: jl = 0 (ml, n0, n1), 1 (n0, ml, n1), 2 (n0, n1, ml); the masks
            // jl == 0 / jl == 2 are sign-extended one-hot bits of loc_info (v_bfe_i32), the
            // selects v_bfi_b32 -- VALU only, no per-lane masks held in SGPRs
            float s2[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t e0 = (uint32_t)__builtin_amdgcn_sbfe((int)inf[v], 16 + 4 * h, 1);
                const uint32_t e2 = (uint32_t)__builtin_amdgcn_sbfe((int)inf[v], 18 + 4 * h, 1);
                const uint32_t ml = __float_as_uint(h ? lv.y : lv.x);
                const uint32_t n0 = __float_as_uint(h ? cv[0].y : cv[0].x), n1 = __float_as_uint(h ? cv[1].y : cv[1].x);
                const float a0 = __uint_as_float(bfi_u32(e0, ml, n0));
                const uint32_t u = bfi_u32(e0, n0, ml);
                const float a1 = __uint_as_float(bfi_u32(e2, n1, u));
                const float a2 = __uint_as_float(bfi_u32(e2, ml, n1));
                s2[h] = (((h ? Lv.y : Lv.x) + a0) + a1) + a2;
            }
            return make_float2(s2[0], s2[1]);
        }
        float s2[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int jl = (inf[v] >> (8 + 2 * h)) & 3;
            const float ml = h ? lv.y : lv.x;
            float s = h ? Lv.y : Lv.x;
#pragma unroll
            for (int j = 0; j <= DN; ++j) {
                const float nl = j == 0 ? 0.0f : (h ? cv[j - 1].y : cv[j - 1].x);
                const float nl2 = j < DN ? (h ? cv[j].y : cv[j].x) : 0.0f;
                s += j < jl ? nl2 : (j == jl ? ml : nl);
            }
            s2[h] = s;
        }
        return make_float2(s2[0], s2[1]);
    };

    int *curve = reinterpret_cast<int *>(smem + (((size_t)(a.loc_words + 64 > n ? a.loc_words + 64 : n) * 4 + 15) &
                                                  ~(size_t)15));
    uint32_t *syn = reinterpret_cast<uint32_t *>(reinterpret_cast<unsigned char *>(curve) +
                                                 (((size_t)(iters + 1) * 4 + 15) & ~(size_t)15));
    const int nsw = (2 * a.loc_P + 31) >> 5;  // MSET: syndrome words (bit 2q + h: check h of pair q)
    // MSET / hard-decision ET: the thread's current decisions, bits 2v, 2v + 1 of var pair v
    using HB = std::conditional_t<(4 * KP > 32), uint64_t, uint32_t>;
    static_assert(!MSET || sizeof(HB) == 4, "MSET: 32-bit decision word");
    HB hbits = 0;
    HB lpar = 0;  // SGN: the parity of each check's two local decisions (see bits_parity)
    // MSET: the decisions that changed in a variable phase (chm, bit 2v + h: hbits before XOR
    // after) flip the syndrome bits of their checks -- the local one (pair q = tid + (v/2) T, bit
    // 2q + h) and the non-local ones (from the slot's packed LDS positions, re-read from L2:
    // a select chain over the register copies measured 15 % slower).
    // Each lane walks its own marks after the phase, so the wave loops max-over-lanes times
    // instead of running a var pair's flips whenever one lane of the wave changed it.
    uint32_t chm = 0u;
    auto syn_flush = [&]() {
        uint32_t mk = chm;
        chm = 0u;
        const uint32_t P4 = 4u * (uint32_t)a.loc_P;
        constexpr int NF = 2;  // flips per trip (1: -0.4 %, 4: -1.5 %, profiles/r05_ab_flip_batch_locvar.txt)
        while (__builtin_amdgcn_ballot_w64(mk != 0u)) {
            // NF flips per trip: every flip's non-local positions loaded before the first use
            // (one L2 round trip per NF flips; rows u < DVM exist for every var pair, so the
            // loads need no guard), the 16-bit half by a bit-field extract (no branch)
            int bit[NF];
            bool on[NF];
            uint32_t raw[NF][DVA];
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                bit[f] = mk ? (int)__builtin_ctz(mk) : 0;
                on[f] = mk != 0u && tid + (bit[f] >> 2) * T < a.loc_P;  // var pair v = bit / 2, pair slot v / 2
                mk &= mk - 1u;
            }
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int u = 0; u < DVM; ++u) raw[f][u] = (uint32_t)a.loc_pos[((bit[f] >> 1) * DVP + u) * T + tid];
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                if (on[f]) {
                    const int v = bit[f] >> 1, h = bit[f] & 1;
                    const int q = tid + (v >> 1) * T;
                    const uint32_t bl = 2u * (uint32_t)q + (uint32_t)h;
                    atomicXor(&syn[bl >> 5], 1u << (bl & 31));
                    const int dn = (v & 1) ? DVN1 : DVN0;
#pragma unroll
                    for (int u = 0; u < DVM; ++u) {
                        if (u < dn) {
                            uint32_t w = __builtin_amdgcn_ubfe(raw[f][u], 16u * (uint32_t)h, 16u);
                            w = w >= P4 ? w - P4 : w;
                            const uint32_t bn = 2u * (w >> 2) + (w & 1u);
                            atomicXor(&syn[bn >> 5], 1u << (bn & 31));
                        }
                    }
                }
            }
        }
    };
    // EP (early stop, posteriors asked for): a persistent grid takes codewords from a global
    // counter (frames stop at different iterations) and keeps each variable pair's product of
    // incoming c->v ratios (min-sum: its posterior sum) of the latest variable phase in the
    // workgroup's slab, a.scratch + blockIdx.x * VP * T float2 (lane-contiguous stores, L2-
    // resident: 40 KB per workgroup); the stopping iteration's posteriors come from there.
    // The slab is written only in variable phases that follow a check phase with at most
    // LDPC_LOC_EP_W0 threads holding an unsatisfied check (frames converge through nearly
    // satisfied syndromes); a frame that stops without a slab from its last variable phase
    // is decoded again from its channel LLRs -- the same deterministic trajectory -- with
    // the slab written in that variable phase (redo_it).
    static_assert(!EP || (ET && !MC), "EP: early-stop decodes with posteriors");
    constexpr bool ep = EP;
    float2 *slab = ep ? reinterpret_cast<float2 *>(a.scratch) + (size_t)blockIdx.x * VP * T : nullptr;
    // persistent grid (a.work: EP, and early stop without posteriors when LDPC_LOC_PERSIST):
    // codewords come from a global counter; thread 0 claims the next one a codeword ahead, so
    // the atomic's latency hides behind the current decode
    __shared__ int next_b;
    const bool per = a.work != nullptr;
    uint32_t claim = 0u;
    for (int round = 0;; ++round) {
        if (per && tid == 0) next_b = round == 0 ? (int)atomicAdd(a.work, 1u) : (int)claim;
        __syncthreads();  // the previous codeword's outputs are out of LDS; next_b visible
        const int b = per ? __builtin_amdgcn_readfirstlane(next_b) : (int)blockIdx.x + round * (int)gridDim.x;
        if (b >= a.B) break;
        if (per && tid == 0) claim = atomicAdd(a.work, 1u);
        const uint64_t cw = a.first_cw + (uint64_t)b;
        int redo_it = -1;  // EP: the variable phase whose slab a second pass must write
    restart:
        int slab_it = -2;  // EP: the variable phase that last wrote the slab
        bool slab_now = false;
        if constexpr (ET) {
            if (tid == 0) stop_flag[0] = stop_flag[1] = 0u;  // visible after the staging barrier
        }
        int err0 = 0;
        if constexpr (MC) {
            for (int i = tid; i <= iters; i += T) curve[i] = 0;
            if constexpr (MSET)
                for (int i = tid; i < nsw; i += T) syn[i] = 0u;
            for (int g4 = tid; g4 < (n + 3) >> 2; g4 += T) {  // one Philox block per four variables
                const uint4 r = chan_block(a.ch, cw, g4);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (4 * g4 + q >= n) break;
                    const float l = chan_soft_word(a.ch, r, q);
                    msg[4 * g4 + q] = to_msg<ALGO>(l);
                    err0 += (l < 0.0f);
                }
            }
        } else {
            if constexpr (MSET)
                for (int i = tid; i < nsw; i += T) syn[i] = 0u;
            for (int v = tid; v < n; v += T) msg[v] = to_msg<ALGO>(a.llr[(size_t)b * n + v]);
        }
        __syncthreads();
        if constexpr (MC) {
            const int w = wave_sum(err0);
            if ((tid & (kWave - 1)) == 0) atomicAdd(&curve[0], w);
        }
#pragma unroll
        for (int k = 0; k < KP; ++k) {
#pragma unroll
            for (int u = 0; u < DVN0; ++u) sp[2 * k][u] = load_sp(2 * k, u);
#pragma unroll
            for (int u = 0; u < DVN1; ++u) sp[2 * k + 1][u] = load_sp(2 * k + 1, u);
        }
        float2 L[VP];  // SPA: E = 2^channel (clamped); min-sum: channel LLR
        if constexpr (MC) {  // (the other decodes: neutral to 0.5 % slower with the batch, registers)
            int vv[2 * VP];
            load_vars(vv);
#pragma unroll
            for (int v = 0; v < VP; ++v)
                L[v] = make_float2(vv[2 * v] >= 0 ? msg[vv[2 * v]] : 0.0f, vv[2 * v + 1] >= 0 ? msg[vv[2 * v + 1]] : 0.0f);
        } else {
#pragma unroll
            for (int v = 0; v < VP; ++v) {
                const int v0 = ld_fresh(a.loc_var, (v * 2 + 0) * T + tid), v1 = ld_fresh(a.loc_var, (v * 2 + 1) * T + tid);
                L[v] = make_float2(v0 >= 0 ? msg[v0] : 0.0f, v1 >= 0 ? msg[v1] : 0.0f);
            }
        }
        __syncthreads();
        float2 loc[VP];
        auto init = [&](auto dn_tag, int v) {
            constexpr int DN = decltype(dn_tag)::value;
            float2 w;
            if constexpr (SPA) {
                w = make_float2(__builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(L[v].x, -23.0f, 23.0f)),
                                __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(L[v].y, -23.0f, 23.0f)));
                if constexpr (ET)  // the channel decision in the LSB
                    w = make_float2(__uint_as_float(bfi_lsb(__float_as_uint(w.x), (uint32_t)(L[v].x < 0.0f))),
                                    __uint_as_float(bfi_lsb(__float_as_uint(w.y), (uint32_t)(L[v].y < 0.0f))));
                L[v] = make_float2(__builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(L[v].x, -126.0f, 126.0f)),
                                   __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(L[v].y, -126.0f, 126.0f)));
            } else {
                w = L[v];
                if constexpr (MSET) {  // the channel decisions' syndrome
                    const int d0 = (int)(w.x < 0.0f) | ((int)(w.y < 0.0f) << 1);
                    hbits |= (uint32_t)d0 << (2 * v);
                    chm |= (uint32_t)d0 << (2 * v);
                }
            }
            loc[v] = w;
#pragma unroll
            for (int u = 0; u < DN; ++u) {
                at(pos_lo_x4(sp[v][u])) = w.x;
                at(pos_hi_x4(sp[v][u])) = w.y;
            }
        };
        hbits = 0u;
#pragma unroll
        for (int k = 0; k < KP; ++k) {
            init(int_c<DVN0>{}, 2 * k);
            init(int_c<DVN1>{}, 2 * k + 1);
        }
        if constexpr (MSET) syn_flush();
        // variable phase of var pair v; returns the pair's hard decisions (bit 0: .x, 1: .y)
        auto var_pair = [&](auto dn_tag, auto abs_tag, int v) -> int {
            constexpr int DN = decltype(dn_tag)::value;
            constexpr int DV = DN + 1;
            uint32_t a0[DVA], a1[DVA];
            float2 cv[DVA];
            gather(dn_tag, abs_tag, v, sp[v], cv, a0, a1);
            int dec = 0;
            if constexpr (SPA) {
                // edges e_0 = local, e_{1+u} = non-local u: R_j = E prod_{k != j} e_k
                float2 pre[DV];
                pre[0] = L[v];
                if constexpr (DV > 1) pre[1] = pre[0] * loc[v];
#pragma unroll
                for (int j = 2; j < DV; ++j) pre[j] = pre[j - 1] * cv[j - 2];
                uint32_t sx = 0, sy = 0;  // ET: the decision rides in every outgoing mantissa LSB
                if constexpr (MC || ET) {
                    // P < 1 on the bits: P is a product of positive clamped ratios, so
                    // bits(P) - bits(1.0) is negative exactly when P < 1 (no compare / select)
                    const float2 P = DN > 0 ? pre[DV - 1] * cv[DN > 0 ? DN - 1 : 0] : pre[DV - 1];
                    const uint32_t dx = (__float_as_uint(P.x) + 0xC0800000u) >> 31;
                    const uint32_t dy = (__float_as_uint(P.y) + 0xC0800000u) >> 31;
                    dec = (int)(dx | dy << 1);
                    if constexpr (ET) {
                        sx = dx;
                        sy = dy;
                    }
                }
                auto sgn = [&](float2 R) {
                    if constexpr (ET)  // LSB := decision (one v_bfi_b32 per value)
                        return make_float2(__uint_as_float(bfi_lsb(__float_as_uint(R.x), sx)),
                                           __uint_as_float(bfi_lsb(__float_as_uint(R.y), sy)));
                    return R;
                };
                float2 suf = DN > 0 ? cv[DN > 0 ? DN - 1 : 0] : make_float2(1.0f, 1.0f);
#pragma unroll
                for (int j = DV - 1; j >= 1; --j) {
                    const float2 R = sgn(ratio_wire2(j == DV - 1 ? pre[j] : pre[j] * suf));
                    at(a0[j - 1]) = R.x;
                    at(a1[j - 1]) = R.y;
                    if (j < DV - 1) suf = suf * cv[j - 1];
                }
                if (ep && slab_now) slab[v * T + tid] = loc[v] * suf;  // prod of the incoming c->v ratios
                loc[v] = ratio_wire2(DN > 0 ? L[v] * suf : L[v]);  // local edge: its decision is in lpar
            } else {
                const float2 s = ms_sum(dn_tag, v, L[v], loc[v], cv);
                if (ep && slab_now) slab[v * T + tid] = s;  // the posterior itself
#pragma unroll
                for (int u = 0; u < DN; ++u) {
                    at(a0[u]) = s.x - cv[u].x;
                    at(a1[u]) = s.y - cv[u].y;
                }
                loc[v] = make_float2(s.x - loc[v].x, s.y - loc[v].y);
                // decisions from the sign bits: a min-sum posterior is never -0 (see to_msg)
                if constexpr (MC || ET)
                    dec = (int)((__float_as_uint(s.x) >> 31) | ((__float_as_uint(s.y) >> 31) << 1));
            }
            return dec;
        };
        int it = 0;
        bool stopped = false;
        for (; it < iters; ++it) {
            __syncthreads();  // variable phase (or initialisation) complete
            int unsat = 0;
            {  // the gathers' unpacked addresses stay in the loop
#pragma unroll
                for (int v = 0; v < VP; ++v)
#pragma unroll
                    for (int u = 0; u < DVA; ++u) asm volatile("" : "+v"(sp[v][u]));
            }
            if constexpr (ALGO == 1) {  // the order masks (ms_sum) are re-derived per iteration, not held
#pragma unroll
                for (int v = 0; v < VP; ++v) asm volatile("" : "+v"(inf[v]));
            }
            // ---- check phase ----
            if (LDPC_LOC_PRIO) __builtin_amdgcn_s_setprio(0);
#pragma unroll
            for (int k = 0; k < KP; ++k) {
                int q = tid + k * T;
                asm volatile("" : "+v"(q));  // recomputed per iteration: no per-pair addresses held live
                if (q < a.loc_P) {
                    if constexpr (DLO == DHI) {  // one class: rows of P pairs from word 0
                        unsat |= loc_check_pair<DLO, ALGO, false, ET && SPA>(msg, 0, a.loc_P, q, loc[2 * k],
                                                                             loc[2 * k + 1], a.alpha,
                                                                             (uint32_t)(lpar >> (4 * k)));
                    } else {
                        // class of q by selects on the (scalar) class table -- no per-lane
                        // indexing of kernel arguments
                        int q0 = a.loc_cls_q[0], q1 = a.loc_cls_q[1], W = a.loc_cls_w[0], d = a.loc_cls_d[0];
#pragma unroll
                        for (int j = 1; j < 4; ++j) {
                            const bool in = j < a.loc_ncls && q >= a.loc_cls_q[j];
                            q0 = in ? a.loc_cls_q[j] : q0;
                            q1 = in ? a.loc_cls_q[j + 1] : q1;
                            W = in ? a.loc_cls_w[j] : W;
                            d = in ? a.loc_cls_d[j] : d;
                        }
                        unsat |= loc_check_dispatch<DLO, DHI, ALGO, ET && SPA>(d, msg, W, q1 - q0, q - q0, loc[2 * k],
                                                                               loc[2 * k + 1], a.alpha,
                                                                               (uint32_t)(lpar >> (4 * k)));
                    }
                }
                if (LDPC_LOC_CGROUP > 0 && k % LDPC_LOC_CGROUP == LDPC_LOC_CGROUP - 1)
                    __builtin_amdgcn_sched_barrier(0);  // pairs in flight (VGPR budget)
            }
            if constexpr (MSET)
                for (int i = tid; i < nsw; i += T) unsat |= syn[i] != 0u;
            if constexpr (ET) {
                // the syndrome of the previous variable phase's decisions: stop when every
                // check is satisfied (oracle: after that iteration)
                if constexpr (SGN_LSB) unsat &= 1;  // the parities are in bit 0 of the OR of the pairs' words
                bool more;
                if constexpr (EP) {
                    const uint32_t cnt = block_count(unsat | (it == 0), stop_flag, it & 1);
                    more = cnt != 0u;
                    slab_now = cnt <= (uint32_t)LDPC_LOC_EP_W0 || it == redo_it;
                    if (more && slab_now) slab_it = it;
                } else {
                    more = block_any(unsat | (it == 0), stop_flag, it & 1);
                }
                if (!more) {
                    stopped = true;
                    break;
                }
            } else {
                __syncthreads();
            }
            if (!MC && it == iters - 1) break;  // the last variable phase only forms posteriors
            // ---- variable phase ----
            if (LDPC_LOC_PRIO) __builtin_amdgcn_s_setprio(1);
            int errs = 0;
            HB nh = 0;  // early stop: this phase's decisions, bits 2v, 2v + 1
            {
#pragma unroll
                for (int k = 0; k < KP; ++k) {
                    const int d0 = var_pair(int_c<DVN0>{}, bool_c<ABS0>{}, 2 * k);
                    if (LDPC_LOC_VGROUP == 1) __builtin_amdgcn_sched_barrier(0);
                    const int d1 = var_pair(int_c<DVN1>{}, bool_c<ABS1>{}, 2 * k + 1);
                    if (LDPC_LOC_VGROUP > 0) __builtin_amdgcn_sched_barrier(0);
                    if constexpr (ET) nh |= (HB)(d0 | d1 << 2) << (4 * k);
                    else if constexpr (MC) errs += tid + k * T < a.loc_P ? __builtin_popcount(d0) + __builtin_popcount(d1) : 0;
                }
            }
            if constexpr (ET) {
                if constexpr (MSET) chm = (uint32_t)(nh ^ hbits);
                hbits = nh;
                if constexpr (SGN_LSB) lpar = nh ^ (nh >> 2);  // bit 4k (+1): check 2q (+1)'s local parity
                if constexpr (MC) {  // pair slots k with tid + k T < P hold variables
                    const int lim = a.loc_P - tid, nk = lim <= 0 ? 0 : min(KP, (lim + T - 1) / T);
                    const HB vm = 4 * nk >= 8 * (int)sizeof(HB) ? ~(HB)0 : (((HB)1 << (4 * nk)) - 1);
                    errs = sizeof(HB) == 8 ? __builtin_popcountll((uint64_t)(nh & vm)) : __builtin_popcount((uint32_t)(nh & vm));
                }
                if constexpr (MSET) syn_flush();
            }
            if constexpr (MC) {
                const int w = wave_sum(errs);
                if ((tid & (kWave - 1)) == 0) atomicAdd(&curve[it + 1], w);
            }
        }
        if constexpr (MC) {
            __syncthreads();
            int32_t *tr = a.trial + (size_t)b * (iters + 1);
            const int last = curve[it];
            for (int i = tid; i <= iters; i += T) tr[i] = i <= it ? curve[i] : last;
            if (tid == 0) a.its[b] = it;
            continue;
        }
        if constexpr (ET && !MC) {
            if (stopped && ep && slab_it != it - 1) {  // no slab from the last variable phase: again
                redo_it = it - 1;
                __syncthreads();  // every thread is past its reads of this pass's LDS
                goto restart;
            }
            if (stopped && ep) {
                // posteriors of the stopping iteration from the slab (its last variable phase):
                // SPA log2 E + log2(prod c->v) -- the oracle's L + sum of the c->v messages -- and
                // the decisions that satisfied every check (hbits) as the hard decisions; staged
                // through LDS (posteriors in words [0, n), decision bytes after them: the messages
                // are dead once the stop is known)
                uint8_t *hb = reinterpret_cast<uint8_t *>(msg + n);
#pragma unroll
                for (int v = 0; v < VP; ++v) {
                    const float2 q = slab[v * T + tid];
                    float2 pv;
                    if constexpr (SPA) {
                        pv = make_float2(__builtin_amdgcn_logf(L[v].x) + __builtin_amdgcn_logf(q.x),
                                         __builtin_amdgcn_logf(L[v].y) + __builtin_amdgcn_logf(q.y));
                    } else {
                        pv = q;
                    }
                    const int v0 = ld_fresh(a.loc_var, (v * 2 + 0) * T + tid), v1 = ld_fresh(a.loc_var, (v * 2 + 1) * T + tid);
                    if constexpr (SPA) {  // a clamped E (|LLR| > 87 nats): the channel value itself
                        const float lx = __builtin_amdgcn_logf(L[v].x), ly = __builtin_amdgcn_logf(L[v].y);
                        if (v0 >= 0 && fabsf(lx) >= 125.5f) pv.x = to_msg<ALGO>(a.llr[(size_t)b * n + v0]) + __builtin_amdgcn_logf(q.x);
                        if (v1 >= 0 && fabsf(ly) >= 125.5f) pv.y = to_msg<ALGO>(a.llr[(size_t)b * n + v1]) + __builtin_amdgcn_logf(q.y);
                    }
                    if (v0 >= 0) {
                        msg[v0] = pv.x;
                        hb[v0] = (uint8_t)((hbits >> (2 * v)) & 1);
                    }
                    if (v1 >= 0) {
                        msg[v1] = pv.y;
                        hb[v1] = (uint8_t)((hbits >> (2 * v + 1)) & 1);
                    }
                }
                __syncthreads();
                for (int v = tid; v < n; v += T) {
                    a.post[(size_t)b * n + v] = msg[v] * Domain<ALGO>::out;
                    if (a.hard) a.hard[(size_t)b * n + v] = hb[v];
                }
                if (a.its && tid == 0) a.its[b] = it;
                continue;
            }
        }
        if constexpr (ET) {
            if (stopped) {  // hard decisions of the stopping iteration (no posteriors asked for)
#pragma unroll
                for (int v = 0; v < VP; ++v) {
                    const int v0 = ld_fresh(a.loc_var, (v * 2 + 0) * T + tid), v1 = ld_fresh(a.loc_var, (v * 2 + 1) * T + tid);
                    if (v0 >= 0) msg[v0] = (hbits >> (2 * v)) & 1 ? -1.0f : 1.0f;
                    if (v1 >= 0) msg[v1] = (hbits >> (2 * v + 1)) & 1 ? -1.0f : 1.0f;
                }
                __syncthreads();
                if (a.hard)
                    for (int v = tid; v < n; v += T) a.hard[(size_t)b * n + v] = (uint8_t)(msg[v] < 0.0f);
                if (a.its && tid == 0) a.its[b] = it;
                continue;
            }
        }
        // ---- posteriors (after the last check phase) and outputs ----
        // (variable ids re-read where needed: not kept live through the decode loop)
        float2 pr[VP];
        auto post = [&](auto dn_tag, auto abs_tag, int v) {
            constexpr int DN = decltype(dn_tag)::value;
            uint32_t a0[DVA], a1[DVA], spv[DVA];
            float2 cv[DVA];
#pragma unroll
            for (int u = 0; u < DN; ++u) spv[u] = load_sp(v, u);
            gather(dn_tag, abs_tag, v, spv, cv, a0, a1);
            if constexpr (SPA) {
                float2 s;
                // the channel term from the register-held E = 2^L: log2 E is L to ~1e-7 (no
                // second 40 KB read of the codeword's LLRs); a clamped E (|LLR| > 87 nats) takes
                // the input value itself
                s = make_float2(__builtin_amdgcn_logf(L[v].x), __builtin_amdgcn_logf(L[v].y));
                if (fabsf(s.x) >= 125.5f || fabsf(s.y) >= 125.5f) {
                    const float *lb = a.llr + (size_t)b * n;
                    const int v0 = ld_fresh(a.loc_var, (v * 2 + 0) * T + tid);
                    const int v1 = ld_fresh(a.loc_var, (v * 2 + 1) * T + tid);
                    if (fabsf(s.x) >= 125.5f && v0 >= 0) s.x = to_msg<ALGO>(lb[v0]);
                    if (fabsf(s.y) >= 125.5f && v1 >= 0) s.y = to_msg<ALGO>(lb[v1]);
                }
                s = s + make_float2(__builtin_amdgcn_logf(loc[v].x), __builtin_amdgcn_logf(loc[v].y));
#pragma unroll
                for (int u = 0; u < DN; ++u)
                    s = s + make_float2(__builtin_amdgcn_logf(cv[u].x), __builtin_amdgcn_logf(cv[u].y));
                pr[v] = s;
            } else {
                pr[v] = ms_sum(dn_tag, v, L[v], loc[v], cv);
            }
            __builtin_amdgcn_sched_barrier(0);  // one var pair's gathers in flight (VGPR budget)
        };
#pragma unroll
        for (int k = 0; k < KP; ++k) {
            post(int_c<DVN0>{}, bool_c<ABS0>{}, 2 * k);
            post(int_c<DVN1>{}, bool_c<ABS1>{}, 2 * k + 1);
        }
        __syncthreads();  // all gathers done before the staging overwrites messages
#pragma unroll
        for (int v = 0; v < VP; ++v) {
            const int v0 = ld_fresh(a.loc_var, (v * 2 + 0) * T + tid), v1 = ld_fresh(a.loc_var, (v * 2 + 1) * T + tid);
            if (v0 >= 0) msg[v0] = pr[v].x;
            if (v1 >= 0) msg[v1] = pr[v].y;
        }
        __syncthreads();
        for (int v = tid; v < n; v += T) {
            const float s = msg[v];
            if (a.post) a.post[(size_t)b * n + v] = s * Domain<ALGO>::out;
            if (a.hard) a.hard[(size_t)b * n + v] = (uint8_t)(s < 0.0f);
        }
        if (a.its && tid == 0) a.its[b] = iters;
    }
}

// ---------------------------------------------------------------------------
// 2b. Generic path: any (irregular) CSR graph, check degree <= MAXDC.
//   Messages in LDS when they fit, else in a per-workgroup global scratch
//   slab (GMEM; the slab stays L2 / Infinity-Cache resident).  Channel LLRs
//   are kept beside the messages.  Posterior / hard decision are written to
//   the outputs after every variable phase.
// ---------------------------------------------------------------------------
constexpr int kGenDV = 4;  // variable degrees up to this keep their messages in registers
#ifndef LDPC_LDS36_GRID
#define LDPC_LDS36_GRID 256  // persistent grid of the LDS kernel under early stop (one per CU)
#endif
#ifndef LDPC_IRR_UV
#define LDPC_IRR_UV 1  // variables per load batch in bp_irr_kernel's variable phase (2, 4: no faster)
#endif
#ifndef LDPC_GEN_UC
#define LDPC_GEN_UC 2  // checks per step of the generic kernel's check phase (loads batched)
#endif
#ifndef LDPC_GEN_UV
#define LDPC_GEN_UV 4  // variables per step of the generic kernel's variable phase
#endif

template <int T, int MAXDC, int ALGO, bool ET, bool MC, bool GMEM>
__global__ __launch_bounds__(T) void bp_generic_kernel(BpArgs a) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int tid = threadIdx.x;
    const int n = a.n, m = a.m, E = a.E, iters = a.max_iters;
    unsigned char *base = GMEM ? reinterpret_cast<unsigned char *>(a.scratch) +
                                     (size_t)blockIdx.x * (((size_t)E * 5 + (size_t)n * 4 + 15) & ~(size_t)15)
                               : smem;
    float *msg_all = reinterpret_cast<float *>(base);
    float *Ls = msg_all + E;
    uint8_t *hs = reinterpret_cast<uint8_t *>(Ls + n);
    int *curve = reinterpret_cast<int *>(GMEM ? smem : smem + (((size_t)E * 5 + (size_t)n * 4 + 15) & ~(size_t)15));
    // GMEM: the first S message slots live in LDS, the rest in the L2-resident
    // global slab (generic pointers -> flat loads pick the space per lane).
    const int S = GMEM ? a.lds_slots : 0;
    // explicit address spaces (no generic pointer selects: a select between an LDS
    // and a global pointer trips the gfx950 backend once the loops are unrolled)
    lds_f32 *msg_lds = (lds_f32 *)((lds_u8 *)smem + (MC ? (((size_t)(iters + 1) * 4 + 15) & ~(size_t)15) : 0));
    lds_f32 *msg_l = (lds_f32 *)(lds_u8 *)smem;  // !GMEM: every message in LDS
    auto LD = [&](int e) -> float {
        if constexpr (GMEM) return e < S ? msg_lds[e] : msg_all[e];
        else return msg_l[e];
    };
    auto ST = [&](int e, float x) {
        if constexpr (GMEM) {
            if (e < S) msg_lds[e] = x;
            else msg_all[e] = x;
        } else {
            msg_l[e] = x;
        }
    };

    for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
        const uint64_t cw = a.first_cw + (uint64_t)b;
        __syncthreads();  // previous codeword fully drained
        if (MC) {
            for (int i = tid; i <= iters; i += T) curve[i] = 0;
        }
        __syncthreads();
        int err0 = 0;
        for (int v = tid; v < n; v += T) {
            const float l = MC ? chan_soft(a.ch, cw, v) : a.llr[(size_t)b * n + v];
            const float l2 = to_msg<ALGO>(l);
            Ls[v] = l2;
            err0 += (l < 0.0f);
            for (int e = a.vptr[v]; e < a.vptr[v + 1]; ++e) ST(a.vslot[e], l2);
            if (!MC) {
                if (a.post) a.post[(size_t)b * n + v] = l;
                if (a.hard) a.hard[(size_t)b * n + v] = (uint8_t)(l < 0.0f);
            }
        }
        if (MC) {
            const int w = wave_sum(err0);
            if ((tid & (kWave - 1)) == 0) atomicAdd(&curve[0], w);
        }
        __syncthreads();
        int it = 0;
        for (; it < iters; ++it) {
            if (it > 0) __syncthreads();  // variable phase (messages, hs) complete
            int unsat = 0;                // ET: syndrome of the previous hard decisions
            // LDPC_GEN_UC checks per step: every load of the step is issued before
            // the first use, so the L2 latency of the CSR and slab reads overlaps
            for (int c0 = tid; c0 < m; c0 += T * LDPC_GEN_UC) {
                int s0[LDPC_GEN_UC], d[LDPC_GEN_UC];
#pragma unroll
                for (int u = 0; u < LDPC_GEN_UC; ++u) {
                    const int c = c0 + u * T, cc = c < m ? c : m - 1;
                    s0[u] = a.cptr[cc];
                    d[u] = c < m ? a.cptr[cc + 1] - s0[u] : 0;
                }
                if (ET && it > 0) {
#pragma unroll
                    for (int u = 0; u < LDPC_GEN_UC; ++u) {
                        int par = 0;
                        for (int q = 0; q < d[u]; ++q) par ^= hs[s0[u] + q];
                        unsat |= par;
                    }
                }
                float x[LDPC_GEN_UC][MAXDC];
#pragma unroll
                for (int u = 0; u < LDPC_GEN_UC; ++u)
#pragma unroll
                    for (int q = 0; q < MAXDC; ++q) x[u][q] = q < d[u] ? LD(s0[u] + q) : __builtin_inff();
#pragma unroll
                for (int u = 0; u < LDPC_GEN_UC; ++u) {
                    check_update<ALGO, MAXDC>(x[u], a.alpha, d[u]);
#pragma unroll
                    for (int q = 0; q < MAXDC; ++q)
                        if (q < d[u]) ST(s0[u] + q, x[u][q]);
                }
            }
            if constexpr (ET) {
                if (!__syncthreads_or(unsat | (it == 0))) break;
            } else {
                __syncthreads();
            }
            int errs = 0;
            // decisions leave the kernel only when they can be final: the last
            // fixed-count iteration, or every iteration under early stop
            const bool out_now = !MC && (ET || it == iters - 1);
            // LDPC_GEN_UV variables per step, loads batched as in the check phase
            for (int v0 = tid; v0 < n; v0 += T * LDPC_GEN_UV) {
                int e0[LDPC_GEN_UV], dg[LDPC_GEN_UV];
                float sv[LDPC_GEN_UV];
#pragma unroll
                for (int u = 0; u < LDPC_GEN_UV; ++u) {
                    const int v = v0 + u * T, vc = v < n ? v : n - 1;  // clamped: loads stay unconditional
                    e0[u] = a.vptr[vc];
                    dg[u] = v < n ? a.vptr[vc + 1] - e0[u] : 0;
                    sv[u] = Ls[vc];
                }
                int sl[LDPC_GEN_UV][kGenDV];
                float cv[LDPC_GEN_UV][kGenDV];
#pragma unroll
                for (int u = 0; u < LDPC_GEN_UV; ++u)
#pragma unroll
                    for (int j = 0; j < kGenDV; ++j) sl[u][j] = j < dg[u] ? a.vslot[e0[u] + j] : 0;
#pragma unroll
                for (int u = 0; u < LDPC_GEN_UV; ++u)
#pragma unroll
                    for (int j = 0; j < kGenDV; ++j) cv[u][j] = j < dg[u] ? LD(sl[u][j]) : 0.0f;
#pragma unroll
                for (int u = 0; u < LDPC_GEN_UV; ++u) {
                    const int v = v0 + u * T;
                    if (v >= n) continue;
                    float s = sv[u];
                    if (dg[u] <= kGenDV) {  // messages and slots read once, kept in registers
#pragma unroll
                        for (int j = 0; j < kGenDV; ++j) s += cv[u][j];  // absent edges add +0
#pragma unroll
                        for (int j = 0; j < kGenDV; ++j)
                            if (j < dg[u]) {
                                ST(sl[u][j], s - cv[u][j]);
                                if (ET) hs[sl[u][j]] = (uint8_t)(s < 0.0f);
                            }
                    } else {
                        const int e1 = e0[u] + dg[u];
                        for (int e = e0[u]; e < e1; ++e) s += LD(a.vslot[e]);
                        for (int e = e0[u]; e < e1; ++e) {
                            const int slot = a.vslot[e];
                            ST(slot, s - LD(slot));
                            if (ET) hs[slot] = (uint8_t)(s < 0.0f);
                        }
                    }
                    errs += (s < 0.0f);
                    if (out_now) {
                        if (a.post) a.post[(size_t)b * n + v] = s * Domain<ALGO>::out;
                        if (a.hard) a.hard[(size_t)b * n + v] = (uint8_t)(s < 0.0f);
                    }
                }
            }
            if (MC) {
                const int w = wave_sum(errs);
                if ((tid & (kWave - 1)) == 0) atomicAdd(&curve[it + 1], w);
            }
        }
        __syncthreads();
        if (MC) {
            int32_t *tr = a.trial + (size_t)b * (iters + 1);
            const int last = curve[it];
            for (int i = tid; i <= iters; i += T) tr[i] = i <= it ? curve[i] : last;
        }
        if ((MC || a.its) && tid == 0) a.its[b] = it;
    }
}

// ---------------------------------------------------------------------------
// 2b'. Irregular graphs (variable degree <= 4, check degree <= 8), one codeword
// per 1024-thread workgroup, host-built layout (build_irr_layout, capi.cpp):
//   check c = k*1024 + t is thread t's row-k check; its slot j sits at position
//   (k*DC + j)*1024 + t, so a row's reads and writes are lane-contiguous (LDS
//   conflict-free, coalesced in the slab).  Absent slots (degree < DC) hold the
//   rule's neutral input (min-sum +inf; sum-product skips them by degree) and are never
//   written, so the update runs on DC entries without a degree test (x1 and
//   min(+inf, .) change nothing: same values as oracle check_update_*(x, d)).
//   Positions [0, S) are in LDS, [S, P) in a per-workgroup global slab (whole
//   rows, so the row loop branches uniformly); the grid is one workgroup per CU
//   so the slabs stay L2-resident.
//   Lane p = i*1024 + t is thread t's i-th variable; lanes are sorted by degree
//   and each degree class is padded to whole 64-lane rows, so "edge j present"
//   is wave-uniform (readfirstlane).  Positions (2 x 16 bit per VGPR) and channel
//   LLRs stay in VGPRs for the whole decode; one variable's messages may sit in
//   LDS or in the slab (per-lane branch).
//   ET: the variable phase XORs the hard decision of every negative posterior
//   into a per-check syndrome bit array in LDS, tested after the phase.
// ---------------------------------------------------------------------------
template <int DC, int VPT, int ALGO, bool ET, bool MC>
__global__ __launch_bounds__(kIrrT) void bp_irr_kernel(BpArgs a) {
    constexpr int T = kIrrT;
    extern __shared__ __align__(16) unsigned char smem[];
    const int tid = threadIdx.x;
    const int n = a.n, m = a.m, iters = a.max_iters, KC = a.irr_KC, S = a.irr_S;
    lds_f32 *ml = (lds_f32 *)(lds_u8 *)smem;  // [S]
    uint32_t *syn = reinterpret_cast<uint32_t *>(smem + (((size_t)S * 4 + 15) & ~(size_t)15));  // [m/32]
    const int nsyn = (m + 31) >> 5;
    int *curve = reinterpret_cast<int *>(syn + ((nsyn + 3) & ~3));  // [iters+1]
    float *slab = a.scratch + (size_t)blockIdx.x * a.irr_P;
    auto LD = [&](uint32_t q) -> float { return (int)q < S ? (float)ml[q] : slab[q]; };
    auto ST = [&](uint32_t q, float x) {
        if ((int)q < S) ml[q] = x;
        else slab[q] = x;
    };
    constexpr float neutral = ALGO == 0 ? 1.0f : __builtin_inff();
    const uint64_t cd = (uint32_t)a.irr_cdeg[tid] | ((uint64_t)(uint32_t)a.irr_cdeg[T + tid] << 32);
    uint32_t pp[2 * VPT];
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        pp[2 * i] = (uint32_t)a.irr_lane[(size_t)T * VPT + i * T + tid];
        pp[2 * i + 1] = (uint32_t)a.irr_lane[(size_t)2 * T * VPT + i * T + tid];
    }
    auto POS = [&](int i, int j) -> uint32_t {
        const uint32_t w = pp[2 * i + (j >> 1)];
        return (j & 1) ? (w >> 16) : (w & 0xFFFFu);
    };

    for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
        const uint64_t cw = a.first_cw + (uint64_t)b;
        __syncthreads();  // previous codeword drained (messages, curve, syndrome)
        if (MC) {
            for (int i = tid; i <= iters; i += T) curve[i] = 0;
        }
        // absent check slots -> neutral
        for (int k = 0; k < KC; ++k) {
            const int d = (int)((cd >> (4 * k)) & 15u);
            for (int j = d; j < DC; ++j) ST((uint32_t)((k * DC + j) * T + tid), neutral);
        }
        // channel LLRs and the first variable-to-check messages
        float L[VPT];
        int err0 = 0;
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            const int v = a.irr_lane[i * T + tid];
            float l = 0.0f;
            if (v >= 0) l = MC ? chan_soft(a.ch, cw, v) : a.llr[(size_t)b * n + v];
            err0 += (v >= 0) & (l < 0.0f);
            L[i] = to_msg<ALGO>(l);
            const float w = v2c_rwire<ALGO>(L[i]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (__builtin_amdgcn_readfirstlane(POS(i, j)) != 0xFFFFu) ST(POS(i, j), w);
        }
        if (ET)
            for (int i = tid; i < nsyn; i += T) syn[i] = 0u;
        __syncthreads();
        if (MC) {
            const int w = wave_sum(err0);
            if ((tid & (kWave - 1)) == 0) atomicAdd(&curve[0], w);
        }
        float pr[(ET && !MC) ? VPT : 1];
        if constexpr (ET && !MC) {
#pragma unroll
            for (int i = 0; i < VPT; ++i) pr[i] = L[i];
        }
        // variable phase; FINAL = the last fixed-count iteration: outputs instead of messages
        auto var_phase = [&](auto final_tag) {
            constexpr bool FINAL = decltype(final_tag)::value;
            int errs = 0;
            // launder the packed positions: unpacked (and slab addresses) hoisted out
            // of the iteration loop would need ~4*VPT more VGPRs
#pragma unroll
            for (int q = 0; q < 2 * VPT; ++q) asm volatile("" : "+v"(pp[q]));
            // LDPC_IRR_UV variables per step: all their loads issue before the first
            // store (stores and later loads may alias as far as the compiler knows)
#pragma unroll
            for (int i0 = 0; i0 < VPT; i0 += LDPC_IRR_UV) {
                bool has[LDPC_IRR_UV][4];
                float cv[LDPC_IRR_UV][4];
#pragma unroll
                for (int u = 0; u < LDPC_IRR_UV; ++u)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int i = i0 + u;
                        has[u][j] = i < VPT && __builtin_amdgcn_readfirstlane(POS(i < VPT ? i : 0, j)) != 0xFFFFu;
                        cv[u][j] = has[u][j] ? LD(POS(i < VPT ? i : 0, j)) : 0.0f;
                    }
#pragma unroll
                for (int u = 0; u < LDPC_IRR_UV; ++u) {
                    const int i = i0 + u;
                    if (i >= VPT) break;
                    float s = L[i];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (has[u][j]) s += cv[u][j];
                    if constexpr (!FINAL) {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (has[u][j]) ST(POS(i, j), v2c_rwire<ALGO>(s - cv[u][j]));
                    }
                    if constexpr (ET) {
                        if (s < 0.0f) {
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const int q = (int)POS(i, j);
                                if (has[u][j] && q < KC * DC * T) {  // a check slot (not a dummy)
                                    const int c = (q / (DC * T)) * T + (q % T);
                                    atomicXor(&syn[c >> 5], 1u << (c & 31));
                                }
                            }
                        }
                        if constexpr (!MC) pr[i] = s;
                    }
                    if constexpr (MC) errs += (s < 0.0f);
                    if constexpr (FINAL && !MC) {
                        const int v = a.irr_lane[i * T + tid];
                        if (v >= 0) {
                            if (a.post) a.post[(size_t)b * n + v] = s * Domain<ALGO>::out;
                            if (a.hard) a.hard[(size_t)b * n + v] = (uint8_t)(s < 0.0f);
                        }
                    }
                }
            }
            return errs;
        };

        int it = 0;
        for (; it < iters; ++it) {
            if (!ET && it > 0) __syncthreads();  // variable phase complete (ET: its syndrome barriers)
            // ---- check phase ----
            for (int k = 0; k < KC; ++k) {
                const int d = (int)((cd >> (4 * k)) & 15u);
                const int q0 = k * DC * T + tid;
                float x[DC];
                const bool in_lds = (k + 1) * DC * T <= S;  // uniform: whole rows
                if (in_lds) {
#pragma unroll
                    for (int j = 0; j < DC; ++j) x[j] = ml[q0 + j * T];
                } else {
#pragma unroll
                    for (int j = 0; j < DC; ++j) x[j] = slab[q0 + j * T];
                }
                if constexpr (ALGO == 1 && DC == 6) check_update_ms6(x, a.alpha);
                else check_update<ALGO, DC, true>(x, a.alpha, d);
                if (in_lds) {
#pragma unroll
                    for (int j = 0; j < DC; ++j)
                        if (j < d) ml[q0 + j * T] = x[j];
                } else {
#pragma unroll
                    for (int j = 0; j < DC; ++j)
                        if (j < d) slab[q0 + j * T] = x[j];
                }
            }
            __syncthreads();
            // fixed-count decode: the last variable phase runs after the loop
            if (!ET && !MC && it == iters - 1) break;
            const int errs = var_phase(std::false_type{});
            if (MC) {
                const int w = wave_sum(errs);
                if ((tid & (kWave - 1)) == 0) atomicAdd(&curve[it + 1], w);
            }
            if constexpr (ET) {
                __syncthreads();  // syndrome complete
                int unsat = 0;
                for (int i = tid; i < nsyn; i += T) unsat |= (syn[i] != 0u);
                const bool more = __syncthreads_or(unsat);
                for (int i = tid; i < nsyn; i += T) syn[i] = 0u;  // every read is before that barrier
                if (!more) {
                    ++it;
                    break;
                }
            }
        }
        if (!ET && !MC && iters > 0) {
            (void)var_phase(std::true_type{});
            it = iters;
        }
        if constexpr (ET && !MC) {
#pragma unroll
            for (int i = 0; i < VPT; ++i) {
                const int v = a.irr_lane[i * T + tid];
                if (v >= 0) {
                    if (a.post) a.post[(size_t)b * n + v] = pr[i] * Domain<ALGO>::out;
                    if (a.hard) a.hard[(size_t)b * n + v] = (uint8_t)(pr[i] < 0.0f);
                }
            }
        }
        if (!ET && !MC && iters == 0) {
#pragma unroll
            for (int i = 0; i < VPT; ++i) {
                const int v = a.irr_lane[i * T + tid];
                if (v >= 0) {
                    if (a.post) a.post[(size_t)b * n + v] = L[i] * Domain<ALGO>::out;
                    if (a.hard) a.hard[(size_t)b * n + v] = (uint8_t)(L[i] < 0.0f);
                }
            }
        }
        if constexpr (MC) {
            __syncthreads();
            int32_t *tr = a.trial + (size_t)b * (iters + 1);
            const int last = curve[it];
            for (int i = tid; i <= iters; i += T) tr[i] = i <= it ? curve[i] : last;
            if (tid == 0) a.its[b] = it;
        } else {
            if (a.its && tid == 0) a.its[b] = it;
        }
    }
}


// ===========================================================================
// 3. Stand-alone channel (rocRAND philox4x32_10 device API)
// ===========================================================================
__global__ __launch_bounds__(256) void channel_kernel(int kind, float p, float p2, uint64_t seed,
                                                      uint64_t first_cw, int n, int B, void *out) {
    const int groups = (n + 3) >> 2;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)groups * B) return;
    const int b = (int)(idx / groups), g = (int)(idx % groups);
    rocrand_state_philox4x32_10 st;
    rocrand_init(seed, first_cw + (uint64_t)b, 4ull * (uint64_t)g, &st);
    const uint4 r = rocrand4(&st);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
    float val[4];
    if (kind == 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float ua = u01(w[2 * h]), ub = u01(w[2 * h + 1]);
            const float rad = sqrtf(-2.0f * logf(ua));
            const float ang = 6.28318530717958647692f * ub;
            val[2 * h] = (1.0f + p * (rad * cosf(ang))) * p2;
            val[2 * h + 1] = (1.0f + p * (rad * sinf(ang))) * p2;
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int v = 4 * g + i;
        if (v >= n) break;
        const size_t o = (size_t)b * n + v;
        const float u = u01(w[i]);
        if (kind == 0) static_cast<uint8_t *>(out)[o] = u < p ? 2 : 0;
        else if (kind == 1) static_cast<float *>(out)[o] = u < p ? -p2 : p2;
        else static_cast<float *>(out)[o] = val[i];
    }
}

// ===========================================================================
// 4. Monte-Carlo statistics: sequential stop rule + counter reduction
// ===========================================================================
// Trial b is a frame error when its final count f satisfies f > X && f != 0
// (parallel_simulator_expurgated.py:238-243; X = -1 gives parallel_simulator.py:227-231).
__global__ __launch_bounds__(1024) void mc_cutoff_kernel(const int32_t *trial, int B, int iters, int X,
                                                         int64_t stop, const int64_t *counters,
                                                         int32_t *cutoff) {
    __shared__ int cnt[1024];
    __shared__ int res;
    const int tid = threadIdx.x;
    if (stop <= 0) {
        if (tid == 0) *cutoff = B;
        return;
    }
    const int64_t remaining = stop - counters[1];
    if (remaining <= 0) {
        if (tid == 0) *cutoff = 0;
        return;
    }
    const int chunk = (B + 1023) / 1024;
    const int b0 = tid * chunk, b1 = min(B, b0 + chunk);
    int c = 0;
    for (int b = b0; b < b1; ++b) {
        const int f = trial[(size_t)b * (iters + 1) + iters];
        c += (f > X && f != 0);
    }
    cnt[tid] = c;
    if (tid == 0) res = B;
    __syncthreads();
    if (tid == 0) {  // exclusive scan (1024 adds)
        int acc = 0;
        for (int i = 0; i < 1024; ++i) {
            const int t = cnt[i];
            cnt[i] = acc;
            acc += t;
        }
    }
    __syncthreads();
    const int64_t before = cnt[tid];
    if (before < remaining && before + c >= remaining) {
        int64_t acc = before;
        for (int b = b0; b < b1; ++b) {
            const int f = trial[(size_t)b * (iters + 1) + iters];
            acc += (f > X && f != 0);
            if (acc >= remaining) {
                res = b + 1;
                break;
            }
        }
    }
    __syncthreads();
    if (tid == 0) *cutoff = res;
}

__global__ __launch_bounds__(256) void mc_reduce_kernel(const int32_t *trial, const int32_t *its, int B,
                                                        int iters, int X, const int32_t *cutoff_p,
                                                        int64_t *counters) {
    __shared__ long long red[4][256 / kWave];
    const int tid = threadIdx.x;
    const int cutoff = min(B, *cutoff_p);
    const int per = (B + gridDim.x - 1) / gridDim.x;
    const int b0 = blockIdx.x * per, b1 = min(cutoff, b0 + per);
    if (b0 >= b1) return;
    // error curve columns, coalesced over t
    for (int t = tid; t <= iters; t += 256) {
        long long s = 0;
        for (int b = b0; b < b1; ++b) {
            const int32_t *row = trial + (size_t)b * (iters + 1);
            if (row[iters] > X) s += row[t];
        }
        if (s) atomicAdd(reinterpret_cast<unsigned long long *>(counters + LDPC_MC_NCOUNT + t),
                         (unsigned long long)s);
    }
    long long fr = 0, bits = 0, itn = 0;
    for (int b = b0 + tid; b < b1; b += 256) {
        const int f = trial[(size_t)b * (iters + 1) + iters];
        if (f > X) {
            fr += (f != 0);
            bits += f;
        }
        itn += its ? its[b] : 0;
    }
    long long v[3] = {fr, bits, itn};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        long long x = v[q];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, kWave);
        if ((tid & 63) == 0) red[q][tid / kWave] = x;
    }
    __syncthreads();
    if (tid == 0) {
        long long s[3] = {0, 0, 0};
        for (int q = 0; q < 3; ++q)
            for (int w = 0; w < 256 / kWave; ++w) s[q] += red[q][w];
        unsigned long long *c = reinterpret_cast<unsigned long long *>(counters);
        atomicAdd(c + 0, (unsigned long long)(b1 - b0));
        atomicAdd(c + 1, (unsigned long long)s[0]);
        atomicAdd(c + 2, (unsigned long long)s[1]);
        atomicAdd(c + 3, (unsigned long long)s[2]);
    }
}

// ===========================================================================
// 6. ML ("optimal") erasure decoding -- optimal_decode, parallel_simulator.py:60-129
//    (system set-up of ml_decoder.c:7-36, GF(2) row_reduce of the galois package)
// ===========================================================================
//
// One workgroup per word.  Thread t holds ROW POSITION t of the augmented system
// [A | target] in registers as W 64-bit words (A = H restricted to the erased
// columns that are still unknown, target = parity of the known 1-bits of each
// active check), so elimination needs no LDS for the matrix: per column j one
// ballot + LDS atomicMin finds the pivot row (first position >= j with bit j set,
// galois' choice); each wave's first candidate row is staged in LDS before the
// barrier, so one barrier per column suffices; rows p and q swap through LDS, and
// every other row holding bit j XORs the pivot in (Gauss-Jordan, above and below).
// Because the reference looks for the FIRST column whose diagonal entry of the
// reduced matrix is not 1, elimination stops at the first column without a pivot
// (all earlier columns are pivots, so that column IS the first diagonal miss):
// that unknown is given up, every check holding it is dropped, and the system is
// rebuilt from the graph and reduced again -- the reference's loop (:93-108).
// When every remaining column has a pivot the solution is read off the augmented
// bit of rows 0..ncols-1 (:110-121).  Words with no erasure or more erasures than
// checks are returned unchanged (:66-70).  m <= 1000 (the 1000-unknown cap of
// :96 can then never bind); n <= 32767.
//
// Per-word LDS (dynamic): cand[2][T/64][W], swp[2][W] (u64); best[3], wsum[16] (int);
// code[n] (int16: column of an active unknown, -1/-2 known 0/1, -3 given up);
// state[n] (u8: 0/1 known, 2 unknown, 3 given up, 4/5 solved 0/1);
// rowchk[m], colvar[m] (int16); achk[m] (u8).

// Register-array helpers with static indices only (a data-dependent index would
// push R[] to scratch): set bit k by masks, and drop the front word (the
// elimination window: columns left of the current 64-column block are never read
// again, and every row's bit j sits in word 0).
template <int W>
__device__ __forceinline__ void ml_set_bit(uint64_t (&R)[W], int k) {
    const int kw = k >> 6;
    const uint64_t b = 1ull << (k & 63);
#pragma unroll
    for (int w = 0; w < W; ++w) R[w] |= (0ull - (uint64_t)(kw == w)) & b;
}

template <int W>
__device__ __forceinline__ void ml_shift(uint64_t (&R)[W]) {
#pragma unroll
    for (int w = 0; w + 1 < W; ++w) R[w] = R[w + 1];
    R[W - 1] = 0;
}

// cptr == nullptr: regular lists, check c owns slots [c*dc, c*dc+dc) of
// cvar + b*cvar_stride (ensemble mode: word b decodes on its own graph b).
template <int W>
__global__ __launch_bounds__(1024) void ml_kernel(const int32_t *__restrict__ cptr, const int32_t *__restrict__ cvar,
                                                  int64_t cvar_stride, int dc, int n, int m,
                                                  const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                  int32_t *__restrict__ unsolved) {
    extern __shared__ __align__(16) unsigned char ml_lds[];
    const int NW = blockDim.x >> 6;
    uint64_t *cand = reinterpret_cast<uint64_t *>(ml_lds);  // [2][NW][W] each wave's first candidate row
    uint64_t *swp = cand + 2 * NW * W;                       // [2][W] row at the pivot position
    int *best = reinterpret_cast<int *>(swp + 2 * W);        // [3]
    int *wsum = best + 3;                                    // [16]
    int16_t *code = reinterpret_cast<int16_t *>(wsum + 16); // [n]
    int16_t *rowchk = code + n;                             // [m]
    int16_t *colvar = rowchk + m;                           // [m]
    uint8_t *state = reinterpret_cast<uint8_t *>(colvar + m);  // [n]
    uint8_t *achk = state + n;                              // [m]

    const int tid = threadIdx.x, T = blockDim.x;
    const int lane = tid & 63, wave = tid >> 6;
    const size_t b = blockIdx.x;
    const uint8_t *w_in = in + b * n;
    uint8_t *w_out = out + b * n;
    const int32_t *gv = cvar + (int64_t)b * cvar_stride;

    int ne_local = 0;
    for (int v = tid; v < n; v += T) {
        const uint8_t x = w_in[v];
        state[v] = x == 2 ? 2 : (x ? 1 : 0);
        ne_local += (x == 2);
    }
    for (int c = tid; c < m; c += T) achk[c] = 1;
    if (tid < 3) best[tid] = INT_MAX;
    int ne = 0;
    (void)block_excl_scan(ne_local, wsum, ne);  // (its barriers also publish state / achk / best)
    if (ne == 0 || ne > m) {
        for (int v = tid; v < n; v += T) w_out[v] = w_in[v];
        if (tid == 0) unsolved[b] = ne;
        return;
    }
    const int vper = (n + T - 1) / T, cper = (m + T - 1) / T;
    int marks = 0;
    for (;;) {
        // --- columns: the active unknowns in position order
        const int v0 = min(n, tid * vper), v1 = min(n, v0 + vper);
        int cnt = 0;
        for (int v = v0; v < v1; ++v) cnt += (state[v] == 2);
        int ncols = 0;
        int col = block_excl_scan(cnt, wsum, ncols);
        for (int v = v0; v < v1; ++v) {
            const int st = state[v];
            if (st == 2) {
                colvar[col] = (int16_t)v;
                code[v] = (int16_t)col++;
            } else {
                code[v] = (int16_t)(st == 3 ? -3 : -1 - st);
            }
        }
        // --- rows: the active checks in index order
        const int c0 = min(m, tid * cper), c1 = min(m, c0 + cper);
        cnt = 0;
        for (int c = c0; c < c1; ++c) cnt += achk[c];
        int nrows = 0;
        int pos = block_excl_scan(cnt, wsum, nrows);  // barrier: code[] / colvar[] complete
        for (int c = c0; c < c1; ++c)
            if (achk[c]) rowchk[pos++] = (int16_t)c;
        __syncthreads();
        // --- build row `tid` of [A | target]
        uint64_t R[W];
#pragma unroll
        for (int w = 0; w < W; ++w) R[w] = 0;
        int s_lo = 0, s_hi = 0;
        if (tid < nrows) {
            const int c = rowchk[tid];
            s_lo = cptr ? cptr[c] : c * dc;
            s_hi = cptr ? cptr[c + 1] : s_lo + dc;
            int tgt = 0;
            for (int s = s_lo; s < s_hi; ++s) {
                const int v = gv[s];
                const int k = code[v];
                if (k >= 0) {
                    ml_set_bit<W>(R, k);  // H is a 0/1 matrix: set, not toggle
                } else if (k == -2) {
                    bool dup = false;     // a variable listed twice in a check counts once
                    for (int s2 = s_lo; s2 < s; ++s2) dup |= (gv[s2] == v);
                    tgt ^= dup ? 0 : 1;
                }
            }
            if (tgt) ml_set_bit<W>(R, ncols);
        }
        // --- Gauss-Jordan in galois' pivot order until the first column without a pivot.
        // Window: R[0] holds columns [64*shift, 64*shift+64) of the row.  One barrier
        // per column: every wave's first candidate row is published before the barrier
        // (with the row at the pivot position, for the swap), so the winner's row is
        // already in LDS once the pivot position is known.  cand/swp are double-
        // buffered by column parity, best[] triple-buffered (the atomicMin of column
        // j+1 may run before a slow thread reads best[] of column j).
        int free_col = -1, shift = 0, b3 = 0, j = 0;
        // One 64-column block at a time with the L = live words of the window only
        // (words past the augmented column are zero in every row), so the column
        // step is branch-free and its cost shrinks as the elimination advances.
        auto block = [&](auto live_tag) {
            constexpr int L = decltype(live_tag)::value;
            const int jend = min(ncols, 64 * (shift + 1));
            for (; j < jend; ++j) {
                const int buf = j & 1;
                const bool bit = (R[0] >> (j & 63)) & 1ull;
                const uint64_t bal = __ballot(bit && tid >= j && tid < nrows);
                if (bal && lane == (int)__ffsll((long long)bal) - 1) {
                    uint64_t *cw = cand + (buf * NW + wave) * W;
#pragma unroll
                    for (int w = 0; w < L; ++w) cw[w] = R[w];
                    atomicMin(&best[b3], tid);
                }
                if (tid == j) {
#pragma unroll
                    for (int w = 0; w < L; ++w) swp[buf * W + w] = R[w];
                }
                __syncthreads();
                const int q = best[b3];
                const int b_old = b3 == 0 ? 2 : b3 - 1;  // buffer of column j-1 == column j+2
                if (tid == 0) best[b_old] = INT_MAX;
                b3 = b3 == 2 ? 0 : b3 + 1;
                if (q == INT_MAX) {
                    free_col = j;
                    return;
                }
                const uint64_t *pb = cand + (buf * NW + (q >> 6)) * W;
                const bool take = (tid == j) && (q != j);               // row j becomes the pivot row
                const uint64_t msk = (bit && tid != q) ? ~0ull : 0ull;  // rows holding bit j XOR it in
#pragma unroll
                for (int w = 0; w < L; ++w) {
                    const uint64_t pw = pb[w];
                    R[w] = take ? pw : (R[w] ^ (pw & msk));
                }
                if (tid == q && q != j) {  // the old row j moves to position q
#pragma unroll
                    for (int w = 0; w < L; ++w) R[w] = swp[buf * W + w];
                }
            }
            if (j < ncols) {  // next block: drop the front word
#pragma unroll
                for (int w = 0; w + 1 < L; ++w) R[w] = R[w + 1];
                R[L - 1] = 0;
                ++shift;
            }
        };
        while (j < ncols && free_col < 0) {
            switch (min(W, (ncols >> 6) - shift + 1)) {  // live words: columns [64*shift, ncols]
#define LDPC_ML_LIVE(LL) \
    case LL:             \
        if constexpr (LL <= W) block(std::integral_constant<int, LL>{}); \
        break;
                LDPC_ML_LIVE(1) LDPC_ML_LIVE(2) LDPC_ML_LIVE(3) LDPC_ML_LIVE(4)
                LDPC_ML_LIVE(5) LDPC_ML_LIVE(6) LDPC_ML_LIVE(7) LDPC_ML_LIVE(8)
                LDPC_ML_LIVE(9) LDPC_ML_LIVE(10) LDPC_ML_LIVE(11) LDPC_ML_LIVE(12)
                LDPC_ML_LIVE(13) LDPC_ML_LIVE(14) LDPC_ML_LIVE(15) LDPC_ML_LIVE(16)
#undef LDPC_ML_LIVE
                default: block(std::integral_constant<int, W>{});
            }
        }
        if (free_col < 0) {
            // full column rank: unknown j = augmented bit (column ncols) of row j
            while (shift < (ncols >> 6)) {
                ml_shift<W>(R);
                ++shift;
            }
            if (tid < ncols) {
                const int v = colvar[tid];
                state[v] = (uint8_t)(4 + ((R[0] >> (ncols & 63)) & 1ull));
            }
            __syncthreads();
            break;
        }
        // --- give the unknown up: drop it and every check that holds it
        const int vf = colvar[free_col];
        if (tid < nrows) {
            bool has = false;
            for (int s = s_lo; s < s_hi; ++s) has |= (gv[s] == vf);
            if (has) achk[rowchk[tid]] = 0;
        }
        if (tid == 0) state[vf] = 3;
        ++marks;
        __syncthreads();
    }
    for (int v = tid; v < n; v += T) {
        const int st = state[v];
        w_out[v] = st == 3 ? 2 : (st >= 4 ? (uint8_t)(st - 4) : w_in[v]);
    }
    if (tid == 0) unsolved[b] = marks;
}

// ===========================================================================
// Launch-side kernel selection
// ===========================================================================
constexpr size_t kLdsMax = 160 * 1024;


ChanArgs make_chan(int kind, float p, float p2, uint64_t seed) {
    ChanArgs c;
    c.kind = kind;
    c.p = p;
    c.p2 = p2;
    c.k0 = (uint32_t)seed;
    c.k1 = (uint32_t)(seed >> 32);
    return c;
}

size_t bec_lds_bytes(const ldpc_graph &g, int iters) {
    return (size_t)((iters * 4 + 15) & ~15) + (size_t)((g.n + 15) & ~15) + (size_t)g.m;
}

template <bool MC>
hipError_t run_bec(const ldpc_graph &g, BecArgs a, int B, hipStream_t stream) {
    const size_t lds = bec_lds_bytes(g, a.max_iters);
    if (lds > kLdsMax - 1024) return hipErrorInvalidValue;
    if (B <= 0) return hipSuccess;
    if (g.n >= 4096) {
        auto k = bec_kernel<1024, MC>;
        hipError_t e = allow_lds(k, lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k, dim3(B), dim3(1024), lds, stream, a);
    } else {
        auto k = bec_kernel<256, MC>;
        hipError_t e = allow_lds(k, lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k, dim3(B), dim3(256), lds, stream, a);
    }
    return hipGetLastError();
}

// Bit-sliced BEC Monte-Carlo (bec_mc_bits_kernel): plane word (u32 x W words per
// variable, or u8 = 8 codewords for graphs whose u32 planes do not fit) and
// workgroup size for this graph and batch; false when not even u8 planes fit.
size_t bec_bits_lds_bytes(const ldpc_graph &g, int W, int bytes_per_word) {
    const int NB = 8 * bytes_per_word * W;
    return ((((size_t)g.n + g.m) * W * bytes_per_word + 15) & ~(size_t)15) + (size_t)8 * NB + 16;
}
bool bec_bits_shape(const ldpc_graph &g, int B, int &W, int &T, int &bytes) {
    T = g.n > 4096 ? 512 : 256;
    bytes = 4;
    for (int w : {4, 2, 1}) {
        // enough workgroups to fill 256 CUs several times over, LDS for >= 2 per CU
        if (bec_bits_lds_bytes(g, w, 4) <= 72 * 1024 && ((int64_t)B + 32 * w - 1) / (32 * w) >= 1024) {
            W = w;
            return true;
        }
    }
    W = 1;
    if (bec_bits_lds_bytes(g, 1, 4) <= kLdsMax - 4096) return true;
    T = 1024;
    bytes = 1;
    return bec_bits_lds_bytes(g, 1, 1) <= kLdsMax - 4096;
}

// bec_dec_bits_kernel: H = 16 (u32) or 4 (u8) codewords per plane word
size_t bec_dec_bits_lds_bytes(const ldpc_graph &g, int W, int bytes_per_word) {
    const int NB = 4 * bytes_per_word * W;
    return ((((size_t)g.n + g.m) * W * bytes_per_word + 15) & ~(size_t)15) + (size_t)4 * NB + 4 * W + 16;
}
bool bec_dec_bits_shape(const ldpc_graph &g, int B, int &W, int &T, int &bytes) {
    T = g.n > 4096 ? 512 : 256;
    bytes = 4;
    if (B < 64) return false;  // a few words (the drop-in's B = 1): one workgroup per codeword
    for (int w : {4, 2, 1}) {
        if (bec_dec_bits_lds_bytes(g, w, 4) <= 72 * 1024 && ((int64_t)B + 16 * w - 1) / (16 * w) >= 1024) {
            W = w;
            return true;
        }
    }
    W = 1;
    if (bec_dec_bits_lds_bytes(g, 1, 4) <= kLdsMax - 4096) return true;
    T = 1024;
    bytes = 1;
    return bec_dec_bits_lds_bytes(g, 1, 1) <= kLdsMax - 4096;
}

template <int T, int W, typename P>
hipError_t launch_bec_dec_bits(const ldpc_graph &g, const BecArgs &a, int B, hipStream_t stream) {
    const size_t lds = bec_dec_bits_lds_bytes(g, W, (int)sizeof(P));
    auto k = bec_dec_bits_kernel<T, W, P>;
    hipError_t e = allow_lds(k, lds);
    if (e != hipSuccess) return e;
    constexpr int NB = 4 * (int)sizeof(P) * W;
    const unsigned grid = (unsigned)(((int64_t)B + NB - 1) / NB);
    hipLaunchKernelGGL(k, dim3(grid), dim3(T), lds, stream, a, B);
    return hipGetLastError();
}

template <int T, int W, typename P>
hipError_t launch_bec_bits(const ldpc_graph &g, const BecArgs &a, int B, hipStream_t stream) {
    const size_t lds = bec_bits_lds_bytes(g, W, (int)sizeof(P));
    auto k = bec_mc_bits_kernel<T, W, P>;
    hipError_t e = allow_lds(k, lds);
    if (e != hipSuccess) return e;
    constexpr int NB = 8 * (int)sizeof(P) * W;
    const unsigned grid = (unsigned)(((int64_t)B + NB - 1) / NB);
    hipLaunchKernelGGL(k, dim3(grid), dim3(T), lds, stream, a, B);
    return hipGetLastError();
}

BecArgs bec_args(const ldpc_graph &g) {
    BecArgs a{};
    a.cvar = g.cvar;
    a.cptr = g.cptr;
    a.vptr = g.vptr;
    a.vchk = g.vchk;
    a.n = g.n;
    a.m = g.m;
    a.dv = g.dv;
    a.dc = g.dc;
    return a;
}

// --- soft path selection ---------------------------------------------------
enum class BpPath { Loc, Lds36, Irr, Generic8, Generic16, Generic32, GenericG8, GenericG16, GenericG32, None };

#ifndef LDPC_LDS36_MINSUM
#define LDPC_LDS36_MINSUM 1  // (3,6) min-sum on bp_lds_kernel rather than bp_loc_kernel
#endif
#ifndef LDPC_LOC
#define LDPC_LOC 1  // fixed-count decode on bp_loc_kernel when the graph has a local-edge layout
#endif
#ifndef LDPC_LOC_MSMC
#define LDPC_LOC_MSMC 1  // (3,6) min-sum Monte-Carlo (with or without early stop) on bp_loc_kernel
#endif
#ifndef LDPC_LOC_HARD_ET
#define LDPC_LOC_HARD_ET 1  // early-stop decodes without posteriors on bp_loc_kernel
#endif
#ifndef LDPC_LOC_ET_POST
#define LDPC_LOC_ET_POST 1  // early-stop decodes with posteriors on bp_loc_kernel (slab, persistent grid)
#endif
// bp_loc_kernel shapes: (check-degree range, non-local edges per variable, absent edges)
// x (threads, check pairs per thread)
// Early stop with posteriors on bp_loc_kernel: persistent workgroups (two per CU, the most
// any bp_loc_kernel shape keeps resident), each with a VP x T float2 slab in scratch.
// The CU count is queried for the current device on every call (no shared cache: devices
// launch from their own host threads, and the slab size and the grid must agree per device).
int loc_ep_grid() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    return 2 * cus;
}
size_t loc_ep_slab_floats(const ldpc_graph &g) {
    return (size_t)loc_ep_grid() * (size_t)(2 * g.loc_KP) * (size_t)g.loc_T * 2;
}

int loc_variant_of(const ldpc_graph &g) {
    return loc_variant(g.loc_dlo, g.loc_dhi, g.loc_DVN, g.loc_dvn0, g.loc_dvn1, g.loc_abs0, g.loc_abs1, g.loc_T,
                       g.loc_KP);
}
bool loc_shape(const ldpc_graph &g, int &T, int &KP) {
    if (loc_variant_of(g) == kLocNone) return false;
    T = g.loc_T;
    KP = g.loc_KP;
    return true;
}
// messages | MC: per-iteration curve (16-byte padded) | min-sum MC: syndrome bits
size_t loc_lds_bytes(const ldpc_graph &g, int iters = 0, bool mc = false, bool syn = false) {
    return (((size_t)std::max(g.loc_words + 64, g.n) * 4 + 15) & ~(size_t)15) +
           (mc ? (((size_t)(iters + 1) * 4 + 15) & ~(size_t)15) : 0) + (syn ? (size_t)((g.m + 31) / 32) * 4 : 0);
}

// bp_irr_kernel: LDS bytes (messages, syndrome bits, curve) and whether the slab is used
size_t irr_lds_bytes(const ldpc_graph &g, int iters) {
    const int nsyn = (g.m + 31) >> 5;
    return (((size_t)g.irr_S * 4 + 15) & ~(size_t)15) + (size_t)((nsyn + 3) & ~3) * 4 + (size_t)(iters + 1) * 4;
}
bool irr_slab(const ldpc_graph &g) { return g.irr_S < g.irr_P; }

size_t lds36_bytes(const ldpc_graph &g, int iters, bool et, bool mc) {
    const size_t Ep = (size_t)lds_pair_span(g.m, 6) + kLdsDummy;
    size_t s = Ep * 4;
    if (et || mc) s = (Ep * 5 + 15) & ~(size_t)15;
    if (mc) s += (size_t)(iters + 1) * 4;
    return s;
}

size_t generic_lds_bytes(const ldpc_graph &g, int iters, bool mc) {
    return (((size_t)g.E * 5 + (size_t)g.n * 4 + 15) & ~(size_t)15) + (mc ? (size_t)(iters + 1) * 4 : 0);
}

BpPath choose_path(const ldpc_graph &g, int iters, bool et, bool mc, int algo = 0, bool hard_only = false) {
    if (!g.consistent) return BpPath::None;
    int lT = 0, lKP = 0;
    // min-sum on (3,6) codes with one 1024-thread local-edge workgroup per CU: bp_lds_kernel
    // is faster (its variable sums need no reordering); with the two-workgroup 512-thread
    // shape the local-edge kernel wins (bench code: 2.00 vs 1.74 M cw/s); the local-edge
    // kernel for everything else it covers
    // (Monte-Carlo with or without early stop; early-stop decodes with hard decisions only;
    // early-stop decodes that return posteriors when the message LDS can stage n posteriors +
    // n decision bytes (ep_ok: the persistent grid with per-workgroup slabs); min-sum early
    // stop: one check class)
    const bool lds36_ms = LDPC_LDS36_MINSUM && algo == 1 && g.lane_var && g.dv == 3 && g.dc == 6 && g.loc_T != 512;
    const bool one_cls = loc_variant_of(g) == kLocReg36;  // the one-class (3,6) instantiation
    // early stop with posteriors stages n posteriors + n decision bytes in the message LDS
    const bool ep_ok = LDPC_LOC_ET_POST && (size_t)std::max(g.loc_words + 64, g.n) * 4 >= (size_t)g.n * 5;
    const bool mode_ok = mc ? (algo == 0 || (LDPC_LOC_MSMC && one_cls))
                            : (!et || (LDPC_LOC_HARD_ET && (hard_only || ep_ok) && (algo == 0 || one_cls)));
    const bool mset = et && algo == 1;
    if (LDPC_LOC && mode_ok && iters > 0 && !lds36_ms && loc_shape(g, lT, lKP) &&
        loc_lds_bytes(g, iters, mc || mset, mset) <= kLdsMax - 2048)
        return BpPath::Loc;
    if (g.lane_var && g.dv == 3 && g.dc == 6 && lds36_bytes(g, iters, et, mc) <= kLdsMax - 2048)
        return BpPath::Lds36;
    if (g.irr_lane && irr_lds_bytes(g, iters) <= kLdsMax - 1024) return BpPath::Irr;
    const int d = g.max_cdeg;
    if (d > 32) return BpPath::None;
    const bool lds = generic_lds_bytes(g, iters, mc) <= kLdsMax - 2048;
    if (d <= 8) return lds ? BpPath::Generic8 : BpPath::GenericG8;
    if (d <= 16) return lds ? BpPath::Generic16 : BpPath::GenericG16;
    return lds ? BpPath::Generic32 : BpPath::GenericG32;
}

template <int VPT, int T, int ALGO, bool ET, bool MC>
hipError_t launch_lds36_vpt(const ldpc_graph &g, BpArgs a, size_t lds, hipStream_t s) {
    auto k = bp_lds_kernel<3, 6, T, VPT, ALGO, ET, MC>;
    hipError_t e = allow_lds(k, lds);
    if (e != hipSuccess) return e;
    // with early stop, one persistent workgroup per CU looping over codewords beats a
    // workgroup per codeword (+6 %: frames end at different iterations); fixed-count
    // decodes are indifferent (within 0.4 %)
    const bool persistent = ET || (LDPC_LDS36_PREFETCH && !MC);  // fixed-count decode: +1 % with the prefetch
    const int grid = persistent && a.B > LDPC_LDS36_GRID ? LDPC_LDS36_GRID : a.B;
    hipLaunchKernelGGL(k, dim3(grid), dim3(T), lds, s, a);
    return hipGetLastError();
}

template <int ALGO, bool ET, bool MC>
hipError_t launch_lds36(const ldpc_graph &g, BpArgs a, hipStream_t s) {
    const size_t lds = lds36_bytes(g, a.max_iters, ET, MC);
    a.lane_var = g.lane_var;
    a.lane_slot = g.lane_slot;
    a.E = lds_pair_span(g.m, 6);  // message positions (lds_pair_pos), dummies after
#define LDS36_CASE(TT, VV) \
    if (g.lane_T == TT && g.lane_VPT == VV) return launch_lds36_vpt<VV, TT, ALGO, ET, MC>(g, a, lds, s);
    LDS36_CASE(256, 1) LDS36_CASE(256, 2) LDS36_CASE(256, 3) LDS36_CASE(256, 5) LDS36_CASE(256, 9)
    LDS36_CASE(1024, 2) LDS36_CASE(1024, 3) LDS36_CASE(1024, 5) LDS36_CASE(1024, 6) LDS36_CASE(1024, 9)
    LDS36_CASE(1024, 10) LDS36_CASE(1024, 11) LDS36_CASE(1024, 14)
#undef LDS36_CASE
    return hipErrorInvalidValue;
}

#ifndef LDPC_GMEM_T
#define LDPC_GMEM_T 1024  // one 1024-thread workgroup per CU ...
#endif
#ifndef LDPC_GMEM_GRID
#define LDPC_GMEM_GRID 256  // ... so the per-workgroup slabs stay cache-resident
#endif
#ifndef LDPC_GMEM_HYB
#define LDPC_GMEM_HYB 1  // first ~38k message slots in LDS, the rest in the slab
#endif
template <int MAXDC, int ALGO, bool ET, bool MC, bool GMEM>
hipError_t launch_generic(const ldpc_graph &g, BpArgs a, hipStream_t s) {
    constexpr int T = GMEM ? LDPC_GMEM_T : 256;
    auto k = bp_generic_kernel<T, MAXDC, ALGO, ET, MC, GMEM>;
    size_t lds = GMEM ? (MC ? (((size_t)(a.max_iters + 1) * 4 + 15) & ~(size_t)15) : 0)
                      : generic_lds_bytes(g, a.max_iters, MC);
    int grid = a.B;
    if (GMEM) grid = a.B < LDPC_GMEM_GRID ? a.B : LDPC_GMEM_GRID;
    if (GMEM && (!a.scratch || a.scratch_bytes < (((size_t)g.E * 5 + (size_t)g.n * 4 + 15) & ~(size_t)15) * (size_t)grid))
        return hipErrorInvalidValue;
    if (GMEM) {  // fill the rest of the CU's LDS with the first message slots
        const size_t room = kLdsMax - 4096 - lds;
        a.lds_slots = LDPC_GMEM_HYB ? (int)std::min<size_t>((size_t)g.E, room / 4) : 0;
        lds += (size_t)a.lds_slots * 4;
    }
    hipError_t e = allow_lds(k, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(grid), dim3(T), lds, s, a);
    return hipGetLastError();
}

template <int DLO, int DHI, int D0, int D1, bool A0, bool A1, int T, int KP, int ALGO, bool ET, bool MC>
hipError_t launch_loc_shape(const ldpc_graph &g, BpArgs a, hipStream_t s) {
    const size_t lds = loc_lds_bytes(g, a.max_iters, MC || (ET && ALGO == 1), ET && ALGO == 1);
    if constexpr (ET && !MC) {
        if (a.post) {  // early stop with posteriors: persistent grid, slab + counter in scratch
            auto k = bp_loc_kernel<DLO, DHI, D0, D1, KP, T, ALGO, A0, A1, true, false, true>;
            hipError_t e = allow_lds(k, lds);
            if (e != hipSuccess) return e;
            if (!a.scratch || a.scratch_bytes < loc_ep_slab_floats(g) * 4 + sizeof(uint32_t)) return hipErrorInvalidValue;
            const unsigned grid = (unsigned)std::min<int>(a.B, loc_ep_grid());
            a.work = reinterpret_cast<uint32_t *>(a.scratch + loc_ep_slab_floats(g));
            e = hipMemsetAsync(a.work, 0, sizeof(uint32_t), s);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(k, dim3(grid), dim3(T), lds, s, a);
            return hipGetLastError();
        }
    }
    auto k = bp_loc_kernel<DLO, DHI, D0, D1, KP, T, ALGO, A0, A1, ET, MC>;
    hipError_t e = allow_lds(k, lds);
    if (e != hipSuccess) return e;
    unsigned grid = (unsigned)a.B;
    if ((ET || LDPC_LOC_PERSIST > 1) && LDPC_LOC_PERSIST && a.scratch &&
        a.scratch_bytes >= sizeof(uint32_t)) {  // persistent grid on a codeword counter
        grid = (unsigned)std::min<int>(a.B, loc_ep_grid());
        a.work = reinterpret_cast<uint32_t *>(a.scratch);
        if ((e = hipMemsetAsync(a.work, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(T), lds, s, a);
    return hipGetLastError();
}

template <int DLO, int DHI, int D0, int D1, bool A0, bool A1, int ALGO, bool ET, bool MC>
hipError_t launch_loc_deg(const ldpc_graph &g, const BpArgs &a, int T, int KP, hipStream_t s) {
#define LOC_SHAPE(TT, KK) \
    if (T == TT && KP == KK) return launch_loc_shape<DLO, DHI, D0, D1, A0, A1, TT, KK, ALGO, ET, MC>(g, a, s);
    LOC_SHAPE(256, 1) LOC_SHAPE(256, 2) LOC_SHAPE(256, 3) LOC_SHAPE(256, 4)
    LOC_SHAPE(1024, 2) LOC_SHAPE(1024, 3)
    if constexpr (DLO != DHI) {  // 512 threads, 2 waves per SIMD: the RSU-type shape only
        LOC_SHAPE(512, 8) LOC_SHAPE(512, 10)
    } else {  // 512 threads, two workgroups per CU
        LOC_SHAPE(512, 5)
    }
#undef LOC_SHAPE
    return hipErrorInvalidValue;
}

template <int ALGO, bool ET, bool MC>
hipError_t launch_loc(const ldpc_graph &g, BpArgs a, hipStream_t s) {
    int T = 0, KP = 0;
    if (!loc_shape(g, T, KP)) return hipErrorInvalidValue;
    a.loc_var = g.loc_var;
    a.loc_pos = g.loc_pos;
    a.loc_info = g.loc_info;
    a.loc_P = g.loc_P;
    a.loc_ncls = g.loc_ncls;
    a.loc_words = g.loc_words;
    for (int i = 0; i < 5; ++i) {
        a.loc_cls_q[i] = g.loc_cls_q[i];
        a.loc_cls_w[i] = g.loc_cls_w[i];
    }
    for (int i = 0; i < 4; ++i) a.loc_cls_d[i] = g.loc_cls_d[i];
    // the template family from the whole layout shape (loc_variant), not the degrees alone
    if (loc_variant_of(g) == kLocReg36) return launch_loc_deg<6, 6, 2, 2, false, false, ALGO, ET, MC>(g, a, T, KP, s);
    if constexpr (ET && ALGO == 1) return hipErrorInvalidValue;  // min-sum early stop: one check class only
    else return launch_loc_deg<5, 6, 1, 3, false, true, ALGO, ET, MC>(g, a, T, KP, s);
}

template <int DC, int VPT, int ALGO, bool ET, bool MC>
hipError_t launch_irr_shape(const ldpc_graph &g, const BpArgs &a, hipStream_t s) {
    auto k = bp_irr_kernel<DC, VPT, ALGO, ET, MC>;
    const size_t lds = irr_lds_bytes(g, a.max_iters);
    hipError_t e = allow_lds(k, lds);
    if (e != hipSuccess) return e;
    const int grid = irr_slab(g) ? std::min(a.B, LDPC_GMEM_GRID) : a.B;
    hipLaunchKernelGGL(k, dim3(grid), dim3(kIrrT), lds, s, a);
    return hipGetLastError();
}

template <int ALGO, bool ET, bool MC>
hipError_t launch_irr(const ldpc_graph &g, BpArgs a, hipStream_t s) {
    a.irr_lane = g.irr_lane;
    a.irr_cdeg = g.irr_cdeg;
    a.irr_KC = g.irr_KC;
    a.irr_S = g.irr_S;
    a.irr_P = g.irr_P;
    if (irr_slab(g) && (!a.scratch || a.scratch_bytes < (size_t)g.irr_P * 4 * (size_t)std::min(a.B, LDPC_GMEM_GRID)))
        return hipErrorInvalidValue;
#define IRR_CASE(DC, VPT) \
    if (g.irr_DC == DC && g.irr_VPT == VPT) return launch_irr_shape<DC, VPT, ALGO, ET, MC>(g, a, s);
    IRR_CASE(6, 5) IRR_CASE(6, 10) IRR_CASE(6, 20) IRR_CASE(8, 5) IRR_CASE(8, 10) IRR_CASE(8, 20)
#undef IRR_CASE
    return hipErrorInvalidValue;
}

template <int ALGO, bool ET, bool MC>
hipError_t dispatch_bp(const ldpc_graph &g, BpArgs a, hipStream_t s) {
    switch (choose_path(g, a.max_iters, ET, MC, ALGO, a.post == nullptr)) {
        case BpPath::Loc: return launch_loc<ALGO, ET, MC>(g, a, s);
        case BpPath::Lds36: return launch_lds36<ALGO, ET, MC>(g, a, s);
        case BpPath::Irr: return launch_irr<ALGO, ET, MC>(g, a, s);
        case BpPath::Generic8: return launch_generic<8, ALGO, ET, MC, false>(g, a, s);
        case BpPath::Generic16: return launch_generic<16, ALGO, ET, MC, false>(g, a, s);
        case BpPath::Generic32: return launch_generic<32, ALGO, ET, MC, false>(g, a, s);
        case BpPath::GenericG8: return launch_generic<8, ALGO, ET, MC, true>(g, a, s);
        case BpPath::GenericG16: return launch_generic<16, ALGO, ET, MC, true>(g, a, s);
        case BpPath::GenericG32: return launch_generic<32, ALGO, ET, MC, true>(g, a, s);
        default: return hipErrorInvalidValue;
    }
}

template <bool MC>
hipError_t dispatch_bp_algo(const ldpc_graph &g, BpArgs a, int algo, int et, hipStream_t s) {
    if (algo == 0) return et ? dispatch_bp<0, true, MC>(g, a, s) : dispatch_bp<0, false, MC>(g, a, s);
    return et ? dispatch_bp<1, true, MC>(g, a, s) : dispatch_bp<1, false, MC>(g, a, s);
}

BpArgs bp_args(const ldpc_graph &g, int B, int iters, float alpha) {
    BpArgs a{};
    a.cptr = g.cptr;
    a.cvar = g.cvar;
    a.vptr = g.vptr;
    a.vslot = g.vslot;
    a.n = g.n;
    a.m = g.m;
    a.E = g.E;
    a.B = B;
    a.max_iters = iters;
    a.alpha = alpha;
    return a;
}

}  // namespace

// ===========================================================================
// Launchers (ldpc_internal.hpp)
// ===========================================================================
hipError_t launch_bec_decode(const ldpc_graph &g, uint8_t *d_words, int B, int max_iters,
                             int32_t *d_errors, int32_t *d_its, hipStream_t stream) {
    BecArgs a = bec_args(g);
    a.words = d_words;
    a.errors = d_errors;
    a.its = d_its;
    a.max_iters = max_iters;
    int W = 0, T = 0, bytes = 0;
    if (LDPC_BEC_DEC_BITS && bec_dec_bits_shape(g, B, W, T, bytes)) {
        if (bytes == 1) return launch_bec_dec_bits<1024, 1, uint8_t>(g, a, B, stream);
        if (T == 256) {
            if (W == 4) return launch_bec_dec_bits<256, 4, uint32_t>(g, a, B, stream);
            if (W == 2) return launch_bec_dec_bits<256, 2, uint32_t>(g, a, B, stream);
            return launch_bec_dec_bits<256, 1, uint32_t>(g, a, B, stream);
        }
        if (W == 4) return launch_bec_dec_bits<512, 4, uint32_t>(g, a, B, stream);
        if (W == 2) return launch_bec_dec_bits<512, 2, uint32_t>(g, a, B, stream);
        return launch_bec_dec_bits<512, 1, uint32_t>(g, a, B, stream);
    }
    return run_bec<false>(g, a, B, stream);
}

size_t bp_scratch_bytes(const ldpc_graph &g, int B, int iters, int algo, bool ep) {
    algo = algo ? 1 : 0;  // as dispatch_bp_algo maps it: the slab decision must follow the path that runs
    // the per-workgroup posterior slabs only when the early-stop-with-posteriors decode will run
    // on bp_loc_kernel (choose_path may send it to bp_lds_kernel / bp_irr_kernel instead)
    const bool ep_slab = ep && g.loc_KP && choose_path(g, iters, true, false, algo, false) == BpPath::Loc;
    const int grid = B < LDPC_GMEM_GRID ? B : LDPC_GMEM_GRID;
    // the irregular kernel's slab (if any) and, for iteration counts that push
    // it off LDS, the generic kernel's: enough for whichever path runs
    const size_t irr = g.irr_lane && irr_slab(g) ? (size_t)g.irr_P * 4 * (size_t)grid : 0;
    const size_t per = ((size_t)g.E * 5 + (size_t)g.n * 4 + 15) & ~(size_t)15;
    const size_t gen = generic_lds_bytes(g, 0, true) + 4096 <= kLdsMax ? 0 : per * (size_t)grid;
    // bp_loc_kernel early stop: the codeword counter of its persistent grid (+ the per-workgroup
    // slabs before it when posteriors are asked for)
    const size_t loc = g.loc_KP ? (ep_slab ? loc_ep_slab_floats(g) * 4 : 0) + 64 : 0;
    return std::max(std::max(irr, gen), loc);
}

const char *bp_kernel_name(const ldpc_graph &g, int early_stop) {
    // early_stop 2: early stop, hard decisions only (no posteriors)
    switch (choose_path(g, 50, early_stop != 0, false, 0, early_stop == 2)) {
        case BpPath::Loc: return "bp_loc_kernel";
        case BpPath::Lds36: return "bp_lds_kernel<3,6>";
        case BpPath::Irr: return irr_slab(g) ? "bp_irr_kernel<lds+slab>" : "bp_irr_kernel<lds>";
        case BpPath::Generic8: return "bp_generic_kernel<8,lds>";
        case BpPath::Generic16: return "bp_generic_kernel<16,lds>";
        case BpPath::Generic32: return "bp_generic_kernel<32,lds>";
        case BpPath::GenericG8: return "bp_generic_kernel<8,gmem>";
        case BpPath::GenericG16: return "bp_generic_kernel<16,gmem>";
        case BpPath::GenericG32: return "bp_generic_kernel<32,gmem>";
        default: return "none";
    }
}

hipError_t launch_bp_decode(const ldpc_graph &g, const float *d_llr, int B, int max_iters, int algo,
                            float alpha, int early_stop, float *d_post, uint8_t *d_hard,
                            int32_t *d_its, hipStream_t stream, float *d_scratch, size_t scratch_bytes) {
    if (B <= 0) return hipSuccess;
    BpArgs a = bp_args(g, B, max_iters, alpha);
    a.llr = d_llr;
    a.post = d_post;
    a.hard = d_hard;
    a.its = d_its;
    a.scratch = d_scratch;
    a.scratch_bytes = d_scratch ? scratch_bytes : 0;
    return dispatch_bp_algo<false>(g, a, algo, early_stop, stream);
}

hipError_t launch_channel(int channel, float p, float p2, uint64_t seed, uint64_t first_cw, int n, int B,
                          void *d_out, hipStream_t stream) {
    if (B <= 0 || n <= 0) return hipSuccess;
    const size_t total = (size_t)((n + 3) / 4) * (size_t)B;
    const unsigned grid = (unsigned)((total + 255) / 256);
    hipLaunchKernelGGL(channel_kernel, dim3(grid), dim3(256), 0, stream, channel, p, p2, seed, first_cw, n, B,
                       d_out);
    return hipGetLastError();
}

hipError_t launch_mc_decode(const ldpc_graph &g, int channel, float p, float p2, uint64_t seed,
                            uint64_t first_cw, int B, int max_iters, int algo, float alpha, int early_stop,
                            int32_t *trial, int32_t *trial_its, hipStream_t stream, float *d_scratch,
                            size_t scratch_bytes) {
    if (B <= 0) return hipSuccess;
    if (channel == 0) {
        BecArgs a = bec_args(g);
        a.max_iters = max_iters;
        a.ch = make_chan(channel, p, p2, seed);
        a.first_cw = first_cw;
        a.trial = trial;
        a.its = trial_its;
        int W = 0, T = 0, bytes = 0;
        if (LDPC_BEC_BITS && bec_bits_shape(g, B, W, T, bytes)) {
            if (bytes == 1) return launch_bec_bits<1024, 1, uint8_t>(g, a, B, stream);
            if (T == 256) {
                if (W == 4) return launch_bec_bits<256, 4, uint32_t>(g, a, B, stream);
                if (W == 2) return launch_bec_bits<256, 2, uint32_t>(g, a, B, stream);
                return launch_bec_bits<256, 1, uint32_t>(g, a, B, stream);
            }
            if (W == 4) return launch_bec_bits<512, 4, uint32_t>(g, a, B, stream);
            if (W == 2) return launch_bec_bits<512, 2, uint32_t>(g, a, B, stream);
            return launch_bec_bits<512, 1, uint32_t>(g, a, B, stream);
        }
        return run_bec<true>(g, a, B, stream);
    }
    BpArgs a = bp_args(g, B, max_iters, alpha);
    a.ch = make_chan(channel, p, p2, seed);
    a.first_cw = first_cw;
    a.trial = trial;
    a.its = trial_its;
    a.scratch = d_scratch;
    a.scratch_bytes = d_scratch ? scratch_bytes : 0;
    return dispatch_bp_algo<true>(g, a, algo, early_stop, stream);
}

hipError_t launch_mc_bec_ensemble(int n, int dv, int dc, const int32_t *check_lookup, const int32_t *variable_lookup,
                                  float p, uint64_t seed, uint64_t first_cw, int B, int max_iters, int32_t *trial,
                                  int32_t *trial_its, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
#ifndef LDPC_ENS_PEEL
#define LDPC_ENS_PEEL 1  // ensemble MC on the frontier-peeling decoder (peel.hip) where it fits
#endif
    if (LDPC_ENS_PEEL) {
        const hipError_t e = launch_mc_bec_peel(n, dv, dc, check_lookup, variable_lookup, p, seed, first_cw, B,
                                                max_iters, trial, trial_its, stream);
        if (e != hipErrorNotSupported) return e;
    }
    ldpc_graph g{};
    g.n = n;
    g.m = n * dv / dc;
    g.dv = dv;
    g.dc = dc;
    BecArgs a = bec_args(g);
    a.cvar = check_lookup;
    a.vchk = variable_lookup;
    a.graph_stride = (int64_t)n * dv;
    a.max_iters = max_iters;
    a.ch = make_chan(0, p, 0.0f, seed);
    a.first_cw = first_cw;
    a.trial = trial;
    a.its = trial_its;
    return run_bec<true>(g, a, B, stream);
}

hipError_t launch_mc_reduce(const int32_t *trial, const int32_t *trial_its, int B, int max_iters,
                            int expurgation, int64_t stop_frame_errors, int64_t *d_counters,
                            int32_t *d_cutoff, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(mc_cutoff_kernel, dim3(1), dim3(1024), 0, stream, trial, B, max_iters, expurgation,
                       stop_frame_errors, d_counters, d_cutoff);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int blocks = B < 1024 ? (B + 63) / 64 : 256;
    hipLaunchKernelGGL(mc_reduce_kernel, dim3(blocks), dim3(256), 0, stream, trial, trial_its, B, max_iters,
                       expurgation, d_cutoff, d_counters);
    return hipGetLastError();
}

size_t ml_lds_bytes(int n, int m, int W, int T) {
    return (size_t)8 * (2 * (T / 64) + 2) * W + 4 * 19 + (size_t)2 * n + (size_t)4 * m + (size_t)n + (size_t)m + 16;
}

int ml_words(int m) {
    const int need = (m + 1 + 63) / 64;
    for (int w : {1, 2, 4, 8, 16})
        if (w >= need) return w;
    return 0;
}

hipError_t launch_ml_decode(const int32_t *cptr, const int32_t *cvar, int64_t cvar_stride, int dc, int n, int m,
                            const uint8_t *d_in, int B, uint8_t *d_out, int32_t *d_unsolved, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    const int W = ml_words(m);
    const int T = std::min(1024, std::max(64, (m + 63) / 64 * 64));
    const size_t lds = ml_lds_bytes(n, m, W, T);
#define LDPC_ML_CASE(WW)                                                                                    \
    case WW: {                                                                                              \
        hipError_t e = allow_lds(ml_kernel<WW>, lds);                                                       \
        if (e != hipSuccess) return e;                                                                      \
        hipLaunchKernelGGL(ml_kernel<WW>, dim3(B), dim3(T), lds, stream, cptr, cvar, cvar_stride, dc, n, m, \
                           d_in, d_out, d_unsolved);                                                        \
        return hipGetLastError();                                                                           \
    }
    switch (W) {
        LDPC_ML_CASE(1)
        LDPC_ML_CASE(2)
        LDPC_ML_CASE(4)
        LDPC_ML_CASE(8)
        LDPC_ML_CASE(16)
        default: return hipErrorInvalidValue;
    }
#undef LDPC_ML_CASE
}

hipError_t launch_mc_reduce_cut(const int32_t *trial, const int32_t *trial_its, int B, int max_iters, int expurgation,
                                const int32_t *d_cutoff, int64_t *d_counters, hipStream_t stream) {
    if (B <= 0) return hipSuccess;
    const int blocks = B < 1024 ? (B + 63) / 64 : 256;
    hipLaunchKernelGGL(mc_reduce_kernel, dim3(blocks), dim3(256), 0, stream, trial, trial_its, B, max_iters,
                       expurgation, d_cutoff, d_counters);
    return hipGetLastError();
}

}  // namespace ldpc
