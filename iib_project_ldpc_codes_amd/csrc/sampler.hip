// Random (dv, dc) and irregular configuration-model graphs on the device (gfx950): the law of
// random_code_generator.c:21-67 -- a uniform socket permutation conditioned on every check
// being simple.  Layout and rationale: DESIGN.md (graph samplers).
#include <cstdlib>

#include "device_common.hpp"
#include "ldpc_internal.hpp"
#include "ldpc_mi355x.h"

namespace ldpc {
namespace {

// ===========================================================================
// 2c. Random regular (dv, dc) graphs: the law of random_code_generator.c:21-67
//
// Configuration model: a uniform permutation of the n*dv sockets, check c =
// positions [c*dc, c*dc+dc), variable of a socket = socket / dv, and a whole-
// graph redraw whenever a check holds a variable twice (:39-47) -- i.e. a
// uniformly random permutation conditioned on every check being simple.  For
// (3, 6) that condition holds with probability ~0.0074, so a graph costs ~135
// permutations; they are drawn in parallel by one workgroup per graph with the
// Rao-Sandelius method, which is exactly uniform:
//   1. every socket s draws a bucket in [0, K) (K = workgroup size, the top
//      log2 K bits of word (s>>6)&3 of Philox ctr {(s>>8)<<6 | s&63,
//      tag|att<<2|0, g_lo, g_hi}, key = seed); a stable counting sort (bucket-major, socket order within a
//      bucket) lays the buckets out back to back -- per-wave ranks come from
//      log2 K ballots, offsets from a workgroup scan;
//   2. thread t Fisher-Yates-shuffles bucket t from its end, drawing j uniform on
//      [0, i] by Lemire's multiply-with-rejection from its own Philox stream
//      ctr {t<<20 | block, tag|att<<2|1, g_lo, g_hi};
//   3. every check is tested for a repeated variable; any failure redraws the
//      whole permutation (att + 1).
// Variable ids (socket / dv) are permuted instead of sockets: every output
// depends on a socket only through its variable.  The permutation lives in LDS
// (u16) when n*dv < 65536, else in the caller's check_lookup row.
// Output: check_lookup[g][E] (variable ids, check-major) and variable_lookup
// [g][E] (each variable's checks ascending), the reference's edge-list format.
// oracle_sample_regular restates this bit for bit.
// ===========================================================================
constexpr uint32_t kSampleTag = 0x80000000u;  // never 0: channel draws use ctr[1] = 0

struct BucketRng {  // sequential Philox stream of one bucket
    uint32_t k0, k1, c0, c1, g0, g1;
    uint32_t k = 0;
    uint4 blk;
    __device__ __forceinline__ uint32_t next() {
        const uint32_t w = k & 3;
        if (w == 0) blk = philox_block(c0 | (k >> 2), c1, g0, g1, k0, k1);
        ++k;
        return pick4(blk, (int)w);
    }
    __device__ __forceinline__ uint32_t below(uint32_t range) {  // uniform on [0, range)
        uint64_t m = (uint64_t)next() * range;
        uint32_t l = (uint32_t)m;
        if (l < range) {
            const uint32_t t = (0u - range) % range;
            while (l < t) {
                m = (uint64_t)next() * range;
                l = (uint32_t)m;
            }
        }
        return (uint32_t)(m >> 32);
    }
};

// Degree structure: regular (vsock == nullptr: socket s belongs to variable s/dv,
// check c owns slots [c*dc, c*dc+dc)) or CSR (vsock[s] = variable of socket s,
// check c owns slots [cptr[c], cptr[c+1])).  Output, per graph: the variable of
// every slot (check_lookup / CSR check_var) and the variable side -- regular:
// variable_lookup[v*dv + k] = k-th check of v (ascending); CSR: var_slot[vptr[v]
// + k] = k-th slot of v (ascending).
struct SampleShape {
    int n, m, E, dv, dc;
    const int32_t *vsock, *cptr, *vptr;
};

// Variable side of a sampled graph from its check side (chk[x] = variable of
// slot x, global): regular rows get check ids, CSR rows slot ids, each row
// ascending (claims by atomic CAS, then a per-row insertion sort).
__device__ void sample_emit_var_side(const SampleShape &sh, const int32_t *chk, int32_t *vl) {
    const int tid = threadIdx.x, T = blockDim.x;
    const int n = sh.n, E = sh.E, dv = sh.dv, dc = sh.dc;
    const bool csr = sh.vsock != nullptr;
    for (int x = tid; x < E; x += T) vl[x] = -1;
    __threadfence_block();
    __syncthreads();
    for (int x = tid; x < E; x += T) {
        const int v = chk[x];
        int32_t *row = vl + (csr ? sh.vptr[v] : (size_t)v * dv);
        const int deg = csr ? sh.vptr[v + 1] - sh.vptr[v] : dv;
        const int val = csr ? x : x / dc;
        for (int k = 0; k < deg; ++k)
            if (atomicCAS(&row[k], -1, val) == -1) break;
    }
    __threadfence_block();
    __syncthreads();
    for (int v = tid; v < n; v += T) {
        int32_t *r = vl + (csr ? sh.vptr[v] : (size_t)v * dv);
        const int deg = csr ? sh.vptr[v + 1] - sh.vptr[v] : dv;
        for (int x = 1; x < deg; ++x) {
            const int key = r[x];
            int y = x - 1;
            while (y >= 0 && r[y] > key) {
                r[y + 1] = r[y];
                --y;
            }
            r[y + 1] = key;
        }
    }
}

// Graphs with kSeqMinE (8192) <= n*dv <= kSeqMaxE: sequential-draw sampler, one attempt per
// workgroup of kSeqNW waves.  The same law -- a uniform socket permutation conditioned on every
// check being simple -- drawn slot by slot, so a bad check is seen as soon as its last slot is
// drawn and the attempt stops there (a failing (3,6) attempt at n = 64,800 stops after ~1/5 of
// the graph instead of paying a whole permutation):
//   * slot x (in order) takes a uniform unused entry of the pool: its words -- word j = word
//     2(j&1) + (x&1) of Philox4x32-7 ctr {x>>1 | (j>>1)<<20, tag|att<<2|3, g_lo, g_hi}, i.e. one block
//     holds words 2k, 2k+1 of the slot pair x>>1 -- give Lemire draws on [0, R) until one lands
//     on an unused pool index (a bitmap in LDS); 1024 words without one reject the attempt
//     (probability < (1/2)^1000);
//   * the pool starts as all R = E sockets; when R' = ceil(R/2) entries are left the unused ones
//     are compacted in order into a new pool (global scratch, the variable_lookup row) with a
//     fresh bitmap, so no draw ever sees more than half its pool used; the last <= kSeqFinal
//     entries are Fisher-Yates-shuffled by one lane (stream {blk, tag|1<<30|att<<2|3, g});
//   * a round draws up to kSeqSlots (256) consecutive slots, two per lane (the pair of one Philox
//     block: its words 0-1 are both slots' first two words), against the bitmap of the slots
//     before the round; LDS atomic ORs mark the picks, and when two slots picked the same entry
//     the round keeps the slots below the second-lowest slot of the group of the lowest slot that
//     saw its bit already set (found with the group's owner; at least the round's first slot,
//     which is always right, and at most the exact cut) -- a slot's result is its first draw not
//     used by an earlier slot, so the later slots simply redraw next round from the updated
//     bitmap: exactly the sequential process, for any atomic order (tests/test_seq_sampler_rounds.py);
//   * every check whose slots are all drawn is tested (variable ids kept in an LDS ring of the
//     last kSeqRing slots); a repeat rejects the attempt (att+1).
// LDS per attempt at n = 64,800: the bitmap (24.3 KB) + ring, retry lists and sync words (2.4 KB),
// so six attempts -- twelve waves -- per CU.  The waves of an attempt meet at two LDS-only
// barriers per round (draws | marks | cut), two more in the rare rounds with a collision.
// The variable side is built with per-variable occurrence counters packed fb bits per variable
// into the bitmap's LDS (fb = 0: global CAS, sample_emit_var_side).
// oracle_sample_regular / oracle_sample_csr restate it bit for bit.
constexpr int kSeqFinal = 64;
// the draws' Philox4x32 rounds: 7, the crush-resistant minimum (Salmon et al., SC'11, Table 2;
// 10 is Random123's default with a safety margin -- the channels keep 10, rocRAND's stream):
// 28 VALU per block instead of 40, -5 % per graph
constexpr int kSeqPhiloxRounds = 7;
constexpr int kSeqFirstBlocks = 2;  // Philox blocks every slot pair draws up front (2 words per slot each)
constexpr int kSeqSplit = 2;        // a stage ends when ceil(R / 2) pool entries are left (f <= 1/2)
constexpr int kSeqNW = 2;                      // waves per attempt
constexpr int kSeqT = kSeqNW * kWave;          // threads per attempt
constexpr int kSeqSlots = 2 * kSeqT;           // slots per round: two per lane
constexpr int kSeqRing = 512;                  // ring: a round + the longest check it completes
static_assert(kSeqSlots + kSeqMaxCdeg <= kSeqRing, "the ring must hold a round and the check it completes");
static_assert(kSeqNW == 2, "the cut words hold two waves");
static_assert(kSeqMaxE <= (1 << 19), "first-pass keys: an entry in 19 bits, the word index above bit 20");
// LDS sync words of an attempt: reject flags by round parity [0, 2), per parity and wave the two lowest
// colliding slots and the lowest one's pick [2, 14), the pick's owner per wave [14, 16), the
// claim broadcast [16, 19)
enum { kSyFlag = 0, kSyCut = 2, kSyOwn = 14, kSyClaim = 16, kSeqSync = 24 };
// LDS of an attempt: sy [kSeqSync] | tl [kSeqNW][2 kWave] | fin [kSeqFinal] | ring [kSeqRing] RT | bitmap [bw]
// (the bitmap last: its LDS address is a constant, folded into the ds instructions' offsets)
constexpr uint32_t kSeqRingOff = 4u * (kSeqSync + 2 * kSeqT + kSeqFinal);
template <typename RT>
__host__ __device__ constexpr uint32_t seq_bm_off() {
    return kSeqRingOff + (uint32_t)sizeof(RT) * kSeqRing;
}

// LDS ordering between the lanes of one wave (LDS instructions of a wave execute in order):
// a compiler barrier only
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}
// the attempt's waves: an s_barrier ordering LDS only (no wait for outstanding global stores,
// which a __syncthreads fence would add to every round)
__device__ __forceinline__ void seq_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ int wave_excl_scan(int v, int &total) {
    const int lane = threadIdx.x & 63;
    int incl = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const int y = __shfl_up(incl, d, kWave);
        if (lane >= d) incl += y;
    }
    total = __shfl(incl, kWave - 1, kWave);
    return incl - v;
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// The bitmap as an LDS byte address: the sampler kernels have no static LDS, so dynamic LDS
// starts at address 0 (checked at kernel entry) and the bitmap at the constant offset
// seq_bm_off<RT>() -- entry e's word is one ds instruction with that offset folded in (through
// the extern array the compiler adds the array's address, 0, with one VALU per access).
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ lds_u32 *bm_word(uint32_t bmoff, int e) {
    return (lds_u32 *)(size_t)(bmoff + (((uint32_t)e >> 3) & ~3u));
}

// Shared state of one workgroup's sequential-draw attempts (LDS pointers, graph id, key).
struct SeqCtx {
    SampleShape sh;
    uint32_t k0, k1, g0, g1;
    uint32_t mdv;  // regular: socket / dv as a multiply-high by ceil(2^32 / dv) (0: divide)
    uint32_t mdc;  // regular: slot / dc likewise (exact below 2^21 for every dc <= 256)
    uint32_t *bm;  // [bw] pool bitmap
    void *ring;    // [kSeqRing] variable of slot x at x % kSeqRing (u16 when n <= 65536, else int)
    int *fin;      // [kSeqFinal] last pool entries
    int *tl;       // [kSeqNW][2 * kWave] retry task lists (second half: writes of lanes without a task)
    int *sy;       // [kSeqSync] sync words
};

template <bool CSR>
__device__ __forceinline__ int seq_var_of(const SeqCtx &c, int s) {
    return CSR ? c.sh.vsock[s] : (c.mdv ? (int)__umulhi((uint32_t)s, c.mdv) : s / c.sh.dv);
}

__device__ __forceinline__ void seq_clear_bm(uint32_t *bm, int words) {  // every thread of the workgroup
    uint4 *b4 = reinterpret_cast<uint4 *>(bm);
    for (int w = (int)threadIdx.x; w < (words + 3) >> 2; w += (int)blockDim.x) b4[w] = make_uint4(0u, 0u, 0u, 0u);
}

constexpr uint32_t kSeqNone = 0xFFFFFFFFu;  // search: no simple attempt found (yet)

// Diagnostics build only (-DLDPC_SEQ_STATS=1, scripts/build_sampler_variant.sh): the passes count
// attempts, rounds, kept slots and collision rounds into g_seq_stats (ldpc_debug_seq_stats);
// the product build compiles every SEQ_STAT to nothing.
#ifndef LDPC_SEQ_STATS
#define LDPC_SEQ_STATS 0
#endif
enum SeqStat { kStAttempts, kStAborted, kStRounds, kStKept, kStLaneIters, kStSpreadIters, kStCollRounds, kStAbortRounds,
               kStCount };
__device__ unsigned long long g_seq_stats[2 * kStCount];  // search pass, then emit pass
#if LDPC_SEQ_STATS
#define SEQ_STAT(pass, i, v)                                                                            \
    do {                                                                                                \
        if (threadIdx.x == 0) atomicAdd(&g_seq_stats[(pass) * kStCount + (i)], (unsigned long long)(v)); \
    } while (0)
#else
#define SEQ_STAT(pass, i, v) \
    do {                     \
    } while (0)
#endif

// Attempt `att` of the sequential draw (the whole workgroup; every return value and loop trip
// is workgroup-uniform).  out != nullptr: every slot's variable also goes to out[x].  pools: >= E
// ints of global scratch (the stage pools, two halves used alternately).  best != nullptr
// (search): the attempt is abandoned once *best (the lowest simple attempt found by any
// workgroup) is below att -- it can no longer be the graph's first simple attempt.
// Returns true when the attempt drew a simple graph.  On entry the LDS of the previous attempt
// may still be read by other waves: the caller has passed a barrier.
template <bool CSR, typename RT, int PASS>
__device__ bool seq_attempt(const SeqCtx &c, int att, int32_t *out, int32_t *pools, const uint32_t *best) {
    constexpr int T = kSeqT, S = kSeqSlots;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int E = c.sh.E, m = c.sh.m, dc = c.sh.dc;
    const uint32_t g0 = c.g0, g1 = c.g1;
    const PhiloxKeys K = philox_keys(c.k0, c.k1);  // the round loop's Philox keys in VGPRs
    uint32_t *const bm = c.bm;
    constexpr uint32_t bmo = seq_bm_off<RT>();
    RT *const ring = reinterpret_cast<RT *>(c.ring);
    int *const tl = c.tl + wave * 2 * kWave;
    int *const sy = c.sy;
    const uint32_t c1 = kSampleTag | ((uint32_t)att << 2) | 3u;
    int R = E, x0 = 0, cdone = 0, nround = 0, par = 0;
    uint32_t bseen = kSeqNone;  // search (wave 0): *best as last loaded
    (void)PASS;

    // checks whose slots all lie below `upto`, from cdone on (one wave per round): a repeated
    // variable sets the reject flag of this round (read by every wave after the next round's
    // first barrier)
    auto validate = [&](int upto) {
        int cend = cdone;
        if constexpr (CSR) {
            for (;;) {
                const int cc = cend + lane;
                const uint64_t f = __ballot(cc < m && c.sh.cptr[cc + 1] <= upto);  // a prefix of the lanes
                cend += __popcll(f);
                if (f != ~0ull) break;
            }
            cend = uni(cend);
        } else {
            cend = uni((int)__umulhi((uint32_t)upto, c.mdc));
        }
        if (wave == (par & (kSeqNW - 1))) {  // one wave per round, alternating
            bool b = false;
            for (int cb = cdone; cb < cend; cb += kWave) {
                const int cc = cb + lane;
                if (cc < cend) {
                    const int lo = CSR ? c.sh.cptr[cc] : cc * dc, d = CSR ? c.sh.cptr[cc + 1] - lo : dc;
                    if (!CSR && d == 6 && sizeof(RT) == 2) {
                        // (3,6), u16 ring: the six variables as three u16 pairs (lo even: no pair
                        // straddles the ring's end); the 15 pairs compared as nine packed XORs
                        // (each pair within a word, and two words against each other straight
                        // and half-swapped), a zero half = a repeated variable
                        const lds_u32 *r32 = (const lds_u32 *)(size_t)kSeqRingOff;  // the ring (see bm_word)
                        const int p = lo & (kSeqRing - 1);
                        const uint32_t w0 = r32[p >> 1], w1 = r32[((p + 2) & (kSeqRing - 1)) >> 1],
                                       w2 = r32[((p + 4) & (kSeqRing - 1)) >> 1];
                        const uint32_t s0 = __builtin_amdgcn_alignbit(w0, w0, 16), s1 = __builtin_amdgcn_alignbit(w1, w1, 16),
                                       s2 = __builtin_amdgcn_alignbit(w2, w2, 16);
                        auto h = [](uint32_t x) { return __builtin_bit_cast(u16x2, x); };
                        u16x2 mn = __builtin_elementwise_min(h(w0 ^ s0), h(w1 ^ s1));
                        mn = __builtin_elementwise_min(mn, h(w2 ^ s2));
                        mn = __builtin_elementwise_min(mn, h(w0 ^ w1));
                        mn = __builtin_elementwise_min(mn, h(w0 ^ s1));
                        mn = __builtin_elementwise_min(mn, h(w0 ^ w2));
                        mn = __builtin_elementwise_min(mn, h(w0 ^ s2));
                        mn = __builtin_elementwise_min(mn, h(w1 ^ w2));
                        mn = __builtin_elementwise_min(mn, h(w1 ^ s2));
                        b |= mn.x == 0 || mn.y == 0;
                    } else if (!CSR && d == 6) {
                        int v[6];
#pragma unroll
                        for (int u = 0; u < 6; u += 2) {
                            const int2 w = *reinterpret_cast<const int2 *>(ring + ((lo + u) & (kSeqRing - 1)));
                            v[u] = w.x;
                            v[u + 1] = w.y;
                        }
#pragma unroll
                        for (int u = 0; u < 6; ++u)
#pragma unroll
                            for (int w = u + 1; w < 6; ++w) b |= v[u] == v[w];
                    } else if (d <= 8) {
                        int v[8];
#pragma unroll
                        for (int a = 0; a < 8; ++a) v[a] = a < d ? (int)ring[(lo + a) & (kSeqRing - 1)] : -1 - a;
#pragma unroll
                        for (int a = 0; a < 8; ++a)
#pragma unroll
                            for (int e = a + 1; e < 8; ++e) b |= v[a] == v[e];
                    } else {
                        for (int a = 0; a < d && !b; ++a) {
                            const int va = (int)ring[(lo + a) & (kSeqRing - 1)];
                            for (int e = a + 1; e < d; ++e) b |= va == (int)ring[(lo + e) & (kSeqRing - 1)];
                        }
                    }
                }
            }
            if (__ballot(b) != 0ull && lane == 0) sy[kSyFlag + par] = 1;
        }
        cdone = cend;
    };

    // the rounds of one stage (slots x0 .. xend - 1); POOL: the pool is the global row at
    // pools + cur (stage 0: the sockets themselves -- no global load in its rounds).  Thread tid
    // draws slots base + 2 tid + q (q = 0, 1) from Philox block (base >> 1) + tid.
    // Returns false when the attempt is rejected.
    auto rounds = [&](auto pool_tag, int xend, int cur) -> bool {
        constexpr bool POOL = decltype(pool_tag)::value;
        const int32_t *pool = pools + cur;
        const uint32_t lt = (0u - (uint32_t)R) % (uint32_t)R;  // Lemire: reject low words below this
        // entry of word w, or -1 when Lemire's test or the bitmap rejects it
        auto try_word = [&](uint32_t w) -> int {
            const uint64_t mm = (uint64_t)w * (uint32_t)R;
            const int e = (int)(mm >> 32);
            const bool used = (*bm_word(bmo, e) >> (e & 31)) & 1u;
            return ((uint32_t)mm < lt || used) ? -1 : e;
        };
        while (x0 < xend) {
            if (best && wave == 0 && (++nround & 15) == 0) {  // search: a lower simple attempt makes this one moot
                // (the value loaded 16 rounds ago: the load's latency never stalls a round)
                if (__builtin_amdgcn_readfirstlane(bseen) < (uint32_t)att) {
                    if (lane == 0) sy[kSyFlag + par] = 1;
                    SEQ_STAT(PASS, kStAborted, 1);
                    SEQ_STAT(PASS, kStAbortRounds, nround);
                }
                bseen = __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            SEQ_STAT(PASS, kStRounds, 1);
            const int base = x0 & ~1;
            const uint32_t blk = (uint32_t)(base >> 1) + (uint32_t)tid;
            // the first 2 kSeqFirstBlocks words of both slots: kSeqFirstBlocks blocks (their
            // ten-step chains interleaved), all their bitmap reads in one LDS round trip
            uint4 Wf[kSeqFirstBlocks];
            {
                uint32_t cc[kSeqFirstBlocks];
#pragma unroll
                for (int f = 0; f < kSeqFirstBlocks; ++f) cc[f] = blk | ((uint32_t)f << 20);
                philox_blocks<kSeqFirstBlocks, kSeqPhiloxRounds>(cc, c1, g0, g1, K, Wf);
            }
            // word j of a slot keys as (j << 20) | entry, all ones when the entry is used (the
            // bitmap bit sign-extended by v_bfe_i32): the slot's pick is its lowest key.  Lemire's
            // rejection (low product word below lt: probability R / 2^32 per word) is tested for
            // the whole wave at once; only a wave holding such a word re-keys with the test.
            constexpr int NWF = 2 * kSeqFirstBlocks;
            int i[2];
            bool act[2], need[2];
            uint32_t key[2][NWF], low[2][NWF], mn[2];
            uint32_t lmin = 0xFFFFFFFFu;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int x = base + 2 * tid + q;
                act[q] = x >= x0 && x < xend;
                mn[q] = 0xFFFFFFFFu;
#pragma unroll
                for (int j = 0; j < NWF; ++j) {
                    const uint4 &W = Wf[j >> 1];
                    const uint32_t w = (j & 1) ? (q ? W.w : W.z) : (q ? W.y : W.x);
                    const uint64_t mm = (uint64_t)w * (uint32_t)R;
                    const uint32_t e = (uint32_t)(mm >> 32);
                    low[q][j] = (uint32_t)mm;
                    const uint32_t used = (uint32_t)__builtin_amdgcn_sbfe((int)*bm_word(bmo, (int)e), e, 1u);
                    key[q][j] = e | used | ((uint32_t)j << 20);
                    mn[q] = min(mn[q], key[q][j]);
                    lmin = min(lmin, low[q][j]);
                }
            }
            if (__ballot(lmin < lt)) {  // rare: exact Lemire
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    mn[q] = 0xFFFFFFFFu;
#pragma unroll
                    for (int j = 0; j < NWF; ++j) mn[q] = min(mn[q], low[q][j] < lt ? 0xFFFFFFFFu : key[q][j]);
                }
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                i[q] = __builtin_amdgcn_sbfe((int)mn[q], 0u, 20u);  // the entry (< 2^19), or -1 (all ones)
                need[q] = act[q] && i[q] < 0;
            }
            // later stages: the pool entries of the first draws are loaded now, so the global
            // load's latency overlaps the retries and the marking (a retried slot reloads)
            int pre[2] = {0, 0};
            if constexpr (POOL) {
#pragma unroll
                for (int q = 0; q < 2; ++q) pre[q] = pool[max(i[q], 0)];
            }
            const bool firstok0 = !need[0], firstok1 = !need[1];
            // retries, within the wave: while many slots still look every lane draws the next
            // block of its own pair; once at most 16 do, the wave spreads them -- L = 4..16 lanes
            // per slot, each trying one of the slot's next L words, the lowest passing word wins
            // (a slot's words are tried in order, so the result is the same)
            uint32_t j0 = 2 * kSeqFirstBlocks;  // next word index of every slot still looking (even)
            bool over = false;
            for (bool any = __ballot(need[0] || need[1]) != 0ull; any;) {  // (uniform; most rounds: none)
                const uint64_t mq0 = __ballot(need[0]), mq1 = __ballot(need[1]);
                const int C = __popcll(mq0) + __popcll(mq1);
                if (C == 0) break;
                if (j0 >= 1024u) {  // a slot rejected 1024 words: reject the attempt
                    over = true;
                    break;
                }
                if (C > 16) {  // (spreading would give each slot at most two lanes: the same words, more work)
                    SEQ_STAT(PASS, kStLaneIters, 1);
                    const uint4 W = philox_block<kSeqPhiloxRounds>(blk | (j0 << 19), c1, g0, g1, K);  // (j0 >> 1) << 20
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        int e = try_word(q ? W.y : W.x);
                        if (e < 0) e = try_word(q ? W.w : W.z);
                        i[q] = need[q] ? e : i[q];
                        need[q] = need[q] && e < 0;
                    }
                    j0 += 2;
                    continue;
                }
                SEQ_STAT(PASS, kStSpreadIters, 1);
                // spread: slot p (q-major order) gets lanes [p*L, p*L + L), lane p*L + k' tries
                // word j0 + k'
                const int lg1 = C <= 4 ? 4 : (C <= 8 ? 3 : (C <= 16 ? 2 : 1));  // L * C <= 64
                const int L = 1 << lg1;
                const uint32_t lmask = (uint32_t)((1ull << L) - 1ull);
                const uint32_t b0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(mq0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mq0, 0u));
                const uint32_t b1 = __builtin_amdgcn_mbcnt_hi((uint32_t)(mq1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mq1, 0u));
                const int pos[2] = {(int)b0, (int)__popcll(mq0) + (int)b1};
                tl[need[0] ? pos[0] : kWave + lane] = lane;
                tl[need[1] ? pos[1] : kWave + lane] = lane | 64;
                wave_sync();
                const int p = lane >> lg1, kl = lane & (L - 1);
                const int ent = tl[p < C ? p : 0];
                const int own = ent & 63, qq = ent >> 6;
                const uint32_t jj = j0 + (uint32_t)kl;
                const uint32_t ob = (uint32_t)(base >> 1) + (uint32_t)(wave * kWave + own);
                const uint4 W = philox_block<kSeqPhiloxRounds>(ob | ((jj >> 1) << 20), c1, g0, g1, K);
                const int eh = (p < C && jj < 1024u) ? try_word(pick4(W, 2 * (int)(jj & 1u) + qq)) : -1;
                const uint64_t okm = __ballot(eh >= 0);
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int s0 = need[q] ? pos[q] << lg1 : 0;
                    const uint32_t seg = (uint32_t)(okm >> s0) & lmask;
                    const int src = seg ? s0 + (int)__builtin_ctz(seg) : lane;
                    const int got = __shfl(eh, src, kWave);
                    const bool hit = need[q] && seg != 0u;
                    i[q] = hit ? got : i[q];
                    need[q] = need[q] && seg == 0u;
                }
                j0 += (uint32_t)L;
                wave_sync();  // tl is rewritten by the next spread
            }
            int val[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const bool fok = q ? firstok1 : firstok0;
                const int ii = max(i[q], 0);
                if constexpr (POOL) val[q] = fok ? pre[q] : pool[ii];
                else val[q] = seq_var_of<CSR>(c, ii);
            }
            if (over && lane == 0) sy[kSyFlag + par] = 1;
            seq_sync();  // (A) every wave's draws read the bitmap of the slots before the round
            if (uni(sy[kSyFlag + (par ^ 1)])) return false;  // the previous round rejected the attempt
            // mark the picks; a pick whose bit was already set (by another slot of the round)
            // is a collision, and the round keeps the slots below the lowest such slot
            bool dup[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const bool mk = act[q] && !need[q];
                const uint32_t bit = mk ? 1u << (i[q] & 31) : 0u;
                const uint32_t old =
                    __hip_atomic_fetch_or(bm_word(bmo, mk ? i[q] : 0), bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                dup[q] = need[q] || (old & bit) != 0u;  // need: a slot without a word (over)
            }
            {
                // this wave's two lowest colliding slots and the lowest one's pick (the cut below)
                const uint64_t d0 = __ballot(dup[0]), d1 = __ballot(dup[1]);
                int c1 = S, c2 = S, e1 = -1;
                if (d0 | d1) {  // (uniform; most rounds have no collision)
                    const uint64_t d0b = d0 & (d0 - 1), d1b = d1 & (d1 - 1);
                    const int la = d0 ? (int)__builtin_ctzll(d0) : 64, lb = d1 ? (int)__builtin_ctzll(d1) : 64;
                    const int ca = 2 * la, ca2 = d0b ? 2 * (int)__builtin_ctzll(d0b) : 128;  // slots 2 l + q of the wave
                    const int cb = 2 * lb + 1, cb2 = d1b ? 2 * (int)__builtin_ctzll(d1b) + 1 : 129;
                    const int m1 = min(ca, cb), m2 = ca < cb ? min(ca2, cb) : min(cb2, ca);
                    e1 = ca < cb ? __builtin_amdgcn_readlane(i[0], la) : __builtin_amdgcn_readlane(i[1], lb);
                    c1 = wave * 2 * kWave + m1;
                    c2 = m2 < 128 ? wave * 2 * kWave + m2 : S;
                }
                if (lane == 0) {
                    int *cw = sy + kSyCut + 6 * par + 3 * wave;
                    cw[0] = c1;
                    cw[1] = c2;
                    cw[2] = e1;
                }
            }
            // ring: both slots of the pair in one store (base is even); a slot below x0 (x0 odd)
            // keeps its value, slots at or above the cut are redrawn (and rewritten) before any
            // check that holds them is tested
            {
                const int p = (base + 2 * tid) & (kSeqRing - 1);
                int v0 = val[0];
                if (tid == 0 && (x0 & 1)) v0 = (int)ring[p];
                if constexpr (sizeof(RT) == 2)
                    *reinterpret_cast<uint32_t *>(ring + p) = (uint32_t)v0 | ((uint32_t)val[1] << 16);
                else
                    *reinterpret_cast<int2 *>(ring + p) = make_int2(v0, val[1]);
            }
            seq_sync();  // (B) marks, cut words and ring
            const int tend = min(S, xend - base);
            const int *cw = sy + kSyCut + 6 * par;
            const int a1 = uni(cw[0]), b1 = uni(cw[3]);
            const int D = min(a1, b1);  // the lowest slot that found its bit set
            int t = min(D, tend);
            if (t < tend) {  // a collision
                SEQ_STAT(PASS, kStCollRounds, 1);
                // The round keeps the slots below the second-lowest slot of every group of equal
                // picks.  D's group: if its owner (the slot that set the bit) is below D, D is
                // that group's second-lowest and no other group's is lower -- t = D exactly;
                // otherwise every group's second-lowest is at least min(owner, the next
                // colliding slot d2) -- t = that (a slot of another group may be cut early: it
                // redraws next round, the same result).  Never fewer than the round's first slot.
                const int a2 = uni(cw[1]), b2 = uni(cw[4]);
                const int d2 = a1 <= b1 ? min(a2, b1) : min(b2, a1);
                const int eD = uni(a1 <= b1 ? cw[2] : cw[5]);
                bool own[2];
#pragma unroll
                for (int q = 0; q < 2; ++q) own[q] = act[q] && !dup[q] && i[q] == eD;
                const uint64_t o0 = __ballot(own[0]), o1 = __ballot(own[1]);
                int om = S;
                if (o0) om = 2 * (wave * kWave + (int)__builtin_ctzll(o0));
                if (o1) om = min(om, 2 * (wave * kWave + (int)__builtin_ctzll(o1)) + 1);
                if (lane == 0) sy[kSyOwn + wave] = om;
#pragma unroll
                for (int q = 0; q < 2; ++q)  // undo every pick of the round ...
                    if (act[q] && !dup[q])
                        __hip_atomic_fetch_and(bm_word(bmo, i[q]), ~(1u << (i[q] & 31)), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                seq_sync();
                const int oD = min(uni(sy[kSyOwn]), uni(sy[kSyOwn + 1]));
                t = min(max(oD < D ? D : min(oD, d2), x0 - base + 1), tend);
#pragma unroll
                for (int q = 0; q < 2; ++q)  // ... and redo the kept ones
                    if (act[q] && !need[q] && 2 * tid + q < t)
                        __hip_atomic_fetch_or(bm_word(bmo, i[q]), 1u << (i[q] & 31), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                seq_sync();
            }
            if (out) {
                const int s = base + 2 * tid;
                if (act[0] && act[1] && 2 * tid + 1 < t) {
                    *reinterpret_cast<int2 *>(out + s) = make_int2(val[0], val[1]);  // s even: 8-byte aligned
                } else {
                    if (act[0] && 2 * tid < t) out[s] = val[0];
                    if (act[1] && 2 * tid + 1 < t) out[s + 1] = val[1];
                }
            }
            SEQ_STAT(PASS, kStKept, base + t - x0);
            x0 = base + t;
            validate(x0);
            par ^= 1;
        }
        return true;
    };
    // compact the unused entries of the stage's pool (R entries), in order, into dst (wave 0)
    auto compact = [&](auto pool_tag, int cur, auto *dst) {
        constexpr bool POOL = decltype(pool_tag)::value;
        const int32_t *pool = pools + cur;
        const int words = (R + 31) >> 5;
        int obase = 0;
        for (int w0 = 0; w0 < words; w0 += kWave) {
            const int w = w0 + lane;
            uint32_t un = 0u;
            if (w < words) {
                un = ~bm[w];
                const int valid = R - w * 32;
                if (valid < 32) un &= (1u << valid) - 1u;
            }
            int tot = 0;
            int o = obase + wave_excl_scan(__popc(un), tot);
            while (un) {
                const int b = __ffs(un) - 1;
                un &= un - 1u;
                const int idx = w * 32 + b;
                dst[o++] = POOL ? pool[idx] : seq_var_of<CSR>(c, idx);
            }
            obase += tot;
        }
    };

    seq_clear_bm(bm, (R + 31) >> 5);
    if (tid < 2) sy[kSyFlag + tid] = 0;
    __syncthreads();
    int cur = -1;  // offset of the current pool in `pools` (-1: stage 0, the sockets)
    while (R > kSeqFinal) {
        const int Rn = (R + kSeqSplit - 1) / kSeqSplit, xend = E - Rn;
        const bool ok = cur < 0 ? rounds(bool_c<false>{}, xend, 0) : rounds(bool_c<true>{}, xend, cur);
        if (!ok) return false;
        if (wave == 0) {
            if (Rn <= kSeqFinal) {  // the last entries go to LDS
                if (cur < 0) compact(bool_c<false>{}, 0, c.fin);
                else compact(bool_c<true>{}, cur, c.fin);
            } else {  // the next pool: pools[0 ..) and pools[ceil(E/2) ..) alternately
                const int nx = cur == 0 ? (E + 1) / 2 : 0;
                if (cur < 0) compact(bool_c<false>{}, 0, pools + nx);
                else compact(bool_c<true>{}, cur, pools + nx);
            }
        }
        if (Rn > kSeqFinal) cur = cur == 0 ? (E + 1) / 2 : 0;
        __syncthreads();  // the new pool (global or LDS) is visible to every wave
        R = Rn;
        seq_clear_bm(bm, (R + 31) >> 5);
        __syncthreads();
    }
    // last R <= kSeqFinal entries (in fin): Fisher-Yates by thread 0, then the last slots
    int *const fin = c.fin;
    if (R == E && tid < E) fin[tid] = seq_var_of<CSR>(c, tid);  // tiny graphs: no compaction ran
    seq_sync();
    if (tid == 0) {
        BucketRng rng{c.k0, c.k1, 0u, c1 | (1u << 30), g0, g1};
        for (int a = R - 1; a >= 1; --a) {
            const int j = (int)rng.below((uint32_t)a + 1u);
            const int tmp = fin[a];
            fin[a] = fin[j];
            fin[j] = tmp;
        }
    }
    seq_sync();
    if (tid < R) {
        const int x = x0 + tid;
        if (out) out[x] = fin[tid];
        ring[x & (kSeqRing - 1)] = (RT)fin[tid];
    }
    seq_sync();
    validate(E);
    seq_sync();
    return uni(sy[kSyFlag] | sy[kSyFlag + 1]) == 0;
}

// Emit pass (and the whole sampler when start == nullptr): one workgroup per graph draws
// attempts start[g], start[g] + 1, ... in order until one is simple (start[g] = the first simple
// attempt found by sample_search_kernel, so normally exactly one attempt), writes its slots to
// check_lookup[g], then builds the variable side.  attempts[g] = attempts drawn from 0
// (negative: max_attempts without a simple graph -- then the identity configuration).
template <typename RT>
__host__ __device__ constexpr size_t seq_lds_bytes(int bw) {
    return (size_t)4 * (bw + kSeqFinal + 2 * kSeqT + kSeqSync) + sizeof(RT) * kSeqRing;
}

template <typename RT>
__device__ __forceinline__ SeqCtx seq_ctx(const SampleShape &sh, uint32_t k0, uint32_t k1, uint64_t gid, uint32_t mdv,
                                         unsigned char *smem, int bw) {
    (void)bw;
    // bm_word: dynamic LDS at LDS address 0 (no static LDS in these kernels)
    if ((uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char *)smem != 0u) __builtin_trap();
    int *sy = reinterpret_cast<int *>(smem);
    int *tl = sy + kSeqSync;
    int *fin = tl + 2 * kSeqT;
    RT *ring = reinterpret_cast<RT *>(fin + kSeqFinal);
    uint32_t *bm = reinterpret_cast<uint32_t *>(ring + kSeqRing);  // last: every other offset is a constant
    const uint32_t mdc = sh.vsock ? 0u : (uint32_t)((0x100000000ull + (uint32_t)sh.dc - 1u) / (uint32_t)sh.dc);
    return SeqCtx{sh, k0, k1, (uint32_t)gid, (uint32_t)(gid >> 32), mdv, mdc, bm, ring, fin, tl, sy};
}

template <bool CSR, typename RT>  // CSR: irregular degree structure (sh.vsock / cptr / vptr); RT: ring entries
__global__ __launch_bounds__(kSeqT) void sample_seq_kernel(SampleShape sh, uint32_t k0, uint32_t k1,
                                                           uint64_t first_graph, int32_t *check_lookup,
                                                           int32_t *variable_lookup, int32_t *attempts,
                                                           int max_attempts, int bw, int fb, uint32_t mdv,
                                                           const uint32_t *start, const uint32_t *homewin) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int n = sh.n, E = sh.E, dv = sh.dv, dc = sh.dc;
    constexpr bool csr = CSR;
    const int tid = threadIdx.x;
    const SeqCtx c = seq_ctx<RT>(sh, k0, k1, first_graph + blockIdx.x, mdv, smem, bw);
    uint32_t *bm = c.bm;
    int32_t *out = check_lookup + (size_t)blockIdx.x * E;
    int32_t *vl = variable_lookup + (size_t)blockIdx.x * E;

    int att = start ? (int)min(start[blockIdx.x], (uint32_t)max_attempts) : 0;
    bool ok = false;
    if (homewin && att < max_attempts && homewin[blockIdx.x] == (uint32_t)att) {
        ok = true;  // the search's home workgroup drew this attempt into check_lookup[g] already
        ++att;
    }
    while (!ok && att < max_attempts) {
        ok = seq_attempt<CSR, RT, 1>(c, att, out, vl, nullptr);
        SEQ_STAT(1, kStAttempts, 1);
        ++att;
        __syncthreads();
    }
    if (attempts && tid == 0) attempts[blockIdx.x] = ok ? att : -att;
    if (!ok)  // max_attempts without a simple graph: the identity configuration (in-range ids)
        for (int x = tid; x < E; x += kSeqT) out[x] = seq_var_of<CSR>(c, x);
    __threadfence_block();
    __syncthreads();
    if (fb < 0) return;  // the variable side is built by sample_var_side_kernel
    if (fb == 0) {
        sample_emit_var_side(sh, out, vl);
        return;
    }
    // variable side: occurrence rank of each slot's variable from fb-bit LDS counters
    // (slot order, so rows come out nearly ascending), then a per-row insertion sort
    seq_clear_bm(bm, bw);
    __syncthreads();
    const uint32_t fmask = (1u << fb) - 1u;
    for (int x = tid; x < E; x += kSeqT) {
        const int v = out[x];
        const uint32_t pos = (uint32_t)v * (uint32_t)fb;
        const uint32_t old = atomicAdd(&bm[pos >> 5], 1u << (pos & 31));
        const int rank = (int)((old >> (pos & 31)) & fmask);
        if (csr) vl[sh.vptr[v] + rank] = x;
        else vl[(size_t)v * dv + rank] = x / dc;
    }
    __threadfence_block();
    __syncthreads();
    for (int v = tid; v < n; v += kSeqT) {
        int32_t *r = vl + (csr ? sh.vptr[v] : (size_t)v * dv);
        const int deg = csr ? sh.vptr[v + 1] - sh.vptr[v] : dv;
        for (int x = 1; x < deg; ++x) {
            const int key = r[x];
            int y = x - 1;
            while (y >= 0 && r[y] > key) {
                r[y + 1] = r[y];
                --y;
            }
            r[y + 1] = key;
        }
    }
}

// Variable side of G sampled graphs (after the emit pass): workgroup (g, k) builds the rows of
// variables [k V, (k + 1) V) of graph g in LDS -- every slot of the graph whose variable is in
// the chunk takes the next occurrence rank from fb-bit LDS counters, each row is sorted
// (variable_lookup rows ascending as random_code_generator.c:57-62; regular: check ids, CSR:
// slot ids) -- and writes them out in one coalesced pass, instead of E scattered 4-byte stores
// per graph.  Rows are u16 in LDS when every entry is below 65,536 (so a (3,6) n = 64,800 graph
// takes three chunks); the chunks of one graph read its check side from L2 / MALL and their
// workgroup ids share an XCD (ids congruent mod 8).
template <int T, typename Row>
__global__ __launch_bounds__(T) void sample_var_side_kernel(SampleShape sh, const int32_t *check_lookup,
                                                            int32_t *variable_lookup, int G, int V, int fb,
                                                            int maxdeg) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int n = sh.n, E = sh.E, dv = sh.dv, dc = sh.dc;
    const bool csr = sh.vsock != nullptr;
    const int nch = (n + V - 1) / V;
    // id = (g / 8) * 8 * nch + k * gl + g % 8, gl = graphs in g's group of 8
    const int id = (int)blockIdx.x, grp = id / (8 * nch), rem = id - grp * 8 * nch;
    const int gl = min(8, G - grp * 8);
    const int k = rem / gl, g = grp * 8 + rem % gl;
    const int v0 = k * V, v1 = min(n, v0 + V);
    const int r0 = csr ? sh.vptr[v0] : v0 * dv, r1 = csr ? sh.vptr[v1] : v1 * dv;
    uint32_t *cnt = reinterpret_cast<uint32_t *>(smem);                     // [V * fb bits]
    Row *rows = reinterpret_cast<Row *>(cnt + ((V * fb + 31) / 32 + 3) / 4 * 4);  // [V * maxdeg]
    const int tid = threadIdx.x;
    const int32_t *out = check_lookup + (size_t)g * E;
    int32_t *vl = variable_lookup + (size_t)g * E;
    for (int w = tid; w < (V * fb + 31) / 32; w += T) cnt[w] = 0u;
    __syncthreads();
    const uint32_t fmask = (1u << fb) - 1u;
    auto take = [&](int x, int v) {
        if (v < v0 || v >= v1) return;
        const uint32_t pos = (uint32_t)(v - v0) * (uint32_t)fb;
        const uint32_t old = atomicAdd(&cnt[pos >> 5], 1u << (pos & 31));
        const int rank = (int)((old >> (pos & 31)) & fmask);
        rows[(csr ? sh.vptr[v] : v * dv) - r0 + rank] = (Row)(csr ? x : x / dc);
    };
    int x = tid;
    for (; x + 3 * T < E; x += 4 * T) {  // four loads in flight per thread
        const int va = out[x], vb = out[x + T], vc = out[x + 2 * T], vd = out[x + 3 * T];
        take(x, va);
        take(x + T, vb);
        take(x + 2 * T, vc);
        take(x + 3 * T, vd);
    }
    for (; x < E; x += T) take(x, out[x]);
    __syncthreads();
    for (int v = v0 + tid; v < v1; v += T) {
        Row *r = rows + ((csr ? sh.vptr[v] : v * dv) - r0);
        const int deg = csr ? sh.vptr[v + 1] - sh.vptr[v] : dv;
        for (int y0 = 1; y0 < deg; ++y0) {
            const Row key = r[y0];
            int y = y0 - 1;
            while (y >= 0 && r[y] > key) {
                r[y + 1] = r[y];
                --y;
            }
            r[y + 1] = key;
        }
    }
    __syncthreads();
    for (int i = tid; i < r1 - r0; i += T) vl[r0 + i] = (int32_t)rows[i];
}

// Search pass: finds, for each of G graphs, its first simple attempt -- the attempt the
// sequential sampler would return -- with the attempts of a graph spread over workgroups.
// Persistent workgroups of kSeqNW waves (one attempt at a time); ctl (global): [0] next graph to
// open, [1] unused, best[G] (kSeqNone: none yet), natt[G] (next attempt index to claim),
// homewin[G] (the simple attempt the graph's home workgroup drew into check_lookup[g], kSeqNone:
// none).  A workgroup claims attempts of its home graph until the graph has a simple attempt
// (then opens the next graph); when every graph is open it helps: it probes for a graph still
// without one and claims that graph's attempts until it has one.  Every attempt below a graph's
// final best is claimed and runs to completion (an attempt is abandoned only once best is below
// it), so best = the lowest simple attempt, exactly the sequential result, for any schedule.
// Attempts >= max_attempts are never drawn (best stays kSeqNone).  Pool rows (E ints per
// workgroup): variable_lookup rows (grid <= G), rebuilt by the variable-side pass.  The workgroup
// that opens a graph draws its attempts into check_lookup[g] and records a simple one in
// homewin[g]; the emit pass skips g when homewin[g] == best[g] and redraws attempt best otherwise.
template <bool CSR, typename RT>
__global__ __launch_bounds__(kSeqT) void sample_search_kernel(SampleShape sh, uint32_t k0, uint32_t k1,
                                                              uint64_t first_graph, int G, int32_t *scratch_a,
                                                              int32_t *scratch_b, uint32_t *ctl, int max_attempts,
                                                              int bw, uint32_t mdv) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t *best = ctl + 2, *natt = ctl + 2 + G, *homewin = ctl + 2 + 2 * G, *wk = ctl + 2 + 3 * G;
    int32_t *pools = scratch_b + (size_t)blockIdx.x * sh.E;  // grid <= G: variable_lookup row w
    const uint32_t um = (uint32_t)max_attempts;
    SeqCtx c = seq_ctx<RT>(sh, k0, k1, first_graph, mdv, smem, bw);
    int *const sy = c.sy;
    int home = -1;         // (wave 0) the graph whose attempts this workgroup claims
    bool helping = false;  // every graph is open: homes are picked among the open ones
    uint32_t probe = (uint32_t)blockIdx.x * 0x9E3779B9u + 0x7F4A7C15u;
    for (;;) {
        // wave 0 claims (graph, attempt) -- lane 0 on the home graph, the wave probing for a new
        // home when helping -- and hands it to the workgroup through LDS
        if (wave == 0) {
            int g = -1, att = 0;
            for (;;) {
                if (lane == 0) {
                    for (;;) {
                        if (home < 0 && !helping) {
                            home = (int)atomicAdd(&ctl[0], 1u);
                            if (home >= G) { home = -1; helping = true; }
                            else atomicAdd(&wk[home], 1u);
                        }
                        if (home < 0) break;  // helping without a home: probe below
                        if (__hip_atomic_load(&best[home], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kSeqNone) {
                            const uint32_t a = atomicAdd(&natt[home], 1u);
                            if (a < um) { g = home; att = (int)a; break; }
                        }
                        atomicSub(&wk[home], 1u);
                        home = -1;  // resolved or out of attempts
                    }
                }
                g = uni(g);
                att = uni(att);
                helping = uni((int)helping) != 0;
                if (g >= 0) break;
                // help: probe the graphs from a pseudo-random start (wrapping), 256 per step with
                // their loads issued together, for graphs without a simple attempt and with
                // attempts left, and join the one with the fewest workers in the first step that
                // has any (workers of one graph run attempts past its first simple one until that
                // one completes: spreading the helpers keeps that waste low); none anywhere:
                // this workgroup is done
                probe = probe * 1664525u + 1013904223u;
                const uint32_t start = (uint32_t)(((uint64_t)probe * (uint32_t)G) >> 32);
                int found = -1;
                for (uint32_t k = 0; k < (uint32_t)G && found < 0; k += 4 * kWave) {
                    uint32_t key = 0xFFFFFFFFu;  // (workers << 8 | u * 64 + lane... ) of this lane's best open graph
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const uint32_t off = k + (uint32_t)(u * kWave + lane);
                        uint32_t cg = start + off;
                        if (cg >= (uint32_t)G) cg -= (uint32_t)G;
                        const bool open =
                            off < (uint32_t)G &&
                            __hip_atomic_load(&best[cg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kSeqNone &&
                            __hip_atomic_load(&natt[cg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < um;
                        const uint32_t w = min(__hip_atomic_load(&wk[cg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), 0xFFFFu);
                        if (open) key = min(key, (w << 16) | (uint32_t)(u * kWave + lane));
                    }
                    // wave minimum of the keys (fewest workers, then the lowest offset)
#pragma unroll
                    for (int d = 1; d < kWave; d <<= 1) key = min(key, (uint32_t)__shfl_xor((int)key, d, kWave));
                    key = (uint32_t)uni((int)key);
                    if (key != 0xFFFFFFFFu) {
                        uint32_t cg = start + k + (key & 0xFFFFu);
                        if (cg >= (uint32_t)G) cg -= (uint32_t)G;
                        found = (int)cg;
                    }
                }
                if (found < 0) break;  // nothing left to claim anywhere (g < 0)
                if (lane == 0) atomicAdd(&wk[found], 1u);
                home = found;
            }
            if (lane == 0) {
                sy[kSyClaim] = g;
                sy[kSyClaim + 1] = att;
                sy[kSyClaim + 2] = helping ? 0 : 1;
            }
        }
        seq_sync();
        const int g = uni(sy[kSyClaim]);
        if (g < 0) break;
        const int att = uni(sy[kSyClaim + 1]);
        // the workgroup that opened graph g is the only one writing its check_lookup row: its
        // attempts draw into it (a simple one is then the graph itself unless a helper's lower
        // attempt wins -- the emit pass redraws exactly those graphs); helpers only search
        const bool solo = uni(sy[kSyClaim + 2]) != 0;
        const uint64_t gid = first_graph + (uint64_t)g;
        c.g0 = (uint32_t)gid;
        c.g1 = (uint32_t)(gid >> 32);
        const bool ok = seq_attempt<CSR, RT, 0>(c, att, solo ? scratch_a + (size_t)g * sh.E : nullptr, pools, &best[g]);
        SEQ_STAT(0, kStAttempts, 1);
        if (ok && tid == 0) {
            atomicMin(&best[g], (uint32_t)att);
            if (solo) homewin[g] = (uint32_t)att;
        }
        __syncthreads();
    }
}

template <int T, typename Idx, bool LDSBUF>
__global__ __launch_bounds__(T) void sample_regular_kernel(SampleShape sh, uint32_t k0, uint32_t k1,
                                                           uint64_t first_graph, int32_t *check_lookup,
                                                           int32_t *variable_lookup, int32_t *attempts,
                                                           int max_attempts) {
    constexpr int NW = T / kWave;
    constexpr int LOGK = T == 256 ? 8 : (T == 512 ? 9 : 10);
    extern __shared__ __align__(16) unsigned char smem[];
    int *cnt = reinterpret_cast<int *>(smem);  // [T buckets][NW waves]
    int *wsum = cnt + T * NW;                  // [16]
    const int E = sh.E, m = sh.m, dv = sh.dv, dc = sh.dc;
    const bool csr = sh.vsock != nullptr;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t gid = first_graph + blockIdx.x;
    const uint32_t g0 = (uint32_t)gid, g1 = (uint32_t)(gid >> 32);
    int32_t *chk = check_lookup + (size_t)blockIdx.x * E;
    Idx *buf = LDSBUF ? reinterpret_cast<Idx *>(wsum + 16) : reinterpret_cast<Idx *>(chk);
    const int chunk = ((E + NW - 1) / NW + 255) / 256 * 256;
    const int s_lo = min(E, wave * chunk), s_hi = min(E, s_lo + chunk);
    const uint64_t lt_mask = (1ull << lane) - 1;

    // bucket of socket s = base + lane (base a multiple of 64) from word (s>>6)&3 of
    // the Philox block {(s>>8)<<6 | lane, c1, g}: one block per lane per 256 sockets;
    // peers = the lanes of this 64-socket group in the same bucket
    auto group = [&](int base, const uint4 &r, uint32_t &bk, uint64_t &peers) {
        const int s = base + lane;
        const bool valid = s < s_hi;
        bk = valid ? pick4(r, (base >> 6) & 3) >> (32 - LOGK) : 0u;
        peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < LOGK; ++bit) {
            const bool on = (bk >> bit) & 1u;
            const uint64_t bal = __ballot(valid && on);
            peers &= on ? bal : ~bal;
        }
        return valid;
    };

    int att = 0;
    bool ok = false;
    while (!ok && att < max_attempts) {
        const uint32_t c1 = kSampleTag | ((uint32_t)att << 2);
        for (int i = tid; i < T * NW; i += T) cnt[i] = 0;
        __syncthreads();
        // 1a. bucket sizes per (bucket, wave)
        for (int b256 = s_lo; b256 < s_hi; b256 += 256) {
            const uint4 r = philox_block((uint32_t)(((b256 >> 8) << 6) | lane), c1, g0, g1, k0, k1);
            for (int base = b256; base < min(s_hi, b256 + 256); base += 64) {
                uint32_t bk;
                uint64_t peers;
                if (group(base, r, bk, peers) && (peers & lt_mask) == 0) cnt[bk * NW + wave] += __popcll(peers);
            }
        }
        __syncthreads();
        // 1b. offsets: bucket-major, wave-minor (= socket order inside a bucket)
        int size = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) size += cnt[tid * NW + w];
        int total = 0;
        const int start = block_excl_scan(size, wsum, total);
        {
            int run = start;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const int c = cnt[tid * NW + w];
                cnt[tid * NW + w] = run;
                run += c;
            }
        }
        __syncthreads();
        // 1c. stable scatter of the variable ids
        for (int b256 = s_lo; b256 < s_hi; b256 += 256) {
            const uint4 r = philox_block((uint32_t)(((b256 >> 8) << 6) | lane), c1, g0, g1, k0, k1);
            for (int base = b256; base < min(s_hi, b256 + 256); base += 64) {
                uint32_t bk;
                uint64_t peers;
                if (group(base, r, bk, peers)) {
                    const int s = base + lane;
                    const int dst = cnt[bk * NW + wave] + __popcll(peers & lt_mask);
                    buf[dst] = (Idx)(csr ? sh.vsock[s] : s / dv);
                    if ((peers & lt_mask) == 0) cnt[bk * NW + wave] += __popcll(peers);
                }
            }
        }
        __syncthreads();
        // 2. Fisher-Yates inside bucket `tid`
        {
            BucketRng rng{k0, k1, (uint32_t)tid << 20, c1 | 1u, g0, g1};
            Idx *bb = buf + start;
            for (int i = size - 1; i >= 1; --i) {
                const int j = (int)rng.below((uint32_t)i + 1u);
                const Idx t = bb[i];
                bb[i] = bb[j];
                bb[j] = t;
            }
        }
        __syncthreads();
        // 3. every check simple?
        int bad = 0;
        for (int c = tid; c < m; c += T) {
            const int lo = csr ? sh.cptr[c] : c * dc, d = csr ? sh.cptr[c + 1] - lo : dc;
            const Idx *r = buf + lo;
            for (int x = 0; x < d && !bad; ++x)
                for (int y = x + 1; y < d; ++y) bad |= (r[x] == r[y]);
        }
        ok = !__syncthreads_or(bad);
        ++att;
    }
    if (attempts && tid == 0) attempts[blockIdx.x] = ok ? att : -att;
    // check_lookup (variable ids per slot); variable_lookup rows claimed by CAS, then sorted
    int32_t *vl = variable_lookup + (size_t)blockIdx.x * E;
    if (LDSBUF)
        for (int x = tid; x < E; x += T) chk[x] = buf[x];
    sample_emit_var_side(sh, chk, vl);
}

}  // namespace

static hipError_t launch_sample(const SampleShape &sh, int max_cdeg, int max_vdeg, uint64_t seed,
                                uint64_t first_graph, int G, int32_t *check_lookup, int32_t *variable_lookup,
                                int32_t *attempts, int max_attempts, uint32_t *ctl, hipStream_t stream) {
    if (G <= 0) return hipSuccess;
    const int E = sh.E;
    const int K = sample_buckets(E);
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const size_t ctl_lds = (size_t)4 * (K * (K / kWave) + 16);
    const bool u16 = sh.n <= 65536;
#define LDPC_SAMPLE(TT, IDX, LDSB)                                                                             \
    do {                                                                                                       \
        auto k = sample_regular_kernel<TT, IDX, LDSB>;                                                         \
        const size_t lds = ctl_lds + (LDSB ? (size_t)2 * E : 0);                                                   \
        hipError_t e = allow_lds(k, lds);                                                                      \
        if (e != hipSuccess) return e;                                                                         \
        hipLaunchKernelGGL(k, dim3(G), dim3(TT), lds, stream, sh, k0, k1, first_graph, check_lookup,           \
                           variable_lookup, attempts, max_attempts);                                           \
        return hipGetLastError();                                                                              \
    } while (0)
    const bool seq = E >= kSeqMinE && E <= kSeqMaxE && max_cdeg <= kSeqMaxCdeg;
    if (K == 256 && u16 && !seq) LDPC_SAMPLE(256, uint16_t, true);
    if (K == 512 && u16 && !seq) LDPC_SAMPLE(512, uint16_t, true);
    if (seq) {
        // bitmap words (a multiple of 4: cleared with 16-byte stores); rank counters of
        // fb bits per variable share them when they fit
        int bw = ((E + 31) / 32 + 3) & ~3;
        const int fb = max_vdeg <= 3 ? 2 : (max_vdeg <= 15 ? 4 : (max_vdeg <= 255 ? 8 : 0));
        const int fbu = fb && (long)sh.n * fb <= (long)bw * 32 ? fb : 0;
        const bool r16 = sh.n <= 65536;  // variable ids fit the u16 ring
        const size_t lds = r16 ? seq_lds_bytes<uint16_t>(bw) : seq_lds_bytes<int>(bw);
        auto kern = sh.vsock ? (r16 ? sample_seq_kernel<true, uint16_t> : sample_seq_kernel<true, int>)
                             : (r16 ? sample_seq_kernel<false, uint16_t> : sample_seq_kernel<false, int>);
        hipError_t e = allow_lds(kern, lds);
        if (e != hipSuccess) return e;
        const uint32_t mdv =
            sh.vsock == nullptr && sh.dv > 1 && sh.dv < 256 ? (uint32_t)((0x100000000ull + sh.dv - 1) / sh.dv) : 0u;
        const uint32_t *start = nullptr, *homewin = nullptr;
        if (ctl) {
            // search pass: persistent workgroups of kSeqNW waves, as many as fit the device (LDS
            // bound), at most one pool row each in the 2G rows of the two outputs
            int dev = 0, cus = 0;
            e = hipGetDevice(&dev);
            if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            if (e != hipSuccess) return e;
            const long per_cu = std::max<long>(1, std::min<long>(32, (long)(160 * 1024) / (long)lds));
            const int W = (int)std::min<long>((long)G, (long)cus * per_cu);
            auto sk = sh.vsock ? (r16 ? sample_search_kernel<true, uint16_t> : sample_search_kernel<true, int>)
                               : (r16 ? sample_search_kernel<false, uint16_t> : sample_search_kernel<false, int>);
            if ((e = allow_lds(sk, lds)) != hipSuccess) return e;
            if ((e = hipMemsetAsync(ctl, 0, 8, stream)) != hipSuccess) return e;
            if ((e = hipMemsetAsync(ctl + 2, 0xFF, (size_t)4 * G, stream)) != hipSuccess) return e;
            if ((e = hipMemsetAsync(ctl + 2 + G, 0, (size_t)4 * G, stream)) != hipSuccess) return e;
            if ((e = hipMemsetAsync(ctl + 2 + 2 * G, 0xFF, (size_t)4 * G, stream)) != hipSuccess) return e;
            if ((e = hipMemsetAsync(ctl + 2 + 3 * G, 0, (size_t)4 * G, stream)) != hipSuccess) return e;
            // graphs' home waves draw into check_lookup; pool rows: wave w uses variable_lookup row w
            hipLaunchKernelGGL(sk, dim3(W), dim3(kSeqT), lds, stream, sh, k0, k1, first_graph, G, check_lookup,
                               variable_lookup, ctl, max_attempts, bw, mdv);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            start = ctl + 2;
            homewin = ctl + 2 + 2 * G;
        }
        // variable side: chunks of V variables per workgroup after the emit pass, rows of at most
        // max_vdeg entries staged in LDS (u16 entries when they fit) within ~150 KB
        const bool u16rows = sh.vsock ? sh.E <= 65536 : sh.m <= 65536;
        const size_t rb = u16rows ? 2 : 4;
        int V = 0;
        if (fb) {
            const size_t bits = 8 * rb * (size_t)max_vdeg + (size_t)fb;  // LDS bits per variable
            V = (int)std::min<size_t>((size_t)sh.n, (size_t)150 * 1024 * 8 / bits) & ~63;
            if (V < 64) V = 0;
        }
        hipLaunchKernelGGL(kern, dim3(G), dim3(kSeqT), lds, stream, sh, k0, k1, first_graph,
                           check_lookup, variable_lookup, attempts, max_attempts, bw, V ? -1 : fbu, mdv, start,
                           homewin);
        if ((e = hipGetLastError()) != hipSuccess || !V) return e;
        const int nch = (sh.n + V - 1) / V;
        const size_t vs_lds = (size_t)4 * (((long)V * fb + 31) / 32 + 3) / 4 * 4 + rb * (size_t)V * max_vdeg;
        auto vk = u16rows ? sample_var_side_kernel<1024, uint16_t> : sample_var_side_kernel<1024, int32_t>;
        if ((e = allow_lds(vk, vs_lds)) != hipSuccess) return e;
        hipLaunchKernelGGL(vk, dim3((unsigned)G * nch), dim3(1024), vs_lds, stream, sh, check_lookup, variable_lookup,
                           G, V, fb, max_vdeg);
        return hipGetLastError();
    }
    LDPC_SAMPLE(1024, int32_t, false);
#undef LDPC_SAMPLE
}

hipError_t seq_stats(uint64_t *out, int reset) {
    if (!LDPC_SEQ_STATS) return hipErrorNotSupported;
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_seq_stats), sizeof(unsigned long long) * 2 * kStCount);
    if (e == hipSuccess && reset) {
        static const unsigned long long z[2 * kStCount] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_seq_stats), z, sizeof(z));
    }
    return e;
}

hipError_t launch_sample_regular(int n, int dv, int dc, uint64_t seed, uint64_t first_graph, int G,
                                 int32_t *check_lookup, int32_t *variable_lookup, int32_t *attempts,
                                 int max_attempts, uint32_t *ctl, hipStream_t stream) {
    const SampleShape sh{n, n * dv / dc, n * dv, dv, dc, nullptr, nullptr, nullptr};
    return launch_sample(sh, dc, dv, seed, first_graph, G, check_lookup, variable_lookup, attempts, max_attempts,
                         ctl, stream);
}

hipError_t launch_sample_csr(int n, int m, int E, const int32_t *d_vsock, const int32_t *d_cptr,
                             const int32_t *d_vptr, int max_cdeg, int max_vdeg, uint64_t seed, uint64_t first_graph,
                             int G, int32_t *check_var, int32_t *var_slot, int32_t *attempts, int max_attempts,
                             uint32_t *ctl, hipStream_t stream) {
    const SampleShape sh{n, m, E, 0, 0, d_vsock, d_cptr, d_vptr};
    return launch_sample(sh, max_cdeg, max_vdeg, seed, first_graph, G, check_var, var_slot, attempts, max_attempts,
                         ctl, stream);
}

}  // namespace ldpc
