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

// Graphs with kSeqMinE (8192) <= n*dv <= kSeqMaxE: sequential-draw sampler, one wave per
// graph.  The same law -- a uniform socket permutation conditioned on every check
// being simple -- drawn slot by slot, so a bad check is seen as soon as its last
// slot is drawn and the attempt stops there (a failing (3,6) attempt at n = 64,800
// stops after ~1/5 of the graph instead of paying a whole permutation):
//   * slot x (in order) takes a uniform unused entry of the pool: its words --
//     word j = word x&3 of Philox ctr {x>>2 | j<<20, tag|att<<2|3, g_lo, g_hi} --
//     give Lemire draws on [0, R) until one lands on an unused pool index (a
//     bitmap in LDS); 1024 words without one reject the attempt (probability
//     < (3/4)^1000);
//   * the pool starts as all R = E sockets; when R' = ceil(R/4) entries are left
//     the unused ones are compacted in order into a new pool (global scratch,
//     the variable_lookup row) with a fresh bitmap, so no draw ever sees more
//     than 3/4 of its pool used; the last <= kSeqFinal entries are
//     Fisher-Yates-shuffled by one lane (stream {blk, tag|1<<30|att<<2|3, g});
//   * up to 256 consecutive slots are drawn per round, the four of block x>>2 by
//     one lane (one Philox block per lane per word index), against the bitmap of
//     the slots before the round; LDS atomic ORs mark the picks, and when two
//     slots picked the same entry the round keeps only the slots below the
//     second-lowest slot of every such group (the later slots redraw next round
//     from the updated bitmap -- a slot's result is its first draw not used by an
//     earlier slot, exactly the sequential process);
//   * every check whose slots are all drawn is tested (variable ids kept in an
//     LDS ring of the last kSeqRing slots); a repeat redraws from slot 0 (att+1).
// ~25.6 KB of LDS per wave at n = 64,800 (the bitmap), so six graphs per CU.
// The variable side is built with per-variable occurrence counters packed fb bits
// per variable into the bitmap's LDS (fb = 0: global CAS, sample_emit_var_side).
// oracle_sample_regular / oracle_sample_csr restate it bit for bit.
constexpr int kSeqFinal = 64, kSeqRing = 1024;  // ring: a round (<= 512 slots) + the check it completes
#ifndef LDPC_SEQ_FIRST_WORDS
#define LDPC_SEQ_FIRST_WORDS 3  // words every slot draws up front (then only ~f^3 of the slots retry)
#endif
constexpr int kSeqFirstWords = LDPC_SEQ_FIRST_WORDS;
#ifndef LDPC_SEQ_WIDE_R
#define LDPC_SEQ_WIDE_R 0  // > 0: pools of at least this many entries draw 512 slots per round
#endif                     // (measured slower at n = 64,800: more registers, costlier collisions)
constexpr int kSeqWideR = LDPC_SEQ_WIDE_R;
#ifndef LDPC_SEQ_VKEYS
#define LDPC_SEQ_VKEYS 1  // the attempt's Philox key schedule in VGPRs (PhiloxKeys)
#endif

// LDS ordering between the lanes of one wave (LDS instructions of a wave execute in order):
// a compiler barrier only -- no s_barrier, no wait for the outstanding global stores that a
// workgroup-scope fence (__syncthreads) would add to every round
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
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

// Shared state of one wave's sequential-draw attempts (LDS pointers, graph id, key).
struct SeqCtx {
    SampleShape sh;
    uint32_t k0, k1, g0, g1;
    uint32_t mdv;   // regular: socket / dv as a multiply-high by ceil(2^32 / dv) (0: divide)
    uint32_t *bm;   // [bw] pool bitmap
    void *ring;     // [kSeqRing] variable of slot x at x % kSeqRing (u16 when n <= 65536, else int)
    int *fin;       // [kSeqFinal] last pool entries
    int *tl;        // [2 * kWave] retry task list (second half: writes of lanes without a task)
};

template <bool CSR>
__device__ __forceinline__ int seq_var_of(const SeqCtx &c, int s) {
    return CSR ? c.sh.vsock[s] : (c.mdv ? (int)__umulhi((uint32_t)s, c.mdv) : s / c.sh.dv);
}

__device__ __forceinline__ void seq_clear_bm(uint32_t *bm, int words) {
    uint4 *b4 = reinterpret_cast<uint4 *>(bm);
    for (int w = (int)(threadIdx.x & 63); w < (words + 3) >> 2; w += kWave) b4[w] = make_uint4(0u, 0u, 0u, 0u);
    wave_sync();
}

constexpr uint32_t kSeqNone = 0xFFFFFFFFu;  // search: no simple attempt found (yet)

// Diagnostics build only (-DLDPC_SEQ_STATS=1, scripts/build_variants.sh): the search pass
// accumulates per-launch counts and s_memtime cycles by phase into g_seq_stats
// (ldpc_debug_seq_stats); the product build compiles every SEQ_STAT to nothing.
#ifndef LDPC_SEQ_STATS
#define LDPC_SEQ_STATS 0
#endif
enum SeqStat {
    kStAttempts, kStAborted, kStRounds, kStKept, kStLaneIters, kStSpreadIters, kStCollRounds, kStProbes,
    kStCycAttempt, kStCycDraw, kStCycRetry, kStCycMark, kStCycRingVal, kStCycCompact, kStCycClaim, kStValFail,
    kStCount
};
__device__ unsigned long long g_seq_stats[2 * kStCount];  // search pass, then emit pass
struct SeqStats {
    unsigned long long v[kStCount];
    uint64_t t;  // last time stamp
    __device__ void zero() {
        for (int i = 0; i < kStCount; ++i) v[i] = 0;
        t = __builtin_amdgcn_s_memtime();
    }
    __device__ void lap(int i) {  // cycles since the last stamp into v[i]
        const uint64_t now = __builtin_amdgcn_s_memtime();
        v[i] += now - t;
        t = now;
    }
    __device__ void flush(int pass = 0) {
        if ((threadIdx.x & 63) == 0)
            for (int i = 0; i < kStCount; ++i)
                if (v[i]) atomicAdd(&g_seq_stats[pass * kStCount + i], v[i]);
    }
};
#if LDPC_SEQ_STATS
#define SEQ_STAT(st, expr) \
    do {                   \
        if (st) { expr; }  \
    } while (0)
#else
#define SEQ_STAT(st, expr) \
    do {                   \
    } while (0)
#endif

// Attempt `att` of the sequential draw (one wave).  EMIT: every slot's variable also goes to
// out[x] (the emit pass); otherwise only the verdict matters (the search pass).  pools: >= E
// ints of global scratch (the stage pools, two halves used alternately).  best != nullptr
// (search): the attempt is abandoned once *best (the lowest simple attempt found by any
// wave) is below att -- it can no longer be the graph's first simple attempt.
// Returns true when the attempt drew a simple graph.
template <bool CSR, bool EMIT, typename RT>
__device__ __forceinline__ bool seq_attempt(const SeqCtx &c, int att, int32_t *out, int32_t *pools,
                                            const uint32_t *best, SeqStats *st = nullptr) {
    const int lane = threadIdx.x & 63;
    const int E = c.sh.E, m = c.sh.m, dc = c.sh.dc;
    const uint32_t k0 = c.k0, k1 = c.k1, g0 = c.g0, g1 = c.g1;
#if LDPC_SEQ_VKEYS
    const PhiloxKeys K = philox_keys(k0, k1);  // the round loop's Philox keys in VGPRs
#define LDPC_SEQ_KEYS K
#else
#define LDPC_SEQ_KEYS k0, k1
#endif
    uint32_t *const bm = c.bm;
    RT *const ring = reinterpret_cast<RT *>(c.ring);
    int *const tl = c.tl;
    const uint32_t c1 = kSampleTag | ((uint32_t)att << 2) | 3u;
    int R = E, x0 = 0, cdone = 0, nround = 0;
    uint32_t bseen = kSeqNone;  // search: *best as last loaded
    bool bad = false;
    // checks whose slots all lie below `upto`, from cdone on: any repeated variable?
    auto validate = [&](int upto) -> bool {
        int cend = cdone;
        if constexpr (CSR) {
            for (;;) {
                const int cc = cend + lane;
                const uint64_t f = __ballot(cc < m && c.sh.cptr[cc + 1] <= upto);  // a prefix of the lanes
                cend += __popcll(f);
                if (f != ~0ull) break;
            }
        } else {
            cend = __builtin_amdgcn_readfirstlane(upto / dc);
        }
        bool b = false;
        for (int cb = cdone; cb < cend; cb += kWave) {
            const int cc = cb + lane;
            if (cc < cend) {
                const int lo = CSR ? c.sh.cptr[cc] : cc * dc, d = CSR ? c.sh.cptr[cc + 1] - lo : dc;
                if (!CSR && d == 6) {  // (3,6): slots in aligned pairs (lo even: no pair straddles the ring's end)
                    uint32_t v[6];
#pragma unroll
                    for (int u = 0; u < 6; u += 2) {
                        const int p = (lo + u) & (kSeqRing - 1);
                        if constexpr (sizeof(RT) == 2) {
                            const uint32_t w = *reinterpret_cast<const uint32_t *>(ring + p);
                            v[u] = w & 0xFFFFu;
                            v[u + 1] = w >> 16;
                        } else {
                            const int2 w = *reinterpret_cast<const int2 *>(ring + p);
                            v[u] = (uint32_t)w.x;
                            v[u + 1] = (uint32_t)w.y;
                        }
                    }
                    uint32_t mn = 0xFFFFFFFFu;  // zero iff two slots hold the same variable
#pragma unroll
                    for (int u = 0; u < 6; ++u)
#pragma unroll
                        for (int w = u + 1; w < 6; ++w) mn = min(mn, v[u] ^ v[w]);
                    b |= mn == 0u;
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
        cdone = cend;
        return __ballot(b) == 0ull;
    };

    // the rounds of one stage (slots x0 .. xend - 1); POOL: the pool is the global row at
    // pools + cur (stage 0: the sockets themselves -- the regular form has no global load in
    // its rounds, so no round waits on earlier stores).  NB: Philox blocks per lane per word
    // index, i.e. up to 256 NB consecutive slots per round -- lane L draws the four slots of
    // block x0/4 + L + 64 b (b < NB), relative slot 256 b + 4 L + q.
    auto rounds = [&](auto pool_tag, auto nb_tag, int xend, int cur) {
        constexpr bool POOL = decltype(pool_tag)::value;
        constexpr int NB = decltype(nb_tag)::value;
        constexpr int NS = 4 * NB;  // slots per lane
        const int32_t *pool = pools + cur;
        const uint32_t lt = (0u - (uint32_t)R) % (uint32_t)R;  // Lemire: reject low words below this
        // entry of word w, or -1 when Lemire's test or the bitmap rejects it
        auto try_word = [&](uint32_t w) -> int {
            const uint64_t mm = (uint64_t)w * (uint32_t)R;
            const int e = (int)(mm >> 32);
            const bool used = (bm[e >> 5] >> (e & 31)) & 1u;
            return ((uint32_t)mm < lt || used) ? -1 : e;
        };
        auto rel = [&](int k, int l) { return 256 * (k >> 2) + 4 * l + (k & 3); };  // slot k of lane l
        // The first words of every slot of the round at base bs: the NB x kSeqFirstWords Philox
        // blocks of the lane, computed round-interleaved (philox_blocks: their ten-step product
        // chains overlap).  (Computing the next round's blocks in this round's atomics' latency
        // measured slower: the search pass is issue-bound; scripts/ablations/README.md.)
        uint4 Wn[NB * kSeqFirstWords];
        auto first_words = [&](int bs) {
            uint32_t cc[NB * kSeqFirstWords];
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int j = 0; j < kSeqFirstWords; ++j)
                    cc[b * kSeqFirstWords + j] = ((uint32_t)(bs >> 2) + (uint32_t)(lane + 64 * b)) | ((uint32_t)j << 20);
            philox_blocks<NB * kSeqFirstWords>(cc, c1, g0, g1, LDPC_SEQ_KEYS, Wn);
        };
        while (x0 < xend) {
            if (best && (++nround & 15) == 0) {  // search: a lower simple attempt makes this one moot
                // (the value loaded 16 rounds ago: the load's latency never stalls a round)
                if (__builtin_amdgcn_readfirstlane(bseen) < (uint32_t)att) {
                    SEQ_STAT(st, st->v[kStAborted]++);
                    bad = true;
                    return;
                }
                bseen = __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            SEQ_STAT(st, st->v[kStRounds]++; st->lap(kStCycRingVal));
            // Word j of slot x is word x&3 of Philox {x>>2 | j<<20, c1, g}.  A slot takes its
            // first word that passes Lemire's test and whose entry is unused (bitmap of the
            // slots before the round).  Every slot first tries words 0 .. kSeqFirstWords-1 at
            // once (independent Philox blocks: instruction-level parallelism for a wave that is
            // mostly waiting, and one LDS round trip for their bitmap reads).  Retries: while
            // many slots still look, every lane draws the next block of its own slots; once at
            // most 32 do, the wave spreads them -- L = 2..16 lanes per slot, each trying one of
            // the slot's next L words, the lowest passing word wins (a slot's words are tried in
            // order, so the result is the same).
            const int base = x0 & ~3;
            uint32_t bb[NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) bb[b] = (uint32_t)(base >> 2) + (uint32_t)(lane + 64 * b);
            first_words(base);
            int i[NS];
            bool act[NS], need[NS];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int k = 4 * b + q, x = base + rel(k, lane);
                    act[k] = x >= x0 && x < xend;
                    int e[kSeqFirstWords];
#pragma unroll
                    for (int j = 0; j < kSeqFirstWords; ++j) e[j] = try_word(pick4(Wn[b * kSeqFirstWords + j], q));
                    i[k] = e[kSeqFirstWords - 1];
#pragma unroll
                    for (int j = kSeqFirstWords - 2; j >= 0; --j) i[k] = e[j] >= 0 ? e[j] : i[k];
                    need[k] = act[k] && i[k] < 0;
                }
            }
            // later stages: the pool entries of the first draws are loaded now, so the global
            // load's latency overlaps the retries and the marking (a retried slot reloads)
            int pre[NS];
            if constexpr (POOL) {
#pragma unroll
                for (int k = 0; k < NS; ++k) pre[k] = pool[max(i[k], 0)];
            }
            SEQ_STAT(st, st->lap(kStCycDraw));
            bool firstok[NS];  // the slot kept its first draw (no retry): pre[k] is its value
#pragma unroll
            for (int k = 0; k < NS; ++k) firstok[k] = !need[k];
            uint32_t j0 = kSeqFirstWords;  // next word index of every slot still looking
            for (;;) {
                uint64_t mq[NS];
                int C = 0;
#pragma unroll
                for (int k = 0; k < NS; ++k) {
                    mq[k] = __ballot(need[k]);
                    C += __popcll(mq[k]);
                }
                if (C == 0) break;
                if (j0 >= 1024u) { bad = true; return; }  // a slot rejected 1024 words: reject the attempt
                if (C > 32) {  // per lane: the next block of the lane's own slots
                    SEQ_STAT(st, st->v[kStLaneIters]++);
#pragma unroll
                    for (int b = 0; b < NB; ++b) {
                        const uint4 W = philox_block(bb[b] | (j0 << 20), c1, g0, g1, LDPC_SEQ_KEYS);
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int k = 4 * b + q;
                            const int e = try_word(pick4(W, q));
                            i[k] = need[k] ? e : i[k];
                            need[k] = need[k] && e < 0;
                        }
                    }
                    ++j0;
                    continue;
                }
                SEQ_STAT(st, st->v[kStSpreadIters]++);
                // spread: slot p (k-major order) gets lanes [p*L, p*L + L), lane p*L + k' tries
                // word j0 + k'
                const int lg1 = C <= 4 ? 4 : (C <= 8 ? 3 : (C <= 16 ? 2 : 1));  // L * C <= 64
                const int L = 1 << lg1;
                const uint32_t lmask = (uint32_t)((1ull << L) - 1ull);
                int pos[NS];
                int pre = 0;
#pragma unroll
                for (int k = 0; k < NS; ++k) {
                    const uint32_t below =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(mq[k] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mq[k], 0u));
                    pos[k] = pre + (int)below;
                    pre += __popcll(mq[k]);
                    tl[need[k] ? pos[k] : kWave + lane] = lane | (k << 6);
                }
                wave_sync();
                const int p = lane >> lg1, kl = lane & (L - 1);
                const int ent = tl[p < C ? p : 0];
                const int own = ent & 63, kk = ent >> 6;
                const uint32_t jj = j0 + (uint32_t)kl;
                const uint32_t ob = (uint32_t)(base >> 2) + (uint32_t)(own + 64 * (kk >> 2));
                const uint4 W = philox_block(ob | (jj << 20), c1, g0, g1, LDPC_SEQ_KEYS);
                const int eh = (p < C && jj < 1024u) ? try_word(pick4(W, kk & 3)) : -1;
                const uint64_t okm = __ballot(eh >= 0);
#pragma unroll
                for (int k = 0; k < NS; ++k) {
                    const int s0 = need[k] ? pos[k] << lg1 : 0;
                    const uint32_t seg = (uint32_t)(okm >> s0) & lmask;
                    const int src = seg ? s0 + (int)__builtin_ctz(seg) : lane;
                    const int got = __shfl(eh, src, kWave);
                    const bool hit = need[k] && seg != 0u;
                    i[k] = hit ? got : i[k];
                    need[k] = need[k] && seg == 0u;
                }
                j0 += (uint32_t)L;
                wave_sync();  // tl is rewritten by the next spread
            }
            SEQ_STAT(st, st->lap(kStCycRetry));
            int val[NS];
            bool dup[NS];
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                val[k] = 0;
                if (act[k]) {
                    if constexpr (POOL) val[k] = firstok[k] ? pre[k] : pool[i[k]];
                    else val[k] = seq_var_of<CSR>(c, i[k]);
                }
            }
            bool anyd = false;
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                const uint32_t bit = 1u << (i[k] & 31);
                dup[k] = act[k] && (atomicOr(&bm[i[k] >> 5], bit) & bit) != 0u;
                anyd |= dup[k];
            }
            int t = min(256 * NB, xend - base);  // kept: slots base + [x0 - base, t)
            if (__ballot(anyd)) {
                SEQ_STAT(st, st->v[kStCollRounds]++);
                // keep the slots below the second-lowest slot of every group of equal picks (the
                // first invalid slot of the group; which slot saw the bit set depends on the
                // atomic order, so each group is found from its members' picks)
                uint64_t dm[NS];
#pragma unroll
                for (int k = 0; k < NS; ++k) dm[k] = __ballot(dup[k]);
#pragma unroll
                for (int k = 0; k < NS; ++k) {
                    while (dm[k]) {
                        const int ip = __shfl(i[k], (int)__builtin_ctzll(dm[k]), kWave);
                        int lo1 = 1 << 30, lo2 = 1 << 30;  // the group's two lowest slots
#pragma unroll
                        for (int r = 0; r < NS; ++r) {
                            const uint64_t g = __ballot(act[r] && i[r] == ip);
                            dm[r] &= ~g;
                            if (g) {
                                const int s1 = rel(r, (int)__builtin_ctzll(g));
                                const uint64_t g2 = g & (g - 1);
                                const int s2 = g2 ? rel(r, (int)__builtin_ctzll(g2)) : 1 << 30;
                                if (s1 < lo1) { lo2 = min(lo1, s2); lo1 = s1; }
                                else lo2 = min(lo2, s1);
                            }
                        }
                        t = __builtin_amdgcn_readfirstlane(min(t, lo2));
                    }
                }
#pragma unroll
                for (int k = 0; k < NS; ++k)  // undo every pick of the round ...
                    if (act[k] && !dup[k]) atomicAnd(&bm[i[k] >> 5], ~(1u << (i[k] & 31)));
#pragma unroll
                for (int k = 0; k < NS; ++k)  // ... and redo the kept ones
                    if (act[k] && rel(k, lane) < t) atomicOr(&bm[i[k] >> 5], 1u << (i[k] & 31));
            }
            SEQ_STAT(st, st->lap(kStCycMark));
            // ring: each block's four slots in one store (base is a multiple of 4); slots below
            // x0 keep their values, slots at or above t are redrawn (and rewritten) before any
            // check that holds them is tested
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const int p = (base + 256 * b + 4 * lane) & (kSeqRing - 1);
                int nv[4] = {val[4 * b], val[4 * b + 1], val[4 * b + 2], val[4 * b + 3]};
                if (b == 0 && (x0 & 3)) {  // the first block has slots below x0 (lane 0): keep their values
#pragma unroll
                    for (int q = 0; q < 4; ++q) nv[q] = act[q] ? nv[q] : (int)ring[p + q];
                }
                if constexpr (sizeof(RT) == 2)
                    *reinterpret_cast<uint2 *>(ring + p) =
                        make_uint2((uint32_t)nv[0] | ((uint32_t)nv[1] << 16), (uint32_t)nv[2] | ((uint32_t)nv[3] << 16));
                else
                    *reinterpret_cast<int4 *>(ring + p) = make_int4(nv[0], nv[1], nv[2], nv[3]);
            }
            if (EMIT && out) {
#pragma unroll
                for (int k = 0; k < NS; ++k) {
                    const int s = rel(k, lane);
                    if (act[k] && s < t) out[base + s] = val[k];
                }
            }
            SEQ_STAT(st, st->v[kStKept] += (unsigned long long)(base + t - x0));
            x0 = __builtin_amdgcn_readfirstlane(base + t);  // uniform: scalar loop control
            wave_sync();
            if (!validate(x0)) {
                SEQ_STAT(st, st->v[kStValFail]++);
                bad = true;
                return;
            }
        }
    };
    // compact the unused entries of the stage's pool (R entries), in order, into dst
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
    int cur = -1;  // offset of the current pool in `pools` (-1: stage 0, the sockets)
    while (R > kSeqFinal && !bad) {
        const int Rn = (R + 3) >> 2, xend = E - Rn;
        // wide rounds (two blocks per lane) while the pool is large: the birthday bound lets
        // ~400 of 512 slots through a round at R ~ 2e5, ~240 of 256 with one block
        if (kSeqWideR > 0 && R >= kSeqWideR) {
            if (cur < 0) rounds(bool_c<false>{}, int_c<2>{}, xend, 0);
            else rounds(bool_c<true>{}, int_c<2>{}, xend, cur);
        } else {
            if (cur < 0) rounds(bool_c<false>{}, int_c<1>{}, xend, 0);
            else rounds(bool_c<true>{}, int_c<1>{}, xend, cur);
        }
        if (bad) break;
        SEQ_STAT(st, st->lap(kStCycRingVal));
        if (Rn <= kSeqFinal) {  // the last entries go to LDS
            if (cur < 0) compact(bool_c<false>{}, 0, c.fin);
            else compact(bool_c<true>{}, cur, c.fin);
        } else {  // the next pool: pools[0 ..) and pools[E/2 ..) alternately (R' <= E/4 + 1)
            const int nx = cur == 0 ? E / 2 : 0;
            if (cur < 0) compact(bool_c<false>{}, 0, pools + nx);
            else compact(bool_c<true>{}, cur, pools + nx);
            cur = nx;
        }
        __threadfence_block();
        __syncthreads();
        R = Rn;
        seq_clear_bm(bm, (R + 31) >> 5);
        SEQ_STAT(st, st->lap(kStCycCompact));
    }
    if (bad) return false;
    // last R <= kSeqFinal entries (in fin): Fisher-Yates by lane 0, then the last slots
    int *const fin = c.fin;
    if (R == E && lane < E) fin[lane] = seq_var_of<CSR>(c, lane);  // tiny graphs: no compaction ran
    wave_sync();
    if (lane == 0) {
        BucketRng rng{k0, k1, 0u, c1 | (1u << 30), g0, g1};
        for (int a = R - 1; a >= 1; --a) {
            const int j = (int)rng.below((uint32_t)a + 1u);
            const int tmp = fin[a];
            fin[a] = fin[j];
            fin[j] = tmp;
        }
    }
    wave_sync();
    if (lane < R) {
        const int x = x0 + lane;
        if (EMIT && out) out[x] = fin[lane];
        ring[x & (kSeqRing - 1)] = (RT)fin[lane];
    }
    wave_sync();
    return validate(E);
}
#undef LDPC_SEQ_KEYS

// Emit pass (and the whole sampler when start == nullptr): one wave per graph draws attempts
// start[g], start[g] + 1, ... in order until one is simple (start[g] = the first simple attempt
// found by sample_search_kernel, so normally exactly one attempt), writes its slots to
// check_lookup[g], then builds the variable side.  attempts[g] = attempts drawn from 0
// (negative: max_attempts without a simple graph -- then the identity configuration).
// LDS of a sequential-draw wave: bitmap [bw] | fin [kSeqFinal] | tl [2 kWave] | ring [kSeqRing] RT
template <typename RT>
__host__ __device__ constexpr size_t seq_lds_bytes(int bw) {
    return (size_t)4 * (bw + kSeqFinal + 2 * kWave) + sizeof(RT) * kSeqRing;
}

template <bool CSR, typename RT>  // CSR: irregular degree structure (sh.vsock / cptr / vptr); RT: ring entries
__global__ __launch_bounds__(kWave) void sample_seq_kernel(SampleShape sh, uint32_t k0, uint32_t k1,
                                                           uint64_t first_graph, int32_t *check_lookup,
                                                           int32_t *variable_lookup, int32_t *attempts,
                                                           int max_attempts, int bw, int fb, uint32_t mdv,
                                                           const uint32_t *start, const uint32_t *homewin) {
    extern __shared__ __align__(16) unsigned char smem[];
    uint32_t *bm = reinterpret_cast<uint32_t *>(smem);  // [bw] pool bitmap, later rank counters
    int *fin = reinterpret_cast<int *>(bm + bw);        // [kSeqFinal]
    int *tl = fin + kSeqFinal;                          // [2 * kWave]
    RT *ring = reinterpret_cast<RT *>(tl + 2 * kWave);  // [kSeqRing]
    const int n = sh.n, E = sh.E, dv = sh.dv, dc = sh.dc;
    constexpr bool csr = CSR;
    const int lane = threadIdx.x;
    const uint64_t gid = first_graph + blockIdx.x;
    const SeqCtx c{sh, k0, k1, (uint32_t)gid, (uint32_t)(gid >> 32), mdv, bm, ring, fin, tl};
    int32_t *out = check_lookup + (size_t)blockIdx.x * E;
    int32_t *vl = variable_lookup + (size_t)blockIdx.x * E;

    int att = start ? (int)min(start[blockIdx.x], (uint32_t)max_attempts) : 0;
    bool ok = false;
    if (homewin && att < max_attempts && homewin[blockIdx.x] == (uint32_t)att) {
        ok = true;  // the search's home wave drew this attempt into check_lookup[g] already
        ++att;
    }
    while (!ok && att < max_attempts) {
#if LDPC_SEQ_STATS
        SeqStats stats;
        stats.zero();
        const uint64_t t_att = __builtin_amdgcn_s_memtime();
        ok = seq_attempt<CSR, true, RT>(c, att, out, vl, nullptr, &stats);
        stats.lap(kStCycRingVal);
        stats.v[kStAttempts]++;
        stats.v[kStCycAttempt] += __builtin_amdgcn_s_memtime() - t_att;
        stats.flush(1);
#else
        ok = seq_attempt<CSR, true, RT>(c, att, out, vl, nullptr);
#endif
        ++att;
    }
    if (attempts && lane == 0) attempts[blockIdx.x] = ok ? att : -att;
    if (!ok)  // max_attempts without a simple graph: the identity configuration (in-range ids)
        for (int x = lane; x < E; x += kWave) out[x] = seq_var_of<CSR>(c, x);
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
    const uint32_t fmask = (1u << fb) - 1u;
    for (int xb = 0; xb < E; xb += kWave) {
        const int x = xb + lane;
        if (x < E) {
            const int v = out[x];
            const uint32_t pos = (uint32_t)v * (uint32_t)fb;
            const uint32_t old = atomicAdd(&bm[pos >> 5], 1u << (pos & 31));
            const int rank = (int)((old >> (pos & 31)) & fmask);
            if (csr) vl[sh.vptr[v] + rank] = x;
            else vl[(size_t)v * dv + rank] = x / dc;
        }
    }
    __threadfence_block();
    __syncthreads();
    for (int v = lane; v < n; v += kWave) {
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
// sequential sampler would return -- with the attempts of a graph spread over waves.
// Persistent single-wave workgroups; ctl (global): [0] next graph to open, [1] unused,
// best[G] (kSeqNone: none yet), natt[G] (next attempt index to claim), homewin[G] (the simple
// attempt the graph's home wave drew into check_lookup[g], kSeqNone: none).  A wave claims attempts of its home graph until the
// graph has a simple attempt (then opens the next graph); when every graph is open it helps:
// it probes for a graph still without one and claims that graph's attempts until it has one.  Every attempt below a graph's
// final best is claimed and runs to completion (an attempt is abandoned only once best is
// below it), so best = the lowest simple attempt, exactly the sequential result, for any
// schedule.  Attempts >= max_attempts are never drawn (best stays kSeqNone).  Pool rows (E
// ints per wave): variable_lookup rows (grid <= G), rebuilt by the variable-side pass.  The
// wave that opens a graph draws its attempts into check_lookup[g] and records a simple one in
// homewin[g]; the emit pass skips g when homewin[g] == best[g] and redraws attempt best otherwise.
template <bool CSR, typename RT>
__global__ __launch_bounds__(kWave) void sample_search_kernel(SampleShape sh, uint32_t k0, uint32_t k1,
                                                              uint64_t first_graph, int G, int32_t *scratch_a,
                                                              int32_t *scratch_b, uint32_t *ctl, int max_attempts,
                                                              int bw, uint32_t mdv) {
    extern __shared__ __align__(16) unsigned char smem[];
    uint32_t *bm = reinterpret_cast<uint32_t *>(smem);
    int *fin = reinterpret_cast<int *>(bm + bw);
    int *tl = fin + kSeqFinal;
    RT *ring = reinterpret_cast<RT *>(tl + 2 * kWave);
    const int lane = threadIdx.x;
    uint32_t *best = ctl + 2, *natt = ctl + 2 + G, *homewin = ctl + 2 + 2 * G;
    int32_t *pools = scratch_b + (size_t)blockIdx.x * sh.E;  // grid <= G: variable_lookup row w
    const uint32_t um = (uint32_t)max_attempts;
    int home = -1;         // the graph whose attempts this wave claims
    bool helping = false;  // every graph is open: homes are picked among the open ones
    uint32_t probe = (uint32_t)blockIdx.x * 0x9E3779B9u + 0x7F4A7C15u;
    for (;;) {
        // claim (graph, attempt) on the home graph (lane 0)
        const uint64_t t_claim = LDPC_SEQ_STATS ? __builtin_amdgcn_s_memtime() : 0;
        int g = -1, att = 0;
        if (lane == 0) {
            for (;;) {
                if (home < 0 && !helping) {
                    home = (int)atomicAdd(&ctl[0], 1u);
                    if (home >= G) { home = -1; helping = true; }
                }
                if (home < 0) break;  // helping without a home: probe below
                if (__hip_atomic_load(&best[home], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kSeqNone) {
                    const uint32_t a = atomicAdd(&natt[home], 1u);
                    if (a < um) { g = home; att = (int)a; break; }
                }
                home = -1;  // resolved or out of attempts
            }
        }
        // lane 0's claim, as wave-uniform (scalar) values
        g = __builtin_amdgcn_readfirstlane(g);
        att = __builtin_amdgcn_readfirstlane(att);
        helping = __builtin_amdgcn_readfirstlane((int)helping) != 0;
        if (g < 0) {
            // help: probe the graphs from a pseudo-random start (wrapping) for one without a
            // simple attempt and with attempts left -- 256 graphs per step, their loads issued
            // together -- and make it the home; none anywhere: this wave is done
            probe = probe * 1664525u + 1013904223u;
            const uint32_t start = (uint32_t)(((uint64_t)probe * (uint32_t)G) >> 32);
            int found = -1;
            for (uint32_t k = 0; k < (uint32_t)G && found < 0; k += 4 * kWave) {
                bool open[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t off = k + (uint32_t)(u * kWave + lane);
                    uint32_t cg = start + off;
                    if (cg >= (uint32_t)G) cg -= (uint32_t)G;
                    open[u] = off < (uint32_t)G &&
                              __hip_atomic_load(&best[cg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kSeqNone &&
                              __hip_atomic_load(&natt[cg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < um;
                }
#pragma unroll
                for (int u = 0; u < 4 && found < 0; ++u) {
                    const uint64_t f = __ballot(open[u]);
                    if (f) {
                        uint32_t cg = start + k + (uint32_t)(u * kWave) + (uint32_t)__builtin_ctzll(f);
                        if (cg >= (uint32_t)G) cg -= (uint32_t)G;
                        found = (int)cg;
                    }
                }
            }
            if (found < 0) break;  // nothing left to claim anywhere
            home = found;
#if LDPC_SEQ_STATS
            if (lane == 0) atomicAdd(&g_seq_stats[kStProbes], 1ull);
#endif
            continue;
        }
#if LDPC_SEQ_STATS
        if (lane == 0) atomicAdd(&g_seq_stats[kStCycClaim], __builtin_amdgcn_s_memtime() - t_claim);
#else
        (void)t_claim;
#endif
        const uint64_t gid = first_graph + (uint64_t)g;
        const SeqCtx c{sh, k0, k1, (uint32_t)gid, (uint32_t)(gid >> 32), mdv, bm, ring, fin, tl};
#if LDPC_SEQ_STATS
        SeqStats stats;
        stats.zero();
        SeqStats *stp = &stats;
#else
        SeqStats *stp = nullptr;
#endif
        const uint64_t t_att = LDPC_SEQ_STATS ? __builtin_amdgcn_s_memtime() : 0;
        (void)t_att;
        // the wave that opened graph g is the only one writing its check_lookup row: its attempts
        // draw into it (a simple one is then the graph itself unless a helper's lower attempt wins
        // -- the emit pass redraws exactly those graphs); helpers only search
        const bool solo = !helping;
        // one instantiation for both roles (out == nullptr: search only): half the code, and a
        // simpler control-flow graph for the round loop
        const bool ok = seq_attempt<CSR, true, RT>(c, att, solo ? scratch_a + (size_t)g * sh.E : nullptr, pools,
                                                   &best[g], stp);
        SEQ_STAT(stp, stp->lap(kStCycRingVal); stp->v[kStAttempts]++;
                 stp->v[kStCycAttempt] += __builtin_amdgcn_s_memtime() - t_att; stp->flush());
        if (ok && lane == 0) {
            atomicMin(&best[g], (uint32_t)att);
            if (solo) homewin[g] = (uint32_t)att;
        }
        __threadfence_block();
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
            // search pass: persistent single-wave workgroups, as many as fit the device (LDS
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
            // graphs' home waves draw into check_lookup; pool rows: wave w uses variable_lookup row w
            hipLaunchKernelGGL(sk, dim3(W), dim3(kWave), lds, stream, sh, k0, k1, first_graph, G, check_lookup,
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
        hipLaunchKernelGGL(kern, dim3(G), dim3(kWave), lds, stream, sh, k0, k1, first_graph,
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
