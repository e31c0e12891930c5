// Ensemble BEC Monte-Carlo decode by frontier peeling (gfx950): the decoder of
// message_passing.c:7-82 for the all-zero codeword of parallel_simulator.py:222, one
// workgroup per trial, each trial on its own device-sampled graph (configs[4]).
//
// With every known bit 0, iteration i of message_passing resolves exactly the erased
// variables v that some check c holds as its only erased slot at the start of i (the check
// message to v is known iff no OTHER slot of c is erased, :28-44; a variable listed twice in
// c never qualifies), and the known value is 0.  So the decode needs, per check, the number
// of erased slots and -- when that number is 1 -- which variable it is.  One u32 per check
// in LDS holds count << 24 | (sum of the erased slots' variable ids): when the count is 1 the
// sum is the variable, and resolving v subtracts (1 << 24) + v from each of v's checks (once
// per edge, so multi-edges stay exact) in ONE atomic.  Iteration i processes only its
// frontier -- the checks whose count was 1 at its start -- and a decrement that takes a count
// from 2 to 1 files that check for iteration i + 1; the per-iteration erasure counts, the stall
// rule (:16-19) and the zero-count break (:76-78) are the reference's, so trial[b][*] and
// its[b] equal bec_kernel's (and the oracle's) exactly.  Work per trial: one pass over the
// check side (E coalesced reads) plus dv reads per resolved variable, instead of E gathers per
// iteration.  A frontier list that overflows its LDS capacity marks the next iteration for a
// full scan (a frontier bitmap snapshot first, so no check is processed in the iteration its
// count reached 1).
#include "device_common.hpp"
#include "ldpc_internal.hpp"

#include <atomic>

namespace ldpc {
namespace {

// Scan-path evidence, always on (a few atomics per trial at most): [0] iterations that ran
// the bitmap-snapshot scan because the frontier list overflowed, [1] trials with at least one
// such iteration, [2] trials decoded (ldpc_debug_peel_stats).
__device__ unsigned long long g_peel_stats[3];

// Test-only frontier capacity override (ldpc_debug_peel_cap); 0 = the LDS budget's capacity.
std::atomic<int> g_peel_cap{0};

struct PeelArgs {
    const int32_t *cvar, *vchk;  // graph b at + b * graph_stride: check-major slots, v's checks
    int64_t graph_stride;
    int n, m, dv, dc, max_iters, F;  // F: capacity of each frontier list (u16 entries)
    ChanArgs ch;
    uint64_t first_cw;
    int32_t *trial, *its;  // [B][max_iters + 1], [B]
};

template <int T>
__global__ __launch_bounds__(T) void bec_peel_kernel(PeelArgs a) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int red[T / kWave];
    __shared__ int ctl[4];  // list lengths [2], overflow flags [2]
    const int tid = threadIdx.x;
    const size_t b = blockIdx.x;
    const int n = a.n, m = a.m, dv = a.dv, dc = a.dc, iters = a.max_iters, F = a.F;
    const int vw = (n + 31) >> 5, fw = (m + 31) >> 5;
    uint32_t *st = reinterpret_cast<uint32_t *>(smem);  // [m] count << 24 | sum of erased ids
    uint32_t *vf = st + m;                              // [vw] erased variables
    uint32_t *fb = vf + vw;                             // [fw] frontier snapshot (scan mode)
    uint16_t *fl = reinterpret_cast<uint16_t *>(fb + fw);  // [2][F] frontier lists
    const int32_t *cvar = a.cvar + b * (size_t)a.graph_stride;
    const int32_t *vchk = a.vchk + b * (size_t)a.graph_stride;
    int32_t *tr = a.trial + b * (size_t)(iters + 1);
    const uint64_t cw = a.first_cw + b;

    for (int w = tid; w < vw; w += T) vf[w] = 0u;
    for (int w = tid; w < fw; w += T) fb[w] = 0u;
    if (tid < 4) ctl[tid] = 0;
    __syncthreads();
    // channel: chan_bec's stream, one Philox block per lane per four variables
    int cnt = 0;
    for (int g4 = tid; g4 < (n + 3) >> 2; g4 += T) {
        const uint4 r = philox_block((uint32_t)g4, 0u, (uint32_t)cw, (uint32_t)(cw >> 32), a.ch.k0, a.ch.k1);
        uint32_t nib = 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * g4 + q < n && u01(pick4(r, q)) < a.ch.p) nib |= 1u << q;
        if (nib) {
            atomicOr(&vf[g4 >> 3], nib << ((4 * g4) & 31));
            cnt += __popc(nib);
        }
    }
    const int initial = block_sum<T>(cnt, red);  // (its barriers also complete vf)
    auto push = [&](int list, int c) {
        const int i = atomicAdd(&ctl[list], 1);
        if (i < F) fl[list * F + i] = (uint16_t)c;
        else ctl[2 + list] = 1;
    };
    // check side: erased count and id sum; the first frontier
    for (int c = tid; c < m; c += T) {
        uint32_t k = 0u, s = 0u;
        for (int j = 0; j < dc; ++j) {
            const int v = cvar[c * dc + j];
            if ((vf[v >> 5] >> (v & 31)) & 1u) { ++k; s += (uint32_t)v; }
        }
        st[c] = k << 24 | s;
        if (k == 1u) push(0, c);
    }
    if (tid == 0) tr[0] = initial;
    __syncthreads();

    int cur = initial, it = 0, its = iters, cl = 0;
    bool fill = false;  // stalled: the remaining counts repeat (message_passing.c:16-19)
    bool scanned = false;
    for (; it < iters; ++it) {
        const int len = ctl[cl], ovf = ctl[2 + cl];
        int resolved = 0;
        if (ovf && tid == 0) {
            atomicAdd(&g_peel_stats[0], 1ull);
            if (!scanned) atomicAdd(&g_peel_stats[1], 1ull);
            scanned = true;
        }
        auto process = [&](int c) {
            const uint32_t s = st[c];
            if ((s >> 24) != 1u) return;  // resolved meanwhile (its variable was the only erasure)
            const int v = (int)(s & 0xFFFFFFu);
            const uint32_t bit = 1u << (v & 31);
            if (!(atomicAnd(&vf[v >> 5], ~bit) & bit)) return;  // another check resolved v first
            ++resolved;
            for (int e = 0; e < dv; ++e) {
                const int c2 = vchk[(size_t)v * dv + e];
                const uint32_t old = atomicAdd(&st[c2], 0u - ((1u << 24) + (uint32_t)v));
                if ((old >> 24) == 2u) push(cl ^ 1, c2);
            }
        };
        if (!ovf) {
            for (int i = tid; i < len; i += T) process(fl[cl * F + i]);
        } else {  // the list overflowed: snapshot every check with count 1, then process them
            for (int w = tid; w < fw; w += T) {
                uint32_t bits = 0u;
                for (int j = 0; j < 32 && w * 32 + j < m; ++j) bits |= (uint32_t)((st[w * 32 + j] >> 24) == 1u) << j;
                fb[w] = bits;
            }
            __syncthreads();
            for (int w = tid; w < fw; w += T) {
                uint32_t bits = fb[w];
                fb[w] = 0u;
                while (bits) {
                    const int j = __ffs(bits) - 1;
                    bits &= bits - 1u;
                    process(w * 32 + j);
                }
            }
        }
        const int total = block_sum<T>(resolved, red);  // barriers: every update of the iteration done
        cur -= total;
        if (tid == 0) {
            tr[it + 1] = cur;
            ctl[cl] = 0;  // this iteration's list is free for iteration it + 2
            ctl[2 + cl] = 0;
        }
        __syncthreads();
        if (cur == 0) { its = it; break; }  // message_passing.c:76-78 (returns this it)
        if (total == 0) { fill = true; ++it; break; }  // fixed point: every later count repeats
        cl ^= 1;
    }
    // remaining curve entries: the stall value, or zeros after the break (the reference's
    // errors[] stay 0 there)
    for (int i = it + 1 + tid; i <= iters; i += T) tr[i] = fill ? cur : 0;
    if (tid == 0) {
        a.its[b] = its;
        atomicAdd(&g_peel_stats[2], 1ull);
    }
}

}  // namespace

// Bytes of LDS the peeling decoder needs with frontier lists of F entries each.
static size_t peel_lds(int n, int m, int F) {
    return (size_t)4 * (m + ((n + 31) >> 5) + ((m + 31) >> 5)) + (size_t)4 * F;
}

hipError_t launch_mc_bec_peel(int n, int dv, int dc, const int32_t *check_lookup, const int32_t *variable_lookup,
                              float p, uint64_t seed, uint64_t first_cw, int B, int max_iters, int32_t *trial,
                              int32_t *trial_its, hipStream_t stream) {
    const int m = n * dv / dc;
    constexpr size_t kBudget = 160 * 1024 - 1024;  // the kernel's static LDS beside the dynamic part
    if (m > 65536 || dc > 255 || (long)dc * n >= (1L << 24) || peel_lds(n, m, 256) > kBudget)
        return hipErrorNotSupported;
    if (B <= 0) return hipSuccess;
    int F = (int)std::min<size_t>((size_t)m, (kBudget - peel_lds(n, m, 0)) / 4);
    if (const int cap = g_peel_cap.load(); cap > 0) F = std::min(F, cap);
    PeelArgs a;
    a.cvar = check_lookup;
    a.vchk = variable_lookup;
    a.graph_stride = (int64_t)n * dv;
    a.n = n;
    a.m = m;
    a.dv = dv;
    a.dc = dc;
    a.max_iters = max_iters;
    a.F = F;
    a.ch.kind = 0;
    a.ch.p = p;
    a.ch.p2 = 0.0f;
    a.ch.k0 = (uint32_t)seed;
    a.ch.k1 = (uint32_t)(seed >> 32);
    a.first_cw = first_cw;
    a.trial = trial;
    a.its = trial_its;
    const size_t lds = peel_lds(n, m, F);
    hipError_t e = allow_lds(bec_peel_kernel<1024>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(bec_peel_kernel<1024>, dim3(B), dim3(1024), lds, stream, a);
    return hipGetLastError();
}

hipError_t peel_stats(uint64_t *out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_peel_stats), sizeof(unsigned long long) * 3);
    if (e == hipSuccess && reset) {
        static const unsigned long long z[3] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_peel_stats), z, sizeof(z));
    }
    return e;
}

void peel_cap(int F) { g_peel_cap = F > 0 ? F : 0; }

}  // namespace ldpc
