// Internal declarations shared by the C ABI (capi.cpp) and the kernels
// (ldpc_kernels.hip).  Not part of the public ABI (see include/ldpc_mi355x.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

// Device-resident Tanner graph.  Slot e = position in the check-major edge
// list (the reference's check_lookup order, random_code_generator.c:34-36).
struct ldpc_graph {
    int n = 0, m = 0, k = 0, E = 0;
    int dv = 0, dc = 0;          // > 0 when every variable / check has that degree
    int max_vdeg = 0, max_cdeg = 0;
    bool consistent = false;     // vslot defined: soft decoding allowed
    int device = 0;
    // device arrays
    int32_t *cvar = nullptr;     // [E]   variable of each slot (check-major)
    int32_t *cptr = nullptr;     // [m+1] check c owns slots [cptr[c], cptr[c+1])
    int32_t *vptr = nullptr;     // [n+1] variable v owns edges [vptr[v], vptr[v+1])
    int32_t *vchk = nullptr;     // [E']  BEC: check id of each variable edge, -1 when
                                 //       that check holds v != 1 times (never assigns)
    int32_t *vslot = nullptr;    // [E]   soft: slot of each variable edge (consistent only)
    int vchk_len = 0;
    // Conflict-aware lane layout of the LDS-resident (3,6) kernel (see
    // build_lane_layout in capi.cpp): position p = t + i*T is thread t's i-th
    // variable; every 32 consecutive positions form one half-wave LDS access.
    int lane_T = 0, lane_VPT = 0;
    int32_t *lane_var = nullptr;   // [T*VPT]    variable id, -1 = padding lane
    int32_t *lane_slot = nullptr;  // [T*VPT*dv] LDS position per edge (lds_pair_pos; padding
                                   //            lanes: dummy positions >= lds_pair_span)
    // Layout of the irregular kernel (bp_irr_kernel; build_irr_layout in capi.cpp):
    // check c = k*1024 + t (thread t, row k < irr_KC), its slot j at position
    // (k*irr_DC + j)*1024 + t; positions [0, irr_S) live in LDS, [irr_S, irr_P) in a
    // per-workgroup global slab.  Lane p = i*1024 + t is thread t's i-th variable.
    int irr_VPT = 0, irr_KC = 0, irr_DC = 0, irr_S = 0, irr_P = 0;
    int32_t *irr_lane = nullptr;  // [3][1024*VPT]: variable id (-1 pad), positions j0|j1<<16, j2|j3<<16
                                  // (0xFFFF = no edge; lanes of one 64-lane row share a degree)
    int32_t *irr_cdeg = nullptr;  // [2][1024]: degrees of thread t's checks, 4 bits per row k
    // Local-edge layout of bp_loc_kernel (build_loc_layout, loc_layout.cpp); loc_KP == 0: none
    int loc_T = 0, loc_KP = 0, loc_DVN = 0, loc_P = 0, loc_ncls = 0, loc_words = 0, loc_dlo = 0, loc_dhi = 0;
    int loc_dvn0 = 0, loc_dvn1 = 0;       // non-local edges per variable, local slot 0 / 1 (max)
    bool loc_abs0 = false, loc_abs1 = false;  // some variable of that slot has fewer
    int loc_cls_q[5] = {0}, loc_cls_d[4] = {0}, loc_cls_w[5] = {0};
    int32_t *loc_var = nullptr;   // [2*KP][2][T] variable id of var pair (thread, pair slot) half h, -1 pad
    int32_t *loc_pos = nullptr;   // [2*KP][DVN][T] non-local edge u's LDS words, h=0 | h=1 << 16
    int32_t *loc_info = nullptr;  // [2*KP][T] bit u + 4h: edge u present; bits 8+2h: local edge index jl;
                                  // bit 16 + 4h + jl: the same one-hot (min-sum order masks)
};

// Local-edge layout (loc_layout.cpp): see the comment there.
constexpr int kLocMaxD = 8, kLocMaxCls = 4;
struct LocLayout {
    int T = 1024, KP = 0, DVN = 0, P = 0, ncls = 0, words = 0;
    int DVN0 = 0, DVN1 = 0;     // non-local edges per variable of local slot 0 / 1 (max)
    bool ABS0 = false, ABS1 = false;  // some variable of that slot has fewer
    long conflicts = 0;  // sum over (instruction, half wave) of the busiest bank's extra lanes
    int cls_q[kLocMaxCls + 1] = {0}, cls_d[kLocMaxCls] = {0}, cls_w[kLocMaxCls + 1] = {0};
    std::vector<int32_t> var, pos, info;
};
bool build_loc_layout(int n, int m, const std::vector<int32_t> &cptr, const std::vector<int32_t> &cvar,
                      const std::vector<int32_t> &vptr, const std::vector<int32_t> &vslot, LocLayout &L);

// Check-degree range of a layout's classes (a mixed class counts its smaller check); false
// when a mixed class is not (dhi - 1, dhi) -- the kernel pads a mixed pair's smaller check by
// exactly one input.
inline bool loc_degree_range(const LocLayout &L, int &dlo, int &dhi) {
    dlo = 99;
    dhi = 0;
    for (int i = 0; i < L.ncls; ++i) {
        dlo = std::min(dlo, L.cls_d[i] >> 8 ? L.cls_d[i] >> 8 : L.cls_d[i]);
        dhi = std::max(dhi, L.cls_d[i] & 255);
    }
    bool ok = true;
    for (int i = 0; i < L.ncls; ++i)
        if (L.cls_d[i] >> 8) ok &= (L.cls_d[i] & 255) == dhi && (L.cls_d[i] >> 8) == dhi - 1;
    return ok;
}

// The bp_loc_kernel instantiation family a local-edge layout runs on -- decided from the
// WHOLE shape, never from the check degrees alone (a check-regular degree-6 graph with
// variable degrees {2, 4} has loc_dlo == 6 but needs the RSU family's DVN = 3 rows):
//   kLocReg36: <DLO=6, DHI=6, DVN0=2, DVN1=2, ABS0=ABS1=false> -- every check degree 6 and every
//              variable degree 3 (the (3,6) codes); shapes T=256 KP 1-4, T=1024 KP 2-3, T=512 KP 5
//   kLocRsu:   <DLO=5, DHI=6, DVN0=1, DVN1=3, ABS0=false, ABS1=true> -- check degrees 5..6, every
//              slot-0 variable degree 2, slot-1 variables degree 2..4; T=256 KP 1-4, T=1024 KP 2-3,
//              T=512 KP 8 / 10
//   kLocNone:  no instantiation (the graph runs on bp_lds / bp_irr / bp_generic)
enum LocVariant { kLocNone = 0, kLocReg36 = 1, kLocRsu = 2 };
inline int loc_variant(int dlo, int dhi, int DVN, int dvn0, int dvn1, bool abs0, bool abs1, int T, int KP) {
    if (KP <= 0) return kLocNone;
    const bool reg36 = dlo == 6 && dhi == 6 && DVN == 2 && dvn0 == 2 && dvn1 == 2 && !abs0 && !abs1;
    const bool rsu = !reg36 && dlo >= 5 && dhi == 6 && DVN == 3 && dvn0 == 1 && !abs0 && dvn1 <= 3;
    const bool common = (T == 256 && KP >= 1 && KP <= 4) || (T == 1024 && KP >= 2 && KP <= 3);
    if (reg36 && (common || (T == 512 && KP == 5))) return kLocReg36;
    if (rsu && (common || (T == 512 && (KP == 8 || KP == 10)))) return kLocRsu;
    return kLocNone;
}

// Irregular kernel (bp_irr_kernel): 1024 threads; LDS room for messages (bytes)
// after the early-stop syndrome bits and the Monte-Carlo curve.
constexpr int kIrrT = 1024;
constexpr size_t kIrrLdsMsgBytes = 148 * 1024;

// Threads per workgroup and variables per thread of the LDS-resident kernel
// for block length n: >= 2 % spare lanes for the conflict-aware layout.  (At
// n = 10^4, 3 % spare = 11 variables per thread packs with ~1.02 LDS cycles per
// half-wave access, 2 % = 10 per thread with ~1.5 -- and is 5 % faster: the
// variable phase is bound by per-lane work, not bank conflicts.)  Must match the
// instantiations in ldpc_kernels.hip.
#ifndef LDPC_LDS_SPARE
#define LDPC_LDS_SPARE 102  // lanes >= n * SPARE / 100 (fewer lanes beat fewer bank conflicts)
#endif
inline bool lds_shape(int n, int &T, int &VPT) {
    static const int v256[] = {1, 2, 3, 5, 9};
    static const int v1024[] = {2, 3, 5, 6, 9, 10, 11, 14};
    const long need = ((long)n * LDPC_LDS_SPARE + 99) / 100;
    if (n <= 2048) {
        T = 256;
        for (int v : v256)
            if (256L * v >= need) { VPT = v; return true; }
    }
    T = 1024;
    for (int v : v1024)
        if (1024L * v >= need) { VPT = v; return true; }
    return false;
}
constexpr int kLdsDummy = 3 * 32 + 4;  // dummy message slots after the real ones (DV=3)

// Message positions of the LDS-resident (3,6) kernel.  Checks are paired
// (2q, 2q+1) and their edges interleaved, [pair q][edge][check of the pair], so
// one LDS access moves the same edges of both checks and the check update runs
// on float2 (both checks in every packed VALU op).  With a 2*dc = 12-dword pair
// stride the check phase's ds_read_b128 / ds_write_b128 are conflict-free.
inline int lds_pair_pos(int slot, int dc) {
    const int c = slot / dc, j = slot % dc;
    return (c >> 1) * 2 * dc + 2 * j + (c & 1);
}
// Positions spanned by the m checks (an odd m leaves one phantom check).
inline int lds_pair_span(int m, int dc) { return ((m + 1) / 2) * 2 * dc; }

namespace ldpc {

void set_error(const std::string &msg);

// Kernel launchers (ldpc_kernels.hip).  All asynchronous on `stream`.
// Return hipSuccess or the launch error.
hipError_t launch_bec_decode(const ldpc_graph &g, uint8_t *d_words, int B, int max_iters,
                             int32_t *d_errors, int32_t *d_its, hipStream_t stream);

hipError_t launch_bp_decode(const ldpc_graph &g, const float *d_llr, int B, int max_iters, int algo,
                            float alpha, int early_stop, float *d_post, uint8_t *d_hard,
                            int32_t *d_its, hipStream_t stream, float *d_scratch, size_t scratch_bytes);

// Bytes of global scratch launch_bp_decode / launch_mc_decode need for this graph/batch (0
// when the messages fit in LDS); ep_slab: an early-stop decode that returns posteriors (the
// local-edge kernel's per-workgroup slabs; no other mode uses them).
// ep: an early-stop decode that returns posteriors (the slabs are sized only if it runs on bp_loc_kernel).
// The launchers check the layout of the path that runs against scratch_bytes and refuse
// (hipErrorInvalidValue) one that would not fit, so a sizing rule that drifts from the dispatch
// fails loudly instead of writing past the buffer.
size_t bp_scratch_bytes(const ldpc_graph &g, int B, int iters, int algo, bool ep);

hipError_t launch_channel(int channel, float p, float p2, uint64_t seed, uint64_t first_cw, int n,
                          int B, void *d_out, hipStream_t stream);

// Monte-Carlo: fused channel + decode writing per-trial curves into `trial`
// ([B][max_iters+1] int32) and its into `trial_its` ([B]); then the reducer.
hipError_t launch_mc_decode(const ldpc_graph &g, int channel, float p, float p2, uint64_t seed,
                            uint64_t first_cw, int B, int max_iters, int algo, float alpha,
                            int early_stop, int32_t *trial, int32_t *trial_its, hipStream_t stream,
                            float *d_scratch, size_t scratch_bytes);
hipError_t launch_mc_reduce(const int32_t *trial, const int32_t *trial_its, int B, int max_iters,
                            int expurgation, int64_t stop_frame_errors, int64_t *d_counters,
                            int32_t *d_cutoff, hipStream_t stream);

// Buckets (= threads per workgroup) of the parallel graph sampler for n*dv
// sockets; the permutation is in LDS (u16) when n*dv < 65536.  Must match
// oracle_sample_regular.
inline int sample_buckets(int E) { return E <= 16384 ? 256 : (E < 65536 ? 512 : 1024); }
// Sequential-draw sampler (sample_seq_kernel, one wave per graph) for
// kSeqMinE <= n*dv <= kSeqMaxE with check degrees <= kSeqMaxCdeg; the oracle's
// SEQ_* constants must equal these.  Larger graphs: one level, K = 1024.
constexpr int kSeqMinE = 8192, kSeqMaxE = 393216, kSeqMaxCdeg = 192;

// Random regular graphs on the device (law of random_code_generator.c), one
// workgroup per graph; attempts[g] = number of permutations drawn (negative if
// max_attempts was hit without a valid graph).
// ctl: device scratch of sample_ctl_words(G) words for the sequential sampler's search pass
// (nullptr: the single-pass form, one wave draws a graph's attempts in order).
hipError_t launch_sample_regular(int n, int dv, int dc, uint64_t seed, uint64_t first_graph, int G,
                                 int32_t *check_lookup, int32_t *variable_lookup, int32_t *attempts,
                                 int max_attempts, uint32_t *ctl, hipStream_t stream);
inline size_t sample_ctl_words(int G) { return 2 + 4 * (size_t)G; }
// Diagnostics builds (-DLDPC_SEQ_STATS=1): the search and emit passes' per-phase counters
// (2 x kStCount words, see SeqStat in sampler.hip); hipErrorNotSupported in the product build.
hipError_t seq_stats(uint64_t *out, int reset);
// Irregular form: socket s of variable d_vsock[s]; check c owns slots [cptr[c], cptr[c+1]);
// outputs check_var[g][E] and var_slot[g][E] (CSR, each variable's slots ascending).
hipError_t launch_sample_csr(int n, int m, int E, const int32_t *d_vsock, const int32_t *d_cptr,
                             const int32_t *d_vptr, int max_cdeg, int max_vdeg, uint64_t seed, uint64_t first_graph,
                             int G, int32_t *check_var, int32_t *var_slot, int32_t *attempts, int max_attempts,
                             uint32_t *ctl, hipStream_t stream);
// Frontier-peeling form of the ensemble BEC Monte-Carlo (peel.hip): regular (dv, dc) graphs
// whose check state fits LDS; hipErrorNotSupported otherwise (launch_mc_bec_ensemble then
// runs bec_kernel).
hipError_t launch_mc_bec_peel(int n, int dv, int dc, const int32_t *check_lookup, const int32_t *variable_lookup,
                              float p, uint64_t seed, uint64_t first_cw, int B, int max_iters, int32_t *trial,
                              int32_t *trial_its, hipStream_t stream);
// Scan-path evidence of the peeling decoder (device global, this device): [0] overflowed
// iterations, [1] trials that overflowed, [2] trials decoded.
hipError_t peel_stats(uint64_t *out, int reset);
// Test-only cap on the frontier-list capacity (F > 0), 0 restores the LDS budget's capacity.
void peel_cap(int F);
// BEC Monte-Carlo where trial b decodes on graph b of (check_lookup, variable_lookup).
hipError_t launch_mc_bec_ensemble(int n, int dv, int dc, const int32_t *check_lookup, const int32_t *variable_lookup,
                                  float p, uint64_t seed, uint64_t first_cw, int B, int max_iters, int32_t *trial,
                                  int32_t *trial_its, hipStream_t stream);

// ML ("optimal") erasure decoding, one workgroup per word (m <= 1000).
// cptr == nullptr: regular lists (check c = slots [c*dc, c*dc+dc)), word b reads
// cvar + b*cvar_stride.
hipError_t launch_ml_decode(const int32_t *cptr, const int32_t *cvar, int64_t cvar_stride, int dc, int n, int m,
                            const uint8_t *d_in, int B, uint8_t *d_out, int32_t *d_unsolved, hipStream_t stream);
// mc_reduce with a cutoff computed by an earlier launch_mc_reduce (trial_its may be null).
hipError_t launch_mc_reduce_cut(const int32_t *trial, const int32_t *trial_its, int B, int max_iters, int expurgation,
                                const int32_t *d_cutoff, int64_t *d_counters, hipStream_t stream);

// Kernel-choice introspection for tests / bench ("lds36", "generic", ...).
const char *bp_kernel_name(const ldpc_graph &g, int early_stop);

}  // namespace ldpc
