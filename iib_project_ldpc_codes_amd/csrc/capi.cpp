// C ABI of libldpc_mi355x.so (declared in include/ldpc_mi355x.h).
//
// Host side of the boundary: argument validation, graph preparation (edge
// lists -> device CSR / slot form), device workspaces and the synchronous
// host-pointer convenience forms.  There is no CPU compute path: without a
// visible HIP device every entry point fails with LDPC_ENODEV.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "ldpc_internal.hpp"

#ifndef LDPC_IRR
#define LDPC_IRR 1  // irregular graphs on bp_irr_kernel when in range
#endif
#ifndef LDPC_LOC_LAYOUT
#define LDPC_LOC_LAYOUT 1  // build the local-edge layout (bp_loc_kernel) for rate-1/2 graphs
#endif
#include "ldpc_mi355x.h"

namespace ldpc {
namespace {
thread_local std::string g_err;
std::mutex g_mu;     // the drop-in graph cache and the host-buffer entry points
std::mutex g_ws_mu;  // the workspace map (each workspace has its own lock)

// Grow-only device buffer.
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
};

// Lock order: g_mu before Workspace::mu; the device-pointer Monte-Carlo entry takes only its
// workspace's lock, so launches on different devices / streams never serialise on g_mu.
struct Workspace {
    std::mutex mu;
    DevBuf trial, its, cutoff, scratch, words, llr, post, hard, errors, itsb, gchk, gvar, gatt, mlw, mlo, mlu, shape,
        sctl;  // sampler search control (sample_ctl_words)
};
std::map<std::pair<int, void *>, Workspace> g_ws;  // (device, stream)

Workspace &workspace(void *stream) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_ws_mu);
    return g_ws[std::make_pair(dev, stream)];  // std::map nodes never move
}
}  // namespace

void set_error(const std::string &msg) { g_err = msg; }
}  // namespace ldpc

using namespace ldpc;

#define LDPC_HIP(expr)                                                                            \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess) {                                                                   \
            set_error(std::string(#expr) + ": " + hipGetErrorString(_e));                         \
            return LDPC_EHIP;                                                                     \
        }                                                                                         \
    } while (0)

#define LDPC_REQUIRE(cond, msg)          \
    do {                                 \
        if (!(cond)) {                   \
            set_error(msg);              \
            return LDPC_EINVAL;          \
        }                                \
    } while (0)

static int require_device() {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) {
        set_error("libldpc_mi355x: no HIP device visible (this library has no CPU path; run on an MI355X)");
        return LDPC_ENODEV;
    }
    return LDPC_OK;
}

// ---------------------------------------------------------------------------
// Graph preparation
// ---------------------------------------------------------------------------
namespace {
struct HostGraph {
    int n = 0, m = 0, k = 0, dv = 0, dc = 0;
    std::vector<int32_t> cvar, cptr, vptr, vchk, vslot;
    bool consistent = false;
    int max_vdeg = 0, max_cdeg = 0;
};

// Regular edge lists in the reference format (random_code_generator.c:34-36, :57-62).
int host_graph_from_lists(const int32_t *v2c, const int32_t *c2v, int n, int k, int dv, int dc, HostGraph &h) {
    LDPC_REQUIRE(v2c && c2v, "null edge list");
    LDPC_REQUIRE(n > 0 && dv > 0 && dc > 0 && k >= 0 && k < n, "bad (n, k, dv, dc)");
    const int m = n - k;
    h.n = n; h.m = m; h.k = k; h.dv = dv; h.dc = dc;
    h.max_vdeg = dv; h.max_cdeg = dc;
    const size_t Ec = (size_t)m * dc, Ev = (size_t)n * dv;
    h.cvar.assign(c2v, c2v + Ec);
    for (size_t e = 0; e < Ec; ++e)
        LDPC_REQUIRE(h.cvar[e] >= 0 && h.cvar[e] < n, "check_to_variable_list entry out of range [0, n)");
    for (size_t e = 0; e < Ev; ++e)
        LDPC_REQUIRE(v2c[e] >= 0 && v2c[e] < m, "variable_to_check_list entry out of range [0, n-k)");
    h.cptr.resize(m + 1);
    for (int c = 0; c <= m; ++c) h.cptr[c] = c * dc;
    h.vptr.resize(n + 1);
    for (int v = 0; v <= n; ++v) h.vptr[v] = v * dv;
    h.vchk.resize(Ev);
    h.vslot.assign(Ev, -1);
    bool ok = (Ec == Ev);
    for (int v = 0; v < n; ++v) {
        for (int j = 0; j < dv; ++j) {
            const int c = v2c[(size_t)v * dv + j];
            int occ = 0, rep = 0, found = -1;
            for (int jj = 0; jj < j; ++jj) rep += (v2c[(size_t)v * dv + jj] == c);
            for (int s = 0; s < dc; ++s) {
                if (h.cvar[(size_t)c * dc + s] == v) {
                    if (occ == rep) found = c * dc + s;
                    ++occ;
                }
            }
            h.vchk[(size_t)v * dv + j] = occ == 1 ? c : -1;
            if (found < 0) ok = false;
            h.vslot[(size_t)v * dv + j] = found;
        }
    }
    h.consistent = ok;
    return LDPC_OK;
}

int host_graph_from_csr(const int32_t *cptr, const int32_t *cvar, const int32_t *vptr, const int32_t *vslot, int n,
                        int m, HostGraph &h) {
    LDPC_REQUIRE(cptr && cvar && vptr && vslot && n > 0 && m > 0, "bad CSR graph arguments");
    LDPC_REQUIRE(cptr[0] == 0 && vptr[0] == 0 && cptr[m] == vptr[n] && cptr[m] > 0, "CSR pointers disagree");
    const int E = cptr[m];
    h.n = n; h.m = m; h.k = n - m;
    h.cptr.assign(cptr, cptr + m + 1);
    h.vptr.assign(vptr, vptr + n + 1);
    h.cvar.assign(cvar, cvar + E);
    h.vslot.assign(vslot, vslot + E);
    std::vector<int32_t> slot_check(E);
    for (int c = 0; c < m; ++c) {
        LDPC_REQUIRE(cptr[c + 1] >= cptr[c], "check_ptr not monotone");
        h.max_cdeg = std::max(h.max_cdeg, cptr[c + 1] - cptr[c]);
        for (int s = cptr[c]; s < cptr[c + 1]; ++s) {
            LDPC_REQUIRE(cvar[s] >= 0 && cvar[s] < n, "check_var out of range");
            slot_check[s] = c;
        }
    }
    std::vector<char> seen(E, 0);
    h.vchk.resize(E);
    for (int v = 0; v < n; ++v) {
        LDPC_REQUIRE(vptr[v + 1] >= vptr[v], "var_ptr not monotone");
        h.max_vdeg = std::max(h.max_vdeg, vptr[v + 1] - vptr[v]);
        for (int e = vptr[v]; e < vptr[v + 1]; ++e) {
            const int s = vslot[e];
            LDPC_REQUIRE(s >= 0 && s < E && !seen[s] && cvar[s] == v, "var_slot is not a slot permutation");
            seen[s] = 1;
            const int c = slot_check[s];
            int occ = 0;
            for (int q = cptr[c]; q < cptr[c + 1]; ++q) occ += (cvar[q] == v);
            h.vchk[e] = occ == 1 ? c : -1;
        }
    }
    bool reg_c = true, reg_v = true;
    for (int c = 0; c < m; ++c) reg_c &= (cptr[c + 1] - cptr[c] == h.max_cdeg);
    for (int v = 0; v < n; ++v) reg_v &= (vptr[v + 1] - vptr[v] == h.max_vdeg);
    if (reg_c && reg_v) {
        h.dc = h.max_cdeg;
        h.dv = h.max_vdeg;
    }
    h.consistent = true;
    return LDPC_OK;
}

template <typename T>
hipError_t upload(T **dst, const std::vector<T> &src) {
    *dst = nullptr;
    if (src.empty()) return hipSuccess;
    hipError_t e = hipMalloc(reinterpret_cast<void **>(dst), src.size() * sizeof(T));
    if (e != hipSuccess) return e;
    return hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice);
}

// Conflict-aware lane layout for the LDS-resident kernel (bp_lds_kernel).
// Lane positions p = t + i*T are cut into groups of 32 (one half-wave
// ds_read/ds_write_b32); a group's accesses to edge j of its variables cost
// one LDS cycle per distinct address on the busiest bank (bank = slot mod 32).
// Variables are placed most-constrained first into the first group whose
// banks for all dv edges are still free, then conflicting ones are moved to
// conflict-free groups with room.  Slots are mapped to the kernel's LDS
// positions first (lds_pair_pos).  Padding lanes get dummy positions S + 32 j + f
// (S = lds_pair_span) on banks the group leaves free.
// Measured on a (3,6) n=10000 graph: 3.44 -> ~1.02 cycles per half-wave access
// at T*VPT = 1.126 n.
void build_lane_layout(const HostGraph &h, int T, int VPT, std::vector<int32_t> &lane_var,
                       std::vector<int32_t> &lane_slot) {
    const int n = h.n, dv = h.dv, E = lds_pair_span(h.m, h.dc);
    const int P = T * VPT, G = P / 32;
    std::vector<int> pos((size_t)n * dv), bank((size_t)n * dv);
    std::vector<int> deg((size_t)dv * 32, 0);
    for (int v = 0; v < n; ++v)
        for (int j = 0; j < dv; ++j) {
            pos[(size_t)v * dv + j] = lds_pair_pos(h.vslot[(size_t)v * dv + j], h.dc);
            bank[(size_t)v * dv + j] = pos[(size_t)v * dv + j] & 31;
            deg[(size_t)j * 32 + bank[(size_t)v * dv + j]]++;
        }
    std::vector<int> order(n), score(n);
    for (int v = 0; v < n; ++v) {
        order[v] = v;
        int sc = 0;
        for (int j = 0; j < dv; ++j) sc += deg[(size_t)j * 32 + bank[(size_t)v * dv + j]];
        score[v] = sc;
    }
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return score[x] > score[y]; });
    std::vector<int> occ((size_t)G * dv * 32, 0), fill(G, 0), where(n, -1);
    auto conflicts = [&](int q, int v) {
        int c = 0;
        for (int j = 0; j < dv; ++j) c += occ[((size_t)q * dv + j) * 32 + bank[(size_t)v * dv + j]];
        return c;
    };
    auto put = [&](int q, int v, int d) {
        for (int j = 0; j < dv; ++j) occ[((size_t)q * dv + j) * 32 + bank[(size_t)v * dv + j]] += d;
        fill[q] += d;
        where[v] = d > 0 ? q : -1;
    };
    int gi = 0;
    for (int v : order) {
        int best = -1, bestc = 1 << 30;
        for (int k = 0; k < G; ++k) {
            const int q = (gi + k) % G;
            if (fill[q] >= 32) continue;
            const int c = conflicts(q, v);
            if (c < bestc) { bestc = c; best = q; if (c == 0) break; }
        }
        put(best, v, 1);
        gi = (best + 1) % G;
    }
    for (int round = 0; round < 8; ++round) {
        int moved = 0;
        for (int v = 0; v < n; ++v) {
            const int q = where[v];
            put(q, v, -1);
            if (conflicts(q, v) == 0) { put(q, v, 1); continue; }
            int r = -1;
            for (int k = 0; k < G; ++k)
                if (fill[k] < 32 && conflicts(k, v) == 0) { r = k; break; }
            put(r >= 0 ? r : q, v, 1);
            moved += (r >= 0);
        }
        if (!moved) break;
    }
    lane_var.assign(P, -1);
    lane_slot.assign((size_t)P * dv, 0);
    std::vector<int> cursor(G, 0);
    for (int v = 0; v < n; ++v) {
        const int q = where[v], p = q * 32 + cursor[q]++;
        lane_var[p] = v;
        for (int j = 0; j < dv; ++j) lane_slot[(size_t)p * dv + j] = pos[(size_t)v * dv + j];
    }
    for (int q = 0; q < G; ++q) {
        std::vector<char> used((size_t)dv * 32, 0);  // [edge j][bank]
        for (int l = 0; l < cursor[q]; ++l)
            for (int j = 0; j < dv; ++j) used[(size_t)j * 32 + (lane_slot[((size_t)q * 32 + l) * dv + j] & 31)] = 1;
        for (int l = cursor[q]; l < 32; ++l) {
            for (int j = 0; j < dv; ++j) {
                // dummy position E + 32 j + f lands on bank (E + f) mod 32: take a free one
                int f = 0;
                for (int t = 0; t < 32; ++t)
                    if (!used[(size_t)j * 32 + ((E + t) & 31)]) { f = t; break; }
                used[(size_t)j * 32 + ((E + f) & 31)] = 1;
                lane_slot[((size_t)q * 32 + l) * dv + j] = E + 32 * j + f;
            }
        }
    }
}

// Layout of the irregular kernel (bp_irr_kernel, ldpc_internal.hpp): rows of
// 1024 checks, DC = 6 or 8 slots per check (absent slots hold the check rule's
// neutral value), positions k-major so a row's slots are lane-contiguous (LDS
// conflict-free / coalesced in the slab) and whole rows are either in LDS or in
// the slab; variables sorted by degree, every degree class padded to whole
// 64-lane rows so the degree is wave-uniform; padding lanes of a class get
// private dummy positions after the checks'.  Returns false when the graph is
// outside the kernel's range (variable degree > 4, check degree > 8, > 16 rows,
// > 20 variables per thread, positions beyond 16 bits).
bool build_irr_layout(const HostGraph &h, int &VPT, int &KC, int &DC, int &S, int &P,
                      std::vector<int32_t> &lane, std::vector<int32_t> &cdeg) {
    const int T = kIrrT, n = h.n, m = h.m;
    if (h.max_vdeg > 4 || h.max_cdeg > 8 || n <= 0 || m <= 0) return false;
    DC = h.max_cdeg <= 6 ? 6 : 8;
    KC = (m + T - 1) / T;
    if (KC > 16) return false;
    const int PC = KC * DC * T;  // check positions
    std::vector<int> slot_check(h.cvar.size());
    for (int c = 0; c < m; ++c)
        for (int x = h.cptr[c]; x < h.cptr[c + 1]; ++x) slot_check[x] = c;
    auto pos_of = [&](int slot) {
        const int c = slot_check[slot], j = slot - h.cptr[c];
        return ((c / T) * DC + j) * T + (c % T);
    };
    // rows that fit LDS (whole rows; the rest go to the slab)
    const int rows_lds = (int)std::min<size_t>((size_t)KC, kIrrLdsMsgBytes / ((size_t)DC * T * 4));
    std::vector<int> order(n);
    for (int v = 0; v < n; ++v) order[v] = v;
    auto deg = [&](int v) { return h.vptr[v + 1] - h.vptr[v]; };
    // within a degree class, lanes sorted by which of their edges live in the slab:
    // a 64-lane row then mostly takes one side per edge (the other side's path is skipped)
    auto slab_mask = [&](int v) {
        int msk = 0;
        for (int j = 0; j < deg(v); ++j)
            if (slot_check[h.vslot[h.vptr[v] + j]] / T >= rows_lds) msk |= 1 << j;
        return msk;
    };
    std::vector<int> key(n);
    for (int v = 0; v < n; ++v) key[v] = -deg(v) * 64 + slab_mask(v);
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return key[x] < key[y]; });
    // lanes: degree classes padded to 64
    std::vector<int> lv;  // var id per lane, -(d+1) for a padding lane of degree d
    for (size_t a = 0; a < order.size();) {
        const int d = deg(order[a]);
        size_t b = a;
        while (b < order.size() && deg(order[b]) == d) lv.push_back(order[b++]);
        while (lv.size() % 64) lv.push_back(-(d + 1));
        a = b;
    }
    const int need = (int)((lv.size() + T - 1) / T);
    VPT = 0;
    for (int v : {1, 2, 5, 10, 20})
        if (v >= need) { VPT = v; break; }
    if (!VPT) return false;
    const int L = T * VPT;
    lane.assign((size_t)3 * L, 0);
    int dummy = PC;
    for (int q = 0; q < L; ++q) {
        int p4[4] = {0xFFFF, 0xFFFF, 0xFFFF, 0xFFFF};
        int var = -1;
        if (q < (int)lv.size() && lv[q] >= 0) {
            var = lv[q];
            for (int j = 0; j < deg(var); ++j) p4[j] = pos_of(h.vslot[h.vptr[var] + j]);
        } else if (q < (int)lv.size()) {
            for (int j = 0; j < -lv[q] - 1; ++j) p4[j] = dummy++;
        }
        lane[q] = var;
        lane[(size_t)L + q] = p4[0] | (p4[1] << 16);
        lane[(size_t)2 * L + q] = p4[2] | (p4[3] << 16);
    }
    P = dummy;
    if (P >= 0xFFFF) return false;
    // whole rows in LDS while they fit (the dummies too when everything fits)
    S = rows_lds == KC && (size_t)P * 4 <= kIrrLdsMsgBytes ? P : rows_lds * DC * T;
    cdeg.assign((size_t)2 * T, 0);
    for (int t = 0; t < T; ++t)
        for (int k = 0; k < KC; ++k) {
            const int c = k * T + t;
            const int d = c < m ? h.cptr[c + 1] - h.cptr[c] : 0;
            cdeg[(size_t)(k >> 3) * T + t] |= d << (4 * (k & 7));
        }
    return true;
}

// layouts = false: the BEC arrays only (the drop-in message_passing; no soft-decoder layouts)
int device_graph(const HostGraph &h, ldpc_graph **out, bool layouts = true) {
    int rc = require_device();
    if (rc) return rc;
    ldpc_graph *g = new ldpc_graph();
    g->n = h.n; g->m = h.m; g->k = h.k;
    g->E = (int)h.cvar.size();
    g->dv = h.dv; g->dc = h.dc;
    g->max_vdeg = h.max_vdeg; g->max_cdeg = h.max_cdeg;
    g->consistent = h.consistent;
    g->vchk_len = (int)h.vchk.size();
    (void)hipGetDevice(&g->device);
    hipError_t e = upload(&g->cvar, h.cvar);
    if (e == hipSuccess) e = upload(&g->cptr, h.cptr);
    if (e == hipSuccess) e = upload(&g->vptr, h.vptr);
    if (e == hipSuccess) e = upload(&g->vchk, h.vchk);
    if (e == hipSuccess && h.consistent) e = upload(&g->vslot, h.vslot);
    int T = 0, VPT = 0;
    if (e == hipSuccess && layouts && h.consistent && h.dv == 3 && h.dc == 6 && lds_shape(h.n, T, VPT) &&
        (size_t)(lds_pair_span(h.m, h.dc) + kLdsDummy) * 4 <= 150 * 1024) {
        std::vector<int32_t> lv, ls;
        build_lane_layout(h, T, VPT, lv, ls);
        e = upload(&g->lane_var, lv);
        if (e == hipSuccess) e = upload(&g->lane_slot, ls);
        g->lane_T = T;
        g->lane_VPT = VPT;
    }
    // LDPC_NO_LOC_LAYOUT=1 in the environment: no local-edge layout (tests run the
    // other kernels on the same graphs)
    const char *noloc = getenv("LDPC_NO_LOC_LAYOUT");
    if (e == hipSuccess && layouts && h.consistent && LDPC_LOC_LAYOUT && !(noloc && noloc[0] == '1')) {
        LocLayout L;
        // threads: 256 for up to 1024 check pairs (4 per thread); (3,6) codes up to 2560 pairs:
        // 512 threads x 5 pairs, two workgroups per CU when both fit the LDS (the bench code:
        // +29 % over one 1024-thread workgroup, whose barriers idle the CU); 1024 for up to
        // 3072 (3 per thread: 4 do not fit 128 VGPRs), else 512 threads with 256 VGPRs (up to
        // 10 per thread)
        const int P = h.m / 2;
        const bool r36 = h.dv == 3 && h.dc == 6;
        L.T = P <= 1024 ? 256 : (r36 && P <= 2560 ? 512 : (P <= 3072 ? 1024 : 512));
        if (const char *t = getenv("LDPC_LOC_T")) L.T = atoi(t);  // shape experiments
        bool built = build_loc_layout(h.n, h.m, h.cptr, h.cvar, h.vptr, h.vslot, L);
        if (built && r36 && L.T == 512 && L.KP == 5 && (size_t)std::max(L.words + 64, h.n) * 4 > 80 * 1024) {
            L = LocLayout();  // two workgroups would not fit one CU's LDS
            L.T = 1024;
            built = build_loc_layout(h.n, h.m, h.cptr, h.cvar, h.vptr, h.vslot, L);
        }
        if (built) {
            e = upload(&g->loc_var, L.var);
            if (e == hipSuccess) e = upload(&g->loc_pos, L.pos);
            if (e == hipSuccess) e = upload(&g->loc_info, L.info);
            g->loc_T = L.T; g->loc_KP = L.KP; g->loc_DVN = L.DVN; g->loc_P = L.P;
            g->loc_ncls = L.ncls; g->loc_words = L.words;
            int dlo = 99, dhi = 0;
            const bool mix_ok = loc_degree_range(L, dlo, dhi);
            g->loc_dlo = dlo; g->loc_dhi = dhi;
            if (!mix_ok) g->loc_KP = 0;
            for (int i = 0; i <= L.ncls; ++i) { g->loc_cls_q[i] = L.cls_q[i]; g->loc_cls_w[i] = L.cls_w[i]; }
            for (int i = 0; i < L.ncls; ++i) g->loc_cls_d[i] = L.cls_d[i];
            g->loc_dvn0 = L.DVN0; g->loc_dvn1 = L.DVN1;
            g->loc_abs0 = L.ABS0; g->loc_abs1 = L.ABS1;
        }
    }
    if (e == hipSuccess && layouts && h.consistent && !g->lane_var && LDPC_IRR) {
        std::vector<int32_t> ln, cd;
        int VPT_ = 0, KC = 0, DC = 0, S = 0, P = 0;
        if (build_irr_layout(h, VPT_, KC, DC, S, P, ln, cd)) {
            e = upload(&g->irr_lane, ln);
            if (e == hipSuccess) e = upload(&g->irr_cdeg, cd);
            g->irr_VPT = VPT_; g->irr_KC = KC; g->irr_DC = DC; g->irr_S = S; g->irr_P = P;
        }
    }
    if (e != hipSuccess) {
        set_error(std::string("graph upload: ") + hipGetErrorString(e));
        ldpc_graph_destroy(g);
        return LDPC_EHIP;
    }
    *out = g;
    return LDPC_OK;
}

// Drop-in state (message_passing, one word per call): the reference re-sends the same
// fixed-code lists on every call (parallel_simulator.py:360, fresh numpy copies each time), so
// the last lists are kept on the host and compared exactly (memcmp: no hash to collide); their
// BEC-only device graph, a stream, and pinned staging for the word / error curve in one
// transfer each way.
struct DropInCache {
    int n = -1, k = -1, dv = -1, dc = -1, dev = -1;
    std::vector<int32_t> v2c, c2v;  // the lists of the cached graph
    ldpc_graph *g = nullptr;
    hipStream_t s = nullptr;
    unsigned char *pin = nullptr, *dbuf = nullptr;  // [word u8 | errors i32 | its i32]
    size_t bytes = 0;
};
DropInCache g_dropin;
}  // namespace

extern "C" {

const char *ldpc_last_error(void) { return g_err.c_str(); }

int ldpc_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

int ldpc_set_device(int device) {
    int rc = require_device();
    if (rc) return rc;
    LDPC_HIP(hipSetDevice(device));
    return LDPC_OK;
}

int ldpc_sync(void *stream) {
    int rc = require_device();
    if (rc) return rc;
    LDPC_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return LDPC_OK;
}

int ldpc_graph_create(const int32_t *variable_to_check_list, const int32_t *check_to_variable_list, int n, int k,
                      int dv, int dc, ldpc_graph **out) {
    LDPC_REQUIRE(out, "null output handle");
    HostGraph h;
    int rc = host_graph_from_lists(variable_to_check_list, check_to_variable_list, n, k, dv, dc, h);
    if (rc) return rc;
    return device_graph(h, out);
}

int ldpc_graph_create_csr(const int32_t *check_ptr, const int32_t *check_var, const int32_t *var_ptr,
                          const int32_t *var_slot, int n, int m, ldpc_graph **out) {
    LDPC_REQUIRE(out, "null output handle");
    HostGraph h;
    int rc = host_graph_from_csr(check_ptr, check_var, var_ptr, var_slot, n, m, h);
    if (rc) return rc;
    return device_graph(h, out);
}

void ldpc_graph_destroy(ldpc_graph *g) {
    if (!g) return;
    (void)hipFree(g->cvar);
    (void)hipFree(g->cptr);
    (void)hipFree(g->vptr);
    (void)hipFree(g->vchk);
    (void)hipFree(g->vslot);
    (void)hipFree(g->lane_var);
    (void)hipFree(g->lane_slot);
    (void)hipFree(g->irr_lane);
    (void)hipFree(g->irr_cdeg);
    (void)hipFree(g->loc_var);
    (void)hipFree(g->loc_pos);
    (void)hipFree(g->loc_info);
    delete g;
}

int ldpc_graph_info(const ldpc_graph *g, int32_t *n, int32_t *m, int32_t *num_edges) {
    LDPC_REQUIRE(g, "null graph");
    if (n) *n = g->n;
    if (m) *m = g->m;
    if (num_edges) *num_edges = g->E;
    return LDPC_OK;
}

int ldpc_debug_lane_layout(const int32_t *variable_to_check_list, const int32_t *check_to_variable_list, int n,
                           int k, int dv, int dc, int32_t *T, int32_t *VPT, int32_t *lane_var, int32_t *lane_slot) {
    LDPC_REQUIRE(T && VPT, "null T / VPT");
    HostGraph h;
    int rc = host_graph_from_lists(variable_to_check_list, check_to_variable_list, n, k, dv, dc, h);
    if (rc) return rc;
    int t = 0, v = 0;
    LDPC_REQUIRE(h.consistent && lds_shape(n, t, v), "no LDS-resident layout for this graph");
    *T = t;
    *VPT = v;
    if (!lane_var || !lane_slot) return LDPC_OK;
    std::vector<int32_t> lv, ls;
    build_lane_layout(h, t, v, lv, ls);
    std::copy(lv.begin(), lv.end(), lane_var);
    std::copy(ls.begin(), ls.end(), lane_slot);
    return LDPC_OK;
}

int ldpc_debug_irr_layout(const int32_t *check_ptr, const int32_t *check_var, const int32_t *var_ptr,
                          const int32_t *var_slot, int n, int m, int32_t *shape, int32_t *lane, int32_t *cdeg) {
    LDPC_REQUIRE(shape, "null shape");
    HostGraph h;
    int rc = host_graph_from_csr(check_ptr, check_var, var_ptr, var_slot, n, m, h);
    if (rc) return rc;
    std::vector<int32_t> ln, cd;
    int VPT = 0, KC = 0, DC = 0, S = 0, P = 0;
    if (!h.consistent || !build_irr_layout(h, VPT, KC, DC, S, P, ln, cd)) {
        set_error("graph outside the irregular kernel's range");
        return LDPC_EUNSUP;
    }
    shape[0] = VPT; shape[1] = KC; shape[2] = DC; shape[3] = S; shape[4] = P;
    if (lane) std::copy(ln.begin(), ln.end(), lane);
    if (cdeg) std::copy(cd.begin(), cd.end(), cdeg);
    return LDPC_OK;
}

int ldpc_debug_loc_layout(const int32_t *check_ptr, const int32_t *check_var, const int32_t *var_ptr,
                          const int32_t *var_slot, int n, int m, int T, int32_t *shape, int32_t *var, int32_t *pos,
                          int32_t *info) {
    LDPC_REQUIRE(shape, "null shape");
    LDPC_REQUIRE(T == 256 || T == 512 || T == 1024, "T must be 256, 512 or 1024");
    HostGraph h;
    int rc = host_graph_from_csr(check_ptr, check_var, var_ptr, var_slot, n, m, h);
    if (rc) return rc;
    LocLayout L;
    L.T = T;
    if (!h.consistent || !build_loc_layout(h.n, h.m, h.cptr, h.cvar, h.vptr, h.vslot, L)) {
        set_error("graph has no local-edge layout (needs n = 2m, a perfect local matching, even degree classes)");
        return LDPC_EUNSUP;
    }
    shape[0] = L.T; shape[1] = L.KP; shape[2] = L.DVN; shape[3] = L.P; shape[4] = L.words;
    shape[5] = L.ncls; shape[6] = (int32_t)std::min<long>(L.conflicts, 0x7fffffff);
    for (int i = 0; i < kLocMaxCls; ++i) {
        shape[7 + i] = L.cls_q[i];
        shape[7 + kLocMaxCls + 1 + i] = L.cls_d[i];
        shape[7 + 2 * kLocMaxCls + 1 + i] = L.cls_w[i];
    }
    shape[7 + kLocMaxCls] = L.cls_q[kLocMaxCls];
    shape[7 + 3 * kLocMaxCls + 1] = L.cls_w[kLocMaxCls];
    shape[22] = L.DVN0 | (L.ABS0 ? 256 : 0);
    shape[23] = L.DVN1 | (L.ABS1 ? 256 : 0);
    if (var) std::copy(L.var.begin(), L.var.end(), var);
    if (pos) std::copy(L.pos.begin(), L.pos.end(), pos);
    if (info) std::copy(L.info.begin(), L.info.end(), info);
    return LDPC_OK;
}

int ldpc_debug_loc_variant(const int32_t *check_ptr, const int32_t *check_var, const int32_t *var_ptr,
                           const int32_t *var_slot, int n, int m, int T, int32_t *variant) {
    LDPC_REQUIRE(variant, "null variant");
    LDPC_REQUIRE(T == 256 || T == 512 || T == 1024, "T must be 256, 512 or 1024");
    HostGraph h;
    int rc = host_graph_from_csr(check_ptr, check_var, var_ptr, var_slot, n, m, h);
    if (rc) return rc;
    LocLayout L;
    L.T = T;
    *variant = kLocNone;
    if (!h.consistent || !build_loc_layout(h.n, h.m, h.cptr, h.cvar, h.vptr, h.vslot, L)) return LDPC_OK;
    int dlo = 0, dhi = 0;
    if (!loc_degree_range(L, dlo, dhi)) return LDPC_OK;
    *variant = loc_variant(dlo, dhi, L.DVN, L.DVN0, L.DVN1, L.ABS0, L.ABS1, L.T, L.KP);
    return LDPC_OK;
}

const char *ldpc_bp_kernel_name(const ldpc_graph *g, int early_stop) {
    return g ? bp_kernel_name(*g, early_stop) : "none";
}

// --------------------------- BEC -------------------------------------------
int ldpc_bec_decode_batch_dev(const ldpc_graph *g, uint8_t *d_words, int B, int max_iters, int32_t *d_errors,
                              int32_t *d_its, void *stream) {
    LDPC_REQUIRE(g && (B == 0 || (d_words && d_errors && d_its)) && B >= 0 && max_iters >= 0, "bad BEC batch arguments");
    if (B == 0 || max_iters == 0) {
        if (B && d_its) LDPC_HIP(hipMemsetAsync(d_its, 0, sizeof(int32_t) * B, static_cast<hipStream_t>(stream)));
        return LDPC_OK;
    }
    LDPC_HIP(launch_bec_decode(*g, d_words, B, max_iters, d_errors, d_its, static_cast<hipStream_t>(stream)));
    return LDPC_OK;
}

// Caller holds g_mu (the workspace and, for the drop-in, the cached graph stay valid).
static int bec_host_locked(const ldpc_graph *g, uint8_t *words, int B, int max_iters, int32_t *errors,
                           int32_t *its) {
    const size_t n = g->n;
    for (size_t i = 0; i < (size_t)B * n; ++i)
        LDPC_REQUIRE(words[i] <= 2, "channel word value outside {0, 1, 2}");
    Workspace &ws = workspace(nullptr);
    std::lock_guard<std::mutex> wl(ws.mu);
    LDPC_HIP(ws.words.ensure((size_t)B * n));
    LDPC_HIP(ws.errors.ensure(sizeof(int32_t) * (size_t)B * (max_iters > 0 ? max_iters : 1)));
    LDPC_HIP(ws.itsb.ensure(sizeof(int32_t) * (size_t)B));
    uint8_t *dw = static_cast<uint8_t *>(ws.words.p);
    int32_t *de = static_cast<int32_t *>(ws.errors.p), *di = static_cast<int32_t *>(ws.itsb.p);
    LDPC_HIP(hipMemcpy(dw, words, (size_t)B * n, hipMemcpyHostToDevice));
    if (max_iters > 0)
        LDPC_HIP(hipMemcpy(de, errors, sizeof(int32_t) * (size_t)B * max_iters, hipMemcpyHostToDevice));
    int rc = ldpc_bec_decode_batch_dev(g, dw, B, max_iters, de, di, nullptr);
    if (rc) return rc;
    LDPC_HIP(hipDeviceSynchronize());
    LDPC_HIP(hipMemcpy(words, dw, (size_t)B * n, hipMemcpyDeviceToHost));
    if (max_iters > 0)
        LDPC_HIP(hipMemcpy(errors, de, sizeof(int32_t) * (size_t)B * max_iters, hipMemcpyDeviceToHost));
    LDPC_HIP(hipMemcpy(its, di, sizeof(int32_t) * (size_t)B, hipMemcpyDeviceToHost));
    return LDPC_OK;
}

static int bec_host(const ldpc_graph *g, uint8_t *words, int B, int max_iters, int32_t *errors, int32_t *its) {
    std::lock_guard<std::mutex> lk(g_mu);
    return bec_host_locked(g, words, B, max_iters, errors, its);
}

int ldpc_bec_decode_batch(const int32_t *variable_to_check_list, const int32_t *check_to_variable_list, int n,
                          int k, int dv, int dc, uint8_t *words, int B, int max_iters, int32_t *errors,
                          int32_t *its) {
    LDPC_REQUIRE((B == 0 || (words && errors && its)) && B >= 0 && max_iters >= 0, "bad BEC batch arguments");
    ldpc_graph *g = nullptr;
    int rc = ldpc_graph_create(variable_to_check_list, check_to_variable_list, n, k, dv, dc, &g);
    if (rc) return rc;
    rc = B ? bec_host(g, words, B, max_iters, errors, its) : LDPC_OK;
    ldpc_graph_destroy(g);
    return rc;
}

// Drop-in for message_passing.c:7.
int message_passing(int *Mvc, int iterations, int *variable_to_check_list, int *check_to_variable_list,
                    int *errors, int n, int k, int dv, int dc) {
    if (iterations <= 0) return 0;  // the reference loop body never runs
    LDPC_REQUIRE(Mvc && errors && variable_to_check_list && check_to_variable_list, "null Mvc / errors / lists");
    LDPC_REQUIRE(n > 0 && dv > 0 && dc > 0 && k >= 0 && k < n, "bad (n, k, dv, dc)");
    int rc = require_device();
    if (rc) return rc;
    // One lock across the cache lookup and the decode: another thread replacing the cached
    // graph cannot free it while this call still uses it.
    std::lock_guard<std::mutex> lk(g_mu);
    DropInCache &c = g_dropin;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const size_t Ev = (size_t)n * dv, Ec = (size_t)(n - k) * dc;
    const bool same_shape = c.g && c.n == n && c.k == k && c.dv == dv && c.dc == dc && c.dev == dev;
    if (!(same_shape && !memcmp(c.v2c.data(), variable_to_check_list, Ev * 4) &&
          !memcmp(c.c2v.data(), check_to_variable_list, Ec * 4))) {
        HostGraph hg;
        rc = host_graph_from_lists(variable_to_check_list, check_to_variable_list, n, k, dv, dc, hg);
        if (rc) return rc;
        ldpc_graph *g = c.g;
        if (same_shape && g->consistent == hg.consistent && g->vchk_len == (int)hg.vchk.size()) {
            // another graph of the same shape (an ensemble run: a new code per trial): new
            // contents in the same device arrays
            LDPC_HIP(hipMemcpy(g->cvar, hg.cvar.data(), 4 * hg.cvar.size(), hipMemcpyHostToDevice));
            LDPC_HIP(hipMemcpy(g->cptr, hg.cptr.data(), 4 * hg.cptr.size(), hipMemcpyHostToDevice));
            LDPC_HIP(hipMemcpy(g->vptr, hg.vptr.data(), 4 * hg.vptr.size(), hipMemcpyHostToDevice));
            LDPC_HIP(hipMemcpy(g->vchk, hg.vchk.data(), 4 * hg.vchk.size(), hipMemcpyHostToDevice));
            if (hg.consistent) LDPC_HIP(hipMemcpy(g->vslot, hg.vslot.data(), 4 * hg.vslot.size(), hipMemcpyHostToDevice));
            g->max_vdeg = hg.max_vdeg;
            g->max_cdeg = hg.max_cdeg;
        } else {
            if (c.g) ldpc_graph_destroy(c.g);
            c.g = nullptr;
            if (c.s && c.dev != dev) {  // the stream and buffers belong to the old device
                (void)hipStreamDestroy(c.s);
                (void)hipHostFree(c.pin);
                (void)hipFree(c.dbuf);
                c.s = nullptr;
                c.pin = c.dbuf = nullptr;
                c.bytes = 0;
            }
            rc = device_graph(hg, &c.g, false);
            if (rc) return rc;
            c.n = n; c.k = k; c.dv = dv; c.dc = dc; c.dev = dev;
        }
        c.v2c.assign(variable_to_check_list, variable_to_check_list + Ev);
        c.c2v.assign(check_to_variable_list, check_to_variable_list + Ec);
    }
    if (!c.s) LDPC_HIP(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
    const size_t wb = ((size_t)n + 15) & ~(size_t)15, eb = (size_t)4 * iterations;
    const size_t need = wb + eb + 16;
    if (need > c.bytes) {
        (void)hipHostFree(c.pin);
        (void)hipFree(c.dbuf);
        c.pin = c.dbuf = nullptr;
        c.bytes = 0;
        LDPC_HIP(hipHostMalloc(reinterpret_cast<void **>(&c.pin), need, hipHostMallocDefault));
        LDPC_HIP(hipMalloc(reinterpret_cast<void **>(&c.dbuf), need));
        c.bytes = need;
    }
    uint8_t *pw = c.pin;
    for (int v = 0; v < n; ++v) {
        LDPC_REQUIRE(Mvc[v] >= 0 && Mvc[v] <= 2, "Mvc value outside {0, 1, 2}");
        pw[v] = (uint8_t)Mvc[v];
    }
    memcpy(c.pin + wb, errors, eb);  // the reference accumulates into the caller's errors[]
    LDPC_HIP(hipMemcpyAsync(c.dbuf, c.pin, wb + eb, hipMemcpyHostToDevice, c.s));
    rc = ldpc_bec_decode_batch_dev(c.g, c.dbuf, 1, iterations, reinterpret_cast<int32_t *>(c.dbuf + wb),
                                   reinterpret_cast<int32_t *>(c.dbuf + wb + eb), c.s);
    if (rc) return rc;
    LDPC_HIP(hipMemcpyAsync(c.pin, c.dbuf, wb + eb + 4, hipMemcpyDeviceToHost, c.s));
    LDPC_HIP(hipStreamSynchronize(c.s));
    for (int v = 0; v < n; ++v) Mvc[v] = pw[v];
    memcpy(errors, c.pin + wb, eb);
    int32_t it = 0;
    memcpy(&it, c.pin + wb + eb, 4);
    return it;
}

// --------------------------- soft ------------------------------------------
int ldpc_bp_decode_batch_dev(const ldpc_graph *g, const float *d_llr, int B, int max_iters, int algo, float alpha,
                             int early_stop, float *d_post, uint8_t *d_hard, int32_t *d_its, void *stream) {
    LDPC_REQUIRE(g && (B == 0 || d_llr) && B >= 0 && max_iters >= 0, "bad soft batch arguments");
    LDPC_REQUIRE(algo == LDPC_ALGO_SPA || algo == LDPC_ALGO_MINSUM, "algo must be LDPC_ALGO_SPA or LDPC_ALGO_MINSUM");
    if (!g->consistent) {
        set_error("soft decoding needs consistent edge lists (each (v,c) pair listed equally often on both sides)");
        return LDPC_EINVAL;
    }
    if (!strcmp(bp_kernel_name(*g, early_stop), "none")) {
        set_error("no soft kernel for this graph (check degree > 32)");
        return LDPC_EUNSUP;
    }
    if (B == 0) return LDPC_OK;
    float *scratch = nullptr;
    const size_t sb = bp_scratch_bytes(*g, B, max_iters, algo, early_stop && d_post);
    if (sb) {
        std::lock_guard<std::mutex> lk(g_mu);
        Workspace &ws = workspace(stream);
        std::lock_guard<std::mutex> wl(ws.mu);
        LDPC_HIP(ws.scratch.ensure(sb));
        scratch = static_cast<float *>(ws.scratch.p);
    }
    LDPC_HIP(launch_bp_decode(*g, d_llr, B, max_iters, algo, alpha, early_stop, d_post, d_hard, d_its,
                              static_cast<hipStream_t>(stream), scratch, sb));
    return LDPC_OK;
}

int ldpc_bp_decode_batch(const int32_t *variable_to_check_list, const int32_t *check_to_variable_list, int n, int k,
                         int dv, int dc, const float *llr, int B, int max_iters, int algo, float alpha,
                         int early_stop, float *post, uint8_t *hard, int32_t *its) {
    LDPC_REQUIRE((B == 0 || llr) && B >= 0, "bad soft batch arguments");
    LDPC_REQUIRE(algo == LDPC_ALGO_SPA || algo == LDPC_ALGO_MINSUM, "algo must be LDPC_ALGO_SPA or LDPC_ALGO_MINSUM");
    ldpc_graph *g = nullptr;
    int rc = ldpc_graph_create(variable_to_check_list, check_to_variable_list, n, k, dv, dc, &g);
    if (rc) return rc;
    if (B == 0) {  // validated graph, nothing to decode
        ldpc_graph_destroy(g);
        return LDPC_OK;
    }
    {
        std::lock_guard<std::mutex> lk(g_mu);
        Workspace &ws = workspace(nullptr);
        std::lock_guard<std::mutex> wl(ws.mu);
        const size_t nb = (size_t)B * n;
        hipError_t e = ws.llr.ensure(nb * 4);
        if (e == hipSuccess) e = ws.post.ensure(nb * 4);
        if (e == hipSuccess) e = ws.hard.ensure(nb);
        if (e == hipSuccess) e = ws.itsb.ensure((size_t)B * 4 + 4);
        if (e == hipSuccess) e = hipMemcpy(ws.llr.p, llr, nb * 4, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            ldpc_graph_destroy(g);
            set_error(std::string("soft batch staging: ") + hipGetErrorString(e));
            return LDPC_EHIP;
        }
        float *dl = static_cast<float *>(ws.llr.p), *dp = static_cast<float *>(ws.post.p);
        uint8_t *dh = static_cast<uint8_t *>(ws.hard.p);
        int32_t *di = static_cast<int32_t *>(ws.itsb.p);
        rc = 0;
        // scratch taken inside the _dev call (needs the lock released)
        if (e == hipSuccess) e = ws.scratch.ensure(bp_scratch_bytes(*g, B, max_iters, algo, early_stop && post));
        if (B > 0) {
            // no posteriors asked for: early stop may take the hard-decision path (bp_loc_kernel)
            e = launch_bp_decode(*g, dl, B, max_iters, algo, alpha, early_stop, post ? dp : nullptr, dh, di, nullptr,
                                 static_cast<float *>(ws.scratch.p), ws.scratch.cap);
            if (e == hipSuccess) e = hipDeviceSynchronize();
            if (e == hipSuccess && post) e = hipMemcpy(post, dp, nb * 4, hipMemcpyDeviceToHost);
            if (e == hipSuccess && hard) e = hipMemcpy(hard, dh, nb, hipMemcpyDeviceToHost);
            if (e == hipSuccess && its) e = hipMemcpy(its, di, (size_t)B * 4, hipMemcpyDeviceToHost);
            if (e != hipSuccess) {
                set_error(std::string("soft batch: ") + hipGetErrorString(e));
                rc = LDPC_EHIP;
            }
        }
    }
    ldpc_graph_destroy(g);
    return rc;
}

// --------------------------- channels / MC ---------------------------------
static int channel_params(int channel, float param, float *p, float *p2) {
    LDPC_REQUIRE(channel >= 0 && channel <= 2, "channel must be LDPC_CH_BEC, LDPC_CH_BSC or LDPC_CH_AWGN");
    *p = param;
    *p2 = 0.0f;
    if (channel == LDPC_CH_BSC) {
        LDPC_REQUIRE(param > 0.0f && param < 0.5f, "BSC crossover probability must be in (0, 0.5)");
        *p2 = (float)std::log((1.0 - (double)param) / (double)param);
    } else if (channel == LDPC_CH_AWGN) {
        LDPC_REQUIRE(param > 0.0f, "AWGN sigma must be > 0");
        *p2 = (float)(2.0 / ((double)param * (double)param));
    } else {
        LDPC_REQUIRE(param >= 0.0f && param <= 1.0f, "erasure probability must be in [0, 1]");
    }
    return LDPC_OK;
}

int ldpc_channel_dev(int channel, float param, uint64_t seed, uint64_t first_cw, int n, int B, void *d_out,
                     void *stream) {
    LDPC_REQUIRE((B == 0 || d_out) && n > 0 && B >= 0, "bad channel arguments");
    float p, p2;
    int rc = channel_params(channel, param, &p, &p2);
    if (rc) return rc;
    if (B == 0) return LDPC_OK;
    LDPC_HIP(launch_channel(channel, p, p2, seed, first_cw, n, B, d_out, static_cast<hipStream_t>(stream)));
    return LDPC_OK;
}

int ldpc_mc_batch_dev(const ldpc_graph *g, int channel, float param, uint64_t seed, uint64_t first_cw, int B,
                      int max_iters, int algo, float alpha, int early_stop, int expurgation,
                      int64_t stop_frame_errors, int64_t *d_counters, void *stream) {
    LDPC_REQUIRE(g && d_counters && B >= 0 && max_iters >= 0, "bad MC arguments");
    float p, p2;
    int rc = channel_params(channel, param, &p, &p2);
    if (rc) return rc;
    if (channel != LDPC_CH_BEC) {
        LDPC_REQUIRE(algo == LDPC_ALGO_SPA || algo == LDPC_ALGO_MINSUM, "bad algo");
        LDPC_REQUIRE(g->consistent, "soft decoding needs consistent edge lists");
    }
    if (B == 0) return LDPC_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    Workspace &ws = workspace(stream);  // this (device, stream)'s lock only: devices launch in parallel
    std::lock_guard<std::mutex> wl(ws.mu);
    LDPC_HIP(ws.trial.ensure(sizeof(int32_t) * (size_t)B * (max_iters + 1)));
    LDPC_HIP(ws.its.ensure(sizeof(int32_t) * (size_t)B));
    LDPC_HIP(ws.cutoff.ensure(16));
    float *scratch = nullptr;
    size_t sbytes = 0;
    if (channel != LDPC_CH_BEC) {
        const size_t sb = bp_scratch_bytes(*g, B, max_iters, algo, false);
        if (sb) {
            LDPC_HIP(ws.scratch.ensure(sb));
            scratch = static_cast<float *>(ws.scratch.p);
            sbytes = ws.scratch.cap;
        }
    }
    int32_t *trial = static_cast<int32_t *>(ws.trial.p), *its = static_cast<int32_t *>(ws.its.p);
    LDPC_HIP(launch_mc_decode(*g, channel, p, p2, seed, first_cw, B, max_iters, algo, alpha, early_stop, trial, its,
                              s, scratch, sbytes));
    LDPC_HIP(launch_mc_reduce(trial, its, B, max_iters, expurgation, stop_frame_errors, d_counters,
                              static_cast<int32_t *>(ws.cutoff.p), s));
    return LDPC_OK;
}

// --------------------------- random graphs / ensemble MC -------------------
static int check_regular_shape(int n, int dv, int dc) {
    LDPC_REQUIRE(n > 0 && dv > 0 && dc > 1 && (long)n * dv % dc == 0 && (long)n * dv < (1L << 30),
                 "need n*dv divisible by dc (regular configuration model)");
    return LDPC_OK;
}

int ldpc_sample_regular_dev(int n, int dv, int dc, uint64_t seed, uint64_t first_graph, int G,
                            int32_t *d_check_lookup, int32_t *d_variable_lookup, int32_t *d_attempts, void *stream) {
    int rc = check_regular_shape(n, dv, dc);
    if (rc) return rc;
    LDPC_REQUIRE(d_check_lookup && d_variable_lookup && G >= 0, "bad sampler arguments");
    rc = require_device();
    if (rc) return rc;
    Workspace &ws = workspace(stream);
    std::lock_guard<std::mutex> wl(ws.mu);
    LDPC_HIP(ws.sctl.ensure(4 * sample_ctl_words(G)));
    LDPC_HIP(launch_sample_regular(n, dv, dc, seed, first_graph, G, d_check_lookup, d_variable_lookup, d_attempts,
                                   1 << 20, static_cast<uint32_t *>(ws.sctl.p), static_cast<hipStream_t>(stream)));
    return LDPC_OK;
}

int ldpc_debug_seq_stats(uint64_t *out, int reset) {
    LDPC_REQUIRE(out, "null output");
    int rc = require_device();
    if (rc) return rc;
    const hipError_t e = seq_stats(out, reset);
    if (e == hipErrorNotSupported) {
        set_error("sampler statistics need a -DLDPC_SEQ_STATS=1 build");
        return LDPC_EUNSUP;
    }
    LDPC_HIP(e);
    return LDPC_OK;
}

int ldpc_debug_peel_stats(uint64_t *out, int reset) {
    LDPC_REQUIRE(out, "null output");
    int rc = require_device();
    if (rc) return rc;
    LDPC_HIP(peel_stats(out, reset));
    return LDPC_OK;
}

int ldpc_debug_peel_cap(int F) {
    peel_cap(F);
    return LDPC_OK;
}

int ldpc_sample_regular(int n, int dv, int dc, uint64_t seed, uint64_t first_graph, int G, int32_t *check_lookup,
                        int32_t *variable_lookup, int32_t *attempts) {
    int rc = check_regular_shape(n, dv, dc);
    if (rc) return rc;
    LDPC_REQUIRE(check_lookup && variable_lookup && G >= 0, "bad sampler arguments");
    rc = require_device();
    if (rc) return rc;
    const size_t E = (size_t)n * dv;
    std::lock_guard<std::mutex> lk(g_mu);
    Workspace &ws = workspace(nullptr);
    std::lock_guard<std::mutex> wl(ws.mu);
    LDPC_HIP(ws.gchk.ensure(E * G * 4));
    LDPC_HIP(ws.gvar.ensure(E * G * 4));
    LDPC_HIP(ws.gatt.ensure((size_t)G * 4 + 4));
    LDPC_HIP(ws.sctl.ensure(4 * sample_ctl_words(G)));
    LDPC_HIP(launch_sample_regular(n, dv, dc, seed, first_graph, G, static_cast<int32_t *>(ws.gchk.p),
                                   static_cast<int32_t *>(ws.gvar.p), static_cast<int32_t *>(ws.gatt.p), 1 << 20,
                                   static_cast<uint32_t *>(ws.sctl.p), nullptr));
    LDPC_HIP(hipDeviceSynchronize());
    LDPC_HIP(hipMemcpy(check_lookup, ws.gchk.p, E * G * 4, hipMemcpyDeviceToHost));
    LDPC_HIP(hipMemcpy(variable_lookup, ws.gvar.p, E * G * 4, hipMemcpyDeviceToHost));
    if (attempts) LDPC_HIP(hipMemcpy(attempts, ws.gatt.p, (size_t)G * 4, hipMemcpyDeviceToHost));
    return LDPC_OK;
}

// Irregular configuration model: degree structure (host arrays) -> device shape buffer
// [vsock E | cptr m+1 | vptr n+1] on the workspace of `stream` (caller holds g_mu).
static int csr_shape_upload(int n, int m, const int32_t *var_ptr, const int32_t *check_ptr, Workspace &ws,
                            void *stream, int *E_out, const int32_t **vsock, const int32_t **cptr,
                            const int32_t **vptr, int *max_cdeg, int *max_vdeg) {
    LDPC_REQUIRE(n > 0 && m > 0 && var_ptr && check_ptr, "bad degree structure");
    LDPC_REQUIRE(var_ptr[0] == 0 && check_ptr[0] == 0, "var_ptr / check_ptr must start at 0");
    *max_cdeg = *max_vdeg = 0;
    for (int v = 0; v < n; ++v) {
        LDPC_REQUIRE(var_ptr[v + 1] >= var_ptr[v], "var_ptr must be non-decreasing");
        *max_vdeg = std::max(*max_vdeg, var_ptr[v + 1] - var_ptr[v]);
    }
    for (int c = 0; c < m; ++c) {
        LDPC_REQUIRE(check_ptr[c + 1] >= check_ptr[c], "check_ptr must be non-decreasing");
        *max_cdeg = std::max(*max_cdeg, check_ptr[c + 1] - check_ptr[c]);
    }
    const int E = var_ptr[n];
    LDPC_REQUIRE(E > 0 && E == check_ptr[m], "socket counts differ: var_ptr[n] != check_ptr[m]");
    std::vector<int32_t> h((size_t)E + m + 1 + n + 1);
    for (int v = 0; v < n; ++v)
        for (int e = var_ptr[v]; e < var_ptr[v + 1]; ++e) h[e] = v;
    std::copy(check_ptr, check_ptr + m + 1, h.begin() + E);
    std::copy(var_ptr, var_ptr + n + 1, h.begin() + E + m + 1);
    // an earlier sampler launch on this stream may still read the shape buffer
    LDPC_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    LDPC_HIP(ws.shape.ensure(h.size() * 4));
    LDPC_HIP(hipMemcpy(ws.shape.p, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    const int32_t *base = static_cast<const int32_t *>(ws.shape.p);
    *E_out = E;
    *vsock = base;
    *cptr = base + E;
    *vptr = base + E + m + 1;
    return LDPC_OK;
}

int ldpc_sample_csr_dev(int n, int m, const int32_t *var_ptr, const int32_t *check_ptr, uint64_t seed,
                        uint64_t first_graph, int G, int32_t *d_check_var, int32_t *d_var_slot, int32_t *d_attempts,
                        void *stream) {
    LDPC_REQUIRE(d_check_var && d_var_slot && G >= 0, "bad sampler arguments");
    int rc = require_device();
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_mu);
    Workspace &ws = workspace(stream);
    std::lock_guard<std::mutex> wl(ws.mu);
    int E = 0, mxc = 0, mxv = 0;
    const int32_t *vs, *cp, *vp;
    rc = csr_shape_upload(n, m, var_ptr, check_ptr, ws, stream, &E, &vs, &cp, &vp, &mxc, &mxv);
    if (rc) return rc;
    LDPC_HIP(ws.sctl.ensure(4 * sample_ctl_words(G)));
    LDPC_HIP(launch_sample_csr(n, m, E, vs, cp, vp, mxc, mxv, seed, first_graph, G, d_check_var, d_var_slot, d_attempts,
                               1 << 20, static_cast<uint32_t *>(ws.sctl.p), static_cast<hipStream_t>(stream)));
    return LDPC_OK;
}

int ldpc_sample_csr(int n, int m, const int32_t *var_ptr, const int32_t *check_ptr, uint64_t seed,
                    uint64_t first_graph, int G, int32_t *check_var, int32_t *var_slot, int32_t *attempts) {
    LDPC_REQUIRE(check_var && var_slot && G >= 0, "bad sampler arguments");
    int rc = require_device();
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_mu);
    Workspace &ws = workspace(nullptr);
    std::lock_guard<std::mutex> wl(ws.mu);
    int E = 0, mxc = 0, mxv = 0;
    const int32_t *vs, *cp, *vp;
    rc = csr_shape_upload(n, m, var_ptr, check_ptr, ws, nullptr, &E, &vs, &cp, &vp, &mxc, &mxv);
    if (rc) return rc;
    LDPC_HIP(ws.gchk.ensure((size_t)E * G * 4));
    LDPC_HIP(ws.gvar.ensure((size_t)E * G * 4));
    LDPC_HIP(ws.gatt.ensure((size_t)G * 4 + 4));
    LDPC_HIP(ws.sctl.ensure(4 * sample_ctl_words(G)));
    LDPC_HIP(launch_sample_csr(n, m, E, vs, cp, vp, mxc, mxv, seed, first_graph, G, static_cast<int32_t *>(ws.gchk.p),
                               static_cast<int32_t *>(ws.gvar.p), static_cast<int32_t *>(ws.gatt.p), 1 << 20,
                               static_cast<uint32_t *>(ws.sctl.p), nullptr));
    LDPC_HIP(hipDeviceSynchronize());
    LDPC_HIP(hipMemcpy(check_var, ws.gchk.p, (size_t)E * G * 4, hipMemcpyDeviceToHost));
    LDPC_HIP(hipMemcpy(var_slot, ws.gvar.p, (size_t)E * G * 4, hipMemcpyDeviceToHost));
    if (attempts) LDPC_HIP(hipMemcpy(attempts, ws.gatt.p, (size_t)G * 4, hipMemcpyDeviceToHost));
    return LDPC_OK;
}

int ldpc_mc_ensemble_batch_dev(int n, int dv, int dc, int channel, float param, uint64_t seed, uint64_t first_cw,
                               int B, int max_iters, int expurgation, int64_t stop_frame_errors, int64_t *d_counters,
                               void *stream) {
    int rc = check_regular_shape(n, dv, dc);
    if (rc) return rc;
    LDPC_REQUIRE(channel == LDPC_CH_BEC, "ensemble Monte-Carlo is BEC-only (as parallel_simulator.py:168-272)");
    LDPC_REQUIRE(d_counters && B >= 0 && max_iters >= 0, "bad MC arguments");
    float p, p2;
    rc = channel_params(channel, param, &p, &p2);
    if (rc) return rc;
    rc = require_device();
    if (rc) return rc;
    if (B == 0) return LDPC_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t E = (size_t)n * dv;
    Workspace &ws = workspace(stream);  // this (device, stream)'s lock only: devices launch in parallel
    std::lock_guard<std::mutex> wl(ws.mu);
    LDPC_HIP(ws.gchk.ensure(E * B * 4));
    LDPC_HIP(ws.gvar.ensure(E * B * 4));
    LDPC_HIP(ws.trial.ensure(sizeof(int32_t) * (size_t)B * (max_iters + 1)));
    LDPC_HIP(ws.its.ensure(sizeof(int32_t) * (size_t)B));
    LDPC_HIP(ws.cutoff.ensure(16));
    int32_t *chk = static_cast<int32_t *>(ws.gchk.p), *var = static_cast<int32_t *>(ws.gvar.p);
    int32_t *trial = static_cast<int32_t *>(ws.trial.p), *its = static_cast<int32_t *>(ws.its.p);
    LDPC_HIP(ws.sctl.ensure(4 * sample_ctl_words(B)));
    LDPC_HIP(launch_sample_regular(n, dv, dc, seed, first_cw, B, chk, var, nullptr, 1 << 20,
                                   static_cast<uint32_t *>(ws.sctl.p), s));
    LDPC_HIP(launch_mc_bec_ensemble(n, dv, dc, chk, var, p, seed, first_cw, B, max_iters, trial, its, s));
    LDPC_HIP(launch_mc_reduce(trial, its, B, max_iters, expurgation, stop_frame_errors, d_counters,
                              static_cast<int32_t *>(ws.cutoff.p), s));
    return LDPC_OK;
}

// --------------------------- ML ("optimal") erasure decoding ---------------
static int ml_check_shape(int n, int m) {
    LDPC_REQUIRE(m >= 1 && m <= 1000, "ML decoding supports 1 <= n-k <= 1000 checks");
    LDPC_REQUIRE(n >= 1 && n <= 32767, "ML decoding supports n <= 32767");
    return LDPC_OK;
}

int ldpc_ml_decode_batch_dev(const ldpc_graph *g, const uint8_t *d_words, int B, uint8_t *d_out,
                             int32_t *d_unsolved, void *stream) {
    LDPC_REQUIRE(g && (B == 0 || (d_words && d_out && d_unsolved)) && B >= 0, "bad ML batch arguments");
    int rc = ml_check_shape(g->n, g->m);
    if (rc) return rc;
    if (B == 0) return LDPC_OK;
    LDPC_HIP(launch_ml_decode(g->cptr, g->cvar, 0, 0, g->n, g->m, d_words, B, d_out, d_unsolved,
                              static_cast<hipStream_t>(stream)));
    return LDPC_OK;
}

int ldpc_ml_decode_batch(const ldpc_graph *g, const uint8_t *words, int B, uint8_t *out, int32_t *unsolved) {
    LDPC_REQUIRE(g && (B == 0 || (words && out && unsolved)) && B >= 0, "bad ML batch arguments");
    int rc = ml_check_shape(g->n, g->m);
    if (rc) return rc;
    if (B == 0) return LDPC_OK;
    const size_t bytes = (size_t)B * g->n;
    std::lock_guard<std::mutex> lk(g_mu);
    Workspace &ws = workspace(nullptr);
    std::lock_guard<std::mutex> wl(ws.mu);
    LDPC_HIP(ws.mlw.ensure(bytes));
    LDPC_HIP(ws.mlo.ensure(bytes));
    LDPC_HIP(ws.mlu.ensure(sizeof(int32_t) * (size_t)B));
    uint8_t *dw = static_cast<uint8_t *>(ws.mlw.p), *dout = static_cast<uint8_t *>(ws.mlo.p);
    int32_t *du = static_cast<int32_t *>(ws.mlu.p);
    LDPC_HIP(hipMemcpy(dw, words, bytes, hipMemcpyHostToDevice));
    LDPC_HIP(launch_ml_decode(g->cptr, g->cvar, 0, 0, g->n, g->m, dw, B, dout, du, nullptr));
    LDPC_HIP(hipDeviceSynchronize());
    LDPC_HIP(hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost));
    LDPC_HIP(hipMemcpy(unsolved, du, sizeof(int32_t) * (size_t)B, hipMemcpyDeviceToHost));
    return LDPC_OK;
}

int ldpc_ml_ensemble_decode_dev(int n, int dv, int dc, const int32_t *d_check_lookup, const uint8_t *d_words, int B,
                                uint8_t *d_out, int32_t *d_unsolved, void *stream) {
    int rc = check_regular_shape(n, dv, dc);
    if (rc) return rc;
    LDPC_REQUIRE((B == 0 || (d_check_lookup && d_words && d_out && d_unsolved)) && B >= 0, "bad ML batch arguments");
    rc = ml_check_shape(n, n * dv / dc);
    if (rc) return rc;
    rc = require_device();
    if (rc) return rc;
    if (B == 0) return LDPC_OK;
    LDPC_HIP(launch_ml_decode(nullptr, d_check_lookup, (int64_t)n * dv, dc, n, n * dv / dc, d_words, B, d_out,
                              d_unsolved, static_cast<hipStream_t>(stream)));
    return LDPC_OK;
}

int ldpc_mc_ml_batch_dev(const ldpc_graph *g, int n, int dv, int dc, float eps, uint64_t seed, uint64_t first_cw,
                         int B, int max_iters, int message_passing, int expurgation, int64_t stop_frame_errors,
                         int64_t *d_counters_mp, int64_t *d_counters_ml, void *stream) {
    LDPC_REQUIRE(d_counters_ml && B >= 0 && max_iters >= 0, "bad MC arguments");
    LDPC_REQUIRE(!message_passing || d_counters_mp, "message_passing needs d_counters_mp");
    float p, p2;
    int rc = channel_params(LDPC_CH_BEC, eps, &p, &p2);
    if (rc) return rc;
    const bool ens = (g == nullptr);
    if (ens) {
        rc = check_regular_shape(n, dv, dc);
        if (rc) return rc;
        rc = require_device();
        if (rc) return rc;
    } else {
        n = g->n;
    }
    const int m = ens ? n * dv / dc : g->m;
    rc = ml_check_shape(n, m);
    if (rc) return rc;
    if (B == 0) return LDPC_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    Workspace &ws = workspace(stream);  // this (device, stream)'s lock only
    std::lock_guard<std::mutex> wl(ws.mu);
    LDPC_HIP(ws.mlw.ensure((size_t)B * n));
    LDPC_HIP(ws.mlo.ensure((size_t)B * n));
    LDPC_HIP(ws.mlu.ensure(sizeof(int32_t) * (size_t)B));
    LDPC_HIP(ws.cutoff.ensure(16));
    uint8_t *dw = static_cast<uint8_t *>(ws.mlw.p), *dout = static_cast<uint8_t *>(ws.mlo.p);
    int32_t *du = static_cast<int32_t *>(ws.mlu.p), *cut = static_cast<int32_t *>(ws.cutoff.p);
    int32_t *chk = nullptr, *var = nullptr;
    if (ens) {
        const size_t E = (size_t)n * dv;
        LDPC_HIP(ws.gchk.ensure(E * B * 4));
        LDPC_HIP(ws.gvar.ensure(E * B * 4));
        chk = static_cast<int32_t *>(ws.gchk.p);
        var = static_cast<int32_t *>(ws.gvar.p);
        LDPC_HIP(ws.sctl.ensure(4 * sample_ctl_words(B)));
        LDPC_HIP(launch_sample_regular(n, dv, dc, seed, first_cw, B, chk, var, nullptr, 1 << 20,
                                       static_cast<uint32_t *>(ws.sctl.p), s));
    }
    // channel words of trials first_cw.. (the same Philox draws the fused BP kernels make)
    LDPC_HIP(launch_channel(LDPC_CH_BEC, p, p2, seed, first_cw, n, B, dw, s));
    if (ens)
        LDPC_HIP(launch_ml_decode(nullptr, chk, (int64_t)n * dv, dc, n, m, dw, B, dout, du, s));
    else
        LDPC_HIP(launch_ml_decode(g->cptr, g->cvar, 0, 0, n, m, dw, B, dout, du, s));
    if (message_passing) {
        LDPC_HIP(ws.trial.ensure(sizeof(int32_t) * (size_t)B * (max_iters + 1)));
        LDPC_HIP(ws.its.ensure(sizeof(int32_t) * (size_t)B));
        int32_t *trial = static_cast<int32_t *>(ws.trial.p), *its = static_cast<int32_t *>(ws.its.p);
        if (ens)
            LDPC_HIP(launch_mc_bec_ensemble(n, dv, dc, chk, var, p, seed, first_cw, B, max_iters, trial, its, s));
        else
            LDPC_HIP(launch_mc_decode(*g, LDPC_CH_BEC, p, p2, seed, first_cw, B, max_iters, 0, 1.0f, 0, trial, its,
                                      s, nullptr, 0));
        // the stop rule counts message-passing frame errors (parallel_simulator.py:226-231)
        LDPC_HIP(launch_mc_reduce(trial, its, B, max_iters, expurgation, stop_frame_errors, d_counters_mp, cut, s));
        LDPC_HIP(launch_mc_reduce_cut(du, nullptr, B, 0, -1, cut, d_counters_ml, s));
    } else {
        // ML only: the stop rule counts ML frame errors (:240-241)
        LDPC_HIP(launch_mc_reduce(du, nullptr, B, 0, -1, stop_frame_errors, d_counters_ml, cut, s));
    }
    return LDPC_OK;
}

}  // extern "C"
