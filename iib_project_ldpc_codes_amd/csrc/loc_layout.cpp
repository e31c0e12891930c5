// Local-edge layout of bp_loc_kernel (ldpc_kernels.hip), built on the host.
// (cls_d[k] = dy, or dy | dx << 8 for a mixed class: see "checks sorted by degree".)
//
// Every variable gets ONE "local" edge: a perfect b-matching pairs each check with exactly
// two of its variables (greedy + augmenting paths on variables x check slots), and a check pair's
// four local variables live in the thread that updates that check pair.  A local edge's
// message then never leaves that thread's registers: the check phase reads and writes it
// as the check's input / output and the variable phase as the variable's.  Only the other
// E - n edges go through LDS -- a third of the LDS traffic of a (3,6) code, and the
// messages of the irregular rate-1/2 ensembles (E = 57 k at n = 20,000) fit in one CU's
// LDS.  Requires n = 2m (rate-1/2 designs), m even, check degrees 2..8 in at most
// kLocMaxCls classes of pairs, variable degrees 1..4.
//
// Check pairs: checks sorted by degree (classes contiguous), consecutive checks of one
// class form pair q; thread t owns pairs t, t + T, ...  Non-local slot u (0 .. D-3) of
// the pair's checks (h = 0 / 1) sits at LDS word
//     W_c + (u/2)*4*N_c + 4i + 2(u%2) + h     (u < 2*floor((D-2)/2): float4 rows)
//     W_c + (D-2)/2*4*N_c + 2i + h            (u = D-3 for odd D-2: a float2 row)
// (class c: degree D, N_c pairs, first word W_c, i = q - first pair of the class), so
// every row is read / written lane-contiguously by ds_read_b128 / ds_read_b64.
// Variables: thread t's var pair v = 2k + s (k = its k-th pair, s = local slot) holds the
// two checks' s-th local variables (.x check 2q-side h = 0, .y h = 1); its non-local edges
// in variable_to_check_list order are gathered from the positions above.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <deque>
#include <vector>

#include "ldpc_internal.hpp"

#ifndef LDPC_LOC_SEARCH
#define LDPC_LOC_SEARCH 10  // local-search moves per edge of the bank-conflict pass (0: off)
#endif
#ifndef LDPC_LOC_T0
#define LDPC_LOC_T0 0.0  // annealing start temperature of that pass (0: greedy)
#endif

namespace {
// Assign every left node to one right node of its adjacency, right node r taking at most
// cap[r] of them.  Greedy (fewest candidates first), then BFS augmenting paths.
bool assign(const std::vector<std::vector<int>> &adj, std::vector<int> cap, int NR, std::vector<int> &to) {
    const int NL = (int)adj.size();
    std::vector<std::vector<int>> held(NR);
    std::vector<int> order(NL);
    to.assign(NL, -1);
    for (int v = 0; v < NL; ++v) order[v] = v;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return adj[a].size() < adj[b].size(); });
    for (int v : order)
        for (int c : adj[v])
            if (cap[c] > 0) {
                --cap[c];
                held[c].push_back(v);
                to[v] = c;
                break;
            }
    // augment: BFS over left nodes; from v try each right node c; free capacity ends the
    // path, otherwise continue from the left nodes c holds
    std::vector<int> from_v(NL), via_c(NL), mark(NL, -1);
    for (int root = 0; root < NL; ++root) {
        if (to[root] >= 0) continue;
        std::deque<int> qu{root};
        mark[root] = root;
        from_v[root] = -1;
        int end_v = -1, end_c = -1;
        while (!qu.empty() && end_v < 0) {
            const int v = qu.front();
            qu.pop_front();
            for (int c : adj[v]) {
                if (c == to[v]) continue;
                if (cap[c] > 0) { end_v = v; end_c = c; break; }
                for (int w : held[c])
                    if (mark[w] != root) {
                        mark[w] = root;
                        from_v[w] = v;
                        via_c[w] = c;  // v takes c, w leaves c
                        qu.push_back(w);
                    }
            }
        }
        if (end_v < 0) return false;
        // walk back: end_v takes end_c; each w (reached via c from from_v[w]) gives c to from_v[w]
        int v = end_v, c = end_c;
        --cap[c];
        while (v >= 0) {
            const int old = to[v];
            held[c].push_back(v);
            to[v] = c;
            if (old >= 0) held[old].erase(std::find(held[old].begin(), held[old].end(), v));
            if (from_v[v] < 0) break;
            c = via_c[v];  // the right node v gave up is the one its predecessor takes
            v = from_v[v];
        }
    }
    return true;
}

// Local edges: every variable to one of its checks, every check exactly two variables.
// First try to give every check one variable of the smallest degree (its local slot 0;
// the kernel then gathers fewer non-local edges for slot 0 -- fewer VGPRs), then the
// others; else a plain b-matching.  vloc[v] = check, slot0[c] = the min-degree variable
// or -1.
bool local_matching(int n, int m, const std::vector<int32_t> &cptr, const std::vector<int32_t> &cvar,
                    const std::vector<int32_t> &vptr, std::vector<int> &vloc, std::vector<int> &slot0) {
    std::vector<std::vector<int>> vch(n), cvs(m);
    for (int c = 0; c < m; ++c)
        for (int e = cptr[c]; e < cptr[c + 1]; ++e) {
            const int v = cvar[e];
            if (std::find(vch[v].begin(), vch[v].end(), c) == vch[v].end()) {
                vch[v].push_back(c);
                cvs[c].push_back(v);
            }
        }
    int dmin = 1 << 30;
    for (int v = 0; v < n; ++v) dmin = std::min(dmin, vptr[v + 1] - vptr[v]);
    slot0.assign(m, -1);
    {
        // stage A: each check one min-degree variable
        std::vector<std::vector<int>> adjA(m);
        for (int c = 0; c < m; ++c)
            for (int v : cvs[c])
                if (vptr[v + 1] - vptr[v] == dmin) adjA[c].push_back(v);
        std::vector<int> toA;
        if (assign(adjA, std::vector<int>(n, 1), n, toA)) {
            std::vector<char> used(n, 0);
            for (int c = 0; c < m; ++c) used[toA[c]] = 1;
            std::vector<int> rest;
            for (int v = 0; v < n; ++v)
                if (!used[v]) rest.push_back(v);
            std::vector<std::vector<int>> adjB(rest.size());
            for (size_t j = 0; j < rest.size(); ++j) adjB[j] = vch[rest[j]];
            std::vector<int> toB;
            if (assign(adjB, std::vector<int>(m, 1), m, toB)) {
                vloc.assign(n, -1);
                for (int c = 0; c < m; ++c) { vloc[toA[c]] = c; slot0[c] = toA[c]; }
                for (size_t j = 0; j < rest.size(); ++j) vloc[rest[j]] = toB[j];
                return true;
            }
        }
    }
    std::fill(slot0.begin(), slot0.end(), -1);
    return assign(vch, std::vector<int>(m, 2), m, vloc);
}
}  // namespace

bool build_loc_layout(int n, int m, const std::vector<int32_t> &cptr, const std::vector<int32_t> &cvar,
                      const std::vector<int32_t> &vptr, const std::vector<int32_t> &vslot, LocLayout &L) {
    if (n != 2 * m || m < 2) return false;
    int maxv = 0;
    for (int v = 0; v < n; ++v) maxv = std::max(maxv, vptr[v + 1] - vptr[v]);
    if (maxv < 1 || maxv > 4) return false;
    // checks sorted by degree; pair q = (corder[2q], corder[2q+1]); classes = runs of pairs
    // with equal degrees (dx, dy) -- a pair straddling two degrees is "mixed": its rows
    // are sized for dy and the smaller check (h = 0) leaves its extra rows as pads
    if (m % 2) return false;
    std::vector<int> corder(m);
    for (int c = 0; c < m; ++c) {
        const int d = cptr[c + 1] - cptr[c];
        if (d < 2 || d > kLocMaxD) return false;
        corder[c] = c;
    }
    std::stable_sort(corder.begin(), corder.end(),
                     [&](int x, int y) { return cptr[x + 1] - cptr[x] < cptr[y + 1] - cptr[y]; });
    std::vector<int> vloc, slot0;
    if (!local_matching(n, m, cptr, cvar, vptr, vloc, slot0)) return false;
    L.P = m / 2;
    L.ncls = 0;
    int w0 = 0;
    for (int q = 0; q < L.P; ++q) {
        const int dx = cptr[corder[2 * q] + 1] - cptr[corder[2 * q]];
        const int dy = cptr[corder[2 * q + 1] + 1] - cptr[corder[2 * q + 1]];
        const int code = dx == dy ? dy : (dy | (dx << 8));
        if (L.ncls == 0 || L.cls_d[L.ncls - 1] != code) {
            if (L.ncls == kLocMaxCls) return false;
            if (L.ncls) w0 += 2 * ((L.cls_d[L.ncls - 1] & 255) - 2) * (q - L.cls_q[L.ncls - 1]);
            L.cls_d[L.ncls] = code;
            L.cls_q[L.ncls] = q;
            L.cls_w[L.ncls] = w0;
            ++L.ncls;
        }
    }
    w0 += 2 * ((L.cls_d[L.ncls - 1] & 255) - 2) * (L.P - L.cls_q[L.ncls - 1]);
    L.cls_q[L.ncls] = L.P;
    L.cls_w[L.ncls] = w0;
    L.words = w0;
    // LDS word of every slot (-1: local), local slot index per variable
    std::vector<int32_t> word(cvar.size(), -1);
    std::vector<int> loc_s(n, -1);                 // local slot (0/1) of v in its check
    std::vector<int> loc_slot(n, -1);              // the CSR slot of v's local edge
    std::vector<int> loc_var(2 * (size_t)m, -1);   // [check][s]
    for (int k = 0; k < L.ncls; ++k) {
        const int D = L.cls_d[k] & 255, Nc = L.cls_q[k + 1] - L.cls_q[k], U = D - 2;
        for (int i = 0; i < Nc; ++i)
            for (int h = 0; h < 2; ++h) {
                const int c = corder[2 * (L.cls_q[k] + i) + h];
                const int Uc = cptr[c + 1] - cptr[c] - 2;  // < U for a mixed pair's smaller check
                int u = 0, s = 0;
                for (int e = cptr[c]; e < cptr[c + 1]; ++e) {
                    const int v = cvar[e];
                    if (vloc[v] == c && loc_slot[v] < 0) {  // the first occurrence is the local edge
                        const int sl = slot0[c] < 0 ? s : (v == slot0[c] ? 0 : 1);
                        loc_slot[v] = e;
                        loc_s[v] = sl;
                        loc_var[2 * (size_t)c + sl] = v;
                        ++s;
                        continue;
                    }
                    const int wd = (u < 2 * (U / 2)) ? L.cls_w[k] + (u / 2) * 4 * Nc + 4 * i + 2 * (u % 2) + h
                                                     : L.cls_w[k] + (U / 2) * 4 * Nc + 2 * i + h;
                    word[e] = wd;
                    ++u;
                }
                if (s != 2 || u != Uc) return false;
            }
    }
    L.DVN = maxv - 1;
    const int DVN = std::max(L.DVN, 1);
    L.DVN0 = 0;
    L.DVN1 = 0;
    for (int v = 0; v < n; ++v) {
        int &d = loc_s[v] == 0 ? L.DVN0 : L.DVN1;
        d = std::max(d, vptr[v + 1] - vptr[v] - 1);
    }
    L.ABS0 = L.ABS1 = false;
    for (int v = 0; v < n; ++v) {
        const int nd = vptr[v + 1] - vptr[v] - 1;
        if (loc_s[v] == 0) L.ABS0 |= nd != L.DVN0;
        else L.ABS1 |= nd != L.DVN1;
    }
    L.KP = (L.P + L.T - 1) / L.T;
    if (L.T == 512) L.KP = L.KP <= 5 ? 5 : (L.KP <= 8 ? 8 : 10);  // the instantiated 512-thread shapes
    if ((long)L.KP * L.T < L.P || L.words + 64 >= 65536) return false;  // beyond 16-bit words / the shapes
    // Bank-conflict search.  A variable's non-local edge u is gathered (and written) by
    // one instruction (var pair slot, u, half) of its thread; the 32 lanes of a half wave
    // conflict on LDS bank = word mod 32.  Cost = sum over (instruction, half wave) of the
    // busiest bank's extra lanes.  Moves (each applied only if it does not raise the cost;
    // optional annealing): (r) swap the rows of two non-local edges of one check -- the
    // check rule is symmetric; (h) swap the two checks of a pair -- their rows' word
    // parity and their local variables' halves; (p) swap two pairs of one degree class --
    // their rows and the threads holding their local variables.  Deterministic (fixed
    // xorshift seed).
    {
        const int G = L.T / 32, VP = 2 * L.KP;
        const size_t E = cvar.size();
        std::vector<int> urow(E, -1), cls_of_q(L.P), pos_in_check(m);
        std::vector<int> vslot_u(E, -1);  // var-side non-local index of the edge at slot e
        for (int k = 0; k < L.ncls; ++k)
            for (int q = L.cls_q[k]; q < L.cls_q[k + 1]; ++q) cls_of_q[q] = k;
        std::vector<int> qof(m), hof(m);
        auto place = [&]() {
            for (int q = 0; q < L.P; ++q)
                for (int h = 0; h < 2; ++h) { qof[corder[2 * q + h]] = q; hof[corder[2 * q + h]] = h; }
        };
        place();
        auto place_pair = [&](int q) {
            for (int h = 0; h < 2; ++h) { qof[corder[2 * q + h]] = q; hof[corder[2 * q + h]] = h; }
        };
        for (int c = 0; c < m; ++c) {
            int u = 0;
            for (int e = cptr[c]; e < cptr[c + 1]; ++e)
                if (word[e] >= 0) urow[e] = u++;
        }
        for (int v = 0; v < n; ++v) {
            int u = 0;
            for (int e = vptr[v]; e < vptr[v + 1]; ++e)
                if (vslot[e] != loc_slot[v]) vslot_u[vslot[e]] = u++;
        }
        std::vector<int> slot_check(E);
        for (int c = 0; c < m; ++c)
            for (int e = cptr[c]; e < cptr[c + 1]; ++e) slot_check[e] = c;
        auto wordf = [&](int e) {
            const int c = slot_check[e], q = qof[c], k = cls_of_q[q], D = L.cls_d[k] & 255, U = D - 2, u = urow[e];
            const int Nc = L.cls_q[k + 1] - L.cls_q[k], i = q - L.cls_q[k], h = hof[c];
            return (u < 2 * (U / 2)) ? L.cls_w[k] + (u / 2) * 4 * Nc + 4 * i + 2 * (u % 2) + h
                                     : L.cls_w[k] + (U / 2) * 4 * Nc + 2 * i + h;
        };
        auto cellf = [&](int e) {
            const int v = cvar[e], c = vloc[v], q = qof[c], t = q % L.T, vi = 2 * (q / L.T) + loc_s[v];
            return ((vi * DVN + vslot_u[e]) * 2 + hof[c]) * G + t / 32;
        };
        const size_t ncell = (size_t)VP * DVN * 2 * G;
        std::vector<int> cnt(ncell * 32, 0), cw(E, -1), cc(E, -1);
        for (size_t e = 0; e < E; ++e)
            if (urow[e] >= 0) {
                cw[e] = wordf((int)e);
                cc[e] = cellf((int)e);
                ++cnt[(size_t)cc[e] * 32 + (cw[e] & 31)];
            }
        // search objective: the busiest bank's extra lanes (the cycles) weighted, plus every
        // extra lane (smooth: a cell only gets cheaper once all its collisions are gone)
        auto cost = [&](int cl) {
            int mx = 0, ex = 0;
            for (int b = 0; b < 32; ++b) {
                const int c = cnt[(size_t)cl * 32 + b];
                mx = std::max(mx, c);
                ex += c > 1 ? c - 1 : 0;
            }
            return (mx > 0 ? mx - 1 : 0) * 8 + ex;
        };
        auto cycles = [&](int cl) {
            int mx = 0;
            for (int b = 0; b < 32; ++b) mx = std::max(mx, cnt[(size_t)cl * 32 + b]);
            return mx > 0 ? mx - 1 : 0;
        };
        std::vector<std::vector<int>> nl(m), vnl(n);  // non-local slots of each check / variable
        for (int c = 0; c < m; ++c)
            for (int e = cptr[c]; e < cptr[c + 1]; ++e)
                if (urow[e] >= 0) nl[c].push_back(e);
        for (size_t e = 0; e < E; ++e)
            if (urow[e] >= 0) vnl[cvar[e]].push_back((int)e);
        // affected edges of a set of checks: their non-local slots (words) and the non-local
        // edges of their local variables (cells)
        std::vector<int> aff, touched;
        std::vector<char> mark_e(E, 0);
        std::vector<int> mark_c(ncell, 0);
        int stamp = 0;
        auto collect = [&](const int *cs, int nc) {
            aff.clear();
            for (int j = 0; j < nc; ++j) {
                const int c = cs[j];
                for (int e : nl[c]) if (!mark_e[e]) { mark_e[e] = 1; aff.push_back(e); }
                for (int s2 = 0; s2 < 2; ++s2)
                    for (int e : vnl[loc_var[2 * (size_t)c + s2]]) if (!mark_e[e]) { mark_e[e] = 1; aff.push_back(e); }
            }
            for (int e : aff) mark_e[e] = 0;
        };
        auto cost_of = [&](const std::vector<int> &cells) {
            int sum = 0;
            for (int cl : cells) sum += cost(cl);
            return sum;
        };
        auto remove_aff = [&]() {
            ++stamp;
            touched.clear();
            for (int e : aff)
                if (mark_c[cc[e]] != stamp) { mark_c[cc[e]] = stamp; touched.push_back(cc[e]); }
            for (int e : aff) --cnt[(size_t)cc[e] * 32 + (cw[e] & 31)];
        };
        std::vector<int> old_w, old_c, new_w, new_c;
        uint64_t x = 0x9E3779B97F4A7C15ull;
        auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
        long moves = (long)E * LDPC_LOC_SEARCH;
        double T0 = LDPC_LOC_T0;
        if (const char *ev = getenv("LDPC_LOC_SEARCH")) moves = (long)E * atol(ev);  // experiments
        if (const char *ev = getenv("LDPC_LOC_T0")) T0 = atof(ev);
        for (long it = 0; it < moves; ++it) {
            const double temp = T0 * (1.0 - (double)it / (double)moves);
            const int kind = (int)(rnd() % 8);  // 0-5: row swap, 6: half swap, 7: pair swap
            int cs[4], ncs = 0, ea = -1, eb = -1, q1 = -1, q2 = -1;
            if (kind < 6) {
                const int c = (int)(rnd() % (uint64_t)m), U = (int)nl[c].size();
                if (U < 2) continue;
                ea = nl[c][rnd() % U];
                eb = nl[c][rnd() % U];
                if (ea == eb) continue;
                aff.assign({ea, eb});
            } else if (kind == 6) {
                q1 = (int)(rnd() % (uint64_t)L.P);
                if (L.cls_d[cls_of_q[q1]] >> 8) continue;  // a mixed pair keeps its smaller check at h = 0
                cs[ncs++] = corder[2 * q1];
                cs[ncs++] = corder[2 * q1 + 1];
                collect(cs, ncs);
            } else {
                q1 = (int)(rnd() % (uint64_t)L.P);
                const int k = cls_of_q[q1], Nc = L.cls_q[k + 1] - L.cls_q[k];
                q2 = L.cls_q[k] + (int)(rnd() % (uint64_t)Nc);
                if (q1 == q2) continue;
                cs[ncs++] = corder[2 * q1];
                cs[ncs++] = corder[2 * q1 + 1];
                cs[ncs++] = corder[2 * q2];
                cs[ncs++] = corder[2 * q2 + 1];
                collect(cs, ncs);
            }
            auto apply = [&]() {  // every move is its own inverse
                if (kind < 6) std::swap(urow[ea], urow[eb]);
                else if (kind == 6) { std::swap(corder[2 * q1], corder[2 * q1 + 1]); place_pair(q1); }
                else {
                    std::swap(corder[2 * q1], corder[2 * q2]);
                    std::swap(corder[2 * q1 + 1], corder[2 * q2 + 1]);
                    place_pair(q1);
                    place_pair(q2);
                }
            };
            // touched cells = the affected edges' cells before and after the move
            remove_aff();
            old_w.resize(aff.size());
            old_c.resize(aff.size());
            new_w.resize(aff.size());
            new_c.resize(aff.size());
            for (size_t j = 0; j < aff.size(); ++j) { old_w[j] = cw[aff[j]]; old_c[j] = cc[aff[j]]; }
            apply();
            for (size_t j = 0; j < aff.size(); ++j) {
                new_w[j] = wordf(aff[j]);
                new_c[j] = cellf(aff[j]);
                if (mark_c[new_c[j]] != stamp) { mark_c[new_c[j]] = stamp; touched.push_back(new_c[j]); }
            }
            apply();
            for (size_t j = 0; j < aff.size(); ++j) ++cnt[(size_t)old_c[j] * 32 + (old_w[j] & 31)];
            const int before = cost_of(touched);
            for (size_t j = 0; j < aff.size(); ++j) --cnt[(size_t)old_c[j] * 32 + (old_w[j] & 31)];
            for (size_t j = 0; j < aff.size(); ++j) ++cnt[(size_t)new_c[j] * 32 + (new_w[j] & 31)];
            const int after = cost_of(touched);
            const bool accept = after <= before ||
                                (temp > 0 && (double)(rnd() >> 11) * 0x1p-53 < exp((before - after) / temp));
            if (accept) {
                apply();
                for (size_t j = 0; j < aff.size(); ++j) { cw[aff[j]] = new_w[j]; cc[aff[j]] = new_c[j]; }
            } else {
                for (size_t j = 0; j < aff.size(); ++j) {
                    --cnt[(size_t)new_c[j] * 32 + (new_w[j] & 31)];
                    ++cnt[(size_t)old_c[j] * 32 + (old_w[j] & 31)];
                }
            }
        }
        long total = 0;
        for (size_t cl = 0; cl < ncell; ++cl) total += cycles((int)cl);
        L.conflicts = total;
        for (size_t e = 0; e < E; ++e)
            if (urow[e] >= 0) word[e] = wordf((int)e);
    }
    // thread layout
    const int VP = 2 * L.KP, T = L.T;
    L.var.assign((size_t)VP * 2 * T, -1);
    L.pos.assign((size_t)VP * DVN * T, 0);
    L.info.assign((size_t)VP * T, 0);
    const int dummy = L.words;  // + (t & 63): absent edges (their gathers are replaced by the neutral value)
    for (int t = 0; t < T; ++t)
        for (int kk = 0; kk < L.KP; ++kk) {
            const int q = t + kk * T;
            for (int s = 0; s < 2; ++s) {
                const int vi = 2 * kk + s;
                uint32_t info = 0, pk[4] = {0, 0, 0, 0};
                for (int h = 0; h < 2; ++h) {
                    int v = -1;
                    if (q < L.P) v = loc_var[2 * (size_t)corder[2 * q + h] + s];
                    L.var[((size_t)vi * 2 + h) * T + t] = v;
                    int u = 0, jl = 0;
                    if (v >= 0)
                        for (int e = vptr[v]; e < vptr[v + 1]; ++e) {
                            if (vslot[e] == loc_slot[v]) { jl = e - vptr[v]; continue; }
                            pk[u] |= (uint32_t)word[vslot[e]] << (16 * h);
                            info |= 1u << (u + 4 * h);
                            ++u;
                        }
                    for (; u < DVN; ++u) pk[u] |= (uint32_t)(dummy + (t & 63)) << (16 * h);
                    info |= (uint32_t)jl << (8 + 2 * h);
                    if (v >= 0 && jl < 4) info |= 1u << (16 + 4 * h + jl);  // one-hot copy (min-sum masks)
                }
                for (int u = 0; u < DVN; ++u) L.pos[((size_t)vi * DVN + u) * T + t] = (int32_t)pk[u];
                L.info[(size_t)vi * T + t] = (int32_t)info;
            }
        }
    return L.words + 64 < 65536;
}
