"""Irregular LDPC ensembles (lambda, rho) and their configuration-model graphs.

Extends the reference's regular (dv, dc) generator (random_code_generator.c:21-67)
to edge-perspective degree distributions, as SURVEY.md 8f-4 asks for config 4
(BASELINE.json configs[3]: irregular lambda/rho, n = 20000, BI-AWGN).  The law is
the reference's: a uniformly random socket matching, whole-graph redraw while a
check holds a variable twice.  Graphs come out in CSR slot form for
ldpc_graph_create_csr.

``RSU_DL4`` is the rate-1/2 ensemble with maximum variable degree 4 of
Richardson-Shokrollahi-Urbanke, "Design of capacity-approaching irregular LDPC
codes" (IEEE T-IT 2001); the BEC / BI-AWGN thresholds quoted in DESIGN.md are
computed by iib_project_ldpc_codes_amd.de, not taken from the paper.
"""
from dataclasses import dataclass

import numpy as np

from .graph import TannerGraph


@dataclass(frozen=True)
class Ensemble:
    """Edge-perspective degree distributions: lam[i] / rho[i] = fraction of edges
    attached to variable / check nodes of degree i (lam(x) = sum lam_i x^(i-1))."""
    lam: dict
    rho: dict

    def _int(self, d):
        return sum(f / i for i, f in d.items())

    @property
    def design_rate(self):
        return 1.0 - self._int(self.rho) / self._int(self.lam)

    def node_fractions(self, side="var"):
        d = self.lam if side == "var" else self.rho
        tot = self._int(d)
        return {i: (f / i) / tot for i, f in d.items()}

    def lam_poly(self, x):
        return sum(f * x ** (i - 1) for i, f in self.lam.items())

    def rho_poly(self, x):
        return sum(f * x ** (i - 1) for i, f in self.rho.items())


REGULAR_36 = Ensemble({3: 1.0}, {6: 1.0})
RSU_DL4 = Ensemble({2: 0.38354, 3: 0.04237, 4: 0.57409}, {5: 0.24123, 6: 0.75877})


def degree_sequences(ens, n):
    """Integer node-degree sequences with equal socket counts on both sides.
    Variables: n nodes split by node fraction (largest remainders); checks: sized so
    that sum of check degrees == sum of variable degrees."""
    def split(frac, total):
        keys = sorted(frac)
        raw = np.array([frac[k] * total for k in keys])
        cnt = np.floor(raw).astype(int)
        for idx in np.argsort(-(raw - cnt))[: total - cnt.sum()]:
            cnt[idx] += 1
        return np.repeat(np.array(keys), cnt)

    vdeg = split(ens.node_fractions("var"), n)
    E = int(vdeg.sum())
    cfrac = ens.node_fractions("check")
    mean_dc = sum(k * f for k, f in cfrac.items())
    m = int(round(E / mean_dc))
    cdeg = split(cfrac, m)
    # fix the socket count mismatch on the check side, one socket at a time
    diff = E - int(cdeg.sum())
    keys = sorted(cfrac)
    i = 0
    while diff != 0:
        j = i % m
        if diff > 0 and cdeg[j] < keys[-1]:
            cdeg[j] += 1
            diff -= 1
        elif diff < 0 and cdeg[j] > keys[0]:
            cdeg[j] -= 1
            diff += 1
        i += 1
    return vdeg.astype(np.int32), cdeg.astype(np.int32)


def sample_irregular(ens, n, seed=0, max_retries=100000, deg2="random", min_cycle=40):
    """Configuration-model graph of ``ens`` with n variables (host, numpy PCG64).

    deg2="random": every socket matched uniformly (the reference's law).  With a
    large fraction of degree-2 variables this leaves low-weight codewords -- two
    degree-2 variables on the same two checks, short cycles of degree-2 nodes --
    and an error floor (FER ~ 1e-1 for RSU_DL4 at n = 20000).
    deg2="zigzag": the degree-2 variables form a path through a random order of
    all checks (IRA-style) plus chords whose cycles through the path hold at
    least ``min_cycle`` degree-2 variables; the other variables are matched
    uniformly to the remaining check sockets.  Same degree distributions.  (The
    chord test covers cycles through one or two chords only: cycles through three
    or more chords, and codewords joining path segments through two degree-4
    variables, remain -- they set its error floor, see DESIGN.md.)
    deg2="path": a ring of m degree-2 variables through all checks and nothing
    else: degree-2 variables beyond m become degree 3 (their extra sockets raise
    the lowest check degrees, 5 -> 6), so the only all-degree-2 codeword is the
    whole ring (weight m) and every lighter one needs variables of degree >= 3;
    configs[3]'s code.  Each check then holds two degree-2 variables
    (bp_loc_kernel's local slot 0)."""
    if deg2 in ("zigzag", "path"):
        return _sample_zigzag(ens, n, seed, min_cycle, max_retries, chords=deg2 == "zigzag")
    vdeg, cdeg = degree_sequences(ens, n)
    rng = np.random.default_rng(seed)
    E = int(vdeg.sum())
    m = cdeg.size
    var_of_socket = np.repeat(np.arange(n, dtype=np.int32), vdeg)
    cptr = np.zeros(m + 1, np.int32)
    cptr[1:] = np.cumsum(cdeg)
    check_of_slot = np.repeat(np.arange(m, dtype=np.int32), cdeg)
    for _ in range(max_retries):
        cvar = var_of_socket[rng.permutation(E)]
        key = check_of_slot.astype(np.int64) * n + cvar
        if np.unique(key).size == E:  # no check holds a variable twice
            break
    else:
        raise RuntimeError("sample_irregular: too many redraws")
    # var side: each variable's edges in ascending check order
    order = np.lexsort((check_of_slot, cvar))
    vptr = np.zeros(n + 1, np.int32)
    vptr[1:] = np.cumsum(vdeg)
    vslot = order.astype(np.int32)
    return TannerGraph.from_csr(cptr, cvar.astype(np.int32), vptr, vslot)


def degree_ptrs(ens, n):
    """(var_ptr, check_ptr) of the degree sequences (sockets of variable v at
    var_ptr[v].., slots of check c at check_ptr[c]..)."""
    vdeg, cdeg = degree_sequences(ens, n)
    vptr = np.zeros(n + 1, np.int32)
    vptr[1:] = np.cumsum(vdeg)
    cptr = np.zeros(cdeg.size + 1, np.int32)
    cptr[1:] = np.cumsum(cdeg)
    return vptr, cptr


def sample_irregular_device(ens, n, seed=0, graph_id=0):
    """Graph `graph_id` of the on-device sampler (ldpc_sample_csr): the law of
    sample_irregular(deg2="random") -- uniform socket matching, whole-graph redraw
    while a check holds a variable twice -- drawn by the same counter-based
    generator as the regular device sampler (any graph can be regenerated)."""
    from . import _native
    vptr, cptr = degree_ptrs(ens, n)
    E = int(vptr[-1])
    cvar = np.zeros(E, np.int32)
    vslot = np.zeros(E, np.int32)
    att = np.zeros(1, np.int32)
    rc = _native.lib().ldpc_sample_csr(n, len(cptr) - 1, vptr.ctypes.data, cptr.ctypes.data, int(seed),
                                       int(graph_id), 1, cvar.ctypes.data, vslot.ctypes.data, att.ctypes.data)
    _native.check(rc, "ldpc_sample_csr")
    if att[0] <= 0:
        raise RuntimeError("sampler hit its attempt cap")
    return TannerGraph.from_csr(cptr, cvar, vptr, vslot)


def _csr_from_pairs(n, m, cdeg, var_check_pairs):
    """CSR slot form from (variable, check) edge pairs; slots check-major, each check's
    variables in the pair order, each variable's edges in ascending check order."""
    v = np.asarray([p[0] for p in var_check_pairs], np.int32)
    c = np.asarray([p[1] for p in var_check_pairs], np.int32)
    order = np.lexsort((np.arange(v.size), c))  # check-major, stable
    cvar = v[order]
    slot_check = c[order]
    cptr = np.zeros(m + 1, np.int32)
    cptr[1:] = np.cumsum(np.bincount(c, minlength=m))
    assert np.array_equal(np.diff(cptr), cdeg)
    vord = np.lexsort((slot_check, cvar))
    vptr = np.zeros(n + 1, np.int32)
    vptr[1:] = np.cumsum(np.bincount(cvar, minlength=n))
    return TannerGraph.from_csr(cptr, cvar, vptr, vord.astype(np.int32))


def _sample_zigzag(ens, n, seed, min_cycle, max_retries, chords=True):
    ring = not chords
    rng = np.random.default_rng(seed)
    vdeg, cdeg = degree_sequences(ens, n)
    m = cdeg.size
    if ring:
        extra = np.nonzero(vdeg == 2)[0][m:]  # the ring holds m of them
        vdeg[extra] = 3
        for _ in range(extra.size):  # one more socket on a lowest-degree check each
            cdeg[int(np.argmin(cdeg))] += 1
    rng.shuffle(cdeg)
    d2 = np.nonzero(vdeg == 2)[0]
    others = np.nonzero(vdeg != 2)[0]
    if d2.size < m - 1:
        raise ValueError("zigzag needs at least m-1 degree-2 variables")
    for _ in range(max_retries):
        order = rng.permutation(m)            # path order of the checks
        pos = np.empty(m, np.int64)
        pos[order] = np.arange(m)
        used = np.zeros(m, np.int64)
        pairs = []
        for i in range(m if ring else m - 1):  # the path (ring): variable d2[i] on checks order[i], order[i+1]
            a, b = order[i], order[(i + 1) % m]
            pairs += [(d2[i], a), (d2[i], b)]
            used[a] += 1
            used[b] += 1
        if ring and d2.size != m:
            raise ValueError("ring needs exactly m degree-2 variables")
        chords = []
        ok = True
        for v in [] if ring else d2[m - 1:]:  # chords between far-apart checks with spare sockets
            for _try in range(1000):
                a, b = rng.integers(0, m, 2)
                if used[a] >= cdeg[a] or used[b] >= cdeg[b] or a == b:
                    continue
                pa, pb = sorted((pos[a], pos[b]))
                if pb - pa + 1 < min_cycle:
                    continue
                # cycles through two chords: |pa - qa| + |pb - qb| + 2 variables on the cycle
                if any(abs(pa - qa) + abs(pb - qb) + 2 < min_cycle or abs(pa - qb) + abs(pb - qa) + 2 < min_cycle
                       for qa, qb in chords):
                    continue
                chords.append((pa, pb))
                pairs += [(v, a), (v, b)]
                used[a] += 1
                used[b] += 1
                break
            else:
                ok = False
                break
        if not ok:
            continue
        # remaining check sockets, matched uniformly to the other variables' sockets
        rest = np.repeat(np.arange(m), cdeg - used)
        vs = np.repeat(others, vdeg[others])
        if rest.size != vs.size:
            raise RuntimeError("socket count mismatch")
        for _r in range(max_retries):
            perm = rng.permutation(rest.size)
            cs = rest[perm]
            key = cs.astype(np.int64) * n + vs
            if np.unique(key).size == key.size:
                break
        else:
            continue
        if ring:
            cs = _ring_repair(cs, vs, vdeg, pos, m, rng, min_cycle, max_retries)
            if cs is None:
                continue
        pairs += list(zip(vs.tolist(), cs.tolist()))
        return _csr_from_pairs(n, m, cdeg, pairs)
    raise RuntimeError("zigzag sampler: too many retries")


def _ring_hops(cs, vs, vdeg, pos, m):
    """Every pair of checks of one higher-degree variable ("hop") as ring positions:
    arrays (socket_a, socket_b, variable, position_a, position_b)."""
    sa, sb = [], []
    start = 0
    vdeg_s = vdeg[vs]
    while start < vs.size:  # sockets are grouped by variable (np.repeat order)
        d = int(vdeg_s[start])
        stop = start
        while stop < vs.size and vdeg_s[stop] == d:
            stop += 1
        base = np.arange(start, stop, d)
        for i in range(d):
            for j in range(i + 1, d):
                sa.append(base + i)
                sb.append(base + j)
        start = stop
    sa = np.concatenate(sa)
    sb = np.concatenate(sb)
    return sa, sb, vs[sa], pos[cs[sa]], pos[cs[sb]]


def _ring_dist(x, y, m):
    d = np.abs(x - y)
    return np.minimum(d, m - d)


def _ring_violations(cs, vs, vdeg, pos, m, min_cycle):
    """Sockets to move so that no small trapping set is left through the ring:
    (1) a higher-degree variable's checks >= min_cycle - 1 apart on the ring (a cycle
    through it and the ring holds >= min_cycle variables; a degree-3 variable closing
    a short ring segment is an (a, 1) trapping set); (2) two higher-degree variables
    v, w joined by k ring segments of <= R = min_cycle // 4 degree-2 variables each
    (distinct checks on both sides) with (deg v - k) + (deg w - k) <= 2 odd checks
    left: two degree-3 variables twice joined, or two degree-4 ones thrice (the
    theta-shaped (8, 2) sets of DESIGN.md's floor analysis)."""
    sa, sb, hv, pa, pb = _ring_hops(cs, vs, vdeg, pos, m)
    bad = set(sa[_ring_dist(pa, pb, m) < min_cycle - 1].tolist())
    R = max(min_cycle // 4, 1)
    p = pos[cs]
    o = np.argsort(p, kind="stable")
    pp = np.concatenate([p[o], p[o] + m])
    oo = np.concatenate([o, o])
    N = o.size
    K = int((np.searchsorted(pp, pp[:N] + R, side="right") - np.arange(N)).max())
    A, Bs = [], []
    for k in range(1, K):
        t = np.nonzero(pp[k:N + k] - pp[:N] <= R)[0]
        A.append(oo[t])
        Bs.append(oo[t + k])
    s1 = np.concatenate(A)
    s2 = np.concatenate(Bs)
    v1, v2 = vs[s1], vs[s2]
    keep = v1 != v2
    s1, s2, v1, v2 = s1[keep], s2[keep], v1[keep], v2[keep]
    sw = v1 > v2
    s1, s2 = np.where(sw, s2, s1), np.where(sw, s1, s2)
    v1, v2 = vs[s1], vs[s2]
    n = int(vs.max()) + 1
    pair = v1.astype(np.int64) * n + v2
    if pair.size:
        ka = np.unique(np.stack([pair, s1]), axis=1)[0]
        kb = np.unique(np.stack([pair, s2]), axis=1)[0]
        ua, ca = np.unique(ka, return_counts=True)
        ub, cb = np.unique(kb, return_counts=True)
        kk = np.minimum(ca, cb)  # ua == ub: the same pair keys
        da, db = vdeg[ua // n], vdeg[ub % n]
        hit = ua[(da - kk) + (db - kk) <= 2]
        if hit.size:
            first = np.unique(pair, return_index=True)
            idx = first[1][np.searchsorted(first[0], hit)]
            bad.update(s1[idx].tolist())
    return np.array(sorted(bad), np.int64)


def _ring_repair(cs, vs, vdeg, pos, m, rng, min_cycle, max_rounds):
    """Swap the sockets of violating variables with random ones until no short cycle
    through the ring remains (_ring_violations); None when it does not settle."""
    cs = cs.copy()
    for _ in range(min(max_rounds, 200)):
        bad = _ring_violations(cs, vs, vdeg, pos, m, min_cycle)
        if bad.size == 0:
            return cs
        tgt = rng.integers(0, cs.size, bad.size)
        for a, b in zip(bad.tolist(), tgt.tolist()):
            cs[a], cs[b] = cs[b], cs[a]
    return None
