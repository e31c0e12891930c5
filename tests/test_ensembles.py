"""Irregular ensembles + density evolution, host side."""
import json
import os

import numpy as np
import pytest

from iib_project_ldpc_codes_amd import de, ensembles

GOLD = os.path.join(os.path.dirname(__file__), "golden", "de_golden.json")


def test_bec_de_reproduces_reference_values():
    g = json.load(open(GOLD))
    r = de.regular(3, 6)
    np.testing.assert_allclose(de.bec_de(r, 0.4, 10), g["density_evolution_0.4_10_3_6"], rtol=1e-12)
    np.testing.assert_allclose(de.bec_de(r, 0.2, 10, 1e-9), g["density_evolution_0.2_10_3_6_1e-9"], rtol=1e-12)
    np.testing.assert_allclose(de.bec_de(r, 0.45, 30), g["density_evolution_0.45_30_3_6"], rtol=1e-12)
    assert de.bec_threshold(r) == pytest.approx(g["calc_threshold_3_6"], abs=1e-9)


def test_irregular_bec_threshold_beats_regular():
    t = de.bec_threshold(ensembles.RSU_DL4, iterations=20000, tol=1e-6)
    assert 0.44 < t < 0.5  # below capacity 1 - R = 0.5, above the (3,6) 0.4294


def test_awgn_ga_threshold_regular36():
    # Gaussian-approximation threshold of (3,6): ~0.874 (exact DE 0.881)
    assert 0.86 < de.awgn_threshold(de.regular(3, 6), tol=2e-3) < 0.89


def test_design_rate_and_degrees():
    e = ensembles.RSU_DL4
    assert e.design_rate == pytest.approx(0.5, abs=1e-5)
    vdeg, cdeg = ensembles.degree_sequences(e, 20000)
    assert vdeg.size == 20000 and vdeg.sum() == cdeg.sum()
    frac = e.node_fractions("var")
    for d, f in frac.items():
        assert abs(np.mean(vdeg == d) - f) < 1e-3


def test_sample_irregular_graph_valid():
    g = ensembles.sample_irregular(ensembles.RSU_DL4, 2000, seed=3)
    cptr, cvar, vptr, vslot = g.csr
    assert cptr[-1] == vptr[-1] == cvar.size == vslot.size
    assert np.array_equal(np.sort(vslot), np.arange(vslot.size))
    for v in range(0, 2000, 37):
        sl = vslot[vptr[v]:vptr[v + 1]]
        assert np.all(cvar[sl] == v)
    for c in range(0, g.m, 29):
        row = cvar[cptr[c]:cptr[c + 1]]
        assert len(set(row)) == row.size


def test_zigzag_construction_preserves_degrees_and_removes_weight2():
    e = ensembles.RSU_DL4
    g = ensembles.sample_irregular(e, 4000, seed=2, deg2="zigzag", min_cycle=30)
    cptr, cvar, vptr, vslot = g.csr
    vdeg, cdeg = ensembles.degree_sequences(e, 4000)
    np.testing.assert_array_equal(np.sort(np.diff(vptr)), np.sort(vdeg))
    np.testing.assert_array_equal(np.sort(np.diff(cptr)), np.sort(cdeg))
    assert np.array_equal(np.sort(vslot), np.arange(vslot.size))
    # no two degree-2 variables on the same pair of checks (weight-2 codewords)
    slot_check = np.repeat(np.arange(g.m), np.diff(cptr))
    pairs = set()
    for v in np.nonzero(np.diff(vptr) == 2)[0]:
        p = tuple(sorted(slot_check[vslot[vptr[v]:vptr[v + 1]]]))
        assert p not in pairs
        pairs.add(p)


def _ring_order(g):
    """Check order along the degree-2 ring of a deg2="path" graph (asserts it is one cycle)."""
    cptr, cvar, vptr, vslot = g.csr
    slot_check = np.repeat(np.arange(g.m), np.diff(cptr))
    vdeg = np.diff(vptr)
    nb = [[] for _ in range(g.m)]
    for v in np.nonzero(vdeg == 2)[0]:
        a, b = slot_check[vslot[vptr[v]:vptr[v + 1]]]
        nb[a].append(b)
        nb[b].append(a)
    assert all(len(x) == 2 for x in nb)  # every check on exactly two ring variables
    order, prev, c = [0], -1, 0
    while True:
        nxt = nb[c][0] if nb[c][0] != prev else nb[c][1]
        if nxt == 0:
            break
        order.append(nxt)
        prev, c = c, nxt
    assert len(order) == g.m  # one ring through all checks: the only all-degree-2 codeword
    pos = np.empty(g.m, np.int64)
    pos[order] = np.arange(g.m)
    return pos, slot_check, vdeg


def test_ring_construction_short_cycle_free():
    """deg2="path": a ring of m degree-2 variables; no higher-degree variable closes a
    ring segment shorter than min_cycle - 1, and no two degree-3 variables are joined by
    two segments of <= min_cycle // 4 (the (a, 1) / (a, 2) trapping sets of the floor)."""
    e, n, L = ensembles.RSU_DL4, 4000, 24
    g = ensembles.sample_irregular(e, n, seed=2, deg2="path", min_cycle=L)
    cptr, cvar, vptr, vslot = g.csr
    assert np.array_equal(np.sort(vslot), np.arange(vslot.size))
    vdeg0, cdeg0 = ensembles.degree_sequences(e, n)
    assert cptr[-1] == vdeg0.sum() + np.count_nonzero(vdeg0 == 2) - g.m  # surplus degree 2 -> 3
    pos, slot_check, vdeg = _ring_order(g)
    m, R = g.m, L // 4
    near = {}
    for v in np.nonzero(vdeg > 2)[0]:
        p = np.sort(pos[slot_check[vslot[vptr[v]:vptr[v + 1]]]])
        d = np.diff(np.append(p, p[0] + m))
        assert d.min() >= L - 1, (v, p)
        if vdeg[v] == 3:
            near[v] = p
    items = list(near.items())
    for i, (v, p) in enumerate(items):  # (3,3) pairs joined twice (brute force, n small)
        for w, q in items[i + 1:]:
            dd = np.abs(p[:, None] - q[None, :])
            dd = np.minimum(dd, m - dd) <= R
            assert not (dd.any(axis=1).sum() >= 2 and dd.any(axis=0).sum() >= 2), (v, w)


def test_oracle_csr_sampler_regular_structure_equals_regular_sampler():
    """ldpc_sample_csr with v*dv / c*dc pointers is the regular generator."""
    from oracle import oracle
    n, dv, dc = 300, 3, 6
    vptr = np.arange(n + 1, dtype=np.int32) * dv
    cptr = np.arange(n * dv // dc + 1, dtype=np.int32) * dc
    for g in range(5):
        chk, var, att = oracle.sample_regular(n, dv, dc, 9, g)
        cv, vs, att2 = oracle.sample_csr(vptr, cptr, 9, g)
        assert att == att2
        np.testing.assert_array_equal(cv, chk)
        np.testing.assert_array_equal(vs // dc, var)  # slots -> checks


def test_oracle_csr_sampler_irregular_law():
    """Irregular RSU graphs: degrees as specified, no check holds a variable twice,
    variable side consistent, and the 4-cycle statistic matches the host
    configuration-model sampler (same law, different generator)."""
    from oracle import oracle
    from iib_project_ldpc_codes_amd import ensembles
    n = 200
    vptr, cptr = ensembles.degree_ptrs(ensembles.RSU_DL4, n)
    m = len(cptr) - 1

    def four_cycles(cp, cv):
        H = np.zeros((m, n), np.int32)
        for c in range(m):
            H[c, cv[cp[c]:cp[c + 1]]] = 1
        O = H @ H.T
        np.fill_diagonal(O, 0)
        return (O * (O - 1) // 2).sum() // 2

    dev, host = [], []
    for g in range(400):
        cv, vs, att = oracle.sample_csr(vptr, cptr, 4, g)
        assert att > 0
        for c in range(m):
            row = cv[cptr[c]:cptr[c + 1]]
            assert len(set(row.tolist())) == len(row)
        assert np.array_equal(np.bincount(cv, minlength=n), np.diff(vptr))
        for v in (0, n // 2, n - 1):
            sl = vs[vptr[v]:vptr[v + 1]]
            assert np.all(cv[sl] == v) and np.all(np.diff(sl) > 0)
        dev.append(four_cycles(cptr, cv))
        hg = ensembles.sample_irregular(ensembles.RSU_DL4, n, seed=g)
        hcp, hcv, _, _ = hg.to_csr()
        host.append(four_cycles(hcp, hcv))
    dev, host = np.array(dev, float), np.array(host, float)
    se = np.sqrt(dev.var() / len(dev) + host.var() / len(host))
    assert abs(dev.mean() - host.mean()) < 4 * se
