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
