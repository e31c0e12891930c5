"""Host-only checks of the local-edge layout of bp_loc_kernel (csrc/loc_layout.cpp) through
ldpc_debug_loc_layout (no device needed):

* every variable sits in exactly one (thread, var-pair slot, half) lane, as one of the two
  local variables of the check pair that thread updates;
* every non-local edge has its own LDS word inside its check pair's rows, and the rows of
  a check hold exactly its non-local edges (with the local ones that is every edge once);
* absent edges (ABS) point at the thread's private dummy word and are flagged absent;
* the rows hold exactly the non-local edges plus the pads of mixed-degree pairs;
* the bank-conflict search lowers the cost well below a random row order.
"""
import ctypes as ct

import numpy as np
import pytest

from iib_project_ldpc_codes_amd import _native, ensembles
from iib_project_ldpc_codes_amd.graph import TannerGraph


def layout(g, T, search=True):
    cptr, cvar, vptr, vslot = [np.ascontiguousarray(a, np.int32) for a in g.to_csr()]
    shape = np.zeros(24, np.int32)
    L = _native.lib()
    rc = L.ldpc_debug_loc_layout(cptr.ctypes.data, cvar.ctypes.data, vptr.ctypes.data, vslot.ctypes.data, g.n, g.m,
                                 T, shape.ctypes.data, None, None, None)
    assert rc == 0, _native.last_error()
    T_, KP, DVN, P, words = shape[:5]
    VP, D = 2 * KP, max(DVN, 1)
    var = np.zeros(VP * 2 * T, np.int32)
    pos = np.zeros(VP * D * T, np.int32)
    info = np.zeros(VP * T, np.int32)
    assert L.ldpc_debug_loc_layout(cptr.ctypes.data, cvar.ctypes.data, vptr.ctypes.data, vslot.ctypes.data, g.n,
                                   g.m, T, shape.ctypes.data, var.ctypes.data, pos.ctypes.data, info.ctypes.data) == 0
    return shape, var.reshape(VP, 2, T), pos.reshape(VP, D, T), info.reshape(VP, T), (cptr, cvar, vptr, vslot)


def check_invariants(g, T):
    shape, var, pos, info, (cptr, cvar, vptr, vslot) = layout(g, T)
    T_, KP, DVN, P, words, ncls, conflicts = shape[:7]
    assert T_ == T and P == g.m // 2 and KP == -(-P // T)
    # each variable exactly once
    ids = var[var >= 0]
    assert np.array_equal(np.sort(ids), np.arange(g.n))
    # non-local words: distinct, inside [0, words), E - n of them
    D = max(DVN, 1)
    seen = []
    for vi in range(2 * KP):
        for h in range(2):
            for t in range(T):
                v = var[vi, h, t]
                if v < 0:
                    continue
                deg = vptr[v + 1] - vptr[v]
                bits = info[vi, t]
                assert bin((bits >> (4 * h)) & 15).count("1") == deg - 1
                jl = (bits >> (8 + 2 * h)) & 3
                assert 0 <= jl < deg
                assert (bits >> (16 + 4 * h)) & 15 == 1 << jl  # one-hot copy of jl
                for u in range(DVN):
                    w = (pos[vi, u, t] >> (16 * h)) & 0xFFFF
                    if u < deg - 1:
                        assert w < words
                        seen.append(w)
                    else:
                        assert w == words + (t & 63)
    seen = np.array(seen)
    assert len(seen) == vptr[-1] - g.n and len(np.unique(seen)) == len(seen)
    assert 0 <= words - len(seen) <= 2 * ncls  # a mixed pair's smaller check leaves pad words
    return conflicts


def test_loc_layout_regular_headline_code(monkeypatch):
    g = TannerGraph.random_regular(10000, 3, 6, seed=1)
    conflicts = check_invariants(g, 1024)
    monkeypatch.setenv("LDPC_LOC_SEARCH", "0")  # the layout before the bank-conflict search
    unsearched = layout(g, 1024)[0][6]
    # 6 var-pair slots x 2 edges x 2 halves x 32 half waves = 768 instruction-groups: the
    # unsearched layout costs ~2 extra lanes per group, the searched one at most 1
    assert conflicts <= 768 and conflicts < 0.5 * unsearched, (conflicts, unsearched)


@pytest.mark.parametrize("n", [2000, 20000])
def test_loc_layout_rsu_ensemble(n):
    g = ensembles.sample_irregular(ensembles.RSU_DL4, n, seed=1, deg2="zigzag")
    check_invariants(g, 256 if n <= 2048 else 1024)


def test_loc_layout_small_regular():
    g = TannerGraph.random_regular(1000, 3, 6, seed=3)
    check_invariants(g, 256)


def test_loc_layout_refuses_other_rates():
    g = TannerGraph.random_regular(1200, 3, 4, seed=3)  # rate 1/4: n != 2m
    cptr, cvar, vptr, vslot = [np.ascontiguousarray(a, np.int32) for a in g.to_csr()]
    shape = np.zeros(24, np.int32)
    rc = _native.lib().ldpc_debug_loc_layout(cptr.ctypes.data, cvar.ctypes.data, vptr.ctypes.data, vslot.ctypes.data,
                                             g.n, g.m, 256, shape.ctypes.data, None, None, None)
    assert rc == _native.LDPC_EUNSUP


def loc_variant(g, T):
    cptr, cvar, vptr, vslot = [np.ascontiguousarray(a, np.int32) for a in g.to_csr()]
    out = np.zeros(1, np.int32)
    rc = _native.lib().ldpc_debug_loc_variant(cptr.ctypes.data, cvar.ctypes.data, vptr.ctypes.data,
                                              vslot.ctypes.data, g.n, g.m, T, out.ctypes.data)
    assert rc == 0, _native.last_error()
    return int(out[0])


def test_loc_variant_from_whole_shape():
    """The bp_loc_kernel family is chosen from the whole layout shape (advisor round 2): a
    check-regular degree-6 graph with variable degrees {2, 4} (loc_dlo == 6, DVN = 3) must
    take the RSU family (2), never the (3,6) family (1) whose rows hold DVN = 2 edges."""
    from tests.graph_util import check6_var24
    g = check6_var24(500, seed=3)
    shape = layout(g, 256)[0]
    assert shape[2] == 3 and (shape[22] & 255) == 1  # DVN 3, slot 0 = the degree-2 variables
    assert all((d & 255) == 6 and not d >> 8 for d in shape[12:12 + shape[5]])  # every class degree 6
    assert loc_variant(g, 256) == 2
    g5 = check6_var24(5000, seed=4)
    assert loc_variant(g5, 1024) == 2
    assert loc_variant(g5, 512) == 0  # KP = 5 at T = 512: the RSU family has no such shape (another kernel runs)
    assert loc_variant(TannerGraph.random_regular(1000, 3, 6, seed=2), 256) == 1
    assert loc_variant(TannerGraph.random_regular(10000, 3, 6, seed=1), 512) == 1
    assert loc_variant(ensembles.sample_irregular(ensembles.RSU_DL4, 2000, seed=21, deg2="zigzag"), 256) == 2
