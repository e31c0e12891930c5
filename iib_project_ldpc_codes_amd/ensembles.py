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


def sample_irregular(ens, n, seed=0, max_retries=100000):
    """Configuration-model graph of ``ens`` with n variables (host, numpy PCG64)."""
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
