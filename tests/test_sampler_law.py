"""Sampler law, whole distributions (not only means): both device-sampler restatements --
the one-level Rao-Sandelius form (oracle default below n*dv = 8192) and the sequential-draw
form (forced) -- against the reference generator (random_code_generator.c:21-67 compiled
unchanged into oracle/_ref):

* the histogram of the number of length-4 cycles, two-sample chi-square homogeneity test;
* the variable held by fixed slots (first, middle, last) over many graphs, chi-square
  goodness of fit to uniform -- the law is a uniform socket permutation conditioned on
  simple checks, so every slot's variable is uniform over the n variables.

Seeds are fixed (the reference's glibc rand() stream is seeded with oracle.ref_srand before its
samples are drawn), so the tests are deterministic and independent of test order; the thresholds are p >= 1e-3."""
import numpy as np
import pytest
from scipy import stats

from oracle import oracle


def _c4(chk, n, m, dc=6):
    H = np.zeros((m, n), np.int64)
    H[np.repeat(np.arange(m), dc), chk] = 1
    O = H @ H.T
    np.fill_diagonal(O, 0)
    return int((O * (O - 1) // 2).sum() // 2)


def _homogeneity(a, b):
    """chi-square homogeneity p-value of two samples of small non-negative integers, bins
    merged from the top until every expected count is >= 5."""
    hi = max(max(a), max(b))
    ca = np.bincount(a, minlength=hi + 1).astype(float)
    cb = np.bincount(b, minlength=hi + 1).astype(float)
    # merge tail bins
    while len(ca) > 2 and (ca[-1] + cb[-1]) < 10:
        ca[-2] += ca[-1]
        cb[-2] += cb[-1]
        ca, cb = ca[:-1], cb[:-1]
    keep = (ca + cb) > 0
    return stats.chi2_contingency(np.vstack([ca[keep], cb[keep]]))[1]


@pytest.fixture
def force_seq():
    oracle.sampler_force_seq(True)
    yield
    oracle.sampler_force_seq(False)


def _ours(n, N, seed):
    return [oracle.sample_regular(n, 3, 6, seed, g)[0] for g in range(N)]


def _check_c4_and_slots(n, ours, ref):
    m = n // 2
    p = _homogeneity([_c4(c, n, m) for c in ours], [_c4(c, n, m) for c in ref])
    assert p >= 1e-3, ("4-cycle histogram", n, p)
    E = 3 * n
    for slot in (0, E // 2, E - 1):
        vals = np.array([c[slot] for c in ours])
        p = stats.chisquare(np.bincount(vals, minlength=n))[1]
        assert p >= 1e-3, ("slot uniformity", n, slot, p)


def test_one_level_sampler_law_full_distribution():
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built")
    n, N = 40, 2000
    oracle.ref_srand(7)  # the reference draws from glibc rand(): seed it, so the test does not depend on test order
    ref = [oracle.ref_generate_random_code(n, 3, 6)[0] for _ in range(N)]
    _check_c4_and_slots(n, _ours(n, N, 101), ref)


@pytest.mark.parametrize("n,N", [(40, 2000), (400, 800)])
def test_seq_sampler_law_full_distribution(force_seq, n, N):
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built")
    oracle.ref_srand(11 + n)
    ref = [oracle.ref_generate_random_code(n, 3, 6)[0] for _ in range(N)]
    _check_c4_and_slots(n, _ours(n, N, 202), ref)
