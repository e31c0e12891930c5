"""ML ("optimal") erasure decoder oracle, CPU only.

Pins, in the absence of galois (not installed, so the reference's
optimal_decode cannot run here -- see DESIGN.md):
  * the system set-up against the reference's own ml_decoder.c (golden
    vectors in tests/golden/ml_golden.npz, made by make_golden.py ml);
  * the C oracle's elimination loop against an independent numpy restatement
    of parallel_simulator.py:60-129 (tests/ml_restated.py);
  * the ensemble bit-error rates against the ML values the reference's author
    plotted (tools/plotting.py:51, :53, :57; n = 100), statistically.
"""
import os

import numpy as np
import pytest

from oracle import oracle
from tests.ml_restated import optimal_decode

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ml_golden.npz")


def _regular_csr(chk, n, dv, dc):
    m = n * dv // dc
    return np.arange(m + 1, dtype=np.int32) * dc, np.asarray(chk, np.int32), m


def _dense(cptr, cvar, n):
    m = len(cptr) - 1
    H = np.zeros((m, n), np.uint8)
    for c in range(m):
        H[c, cvar[cptr[c]:cptr[c + 1]]] = 1
    return H


def test_ml_system_matches_reference_ml_decoder_c():
    z = np.load(GOLD)
    assert int(z["num_cases"][0]) >= 60
    for ci in range(int(z["num_cases"][0])):
        gi = int(z[f"c{ci}_meta"][0])
        n, dv, dc = map(int, z[f"g{gi}_n"])
        cptr, cvar, m = _regular_csr(z[f"g{gi}_c2v"], n, dv, dc)
        # the reference's dense H agrees with the check-side lists
        np.testing.assert_array_equal(_dense(cptr, cvar, n), z[f"g{gi}_H"])
        target, rem = oracle.ml_system(cptr, cvar, z[f"c{ci}_word"], n, m)
        np.testing.assert_array_equal(target, z[f"c{ci}_target"])
        np.testing.assert_array_equal(rem, z[f"c{ci}_remaining"])


def _random_case(rs, trial):
    n = int(rs.choice([12, 24, 30, 60, 100]))
    chk, _, att = oracle.sample_regular(n, 3, 6, 7, trial)
    assert att > 0
    cptr, cvar, m = _regular_csr(chk, n, 3, 6)
    eps = rs.uniform(0.15, 0.62)
    w = np.where(rs.rand(n) < eps, 2, 0)
    if trial % 3 == 0:  # non-codeword known values: inconsistent systems, galois' pivot order matters
        w = np.where(w == 2, 2, rs.randint(0, 2, n))
    return n, m, cptr, cvar, w


def test_oracle_matches_numpy_restatement_random():
    rs = np.random.RandomState(1)
    partial = 0
    for trial in range(300):
        n, m, cptr, cvar, w = _random_case(rs, trial)
        out, uns = oracle.ml_decode_batch(cptr, cvar, w, n, m)
        ref, ref_uns = optimal_decode(_dense(cptr, cvar, n), w)
        np.testing.assert_array_equal(out[0], ref, err_msg=f"trial {trial}")
        assert uns[0] == ref_uns
        partial += 0 < ref_uns < int((w == 2).sum())
    assert partial > 20  # the give-up loop was exercised


def test_oracle_matches_numpy_restatement_irregular_and_multiedge():
    rs = np.random.RandomState(5)
    for trial in range(60):
        n = int(rs.choice([20, 40, 64]))
        m = n // 2
        H = (rs.rand(m, n) < rs.uniform(0.05, 0.2)).astype(np.uint8)
        cptr = np.zeros(m + 1, np.int32)
        cvar = []
        for c in range(m):
            vs = list(np.nonzero(H[c])[0])
            if trial % 4 == 0 and vs:
                vs.append(vs[0])  # a variable listed twice: H stays 0/1
            cvar += vs
            cptr[c + 1] = len(cvar)
        cvar = np.asarray(cvar, np.int32)
        w = np.where(rs.rand(n) < rs.uniform(0.2, 0.6), 2, rs.randint(0, 2, n))
        out, uns = oracle.ml_decode_batch(cptr, cvar, w, n, m)
        ref, ref_uns = optimal_decode(H, w)
        np.testing.assert_array_equal(out[0], ref)
        assert uns[0] == ref_uns


def test_oracle_edge_cases():
    n = 60
    chk, _, _ = oracle.sample_regular(n, 3, 6, 3, 0)
    cptr, cvar, m = _regular_csr(chk, n, 3, 6)
    H = _dense(cptr, cvar, n)
    # no erasures: unchanged, zero count
    w = np.zeros(n, np.uint8)
    out, uns = oracle.ml_decode_batch(cptr, cvar, w, n, m)
    assert uns[0] == 0 and np.array_equal(out[0], w)
    # more erasures than checks: unchanged (parallel_simulator.py:66-70)
    w = np.zeros(n, np.uint8)
    w[: m + 1] = 2
    out, uns = oracle.ml_decode_batch(cptr, cvar, w, n, m)
    assert uns[0] == m + 1 and np.array_equal(out[0], w)
    # exactly m erasures
    w = np.zeros(n, np.uint8)
    w[::2] = 2
    out, uns = oracle.ml_decode_batch(cptr, cvar, w, n, m)
    ref, ref_uns = optimal_decode(H, w)
    assert uns[0] == ref_uns and np.array_equal(out[0], ref)
    # a single erasure is always solvable (every variable sits in a check)
    w = np.zeros(n, np.uint8)
    w[17] = 2
    out, uns = oracle.ml_decode_batch(cptr, cvar, w, n, m)
    assert uns[0] == 0 and out[0][17] == 0


def test_oracle_solves_codewords():
    """Erasing a real codeword and ML-decoding gives it back wherever solvable."""
    rs = np.random.RandomState(9)
    n = 100
    chk, _, _ = oracle.sample_regular(n, 3, 6, 4, 1)
    cptr, cvar, m = _regular_csr(chk, n, 3, 6)
    H = _dense(cptr, cvar, n)
    # a random codeword from the null space of H over GF(2)
    A = H.copy()
    piv, r = [], 0
    for c in range(n):
        p = next((i for i in range(r, m) if A[i, c]), None)
        if p is None:
            continue
        A[[r, p]] = A[[p, r]]
        for i in range(m):
            if i != r and A[i, c]:
                A[i] ^= A[r]
        piv.append(c)
        r += 1
    free = [c for c in range(n) if c not in piv]
    for _ in range(20):
        x = np.zeros(n, np.uint8)
        x[free] = rs.randint(0, 2, len(free))
        for i, c in enumerate(piv):
            x[c] = (A[i, free] @ x[free]) % 2
        assert not ((H.astype(int) @ x) % 2).any()
        w = np.where(rs.rand(n) < 0.35, 2, x)
        out, uns = oracle.ml_decode_batch(cptr, cvar, w, n, m)
        solved = out[0] != 2
        np.testing.assert_array_equal(out[0][solved], x[solved])


# Author's ML simulations (tools/plotting.py:51, :53, :57): BER for n = 100, (3, 6), by erasure
# probability, with the number of trials each value rests on as far as it can be read off the
# value itself (0.045414847161572056 = 5200 / (1145 * 100); 7.53378e-4 = 3100 / (41148 * 100);
# 0.0059553 is rounded -- 10^4 trials assumed).
PLOTTED_ML_BER_N100 = {0.30: (7.533780499659765e-4, 41148), 0.35: (5.9553e-3, 10000),
                       0.40: (4.5414847161572056e-2, 1145)}


def ml_ber_agrees(bits_per_trial, n, eps):
    """Two-sample z-test (3 sigma): our mean vs the plotted value, the per-trial
    standard deviation estimated from our sample for both."""
    ref, n_ref = PLOTTED_ML_BER_N100[eps]
    T = len(bits_per_trial)
    ber = bits_per_trial.mean() / n
    sd = bits_per_trial.std() / n
    return abs(ber - ref) <= 3.0 * sd * np.sqrt(1.0 / T + 1.0 / n_ref), ber, ref


@pytest.mark.parametrize("eps", sorted(PLOTTED_ML_BER_N100))
def test_ensemble_ml_ber_matches_reference_plots(eps):
    """Fresh (3,6) graph per trial (sampler law of random_code_generator.c), BEC(eps)
    word, ML decode: the bit-error rate agrees with the author's plotted ML values
    within the two runs' sampling error."""
    n, m, T = 100, 50, 12000
    rs = np.random.RandomState(int(eps * 1000))
    chks = oracle.sample_regular_batch(n, 3, 6, 11, 0, T)[0]
    words = np.where(rs.rand(T, n) < eps, 2, 0).astype(np.uint8)
    cptr = np.arange(m + 1, dtype=np.int32) * 6
    u = np.array([oracle.ml_decode_batch(cptr, chks[t], words[t], n, m)[1][0] for t in range(T)], np.float64)
    ok, ber, ref = ml_ber_agrees(u, n, eps)
    assert ok, (eps, ber, ref)
