"""Pin the CPU oracle against the reference's own outputs (tests/golden/)."""
import json
import os

import numpy as np
import pytest

from oracle import oracle
from tests.golden_util import load_bec_golden

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load():
    return load_bec_golden()


GRAPHS, CASES = _load()


def test_golden_has_cases():
    assert len(CASES) >= 400 and len(GRAPHS) >= 8


@pytest.mark.parametrize("ci", range(0, len(CASES)))
def test_oracle_message_passing_matches_reference(ci):
    c = CASES[ci]
    n, k, dv, dc, v2c, c2v = GRAPHS[c["gi"]]
    if c["errin"] is None:
        w, err, it = oracle.message_passing(c["word"], c["max_its"], v2c, c2v, n, k, dv, dc)
        err = np.insert(err, 0, int(np.count_nonzero(c["word"] == 2)))  # parallel_simulator.py:165
    else:
        w, err, it = oracle.message_passing(c["word"], c["max_its"], v2c, c2v, n, k, dv, dc, errors=c["errin"])
    assert it == c["it"]
    np.testing.assert_array_equal(w.astype(np.int8), c["out"])
    np.testing.assert_array_equal(err, c["errors"])


def test_oracle_bec_batch_matches_single():
    n, k, dv, dc, v2c, c2v = GRAPHS[3]
    sel = [c for c in CASES if c["gi"] == 3 and c["errin"] is None and c["max_its"] == 20]
    words = np.stack([c["word"] for c in sel])
    w, err, its = oracle.bec_decode_batch(words, 20, v2c, c2v, n, k, dv, dc)
    for b, c in enumerate(sel):
        np.testing.assert_array_equal(w[b], c["out"])
        np.testing.assert_array_equal(err[b], c["errors"][1:])
        assert its[b] == c["it"]


def test_density_evolution_known_answers():
    with open(os.path.join(GOLD, "de_golden.json")) as f:
        g = json.load(f)
    np.testing.assert_allclose(oracle.density_evolution(0.4, 10, 3, 6), g["density_evolution_0.4_10_3_6"], rtol=1e-12)
    np.testing.assert_allclose(oracle.density_evolution(0.2, 10, 3, 6, 1e-9), g["density_evolution_0.2_10_3_6_1e-9"], rtol=1e-12)
    np.testing.assert_allclose(oracle.density_evolution(0.45, 30, 3, 6), g["density_evolution_0.45_30_3_6"], rtol=1e-12)
    assert abs(g["calc_threshold_3_6"] - 0.42943981) < 1e-7


def test_philox_known_answer():
    # Random123 published known-answer vectors for philox4x32-10 (kat_vectors).
    np.testing.assert_array_equal(oracle.philox([0, 0, 0, 0], [0, 0]),
                                  np.array([0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8], np.uint32))
    np.testing.assert_array_equal(oracle.philox([0xffffffff] * 4, [0xffffffff] * 2),
                                  np.array([0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd], np.uint32))
    np.testing.assert_array_equal(
        oracle.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0]),
        np.array([0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1], np.uint32))


def test_oracle_fixed_code_fer_ber_near_reference_probe():
    """The oracle on the reference-generated n=1000 code, eps=0.4, 50 iterations: FER / BER
    near the reference C's 9.05e-2 / 2.13e-2 (6,000 trials here, so the
    tolerance is ~4 sigma of this sample)."""
    n, k, dv, dc, v2c, c2v = GRAPHS[3]
    T = 6000
    words = oracle.channel(oracle.CH_BEC, 0.4, 17, 0, n, T)
    _, err, _ = oracle.bec_decode_batch(words, 50, v2c, c2v, n, k, dv, dc)
    final = err[:, -1]
    fer, ber = float((final > 0).mean()), float(final.sum() / (T * n))
    assert abs(fer - 0.0905) < 0.015, fer
    assert abs(ber - 0.0213) < 0.004, ber


# ------------------------------------------------ soft check rules vs float64
XMAX64 = 23 * np.log(2.0)  # the rules' saturation: |x| is clamped at 23 ln 2 (e^-|x| >= 2^-23)


def _spa_float64(x):
    """Textbook tanh rule in float64: c_j = 2 atanh(prod_{i != j} tanh(x_i / 2)), inputs
    saturated at XMAX64 like the decoders -- independent of the oracle's ratio form."""
    x = np.asarray(x, np.float64)
    t = np.tanh(np.minimum(np.abs(x), XMAX64) / 2) * np.where(x < 0, -1.0, 1.0)
    return np.array([2 * np.arctanh(np.prod(np.delete(t, j))) for j in range(len(x))])


def _minsum_float64(x, alpha):
    x = np.asarray(x, np.float32)
    out = np.empty_like(x)
    for j in range(len(x)):
        rest = np.delete(x, j)
        sign = -1.0 if (np.count_nonzero(rest < 0) % 2) else 1.0
        out[j] = np.float32(sign * float(alpha) * float(np.min(np.abs(rest))))  # one fp32 rounding
    return out


def test_oracle_spa_rule_vs_float64_tanh():
    """The oracle's sum-product check rule (the definition the GPU kernels are held to:
    the exact tanh rule, evaluated in double without cancellation and rounded to fp32)
    against the float64 tanh / atanh rule, over degrees 2-8 and input scales from 0.1 to
    60 nats (saturated inputs included): within one fp32 ulp everywhere."""
    rng = np.random.default_rng(7)
    worst = 0.0
    for _ in range(6000):
        d = int(rng.integers(2, 9))
        scale = rng.choice([0.1, 0.5, 2.0, 5.0, 20.0, 60.0])
        x = (rng.normal(size=d) * scale).astype(np.float32)
        if rng.random() < 0.1:
            x[rng.integers(d)] = np.float32(0.0)
        got = oracle.check_update(x, 0).astype(np.float64)
        want = _spa_float64(x)
        tol = 2.0 ** -23 * np.abs(want) + 1e-30
        worst = max(worst, float(np.max(np.abs(got - want) / tol)))
        assert np.all(np.abs(got - want) <= tol), (x, got, want)
    assert worst > 0.05  # the bound is not vacuous


def test_oracle_spa_rule_saturated_inputs():
    """All inputs beyond the 23 ln 2 clamp: the outputs are the clamped rule's,
    2 atanh(tanh(23 ln2 / 2)^5) = 14.33 nats for degree 6 -- the largest check message the
    decoders produce -- to one ulp, with the exclusive sign (here the input's own sign:
    the total sign product is +)."""
    x = np.array([30.0, -40.0, 25.0, 60.0, -17.0, 90.0], np.float32)
    got = oracle.check_update(x, 0).astype(np.float64)
    want = _spa_float64(x)
    np.testing.assert_allclose(got, want, rtol=2.0 ** -23, atol=0)
    assert np.allclose(np.abs(got), 2 * np.arctanh(np.tanh(23 * np.log(2) / 2) ** 5), rtol=2.0 ** -23)
    assert np.array_equal(np.sign(got), np.sign(x))


@pytest.mark.parametrize("alpha", [1.0, 0.75, 0.8125])
def test_oracle_minsum_rule_vs_float64(alpha):
    """Normalized min-sum: c_j = alpha * min_{i != j} |x_i| * prod_{i != j} sign(x_i), with
    one fp32 rounding of the product -- bit-exact, incl. ties, zeros and huge inputs."""
    rng = np.random.default_rng(9)
    for _ in range(3000):
        d = int(rng.integers(2, 9))
        x = (rng.normal(size=d) * rng.choice([0.5, 5.0, 1e30])).astype(np.float32)
        if rng.random() < 0.2:
            x[rng.integers(d)] = x[rng.integers(d)]  # ties
        if rng.random() < 0.1:
            x[rng.integers(d)] = np.float32(0.0)
        got = oracle.check_update(x, 1, alpha)
        np.testing.assert_array_equal(got, _minsum_float64(x, alpha))
