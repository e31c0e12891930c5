"""The frontier-peeling ensemble decoder's overflow branch (csrc/peel.hip), bit-exact against
the oracle trial by trial.

bec_peel_kernel keeps each iteration's frontier (checks holding exactly one erasure) in an LDS
list of F entries; when a list overflows, the next iteration snapshots every count-1 check
into a bitmap and scans it instead.  At n = 64,800 F = 5,266 and the expected first frontier
m*dc*eps*(1-eps)^5 is ~5,390 at eps = 0.419, so nearly every configs[4] trial there takes the
scan path.  Both tests read ldpc_debug_peel_stats (always collected by the product build) to
prove the branch ran, and compare every trial's erasure curve and iteration count with the
oracle's sampler + message_passing restatement (message_passing.c:7-82, the curve with the
initial count prepended as parallel_simulator.py:165, X = -1 so every curve counts,
parallel_simulator_expurgated.py:238).
"""
import ctypes

import numpy as np
import pytest

from oracle import oracle
from tests.test_gpu_fullsize import _dump

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a visible MI355X"
    return t


def _peel_stats(reset=False):
    from iib_project_ldpc_codes_amd import _native
    out = (ctypes.c_uint64 * 3)()
    _native.check(_native.lib().ldpc_debug_peel_stats(out, int(reset)), "ldpc_debug_peel_stats")
    return [int(x) for x in out]


def _per_trial(torch, n, eps, iters, seed, T):
    """Device: one trial per run_batch call (trial t on graph t, channel subsequence t), so the
    counter deltas are the trial's own curve; returns (curves [T][iters+1], its [T])."""
    from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
    mc = MonteCarlo.ensemble(n, 3, 6, "bec", eps, iters, seed=seed, batch=1, expurgation=-1)
    curves = np.zeros((T, iters + 1), np.int64)
    its = np.zeros(T, np.int64)
    prev = mc.counters.cpu().numpy().copy()
    for t in range(T):
        mc.run_batch(t, 1)
        torch.cuda.synchronize()
        cur = mc.counters.cpu().numpy().copy()
        d = cur - prev
        prev = cur
        assert d[0] == 1
        curves[t] = d[4:]
        its[t] = d[3]
    return curves, its


def _oracle_trials(n, eps, iters, seed, T):
    chk, var, _ = oracle.sample_regular_batch(n, 3, 6, seed, 0, T)
    words = oracle.channel(oracle.CH_BEC, eps, seed, 0, n, T)
    curves = np.zeros((T, iters + 1), np.int64)
    its = np.zeros(T, np.int64)
    for t in range(T):
        _, err, it = oracle.message_passing(words[t], iters, var[t], chk[t], n, n // 2, 3, 6)
        curves[t] = np.insert(err, 0, int(np.count_nonzero(words[t] == 2)))
        its[t] = it
    return curves, its


def _check(torch, name, n, eps, iters, seed, T, cap):
    from iib_project_ldpc_codes_amd import _native
    _native.check(_native.lib().ldpc_debug_peel_cap(cap), "ldpc_debug_peel_cap")
    try:
        _peel_stats(reset=True)
        got_c, got_i = _per_trial(torch, n, eps, iters, seed, T)
        st = _peel_stats()
    finally:
        _native.lib().ldpc_debug_peel_cap(0)
    want_c, want_i = _oracle_trials(n, eps, iters, seed, T)
    stats = {"n": n, "eps": eps, "iterations": iters, "trials": T, "frontier_cap": cap or "lds budget",
             "scan_iterations": st[0], "trials_scanned": st[1], "trials_decoded": st[2],
             "frame_errors": int((want_c[:, -1] != 0).sum()), "mean_its": float(want_i.mean()),
             "identical_trials": int(np.all(got_c == want_c, axis=1).sum())}
    _dump(name, stats)
    assert st[2] == T, stats  # every trial ran on the peeling decoder
    np.testing.assert_array_equal(got_c, want_c)
    np.testing.assert_array_equal(got_i, want_i)
    return stats


def test_peel_overflow_forced_small_n(torch):
    """n = 1,000 with the frontier lists capped at 8 entries: the scan branch runs in (nearly)
    every trial, deterministically; 96 trials at eps = 0.42, 60 iterations."""
    stats = _check(torch, "peel_overflow_forced_n1000", 1000, 0.42, 60, 31, 96, 8)
    assert stats["trials_scanned"] >= 90 and stats["scan_iterations"] > stats["trials_scanned"], stats


def test_peel_overflow_cfg4_n64800_eps0419(torch):
    """configs[4] at the campaign point eps = 0.419, 200 iterations, the product frontier
    capacity (5,266): 32 trials, most of them through the scan branch."""
    stats = _check(torch, "peel_overflow_cfg4_n64800_eps0.419", 64800, 0.419, 200, 41, 32, 0)
    assert stats["trials_scanned"] >= 16, stats
