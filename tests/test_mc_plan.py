"""ldpc_mc_run's round accounting on the CPU (csrc/mc_plan.hpp through the host-only
ldpc_debug_mc_plan, which runs the device run's own driver loop on a synthetic trial
sequence): for ndev = 1..8 slots, every batch size, trial limit and frame-error stop, the
counters equal the reference's sequential loop

    while frame_errors < stop and trials < num_tests: run trial   (parallel_simulator.py:198)

including crossings in the first, a middle and the last slot of a round and rounds clamped
by num_tests (the case the round-2 advisor found: the crossing slot's re-run must keep the
batch it first ran, not one re-clamped from counters that already hold earlier slots)."""
import numpy as np
import pytest

from iib_project_ldpc_codes_amd import _native


def sequential(fe, num_tests, stop):
    t = f = 0
    while (stop <= 0 or f < stop) and (num_tests <= 0 or t < num_tests):
        f += int(fe[t] != 0)
        t += 1
    return t, f


def plan(fe, num_tests, stop, batch, ndev):
    fe = np.ascontiguousarray(fe, np.uint8)
    out = np.zeros(3, np.int64)
    rc = _native.lib().ldpc_debug_mc_plan(fe.ctypes.data, fe.size, num_tests, stop, batch, ndev, out.ctypes.data)
    assert rc == 0, _native.last_error()
    return int(out[0]), int(out[1]), int(out[2])


def rounds_expected(trials, batch, ndev):
    return -(-trials // (batch * ndev)) if trials else 0


@pytest.mark.parametrize("ndev", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("batch", [1, 5, 64])
def test_plan_equals_sequential_random(ndev, batch):
    rng = np.random.default_rng(1000 * ndev + batch)
    for trial in range(60):
        N = int(rng.integers(1, 4000))
        p = float(rng.choice([0.0, 0.001, 0.02, 0.3, 1.0]))
        fe = (rng.random(N + 3 * batch * ndev) < p).astype(np.uint8)
        num_tests = int(rng.integers(1, N + 1))
        stop = int(rng.choice([0, 1, 2, 7, 50, 200]))
        t, f, r = plan(fe, num_tests, stop, batch, ndev)
        assert (t, f) == sequential(fe, num_tests, stop), (N, p, num_tests, stop)
        assert r == rounds_expected(t, batch, ndev)


@pytest.mark.parametrize("ndev", [2, 4, 8])
@pytest.mark.parametrize("where", ["first", "middle", "last"])
@pytest.mark.parametrize("clamped", [False, True])
def test_plan_crossing_slot(ndev, where, clamped):
    """The stop is crossed inside slot 0, a middle slot or the last slot of the final round;
    with `clamped` that round is also the one num_tests cuts short (the later slots run
    fewer than `batch` trials or none)."""
    batch, stop, rounds = 16, 10, 3
    slot = {"first": 0, "middle": ndev // 2, "last": ndev - 1}[where]
    N = (rounds + 1) * batch * ndev
    fe = np.zeros(N, np.uint8)
    # stop - 1 frame errors spread over the earlier rounds, the last one inside `slot` of the final round
    early = np.linspace(0, (rounds - 1) * batch * ndev - 1, stop - 1).astype(int)
    fe[early] = 1
    last_round0 = (rounds - 1) * batch * ndev
    cross = last_round0 + slot * batch + 5
    fe[cross] = 1
    fe[cross + 1:] = 1  # every trial after the crossing one is an error too (must not be counted)
    num_tests = last_round0 + slot * batch + 9 if clamped else 0
    t, f, r = plan(fe, num_tests, stop, batch, ndev)
    assert (t, f) == sequential(fe, num_tests, stop) == (cross + 1, stop)
    assert r == rounds


@pytest.mark.parametrize("ndev", [2, 3, 4, 8])
def test_plan_crossing_in_clamped_round_keeps_first_batch(ndev):
    """Round-2 advisor case: num_tests > 0 and the crossing in the round that num_tests
    clamps, in a slot after earlier kept slots: the re-run must decode the slot's own
    (unclamped) batch up to the cut."""
    batch = 32
    rounds = 2
    N = rounds * batch * ndev
    num_tests = N - batch // 2  # the last slot of round 1 runs half a batch
    for slot in range(1, ndev):
        fe = np.zeros(N, np.uint8)
        first = (rounds - 1) * batch * ndev + slot * batch
        fe[first + batch - 3] = 1 if slot < ndev - 1 else 0
        fe[first + batch // 2 - 2] = 1
        stop = int(fe.sum())
        t, f, r = plan(fe, num_tests, stop, batch, ndev)
        assert (t, f) == sequential(fe, num_tests, stop), slot


def test_plan_trial_limit_only():
    fe = np.zeros(1000, np.uint8)
    for ndev in (1, 2, 5, 8):
        for num_tests in (1, 7, 63, 64, 65, 999):
            t, f, r = plan(fe, num_tests, 0, 8, ndev)
            assert (t, f) == (num_tests, 0)
            assert r == rounds_expected(num_tests, 8, ndev)


def test_plan_reports_reading_past_the_sequence():
    fe = np.zeros(10, np.uint8)
    out = np.zeros(3, np.int64)
    rc = _native.lib().ldpc_debug_mc_plan(fe.ctypes.data, fe.size, 0, 5, 4, 2, out.ctypes.data)
    assert rc == _native.LDPC_EINVAL
