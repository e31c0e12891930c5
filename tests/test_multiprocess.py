"""World-size-2 gloo test of the Monte-Carlo sharding + counter all-reduce (CPU only).

The per-batch executor is the oracle (BEC channel + message_passing restatement), so this
checks the distributed logic -- trial partition by rank, one all-reduce per round, global
stop rule -- independently of the GPU kernels (which tests/test_gpu_parity.py pins to the
same oracle counters)."""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle

N, ITERS, B, EPS, SEED = 200, 20, 32, 0.42, 11


def oracle_batch_counters(g, first_cw, Bn, iters, X=-1, remaining=0):
    """Counters of trials first_cw.. on the oracle; remaining > 0 applies the sequential
    stop (parallel_simulator.py:198): keep trials up to the one that brings the frame
    errors to `remaining`."""
    words = oracle.channel(oracle.CH_BEC, EPS, SEED, first_cw, g.n, Bn)
    _, err, its = oracle.bec_decode_batch(words, iters, g.variable_lookup, g.check_lookup, g.n, g.k, g.dv, g.dc)
    c = np.zeros(4 + iters + 1, np.int64)
    for b in range(Bn):
        curve = np.insert(err[b], 0, int(np.count_nonzero(words[b] == 2)))
        if curve[-1] > X:
            c[4:] += curve
            c[1] += curve[-1] != 0
            c[2] += curve[-1]
        c[0] += 1
        c[3] += its[b]
        if remaining and c[1] >= remaining:
            break
    return c


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, num_tests, stop_frames, time_limit, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from iib_project_ldpc_codes_amd.graph import TannerGraph
        from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
        g = TannerGraph.random_regular(N, 3, 6, seed=5)  # every rank builds the same code
        seen = []

        def executor(first_cw, Bn, stop, counters):
            # the device executor's contract: the in-batch cut counts from counters[1]
            seen.append((first_cw, Bn, stop))
            rem = int(stop - counters[1]) if stop else 0
            if stop and rem <= 0:
                return
            counters += torch.from_numpy(oracle_batch_counters(g, first_cw, Bn, ITERS, remaining=rem))
            if time_limit is not None and rank == world - 1:
                time.sleep(0.05)  # this rank's clock runs out later than rank 0's

        mc = MonteCarlo(g, "bec", EPS, ITERS, seed=SEED, batch=B, executor=executor)
        res = mc.run(num_tests=num_tests, stop_frame_errors=stop_frames, time_limit=time_limit)
        q.put((rank, seen, res["raw_counters"].tolist(), mc.rounds))
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda o: o[0])


def sequential_counters(g, num_tests, stop_frames):
    """One process, trial by trial: `while block_error < stop and i < num_tests`."""
    T = num_tests if num_tests else 64 * B
    return oracle_batch_counters(g, 0, T, ITERS, remaining=stop_frames)


@pytest.mark.parametrize("world,num_tests", [(2, 5 * B), (2, 5 * B + 7), (3, 4 * B + 5)])
def test_sharded_mc_matches_single_process(world, num_tests):
    """No frame-error stop: exactly num_tests trials (the last round clamped in trial order)."""
    out = _spawn(_worker, world, num_tests, 0, None)
    rounds = out[0][3]
    assert all(o[3] == rounds for o in out)
    # rank r ran batches (round*W + r)*B: disjoint, covering [0, num_tests)
    runs = sorted((s, n) for o in out for s, n, _ in o[1] if n > 0)
    assert [s for s, _ in runs] == [i * B for i in range(len(runs))]
    assert sum(n for _, n in runs) == num_tests
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    g = TannerGraph.random_regular(N, 3, 6, seed=5)
    want = oracle_batch_counters(g, 0, num_tests, ITERS)
    for o in out:
        np.testing.assert_array_equal(np.array(o[2]), want)


@pytest.mark.parametrize("world,stop", [(2, 5), (2, 17), (3, 11), (4, 40)])
def test_sharded_stop_rule_is_sequential(world, stop):
    """The global frame-error stop cuts at exactly the same trial as one process
    (parallel_simulator.py:198), whichever rank's batch holds the crossing."""
    out = _spawn(_worker, world, 0, stop, None)
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    g = TannerGraph.random_regular(N, 3, 6, seed=5)
    want = sequential_counters(g, 0, stop)
    assert want[1] == stop
    for o in out:
        np.testing.assert_array_equal(np.array(o[2]), want)
    assert len({o[3] for o in out}) == 1


def test_sharded_time_limit_is_collective():
    """A time limit ends every rank on the same round (no rank left waiting in an
    all-reduce), and the counters are the trials of the rounds run."""
    world = 2
    out = _spawn(_worker, world, 0, 0, 0.12)
    rounds = {o[3] for o in out}
    assert len(rounds) == 1
    r = rounds.pop()
    assert r >= 1
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    g = TannerGraph.random_regular(N, 3, 6, seed=5)
    want = oracle_batch_counters(g, 0, r * world * B, ITERS)
    for o in out:
        np.testing.assert_array_equal(np.array(o[2]), want)


def _worker_ml(rank, world, port, num_tests, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from iib_project_ldpc_codes_amd.graph import TannerGraph
        from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
        g = TannerGraph.random_regular(N, 3, 6, seed=5)
        cptr, cvar, _, _ = g.to_csr()
        holder = {}

        def executor(first_cw, Bn, stop, counters):  # ML-only batch on the oracle
            words = oracle.channel(oracle.CH_BEC, EPS, SEED, first_cw, g.n, Bn).astype(np.uint8)
            _, uns = oracle.ml_decode_batch(cptr, cvar, words, g.n, g.m)
            c = holder["mc"].counters_ml
            c[0] += Bn
            c[1] += int((uns > 0).sum())
            c[2] += int(uns.sum())
            c[4] += int(uns.sum())

        mc = MonteCarlo(g, "bec", EPS, ITERS, seed=SEED, batch=B, executor=executor, optimal=True,
                        message_passing=False)
        holder["mc"] = mc
        res = mc.run(num_tests=num_tests, stop_frame_errors=10 ** 9)
        q.put((rank, res["ml_num_tests"], res["ml_frame_errors"], res["ml_bit_errors"], mc.rounds))
    finally:
        dist.destroy_process_group()


def test_sharded_ml_mc_matches_single_process():
    """Optimal (ML-only) mode: the ML counters are all-reduced with the others and the
    trial-count stop uses them (message_passing=False)."""
    world = 2
    num_tests = 3 * B
    out = _spawn(_worker_ml, world, num_tests)
    rounds = out[0][4]
    assert all(o[4] == rounds for o in out)
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    g = TannerGraph.random_regular(N, 3, 6, seed=5)
    cptr, cvar, _, _ = g.to_csr()
    T = num_tests
    words = oracle.channel(oracle.CH_BEC, EPS, SEED, 0, g.n, T).astype(np.uint8)
    _, uns = oracle.ml_decode_batch(cptr, cvar, words, g.n, g.m)
    for o in out:
        assert o[1] == T and o[2] == int((uns > 0).sum()) and o[3] == int(uns.sum())
