"""World-size-2 gloo test of the Monte-Carlo sharding + counter all-reduce (CPU only).

The per-batch executor is the oracle (BEC channel + message_passing restatement), so this
checks the distributed logic -- trial partition by rank, one all-reduce per round, global
stop rule -- independently of the GPU kernels (which tests/test_gpu_parity.py pins to the
same oracle counters)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle

N, ITERS, B, EPS, SEED = 200, 20, 32, 0.42, 11


def oracle_batch_counters(g, first_cw, Bn, iters, X=-1):
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
    return c


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, num_tests, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from iib_project_ldpc_codes_amd.graph import TannerGraph
        from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
        g = TannerGraph.random_regular(N, 3, 6, seed=5)  # every rank builds the same code
        seen = []

        def executor(first_cw, Bn, stop, counters):
            seen.append(first_cw)
            counters += torch.from_numpy(oracle_batch_counters(g, first_cw, Bn, ITERS))

        mc = MonteCarlo(g, "bec", EPS, ITERS, seed=SEED, batch=B, executor=executor)
        res = mc.run(num_tests=num_tests, stop_frame_errors=10 ** 9)
        q.put((rank, seen, res["raw_counters"].tolist(), mc.rounds))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_mc_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    num_tests = 5 * B
    procs = [ctx.Process(target=_worker, args=(r, world, port, num_tests, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    rounds = out[0][3]
    assert all(o[3] == rounds for o in out)
    # rank r ran batches (round*W + r)*B: disjoint, covering [0, rounds*W*B)
    starts = sorted(s for o in out for s in o[1])
    assert starts == [i * B for i in range(rounds * world)]
    assert rounds * world * B >= num_tests
    # both ranks see the same global counters == one process over the same trials
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    g = TannerGraph.random_regular(N, 3, 6, seed=5)
    want = oracle_batch_counters(g, 0, rounds * world * B, ITERS)
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
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    num_tests = 3 * B
    procs = [ctx.Process(target=_worker_ml, args=(r, world, port, num_tests, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rounds = out[0][4]
    assert all(o[4] == rounds for o in out) and rounds * world * B >= num_tests
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    g = TannerGraph.random_regular(N, 3, 6, seed=5)
    cptr, cvar, _, _ = g.to_csr()
    T = rounds * world * B
    words = oracle.channel(oracle.CH_BEC, EPS, SEED, 0, g.n, T).astype(np.uint8)
    _, uns = oracle.ml_decode_batch(cptr, cvar, words, g.n, g.m)
    for o in out:
        assert o[1] == T and o[2] == int((uns > 0).sum()) and o[3] == int(uns.sum())
