"""Counter snapshots (iib_project_ldpc_codes_amd/snapshot.py): checkpoint, resume, merge.

CPU only: the batch executor is the oracle (BEC channel + message_passing restatement), as in
tests/test_multiprocess.py.  A run split by a time limit and resumed from its snapshot -- in one
process, or over two gloo ranks -- counts exactly what one uninterrupted sequential run counts;
merging two seeds' snapshots equals the counter sum (tools/combine_data.py:64-95, exactly)."""
import json
import os

import numpy as np
import pytest
import torch

from iib_project_ldpc_codes_amd import snapshot
from tests.test_multiprocess import B, EPS, ITERS, N, SEED, _spawn, oracle_batch_counters


def _graph():
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    return TannerGraph.random_regular(N, 3, 6, seed=5)


def _mc(g, seed=SEED, calls=None, **kw):
    from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo

    def executor(first_cw, Bn, stop, counters):
        if calls is not None:
            calls.append((first_cw, Bn))
        rem = int(stop - counters[1]) if stop else 0
        if stop and rem <= 0:
            return
        words_seed = seed
        c = oracle_batch_counters_seed(g, first_cw, Bn, words_seed, rem)
        counters += torch.from_numpy(c)
    return MonteCarlo(g, "bec", EPS, ITERS, seed=seed, batch=B, executor=executor, **kw)


def oracle_batch_counters_seed(g, first_cw, Bn, seed, remaining=0):
    if seed == SEED:
        return oracle_batch_counters(g, first_cw, Bn, ITERS, remaining=remaining)
    from oracle import oracle
    words = oracle.channel(oracle.CH_BEC, EPS, seed, first_cw, g.n, Bn)
    _, err, its = oracle.bec_decode_batch(words, ITERS, g.variable_lookup, g.check_lookup, g.n, g.k, g.dv, g.dc)
    c = np.zeros(4 + ITERS + 1, np.int64)
    for b in range(Bn):
        curve = np.insert(err[b], 0, int(np.count_nonzero(words[b] == 2)))
        c[4:] += curve
        c[1] += curve[-1] != 0
        c[2] += curve[-1]
        c[0] += 1
        c[3] += its[b]
        if remaining and c[1] >= remaining:
            break
    return c


def test_checkpoint_resume_equals_uninterrupted(tmp_path):
    g = _graph()
    path = str(tmp_path / "run.json")
    # piece 1: stopped after 3 rounds by num_tests (a stand-in for a lease running out)
    mc = _mc(g)
    mc.run(num_tests=3 * B, stop_frame_errors=0, checkpoint=path)
    snap = snapshot.load(path)
    assert snap["trial_ranges"] == [[0, 3 * B]] and snap["counters"][0] == 3 * B
    # piece 2: a new process resumes at trial 3B and finishes the 200-frame-error run
    calls = []
    mc2 = _mc(g, calls=calls)
    mc2.restore(snap)
    stop = snap["counters"][1] + 15  # the 200 of parallel_simulator.py:198, scaled down
    res = mc2.run(num_tests=0, stop_frame_errors=stop, checkpoint=path)
    assert calls[0][0] == 3 * B
    want = oracle_batch_counters(g, 0, 64 * B, ITERS, remaining=stop)
    np.testing.assert_array_equal(res["raw_counters"], want)
    np.testing.assert_array_equal(snapshot.load(path)["counters"], want)


def test_resume_after_frame_error_stop_continues_after_the_cut(tmp_path):
    """Advisor round 2: a run stopped by the frame-error rule (in-batch cut) ends its trial
    range at the first trial it did not count, so resuming it with a higher stop counts
    exactly what one uninterrupted run to the higher stop counts (no skipped trials)."""
    g = _graph()
    mc = _mc(g)
    first = oracle_batch_counters(g, 0, 64 * B, ITERS)
    s1 = 5
    mc.run(num_tests=0, stop_frame_errors=s1)
    snap = mc.snapshot()
    assert snap["counters"][1] == s1
    assert snap["trial_ranges"][0][1] == snap["counters"][0] < mc.next_trial()  # cut inside a batch
    mc2 = _mc(g)
    mc2.restore(snap)
    s2 = s1 + 7
    res = mc2.run(num_tests=0, stop_frame_errors=s2)
    want = oracle_batch_counters(g, 0, 64 * B, ITERS, remaining=s2)
    np.testing.assert_array_equal(res["raw_counters"], want)
    assert first[1] > s2  # the sequence holds enough frame errors for both stops


def test_restore_rejects_other_configuration(tmp_path):
    g = _graph()
    mc = _mc(g)
    mc.run(num_tests=B, stop_frame_errors=0)
    snap = mc.snapshot()
    with pytest.raises(ValueError):
        _mc(g, seed=SEED + 1).restore(snap)
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    with pytest.raises(ValueError):
        _mc(TannerGraph.random_regular(N, 3, 6, seed=6)).restore(snap)


def test_merge_seeds_and_ranges(tmp_path):
    g = _graph()
    a = _mc(g)
    a.run(num_tests=2 * B, stop_frame_errors=0)
    b = _mc(g, seed=SEED + 100)
    b.run(num_tests=3 * B, stop_frame_errors=0)
    m = snapshot.merge([a.snapshot(), b.snapshot()])
    want = oracle_batch_counters(g, 0, 2 * B, ITERS) + oracle_batch_counters_seed(g, 0, 3 * B, SEED + 100)
    np.testing.assert_array_equal(m["counters"], want)
    r = snapshot.results(m)
    assert r["num_tests"] == 5 * B
    # overlapping trials of one seed are refused; disjoint ranges of one seed are summed
    with pytest.raises(ValueError):
        snapshot.merge([a.snapshot(), a.snapshot()])
    c = _mc(g)
    c.restore(a.snapshot())
    c.counters.zero_()  # only the new trials: [2B, 4B)
    c.trial_base0 = c.trial_base
    c.run(num_tests=2 * B, stop_frame_errors=0)
    m2 = snapshot.merge([a.snapshot(), c.snapshot()])
    np.testing.assert_array_equal(m2["counters"], oracle_batch_counters(g, 0, 4 * B, ITERS))
    with pytest.raises(ValueError):
        snapshot.restore(_mc(g), m2)  # two trial ranges: not resumable


def test_write_csv_reference_format(tmp_path, monkeypatch):
    from iib_project_ldpc_codes_amd import parallel_simulator as ps
    monkeypatch.setattr(ps, "base_directory", str(tmp_path) + os.sep)
    g = _graph()
    mc = _mc(g)
    mc.run(num_tests=2 * B, stop_frame_errors=0)
    snap = mc.snapshot()
    path = snapshot.write_csv(snap, g.k, 3, 6)
    name = os.path.basename(path)
    assert name.startswith(f"regular_code_BEC={EPS}_n={N}_k={g.k}_dv=3_dc=6_it={ITERS}_num={2 * B}_time=")
    rows = open(path).read().strip().split("\n")
    assert len(rows) == ITERS + 1 + 2 and rows[-2].startswith("Message passing block-wise error")
    json.dumps(snap)  # plain JSON


def _resume_worker(rank, world, port, path, stop, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = _graph()
        mc = _mc(g)
        mc.restore(snapshot.load(path))
        res = mc.run(num_tests=0, stop_frame_errors=stop)
        q.put((rank, res["raw_counters"].tolist()))
    finally:
        dist.destroy_process_group()


def test_resume_on_two_ranks_equals_sequential(tmp_path):
    """A one-process piece, then two gloo ranks resuming from its snapshot: exact counts."""
    g = _graph()
    path = str(tmp_path / "run.json")
    _mc(g).run(num_tests=2 * B, stop_frame_errors=0, checkpoint=path)
    stop = snapshot.load(path)["counters"][1] + 23
    out = _spawn(_resume_worker, 2, path, stop)
    want = oracle_batch_counters(g, 0, 64 * B, ITERS, remaining=stop)
    for _, c in out:
        np.testing.assert_array_equal(np.array(c), want)


def test_ensemble_snapshot_records_sampler_stream():
    """An ensemble run's snapshot names the device sampler's stream rule; a snapshot of the
    round 3-5 stream (SAMPLER_RULE_R3, also the one written before the field existed) or of any
    other rule does not resume."""
    from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo

    def executor(first_cw, Bn, stop, counters):
        counters[0] += Bn

    def fresh():
        return MonteCarlo.ensemble(64800, 3, 6, "bec", 0.42, 200, seed=3, batch=16, expurgation=3, executor=executor)

    mc = fresh()
    mc.run(48, stop_frame_errors=0)
    snap = mc.snapshot()
    assert snap["config"]["graph"]["sampler"] == snapshot.SAMPLER_RULE
    same = fresh()
    same.restore(json.loads(json.dumps(snap)))
    assert same.next_trial() == 48
    old = json.loads(json.dumps(snap))
    del old["config"]["graph"]["sampler"]
    r3 = json.loads(json.dumps(snap))
    r3["config"]["graph"]["sampler"] = snapshot.SAMPLER_RULE_R3
    other = json.loads(json.dumps(snap))
    other["config"]["graph"]["sampler"] = "another-stream"
    for bad in (old, r3, other):
        with pytest.raises(ValueError):
            fresh().restore(bad)
