"""Counter snapshots: checkpoint / resume a Monte-Carlo run and merge runs exactly.

The reference keeps no state between runs; long campaigns are split over processes and HPC jobs
whose per-iteration CSV curves are merged afterwards by tools/combine_data.py:64-95 (curves
re-scaled by num*n, summed, divided by the total num).  Here a run's state is its int64
counter vector (montecarlo.MonteCarlo: [trials, frame_errors, bit_errors, iterations,
curve[0..max_iters]]) plus the next trial index, so

* ``save(mc, path)`` writes that state (JSON, atomically) -- MonteCarlo.run(checkpoint=path)
  does it every ``checkpoint_every`` rounds, so a run cut off by a lease or time limit loses
  at most that many rounds;
* ``restore(mc, snap)`` continues a run at the next trial index (same Philox streams, so a
  run split into pieces counts exactly what one uninterrupted run counts);
* ``merge(snaps)`` sums runs of one configuration whose trials are disjoint (different seeds,
  or disjoint trial ranges of one seed) -- exact integer sums where combine_data.py re-derives
  counts from rounded floats;
* ``write_csv(snap, ...)`` emits the reference's message-passing CSV (parallel_simulator.py:
  26-42 row format, :250-260 filename schema) for tools/plotting.py.
"""
import hashlib
import json
import os

import numpy as np

VERSION = 1


# The device sampler's graph stream (csrc/sampler.hip: which graph trial t gets): a resumed
# ensemble run must draw its remaining graphs from the stream its first part drew from.
# Round 6 changed the sequential-draw stream (one Philox4x32-7 block = two words of a slot pair,
# was one Philox4x32-10 word of four slots; stages end at half the pool, was a quarter):
# SAMPLER_RULE_R3 is the stream of rounds 3-5, and of the snapshots written before the field
# existed (round 3) -- they no longer resume.
SAMPLER_RULE = "one-level-rs/philox4x32-10<8192<=seq-draw-pair-words/philox4x32-7/split2<=393216"
SAMPLER_RULE_R3 = "one-level-rs<8192<=seq-draw<=393216/philox4x32-10"


def graph_fingerprint(graph):
    """Identity of the code a run decodes: the edge lists' digest, or the ensemble parameters
    (with the device sampler's stream rule)."""
    if not hasattr(graph, "variable_lookup") and hasattr(graph, "dv"):  # montecarlo._Ensemble
        return {"kind": "ensemble", "n": int(graph.n), "dv": int(graph.dv), "dc": int(graph.dc),
                "sampler": SAMPLER_RULE}
    h = hashlib.sha1()
    if getattr(graph, "csr", None) is not None:
        for a in graph.csr:
            h.update(np.ascontiguousarray(a, np.int32).tobytes())
    else:
        h.update(np.ascontiguousarray(graph.variable_lookup, np.int32).tobytes())
        h.update(np.ascontiguousarray(graph.check_lookup, np.int32).tobytes())
    return {"kind": "fixed", "n": int(graph.n), "sha1": h.hexdigest()}


def config(mc):
    return {"graph": graph_fingerprint(mc.graph), "channel": int(mc.channel), "param": float(mc.param),
            "max_iters": int(mc.max_iters), "algo": int(mc.algo), "alpha": float(mc.alpha),
            "early_stop": bool(mc.early_stop), "expurgation": int(mc.expurgation),
            "optimal": bool(mc.optimal), "message_passing": bool(mc.message_passing)}


def from_counters(mc, g):
    """Snapshot dict from global counters g (numpy, BP counters then ML counters).

    The trial range ends at the first trial NOT counted.  The stop rule counts trials in
    global trial order from the run's first trial (the in-batch cut, later ranks' dropped
    batches, the num_tests clamp), so the counted trials are exactly [trial_base0,
    trial_base0 + trials) -- which is next_trial() only when every round ran whole batches.
    Resuming a stopped run with a higher stop then continues right after the cut."""
    nc = len(mc.counters)
    _, trials = mc._frames_trials(g[:nc], g[nc:])
    return {"version": VERSION, "config": config(mc), "seed": int(mc.seed),
            "trial_ranges": [[int(mc.trial_base0), int(mc.trial_base0) + int(trials)]],
            "counters": [int(x) for x in g[:nc]],
            "counters_ml": [int(x) for x in g[nc:]] if mc.optimal else None}


def save(snap, path):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(snap, f)
    os.replace(tmp, path)


def load(path):
    with open(path) as f:
        snap = json.load(f)
    if snap.get("version") != VERSION:
        raise ValueError(f"{path}: snapshot version {snap.get('version')} (want {VERSION})")
    return snap


def restore(mc, snap):
    """Continue `mc` from `snap`: same configuration and seed required.  Rank 0 carries the
    restored counts (the per-round all-reduce sums them in); every rank continues at the
    snapshot's next trial index."""
    have = json.loads(json.dumps(snap["config"]))
    if have.get("graph", {}).get("kind") == "ensemble":
        have["graph"].setdefault("sampler", SAMPLER_RULE_R3)  # pre-field snapshots: the round-3 stream
    if have != config(mc) or snap["seed"] != mc.seed:
        raise ValueError("snapshot is of a different run configuration, sampler stream or seed")
    if len(snap["trial_ranges"]) != 1:
        raise ValueError("a merged snapshot cannot be resumed (its trials are not one range)")
    t = mc.torch
    c = np.asarray(snap["counters"], np.int64)
    mc.counters.copy_(t.from_numpy(c if mc.rank == 0 else np.zeros_like(c)).to(mc.counters.device))
    if mc.optimal:
        cm = np.asarray(snap["counters_ml"], np.int64)
        mc.counters_ml.copy_(t.from_numpy(cm if mc.rank == 0 else np.zeros_like(cm)).to(mc.counters.device))
    mc.trial_base0 = int(snap["trial_ranges"][0][0])
    mc.trial_base = int(snap["trial_ranges"][0][1])
    mc.rounds = 0


def _disjoint(ranges_a, ranges_b):
    return all(a1 <= b0 or b1 <= a0 for a0, a1 in ranges_a for b0, b1 in ranges_b)


def merge(snaps):
    """Sum snapshots of one configuration over disjoint trials (tools/combine_data.py:64-95,
    exactly).  Snapshots of one seed must cover disjoint trial ranges; different seeds are
    independent Philox streams."""
    if not snaps:
        raise ValueError("nothing to merge")
    cfg = snaps[0]["config"]
    by_seed = {}
    out_c = np.zeros(len(snaps[0]["counters"]), np.int64)
    out_ml = None if snaps[0]["counters_ml"] is None else np.zeros(len(snaps[0]["counters_ml"]), np.int64)
    for s in snaps:
        if s["config"] != cfg:
            raise ValueError("snapshots of different configurations cannot be merged")
        prev = by_seed.setdefault(s["seed"], [])
        if not _disjoint(prev, s["trial_ranges"]):
            raise ValueError(f"snapshots of seed {s['seed']} overlap in trials")
        prev.extend(s["trial_ranges"])
        out_c += np.asarray(s["counters"], np.int64)
        if out_ml is not None:
            out_ml += np.asarray(s["counters_ml"], np.int64)
    seeds = sorted(by_seed)
    return {"version": VERSION, "config": cfg, "seed": seeds[0] if len(seeds) == 1 else None,
            "seeds": {str(k): v for k, v in by_seed.items()},
            "trial_ranges": by_seed[seeds[0]] if len(seeds) == 1 else [],
            "counters": [int(x) for x in out_c],
            "counters_ml": None if out_ml is None else [int(x) for x in out_ml]}


def results(snap):
    """The same dict MonteCarlo.results gives, from a snapshot."""
    n = snap["config"]["graph"]["n"]
    g = np.asarray(snap["counters"], np.int64)
    t = int(g[0])
    curve = g[4:].astype(np.float64)
    return {"num_tests": t, "frame_errors": int(g[1]), "bit_errors": int(g[2]), "iterations": int(g[3]),
            "fer": g[1] / t if t else float("nan"), "ber": g[2] / (t * n) if t else float("nan"),
            "error_curve": curve / (n * t) if t else curve, "raw_counters": g}


def write_csv(snap, k, dv, dc, prefix="regular_code"):
    """Reference CSV (message passing rows, parallel_simulator.py:26-42) for a BEC snapshot;
    returns the file path (parallel_simulator.py:250-260 name schema, num = merged trials)."""
    from . import parallel_simulator as ps
    r = results(snap)
    n = snap["config"]["graph"]["n"]
    name = ps._filename(prefix, {"BEC": snap["config"]["param"]}, n, k, dv, dc, snap["config"]["max_iters"],
                        r["num_tests"])
    ps.write_message_passing_file(name, r["error_curve"], r["fer"], r["ber"])
    return ps._out_path(name)
