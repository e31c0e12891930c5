"""Device Monte-Carlo engine (the trial loop of parallel_simulator.py:198-244 / :354-379).

One fused launch per batch: channel (Philox) -> decode -> per-trial error
curve; a second launch applies the expurgation filter
(parallel_simulator_expurgated.py:238) and the sequential 200-frame-error stop
rule (parallel_simulator.py:198) and accumulates int64 counters on the device.

Multi-GPU (one process per GPU, torch.distributed): trials shard by index --
rank r of W runs the batch of trials [(round*W + r)*B, +B); the only collective
is one all-reduce per round of [counter deltas | per-rank frame errors | time
flag] (RCCL over xGMI with backend "nccl", gloo on CPU).  The stop rule is the
reference's sequential one in global trial order: in the round that crosses
stop_frame_errors, ranks before the crossing keep their whole batch, the
crossing rank re-runs its batch (Philox streams are keyed by trial index, so
the re-run is identical) with the in-batch cut at its share of the remaining
frame errors, and later ranks drop theirs -- the counters then equal one
process's `while block_error < 200 and i < num_tests` loop exactly.
"""
import time

import numpy as np

from . import _native
from .decoder import ALGOS, CHANNELS


def device_executor(mc):
    """Batch executor backed by ldpc_mc_batch_dev on the current HIP device."""
    torch = mc.torch

    def run(first_cw, B, stop_frame_errors, counters, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream()
        rc = _native.lib().ldpc_mc_batch_dev(mc.graph.handle(), mc.channel, mc.param, mc.seed, int(first_cw),
                                             int(B), mc.max_iters, mc.algo, mc.alpha, int(mc.early_stop),
                                             mc.expurgation, int(stop_frame_errors), counters.data_ptr(),
                                             s.cuda_stream)
        _native.check(rc, "ldpc_mc_batch_dev")
    return run


def ensemble_executor(mc, n, dv, dc):
    """Batch executor for ensemble mode: trial t decodes on its own random (dv, dc)
    graph t (ldpc_mc_ensemble_batch_dev; parallel_simulator.py:198-231 draws a fresh
    code per trial)."""
    torch = mc.torch

    def run(first_cw, B, stop_frame_errors, counters, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream()
        rc = _native.lib().ldpc_mc_ensemble_batch_dev(n, dv, dc, mc.channel, mc.param, mc.seed, int(first_cw), int(B),
                                                      mc.max_iters, mc.expurgation, int(stop_frame_errors),
                                                      counters.data_ptr(), s.cuda_stream)
        _native.check(rc, "ldpc_mc_ensemble_batch_dev")
    return run


def ml_executor(mc):
    """Batch executor of the "optimal" modes (ldpc_mc_ml_batch_dev): ML decoding of each
    trial's BEC word, plus message passing on the same word when mc.message_passing."""
    torch = mc.torch
    ens = isinstance(mc.graph, _Ensemble)

    def run(first_cw, B, stop_frame_errors, counters, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream()
        g = mc.graph
        rc = _native.lib().ldpc_mc_ml_batch_dev(None if ens else g.handle(), g.n, g.dv if ens else 0,
                                                g.dc if ens else 0, mc.param, mc.seed, int(first_cw), int(B),
                                                mc.max_iters, int(mc.message_passing), mc.expurgation,
                                                int(stop_frame_errors),
                                                counters.data_ptr() if mc.message_passing else None,
                                                mc.counters_ml.data_ptr(), s.cuda_stream)
        _native.check(rc, "ldpc_mc_ml_batch_dev")
    return run


class _Ensemble:
    """Stand-in for a graph in ensemble mode (only n is needed by the counters)."""

    def __init__(self, n, dv, dc):
        self.n, self.dv, self.dc = n, dv, dc


class MonteCarlo:
    """counters = [trials, frame_errors, bit_errors, iterations, curve[0..max_iters]] (int64).

    optimal=True adds ML ("optimal") decoding of every trial's BEC word
    (parallel_simulator.py `optimal`, modes 1/2/4/5): counters_ml = [trials,
    ML frame errors, ML bit errors, 0, ML bit errors]; message_passing=False
    drops the BP decode and the stop rule then counts ML frame errors."""

    def __init__(self, graph, channel, param, max_iters, algo="spa", alpha=1.0, early_stop=True,
                 expurgation=-1, seed=0, batch=4096, process_group=None, executor=None, device=None,
                 optimal=False, message_passing=True):
        import torch
        self.torch = torch
        self.graph = graph
        self.channel = CHANNELS[channel]
        self.param = float(param)
        self.max_iters = int(max_iters)
        self.algo = ALGOS[algo]
        self.alpha = float(alpha)
        self.early_stop = bool(early_stop)
        self.expurgation = int(expurgation)
        self.seed = int(seed)
        self.batch = int(batch)
        self.pg = process_group
        dist = torch.distributed
        self.dist = dist if (dist.is_available() and dist.is_initialized()) else None
        self.rank = self.dist.get_rank(process_group) if self.dist else 0
        self.world = self.dist.get_world_size(process_group) if self.dist else 1
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if executor is None else torch.device("cpu")
        self.device = torch.device(device)
        self.counters = torch.zeros(_native.MC_NCOUNT + self.max_iters + 1, dtype=torch.int64, device=self.device)
        self.optimal = bool(optimal)
        self.message_passing = bool(message_passing) or not self.optimal
        self.counters_ml = (torch.zeros(_native.MC_NCOUNT + 1, dtype=torch.int64, device=self.device)
                            if self.optimal else None)
        if self.optimal and self.channel != CHANNELS["bec"]:
            raise ValueError("ML (optimal) decoding is defined for the BEC only")
        if executor is None:
            if self.optimal:
                executor = ml_executor(self)
            elif isinstance(graph, _Ensemble):
                executor = ensemble_executor(self, graph.n, graph.dv, graph.dc)
            else:
                executor = device_executor(self)
        self.executor = executor
        self.rounds = 0
        self.trial_base = 0   # first trial index of round 0 (a restored run continues here)
        self.trial_base0 = 0  # first trial index of the whole run (snapshot trial range)

    def next_trial(self):
        """Index of the first trial the next round runs (all ranks)."""
        return self.trial_base + self.rounds * self.world * self.batch

    def snapshot(self, g=None):
        """Counter snapshot of the run so far (collective when g is None; see snapshot.py)."""
        from . import snapshot
        return snapshot.from_counters(self, self._global() if g is None else g)

    def restore(self, snap):
        """Continue from a snapshot (snapshot.load(path)); see snapshot.restore."""
        from . import snapshot
        snapshot.restore(self, snap)

    @classmethod
    def ensemble(cls, n, dv, dc, channel, param, max_iters, **kw):
        """Fresh random (dv, dc) code per trial (BEC; parallel_simulator.run_simulation)."""
        return cls(_Ensemble(n, dv, dc), channel, param, max_iters, **kw)

    def run_batch(self, first_cw, B, stop_frame_errors=0, stream=None):
        if stream is None:
            self.executor(first_cw, B, stop_frame_errors, self.counters)
        else:
            self.executor(first_cw, B, stop_frame_errors, self.counters, stream)

    def _global(self):
        c = self.counters.clone()
        if self.optimal:
            c = self.torch.cat([c, self.counters_ml])
        if self.dist is not None and self.world > 1:
            if self.dist.get_backend(self.pg) == "gloo":
                c = c.cpu()
            self.dist.all_reduce(c, group=self.pg)
        return c.cpu().numpy()

    def _frames_trials(self, c, c_ml):
        """(frame errors, trials) the stop rules count: BP counters, or ML ones when
        message passing is off (parallel_simulator.py:226-231 / :240-241)."""
        src = c if self.message_passing else c_ml
        return int(src[1]), int(src[0])

    def _run_delta(self, first_cw, B, stop):
        """Run one batch into fresh zero counters; return (delta, delta_ml)."""
        saved = self.counters, self.counters_ml
        self.counters = self.torch.zeros_like(saved[0])
        self.counters_ml = None if saved[1] is None else self.torch.zeros_like(saved[1])
        try:
            if B > 0:
                self.run_batch(first_cw, B, stop)
            return self.counters, self.counters_ml
        finally:
            self.counters, self.counters_ml = saved

    def _add(self, delta):
        self.counters += delta[0]
        if delta[1] is not None:
            self.counters_ml += delta[1]

    def _allreduce(self, vec):
        if self.dist.get_backend(self.pg) == "gloo":
            vec = vec.cpu()
        self.dist.all_reduce(vec, group=self.pg)
        return vec.cpu().numpy()

    def _batch_size(self, num_tests, trials_before, slot):
        """Trials this rank runs in the round: the reference stops at exactly num_tests
        (parallel_simulator.py:198), so the round's last batches are clamped in trial order."""
        if not num_tests:
            return self.batch
        return int(max(0, min(self.batch, num_tests - trials_before - slot * self.batch)))

    def run(self, num_tests, stop_frame_errors=200, time_limit=None, checkpoint=None, checkpoint_every=1):
        """Run rounds until the global counters reach stop_frame_errors frame errors or
        num_tests trials, or time_limit seconds pass (parallel_simulator.py:198).  Counts
        equal one sequential process's over the same trials; the time limit is decided
        collectively (every rank leaves on the same round).  checkpoint: snapshot path rank 0
        rewrites every checkpoint_every rounds and at the end (snapshot.py)."""
        from . import snapshot
        t0 = time.time()
        g = self._global()
        nc = len(self.counters)
        frames, trials = self._frames_trials(g[:nc], g[nc:])
        while True:
            if stop_frame_errors and frames >= stop_frame_errors:
                break
            if num_tests and trials >= num_tests:
                break
            first_cw = self.trial_base + (self.rounds * self.world + self.rank) * self.batch
            B = self._batch_size(num_tests, trials, self.rank)
            if self.world == 1:
                # one process: the exact sequential stop happens inside the batch
                self.run_batch(first_cw, B, stop_frame_errors)
                self.rounds += 1
                g = self._global()
                expired = time_limit is not None and time.time() - t0 > time_limit
            else:
                delta = self._run_delta(first_cw, B, 0)
                f_mine = self._frames_trials(*[None if d is None else d.cpu() for d in delta])[0]
                onehot = self.torch.zeros(self.world + 1, dtype=self.torch.int64, device=self.device)
                onehot[self.rank] = f_mine
                onehot[self.world] = int(time_limit is not None and time.time() - t0 > time_limit)
                parts = [delta[0]] + ([delta[1]] if delta[1] is not None else []) + [onehot]
                red = self._allreduce(self.torch.cat(parts))
                per_rank = red[-(self.world + 1):-1]
                expired = bool(red[-1])
                if stop_frame_errors and frames + int(per_rank.sum()) >= stop_frame_errors:
                    quota = stop_frame_errors - frames - int(per_rank[:self.rank].sum())
                    if quota <= 0:
                        delta = (self.torch.zeros_like(delta[0]),
                                 None if delta[1] is None else self.torch.zeros_like(delta[1]))
                    elif quota <= f_mine:
                        # the crossing rank: cut at its share, in trial order
                        delta = self._run_delta(first_cw, B, quota)
                    self._add(delta)
                    self.rounds += 1
                    g = self._global()
                    break
                self._add(delta)
                self.rounds += 1
                g = g + red[:len(red) - (self.world + 1)]
            frames, trials = self._frames_trials(g[:nc], g[nc:])
            if checkpoint and self.rank == 0 and self.rounds % max(1, checkpoint_every) == 0:
                snapshot.save(self.snapshot(g), checkpoint)
            if expired:
                break
        if checkpoint and self.rank == 0:
            snapshot.save(self.snapshot(g), checkpoint)
        return self.results(g)

    def results(self, g=None):
        g = self._global() if g is None else g
        n = self.graph.n
        nc = len(self.counters)
        out = {}
        if self.optimal:
            ml = g[nc:]
            t = int(ml[0])
            out = {"ml_num_tests": t, "ml_frame_errors": int(ml[1]), "ml_bit_errors": int(ml[2]),
                   "ml_fer": ml[1] / t if t else float("nan"), "ml_ber": ml[2] / (t * n) if t else float("nan")}
            g = g[:nc]
            if not self.message_passing:
                out.update({"num_tests": t, "raw_counters": g})
                return out
        trials = int(g[0])
        curve = g[_native.MC_NCOUNT:].astype(np.float64)
        return {**out,
            "num_tests": trials,
            "frame_errors": int(g[1]),
            "bit_errors": int(g[2]),
            "iterations": int(g[3]),
            "fer": g[1] / trials if trials else float("nan"),
            "ber": g[2] / (trials * n) if trials else float("nan"),
            "error_curve": curve / (n * trials) if trials else curve,
            "raw_counters": g,
        }


def mc_run(graph, channel, param, max_iters, devices=(0,), num_tests=0, stop_frame_errors=200, algo="spa",
           alpha=1.0, early_stop=True, expurgation=-1, seed=0, batch=4096, time_limit=None):
    """A whole run over several devices of THIS process through the C ABI's ldpc_mc_run
    (one RCCL all-reduce per round, exact sequential stop rule; no torch.distributed).
    graph: a TannerGraph (fixed code; irregular graphs go through ldpc_mc_run_csr) or
    ``("ensemble", n, dv, dc)`` for a fresh code per trial.  Returns the same dict as
    MonteCarlo.results."""
    import ctypes as ct
    L = _native.lib()
    C = _native.MC_NCOUNT + int(max_iters) + 1
    counters = np.zeros(C, np.int64)
    rounds = np.zeros(1, np.int64)
    devs = np.ascontiguousarray(devices, dtype=np.int32)
    common = (CHANNELS[channel], float(param), ALGOS[algo], float(alpha), int(bool(early_stop)), int(seed),
              int(max_iters), int(expurgation), int(num_tests or 0), int(stop_frame_errors or 0), int(batch),
              float(time_limit or 0.0), devs.ctypes.data, len(devs), counters.ctypes.data, rounds.ctypes.data)
    if isinstance(graph, tuple) and graph[0] == "ensemble":
        _, n, dv, dc = graph
        rc = L.ldpc_mc_run(None, None, n, n - n * dv // dc, dv, dc, *common)
        name = "ldpc_mc_run"
    elif graph.csr is None:
        v2c = np.ascontiguousarray(graph.variable_lookup, np.int32)
        c2v = np.ascontiguousarray(graph.check_lookup, np.int32)
        n = graph.n
        rc = L.ldpc_mc_run(v2c.ctypes.data, c2v.ctypes.data, graph.n, graph.k, graph.dv, graph.dc, *common)
        name = "ldpc_mc_run"
    else:
        cptr, cvar, vptr, vslot = [np.ascontiguousarray(a, np.int32) for a in graph.to_csr()]
        n = graph.n
        rc = L.ldpc_mc_run_csr(cptr.ctypes.data, cvar.ctypes.data, vptr.ctypes.data, vslot.ctypes.data, graph.n,
                               graph.m, *common)
        name = "ldpc_mc_run_csr"
    _native.check(rc, name)
    trials = int(counters[0])
    curve = counters[_native.MC_NCOUNT:].astype(np.float64)
    return {"num_tests": trials, "frame_errors": int(counters[1]), "bit_errors": int(counters[2]),
            "iterations": int(counters[3]), "fer": counters[1] / trials if trials else float("nan"),
            "ber": counters[2] / (trials * n) if trials else float("nan"),
            "error_curve": curve / (n * trials) if trials else curve, "raw_counters": counters,
            "rounds": int(rounds[0]), "devices": [int(d) for d in devs]}
