"""Device Monte-Carlo engine (the trial loop of parallel_simulator.py:198-244 / :354-379).

One fused launch per batch: channel (Philox) -> decode -> per-trial error
curve; a second launch applies the expurgation filter
(parallel_simulator_expurgated.py:238) and the sequential 200-frame-error stop
rule (parallel_simulator.py:198) and accumulates int64 counters on the device.

Multi-GPU (one process per GPU, torch.distributed): trials shard by index --
rank r of W runs batches (round * W + r); the only collective is one
all-reduce of the counter vector per round (RCCL over xGMI with backend
"nccl", gloo on CPU), used for the global stop rule and the final result.
"""
import time

import numpy as np

from . import _native
from .decoder import ALGOS, CHANNELS


class MonteCarlo:
    def __init__(self, graph, channel, param, max_iters, algo="spa", alpha=1.0, early_stop=True,
                 expurgation=-1, seed=0, batch=4096, process_group=None):
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
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.counters = torch.zeros(_native.MC_NCOUNT + self.max_iters + 1, dtype=torch.int64, device=self.device)
        self.rounds = 0

    def run_batch(self, first_cw, B, stop_frame_errors=0, stream=None):
        s = stream if stream is not None else self.torch.cuda.current_stream()
        rc = _native.lib().ldpc_mc_batch_dev(self.graph.handle(), self.channel, self.param, self.seed,
                                             int(first_cw), int(B), self.max_iters, self.algo, self.alpha,
                                             int(self.early_stop), self.expurgation, int(stop_frame_errors),
                                             self.counters.data_ptr(), s.cuda_stream)
        _native.check(rc, "ldpc_mc_batch_dev")

    def _global(self):
        c = self.counters.clone()
        if self.dist is not None and self.world > 1:
            backend = self.dist.get_backend(self.pg)
            if backend == "gloo":
                c = c.cpu()
                self.dist.all_reduce(c, group=self.pg)
            else:
                self.dist.all_reduce(c, group=self.pg)
        return c.cpu().numpy()

    def run(self, num_tests, stop_frame_errors=200, time_limit=None):
        """Run until stop_frame_errors frame errors (global), num_tests trials or time_limit seconds."""
        t0 = time.time()
        first_round = self.rounds
        while True:
            r = self.rounds
            first_cw = (r * self.world + self.rank) * self.batch
            # single process: exact sequential stop inside the batch
            stop = stop_frame_errors if self.world == 1 else 0
            self.run_batch(first_cw, self.batch, stop)
            self.rounds += 1
            g = self._global()
            if stop_frame_errors and g[1] >= stop_frame_errors:
                break
            if num_tests and g[0] >= num_tests:
                break
            if time_limit is not None and time.time() - t0 > time_limit:
                break
            if self.rounds - first_round > 10 ** 9:
                break
        return self.results(g)

    def results(self, g=None):
        g = self._global() if g is None else g
        n = self.graph.n
        trials = int(g[0])
        curve = g[_native.MC_NCOUNT:].astype(np.float64)
        return {
            "num_tests": trials,
            "frame_errors": int(g[1]),
            "bit_errors": int(g[2]),
            "iterations": int(g[3]),
            "fer": g[1] / trials if trials else float("nan"),
            "ber": g[2] / (trials * n) if trials else float("nan"),
            "error_curve": curve / (n * trials) if trials else curve,
            "raw_counters": g,
        }
