"""Thread scaling of the CPU baselines on this host: the reference's message_passing
(oracle/_ref/ref_bench.so) and the oracle restatement, configs[0] shape."""
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
from oracle import oracle
from iib_project_ldpc_codes_amd.graph import TannerGraph
g = TannerGraph.random_regular(1000, 3, 6, seed=1)
w = oracle.channel(oracle.CH_BEC, 0.40, 5, 0, g.n, 2048)
print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())
for th in (1, 2, 4, 8, 16):
    t = time.perf_counter(); _, _, _, u = oracle.ref_bench_message_passing(w, 50, g.check_lookup, g.variable_lookup, g.n, g.k, 3, 6, th)
    t1 = time.perf_counter() - t
    oracle.set_num_threads(th)
    t = time.perf_counter(); oracle.bec_decode_batch(w, 50, g.variable_lookup, g.check_lookup, g.n, g.k, 3, 6)
    t2 = time.perf_counter() - t
    print(f"threads {th:3d} (omp {u}): ref {2048 / t1:9.0f} w/s   oracle {2048 / t2:9.0f} w/s", flush=True)
