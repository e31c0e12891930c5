"""Multi-rank Monte-Carlo on the device path: W processes (gloo process group, all on
cuda:0 -- the one GPU of the test box) run montecarlo.MonteCarlo with the HIP executor and
the global 200-frame-error stop rule; their counters must equal one process's sequential
run over the same trials exactly (parallel_simulator.py:198: `while block_error < 200 and
i < num_tests`).  The 8-GPU RCCL form differs only in the backend of the all-reduce."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CASES = {
    "bec": dict(channel="bec", param=0.42, n=1000, iters=40, algo="spa", early_stop=True, batch=256),
    "bsc_minsum": dict(channel="bsc", param=0.07, n=1000, iters=50, algo="minsum", early_stop=True, batch=256),
    "awgn_spa": dict(channel="awgn", param=0.88, n=1000, iters=50, algo="spa", early_stop=False, batch=256),
}
SEED, STOP = 31, 200


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mc(case):
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
    c = CASES[case]
    g = TannerGraph.random_regular(c["n"], 3, 6, seed=4)
    return MonteCarlo(g, c["channel"], c["param"], c["iters"], algo=c["algo"], alpha=0.75 if c["algo"] == "minsum"
                      else 1.0, early_stop=c["early_stop"], seed=SEED, batch=c["batch"])


def _worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mc = _mc(case)
        res = mc.run(num_tests=0, stop_frame_errors=STOP)
        q.put((rank, res["raw_counters"].tolist(), mc.rounds))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", sorted(CASES))
def test_two_ranks_equal_sequential(case):
    import torch
    ref = _mc(case)
    want = ref.run(num_tests=0, stop_frame_errors=STOP)["raw_counters"]
    torch.cuda.synchronize()
    assert want[1] == STOP
    assert want[0] > ref.batch  # the crossing is past the first batch: rank 1's share matters
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, counters, rounds in out:
        np.testing.assert_array_equal(np.array(counters), want, err_msg=f"rank {rank}")


# ------------------------------------------- ldpc_mc_run (one process, RCCL over devices)
@pytest.mark.parametrize("case", sorted(CASES))
def test_mc_run_one_device_equals_montecarlo(case):
    """ldpc_mc_run through ctypes on device 0 (RCCL communicator of one rank): same
    counters as montecarlo.MonteCarlo's sequential run, stop rule inside a batch."""
    from iib_project_ldpc_codes_amd import montecarlo
    c = CASES[case]
    ref = _mc(case)
    want = ref.run(num_tests=0, stop_frame_errors=STOP)["raw_counters"]
    got = montecarlo.mc_run(ref.graph, c["channel"], c["param"], c["iters"], devices=(0,), num_tests=0,
                            stop_frame_errors=STOP, algo=c["algo"], alpha=ref.alpha, early_stop=c["early_stop"],
                            seed=SEED, batch=c["batch"])
    np.testing.assert_array_equal(got["raw_counters"], want)
    assert got["rounds"] == ref.rounds


def test_mc_run_num_tests_clamp_and_ensemble():
    """num_tests is met exactly (last batch clamped) -- fixed code and ensemble mode."""
    import torch
    from iib_project_ldpc_codes_amd import montecarlo
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
    g = TannerGraph.random_regular(1000, 3, 6, seed=4)
    got = montecarlo.mc_run(g, "bec", 0.42, 40, devices=(0,), num_tests=1000, stop_frame_errors=0, seed=3,
                            batch=256)
    ref = MonteCarlo(g, "bec", 0.42, 40, seed=3, batch=256)
    for first, B in ((0, 256), (256, 256), (512, 256), (768, 232)):
        ref.run_batch(first, B)
    torch.cuda.synchronize()
    assert got["num_tests"] == 1000
    np.testing.assert_array_equal(got["raw_counters"], ref.counters.cpu().numpy())
    ens = montecarlo.mc_run(("ensemble", 200, 3, 6), "bec", 0.40, 20, devices=(0,), num_tests=150,
                            stop_frame_errors=0, seed=17, batch=96, expurgation=1)
    mce = MonteCarlo.ensemble(200, 3, 6, "bec", 0.40, 20, seed=17, batch=96, expurgation=1)
    mce.run_batch(0, 96)
    mce.run_batch(96, 54)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ens["raw_counters"], mce.counters.cpu().numpy())
