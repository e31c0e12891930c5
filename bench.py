"""Headline benchmark: decoded codewords/s + info-bit Gb/s, (3,6) n=10000, 50-iteration BP.

Workload (BASELINE.json configs[1]): (3,6)-regular n=10000 (k=5000), BI-AWGN
channel LLRs (sigma=0.85, Eb/N0 ~ 1.4 dB), fp32 sum-product, batch 65536
codewords, exactly 50 flooding iterations per codeword (no early stop), one
MI355X per rank.  One step = one ldpc_bp_decode_batch_dev launch over the
65536 HBM-resident LLR frames (posterior + hard decision written back).
Weak scaling: every rank decodes its own 65536-frame batch.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line.  roofline: SURVEY.md 8(d) algorithmic bytes per
codeword-iteration B_it = 2*E*4 + 2*n*4 = 320,000 B over the measured average
kernel duration (HIP events on the launch stream).  cpu_baseline: the oracle's
OpenMP fp32 sum-product (oracle/ldpc_oracle.c, "port": the reference has no
soft decoder) on a bounded sample of the same frames.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_BITS, DV, DC = 10000, 3, 6
ITERS = 50
BATCH = 65536
SIGMA = 0.85
HBM_PEAK_GBPS = 8000.0
# LDS rates per CU per clock by instruction (MI355X_MICROARCH.md, LDS table), 256 CUs at ~2.4 GHz
LDS_CHIP = 256 * 2.4e9
LDS_B_PER_CLK = {"ds_read_b128": 256.0, "ds_read_b32": 128.0, "ds_write_b128": 79.0, "ds_write_b32": 64.0}


def lds_roofline(n, m, dc, dv, cw_iters_per_s):
    """The LDS-resident kernel's own bound: every iteration reads and writes each edge message
    once in the check phase (check pairs, contiguous ds_read_b128 / ds_write_b128) and once in the
    variable phase (gathered, ds_read_b32 / ds_write_b32).  Peak = those bytes at the
    instruction rates."""
    chk = m * dc * 4
    var = n * dv * 4
    t_peak = (chk / LDS_B_PER_CLK["ds_read_b128"] + chk / LDS_B_PER_CLK["ds_write_b128"]
              + var / LDS_B_PER_CLK["ds_read_b32"] + var / LDS_B_PER_CLK["ds_write_b32"]) / LDS_CHIP
    bytes_it = 2 * (chk + var)
    peak = bytes_it / t_peak / 1e9
    achieved = bytes_it * cw_iters_per_s / 1e9
    return {"bound": "lds", "achieved": achieved, "peak": peak, "unit": "GB/s", "frac": achieved / peak,
            "bytes_per_codeword_iteration": bytes_it,
            "note": "informational: the unit this kernel is closest to (messages live in LDS); peak = the "
                    "per-instruction LDS rates of MI355X_MICROARCH.md for this access mix; the kernel "
                    "itself is VALU-bound (DESIGN.md 3.1)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    return ap.parse_args()


def cpu_baseline(graph, llr_host, seconds):
    """Oracle fp32 SPA, OpenMP over frames, bounded to ~`seconds` of wall time."""
    os.environ.setdefault("OMP_NUM_THREADS", str(min(16, os.cpu_count() or 1)))
    from oracle import oracle
    threads = oracle.num_threads()
    csr = oracle.csr_from_lists(graph.variable_lookup, graph.check_lookup, graph.n, graph.m, DV, DC)
    chunk = max(threads, 1) * 2
    done = 0
    t0 = time.perf_counter()
    while True:
        sl = llr_host[done % llr_host.shape[0]:done % llr_host.shape[0] + chunk]
        if sl.shape[0] < chunk:
            sl = llr_host[:chunk]
        oracle.bp_decode_batch(csr, sl, ITERS, 0)
        done += sl.shape[0]
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": done / el, "unit": "codewords/s", "cores": threads, "kind": "port",
            "sample": f"{done} frames of the bench workload ((3,6) n=10000 BI-AWGN sigma={SIGMA}, "
                      f"fp32 sum-product, 50 iterations) in {el:.1f} s, oracle/ldpc_oracle.c OpenMP "
                      f"x{threads} threads (reference has no soft decoder)"}


def valu_roofline(cw_iters_per_s):
    """The unit that bounds the LDS kernel: vector-instruction issue.  VALU
    wave-instructions per codeword-iteration come from the committed PMC profile of this kernel
    (SQ_INSTS_VALU per launch / codeword-iterations); the live rate times that count is compared
    with 256 CUs x 4 SIMDs issuing one wave64 VALU instruction per 4 cycles at 2.4 GHz
    (transcendentals take 8, so frac understates the busy time: busy_frac_pmc is the profile's
    SQ_ACTIVE_INST_VALU share at its own clock)."""
    p = os.path.join(ROOT, "profiles", "r01f_pmc_summary.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    c, ns = d["counters"], d["dispatch_ns"]
    per_it = c["SQ_INSTS_VALU"] / (BATCH * ITERS)
    peak = 256 * 4 * 2.4e9 / 4
    clock = c["GRBM_GUI_ACTIVE"] / 8 / (ns["GRBM_GUI_ACTIVE"] * 1e-9)
    busy = c["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * ns["SQ_ACTIVE_INST_VALU"] * 1e-9 * clock)
    achieved = per_it * cw_iters_per_s
    return {"bound": "valu", "achieved": achieved / 1e9, "peak": peak / 1e9, "unit": "G wave-instr/s",
            "frac": achieved / peak, "valu_instr_per_codeword_iteration": per_it, "busy_frac_pmc": busy,
            "note": "informational: the LDS-resident kernel is VALU-bound; instruction count from "
                    "profiles/r01f_pmc_summary.json"}


def load_traffic():
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % max(ndev, 1))
    backend = os.environ.get("LDPC_DIST_BACKEND", "nccl")  # gloo: rehearse N ranks on one GPU
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local % max(ndev, 1)))
        else:
            dist.init_process_group(backend)

    from iib_project_ldpc_codes_amd import decoder
    from iib_project_ldpc_codes_amd.graph import TannerGraph

    B = args.batch
    g = TannerGraph.random_regular(N_BITS, DV, DC, seed=1)  # identical code on every rank
    k = g.k
    E = g.num_edges
    stream = torch.cuda.current_stream()
    llr = decoder.channel_dev("awgn", SIGMA, 2026, rank * B, g.n, B)  # HBM-resident input
    post = torch.empty_like(llr)
    hard = torch.empty(llr.shape, dtype=torch.uint8, device=llr.device)
    its = torch.empty((B,), dtype=torch.int32, device=llr.device)

    def step():
        decoder.bp_decode_dev(g, llr, ITERS, "spa", early_stop=False, post=post, hard=hard, its=its,
                              stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        step()
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])

    fer = float(hard.any(dim=1).float().mean().item())
    total_cw = world * B * args.steps
    value = total_cw / elapsed
    b_it = 2 * E * 4 + 2 * g.n * 4
    achieved = b_it * B * ITERS / (kernel_ms * 1e-3) / 1e9
    kernel_cw_iters = B * ITERS / (kernel_ms * 1e-3)
    traffic = load_traffic()

    extras = {}
    if not args.no_extras and rank == 0:
        # same frames with syndrome early termination (max 50 iterations)
        decoder.bp_decode_dev(g, llr, ITERS, "spa", early_stop=True, post=post, hard=hard, its=its, stream=stream)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        decoder.bp_decode_dev(g, llr, ITERS, "spa", early_stop=True, post=post, hard=hard, its=its, stream=stream)
        b.record(stream)
        torch.cuda.synchronize()
        et_ms = a.elapsed_time(b)
        extras["early_stop_spa"] = {"codewords_per_s": B / (et_ms * 1e-3),
                                    "mean_iterations": float(its.float().mean().item())}
        a.record(stream)
        decoder.bp_decode_dev(g, llr, ITERS, "minsum", alpha=0.75, post=post, hard=hard, its=its, stream=stream)
        b.record(stream)
        torch.cuda.synchronize()
        extras["minsum_50it_codewords_per_s"] = B / (a.elapsed_time(b) * 1e-3)
        # BEC Monte-Carlo on a fixed code (channel + decode + counters, bit-sliced kernel): the
        # device engine of run_simulation_fixed_ldpc at the configs[0] / configs[4] shapes
        from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
        for key, n_b, eps, its_b, Bb in (("bec_mc_cfg1_n1000_eps0.4_50it", 1000, 0.40, 50, 262144),
                                         ("bec_mc_cfg5_n64800_eps0.4_200it", 64800, 0.40, 200, 4096)):
            gb = TannerGraph.random_regular(n_b, DV, DC, seed=1)
            mc = MonteCarlo(gb, "bec", eps, its_b, seed=9, batch=Bb)
            mc.run_batch(0, Bb)
            torch.cuda.synchronize()
            a.record(stream)
            mc.run_batch(Bb, Bb)
            b.record(stream)
            torch.cuda.synchronize()
            cnt = mc.counters.cpu().numpy()
            extras[key] = {"trials_per_s": Bb / (a.elapsed_time(b) * 1e-3), "batch": Bb,
                           "fer": float(cnt[1] / cnt[0]), "mean_iterations": float(cnt[3] / cnt[0])}
        # BEC erasure decoding (message_passing.c semantics, bit-exact): configs[0] and configs[4] shapes
        for key, n_b, eps, its_b, Bb in (("bec_cfg1_n1000_eps0.4_50it", 1000, 0.40, 50, 65536),
                                         ("bec_cfg5_n64800_eps0.4_200it", 64800, 0.40, 200, 4096)):
            gb = TannerGraph.random_regular(n_b, DV, DC, seed=1)
            w0 = decoder.channel_dev("bec", eps, 5, 0, n_b, Bb)
            w = w0.clone()
            decoder.bec_decode_dev(gb, w, its_b)
            w = w0.clone()
            torch.cuda.synchronize()
            a.record(stream)
            _, _, its_bec = decoder.bec_decode_dev(gb, w, its_b)
            b.record(stream)
            torch.cuda.synchronize()
            extras[key] = {"codewords_per_s": Bb / (a.elapsed_time(b) * 1e-3),
                           "mean_iterations": float(its_bec.float().mean().item()), "batch": Bb}
            del w, w0
        # configs[3] shape: irregular RSU rate-1/2 ensemble (density-evolution lambda/rho),
        # n = 20000, BI-AWGN sum-product, 100 iterations, fixed count and with early stop
        from iib_project_ldpc_codes_amd import ensembles
        gi = ensembles.sample_irregular(ensembles.RSU_DL4, 20000, seed=1)
        Bi = 8192
        llr_i = decoder.channel_dev("awgn", 0.80, 7, 0, gi.n, Bi)
        for key, et in (("irregular_cfg4_n20000_spa_100it", False), ("irregular_cfg4_n20000_spa_early_stop", True)):
            _, _, its_i = decoder.bp_decode_dev(gi, llr_i, 100, "spa", early_stop=et, want_post=False)
            torch.cuda.synchronize()
            a.record(stream)
            _, _, its_i = decoder.bp_decode_dev(gi, llr_i, 100, "spa", early_stop=et, want_post=False)
            b.record(stream)
            torch.cuda.synchronize()
            extras[key] = {"codewords_per_s": Bi / (a.elapsed_time(b) * 1e-3), "batch": Bi, "sigma": 0.80,
                           "mean_iterations": float(its_i.float().mean().item()),
                           "kernel": gi.kernel_name(early_stop=et)}
        del llr_i
        # "optimal" modes: ML erasure decoding (parallel_simulator.py:60-129), n = 1000, eps = 0.45
        gm = TannerGraph.random_regular(1000, DV, DC, seed=1)
        wm = decoder.channel_dev("bec", 0.45, 5, 0, gm.n, 32768)
        decoder.ml_decode_dev(gm, wm)
        torch.cuda.synchronize()
        a.record(stream)
        decoder.ml_decode_dev(gm, wm)
        b.record(stream)
        torch.cuda.synchronize()
        extras["ml_n1000_eps0.45"] = {"words_per_s": 32768 / (a.elapsed_time(b) * 1e-3), "batch": 32768}

    cpu = None
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(g, llr[:256].cpu().numpy(), args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "decoded codewords/sec + info-bit Gb/s, (3,6) n=10k 50-iter BP, 1/2/4/8 MI355X",
            "value": value,
            "unit": "codewords/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: BI-AWGN LLRs (Philox, all-zero codeword), seeded (3,6) configuration-model code",
            "config": {"workload": "(3,6)-regular n=10000 BI-AWGN sum-product fp32, batch 65536, 50 iterations "
                                   "(BASELINE.json configs[1])",
                       "n": g.n, "k": k, "edges": E, "batch_per_gpu": B, "iterations": ITERS,
                       "sigma": SIGMA, "early_stop": False, "parallelism": f"trials sharded x{world}",
                       "kernel": g.kernel_name(False)},
            "info_bit_gbps": value * k / 1e9,
            "codeword_iterations_per_s": value * ITERS,
            "kernel_ms_per_launch": kernel_ms,
            "fer_at_sigma": fer,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS,
                         "traffic": traffic.get("bytes_per_launch") if traffic else None,
                         "algorithmic_bytes_per_codeword_iteration": b_it,
                         "note": "algorithmic bytes = SURVEY.md 8(d) streaming model; this kernel keeps the "
                                 "messages in LDS, so its measured HBM traffic is "
                                 + (f"{traffic['bytes_per_codeword'] / 1e3:.0f} KB" if traffic else "~100 KB")
                                 + " per codeword (channel LLRs in, posteriors + decisions out), not "
                                 f"{b_it * ITERS / 1e6:.0f} MB; the kernel is VALU-bound (DESIGN.md 3.1)"},
            "lds_roofline": lds_roofline(g.n, g.m, DC, DV, kernel_cw_iters),
            "valu_roofline": valu_roofline(kernel_cw_iters),
            "cpu_baseline": cpu,
            "extras": extras,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
