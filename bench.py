"""Headline benchmark: decoded codewords/s + info-bit Gb/s, (3,6) n=10000, 50-iteration BP.

Workload (BASELINE.json configs[1]): (3,6)-regular n=10000 (k=5000), BI-AWGN
channel LLRs (sigma=0.85, Eb/N0 ~ 1.4 dB), fp32 sum-product, batch 65536
codewords, exactly 50 flooding iterations per codeword (no early stop), one
MI355X per rank.  One step = one ldpc_bp_decode_batch_dev launch over the
65536 HBM-resident LLR frames (posterior + hard decision written back).
Weak scaling: every rank decodes its own 65536-frame batch.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line.  roofline: the decode kernel keeps every edge
message in LDS, so its binding unit is on-chip: LDS-array cycles (per CU,
PMC SQ_LDS_IDX_ACTIVE) or VALU-busy cycles (per SIMD, PMC SQ_ACTIVE_INST_VALU)
per codeword-iteration, both measured by counters in the committed profile of
this kernel (ISSUE_PROFILE below, scripts/issue_model.py), x the live
codeword-iteration rate of the kernel (HIP events on the launch stream) over
the unit's peak; the larger fraction is `roofline` (the issue model at the
measured VALU prices rides beside it).  roofline.hbm_model
keeps SURVEY.md 8(d)'s streaming byte model (2*E*4 + 2*n*4 = 320,000 B per
codeword-iteration, above the HBM peak by design) beside the measured HBM
traffic (PMC FETCH_SIZE/WRITE_SIZE).  cpu_baseline: the oracle's OpenMP fp32
sum-product ("port": the reference has no soft decoder) on all host cores this
job may use and on one core, plus the reference's own message_passing.c (BEC
hot path, configs[0] shape) on the same cores -- bounded samples, stated.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from iib_project_ldpc_codes_amd.launch import launch_plan, spawn_ranks  # noqa: E402,F401

N_BITS, DV, DC = 10000, 3, 6
ITERS = 50
BATCH = 65536
SIGMA = 0.85
HBM_PEAK_GBPS = 8000.0
def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); without torchrun's WORLD_SIZE, bench.py starts them itself")
    ap.add_argument("--rehearse-on-one-gpu", action="store_true",
                    help="allow more ranks than visible GPUs (ranks share devices, gloo collectives): "
                         "a rehearsal of the N-rank path on a one-GPU box, not a scaling measurement")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    return ap.parse_args(argv)


def host_cores():
    """Host cores this process may use: the CPU affinity set, capped by a cgroup CPU quota
    (the GPU box hands each one-GPU job a share of a larger machine; os.cpu_count() reports
    the whole machine).  Returns (cores, os_cpu_count, detail)."""
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = total
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    cores = min(aff, quota) if quota else aff
    env = {k: v for k, v in os.environ.items() if k.startswith(("OMP_", "GOMP_"))}
    return cores, total, {"os_cpu_count": total, "affinity": aff, "cgroup_quota_cpus": quota, "omp_env": env}


def _timed(fn, chunk, seconds):
    """Call fn(i) on successive chunks until `seconds` of wall time; returns (items, elapsed)."""
    done, i = 0, 0
    t0 = time.perf_counter()
    while True:
        done += fn(i)
        i += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return done, el


def cpu_baseline(graph, llr_host, seconds):
    """CPU baselines timed on this host in the same run (rank 0, N=1), on bounded samples.

    value: the oracle's fp32 sum-product in the GPU kernel's formulation (oracle/ldpc_oracle.c
    algo 2, "port": the reference has no soft decoder) on every host core this job may use;
    single_core: the same on one thread; bec_reference_path: the reference's own message_passing.c (compiled unchanged into
    oracle/_ref/ref_bench.so, one word per call as parallel_simulator.py:131-166) at the
    configs[0] shape, all cores and one core."""
    from oracle import oracle
    cores, total, detail = host_cores()
    csr = oracle.csr_from_lists(graph.variable_lookup, graph.check_lookup, graph.n, graph.m, DV, DC)
    F = llr_host.shape[0]

    def spa(threads, secs):
        oracle.set_num_threads(threads)
        chunk = 2 * threads

        def fn(i):
            lo = (i * chunk) % F
            sl = llr_host[lo:lo + chunk] if lo + chunk <= F else llr_host[:chunk]
            oracle.bp_decode_batch(csr, sl, ITERS, 2)  # algo 2: fp32, the GPU kernel's check formulation
            return sl.shape[0]
        return _timed(fn, chunk, secs)

    done_all, el_all = spa(cores, seconds * 0.45)
    done_one, el_one = spa(1, seconds * 0.2)
    out = {"value": done_all / el_all, "unit": "codewords/s", "cores": cores, "kind": "port",
           "sample": f"{done_all} frames of the bench workload ((3,6) n=10000 BI-AWGN sigma={SIGMA}, fp32 "
                     f"sum-product, 50 iterations; drawn from the first {F} frames of the batch) in "
                     f"{el_all:.1f} s, oracle/ldpc_oracle.c algo 2 (fp32, the kernel's elementary-symmetric check "
                     f"form) OpenMP x{cores} threads (the reference has no soft decoder)",
           "host": detail,
           "single_core": {"value": done_one / el_one, "unit": "codewords/s", "cores": 1,
                           "sample": f"{done_one} frames in {el_one:.1f} s"}}
    if total != cores:
        # one thread per CPU os.cpu_count() reports, for the record: the job's cgroup quota caps
        # what they can use, so this is not more compute than `value`'s `cores` threads
        done_os, el_os = spa(total, seconds * 0.15)
        out["os_cpu_count_threads"] = {"value": done_os / el_os, "unit": "codewords/s", "threads": total,
                                       "cgroup_quota_cpus": detail["cgroup_quota_cpus"],
                                       "sample": f"{done_os} frames in {el_os:.1f} s"}
    # the reference hot path itself: message_passing.c at configs[0] (n=1000, eps=0.4, 50 iterations)
    gb = graph_cfg0()
    words = oracle.channel(oracle.CH_BEC, 0.40, 5, 0, gb.n, 4096)
    kind = "reference" if oracle.ref_bench_available() else "port"

    used = []

    def bec(threads, secs):
        if kind == "reference":
            # a fresh interpreter (no torch / HIP runtime threads): the reference's C on the
            # host cores exactly as a CPU-only run would use them
            import multiprocessing as mp
            with mp.get_context("spawn").Pool(1) as pool:
                done, el, u = pool.apply(oracle.ref_bench_timed, (words, 50, gb.check_lookup, gb.variable_lookup,
                                                                  gb.n, gb.k, DV, DC, threads, secs))
            used.append(u)
            return done, el
        oracle.set_num_threads(threads)
        chunk = 64 * threads

        def fn(i):
            lo = (i * chunk) % words.shape[0]
            sl = words[lo:lo + chunk] if lo + chunk <= words.shape[0] else words[:chunk]
            oracle.bec_decode_batch(sl, 50, gb.variable_lookup, gb.check_lookup, gb.n, gb.k, DV, DC)
            return sl.shape[0]
        return _timed(fn, chunk, secs)

    b_all, e_all = bec(cores, seconds * 0.2)
    b_one, e_one = bec(1, seconds * 0.15)
    out["bec_reference_path"] = {
        "value": b_all / e_all, "unit": "codewords/s", "cores": cores, "kind": kind,
        "single_core": b_one / e_one, "threads_reported_by_openmp": sorted(set(used)),
        "sample": f"configs[0] shape: (3,6) n=1000 BEC eps=0.4, 50 iterations; {b_all} words in {e_all:.1f} s "
                  f"on {cores} threads, {b_one} in {e_one:.1f} s on one; "
                  + ("reference message_passing.c compiled unchanged (oracle/_ref/ref_bench.so)"
                     if kind == "reference" else "oracle restatement (reference build absent)")}
    oracle.set_num_threads(cores)
    return out


DROPIN_NS = (1000, 10000)
DROPIN_EPS = 0.40


def dropin_words(n, count, seed):
    """BEC channel words of the all-zero codeword (0 / 2 = erased, int32 like
    parallel_simulator.py:151), synthetic, eps = DROPIN_EPS."""
    import numpy as np
    rng = np.random.default_rng(seed)
    return np.where(rng.random((count, n)) < DROPIN_EPS, 2, 0).astype(np.int32)


def _call_loop(call, words, seconds):
    """One call per word, cycling through `words`, for `seconds`: (calls, elapsed)."""
    return _timed(lambda i: (call(words[i % len(words)]), 1)[1], 1, seconds)


def dropin_gpu_rates(seconds):
    """The reference's literal call surface on this library: one message_passing call per word
    through ctypes with the marshalling of parallel_simulator.py:131-166 (the mirror's
    regular_LDPC_code.message_pass_decode: int32 copies of the lists and the word, errors[],
    the call), 50 iterations, at n = 1000 and 10000.  fixed_code: the same lists every call
    (parallel_simulator.py:354-379, the cached device graph); new_graph_each_call: two codes
    of the same shape alternating (the ensemble loop, :198-223, re-sends a new code per trial)."""
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    from iib_project_ldpc_codes_amd.parallel_simulator import regular_LDPC_code
    out = {}
    for n in DROPIN_NS:
        ga, gb = (TannerGraph.random_regular(n, DV, DC, seed=s) for s in (1, 2))
        code = regular_LDPC_code(None, n, ga.k, DV, DC)
        words = dropin_words(n, 64, 11)
        lists = [(ga.check_lookup, ga.variable_lookup), (gb.check_lookup, gb.variable_lookup)]
        code.message_pass_decode(words[0], ITERS, *lists[0])  # graph upload, stream, staging
        c_fix, e_fix = _call_loop(lambda w: code.message_pass_decode(w, ITERS, *lists[0]), words, seconds)
        state = [0]

        def alt(w):
            state[0] ^= 1
            return code.message_pass_decode(w, ITERS, *lists[state[0]])
        c_alt, e_alt = _call_loop(alt, words, seconds * 0.5)
        out[f"n{n}"] = {
            "fixed_code": {"calls_per_s": c_fix / e_fix, "us_per_call": e_fix / c_fix * 1e6, "calls": c_fix},
            "new_graph_each_call": {"calls_per_s": c_alt / e_alt, "us_per_call": e_alt / c_alt * 1e6,
                                    "calls": c_alt}}
    return out


def dropin_reference_rates(seconds):
    """The reference's own message_passing.c (oracle/_ref/message_passing.so, built unchanged from
    the reference sources, one host core) driven exactly as parallel_simulator.py:131-166 does
    (oracle.ref_message_pass_decode: the same marshalling, ct.CDLL per call), on the words and
    codes of dropin_gpu_rates."""
    from oracle import oracle
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    if not oracle.ref_available():
        return None
    out = {}
    for n in DROPIN_NS:
        ga = TannerGraph.random_regular(n, DV, DC, seed=1)
        words = dropin_words(n, 64, 11)
        c, e = _call_loop(lambda w: oracle.ref_message_pass_decode(w, ITERS, ga.check_lookup, ga.variable_lookup,
                                                                    n, ga.k, DV, DC), words, seconds)
        out[f"n{n}"] = {"calls_per_s": c / e, "us_per_call": e / c * 1e6, "calls": c, "cores": 1}
    return out


def graph_cfg0():
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    return TannerGraph.random_regular(1000, DV, DC, seed=1)


ISSUE_PROFILE = os.path.join(ROOT, "profiles", "r06_issue_model.json")
SIMDS, CUS, CLOCK_HZ = 1024, 256, 2.4e9


def onchip_rooflines(cw_iters_per_s, kernel):
    """The units the LDS-resident kernel can saturate, per codeword-iteration, from the committed
    issue model of this kernel (ISSUE_PROFILE, scripts/issue_model.py: its ISA blocks x their
    execution counts, completed by the PMC counters of one profiled launch):
      valu: VALU-busy cycles per codeword-iteration MEASURED by PMC SQ_ACTIVE_INST_VALU (x 4: one
            quad-cycle per wave64 instruction, two per transcendental) over 1024 SIMDs x 2.4 GHz
            -- the roofline's frac, a counter, not a price choice; beside it the issue model at
            the chip-wide probe's prices (plain 4.2, packed f32 5.3, transcendental 8.2 cycles;
            scripts/diag/valu_rate.hip) and the band those prices span: packed ops at 4.0 (what
            the counter charges) .. 5.3 (distinct operand pairs) .. 7.5 (one register pair read
            three times -- above 1.0 of peak with this mix, so not the headline's price);
      lds:  LDS-array cycles per codeword-iteration MEASURED by SQ_LDS_IDX_ACTIVE (every array
            cycle, bank conflicts included) over 256 CUs x 2.4 GHz; beside it the older transfer
            model (MI355X_MICROARCH.md per-instruction costs plus SQ_LDS_BANK_CONFLICT).
    achieved = cycles per codeword-iteration x the live codeword-iteration rate of this run's
    kernel (HIP events).  Returns (valu, lds), or (None, None) when the committed model is of
    another kernel than the one that ran."""
    if not os.path.exists(ISSUE_PROFILE):
        return None, None
    with open(ISSUE_PROFILE) as f:
        d = json.load(f)
    if d.get("kernel_family") != kernel.split("<")[0]:  # the model describes another kernel: no roofline from it
        return None, None
    rel = os.path.relpath(ISSUE_PROFILE, ROOT)
    peak = SIMDS * CLOCK_HZ
    pmc = d.get("pmc_per_codeword_iteration", {})
    wi = d["wave_instr_per_codeword_iteration"]
    prices = d["cycles"]["valu"]

    def priced(packed):
        return (wi["packed"] * packed + wi["plain"] * prices["plain"] + wi["trans"] * prices["trans"])

    v_cyc = d["valu_issue_cycles_per_codeword_iteration"]
    model = {"frac": v_cyc * cw_iters_per_s / peak, "issue_cycles_per_codeword_iteration": v_cyc,
             "wave_instr_per_codeword_iteration": wi, "cycles_per_wave_instr": prices,
             "price_band_frac": {f"packed_{pk:g}": priced(pk) * cw_iters_per_s / peak for pk in (4.0, 5.3, 7.5)},
             "note": "packed price 4.0 = the counter's charge; 5.3 = chip-wide probe, distinct operand pairs; "
                     "7.5 = probe with one register pair read three times (gives > 1.0 here: infeasible)"}
    alg = algorithmic_valu_cycles(prices)
    model["algorithmic"] = {"issue_cycles_per_codeword_iteration": alg["cycles"],
                            "frac": alg["cycles"] * cw_iters_per_s / peak, "definition": alg["definition"]}
    busy = pmc.get("SQ_ACTIVE_INST_VALU")
    if busy:  # the measured VALU-busy cycles (quad-cycles x 4)
        cyc = busy * 4
        valu = {"bound": "valu", "achieved": cyc * cw_iters_per_s / 1e9, "peak": peak / 1e9,
                "unit": "G SIMD-VALU-busy-cycles/s", "frac": cyc * cw_iters_per_s / peak,
                "source": "PMC SQ_ACTIVE_INST_VALU x 4 per codeword-iteration (profiled launch of this kernel) "
                          "x this run's live codeword-iteration rate",
                "valu_busy_cycles_per_codeword_iteration": cyc,
                "profiled_launch_valu_active_frac": d.get("profiled_valu_active_frac"),
                "issue_model": model, "profile": rel, "profile_git": d.get("git")}
    else:  # an older profile without the counter: the model
        valu = dict(model, bound="valu", achieved=v_cyc * cw_iters_per_s / 1e9, peak=peak / 1e9,
                    unit="G SIMD-issue-cycles/s", source="issue model (measured prices)", profile=rel,
                    profile_git=d.get("git"))
    t_cyc = d["lds_cycles_per_codeword_iteration"]
    conf = d["lds_bank_conflict_cycles_per_codeword_iteration"]
    tmodel = {"frac": (t_cyc + conf) * cw_iters_per_s / (CUS * CLOCK_HZ),
              "cycles_per_codeword_iteration": t_cyc + conf, "conflict_free_cycles": t_cyc,
              "bank_conflict_cycles": conf, "cycles_per_wave_instr": d["cycles"]["lds"],
              "lds_instr_per_codeword_iteration": d["lds_instr_per_codeword_iteration"]}
    idx = pmc.get("SQ_LDS_IDX_ACTIVE")
    if idx:
        lds = {"bound": "lds", "achieved": idx * cw_iters_per_s / 1e9, "peak": CUS * CLOCK_HZ / 1e9,
               "unit": "G LDS-array-cycles/s", "frac": idx * cw_iters_per_s / (CUS * CLOCK_HZ),
               "array_cycles_per_codeword_iteration": idx, "source": "PMC SQ_LDS_IDX_ACTIVE (measured)",
               "transfer_model": tmodel, "profile": rel, "profile_git": d.get("git")}
    else:  # an older profile without the array counter: the model
        lds = {"bound": "lds", "achieved": (t_cyc + conf) * cw_iters_per_s / 1e9, "peak": CUS * CLOCK_HZ / 1e9,
               "unit": "G LDS-cycles/s", "frac": tmodel["frac"], "source": "transfer model + SQ_LDS_BANK_CONFLICT",
               "transfer_model": tmodel, "profile": rel, "profile_git": d.get("git")}
    return valu, lds


def algorithmic_valu_cycles(prices=None):
    """The minimum VALU issue work of the headline decode per codeword-iteration in its chosen
    formulation (no unpacks, clamps, sign handling, staging or loop control), SIMD-cycles at the
    issue-model prices (packed f32 and transcendental, per wave64 instruction):
      check phase, per check pair (both degree-6 checks on float2, elementary-symmetric rule):
        prefix (E, O) 4 x 2 packed ops, suffix 3 x (2 v_pk_mul + 4 v_pk_fma) + 4 for the last step
        (its prefix set is {R_0}: no product), six output ratios 6 v_pk_mul + 12 v_rcp_f32
        = 36 packed + 12 transcendental;
      variable phase, per variable pair (degree 3: one local + two gathered ratios on float2):
        R_j = E prod_{k != j} r_k by prefix / suffix products = 5 v_pk_mul.
    For (3,6) n = 10,000: P = 2,500 check pairs, 5,000 variable pairs, 64 lanes per wave."""
    pk, tr = (prices or {}).get("packed", 4.0), (prices or {}).get("trans", 8.0)
    P, VPAIRS = (N_BITS // 2) // 2, N_BITS // 2
    check = (36 * pk + 12 * tr) * P / 64
    var = 5 * pk * VPAIRS / 64
    return {"cycles": check + var,
            "definition": f"check pair: 36 v_pk_* x{pk:g} + 12 v_rcp x{tr:g} cycles per 64 pairs; variable pair: "
                          f"5 v_pk_mul x{pk:g} per 64 pairs; P=2500, 5000 variable pairs (bench.py algorithmic_valu_cycles)"}


def load_traffic():
    for name in ("r06_pmc_traffic.json", "r05a_pmc_traffic.json", "r04b_pmc_traffic.json", "r03a_pmc_traffic.json",
                 "pmc_traffic.json"):
        p = os.path.join(ROOT, "profiles", name)
        if os.path.exists(p):
            with open(p) as f:
                d = json.load(f)
            d["source"] = "profiles/" + name
            return d
    return None


def main():
    args = parse()
    import torch
    mode, info = launch_plan(args.gpus, os.environ, torch.cuda.device_count(), args.rehearse_on_one_gpu)
    if mode == "error":
        print(f"bench.py: {info}", file=sys.stderr, flush=True)
        return 2
    if mode == "spawn":
        return spawn_ranks(info, sys.argv[1:], script=os.path.abspath(__file__))
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

    # one collective over all ranks after the timed region: the frame errors of every rank's
    # own batch (RCCL over xGMI with the nccl backend) -- proves all N ranks joined and decoded
    fe_local = hard.any(dim=1).sum().to(torch.int64).reshape(1)
    fe_all, ranks_joined = int(fe_local.item()), 1
    if world > 1:
        vec = torch.stack([fe_local[0], torch.ones((), dtype=torch.int64, device=fe_local.device)])
        if backend != "nccl":
            vec = vec.cpu()
        dist.all_reduce(vec)
        fe_all, ranks_joined = int(vec[0]), int(vec[1])
    fer = fe_all / (world * B)
    total_cw = world * B * args.steps
    value = total_cw / elapsed
    b_it = 2 * E * 4 + 2 * g.n * 4
    achieved = b_it * B * ITERS / (kernel_ms * 1e-3) / 1e9
    kernel_cw_iters = B * ITERS / (kernel_ms * 1e-3)
    traffic = load_traffic()

    extras = {}
    if not args.no_extras and rank == 0 and world == 1:  # the N = 1 line carries the extras
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def best_ms(fn, reps=3):  # one untimed launch, then the fastest of `reps` (HIP events)
            fn()
            torch.cuda.synchronize()
            out = []
            for _ in range(reps):
                a.record(stream)
                fn()
                b.record(stream)
                torch.cuda.synchronize()
                out.append(a.elapsed_time(b))
            return min(out)

        # same frames with syndrome early termination (max 50 iterations), posteriors of the
        # stopping iteration
        et_ms = best_ms(lambda: decoder.bp_decode_dev(g, llr, ITERS, "spa", early_stop=True, post=post, hard=hard,
                                                      its=its, stream=stream))
        extras["early_stop_spa"] = {"codewords_per_s": B / (et_ms * 1e-3),
                                    "mean_iterations": float(its.float().mean().item()),
                                    "kernel": g.kernel_name(early_stop=True)}
        # the same with hard decisions only (no posteriors)
        hd_ms = best_ms(lambda: decoder.bp_decode_dev(g, llr, ITERS, "spa", early_stop=True, post=None, hard=hard,
                                                      its=its, stream=stream, want_post=False))
        extras["early_stop_spa_hard_only"] = {"codewords_per_s": B / (hd_ms * 1e-3),
                                              "codeword_iterations_per_s": float(its.sum().item()) / (hd_ms * 1e-3),
                                              "mean_iterations": float(its.float().mean().item()),
                                              "kernel": g.kernel_name(early_stop=True, hard_only=True)}
        ms_ms = best_ms(lambda: decoder.bp_decode_dev(g, llr, ITERS, "minsum", alpha=0.75, post=post, hard=hard,
                                                      its=its, stream=stream))
        extras["minsum_50it_codewords_per_s"] = B / (ms_ms * 1e-3)
        es_ms = best_ms(lambda: decoder.bp_decode_dev(g, llr, ITERS, "minsum", alpha=0.75, early_stop=True, post=post,
                                                      hard=hard, its=its, stream=stream))
        extras["early_stop_minsum"] = {"codewords_per_s": B / (es_ms * 1e-3),
                                       "mean_iterations": float(its.float().mean().item()),
                                       "kernel": g.kernel_name(early_stop=True)}
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
        gi = ensembles.sample_irregular(ensembles.RSU_DL4, 20000, seed=1, deg2="path")  # ring code
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
                           "kernel": gi.kernel_name(early_stop=et, hard_only=True)}
        del llr_i
        # configs[3] Monte-Carlo as scripts/fer_sweep.py runs it (fused channel, sign-bit early stop)
        Bm = 65536
        mc = MonteCarlo(gi, "awgn", 0.84, 100, algo="spa", early_stop=True, seed=9, batch=Bm)
        mc.run_batch(0, Bm)
        torch.cuda.synchronize()
        a.record(stream)
        mc.run_batch(Bm, Bm)
        b.record(stream)
        torch.cuda.synchronize()
        cnt = mc.counters.cpu().numpy()
        extras["irregular_cfg4_mc_sigma0.84_early_stop"] = {
            "trials_per_s": Bm / (a.elapsed_time(b) * 1e-3), "batch": Bm, "mean_iterations": float(cnt[3] / cnt[0]),
            "fer": float(cnt[1] / cnt[0])}
        # configs[2] shape: BSC normalized min-sum Monte-Carlo, (3,6) n = 10,000 (fused channel,
        # LDS-syndrome early stop, 50 iterations), p = 0.07.  The code is the headline law's seed-1
        # draw with distinct columns (scripts/fer_sweep.py cfg3): the plain draw holds one pair of
        # identical columns, a weight-2 codeword that one channel flip turns into a tie (FER 2p(1-p))
        gd = TannerGraph.random_regular(N_BITS, DV, DC, seed=1, distinct_columns=True)
        Bm = 65536
        mc = MonteCarlo(gd, "bsc", 0.07, ITERS, algo="minsum", alpha=0.75, early_stop=True, seed=11, batch=Bm)
        mc.run_batch(0, Bm)
        torch.cuda.synchronize()
        nb = 3  # three batches between the events: the mean rate, not one batch's
        a.record(stream)
        for r in range(nb):
            mc.run_batch((1 + r) * Bm, Bm)
        b.record(stream)
        torch.cuda.synchronize()
        cnt = mc.counters.cpu().numpy()
        extras["bsc_minsum_mc_cfg2_p0.07_early_stop"] = {
            "trials_per_s": nb * Bm / (a.elapsed_time(b) * 1e-3), "batch": Bm, "batches_timed": nb,
            "mean_iterations": float(cnt[3] / cnt[0]), "fer": float(cnt[1] / cnt[0])}
        # configs[4] shape: expurgated (3,6) ensemble, a fresh device-sampled n = 64,800 graph per
        # trial (sample_seq_kernel) + 200-iteration BEC decode + counters, eps = 0.42, X = 3
        # (parallel_simulator_expurgated.py:169-285)
        Be = 16384
        mc = MonteCarlo.ensemble(64800, DV, DC, "bec", 0.42, 200, seed=7, batch=Be, expurgation=3)
        mc.run_batch(0, 256)
        torch.cuda.synchronize()
        a.record(stream)
        mc.run_batch(256, Be)
        b.record(stream)
        torch.cuda.synchronize()
        cnt = mc.counters.cpu().numpy()
        extras["ensemble_mc_cfg5_n64800_eps0.42_200it_X3"] = {
            "trials_per_s": Be / (a.elapsed_time(b) * 1e-3), "batch": Be, "mean_iterations": float(cnt[3] / cnt[0]),
            "frame_errors": int(cnt[1]), "trials": int(cnt[0])}
        del mc
        # the same at the FER campaigns' batch (scripts/fer_campaign.sh: 65,536 graphs per launch,
        # ~100 GB of edge lists): the sampler's tail (the last graphs' helpers) amortised 4x
        Bc = 65536
        mc = MonteCarlo.ensemble(64800, DV, DC, "bec", 0.42, 200, seed=7, batch=Bc, expurgation=3)
        mc.run_batch(0, 256)
        torch.cuda.synchronize()
        a.record(stream)
        mc.run_batch(256, Bc)
        b.record(stream)
        torch.cuda.synchronize()
        cnt = mc.counters.cpu().numpy()
        extras["ensemble_mc_cfg5_n64800_eps0.42_200it_X3_campaign_batch"] = {
            "trials_per_s": Bc / (a.elapsed_time(b) * 1e-3), "batch": Bc, "mean_iterations": float(cnt[3] / cnt[0]),
            "frame_errors": int(cnt[1]), "trials": int(cnt[0])}
        del mc
        torch.cuda.empty_cache()
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

    dropin = None
    if rank == 0 and world == 1 and not args.no_extras:
        dropin = {"what": "one message_passing call per word through ctypes, parallel_simulator.py:131-166 "
                          "marshalling, (3,6) BEC eps=0.4, 50 iterations, synthetic words",
                  "gpu": dropin_gpu_rates(2.0)}
        extras["dropin_message_passing"] = dropin
    cpu = None
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(g, llr[:1024].cpu().numpy(), args.cpu_seconds)
        if dropin is not None:
            dropin["reference_c_one_core"] = dropin_reference_rates(2.0)
            for key, ref in (dropin["reference_c_one_core"] or {}).items():
                gpu = dropin["gpu"][key]["fixed_code"]["calls_per_s"]
                dropin["gpu"][key]["fixed_code"]["vs_reference_c"] = gpu / ref["calls_per_s"]

    hbm_model = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                 "frac": achieved / HBM_PEAK_GBPS, "algorithmic_bytes_per_codeword_iteration": b_it,
                 "note": "SURVEY.md 8(d) streaming model (every edge message read + written through HBM "
                         "each iteration); this kernel keeps the messages in LDS, so the model exceeds the "
                         "HBM peak and is informational only"}
    if traffic:
        hbm_meas = traffic["bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9 * (B / traffic["batch"])
        hbm_model["measured_traffic_bytes_per_launch"] = traffic["bytes_per_launch"] * B / traffic["batch"]
        hbm_model["measured_GBps"] = hbm_meas
        hbm_model["measured_frac"] = hbm_meas / HBM_PEAK_GBPS
        hbm_model["measured_bytes_per_codeword"] = traffic["bytes_per_codeword"]
        hbm_model["traffic_profile"] = traffic.get("source", "profiles/pmc_traffic.json")
    valu_roof, lds_roof = onchip_rooflines(kernel_cw_iters, g.kernel_name(False))
    if lds_roof is None:  # no issue-model profile: report the measured HBM use as the roofline
        roof = {"bound": "hbm", "achieved": hbm_model.get("measured_GBps"), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": hbm_model.get("measured_frac")}
    else:  # the binding unit is the one with the larger fraction
        roof = dict(max((lds_roof, valu_roof), key=lambda r: r["frac"]))
        roof["other_units"] = {r["bound"]: {"frac": r["frac"], "achieved": r["achieved"], "peak": r["peak"],
                                            "unit": r["unit"]} for r in (lds_roof, valu_roof) if r["bound"] != roof["bound"]}
    roof["traffic"] = hbm_model.get("measured_traffic_bytes_per_launch")
    roof["hbm_model"] = hbm_model

    if rank == 0:
        line = {
            "metric": "decoded codewords/sec + info-bit Gb/s, (3,6) n=10k 50-iter BP, 1/2/4/8 MI355X",
            "value": value,
            "unit": "codewords/s",
            "n_gpus": world,
            "rccl_ranks": ranks_joined if (world > 1 and backend == "nccl") else None,
            "dist": {"ranks_joined": ranks_joined, "backend": backend if world > 1 else None,
                     "devices_visible": torch.cuda.device_count(),
                     "rehearsal_shared_gpu": bool(args.rehearse_on_one_gpu and world > torch.cuda.device_count()),
                     "frame_errors_all_ranks": fe_all},
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
            "roofline": roof,
            "valu_roofline": valu_roof,
            "lds_roofline": lds_roof,
            "cpu_baseline": cpu,
            "extras": extras,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
