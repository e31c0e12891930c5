"""Issue model of the headline decode kernel per codeword-iteration -> profiles/<tag>_issue_model.json.

usage: python scripts/issue_model.py <kernels.s> <pmc_summary.json> <out.json> [git-sha] [--kernel loc|lds36]

<kernels.s>: `hipcc --cuda-device-only -S` of csrc/ldpc_kernels.hip with the Makefile's flags;
<pmc_summary.json>: scripts/pmc_summary.py output for one bench launch (B = 65,536, 50 iterations).

The two on-chip units an LDS-resident decode kernel can saturate, per codeword-iteration:

* VALU issue (per SIMD): wave-instructions by class x issue cycles of one wave64 instruction
  on its SIMD (measured, VALU_CYC below: plain 4.2, packed f32 5.3, transcendentals 8.2).  packed = the ISA's v_pk_* of every block x its wave-executions;
  trans = PMC SQ_INSTS_VALU_TRANS_F32; plain = PMC SQ_INSTS_VALU - packed - trans.
  Peak: 1024 SIMDs.
* LDS (per CU): the blocks' ds_* wave-instructions x their conflict-free LDS cycles
  (MI355X_MICROARCH.md LDS table: ds_read_b128 4, ds_write_b128 13, ds_read_b32 2,
  ds_write_b32 4) -- the algorithmic LDS work.  PMC SQ_LDS_BANK_CONFLICT is reported beside it
  as waste (like HBM traffic above the algorithmic bytes); it is not added, because the
  counter also tallies store conflicts that hide under a ds_write_b32's 4-cycle address +
  data transfer (2 LDS-array cycles).  Peak: 256 CUs.

Wave-executions per codeword-iteration:

--kernel loc (default; bp_loc_kernel<6,6,2,2,5,512,SPA>, the bench code's local-edge
  layout, two 512-thread workgroups per CU): the check phase is KP = 5 straight blocks (one
  per check pair slot k; each two ds_read_b128 + two ds_write_b128 -- a pair's 2 x 4
  non-local inputs and outputs), block k runs in the waves holding a lane t with
  t + k*T < P (P = m/2 = 2500, T = 512: 8 waves each); the variable phase is one block
  (8*KP ds_read_b32 + 8*KP ds_write_b32: the 4*KP local variables' 2 non-local edges each)
  run by all T/64 = 8 waves in ITERS - 1 of the ITERS iterations (the last iteration's
  variable phase is the posterior epilogue); every other block (staging, init, epilogue)
  counts once per wave per codeword, i.e. 8/ITERS.  --kernel loc1024: the round-2
  one-workgroup shape <6,6,2,2,3,1024> (16, 16, 8 waves; 16).
--kernel lds36 (round-2 bp_lds_kernel<3,6,1024,10,SPA>): the check phase's two-pair loop body
  (16 wave-executions) after a one-pair prologue (8), the variable block once per wave (16).
"""
import collections
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from valu_mix import blocks, mix  # noqa: E402

N, DV, DC, B, ITERS = 10000, 3, 6, 65536, 50
LDS_CYC = {"ds_read_b128": 4, "ds_write_b128": 13, "ds_read_b32": 2, "ds_write_b32": 4,
           "ds_read_b64": 2, "ds_write_b64": 6, "ds_write2st64_b32": 8, "ds_write2_b32": 8,
           "ds_read2_b32": 4, "ds_read2st64_b32": 4, "ds_read2_b64": 4, "ds_write2_b64": 13,
           "ds_read_u8": 2, "ds_write_b8": 4, "ds_read_u16": 2, "ds_write_b16": 4, "ds_bpermute_b32": 2,
           "ds_swizzle_b32": 2, "ds_add_u32": 4, "ds_or_b32": 4, "ds_read_b96": 4, "ds_write_b96": 13}
# Issue cycles of one wave64 VALU instruction on its SIMD, measured on the whole chip by
# scripts/diag/valu_rate.hip (HIP events around 5 launches of 256 x W workgroups, W = 8 waves per
# SIMD, throughput at the in-kernel clock; profiles/r05_valu_rate*.jsonl): v_add / v_fma / v_xor /
# v_mul_lo 4.1-4.3 (4.2), v_pk_mul / v_pk_fma / v_pk_add with distinct operand pairs 5.2-5.3 (5.3),
# v_rcp_f32 8.2 -- not the 2 / 4 / 8 of rounds 2-4 (MI355X_MICROARCH.md's SIMD-32 figure for a
# wave64 v_fma_f32).  PMC SQ_ACTIVE_INST_VALU counts one quad-cycle per plain or packed
# instruction and two per transcendental (4 / 4 / 8: the headline launch's count to 0.1 %), so
# it undercounts the packed ops' measured cost; both are reported.
VALU_CYC = {"packed": 5.3, "plain": 4.2, "trans": 8.2}
KERNELS = {
    "loc": ("_ZN4ldpc12_GLOBAL__N_113bp_loc_kernelILi6ELi6ELi2ELi2ELi5ELi512ELi0ELb0ELb0ELb0ELb0ELb0EEEvNS0_6BpArgsE",
            "bp_loc_kernel<6,6,2,2,KP=5,T=512,SPA,fixed-count>", 512, 5),
    "loc1024": ("_ZN4ldpc12_GLOBAL__N_113bp_loc_kernelILi6ELi6ELi2ELi2ELi3ELi1024ELi0ELb0ELb0ELb0ELb0ELb0EEEvNS0_6BpArgsE",
                "bp_loc_kernel<6,6,2,2,KP=3,T=1024,SPA,fixed-count>", 1024, 3),
    "loc_et": ("_ZN4ldpc12_GLOBAL__N_113bp_loc_kernelILi6ELi6ELi2ELi2ELi5ELi512ELi0ELb0ELb0ELb1ELb0ELb0EEEvNS0_6BpArgsE",
               "bp_loc_kernel<6,6,2,2,KP=5,T=512,SPA,early-stop>", 512, 5),
    "loc_ep": ("_ZN4ldpc12_GLOBAL__N_113bp_loc_kernelILi6ELi6ELi2ELi2ELi5ELi512ELi0ELb0ELb0ELb1ELb0ELb1EEEvNS0_6BpArgsE",
               "bp_loc_kernel<6,6,2,2,KP=5,T=512,SPA,early-stop+posteriors>", 512, 5),
    "loc_ms": ("_ZN4ldpc12_GLOBAL__N_113bp_loc_kernelILi6ELi6ELi2ELi2ELi5ELi512ELi1ELb0ELb0ELb0ELb0ELb0EEEvNS0_6BpArgsE",
               "bp_loc_kernel<6,6,2,2,KP=5,T=512,min-sum,fixed-count>", 512, 5),
    "lds36": ("_ZN4ldpc12_GLOBAL__N_113bp_lds_kernelILi3ELi6ELi1024ELi10ELi0ELb0ELb0EEEvNS0_6BpArgsE",
              "bp_lds_kernel<3,6,1024,10,SPA,fixed-count>", 1024, None),
}


def loc_parts(bb, T, KP, stats=None):
    """stats (scripts/diag/decode_launch.py output): early-stop launches -- per codeword-iteration
    the check blocks run check_phases / sum_its times, the variable block variable_phases /
    sum_its, the per-codeword blocks batch / sum_its (fixed count: 1, (ITERS-1)/ITERS, 1/ITERS)."""
    P = (N * DV // DC) // 2
    waves = T // 64
    if stats:
        r_chk = stats["check_phases"] / stats["sum_its"]
        r_var = stats["variable_phases"] / stats["sum_its"]
        r_cw = stats["batch"] / stats["sum_its"]
    else:
        r_chk, r_var, r_cw = 1.0, (ITERS - 1) / ITERS, 1.0 / ITERS
    # check slot k: the block storing the pair's two ds_write_b128 (the early-stop builds load
    # one of the two b128 inputs as a b128 and the other through two narrower reads)
    # (round 5: the one-class check phase has no per-pair branch -- one block holding all KP
    # pairs' 2 * KP ds_write_b128, run by every wave)
    chk = [i for i, (_, ins) in enumerate(bb) if ins.count("ds_write_b128") == 2]
    one = [i for i, (_, ins) in enumerate(bb) if ins.count("ds_write_b128") == 2 * KP]
    if len(one) == 1 and len(chk) != KP:
        chk = one
    assert len(chk) in (KP, 1), len(chk)
    # variable phase: the blocks after the check slots holding its 8*KP ds_read_b32 / ds_write_b32
    # (one block; split in ten by the slab-store branches in the early-stop-with-posteriors build)
    # (searched from the last check slot on, wrapping: the compiler may rotate the loop so the
    # variable block precedes the check blocks in the code)
    var, nr = [], 0
    for i in list(range(chk[-1] + 1, len(bb))) + list(range(0, chk[0])):
        ins = bb[i][1]
        if ins.count("ds_read_b32") >= 4 and ins.count("ds_write_b32") >= 4:
            var.append(i)
            nr += ins.count("ds_read_b32")
            if nr >= 8 * KP:
                break
    assert nr == 8 * KP and sum(bb[i][1].count("ds_write_b32") for i in var) == 8 * KP, (var, nr)
    execs = {}
    for k, i in enumerate(chk):
        lanes = min(max(P - k * T, 0), T) if len(chk) == KP else T
        execs[i] = (lanes + 63) // 64 * r_chk
    for i in var:
        execs[i] = waves * r_var
    parts = []
    for i, (_, ins) in enumerate(bb):
        parts.append((ins, execs.get(i, waves * r_cw)))
    return parts, {"check_slot_waves": [execs[i] for i in chk], "variable": execs[var[0]], "variable_blocks": len(var),
                   "other_blocks": waves * r_cw}


def lds36_parts(bb, T):
    one = [ins for _, ins in bb if ins.count("ds_read_b128") == 3]
    two = [ins for _, ins in bb if ins.count("ds_read_b128") == 6]
    var = max((ins for _, ins in bb), key=lambda ins: ins.count("ds_read_b32"))
    assert len(one) == 1 and len(two) == 1 and var.count("ds_read_b32") == 3 * 10
    P = (N * DV // DC) // 2
    trips = [len(range(t, P, T)) for t in range(T)]
    n_one = sum(1 for w in range(T // 64) if any(trips[t] % 2 for t in range(64 * w, 64 * w + 64)))
    n_two = sum(max(trips[t] // 2 for t in range(64 * w, 64 * w + 64)) for w in range(T // 64))
    assert n_one + 2 * n_two == 40
    return [(one[0], n_one), (two[0], n_two), (var, T // 64)], \
        {"check_one_pair": n_one, "check_two_pairs": n_two, "variable": T // 64}


def main():
    argv = [a for a in sys.argv[1:] if not a.startswith("--")]
    kind = "loc"
    if "--kernel" in sys.argv:
        kind = sys.argv[sys.argv.index("--kernel") + 1]
        argv.remove(kind)
    stats = None
    if "--stats" in sys.argv:  # an early-stop launch: its iteration statistics
        sp = sys.argv[sys.argv.index("--stats") + 1]
        argv.remove(sp)
        stats = json.load(open(sp))
    src, pmc_path, out_path = argv[:3]
    sha = argv[3] if len(argv) > 3 else None
    sym, label, T, KP = KERNELS[kind]
    lines = open(src).read().split("\n")
    a = next(k for k, l in enumerate(lines) if l.startswith(sym + ":"))
    b = next(k for k in range(a, len(lines)) if "s_endpgm" in lines[k])
    bb = blocks(lines[a:b])
    parts, wx = loc_parts(bb, T, KP, stats) if kind.startswith("loc") else lds36_parts(bb, T)
    valu = collections.Counter()
    lds = collections.Counter()
    for ins, k in parts:
        for c, v in mix(ins).items():
            valu[c] += v * k
        for op in ins:
            if op.startswith("ds_"):
                assert op in LDS_CYC, op
                lds[op] += k
    d = json.load(open(pmc_path))["counters"]
    units = stats["sum_its"] if stats else B * ITERS  # codeword-iterations of the profiled launch
    total = d["SQ_INSTS_VALU"] / units
    trans = d["SQ_INSTS_VALU_TRANS_F32"] / units
    per = {"packed": valu["packed"], "trans": trans, "plain": total - valu["packed"] - trans}
    conflict = d["SQ_LDS_BANK_CONFLICT"] / units
    lds_cycles = sum(LDS_CYC[op] * n for op, n in lds.items())
    out = {
        "kernel": label,
        "kernel_family": label.split("<")[0],
        "git": sha,
        "codeword_iterations_per_launch": units,
        "launch_stats": stats,
        "wave_instr_per_codeword_iteration": per,
        "valu_issue_cycles_per_codeword_iteration": sum(per[c] * VALU_CYC[c] for c in VALU_CYC),
        "lds_instr_per_codeword_iteration": dict(lds),
        "lds_bank_conflict_cycles_per_codeword_iteration": conflict,
        "lds_cycles_per_codeword_iteration": lds_cycles,
        "cycles": {"valu": VALU_CYC, "lds": LDS_CYC},
        "check": {"isa_valu_per_codeword_iteration": valu["packed"] + valu["plain"] + valu["trans"],
                  "isa_trans_per_codeword_iteration": valu["trans"],
                  "pmc_valu_per_codeword_iteration": total,
                  "isa_lds_per_codeword_iteration": sum(lds.values()),
                  "pmc_lds_per_codeword_iteration": d.get("SQ_INSTS_LDS", 0) / units,
                  "isa_pk_mul_fma": valu["pk_mul_fma"],
                  "pmc_mul_fma_f32": (d.get("SQ_INSTS_VALU_MUL_F32", 0) + d.get("SQ_INSTS_VALU_FMA_F32", 0)) / units},
        "wave_executions": wx,
        "pmc_per_codeword_iteration": {k: v / units for k, v in d.items() if k.startswith("SQ_")},
    }
    if "GRBM_GUI_ACTIVE" in d and "SQ_ACTIVE_INST_VALU" in d:  # the profiled launch's own VALU-busy fraction
        out["profiled_valu_active_frac"] = d["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * d["GRBM_GUI_ACTIVE"] / 8)
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
