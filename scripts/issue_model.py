"""Issue model of the headline decode kernel per codeword-iteration -> profiles/<tag>_issue_model.json.

usage: python scripts/issue_model.py <kernels.s> <pmc_summary.json> <out.json> [git-sha]

<kernels.s>: `hipcc --cuda-device-only -S` of csrc/ldpc_kernels.hip with the Makefile's flags;
<pmc_summary.json>: scripts/pmc_summary.py output for one bench launch (B = 65,536, 50 iterations).

The two on-chip units the LDS-resident kernel can saturate, per codeword-iteration of
bp_lds_kernel<3,6,1024,10,SPA> (fixed count):

* VALU issue (per SIMD): wave-instructions by class x issue cycles of one wave64 instruction
  on its SIMD (MI355X_MICROARCH.md: v_fma_f32 2 cycles on the SIMD-32, packed f32 twice that,
  transcendentals 8).  packed = the ISA's v_pk_* of the check and variable blocks x their
  wave-executions; trans = PMC SQ_INSTS_VALU_TRANS_F32; plain = PMC SQ_INSTS_VALU - packed -
  trans.  Peak: 1024 SIMDs.
* LDS (per CU): the blocks' ds_* wave-instructions x their conflict-free LDS cycles
  (MI355X_MICROARCH.md LDS table: ds_read_b128 4, ds_write_b128 13, ds_read_b32 2,
  ds_write_b32 4) -- the algorithmic LDS work.  PMC SQ_LDS_BANK_CONFLICT is reported beside it
  as waste (like HBM traffic above the algorithmic bytes); it is not added, because the
  counter also tallies store conflicts that hide under a ds_write_b32's 4-cycle address +
  data transfer (2 LDS-array cycles).  Peak: 256 CUs.

Wave-executions: the check phase's P = m/2 = 2500 pairs over T = 1024 threads (thread t owns
pairs t, t+T, t+2T < P); the loop runs two pairs per iteration after a one-pair prologue for
odd trip counts, so the prologue block runs in the waves holding a lane with 3 pairs (8) and
the two-pair block once in every wave (16); the variable block runs once per wave (16).
"""
import collections
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from valu_mix import KERNEL, blocks, mix  # noqa: E402

N, DV, DC, T, B, ITERS = 10000, 3, 6, 1024, 65536, 50
LDS_CYC = {"ds_read_b128": 4, "ds_write_b128": 13, "ds_read_b32": 2, "ds_write_b32": 4,
           "ds_read_b64": 2, "ds_write_b64": 6}
VALU_CYC = {"packed": 4.0, "plain": 2.0, "trans": 8.0}


def wave_execs():
    P = (N * DV // DC) // 2
    trips = [len(range(t, P, T)) for t in range(T)]
    pro = sum(1 for w in range(T // 64) if any(trips[t] % 2 for t in range(64 * w, 64 * w + 64)))
    two = sum(max(trips[t] // 2 for t in range(64 * w, 64 * w + 64)) for w in range(T // 64))
    return pro, two, T // 64


def main():
    src, pmc_path, out_path = sys.argv[1:4]
    sha = sys.argv[4] if len(sys.argv) > 4 else None
    lines = open(src).read().split("\n")
    a = next(k for k, l in enumerate(lines) if l.startswith(KERNEL + ":"))
    b = next(k for k in range(a, len(lines)) if "s_endpgm" in lines[k])
    bb = blocks(lines[a:b])
    one = [ins for _, ins in bb if ins.count("ds_read_b128") == 3]
    two = [ins for _, ins in bb if ins.count("ds_read_b128") == 6]
    var = max((ins for _, ins in bb), key=lambda ins: ins.count("ds_read_b32"))
    assert len(one) == 1 and len(two) == 1 and var.count("ds_read_b32") == 3 * 10
    n_one, n_two, n_var = wave_execs()
    assert n_one + 2 * n_two == 40
    parts = [(one[0], n_one), (two[0], n_two), (var, n_var)]
    valu = collections.Counter()
    lds = collections.Counter()
    for ins, k in parts:
        for c, v in mix(ins).items():
            valu[c] += v * k
        for op in ins:
            if op in LDS_CYC:
                lds[op] += k
    d = json.load(open(pmc_path))["counters"]
    units = B * ITERS
    total = d["SQ_INSTS_VALU"] / units
    trans = d["SQ_INSTS_VALU_TRANS_F32"] / units
    per = {"packed": valu["packed"], "trans": trans, "plain": total - valu["packed"] - trans}
    conflict = d["SQ_LDS_BANK_CONFLICT"] / units
    lds_cycles = sum(LDS_CYC[op] * n for op, n in lds.items())
    out = {
        "kernel": "bp_lds_kernel<3,6,1024,10,SPA,fixed-count>",
        "git": sha,
        "wave_instr_per_codeword_iteration": per,
        "valu_issue_cycles_per_codeword_iteration": sum(per[c] * VALU_CYC[c] for c in VALU_CYC),
        "lds_instr_per_codeword_iteration": dict(lds),
        "lds_bank_conflict_cycles_per_codeword_iteration": conflict,
        "lds_cycles_per_codeword_iteration": lds_cycles,
        "cycles": {"valu": VALU_CYC, "lds": LDS_CYC},
        "check": {"isa_valu_per_codeword_iteration": valu["packed"] + valu["plain"] + valu["trans"],
                  "pmc_valu_per_codeword_iteration": total,
                  "isa_lds_per_codeword_iteration": sum(lds.values()),
                  "pmc_lds_per_codeword_iteration": d.get("SQ_INSTS_LDS", 0) / units,
                  "isa_pk_mul_fma": valu["pk_mul_fma"],
                  "pmc_mul_fma_f32": (d.get("SQ_INSTS_VALU_MUL_F32", 0) + d.get("SQ_INSTS_VALU_FMA_F32", 0)) / units},
        "wave_executions": {"check_one_pair": n_one, "check_two_pairs": n_two, "variable": n_var},
        "pmc_per_codeword_iteration": {k: v / units for k, v in d.items() if k.startswith("SQ_")},
    }
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
