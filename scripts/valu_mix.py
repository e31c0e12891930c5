"""VALU instruction mix of the headline decode kernel per codeword-iteration -> profiles/<tag>_valu_mix.json.

usage: python scripts/valu_mix.py <kernels.s> <pmc_summary.json> <out.json> [git-sha]

<kernels.s>: `hipcc --cuda-device-only -S` of csrc/ldpc_kernels.hip (same flags as the Makefile);
<pmc_summary.json>: scripts/pmc_summary.py output of one bench launch (B = 65,536, 50 iterations)
with SQ_INSTS_VALU and SQ_INSTS_VALU_TRANS_F32 (and the ADD/MUL/FMA_F32 class counters, which
count a packed v_pk_* instruction once, in its class).

Per codeword-iteration of bp_lds_kernel<3,6,1024,10,SPA>:
  * the check phase runs its loop body once per (wave, pair round): pairs P = m/2 = 2500 over
    T = 1024 threads -> rounds of 1024, 1024, 452 pairs -> 16 + 16 + 8 = 40 wave-executions;
  * the variable phase runs its straight-line block once per wave: T/64 = 16.
packed = the v_pk_* instructions of those two blocks x their execution counts (ISA);
trans = SQ_INSTS_VALU_TRANS_F32 (PMC); plain = SQ_INSTS_VALU - packed - trans (PMC).
The ISA's v_pk_mul_f32 + v_pk_fma_f32 count is checked against PMC MUL_F32 + FMA_F32 (those
classes hold no unpacked f32 multiplies outside the blocks but a handful per codeword).
"""
import collections
import json
import sys

KERNEL = "_ZN4ldpc12_GLOBAL__N_113bp_lds_kernelILi3ELi6ELi1024ELi10ELi0ELb0ELb0EEEvNS0_6BpArgsE"
N, DV, DC, T, B, ITERS = 10000, 3, 6, 1024, 65536, 50
TRANS = ("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")


def blocks(lines):
    """Split into basic blocks at labels and `; %bb.` markers: [(label, [instr...])]."""
    out, cur, name = [], [], "entry"
    for l in lines:
        s = l.strip()
        if s.startswith(".LBB") and s.split()[0].endswith(":") or s.startswith("; %bb."):
            out.append((name, cur))
            name, cur = s.split()[0].rstrip(":") if s.startswith(".LBB") else s.split()[1], []
            continue
        if not s or s.startswith((";", ".")):
            continue
        cur.append(s.split()[0])
    out.append((name, cur))
    return out


def mix(instrs):
    c = collections.Counter()
    for op in instrs:
        if not op.startswith("v_"):
            continue
        c["trans" if op.startswith(TRANS) else "packed" if op.startswith("v_pk_") else "plain"] += 1
        if op.startswith(("v_pk_mul_f32", "v_pk_fma_f32")):
            c["pk_mul_fma"] += 1
    return c


def main():
    src, pmc_path, out_path = sys.argv[1:4]
    sha = sys.argv[4] if len(sys.argv) > 4 else None
    lines = open(src).read().split("\n")
    a = next(k for k, l in enumerate(lines) if l.startswith(KERNEL + ":"))
    b = next(k for k in range(a, len(lines)) if "s_endpgm" in lines[k])
    bb = blocks(lines[a:b])
    # check-phase loop body: the block with the ds_read_b128s that branches back to itself
    chk = [(n, ins) for n, ins in bb if ins.count("ds_read_b128") >= 3 and any(i == "s_cbranch_execnz" for i in ins)]
    # variable-phase block: the straight-line block with the 30 gathers (ds_read_b32) per wave
    var = max(bb, key=lambda x: x[1].count("ds_read_b32"))
    assert len(chk) == 1, chk
    mc, mv = mix(chk[0][1]), mix(var[1])
    pairs = (N * DV // DC) // 2
    wave_exec_chk = 0
    for r in range(0, pairs, T):
        act = min(T, pairs - r)
        wave_exec_chk += (act + 63) // 64
    wave_exec_var = T // 64
    d = json.load(open(pmc_path))["counters"]
    units = B * ITERS
    total = d["SQ_INSTS_VALU"] / units
    trans = d["SQ_INSTS_VALU_TRANS_F32"] / units
    packed = mc["packed"] * wave_exec_chk + mv["packed"] * wave_exec_var
    static_total = sum(mc[k] for k in ("packed", "plain", "trans")) * wave_exec_chk + \
        sum(mv[k] for k in ("packed", "plain", "trans")) * wave_exec_var
    out = {
        "kernel": "bp_lds_kernel<3,6,1024,10,SPA,fixed-count>",
        "git": sha,
        "wave_instr_per_codeword_iteration": {"packed": packed, "trans": trans, "plain": total - packed - trans},
        "pmc_per_codeword_iteration": {k: v / units for k, v in d.items() if k.startswith("SQ_INSTS_VALU")},
        "isa": {"check_body": dict(mc), "check_wave_executions": wave_exec_chk,
                "variable_block": dict(mv), "variable_wave_executions": wave_exec_var,
                "static_valu_per_codeword_iteration": static_total,
                "pk_mul_fma_per_codeword_iteration": mc["pk_mul_fma"] * wave_exec_chk + mv["pk_mul_fma"] * wave_exec_var},
        "method": "packed from the ISA blocks x execution counts; trans and total from PMC (one launch, B=65536, 50 it)",
    }
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
