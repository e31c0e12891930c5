"""Per-instantiation ISA summary of a kernel family in a hipcc -S file: instruction count,
VGPRs, spills, scratch ops, and the counts of selected mnemonics.
usage: python scripts/diag/isa_kern.py file.s <mangled-substring> [mnemonic ...]"""
import collections, re, sys
src, key = sys.argv[1], sys.argv[2]
extra = sys.argv[3:]
lines = open(src).read().split('\n')
i = 0
while i < len(lines):
    l = lines[i]
    if key in l and l.endswith(':') is False and re.match(r'^_Z\S+:', l) and key in l.split(':')[0]:
        name = l.split(':')[0]
        j = i
        while 's_endpgm' not in lines[j]:
            j += 1
        body = [x.strip() for x in lines[i:j] if x.strip() and not x.strip().startswith((';', '.', '_'))]
        mix = collections.Counter(re.sub(r'_e(32|64)$', '', x.split()[0]) for x in body)
        meta = {}
        for k in range(j, min(j + 400, len(lines))):
            m = re.match(r'\s*\.(vgpr_count|vgpr_spill_count|sgpr_count|private_segment_fixed_size|agpr_count):\s*(\d+)', lines[k])
            if m:
                meta[m.group(1)] = int(m.group(2))
            m = re.search(r'; (NumVgprs|ScratchSize|Occupancy|NumAgprs): (\d+)', lines[k])
            if m:
                meta[m.group(1)] = int(m.group(2))
        args = re.search(r'bp_loc_kernelI(.*)EEvNS', name)
        tag = args.group(1) if args else name[:80]
        tag = tag.replace('Li', '').replace('ELb', ',').replace('E', ',')
        print(f"{tag:40s} instr {len(body):5d} vgpr {meta.get('NumVgprs','?'):>3} scratch {meta.get('ScratchSize','?'):>4} "
              f"scr_ld {mix['scratch_load_dword']:3d} scr_st {mix['scratch_store_dword']:3d} "
              + " ".join(f"{e} {mix[e]}" for e in extra))
        i = j
    i += 1
