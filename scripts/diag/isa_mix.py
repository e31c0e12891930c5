"""Instruction mix of the barrier-delimited regions of one kernel in a .s file.
usage: python scripts/diag/isa_mix.py file.s <kernel-name-substring>"""
import collections, sys
src, key = sys.argv[1], sys.argv[2]
s = open(src).read()
lines = s.split('\n')
start = next(k for k, l in enumerate(lines) if l.startswith(key) and ':' in l)
end = next(k for k in range(start, len(lines)) if 's_endpgm' in lines[k])
body = lines[start:end]
cuts = [k for k, l in enumerate(body) if 's_barrier' in l] + [len(body)]
prev = 0
for c in cuts:
    mix = collections.Counter(l.strip().split()[0] for l in body[prev:c]
                              if l.strip() and not l.strip().startswith((';', '.')))
    if sum(mix.values()) > 60:
        print(f"[{prev}:{c}] {sum(mix.values())} :", ", ".join(f"{k} {v}" for k, v in mix.most_common(16)))
    prev = c
