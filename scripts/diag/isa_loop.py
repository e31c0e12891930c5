"""Instruction mix of the decode-iteration loop (the loop holding the most packed-FP / min-sum
work) of one kernel instantiation in a hipcc -S file.
usage: python scripts/diag/isa_loop.py file.s <mangled-substring> [label]"""
import collections, re, sys
lines = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
i = next(k for k, l in enumerate(lines) if re.match(r'^_Z\S+:', l) and key in l)
j = i
while 's_endpgm' not in lines[j]:
    j += 1
b = lines[i:j]
loops = []
for h, l in enumerate(b):
    m = re.match(r'(\.LBB\d+_\d+):', l.strip())
    if not m:
        continue
    lab = m.group(1)
    back = [k for k, x in enumerate(b) if k > h and re.search(r's_c?branch\w*\s+' + re.escape(lab) + r'$', x.strip())]
    if not back:
        continue
    seg = [x.strip() for x in b[h:max(back) + 1] if x.strip() and not x.strip().startswith(('.', ';'))]
    if 's_barrier' not in ' '.join(seg):
        continue
    loops.append((lab, seg))
# the innermost loop that still holds a barrier (the iteration loop; the codeword loop holds it too)
lab, seg = min(loops, key=lambda t: len(t[1]))
mix = collections.Counter(re.sub(r'_e(32|64)$', '', x.split()[0]) for x in seg)
valu = sum(v for k, v in mix.items() if k.startswith('v_'))
print(f"loop {lab}: {len(seg)} instr, {valu} VALU:", ", ".join(f"{k} {v}" for k, v in mix.most_common(40)))
