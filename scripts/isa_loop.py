"""Instruction histogram of the PGD inner loop(s) of one kernel in a gfx950 assembly file
(the innermost loops holding the evaluation's cross-lane reduction, v_permlane32_swap).
usage: isa_loop.py <file.s> <mangled-kernel-name-substring>"""
import re, sys
from collections import Counter
path, name = sys.argv[1], sys.argv[2]
L = open(path).read().split('\n')
start = next(i for i, l in enumerate(L) if l.startswith('_ZN') and name in l.split(':')[0] and ':' in l)
end = next(i for i in range(start, len(L)) if L[i].startswith('.Lfunc_end'))
F = L[start:end]
# basic blocks with their innermost loop (header, depth) from the assembler's comments
blocks, cur, pending = [], None, False
for l in F:
    if l.startswith('.LBB'):
        cur = {"label": l.split(':')[0], "hdr": None, "depth": 0, "ins": []}
        blocks.append(cur)
        pending = True
    if cur is None:
        continue
    if pending and ';' in l:
        c = l.split(';', 1)[1]
        m = re.search(r'Loop Header: Depth=(\d+)', c)
        if m and cur["hdr"] is None:
            cur["hdr"], cur["depth"] = cur["label"][1:], int(m.group(1))
        m = re.search(r'Header=(BB\d+_\d+) Depth=(\d+)', c)
        if m and cur["hdr"] is None:
            cur["hdr"], cur["depth"] = m.group(1), int(m.group(2))
    if l.startswith('\t') and not l.strip().startswith(';') and not l.strip().startswith('.'):
        pending = False
        cur["ins"].append(l.split()[0])
loops = {}
for b in blocks:
    if b["hdr"]:
        loops.setdefault(b["hdr"], []).append(b)
cand = [h for h, bs in loops.items() if any('v_permlane32_swap_b32_e32' in b["ins"] for b in bs)]
dmax = max(loops[h][0]["depth"] for h in cand)
cand = [h for h in cand if loops[h][0]["depth"] == dmax][:1]     # one of the two alternating inner loops
tot = Counter()
for h in cand:
    bs = loops[h]
    c = Counter(i for b in bs for i in b["ins"])
    tot += c
    print(f"loop {h} depth {bs[0]['depth']}: {sum(c.values())} instructions in {len(bs)} blocks")
valu = {k: v for k, v in tot.items() if k.startswith('v_')}
f64 = sum(v for k, v in valu.items() if k.endswith('f64') or '_f64_' in k)
print(f"all cand loops: VALU {sum(valu.values())} (f64 {f64}), SALU {sum(v for k, v in tot.items() if k.startswith('s_'))}")
for k, v in tot.most_common(40):
    print(f"{v:5d} {k}")
