"""Instruction mix per basic block (>= MIN instructions) of one kernel in a hipcc --save-temps .s file.
    python tools/isa_blocks.py FILE.s KERNEL_SUBSTRING [MIN]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
names = re.findall(r'^(_Z[^:\s]+):', s, re.M)
name = next(n for n in names if sys.argv[2] in n)
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
blocks, cur = [], None
for ln in s[i:j].split('\n'):
    t = ln.strip()
    if re.match(r'^(\.LBB\S+|; %bb\.\d+):', t):
        cur = [t.split(':')[0], []]
        blocks.append(cur)
        continue
    if cur is None or not t or t.startswith(';') or t.startswith('.'):
        continue
    cur[1].append(t.split()[0])
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 100
print(name)
for lab, ins in blocks:
    if len(ins) < mn:
        continue
    c = Counter(ins)
    mf = sum(v for k, v in c.items() if k.startswith('v_mfma'))
    va = sum(v for k, v in c.items() if k.startswith('v_') and not k.startswith('v_mfma'))
    print(f'{lab:12s} n={len(ins):4d} mfma={mf:3d} valu={va:3d} ' +
          ' '.join(f'{k}:{v}' for k, v in c.most_common() if not k.startswith('v_mfma'))[:400])
