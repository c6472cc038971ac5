"""Top kernel families of a bench.py --profile-json file: share of GPU time, ms per forward, TF.
    python tools/prof_top.py gpurun_out/c3_prof.json [N]"""
import json
import sys

d = json.load(open(sys.argv[1]))
fam = d['families']
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(f['ms'] for f in fam.values())
fwd = max(max((op['launches'] for op in d['ops'] if op['label'] == k), default=1) for k in fam) if fam else 1
for k, f in sorted(fam.items(), key=lambda kv: -kv[1]['ms'])[:n]:
    tf = f['flops'] / (f['ms'] * 1e-3) / 1e12 if f['ms'] > 0 and f['flops'] > 0 else 0.0
    gbs = f['bytes'] / (f['ms'] * 1e-3) / 1e9 if f['ms'] > 0 else 0.0
    print(f"{100 * f['ms'] / tot:6.2f} %  {f['ms'] / fwd:8.3f} ms/fwd  {f['launches'] // fwd:4d} x  {tf:7.1f} TF  "
          f"{gbs:7.0f} GB/s  {k}")
print(f'total {tot / fwd:.3f} ms per observed forward ({fwd} observed)')
