#!/bin/bash
# Register / spill / LDS summary per kernel of one source: tools/resusage.sh csrc/conv_wino.hip [EXTRA flags]
src=$1; shift
cd "$(dirname "$src")" || exit 2
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include "$@" \
  -Rpass-analysis=kernel-resource-usage -c "$(basename "$src")" -o /tmp/resusage.o 2>&1 |
  python3 -c "
import re, sys
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r'remark: +(Function Name|VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)', line)
    if not m: continue
    k, v = m.groups()
    if k == 'Function Name':
        cur = {'name': v}; rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    print('%-90s v%-4s a%-3s vsp%-4s ssp%-4s lds%-7s occ%s' % (r['name'][:90], r.get('VGPRs'), r.get('AGPRs'), r.get('VGPRs Spill'), r.get('SGPRs Spill'), r.get('LDS Size [bytes/block]'), r.get('Occupancy [waves/SIMD]')))
"
