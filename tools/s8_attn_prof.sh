#!/bin/bash
# Per-op HIP-event times of the C3 forward with and without DM_ATTN_OPT=4 (two alternations).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-json gpurun_out/s8_base_$i.json > /dev/null 2>&1 || exit 1
  DM_ATTN_OPT=4 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-json gpurun_out/s8_opt4_$i.json > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import json
for tag in ('base', 'opt4'):
    for i in (1, 2):
        f = json.load(open(f'gpurun_out/s8_{tag}_{i}.json'))['families']
        a = f.get('attn_block4_kernel<8>')
        print(tag, i, 'attn_block4 us/launch', round(a['ms'] / a['launches'] * 1e3, 2))
PY
