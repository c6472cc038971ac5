#!/bin/bash
# Round-4 batch 5: attention S-operand prefetch (DM_ATTN_OPT=2) bit-identity check and same-box A/B.
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 200 python3 - <<'PY' || exit 1
import os, sys, torch
sys.path[:0] = ['.', 'diffusion-models-pytorch_amd']
from tests.test_gpu_parity import _model
import json
meta = json.load(open('tests/golden/forward.json'))
cuda = torch.device('cuda', 0)
g = torch.Generator().manual_seed(36)
x = torch.randn((4, 3, 32, 32), generator=g).to(cuda)
t = torch.randint(0, 1000, (4, ), generator=g).to(cuda)
outs = {}
for opt in ('0', '2'):
    os.environ['DM_ATTN_OPT'] = opt
    m, _ = _model(meta, 'cifar10', cuda)
    outs[opt] = m(x, t)
    del m
print('DM_ATTN_OPT=2 bit-identical:', torch.equal(outs['0'], outs['2']))
PY
VAR=DM_ATTN_OPT VAL=2 N=2 bash tools/env_ab.sh
