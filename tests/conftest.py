import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'diffusion-models-pytorch_amd')
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a ROCm GPU (MI355X) and the built libdm_hip.so')
    config.addinivalue_line('markers', 'slow: long-running test')


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    with open(os.path.join(GOLDEN, name + '.json')) as f:
        meta = json.load(f)
    return arrays, meta


TOL = 1e-4   # BASELINE.json north_star: fp32 max-abs vs the reference


def drift_bound(drift):
    """Per-step bound of a free-running trajectory: the 1e-4 budget, or 1.5x the reference's own
    float32-vs-float64 drift on the same trajectory (tests/golden/drift.npz, ddpm1000.npz, ddpmcfg.npz,
    made by make_golden_r2.py) where that drift alone already approaches the budget."""
    return max(TOL, 1.5 * float(drift))


@pytest.fixture(scope='session')
def golden():
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = load_golden(name)
        return cache[name]
    return get


_REPORT = {}


@pytest.fixture(scope='session')
def report():
    """record(name, value): measured parity margins, written to gpurun_out/parity_report.json."""
    def record(name, value):
        _REPORT[name] = float(value)
    return record


def pytest_sessionfinish(session, exitstatus):
    if _REPORT:
        out = os.path.join(ROOT, 'gpurun_out')
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, 'parity_report.json'), 'w') as f:
            json.dump(_REPORT, f, indent=1, sort_keys=True)


@pytest.fixture(scope='session')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no ROCm GPU visible')
    return torch.device('cuda:0')
