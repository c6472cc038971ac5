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


def check_free_running(got, ref32, ref64, drift, i):
    """Step i of a free-running trajectory against the reference (tests/golden/drift.npz, ddpm1000.npz,
    ddpmcfg.npz; make_golden_r2.py ran the reference module in float32 AND in float64 on the same inputs).

    Where the reference's own fp32 run stays within 1e-4 of its float64 run, the engine must match the
    fp32 reference within 1e-4. Where the reference itself drifts further (x0 = sqrt(1/a_t) x - ...
    amplifies rounding ~160x at t ~ 1000, CFG adds a (2s - 1) gain), the engine must be at least as
    accurate as the reference: its distance to the float64 trajectory at most 1.5x the drift the fp32
    reference has accumulated by step i (max over steps <= i), and hence within 2.5x of that drift of
    the fp32 reference. Returns (error vs fp32 reference, error vs float64 run)."""
    import numpy as np
    got = np.asarray(got, dtype=np.float64)
    d = float(np.max(drift[:i + 1]))
    e32 = float(np.abs(got - ref32).max())
    e64 = float(np.abs(got - ref64).max())
    assert e64 <= max(TOL, 1.5 * d), f'step {i}: {e64:.3e} from the float64 run, reference drift {d:.3e}'
    assert e32 <= max(TOL, 2.5 * d), f'step {i}: {e32:.3e} from the fp32 reference, reference drift {d:.3e}'
    return e32, e64


def check_chaos_envelope(golden, name, worst64, report, key):
    """The engine's free-running distance to the float64 trajectory (max over steps) against the spread of
    the REFERENCE's own fp32 runs with the model output perturbed at the level the engine's forwards differ
    from the reference's (2^-20 relative, 8 seeds; tests/golden/chaos.npz, make_golden_r3.py make_chaos):
    it must lie inside that envelope (<= the worst perturbed run). Reports where it lies: the fraction of
    perturbed reference runs that end further from float64 than the engine does."""
    import numpy as np
    g, _ = golden('chaos')
    runs = g[f'{name}_e64_p20'].max(axis=1)
    report(f'{key}_chaos_envelope_2^-20_max', float(runs.max()))
    report(f'{key}_chaos_envelope_2^-22_max', float(g[f'{name}_e64_p22'].max()))
    report(f'{key}_perturbed_reference_runs_further_than_engine', float(np.mean(runs > worst64)))
    assert worst64 <= max(TOL, float(runs.max())), (worst64, list(runs))


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
