"""Every environment switch the library reads (refresh_toggles in csrc/api.hip, the only place they are read) has a
row in DESIGN.md's toggle table, with the test that uses it as an oracle. CPU-only: source text checks."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read(*parts):
    with open(os.path.join(ROOT, *parts), encoding='utf-8') as f:
        return f.read()


def test_every_library_toggle_is_documented():
    api = _read('diffusion-models-pytorch_amd', 'csrc', 'api.hip')
    read = set(re.findall(r'(?:getenv|env_is)\("(DM_[A-Z0-9_]+)"', api))
    assert read, 'no toggles found in api.hip'
    design = _read('DESIGN.md')
    rows = {m.group(1) for m in re.finditer(r'^\| `(DM_[A-Z0-9_]+)', design, re.M)}
    missing = sorted(read - rows)
    assert not missing, f'toggles read in api.hip without a DESIGN.md table row: {missing}'


def test_toggles_read_only_in_api():
    """No other library source reads the environment for a DM_ switch (one snapshot per plan build)."""
    csrc = os.path.join(ROOT, 'diffusion-models-pytorch_amd', 'csrc')
    for name in sorted(os.listdir(csrc)):
        if not name.endswith(('.hip', '.h')) or name == 'api.hip':
            continue
        text = _read('diffusion-models-pytorch_amd', 'csrc', name)
        assert not re.search(r'getenv\("DM_', text), f'{name} reads a DM_ switch outside refresh_toggles'
