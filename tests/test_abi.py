"""The C-ABI library loads without a GPU and exports every symbol declared in
include/dm_hip.h; host-only entry points validate their arguments."""
import ctypes

import pytest

import dmhip
from dmhip._lib import UNetArch


def test_library_exports_every_header_symbol():
    L = dmhip.load()
    names = dmhip.exported_symbols()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert L.dm_abi_version() == 2  # (include/dm_hip.h DM_ABI_VERSION: dm_conv_desc grew in version 2)


def test_abi_version_matches_header_and_conv_desc_layout():
    """DM_ABI_VERSION in the header, the binding's expectation and the library agree, and the ctypes dm_conv_desc
    ends with the fields version 2 added (a version-1 caller's shorter struct must be refused)."""
    import re
    from dmhip import _lib
    hdr = open(_lib._HEADER).read()
    v = int(re.search(r'#define DM_ABI_VERSION (\d+)', hdr).group(1))
    assert v == _lib.ABI_VERSION == dmhip.load().dm_abi_version() == 2
    fields = [f[0] for f in dmhip.ConvDesc._fields_]
    assert fields[-2:] == ['w_wino', 'w_wino_fold'], fields


def _arch(dim=128, mults=(1, 2, 2, 2), attn=(0, 1, 0, 0), nres=2, heads=1, cin=3, cout=3):
    a = UNetArch()
    a.in_channels, a.out_channels, a.dim, a.n_stages = cin, cout, dim, len(mults)
    for i, (m, at) in enumerate(zip(mults, attn)):
        a.dim_mults[i], a.use_attn[i] = m, at
    a.num_res_blocks, a.n_heads = nres, heads
    return a


def test_param_count_matches_reference_registration():
    from models.unet import UNet
    L = dmhip.load()
    for kw, ours in [(dict(), dict()), (dict(dim=64, cin=1, cout=1), dict(dim=64, in_channels=1, out_channels=1)),
                     (dict(dim=32, mults=(1, 2), attn=(0, 1), nres=1, heads=2),
                      dict(dim=32, dim_mults=[1, 2], use_attn=[False, True], num_res_blocks=1, n_heads=2))]:
        n = ctypes.c_int()
        assert L.dm_unet_param_count(ctypes.byref(_arch(**kw)), ctypes.byref(n)) == 0
        assert n.value == len(UNet(**ours).state_dict())


def test_create_rejects_bad_arguments():
    L = dmhip.load()
    h = ctypes.c_void_p()
    arr = (ctypes.c_void_p * 1)()
    num = (ctypes.c_int64 * 1)()
    rc = L.dm_unet_create(ctypes.byref(_arch()), arr, num, 1, None, ctypes.byref(h))
    assert rc == dmhip._lib.DM_ERR_ARG
    assert b'expected 328 parameter tensors' in L.dm_last_error()
    bad = _arch(dim=100)
    n = ctypes.c_int()
    assert L.dm_unet_param_count(ctypes.byref(bad), ctypes.byref(n)) == dmhip._lib.DM_ERR_ARG
    with pytest.raises(ValueError):
        dmhip._lib.check(dmhip._lib.DM_ERR_ARG, 'x')


def test_library_built_from_these_sources():
    """dm_build_info's source fingerprint equals the tree's (csrc/Makefile SRC_HASH): the libdm_hip.so the
    tests load -- here and, in tests/test_gpu_r3.py, on the GPU box -- was built from these sources."""
    info = dmhip._lib.build_info()
    assert info.startswith('src=') and 'arch=gfx950' in info, info
    assert info.split()[0] == 'src=' + dmhip._lib.source_hash(), (info, dmhip._lib.source_hash())
