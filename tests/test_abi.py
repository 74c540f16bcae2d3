"""C-ABI checks that run without a GPU: the library loads, exports every symbol
include/azg_pv.h declares, and its flat layout equals the reference module's
parameter / BatchNorm order (network.py:41-73).  No compute calls."""
import ctypes
import os
import re

import pytest
import torch.nn as nn

from conftest import REPO

import _native
from oracle.ref_net import RefNet

HEADER = os.path.join(REPO, "include", "azg_pv.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\*?\s+\**(azg_pv_[a-z_0-9]+)\s*\(", txt, re.M)))


def test_header_declares_expected_entry_points():
    syms = header_symbols()
    assert set(syms) == set(_native.EXPORTS), syms


def test_library_exports_every_header_symbol():
    lib = _native.load_library()
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert lib.azg_pv_abi_version() == _native.ABI_VERSION


@pytest.mark.parametrize("blocks,ch", [(3, 64), (6, 128), (10, 256), (0, 64)])
def test_flat_layout_matches_module_order(blocks, ch):
    lib = _native.load_library()
    cfg = _native.AzgConfig(blocks, ch, 15, 3)
    h = ctypes.c_void_p()
    _native.check(lib.azg_pv_create(ctypes.byref(cfg), ctypes.byref(h)), lib)
    try:
        net = RefNet(blocks, ch)
        params = list(net.parameters())
        n = lib.azg_pv_num_param_tensors(h)
        assert n == len(params)
        offs = (ctypes.c_int64 * n)()
        nums = (ctypes.c_int64 * n)()
        _native.check(lib.azg_pv_param_layout(h, offs, nums), lib)
        o = 0
        for i, p in enumerate(params):
            assert offs[i] == o and nums[i] == p.numel()
            o += p.numel()
        assert lib.azg_pv_param_count(h) == o
        bns = [m for m in net.modules() if isinstance(m, nn.BatchNorm2d)]
        assert lib.azg_pv_bn_count(h) == sum(2 * b.num_features for b in bns)
    finally:
        lib.azg_pv_destroy(h)


def test_create_rejects_bad_config():
    lib = _native.load_library()
    h = ctypes.c_void_p()
    for cfg in [(6, 96, 15, 3), (6, 128, 19, 3), (6, 128, 15, 4)]:
        rc = lib.azg_pv_create(ctypes.byref(_native.AzgConfig(*cfg)), ctypes.byref(h))
        assert rc != 0
        assert lib.azg_pv_last_error()


def test_no_cpu_fallback():
    from network import PyTorchModel
    with pytest.raises(RuntimeError, match="HIP"):
        PyTorchModel(device="cpu")
