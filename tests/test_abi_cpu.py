"""CPU checks of the C-ABI library: it loads without a GPU, exports every symbol that
include/ffc_amd.h declares, and its struct layouts match the ctypes mirror."""
import ctypes
import os
import re

import pytest

from conftest import ROOT
from fastfourierconvolution_amd import _lib

HEADER = os.path.join(ROOT, "include", "ffc_amd.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ffc_[a-z0-9_]+)\s*\(", text)))


def test_library_builds_and_loads():
    lib = _lib.load()
    assert lib.ffc_abi_version() == 4


def test_every_declared_symbol_is_exported():
    names = declared_functions()
    assert len(names) >= 14
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(raw, n), n
    bound = {s[0] for s in _lib.SIGNATURES}
    assert set(names) == bound, set(names) ^ bound


def test_struct_layout_matches_binding():
    lib = _lib.load()
    out = (ctypes.c_int * 6)()
    assert lib.ffc_struct_sizes(out, 6) == 0
    assert tuple(out) == (ctypes.sizeof(_lib.ConvSeg), ctypes.sizeof(_lib.ConvPhase), ctypes.sizeof(_lib.ConvJob),
                          ctypes.sizeof(_lib.ConvPSeg), ctypes.sizeof(_lib.ConvPPhase), ctypes.sizeof(_lib.ConvPJob))


def test_argument_validation_without_gpu():
    """invalid shapes are rejected before any launch, with a readable error"""
    lib = _lib.load()
    # Z/Y planes (Re, Im) + the mix weight (2C x ceil32(2C), whole 256-float DMA groups)
    # + BN scale/shift (4C) + the folded input affine (2C)
    assert lib.ffc_fu_lds_bytes(16, 32, 32) == 16 * 16 * 32 * 17 + 4 * 32 * 32 + 4 * 6 * 16
    assert lib.ffc_fu_lds_bytes(16, 64, 64) == 0          # large planes: the staged FU (ffc_fu2d_*)
    assert lib.ffc_fu2d_supported(16, 64, 64, 2) == 1 and lib.ffc_fu2d_supported(32, 128, 128, 1) == 1
    assert lib.ffc_fu2d_supported(65, 64, 64, 1) == 0     # 2C > 128
    assert lib.ffc_fu2d_supported(8, 64, 32, 1) == 0      # not square
    assert lib.ffc_fu_lds_bytes(16, 12, 12) == 0          # not a power of two
    rc = lib.ffc_fu_forward(None, 1, 4, 12, 12, 1, None, None, 0, None, 0, None, None, None, 0, None, None)
    assert rc == -1
    assert b"unsupported" in lib.ffc_last_error()
    rc = lib.ffc_conv_forward(None, 0, None, 0, 0, None)
    assert rc == -1
    # ST prologue workgroups per sample: a power of two dividing conv1's output tiles
    # (ceil32(c)/32 x ceil32(hw)/32), growing while the grid is below 256, at most 8
    assert lib.ffc_st_prologue_split(32, 256, 8, 8, 1, 64) == 2     # 2 x 1 tiles
    assert lib.ffc_st_prologue_split(32, 128, 16, 16, 1, 32) == 2   # 1 x 2 tiles
    assert lib.ffc_st_prologue_split(32, 64, 32, 32, 1, 16) == 8    # 1 x 8 tiles
    assert lib.ffc_st_prologue_split(256, 64, 32, 32, 1, 16) == 1   # the batch fills the GPU
    assert lib.ffc_st_prologue_split(3, 16, 4, 4, 0, 16) == 1       # one tile
    p = ctypes.c_void_p(16)   # never dereferenced: the split check fails first
    rc = lib.ffc_st_prologue_ex(p, 4, 64, 32, 32, 1, None, None, 0, p, 16, 3, p, p, None, None)
    assert rc == -1 and b"split" in lib.ffc_last_error()


def test_product_path_refuses_cpu_tensors():
    import torch
    import contextlib
    import io
    import fastfourierconvolution_amd as F
    with contextlib.redirect_stdout(io.StringIO()):
        m = F.FFC_BN_ACT(8, 8, 3, 0.5, 0.5, 1, 1)
    with pytest.raises(_lib.FFCError, match="no CPU fallback"):
        m((torch.randn(1, 4, 8, 8), torch.randn(1, 4, 8, 8)))


def test_state_dict_names_match_reference(manifest):
    import contextlib
    import io
    import fastfourierconvolution_amd as F
    import torch.nn as nn
    for case in manifest["cases"]:
        kw = dict(case["ctor"])
        for k in ("norm_layer", "activation_layer"):
            if k in kw:
                kw[k] = getattr(nn, kw[k])
        with contextlib.redirect_stdout(io.StringIO()):
            mod = getattr(F, case["kind"])(**kw)
        sd = mod.state_dict()
        assert set(sd) == set(case["specs"]), case["name"]
        for k, spec in case["specs"].items():
            assert list(sd[k].shape) == list(spec[0]), (case["name"], k)
