"""Kernel-level parity on the GPU (through the C ABI): the 1x1 tiled GEMM (ffc_pw_forward) and the
LDS-patch kernel's 4-channel x 16-tap chunks (Conv2d k4 s2), each against a torch fp64 reference of the
same op (normwise <= 1e-5; the kernels compute exact fp32 products with fp32 accumulation)."""
import pytest
import torch
import torch.nn.functional as F

from fastfourierconvolution_amd import _autograd as ag
from fastfourierconvolution_amd import _plan
from fastfourierconvolution_amd import _runtime as rt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _nerr(a, b):
    return ((a.double().cpu() - b.double().cpu()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


PW_CASES = [  # (B, M, [C per segment], H, W, bias, addend, act)
    (8, 128, [128], 16, 9, False, False, 0),       # D ffc1 FU spectral mix (odd plane)
    (5, 200, [64, 48], 8, 5, True, True, 2),        # two segments, M not a tile multiple, LeakyReLU
    (3, 40, [17], 7, 3, False, True, 0),            # tiny, ragged everything
    (16, 512, [512], 4, 3, False, False, 0),        # D ffc3 FU mix
    (2, 16, [64, 64, 32], 32, 32, True, False, 1),  # three segments, ReLU
]


@pytest.mark.parametrize("case", PW_CASES, ids=[f"pw{i}" for i in range(len(PW_CASES))])
def test_pw_gemm_matches_fp64(case):
    B, M, Cs, H, W, use_bias, use_add, act = case
    gen = torch.Generator().manual_seed(7)
    xs = [torch.randn(B, C, H, W, generator=gen) for C in Cs]
    ws = [torch.randn(M, C, 1, 1, generator=gen) / C ** 0.5 for C in Cs]
    bias = torch.randn(M, generator=gen) if use_bias else None
    add = torch.randn(B, M, H, W, generator=gen) if use_add else None
    ref = sum(F.conv2d(x.double(), w.double()) for x, w in zip(xs, ws))
    if bias is not None:
        ref = ref + bias.double()[None, :, None, None]
    if add is not None:
        ref = ref + add.double()
    ref = {0: ref, 1: ref.clamp_min(0), 2: F.leaky_relu(ref, 0.1)}[act]
    segs = [_plan.Seg("pw", C, H, W) for C in Cs]
    wts = [(w.to(DEV), 0, 1, 1, bias.to(DEV) if (bias is not None and i == 0) else None) for i, w in enumerate(ws)]
    cache = {}
    out = ag.run_conv(cache, "k", B, M, segs, wts, [x.to(DEV) for x in xs], act=(act, 0.1),
                      addend=add.to(DEV) if add is not None else None)
    torch.cuda.synchronize()
    (ex, _), = cache.values()     # run_conv's one plan (keyed by "k" + the job shape + plan switches)
    assert ex.kind == "pw"
    assert _nerr(out, ref) <= 1e-5


CONV16_CASES = [  # (B, M, [(C, IH, IW)] segments of Conv2d k4 s2 p1, extra pw segment channels)
    (4, 128, [(64, 32, 32), (64, 32, 32)], 0),      # FFCDiscriminator ffc1 local branch
    (4, 128, [(64, 32, 32)], 64),                   # ffc1 global branch: l2g + conv2 (1x1) in one job
    (32, 512, [(256, 8, 8), (256, 8, 8)], 0),       # ffc3 (4x4 outputs, smaller pixel block config)
    (3, 64, [(3, 64, 64)], 0),                      # ffc0: 3 input channels (padded to 4)
    (2, 40, [(5, 9, 7)], 0),                        # ragged
]


@pytest.mark.parametrize("case", CONV16_CASES, ids=[f"c16_{i}" for i in range(len(CONV16_CASES))])
def test_conv_k4s2_patch_matches_fp64(case):
    B, M, specs, cpw = case
    gen = torch.Generator().manual_seed(11)
    segs, xs, ws, ref = [], [], [], 0
    for C, IH, IW in specs:
        x = torch.randn(B, C, IH, IW, generator=gen)
        w = torch.randn(M, C, 4, 4, generator=gen) / (16 * C) ** 0.5
        segs.append(_plan.Seg("conv", C, IH, IW, 4, 2, 1))
        xs.append(x)
        ws.append((w, 0, 4, 4, None))
        ref = ref + F.conv2d(x.double(), w.double(), stride=2, padding=1)
    if cpw:
        OH, OW = ref.shape[2:]
        x = torch.randn(B, cpw, OH, OW, generator=gen)
        w = torch.randn(M, cpw, 1, 1, generator=gen) / cpw ** 0.5
        segs.append(_plan.Seg("pw", cpw, OH, OW))
        xs.append(x)
        ws.append((w, 0, 1, 1, None))
        ref = ref + F.conv2d(x.double(), w.double())
    pl = _plan.pick_patch_cfg(B, M, segs)
    assert pl is not None and 4 in pl.cc
    cache = {}
    out = ag.run_conv(cache, "k", B, M, segs, [(w.to(DEV), l, kh, kw, b) for w, l, kh, kw, b in ws],
                      [x.to(DEV) for x in xs])
    torch.cuda.synchronize()
    assert next(iter(cache.values()))[0].kind == "patch"
    assert _nerr(out, ref) <= 1e-5
