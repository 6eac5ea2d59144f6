"""ffc_convq_forward (csrc/convq_kernels.hip) against PyTorch's fp32 ConvTranspose2d / 1x1 conv on
the GPU: every (MT, NTW) configuration, ragged batches, channel counts that are not multiples of
16, one to three segments (two ConvT k4 s2 + the direct 1x1 at the output resolution), tiny
inputs whose phases lose taps, bias, addend, BN partial slabs and fused activations.
Tolerance: normwise 1e-5 (fp32-accurate split-bf16 products, SURVEY.md §8c bound 1e-4)."""
import os

import pytest
import torch
import torch.nn.functional as F

from oracle.ffc_oracle import normwise_err

pytestmark = pytest.mark.gpu


def _run(B, C0, C1, Cv, IH, M, cfg, bias=False, addend=False, stats=False, act=0, seed=0, ksplit=None):
    from fastfourierconvolution_amd import _lib, _plan, _runtime as rt
    g = torch.Generator().manual_seed(seed)
    segs, ws, xs = [], [], []
    for C in (C0, C1):
        if C:
            segs.append(_plan.Seg("convT", C, IH, IH, 4, 2, 1))
            ws.append(torch.randn(C, M, 4, 4, generator=g).cuda() / (4 * C) ** 0.5)
            xs.append(torch.randn(B, C, IH, IH, generator=g).cuda())
    if Cv:
        segs.append(_plan.Seg("pw", Cv, 2 * IH, 2 * IH))
        ws.append(torch.randn(M, Cv, 1, 1, generator=g).cuda() / Cv ** 0.5)
        xs.append(torch.randn(B, Cv, 2 * IH, 2 * IH, generator=g).cuda())
    bvec = torch.randn(M, generator=g).cuda() if bias else None
    weights = [(w, 1 if s.kind == "convT" else 0, w.shape[2], w.shape[3], bvec if i == 0 else None)
               for i, (s, w) in enumerate(zip(segs, ws))]
    env = {"FFC_CONVQ_CFG": str(cfg)}
    if ksplit is not None:
        env["FFC_CONVQ_KSPLIT"] = str(ksplit)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ex = rt.ConvExec(B, M, segs, weights, xs[0].device)
        lp = rt.LaunchPlan([ex], xs[0].device) if ex.launch_key[0] == "q" else None
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    if ex.launch_key[0] != "q":
        pytest.skip("no convq plan for this shape / configuration")
    if ksplit is not None:
        assert lp.ksplit == min(ksplit, _plan.convq_chunks(ex.plan))
    ref = 0
    for s, w, x in zip(segs, ws, xs):
        ref = ref + (F.conv_transpose2d(x, w, stride=2, padding=1) if s.kind == "convT" else F.conv2d(x, w))
    if bias:
        ref = ref + bvec[None, :, None, None]
    add = torch.randn(ref.shape, generator=g).cuda() if addend else None
    if addend:
        ref = ref + add
    out = torch.full(ref.shape, float("nan"), device="cuda")
    slab = torch.zeros((lp.stat_rows(0), M, 4), device="cuda") if stats else None
    job = ex.job([(x, None) for x in xs], out, act, 0.1, add, slab)
    lp.launch([job], torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    if lp.ksplit > 1:   # a second launch reproduces the first bit for bit
        first = out.clone()
        lp.launch([job], torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(out, first)
    pre = ref
    if act == 2:
        ref = F.leaky_relu(ref, 0.1)
    elif act == 5:
        ref = F.gelu(ref)
    assert not torch.isnan(out).any()
    err = normwise_err(out.cpu().double(), ref.cpu().double())
    assert err <= 1e-5, err
    if stats:   # merge the {n, mean, M2} rows -> per-channel mean / var of the pre-activation output
        s = slab.double().cpu()
        n = s[..., 0].sum(0)
        mean = (s[..., 0] * s[..., 1]).sum(0) / n
        m2 = (s[..., 2] + s[..., 0] * (s[..., 1] - mean) ** 2).sum(0)
        p = pre.double().cpu()
        torch.testing.assert_close(n, torch.full((M,), float(p.numel() // M), dtype=torch.float64))
        torch.testing.assert_close(mean, p.mean(dim=(0, 2, 3)), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(m2 / n, p.var(dim=(0, 2, 3), unbiased=False), rtol=1e-5, atol=1e-6)
    return lp


@pytest.mark.parametrize("cfg", [0, 1, 2, 3])
@pytest.mark.parametrize("B,C0,C1,Cv,IH,M", [(3, 20, 12, 8, 4, 40), (2, 16, 0, 0, 8, 32), (5, 7, 9, 16, 12, 70),
                                             (1, 33, 0, 5, 16, 64), (4, 16, 16, 0, 4, 32), (2, 64, 64, 16, 16, 32),
                                             (7, 128, 128, 0, 8, 64), (2, 8, 8, 8, 32, 36), (3, 32, 32, 32, 64, 64)])
def test_convq_vs_torch(cfg, B, C0, C1, Cv, IH, M):
    _run(B, C0, C1, Cv, IH, M, cfg, seed=cfg + 10 * B)


@pytest.mark.parametrize("ksplit", [2, 3, 8])
@pytest.mark.parametrize("cfg", [0, 2, 3])
@pytest.mark.parametrize("B,C0,C1,Cv,IH,M", [(3, 20, 12, 8, 4, 40), (5, 7, 9, 16, 12, 70), (7, 128, 128, 0, 8, 64),
                                             (2, 64, 64, 16, 16, 32), (1, 16, 0, 48, 8, 32)])
def test_convq_ksplit(ksplit, cfg, B, C0, C1, Cv, IH, M):
    """K split: contiguous chunk ranges (staged, then direct) per workgroup, partial fragments summed
    in split order by the last arrival, counters re-zeroed (a second launch is bit-identical)"""
    _run(B, C0, C1, Cv, IH, M, cfg, seed=cfg + 3 * B + ksplit, ksplit=ksplit)


@pytest.mark.parametrize("cfg", [0, 2])
def test_convq_ksplit_epilogue(cfg):
    _run(3, 24, 8, 8, 8, 48, cfg, bias=True, addend=True, stats=True, act=2, seed=7, ksplit=4)


@pytest.mark.parametrize("cfg", [0, 2])
def test_convq_epilogue(cfg):
    _run(3, 24, 8, 8, 8, 48, cfg, bias=True, addend=True, stats=True, act=2, seed=5)
    _run(2, 16, 16, 0, 4, 64, cfg, stats=True, act=5, seed=6)


def test_convq_gen64_shapes_used():
    """the generator's ConvT k4 s2 jobs (B = 256 and a B = 32 shard) run on convq"""
    from fastfourierconvolution_amd import _plan, _runtime as rt
    for B in (256, 32):
        for C, IH, M, c in [(256, 4, 128, 64), (128, 8, 64, 32), (64, 16, 32, 16)]:
            segs = [_plan.Seg("convT", C, IH, IH, 4, 2, 1), _plan.Seg("pw", c, 2 * IH, 2 * IH)]
            assert _plan.pick_convq_cfg(B, M, segs) is not None
    assert rt.USE_CONVQ and rt.CONV_ARITH == "split"
