"""Deferred BN + activation + NoiseInjection (rt.PendingAct, ffc_in_tf): the fgan128 conv6 -> conv7
hand-off where the 3x3 head applies conv6's BatchNorm2d + GELU + noise (ffc_bn_act.py:80-83,
noise_injection.py:25-32, fgan128_complete.py:509-514) while staging its input.

The deferred path evaluates the same BN / noise expression as the separate pass; GELU uses a
branch-free erf (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7) instead of erff, so the tests
ask for <= 2e-6 normwise against that pass (bit-identical running statistics) and <= 1e-4
against the fp64 oracle."""
import contextlib
import io

import pytest
import torch
import torch.nn as nn

from oracle.ffc_oracle import ffc_bn_act, noise_injection, normwise_err

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _rand(mod, gen):
    with torch.no_grad():
        for k, v in mod.state_dict().items():
            if not v.is_floating_point() or v.numel() == 0:
                continue
            if k.endswith("running_var"):
                v.copy_(0.5 + torch.rand(v.shape, generator=gen))
            elif k.endswith("running_mean") or k.endswith("bias"):
                v.copy_(0.1 * torch.randn(v.shape, generator=gen))
            elif v.dim() == 1:
                v.copy_(1 + 0.1 * torch.randn(v.shape, generator=gen))
            elif k.endswith("weight") and v.dim() == 4 and v.shape[0] == 1 and v.shape[2:] == (1, 1):
                v.copy_(torch.randn(v.shape, generator=gen))   # NoiseInjection.weight (zeros by default)
            else:
                v.copy_(torch.randn(v.shape, generator=gen) / max(1, v[0].numel()) ** 0.5)
    return mod


def _sd64(mod):
    return {k: (v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu().clone())
            for k, v in mod.state_dict().items()}


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("cin,H,W,B", [(32, 32, 32, 3), (16, 16, 16, 2), (128, 64, 64, 2)])
def test_deferred_head_matches_separate_pass(train, cin, H, W, B):
    """producer FFC_BN_ACT(cin, cin, 3, 0.5, 0.5, BN, GELU) + NoiseInjection on both branches, consumer
    FFC_BN_ACT(cin, 3, 3, 0.5, 0, Tanh): deferred vs the separate pass and vs the oracle"""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    gen = torch.Generator().manual_seed(cin + H + train)
    with contextlib.redirect_stdout(io.StringIO()):
        prod = F.FFC_BN_ACT(cin, cin, 3, 0.5, 0.5, 1, 1, norm_layer=nn.BatchNorm2d, activation_layer=nn.GELU)
        head = F.FFC_BN_ACT(cin, 3, 3, 0.5, 0.0, 1, 1, activation_layer=nn.Tanh)
    nl_mod, ng_mod = F.NoiseInjection(cin // 2), F.NoiseInjection(cin // 2)
    for m in (prod, head, nl_mod, ng_mod):
        _rand(m, gen)
    sd_p, sd_h = _sd64(prod), _sd64(head)
    sd_n = {"l.weight": nl_mod.weight.detach().double(), "g.weight": ng_mod.weight.detach().double()}
    xl = torch.randn((B, cin // 2, H, W), generator=gen)
    xg = torch.randn((B, cin // 2, H, W), generator=gen)
    nl = torch.randn((B, 1, H, W), generator=gen)
    ng = torch.randn((B, 1, H, W), generator=gen)
    prod, head, nl_mod, ng_mod = (m.cuda().train(train) for m in (prod, head, nl_mod, ng_mod))
    state = {k: v.clone() for k, v in prod.state_dict().items()}
    x = (xl.cuda(), xg.cuda())
    obs = rt.LaunchObserver()
    with torch.no_grad():
        if train:
            y0 = prod.forward_noise(x, (nl_mod, nl.cuda()), (ng_mod, ng.cuda()))
        else:
            y0 = prod(x)
        ref_out, _ = head(y0)
        after = {k: v.clone() for k, v in prod.state_dict().items()}
        prod.load_state_dict(state)   # same running stats for the second train-mode forward
        rt.set_observer(obs)
        try:
            if train:
                y1 = prod.forward_deferred(x, (nl_mod, nl.cuda()), (ng_mod, ng.cuda()))
            else:
                y1 = prod.forward_deferred(x)
            assert isinstance(y1[0], rt.PendingAct) and isinstance(y1[1], rt.PendingAct)
            out, og = head(y1)
        finally:
            rt.set_observer(None)
        torch.cuda.synchronize()
    summ = obs.summary()
    assert og == 0 and "conv3_smallm" in summ and "bn_act_noise" not in summ and "bn_act" not in summ
    assert normwise_err(out.cpu(), ref_out.cpu()) <= 2e-6
    for k, v in prod.state_dict().items():   # running stats advanced exactly as on the eager path
        assert torch.equal(v, after[k]), k
    cfg_p = dict(in_channels=cin, out_channels=cin, kernel_size=3, ratio_gin=0.5, ratio_gout=0.5, stride=1,
                 padding=1, norm_layer="BatchNorm2d", activation_layer="GELU")
    cfg_h = dict(in_channels=cin, out_channels=3, kernel_size=3, ratio_gin=0.5, ratio_gout=0.0, stride=1, padding=1,
                 activation_layer="Tanh")
    rl, rg = ffc_bn_act((xl.double(), xg.double()), sd_p, "", cfg_p, train)
    if train:
        rl = noise_injection(rl, sd_n, "l.", nl.double())
        rg = noise_injection(rg, sd_n, "g.", ng.double())
    ro, _ = ffc_bn_act((rl, rg), sd_h, "", cfg_h, train)
    assert normwise_err(out.cpu(), ro) <= TOL


def test_pending_materializes_for_other_consumers():
    """a PendingAct handed to a layer that cannot apply it (a BN'd FFC_BN_ACT) is materialized first:
    same result as the eager pass"""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    gen = torch.Generator().manual_seed(3)
    with contextlib.redirect_stdout(io.StringIO()):
        prod = F.FFC_BN_ACT(16, 16, 3, 0.5, 0.5, 1, 1, norm_layer=nn.BatchNorm2d, activation_layer=nn.GELU)
        nxt = F.FFC_BN_ACT(16, 16, 3, 0.5, 0.5, 1, 1, norm_layer=nn.BatchNorm2d, activation_layer=nn.ReLU)
    prod, nxt = _rand(prod, gen).cuda().eval(), _rand(nxt, gen).cuda().eval()
    x = (torch.randn((2, 8, 16, 16), generator=gen).cuda(), torch.randn((2, 8, 16, 16), generator=gen).cuda())
    with torch.no_grad():
        a = nxt(prod(x))
        p = prod.forward_deferred(x)
        assert isinstance(p[0], rt.PendingAct)
        b = nxt(p)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("train", [True, False])
def test_fgan128_deferred_head_matches_eager(train):
    """FGenerator.forward_float with conv6 -> conv7 deferred == the separate-pass path (GELU erf within 2e-6)"""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import models
    gen = torch.Generator().manual_seed(11)
    with contextlib.redirect_stdout(io.StringIO()):
        g = F.FGenerator(128)
    g = _rand(g, gen).cuda().train(train)
    state = {k: v.clone() for k, v in g.state_dict().items()}
    B = 3
    z = torch.randn((B, 128), generator=gen).cuda()
    noises = [(torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen).cuda(),
               torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen).cuda()) for n in (2, 3, 4, 5, 6)]
    old = models.DEFER_HEAD_INPUT
    try:
        with torch.no_grad():
            models.DEFER_HEAD_INPUT = False
            a = g.forward_float(z, noises if train else None)
            g.load_state_dict(state)
            models.DEFER_HEAD_INPUT = True
            b = g.forward_float(z, noises if train else None)
    finally:
        models.DEFER_HEAD_INPUT = old
    assert normwise_err(a.cpu(), b.cpu()) <= 2e-6


def test_conv3x3_smallm_tf_abi_validation():
    """ffc_conv3x3_smallm_tf rejects a transform without scale/shift before launching anything"""
    import ctypes
    from fastfourierconvolution_amd import _lib
    L = _lib.load()
    x = torch.zeros((1, 4, 8, 8), device="cuda")
    w = torch.zeros((3, 4, 3, 3), device="cuda")
    out = torch.empty((1, 3, 8, 8), device="cuda")
    bad = _lib.InTf(None, None, 0, 0.0, None, None)
    rc = L.ffc_conv3x3_smallm_tf(x.data_ptr(), 4, w.data_ptr(), None, 0, None, None, 1, 8, 8, 3, out.data_ptr(),
                                 0, 0.0, ctypes.byref(bad), None, None)
    assert rc != 0 and b"scale" in L.ffc_last_error()


@pytest.mark.parametrize("C0,C1,M,H,W,noise,act", [(16, 0, 1, 40, 24, True, 5), (6, 5, 4, 33, 20, False, 2),
                                                  (64, 64, 3, 128, 128, True, 5), (8, 8, 2, 72, 96, True, 1)])
def test_conv3x3_smallm_tf_ragged(C0, C1, M, H, W, noise, act):
    """ffc_conv3x3_smallm_tf on ragged tiles / one or two segments against torch: transform
    (act(x*scale + shift) + noise_w * noise, zero padding outside) then Conv2d 3x3 p1 + Tanh"""
    import ctypes
    import torch.nn.functional as Fn
    from fastfourierconvolution_amd import _lib
    L = _lib.load()
    g = torch.Generator().manual_seed(C0 * 7 + H)
    B = 2
    xs = [torch.randn((B, c, H, W), generator=g).cuda() for c in (C0, C1) if c]
    ws = [(torch.randn((M, c, 3, 3), generator=g) / (9 * c) ** 0.5).cuda() for c in (C0, C1) if c]
    tfs, keep, xt = [], [], []
    for x in xs:
        C = x.shape[1]
        sc = (1 + 0.2 * torch.randn(C, generator=g)).cuda()
        sh = (0.1 * torch.randn(C, generator=g)).cuda()
        nw = torch.randn(C, generator=g).cuda() if noise else None
        nz = torch.randn((B, 1, H, W), generator=g).cuda() if noise else None
        keep += [sc, sh, nw, nz]
        tfs.append(_lib.InTf(sc.data_ptr(), sh.data_ptr(), act, 0.1, nw.data_ptr() if noise else None,
                             nz.data_ptr() if noise else None))
        y = x * sc[None, :, None, None] + sh[None, :, None, None]
        y = {5: Fn.gelu, 2: lambda v: Fn.leaky_relu(v, 0.1), 1: torch.relu}[act](y)
        if noise:
            y = y + nw[None, :, None, None] * nz
        xt.append(y)
    out = torch.empty((B, M, H, W), device="cuda")
    rc = L.ffc_conv3x3_smallm_tf(xs[0].data_ptr(), C0, ws[0].data_ptr(), xs[1].data_ptr() if C1 else None, C1,
                                 ws[1].data_ptr() if C1 else None, None, B, H, W, M, out.data_ptr(), 3, 0.0,
                                 ctypes.byref(tfs[0]), ctypes.byref(tfs[1]) if C1 else None, None)
    assert rc == 0, L.ffc_last_error()
    torch.cuda.synchronize()
    ref = sum(Fn.conv2d(y.double(), w.double(), padding=1) for y, w in zip(xt, ws)).tanh()
    assert normwise_err(out.cpu(), ref.cpu()) <= 1e-5
