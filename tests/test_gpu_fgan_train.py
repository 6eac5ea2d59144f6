"""fgan128 training path (fgan128_complete.py:680-703 trains FGenerator): an FFC_BN_ACT layer of the
fgan128 stack (FFCTranspose k4 s2, BatchNorm2d + GELU, SpectralTransform with the spectrum-side
upsample, 64x64 and 128x128 Fourier units on the line-FFT planar transforms) followed by
NoiseInjection on both branches, forward + backward against the fp64 oracle's autograd
(torch.fft in fp64), with the ReLU active sets of the spectral branch taken from the HIP path's own
outputs (as tests/test_gpu_train.py does: the network is piecewise linear there).  Also the
NoiseInjection weight gradient, the nn.Linear of noise_to_feature, and a whole FGenerator train step.
Tolerance: normwise 1e-4."""
import contextlib
import io

import pytest
import torch
import torch.nn as nn

from oracle.ffc_oracle import ffc_bn_act, noise_injection, normwise_err

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _randomize(mod, gen):
    with torch.no_grad():
        for k, v in mod.state_dict().items():
            if not v.is_floating_point() or v.numel() == 0 or k.endswith(("running_mean", "running_var")):
                continue
            if k.endswith("weight") and v.dim() == 4 and v.shape[0] == 1 and v.shape[2:] == (1, 1):
                v.copy_(torch.randn(v.shape, generator=gen))            # NoiseInjection.weight
                continue
            fan = v[0].numel() if v.dim() > 1 else 1
            base = 1.0 if (v.dim() == 1 and k.endswith("weight")) else 0.0
            v.copy_(base + torch.randn(v.shape, generator=gen) / max(1, fan) ** 0.5 * (0.1 if v.dim() == 1 else 1))
    return mod


class _Block(nn.Module):
    def __init__(self, cin, cout, rin):
        super().__init__()
        import fastfourierconvolution_amd as F
        with contextlib.redirect_stdout(io.StringIO()):
            self.conv = F.FFC_BN_ACT(cin, cout, 4, rin, 0.5, stride=2, padding=1, activation_layer=nn.GELU,
                                     norm_layer=nn.BatchNorm2d, upsampling=True, uses_noise=True, uses_sn=True)
        self.lcl = F.NoiseInjection(cout - cout // 2)
        self.glb = F.NoiseInjection(cout // 2)


def test_noise_wgrad_kernel():
    from fastfourierconvolution_amd import _lib
    L = _lib.load()
    g = torch.Generator().manual_seed(1)
    dy = torch.randn((3, 5, 8, 12), generator=g).cuda()
    nz = torch.randn((3, 1, 8, 12), generator=g).cuda()
    dw = torch.empty(5, device="cuda")
    assert L.ffc_noise_wgrad(dy.data_ptr(), nz.data_ptr(), 3, 5, 96, dw.data_ptr(), None) == 0
    torch.testing.assert_close(dw.double().cpu(), (dy.double() * nz.double()).sum((0, 2, 3)).cpu(), rtol=1e-6,
                               atol=1e-6)


@pytest.mark.parametrize("cin,cout,H,rin,B", [(64, 32, 64, 0.5, 2), (64, 64, 32, 0.5, 2), (128, 64, 4, 0.0, 3)])
def test_fgan128_layer_grads_vs_oracle(cin, cout, H, rin, B):
    """NoiseInjection(FFC_BN_ACT(...)) fwd + bwd: input, weight, BN, SE, Fourier-unit and noise-weight
    gradients vs the fp64 oracle (H -> 2H output; H = 64 runs the 128x128 Fourier unit)"""
    from fastfourierconvolution_amd import _autograd as ag
    import oracle.ffc_oracle as O
    from test_gpu_train import _KinkF
    gen = torch.Generator().manual_seed(cin + H)
    blk = _randomize(_Block(cin, cout, rin), gen)
    sd0 = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    cg = int(cin * rin)
    xl = torch.randn((B, cin - cg, H, H), generator=gen)
    xg = torch.randn((B, cg, H, H), generator=gen) if cg else None
    nl = torch.randn((B, 1, 2 * H, 2 * H), generator=gen)
    ng = torch.randn((B, 1, 2 * H, 2 * H), generator=gen)
    cl_ = torch.randn((B, cout - cout // 2, 2 * H, 2 * H), generator=gen)
    cg_ = torch.randn((B, cout // 2, 2 * H, 2 * H), generator=gen)
    blk = blk.cuda().train()
    xs = [xl.cuda().requires_grad_(True)] + ([xg.cuda().requires_grad_(True)] if cg else [])
    ag.RECORD = []
    try:
        yl, yg = blk.conv.forward_noise(tuple(xs) if cg else xs[0], (blk.lcl, nl.cuda()), (blk.glb, ng.cuda()))
        recorded = [t.cpu() for t in ag.RECORD]
    finally:
        ag.RECORD = None
    ((yl * cl_.cuda()).sum() + (yg * cg_.cuda()).sum()).backward()
    params = {k: p for k, p in blk.named_parameters() if p.grad is not None}
    # fp64 oracle on the same inputs, ReLU active sets from the HIP path
    sd = {k: (v.double().clone().requires_grad_(True) if v.is_floating_point() else v.clone()) for k, v in sd0.items()}
    xin = [xl.double().requires_grad_(True)] + ([xg.double().requires_grad_(True)] if cg else [])
    cfg = dict(in_channels=cin, out_channels=cout, kernel_size=4, ratio_gin=rin, ratio_gout=0.5, stride=2,
               padding=1, activation_layer="GELU", norm_layer="BatchNorm2d", upsampling=True)
    old = O.F
    O.F = _KinkF([r.double() for r in recorded if r.dim() == 4], [])
    try:
        ol, og = ffc_bn_act(tuple(xin) if cg else xin[0], sd, "conv.", cfg, True, fft="torch")
    finally:
        O.F = old
    ol = noise_injection(ol, sd, "lcl.", nl.double())
    og = noise_injection(og, sd, "glb.", ng.double())
    assert normwise_err(yl.detach().cpu(), ol.detach()) <= TOL
    assert normwise_err(yg.detach().cpu(), og.detach()) <= TOL
    ((ol * cl_.double()).sum() + (og * cg_.double()).sum()).backward()
    errs = {}
    for j, (mine, ref) in enumerate(zip(xs, xin)):
        errs[f"in{j}"] = normwise_err(mine.grad.cpu(), ref.grad)
    for k, p in params.items():
        key = k
        if key.endswith("weight_orig") or key not in sd:
            continue
        assert sd[key].grad is not None, key
        errs[key] = normwise_err(p.grad.cpu(), sd[key].grad)
    print(f"fgan layer {cin}->{cout} @ {H}: {len(errs)} gradients, worst {max(errs.values()):.2e}")
    assert "lcl.weight" in errs and "glb.weight" in errs
    assert (not cg) or any("fu.conv_layer" in k for k in errs)   # in_cg = 0: no SpectralTransform
    bad = {k: e for k, e in errs.items() if not e <= TOL}
    assert not bad, bad


def test_fgan128_train_step():
    """a whole FGenerator train step (Linear, conv2..conv7, NoiseInjection, 8x8..128x128 Fourier units)
    at B = 2: forward loss vs the fp64 oracle, every parameter receives a finite gradient, an Adam step
    changes the next forward"""
    import fastfourierconvolution_amd as F
    from oracle.ffc_oracle import fgan128_generator
    gen = torch.Generator().manual_seed(4)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FGenerator(128)
    _randomize(G, gen)
    sd = {k: (v.detach().double().clone() if v.is_floating_point() else v.detach().clone())
          for k, v in G.state_dict().items()}
    G = G.cuda().train()
    B = 2
    z = torch.randn((B, 128), generator=gen)
    noises = [(torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen),
               torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen)) for n in (2, 3, 4, 5, 6)]
    out = G.forward_float(z.cuda(), [(a.cuda(), b.cuda()) for a, b in noises])
    loss = out.square().mean()
    loss.backward()
    with torch.no_grad():
        ref = fgan128_generator(z.double(), sd, True, [(a.double(), b.double()) for a, b in noises])
    rel = abs(loss.item() - ref.square().mean().item()) / ref.square().mean().item()
    print(f"fgan128 train step B=2: loss rel err {rel:.2e}")
    assert rel <= TOL
    # the SpectralTransform's lfu parameters are dead in the reference too (spectral_transform.py:66-87)
    missing = [k for k, p in G.named_parameters() if p.requires_grad and ".lfu." not in k and
               (p.grad is None or not torch.isfinite(p.grad).all())]
    assert not missing, missing[:5]
    opt = torch.optim.Adam(G.parameters(), lr=1e-3)
    opt.step()
    out2 = G.forward_float(z.cuda(), [(a.cuda(), b.cuda()) for a, b in noises])
    assert not torch.equal(out2.detach(), out.detach())


def test_fgan128_train_iteration_graph_replay_matches_eager():
    """the fgan128train bench step -- generator_step + discriminator_step (fgan128_complete.py:680-703)
    with the spectral-norm Discriminator, AdamW(capturable), NoiseInjection and weight re-packs keyed by
    weight version -- replayed from one captured hipGraph gives bit-identical G / D weights, BN buffers
    and spectral-norm weight_u / weight_v to the same number of eager iterations"""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd.graphs import capture_step
    from fastfourierconvolution_amd.training import discriminator_step, generator_step
    B = 4
    gen = torch.Generator().manual_seed(5)
    z_g = torch.randn(B, 128, generator=gen).cuda()
    z_d = torch.randn(B, 128, generator=gen).cuda()
    real = (torch.rand(B, 3, 128, 128, generator=gen) * 2 - 1).cuda()
    noises = [tuple(torch.randn(B, 1, s, s, generator=gen).cuda() for _ in range(2)) for s in (8, 16, 32, 64, 128)]
    res = []
    for graph in (False, True):
        torch.manual_seed(0)
        with contextlib.redirect_stdout(io.StringIO()):
            G = F.FGenerator(128)
        D = F.Discriminator()
        G, D = G.cuda().train(), D.cuda().train()
        kw = dict(lr=2e-4, betas=(0.5, 0.999), foreach=True, capturable=True)
        optim_G, optim_D = torch.optim.AdamW(G.parameters(), **kw), torch.optim.AdamW(D.parameters(), **kw)

        def step():
            generator_step(G, D, optim_G, optim_D, z_g, noises)
            discriminator_step(G, D, optim_G, optim_D, z_d, real, noises)
        if graph:
            g = capture_step(step, warmup=2)
            assert g is not None, "capture failed"
            for _ in range(2):
                g.replay()
        else:
            for _ in range(4):
                step()
        torch.cuda.synchronize()
        res.append({n + k: v.detach().cpu().clone() for n, m in (("G.", G), ("D.", D))
                    for k, v in m.state_dict().items()})
    assert any(k.endswith("weight_u") for k in res[0])
    for k in res[0]:
        assert torch.equal(res[0][k], res[1][k]), k
