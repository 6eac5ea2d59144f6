"""BASELINE config 5 pieces on the GPU: spectral-norm FFC stacks (layers/snffc) and the fp16-operand
spectral mix, against the fp64 oracle (oracle/ffc_oracle.py: sn_materialize restates
torch.nn.utils.spectral_norm; the SNFFC golden cases pin it to the reference itself).

Tolerances (normwise max|got - ref| / max|ref|):
  fp32 mix  1e-4  
  fp16 mix  the spectrum and the 1x1 mix weights are rounded to fp16 (11-bit significand, unit
            roundoff 2^-11 = 4.9e-4) and accumulated in fp32; SURVEY.md §7 measured a simulated fp16
            mix at 4.2e-4 normwise for one FU.  Gates: 2e-3 for one Fourier unit, 1e-2 for the whole
            fgan128 stack (five spectral layers, BN renormalising in between).
  fp16 range: the rebuilt spectrum must stay below 65504; with running statistics that do not match
  the activations (random ones) eval-mode activations can grow past it, so the eval test uses the
  running statistics of a warm-up batch, as a trained model has.
"""
import contextlib
import io

import pytest
import torch
import torch.nn as nn

from oracle.ffc_oracle import fgan128_generator, fourier_unit, normwise_err, sn_materialize

pytestmark = pytest.mark.gpu
TOL = 1e-4
TOL_FP16_FU = 2e-3
TOL_FP16_STACK = 1e-2


def _randomize(mod, gen):
    with torch.no_grad():
        for k, v in mod.state_dict().items():
            if not v.is_floating_point():
                continue
            if k.endswith("running_var"):
                v.copy_(0.5 + torch.rand(v.shape, generator=gen))
            elif k.endswith(("running_mean", "bias")):
                v.copy_(0.1 * torch.randn(v.shape, generator=gen))
            elif k.endswith(("weight_u", "weight_v")):
                v.copy_(nn.functional.normalize(torch.randn(v.shape, generator=gen), dim=0))
            elif v.dim() == 1:
                v.copy_(1 + 0.1 * torch.randn(v.shape, generator=gen))
            else:
                v.copy_(torch.randn(v.shape, generator=gen) / max(1, v[0].numel()) ** 0.5)
    return mod


def _sd64(mod):
    return {k: (v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu().clone())
            for k, v in mod.state_dict().items()}


def _sn_dims(model):
    return {name: 1 for name, m in model.named_modules() if isinstance(m, nn.ConvTranspose2d)}


@pytest.mark.parametrize("c,n,up", [(32, 128, 1), (32, 64, 1), (16, 32, 1), (64, 64, 1), (64, 16, 1)])
@pytest.mark.parametrize("train", [True, False])
def test_fp16_mix_fourier_unit(c, n, up, train):
    import fastfourierconvolution_amd as F
    gen = torch.Generator().manual_seed(c + n)
    fu = _randomize(F.FourierUnitSN(c, c), gen)
    sd = _sd64(fu)
    fu = fu.cuda().train(train)
    fu.mix_precision = "fp16"
    x = torch.randn((2, c, n, n), generator=gen)
    with torch.no_grad():
        got = fu(x.cuda()).cpu()
        ref = fourier_unit(x.double(), sd, "", train)
    err = normwise_err(got, ref)
    assert err <= TOL_FP16_FU, err
    assert err > 1e-7   # the fp16 path really ran (exact fp32 would be ~1e-6)


@pytest.mark.parametrize("cin,cout,n_in", [(64, 64, 64), (64, 64, 32), (256, 128, 8), (128, 64, 16)])
def test_fp16_mix_spectral_transform(cin, cout, n_in):
    """SpectralTransform(stride 2, upsample) with the fp16 mix: the upsample-in-the-spectrum path"""
    import fastfourierconvolution_amd as F
    from oracle.ffc_oracle import spectral_transform
    gen = torch.Generator().manual_seed(cin + n_in)
    st = _randomize(F.SpectralTransform(cin, cout, stride=2, upsample=True), gen)
    sd = _sd64(st)
    st = F.set_mix_precision(st.cuda().eval(), "fp16")
    x = torch.randn((2, cin, n_in, n_in), generator=gen)
    with torch.no_grad():
        got = st(x.cuda()).cpu()
        ref = spectral_transform(x.double(), sd, "", 2, True, False)
    err = normwise_err(got, ref)
    assert err <= TOL_FP16_FU, err


def test_fp16_mix_rejects_unsupported():
    import fastfourierconvolution_amd as F
    fu = F.FourierUnitSN(5, 5).cuda()
    fu.mix_precision = "fp16"
    with pytest.raises(NotImplementedError):
        fu(torch.randn(1, 5, 64, 64, device="cuda"))


def _sn_fgan(seed=31):
    import fastfourierconvolution_amd as F
    with contextlib.redirect_stdout(io.StringIO()):
        g = F.spectral_norm_ffc(F.FGenerator(128))
    return _randomize(g, torch.Generator().manual_seed(seed))


@pytest.mark.parametrize("mix", ["fp32", "fp16"])
@pytest.mark.parametrize("train", [False, True])
def test_sn_fgan128_vs_oracle(mix, train):
    """BASELINE config 5 stack: fgan128 with spectral norm on l2l / l2g / g2l and the SpectralTransform
    conv1 / conv2 (what SNFFC / SNFFCTranspose apply), fp32 or fp16 spectral mix"""
    import fastfourierconvolution_amd as F
    g = _sn_fgan()
    dims = _sn_dims(g)
    gen = torch.Generator().manual_seed(8)
    B = 3
    if not train:
        # eval with running statistics of a warm-up batch (a trained model's): random running stats let
        # the eval activations grow layer over layer past fp16's range (65504) in the spectrum
        g = g.cuda()
        for m in g.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.momentum = 1.0
        with torch.no_grad():
            g.train().forward_float(torch.randn((8, 128), generator=gen).cuda())
        for m in g.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.momentum = 0.1
    sd = _sd64(g)
    g = F.set_mix_precision(g.cuda().train(train), mix)
    z = torch.randn((B, 128), generator=gen)
    noises = [(torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen),
               torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen)) for n in (2, 3, 4, 5, 6)]
    with torch.no_grad():
        got = g.forward_float(z.cuda(), [(a.cuda(), b.cuda()) for a, b in noises] if train else None).cpu()
        sn_materialize(sd, dims, train)
        ref = fgan128_generator(z.double(), sd, train, [(a.double(), b.double()) for a, b in noises])
    err = normwise_err(got, ref)
    assert err <= (TOL if mix == "fp32" else TOL_FP16_STACK), err
    if train:   # the power iteration updated u / v like torch's hook on the CPU
        after = g.state_dict()
        for k in [k for k in sd if k.endswith("weight_u")][:6]:
            torch.testing.assert_close(after[k].cpu().double(), sd[k], rtol=1e-4, atol=1e-6, msg=k)


def test_sn_graph_capture_repacks_each_step():
    """train-mode spectral norm changes W / sigma every step: a replayed graph must rerun the power
    iteration and repack the weights, matching an eager step from the same state"""
    import fastfourierconvolution_amd as F
    gen = torch.Generator().manual_seed(2)
    with contextlib.redirect_stdout(io.StringIO()):
        blk = _randomize(F.SNFFC(32, 32, 3, 0.5, 0.5, 1, 1), gen).cuda().train()
    x = (torch.randn(2, 16, 16, 16, generator=gen).cuda(), torch.randn(2, 16, 16, 16, generator=gen).cuda())
    with torch.no_grad():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            blk(x)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out_l, out_g = blk(x)
        state = {k: v.clone() for k, v in blk.state_dict().items()}
        g.replay()
        torch.cuda.synchronize()
        rl, rg = out_l.clone(), out_g.clone()
        assert not torch.equal(state["convl2l.weight_u"], blk.convl2l.weight_u)   # power iteration replayed
        blk.load_state_dict(state)
        el, eg = blk(x)
    torch.testing.assert_close(rl, el, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(rg, eg, rtol=1e-6, atol=1e-6)
