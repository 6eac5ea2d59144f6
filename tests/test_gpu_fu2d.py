"""GPU parity of the large-plane Fourier unit (csrc/fu2d_kernels.hip: r2c -> mix -> c2r) against the
fp64 oracle (oracle/ffc_oracle.py restates fourier_unity.py:32-56 / spectral_transform.py:77-110).
Sizes are the fgan128 generator's FU planes (fgan128_complete.py:474-485: c=32 at 64x64 and
128x128 behind a x2 nearest Upsample) at small batches the oracle finishes in seconds.
Tolerance: normwise max|got - ref| / max|ref| <= 1e-4 in fp32."""
import contextlib
import io

import pytest
import torch

from oracle.ffc_oracle import fourier_unit, normwise_err, spectral_transform

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _randomize(mod, gen):
    with torch.no_grad():
        for k, v in mod.state_dict().items():
            if not v.is_floating_point():
                continue
            if k.endswith("running_var"):
                v.copy_(0.5 + torch.rand(v.shape, generator=gen))
            elif k.endswith("running_mean") or k.endswith("bias"):
                v.copy_(0.1 * torch.randn(v.shape, generator=gen))
            elif v.dim() == 1:
                v.copy_(1 + 0.1 * torch.randn(v.shape, generator=gen))
            else:
                v.copy_(torch.randn(v.shape, generator=gen) / max(1, v[0].numel()) ** 0.5)
    return mod


def _sd64(mod):
    return {k: (v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu().clone())
            for k, v in mod.state_dict().items()}


@pytest.mark.parametrize("c,n,B", [(4, 64, 3), (32, 64, 2), (32, 128, 2), (64, 64, 2), (3, 128, 1)])
@pytest.mark.parametrize("train", [True, False])
def test_fu2d_standalone_vs_oracle(c, n, B, train):
    """FourierUnitSN on planes beyond the fused kernel (up = 1 path of the staged FU)"""
    import fastfourierconvolution_amd as F
    gen = torch.Generator().manual_seed(c * 1000 + n)
    fu = _randomize(F.FourierUnitSN(c, c), gen)
    sd = _sd64(fu)
    fu = fu.cuda().train(train)
    x = torch.randn((B, c, n, n), generator=gen)
    with torch.no_grad():
        got = fu(x.cuda()).cpu()
        ref = fourier_unit(x.double(), sd, "", train)
    assert normwise_err(got, ref) <= TOL
    if train:   # running statistics of fu.bn after the forward
        after = fu.state_dict()
        torch.testing.assert_close(after["bn.running_mean"].cpu().double(), sd["bn.running_mean"], rtol=1e-4,
                                   atol=1e-5)
        torch.testing.assert_close(after["bn.running_var"].cpu().double(), sd["bn.running_var"], rtol=1e-4,
                                   atol=1e-5)
        assert int(after["bn.num_batches_tracked"]) == int(sd["bn.num_batches_tracked"])


@pytest.mark.parametrize("n", [32])
def test_fu2d_forced_matches_fused(n):
    """at 32x32 both the fused per-sample FU and the staged FU apply: both match the oracle"""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    gen = torch.Generator().manual_seed(7)
    fu = _randomize(F.FourierUnitSN(16, 16), gen)
    sd = _sd64(fu)
    fu = fu.cuda().eval()
    x = torch.randn((4, 16, n, n), generator=gen)
    with torch.no_grad():
        fused = fu(x.cuda()).cpu()
        rt.FORCE_FU2D = True
        try:
            staged = fu(x.cuda()).cpu()
        finally:
            rt.FORCE_FU2D = False
        ref = fourier_unit(x.double(), sd, "", False)
    assert normwise_err(fused, ref) <= TOL
    assert normwise_err(staged, ref) <= TOL


@pytest.mark.parametrize("cin,cout,n_in,B", [(64, 64, 32, 2), (64, 64, 64, 2), (32, 16, 64, 3)])
@pytest.mark.parametrize("train", [True, False])
def test_st_upsample_large_vs_oracle(cin, cout, n_in, B, train):
    """SpectralTransform(stride=2, upsample=True) whose FU runs at 2*n_in: the x2 nearest upsample is
    applied in the spectrum (mix stage) instead of on the activation"""
    import fastfourierconvolution_amd as F
    gen = torch.Generator().manual_seed(cin + n_in)
    st = _randomize(F.SpectralTransform(cin, cout, stride=2, upsample=True), gen)
    sd = _sd64(st)
    st = st.cuda().train(train)
    x = torch.randn((B, cin, n_in, n_in), generator=gen)
    with torch.no_grad():
        got = st(x.cuda()).cpu()
        ref = spectral_transform(x.double(), sd, "", 2, True, train)
    assert normwise_err(got, ref) <= TOL
    if train:
        after = st.state_dict()
        for k in ("bn1.running_mean", "bn1.running_var", "fu.bn.running_mean", "fu.bn.running_var"):
            torch.testing.assert_close(after[k].cpu().double(), sd[k], rtol=1e-4, atol=1e-5, msg=k)


@pytest.mark.parametrize("c,n,up,train", [(32, 128, 2, True), (32, 64, 2, False), (16, 32, 1, True), (32, 32, 2, False)])
def test_fu2d_column_fused_matches_unfused(c, n, up, train):
    """mix pass 1 with the inverse column FFT fused in + rows-only C2R == the unfused pass 1 + C2R,
    and both match the oracle"""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    from oracle.ffc_oracle import fourier_unit
    gen = torch.Generator().manual_seed(n + c)
    fu = _randomize(F.FourierUnitSN(c, c), gen)
    sd = _sd64(fu)
    fu = fu.cuda().train(train)
    t = torch.randn((2, c, n // up, n // up), generator=gen).cuda()
    outs = []
    for cols in (True, False):
        rt.FU_COLS = cols
        try:
            fu.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in sd.items()})
            with torch.no_grad():
                outs.append(fu._run(t, up=up).cpu())
        finally:
            rt.FU_COLS = True
    s = torch.repeat_interleave(torch.repeat_interleave(t.cpu().double(), up, 2), up, 3)
    ref = fourier_unit(s, sd, "", train)
    assert normwise_err(outs[0], ref) <= TOL and normwise_err(outs[1], ref) <= TOL
    assert normwise_err(outs[0], outs[1]) <= 1e-5


def test_fu2d_deterministic():
    import fastfourierconvolution_amd as F
    gen = torch.Generator().manual_seed(3)
    fu = _randomize(F.FourierUnitSN(32, 32), gen).cuda().train()
    x = torch.randn((2, 32, 128, 128), generator=gen).cuda()
    with torch.no_grad():
        a = fu(x)
        b = fu(x)
    assert torch.equal(a, b)


def test_fu2d_graph_capture():
    """the staged FU is allocation- and sync-free: it captures into a hipGraph and replays"""
    import fastfourierconvolution_amd as F
    gen = torch.Generator().manual_seed(4)
    with contextlib.redirect_stdout(io.StringIO()):
        st = _randomize(F.SpectralTransform(64, 64, stride=2, upsample=True), gen).cuda().eval()
    x = torch.randn((2, 64, 64, 64), generator=gen).cuda()
    with torch.no_grad():
        ref = st(x)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            st(x)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = st(x)
        g.replay()
        torch.cuda.synchronize()
    assert torch.equal(out, ref)


def _fgan_state(seed=21):
    import fastfourierconvolution_amd as F
    with contextlib.redirect_stdout(io.StringIO()):
        g = F.FGenerator(128)
    return _randomize(g, torch.Generator().manual_seed(seed))


@pytest.mark.parametrize("train", [True, False])
def test_fgan128_generator_vs_oracle(train):
    """BASELINE config 4 stack (fgan128_complete.py:442-522) at B=4 against the fp64 oracle, train mode
    with explicit NoiseInjection noise"""
    from oracle.ffc_oracle import fgan128_generator
    g = _fgan_state()
    sd = _sd64(g)
    g = g.cuda().train(train)
    gen = torch.Generator().manual_seed(5)
    B = 4
    z = torch.randn((B, 128), generator=gen)
    noises = [(torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen),
               torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen)) for n in (2, 3, 4, 5, 6)]
    with torch.no_grad():
        got = g.forward_float(z.cuda(), [(a.cuda(), b.cuda()) for a, b in noises] if train else None).cpu()
        ref = fgan128_generator(z.double(), sd, train, [(a.double(), b.double()) for a, b in noises])
    assert got.shape == (B, 3, 128, 128)
    assert normwise_err(got, ref) <= TOL


def test_fgan128_eval_quantization():
    """eval forward returns the uint8 image of fgan128_complete.py:516-521"""
    from oracle.ffc_oracle import quantize_u8
    g = _fgan_state().cuda().eval()
    z = torch.randn((3, 128), generator=torch.Generator().manual_seed(9)).cuda()
    with torch.no_grad():
        fl = g.forward_float(z)
        q = g(z)
    assert q.dtype == torch.uint8 and q.shape == (3, 3, 128, 128)
    assert torch.equal(q.cpu(), quantize_u8(fl.cpu()))


def test_noise_injection_kernel():
    import fastfourierconvolution_amd as F
    ni = F.NoiseInjection(6)
    with torch.no_grad():
        ni.weight.copy_(torch.randn(1, 6, 1, 1))
    ni = ni.cuda()
    x = torch.randn(2, 6, 8, 8, device="cuda")
    n = torch.randn(2, 1, 8, 8, device="cuda")
    torch.testing.assert_close(ni(x, n), x + ni.weight * n, rtol=0, atol=1e-6)


@pytest.mark.parametrize("cin,M,H,W,bias,rin", [(128, 3, 128, 128, False, 0.5), (16, 1, 40, 24, True, 0.0),
                                                 (6, 4, 33, 20, False, 0.5), (64, 3, 96, 72, False, 0.5)])
def test_conv3x3_smallm_head_vs_oracle(cin, M, H, W, bias, rin):
    """FFC_BN_ACT(cin, M, 3, 0.5, 0, 1, 1, Tanh) (the fgan128 head conv7, fgan128_complete.py:484):
    the direct small-M 3x3 kernel, ragged tiles included"""
    import torch.nn as nn
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    from oracle.ffc_oracle import ffc_bn_act
    gen = torch.Generator().manual_seed(cin + H)
    with contextlib.redirect_stdout(io.StringIO()):
        blk = _randomize(F.FFC_BN_ACT(cin, M, 3, rin, 0.0, 1, 1, bias=bias, activation_layer=nn.Tanh), gen)
    sd = _sd64(blk)
    cfg = dict(in_channels=cin, out_channels=M, kernel_size=3, ratio_gin=rin, ratio_gout=0.0, stride=1, padding=1,
               activation_layer="Tanh")
    blk = blk.cuda()
    cg = int(cin * rin)
    xl = torch.randn((2, cin - cg, H, W), generator=gen)
    xg = torch.randn((2, cg, H, W), generator=gen) if cg else None
    obs = rt.LaunchObserver()
    rt.set_observer(obs)
    try:
        with torch.no_grad():
            out, og = blk((xl.cuda(), xg.cuda()) if cg else xl.cuda())
    finally:
        rt.set_observer(None)
    assert og == 0 and "conv3_smallm" in obs.summary()
    ref, _ = ffc_bn_act((xl.double(), xg.double()) if cg else xl.double(), sd, "", cfg, True)
    assert normwise_err(out.cpu(), ref) <= TOL


@pytest.mark.parametrize("H,pool", [(64, False), (64, True), (128, False)])
def test_se_gate_wide_planes(H, pool):
    """SELayer gate on large planes (plane-mean kernel + per-sample FC) vs the oracle's se_layer"""
    import fastfourierconvolution_amd as F
    import torch.nn.functional as Fn
    gen = torch.Generator().manual_seed(H)
    se = _randomize(F.SELayer(64), gen)
    sd = _sd64(se)
    x = torch.randn((3, 64, H, H), generator=gen)
    g = se.cuda().gate(x.cuda(), pool).cpu()
    xr = Fn.avg_pool2d(x.double(), 2) if pool else x.double()
    y = xr.mean(dim=(2, 3))                      # spectral_transform.py:23-28
    ref = torch.sigmoid(Fn.linear(torch.relu(Fn.linear(y, sd["fc.0.weight"])), sd["fc.2.weight"]))
    assert normwise_err(g, ref) <= 1e-5
