"""CPU checks of the training path's host logic and kernel math (no GPU):
  * every conv / convT of the config-3 generator and discriminator has an adjoint segment that
    the implicit-GEMM planner accepts and that returns to the input size (data gradients run on
    the forward conv kernels);
  * a numpy emulation of ffc_rfft2_planes / ffc_irfft2_planes (csrc/train_kernels.hip index math:
    twiddle tables, interior-bin weights, Re/Im interleave) equals rfftn / irfftn(ortho), and the
    scaled variants are exact adjoints of each other (SURVEY.md §8a FFT adjoints)."""
import numpy as np
import pytest

from fastfourierconvolution_amd import _plan
from fastfourierconvolution_amd._autograd import adjoint_seg, wgrad_splits


def _layers():
    """(kind, C_in, IH, k, s, p, C_out) of every local conv in FFCGenerator(100, 3, 64) and
    FFCDiscriminator(3, 64) (models/ffc_generator.py:24-28, models/ffc_discriminator.py:26-31)"""
    g = [("convT", 100, 1, 4, 1, 0, 256), ("convT", 256, 4, 4, 2, 1, 128), ("convT", 128, 8, 4, 2, 1, 64),
         ("convT", 64, 16, 4, 2, 1, 32), ("convT", 32, 32, 4, 2, 1, 3)]
    d = [("conv", 3, 64, 4, 2, 1, 64), ("conv", 64, 32, 4, 2, 1, 128), ("conv", 128, 16, 4, 2, 1, 256),
         ("conv", 256, 8, 4, 2, 1, 512), ("conv", 512, 4, 4, 1, 0, 1)]
    return g + d


@pytest.mark.parametrize("layer", _layers())
def test_adjoint_segments_plan(layer):
    kind, C, IH, k, s, p, M = layer
    sg = _plan.Seg(kind, C, IH, IH, k, s, p)
    OH, OW = _plan.seg_out(sg)
    adj = adjoint_seg(sg, M, OH, OW)
    assert _plan.seg_out(adj) == (IH, IH)
    # x_l receives both convl2l and convl2g gradients: one two-segment job
    plan = _plan.plan_job(256, C, (adj, adjoint_seg(sg, M // 2 or 1, OH, OW)))
    assert (plan.OH, plan.OW) == (IH, IH)


def test_pw_adjoint():
    sg = _plan.Seg("pw", 64, 8, 5)
    adj = adjoint_seg(sg, 128, 8, 5)
    assert adj == _plan.Seg("pw", 128, 8, 5)


def test_wgrad_splits_bounded():
    for B in (1, 2, 8, 256):
        for Mu, NT, P in ((128, 1024, 16), (3, 512, 1024), (512, 512, 12), (16, 256, 1)):
            S = wgrad_splits(B, Mu, NT, P)
            K = B * P
            assert 1 <= S <= min(1024, max(1, K // 64)) and S * Mu * NT <= max(Mu * NT, 32 << 20)


def _tw(N):
    j = np.arange(N)
    return np.exp(-2j * np.pi * j / N)


def _interior(W):
    kw = np.arange(W // 2 + 1)
    return (kw != 0) & (2 * kw != W)


def emu_rfft2(x, iscale):
    """csrc/train_kernels.hip rfft2_kernel: row DFT via tw[(kw*w) mod W], column DFT, ortho scale"""
    P, H, W = x.shape
    Wp = W // 2 + 1
    twW, twH = _tw(W), _tw(H)
    R = np.einsum("phw,kw->phk", x, twW[(np.arange(Wp)[:, None] * np.arange(W)[None, :]) % W])
    X = np.einsum("phk,qh->pqk", R, twH[(np.arange(H)[:, None] * np.arange(H)[None, :]) % H])
    X = X / np.sqrt(H * W) * np.where(_interior(W), iscale, 1.0)
    Z = np.empty((2 * P, H, Wp))
    Z[0::2], Z[1::2] = X.real, X.imag
    return Z


def emu_irfft2(Z, H, W, iscale):
    """irfft2_kernel: conj column DFT, interior weight 2*iscale, C2R row sum of Re(v * conj(t))"""
    X = Z[0::2] + 1j * Z[1::2]
    Wp = W // 2 + 1
    twW, twH = _tw(W), _tw(H)
    R = np.einsum("pqk,hq->phk", X, np.conj(twH[(np.arange(H)[:, None] * np.arange(H)[None, :]) % H]))
    R = R * np.where(_interior(W), 2 * iscale, 1.0)
    T = twW[(np.arange(Wp)[None, :] * np.arange(W)[:, None]) % W]      # [w][kw]
    y = (R.real[:, :, None, :] * T.real[None, None] + R.imag[:, :, None, :] * T.imag[None, None]).sum(-1)
    return y / np.sqrt(H * W)


@pytest.mark.parametrize("H,W", [(4, 4), (8, 8), (16, 16), (32, 32), (8, 16), (5, 6)])
def test_dft_emulation_matches_numpy_and_adjoints(H, W):
    rng = np.random.default_rng(H * 100 + W)
    x = rng.standard_normal((3, H, W))
    Z = emu_rfft2(x, 1.0)
    X = np.fft.rfftn(x, axes=(-2, -1), norm="ortho")
    np.testing.assert_allclose(Z[0::2] + 1j * Z[1::2], X, atol=1e-12)
    Zr = rng.standard_normal(Z.shape)            # non-Hermitian spectra are normal in the FU
    y = emu_irfft2(Zr, H, W, 1.0)
    np.testing.assert_allclose(y, np.fft.irfftn(Zr[0::2] + 1j * Zr[1::2], s=(H, W), axes=(-2, -1), norm="ortho"),
                               atol=1e-12)
    # <irfft(Zr), v> == <Zr, rfft_x2(v)>  and  <rfft(x), Zr> == <x, irfft_x0.5(Zr)>
    v = rng.standard_normal(y.shape)
    assert np.isclose((y * v).sum(), (Zr * emu_rfft2(v, 2.0)).sum())
    assert np.isclose((Z * Zr).sum(), (x * emu_irfft2(Zr, H, W, 0.5)).sum())
