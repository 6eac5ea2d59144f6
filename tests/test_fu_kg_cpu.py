"""CPU emulation of the round-6 fused-FU pieces (csrc/fft_common.h rfft_reg / irfft_reg,
csrc/fu_kernels.hip fu_pass0_kg_kernel's bin-group spill layout and fu_spill_bin), in numpy.

The real-input row transforms of FourierUnitSN.forward (rfftn / irfftn, /root/reference/layers/ffc/
fourier_unity.py:38,56) run on ONE N/2-point complex FFT; the kernels' arithmetic is restated here
step for step and checked against numpy's FFT (parity of the formulas; the GPU tests check the
kernels against the fp64 oracle)."""
import numpy as np
import pytest

TW = np.arange(128) * 2 * np.pi / 128
TWC, TWS = np.cos(TW), np.sin(TW)


def rfft_split(x):
    """fft_common.h rfft_reg<N>"""
    N = x.shape[-1]
    M = N // 2
    Z = np.fft.fft(x[..., 0::2] + 1j * x[..., 1::2])   # fft_reg<M, false>
    zr, zi = Z.real, Z.imag
    Xr = np.zeros(x.shape[:-1] + (M + 1,))
    Xi = np.zeros_like(Xr)
    Xr[..., 0] = zr[..., 0] + zi[..., 0]
    Xr[..., M] = zr[..., 0] - zi[..., 0]
    for k in range(1, M):
        ar, ai, br, bi = zr[..., k], zi[..., k], zr[..., M - k], zi[..., M - k]
        er, ei = 0.5 * (ar + br), 0.5 * (ai - bi)
        orr, oi = 0.5 * (ai + bi), 0.5 * (br - ar)
        if 4 * k == N:
            Xr[..., k], Xi[..., k] = er + oi, ei - orr
        else:
            c, s = TWC[k * (128 // N)], TWS[k * (128 // N)]
            Xr[..., k], Xi[..., k] = er + (orr * c + oi * s), ei + (oi * c - orr * s)
    return Xr, Xi


def irfft_split(Xr, Xi):
    """fft_common.h irfft_reg<N> (unnormalised; Im of bins 0 and N/2 ignored)"""
    M = Xr.shape[-1] - 1
    N = 2 * M
    zr = np.zeros(Xr.shape[:-1] + (M,))
    zi = np.zeros_like(zr)
    zr[..., 0] = Xr[..., 0] + Xr[..., M]
    zi[..., 0] = Xr[..., 0] - Xr[..., M]
    for k in range(1, M):
        ar, ai, br, bi = Xr[..., k], Xi[..., k], Xr[..., M - k], Xi[..., M - k]
        sr, si = ar + br, ai - bi
        dr, di = ar - br, ai + bi
        if 4 * k == N:
            tr, ti = -di, dr
        else:
            c, s = TWC[k * (128 // N)], TWS[k * (128 // N)]
            tr, ti = dr * c - di * s, dr * s + di * c
        zr[..., k], zi[..., k] = sr - ti, si + tr
    z = np.fft.ifft(zr + 1j * zi) * M                  # fft_reg<M, true>: unnormalised
    x = np.zeros(Xr.shape[:-1] + (N,))
    x[..., 0::2], x[..., 1::2] = z.real, z.imag
    return x


@pytest.mark.parametrize("N", [4, 8, 16, 32, 64, 128])
def test_rfft_split_matches_rfft(N):
    rng = np.random.default_rng(N)
    x = rng.standard_normal((7, N))
    Xr, Xi = rfft_split(x)
    ref = np.fft.rfft(x)
    np.testing.assert_allclose(Xr + 1j * Xi, ref, rtol=0, atol=1e-12 * N)


@pytest.mark.parametrize("N", [4, 8, 16, 32, 64, 128])
def test_irfft_split_matches_c2r(N):
    """irfftn's C2R over W as the reference runs it: the Im of bins 0 and W/2 dropped, the rest of a
    non-Hermitian row taken as given"""
    rng = np.random.default_rng(100 + N)
    M = N // 2
    X = rng.standard_normal((5, M + 1)) + 1j * rng.standard_normal((5, M + 1))
    x = irfft_split(X.real, X.imag)
    ref = np.fft.irfft(X, n=N) * N
    np.testing.assert_allclose(x, ref, rtol=0, atol=1e-12 * N)


def spill_bin(m, H, W, G):
    """fu_kernels.hip fu_spill_bin<H, W, G>"""
    WP = W // 2 + 1
    KW0 = -(-WP // G)
    KWL = WP - (G - 1) * KW0
    ZPL = H * KW0
    g = min(m // ZPL, G - 1)
    rem = m - g * ZPL
    kwg = KW0 if g < G - 1 else KWL
    y, kk = rem // kwg, rem % kwg
    return y * WP + g * KW0 + kk


@pytest.mark.parametrize("HW", [8, 16, 32])
def test_bin_group_spill_layout_is_a_permutation(HW):
    """pass 0's group GI writes bin (y, K0 + kk) at GI * ZPL + y * KW + kk; pass 1's decode maps it
    back to y * WP + K0 + kk, and every bin of the channel is written exactly once"""
    H = W = HW
    G = 2
    WP = W // 2 + 1
    KW0 = -(-WP // G)
    ZPL = H * KW0
    seen = {}
    for GI in range(G):
        K0 = GI * KW0
        KW = KW0 if GI < G - 1 else WP - (G - 1) * KW0
        assert KW >= 1
        for y in range(H):
            for kk in range(KW):
                m = GI * ZPL + y * KW + kk
                assert m not in seen
                seen[m] = y * WP + K0 + kk
    assert sorted(seen) == list(range(H * WP))
    for m, n in seen.items():
        assert spill_bin(m, H, W, G) == n
