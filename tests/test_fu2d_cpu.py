"""CPU emulation of the large-plane Fourier unit's index math (csrc/fu2d_kernels.hip).

Each check restates one kernel step in numpy with the kernel's own index arithmetic and compares
it with numpy's FFT (which agrees with the reference's torch.fft semantics):
  - the N = N1*N2 line FFT split over N1 lanes (stage_a / stage_b / line_fft),
  - r2c's row-pair packing z = a + i b and the half-spectrum separation,
  - c2r's Hermitian extension (Im of bins 0 and W/2 dropped) and row-pair synthesis,
  - the mix stage's rebuild of rfftn(ortho) of the x2 nearest-upsampled plane from the 4x
    smaller T through X = T[kh mod h][kw mod w] (1 + W_H^kh)(1 + W_W^kw) / sqrt(HW).
"""
import numpy as np
import pytest


def split(n):
    n1 = 8 if n >= 64 else (4 if n >= 16 else 2)
    return n1, n // n1


def line_fft(x, inv=False):
    """stage_a + stage_b + natural-order write, lane by lane"""
    n = x.shape[0]
    n1, n2 = split(n)
    sign = 1.0 if inv else -1.0
    line = x.astype(np.complex128).copy()
    # stage A: lane jj transforms x[jj + n1*m] over m, twiddles W_N^{jj*k2}, writes at jj + n1*k2
    stage = np.empty_like(line)
    for jj in range(n1):
        v = line[jj + n1 * np.arange(n2)]
        f = np.fft.ifft(v) * n2 if inv else np.fft.fft(v)
        f = f * np.exp(sign * 2j * np.pi * jj * np.arange(n2) / n)
        stage[jj + n1 * np.arange(n2)] = f
    # stage B: k2 column = stage[n1' + n1*k2], transform over n1', output index k2 + n2*k1
    out = np.empty_like(line)
    for k2 in range(n2):
        v = stage[np.arange(n1) + n1 * k2]
        f = np.fft.ifft(v) * n1 if inv else np.fft.fft(v)
        out[k2 + n2 * np.arange(n1)] = f
    return out


@pytest.mark.parametrize("n", [8, 16, 32, 64, 128])
@pytest.mark.parametrize("inv", [False, True])
def test_line_fft_split(n, inv):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    want = np.fft.ifft(x) * n if inv else np.fft.fft(x)
    np.testing.assert_allclose(line_fft(x, inv), want, rtol=1e-12, atol=1e-12)


def r2c_plane(s):
    """fu2d_r2c_kernel: row pairs packed as a + i b, separated into two half spectra, then columns"""
    h, w = s.shape
    wpt = w // 2 + 1
    Z = np.empty((h, wpt), np.complex128)
    k = np.arange(wpt)
    for g in range(h // 2):
        z = line_fft(s[2 * g] + 1j * s[2 * g + 1])
        zk, zm = z[k & (w - 1)], z[(w - k) & (w - 1)]
        Z[2 * g] = 0.5 * (zk.real + zm.real) + 0.5j * (zk.imag - zm.imag)
        Z[2 * g + 1] = 0.5 * (zk.imag + zm.imag) - 0.5j * (zk.real - zm.real)
    for c in range(wpt):
        Z[:, c] = line_fft(Z[:, c])
    return Z


@pytest.mark.parametrize("n", [16, 32, 64, 128])
def test_r2c_plane(n):
    s = np.random.default_rng(1).standard_normal((n, n))
    np.testing.assert_allclose(r2c_plane(s), np.fft.rfft2(s), rtol=1e-10, atol=1e-9)


def c2r_plane(Y):
    """fu2d_c2r_kernel: inverse columns, then row pairs z = A_ext + i B_ext -> inverse FFT"""
    H, WP = Y.shape
    W = 2 * (WP - 1)
    Z = Y.astype(np.complex128).copy()
    for c in range(WP):
        Z[:, c] = line_fft(Z[:, c], inv=True)
    out = np.empty((H, W))
    for g in range(H // 2):
        A, B = Z[2 * g].copy(), Z[2 * g + 1].copy()
        A[0] = A[0].real
        A[W // 2] = A[W // 2].real
        B[0] = B[0].real
        B[W // 2] = B[W // 2].real
        Ae = np.array([A[k] if k <= W // 2 else np.conj(A[W - k]) for k in range(W)])
        Be = np.array([B[k] if k <= W // 2 else np.conj(B[W - k]) for k in range(W)])
        z = line_fft(Ae + 1j * Be, inv=True)
        out[2 * g], out[2 * g + 1] = z.real, z.imag
    return out / (H * W)


@pytest.mark.parametrize("n", [32, 64, 128])
def test_c2r_plane_non_hermitian(n):
    """torch irfftn semantics on a non-Hermitian half spectrum (SURVEY.md §7 'Hard parts')"""
    rng = np.random.default_rng(2)
    Y = rng.standard_normal((n, n // 2 + 1)) + 1j * rng.standard_normal((n, n // 2 + 1))
    want = np.fft.irfft(np.fft.ifft(Y, axis=0), n=n, axis=1)
    np.testing.assert_allclose(c2r_plane(Y), want, rtol=1e-10, atol=1e-12)


def mix_rebuild(T, H, W, up):
    """fu2d_mix_kernel's per-bin source index / conjugation / factor"""
    h, w = H // up, W // up
    WP = W // 2 + 1
    X = np.empty((H, WP), np.complex128)
    for kh in range(H):
        for kw in range(WP):
            if up == 1:
                v = T[kh, kw]
                f = 1.0
            else:
                khp, kwp = kh & (h - 1), kw & (w - 1)
                v = T[khp, kwp] if kwp <= w // 2 else np.conj(T[(h - khp) & (h - 1), w - kwp])
                f = (1 + np.exp(-2j * np.pi * kh / H)) * (1 + np.exp(-2j * np.pi * kw / W))
            X[kh, kw] = v * f / np.sqrt(H * W)
    return X


@pytest.mark.parametrize("n,up", [(32, 2), (64, 2), (128, 2), (64, 1)])
def test_upsample_identity(n, up):
    t = np.random.default_rng(3).standard_normal((n // up, n // up))
    s = np.repeat(np.repeat(t, up, 0), up, 1)
    np.testing.assert_allclose(mix_rebuild(np.fft.rfft2(t), n, n, up), np.fft.rfft2(s, norm="ortho"),
                               rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("H", [16, 32, 64, 128])
def test_c2r_packed_dc_nyquist_columns(H):
    """fu2d_c2r_kernel step 2: columns 0 and W/2 (whose Im the row C2R drops after the column IFFT) run
    as ONE complex IFFT of z = a_h + i b_h, a_h[k] = (a[k] + conj(a[-k])) / 2 -- numpy emulation
    against irfftn(Y, s=(H, W)) (torch's C2R semantics ignore Im of bins 0 and W/2)"""
    W = H
    rng = np.random.default_rng(H)
    Y = rng.standard_normal((H, W // 2 + 1)) + 1j * rng.standard_normal((H, W // 2 + 1))
    cols = np.fft.ifft(Y, axis=0) * H                      # unnormalised inverse column FFT
    a, b = Y[:, 0], Y[:, W // 2]
    neg = (-np.arange(H)) % H
    z = 0.5 * (a + np.conj(a[neg])) + 1j * 0.5 * (b + np.conj(b[neg]))
    zc = np.fft.ifft(z) * H
    cols[:, 0] = zc.real
    cols[:, W // 2] = zc.imag                                # only the Re parts are used below
    rows = np.fft.irfft(cols.real * (np.arange(W // 2 + 1) % (W // 2) == 0) + cols * (np.arange(W // 2 + 1) % (W // 2) != 0),
                        n=W, axis=1) * W
    ref = np.fft.irfftn(Y, s=(H, W)) * H * W
    np.testing.assert_allclose(rows, ref, rtol=0, atol=1e-9 * np.abs(ref).max())

