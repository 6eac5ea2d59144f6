"""CPU emulation of the cross-lane column DFTs of the fused Fourier unit (csrc/fft_common.h lane_xor,
lane_fft_dif, lane_ifft_dit; used by csrc/fu_kernels.hip fu_kernel and fu_pass1_split_kernel), in numpy.

After the row R2C a lane holds one spectrum row; the column DFT of FourierUnitSN.forward's rfftn /
irfftn (/root/reference/layers/ffc/fourier_unity.py:38,56) runs across the H lanes of a channel with
butterfly partners y ^ D reached by DPP moves and ds_swizzle.  The lane moves are emulated from their
ISA definitions (quad_perm, row_mirror, row_half_mirror, swizzle bit-mask mode) so the composites the
kernel uses for D = 4 and 8 are checked to be the xor partner, and the stage arithmetic (table
twiddles, sign trick, scale folding, bit-reversed rows) is restated step for step against numpy's
FFT.  The GPU tests check the kernels against the fp64 oracle."""
import numpy as np
import pytest

TW = np.arange(128) * 2 * np.pi / 128
TWC, TWS = np.cos(TW), np.sin(TW)
LANES = np.arange(64)


def dpp(v, ctrl):
    """v_mov_b32_dpp on a (..., 64) array of lane values: the value lane i reads"""
    i = LANES
    if ctrl in (0xB1, 0x4E, 0x1B):   # quad_perm
        sel = [(ctrl >> (2 * q)) & 3 for q in range(4)]
        src = (i & ~3) | np.array(sel)[i & 3]
    elif ctrl == 0x141:              # row_half_mirror
        src = (i & ~7) | (7 - (i & 7))
    elif ctrl == 0x140:              # row_mirror
        src = (i & ~15) | (15 - (i & 15))
    else:
        raise ValueError(ctrl)
    return v[..., src]


def swizzle(v, pattern):
    """ds_swizzle_b32 bit-mask mode (offset bit 15 = 0): within groups of 32 lanes"""
    assert pattern & 0x8000 == 0
    and_m, or_m, xor_m = pattern & 0x1F, (pattern >> 5) & 0x1F, (pattern >> 10) & 0x1F
    i = LANES
    src = (i & ~31) | (((i & 31) & and_m | or_m) ^ xor_m)
    return v[..., src]


def lane_xor(v, D):
    """fft_common.h lane_xor<D>"""
    if D == 1:
        return dpp(v, 0xB1)
    if D == 2:
        return dpp(v, 0x4E)
    if D == 4:
        return dpp(dpp(v, 0x141), 0x1B)
    if D == 8:
        return dpp(dpp(v, 0x140), 0x141)
    if D == 16:
        return swizzle(v, 0x401F)
    raise ValueError(D)


def lane_tw(y, D, inv):
    j = y & (D - 1)
    up = (y & D) != 0
    tc, ts = TWC[j * (64 // D)], TWS[j * (64 // D)]
    return np.where(up, tc, 1.0), np.where(up, ts if inv else -ts, 0.0)


def lane_fft_dif(re, im, N, scale):
    """fft_common.h lane_fft_dif<N, K>: re / im (K, 64), lane y % N = row y of its group"""
    y = LANES % N
    D = N // 2
    while D >= 1:
        sg = np.where(y & D, -1.0, 1.0)
        c, s = lane_tw(y, D, False)
        pr, pi = lane_xor(re, D), lane_xor(im, D)
        tr, ti = sg * re + pr, sg * im + pi
        if D == 1:
            re, im = tr * scale, ti * scale
        else:
            re, im = tr * c - ti * s, tr * s + ti * c
        D //= 2
    return re, im


def lane_ifft_dit(re, im, N, scale):
    """fft_common.h lane_ifft_dit<N, K>"""
    y = LANES % N
    D = 1
    while D < N:
        sg = np.where(y & D, -1.0, 1.0)
        c, s = lane_tw(y, D, True)
        if D == 1:
            ur, ui = re * scale, im * scale
        else:
            ur, ui = re * c - im * s, re * s + im * c
        pr, pi = lane_xor(ur, D), lane_xor(ui, D)
        re, im = sg * ur + pr, sg * ui + pi
        D *= 2
    return re, im


def brev(y, N):
    bits = N.bit_length() - 1
    return np.array([int(format(v, f"0{bits}b")[::-1], 2) for v in np.atleast_1d(y)])


@pytest.mark.parametrize("D", [1, 2, 4, 8, 16])
def test_lane_moves_are_xor_partners(D):
    """the DPP composites (FFC_LANE_SWZ=0) and the default ds_swizzle pattern (D << 10) | 0x1F"""
    v = LANES.astype(float)
    assert np.array_equal(lane_xor(v, D), LANES ^ D)
    assert np.array_equal(swizzle(v, (D << 10) | 0x1F), LANES ^ D)


@pytest.mark.parametrize("N", [2, 4, 8, 16, 32])
def test_lane_dif_forward_is_the_column_dft(N):
    """64 // N channels per wave, K = 5 columns; lane y ends with scale * X[bitrev(y)]"""
    rng = np.random.default_rng(N)
    K = 5
    x = rng.standard_normal((K, 64)) + 1j * rng.standard_normal((K, 64))
    scale = 0.125
    re, im = lane_fft_dif(x.real.copy(), x.imag.copy(), N, scale)
    got = re + 1j * im
    want = np.fft.fft(x.reshape(K, 64 // N, N), axis=-1) * scale        # natural order per group
    y = LANES % N
    want_lane = want.reshape(K, 64 // N, N)[:, LANES // N, brev(y, N)]   # X[bitrev(y)] at lane y
    np.testing.assert_allclose(got, want_lane, rtol=0, atol=1e-12 * N)


@pytest.mark.parametrize("N", [2, 4, 8, 16, 32])
def test_lane_dit_inverse_undoes_the_forward(N):
    rng = np.random.default_rng(100 + N)
    K = 3
    X = rng.standard_normal((K, 64)) + 1j * rng.standard_normal((K, 64))   # natural bins per group
    y = LANES % N
    lanes_in = X.reshape(K, 64 // N, N)[:, LANES // N, brev(y, N)]         # lane y reads row bitrev(y)
    re, im = lane_ifft_dit(lanes_in.real.copy(), lanes_in.imag.copy(), N, 0.5)
    want = np.fft.ifft(X.reshape(K, 64 // N, N), axis=-1) * N * 0.5       # unnormalised inverse
    np.testing.assert_allclose(re + 1j * im, want.reshape(K, 64), rtol=0, atol=1e-12 * N)


@pytest.mark.parametrize("H,W", [(8, 8), (16, 16), (32, 32)])
def test_fused_rows_then_lane_columns_is_rfft2_ortho(H, W):
    """pass 0 of fu_kernel on one wave: rows (np.fft.rfft as the row R2C), lane columns, the store
    to row bitrev(y) -- equals rfftn(s, norm='ortho') (fourier_unity.py:38); the inverse path
    (row bitrev(y) in, lane inverse columns, row irfft) restores s (fourier_unity.py:56)"""
    rng = np.random.default_rng(H)
    C = 64 // H
    s = rng.standard_normal((C, H, W))
    rows = np.fft.rfft(s, axis=-1).reshape(C * H, W // 2 + 1).T            # (K, 64): lane = (ch, y)
    norm = 1.0 / np.sqrt(H * W)
    re, im = lane_fft_dif(rows.real.copy(), rows.imag.copy(), H, norm)
    y = LANES % H
    Z = np.zeros((C, H, W // 2 + 1), complex)
    Z[LANES // H, brev(y, H), :] = (re + 1j * im).T
    np.testing.assert_allclose(Z, np.fft.rfftn(s, axes=(-2, -1), norm="ortho"), rtol=0, atol=1e-12)
    lanes_in = Z[LANES // H, brev(y, H), :].T
    re, im = lane_ifft_dit(lanes_in.real.copy(), lanes_in.imag.copy(), H, norm)
    back = np.fft.irfft((re + 1j * im).T, n=W, axis=-1) * W                 # irfft_reg is unnormalised
    np.testing.assert_allclose(back.reshape(C, H, W), s, rtol=0, atol=1e-12)
