"""CPU emulation of the fp32-accurate split-bf16 MFMA products (csrc/convp_kernels.hip split3 /
mfma_split3), bit for bit in numpy:
  * every finite fp32 value with |a| >= 2^-100 (signed, any larger exponent) splits EXACTLY into
    three bf16 pieces hi + mid + lo, each representable in bf16 (low 16 bits of its fp32 pattern
    zero); below that lo may fall into the fp32 subnormal range (an absolute error < 2^-126);
  * the six kept piece products (order <= 2) reproduce a*b to < 2^-21 |a b| per product, and a
    K = 4096 dot product of such products (fp32 accumulation, as the MFMA) stays within fp32
    accumulation error of the fp64 dot product, far inside the path's 1e-4 normwise gate."""
import numpy as np

M16 = np.uint32(0xFFFF0000)


def split3(a):
    """numpy restatement of split3(): truncation split, fp32 subtractions"""
    a = np.asarray(a, dtype=np.float32)
    u = a.view(np.uint32)
    hi = (u & M16).view(np.float32)
    r1 = (a - hi).astype(np.float32)
    mid = (r1.view(np.uint32) & M16).view(np.float32)
    lo = (r1 - mid).astype(np.float32)
    return hi, mid, lo


def _bf16_exact(x):
    return np.all((x.view(np.uint32) & np.uint32(0xFFFF)) == 0)


def _values(n, seed=0):
    rng = np.random.default_rng(seed)
    parts = [rng.standard_normal(n).astype(np.float32),
             (rng.standard_normal(n) * 0.02).astype(np.float32),
             (rng.standard_normal(n) * 1e4).astype(np.float32),
             np.ldexp(rng.uniform(1, 2, n), rng.integers(-120, 120, n)).astype(np.float32),
             rng.integers(0, 2**32 - 1, n, dtype=np.uint64).astype(np.uint32).view(np.float32)]
    v = np.concatenate(parts)
    return v[np.isfinite(v) & (np.abs(v) < 1e30) & (np.abs(v) >= 2.0 ** -100)]


def test_split_is_exact():
    a = _values(200_000)
    hi, mid, lo = split3(a)
    for p in (hi, mid, lo):
        assert _bf16_exact(p)
    recon = hi.astype(np.float64) + mid.astype(np.float64) + lo.astype(np.float64)
    np.testing.assert_array_equal(recon, a.astype(np.float64))


def test_six_products_error_bound():
    a, b = _values(50_000, 1), _values(50_000, 2)
    n = min(a.size, b.size)
    a, b = a[:n], b[:n]
    ok = (np.abs(a.astype(np.float64) * b) < 1e30) & (np.abs(a.astype(np.float64) * b) > 1e-30)
    a, b = a[ok], b[ok]
    ah, am, al = (x.astype(np.float64) for x in split3(a))
    bh, bm, bl = (x.astype(np.float64) for x in split3(b))
    kept = al * bh + ah * bl + am * bm + am * bh + ah * bm + ah * bh
    exact = a.astype(np.float64) * b.astype(np.float64)
    rel = np.abs(kept - exact) / np.abs(exact)
    assert rel.max() < 2.0 ** -21


def test_dot_product_matches_fp64():
    rng = np.random.default_rng(3)
    K = 4096
    w = (rng.standard_normal((32, K)) * 0.02).astype(np.float32)
    x = rng.standard_normal((K, 64)).astype(np.float32)
    wh, wm, wl = split3(w)
    xh, xm, xl = split3(x)
    acc = np.zeros((32, 64), np.float32)
    for pa, pb in ((wl, xh), (wh, xl), (wm, xm), (wm, xh), (wh, xm), (wh, xh)):   # mfma_split3 order
        acc = (acc + (pa.astype(np.float64) @ pb.astype(np.float64)).astype(np.float32)).astype(np.float32)
    ref = w.astype(np.float64) @ x.astype(np.float64)
    err = np.abs(acc - ref).max() / np.abs(ref).max()
    assert err < 1e-6
