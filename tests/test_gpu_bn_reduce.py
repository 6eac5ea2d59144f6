"""BN slab reduction (csrc/bn_se_kernels.hip): the one-block-per-channel merge for small slabs and the
two-level coalesced merge for large ones (>= 1024 rows: 16-channel x row-range partials + a
fixed-order merge) against an fp64 restatement of the merge (raw moments {n, sum, sumsq} of Chan
partials {n, mean, M2}) and nn.BatchNorm2d's finalize (torch/nn/modules/batchnorm.py semantics as
layers/ffc/ffc_bn_act.py uses them)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _slab(nrows, C, gen):
    n = torch.randint(1, 64, (nrows, C), generator=gen).double()
    mean = torch.randn((nrows, C), generator=gen, dtype=torch.float64)
    m2 = torch.rand((nrows, C), generator=gen, dtype=torch.float64) * n
    slab = torch.stack([n, mean, m2, torch.zeros_like(n)], dim=-1).float()
    s64 = slab.double()
    ref = torch.stack([s64[..., 0].sum(0), (s64[..., 0] * s64[..., 1]).sum(0),
                       (s64[..., 2] + s64[..., 0] * s64[..., 1] ** 2).sum(0)], dim=-1)
    return slab, ref


@pytest.mark.parametrize("nrows,C", [(300, 64), (1024, 16), (5000, 72), (16384, 256), (2047, 3)])
def test_bn_reduce_moments(nrows, C):
    from fastfourierconvolution_amd import _lib
    L = _lib.load()
    gen = torch.Generator().manual_seed(nrows + C)
    slab, ref = _slab(nrows, C, gen)
    ws = L.ffc_bn_reduce_ws_doubles(nrows, C)
    assert (ws > 0) == (nrows >= 1024)
    buf = torch.full((3 * C + ws,), float("nan"), dtype=torch.float64, device="cuda")
    rc = L.ffc_bn_reduce(slab.cuda().data_ptr(), nrows, C, buf.data_ptr(), None)
    assert rc == 0, L.ffc_last_error()
    got = buf[:3 * C].view(C, 3).cpu()
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-8)
    # deterministic: a second run gives the same bits
    buf2 = torch.full_like(buf, float("nan"))
    assert L.ffc_bn_reduce(slab.cuda().data_ptr(), nrows, C, buf2.data_ptr(), None) == 0
    assert torch.equal(buf[:3 * C], buf2[:3 * C])


@pytest.mark.parametrize("nrows,C,momentum", [(4096, 64, 0.1), (8192, 128, None), (512, 32, 0.1)])
def test_bn_reduce_finalize_large(nrows, C, momentum):
    """scale / shift and the running-stat update from a large slab vs nn.BatchNorm2d's formulas"""
    from fastfourierconvolution_amd import _lib
    L = _lib.load()
    gen = torch.Generator().manual_seed(7 + nrows)
    slab, ref = _slab(nrows, C, gen)
    gamma = (1 + 0.1 * torch.randn(C, generator=gen)).cuda()
    beta = (0.1 * torch.randn(C, generator=gen)).cuda()
    rm = (0.1 * torch.randn(C, generator=gen)).cuda()
    rv = (0.5 + torch.rand(C, generator=gen)).cuda()
    nbt = torch.tensor(3, dtype=torch.int64, device="cuda")
    rm0, rv0 = rm.clone(), rv.clone()
    scale = torch.empty(C, device="cuda")
    shift = torch.empty(C, device="cuda")
    buf = torch.empty(3 * C + L.ffc_bn_reduce_ws_doubles(nrows, C), dtype=torch.float64, device="cuda")
    mom = -1.0 if momentum is None else momentum
    rc = L.ffc_bn_reduce_finalize(slab.cuda().data_ptr(), nrows, C, buf.data_ptr(), gamma.data_ptr(),
                                  beta.data_ptr(), rm.data_ptr(), rv.data_ptr(), nbt.data_ptr(), 1, mom, 1e-5, 1.0,
                                  scale.data_ptr(), shift.data_ptr(), None)
    assert rc == 0, L.ffc_last_error()
    torch.cuda.synchronize()
    n, s, q = ref[:, 0], ref[:, 1], ref[:, 2]
    mu = s / n
    var = (q / n - mu * mu).clamp_min(0)
    f = 1.0 / 4 if momentum is None else momentum
    sc_ref = gamma.cpu().double() / torch.sqrt(var.float().double() + 1e-5)
    torch.testing.assert_close(scale.cpu().double(), sc_ref, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(shift.cpu().double(), beta.cpu().double() - mu.float().double() * sc_ref,
                               rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rm.cpu().double(), (1 - f) * rm0.cpu().double() + f * mu, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(rv.cpu().double(), (1 - f) * rv0.cpu().double() + f * var * n / (n - 1),
                               rtol=1e-5, atol=1e-6)
    assert int(nbt.item()) == 4


def test_batched_finalize_and_apply_match_single_calls():
    """ffc_bn_reduce_finalize_batch / ffc_bn_act_apply_batch (one launch for a layer's BNs) against the
    single calls, bit for bit: a small slab, a large (two-level) slab and a momentum=None BN; apply
    with and without noise, plus a tensor the plane kernel does not take (HW = 36)"""
    import ctypes
    from fastfourierconvolution_amd import _lib
    L = _lib.load()
    gen = torch.Generator().manual_seed(9)
    specs = [(300, 64, 0.1), (2000, 32, 0.1), (50, 16, None)]
    slabs = [_slab(n, C, gen)[0].cuda() for n, C, _ in specs]

    def params(C):
        return [t.cuda() for t in (1 + 0.1 * torch.randn(C, generator=gen), 0.1 * torch.randn(C, generator=gen),
                                   0.1 * torch.randn(C, generator=gen), 0.5 + torch.rand(C, generator=gen))]
    ps = [params(C) for _, C, _ in specs]
    runs = []
    for batched in (False, True):
        st = [[t.clone() for t in p] + [torch.tensor(2, dtype=torch.int64, device="cuda")] for p in ps]
        out = [(torch.empty(C, device="cuda"), torch.empty(C, device="cuda")) for _, C, _ in specs]
        bufs = [torch.empty(3 * C + L.ffc_bn_reduce_ws_doubles(n, C), dtype=torch.float64, device="cuda")
                for n, C, _ in specs]
        args = [(slabs[i].data_ptr(), n, C, bufs[i].data_ptr(), *(t.data_ptr() for t in st[i]), 1,
                 -1.0 if m is None else m, 1e-5, 1.0, out[i][0].data_ptr(), out[i][1].data_ptr())
                for i, (n, C, m) in enumerate(specs)]
        if batched:
            arr = (_lib.BnRfItem * 3)(*[_lib.BnRfItem(*a) for a in args])
            assert L.ffc_bn_reduce_finalize_batch(arr, 3, None) == 0, L.ffc_last_error()
        else:
            for a in args:
                assert L.ffc_bn_reduce_finalize(*a, None) == 0, L.ffc_last_error()
        torch.cuda.synchronize()
        runs.append((out, st))
    for (s0, h0), (s1, h1) in zip(runs[0][0], runs[1][0]):
        assert torch.equal(s0, s1) and torch.equal(h0, h1)
    for a, b in zip(runs[0][1], runs[1][1]):
        for t0, t1 in zip(a, b):
            assert torch.equal(t0, t1)
    # apply
    xs = [torch.randn((2, 8, 32, 32), generator=gen).cuda(), torch.randn((2, 4, 16, 16), generator=gen).cuda(),
          torch.randn((3, 5, 6, 6), generator=gen).cuda()]
    nzs = [torch.randn((2, 1, 32, 32), generator=gen).cuda(), None, None]
    sc = [torch.rand(x.shape[1], generator=gen).cuda() + 0.5 for x in xs]
    sh = [0.1 * torch.randn(x.shape[1], generator=gen).cuda() for x in xs]
    nw = [torch.randn(x.shape[1], generator=gen).cuda() for x in xs]
    acts = [5, 1, 2]
    ref = [x.clone() for x in xs]
    for i, x in enumerate(ref):
        B, C, H, W = x.shape
        if nzs[i] is not None:
            rc = L.ffc_bn_act_noise_apply(x.data_ptr(), x.data_ptr(), B, C, H * W, sc[i].data_ptr(), sh[i].data_ptr(),
                                          acts[i], 0.1, nw[i].data_ptr(), nzs[i].data_ptr(), None)
        else:
            rc = L.ffc_bn_act_apply(x.data_ptr(), x.data_ptr(), B, C, H * W, sc[i].data_ptr(), sh[i].data_ptr(),
                                    acts[i], 0.1, None)
        assert rc == 0
    got = [x.clone() for x in xs]
    arr = (_lib.BnApplyItem * 3)(*[_lib.BnApplyItem(x.data_ptr(), x.data_ptr(), x.shape[0], x.shape[1],
                                                    x.shape[2] * x.shape[3], sc[i].data_ptr(), sh[i].data_ptr(),
                                                    acts[i], 0.1, nw[i].data_ptr() if nzs[i] is not None else None,
                                                    nzs[i].data_ptr() if nzs[i] is not None else None)
                                   for i, x in enumerate(got)])
    assert L.ffc_bn_act_apply_batch(arr, 3, None) == 0, L.ffc_last_error()
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
