"""BN folded into its consumer (ffc_bn_fold, csrc/bn_common.h) and the fused FU's pass 1 fed from
pass 0's spilled mix output (ffc_fu_forward_ex yspill) against the separate reduce/finalize launch
and the recompute: SpectralTransform (layers/ffc/spectral_transform.py:79-108 with
FourierUnitSN, fourier_unity.py:32-56) in train mode on the fused per-sample FU path, momentum
0.1 and None (cumulative average), several steps (running statistics, num_batches_tracked).
Outputs within 1e-6 normwise (the folded merge order differs from bn_reduce_finalize's only in
fp64 rounding); buffers within 1e-6; num_batches_tracked exact; the default path bitwise
deterministic."""
import contextlib
import copy
import io

import pytest
import torch

from oracle.ffc_oracle import normwise_err

pytestmark = pytest.mark.gpu


def _st(cin, cout, momentum, seed):
    import fastfourierconvolution_amd as F
    torch.manual_seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        st = F.SpectralTransform(cin, cout, stride=2, upsample=True)
    for m in st.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.momentum = momentum
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    return st.cuda().train()


def _run(st, xs, fold, spill):
    from fastfourierconvolution_amd import _runtime as rt
    old = rt.BN_FOLD, rt.FU_SPILL, rt.FU_PATH
    rt.BN_FOLD, rt.FU_SPILL, rt.FU_PATH = fold, spill, "fused"
    try:
        with torch.no_grad():
            outs = [st(x).clone() for x in xs]
        torch.cuda.synchronize()
    finally:
        rt.BN_FOLD, rt.FU_SPILL, rt.FU_PATH = old
    return outs, {k: v.detach().clone() for k, v in st.state_dict().items()}


@pytest.mark.parametrize("momentum", [0.1, None])
@pytest.mark.parametrize("cin,cout,hw,B", [(64, 64, 4, 12), (32, 32, 8, 5), (16, 16, 16, 3)])
def test_fold_and_spill_match_separate_launches(momentum, cin, cout, hw, B):
    base = _st(cin, cout, momentum, seed=cin + hw)
    g = torch.Generator().manual_seed(hw)
    xs = [torch.randn((B, cin, hw, hw), generator=g).cuda() for _ in range(3)]
    ref_out, ref_sd = _run(copy.deepcopy(base), xs, False, False)
    for fold, spill in [(True, False), (False, True), (True, True)]:
        out, sd = _run(copy.deepcopy(base), xs, fold, spill)
        for a, b in zip(out, ref_out):
            assert normwise_err(a.double().cpu(), b.double().cpu()) <= 1e-6, (fold, spill)
        for k, v in ref_sd.items():
            if k.endswith("num_batches_tracked"):
                assert int(sd[k]) == int(v), (k, fold, spill)
            elif k.endswith("running_mean") or k.endswith("running_var"):
                torch.testing.assert_close(sd[k], v, rtol=1e-6, atol=1e-7, msg=f"{k} {fold} {spill}")


def test_folded_path_deterministic():
    base = _st(32, 32, 0.1, seed=3)
    xs = [torch.randn((9, 32, 8, 8), generator=torch.Generator().manual_seed(2)).cuda()]
    a, sa = _run(copy.deepcopy(base), xs, True, True)
    b, sb = _run(copy.deepcopy(base), xs, True, True)
    assert torch.equal(a[0], b[0])
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def _run_split(st, xs, split):
    from fastfourierconvolution_amd import _runtime as rt
    old = rt.ST_SPLIT, rt.FU_PATH
    rt.ST_SPLIT, rt.FU_PATH = split, "fused"
    try:
        with torch.no_grad():
            outs = [st(x).clone() for x in xs]
        torch.cuda.synchronize()
    finally:
        rt.ST_SPLIT, rt.FU_PATH = old
    return outs, {k: v.detach().clone() for k, v in st.state_dict().items()}


@pytest.mark.parametrize("cin,cout,hw,B", [(64, 128, 4, 8), (32, 32, 8, 5), (16, 16, 16, 3), (64, 32, 16, 32)])
def test_st_prologue_split_matches_one_workgroup_per_sample(cin, cout, hw, B):
    """ffc_st_prologue_ex over several workgroups per sample (each its share of conv1's output
    tiles, B * split slab rows) against one workgroup per sample: the same outputs and BN buffers
    up to the K-split summation order of conv1 (1e-6 normwise)"""
    from fastfourierconvolution_amd import _lib
    h = hw  # upsample=True: no pooling, conv1 on the input plane
    assert _lib.load().ffc_st_prologue_split(B, cin, h, h, 0, cout // 2) > 1
    base = _st(cin, cout, 0.1, seed=cin + hw + B)
    g = torch.Generator().manual_seed(B)
    xs = [torch.randn((B, cin, hw, hw), generator=g).cuda() for _ in range(2)]
    ref_out, ref_sd = _run_split(copy.deepcopy(base), xs, False)
    out, sd = _run_split(copy.deepcopy(base), xs, True)
    for a, b in zip(out, ref_out):
        assert normwise_err(a.double().cpu(), b.double().cpu()) <= 1e-6
    for k, v in ref_sd.items():
        if k.endswith("num_batches_tracked"):
            assert int(sd[k]) == int(v), k
        elif k.endswith("running_mean") or k.endswith("running_var"):
            torch.testing.assert_close(sd[k], v, rtol=1e-6, atol=1e-7, msg=k)


# --------------------------------------------------------------------------- round 5: per-channel folds
def _run_chfold(st, xs, chfold, path):
    from fastfourierconvolution_amd import _runtime as rt
    old = rt.BN_CHFOLD, rt.FU_PATH, rt.FU_SPILL
    rt.BN_CHFOLD, rt.FU_PATH, rt.FU_SPILL = chfold, path, True
    try:
        with torch.no_grad():
            outs = [st(x).clone() for x in xs]
        torch.cuda.synchronize()
    finally:
        rt.BN_CHFOLD, rt.FU_PATH, rt.FU_SPILL = old
    return outs, {k: v.detach().clone() for k, v in st.state_dict().items()}


@pytest.mark.parametrize("momentum", [0.1, None])
@pytest.mark.parametrize("path,cin,cout,hw,B", [("staged", 32, 64, 8, 6), ("staged", 64, 32, 16, 3),
                                                ("fused", 64, 128, 4, 7), ("fused", 32, 64, 8, 5),
                                                ("fused", 16, 32, 16, 4)])
def test_channel_folds_match_separate_launches(momentum, path, cin, cout, hw, B):
    """bn1 folded into the staged r2c (one channel per plane workgroup), the FU's BN into the staged
    c2r (two channels per plane) and into the fused FU's split pass 1 (2 x 64/H channels per wave),
    ffc::bn_fold_channels, against the separate finalize launches (FFC_BN_CHFOLD=0): outputs within
    1e-6 normwise, running statistics within 1e-6, num_batches_tracked exact, over three steps.
    momentum None takes the separate launches (the per-channel leaders cannot read
    num_batches_tracked), and must still agree."""
    from fastfourierconvolution_amd import _runtime as rt
    base = _st(cin, cout, momentum, seed=cin + hw + 1)
    g = torch.Generator().manual_seed(hw + 1)
    xs = [torch.randn((B, cin, hw, hw), generator=g).cuda() for _ in range(3)]
    ref_out, ref_sd = _run_chfold(copy.deepcopy(base), xs, False, path)
    L = rt.lib()
    calls = {"r2c": 0, "c2r": 0}
    o_r2c, o_c2r, o_r2cm = L.ffc_fu2d_r2c_ex, L.ffc_fu2d_c2r_fold, L.ffc_fu2d_r2c_mix

    def r2c(*a):
        calls["r2c"] += a[8] is not None
        return o_r2c(*a)

    def r2cm(*a):   # the R2C inside mix pass 0 (small t planes), fold argument 9
        calls["r2c"] += a[9] is not None
        return o_r2cm(*a)

    def c2r(*a):
        calls["c2r"] += 1
        return o_c2r(*a)
    L.ffc_fu2d_r2c_ex, L.ffc_fu2d_c2r_fold, L.ffc_fu2d_r2c_mix = r2c, c2r, r2cm
    try:
        out, sd = _run_chfold(copy.deepcopy(base), xs, True, path)
    finally:
        L.ffc_fu2d_r2c_ex, L.ffc_fu2d_c2r_fold, L.ffc_fu2d_r2c_mix = o_r2c, o_c2r, o_r2cm
    if path == "staged" and momentum is not None:
        assert calls["r2c"] == 3 and calls["c2r"] == 3, calls
    for a, b in zip(out, ref_out):
        assert normwise_err(a.double().cpu(), b.double().cpu()) <= 1e-6
    for k, v in ref_sd.items():
        if k.endswith("num_batches_tracked"):
            assert int(sd[k]) == int(v) == 3, k
        elif k.endswith("running_mean") or k.endswith("running_var"):
            torch.testing.assert_close(sd[k], v, rtol=1e-6, atol=1e-7, msg=k)
    again, _ = _run_chfold(copy.deepcopy(base), xs, True, path)
    assert all(torch.equal(a, b) for a, b in zip(out, again))   # deterministic


# --------------------------------------------------------------------------- round 5: R2C inside mix pass 0
@pytest.mark.parametrize("chfold", [True, False])
@pytest.mark.parametrize("cin,cout,hw,B", [(32, 64, 8, 6), (64, 64, 16, 3), (32, 32, 8, 5), (16, 32, 16, 4)])
def test_r2c_mix_matches_separate_launches(chfold, cin, cout, hw, B):
    """ffc_fu2d_r2c_mix (bn1 + ReLU + R2C of the sample recomputed in every mix pass-0 workgroup, T
    in LDS) against the separate r2c + mix launches (FFC_FU2D_R2CMIX=0), staged FU, train-mode BN,
    bn1 folded per channel (chfold) or finalized by its own launch: outputs within 1e-6 normwise
    (the FFT order differs), running statistics within 1e-6, num_batches_tracked exact, three steps"""
    from fastfourierconvolution_amd import _runtime as rt
    L = rt.lib()
    C, up = cout // 2, 2
    assert L.ffc_fu2d_r2c_mix_supported(C, hw * up, hw * up, up)
    base = _st(cin, cout, 0.1, seed=cin + hw + B + 7)
    g = torch.Generator().manual_seed(hw + B)
    xs = [torch.randn((B, cin, hw, hw), generator=g).cuda() for _ in range(3)]
    old = rt.FU2D_R2CMIX, rt.BN_CHFOLD
    n = {"fused": 0}
    o = L.ffc_fu2d_r2c_mix

    def spy(*a):
        n["fused"] += 1
        return o(*a)
    try:
        rt.BN_CHFOLD = chfold
        rt.FU2D_R2CMIX = False
        ref_out, ref_sd = _run_chfold(copy.deepcopy(base), xs, chfold, "staged")
        rt.FU2D_R2CMIX = True
        L.ffc_fu2d_r2c_mix = spy
        out, sd = _run_chfold(copy.deepcopy(base), xs, chfold, "staged")
    finally:
        rt.FU2D_R2CMIX, rt.BN_CHFOLD = old
        L.ffc_fu2d_r2c_mix = o
    assert n["fused"] == 3
    for a, b in zip(out, ref_out):
        assert normwise_err(a.double().cpu(), b.double().cpu()) <= 1e-6
    for k, v in ref_sd.items():
        if k.endswith("num_batches_tracked"):
            assert int(sd[k]) == int(v) == 3, k
        elif k.endswith("running_mean") or k.endswith("running_var"):
            torch.testing.assert_close(sd[k], v, rtol=1e-6, atol=1e-7, msg=k)


@pytest.mark.parametrize("path", ["staged", "fused"])
@pytest.mark.parametrize("cin,cout,hw,B", [(64, 32, 16, 32), (64, 32, 16, 64), (64, 32, 16, 86), (128, 64, 8, 32),
                                           (128, 64, 8, 86), (256, 128, 4, 32)])
def test_fu_repeat_bitwise(path, cin, cout, hw, B):
    """both Fourier-unit paths (staged: r2c_mix + c2r; fused: pass 0 + split pass 1) at the
    strong-scaling shard sizes, with the library's default BN folds, twenty fresh train forwards of
    one SpectralTransform on one input: bitwise equal outputs and buffers (a
    per-channel bn1 fold inside ffc_fu2d_r2c_mix corrupted T of whole channels in co-resident
    workgroups; one-run parity checks passed it)"""
    from fastfourierconvolution_amd import _runtime as rt
    torch.manual_seed(cin + hw + B)
    base = _st(cin, cout, 0.1, seed=cin + B)
    x = torch.randn((B, cin, hw, hw), generator=torch.Generator().manual_seed(B)).cuda()
    outs, sds = [], []
    for _ in range(20):
        out, sd = _run_chfold(copy.deepcopy(base), [x], rt.BN_CHFOLD, path)
        outs.append(out[0])
        sds.append(sd)
    bad = [i for i, o in enumerate(outs) if not torch.equal(o, outs[0])]
    assert not bad, f"runs {bad} differ from run 0"
    for sd in sds[1:]:
        for k in sd:
            assert torch.equal(sd[k], sds[0][k]), k


# --------------------------------------------------------------------------- round 6: bin groups
def _run_kg(st, xs, kg):
    from fastfourierconvolution_amd import _runtime as rt
    old = rt.FU_KGROUPS, rt.FU_PATH
    rt.FU_KGROUPS, rt.FU_PATH = kg, "fused"
    try:
        with torch.no_grad():
            outs = [st(x).clone() for x in xs]
        torch.cuda.synchronize()
    finally:
        rt.FU_KGROUPS, rt.FU_PATH = old
    return outs, {k: v.detach().clone() for k, v in st.state_dict().items()}


@pytest.mark.parametrize("momentum", [0.1, None])
@pytest.mark.parametrize("cin,cout,hw,B", [(256, 128, 4, 64), (128, 64, 8, 86), (64, 32, 16, 256),
                                           (64, 64, 8, 7), (32, 32, 16, 5)])
def test_bin_groups_match_one_workgroup_per_sample(momentum, cin, cout, hw, B):
    """fused FU pass 0 over two bin groups (fu_pass0_kg_kernel: slab rows B x 2, bin-group spill
    layout, real-input row FFTs on N/2-point complex FFTs) against one workgroup per sample:
    SpectralTransform train forwards (gen64 ffc1-ffc3 shapes and odd batches), three steps"""
    from fastfourierconvolution_amd import _runtime as rt
    L = rt.lib()
    base = _st(cin, cout, momentum, seed=cin + hw + B)
    c = cout // 2
    if L.ffc_fu_kgroups(B, c, 2 * hw, 2 * hw) != 2:
        pytest.skip("bin groups off (FFC_FU_KGROUPS=2 turns them on; tests/test_gpu_fu_kg_env.py runs them)")
    g = torch.Generator().manual_seed(hw + B)
    xs = [torch.randn((B, cin, hw, hw), generator=g).cuda() for _ in range(3)]
    ref_out, ref_sd = _run_kg(copy.deepcopy(base), xs, False)
    out, sd = _run_kg(copy.deepcopy(base), xs, True)
    for a, b in zip(out, ref_out):
        err = normwise_err(a.double().cpu(), b.double().cpu())
        assert err <= 2e-6, err
    for k, v in ref_sd.items():
        if k.endswith("num_batches_tracked"):
            assert int(sd[k]) == int(v), k
        elif k.endswith("running_mean") or k.endswith("running_var"):
            torch.testing.assert_close(sd[k], v, rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.parametrize("B", [64, 86, 256])
def test_bin_groups_repeat_bitwise(B):
    """the bin-group path repeated at the strong-scaling shard / full batch sizes: bitwise-equal
    outputs and buffers (no cross-workgroup ordering left to chance)"""
    from fastfourierconvolution_amd import _runtime as rt
    if rt.lib().ffc_fu_kgroups(B, 16, 32, 32) != 2:
        pytest.skip("bin groups off (FFC_FU_KGROUPS=2 turns them on; tests/test_gpu_fu_kg_env.py runs them)")
    base = _st(64, 32, 0.1, seed=B)
    xs = [torch.randn((B, 64, 16, 16), generator=torch.Generator().manual_seed(B)).cuda()]
    first, sd0 = _run_kg(copy.deepcopy(base), xs, True)
    for _ in range(12):
        o, sd = _run_kg(copy.deepcopy(base), xs, True)
        assert torch.equal(o[0], first[0])
        for k in sd0:
            assert torch.equal(sd[k], sd0[k]), k
