"""CPU checks of the host-side conv planner (fastfourierconvolution_amd/_plan.py).

The GEMM the HIP kernel runs is emulated here with exactly the kernel's index math
(k-table entry -> input coordinate my*mult + off, weight index (ky, kx)) and compared to
torch's CPU conv2d / conv_transpose2d in fp64.  This pins the phase decomposition and
tap tables without a GPU.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from fastfourierconvolution_amd import _plan


def emulate(plan, xs, ws, layouts):
    """out[b, m, oy, ox] via the plan's per-phase GEMMs (float64)."""
    B, M = plan.B, plan.M
    out = torch.zeros((B, M, plan.OH, plan.OW), dtype=torch.float64)
    for pi, ph in enumerate(plan.phases):
        ent = plan.ktab[plan.kt_off[pi]: plan.kt_off[pi] + ph.K]
        K = len(ent)
        A = torch.zeros((M, K), dtype=torch.float64)
        Bm = torch.zeros((K, B, ph.PH, ph.PW), dtype=torch.float64)
        my = torch.arange(ph.PH)[:, None]
        mx = torch.arange(ph.PW)[None, :]
        for k, (sx, oy, ox, kk) in enumerate(ent):
            seg = sx & 15
            if seg == 15:
                continue
            ch = sx >> 4
            ky, kx = kk & 0xFFFF, kk >> 16
            sg = plan.segs[seg]
            w = ws[seg]
            A[:, k] = w[:, ch, ky, kx] if layouts[seg] == 0 else w[ch, :, ky, kx]
            mul_y, mul_x = plan.mults[seg]
            iy = my * mul_y + oy
            ix = mx * mul_x + ox
            valid = (iy >= 0) & (iy < sg.IH) & (ix >= 0) & (ix < sg.IW)
            x = xs[seg]
            if sg.pool:
                x = F.avg_pool2d(x, 2, 2)
            vals = x[:, ch][:, iy.clamp(0, sg.IH - 1), ix.clamp(0, sg.IW - 1)]
            Bm[k] = torch.where(valid[None], vals, torch.zeros(()))
        res = torch.einsum("mk,kbyx->bmyx", A, Bm)
        out[:, :, ph.py::plan.Sy, ph.px::plan.Sx] = res
    return out


def ref_out(sg, x, w):
    if sg.pool:
        x = F.avg_pool2d(x, 2, 2)
    if sg.kind == "convT":
        return F.conv_transpose2d(x, w, None, sg.s, sg.p, sg.op, 1, sg.d)
    if sg.kind == "conv":
        return F.conv2d(x, w, None, sg.s, sg.p, sg.d)
    return F.conv2d(x, w)


def make(sg, B, M, gen):
    H, W = (2 * sg.IH, 2 * sg.IW) if sg.pool else (sg.IH, sg.IW)
    x = torch.randn((B, sg.C, H, W), generator=gen, dtype=torch.float64)
    if sg.kind == "convT":
        w = torch.randn((sg.C, M, sg.k, sg.k), generator=gen, dtype=torch.float64)
        return x, w, 1
    return x, torch.randn((M, sg.C, sg.k, sg.k), generator=gen, dtype=torch.float64), 0


CASES = {
    "convT_k4s2p1": [_plan.Seg("convT", 5, 4, 4, 4, 2, 1)],
    "convT_k4s2p1_two_inputs": [_plan.Seg("convT", 3, 8, 8, 4, 2, 1), _plan.Seg("convT", 4, 8, 8, 4, 2, 1)],
    "convT_plus_pw": [_plan.Seg("convT", 3, 8, 8, 4, 2, 1), _plan.Seg("pw", 2, 16, 16)],
    "convT_1x1_input_ffc0": [_plan.Seg("convT", 7, 1, 1, 4, 1, 0)],
    "convT_k3s2p1_op1": [_plan.Seg("convT", 3, 5, 7, 3, 2, 1, 1, 1)],
    "convT_k4s1p0_dil2": [_plan.Seg("convT", 2, 5, 5, 4, 1, 0, 2)],
    "conv_k4s2p1": [_plan.Seg("conv", 3, 16, 16, 4, 2, 1)],
    "conv_k4s2p1_odd": [_plan.Seg("conv", 3, 9, 11, 4, 2, 1)],
    "conv_k4s1p0_to1x1": [_plan.Seg("conv", 6, 4, 4, 4, 1, 0)],
    "conv_k3s1p1_two_inputs": [_plan.Seg("conv", 4, 8, 8, 3, 1, 1), _plan.Seg("conv", 5, 8, 8, 3, 1, 1)],
    "conv_k3s2p1_dil2": [_plan.Seg("conv", 3, 12, 12, 3, 2, 2, 2)],
    "conv_plus_pw_stride2": [_plan.Seg("conv", 3, 16, 16, 4, 2, 1), _plan.Seg("pw", 5, 8, 8)],
    "pw_pool": [_plan.Seg("pw", 6, 4, 4, pool=True)],
    "three_segments": [_plan.Seg("conv", 2, 6, 6, 3, 1, 1), _plan.Seg("conv", 3, 6, 6, 3, 1, 1),
                       _plan.Seg("pw", 4, 6, 6)],
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_plan_matches_torch(name):
    segs = CASES[name]
    gen = torch.Generator().manual_seed(1)
    B, M = 2, 5
    plan = _plan.plan_job(B, M, segs)
    xs, ws, lays = [], [], []
    ref = 0
    for sg in segs:
        x, w, lay = make(sg, B, M, gen)
        xs.append(x)
        ws.append(w)
        lays.append(lay)
        ref = ref + ref_out(sg, x, w)
    got = emulate(plan, xs, ws, lays)
    assert got.shape == ref.shape
    assert torch.allclose(got, ref, atol=1e-10, rtol=1e-10)
    # every Kpad is a multiple of the k chunk, pads are marked
    for pi, ph in enumerate(plan.phases):
        assert ph.Kpad % _plan.BK == 0 and ph.Kpad >= ph.K
        pads = plan.ktab[plan.kt_off[pi] + ph.K: plan.kt_off[pi] + ph.Kpad]
        assert (pads[:, 0] == 15).all()


def test_generator_layer_plans():
    """FFCGenerator ffc1 shapes: 4 phases, 4 taps per input channel per phase."""
    segs = [_plan.Seg("convT", 256, 4, 4, 4, 2, 1), _plan.Seg("convT", 256, 4, 4, 4, 2, 1)]
    plan = _plan.plan_job(256, 128, segs)
    assert (plan.Sy, plan.Sx) == (2, 2) and len(plan.phases) == 4
    assert all(ph.K == 512 * 4 for ph in plan.phases)
    ffc0 = _plan.plan_job(256, 256, [_plan.Seg("convT", 100, 1, 1, 4, 1, 0)])
    assert len(ffc0.phases) == 16 and all(ph.K == 100 for ph in ffc0.phases)


@pytest.mark.parametrize("n", [1, 7, 8, 9, 63, 64, 100, 257, 1000])
def test_xcd_remap_bijective(n):
    r = _plan.xcd_remap(n)
    assert sorted(r.tolist()) == list(range(n))


@pytest.mark.parametrize("cfg", [0, 1, 2])
def test_tiles_cover_every_output_once(cfg):
    pa = _plan.plan_job(3, 70, [_plan.Seg("convT", 4, 5, 5, 4, 2, 1)])
    pb = _plan.plan_job(3, 33, [_plan.Seg("convT", 4, 5, 5, 4, 2, 1), _plan.Seg("pw", 2, 10, 10)])
    tiles, nslots = _plan.build_tiles([pa, pb], cfg)
    BM, BN, _ = _plan.TILE_CFGS[cfg]
    seen = set()
    for jx, m0, n0, slot in tiles.tolist():
        j, p = jx & 0xFF, jx >> 8
        key = (j, p, m0, n0)
        assert key not in seen
        seen.add(key)
        assert 0 <= slot < nslots[j]
    for j, pl in enumerate((pa, pb)):
        for p, ph in enumerate(pl.phases):
            for n0 in range(0, pl.B * ph.PH * ph.PW, BN):
                for m0 in range(0, pl.M, BM):
                    assert (j, p, m0, n0) in seen
    assert len(seen) == len(tiles)


def test_rejects_mixed_strides():
    with pytest.raises(ValueError):
        _plan.plan_job(1, 4, [_plan.Seg("convT", 2, 4, 4, 4, 2, 1), _plan.Seg("conv", 2, 8, 8, 3, 1, 1)])


def emulate_patch(plan, xs, ws, layouts):
    """the LDS-patch kernel's index math: A from the packing table, B from taptab offsets"""
    B, M = plan.B, plan.M
    out = torch.zeros((B, M, plan.OH, plan.OW), dtype=torch.float64)
    for ph in plan.phases:
        K = ph["Kpad"]
        ent = plan.ktab[ph["kt_off"]: ph["kt_off"] + K]
        A = torch.zeros((M, K), dtype=torch.float64)
        Bm = torch.zeros((K, B, ph["PH"], ph["PW"]), dtype=torch.float64)
        my = torch.arange(ph["PH"])[:, None]
        mx = torch.arange(ph["PW"])[None, :]
        for s, sg in enumerate(plan.segs):
            T = ph["T"][s]
            PR, PC = plan.prc[s]
            mul_y, mul_x = plan.mults[s]
            x = F.avg_pool2d(xs[s], 2, 2) if sg.pool else xs[s]
            for kk in range(plan.cpad[s] * T):
                k = ph["kseg"][s] + kk
                ch, t = divmod(kk, T)
                sx, oy, ox, kyx = ent[k]
                if ch >= sg.C:
                    assert sx == 15
                    continue
                if sx == 15:   # a 3x3 job's zero-weight 4th tap row / column (4x4 taps)
                    assert T == 16 and sg.k == 3
                    continue
                assert sx == (s | (ch << 4))
                tt = plan.taptab[ph["tap_base"][s] + t]
                dy, dx = int(tt) >> 16, int(tt) & 0xFFFF
                if T == 16:   # kernel view: lane half 1 reads taps 8..15 as taps 0..7 shifted by tap_h
                    assert plan.cc[s] == 4 and plan.cpad[s] % 4 == 0
                    if t >= 8:
                        t0 = int(plan.taptab[ph["tap_base"][s] + t - 8])
                        th = ph["tap_h"][s]
                        assert (dy, dx) == ((t0 >> 16) + (th >> 16), (t0 & 0xFFFF) + (th & 0xFFFF))
                else:
                    assert plan.cc[s] == 16 and plan.cpad[s] % 16 == 0
                assert (dy, dx) == (oy - plan.org[s][0], ox - plan.org[s][1])
                # every in-block pixel stays inside the patch, also shifted by the 16-byte row alignment
                PCa = plan.rowlen[s]
                al = plan.org[s][1] % 4 == 0 and (plan.TC * mul_x) % 4 == 0
                xs_max = 3 if plan.vec4[s] and not al else 0
                assert (plan.TR - 1) * mul_y + dy < PR and (plan.TC - 1) * mul_x + dx + xs_max < PCa
                ky, kx = kyx & 0xFFFF, kyx >> 16
                A[:, k] = ws[s][:, ch, ky, kx] if layouts[s] == 0 else ws[s][ch, :, ky, kx]
                iy = my * mul_y + plan.org[s][0] + dy
                ix = mx * mul_x + plan.org[s][1] + dx
                valid = (iy >= 0) & (iy < sg.IH) & (ix >= 0) & (ix < sg.IW)
                vals = x[:, ch][:, iy.clamp(0, sg.IH - 1), ix.clamp(0, sg.IW - 1)]
                Bm[k] = torch.where(valid[None], vals, torch.zeros(()))
        out[:, :, ph["py"]::plan.Sy, ph["px"]::plan.Sx] = torch.einsum("mk,kbyx->bmyx", A, Bm)
    return out


PATCH_CASES = {
    "gen_ffc1_l": [_plan.Seg("convT", 20, 4, 4, 4, 2, 1), _plan.Seg("convT", 18, 4, 4, 4, 2, 1)],
    "gen_ffc2_g": [_plan.Seg("convT", 17, 8, 8, 4, 2, 1), _plan.Seg("pw", 5, 16, 16)],
    "gen_ffc4": [_plan.Seg("convT", 6, 32, 32, 4, 2, 1)],
    "odd_sizes": [_plan.Seg("convT", 3, 5, 7, 4, 2, 1)],
    "conv_k4s1p0": [_plan.Seg("conv", 5, 4, 4, 4, 1, 0)],
    "conv_k4s2p1": [_plan.Seg("conv", 5, 8, 8, 4, 2, 1), _plan.Seg("conv", 3, 8, 8, 4, 2, 1)],
    "conv_k4s2p1_pw": [_plan.Seg("conv", 6, 16, 16, 4, 2, 1), _plan.Seg("pw", 5, 8, 8)],
    "conv_k4s2p1_odd": [_plan.Seg("conv", 3, 9, 7, 4, 2, 1)],
    "conv_k3s1p1": [_plan.Seg("conv", 5, 8, 12, 3, 1, 1)],
    # the data gradient of a 3x3 conv (fgan128 Discriminator conv3 / conv5 / conv7): ConvTranspose2d k3 s1 p1
    "convT_k3s1p1": [_plan.Seg("convT", 6, 8, 8, 3, 1, 1)],
    "convT_k3s1p1_odd": [_plan.Seg("convT", 3, 5, 7, 3, 1, 1)],
}


@pytest.mark.parametrize("name", sorted(PATCH_CASES))
@pytest.mark.parametrize("cfg", [None, 1, 3])
def test_patch_plan_matches_torch(name, cfg):
    segs = PATCH_CASES[name]
    gen = torch.Generator().manual_seed(2)
    B, M = 3, 7
    plan = _plan.plan_patch_job(B, M, segs, cfg)
    if plan is None:
        pytest.skip("configuration not applicable to this job")
    xs, ws, lays, ref = [], [], [], 0
    for sg in segs:
        x, w, lay = make(sg, B, M, gen)
        xs.append(x)
        ws.append(w)
        lays.append(lay)
        ref = ref + ref_out(sg, x, w)
    got = emulate_patch(plan, xs, ws, lays)
    assert torch.allclose(got, ref, atol=1e-10, rtol=1e-10)
    tiles = _plan.build_patch_tiles([plan])
    assert len({tuple(t) for t in tiles.tolist()}) == len(tiles) == plan.npb * (-(-M // 32))


def test_generator_layers_use_patch_kernel():
    for M, segs in [(128, [_plan.Seg("convT", 256, 4, 4, 4, 2, 1)] * 2),
                    (64, [_plan.Seg("convT", 128, 8, 8, 4, 2, 1), _plan.Seg("pw", 32, 16, 16)]),
                    (32, [_plan.Seg("convT", 64, 16, 16, 4, 2, 1), _plan.Seg("pw", 16, 32, 32)])]:
        assert _plan.pick_patch_cfg(256, M, segs) is not None


def test_strided_conv_layers_use_patch_kernel():
    """FFCDiscriminator ffc0-3 convs (models/ffc_discriminator.py:26-30) and the generator's ConvT
    data gradients (Conv2d k4 s2 p1) run on the LDS-patch kernel in 4-channel x 16-tap chunks"""
    for M, segs in [(64, [_plan.Seg("conv", 3, 64, 64, 4, 2, 1)]),
                    (128, [_plan.Seg("conv", 64, 32, 32, 4, 2, 1)] * 2),
                    (128, [_plan.Seg("conv", 64, 32, 32, 4, 2, 1), _plan.Seg("pw", 64, 16, 16)]),
                    (256, [_plan.Seg("conv", 128, 16, 16, 4, 2, 1)] * 2),
                    (512, [_plan.Seg("conv", 256, 8, 8, 4, 2, 1)] * 2),
                    (256, [_plan.Seg("conv", 128, 8, 8, 4, 2, 1)] * 2),
                    (32, [_plan.Seg("conv", 3, 64, 64, 4, 2, 1)])]:
        p = _plan.pick_patch_cfg(256, M, segs)
        assert p is not None and 4 in p.cc, segs


def test_patch_cfg_policy_min_blocks():
    """4-phase jobs keep NTW = 4 (cfg 0) down to `min_blocks` workgroups: the split-bf16 products use
    128 (the runtime's choice, _runtime.CONV_ARITH == "split"), the f32 products 512"""
    segs = [_plan.Seg("convT", 128, 8, 8, 4, 2, 1), _plan.Seg("pw", 32, 16, 16)]   # gen64 ffc2 global, M = 64
    p512 = _plan.pick_patch_cfg(256, 64, segs)
    p128 = _plan.pick_patch_cfg(256, 64, segs, 128)
    assert p512.cfg == 1 and p128.cfg == 0
    assert 128 <= p128.npb * 2 < 512   # cfg 0: pixel blocks x 2 M-tiles, between the two thresholds


# --------------------------------------------------------------------------- round 5: plan keys and launch guard
def test_conv_layer_backward_plans_distinct_per_channel_count(monkeypatch):
    """the r04b illegal memory access: two conv_layer backward (adjoint) jobs of one
    layer structure that differ only in the input channel count C -- i.e. in the adjoint's output
    channels M -- must get two plans.  Before 144747e the adjoint key ("adj", spec, i, edges, B, segs)
    had no C, so the second job reused the first one's plan and its kernel wrote B*C1*H*W outputs
    into a B*C2*H*W tensor.  run_conv now keys every plan by (caller key, B, M, segments, device,
    plan switches), whatever the caller's key holds."""
    from fastfourierconvolution_amd import _autograd as ag
    from fastfourierconvolution_amd import _runtime as rt
    made = []

    class FakeExec:
        def __init__(self, B, M, segs, weights, dev, pw_ok=False, convq_cfg=None):
            self.plan = _plan.plan_job(B, M, segs)
            self.flops, self.kind = 0.0, "gemm"
            made.append((B, M, tuple(segs)))

        def ensure_packed(self, weights):
            pass

        job = rt.ConvExec.job
        check_launch = rt.ConvExec.check_launch

        def base_job(self):
            return None

    class FakeLaunch:
        def __init__(self, execs, dev):
            pass

        def launch(self, jobs, stream, flops=0.0):
            pass

    class FakeJob:
        def __init__(self):
            self.seg = [FakeJob.Seg() for _ in range(4)]

        class Seg:
            pass
    monkeypatch.setattr(rt, "ConvExec", FakeExec)
    monkeypatch.setattr(rt, "LaunchPlan", FakeLaunch)
    monkeypatch.setattr(FakeExec, "base_job", lambda self: FakeJob())
    monkeypatch.setattr(ag, "_stream", lambda t: 0)
    cache = {}
    B, H = 2, 8
    g = torch.zeros(B, 16, 2 * H, 2 * H)            # the gradient of a ConvT(C -> 16, k4 s2 p1) output
    adj = _plan.Seg("conv", 16, 2 * H, 2 * H, 4, 2, 1)   # its adjoint: Conv2d k4 s2 p1 back to H x H
    outs = []
    for C in (8, 24):                                # same structure and gradient, different C
        key = ("adj", "spec", 0, (0,), B, (adj,))    # the round-4 key: no C
        w = (torch.zeros(C, 16, 4, 4), 0, 4, 4, None)
        outs.append(ag.run_conv(cache, key, B, C, (adj,), [w], [g], out_shape=(B, C, H, H)))
    assert [m[1] for m in made] == [8, 24], made     # two plans, one per output channel count
    assert len(cache) == 2
    assert [tuple(o.shape) for o in outs] == [(B, 8, H, H), (B, 24, H, H)]


def test_conv_launch_guard_rejects_mismatched_tensors():
    """ConvExec.check_launch (the host-side guard before every conv launch): a plan used with an output,
    addend or input of other extents raises FFCError instead of launching a kernel that would write
    (or read) past the tensor; (B, M, k, k) views of a (B, M k k, 1, 1) output are accepted"""
    from fastfourierconvolution_amd import _runtime as rt
    ex = rt.ConvExec.__new__(rt.ConvExec)
    segs = (_plan.Seg("convT", 16, 8, 8, 4, 2, 1), _plan.Seg("pw", 12, 16, 16))
    ex.plan = _plan.plan_job(4, 32, segs)
    x0, x1 = torch.zeros(4, 16, 8, 8), torch.zeros(4, 12, 16, 16)
    out = torch.zeros(4, 32, 16, 16)
    ex.check_launch([(x0, None), (x1, None)], out, addend=torch.zeros(4, 32, 16, 16))
    bad = [
        ([(x0, None), (x1, None)], torch.zeros(4, 24, 16, 16), None),      # fewer output channels
        ([(x0, None), (x1, None)], torch.zeros(4, 40, 16, 16), None),      # more
        ([(x0, None), (x1, None)], torch.zeros(4, 32, 16, 16)[:, :, :, :8], None),   # strided view
        ([(x0, None), (x1, None)], out, torch.zeros(4, 32, 8, 8)),          # addend
        ([(torch.zeros(4, 8, 8, 8), None), (x1, None)], out, None),         # input channels
        ([(torch.zeros(2, 16, 8, 8), None), (x1, None)], out, None),        # batch
        ([(x0, None)], out, None),                                          # segment count
        ([(x0, torch.zeros(4, 15)), (x1, None)], out, None),                # gate size
    ]
    for inputs, o, add in bad:
        with pytest.raises(rt.FFCError):
            ex.check_launch(inputs, o, add)
    ex1 = rt.ConvExec.__new__(rt.ConvExec)
    ex1.plan = _plan.plan_job(4, 32 * 16, (_plan.Seg("pw", 100, 1, 1),))   # ffc0's outer-product form
    ex1.check_launch([(torch.zeros(4, 100, 1, 1), None)], torch.zeros(4, 32, 4, 4))
    pool = rt.ConvExec.__new__(rt.ConvExec)                # a 2x2-pooled segment reads the 2x input
    pool.plan = _plan.plan_job(4, 8, (_plan.Seg("pw", 12, 8, 8, pool=True),))
    pool.check_launch([(torch.zeros(4, 12, 16, 16), None)], torch.zeros(4, 8, 8, 8))
    with pytest.raises(rt.FFCError):
        pool.check_launch([(torch.zeros(4, 12, 8, 8), None)], torch.zeros(4, 8, 8, 8))


def test_st_split_max_rounds_to_power_of_two():
    from fastfourierconvolution_amd import _runtime as rt
    assert [rt._pow2_floor(v) for v in ("0", "1", "3", "6", "8", "12", -4)] == [1, 1, 2, 4, 8, 8, 1]
