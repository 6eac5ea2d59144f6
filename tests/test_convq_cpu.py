"""Host logic of the convq plans (ffc_convq_forward, csrc/convq_kernels.hip) on the CPU.

A numpy emulation walks exactly the index arithmetic the kernel uses -- pixel blocks, the
4 phases, per-chunk patches at (r0 * mult + org), tap offsets relative to the patch origin, the
(chunk, tap, channel) K order of the packed weights, direct 1x1 segments at (oy, ox) -- with
fp64 products in place of the split-bf16 MFMAs, and compares it with torch's ConvTranspose2d /
1x1 conv.  It also checks every patch read a valid pixel makes stays inside the staged patch and
that the staging fits the kernel's registers (QEMAX x 256 units).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from fastfourierconvolution_amd import _plan

MAX_UNITS = 256   # staging units per chunk: 8 channels x 4 pixels each, one per staging thread


def _pack(plan, weights):
    """A[phase][m][k] from the plan's ktab (what ffc_conv_pack does): convT weight (I, O, kh, kw),
    1x1 conv weight (O, I, 1, 1)"""
    A = []
    for ph in plan.phases:
        ent = plan.ktab[ph["kt_off"]: ph["kt_off"] + ph["K"]]
        a = np.zeros((plan.M, ph["K"]))
        for k, (sx, oy, ox, kk) in enumerate(ent):
            seg = sx & 15
            if seg == 15:
                continue
            ch, ky, kx = sx >> 4, kk & 0xFFFF, kk >> 16
            w, kind = weights[seg]
            a[:, k] = w[ch, :, ky, kx] if kind == "convT" else w[:, ch, ky, kx]
        A.append(a)
    return A


def _emulate(plan, xs, A):
    B, M, OH, OW = plan.B, plan.M, plan.OH, plan.OW
    out = np.zeros((B, M, OH, OW))
    NS, TR, TC = plan.NS, plan.TR, plan.TC
    npb = plan.npb
    mt, ntw = _plan.CONVQ_CFGS[plan.cfg]
    for pb in range(npb):
        bs, prem = divmod(pb, plan.nrb * plan.ncb)
        rb, cb = divmod(prem, plan.ncb)
        b0, r0, c0 = bs * NS, rb * TR, cb * TC
        for si, sg in enumerate(plan.segs):   # staging fits the kernel's registers
            if not plan.direct[si]:
                PR, PC = plan.prc[si]
                assert PC % 4 == 0 and 2 * NS * PR * (PC // 4) <= MAX_UNITS
        for p, ph in enumerate(plan.phases):
            for q in range(32 * ntw):
                ns, rem = divmod(q, TR * TC)
                r, c = divmod(rem, TC)
                if not (ns < NS and b0 + ns < B and r0 + r < ph["PH"] and c0 + c < ph["PW"]):
                    continue
                b, oy, ox = b0 + ns, (r0 + r) * 2 + ph["py"], (c0 + c) * 2 + ph["px"]
                acc = np.zeros(M)
                for si, sg in enumerate(plan.segs):
                    T, kseg = ph["T"][si], ph["kseg"][si]
                    x = xs[si]
                    if plan.direct[si]:
                        if T == 0:
                            continue
                        for c0_ in range(0, plan.cpad[si], 16):
                            for cc in range(16):
                                ch = c0_ + cc
                                if ch < sg.C:
                                    acc += A[p][:, kseg + c0_ + cc] * x[b, ch, oy, ox]
                        continue
                    PR, PC = plan.prc[si]
                    my_, mx_ = plan.mults[si]
                    org_y, org_x = plan.org[si]
                    iy0, ix0 = r0 * my_ + org_y, c0 * mx_ + org_x
                    xoff = ix0 - (ix0 & ~3)     # image column of patch column 0 (aligned 4-pixel groups)
                    taps = plan.taptab[ph["tap_base"][si]: ph["tap_base"][si] + T]
                    for ci, c0_ in enumerate(range(0, plan.cpad[si], 16)):
                        for t in range(T):
                            dy, dx = int(taps[t]) >> 16, int(taps[t]) & 0xFFFF
                            pr, pc = r * my_ + dy, c * mx_ + dx
                            assert 0 <= pr < PR and 0 <= pc + xoff < PC, "patch read outside the staged patch"
                            iy, ix = iy0 + pr, ix0 + pc
                            if not (0 <= iy < sg.IH and 0 <= ix < sg.IW):
                                continue
                            for cc in range(16):
                                ch = c0_ + cc
                                if ch < sg.C:
                                    acc += A[p][:, kseg + c0_ * T + 16 * t + cc] * x[b, ch, iy, ix]
                out[b, :, oy, ox] = acc
    return out


@pytest.mark.parametrize("cfg", [0, 1, 2, 3])
@pytest.mark.parametrize("B,C0,C1,Cv,IH,M", [(3, 20, 12, 8, 4, 40), (2, 16, 0, 0, 8, 32), (5, 7, 9, 16, 12, 70),
                                             (1, 33, 0, 5, 16, 64), (4, 16, 16, 0, 4, 32), (2, 8, 8, 8, 32, 36)])
def test_convq_plan_emulation(cfg, B, C0, C1, Cv, IH, M):
    rng = np.random.default_rng(cfg * 100 + B * 7 + IH)
    segs, weights, xs = [], [], []
    for C in (C0, C1):
        if C:
            segs.append(_plan.Seg("convT", C, IH, IH, 4, 2, 1))
            weights.append((rng.standard_normal((C, M, 4, 4)), "convT"))
            xs.append(rng.standard_normal((B, C, IH, IH)))
    if Cv:
        segs.append(_plan.Seg("pw", Cv, 2 * IH, 2 * IH))
        weights.append((rng.standard_normal((M, Cv, 1, 1)), "pw"))
        xs.append(rng.standard_normal((B, Cv, 2 * IH, 2 * IH)))
    plan = _plan.plan_convq_job(B, M, segs, cfg)
    if plan is None:
        pytest.skip("patch does not fit this configuration")
    assert plan.q and plan.mt == _plan.CONVQ_CFGS[cfg][0]
    got = _emulate(plan, xs, _pack(plan, weights))
    ref = 0
    for (w, kind), x in zip(weights, xs):
        xt, wt = torch.from_numpy(x), torch.from_numpy(w)
        ref = ref + (F.conv_transpose2d(xt, wt, stride=2, padding=1) if kind == "convT" else F.conv2d(xt, wt))
    np.testing.assert_allclose(got, ref.numpy(), rtol=1e-10, atol=1e-10)


def test_convq_rejects_unsupported():
    assert _plan.plan_convq_job(2, 8, [_plan.Seg("conv", 8, 8, 8, 4, 2, 1)], 0) is None          # 1 phase
    assert _plan.plan_convq_job(2, 8, [_plan.Seg("convT", 8, 6, 6, 4, 2, 1)], 0) is None         # IW % 4
    assert _plan.plan_convq_job(2, 8, [_plan.Seg("convT", 8, 8, 8, 4, 2, 1, pool=True)], 0) is None
    # gen64 / fgan128 layer shapes all plan (patch fits the staging registers)
    for B, C, IH, M in [(256, 256, 4, 128), (256, 128, 8, 64), (256, 64, 16, 32), (32, 256, 4, 128),
                        (64, 64, 64, 64), (64, 256, 16, 128)]:
        segs = [_plan.Seg("convT", C, IH, IH, 4, 2, 1), _plan.Seg("convT", C, IH, IH, 4, 2, 1)]
        assert _plan.pick_convq_cfg(B, M, segs) is not None, (B, C, IH, M)


@pytest.mark.parametrize("ksplit", [1, 2, 4, 8])
def test_convq_split_tiles(ksplit):
    """K-split tile table: every (job, m0, pixel block) output tile appears once per split, with one
    slot shared by its splits (tile.w = slot * 8 + split); slots are dense 0..nslots-1"""
    segs = [_plan.Seg("convT", 64, 8, 8, 4, 2, 1), _plan.Seg("pw", 16, 16, 16)]
    q = _plan.plan_convq_job(6, 96, segs, 3)
    t = _plan.build_patch_tiles([q], ksplit=ksplit)
    ntiles = q.npb * (-(-q.M // (32 * q.mt)))
    assert t.shape == (ntiles * ksplit, 4)
    if ksplit == 1:
        assert (t[:, 3] == 0).all()
        return
    slot, ks = t[:, 3] >> 3, t[:, 3] & 7
    assert sorted(set(slot.tolist())) == list(range(ntiles))
    for s in range(ntiles):
        rows = t[slot == s]
        assert sorted(ks[slot == s].tolist()) == list(range(ksplit))
        assert (rows[:, :3] == rows[0, :3]).all()
    assert len({tuple(r) for r in t[:, :3].tolist()}) == ntiles
    st = _plan.convq_slot_tiles(t)
    assert st.shape == (ntiles, 4) and (st[:, 3] == 0).all()
    for s in range(ntiles):
        assert (t[slot == s][0, :3] == st[s, :3]).all()


def test_convq_ksplit_choice():
    """small batches split K (more workgroups than 256 CUs' worth of output tiles), large ones do
    not; at least 4 chunks per split; FFC_CONVQ_KSPLIT forces"""
    import os
    segs = [_plan.Seg("convT", 256, 4, 4, 4, 2, 1), _plan.Seg("convT", 256, 4, 4, 4, 2, 1),
            _plan.Seg("pw", 64, 8, 8)]
    big_segs = [_plan.Seg("convT", 64, 16, 16, 4, 2, 1), _plan.Seg("convT", 64, 16, 16, 4, 2, 1),
                _plan.Seg("pw", 16, 32, 32)]
    small, big = _plan.pick_convq_cfg(32, 128, segs), _plan.pick_convq_cfg(256, 32, big_segs)
    assert small.ksplit > 1 and _plan.convq_chunks(small) >= 4 * small.ksplit
    assert big.ksplit == 1
    os.environ["FFC_CONVQ_KSPLIT"] = "3"
    try:
        assert _plan.pick_convq_cfg(32, 128, segs).ksplit == 3
    finally:
        os.environ.pop("FFC_CONVQ_KSPLIT")
