"""Host-side planning of the implicit-GEMM convolution launches (pure integer bookkeeping).

A *job* computes one output tensor as the sum of up to three convolution segments
(e.g. FFCTranspose's ``convl2l(x_l) + convg2l(x_g)``, layers/ffc/ffc_transpose.py:96-100,
or ``convl2g(x_l) + conv2(x + fu(x))``, :104-106 with spectral_transform.py:108).

Output pixels are split into *phases* ``oy = my*Sy + py`` so that all pixels of a phase
see the same taps: a stride-s transposed conv has s*s phases (4 for the generator's
ConvT k4 s2 p1), a ConvT on a 1x1 input gets one phase per output pixel (ffc0), an
ordinary conv has one phase.  Per phase the k-table lists every (segment, channel, tap)
that can be in bounds; its entry gives the input offset ``iy = my*mult + off``.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import os

import numpy as np

# FFC_CONVQ_TCMAX: convq pixel-block width cap (A/B), read once; part of _runtime.plan_knobs()
CONVQ_TCMAX = int(os.environ.get("FFC_CONVQ_TCMAX", "0"))

BK = 16
MPAD = 128
TILE_CFGS = {0: (128, 128, 2), 1: (64, 128, 2), 2: (32, 256, 4)}  # cfg -> (BM, BN, slab rows per tile)
PAD_ENTRY = (15, 0, 0, 0)


@dataclass(frozen=True)
class Seg:
    """One convolution segment feeding a job.

    kind: 'conv' (nn.Conv2d), 'convT' (nn.ConvTranspose2d) or 'pw' (1x1, stride 1, at the
    output resolution: the 1x1 convs of SpectralTransform).
    C, IH, IW: channels / spatial size seen by the taps (after pooling when pool=True).
    """
    kind: str
    C: int
    IH: int
    IW: int
    k: int = 1
    s: int = 1
    p: int = 0
    d: int = 1
    op: int = 0
    pool: bool = False
    gate: bool = False   # a per-(sample, channel) multiplier is applied on load (SE gate)


def conv_out(n, k, s, p, d):
    return (n + 2 * p - d * (k - 1) - 1) // s + 1


def convT_out(n, k, s, p, d, op):
    return (n - 1) * s - 2 * p + d * (k - 1) + op + 1


def seg_out(sg: Seg):
    if sg.kind == "conv":
        return conv_out(sg.IH, sg.k, sg.s, sg.p, sg.d), conv_out(sg.IW, sg.k, sg.s, sg.p, sg.d)
    if sg.kind == "convT":
        return convT_out(sg.IH, sg.k, sg.s, sg.p, sg.d, sg.op), convT_out(sg.IW, sg.k, sg.s, sg.p, sg.d, sg.op)
    return sg.IH, sg.IW


@dataclass
class Phase:
    py: int
    px: int
    PH: int
    PW: int
    entries: list = field(default_factory=list)  # (seg | ch<<4, off_y, off_x, ky | kx<<16)

    @property
    def K(self):
        return len(self.entries)

    @property
    def Kpad(self):
        return max(BK, -(-self.K // BK) * BK)


@dataclass
class JobPlan:
    B: int
    M: int
    OH: int
    OW: int
    Sy: int
    Sx: int
    segs: tuple
    mults: list          # per segment (mult_y, mult_x)
    phases: list
    ktab: np.ndarray     # int32 [entries, 4]
    kt_off: list
    a_off: list
    a_size: int          # floats in the packed weight buffer

    @property
    def Mpad(self):
        return -(-self.M // MPAD) * MPAD


def choose_phase_stride(segs, OH, OW):
    sT = {sg.s for sg in segs if sg.kind == "convT"}
    if len(sT) > 1:
        raise ValueError("a job's transposed segments must share one stride")
    if any(sg.kind == "conv" for sg in segs) and sT and max(sT) > 1:
        raise ValueError("cannot mix strided transposed and direct convolutions in one job")
    if sT:
        s = sT.pop()
        one_px = all(sg.IH == 1 and sg.IW == 1 for sg in segs if sg.kind == "convT")
        if s == 1 and one_px and OH * OW <= 16:
            return OH, OW  # one phase per output pixel: exactly one tap each
        return s, s
    return 1, 1


def _taps(sg: Seg, S: int, py: int, axis_in: int, PH: int):
    """valid (k index, off) pairs along one axis for phase offset py."""
    out = []
    for kk in range(sg.k):
        if sg.kind == "convT":
            num = py + sg.p - kk * sg.d
            if num % sg.s:
                continue
            off, mult = num // sg.s, S // sg.s
        elif sg.kind == "conv":
            off, mult = py * sg.s - sg.p + kk * sg.d, S * sg.s
        else:
            off, mult = py, S
        if any(0 <= my * mult + off < axis_in for my in range(PH)):
            out.append((kk, off))
    return out


def seg_mult(sg: Seg, S: int):
    if sg.kind == "convT":
        return S // sg.s
    if sg.kind == "conv":
        return S * sg.s
    return S


def plan_job(B: int, M: int, segs) -> JobPlan:
    segs = tuple(segs)
    outs = {seg_out(sg) for sg in segs}
    if len(outs) != 1:
        raise ValueError(f"segments disagree on the output size: {outs}")
    OH, OW = outs.pop()
    if OH <= 0 or OW <= 0:
        raise ValueError("empty output")
    Sy, Sx = choose_phase_stride(segs, OH, OW)
    for sg in segs:
        if sg.kind == "convT" and (Sy % sg.s or Sx % sg.s):
            raise ValueError("phase stride must be a multiple of the transposed stride")
        if sg.kind == "pw" and (sg.IH, sg.IW) != (OH, OW):
            raise ValueError("pointwise segment must be at the output resolution")
    if Sy * Sx > 16:
        raise ValueError("too many phases")
    phases, ktab, kt_off, a_off = [], [], [], []
    Mpad = -(-M // MPAD) * MPAD
    a_total = 0
    for py in range(Sy):
        for px in range(Sx):
            PH = -(-(OH - py) // Sy)
            PW = -(-(OW - px) // Sx)
            if PH <= 0 or PW <= 0:
                continue
            ph = Phase(py, px, PH, PW)
            for si, sg in enumerate(segs):
                ty = _taps(sg, Sy, py, sg.IH, PH)
                tx = _taps(sg, Sx, px, sg.IW, PW)
                for ch in range(sg.C):
                    for ky, oy in ty:
                        for kx, ox in tx:
                            ph.entries.append((si | (ch << 4), oy, ox, ky | (kx << 16)))
            if ph.K == 0:
                ph.entries.append(PAD_ENTRY)  # all-zero phase (e.g. fully cropped): still write outputs
            kt_off.append(len(ktab))
            ktab.extend(ph.entries)
            ktab.extend([PAD_ENTRY] * (ph.Kpad - ph.K))
            a_off.append(a_total)
            a_total += Mpad * ph.Kpad
            phases.append(ph)
    mults = [(seg_mult(sg, Sy), seg_mult(sg, Sx)) for sg in segs]
    return JobPlan(B, M, OH, OW, Sy, Sx, segs, mults, phases, np.asarray(ktab, dtype=np.int32).reshape(-1, 4),
                   kt_off, a_off, a_total)


def pick_tile_cfg(Ms):
    m = max(Ms)
    if m >= 128:
        return 0
    if m > 32:
        return 1
    return 2


def xcd_remap(n: int, nxcd: int = 8):
    """blockIdx -> locality index such that each XCD (blockIdx % 8) gets a contiguous run
    (bijective for any n; cdna_hip_programming.md 'XCD swizzle must be bijective')."""
    q, r = divmod(n, nxcd)
    out = np.empty(n, dtype=np.int64)
    for b in range(n):
        x, slot = b % nxcd, b // nxcd
        base = x * (q + 1) if x < r else r * (q + 1) + (x - r) * q
        out[b] = base + slot
    return out


def build_tiles(plans, cfg):
    """int32 [ntiles, 4] {job | phase<<8, m0, n0, slot}; slots per job returned too."""
    BM, BN, _ = TILE_CFGS[cfg]
    ordered = []
    nslots = []
    for j, pl in enumerate(plans):
        slot = 0
        per_phase = []
        for pi, ph in enumerate(pl.phases):
            npix = pl.B * ph.PH * ph.PW
            lst = []
            for n0 in range(0, npix, BN):
                lst.append((pi, n0, slot))
                slot += 1
            per_phase.append(lst)
        nslots.append(slot)
        # locality order: same n-block across phases and m-tiles next to each other
        depth = max(len(x) for x in per_phase)
        for t in range(depth):
            for lst in per_phase:
                if t < len(lst):
                    pi, n0, sl = lst[t]
                    for m0 in range(0, pl.M, BM):
                        ordered.append((j | (pi << 8), m0, n0, sl))
    n = len(ordered)
    remap = xcd_remap(n)
    tiles = np.asarray([ordered[i] for i in remap], dtype=np.int32).reshape(-1, 4)
    return tiles, nslots


# --------------------------------------------------------------------------- LDS-patch plans
PATCH_CC = 16
PATCH_PMAX = 32
PATCH_CFGS = {0: (4, 4), 1: (4, 2), 2: (1, 2), 3: (1, 1)}   # cfg -> (phases per block, N-tiles per wave)


@dataclass
class PatchPlan:
    B: int
    M: int
    OH: int
    OW: int
    Sy: int
    Sx: int
    segs: tuple
    mults: list
    cpad: list
    org: list            # per segment (org_y, org_x)
    prc: list            # per segment (PR, PC)
    vec4: list           # per segment: staged in 16-byte groups (IW % 4 == 0)
    rowlen: list         # per segment: LDS patch row length in floats (PC, or whole 4-float groups)
    phases: list         # dicts: py, px, PH, PW, T[s], kseg[s], tap_base[s], tap_h[s], Kpad, a_off, kt_off, K
    ktab: np.ndarray     # packing table (same format as JobPlan.ktab)
    taptab: np.ndarray   # int32 patch-relative tap offsets
    a_size: int
    cfg: int
    NS: int
    TR: int
    TC: int
    nrb: int
    ncb: int
    cc: list = field(default_factory=list)   # per segment: channels per chunk (16, or 4 for 16 taps)
    q: bool = False      # ffc_convq_forward plan (K order (chunk, tap, channel), pre-split operands)
    mt: int = 1          # convq: M-tiles of 32 channels per wave (tiles step m0 by 32 * mt)
    direct: list = field(default_factory=list)   # convq: per segment, B read straight from global
    qstride: list = field(default_factory=list)  # convq: per segment LDS (row, sample) pixel strides
    ksplit: int = 1      # convq: K splits per output tile (ffc_convq_forward_split)

    @property
    def Mpad(self):
        return -(-self.M // MPAD) * MPAD

    @property
    def npb(self):
        return -(-self.B // self.NS) * self.nrb * self.ncb


PATCH_MAX_UNITS = 8 * 256   # staging units per chunk (convp_kernels.hip NEMAX x 256 threads)


def patch_units_per_row(PC: int, vec4: bool, aligned: bool = False) -> int:
    """staging units per patch row: 4-float groups covering PC columns from the row start rounded
    down to a multiple of 4 (by up to 3 columns unless every block's start is aligned), or floats"""
    if not vec4:
        return PC
    return -(-PC // 4) if aligned else (PC + 6) // 4


def plan_patch_job(B: int, M: int, segs, cfg: int | None = None):
    """LDS-patch plan, or None when the job does not fit the patch kernel."""
    segs = tuple(segs)
    if any(sg.pool or sg.gate for sg in segs):
        return None                  # LDS-DMA staging copies bytes: no pooling / gating on the way in
    base = plan_job(B, M, segs)      # validates shapes, picks the phase stride
    NP = base.Sy * base.Sx
    if NP not in (1, 4) or len(base.phases) != NP:
        return None
    if cfg is None:
        cfg = 0 if NP == 4 else 2
    np_, ntw = PATCH_CFGS[cfg]
    if np_ != NP:
        return None
    npix = (4 // NP) * ntw * 32
    PHm = max(ph.PH for ph in base.phases)
    PWm = max(ph.PW for ph in base.phases)
    TC = min(PWm, npix)
    TR = min(PHm, max(1, npix // TC))
    NS = max(1, min(B, npix // (TR * TC)))
    nrb, ncb = -(-PHm // TR), -(-PWm // TC)
    # taps per (phase, segment): 1, 2 or 4 in 16-channel chunks; 16 (4 x 4, e.g. Conv2d k4 s2) in
    # 4-channel chunks, one-phase jobs only
    taps = []
    cc = [PATCH_CC] * len(segs)
    for ph in base.phases:
        row = []
        for si, sg in enumerate(segs):
            ty = _taps(sg, base.Sy, ph.py, sg.IH, ph.PH)
            tx = _taps(sg, base.Sx, ph.px, sg.IW, ph.PW)
            if NP == 1 and len(ty) == len(tx) == 3 and (sg.kind == "conv" or (sg.kind == "convT" and sg.s == 1)):
                # 3x3 (FFC k3, BASELINE configs[0] / fgan128's head; the stride-1 ConvTranspose2d k3 is
                # the data gradient of a 3x3 conv, e.g. the fgan128 Discriminator's): run as 4x4 taps in
                # 4-channel chunks with a zero-weight 4th row / column (k index -1), one pixel past the
                # 3rd, taps in ascending offset order (a ConvTranspose2d's offsets fall with k)
                ty, tx = sorted(ty, key=lambda t: t[1]), sorted(tx, key=lambda t: t[1])
                if any(b[1] - a[1] != 1 for a, b in zip(ty, ty[1:])) or any(b[1] - a[1] != 1 for a, b in zip(tx, tx[1:])):
                    return None
                ty = ty + [(-1, ty[-1][1] + 1)]
                tx = tx + [(-1, tx[-1][1] + 1)]
            T = len(ty) * len(tx)
            if T == 16 and NP == 1 and len(ty) == len(tx) == 4:
                cc[si] = 4
            elif T and 4 % T:
                return None
            row.append((ty, tx))
        taps.append(row)
    cpad = [-(-sg.C // cc[si]) * cc[si] for si, sg in enumerate(segs)]
    org, prc, vec4, rowlen = [], [], [], []
    for si, sg in enumerate(segs):
        oys = [o for row in taps for (k, o) in row[si][0]]
        oxs = [o for row in taps for (k, o) in row[si][1]]
        if not oys or not oxs:
            oys, oxs = [0], [0]
        my_, mx_ = base.mults[si]
        oy0, ox0 = min(oys), min(oxs)
        PR = (TR - 1) * my_ + (max(oys) - oy0) + 1
        PC = (TC - 1) * mx_ + (max(oxs) - ox0) + 1
        v4 = sg.IW % 4 == 0
        al = ox0 % 4 == 0 and (TC * mx_) % 4 == 0
        if NS * cc[si] * PR * patch_units_per_row(PC, v4, al) > PATCH_MAX_UNITS:
            return None
        vec4.append(v4)
        rowlen.append(4 * patch_units_per_row(PC, True, al) if v4 else PC)
        org.append((oy0, ox0))
        prc.append((PR, PC))
    phases, ktab, taptab = [], [], []
    a_total = 0
    Mpad = -(-M // MPAD) * MPAD
    for pi, ph in enumerate(base.phases):
        d = dict(py=ph.py, px=ph.px, PH=ph.PH, PW=ph.PW, T=[], kseg=[], tap_base=[], tap_h=[])
        k = 0
        kt_off = len(ktab)
        for si, sg in enumerate(segs):
            ty, tx = taps[pi][si]
            T = len(ty) * len(tx)
            d["T"].append(T)
            d["kseg"].append(k)
            d["tap_base"].append(len(taptab))
            PR, PC = prc[si]
            base_t = len(taptab)
            for (ky, oy) in ty:
                for (kx, ox) in tx:
                    taptab.append(((oy - org[si][0]) << 16) | (ox - org[si][1]))
            th = 0
            if T == 16:   # the kernel reads taps 8..15 as taps 0..7 shifted by one (dy, dx)
                dyx = [(t >> 16, t & 0xFFFF) for t in taptab[base_t:]]
                hy, hx = dyx[8][0] - dyx[0][0], dyx[8][1] - dyx[0][1]
                if hx < 0 or any((dyx[j + 8][0] - dyx[j][0], dyx[j + 8][1] - dyx[j][1]) != (hy, hx)
                                 for j in range(8)):
                    return None
                th = (hy << 16) | hx
            d["tap_h"].append(th)
            for ch in range(cpad[si]):
                for (ky, oy) in ty:
                    for (kx, ox) in tx:
                        ktab.append((si | (ch << 4), oy, ox, ky | (kx << 16))
                                    if ch < sg.C and ky >= 0 and kx >= 0 else PAD_ENTRY)
            k += cpad[si] * T
        if k == 0:
            return None
        d["Kpad"] = k
        d["K"] = k
        d["kt_off"] = kt_off
        d["a_off"] = a_total
        a_total += Mpad * k
        phases.append(d)
    return PatchPlan(B, M, base.OH, base.OW, base.Sy, base.Sx, segs, base.mults, cpad, org, prc, vec4, rowlen, phases,
                     np.asarray(ktab, dtype=np.int32).reshape(-1, 4), np.asarray(taptab or [0], dtype=np.int32),
                     a_total, cfg, NS, TR, TC, nrb, ncb, cc)


# --------------------------------------------------------------------------- convq plans
CONVQ_CFGS = {0: (1, 4), 1: (1, 2), 2: (2, 2), 3: (1, 1)}   # cfg -> (M-tiles, N-tiles) per wave
CONVQ_MAX_UNITS = 256      # staging units per chunk (one per staging thread: 4 pixels x 8 channels)
CONVQ_LDS_BUDGET = 150 * 1024  # LDS bytes per workgroup (one 8-wave workgroup per CU)


def convq_strides(NS, TR, TC, PR, PC, pad=True):
    """LDS (row, sample) pixel strides of the convq patch image.  A B fragment's lane n reads pixel
    p(n) = ns * qsample + r * qrow + c (+ a tap offset) at 48 * p bytes; the 16 lanes of a
    ds_read_b128 group are conflict-free when p(n) = n (mod 16) for every lane, i.e. qrow = TC and
    qsample = TR * TC (mod 16)."""
    if not pad:
        return PC, PR * PC
    qr = PC + ((TC - PC) % 16)
    qs = PR * qr + ((TR * TC - PR * qr) % 16)
    return qr, qs


def convq_lds_bytes(NS, strides):
    """three chunk buffers (csrc/convq_kernels.hip convq_tile)"""
    return 3 * (((max(NS * qs for _, qs in strides) * 96 + 255) // 256) * 256 + 256)


def plan_convq_job(B: int, M: int, segs, cfg: int):
    """ffc_convq_forward plan (4-phase stride-2 jobs: ConvTranspose2d k4 s2 segments staged through
    LDS, 1x1 segments at the output resolution read directly), or None when it does not apply."""
    segs = tuple(segs)
    if any(sg.pool or sg.gate for sg in segs):
        return None
    base = plan_job(B, M, segs)
    if (base.Sy, base.Sx) != (2, 2) or len(base.phases) != 4:
        return None
    mt, ntw = CONVQ_CFGS[cfg]
    npix = 32 * ntw
    PHm = max(ph.PH for ph in base.phases)
    PWm = max(ph.PW for ph in base.phases)
    TC = min(PWm, npix)
    if CONVQ_TCMAX >= 4 and TC > CONVQ_TCMAX:   # A/B: squarer pixel blocks (less halo)
        TC = CONVQ_TCMAX
    TR = min(PHm, max(1, npix // TC))
    NS = max(1, min(B, npix // (TR * TC)))
    nrb, ncb = -(-PHm // TR), -(-PWm // TC)
    direct = [sg.kind == "pw" for sg in segs]
    taps = []
    for ph in base.phases:
        row = []
        for si, sg in enumerate(segs):
            ty = _taps(sg, base.Sy, ph.py, sg.IH, ph.PH)
            tx = _taps(sg, base.Sx, ph.px, sg.IW, ph.PW)
            T = len(ty) * len(tx)
            if (direct[si] and T not in (0, 1)) or T > 4:
                return None
            row.append((ty, tx))
        taps.append(row)
    cpad = [-(-sg.C // 16) * 16 for sg in segs]
    org, prc = [], []
    for si, sg in enumerate(segs):
        my_, mx_ = base.mults[si]
        if direct[si]:
            if (my_, mx_) != (2, 2):
                return None
            org.append((0, 0))
            prc.append((1, 1))
            continue
        oys = [o for row in taps for (k, o) in row[si][0]] or [0]
        oxs = [o for row in taps for (k, o) in row[si][1]] or [0]
        oy0, ox0 = min(oys), min(oxs)
        PR = (TR - 1) * my_ + (max(oys) - oy0) + 1
        PC = (TC - 1) * mx_ + (max(oxs) - ox0) + 1
        if sg.IW % 4:
            return None                    # staged in aligned 4-pixel groups
        PC = 4 * patch_units_per_row(PC, True, False)   # image columns: groups from the aligned start
        if 2 * NS * PR * (PC // 4) > CONVQ_MAX_UNITS:
            return None
        org.append((oy0, ox0))
        prc.append((PR, PC))
    staged = [prc[si] for si in range(len(segs)) if not direct[si]]
    pad = bool(staged) and convq_lds_bytes(NS, [convq_strides(NS, TR, TC, PR, PC) for PR, PC in staged]) \
        <= CONVQ_LDS_BUDGET
    if os.environ.get("FFC_CONVQ_PAD") == "0":
        pad = False
    qstride = [convq_strides(NS, TR, TC, PR, PC, pad) for (PR, PC) in prc]
    if staged and convq_lds_bytes(NS, [qstride[si] for si in range(len(segs)) if not direct[si]]) > 160 * 1024:
        return None
    if any(not direct[si] and B * sg.C * sg.IH * sg.IW * 4 >= 0x7FFFFFFF for si, sg in enumerate(segs)):
        return None                        # staged through 32-bit buffer offsets
    phases, ktab, taptab = [], [], []
    a_total = 0
    Mpad = -(-M // MPAD) * MPAD
    for pi, ph in enumerate(base.phases):
        d = dict(py=ph.py, px=ph.px, PH=ph.PH, PW=ph.PW, T=[], kseg=[], tap_base=[], tap_h=[])
        k = 0
        kt_off = len(ktab)
        for si, sg in enumerate(segs):
            ty, tx = taps[pi][si]
            T = len(ty) * len(tx)
            d["T"].append(T)
            d["kseg"].append(k)
            d["tap_base"].append(len(taptab))
            d["tap_h"].append(0)
            tl = [(ky, oy, kx, ox) for (ky, oy) in ty for (kx, ox) in tx]
            # the kernel runs exactly 4 taps per staged segment (1 per direct one): missing taps (tiny
            # inputs) are padded with zero weights reading the patch origin
            TT = 1 if direct[si] else 4
            d["T"][-1] = TT
            for t in range(TT):
                taptab.append(((tl[t][1] - org[si][0]) << 16) | (tl[t][3] - org[si][1]) if t < T else 0)
            for c0 in range(0, cpad[si], 16):            # K order: chunk, tap, channel
                for t in range(TT):
                    for ch in range(c0, c0 + 16):
                        if t < T and ch < sg.C:
                            ky, oy, kx, ox = tl[t]
                            ktab.append((si | (ch << 4), oy, ox, ky | (kx << 16)))
                        else:
                            ktab.append(PAD_ENTRY)
            k += cpad[si] * TT
        if k == 0:
            return None
        d["Kpad"] = k
        d["K"] = k
        d["kt_off"] = kt_off
        d["a_off"] = a_total
        a_total += Mpad * k
        phases.append(d)
    return PatchPlan(B, M, base.OH, base.OW, base.Sy, base.Sx, segs, base.mults, cpad, org, prc,
                     [not d for d in direct], [pc for (_, pc) in prc], phases,
                     np.asarray(ktab, dtype=np.int32).reshape(-1, 4), np.asarray(taptab or [0], dtype=np.int32),
                     a_total, cfg, NS, TR, TC, nrb, ncb, [16] * len(segs), True, mt, direct, qstride)


CONVQ_SPLIT_FIXED = 17500.0  # cycles: partial stores + the reduce launch (~7 us measured, r02 sweep)


def convq_chunks(q) -> int:
    """16-channel chunks of K per output tile (staged and direct segments)"""
    return sum(c // 16 for c in q.cpad)


def convq_cost(q, ksplit: int = 1) -> float:
    """Cycle estimate of a convq plan, fitted on MI355X (tools/convq_probe.py, r02): the workgroups
    run in rounds of 256 CUs x (2 workgroups per CU for the (1, 1) tile, else 1), each chunk costs
    768 cycles per 32 x 32 MFMA tile of a wave plus ~5500 cycles of fixed per-chunk latency
    (staging hand-off, A loads, barrier); a K split runs ceil(chunks / ksplit) chunks per
    workgroup on ksplit x the workgroups, plus the partial-sum hand-off."""
    wgs = q.npb * (-(-q.M // (32 * q.mt))) * ksplit
    mt, ntw = CONVQ_CFGS[q.cfg]
    slots = 256 * (2 if (mt, ntw) == (1, 1) else 1)
    per_wg = -(-convq_chunks(q) // ksplit) * (768.0 * mt * ntw + 5500.0)
    return -(-wgs // slots) * (per_wg + (CONVQ_SPLIT_FIXED if ksplit > 1 else 0.0))


# Measured (cfg, ksplit) per convq launch group: tools/tune_convq.py sweeps every configuration
# of the timed layer shapes on MI355X and writes convq_tuned.json; the cost model below is the
# fallback for shapes the table does not hold.
_TUNED = None


def job_signature(B, M, segs) -> tuple:
    return (int(B), int(M), tuple((sg.kind, sg.C, sg.IH, sg.IW, sg.k, sg.s, sg.p, sg.d, sg.op, sg.pool, sg.gate)
                                  for sg in segs))


def convq_tuned():
    """{job signature: cfg}, {group signature (sorted job signatures): (cfg, ksplit)}"""
    global _TUNED
    if _TUNED is None:
        import json
        jobs, groups = {}, {}
        path = os.environ.get("FFC_CONVQ_TUNED", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                               "convq_tuned.json"))
        if path and os.path.exists(path):
            with open(path) as f:
                for e in json.load(f)["entries"]:
                    sigs = tuple(sorted((B, M, tuple(tuple(sg) for sg in segs)) for B, M, segs in e["jobs"]))
                    groups[sigs] = (int(e["cfg"]), int(e["ksplit"]))
                    for sg in sigs:
                        jobs[sg] = int(e["cfg"])
        _TUNED = (jobs, groups)
    return _TUNED


def pick_convq_ksplit(q) -> int:
    """K splits for a convq plan: the cheapest of 1, 2, 4, 8 by convq_cost with at least 4 chunks
    per split; FFC_CONVQ_KSPLIT forces one (A/B measurements)"""
    return pick_convq_ksplit_group([q])


def pick_convq_ksplit_group(plans) -> int:
    """one K split for the jobs of one convq launch (they share the grid): the cheapest by the
    summed convq_cost, at least 4 chunks per split in every job; FFC_CONVQ_KSPLIT forces one"""
    cmin = min(convq_chunks(q) for q in plans)
    force = os.environ.get("FFC_CONVQ_KSPLIT")
    if force is not None:
        return max(1, min(8, int(force), cmin))
    tuned = convq_tuned()[1].get(tuple(sorted(job_signature(q.B, q.M, q.segs) for q in plans)))
    if tuned is not None and tuned[0] == plans[0].cfg:
        return max(1, min(tuned[1], cmin))
    ks = [k for k in (1, 2, 4, 8) if k == 1 or cmin >= 4 * k]
    return min(ks, key=lambda k: (sum(convq_cost(q, k) for q in plans), k))


def convq_slot_tiles(tiles) -> np.ndarray:
    """the slot table of a K-split tile table: int32 [nslots, 4] {job, m0, pixel block, 0} in slot
    order (split 0's row of every slot)"""
    first = tiles[(tiles[:, 3] & 7) == 0]
    out = np.zeros((first.shape[0], 4), dtype=np.int32)
    out[first[:, 3] >> 3, :3] = first[:, :3]
    return out


def pick_convq_cfg(B, M, segs):
    """the convq configuration (and K split) with the lowest convq_cost (MT = 2 only when M >= 64);
    FFC_CONVQ_CFG forces the configuration (A/B measurements)"""
    force = os.environ.get("FFC_CONVQ_CFG")
    tuned = convq_tuned()[0].get(job_signature(B, M, segs))
    if os.environ.get("FFC_CONVQ_TUNED_LOG"):
        import sys
        print(f"[convq] tuned cfg {'hit' if tuned is not None else 'miss'}: {job_signature(B, M, segs)}",
              file=sys.stderr)
    if force is not None:
        cands = [int(force)]
    elif tuned is not None:
        cands = [tuned]
    else:
        cands = ([0, 2] if M >= 64 else [0]) + [1, 3]
    plans = [q for q in (plan_convq_job(B, M, segs, c) for c in cands) if q is not None]
    for q in plans:
        q.ksplit = pick_convq_ksplit(q)
    return min(plans, key=lambda q: convq_cost(q, q.ksplit)) if plans else None


def pick_patch_cfg(B, M, segs, min_blocks=512):
    """4-phase jobs: NTW=4 unless that leaves fewer than `min_blocks` workgroups.  512 (2 per CU)
    suits the f32-MFMA products; the split-bf16 products pay a per-group A split that 4 N-tiles
    amortise better than 2, so the runtime passes 128 for them (gen64 on MI355X: 459K -> 478K
    img/s; fgan128 and the training step unchanged, profiles/r01i)."""
    force = os.environ.get("FFC_PATCH_CFG4")   # A/B measurements: force the 4-phase configuration
    if force is not None:
        q = plan_patch_job(B, M, segs, int(force))
        if q is not None:
            return q
    p = plan_patch_job(B, M, segs)
    if p is None:   # a smaller pixel block may still fit the staging limits
        return plan_patch_job(B, M, segs, 1) or plan_patch_job(B, M, segs, 3)
    if p.cfg == 0:
        blocks = p.npb * (-(-M // 32))
        if blocks < min_blocks:
            q = plan_patch_job(B, M, segs, 1)
            if q is not None:
                return q
    return p


def patch_tile_cost(pl) -> int:
    """k-steps a workgroup of this job runs (the phases of a block run concurrently, so the
    slowest phase counts)"""
    return max(ph["Kpad"] for ph in pl.phases)


def build_patch_tiles(plans, nxcd: int = 8, ksplit: int = 1):
    """int32 [ntiles, 4] {job, m0, pixel block, slot * 8 + split}, XCD-remapped (ksplit > 1: each
    output tile (slot) as ksplit consecutive workgroups, one per K range; ffc_convq_forward_split).

    The pixel blocks are cut into nxcd contiguous ranges, one per XCD (blockIdx % 8), so the
    workgroups that share a block's input patch share an L2.  Within an XCD's run the heaviest
    job's tiles come first: a CU's first and second resident workgroups are then one heavy and
    one light tile (dispatch deals an XCD's blocks round-robin over its CUs), and in launches of
    more rounds the light tiles fill in behind the heavy ones (longest-processing-time first)."""
    npb = max(pl.npb for pl in plans)
    order = sorted(range(len(plans)), key=lambda j: -patch_tile_cost(plans[j]))
    ordered = []
    if os.environ.get("FFC_TILE_ORDER") == "interleaved":   # previous order, for A/B measurements
        for pb in range(npb):
            for j, pl in enumerate(plans):
                if pb < pl.npb:
                    for m0 in range(0, pl.M, 32):
                        ordered.append((j, m0, pb, 0))
        remap = xcd_remap(len(ordered), nxcd)
        return np.asarray([ordered[i] for i in remap], dtype=np.int32).reshape(-1, 4)
    slot = 0
    for x in range(nxcd):
        lo, hi = npb * x // nxcd, npb * (x + 1) // nxcd
        for j in order:
            pl = plans[j]
            for pb in range(lo, min(hi, pl.npb)):
                for m0 in range(0, pl.M, 32 * pl.mt):
                    for k in range(ksplit):
                        ordered.append((j, m0, pb, slot * 8 + k if ksplit > 1 else 0))
                    slot += 1
    remap = xcd_remap(len(ordered), nxcd)
    return np.asarray([ordered[i] for i in remap], dtype=np.int32).reshape(-1, 4)
