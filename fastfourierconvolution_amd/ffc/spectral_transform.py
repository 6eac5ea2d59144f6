"""Drop-in ``SELayer`` / ``SpectralTransform`` (reference: layers/ffc/spectral_transform.py:12-110).

Same constructor signatures, submodule names (``downsample``, ``conv1``, ``bn1``, ``act1``, ``fu``,
``lfu``, ``conv2``, ``se_block``) and state_dict keys.  ``lfu`` is constructed (its parameters
are in the reference's checkpoints) but never executed, exactly as in the reference (:94-105).

HIP execution of forward (x -> conv2(s + fu(s))):
  1. SE gate per sample (mean over HW, two tiny FCs)                      ffc_se_gate
  2. conv1 as a 1x1 GEMM with the gate (and the 2x2 avg-pool) fused into its operand load,
     BN partials in its epilogue                                          ffc_conv_forward
  3. bn1 batch statistics (train) / running statistics (eval)             ffc_bn_reduce_finalize
  4. fused Fourier unit: bn1+ReLU and the x2 nearest upsample fused into its loads,
     pass 0 statistics, pass 1 apply + residual s + fu(s)                 ffc_fu_forward
  5. conv2 as a 1x1 GEMM (inside FFC/FFCTranspose this is folded into the local conv GEMM)
SE, conv1 and train-mode BN1 commute with nearest upsampling, so steps 1-3 run at the input
resolution; the running-var unbiasing uses the upsampled count (count_mult = 4).
"""
import torch
import torch.nn as nn

from .. import _autograd as ag
from .. import _plan
from .. import _runtime as rt
from .. import ops
from .._lib import check, ptr
from .fourier_unity import FourierUnitSN


class SELayer(nn.Module):
    def __init__(self, channel, reduction=16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Sequential(
            nn.Linear(channel, channel // reduction, bias=False),
            nn.ReLU(inplace=True),
            nn.Linear(channel // reduction, channel, bias=False),
            nn.Sigmoid(),
        )

    def gate(self, x, pool: bool):
        """(B, C) sigmoid gate on the HIP path (pool: gate of the 2x2-avg-pooled x)."""
        x = rt.require(x, "x")
        B, C, H, W = x.shape
        hid = self.fc[0].out_features
        w1 = rt.require(self.fc[0].weight.detach(), "se.fc.0.weight") if hid > 0 else None
        w2 = rt.require(self.fc[2].weight.detach(), "se.fc.2.weight") if hid > 0 else None
        g = torch.empty((B, C), device=x.device, dtype=torch.float32)
        ps = None if pool else rt.plane_sums_for(x)
        if ps is not None:   # plane sums from the BN-apply pass that wrote x: no second read of x
            with rt.observe("se_gate"):
                check(rt.lib().ffc_se_gate_sums(ptr(ps[0]), ps[1], B, C, H * W, ptr(w1), ptr(w2), hid, ptr(g),
                                                rt.stream_of(x)), "ffc_se_gate_sums")
            return g
        with rt.observe("se_gate", bytes=4.0 * x.numel()):
            check(rt.lib().ffc_se_gate(ptr(x), B, C, H, W, int(pool), ptr(w1), ptr(w2), hid, ptr(g), rt.stream_of(x)),
                "ffc_se_gate")
        return g

    def forward(self, x):
        """x * sigmoid(fc(avg_pool(x))) on the ffc::se_scale op (gate + one per-(b, c) scale launch)."""
        return ag.se_layer(self, rt.require(x, "x"))


class SpectralTransform(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, stride: int = 1, groups: int = 1,
                 enable_lfu: bool = False, upsample: bool = False, num_classes: int = 1):
        super().__init__()
        self._ffc_ctor = ["SpectralTransform", dict(in_channels=in_channels, out_channels=out_channels, stride=stride,
                                                    groups=groups, enable_lfu=enable_lfu, upsample=upsample,
                                                    num_classes=num_classes)]
        self.enable_lfu = enable_lfu
        self.downsample = nn.Identity()
        if stride == 2 and upsample:
            self.downsample = nn.Upsample(scale_factor=2, mode="nearest")
        if stride == 2 and not upsample:
            self.downsample = nn.AvgPool2d(kernel_size=(2, 2), stride=2)
        self.stride = stride
        self.upsample = upsample
        self.groups = groups
        self.conv1 = nn.Conv2d(in_channels, out_channels // 2, kernel_size=1, groups=groups, bias=False)
        self.bn1 = nn.BatchNorm2d(out_channels // 2)
        self.act1 = nn.ReLU(inplace=True)
        self.fu = FourierUnitSN(out_channels // 2, out_channels // 2, groups, num_classes=num_classes)
        if self.enable_lfu:
            self.lfu = FourierUnitSN(out_channels // 2, out_channels // 2, groups, num_classes=num_classes)
        self.conv2 = torch.nn.Conv2d(out_channels // 2, out_channels, kernel_size=1, groups=groups, bias=False)
        self.se_block = SELayer(self.conv1.in_channels)
        self._cache = {}

    # ------------------------------------------------------------------ internals
    def _conv1_T(self, stream):
        """conv1 weight transposed + zero padded for ffc_st_prologue (re-packed when it changes)"""
        w = rt.require(self.conv1.weight.detach(), "conv1.weight")

        def build():
            c, cin = w.shape[0], w.shape[1]
            c1T = torch.empty((cin, -(-c // 32) * 32), device=w.device, dtype=torch.float32)
            check(rt.lib().ffc_pack_transpose(ptr(w), c, cin, ptr(c1T), stream), "ffc_pack_transpose")
            return c1T
        return self.__dict__.setdefault("_packs", rt.PackCache()).get("conv1T", [w], build)

    def _conv1_3(self, stream):
        """conv1 weight as split-bf16 MFMA fragments for ffc_st_prologue_ex3 (None: Cin % 16 != 0 or
        FFC_ST_MFMA=f32)"""
        w = rt.require(self.conv1.weight.detach(), "conv1.weight")
        c, cin = w.shape[0], w.shape[1]
        n = rt.lib().ffc_st_pack_a3_elems(c, cin)
        if not n or not rt.ST_SPLIT_MFMA:
            return None

        def build():
            wc3 = torch.empty(n, device=w.device, dtype=torch.int16)
            check(rt.lib().ffc_st_pack_a3(ptr(w), c, cin, ptr(wc3), stream), "ffc_st_pack_a3")
            return wc3
        return self.__dict__.setdefault("_packs", rt.PackCache()).get("conv1_3", [w], build)

    def _mode(self):
        if self.stride == 2 and self.upsample:
            return 1, 2  # pool, up
        if self.stride == 2:
            return 2, 1
        return 1, 1

    def spectral(self, x):
        """v = s + fu(s), s = relu(bn1(conv1(se(downsample(x))))) — the part of forward before conv2."""
        x = rt.require(x, "x")
        if self.groups != 1:
            raise NotImplementedError("grouped SpectralTransform (groups != 1) is not on the hot path")
        B, Cin, H, W = x.shape
        if Cin != self.conv1.in_channels:
            raise RuntimeError(f"SpectralTransform expected {self.conv1.in_channels} channels, got {Cin}")
        rt.sn_refresh(self.conv1)
        pool = self.stride == 2 and not self.upsample
        up = 2 if (self.stride == 2 and self.upsample) else 1
        if pool and (H % 2 or W % 2):
            raise NotImplementedError("AvgPool2d(2) downsample of an odd-sized input")
        h2, w2 = (H // 2, W // 2) if pool else (H, W)
        c = self.conv1.out_channels
        dev = x.device
        stream = rt.stream_of(x)
        use_batch, _ = rt.bn_mode(self.bn1)
        L = rt.lib()
        hid = self.se_block.fc[0].out_features
        t = torch.empty((B, c, h2, w2), device=dev, dtype=torch.float32)
        if rt.ST_PATH != "pw" and L.ffc_st_prologue_lds_bytes(Cin, H, W, int(pool), hid, c) > 0:
            # one fused launch: [pool] -> SE gate -> conv1 -> per-sample BN1 partials
            se1 = rt.require(self.se_block.fc[0].weight.detach(), "se.fc.0.weight") if hid > 0 else None
            se2 = rt.require(self.se_block.fc[2].weight.detach(), "se.fc.2.weight") if hid > 0 else None
            wc = self._conv1_T(stream)
            # small batches: several workgroups per sample, each with a share of conv1's tiles
            split = min(L.ffc_st_prologue_split(B, Cin, H, W, int(pool), c), rt.st_split_max(B)) if rt.ST_SPLIT else 1
            nrows = B * split
            slab = torch.empty((nrows, c, 4), device=dev, dtype=torch.float32)
            wc3 = self._conv1_3(stream)
            with rt.observe("st_prologue", flops=2.0 * B * c * Cin * h2 * w2):
                check(L.ffc_st_prologue_ex3(ptr(x), B, Cin, H, W, int(pool), ptr(se1), ptr(se2), hid, ptr(wc),
                                            ptr(wc3), c, split, ptr(t), ptr(slab), None, stream), "ffc_st_prologue")
        elif not pool and L.ffc_pw_gate_lds_bytes(Cin, c) > 0:
            # large planes: SE gate (plane means + FCs), then conv1 with the gate folded into the
            # per-sample weights and the bn1 partials in the epilogue (csrc/st_pw.hip)
            gate = self.se_block.gate(x, pool)
            w1 = rt.require(self.conv1.weight.detach(), "conv1.weight")
            nrows = B * L.ffc_pw_gate_blocks(h2 * w2)
            slab = torch.empty((nrows, c, 4), device=dev, dtype=torch.float32) if use_batch else None
            with rt.observe("st_conv1", flops=2.0 * B * c * Cin * h2 * w2, bytes=4.0 * B * (Cin + c) * h2 * w2):
                check(L.ffc_pw_gate_conv(ptr(x), ptr(gate), ptr(w1), B, Cin, c, h2 * w2, ptr(t), ptr(slab), stream),
                      "ffc_pw_gate_conv")
        else:
            gate = self.se_block.gate(x, pool)
            key = ("conv1", B, Cin, h2, w2, pool, str(dev))
            ex = self._cache.get(key)
            if ex is None:
                seg = _plan.Seg("pw", Cin, h2, w2, pool=pool, gate=True)
                ex = rt.ConvExec(B, c, [seg], [rt.conv_weight(self.conv1)], dev)
                lp = rt.LaunchPlan([ex], dev)
                self._cache[key] = ex = (ex, lp)
            ex, lp = ex
            ex.ensure_packed([rt.conv_weight(self.conv1)])
            nrows = lp.stat_rows(0)
            slab = torch.empty((nrows, c, 4), device=dev, dtype=torch.float32) if use_batch else None
            lp.launch([ex.job([(x, gate)], t, stats=slab)], stream, flops=ex.flops)
        fold = rt.bn_fold(self.bn1, c, slab, nrows, float(up * up), dev) if use_batch else None
        if fold is None and use_batch:   # the staged FU's r2c can still fold it channel by channel
            fold = rt.bn_fold_channels(self.bn1, c, slab, nrows, float(up * up), dev)
        if fold is not None:   # bn1 finalized inside the FU's first kernel
            return self.fu._run(t, up=up, in_relu=True, residual=True, in_fold=fold)
        sc1, sh1 = rt.bn_scale_shift(self.bn1, c, slab, nrows if use_batch else 0, float(up * up), dev, stream)
        return self.fu._run(t, up=up, in_scale=sc1, in_shift=sh1, in_relu=True, residual=True)

    def forward(self, x, y=None):
        if y is not None:
            raise TypeError("SpectralTransform: the conditional (y) path is not supported (the reference raises "
                            "in FourierUnitSN, fourier_unity.py:46-47)")
        if ag.wants_grad(self, x):
            v = ag.spectral_v(self, rt.require(x, "x"))
            (out,) = ag.conv_layer(v.shape[0], [(self.conv2.out_channels, 0, 0.0)],
                                   [(0, 0, _plan.Seg("pw", v.shape[1], v.shape[2], v.shape[3]), self.conv2)], [v])
            return out
        return ops.st_forward(self, x)

    def _forward_fused(self, x):
        """forward on the fused inference kernels (the ffc::spectral_transform op runs this)"""
        v = self.spectral(x)
        rt.sn_refresh(self.conv2)
        B, c, H, W = v.shape
        key = ("conv2", B, c, H, W, str(v.device))
        ex = self._cache.get(key)
        if ex is None:
            ex = rt.ConvExec(B, self.conv2.out_channels, [_plan.Seg("pw", c, H, W)], [rt.conv_weight(self.conv2)],
                             v.device)
            self._cache[key] = ex = (ex, rt.LaunchPlan([ex], v.device))
        ex, lp = ex
        ex.ensure_packed([rt.conv_weight(self.conv2)])
        out = torch.empty((B, self.conv2.out_channels, H, W), device=v.device, dtype=torch.float32)
        lp.launch([ex.job([(v, None)], out)], rt.stream_of(v), flops=ex.flops)
        return out
