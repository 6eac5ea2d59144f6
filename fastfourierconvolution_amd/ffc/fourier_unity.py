"""Drop-in ``FourierUnitSN`` (reference: layers/ffc/fourier_unity.py:17-56).

Same constructor, attribute names (``conv_layer``, ``bn``, ``relu``) and state_dict keys;
forward runs the ffc::fourier_unit custom op -- the fused HIP Fourier unit (csrc/fu_kernels.hip,
csrc/fu2d_kernels.hip) -- instead of rfftn -> 1x1 conv -> BatchNorm2d -> ReLU -> irfftn (the
ffc::rfft2 / conv_layer / bn_act / irfft2 training ops under autograd).
"""
import ctypes

import torch
import torch.nn as nn

from .. import _autograd as ag
from .. import _runtime as rt
from .. import ops
from .._lib import check, ptr


class FourierUnitSN(nn.Module):
    def __init__(self, in_channels, out_channels, groups: int = 1, num_classes: int = 1):
        super().__init__()
        self._ffc_ctor = ["FourierUnitSN", dict(in_channels=in_channels, out_channels=out_channels, groups=groups,
                                                num_classes=num_classes)]
        self.groups = groups
        self.conv_layer = torch.nn.Conv2d(in_channels=in_channels * 2, out_channels=out_channels * 2,
                                          kernel_size=1, stride=1, padding=0, groups=self.groups, bias=False)
        self.bn = torch.nn.BatchNorm2d(out_channels * 2)
        self.relu = torch.nn.ReLU(inplace=True)
        self._packs = rt.PackCache()
        # "fp32" (exact, the reference's arithmetic) or "fp16": fp16 operands on the f16 MFMA with fp32
        # accumulation (BASELINE config 5); fp16 runs the staged FU (C in {16, 32, 64})
        self.mix_precision = "fp32"

    # ------------------------------------------------------------------ internals
    def _check(self, C):
        if self.groups != 1:
            raise NotImplementedError("grouped FourierUnitSN mix (groups != 1) is not on the hot path")
        if self.conv_layer.in_channels != 2 * C or self.conv_layer.out_channels != 2 * C:
            raise NotImplementedError("FourierUnitSN with in_channels != out_channels")

    def _packed_mix(self, device, stream):
        w = rt.require(self.conv_layer.weight.detach(), "conv_layer.weight")

        def build():
            C2 = w.shape[0]
            mixT = torch.empty((C2, -(-C2 // 32) * 32), device=device, dtype=torch.float32)
            check(rt.lib().ffc_fu_pack_mix(ptr(w), C2, ptr(mixT), stream), "ffc_fu_pack_mix")
            return mixT
        return self._packs.get("mix", [w], build)

    def _packed_mix3(self, mixT, device, stream):
        """the mix weight's split bf16 pieces in MFMA fragment order (ffc_fu_pack_mix3), or None when
        C % 8 != 0 (the fused kernel then splits wmixT itself)"""
        w = self.conv_layer.weight
        C = w.shape[0] // 2
        n = rt.lib().ffc_fu_mix3_elems(C)
        if n == 0:
            return None

        def build():
            w3 = torch.empty(int(n), device=device, dtype=torch.int16)
            check(rt.lib().ffc_fu_pack_mix3(ptr(mixT), C, ptr(w3), stream), "ffc_fu_pack_mix3")
            return w3
        return self._packs.get("mix3", [rt.require(w.detach(), "conv_layer.weight")], build)

    @staticmethod
    def _fold_ok(C, H, W):
        """the fused kernel's planes hold the in-kernel BN fold's scratch (csrc/bn_common.h)"""
        return 16 * C * H * (W // 2 + 1) >= 8 * 3 * 512 // 4

    def _run(self, t, up=1, in_scale=None, in_shift=None, in_relu=False, residual=False, in_fold=None):
        """fused FU over s = transform(t) (see include/ffc_amd.h ffc_fu_forward_ex).  in_fold: the
        input BN (SpectralTransform.bn1) as an rt.BnFoldDesc, finalized inside pass 0."""
        B, C, th, tw = t.shape
        H, W = th * up, tw * up
        self._check(C)
        L = rt.lib()
        fused = L.ffc_fu_lds_bytes(C, H, W) > 0 and not rt.FORCE_FU2D
        staged_ok = L.ffc_fu2d_supported(C, H, W, up)
        if self.mix_precision == "fp16":
            if not (staged_ok and C in (16, 32, 64)):
                raise NotImplementedError(f"fp16 mix: staged FU with C in {{16, 32, 64}} only; got C={C}, {H}x{W}")
            fused = False
        if fused and staged_ok and (rt.FU_PATH == "staged" or (rt.FU_PATH == "auto" and B < rt.FU_FUSED_MIN_BATCH)):
            fused = False
        if in_fold is not None and fused and in_fold.moments is None and (in_fold.channel_only or
                                                                          not self._fold_ok(C, H, W)):
            in_scale, in_shift = in_fold.materialize(rt.stream_of(t))
            in_fold = None
        if not fused:
            if L.ffc_fu2d_supported(C, H, W, up):
                return self._run2d(t, up, in_scale, in_shift, in_relu, residual, in_fold)
            raise NotImplementedError(f"Fourier unit supports H,W in {{4,8,16,32}} with 16*C*H*(W/2+1) <= 160 KiB "
                                      f"(fused) or square H=W in {{16,32,64,128}} with 2C <= 128 (staged); "
                                      f"got C={C}, {H}x{W}")
        dev = t.device
        stream = rt.stream_of(t)
        mixT = self._packed_mix(dev, stream)
        mix3 = self._packed_mix3(mixT, dev, stream)
        use_batch, _ = rt.bn_mode(self.bn)
        n_r = float(B * C * H * W)              # fused FU moves 4*N_r per read/write
        n_y = float(B * 2 * C * H * (W // 2 + 1))
        sc = sh = mix_fold = yspill = None
        kg = 1
        if use_batch:
            # pass 0 over two bin groups per sample where the library takes them (ffc_fu_kgroups: half
            # the spectrum's columns per workgroup, two workgroups per CU); slab rows = B x groups
            kg = L.ffc_fu_kgroups(B, C, H, W) if (rt.FU_KGROUPS and rt.FU_SPILL and mix3 is not None) else 1
            rows = L.ffc_fu_slab_rows(B, C, H, W, kg)
            slab = torch.empty((rows, 2 * C, 4), device=dev, dtype=torch.float32)
            # pass 0 keeps its mix output Y for pass 1 (no second row R2C + column FFT + mix)
            yspill = torch.empty(int(n_y), device=dev, dtype=torch.float32) if rt.FU_SPILL else None
            # bytes: SURVEY.md §8d's algorithmic basis (fused train FU = 12*N_r: x read in each pass,
            # out written once), never more than the kernel moves (t is read at the pre-upsample size);
            # moved: what this kernel pair actually streams (including the Y spill written and read back)
            mv0 = 4.0 * t.numel() + (4.0 * n_y if rt.FU_SPILL else 0.0)
            with rt.observe("fu_pass0", bytes=min(4.0 * n_r, mv0), moved=mv0):
                check(L.ffc_fu_forward_ex4(ptr(t), B, C, H, W, up, None if in_fold else ptr(in_scale),
                                           None if in_fold else ptr(in_shift), int(in_relu), ptr(mixT), ptr(mix3), 0,
                                           ptr(slab), None, None, 0, None,
                                           ctypes.byref(in_fold.struct) if in_fold else None, None, ptr(yspill),
                                           kg, stream), "ffc_fu_forward(pass 0)")
            if in_fold is not None:          # pass 0's workgroup 0 wrote the folded bn1 affine
                in_scale, in_shift = in_fold.scale, in_fold.shift
            mix_fold = None
            if rt.FU_SPLIT and yspill is not None and H == W and H in (8, 16, 32) and C % (64 // H) == 0:
                # the split pass 1 (one wave per 64 / H channels) folds its 2 * 64 / H channels itself
                mix_fold = rt.bn_fold_channels(self.bn, 2 * C, slab, rows, 1.0, dev, lanes=64 // (2 * 64 // H))
            if mix_fold is None and self._fold_ok(C, H, W):
                mix_fold = rt.bn_fold(self.bn, 2 * C, slab, rows, 1.0, dev)
            if mix_fold is None:
                sc, sh = rt.bn_scale_shift(self.bn, 2 * C, slab, rows, 1.0, dev, stream)
        else:
            if in_fold is not None:
                in_scale, in_shift = in_fold.materialize(stream)
            sc, sh = rt.bn_scale_shift(self.bn, 2 * C, None, 0, 1.0, dev, stream)
        out = torch.empty((B, C, H, W), device=dev, dtype=torch.float32)
        mv1 = (4.0 * n_y if yspill is not None else 4.0 * t.numel()) + 4.0 * t.numel() * bool(residual) + 4.0 * n_r
        with rt.observe("fu_pass1", bytes=min(8.0 * n_r, mv1), moved=mv1):
            check(L.ffc_fu_forward_ex4(ptr(t), B, C, H, W, up, ptr(in_scale), ptr(in_shift), int(in_relu), ptr(mixT),
                                       ptr(mix3), 1, None, ptr(sc), ptr(sh), int(residual), ptr(out), None,
                                       ctypes.byref(mix_fold.struct) if mix_fold else None, ptr(yspill), kg, stream),
                  "ffc_fu_forward(pass 1)")
        return out

    def _packed_mix16(self, device, stream):
        w = rt.require(self.conv_layer.weight.detach(), "conv_layer.weight")

        def build():
            C2 = w.shape[0]
            mix16 = torch.empty((-(-C2 // 32) * 32, C2), device=device, dtype=torch.float16)
            check(rt.lib().ffc_fu_pack_mix_f16(ptr(w), C2, ptr(mix16), stream), "ffc_fu_pack_mix_f16")
            return mix16
        return self._packs.get("mix16", [w], build)

    def _run2d(self, t, up, in_scale, in_shift, in_relu, residual, in_fold=None):
        """large-plane FU: r2c -> mix (pass 0 stats, pass 1 BN/ReLU) -> c2r (include/ffc_amd.h ffc_fu2d_*).
        in_fold: the input BN as an rt.BnFoldDesc -- finalized inside the r2c, one channel per plane
        workgroup, when that fold applies (rt.bn_fold_channels), else by its own launch"""
        B, C, h, w = t.shape
        if in_fold is not None:
            if in_fold.moments is not None:   # SyncBN: already merged over the ranks; per-channel needs momentum
                chf = in_fold if in_fold.bn.momentum is not None else None
            else:
                chf = rt.bn_fold_channels(in_fold.bn, C, in_fold.slab, in_fold.struct.nrows,
                                          in_fold.struct.count_mult, t.device, consumers=B)
            if chf is None:
                in_scale, in_shift = in_fold.materialize(rt.stream_of(t))
                in_fold = None
            else:
                in_fold = chf
        H, W = h * up, w * up
        L = rt.lib()
        dev = t.device
        stream = rt.stream_of(t)
        f16 = self.mix_precision == "fp16"
        mixT = self._packed_mix16(dev, stream) if f16 else self._packed_mix(dev, stream)
        mixfn = L.ffc_fu2d_mix_f16 if f16 else L.ffc_fu2d_mix
        use_batch, _ = rt.bn_mode(self.bn)
        nT = B * C * h * (w // 2 + 1)           # complex bins of T
        nY = B * C * H * (W // 2 + 1)           # complex bins of Y
        mix_flops = 2.0 * (2 * C) ** 2 * (B * H * (W // 2 + 1))   # (2C x 2C) GEMM over every bin
        n_r, n_c = float(B * C * H * W), float(B * C * H * (W // 2 + 1))   # SURVEY.md §8d, full resolution
        # SURVEY.md §8d's R2C bytes, capped at what the kernel moves: with the upsample folded in it
        # reads t (N_r / 4) and writes T (N_c / 4), and counting the full-resolution bytes would credit
        # bytes never transferred
        mvr = 4.0 * t.numel() + 8.0 * nT
        out = torch.empty((B, C, H, W), device=dev, dtype=torch.float32)
        c2r_moved = 8.0 * nY + 4.0 * out.numel() + (4.0 * t.numel() if residual else 0.0)
        c2r_bytes = min(8.0 * n_c + 4.0 * n_r, c2r_moved)                   # SURVEY.md §8d C2R pass
        fused_r2c = (use_batch and rt.FU2D_SPILL and rt.FU2D_R2CMIX and not f16 and
                     L.ffc_fu2d_r2c_mix_supported(C, H, W, up))
        T = None
        if not fused_r2c:
            T = torch.empty((B, C, h, w // 2 + 1, 2), device=dev, dtype=torch.float32)
            with rt.observe("fu2d_r2c", bytes=min(4.0 * n_r + 8.0 * n_c, mvr), moved=mvr):
                check(L.ffc_fu2d_r2c_ex(ptr(t), B, C, h, w, ptr(in_scale), ptr(in_shift), int(in_relu),
                                        ctypes.byref(in_fold.struct) if in_fold else None, ptr(T), stream),
                      "ffc_fu2d_r2c")
        if use_batch:
            rows = L.ffc_fu2d_slab_rows(B, C, H, W)
            slab = torch.empty((rows, 2 * C, 4), device=dev, dtype=torch.float32)
            # spill: pass 0 stores the raw Y and the C2R applies BN + ReLU on load (one mix instead of
            # two, and the statistics are taken from exactly the values they normalise)
            Y = torch.empty((B, C, H, W // 2 + 1, 2), device=dev, dtype=torch.float32) if rt.FU2D_SPILL else None
            if fused_r2c:
                # the R2C inside mix pass 0 (small t planes: every bin-range workgroup recomputes its
                # sample's T in LDS); labelled as the R2C stage, bytes = t in + the spilled Y out
                mv = 4.0 * t.numel() + 8.0 * nY
                with rt.observe("fu2d_r2c", flops=mix_flops, bytes=min(4.0 * n_r + 8.0 * n_c, mv), moved=mv):
                    check(L.ffc_fu2d_r2c_mix(ptr(t), B, C, H, W, up, ptr(in_scale), ptr(in_shift), int(in_relu),
                                             ctypes.byref(in_fold.struct) if in_fold else None, ptr(mixT),
                                             ptr(slab), ptr(Y), stream), "ffc_fu2d_r2c_mix")
            else:
                with rt.observe("fu2d_mix0", flops=mix_flops, bytes=8.0 * nT + (8.0 * nY if Y is not None else 0.0)):
                    check(mixfn(ptr(T), B, C, H, W, up, ptr(mixT), 0, ptr(slab), None, None, ptr(Y), stream),
                          "ffc_fu2d_mix(pass 0)")
            if in_fold is not None:   # the r2c's (or r2c_mix's) leader workgroups wrote the folded bn1 affine
                in_scale, in_shift = in_fold.scale, in_fold.shift
            cfold = rt.bn_fold_channels(self.bn, 2 * C, slab, rows, 1.0, dev, consumers=B) if Y is not None else None
            if cfold is not None:   # the FU's BN finalized inside the C2R (two channels per plane)
                with rt.observe("fu2d_c2r", bytes=c2r_bytes, moved=c2r_moved):
                    check(L.ffc_fu2d_c2r_fold(ptr(Y), B, C, H, W, ptr(t), up, ptr(in_scale), ptr(in_shift),
                                              int(in_relu), int(residual), ctypes.byref(cfold.struct), ptr(out),
                                              stream), "ffc_fu2d_c2r_fold")
                return out
            sc, sh = rt.bn_scale_shift(self.bn, 2 * C, slab, rows, 1.0, dev, stream)
            if Y is not None:
                with rt.observe("fu2d_c2r", bytes=c2r_bytes, moved=c2r_moved):
                    check(L.ffc_fu2d_c2r_bn(ptr(Y), B, C, H, W, ptr(t), up, ptr(in_scale), ptr(in_shift),
                                            int(in_relu), int(residual), ptr(sc), ptr(sh), ptr(out), stream),
                          "ffc_fu2d_c2r_bn")
                return out
        else:
            sc, sh = rt.bn_scale_shift(self.bn, 2 * C, None, 0, 1.0, dev, stream)
        if in_fold is not None and not use_batch:
            in_scale, in_shift = in_fold.scale, in_fold.shift
        if rt.FU_COLS and L.ffc_fu2d_cols_supported(C, H, W, up, int(f16)):
            # pass 1 with the inverse column FFT fused in (column-major Yc), then rows-only C2R
            Yc = torch.empty((B, C, W // 2 + 1, H, 2), device=dev, dtype=torch.float32)
            with rt.observe("fu2d_mix1", flops=mix_flops, bytes=8.0 * nT + 8.0 * nY):
                check(L.ffc_fu2d_mix_cols(ptr(T), B, C, H, W, up, ptr(mixT), int(f16), ptr(sc), ptr(sh), ptr(Yc),
                                          stream), "ffc_fu2d_mix_cols")
            with rt.observe("fu2d_c2r", bytes=c2r_bytes, moved=c2r_moved):
                check(L.ffc_fu2d_c2r_rows(ptr(Yc), B, C, H, W, ptr(t), up, ptr(in_scale), ptr(in_shift),
                                          int(in_relu), int(residual), ptr(out), stream), "ffc_fu2d_c2r_rows")
            return out
        Y = torch.empty((B, C, H, W // 2 + 1, 2), device=dev, dtype=torch.float32)
        with rt.observe("fu2d_mix1", flops=mix_flops, bytes=8.0 * nT + 8.0 * nY):
            check(mixfn(ptr(T), B, C, H, W, up, ptr(mixT), 1, None, ptr(sc), ptr(sh), ptr(Y), stream),
                  "ffc_fu2d_mix(pass 1)")
        with rt.observe("fu2d_c2r", bytes=c2r_bytes, moved=c2r_moved):
            check(L.ffc_fu2d_c2r(ptr(Y), B, C, H, W, ptr(t), up, ptr(in_scale), ptr(in_shift), int(in_relu),
                                 int(residual), ptr(out), stream), "ffc_fu2d_c2r")
        return out

    def forward(self, x, y=None):
        if y is not None:
            # reference: self.bn(ffted, y) -> BatchNorm2d.forward() takes 1 input (fourier_unity.py:46-47)
            raise TypeError("FourierUnitSN: the conditional (y) path is not supported (the reference raises here)")
        x = rt.require(x, "x")
        if ag.wants_grad(self, x):
            return ag.fourier_unit(self, x, residual=False)
        return ops.fu_forward(self, x)
