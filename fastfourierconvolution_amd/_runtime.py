"""Execution layer between the drop-in modules and the C ABI.

Owns: plan caches, weight packing (re-packed only when a weight's version changes),
per-call buffers (allocated from PyTorch's caching allocator, so hipGraph capture via
torch.cuda.graph works), BatchNorm statistics (optionally all-reduced across ranks for
sharded train-mode batches) and the launches themselves.  Every launch goes to
``torch.cuda.current_stream()``.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from . import _lib, _plan
from ._lib import FFCError, check, ptr  # noqa: F401  (re-exported for the layers)

# --------------------------------------------------------------------------- device / stream


def require(t: torch.Tensor, name: str = "input") -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor, got {type(t).__name__}")
    if not t.is_cuda:
        raise FFCError(f"{name}: the FFC hot path runs only on a ROCm/HIP device (tensor is on {t.device}); "
                       "there is no CPU fallback")
    if t.dtype != torch.float32:
        raise FFCError(f"{name}: fp32 required (got {t.dtype})")
    return t.contiguous()


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def lib():
    return _lib.load()


# --------------------------------------------------------------------------- launch observer
class LaunchObserver:
    """Records HIP events around every library launch (on the launch stream) with a label and
    the launch's algorithmic work, for bench.py's live roofline measurement."""

    def __init__(self):
        self.records = []   # (label, start event, end event, work dict)

    def summary(self):
        torch.cuda.synchronize()
        agg = {}
        for label, e0, e1, work in self.records:
            a = agg.setdefault(label, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0, "moved": 0.0})
            a["launches"] += 1
            a["ms"] += e0.elapsed_time(e1)
            a["flops"] += work.get("flops", 0.0)
            a["bytes"] += work.get("bytes", 0.0)
            a["moved"] += work.get("moved", work.get("bytes", 0.0))
        return agg


_OBS = {"obs": None}


def set_observer(obs):
    _OBS["obs"] = obs


class observe:
    """context manager around one launch"""

    def __init__(self, label, **work):
        self.label, self.work = label, work

    def __enter__(self):
        obs = _OBS["obs"]
        if obs is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        obs = _OBS["obs"]
        if obs is not None and exc[0] is None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            obs.records.append((self.label, self.e0, e1, self.work))
        return False


# --------------------------------------------------------------------------- SyncBN hook
_SYNC = {"group": None, "world1": False}


def set_sync_bn_group(group, even_world1: bool = False):
    """Route train-mode BN moments through torch.distributed.all_reduce (RCCL) over ``group``
    (None disables).  See fastfourierconvolution_amd.distributed.enable_sync_bn.
    ``even_world1``: keep the collective in a one-rank group (tests of the RCCL / hipGraph
    machinery on a one-GPU box); a one-rank group is otherwise skipped."""
    _SYNC["group"] = group
    _SYNC["world1"] = bool(even_world1)


def _sync_group():
    g = _SYNC["group"]
    if g is None:
        return None
    import torch.distributed as dist
    if not dist.is_initialized() or (dist.get_world_size(g) == 1 and not _SYNC["world1"]):
        return None
    return g


# --------------------------------------------------------------------------- batch norm
def bn_mode(bn: nn.BatchNorm2d):
    use_batch = bn.training or (bn.running_mean is None and bn.running_var is None)
    update = bn.training and bn.track_running_stats and bn.running_mean is not None
    return use_batch, update


def bn_scale_shift(bn: nn.BatchNorm2d, C: int, slab, nrows: int, count_mult: float, device, stream):
    """-> (scale, shift) fp32 device tensors of length C, nn.BatchNorm2d semantics."""
    if bn.num_features != C:
        raise RuntimeError(f"running_mean should contain {C} elements not {bn.num_features}")
    use_batch, update = bn_mode(bn)
    L = lib()
    scale = torch.empty(C, device=device, dtype=torch.float32)
    shift = torch.empty(C, device=device, dtype=torch.float32)
    momentum = -1.0 if bn.momentum is None else float(bn.momentum)
    gamma = ptr(bn.weight.detach()) if bn.weight is not None else None
    beta = ptr(bn.bias.detach()) if bn.bias is not None else None
    rm = ptr(bn.running_mean) if bn.running_mean is not None else None
    rv = ptr(bn.running_var) if bn.running_var is not None else None
    nbt = ptr(bn.num_batches_tracked) if bn.num_batches_tracked is not None else None
    if use_batch:
        # [C][3] moments + the large-slab scratch behind them (ffc_bn_reduce_ws_doubles)
        mbuf = torch.empty(3 * C + L.ffc_bn_reduce_ws_doubles(nrows, C), device=device, dtype=torch.float64)
        moments = mbuf[:3 * C].view(C, 3)
        grp = _sync_group()
        if grp is None:
            with observe("bn_stats"):
                check(L.ffc_bn_reduce_finalize(ptr(slab), nrows, C, ptr(mbuf), gamma, beta, rm, rv, nbt,
                                               int(update), momentum, float(bn.eps), float(count_mult), ptr(scale),
                                               ptr(shift), stream), "ffc_bn_reduce_finalize")
        else:
            from .distributed import merge_moments
            with observe("bn_stats"):
                check(L.ffc_bn_reduce(ptr(slab), nrows, C, ptr(mbuf), stream), "ffc_bn_reduce")
                merge_moments(moments, group=grp)
                check(L.ffc_bn_finalize(ptr(moments), C, gamma, beta, rm, rv, nbt, 1, int(update), momentum,
                                        float(bn.eps), float(count_mult), ptr(scale), ptr(shift), stream),
                      "ffc_bn_finalize")
    else:
        check(L.ffc_bn_finalize(None, C, gamma, beta, rm, rv, nbt, 0, 0, momentum, float(bn.eps), 1.0,
                                ptr(scale), ptr(shift), stream), "ffc_bn_finalize")
    return scale, shift


def _bn_finalize_batch(items, batch, device, stream):
    """single rank: the batch's reduce + finalize in one launch (ffc_bn_reduce_finalize_batch)"""
    from ._lib import BnRfItem
    L = lib()
    arr = (BnRfItem * len(batch))()
    res, keep = {}, []
    for k, (bn, C, slab, nrows, cm) in enumerate(batch):
        if bn.num_features != C:
            raise RuntimeError(f"running_mean should contain {C} elements not {bn.num_features}")
        _, update = bn_mode(bn)
        scale = torch.empty(C, device=device, dtype=torch.float32)
        shift = torch.empty(C, device=device, dtype=torch.float32)
        mbuf = torch.empty(3 * C + L.ffc_bn_reduce_ws_doubles(nrows, C), device=device, dtype=torch.float64)
        keep.append(mbuf)
        arr[k] = BnRfItem(ptr(slab), nrows, C, ptr(mbuf), ptr(bn.weight.detach()) if bn.weight is not None else None,
                          ptr(bn.bias.detach()) if bn.bias is not None else None,
                          ptr(bn.running_mean) if bn.running_mean is not None else None,
                          ptr(bn.running_var) if bn.running_var is not None else None,
                          ptr(bn.num_batches_tracked) if bn.num_batches_tracked is not None else None,
                          int(update), -1.0 if bn.momentum is None else float(bn.momentum), float(bn.eps), float(cm),
                          ptr(scale), ptr(shift))
        res[id(bn)] = (scale, shift)
    with observe("bn_stats"):
        check(L.ffc_bn_reduce_finalize_batch(arr, len(batch), stream), "ffc_bn_reduce_finalize_batch")
    return [res[id(it[0])] if id(it[0]) in res else bn_scale_shift(it[0], it[1], it[2], it[3], it[4], device, stream)
            for it in items]


def bn_act_apply_batch(items):
    """[(x, scale, shift, act, param, noise_w or None, noise or None[, plane_sum or None])]: y = x in
    place, one launch (ffc_bn_act_apply_batch; the l and g outputs of an FFC_BN_ACT, with fgan128's
    NoiseInjection).  plane_sum (B, C, ffc_plane_chunks(HW)) receives the chunk sums of y."""
    from ._lib import BnApplyItem
    arr = (BnApplyItem * len(items))()
    nbytes = 0.0
    for k, it in enumerate(items):
        x, sc, sh, act, param, nw, nz = it[:7]
        ps = it[7] if len(it) > 7 else None
        B, C = x.shape[:2]
        HW = x.numel() // (B * C)
        arr[k] = BnApplyItem(ptr(x), ptr(x), B, C, HW, ptr(sc), ptr(sh), int(act), float(param), ptr(nw), ptr(nz),
                             ptr(ps))
        nbytes += 8.0 * x.numel() + (4.0 * nz.numel() if nz is not None else 0.0)
    label = "bn_act_noise" if any(it[6] is not None for it in items) else "bn_act"
    with observe(label, bytes=nbytes):
        check(lib().ffc_bn_act_apply_batch(arr, len(items), stream_of(items[0][0])), "ffc_bn_act_apply_batch")


def bn_scale_shift_many(items, device, stream):
    """bn_scale_shift for several BNs whose slabs are ready together (an FFC layer's bn_l and bn_g,
    ffc_bn_act.py:80-83).  items: [(bn, C, slab, nrows, count_mult)] -> [(scale, shift)].  Under
    SyncBN their raw moments travel in ONE all-reduce (one collective per layer instead of one per
    BN: the per-rank step of strong scaling is latency-bound, each collective a round trip)."""
    grp = _sync_group()
    batch = [it for it in items if it[2] is not None and bn_mode(it[0])[0]]
    if len(batch) < 2 or len(batch) > 4:
        return [bn_scale_shift(bn, C, slab, nrows, cm, device, stream) for bn, C, slab, nrows, cm in items]
    if grp is None:
        return _bn_finalize_batch(items, batch, device, stream)
    from .distributed import merge_moments
    L = lib()
    Cs = [it[1] for it in batch]
    # moments of every BN back to back ([sum C][3]); each reduce's scratch lies behind its own
    # moments (the later BNs' moments included: they are reduced afterwards, in stream order)
    offs = [3 * sum(Cs[:i]) for i in range(len(batch))]
    need = max(offs[i] + 3 * Cs[i] + L.ffc_bn_reduce_ws_doubles(batch[i][3], Cs[i]) for i in range(len(batch)))
    mbuf = torch.empty(need, device=device, dtype=torch.float64)
    with observe("bn_stats"):
        for (bn, C, slab, nrows, _), o in zip(batch, offs):
            if bn.num_features != C:
                raise RuntimeError(f"running_mean should contain {C} elements not {bn.num_features}")
            check(L.ffc_bn_reduce(ptr(slab), nrows, C, ptr(mbuf[o:]), stream), "ffc_bn_reduce")
        tot = 3 * sum(Cs)
        merge_moments(mbuf[:tot].view(-1, 3), group=grp)
    res = {}
    for (bn, C, slab, nrows, cm), o in zip(batch, offs):
        use_batch, update = bn_mode(bn)
        scale = torch.empty(C, device=device, dtype=torch.float32)
        shift = torch.empty(C, device=device, dtype=torch.float32)
        momentum = -1.0 if bn.momentum is None else float(bn.momentum)
        with observe("bn_stats"):
            check(L.ffc_bn_finalize(ptr(mbuf[o:]), C, ptr(bn.weight.detach()) if bn.weight is not None else None,
                                    ptr(bn.bias.detach()) if bn.bias is not None else None,
                                    ptr(bn.running_mean) if bn.running_mean is not None else None,
                                    ptr(bn.running_var) if bn.running_var is not None else None,
                                    ptr(bn.num_batches_tracked) if bn.num_batches_tracked is not None else None,
                                    1, int(update), momentum, float(bn.eps), float(cm), ptr(scale), ptr(shift), stream),
                  "ffc_bn_finalize")
        res[id(bn)] = (scale, shift)
    return [res[id(it[0])] if id(it[0]) in res else bn_scale_shift(it[0], it[1], it[2], it[3], it[4], device, stream)
            for it in items]


# Train-mode BNs whose consumer kernel finalizes them in-kernel (ffc_bn_fold) instead of a
# separate ffc_bn_reduce_finalize launch: single rank only (SyncBN all-reduces the moments between
# the merge and the finalize).  FFC_BN_FOLD=0 restores the separate launch (A/B measurements).
BN_FOLD = __import__("os").environ.get("FFC_BN_FOLD", "1") != "0"
# slab rows x channels up to which the fold beats the separate launch (each consumer workgroup
# reads the whole slab; measured on MI355X, r02)
BN_FOLD_MAX = int(__import__("os").environ.get("FFC_BN_FOLD_MAX", "4096"))
# the SE means of a layer's global input taken from the previous layer's BN-apply pass (plane sums
# written as it stores y) instead of a second read of y (FFC_SE_SUMS=0: se_mean_kernel)
SE_SUMS = __import__("os").environ.get("FFC_SE_SUMS", "1") != "0"


def plane_sums_for(x):
    """(sums, chunks) attached to x by the BN-apply pass that wrote it, if x is unchanged since"""
    at = getattr(x, "_ffc_plane_sums", None)
    if at is None or not SE_SUMS:
        return None
    sums, chunks, version = at
    return (sums, chunks) if x._version == version else None


# the fused ST prologue over several workgroups per sample at small batches (FFC_ST_SPLIT=0: one)
ST_SPLIT = __import__("os").environ.get("FFC_ST_SPLIT", "1") != "0"


def _pow2_floor(v: int) -> int:
    """the largest power of two <= max(v, 1) (the prologue split must divide conv1's tile count)"""
    v = max(int(v), 1)
    return 1 << (v.bit_length() - 1)


# cap, rounded to 2^k: 2 since the SE gate went thread-per-channel (B = 32: 0.1755 -> 0.1731 ms with 4
# instead of 8, profiles/r05/an; B = 64 0.2105 -> 0.2092 ms with 2 instead of 4, r05/av; r04 had
# measured them level)
# (FFC_ST_SPLIT_MAX fixes it for every batch).  Round 6: 4 at B <= 32 -- the per-rank batch of the
# 8-way strong split -- B = 32 0.1790 / 0.1798 -> 0.1771 / 0.1774 ms (8: 0.1774 / 0.1777), B = 64 level
# (profiles/r06/st)
_ST_SPLIT_ENV = __import__("os").environ.get("FFC_ST_SPLIT_MAX")
ST_SPLIT_MAX = _pow2_floor(_ST_SPLIT_ENV) if _ST_SPLIT_ENV else 0   # 0: by batch (st_split_max)


def st_split_max(B: int) -> int:
    """the ST prologue's cap on workgroups per sample at batch B"""
    if ST_SPLIT_MAX:
        return ST_SPLIT_MAX
    return 4 if B <= 32 else 2
# ST prologue conv1 on the split-bf16 MFMA products (FFC_ST_MFMA=f32: the exact f32-input MFMA, A/B)
ST_SPLIT_MFMA = __import__("os").environ.get("FFC_ST_MFMA", "split") != "f32"
# the fused FU's pass 1 reads pass 0's mix output instead of recomputing it (FFC_FU_SPILL=0: recompute)
FU_SPILL = __import__("os").environ.get("FFC_FU_SPILL", "1") != "0"


class BnFoldDesc:
    """an ffc_bn_fold for ``bn`` over the partial rows ``slab`` plus the tensors it points at;
    scale / shift receive the folded affine (written by the consumer's workgroup 0)"""

    def __init__(self, bn: nn.BatchNorm2d, C: int, slab, nrows: int, count_mult: float, device, moments=None):
        _, update = bn_mode(bn)
        self.slab = slab
        # SyncBN: the slab's raw moments, reduced and all-reduced over the ranks already ([C][3] fp64,
        # ffc_bn_fold.moments); the consumer finalizes from them
        self.moments = moments
        self.channel_only = False   # made by bn_fold_channels: too many rows for a whole-slab fold
        self.scale = torch.empty(C, device=device, dtype=torch.float32)
        self.shift = torch.empty(C, device=device, dtype=torch.float32)
        self.bn = bn
        self.struct = _lib.BnFold(
            ptr(slab), int(nrows), int(C),
            ptr(bn.weight.detach()) if bn.weight is not None else None,
            ptr(bn.bias.detach()) if bn.bias is not None else None,
            ptr(bn.running_mean) if update else None, ptr(bn.running_var) if update else None,
            ptr(bn.num_batches_tracked) if update else None, int(update),
            -1.0 if bn.momentum is None else float(bn.momentum), float(bn.eps), float(count_mult),
            ptr(self.scale), ptr(self.shift), ptr(moments) if moments is not None else None)

    def materialize(self, stream):
        """(scale, shift) by the separate reduce + finalize launch (consumers without a fold)"""
        if self.moments is not None:   # SyncBN: only the finalize is left (the moments are merged)
            bn, C = self.bn, self.struct.C
            _, update = bn_mode(bn)
            check(lib().ffc_bn_finalize(ptr(self.moments), C, ptr(bn.weight.detach()) if bn.weight is not None else None,
                                        ptr(bn.bias.detach()) if bn.bias is not None else None,
                                        ptr(bn.running_mean) if bn.running_mean is not None else None,
                                        ptr(bn.running_var) if bn.running_var is not None else None,
                                        ptr(bn.num_batches_tracked) if bn.num_batches_tracked is not None else None,
                                        1, int(update), -1.0 if bn.momentum is None else float(bn.momentum),
                                        float(bn.eps), float(self.struct.count_mult), ptr(self.scale),
                                        ptr(self.shift), stream), "ffc_bn_finalize")
            return self.scale, self.shift
        return bn_scale_shift(self.bn, self.struct.C, self.slab, self.struct.nrows, self.struct.count_mult,
                              self.scale.device, stream)


def _bn_fold_synced(bn: nn.BatchNorm2d, C: int, slab, nrows: int, count_mult: float, device, grp):
    """SyncBN: the slab's raw moments by ffc_bn_reduce, all-reduced over ``grp``
    (RCCL), handed to the consumer kernel as a moments fold -- its workgroups finalize in-kernel, so
    the separate ffc_bn_finalize launch of the N > 1 path goes away"""
    if bn.num_features != C:
        raise RuntimeError(f"running_mean should contain {C} elements not {bn.num_features}")
    L = lib()
    stream = torch.cuda.current_stream(device).cuda_stream
    mbuf = torch.empty(3 * C + L.ffc_bn_reduce_ws_doubles(nrows, C), device=device, dtype=torch.float64)
    from .distributed import merge_moments
    with observe("bn_stats"):
        check(L.ffc_bn_reduce(ptr(slab), nrows, C, ptr(mbuf), stream), "ffc_bn_reduce")
        merge_moments(mbuf[:3 * C].view(C, 3), group=grp)
    return BnFoldDesc(bn, C, slab, nrows, count_mult, device, moments=mbuf)


def bn_fold(bn: nn.BatchNorm2d, C: int, slab, nrows: int, count_mult: float, device):
    """a BnFoldDesc when ``bn`` can be finalized inside its consumer (batch statistics, one rank),
    else None (use bn_scale_shift)"""
    use_batch, _ = bn_mode(bn)
    if not (BN_FOLD and use_batch and slab is not None):
        return None
    grp = _sync_group()
    if grp is not None:
        return _bn_fold_synced(bn, C, slab, nrows, count_mult, device, grp) if BN_FOLD_SYNC else None
    if nrows * C > BN_FOLD_MAX:   # every consumer workgroup merges all rows: only small slabs pay
        return None
    if bn.num_features != C:
        raise RuntimeError(f"running_mean should contain {C} elements not {bn.num_features}")
    return BnFoldDesc(bn, C, slab, nrows, count_mult, device)


# SyncBN: reduce + all-reduce the moments, then finalize inside the consumer (ffc_bn_fold.moments)
# instead of a separate ffc_bn_finalize launch (FFC_BN_FOLD_SYNC=0: the old path, A/B)
BN_FOLD_SYNC = __import__("os").environ.get("FFC_BN_FOLD_SYNC", "1") != "0"


# Per-channel in-kernel folds (ffc::bn_fold_channels): consumers whose workgroups / waves need only
# one or a few channels (the staged Fourier unit's r2c / c2r, the fused FU's split pass 1) merge just
# those channels' slab rows -- cheap at any channel count, so the limit is the rows a lane merges.
# FFC_BN_CHFOLD=0 restores the separate finalize launches (A/B); FFC_BN_CHFOLD_LOADS: max slab rows
# per lane.
# Off by default since round 6 (FFC_BN_CHFOLD=1 turns it on): the same fold placed inside
# ffc_fu2d_r2c_mix was reproduced non-deterministic in round 6 (T of whole channels
# wrong in co-resident workgroups, 39 of 40 repeated forwards) and its mechanism is not isolated, so
# the single-rank path finalizes these BNs by their own launch (B = 32: +3 %, B = 256: neutral, r05c)
BN_CHFOLD = __import__("os").environ.get("FFC_BN_CHFOLD", "0") == "1"
BN_CHFOLD_LOADS = int(__import__("os").environ.get("FFC_BN_CHFOLD_LOADS", "16"))
BN_CHFOLD_READS = int(__import__("os").environ.get("FFC_BN_CHFOLD_READS", "16384"))
# mirrors fu_kernels.hip fu_split_on(): FFC_FU_SPLIT=0 runs the fused FU's pass 1 as one workgroup per
# sample, which folds a mix BN over its whole slab (bn_fold_block) -- a channel-only fold descriptor
# (the split pass 1's) must not reach it
FU_SPLIT = __import__("os").environ.get("FFC_FU_SPLIT", "1")[:1] != "0"
# fused FU pass 0 over two bin groups per sample where the library takes them (ffc_fu_kgroups, round
# 6; off unless FFC_FU_KGROUPS=2, which the library reads too -- measured neutral to slower);
# FU_KGROUPS = False keeps one workgroup per sample even then
FU_KGROUPS = True


def bn_fold_channels(bn: nn.BatchNorm2d, C: int, slab, nrows: int, count_mult: float, device, lanes: int = 64,
                     consumers: int = 1):
    """a BnFoldDesc for a per-channel in-kernel fold (``lanes`` lanes merge one channel's rows), or
    None: batch statistics on one rank only, momentum not None (the per-channel leaders cannot read
    num_batches_tracked while another bumps it), at most BN_CHFOLD_LOADS rows per lane, and at most
    BN_CHFOLD_READS slab rows read per channel over its ``consumers`` workgroups (at fgan128's
    B = 512 every 64^2 C2R plane workgroup re-read 1024 rows: C2R 798 -> 1046 us per step, r05l)"""
    use_batch, _ = bn_mode(bn)
    if not (BN_FOLD and BN_CHFOLD and use_batch and slab is not None) or bn.momentum is None:
        return None
    grp = _sync_group()
    if grp is not None:   # moments: every consumer reads 3 doubles per channel, no row gating
        if not BN_FOLD_SYNC:
            return None
        d = _bn_fold_synced(bn, C, slab, nrows, count_mult, device, grp)
        d.channel_only = True
        return d
    if -(-nrows // lanes) > BN_CHFOLD_LOADS or nrows * max(1, consumers) > BN_CHFOLD_READS:
        return None
    if bn.num_features != C:
        raise RuntimeError(f"running_mean should contain {C} elements not {bn.num_features}")
    d = BnFoldDesc(bn, C, slab, nrows, count_mult, device)
    d.channel_only = True
    return d


def act_code(mod: nn.Module):
    """activation module -> (FFC_ACT_* code, parameter).  layers/ffc/ffc_bn_act.py:63-67."""
    if isinstance(mod, nn.Identity):
        return 0, 0.0
    if isinstance(mod, nn.LeakyReLU):
        return 2, float(mod.negative_slope)
    if isinstance(mod, nn.ReLU):
        return 1, 0.0
    if isinstance(mod, nn.Tanh):
        return 3, 0.0
    if isinstance(mod, nn.Sigmoid):
        return 4, 0.0
    if isinstance(mod, nn.GELU) and getattr(mod, "approximate", "none") == "none":
        return 5, 0.0
    raise NotImplementedError(f"activation {type(mod).__name__} has no fused HIP epilogue")


def bn_act_apply(x, scale, shift, act, param, out=None):
    B, C = x.shape[:2]
    HW = x.numel() // (B * C)
    out = x if out is None else out
    with observe("bn_act", bytes=8.0 * x.numel()):
        check(lib().ffc_bn_act_apply(ptr(x), ptr(out), B, C, HW, ptr(scale), ptr(shift), act, float(param),
                                     stream_of(x)), "ffc_bn_act_apply")
    return out


def bn_act_noise_apply(x, scale, shift, act, param, noise_mod, noise=None):
    """x <- act(x*scale + shift) + noise_mod.weight[c] * noise[b] in one pass (noise drawn with normal_()
    as layers/noise_injection.py:26-28 does when not given)"""
    B, C, H, W = x.shape
    if noise is None:
        noise = x.new_empty(B, 1, H, W).normal_()
    noise = require(noise, "noise")
    if tuple(noise.shape) != (B, 1, H, W):
        raise RuntimeError(f"noise must be {(B, 1, H, W)}, got {tuple(noise.shape)}")
    w = require(noise_mod.weight.detach(), "NoiseInjection.weight")
    if w.numel() != C:
        raise RuntimeError(f"NoiseInjection has {w.numel()} channels, tensor has {C}")
    with observe("bn_act_noise", bytes=8.0 * x.numel() + 4.0 * noise.numel()):
        check(lib().ffc_bn_act_noise_apply(ptr(x), ptr(x), B, C, H * W, ptr(scale), ptr(shift), act, float(param),
                                           ptr(w), ptr(noise), stream_of(x)), "ffc_bn_act_noise_apply")
    return x


class PendingAct:
    """A branch output whose BN + activation (+ NoiseInjection) has not been applied yet: the consumer
    applies it while staging its operand (ffc_in_tf), so the separate read + write pass of the whole
    tensor disappears.  ``materialize()`` runs that pass instead (for consumers without the option).
    The noise is drawn when the pending value is created, in the order the eager path draws it."""

    def __init__(self, raw, scale, shift, act, param, noise_mod=None, noise=None):
        B, C, H, W = raw.shape
        self.raw, self.scale, self.shift, self.act, self.param = raw, scale, shift, int(act), float(param)
        self.noise_w = self.noise = None
        if noise_mod is not None:
            if noise is None:
                noise = raw.new_empty(B, 1, H, W).normal_()
            noise = require(noise, "noise")
            if tuple(noise.shape) != (B, 1, H, W):
                raise RuntimeError(f"noise must be {(B, 1, H, W)}, got {tuple(noise.shape)}")
            w = require(noise_mod.weight.detach(), "NoiseInjection.weight")
            if w.numel() != C:
                raise RuntimeError(f"NoiseInjection has {w.numel()} channels, tensor has {C}")
            self.noise_w, self.noise = w, noise
        self.shape = raw.shape

    @classmethod
    def from_tensors(cls, raw, scale, shift, act, param, noise_w=None, noise=None):
        """a PendingAct from its tensors (the outputs / inputs of the deferred ffc::ffc_bn_act op)"""
        p = cls(raw, scale, shift, act, param)
        p.noise_w, p.noise = noise_w, noise
        return p

    def struct(self):
        from ._lib import InTf
        return InTf(ptr(self.scale), ptr(self.shift), self.act, self.param, ptr(self.noise_w), ptr(self.noise))

    def materialize(self):
        x = self.raw
        if self.noise is not None:
            with observe("bn_act_noise", bytes=8.0 * x.numel() + 4.0 * self.noise.numel()):
                B, C, H, W = x.shape
                check(lib().ffc_bn_act_noise_apply(ptr(x), ptr(x), B, C, H * W, ptr(self.scale), ptr(self.shift),
                                                   self.act, self.param, ptr(self.noise_w), ptr(self.noise),
                                                   stream_of(x)), "ffc_bn_act_noise_apply")
            return x
        return bn_act_apply(x, self.scale, self.shift, self.act, self.param)


def materialize(x):
    """PendingAct -> tensor (other values unchanged); tuples element-wise"""
    if type(x) is tuple:
        return tuple(materialize(v) for v in x)
    return x.materialize() if isinstance(x, PendingAct) else x


# --------------------------------------------------------------------------- packed-weight keys
# Packed forms of weights (GEMM A panels, transposed mix / conv1 / Linear weights) are cached by
# (pointer, version, epoch).  The custom ops (ops.py) are functional: the weights arrive as op
# arguments, and one op's plan cache serves every module with the same structure.  Pointer +
# version alone would then hit stale packs when a freed model's weight memory is reused by a new
# model's weight at the same version count, so each weight tensor OBJECT (the view's base for
# views) gets an epoch the first time an op sees it; a new object at a recycled address gets a
# new epoch and is re-packed.
_EPOCH = {"next": 1, "by_id": {}, "by_ptr": {}}
_EPOCH_LOCK = __import__("threading").Lock()


def note_tensors(ts):
    """register the weight tensors an op was called with (see weight_key)"""
    import weakref
    with _EPOCH_LOCK:
        by_id, by_ptr = _EPOCH["by_id"], _EPOCH["by_ptr"]
        for t in ts:
            if t is None or not isinstance(t, torch.Tensor):
                continue
            a = t._base if t._base is not None else t
            e = by_id.get(id(a))
            if e is None or e[0]() is not a:
                k = id(a)
                e = (weakref.ref(a, lambda _r, k=k: _EPOCH["by_id"].pop(k, None)), _EPOCH["next"])
                _EPOCH["next"] += 1
                by_id[k] = e
            by_ptr[t.data_ptr()] = (e[0], e[1])


def weight_key(t):
    """cache key of a weight's packed form: (pointer, version, epoch of the live tensor object noted at
    that pointer; 0 when none is alive there)"""
    if t is None:
        return None
    p = t.data_ptr()
    e = _EPOCH["by_ptr"].get(p)
    a = e[0]() if e is not None else None
    return p, t._version, e[1] if a is not None and a.data_ptr() == p else 0


def _wkey(ts):
    return tuple(weight_key(t) for t in ts)


class StreamPool:
    """Objects that own device buffers (layer templates with their plan caches, packed weights and
    split-K partials; the conv_layer plan cache) handed to ONE caller at a time.

    Concurrent callers -- nn.DataParallel-style threads, each on its own stream (SURVEY.md §8b
    "Threading", /root/reference/train_cond.py:66-68) -- get different objects, and the pool's lock
    covers only the check-out and the return, never the launches.  An object's previous holder may
    have been another thread whose kernels are still queued on ITS stream and read or write the
    object's buffers, so a caller that takes an object last used by another thread makes its current
    stream wait for that stream first.  One thread alone never records or waits on anything (graph
    capture and the timed loops are unaffected)."""

    def __init__(self, factory):
        import threading
        self._factory = factory
        self._free, self._all = [], []
        self._lock = threading.Lock()
        self._last = {}   # id(object) -> (thread id, stream) of its previous holder

    def take(self):
        import threading
        me = threading.get_ident()
        with self._lock:
            obj = self._free.pop() if self._free else None
        if obj is None:
            obj = self._factory()   # built outside the lock (only this caller can see it)
            with self._lock:
                self._all.append(obj)
        last = self._last.get(id(obj))
        if last is not None and last[0] != me:
            cur = torch.cuda.current_stream()
            if torch.cuda.is_current_stream_capturing():
                # a wait on an event recorded outside the capture invalidates it, and so does a host
                # synchronise from the capturing thread (measured r06d): nothing is done
                # here -- graphs.capture_step synchronises the device before it captures, so the
                # previous holder's kernels have retired
                pass
            else:
                cur.wait_stream(last[1])
        return obj

    def give(self, obj):
        import threading
        if torch.cuda.is_initialized():
            self._last[id(obj)] = (threading.get_ident(), torch.cuda.current_stream())
        with self._lock:
            self._free.append(obj)

    @property
    def instances(self) -> int:
        return len(self._all)

    def first(self):
        """an object of the pool for read-only inspection (built if none exists yet)"""
        with self._lock:
            if self._all:
                return self._all[0]
        obj = self.take()
        self.give(obj)
        return obj

    class _Hold:
        def __init__(self, pool):
            self.pool = pool

        def __enter__(self):
            self.obj = self.pool.take()
            return self.obj

        def __exit__(self, *exc):
            self.pool.give(self.obj)
            return False

    def hold(self):
        """``with pool.hold() as obj:`` -- obj held exclusively for the block"""
        return StreamPool._Hold(self)


class PackCache:
    """a few packed forms of weights, keyed by weight_key of their sources (FIFO-bounded)"""

    def __init__(self, cap: int = 16):
        self.cap, self.d = cap, {}

    def get(self, tag, sources, build):
        key = (tag,) + _wkey(sources)
        v = self.d.get(key)
        if v is None:
            if len(self.d) >= self.cap:
                self.d.pop(next(iter(self.d)))
            v = self.d[key] = build()
        return v


# --------------------------------------------------------------------------- convolution jobs


def plan_knobs():
    """the module-level switches plans depend on (tests and A/B runs flip them): part of every plan
    cache key, so a changed switch never meets a plan made under another setting"""
    return (USE_PATCH, PW_KERNEL, CONV_ARITH, PRESPLIT_A, USE_CONVQ, CONVQ_FORCE, USE_OUTER, USE_SMALLM, FORCE_FU2D,
            FU_PATH, FU_FUSED_MIN_BATCH, FU_COLS, FU2D_SPILL, OVERLAP_SPECTRAL, BN_FOLD, BN_FOLD_MAX, FU_SPILL, ST_PATH,
            ST_SPLIT, ST_SPLIT_MAX, SE_SUMS, BN_CHFOLD, BN_CHFOLD_LOADS, BN_CHFOLD_READS, ST_SPLIT_MFMA, FU2D_R2CMIX,
            FU_SPLIT, _plan.CONVQ_TCMAX, FU_KGROUPS, BN_FOLD_SYNC)


def algorithmic_flops(plan) -> float:
    """exact multiply-adds x2 of the job: every (output pixel, in-bounds tap, channel) triple"""
    total = 0
    phases = plan.phases
    for pi, ph in enumerate(phases):
        if isinstance(ph, dict):
            ent = plan.ktab[ph["kt_off"]: ph["kt_off"] + ph["K"]]
            PH, PW = ph["PH"], ph["PW"]
        else:
            ent = plan.ktab[plan.kt_off[pi]: plan.kt_off[pi] + ph.K]
            PH, PW = ph.PH, ph.PW
        for sx, oy, ox, _ in ent:
            seg = sx & 15
            if seg == 15:
                continue
            sg = plan.segs[seg]
            my_, mx_ = plan.mults[seg]
            ny = sum(1 for m in range(PH) if 0 <= m * my_ + oy < sg.IH)
            nx = sum(1 for m in range(PW) if 0 <= m * mx_ + ox < sg.IW)
            total += ny * nx
    return 2.0 * total * plan.B * plan.M


USE_PATCH = True   # LDS-patch kernel where it applies (tests flip this to cover the generic kernel)
# 1x1-only jobs of the training path: "pw" = ffc_pw_forward (tiled GEMM), "patch" / "gemm" = the
# conv kernels (A/B measurements, tests)
PW_KERNEL = __import__("os").environ.get("FFC_PW_KERNEL", "pw")


def pick_pw_cfg(B, M, Q):
    """largest ffc_pw_forward tile that still gives >= 512 workgroups (2 per CU), else the smallest"""
    cands = (0, 1, 2) if M > 64 else (1, 2)
    for c in cands:
        if lib().ffc_pw_tiles(M, B, Q, c) >= 512:
            return c
    return 2
# LDS-patch conv products: "split" = fp32-accurate split-bf16 MFMA (three exact bf16 pieces per
# operand, six piece products), "f32" = v_mfma_f32_32x32x2_f32 (A/B measurements, tests)
CONV_ARITH = __import__("os").environ.get("FFC_CONV_ARITH", "split")
PRESPLIT_A = __import__("os").environ.get("FFC_CONVP_PRESPLIT", "0") == "1"   # A/B knob: A3 planes (off: measured neutral / -1 %)
# stride-2 transposed-conv jobs on ffc_convq_forward (operands split once while staged, warp-specialised,
# persistent workgroups) under the split-bf16 products: taken wherever it plans ("auto" / "1" / "force");
# "0" never (convp for everything, A/B measurements).  Until r02 it lost to convp on large grids; the
# persistent grid (r03) reversed that (tools/convq_probe.py)
USE_CONVQ = __import__("os").environ.get("FFC_CONVQ", "auto") != "0"
CONVQ_FORCE = __import__("os").environ.get("FFC_CONVQ", "auto") in ("1", "force")
USE_OUTER = True   # ConvT on a 1x1 input as one outer-product GEMM (ffc._FFCExec._outer_rewrite)
USE_SMALLM = True  # direct VALU ConvT for <= 4 output channels (ffc_convt_k4s2_smallm)
FORCE_FU2D = False  # large-plane FU stages even where the fused per-sample FU applies (tests)
# SpectralTransform prologue: "auto" = the fused per-sample kernel where the sample fits in LDS
# (st_prologue.hip), else SE gate + gated 1x1 GEMM (st_pw.hip); "pw" forces the latter (A/B runs)
ST_PATH = __import__("os").environ.get("FFC_ST_PATH", "auto")
# Fourier-unit path where both apply: the fused one-workgroup-per-sample kernel fills the chip only
# with B >= ~CUs/4 samples; smaller batches run the staged kernels, which spread every sample over
# many workgroups.  "auto" | "fused" | "staged".  The threshold was 128 until the fused mix ran on
# pre-split weights (r05ad); gen64 B = 64 then measured 0.2161 -> 0.2147 ms fused (r05af)
FU_PATH = __import__("os").environ.get("FFC_FU_PATH", "auto")
FU_FUSED_MIN_BATCH = 64
FU_COLS = True      # staged FU: inverse column FFT fused into mix pass 1, rows-only C2R (H in 32..128)
# staged FU, batch-statistics BN: pass 0 spills the raw Y and the whole-plane C2R applies BN + ReLU on
# load (no second mix); FFC_FU2D_SPILL=0 keeps the two-pass mix
FU2D_SPILL = __import__("os").environ.get("FFC_FU2D_SPILL", "1") != "0"
# staged FU with the spill on small t planes (h in {8, 16}, C in {16, 32}): the R2C inside mix pass 0
# (ffc_fu2d_r2c_mix: one launch instead of two); FFC_FU2D_R2CMIX=0 keeps the separate R2C
FU2D_R2CMIX = __import__("os").environ.get("FFC_FU2D_R2CMIX", "1") != "0"
# Run SpectralTransform's kernels on a side stream beside the local-branch GEMM of the same FFC
# layer ("gemm-first" / "spectral-first": which is issued first).  Off by default: measured on
# MI355X (B=256 generator) 10-18 % slower than one launch pairing the local and global GEMMs,
# because the FU / ST kernels' LDS footprint cannot co-reside with the GEMM workgroups and the
# separate GEMM launches lose the heavy/light tile pairing.
OVERLAP_SPECTRAL = __import__("os").environ.get("FFC_OVERLAP", "off")
if OVERLAP_SPECTRAL in ("0", "off", "false"):
    OVERLAP_SPECTRAL = False

_SIDE = {}


def side_stream(device):
    """one side stream per device (created once, outside any graph capture of later steps)"""
    key = str(device)
    s = _SIDE.get(key)
    if s is None:
        s = _SIDE[key] = torch.cuda.Stream(device=device)
    return s


class ConvExec:
    """One planned + packed job: output = sum of segment convolutions of fixed shapes.

    kind 'patch' -> ffc_convp_forward (LDS input patch, all phases per workgroup),
    kind 'gemm'  -> ffc_conv_forward (generic phase GEMM with gathered B)."""

    def __init__(self, B, M, segs, weights, device, pw_ok=False, convq_cfg=None):
        pw_only = all(sg.kind == "pw" and not sg.pool and not sg.gate for sg in segs)
        pp = (_plan.pick_patch_cfg(B, M, segs, 128 if CONV_ARITH == "split" else 512)
              if USE_PATCH and not (pw_only and PW_KERNEL == "gemm") else None)
        if USE_PATCH and USE_CONVQ and CONV_ARITH == "split" and not pw_only and convq_cfg is not None:
            pp = _plan.plan_convq_job(B, M, segs, convq_cfg) or pp   # the launch group's common cfg
        elif USE_PATCH and USE_CONVQ and CONV_ARITH == "split" and not pw_only:
            # persistent convq (r03) measured faster than convp on every timed stride-2 shape, large
            # grids included (profiles/r03/r03g_probe_fgan128_*.log); convp stays for what it cannot plan
            pp = _plan.pick_convq_cfg(B, M, segs) or pp
        if pw_ok and pw_only and PW_KERNEL == "pw":
            self.kind, self.plan = "pw", _plan.plan_job(B, M, segs)
            self.launch_key = ("pw", pick_pw_cfg(B, M, self.plan.OH * self.plan.OW))
        elif pp is not None:
            self.kind, self.plan = "patch", pp
            self.launch_key = ("q" if pp.q else "patch", pp.cfg)
        else:
            self.kind, self.plan = "gemm", _plan.plan_job(B, M, segs)
            self.launch_key = ("gemm",)
        self.device = device
        self.ktab = torch.from_numpy(self.plan.ktab.copy()).to(device)
        # + tail padding: the patch kernel loads all 4 tap groups of a chunk, used or not
        self.a_floats = max(1, self.plan.a_size) + 256
        # split-bf16 patch conv: A pre-split into three exact bf16 planes (ffc_split_bf16) after every
        # pack, so the kernel loads the pieces instead of splitting each chunk's A in registers
        self.a3_stride = -(-self.a_floats // 8) * 8
        self.use_a3 = self.kind == "patch" and CONV_ARITH == "split" and (PRESPLIT_A or self.plan.q)
        self.has_bias = any(w[4] is not None for w in weights)
        self.M = M
        # packed buffers per weight identity: modules of one structure share this plan,
        # and alternating them must neither re-pack every call nor overwrite a buffer in use
        self._slots = {}   # identity -> (key, A, A3, bias)
        self._packed = None
        self.A = self.A3 = self.bias = None
        self.flops = algorithmic_flops(self.plan)
        self.ensure_packed(weights)

    PACK_SLOTS = 4   # distinct weight sets kept packed per plan

    def _new_buffers(self):
        A = torch.zeros(self.a_floats, device=self.device, dtype=torch.float32)
        A3 = torch.zeros(3 * self.a3_stride, device=self.device, dtype=torch.int16) if self.use_a3 else None
        bias = torch.empty(self.M, device=self.device, dtype=torch.float32) if self.has_bias else None
        return A, A3, bias

    def check_launch(self, inputs, out, addend=None):
        """host-side launch guard: the tensors must have exactly the extents this plan was made for.
        The C ABI takes raw pointers and cannot check them, so a plan reused for another shape (a
        cache-key collision: DESIGN.md §10b) would write past ``out`` instead of failing."""
        pl = self.plan
        want = (pl.B, pl.M, pl.OH, pl.OW)

        def fits(t, n):   # (B, ...) fp32, dense, exactly n elements (a view such as (B, M, k, k) for
            return (t.dim() >= 1 and t.shape[0] == pl.B and t.numel() == n and t.is_contiguous()   # (B, M k k, 1, 1)
                    and t.dtype == torch.float32)
        n_out = pl.B * pl.M * pl.OH * pl.OW
        if not fits(out, n_out):
            raise FFCError(f"conv launch guard: output {tuple(out.shape)} ({out.dtype}, contiguous="
                           f"{out.is_contiguous()}) does not match the plan's {want}")
        if addend is not None and not fits(addend, n_out):
            raise FFCError(f"conv launch guard: addend {tuple(addend.shape)} does not match the plan's {want}")
        if len(inputs) != len(pl.segs):
            raise FFCError(f"conv launch guard: {len(inputs)} inputs for {len(pl.segs)} segments")
        for i, ((x, gate), sg) in enumerate(zip(inputs, pl.segs)):
            n_in = pl.B * sg.C * sg.IH * sg.IW * (4 if sg.pool else 1)   # pooled: the 2x2-pool input
            if not fits(x, n_in):
                raise FFCError(f"conv launch guard: segment {i} input {tuple(x.shape)} (contiguous="
                               f"{x.is_contiguous()}) does not match the plan's ({pl.B}, {sg.C}, "
                               f"{sg.IH * (2 if sg.pool else 1)}, {sg.IW * (2 if sg.pool else 1)})")
            if gate is not None and gate.numel() != pl.B * sg.C:
                raise FFCError(f"conv launch guard: segment {i} gate has {gate.numel()} values, "
                               f"the plan needs {pl.B * sg.C}")

    def pack_job(self):
        """ffc_conv_job describing the packed-weight layout (used by ffc_conv_pack for both kinds)"""
        pl = self.plan
        job = _lib.ConvJob()
        job.nseg = len(pl.segs)
        job.nphase = len(pl.phases)
        job.B, job.M, job.Mpad, job.OH, job.OW, job.Sy, job.Sx = pl.B, pl.M, pl.Mpad, pl.OH, pl.OW, pl.Sy, pl.Sx
        for i, (sg, (my, mx)) in enumerate(zip(pl.segs, pl.mults)):
            sgs = job.seg[i]
            sgs.C, sgs.IH, sgs.IW, sgs.mult_y, sgs.mult_x, sgs.pool = sg.C, sg.IH, sg.IW, my, mx, int(sg.pool)
        for i, ph in enumerate(pl.phases):
            p = job.ph[i]
            if isinstance(ph, dict):
                p.py, p.px, p.PH, p.PW, p.K, p.Kpad = ph["py"], ph["px"], ph["PH"], ph["PW"], ph["K"], ph["Kpad"]
                p.a_off, p.kt_off = ph["a_off"], ph["kt_off"]
            else:
                p.py, p.px, p.PH, p.PW, p.K, p.Kpad = ph.py, ph.px, ph.PH, ph.PW, ph.K, ph.Kpad
                p.a_off, p.kt_off = pl.a_off[i], pl.kt_off[i]
        job.A = self.A.data_ptr()
        job.ktab = self.ktab.data_ptr()
        job.bias = self.bias.data_ptr() if self.bias is not None else None
        return job

    def base_job(self):
        if self.kind in ("gemm", "pw"):
            return self.pack_job()
        pl = self.plan
        job = _lib.ConvPJob()
        job.nseg = len(pl.segs)
        job.nphase = len(pl.phases)
        job.B, job.M, job.Mpad, job.OH, job.OW, job.Sy, job.Sx = pl.B, pl.M, pl.Mpad, pl.OH, pl.OW, pl.Sy, pl.Sx
        job.NS, job.TR, job.TC, job.nrb, job.ncb = pl.NS, pl.TR, pl.TC, pl.nrb, pl.ncb
        for i, sg in enumerate(pl.segs):
            s = job.seg[i]
            s.C, s.Cpad, s.IH, s.IW = sg.C, pl.cpad[i], sg.IH, sg.IW
            s.mult_y, s.mult_x = pl.mults[i]
            s.org_y, s.org_x = pl.org[i]
            s.PR, s.PC = pl.prc[i][0], pl.rowlen[i]
            s.pool = int(sg.pool)
            s.vec4 = int(pl.vec4[i])
            s.cc = pl.cc[i]
            s.direct = int(pl.direct[i]) if pl.q else 0
            if pl.q:
                s.qrow, s.qsample = pl.qstride[i]
        for i, ph in enumerate(pl.phases):
            p = job.ph[i]
            p.py, p.px, p.PH, p.PW, p.Kpad, p.a_off = ph["py"], ph["px"], ph["PH"], ph["PW"], ph["Kpad"], ph["a_off"]
            for si in range(len(pl.segs)):
                p.T[si], p.kseg[si], p.tap_h[si] = ph["T"][si], ph["kseg"][si], ph["tap_h"][si]
                for t in range(min(ph["T"][si], 8)):
                    p.tap[si][t] = int(pl.taptab[ph["tap_base"][si] + t])
        job.A = self.A.data_ptr()
        job.bias = self.bias.data_ptr() if self.bias is not None else None
        if self.A3 is not None:
            job.A3, job.a3_stride = self.A3.data_ptr(), self.a3_stride
        return job

    def ensure_packed(self, weights):
        key = _wkey([w[0] for w in weights] + [w[4] for w in weights])
        if key == self._packed:
            return
        # identity = the weight objects (pointer, epoch) without their versions: an updated weight
        # re-packs into its own slot, another model's weights get a slot of their own
        ident = tuple(None if k is None else (k[0], k[2]) for k in key)
        slot = self._slots.pop(ident, None)
        if slot is not None and slot[0] == key:
            self._slots[ident] = slot
            _, self.A, self.A3, self.bias = slot
            self._packed = key
            return
        if slot is not None:
            bufs = slot[1:]
        elif len(self._slots) >= self.PACK_SLOTS:
            bufs = self._slots.pop(next(iter(self._slots)))[1:]   # oldest slot's buffers
        else:
            bufs = self._new_buffers()
        self.A, self.A3, self.bias = bufs
        self._slots[ident] = (key,) + tuple(bufs)
        n = len(weights)
        job = self.pack_job()
        wp = (ctypes.c_void_p * _lib.MAX_SEG)(*[w[0].data_ptr() for w in weights], *([None] * (_lib.MAX_SEG - n)))
        lay = (ctypes.c_int * _lib.MAX_SEG)(*[w[1] for w in weights], *([0] * (_lib.MAX_SEG - n)))
        kh = (ctypes.c_int * _lib.MAX_SEG)(*[w[2] for w in weights], *([1] * (_lib.MAX_SEG - n)))
        kw = (ctypes.c_int * _lib.MAX_SEG)(*[w[3] for w in weights], *([1] * (_lib.MAX_SEG - n)))
        bp = (ctypes.c_void_p * _lib.MAX_SEG)(*[ptr(w[4]) for w in weights], *([None] * (_lib.MAX_SEG - n)))
        check(lib().ffc_conv_pack(ctypes.byref(job), wp, lay, kh, kw, bp, self.A.data_ptr(),
                                  ptr(self.bias), torch.cuda.current_stream(self.device).cuda_stream),
              "ffc_conv_pack")
        if self.A3 is not None and self.plan.q:
            # fragment-ordered split planes (one coalesced 1 KiB load per A fragment piece)
            check(lib().ffc_convq_pack_a3(ctypes.byref(self.base_job()), self.A.data_ptr(), self.A3.data_ptr(),
                                          torch.cuda.current_stream(self.device).cuda_stream), "ffc_convq_pack_a3")
        elif self.A3 is not None:
            check(lib().ffc_split_bf16(self.A.data_ptr(), self.A.numel(), self.A3.data_ptr(), self.a3_stride,
                                       torch.cuda.current_stream(self.device).cuda_stream), "ffc_split_bf16")
        self._packed = key

    def job(self, inputs, out, act=0, act_param=0.0, addend=None, stats=None):
        self.check_launch(inputs, out, addend)
        job = self.base_job()
        for i, (x, gate) in enumerate(inputs):
            if self.kind == "patch" and self.plan.vec4[i] and x.data_ptr() % 16:
                raise FFCError("patch conv: input segment is not 16-byte aligned")
            job.seg[i].x = x.data_ptr()
            job.seg[i].gate = ptr(gate)
        job.out = out.data_ptr()
        job.addend = ptr(addend)
        job.stats = ptr(stats)
        job.act = act
        job.act_param = act_param
        return job


class LaunchPlan:
    """tile table for a set of jobs of the same kind launched together"""

    def __init__(self, execs, device):
        kinds = {e.launch_key for e in execs}
        if len(kinds) != 1:
            raise ValueError("jobs of one launch must share a kernel configuration")
        self.key = kinds.pop()
        if self.key[0] == "pw":
            self.cfg = self.key[1]
            self._rows = [0 for _ in execs]
            self.ntiles = sum(lib().ffc_pw_tiles(e.plan.M, e.plan.B, e.plan.OH * e.plan.OW, self.cfg) for e in execs)
            self.tiles = None
            return
        self.ksplit, self.part, self.slots, self.nslots = 1, None, None, 0
        if self.key[0] in ("patch", "q"):
            self.cfg = self.key[1]
            if self.key[0] == "q":   # one K split for the launch's jobs (small batches: fill the CUs)
                self.ksplit = _plan.pick_convq_ksplit_group([e.plan for e in execs])
            tiles = _plan.build_patch_tiles([e.plan for e in execs], ksplit=self.ksplit)
            self._rows = [e.plan.npb * 4 for e in execs]
            if self.ksplit > 1:   # partial fragments, added by the reduce launch of ffc_convq_forward_split
                slots = _plan.convq_slot_tiles(tiles)
                self.nslots = slots.shape[0]
                n = lib().ffc_convq_split_floats(self.cfg, self.nslots, self.ksplit)
                if n <= 0:
                    raise RuntimeError("ffc_convq_split_floats: bad configuration")
                self.part = torch.empty(n, device=device, dtype=torch.float32)
                self.slots = torch.from_numpy(slots).to(device)
        else:
            self.cfg = _plan.pick_tile_cfg([e.plan.M for e in execs])
            tiles, nslots = _plan.build_tiles([e.plan for e in execs], self.cfg)
            while tiles.shape[0] < 256 and self.cfg == 0:   # too few tiles to fill 256 CUs: halve BM
                self.cfg = 1
                tiles, nslots = _plan.build_tiles([e.plan for e in execs], self.cfg)
            rpt = _plan.TILE_CFGS[self.cfg][2]
            self._rows = [n * rpt for n in nslots]
        self.ntiles = tiles.shape[0]
        self.tiles = torch.from_numpy(tiles).to(device)

    def stat_rows(self, j):
        return self._rows[j]

    def launch(self, jobs, stream, flops=0.0):
        L = lib()
        with observe("conv_gemm", flops=flops):
            if self.key[0] == "pw":
                for jb in jobs:
                    check(L.ffc_pw_forward(ctypes.byref(jb), self.cfg, stream), "ffc_pw_forward")
            elif self.key[0] == "q":
                arr = (_lib.ConvPJob * len(jobs))(*jobs)
                if self.ksplit > 1:
                    check(L.ffc_convq_forward_split(arr, len(jobs), self.tiles.data_ptr(), self.ntiles,
                                                    self.slots.data_ptr(), self.nslots, self.cfg, self.ksplit,
                                                    self.part.data_ptr(), stream),
                          "ffc_convq_forward_split")
                else:
                    check(L.ffc_convq_forward(arr, len(jobs), self.tiles.data_ptr(), self.ntiles, self.cfg, stream),
                          "ffc_convq_forward")
            elif self.key[0] == "patch":
                arr = (_lib.ConvPJob * len(jobs))(*jobs)
                cfg = self.cfg | (_lib.CONVP_EXACT_F32 if CONV_ARITH == "f32" else 0)
                check(L.ffc_convp_forward(arr, len(jobs), self.tiles.data_ptr(), self.ntiles, cfg, stream),
                      "ffc_convp_forward")
            else:
                arr = (_lib.ConvJob * len(jobs))(*jobs)
                check(L.ffc_conv_forward(arr, len(jobs), self.tiles.data_ptr(), self.ntiles, self.cfg, stream),
                      "ffc_conv_forward")


def sn_refresh(mod):
    """Run a module's torch.nn.utils.spectral_norm pre-hook (W <- W_orig / sigma, with one power
    iteration in training mode) at the point where the reference's forward would call the module
    (layers/snffc/snffc.py:23-33); the HIP path reads module.weight without calling the module.
    The power iteration stays host-driven PyTorch, as in the reference."""
    hooks = getattr(mod, "_forward_pre_hooks", None)
    if not hooks:
        return
    from torch.nn.utils.spectral_norm import SpectralNorm
    for h in hooks.values():
        if isinstance(h, SpectralNorm):
            h(mod, None)
            # keep the normalised weight in one persistent tensor updated in place: its version
            # changes every refresh, so the packed-weight caches (keyed by pointer + version) repack
            w = getattr(mod, h.name)
            buf = mod.__dict__.get("_ffc_sn_" + h.name)
            if buf is None or buf.shape != w.shape or buf.device != w.device:
                buf = w.detach().clone()
                mod.__dict__["_ffc_sn_" + h.name] = buf
            else:
                buf.copy_(w.detach())
            setattr(mod, h.name, buf)


def sn_refresh_train(mod):
    """training path: run the spectral_norm pre-hooks so ``mod.weight`` = weight_orig / sigma is a
    differentiable function of weight_orig (the reference calls the module, which does the same)"""
    hooks = getattr(mod, "_forward_pre_hooks", None)
    if not hooks:
        return
    from torch.nn.utils.spectral_norm import SpectralNorm
    for h in hooks.values():
        if isinstance(h, SpectralNorm):
            h(mod, None)


def conv_weight(mod):
    """(weight, layout, kh, kw, bias) for nn.Conv2d (layout 0) / nn.ConvTranspose2d (layout 1)."""
    w = mod.weight.detach()
    kh, kw = w.shape[2], w.shape[3]
    b = mod.bias.detach() if mod.bias is not None else None
    return (require(w, "weight"), 1 if isinstance(mod, nn.ConvTranspose2d) else 0, kh, kw,
            require(b, "bias") if b is not None else None)


def _square(v, what):
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            raise NotImplementedError(f"non-square {what} {v}")
        return int(v[0])
    return int(v)


def conv_seg(mod, x: torch.Tensor):
    """Seg for an nn.Conv2d / nn.ConvTranspose2d applied to x."""
    if mod.groups != 1:
        raise NotImplementedError("grouped convolutions are not on the FFC hot path (groups=1 in every caller)")
    if getattr(mod, "padding_mode", "zeros") != "zeros":
        raise NotImplementedError("only zero padding")
    if isinstance(mod.padding, str):
        raise NotImplementedError("string padding")
    B, C, H, W = x.shape
    if C != mod.in_channels:
        raise RuntimeError(f"expected input with {mod.in_channels} channels, got {C}")
    k = _square(mod.kernel_size, "kernel")
    s = _square(mod.stride, "stride")
    p = _square(mod.padding, "padding")
    d = _square(mod.dilation, "dilation")
    if isinstance(mod, nn.ConvTranspose2d):
        op = _square(mod.output_padding, "output_padding")
        return _plan.Seg("convT", C, H, W, k, s, p, d, op)
    return _plan.Seg("conv", C, H, W, k, s, p, d)
