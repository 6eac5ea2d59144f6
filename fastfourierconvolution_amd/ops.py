"""The custom-op boundary: every launch of the FFC hot path is reached through a ``torch.ops.ffc.*``
op registered with ``torch.library.custom_op``, over the C ABI of libffc_amd.so
(include/ffc_amd.h).  Each op has a fake (meta) implementation, so FakeTensor tracing,
``torch.export`` and ``torch.library.opcheck`` see the path; the training ops carry their backward
through ``register_autograd`` (the backward is another ffc op).

Training ops (autograd): one per op the reference's forward is made of (see _autograd.py)
  ffc::conv_layer      local convs / ConvT + ST conv2 summed per output branch, 1x1 convs, Linear
                       (ffc.py:89-97, ffc_transpose.py:96-106, spectral_transform.py:89,108,
                       fourier_unity.py:45)                        backward: ffc::conv_layer_backward
  ffc::bn_act          BatchNorm2d + activation (ffc_bn_act.py:73-81, spectral_transform.py:89,
                       fourier_unity.py:46-49)                      backward: ffc::bn_act_backward
  ffc::se_scale        SELayer (spectral_transform.py:12-28)        backward: ffc::se_scale_backward
  ffc::pool2, ffc::up2 AvgPool2d(2) / Upsample(x2) (:44-47)         backward: each other
  ffc::rfft2           rfftn(ortho) + Re/Im interleave (fourier_unity.py:38-42)   backward: ffc::irfft2
  ffc::irfft2          de-interleave + irfftn(s=(H, W), ortho) (:51-56) [+ x]     backward: ffc::rfft2
  ffc::noise_inject    NoiseInjection (layers/noise_injection.py:25-32)  backward: ffc::noise_wgrad

Inference ops (the fused kernels; used under torch.no_grad() / when nothing needs a gradient):
  ffc::ffc_bn_act      one FFC_BN_ACT / FFC / FFCTranspose layer (ffc_bn_act.py:70-83, ffc.py:84-99,
                       ffc_transpose.py:91-110): its local GEMM launch(es), SpectralTransform,
                       BN + activation (+ fgan128's NoiseInjection, + a deferred input transform)
  ffc::spectral_transform   SpectralTransform.forward (spectral_transform.py:77-110)
  ffc::fourier_unit    FourierUnitSN.forward (fourier_unity.py:32-56)
  ffc::linear          nn.Linear (fgan128_complete.py:453-455)
  ffc::quantize_u8     the fgan128 eval-mode uint8 image (fgan128_complete.py:516-521)

A layer op is a function of its arguments: the layer's structure travels as a JSON ``spec``
(constructor arguments and every submodule's mode / BN settings / activation), its parameters and
buffers as tensor lists.  The op runs the spec's *template* -- the same module class built once on
the meta device -- with the argument tensors bound in place of its parameters, so the fused
executor of ffc.py / spectral_transform.py / fourier_unity.py (plan caches, packed weights keyed by
rt.weight_key) serves every module of that structure.
"""
from __future__ import annotations

import contextlib
import functools
import io
import json
import threading
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
from torch import Tensor

from . import _autograd as ag
from . import _plan
from . import _runtime as rt

# =========================================================================== training ops
# ---------------------------------------------------------------- ffc::conv_layer


@torch.library.custom_op("ffc::conv_layer", mutates_args=())
def conv_layer(xs: List[Tensor], ws: List[Tensor], bs: List[Tensor], spec: str) -> List[Tensor]:
    return ag.conv_layer_impl(xs, ws, bs, spec)


@conv_layer.register_fake
def _(xs, ws, bs, spec):
    outs_s, edges = ag.parse_conv_spec(spec)
    outs, pres = [], []
    for j, (M, act, _) in enumerate(outs_s):
        e = next(e for e in edges if e[0] == j)
        y = xs[e[1]].new_empty(ag.conv_layer_out_shape(e, xs[e[1]], M))
        outs.append(y)
        if act == 5:
            pres.append(xs[e[1]].new_empty(y.shape))
    return outs + pres


@torch.library.custom_op("ffc::conv_layer_backward", mutates_args=())
def conv_layer_backward(xs: List[Tensor], ws: List[Tensor], ts: List[Tensor], gouts: List[Optional[Tensor]],
                        needs: List[bool], spec: str) -> List[Tensor]:
    return ag.conv_layer_backward_impl(xs, ws, ts, gouts, needs, spec)


@conv_layer_backward.register_fake
def _(xs, ws, ts, gouts, needs, spec):
    _, edges = ag.parse_conv_spec(spec)
    nb = sum(1 for e in edges if e[9] >= 0)
    srcs = list(xs) + list(ws)
    res = [t.new_empty(t.shape) if needs[k] else t.new_empty(0) for k, t in enumerate(srcs)]
    bias_ch = {}
    for e in edges:
        if e[9] >= 0:
            bias_ch[e[9]] = ws[edges.index(e)].shape[1 if e[2] == "convT" else 0]
    res += [xs[0].new_empty(bias_ch[b]) if needs[len(srcs) + b] else xs[0].new_empty(0) for b in range(nb)]
    return res


def _conv_layer_setup(ctx, inputs, output):
    xs, ws, bs, spec = inputs
    outs_s, _ = ag.parse_conv_spec(spec)
    no = len(outs_s)
    pres = iter(output[no:])
    ts = [next(pres) if act == 5 else output[j] for j, (_, act, _) in enumerate(outs_s)]
    ctx.spec, ctx.n = spec, (len(xs), len(ws), len(bs))
    ctx.needs = [bool(t.requires_grad) for t in list(xs) + list(ws) + list(bs)]
    ctx.save_for_backward(*xs, *ws, *ts)


def _conv_layer_bwd(ctx, grads):
    n_in, ne, nb = ctx.n
    saved = ctx.saved_tensors
    xs, ws, ts = list(saved[:n_in]), list(saved[n_in:n_in + ne]), list(saved[n_in + ne:])
    gouts = list(grads[:len(ts)])
    res = torch.ops.ffc.conv_layer_backward(xs, ws, ts, gouts, ctx.needs, ctx.spec)
    g = [r if need else None for r, need in zip(res, ctx.needs)]
    return g[:n_in], g[n_in:n_in + ne], g[n_in + ne:], None


conv_layer.register_autograd(_conv_layer_bwd, setup_context=_conv_layer_setup)

# ---------------------------------------------------------------- ffc::bn_act


@torch.library.custom_op("ffc::bn_act", mutates_args=())
def bn_act(x: Tensor, weight: Optional[Tensor], bias: Optional[Tensor], running_mean: Optional[Tensor],
           running_var: Optional[Tensor], use_batch: bool, eps: float, act: int, act_param: float) -> List[Tensor]:
    """functional (the running statistics are updated by ffc::bn_update_running)"""
    return ag.bn_act_impl(x, weight, bias, running_mean, running_var, use_batch, eps, act, act_param)


@bn_act.register_fake
def _(x, weight, bias, running_mean, running_var, use_batch, eps, act, act_param):
    C = x.shape[1]
    stats = x.new_empty((C, 3), dtype=torch.float64) if use_batch else x.new_empty((2, C))
    return [torch.empty_like(x), x.new_empty(C), x.new_empty(C), stats]


@torch.library.custom_op("ffc::bn_update_running",
                         mutates_args=("running_mean", "running_var", "num_batches_tracked"))
def bn_update_running(running_mean: Tensor, running_var: Tensor, num_batches_tracked: Optional[Tensor],
                      stats: Tensor, momentum: float, count_mult: float) -> None:
    """nn.BatchNorm2d's running-statistics update from the batch moments ffc::bn_act returned
    (momentum < 0: None, the cumulative average over num_batches_tracked)"""
    ag.bn_update_running_impl(running_mean, running_var, num_batches_tracked, stats, momentum, count_mult)


@bn_update_running.register_fake
def _(running_mean, running_var, num_batches_tracked, stats, momentum, count_mult):
    return None


@torch.library.custom_op("ffc::bn_act_backward", mutates_args=())
def bn_act_backward(x: Tensor, dy: Tensor, scale: Tensor, shift: Tensor, stats: Tensor, weight: Optional[Tensor],
                    use_batch: bool, sync: bool, eps: float, act: int, act_param: float, need_dx: bool,
                    has_weight: bool, has_bias: bool) -> List[Tensor]:
    return ag.bn_act_backward_impl(x, dy, scale, shift, stats, weight, use_batch, sync, eps, act, act_param,
                                   need_dx, has_weight, has_bias)


@bn_act_backward.register_fake
def _(x, dy, scale, shift, stats, weight, use_batch, sync, eps, act, act_param, need_dx, has_weight, has_bias):
    C = x.shape[1]
    return [torch.empty_like(x) if need_dx else x.new_empty(0), x.new_empty(C) if has_weight else x.new_empty(0),
            x.new_empty(C) if has_bias else x.new_empty(0)]


def _bn_act_setup(ctx, inputs, output):
    x, weight, bias, rm, rv, use_batch, eps, act, act_param = inputs
    _, scale, shift, stats = output
    ctx.mark_non_differentiable(scale, shift, stats)
    ctx.use_batch = use_batch
    ctx.sync = ctx.use_batch and rt._sync_group() is not None
    ctx.cfg = (float(eps), int(act), float(act_param))
    ctx.has = (weight is not None, bias is not None)
    ctx.need_dx = bool(x.requires_grad)
    ctx.save_for_backward(x, scale, shift, stats, weight)


def _bn_act_bwd(ctx, grads):
    x, scale, shift, stats, weight = ctx.saved_tensors
    dy = grads[0]
    if dy is None:
        return (None,) * 9
    eps, act, act_param = ctx.cfg
    dx, dw, db = torch.ops.ffc.bn_act_backward(x, dy, scale, shift, stats, weight, ctx.use_batch, ctx.sync, eps, act,
                                               act_param, ctx.need_dx, ctx.has[0], ctx.has[1])
    return (dx if ctx.need_dx else None, dw if ctx.has[0] else None, db if ctx.has[1] else None) + (None,) * 6


bn_act.register_autograd(_bn_act_bwd, setup_context=_bn_act_setup)

# ---------------------------------------------------------------- ffc::se_scale


@torch.library.custom_op("ffc::se_scale", mutates_args=())
def se_scale(x: Tensor, w1: Tensor, w2: Tensor) -> Tensor:
    return ag.se_scale_impl(x, w1, w2)


@se_scale.register_fake
def _(x, w1, w2):
    return torch.empty_like(x)


@torch.library.custom_op("ffc::se_scale_backward", mutates_args=())
def se_scale_backward(x: Tensor, dy: Tensor, w1: Tensor, w2: Tensor) -> List[Tensor]:
    return ag.se_scale_backward_impl(x, dy, w1, w2)


@se_scale_backward.register_fake
def _(x, dy, w1, w2):
    return [torch.empty_like(x), torch.empty_like(w1), torch.empty_like(w2)]


def _se_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _se_bwd(ctx, dy):
    x, w1, w2 = ctx.saved_tensors
    return tuple(torch.ops.ffc.se_scale_backward(x, dy, w1, w2))


se_scale.register_autograd(_se_bwd, setup_context=_se_setup)

# ---------------------------------------------------------------- ffc::pool2 / ffc::up2 (adjoints of each other)


@torch.library.custom_op("ffc::pool2", mutates_args=())
def pool2(x: Tensor, scale: float) -> Tensor:
    return ag.pool2_impl(x, scale)


@pool2.register_fake
def _(x, scale):
    return x.new_empty((x.shape[0], x.shape[1], x.shape[2] // 2, x.shape[3] // 2))


@torch.library.custom_op("ffc::up2", mutates_args=())
def up2(x: Tensor, scale: float) -> Tensor:
    return ag.up2_impl(x, scale)


@up2.register_fake
def _(x, scale):
    return x.new_empty((x.shape[0], x.shape[1], 2 * x.shape[2], 2 * x.shape[3]))


def _scale_setup(ctx, inputs, output):
    ctx.scale = inputs[1]


pool2.register_autograd(lambda ctx, dy: (torch.ops.ffc.up2(dy, ctx.scale), None), setup_context=_scale_setup)
up2.register_autograd(lambda ctx, dy: (torch.ops.ffc.pool2(dy, ctx.scale), None), setup_context=_scale_setup)

# ---------------------------------------------------------------- ffc::rfft2 / ffc::irfft2


@torch.library.custom_op("ffc::rfft2", mutates_args=())
def rfft2(x: Tensor, mirror_scale: float) -> Tensor:
    return ag.rfft2_impl(x, mirror_scale)


@rfft2.register_fake
def _(x, mirror_scale):
    return x.new_empty((x.shape[0], 2 * x.shape[1], x.shape[2], x.shape[3] // 2 + 1))


@torch.library.custom_op("ffc::irfft2", mutates_args=())
def irfft2(Z: Tensor, H: int, W: int, mirror_scale: float, r: Optional[Tensor]) -> Tensor:
    return ag.irfft2_impl(Z, H, W, mirror_scale, r)


@irfft2.register_fake
def _(Z, H, W, mirror_scale, r):
    return Z.new_empty((Z.shape[0], Z.shape[1] // 2, H, W))


def _rfft2_setup(ctx, inputs, output):
    x, ms = inputs
    ctx.hw, ctx.ms = (x.shape[2], x.shape[3]), ms


def _rfft2_bwd(ctx, dZ):
    if ctx.ms != 1.0:
        raise NotImplementedError("ffc::rfft2 backward: mirror_scale 1 only")
    # d/dx of rfftn(ortho): irfftn(ortho) with the mirrored bins halved
    return torch.ops.ffc.irfft2(dZ, ctx.hw[0], ctx.hw[1], 0.5, None), None


def _irfft2_setup(ctx, inputs, output):
    ctx.ms, ctx.has_r = inputs[3], inputs[4] is not None


def _irfft2_bwd(ctx, dy):
    if ctx.ms != 1.0:
        raise NotImplementedError("ffc::irfft2 backward: mirror_scale 1 only")
    # d/dZ of irfftn(ortho): rfftn(ortho) with the mirrored bins doubled
    return torch.ops.ffc.rfft2(dy, 2.0), None, None, None, (dy if ctx.has_r else None)


rfft2.register_autograd(_rfft2_bwd, setup_context=_rfft2_setup)
irfft2.register_autograd(_irfft2_bwd, setup_context=_irfft2_setup)

# ---------------------------------------------------------------- ffc::noise_inject


@torch.library.custom_op("ffc::noise_inject", mutates_args=())
def noise_inject(x: Tensor, weight: Tensor, noise: Tensor) -> Tensor:
    return ag.noise_inject_impl(x, weight, noise)


@noise_inject.register_fake
def _(x, weight, noise):
    return torch.empty_like(x)


@torch.library.custom_op("ffc::noise_wgrad", mutates_args=())
def noise_wgrad(g: Tensor, noise: Tensor) -> Tensor:
    return ag.noise_wgrad_impl(g, noise)


@noise_wgrad.register_fake
def _(g, noise):
    return g.new_empty((1, g.shape[1], 1, 1))


def _noise_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[2])
    ctx.need_w = bool(inputs[1].requires_grad)


def _noise_bwd(ctx, g):
    (noise,) = ctx.saved_tensors
    dw = torch.ops.ffc.noise_wgrad(g, noise).view(ctx.wshape) if ctx.need_w else None
    return g, dw, None


def _noise_setup_shape(ctx, inputs, output):
    _noise_setup(ctx, inputs, output)
    ctx.wshape = tuple(inputs[1].shape)


noise_inject.register_autograd(_noise_bwd, setup_context=_noise_setup_shape)

# =========================================================================== inference ops


@torch.library.custom_op("ffc::linear", mutates_args=())
def linear(z: Tensor, weight: Tensor, bias: Optional[Tensor]) -> Tensor:
    """nn.Linear on the dense HIP GEMM: z (B, K) . weight^T (K, N) + bias"""
    z = rt.require(z, "z")
    N, K = weight.shape
    if z.dim() != 2 or z.shape[1] != K:
        raise RuntimeError(f"linear: z must be (B, {K}), got {tuple(z.shape)}")
    rt.note_tensors([weight, bias])
    w = rt.require(weight.detach(), "weight")
    b = rt.require(bias.detach(), "bias") if bias is not None else None
    with _PACKS.hold() as packs:
        Wt = packs.get("linearT", [w], lambda: w.t().contiguous())
        B = z.shape[0]
        out = torch.empty((B, N), device=z.device, dtype=torch.float32)
        with rt.observe("dense", flops=2.0 * B * K * N):
            rt.check(rt.lib().ffc_dense_forward(rt.ptr(z), rt.ptr(Wt), rt.ptr(b), B, K, N, N, rt.ptr(out), None, 0,
                                                0.0, rt.stream_of(z)), "ffc_dense_forward")
    return out


@linear.register_fake
def _(z, weight, bias):
    return z.new_empty((z.shape[0], weight.shape[0]))


_PACKS = rt.StreamPool(lambda: rt.PackCache(64))   # transposed Linear weights


@torch.library.custom_op("ffc::quantize_u8", mutates_args=())
def quantize_u8(x: Tensor) -> Tensor:
    """fgan128_complete.py:516-521: the float image -> uint8 over its own global min / max"""
    x = rt.require(x, "x")
    out = torch.empty(x.shape, device=x.device, dtype=torch.uint8)
    rt.check(rt.lib().ffc_quantize_u8(rt.ptr(x), rt.ptr(out), x.numel(), rt.stream_of(x)), "ffc_quantize_u8")
    return out


@quantize_u8.register_fake
def _(x):
    return torch.empty_like(x, dtype=torch.uint8)


# ---------------------------------------------------------------- layer templates
_ACTS = {"Identity": nn.Identity, "ReLU": nn.ReLU, "LeakyReLU": nn.LeakyReLU, "Tanh": nn.Tanh,
         "Sigmoid": nn.Sigmoid, "GELU": nn.GELU, "BatchNorm2d": nn.BatchNorm2d}
_ACT_MODS = (nn.Identity, nn.ReLU, nn.LeakyReLU, nn.Tanh, nn.Sigmoid, nn.GELU)


def _module_state(m: nn.Module):
    """the per-submodule settings a layer op depends on besides its tensors"""
    out = []
    for name, sub in m.named_modules():
        e = [name, bool(sub.training)]
        if isinstance(sub, nn.BatchNorm2d):
            e += [sub.momentum, float(sub.eps), bool(sub.affine), bool(sub.track_running_stats), sub.num_features]
        elif isinstance(sub, nn.LeakyReLU):
            e += [float(sub.negative_slope)]
        elif isinstance(sub, nn.GELU):
            e += [sub.approximate]
        elif hasattr(sub, "mix_precision"):
            e += [sub.mix_precision]
        out.append(e)
    return out


def layer_spec(m: nn.Module) -> str:
    """JSON spec of a FFC_BN_ACT / FFC / FFCTranspose / SpectralTransform / FourierUnitSN module"""
    ctor = getattr(m, "_ffc_ctor", None)
    if ctor is None:
        raise NotImplementedError(f"{type(m).__name__} has no layer op")
    return json.dumps({"ctor": ctor, "state": _module_state(m)}, separators=(",", ":"))


class _Template:
    """a layer module of the spec's structure on the meta device, plus its tensor slots"""

    def __init__(self, spec: str):
        from .ffc import FFC, FFC_BN_ACT, FFCTranspose, FourierUnitSN, SpectralTransform
        d = json.loads(spec)
        kind, args = d["ctor"][0], dict(d["ctor"][1])
        cls = {"FFC_BN_ACT": FFC_BN_ACT, "FFC": FFC, "FFCTranspose": FFCTranspose,
               "SpectralTransform": SpectralTransform, "FourierUnitSN": FourierUnitSN}[kind]
        for k in ("norm_layer", "activation_layer"):
            if k in args:
                if args[k] not in _ACTS:
                    raise NotImplementedError(f"{k} {args[k]} has no HIP path")
                args[k] = _ACTS[args[k]]
        # built outside any active tracing / fake mode (a template is a cached object, not graph content)
        from torch.utils._python_dispatch import _disable_current_modes
        with _disable_current_modes(), torch.device("meta"), contextlib.redirect_stdout(io.StringIO()):
            mod = cls(**args)
        subs = dict(mod.named_modules())
        for e in d["state"]:
            name, training = e[0], e[1]
            sub = subs.get(name)
            if sub is None:
                raise NotImplementedError(f"layer op: submodule {name!r} is not part of {kind}'s structure")
            sub.training = training
            if isinstance(sub, nn.BatchNorm2d):
                sub.momentum, sub.eps = e[2], e[3]
                if not e[4]:
                    sub.weight = sub.bias = None
                if not e[5]:
                    sub.track_running_stats = False
                    sub.register_buffer("running_mean", None)
                    sub.register_buffer("running_var", None)
                    sub.register_buffer("num_batches_tracked", None)
            elif isinstance(sub, nn.LeakyReLU):
                sub.negative_slope = e[2]
            elif isinstance(sub, nn.GELU):
                sub.approximate = e[2]
            elif len(e) > 2 and hasattr(sub, "mix_precision"):
                sub.mix_precision = e[2]
        self.kind, self.module = kind, mod
        self.param_names = [n for n, _ in mod.named_parameters()]
        self.buffer_names = [n for n, _ in mod.named_buffers()]
        self._slots = [self._slot(mod, n, "_parameters") for n in self.param_names] + \
                      [self._slot(mod, n, "_buffers") for n in self.buffer_names]
        self._meta = [getattr(sub, kind)[leaf] for sub, kind, leaf in self._slots]

    @staticmethod
    def _slot(mod, name, kind):
        path, _, leaf = name.rpartition(".")
        return (mod.get_submodule(path) if path else mod), kind, leaf

    @contextlib.contextmanager
    def bound(self, params, buffers):
        """this instance with the op's tensors in place of its parameters and buffers (the caller
        holds the instance exclusively: _TemplatePool.bound)"""
        ts = list(params) + list(buffers)
        if len(ts) != len(self._slots):
            raise RuntimeError(f"layer op: {len(ts)} tensors for {len(self._slots)} slots")
        for (sub, kind, leaf), t in zip(self._slots, ts):
            getattr(sub, kind)[leaf] = t
        try:
            yield self.module
        finally:
            for (sub, kind, leaf), t in zip(self._slots, self._meta):
                getattr(sub, kind)[leaf] = t


class _TemplatePool:
    """the template instances of one spec (an rt.StreamPool).  A layer op checks an instance out for
    the whole forward -- binding, launches, unbinding -- and returns it afterwards; the pool's lock
    covers only the check-out and the return.  Concurrent callers (nn.DataParallel-style threads,
    each on its own stream: SURVEY.md §8b "Threading", /root/reference/train_cond.py:66-68) therefore
    run on different instances, and an instance's plan caches, packed weights and split-K partial
    buffers (all kept on its modules) are used by one thread at a time, in stream order."""

    def __init__(self, spec: str):
        self.spec = spec
        self.pool = rt.StreamPool(lambda: _Template(spec))
        first = self.pool.first()
        # structure shared by every instance (fake impls, layer_tensors)
        self.kind, self.module = first.kind, first.module
        self.param_names, self.buffer_names = first.param_names, first.buffer_names

    @property
    def instances(self) -> int:
        return self.pool.instances

    @contextlib.contextmanager
    def bound(self, params, buffers):
        """a template instance of this spec held exclusively, with the op's tensors bound in"""
        rt.note_tensors(params)
        with self.pool.hold() as inst, inst.bound(params, buffers) as m:
            yield m


def template(spec: str) -> _TemplatePool:
    """the spec's template pool under the current plan switches (rt.plan_knobs: the templates' plan
    caches are made under them)"""
    return _template(spec, rt.plan_knobs())


@functools.lru_cache(maxsize=512)
def _template(spec: str, knobs) -> _TemplatePool:
    return _TemplatePool(spec)


def layer_tensors(m: nn.Module, spec: str):
    """(params, buffers) of module m in its template's slot order.  Parameters are read as attributes,
    so a spectral-norm wrapped conv contributes its normalised weight (refreshed by the caller)."""
    tpl = template(spec)

    def get(name):
        path, _, leaf = name.rpartition(".")
        return getattr(m.get_submodule(path) if path else m, leaf)
    return [get(n) for n in tpl.param_names], [get(n) for n in tpl.buffer_names]


# ---------------------------------------------------------------- output shapes of a layer (fake impls)
def _conv_out_hw(conv, H, W):
    if isinstance(conv, nn.ConvTranspose2d):
        k, s, p, d, op = conv.kernel_size[0], conv.stride[0], conv.padding[0], conv.dilation[0], conv.output_padding[0]
        return _plan.convT_out(H, k, s, p, d, op), _plan.convT_out(W, k, s, p, d, op)
    k, s, p, d = conv.kernel_size[0], conv.stride[0], conv.padding[0], conv.dilation[0]
    return _plan.conv_out(H, k, s, p, d), _plan.conv_out(W, k, s, p, d)


def _st_out_shape(st, x):
    B, _, H, W = x.shape
    if st.stride == 2 and st.upsample:
        H, W = 2 * H, 2 * W
    elif st.stride == 2:
        H, W = H // 2, W // 2
    return (B, st.conv2.out_channels, H, W)


def ffc_out_shapes(ffc, x_l, x_g):
    """(shape of out_l or None, shape of out_g or None) of FFC / FFCTranspose ``ffc`` (ffc.py:84-99):
    a branch is None when it is the int 0 of the tuple protocol"""
    from .ffc.spectral_transform import SpectralTransform

    def branch(parts):
        for mod, t in parts:
            if t is None:
                continue
            if isinstance(mod, (nn.Conv2d, nn.ConvTranspose2d)):
                h, w = _conv_out_hw(mod, t.shape[2], t.shape[3])
                return (t.shape[0], mod.out_channels, h, w)
            if isinstance(mod, SpectralTransform):
                return _st_out_shape(mod, t)
            if isinstance(mod, nn.Identity):
                return tuple(t.shape)
        return None
    sl = branch([(ffc.convl2l, x_l), (ffc.convg2l, x_g)]) if ffc.ratio_gout != 1 else None
    sg = branch([(ffc.convl2g, x_l), (ffc.convg2g, x_g)]) if ffc.ratio_gout != 0 else None
    return sl, sg


# ---------------------------------------------------------------- ffc::ffc_bn_act
@torch.library.custom_op("ffc::ffc_bn_act", mutates_args=("buffers",))
def ffc_bn_act(x_l: Optional[Tensor], x_g: Optional[Tensor], params: List[Tensor], buffers: List[Tensor],
               noise: List[Tensor], pending: List[Tensor], pending_act: List[float], defer: bool,
               spec: str) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """one layer's forward.  noise: [] or NoiseInjection (weight_l, noise_l, weight_g, noise_g) applied
    after the BN + activation (fgan128_complete.py:496-515); pending: [] or the deferred BN + activation
    (+ noise) of the inputs, (scale_l, shift_l, weight_l, noise_l, scale_g, ...) with pending_act =
    (act_l, param_l, act_g, param_g) (zero-size tensors for absent parts); defer: return (raw, scale,
    shift) per output branch instead of applying BN + activation (+ noise).
    -> (out_l, out_g, scale_l, shift_l, scale_g, shift_g): zero-size tensors for the int-0 branches of
    the tuple protocol and, unless defer, for the scales / shifts (a fixed-arity tuple: the op
    mutates its buffers, and functionalization takes no list outputs beside mutated arguments)"""
    tpl = template(spec)
    with tpl.bound(params, buffers) as m:
        x_in = _pending_inputs(x_l, x_g, pending, pending_act)
        nz = None
        if noise:
            from .layers_misc import NoiseInjection
            nz = {}
            for k, (w, n) in (("l", noise[0:2]), ("g", noise[2:4])):
                if w.numel():
                    mod = NoiseInjection.__new__(NoiseInjection)
                    nn.Module.__init__(mod)
                    mod._parameters["weight"] = w
                    nz[k] = (mod, n)
        if tpl.kind == "FFC_BN_ACT":
            bn_l, bn_g = m._norm(m.bn_l), m._norm(m.bn_g)
            out = m.ffc._run(x_in, None, rt.act_code(m.act_l), rt.act_code(m.act_g), bn_l, bn_g, noise=nz,
                             defer=defer)
        else:
            out = m._run(x_in, None, noise=nz, defer=defer)
    ref = x_l if x_l is not None else x_g
    res = [ref.new_empty(0) for _ in range(6)]
    for k, o in enumerate(out):
        if isinstance(o, rt.PendingAct):
            res[k], res[2 + 2 * k], res[3 + 2 * k] = o.raw, o.scale, o.shift
        elif isinstance(o, torch.Tensor):
            res[k] = o
    return tuple(res)


def _pending_inputs(x_l, x_g, pending, pending_act):
    if not pending:
        return (x_l if x_l is not None else 0, x_g if x_g is not None else 0)
    xs = []
    for k, x in enumerate((x_l, x_g)):
        sc, sh, w, n = pending[4 * k: 4 * k + 4]
        if x is None:
            xs.append(0)
        elif sc.numel():
            xs.append(rt.PendingAct.from_tensors(x, sc, sh, int(pending_act[2 * k]), pending_act[2 * k + 1],
                                                 w if w.numel() else None, n if n.numel() else None))
        else:
            xs.append(x)
    return tuple(xs)


@ffc_bn_act.register_fake
def _(x_l, x_g, params, buffers, noise, pending, pending_act, defer, spec):
    tpl = template(spec)
    ffc = tpl.module.ffc if tpl.kind == "FFC_BN_ACT" else tpl.module
    ref = x_l if x_l is not None else x_g
    res = [ref.new_empty(0) for _ in range(6)]
    for k, shp in enumerate(ffc_out_shapes(ffc, x_l, x_g)):
        if shp is None:
            continue
        res[k] = ref.new_empty(shp)
        if defer:
            res[2 + 2 * k], res[3 + 2 * k] = ref.new_empty(shp[1]), ref.new_empty(shp[1])
    return tuple(res)


# ---------------------------------------------------------------- ffc::spectral_transform / ffc::fourier_unit
@torch.library.custom_op("ffc::spectral_transform", mutates_args=("buffers",))
def spectral_transform(x: Tensor, params: List[Tensor], buffers: List[Tensor], spec: str) -> Tensor:
    tpl = template(spec)
    with tpl.bound(params, buffers) as m:
        return m._forward_fused(x)


@spectral_transform.register_fake
def _(x, params, buffers, spec):
    return x.new_empty(_st_out_shape(template(spec).module, x))


@torch.library.custom_op("ffc::fourier_unit", mutates_args=("buffers",))
def fourier_unit(x: Tensor, params: List[Tensor], buffers: List[Tensor], spec: str) -> Tensor:
    tpl = template(spec)
    with tpl.bound(params, buffers) as m:
        return m._run(rt.require(x, "x"))


@fourier_unit.register_fake
def _(x, params, buffers, spec):
    return torch.empty_like(x)


# =========================================================================== module-facing helpers
def _refresh_sn(m: nn.Module):
    """spectral-norm pre-hooks of every conv in m, where the reference's module calls would run them"""
    for sub in m.modules():
        if isinstance(sub, (nn.Conv2d, nn.ConvTranspose2d)):
            rt.sn_refresh(sub)


def layer_forward(m: nn.Module, x, noise=None, defer=False):
    """FFC_BN_ACT / FFC / FFCTranspose inference forward through ffc::ffc_bn_act.
    noise: {"l"|"g": (NoiseInjection, noise or None)}; defer: rt.PendingAct outputs.
    -> (out_l, out_g) with the int 0 for absent branches"""
    x_l, x_g = x if type(x) is tuple else (x, 0)
    pend = []
    pact = []
    ins = []
    for v in (x_l, x_g):
        if isinstance(v, rt.PendingAct):
            ins.append(v.raw)
        elif isinstance(v, torch.Tensor):
            ins.append(rt.require(v, "x"))
        else:
            ins.append(None)
    ref = next((t for t in ins if t is not None), None)
    if ref is None:
        raise TypeError("FFC input has no tensor branch")
    e = ref.new_empty(0) if noise or any(isinstance(v, rt.PendingAct) for v in (x_l, x_g)) else None   # placeholder
    if any(isinstance(v, rt.PendingAct) for v in (x_l, x_g)):
        for v in (x_l, x_g):
            if isinstance(v, rt.PendingAct):
                pend += [v.scale, v.shift, v.noise_w if v.noise_w is not None else e,
                         v.noise if v.noise is not None else e]
                pact += [float(v.act), float(v.param)]
            else:
                pend += [e, e, e, e]
                pact += [0.0, 0.0]
    _refresh_sn(m)
    spec = layer_spec(m)
    tpl = template(spec)
    ffc = tpl.module.ffc if tpl.kind == "FFC_BN_ACT" else tpl.module
    shapes = ffc_out_shapes(ffc, ins[0], ins[1])
    nz = []
    if noise:
        for k, shp in zip(("l", "g"), shapes):
            mod, n = noise.get(k, (None, None))
            if mod is None or shp is None:
                nz += [e, e]
                continue
            if n is None:   # drawn here, in branch order, as NoiseInjection draws it (noise_injection.py:26-28)
                n = ref.new_empty((shp[0], 1, shp[2], shp[3])).normal_()
            nz += [mod.weight.detach(), rt.require(n, "noise")]
    params, buffers = layer_tensors(m, spec)
    res = torch.ops.ffc.ffc_bn_act(ins[0], ins[1], params, buffers, nz, pend, pact, bool(defer), spec)
    out = []
    for k, (name, shp) in enumerate(zip(("l", "g"), shapes)):
        if shp is None:
            out.append(0)
        elif defer:
            raw, sc, sh = res[k], res[2 + 2 * k], res[3 + 2 * k]
            act = rt.act_code(m.act_l if name == "l" else m.act_g) if hasattr(m, "act_l") else (0, 0.0)
            w, n = (nz[0:2] if name == "l" else nz[2:4]) if nz else (None, None)
            out.append(rt.PendingAct.from_tensors(raw, sc, sh, act[0], act[1], w if w is not None and w.numel() else None,
                                                  n if n is not None and n.numel() else None))
        else:
            out.append(res[k])
    return tuple(out)


def st_forward(st: nn.Module, x):
    _refresh_sn(st)
    spec = layer_spec(st)
    params, buffers = layer_tensors(st, spec)
    return torch.ops.ffc.spectral_transform(rt.require(x, "x"), params, buffers, spec)


def fu_forward(fu: nn.Module, x):
    spec = layer_spec(fu)
    params, buffers = layer_tensors(fu, spec)
    return torch.ops.ffc.fourier_unit(rt.require(x, "x"), params, buffers, spec)
