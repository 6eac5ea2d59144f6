"""Training path: custom-op autograd for the FFC operator surface (BASELINE config 3,
FFC-DCGAN generator + discriminator forward + backward).

The reference differentiates through ATen.  Here every op the reference's forward is made of
is one ``torch.autograd.Function`` whose forward AND backward launch the HIP kernels of
``libffc_amd.so`` (no torch compute on the path, no CPU fallback):

  reference op (file:line)                                  Function        backward kernels
  FFC / FFCTranspose local convs + ST conv2, summed per     _ConvLayerFn    act_bwd; adjoint conv/convT
    output branch (ffc.py:89-97, ffc_transpose.py:96-106,                   on ffc_conv_forward /
    spectral_transform.py:108), FU conv_layer (fourier_unity               ffc_convp_forward (same weight,
    .py:45), ST conv1 (:89)                                                other layout); ffc_conv_wgrad
  BatchNorm2d (+ activation): bn_l/bn_g (ffc_bn_act.py:       _BNActFn        ffc_bn_bwd
    73-81), ST bn1+act1 (:89), FU bn+relu (:46-49)
  SELayer (spectral_transform.py:23-28, :87)                 _SEFn           ffc_se_bwd + ffc_conv_wgrad
  AvgPool2d(2) / Upsample(x2) downsample (:44-47, :77)       _Pool2Fn/_Up2Fn ffc_up2 / ffc_pool2
  rfftn + Re/Im interleave (fourier_unity.py:38-42)          _RFFT2Fn        ffc_irfft2_planes (x 0.5)
  de-interleave + irfftn (+ x residual) (:51-56, ST :108)     _IRFFT2Fn       ffc_rfft2_planes (x 2)

FFT adjoints (verified in fp64): d/dX of irfftn(ortho) is rfftn(ortho) with the
mirrored bins doubled; d/dx of rfftn(ortho) is irfftn(ortho) with the mirrored bins halved.
The modules switch to this path when autograd is recording and an input or parameter needs a
gradient; under ``torch.no_grad()`` the fused inference kernels run.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _plan
from . import _runtime as rt
from ._lib import FFCError, check, ptr


def wants_grad(module: nn.Module, *tensors) -> bool:
    if not torch.is_grad_enabled():
        return False
    if any(isinstance(t, torch.Tensor) and t.requires_grad for t in tensors):
        return True
    return any(p.requires_grad for p in module.parameters())


def _stream(t):
    return rt.stream_of(t)


def _act_out(t: torch.Tensor, act, param, stream):
    """out-of-place y = act(t) (GELU, which the backward needs the input of)"""
    C = t.shape[1]
    one = torch.ones(C, device=t.device, dtype=torch.float32)
    zero = torch.zeros(C, device=t.device, dtype=torch.float32)
    y = torch.empty_like(t)
    check(rt.lib().ffc_bn_act_apply(ptr(t), ptr(y), t.shape[0], C, t[0, 0].numel(), ptr(one), ptr(zero), act,
                                    float(param), stream), "ffc_bn_act_apply")
    return y


def act_backward(t, dy, act, param):
    """dx = dy * act'(.): t = activation output (GELU: input)"""
    if act == 0:
        return dy
    dy = dy.contiguous()
    dx = torch.empty_like(dy)
    with rt.observe("act_bwd", bytes=12.0 * dy.numel()):
        check(rt.lib().ffc_act_bwd(ptr(t), ptr(dy), ptr(dx), dy.numel(), act, float(param), _stream(dy)),
              "ffc_act_bwd")
    return dx


# --------------------------------------------------------------------------- convolutions
def adjoint_seg(sg: _plan.Seg, M: int, OH: int, OW: int) -> _plan.Seg:
    """the segment whose forward is the adjoint (data gradient) of ``sg`` (output M x OH x OW)"""
    if sg.pool or sg.gate:
        raise NotImplementedError("pooled / gated segments have no training path")
    if sg.kind == "pw":
        return _plan.Seg("pw", M, OH, OW)
    if sg.kind == "conv":
        base = _plan.convT_out(OH, sg.k, sg.s, sg.p, sg.d, 0)
        op = sg.IH - base
        if op != sg.IW - _plan.convT_out(OW, sg.k, sg.s, sg.p, sg.d, 0) or not 0 <= op < max(sg.s, sg.d):
            raise NotImplementedError(f"conv adjoint needs output_padding {op} for {sg}")
        return _plan.Seg("convT", M, OH, OW, sg.k, sg.s, sg.p, sg.d, op)
    adj = _plan.Seg("conv", M, OH, OW, sg.k, sg.s, sg.p, sg.d)
    if _plan.seg_out(adj) != (sg.IH, sg.IW):
        raise NotImplementedError(f"convT adjoint does not return to the input size for {sg}")
    return adj


def run_conv(cache, key, B, M, segs, weights, inputs, out_shape=None, act=(0, 0.0), addend=None):
    """one implicit-GEMM launch: out = act(sum_s conv_s(x_s) [+ addend]) (plans cached in ``cache``)"""
    dev = inputs[0].device
    hit = cache.get(key)
    if hit is None:
        ex = rt.ConvExec(B, M, list(segs), weights, dev, pw_ok=True)
        hit = cache[key] = (ex, rt.LaunchPlan([ex], dev))
    ex, lp = hit
    ex.ensure_packed(weights)
    pl = ex.plan
    out = torch.empty(out_shape or (B, pl.M, pl.OH, pl.OW), device=dev, dtype=torch.float32)
    lp.launch([ex.job([(x, None) for x in inputs], out, act[0], act[1], addend, None)], _stream(out),
              flops=ex.flops)
    return out


def smallm_route(segs, layouts, M):
    """<= 4 output channels: 'full' (Conv2d onto a 1x1 output, ffc_conv_full_smallm), 'convT'
    (ConvTranspose2d k4 s2 p1, ffc_convt_k4s2_smallm), else None (implicit-GEMM kernels)"""
    if M > 4 or not 1 <= len(segs) <= 2 or not rt.USE_SMALLM:
        return None
    if all(sg.kind == "conv" and sg.k == sg.IH == sg.IW and sg.p == 0 and sg.d == 1 and not sg.pool and not sg.gate
           for sg in segs) and all(lay == 0 for lay in layouts):
        return "full"
    if all(sg.kind == "convT" and (sg.k, sg.s, sg.p, sg.d, sg.op) == (4, 2, 1, 1, 0) for sg in segs) and \
            all((sg.IH, sg.IW) == (segs[0].IH, segs[0].IW) for sg in segs) and sum(sg.C for sg in segs) <= 256 and \
            all(lay == 1 for lay in layouts):
        return "convT"
    return None


def conv_forward(cache, key, B, M, segs, weights, inputs, out_shape=None, act=(0, 0.0), addend=None):
    """out = act(sum_s conv_s(x_s) [+ addend]) on the best kernel for the job: the small-M direct
    kernels for <= 4 output channels, the implicit-GEMM kernels otherwise"""
    route = None
    if addend is None and sum(1 for w in weights if w[4] is not None) <= 1:
        route = smallm_route(segs, [w[1] for w in weights], M)
    if route is None and addend is None and len(segs) == 1 and weights[0][4] is None and weights[0][1] == 1:
        sg = segs[0]
        if sg.kind == "convT" and (sg.IH, sg.IW, sg.s, sg.p, sg.d, sg.op) == (1, 1, 1, 0, 1, 0) and sg.C <= 256:
            # ConvTranspose2d on a 1x1 input (FFCGenerator ffc0, models/ffc_generator.py:24): a plain GEMM
            # out (B, M*k*k) = x (B, C) . W (C, M*k*k) on the dense kernel; W needs no packing
            Wt = weights[0][0]
            N = M * sg.k * sg.k
            out = torch.empty((B, M, sg.k, sg.k), device=inputs[0].device, dtype=torch.float32)
            with rt.observe("dense", flops=2.0 * B * sg.C * N):
                check(rt.lib().ffc_dense_forward(ptr(inputs[0]), ptr(Wt), None, B, sg.C, N, N, ptr(out), None,
                                                 act[0], float(act[1]), _stream(out)), "ffc_dense_forward")
            return out
    if route is None:
        return run_conv(cache, key, B, M, segs, weights, inputs, out_shape, act, addend)
    L = rt.lib()
    bias = next((w[4] for w in weights if w[4] is not None), None)
    x1 = inputs[1] if len(inputs) > 1 else None
    w1 = weights[1][0] if len(weights) > 1 else None
    dev = inputs[0].device
    stream = _stream(inputs[0])
    if route == "full":
        sg = segs[0]
        out = torch.empty((B, M, 1, 1), device=dev, dtype=torch.float32)
        K0 = sg.C * sg.k * sg.k
        K1 = segs[1].C * segs[1].k * segs[1].k if x1 is not None else 0
        with rt.observe("conv_full_smallm", flops=2.0 * B * M * (K0 + K1)):
            check(L.ffc_conv_full_smallm(ptr(inputs[0]), K0, ptr(weights[0][0]), ptr(x1), K1, ptr(w1), ptr(bias), B, M,
                                         ptr(out), act[0], float(act[1]), stream), "ffc_conv_full_smallm")
        return out
    C0, C1 = segs[0].C, (segs[1].C if x1 is not None else 0)
    pkey = ("ctpack", key, weights[0][0].data_ptr(), weights[0][0]._version,
            None if w1 is None else (w1.data_ptr(), w1._version))
    wp = cache.get(pkey)
    if wp is None:
        for old in [k for k in cache if k[:2] == ("ctpack", key)]:
            del cache[old]
        wp = cache[pkey] = torch.empty(L.ffc_convt_smallm_pack_floats(C0, C1), device=dev, dtype=torch.float32)
        check(L.ffc_convt_smallm_pack(ptr(weights[0][0]), C0, ptr(w1), C1, M, ptr(wp), stream), "ffc_convt_smallm_pack")
    IH, IW = segs[0].IH, segs[0].IW
    out = torch.empty((B, M, 2 * IH, 2 * IW), device=dev, dtype=torch.float32)
    with rt.observe("convt_smallm", flops=2.0 * B * M * (C0 + C1) * 4 * (2 * IH) * (2 * IW)):
        check(L.ffc_convt_k4s2_smallm(ptr(inputs[0]), C0, ptr(x1), C1, ptr(wp), ptr(bias), B, IH, IW, M, ptr(out),
                                      act[0], float(act[1]), stream), "ffc_convt_k4s2_smallm")
    return out


def wgrad_splits(B, Mu, NT, P, bt=64):
    """split-K count for ffc_conv_wgrad (split-once kernel).  128x128 tiles: >= 512 workgroups and
    <= 1024 k per split; 64x64 tiles: >= 1024 workgroups and <= 4096 k per split; at most 1024 splits,
    >= 64 k each, partial sums capped at 32 M floats.  Fitted on MI355X to every weight gradient of
    the gan64train (B = 256) and fgan128train (B = 64) steps over 4-8 split counts each
    (tools/wgrad_probe.py, profiles/r03/wgrad/): the large tiles lose to the partial-sum traffic
    beyond ~1 k-deep splits, the small ones want the deeper grid"""
    tiles = -(-Mu // bt) * -(-NT // bt)
    K = B * P
    if bt >= 128:
        S = max(-(-512 // max(1, tiles)), K // 1024)
    else:
        S = max(-(-1024 // max(1, tiles)), K // 4096)
    S = min(S, 1024, max(1, K // 64), max(1, (32 << 20) // max(1, Mu * NT)))
    return max(1, S)


def conv_wgrad(U, V, k, s, p, d, dW_shape):
    """ffc_conv_wgrad: dW[m][n][kh][kw] = sum U[b,m,q] V[b,n,q*s-p+k*d] (see include/ffc_amd.h)"""
    B, Mu, PH, PW = U.shape
    _, Nv, VH, VW = V.shape
    NT = Nv * k * k
    S = wgrad_splits(B, Mu, NT, PH * PW, rt.lib().ffc_conv_wgrad_tile(Mu, NT))
    dW = torch.empty(dW_shape, device=U.device, dtype=torch.float32)
    if dW.numel() != Mu * NT:
        raise FFCError(f"weight gradient shape {dW_shape} != ({Mu}, {Nv}, {k}, {k})")
    ws = torch.empty(S * Mu * NT, device=U.device, dtype=torch.float32) if S > 1 else None
    with rt.observe("wgrad", flops=2.0 * B * Mu * NT * PH * PW):
        check(rt.lib().ffc_conv_wgrad(ptr(U), Mu, PH, PW, ptr(V), Nv, VH, VW, B, k, s, p, d, S, ptr(ws), ptr(dW), 0,
                                      _stream(U)), "ffc_conv_wgrad")
    return dW


def channel_sum(g):
    """sum over (B, H, W) per channel (bias gradient)"""
    B, C = g.shape[:2]
    HW = g[0, 0].numel()
    L = rt.lib()
    S = L.ffc_reduce_splits(B, C, HW)
    ws = torch.empty(S * C * 2, device=g.device, dtype=torch.float64)
    mom = torch.empty((C, 3), device=g.device, dtype=torch.float64)
    check(L.ffc_channel_moments(ptr(g), B, C, HW, ptr(ws), S, ptr(mom), _stream(g)), "ffc_channel_moments")
    return mom[:, 1].float()


class ConvLayerSpec:
    """outputs j = act_j(sum of the edges (j, i, seg, layout) applied to inputs i)"""

    def __init__(self, cache, B, outs, edges, n_in):
        self.cache, self.B, self.outs, self.edges, self.n_in = cache, B, outs, edges, n_in


class _ConvLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec: ConvLayerSpec, *args):
        n_in, ne = spec.n_in, len(spec.edges)
        xs = [a.contiguous() if a is not None else None for a in args[:n_in]]
        ws = [w.detach().contiguous() for w in args[n_in:n_in + ne]]
        bs = [b.detach().contiguous() if b is not None else None for b in args[n_in + ne:n_in + 2 * ne]]
        outs, saved_t = [], []
        for j, (M, act, param) in enumerate(spec.outs):
            es = [(e, spec.edges[e]) for e in range(ne) if spec.edges[e][0] == j]
            segs = tuple(ed[2] for _, ed in es)
            wts = [(ws[e], ed[3], ed[2].k, ed[2].k, bs[e]) for e, ed in es]
            fused = act if act != 5 else 0
            y = conv_forward(spec.cache, ("fwd", j, spec.B, segs, tuple(ed[3] for _, ed in es)), spec.B, M, segs, wts,
                             [xs[ed[1]] for _, ed in es], act=(fused, param))
            if act == 5:
                pre = y
                y = _act_out(pre, act, param, _stream(pre))
                saved_t.append(pre)
            else:
                saved_t.append(y)
            if RECORD is not None and act in (1, 2):   # ReLU / LeakyReLU kinks (fgan128 Discriminator)
                RECORD.append(y.detach())
            outs.append(y)
        ctx.spec = spec
        ctx.save_for_backward(*[x if x is not None else torch.empty(0) for x in xs], *ws, *saved_t)
        ctx.has_bias = [b is not None for b in bs]
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        spec = ctx.spec
        n_in, ne, no = spec.n_in, len(spec.edges), len(spec.outs)
        saved = ctx.saved_tensors
        xs, ws, ts = saved[:n_in], saved[n_in:n_in + ne], saved[n_in + ne:]
        gs = []
        for j, (M, act, param) in enumerate(spec.outs):
            g = gouts[j]
            gs.append(None if g is None else act_backward(ts[j], g.contiguous(), act, param))
        grads = [None] * (n_in + 2 * ne)
        for i in range(n_in):
            if not ctx.needs_input_grad[1 + i]:
                continue
            es = [(e, spec.edges[e]) for e in range(ne) if spec.edges[e][1] == i and gs[spec.edges[e][0]] is not None]
            if not es:
                continue
            x = xs[i]
            B, C = x.shape[:2]
            adj = []
            for e, (j, _, sg, lay) in es:
                g = gs[j]
                adj.append((e, adjoint_seg(sg, g.shape[1], g.shape[2], g.shape[3]), lay, g))
            # one launch when the adjoint segments can share a job, else chained through the addend
            groups = [adj]
            try:
                _plan.plan_job(B, C, tuple(a[1] for a in adj))
            except ValueError:
                groups = [[a] for a in adj]
            dx = None
            for grp in groups:
                segs = tuple(a[1] for a in grp)
                wts = [(ws[a[0]], 1 - a[2], a[1].k, a[1].k, None) for a in grp]
                key = ("adj", i, tuple(a[0] for a in grp), spec.B, segs)
                dx = conv_forward(spec.cache, key, B, C, segs, wts, [a[3] for a in grp], out_shape=tuple(x.shape),
                                  addend=dx)
            grads[i] = dx
        for e, (j, i, sg, lay) in enumerate(spec.edges):
            g = gs[j]
            if g is None:
                continue
            if ctx.needs_input_grad[1 + n_in + e]:
                w = ws[e]
                x = xs[i]
                if sg.kind == "convT":
                    grads[n_in + e] = conv_wgrad(x, g, sg.k, sg.s, sg.p, sg.d, tuple(w.shape))
                else:
                    grads[n_in + e] = conv_wgrad(g, x, sg.k, sg.s, sg.p, sg.d, tuple(w.shape))
            if ctx.has_bias[e] and ctx.needs_input_grad[1 + n_in + ne + e]:
                grads[n_in + ne + e] = channel_sum(g)
        return (None, *grads)


def conv_layer(owner_cache, B, outs, edges, inputs):
    """apply _ConvLayerFn.  edges: (out j, input i, Seg, module); modules' weight/bias are the params"""
    spec_edges = [(j, i, sg, 1 if isinstance(m, nn.ConvTranspose2d) else 0) for j, i, sg, m in edges]
    key = ("spec", B, tuple(outs), tuple((j, i, sg, lay) for j, i, sg, lay in spec_edges))
    spec = owner_cache.get(key)
    if spec is None:
        spec = owner_cache[key] = ConvLayerSpec(owner_cache, B, list(outs), spec_edges, len(inputs))
    for _, _, _, m in edges:
        rt.sn_refresh_train(m)
    weights = [m.weight for _, _, _, m in edges]
    biases = [m.bias for _, _, _, m in edges]
    return _ConvLayerFn.apply(spec, *inputs, *weights, *biases)


# --------------------------------------------------------------------------- BatchNorm2d + activation
class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bn, act, param, x, gamma, beta):
        x = x.contiguous()
        B, C = x.shape[:2]
        HW = x[0, 0].numel()
        use_batch, update = rt.bn_mode(bn)
        if bn.num_features != C:
            raise RuntimeError(f"running_mean should contain {C} elements not {bn.num_features}")
        grp = rt._sync_group() if use_batch else None   # SyncBN: global-batch statistics
        L = rt.lib()
        dev, stream = x.device, _stream(x)
        scale = torch.empty(C, device=dev, dtype=torch.float32)
        shift = torch.empty(C, device=dev, dtype=torch.float32)
        momentum = -1.0 if bn.momentum is None else float(bn.momentum)
        g = gamma.detach() if gamma is not None else None
        b = beta.detach() if beta is not None else None
        rm, rv = bn.running_mean, bn.running_var
        nbt = bn.num_batches_tracked
        moments = None
        rstats = (None, None)
        if use_batch:
            S = L.ffc_reduce_splits(B, C, HW)
            ws = torch.empty(S * C * 2, device=dev, dtype=torch.float64)
            moments = torch.empty((C, 3), device=dev, dtype=torch.float64)
            with rt.observe("bn_moments", bytes=4.0 * x.numel()):
                check(L.ffc_channel_moments(ptr(x), B, C, HW, ptr(ws), S, ptr(moments), stream), "ffc_channel_moments")
            if grp is not None:
                from .distributed import merge_moments
                merge_moments(moments, group=grp)
            check(L.ffc_bn_finalize(ptr(moments), C, ptr(g), ptr(b), ptr(rm), ptr(rv), ptr(nbt), 1, int(update),
                                    momentum, float(bn.eps), 1.0, ptr(scale), ptr(shift), stream), "ffc_bn_finalize")
        else:
            rstats = (rm.detach().clone(), rv.detach().clone())
            check(L.ffc_bn_finalize(None, C, ptr(g), ptr(b), ptr(rm), ptr(rv), ptr(nbt), 0, 0, momentum,
                                    float(bn.eps), 1.0, ptr(scale), ptr(shift), stream), "ffc_bn_finalize")
        y = torch.empty_like(x)
        with rt.observe("bn_act", bytes=8.0 * x.numel()):
            check(L.ffc_bn_act_apply(ptr(x), ptr(y), B, C, HW, ptr(scale), ptr(shift), act, float(param), stream),
                  "ffc_bn_act_apply")
        ctx.act, ctx.param, ctx.eps = act, param, float(bn.eps)
        ctx.has_gamma, ctx.has_beta = gamma is not None, beta is not None
        ctx.save_for_backward(x, scale, shift, moments if moments is not None else torch.empty(0),
                              rstats[0] if rstats[0] is not None else torch.empty(0),
                              rstats[1] if rstats[1] is not None else torch.empty(0),
                              g if g is not None else torch.empty(0))
        ctx.use_batch = use_batch
        ctx.grp = grp
        return y

    @staticmethod
    def backward(ctx, dy):
        x, scale, shift, moments, rmean, rvar, gamma = ctx.saved_tensors
        dy = dy.contiguous()
        B, C = x.shape[:2]
        HW = x[0, 0].numel()
        L = rt.lib()
        S = L.ffc_reduce_splits(B, C, HW)
        ws = torch.empty(S * C * 2, device=x.device, dtype=torch.float64)
        coef = torch.empty(C * 3, device=x.device, dtype=torch.float32)
        dgamma = torch.empty(C, device=x.device, dtype=torch.float32) if ctx.has_gamma else None
        dbeta = torch.empty(C, device=x.device, dtype=torch.float32) if ctx.has_beta else None
        dx = torch.empty_like(x) if ctx.needs_input_grad[3] else None
        if ctx.grp is not None:
            # torch.nn.SyncBatchNorm backward: dx from the all-reduced {sum g, sum g*x}, this rank's
            # own sums for dgamma / dbeta (the caller's data-parallel wrapper reduces parameter grads)
            import torch.distributed as dist
            stream = _stream(x)
            sums = torch.empty((C, 2), device=x.device, dtype=torch.float64)
            with rt.observe("bn_bwd", bytes=8.0 * x.numel()):
                check(L.ffc_bn_bwd_sums(ptr(x), ptr(dy), B, C, HW, ptr(scale), ptr(shift), ctx.act, float(ctx.param),
                                        ptr(ws), S, ptr(sums), stream), "ffc_bn_bwd_sums")
            gsums = sums.clone()
            dist.all_reduce(gsums, group=ctx.grp)
            g = ptr(gamma) if ctx.has_gamma else None
            check(L.ffc_bn_bwd_coeff(ptr(sums), C, ptr(moments), ctx.eps, g, ptr(coef), ptr(dgamma), ptr(dbeta),
                                     stream), "ffc_bn_bwd_coeff")
            check(L.ffc_bn_bwd_coeff(ptr(gsums), C, ptr(moments), ctx.eps, g, ptr(coef), None, None, stream),
                  "ffc_bn_bwd_coeff")
            if dx is not None:
                with rt.observe("bn_bwd", bytes=12.0 * x.numel()):
                    check(L.ffc_bn_bwd_apply(ptr(x), ptr(dy), B, C, HW, ptr(scale), ptr(shift), ctx.act,
                                             float(ctx.param), ptr(coef), ptr(dx), stream), "ffc_bn_bwd_apply")
            return None, None, None, dx, dgamma, dbeta
        with rt.observe("bn_bwd", bytes=12.0 * x.numel()):
            check(L.ffc_bn_bwd(ptr(x), ptr(dy), B, C, HW, ptr(scale), ptr(shift), ctx.act, float(ctx.param),
                               ptr(moments) if ctx.use_batch else None,
                               None if ctx.use_batch else ptr(rmean), None if ctx.use_batch else ptr(rvar),
                               ctx.eps, ptr(gamma) if ctx.has_gamma else None, ptr(ws), S, ptr(coef), ptr(dgamma),
                               ptr(dbeta), ptr(dx), _stream(x)), "ffc_bn_bwd")
        return None, None, None, dx, dgamma, dbeta


RECORD = None   # tests: a list collecting every BN + activation output (kink patterns of the path)


def bn_act(bn: nn.BatchNorm2d, x, act=(0, 0.0)):
    y = _BNActFn.apply(bn, act[0], act[1], x, bn.weight, bn.bias)
    if RECORD is not None:
        RECORD.append(y.detach())
    return y


# --------------------------------------------------------------------------- SELayer
class _SEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, w2):
        x = x.contiguous()
        B, C, H, W = x.shape
        hid = w1.shape[0]
        L = rt.lib()
        stream = _stream(x)
        w1d = w1.detach().contiguous() if hid else None
        w2d = w2.detach().contiguous() if hid else None
        gate = torch.empty((B, C), device=x.device, dtype=torch.float32)
        with rt.observe("se_gate", bytes=4.0 * x.numel()):
            check(L.ffc_se_gate(ptr(x), B, C, H, W, 0, ptr(w1d), ptr(w2d), hid, ptr(gate), stream), "ffc_se_gate")
        zeros = torch.zeros(B * C, device=x.device, dtype=torch.float32)
        y = torch.empty_like(x)
        check(L.ffc_bn_act_apply(ptr(x), ptr(y), 1, B * C, H * W, ptr(gate), ptr(zeros), 0, 0.0, stream),
              "ffc_bn_act_apply")
        ctx.hid = hid
        ctx.w_shapes = (tuple(w1.shape), tuple(w2.shape))
        ctx.save_for_backward(x, w1d if hid else torch.empty(0), w2d if hid else torch.empty(0))
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w1, w2 = ctx.saved_tensors
        dy = dy.contiguous()
        B, C, H, W = x.shape
        hid = ctx.hid
        dev = x.device
        dx = torch.empty_like(x)
        vec = (lambda n: torch.empty((B, n, 1, 1), device=dev, dtype=torch.float32)) if hid else (lambda n: None)
        dpre2, hact, dpre1, mean = vec(C), vec(hid), vec(hid), vec(C)
        ws = torch.empty(4 * B * C, device=dev, dtype=torch.float32)
        with rt.observe("se_bwd", bytes=(16.0 if hid else 8.0) * x.numel()):
            check(rt.lib().ffc_se_bwd(ptr(x), ptr(dy), B, C, H, W, ptr(w1) if hid else None, ptr(w2) if hid else None,
                                      hid, ptr(dx), ptr(dpre2), ptr(hact), ptr(dpre1), ptr(mean), ptr(ws), _stream(x)),
                  "ffc_se_bwd")
        dw1 = dw2 = None
        if not hid:   # Linear(C, 0) / Linear(0, C): empty weights get empty gradients
            dw1 = torch.zeros(ctx.w_shapes[0], device=dev) if ctx.needs_input_grad[1] else None
            dw2 = torch.zeros(ctx.w_shapes[1], device=dev) if ctx.needs_input_grad[2] else None
        if hid and ctx.needs_input_grad[1]:
            dw1 = conv_wgrad(dpre1, mean, 1, 1, 0, 1, (hid, C))      # fc.0: (hid, C)
        if hid and ctx.needs_input_grad[2]:
            dw2 = conv_wgrad(dpre2, hact, 1, 1, 0, 1, (C, hid))      # fc.2: (C, hid)
        return dx, dw1, dw2


def se_layer(se, x):
    if se.fc[0].bias is not None or se.fc[2].bias is not None:
        raise NotImplementedError("SELayer with bias")
    return _SEFn.apply(x, se.fc[0].weight, se.fc[2].weight)


# --------------------------------------------------------------------------- pool / upsample
def _pool2(x, scale):
    B, C, H, W = x.shape
    y = torch.empty((B, C, H // 2, W // 2), device=x.device, dtype=torch.float32)
    check(rt.lib().ffc_pool2(ptr(x), B * C, H, W, float(scale), ptr(y), _stream(x)), "ffc_pool2")
    return y


def _up2(x, scale):
    B, C, h, w = x.shape
    y = torch.empty((B, C, 2 * h, 2 * w), device=x.device, dtype=torch.float32)
    check(rt.lib().ffc_up2(ptr(x), B * C, h, w, float(scale), ptr(y), _stream(x)), "ffc_up2")
    return y


class _Pool2Fn(torch.autograd.Function):
    """AvgPool2d(2, 2) (spectral_transform.py:46-47)"""

    @staticmethod
    def forward(ctx, x):
        if x.shape[2] % 2 or x.shape[3] % 2:
            raise NotImplementedError("AvgPool2d(2) downsample of an odd-sized input")
        return _pool2(x.contiguous(), 0.25)

    @staticmethod
    def backward(ctx, dy):
        return _up2(dy.contiguous(), 0.25)


class _Up2Fn(torch.autograd.Function):
    """Upsample(scale_factor=2, mode='nearest') (spectral_transform.py:44-45)"""

    @staticmethod
    def forward(ctx, x):
        return _up2(x.contiguous(), 1.0)

    @staticmethod
    def backward(ctx, dy):
        return _pool2(dy.contiguous(), 1.0)


# --------------------------------------------------------------------------- NoiseInjection, Linear
class _NoiseFn(torch.autograd.Function):
    """NoiseInjection.forward (layers/noise_injection.py:25-32): x + weight * noise; backward
    dx = g, dweight[c] = sum g[:, c] * noise (ffc_noise_wgrad)"""

    @staticmethod
    def forward(ctx, x, weight, noise):
        B, C, H, W = x.shape
        x = x.contiguous()
        out = torch.empty_like(x)
        with rt.observe("noise_inject", bytes=8.0 * x.numel() + 4.0 * noise.numel()):
            check(rt.lib().ffc_noise_inject(ptr(x), ptr(weight.detach().contiguous()), ptr(noise), ptr(out), B, C,
                                            H * W, _stream(x)), "ffc_noise_inject")
        ctx.save_for_backward(noise)
        return out

    @staticmethod
    def backward(ctx, g):
        (noise,) = ctx.saved_tensors
        g = g.contiguous()
        dw = None
        if ctx.needs_input_grad[1]:
            B, C, H, W = g.shape
            dw = torch.empty(C, device=g.device, dtype=torch.float32)
            check(rt.lib().ffc_noise_wgrad(ptr(g), ptr(noise), B, C, H * W, ptr(dw), _stream(g)), "ffc_noise_wgrad")
            dw = dw.view(1, C, 1, 1)
        return (g if ctx.needs_input_grad[0] else None), dw, None


def noise_inject(mod, x, noise=None):
    """NoiseInjection ``mod`` applied to x on the training path (noise drawn with normal_() as the
    reference does when not given)"""
    B, C, H, W = x.shape
    if noise is None:
        noise = x.new_empty(B, 1, H, W).normal_()
    noise = rt.require(noise, "noise").contiguous()
    if tuple(noise.shape) != (B, 1, H, W) or (H * W) % 4:
        raise NotImplementedError("NoiseInjection: noise must be (B, 1, H, W) with H*W % 4 == 0")
    if mod.weight.numel() != C:
        raise RuntimeError(f"NoiseInjection has {mod.weight.numel()} channels, tensor has {C}")
    return _NoiseFn.apply(x, mod.weight, noise)


class _LinearAs1x1:
    """nn.Linear(K, N) seen by conv_layer as a 1x1 Conv2d on a 1x1 input: weight (N, K, 1, 1) is a view
    of the Linear's weight, so its gradient flows back to the parameter"""

    def __init__(self, lin: nn.Linear):
        self.weight = lin.weight.view(lin.out_features, lin.in_features, 1, 1)
        self.bias = lin.bias
        self.out_channels = lin.out_features


def linear(owner_cache, lin: nn.Linear, z):
    """nn.Linear forward + backward (fgan128_complete.py:453-455 noise_to_feature, and the spectral-norm
    fc of the fgan128 Discriminator, :540) -> (B, N)"""
    B, K = z.shape
    rt.sn_refresh_train(lin)   # the 1x1 view below must see this call's W / sigma
    (y,) = conv_layer(owner_cache, B, [(lin.out_features, 0, 0.0)], [(0, 0, _plan.Seg("pw", K, 1, 1), _LinearAs1x1(lin))],
                      [z.reshape(B, K, 1, 1)])
    return y.reshape(B, lin.out_features)


# --------------------------------------------------------------------------- FFTs
def _rfft2(x, iscale):
    B, C, H, W = x.shape
    Z = torch.empty((B, 2 * C, H, W // 2 + 1), device=x.device, dtype=torch.float32)
    with rt.observe("rfft2", bytes=4.0 * x.numel() + 4.0 * Z.numel()):
        check(rt.lib().ffc_rfft2_planes(ptr(x), B * C, H, W, float(iscale), ptr(Z), _stream(x)), "ffc_rfft2_planes")
    return Z


def _irfft2(Z, H, W, iscale, addend=None):
    B, C2 = Z.shape[:2]
    y = torch.empty((B, C2 // 2, H, W), device=Z.device, dtype=torch.float32)
    with rt.observe("irfft2", bytes=4.0 * Z.numel() + 4.0 * y.numel()):
        check(rt.lib().ffc_irfft2_planes(ptr(Z), B * (C2 // 2), H, W, float(iscale), ptr(addend), ptr(y),
                                         _stream(Z)), "ffc_irfft2_planes")
    return y


class _RFFT2Fn(torch.autograd.Function):
    """Z = interleave(rfftn(x, norm='ortho')) (fourier_unity.py:38-42)"""

    @staticmethod
    def forward(ctx, x):
        ctx.hw = x.shape[2:]
        return _rfft2(x.contiguous(), 1.0)

    @staticmethod
    def backward(ctx, dZ):
        H, W = ctx.hw
        return _irfft2(dZ.contiguous(), H, W, 0.5)


class _IRFFT2Fn(torch.autograd.Function):
    """y = irfftn(deinterleave(Z), s=(H, W), norm='ortho') [+ r] (fourier_unity.py:51-56; r: the
    x + fu(x) residual of spectral_transform.py:108)"""

    @staticmethod
    def forward(ctx, Z, H, W, r):
        ctx.has_r = r is not None
        return _irfft2(Z.contiguous(), H, W, 1.0, r.contiguous() if r is not None else None)

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dZ = _rfft2(dy, 2.0) if ctx.needs_input_grad[0] else None
        return dZ, None, None, (dy if ctx.has_r else None)


def fourier_unit(fu, x, residual: bool):
    """FourierUnitSN.forward (fourier_unity.py:32-56) [+ x] on the training path"""
    B, C, H, W = x.shape
    fu._check(C)
    if fu.mix_precision != "fp32":
        raise NotImplementedError("the training path computes the spectral mix in fp32 only (config 5's fp16 "
                                  "mix is forward-only)")
    if (H > 64 or W > 64) and not (H == W and H in (128,)):
        raise NotImplementedError("training-path Fourier unit: planes up to 64x64, or square 128x128")
    Z = _RFFT2Fn.apply(x)
    cache = fu.__dict__.setdefault("_train_cache", {})
    seg = _plan.Seg("pw", 2 * C, H, W // 2 + 1)
    (U,) = conv_layer(cache, B, [(2 * C, 0, 0.0)], [(0, 0, seg, fu.conv_layer)], [Z])
    R = bn_act(fu.bn, U, (1, 0.0))
    return _IRFFT2Fn.apply(R, H, W, x if residual else None)


def spectral_v(st, x):
    """v = s + fu(s), s = relu(bn1(conv1(se(downsample(x))))) (spectral_transform.py:77-108, before conv2)"""
    if st.groups != 1:
        raise NotImplementedError("grouped SpectralTransform (groups != 1) is not on the hot path")
    if st.stride == 2 and st.upsample:
        x = _Up2Fn.apply(x)
    elif st.stride == 2:
        x = _Pool2Fn.apply(x)
    x = se_layer(st.se_block, x)
    B, Cin, H, W = x.shape
    cache = st.__dict__.setdefault("_train_cache", {})
    c = st.conv1.out_channels
    (t,) = conv_layer(cache, B, [(c, 0, 0.0)], [(0, 0, _plan.Seg("pw", Cin, H, W), st.conv1)], [x])
    s = bn_act(st.bn1, t, (1, 0.0))
    return fourier_unit(st.fu, s, residual=True)
