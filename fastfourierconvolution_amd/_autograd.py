"""Training path: the implementations behind the autograd-registered custom ops of ops.py for the
FFC operator surface (BASELINE config 3, FFC-DCGAN generator + discriminator forward + backward),
and the module-facing helpers that compose those ops.

The reference differentiates through ATen.  Here every op the reference's forward is made of
is one ``torch.ops.ffc.*`` custom op whose forward AND backward (another ffc op, wired by
``register_autograd``) launch the HIP kernels of ``libffc_amd.so`` (no torch compute on the path,
no CPU fallback):

  reference op (file:line)                                  custom op          backward op / kernels
  FFC / FFCTranspose local convs + ST conv2, summed per     ffc::conv_layer    ffc::conv_layer_backward:
    output branch (ffc.py:89-97, ffc_transpose.py:96-106,                      act_bwd; adjoint conv/convT on
    spectral_transform.py:108), FU conv_layer (fourier_unity                  ffc_conv_forward / convp (same
    .py:45), ST conv1 (:89), nn.Linear                                        weight, other layout); wgrad
  BatchNorm2d (+ activation): bn_l/bn_g (ffc_bn_act.py:       ffc::bn_act        ffc::bn_act_backward (ffc_bn_bwd)
    73-81), ST bn1+act1 (:89), FU bn+relu (:46-49)
  SELayer (spectral_transform.py:23-28, :87)                 ffc::se_scale      ffc::se_scale_backward
  AvgPool2d(2) / Upsample(x2) downsample (:44-47, :77)       ffc::pool2/up2     each other (adjoints)
  rfftn + Re/Im interleave (fourier_unity.py:38-42)          ffc::rfft2         ffc::irfft2 (mirrored x 0.5)
  de-interleave + irfftn (+ x residual) (:51-56, ST :108)     ffc::irfft2        ffc::rfft2 (mirrored x 2)
  NoiseInjection (noise_injection.py:25-32)                  ffc::noise_inject  ffc::noise_wgrad

FFT adjoints (verified in fp64): d/dX of irfftn(ortho) is rfftn(ortho) with the
mirrored bins doubled; d/dx of rfftn(ortho) is irfftn(ortho) with the mirrored bins halved.
The modules switch to this path when autograd is recording and an input or parameter needs a
gradient; under ``torch.no_grad()`` the fused inference kernels run.
"""
from __future__ import annotations

import functools
import json

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
    # the job's full shape and the plan switches are part of the key (a caller's key alone may leave
    # out the output channels, and one cache serves every module of a structure)
    key = (key, B, M, tuple(segs), str(dev), rt.plan_knobs())
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
    pkey = ("ctpack", key, rt.weight_key(weights[0][0]), rt.weight_key(w1))
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


# --------------------------------------------------------------------------- conv layer (ffc::conv_layer)
# spec (JSON): {"outs": [[M, act, param], ...], "edges": [[j, i, kind, k, s, p, d, op, layout, bias], ...]}:
# output j = act_j(sum over its edges of conv(kind, k, s, p, d, op)(xs[i]) with ws[e] (+ bs[bias])).
# Shapes come from the tensors, so one spec serves every batch size.
# plans / packed weights of every conv_layer op, keyed by (spec, shapes): a pool of caches, each
# held by one caller at a time (rt.StreamPool: a plan's packed weights and split-K partials are
# written on its holder's stream)
_CL_POOL = rt.StreamPool(dict)


@functools.lru_cache(maxsize=4096)
def parse_conv_spec(spec: str):
    d = json.loads(spec)
    return [tuple(o) for o in d["outs"]], [tuple(e) for e in d["edges"]]


def conv_spec(outs, edges) -> str:
    """outs: [(M, act, param)]; edges: [(j, i, Seg, layout, bias index or -1)] -> spec string"""
    return json.dumps({"outs": [[int(M), int(a), float(p)] for M, a, p in outs],
                       "edges": [[j, i, sg.kind, sg.k, sg.s, sg.p, sg.d, sg.op, lay, b] for j, i, sg, lay, b in edges]},
                      separators=(",", ":"))


def _edge_seg(e, x) -> _plan.Seg:
    _, _, kind, k, s, p, d, op, _, _ = e
    if kind == "pw":
        return _plan.Seg("pw", x.shape[1], x.shape[2], x.shape[3])
    return _plan.Seg(kind, x.shape[1], x.shape[2], x.shape[3], k, s, p, d, op)


def conv_layer_out_shape(e, x, M):
    """output shape of edge e (spec tuple) applied to x with M output channels (works on SymInts)"""
    _, _, kind, k, s, p, d, op, _, _ = e
    B, _, H, W = x.shape
    if kind == "conv":
        return (B, M, _plan.conv_out(H, k, s, p, d), _plan.conv_out(W, k, s, p, d))
    if kind == "convT":
        return (B, M, _plan.convT_out(H, k, s, p, d, op), _plan.convT_out(W, k, s, p, d, op))
    return (B, M, H, W)


def conv_layer_impl(xs, ws, bs, spec):
    """ffc::conv_layer: -> outputs, then the pre-activation of every GELU output (the backward's input)"""
    outs_s, edges = parse_conv_spec(spec)
    rt.note_tensors(list(ws) + list(bs))
    xs = [rt.require(x, "conv_layer input") for x in xs]
    ws = [rt.require(w, "conv_layer weight") for w in ws]
    bs = [rt.require(b, "conv_layer bias") for b in bs]
    B = xs[0].shape[0]
    segs = [_edge_seg(e, xs[e[1]]) for e in edges]
    outs, pres = [], []
    for j, (M, act, param) in enumerate(outs_s):
        es = [e for e in range(len(edges)) if edges[e][0] == j]
        sgs = tuple(segs[e] for e in es)
        wts = [(ws[e], edges[e][8], edges[e][3], edges[e][3], bs[edges[e][9]] if edges[e][9] >= 0 else None)
               for e in es]
        fused = act if act != 5 else 0
        with _CL_POOL.hold() as cache:
            y = conv_forward(cache, ("fwd", spec, j, B, sgs), B, M, sgs, wts, [xs[edges[e][1]] for e in es],
                             act=(fused, param))
        if act == 5:
            pres.append(y)
            y = _act_out(y, act, param, _stream(y))
        if RECORD is not None and act in (1, 2):   # ReLU / LeakyReLU kinks (fgan128 Discriminator)
            RECORD.append(y.detach())
        outs.append(y)
    return outs + pres


def conv_layer_backward_impl(xs, ws, ts, gouts, needs, spec):
    """ffc::conv_layer_backward: ts[j] = output j (its pre-activation for GELU); needs: per x, w, b.
    -> [dx per x, dW per w, db per b] (empty tensors where not needed)"""
    outs_s, edges = parse_conv_spec(spec)
    n_in, ne = len(xs), len(ws)
    nb = sum(1 for e in edges if e[9] >= 0)
    gs = []
    for j, (M, act, param) in enumerate(outs_s):
        g = gouts[j]
        gs.append(None if g is None else act_backward(ts[j], g.contiguous(), act, param))
    B = xs[0].shape[0]
    grads = [xs[0].new_empty(0) for _ in range(n_in + ne + nb)]   # distinct: op outputs may not alias
    for i in range(n_in):
        if not needs[i]:
            continue
        es = [(e, edges[e]) for e in range(ne) if edges[e][1] == i and gs[edges[e][0]] is not None]
        x = xs[i]
        if not es:
            grads[i] = torch.zeros_like(x)
            continue
        C = x.shape[1]
        adj = []
        for e, ed in es:
            g = gs[ed[0]]
            adj.append((e, adjoint_seg(_edge_seg(ed, x), g.shape[1], g.shape[2], g.shape[3]), ed[8], g))
        # one launch when the adjoint segments can share a job, else chained through the addend
        groups = [adj]
        try:
            _plan.plan_job(B, C, tuple(a[1] for a in adj))
        except ValueError:
            groups = [[a] for a in adj]
        dx = None
        for grp in groups:
            segs = tuple(a[1] for a in grp)
            wts = [(ws[a[0]].contiguous(), 1 - a[2], a[1].k, a[1].k, None) for a in grp]
            key = ("adj", spec, i, tuple(a[0] for a in grp), B, C, segs)
            with _CL_POOL.hold() as cache:
                dx = conv_forward(cache, key, B, C, segs, wts, [a[3] for a in grp], out_shape=tuple(x.shape),
                                  addend=dx)
        grads[i] = dx
    for e, ed in enumerate(edges):
        j, i, kind, k, s, p, d = ed[:7]
        g = gs[j]
        if needs[n_in + e]:
            w, x = ws[e], xs[i].contiguous()
            if g is None:
                grads[n_in + e] = torch.zeros_like(w)
            elif kind == "convT":
                grads[n_in + e] = conv_wgrad(x, g, k, s, p, d, tuple(w.shape))
            else:
                grads[n_in + e] = conv_wgrad(g, x, k, s, p, d, tuple(w.shape))
        if ed[9] >= 0 and needs[n_in + ne + ed[9]]:
            grads[n_in + ne + ed[9]] = channel_sum(g) if g is not None else xs[0].new_zeros(outs_s[j][0])
    return grads


def conv_layer(B, outs, edges, inputs):
    """the ffc::conv_layer op over modules: edges (out j, input i, Seg, module) whose weight / bias
    are the parameters (spectral norm refreshed first, as the module call would)"""
    spec_edges, ws, bs = [], [], []
    for j, i, sg, m in edges:
        rt.sn_refresh_train(m)
        b = -1
        if m.bias is not None:
            b = len(bs)
            bs.append(m.bias)
        spec_edges.append((j, i, sg, 1 if isinstance(m, nn.ConvTranspose2d) else 0, b))
        ws.append(m.weight)
    ys = torch.ops.ffc.conv_layer(list(inputs), ws, bs, conv_spec(outs, spec_edges))
    return ys[:len(outs)]


# --------------------------------------------------------------------------- BatchNorm2d + activation
def bn_act_impl(x, gamma, beta, running_mean, running_var, use_batch, eps, act, param):
    """ffc::bn_act: y = act(BN(x)) with nn.BatchNorm2d's normalisation (batch statistics when
    use_batch, else the running ones).  -> [y, scale, shift, stats]: stats = the fp64 batch moments
    [C][3] {n, sum x, sum x^2} (all-reduced under SyncBN) with batch statistics, the running
    (mean, var) [2][C] otherwise -- the backward's input and ffc::bn_update_running's"""
    x = rt.require(x, "x")
    B, C = x.shape[:2]
    HW = x[0, 0].numel()
    n_feat = running_mean.numel() if running_mean is not None else (gamma.numel() if gamma is not None else C)
    if n_feat != C:
        raise RuntimeError(f"running_mean should contain {C} elements not {n_feat}")
    grp = rt._sync_group() if use_batch else None   # SyncBN: global-batch statistics
    L = rt.lib()
    dev, stream = x.device, _stream(x)
    scale = torch.empty(C, device=dev, dtype=torch.float32)
    shift = torch.empty(C, device=dev, dtype=torch.float32)
    if use_batch:
        S = L.ffc_reduce_splits(B, C, HW)
        ws = torch.empty(S * C * 2, device=dev, dtype=torch.float64)
        stats = torch.empty((C, 3), device=dev, dtype=torch.float64)
        with rt.observe("bn_moments", bytes=4.0 * x.numel()):
            check(L.ffc_channel_moments(ptr(x), B, C, HW, ptr(ws), S, ptr(stats), stream), "ffc_channel_moments")
        if grp is not None:
            from .distributed import merge_moments
            merge_moments(stats, group=grp)
        check(L.ffc_bn_finalize(ptr(stats), C, ptr(gamma), ptr(beta), None, None, None, 1, 0, 0.1, float(eps), 1.0,
                                ptr(scale), ptr(shift), stream), "ffc_bn_finalize")
    else:
        stats = torch.stack((running_mean.detach(), running_var.detach()))
        check(L.ffc_bn_finalize(None, C, ptr(gamma), ptr(beta), ptr(stats[0]), ptr(stats[1]), None, 0, 0, 0.1,
                                float(eps), 1.0, ptr(scale), ptr(shift), stream), "ffc_bn_finalize")
    y = torch.empty_like(x)
    with rt.observe("bn_act", bytes=8.0 * x.numel()):
        check(L.ffc_bn_act_apply(ptr(x), ptr(y), B, C, HW, ptr(scale), ptr(shift), act, float(param), stream),
              "ffc_bn_act_apply")
    return [y, scale, shift, stats]


def bn_update_running_impl(running_mean, running_var, num_batches_tracked, stats, momentum, count_mult):
    """ffc::bn_update_running: running stats <- batch moments (unbiased variance), nn.BatchNorm2d's rule"""
    C = running_mean.numel()
    scratch = torch.empty(2 * C, device=running_mean.device, dtype=torch.float32)
    check(rt.lib().ffc_bn_finalize(ptr(stats), C, None, None, ptr(running_mean), ptr(running_var),
                                   ptr(num_batches_tracked), 1, 1, float(momentum), 1e-5, float(count_mult),
                                   ptr(scratch), ptr(scratch[C:]), _stream(running_mean)), "ffc_bn_finalize")


def bn_act_backward_impl(x, dy, scale, shift, stats, gamma, use_batch, sync, eps, act, param, need_dx, has_gamma,
                         has_beta):
    """ffc::bn_act_backward -> [dx, dgamma, dbeta] (empty tensors where not needed / absent).
    x is the op's raw input (the saved tensor, not the forward's contiguous copy): the kernels read
    and write dense NCHW, so x is made contiguous here and dx is allocated NCHW-contiguous"""
    x = x.contiguous()
    dy = dy.contiguous()
    B, C = x.shape[:2]
    HW = x[0, 0].numel()
    L = rt.lib()
    S = L.ffc_reduce_splits(B, C, HW)
    ws = torch.empty(S * C * 2, device=x.device, dtype=torch.float64)
    coef = torch.empty(C * 3, device=x.device, dtype=torch.float32)
    dgamma = torch.empty(C, device=x.device, dtype=torch.float32) if has_gamma else None
    dbeta = torch.empty(C, device=x.device, dtype=torch.float32) if has_beta else None
    dx = torch.empty_like(x) if need_dx else None
    stream = _stream(x)
    grp = rt._sync_group() if sync else None
    if grp is not None:
        # torch.nn.SyncBatchNorm backward: dx from the all-reduced {sum g, sum g*x}, this rank's
        # own sums for dgamma / dbeta (the caller's data-parallel wrapper reduces parameter grads)
        import torch.distributed as dist
        sums = torch.empty((C, 2), device=x.device, dtype=torch.float64)
        with rt.observe("bn_bwd", bytes=8.0 * x.numel()):
            check(L.ffc_bn_bwd_sums(ptr(x), ptr(dy), B, C, HW, ptr(scale), ptr(shift), act, float(param),
                                    ptr(ws), S, ptr(sums), stream), "ffc_bn_bwd_sums")
        gsums = sums.clone()
        dist.all_reduce(gsums, group=grp)
        g = ptr(gamma) if has_gamma else None
        check(L.ffc_bn_bwd_coeff(ptr(sums), C, ptr(stats), float(eps), g, ptr(coef), ptr(dgamma), ptr(dbeta),
                                 stream), "ffc_bn_bwd_coeff")
        check(L.ffc_bn_bwd_coeff(ptr(gsums), C, ptr(stats), float(eps), g, ptr(coef), None, None, stream),
              "ffc_bn_bwd_coeff")
        if dx is not None:
            with rt.observe("bn_bwd", bytes=12.0 * x.numel()):
                check(L.ffc_bn_bwd_apply(ptr(x), ptr(dy), B, C, HW, ptr(scale), ptr(shift), act, float(param),
                                         ptr(coef), ptr(dx), stream), "ffc_bn_bwd_apply")
    else:
        with rt.observe("bn_bwd", bytes=12.0 * x.numel()):
            check(L.ffc_bn_bwd(ptr(x), ptr(dy), B, C, HW, ptr(scale), ptr(shift), act, float(param),
                               ptr(stats) if use_batch else None,
                               None if use_batch else ptr(stats[0]), None if use_batch else ptr(stats[1]),
                               float(eps), ptr(gamma) if has_gamma else None, ptr(ws), S, ptr(coef), ptr(dgamma),
                               ptr(dbeta), ptr(dx), stream), "ffc_bn_bwd")
    return [t if t is not None else x.new_empty(0) for t in (dx, dgamma, dbeta)]


RECORD = None   # tests: a list collecting every BN + activation output (kink patterns of the path)


def bn_act(bn: nn.BatchNorm2d, x, act=(0, 0.0)):
    """BatchNorm2d ``bn`` + activation on the ffc::bn_act op (the module's tensors as arguments), then
    the running-statistics update in training mode (ffc::bn_update_running)"""
    use_batch, update = rt.bn_mode(bn)
    y, _, _, stats = torch.ops.ffc.bn_act(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, use_batch,
                                          float(bn.eps), int(act[0]), float(act[1]))
    if update:
        torch.ops.ffc.bn_update_running(bn.running_mean, bn.running_var, bn.num_batches_tracked, stats,
                                        -1.0 if bn.momentum is None else float(bn.momentum), 1.0)
    if RECORD is not None:
        RECORD.append(y.detach())
    return y


# --------------------------------------------------------------------------- SELayer
def se_scale_impl(x, w1, w2):
    """ffc::se_scale: x * sigmoid(w2 . relu(w1 . mean_HW(x))) (hidden width w1.shape[0] may be 0)"""
    x = rt.require(x, "x")
    B, C, H, W = x.shape
    hid = w1.shape[0]
    L = rt.lib()
    stream = _stream(x)
    w1d = w1.contiguous() if hid else None
    w2d = w2.contiguous() if hid else None
    gate = torch.empty((B, C), device=x.device, dtype=torch.float32)
    with rt.observe("se_gate", bytes=4.0 * x.numel()):
        check(L.ffc_se_gate(ptr(x), B, C, H, W, 0, ptr(w1d), ptr(w2d), hid, ptr(gate), stream), "ffc_se_gate")
    zeros = torch.zeros(B * C, device=x.device, dtype=torch.float32)
    y = torch.empty_like(x)
    check(L.ffc_bn_act_apply(ptr(x), ptr(y), 1, B * C, H * W, ptr(gate), ptr(zeros), 0, 0.0, stream),
          "ffc_bn_act_apply")
    return y


def se_scale_backward_impl(x, dy, w1, w2):
    """ffc::se_scale_backward -> [dx, dw1, dw2] (x as saved by the op: made contiguous, as the forward's
    rt.require copy was)"""
    x = x.contiguous()
    dy = dy.contiguous()
    B, C, H, W = x.shape
    hid = w1.shape[0]
    dev = x.device
    dx = torch.empty_like(x)
    if not hid:   # Linear(C, 0) / Linear(0, C): empty weights get empty gradients; the gate is 0.5
        check(rt.lib().ffc_se_bwd(ptr(x), ptr(dy), B, C, H, W, None, None, 0, ptr(dx), None, None, None, None,
                                  ptr(torch.empty(4 * B * C, device=dev)), _stream(x)), "ffc_se_bwd")
        return [dx, torch.zeros_like(w1), torch.zeros_like(w2)]
    vec = lambda n: torch.empty((B, n, 1, 1), device=dev, dtype=torch.float32)  # noqa: E731
    dpre2, hact, dpre1, mean = vec(C), vec(hid), vec(hid), vec(C)
    ws = torch.empty(4 * B * C, device=dev, dtype=torch.float32)
    w1c, w2c = w1.contiguous(), w2.contiguous()
    with rt.observe("se_bwd", bytes=16.0 * x.numel()):
        check(rt.lib().ffc_se_bwd(ptr(x), ptr(dy), B, C, H, W, ptr(w1c), ptr(w2c), hid, ptr(dx), ptr(dpre2), ptr(hact),
                                  ptr(dpre1), ptr(mean), ptr(ws), _stream(x)), "ffc_se_bwd")
    dw1 = conv_wgrad(dpre1, mean, 1, 1, 0, 1, (hid, C))      # fc.0: (hid, C)
    dw2 = conv_wgrad(dpre2, hact, 1, 1, 0, 1, (C, hid))      # fc.2: (C, hid)
    return [dx, dw1, dw2]


def se_layer(se, x):
    if se.fc[0].bias is not None or se.fc[2].bias is not None:
        raise NotImplementedError("SELayer with bias")
    return torch.ops.ffc.se_scale(x, se.fc[0].weight, se.fc[2].weight)


# --------------------------------------------------------------------------- pool / upsample
def pool2_impl(x, scale):
    """ffc::pool2: scale * (sum of each 2x2 block) -- AvgPool2d(2, 2) at scale 0.25 (spectral_transform.py:46-47)"""
    x = rt.require(x, "x")
    B, C, H, W = x.shape
    if H % 2 or W % 2:
        raise NotImplementedError("AvgPool2d(2) downsample of an odd-sized input")
    y = torch.empty((B, C, H // 2, W // 2), device=x.device, dtype=torch.float32)
    check(rt.lib().ffc_pool2(ptr(x), B * C, H, W, float(scale), ptr(y), _stream(x)), "ffc_pool2")
    return y


def up2_impl(x, scale):
    """ffc::up2: scale * nearest x2 -- Upsample(scale_factor=2, mode='nearest') at scale 1 (:44-45)"""
    x = rt.require(x, "x")
    B, C, h, w = x.shape
    y = torch.empty((B, C, 2 * h, 2 * w), device=x.device, dtype=torch.float32)
    check(rt.lib().ffc_up2(ptr(x), B * C, h, w, float(scale), ptr(y), _stream(x)), "ffc_up2")
    return y


# --------------------------------------------------------------------------- NoiseInjection, Linear
def noise_inject_impl(x, weight, noise):
    """ffc::noise_inject: x + weight[c] * noise[b] (layers/noise_injection.py:25-32)"""
    x = rt.require(x, "x")
    B, C, H, W = x.shape
    noise = rt.require(noise, "noise")
    if tuple(noise.shape) != (B, 1, H, W) or (H * W) % 4:
        raise NotImplementedError("NoiseInjection: noise must be (B, 1, H, W) with H*W % 4 == 0")
    if weight.numel() != C:
        raise RuntimeError(f"NoiseInjection has {weight.numel()} channels, tensor has {C}")
    out = torch.empty_like(x)
    with rt.observe("noise_inject", bytes=8.0 * x.numel() + 4.0 * noise.numel()):
        check(rt.lib().ffc_noise_inject(ptr(x), ptr(weight.contiguous()), ptr(noise), ptr(out), B, C, H * W,
                                        _stream(x)), "ffc_noise_inject")
    return out


def noise_wgrad_impl(g, noise):
    """ffc::noise_wgrad: dweight[c] = sum g[:, c] * noise -> (1, C, 1, 1)"""
    g = g.contiguous()
    B, C, H, W = g.shape
    noise = noise.contiguous()   # the saved op input: a strided view (e.g. n[:, :1]) reads as dense (B, 1, H, W)
    if tuple(noise.shape) != (B, 1, H, W):
        raise RuntimeError(f"noise must be {(B, 1, H, W)}, got {tuple(noise.shape)}")
    dw = torch.empty(C, device=g.device, dtype=torch.float32)
    check(rt.lib().ffc_noise_wgrad(ptr(g), ptr(noise), B, C, H * W, ptr(dw), _stream(g)), "ffc_noise_wgrad")
    return dw.view(1, C, 1, 1)


def noise_inject(mod, x, noise=None):
    """NoiseInjection ``mod`` on the ffc::noise_inject op (noise drawn with normal_() as the reference
    does when not given)"""
    B, C, H, W = x.shape
    if noise is None:
        noise = x.new_empty(B, 1, H, W).normal_()
    return torch.ops.ffc.noise_inject(x, mod.weight, rt.require(noise, "noise"))


class _LinearAs1x1:
    """nn.Linear(K, N) seen by conv_layer as a 1x1 Conv2d on a 1x1 input: weight (N, K, 1, 1) is a view
    of the Linear's weight, so its gradient flows back to the parameter"""

    def __init__(self, lin: nn.Linear):
        self.weight = lin.weight.view(lin.out_features, lin.in_features, 1, 1)
        self.bias = lin.bias
        self.out_channels = lin.out_features


def linear(lin: nn.Linear, z):
    """nn.Linear forward + backward (fgan128_complete.py:453-455 noise_to_feature, and the spectral-norm
    fc of the fgan128 Discriminator, :540) -> (B, N)"""
    B, K = z.shape
    rt.sn_refresh_train(lin)   # the 1x1 view below must see this call's W / sigma
    (y,) = conv_layer(B, [(lin.out_features, 0, 0.0)], [(0, 0, _plan.Seg("pw", K, 1, 1), _LinearAs1x1(lin))],
                      [z.reshape(B, K, 1, 1)])
    return y.reshape(B, lin.out_features)


# --------------------------------------------------------------------------- FFTs
def rfft2_impl(x, mirror_scale):
    """ffc::rfft2: interleave(rfftn(x, ortho)) -> (B, 2C, H, W/2+1), mirrored bins x mirror_scale
    (0.5: the adjoint of irfftn)"""
    x = rt.require(x, "x")
    B, C, H, W = x.shape
    Z = torch.empty((B, 2 * C, H, W // 2 + 1), device=x.device, dtype=torch.float32)
    with rt.observe("rfft2", bytes=4.0 * x.numel() + 4.0 * Z.numel()):
        check(rt.lib().ffc_rfft2_planes(ptr(x), B * C, H, W, float(mirror_scale), ptr(Z), _stream(x)),
              "ffc_rfft2_planes")
    return Z


def irfft2_impl(Z, H, W, mirror_scale, r):
    """ffc::irfft2: irfftn(deinterleave(Z), s=(H, W), ortho) [+ r], mirrored bins x mirror_scale
    (2: the adjoint of rfftn)"""
    Z = rt.require(Z, "Z")
    B, C2 = Z.shape[:2]
    y = torch.empty((B, C2 // 2, H, W), device=Z.device, dtype=torch.float32)
    r = rt.require(r, "residual") if r is not None else None
    with rt.observe("irfft2", bytes=4.0 * Z.numel() + 4.0 * y.numel()):
        check(rt.lib().ffc_irfft2_planes(ptr(Z), B * (C2 // 2), H, W, float(mirror_scale), ptr(r), ptr(y),
                                         _stream(Z)), "ffc_irfft2_planes")
    return y


def fourier_unit(fu, x, residual: bool):
    """FourierUnitSN.forward (fourier_unity.py:32-56) [+ x] on the training path"""
    B, C, H, W = x.shape
    fu._check(C)
    if fu.mix_precision != "fp32":
        raise NotImplementedError("the training path computes the spectral mix in fp32 only (config 5's fp16 "
                                  "mix is forward-only)")
    if (H > 64 or W > 64) and not (H == W and H in (128,)):
        raise NotImplementedError("training-path Fourier unit: planes up to 64x64, or square 128x128")
    Z = torch.ops.ffc.rfft2(x, 1.0)
    seg = _plan.Seg("pw", 2 * C, H, W // 2 + 1)
    (U,) = conv_layer(B, [(2 * C, 0, 0.0)], [(0, 0, seg, fu.conv_layer)], [Z])
    R = bn_act(fu.bn, U, (1, 0.0))
    return torch.ops.ffc.irfft2(R, H, W, 1.0, x if residual else None)


def spectral_v(st, x):
    """v = s + fu(s), s = relu(bn1(conv1(se(downsample(x))))) (spectral_transform.py:77-108, before conv2)"""
    if st.groups != 1:
        raise NotImplementedError("grouped SpectralTransform (groups != 1) is not on the hot path")
    if st.stride == 2 and st.upsample:
        x = torch.ops.ffc.up2(x, 1.0)
    elif st.stride == 2:
        x = torch.ops.ffc.pool2(x, 0.25)
    x = se_layer(st.se_block, x)
    B, Cin, H, W = x.shape
    c = st.conv1.out_channels
    (t,) = conv_layer(B, [(c, 0, 0.0)], [(0, 0, _plan.Seg("pw", Cin, H, W), st.conv1)], [x])
    s = bn_act(st.bn1, t, (1, 0.0))
    return fourier_unit(st.fu, s, residual=True)
