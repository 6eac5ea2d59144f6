"""Drop-in ``FFC`` (reference: layers/ffc/ffc.py:10-99) and the shared HIP executor that
FFCTranspose (ffc_transpose.py) and FFC_BN_ACT (ffc_bn_act.py) also use.

The module forwards go through the custom ops of ops.py (``ffc::ffc_bn_act`` for inference, the
per-op training ops under autograd); _FFCExec is the executor those ops run.

Each output branch is ONE implicit-GEMM launch (both branches share it):
  out_l = convl2l(x_l) + convg2l(x_g)                      segments: conv, conv
  out_g = convl2g(x_l) + conv2(v),  v = s + fu(s)          segments: conv, 1x1 at output res
with the FFC_BN_ACT activation fused into the epilogue (or BN partials, then one
BN+activation pass when norm_layer is BatchNorm2d).  ``nn.Identity`` sub-convs keep the
reference semantics: they return their input (usually the int 0 of the tuple protocol).
"""
import ctypes

import torch
import torch.nn as nn

from .. import _autograd as ag
from .. import _plan
from .. import _runtime as rt
from .. import ops
from .spectral_transform import SpectralTransform


def layer_call(mod, ffc, x, y, act_l=(0, 0.0), act_g=(0, 0.0), bn_l=None, bn_g=None, noise=None, defer=False):
    """forward of FFC_BN_ACT / FFC / FFCTranspose ``mod`` whose FFC part is ``ffc``: the training ops
    when autograd needs them, else the fused ffc::ffc_bn_act op"""
    if y is not None and ffc.ratio_gout != 0:
        # the reference passes y into SpectralTransform / FourierUnitSN, whose BatchNorm2d.forward()
        # takes no label (fourier_unity.py:46-47), or into nn.Identity.forward (one argument)
        raise TypeError("FFC: the conditional (y) path is not supported (the reference raises in "
                        "FourierUnitSN, fourier_unity.py:46-47)")
    x_l, x_g = x if type(x) is tuple else (x, 0)
    if ag.wants_grad(mod, x_l, x_g):
        x_l, x_g = rt.materialize(x_l), rt.materialize(x_g)
        return ffc._run_train(x_l, x_g, None, act_l, act_g, bn_l, bn_g, noise)
    return ops.layer_forward(mod, x, noise, defer)


class _FFCExec:
    """mixin: fused execution of an FFC / FFCTranspose layer (run by the ffc::ffc_bn_act op)"""

    def _ffc_cache(self):
        c = self.__dict__.get("_exec_cache")
        if c is None:
            c = self.__dict__["_exec_cache"] = {}
        return c

    def _branch(self, parts):
        """parts: list of (module, input) whose outputs are summed.  -> (segments, weights, inputs, addends)"""
        segs, weights, inputs, addends = [], [], [], []
        for mod, inp in parts:
            if isinstance(mod, (nn.Conv2d, nn.ConvTranspose2d)):
                if not isinstance(inp, torch.Tensor):
                    raise TypeError(f"{type(mod).__name__} got {type(inp).__name__} input")
                rt.sn_refresh(mod)
                segs.append(rt.conv_seg(mod, inp))
                weights.append(rt.conv_weight(mod))
                inputs.append((inp, None))
            elif isinstance(mod, nn.Identity):
                if isinstance(inp, torch.Tensor):
                    addends.append(inp)       # Identity passes a tensor through
            else:
                raise NotImplementedError(f"{type(mod).__name__} in an FFC branch")
        return segs, weights, inputs, addends

    def _run(self, x, y=None, act_l=(0, 0.0), act_g=(0, 0.0), bn_l=None, bn_g=None, noise=None, defer=False):
        """noise: optional {"l"|"g": (NoiseInjection, noise tensor or None)} applied after the branch's
        BN + activation in the same pass (FFC_BN_ACT followed by the fgan128 NoiseInjection).
        defer: return rt.PendingAct outputs instead of running that pass (the consumer applies it).
        Inputs may be PendingAct: a consumer that cannot apply them materializes them first."""
        x_l, x_g = x if type(x) is tuple else (x, 0)
        if isinstance(x_l, rt.PendingAct) or isinstance(x_g, rt.PendingAct):
            out = self._run_pending(x_l, x_g, y, act_l, act_g, bn_l, bn_g, noise)
            if out is not None:
                return out
            x_l, x_g = rt.materialize(x_l), rt.materialize(x_g)
        if ag.wants_grad(self, x_l, x_g):
            return self._run_train(x_l, x_g, y, act_l, act_g, bn_l, bn_g, noise)
        if isinstance(x_l, torch.Tensor):
            x_l = rt.require(x_l, "x_l")
        if isinstance(x_g, torch.Tensor):
            x_g = rt.require(x_g, "x_g")
        ref = x_l if isinstance(x_l, torch.Tensor) else x_g
        if not isinstance(ref, torch.Tensor):
            raise TypeError("FFC input has no tensor branch")
        B, dev = ref.shape[0], ref.device
        stream = rt.stream_of(ref)
        branches = []  # (name, segs, weights, inputs, addends, act, bn, M)
        if self.ratio_gout != 1:
            segs, w, inp, add = self._branch([(self.convl2l, x_l), (self.convg2l, x_g)])
            M = self.convl2l.out_channels if isinstance(self.convl2l, (nn.Conv2d, nn.ConvTranspose2d)) else (
                self.convg2l.out_channels if isinstance(self.convg2l, (nn.Conv2d, nn.ConvTranspose2d)) else None)
            branches.append(("l", segs, w, inp, add, act_l, bn_l, M))
        spectral = (self.ratio_gout != 0 and isinstance(self.convg2g, SpectralTransform) and y is None and
                    isinstance(x_g, torch.Tensor))
        if rt.OVERLAP_SPECTRAL and spectral and branches and branches[0][1]:
            # The local branch does not depend on the spectral chain: its GEMM runs on the main stream
            # while SpectralTransform's latency-bound kernels run on a side stream (fork / join by
            # events, hipGraph-capturable); then the global-branch GEMM consumes v.
            main = torch.cuda.current_stream(dev)
            side = rt.side_stream(dev)
            side.wait_stream(main)
            if rt.OVERLAP_SPECTRAL == "spectral-first":
                with torch.cuda.stream(side):
                    v = self.convg2g.spectral(x_g)
                out_l, _ = self._launch_branches(branches, B, dev, stream, noise)
            else:
                out_l, _ = self._launch_branches(branches, B, dev, stream, noise)
                with torch.cuda.stream(side):
                    v = self.convg2g.spectral(x_g)
            main.wait_stream(side)
            v.record_stream(main)
            segs, w, inp, add = self._branch([(self.convl2g, x_l)])
            rt.sn_refresh(self.convg2g.conv2)
            segs.append(_plan.Seg("pw", v.shape[1], v.shape[2], v.shape[3]))
            w.append(rt.conv_weight(self.convg2g.conv2))
            inp.append((v, None))
            M = self.convl2g.out_channels if isinstance(self.convl2g, (nn.Conv2d, nn.ConvTranspose2d)) else \
                self.convg2g.conv2.out_channels
            _, out_g = self._launch_branches([("g", segs, w, inp, add, act_g, bn_g, M)], B, dev, stream, noise)
            return out_l, out_g
        if self.ratio_gout != 0:
            segs, w, inp, add = self._branch([(self.convl2g, x_l)])
            if not isinstance(self.convg2g, nn.Identity):
                if isinstance(self.convg2g, SpectralTransform):
                    if y is not None:
                        raise TypeError("FFC: the conditional (y) path is not supported (the reference raises in "
                                        "FourierUnitSN, fourier_unity.py:46-47)")
                    if not isinstance(x_g, torch.Tensor):
                        raise TypeError("spectral branch needs a tensor x_g")
                    v = self.convg2g.spectral(x_g)
                    st = self.convg2g
                    rt.sn_refresh(st.conv2)
                    segs.append(_plan.Seg("pw", v.shape[1], v.shape[2], v.shape[3]))
                    w.append(rt.conv_weight(st.conv2))
                    inp.append((v, None))
                else:
                    raise NotImplementedError(type(self.convg2g).__name__)
            M = self.convl2g.out_channels if isinstance(self.convl2g, (nn.Conv2d, nn.ConvTranspose2d)) else (
                self.convg2g.conv2.out_channels if isinstance(self.convg2g, SpectralTransform) else None)
            branches.append(("g", segs, w, inp, add, act_g, bn_g, M))
        return self._launch_branches(branches, B, dev, stream, noise, defer)

    def _run_pending(self, x_l, x_g, y, act_l, act_g, bn_l, bn_g, noise):
        """Inputs with deferred BN + activation (+ noise): the direct 3x3 head (fgan128 conv7: local output
        only, no BN, both inputs convs) reads them through ffc_in_tf.  -> (out_l, 0) or None (not fusable)"""
        if y is not None or noise or bn_l is not None or self.ratio_gout != 0 or ag.wants_grad(self, x_l, x_g):
            return None
        parts = [(self.convl2l, x_l), (self.convg2l, x_g)]
        if not all(isinstance(m, nn.Conv2d) and isinstance(t, (torch.Tensor, rt.PendingAct)) for m, t in parts):
            return None
        raw = [t.raw if isinstance(t, rt.PendingAct) else rt.require(t, "x") for _, t in parts]
        segs, w, inp, add = self._branch([(m, r) for (m, _), r in zip(parts, raw)])
        M = self.convl2l.out_channels
        if self._smallm_kind(segs, w, None, None, M) != "conv3":
            return None
        tfs = [t if isinstance(t, rt.PendingAct) else None for _, t in parts]
        return self._smallm("conv3", segs, w, inp, act_l, M, raw[0].shape[0], raw[0].device,
                            rt.stream_of(raw[0]), tfs=tfs), 0

    def _run_train(self, x_l, x_g, y, act_l, act_g, bn_l, bn_g, noise):
        """training path (autograd recording): the layer's local convs and ST conv2 as one
        _ConvLayerFn (both output branches; their data gradients w.r.t. x_l in one adjoint launch),
        SpectralTransform through its per-op Functions, BN + activation as _BNActFn
        (include/ffc_amd.h "training path")."""
        if y is not None:
            raise TypeError("FFC: the conditional (y) path is not supported (the reference raises in "
                            "FourierUnitSN, fourier_unity.py:46-47)")
        for t, n in ((x_l, "x_l"), (x_g, "x_g")):
            if isinstance(t, torch.Tensor):
                rt.require(t, n)
        ref = x_l if isinstance(x_l, torch.Tensor) else x_g
        if not isinstance(ref, torch.Tensor):
            raise TypeError("FFC input has no tensor branch")
        B = ref.shape[0]
        inputs, idx, outs, edges, names = [], {}, [], [], []

        def inp(t):
            if id(t) not in idx:
                idx[id(t)] = len(inputs)
                inputs.append(t.contiguous())
            return idx[id(t)]

        def branch(parts, extra=None):
            convs = []
            for mod, t in parts:
                if isinstance(mod, (nn.Conv2d, nn.ConvTranspose2d)):
                    if not isinstance(t, torch.Tensor):
                        raise TypeError(f"{type(mod).__name__} got {type(t).__name__} input")
                    convs.append((mod, t))
                elif isinstance(t, torch.Tensor):
                    raise NotImplementedError("identity pass-through of a tensor on the training path")
            return convs + ([extra] if extra else [])

        for name, parts, extra, act, bn in (
                ("l", [(self.convl2l, x_l), (self.convg2l, x_g)], None, act_l, bn_l),
                ("g", [(self.convl2g, x_l)], "st", act_g, bn_g)):
            if (name == "l" and self.ratio_gout == 1) or (name == "g" and self.ratio_gout == 0):
                continue
            ex = None
            if extra and isinstance(self.convg2g, SpectralTransform) and isinstance(x_g, torch.Tensor):
                v = ag.spectral_v(self.convg2g, x_g)
                ex = (self.convg2g.conv2, v, _plan.Seg("pw", v.shape[1], v.shape[2], v.shape[3]))
            elif extra and not isinstance(self.convg2g, nn.Identity):
                raise NotImplementedError(type(self.convg2g).__name__)
            convs = branch(parts)
            if not convs and ex is None:
                continue
            j = len(outs)
            M = (convs[0][0] if convs else ex[0]).out_channels
            outs.append((M,) + (tuple(act) if bn is None else (0, 0.0)))
            for mod, t in convs:
                edges.append((j, inp(t), rt.conv_seg(mod, t), mod))
            if ex is not None:
                edges.append((j, inp(ex[1]), ex[2], ex[0]))
            names.append((name, act, bn))
        res = {"l": 0, "g": 0}
        if outs:
            ys = ag.conv_layer(B, outs, edges, inputs)
            for (name, act, bn), yv in zip(names, ys):
                res[name] = ag.bn_act(bn, yv, act) if bn is not None else yv
        for name, (mod, n) in (noise or {}).items():   # fgan128's NoiseInjection after FFC_BN_ACT
            if isinstance(res[name], torch.Tensor):
                res[name] = ag.noise_inject(mod, res[name], n)
        return res["l"], res["g"]

    def _launch_branches(self, branches, B, dev, stream, noise=None, defer=False):
        """plan / pack / launch the GEMM(s) of the given branches (one launch per kernel kind),
        then BN statistics and BN+activation passes (defer: PendingAct outputs instead of those
        passes).  -> (out_l, out_g)"""
        outs = {"l": 0, "g": 0}
        execs, jobs, post, built = [], [], [], []
        jb_name = {}
        dense = []   # (name, (W (M', C, 1, 1), layout, 1, 1, bias), input, out, act, M')
        for name, segs, w, inp, add, act, bn, M in branches:
            if len(add) > 1:
                raise NotImplementedError("more than one identity pass-through in a branch")
            addend = add[0] if add else None
            if not segs:
                # no convolution: the branch is its pass-through (or the int 0)
                if addend is None:
                    continue
                out = addend.clone()
                outs[name] = out
                post.append((name, out, act, bn, None, 0))
                continue
            smk = self._smallm_kind(segs, w, addend, bn, M)
            if smk is not None:
                out = self._smallm(smk, segs, w, inp, act, M, B, dev, stream)
                outs[name] = out
                continue
            out_shape = None
            if addend is None and bn is None:
                rw = self._outer_rewrite(segs, w, M)
                if rw is not None and len(segs) == 1:
                    # a plain GEMM: batched with the other branch's into one dense launch below
                    segs2, w2, M2, chw = rw
                    out = torch.empty((B,) + chw, device=dev, dtype=torch.float32)
                    outs[name] = out
                    dense.append((name, w2[0], inp[0][0], out, act, M2))
                    continue
                if rw is not None:
                    segs, w, M, chw = rw
                    out_shape = (B,) + chw
            key = (name, B, tuple(segs), str(dev))
            cache = self._ffc_cache()
            ex = cache.get(key)
            if ex is None:
                ex = cache[key] = rt.ConvExec(B, M, segs, w, dev)
            ex.ensure_packed(w)
            pl = ex.plan
            out = torch.empty(out_shape or (B, pl.M, pl.OH, pl.OW), device=dev, dtype=torch.float32)
            if addend is not None and tuple(addend.shape) != tuple(out.shape):
                raise RuntimeError(f"shape mismatch adding pass-through {tuple(addend.shape)} to {tuple(out.shape)}")
            outs[name] = out
            jb_name[id(out)] = name
            execs.append(ex)
            jobs.append((ex, inp, out, act, bn, addend))
            built.append((key, B, M, segs, w))
        if dense:
            self._launch_dense(dense, B, stream)
        # the layer's convq jobs share one launch, so one configuration: when they picked different
        # ones (untuned shapes), rebuild them on the costliest job's (cached: happens once)
        qi = [i for i, jb in enumerate(jobs) if jb[0].launch_key[0] == "q"]
        if len({jobs[i][0].launch_key for i in qi}) > 1:
            # the decision is cached per layer shape, including "this job cannot take that cfg" (it
            # stays on its own kernel): nothing is re-planned or re-packed on later forwards
            cache = self._ffc_cache()
            rkey = ("rebuild",) + tuple(built[i][0] for i in qi)
            dec = cache.get(rkey)
            if dec is None:
                cfg = max((jobs[i][0].plan for i in qi), key=_plan.convq_cost).cfg
                dec = {}
                for i in qi:
                    ckey, cB, cM, csegs, cw = built[i]
                    ex2 = rt.ConvExec(cB, cM, csegs, cw, dev, convq_cfg=cfg)
                    if ex2.launch_key[0] == "q":
                        cache[ckey] = dec[i] = ex2
                cache[rkey] = dec
            for i, ex2 in dec.items():
                ex2.ensure_packed(built[i][4])
                jobs[i] = (ex2,) + jobs[i][1:]
        groups = {}
        for jb in jobs:
            groups.setdefault(jb[0].launch_key, []).append(jb)
        cache = self._ffc_cache()
        for gjobs in groups.values():
            lkey = ("launch",) + tuple(id(j[0]) for j in gjobs)
            lp = cache.get(lkey)
            if lp is None:
                lp = cache[lkey] = rt.LaunchPlan([j[0] for j in gjobs], dev)
            structs = []
            for ji, (ex, inp, out, act, bn, addend) in enumerate(gjobs):
                slab = None
                if bn is not None and rt.bn_mode(bn)[0]:
                    slab = torch.empty((lp.stat_rows(ji), ex.plan.M, 4), device=dev, dtype=torch.float32)
                fused_act = act if bn is None else (0, 0.0)
                structs.append(ex.job(inp, out, fused_act[0], fused_act[1], addend, slab))
                if bn is not None:
                    post.append((jb_name[id(out)], out, act, bn, slab, lp.stat_rows(ji)))
            lp.launch(structs, stream, flops=sum(j[0].flops for j in gjobs))
        noise = noise or {}
        done = set()
        applies = []
        # the layer's slab-backed BNs (bn_l, bn_g) finalized together: one SyncBN all-reduce for both
        slab_bns = [(bn, out.shape[1], slab, nrows, 1.0) for _, out, _, bn, slab, nrows in post
                    if bn is not None and slab is not None]
        ss = dict(zip((id(it[0]) for it in slab_bns), rt.bn_scale_shift_many(slab_bns, dev, stream)))
        for name, out, act, bn, slab, nrows in post:
            C = out.shape[1]
            nz = noise.get(name)
            if bn is not None:
                if slab is not None:
                    sc, sh = ss[id(bn)]
                else:
                    sc, sh = rt.bn_scale_shift(bn, C, slab, nrows, 1.0, dev, stream) if not rt.bn_mode(bn)[0] \
                        else self._bn_from_tensor(bn, out, stream)
            else:
                if act[0] == 0 and nz is None:
                    continue
                sc = torch.ones(C, device=dev, dtype=torch.float32)
                sh = torch.zeros(C, device=dev, dtype=torch.float32)
            if defer:
                outs[name] = rt.PendingAct(out, sc, sh, act[0], act[1], *(nz if nz is not None else (None, None)))
                done.add(name)
                continue
            # the global output's plane sums for the next layer's SE gate (large planes, where the
            # SpectralTransform reads y twice otherwise: spectral_transform.py pw path)
            HW = out.shape[2] * out.shape[3]
            ps = None
            if name == "g" and rt.SE_SUMS and HW % 4 == 0 and HW >= 256:
                chunks = rt.lib().ffc_plane_chunks(HW)
                ps = torch.empty((out.shape[0], out.shape[1], chunks), device=dev, dtype=torch.float32)
            if nz is not None and HW % 4 == 0:
                # the noise drawn here, in branch order, as the single pass does; applied below
                p = rt.PendingAct(out, sc, sh, act[0], act[1], *nz)
                applies.append((out, sc, sh, act[0], act[1], p.noise_w, p.noise, ps))
                done.add(name)
            else:
                applies.append((out, sc, sh, act[0], act[1], None, None, ps))
            if ps is not None:
                out._ffc_plane_sums = (ps, chunks, out._version)
        if applies:   # the layer's BN + activation (+ noise) passes in one launch
            rt.bn_act_apply_batch(applies)
        for name, (mod, n) in noise.items():   # branches without a BN/activation pass of their own
            if name not in done and isinstance(outs[name], torch.Tensor):
                outs[name] = mod(outs[name], n)
        return outs["l"], outs["g"]

    def _outer_rewrite(self, segs, w, M):
        """ConvTranspose2d(k, s=1, p=0) on a 1x1 input (the generator's first layer, ffc0:
        ffc_transpose.py:79-86 on z of shape (B, nz, 1, 1)) is an outer product: out[b, m, y, x] =
        sum_c z[b, c] W[c, m, y, x].  As ONE GEMM with M' = M*k*k "channels" at 1x1 (the output
        (B, M, k, k) has the memory layout of (B, M*k*k, 1, 1)) it fills the GPU with tiles instead
        of 16 tiny per-phase GEMMs.  -> (segments, weights, M', output shape) or None."""
        if M is None or not segs or not rt.USE_OUTER:
            return None
        k = segs[0].k
        for sg in segs:
            if (sg.kind, sg.IH, sg.IW, sg.s, sg.p, sg.d, sg.op, sg.k) != ("convT", 1, 1, 1, 0, 1, 0, k):
                return None
        cache = self._ffc_cache()
        segs2, w2 = [], []
        for sg, (wt, lay, kh, kw, bias) in zip(segs, w):
            key = ("outer", wt.data_ptr(), rt.weight_key(wt), rt.weight_key(bias))
            hit = cache.get(key)
            if hit is None:
                for old in [kk for kk in cache if kk[0] == "outer" and kk[1] == wt.data_ptr()]:
                    del cache[old]
                wr = wt.permute(1, 2, 3, 0).reshape(M * k * k, sg.C, 1, 1).contiguous()   # (C,M,k,k) -> (M k k, C)
                br = bias.repeat_interleave(k * k).contiguous() if bias is not None else None
                rt.note_tensors([wr, br])   # the dense launch's packed-weight key is taken from these
                hit = cache[key] = (wr, br)
            segs2.append(_plan.Seg("pw", sg.C, 1, 1))
            w2.append((hit[0], 0, 1, 1, hit[1]))
        return segs2, w2, M * k * k, (M, k, k)

    def _launch_dense(self, dense, B, stream):
        """outer-product branches (ConvT on a 1x1 input) as ffc_dense_forward launches; two branches with
        the same input and activation share one launch (their weights concatenated along N, cached)"""
        cache = self._ffc_cache()
        groups = []
        for d in dense:
            for g in groups:
                if len(g) == 1 and g[0][2].data_ptr() == d[2].data_ptr() and g[0][4] == d[4]:
                    g.append(d)
                    break
            else:
                groups.append([d])
        for g in groups:
            wts = [d[1] for d in g]
            key = ("dense",) + tuple((wt[0].data_ptr(), rt.weight_key(wt[0]), rt.weight_key(wt[4])) for wt in wts)
            hit = cache.get(key)
            if hit is None:
                for old in [kk for kk in cache if kk[0] == "dense" and kk[1][0] == key[1][0]]:
                    del cache[old]
                Wt = torch.cat([wt[0].reshape(wt[0].shape[0], -1).t() for wt in wts], dim=1).contiguous()
                has_b = any(wt[4] is not None for wt in wts)
                bias = torch.cat([wt[4] if wt[4] is not None else torch.zeros(wt[0].shape[0], device=Wt.device)
                                  for wt in wts]).contiguous() if has_b else None
                hit = cache[key] = (Wt, bias)
            Wt, bias = hit
            x = g[0][2]
            K, N = Wt.shape
            N0 = g[0][5]
            act = g[0][4]
            with rt.observe("dense", flops=2.0 * B * K * N):
                rt.check(rt.lib().ffc_dense_forward(x.data_ptr(), Wt.data_ptr(), rt.ptr(bias), B, K, N, N0,
                                                    g[0][3].data_ptr(), rt.ptr(g[1][3]) if len(g) > 1 else None,
                                                    act[0], act[1], stream), "ffc_dense_forward")

    @staticmethod
    def _smallm_kind(segs, w, addend, bn, M):
        """<= 4 output channels -> direct VALU kernel: 'convT' for ConvT k4 s2 p1 (the generator's last
        layer, models/ffc_generator.py:28), 'conv3' for Conv k3 s1 p1 (the fgan128 head conv7,
        fgan128_complete.py:484), else None"""
        if not rt.USE_SMALLM or addend is not None or bn is not None or M is None or M > 4 or \
                not 1 <= len(segs) <= 2:
            return None
        if sum(1 for x in w if x[4] is not None) > 1:
            return None
        if not all(sg.IH == segs[0].IH and sg.IW == segs[0].IW for sg in segs):
            return None
        if all(sg.kind == "convT" and (sg.k, sg.s, sg.p, sg.d, sg.op) == (4, 2, 1, 1, 0) for sg in segs):
            return "convT"
        if all(sg.kind == "conv" and sg.k == sg.IH == sg.IW and sg.p == 0 and sg.d == 1 and not sg.pool
               for sg in segs) and all(x[1] == 0 for x in w):
            return "full"   # Conv2d onto a 1x1 output (FFCDiscriminator's last layer)
        if segs[0].IW % 4 == 0 and all(sg.kind == "conv" and (sg.k, sg.s, sg.p, sg.d) == (3, 1, 1, 1) for sg in segs):
            return "conv3"
        return None

    def _smallm(self, kind, segs, w, inp, act, M, B, dev, stream, tfs=None):
        IH, IW = segs[0].IH, segs[0].IW
        x1 = inp[1][0] if len(inp) > 1 else None
        w1 = w[1][0] if len(w) > 1 else None
        bias = next((x[4] for x in w if x[4] is not None), None)
        C1 = segs[1].C if x1 is not None else 0
        if kind == "convT":
            # weights packed [C0 + C1][16 taps][4] by a HIP kernel, cached per (pointer, version)
            cache = self._ffc_cache()
            key = ("ctpack", w[0][0].data_ptr(), rt.weight_key(w[0][0]), rt.weight_key(w1))
            wp = cache.get(key)
            if wp is None:
                for old in [kk for kk in cache if kk[0] == "ctpack" and kk[1] == key[1]]:
                    del cache[old]
                wp = cache[key] = torch.empty(rt.lib().ffc_convt_smallm_pack_floats(segs[0].C, C1), device=dev,
                                              dtype=torch.float32)
                rt.check(rt.lib().ffc_convt_smallm_pack(w[0][0].data_ptr(), segs[0].C, rt.ptr(w1), C1, M,
                                                        wp.data_ptr(), stream), "ffc_convt_smallm_pack")
            out = torch.empty((B, M, 2 * IH, 2 * IW), device=dev, dtype=torch.float32)
            flops = 2.0 * B * M * sum(sg.C for sg in segs) * 4 * (2 * IH) * (2 * IW)
            with rt.observe("convt_smallm", flops=flops):
                rt.check(rt.lib().ffc_convt_k4s2_smallm(inp[0][0].data_ptr(), segs[0].C, rt.ptr(x1), C1,
                                                        wp.data_ptr(), rt.ptr(bias), B, IH, IW, M, out.data_ptr(),
                                                        act[0], act[1], stream), "ffc_convt_k4s2_smallm")
            return out
        if kind == "full":
            return ag.conv_forward(self._ffc_cache(), ("inf_full",), B, M, tuple(segs), w,
                                   [x for x, _ in inp], act=act)
        out = torch.empty((B, M, IH, IW), device=dev, dtype=torch.float32)
        flops = 2.0 * B * M * sum(sg.C for sg in segs) * 9 * IH * IW
        if tfs is not None and any(t is not None for t in tfs):
            st = [t.struct() if t is not None else None for t in tfs] + [None]
            with rt.observe("conv3_smallm", flops=flops):
                rt.check(rt.lib().ffc_conv3x3_smallm_tf(inp[0][0].data_ptr(), segs[0].C, w[0][0].data_ptr(),
                                                        rt.ptr(x1), C1, rt.ptr(w1), rt.ptr(bias), B, IH, IW, M,
                                                        out.data_ptr(), act[0], act[1],
                                                        None if st[0] is None else ctypes.byref(st[0]),
                                                        None if st[1] is None else ctypes.byref(st[1]), stream),
                         "ffc_conv3x3_smallm_tf")
            return out
        with rt.observe("conv3_smallm", flops=flops):
            rt.check(rt.lib().ffc_conv3x3_smallm(inp[0][0].data_ptr(), segs[0].C, w[0][0].data_ptr(), rt.ptr(x1), C1,
                                                 rt.ptr(w1), rt.ptr(bias), B, IH, IW, M, out.data_ptr(),
                                                 act[0], act[1], stream), "ffc_conv3x3_smallm")
        return out

    def _bn_from_tensor(self, bn, out, stream):
        """batch statistics of a pass-through branch (no GEMM epilogue to collect them)"""
        B, C = out.shape[:2]
        ex = self._ffc_cache().get(("bnstats", tuple(out.shape), str(out.device)))
        if ex is None:
            seg = _plan.Seg("pw", C, out.shape[2], out.shape[3])
            eye = nn.Conv2d(C, C, 1, bias=False).to(out.device)
            with torch.no_grad():
                eye.weight.zero_()
                eye.weight[:, :, 0, 0] = torch.eye(C, device=out.device)
            ex = (rt.ConvExec(B, C, [seg], [rt.conv_weight(eye)], out.device), eye)
            self._ffc_cache()[("bnstats", tuple(out.shape), str(out.device))] = ex
        cexec, _ = ex
        lp = rt.LaunchPlan([cexec], out.device)
        slab = torch.empty((lp.stat_rows(0), C, 4), device=out.device, dtype=torch.float32)
        tmp = torch.empty_like(out)
        lp.launch([cexec.job([(out, None)], tmp, stats=slab)], stream)
        return rt.bn_scale_shift(bn, C, slab, lp.stat_rows(0), 1.0, out.device, stream)


class FFC(_FFCExec, nn.Module):
    def __init__(self, in_channels: int, out_channels: int, kernel_size: int,
                 ratio_gin: float, ratio_gout: float, stride: int = 1, padding: int = 0,
                 dilation: int = 1, groups: int = 1, bias: bool = False, enable_lfu: bool = True,
                 attention: bool = False, num_classes: int = 1):
        super().__init__()
        assert stride == 1 or stride == 2, "Stride should be 1 or 2."
        self._ffc_ctor = ["FFC", dict(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                                      ratio_gin=ratio_gin, ratio_gout=ratio_gout, stride=stride, padding=padding,
                                      dilation=dilation, groups=groups, bias=bias, enable_lfu=enable_lfu,
                                      num_classes=num_classes)]
        self.stride = stride
        in_cg = int(in_channels * ratio_gin)
        in_cl = in_channels - in_cg
        out_cg = int(out_channels * ratio_gout)
        out_cl = out_channels - out_cg
        print("in_cl, in_cg, out_cl, out_cg")   # the reference prints at construction (ffc.py:38-39)
        print(in_cl, in_cg, out_cl, out_cg)
        self.ratio_gin = ratio_gin
        self.ratio_gout = ratio_gout
        module = nn.Identity if (in_cl == 0 or out_cl == 0) else nn.Conv2d
        self.convl2l = module(in_cl, out_cl, kernel_size, stride, padding, dilation, groups, bias)
        module = nn.Identity if (in_cl == 0 or out_cg == 0) else nn.Conv2d
        self.convl2g = module(in_cl, out_cg, kernel_size, stride, padding, dilation, groups, bias)
        module = nn.Identity if (in_cg == 0 or out_cl == 0) else nn.Conv2d
        self.convg2l = module(in_cg, out_cl, kernel_size, stride, padding, dilation, groups, bias)
        module = nn.Identity if in_cg == 0 or out_cg == 0 else SpectralTransform
        self.convg2g = module(in_cg, out_cg, stride, 1 if groups == 1 else groups // 2, enable_lfu, False,
                              num_classes)

    def forward(self, x, y=None):
        return layer_call(self, self, x, y)
