"""torch.library.opcheck over every ffc:: custom op (schema / mutation declarations, fake vs real
metadata, autograd registration, AOT dispatch with dynamic shapes) on real HIP tensors, plus the
module forward through the op against a direct call of the op."""
import contextlib
import io

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _opcheck(op, args, **kw):
    res = torch.library.opcheck(op, args, kw or None, raise_exception=False)
    bad = {k: v for k, v in res.items() if v != "SUCCESS"}
    assert not bad, f"{op}: {bad}"


def _quiet(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


def test_opcheck_conv_layer():
    from fastfourierconvolution_amd import _autograd as ag
    from fastfourierconvolution_amd import _plan
    x = torch.randn(4, 16, 8, 8, device=DEV, requires_grad=True)
    x2 = torch.randn(4, 8, 8, 8, device=DEV, requires_grad=True)
    w = (0.1 * torch.randn(16, 32, 4, 4, device=DEV)).requires_grad_()     # ConvTranspose2d(16, 32, 4, 2, 1)
    w2 = (0.1 * torch.randn(8, 32, 4, 4, device=DEV)).requires_grad_()
    b = torch.randn(32, device=DEV, requires_grad=True)
    for act in (0, 2, 5):   # Identity, LeakyReLU (fused), GELU (pre-activation output too)
        spec = ag.conv_spec([(32, act, 0.1)], [(0, 0, _plan.Seg("convT", 16, 8, 8, 4, 2, 1), 1, 0),
                                               (0, 1, _plan.Seg("convT", 8, 8, 8, 4, 2, 1), 1, -1)])
        _opcheck(torch.ops.ffc.conv_layer.default, ([x, x2], [w, w2], [b], spec))
    wc = (0.1 * torch.randn(24, 16, 3, 3, device=DEV)).requires_grad_()   # Conv2d 3x3 s1 p1 into two outputs
    spec = ag.conv_spec([(24, 1, 0.0), (24, 0, 0.0)], [(0, 0, _plan.Seg("conv", 16, 8, 8, 3, 1, 1), 0, -1),
                                                       (1, 0, _plan.Seg("conv", 16, 8, 8, 3, 1, 1), 0, -1)])
    _opcheck(torch.ops.ffc.conv_layer.default, ([x], [wc, wc], [], spec))


@pytest.mark.parametrize("use_batch", [True, False])
def test_opcheck_bn_act(use_batch):
    x = torch.randn(4, 16, 8, 8, device=DEV, requires_grad=True)
    g = (1 + 0.1 * torch.randn(16, device=DEV)).requires_grad_()
    b = (0.1 * torch.randn(16, device=DEV)).requires_grad_()
    rm, rv = 0.1 * torch.randn(16, device=DEV), 0.5 + torch.rand(16, device=DEV)
    for act in (1, 5):
        _opcheck(torch.ops.ffc.bn_act.default, (x, g, b, rm, rv, use_batch, 1e-5, act, 0.0))
    _, _, _, stats = torch.ops.ffc.bn_act(x.detach(), g.detach(), b.detach(), rm, rv, True, 1e-5, 1, 0.0)
    nbt = torch.tensor(3, device=DEV, dtype=torch.long)
    _opcheck(torch.ops.ffc.bn_update_running.default, (rm.clone(), rv.clone(), nbt, stats, 0.1, 1.0))


def test_opcheck_small_ops():
    x = torch.randn(4, 16, 8, 8, device=DEV, requires_grad=True)
    _opcheck(torch.ops.ffc.pool2.default, (x, 0.25))
    _opcheck(torch.ops.ffc.up2.default, (x, 1.0))
    _opcheck(torch.ops.ffc.rfft2.default, (x, 1.0))
    Z = torch.randn(4, 32, 8, 5, device=DEV, requires_grad=True)
    _opcheck(torch.ops.ffc.irfft2.default, (Z, 8, 8, 1.0, None))
    _opcheck(torch.ops.ffc.irfft2.default, (Z, 8, 8, 1.0, x))
    for hid in (1, 0):   # SELayer(16): hidden 16 // 16 = 1; SELayer(8): hidden 0 (gate 0.5)
        w1 = (0.3 * torch.randn(hid, 16, device=DEV)).requires_grad_()
        w2 = (0.3 * torch.randn(16, hid, device=DEV)).requires_grad_()
        _opcheck(torch.ops.ffc.se_scale.default, (x, w1, w2))
    w = (0.1 * torch.randn(1, 16, 1, 1, device=DEV)).requires_grad_()
    _opcheck(torch.ops.ffc.noise_inject.default, (x, w, torch.randn(4, 1, 8, 8, device=DEV)))
    z = torch.randn(8, 128, device=DEV)
    _opcheck(torch.ops.ffc.linear.default, (z, torch.randn(256, 128, device=DEV), torch.randn(256, device=DEV)))
    _opcheck(torch.ops.ffc.quantize_u8.default, (torch.randn(2, 3, 16, 16, device=DEV),))


def _layer_args(m, x_l, x_g):
    from fastfourierconvolution_amd import ops
    spec = ops.layer_spec(m)
    params, buffers = ops.layer_tensors(m, spec)
    return (x_l, x_g, [p.detach() for p in params], [b.clone() for b in buffers], [], [], [], False, spec)


@pytest.mark.parametrize("train", [True, False])
def test_opcheck_layer_ops(train):
    import fastfourierconvolution_amd as F
    blk = _quiet(F.FFC_BN_ACT, 32, 32, 3, 0.5, 0.5, 1, 1, norm_layer=nn.BatchNorm2d,
                 activation_layer=nn.ReLU).to(DEV).train(train)
    xl, xg = torch.randn(4, 16, 32, 32, device=DEV), torch.randn(4, 16, 32, 32, device=DEV)
    _opcheck(torch.ops.ffc.ffc_bn_act.default, _layer_args(blk, xl, xg))
    up = _quiet(F.FFC_BN_ACT, 256, 128, 4, 0.5, 0.5, 2, 1, activation_layer=nn.LeakyReLU,
                upsampling=True).to(DEV).train(train)                                 # FFCGenerator ffc2
    _opcheck(torch.ops.ffc.ffc_bn_act.default, _layer_args(up, torch.randn(8, 128, 8, 8, device=DEV),
                                                           torch.randn(8, 128, 8, 8, device=DEV)))
    first = _quiet(F.FFC_BN_ACT, 100, 512, 4, 0, 0.5, 1, 0, activation_layer=nn.LeakyReLU,
                   upsampling=True).to(DEV).train(train)                              # ffc0: x_g is the int 0
    _opcheck(torch.ops.ffc.ffc_bn_act.default, _layer_args(first, torch.randn(8, 100, 1, 1, device=DEV), None))
    from fastfourierconvolution_amd import ops
    st = _quiet(F.SpectralTransform, 64, 64, 2, upsample=True).to(DEV).train(train)
    spec = ops.layer_spec(st)
    p, b = ops.layer_tensors(st, spec)
    _opcheck(torch.ops.ffc.spectral_transform.default, (torch.randn(8, 64, 8, 8, device=DEV),
                                                        [t.detach() for t in p], [t.clone() for t in b], spec))
    fu = F.FourierUnitSN(16, 16).to(DEV).train(train)
    spec = ops.layer_spec(fu)
    p, b = ops.layer_tensors(fu, spec)
    _opcheck(torch.ops.ffc.fourier_unit.default, (torch.randn(4, 16, 32, 32, device=DEV),
                                                  [t.detach() for t in p], [t.clone() for t in b], spec))


def test_module_forward_is_the_op():
    """FFC_BN_ACT.forward under no_grad == the ffc::ffc_bn_act op on the module's tensors, bit for bit
    (eval mode: no running-stat side effects between the calls)"""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import ops
    blk = _quiet(F.FFC_BN_ACT, 32, 32, 3, 0.5, 0.5, 1, 1, norm_layer=nn.BatchNorm2d,
                 activation_layer=nn.ReLU).to(DEV).eval()
    xl, xg = torch.randn(4, 16, 32, 32, device=DEV), torch.randn(4, 16, 32, 32, device=DEV)
    with torch.no_grad():
        ol, og = blk((xl, xg))
        spec = ops.layer_spec(blk)
        p, b = ops.layer_tensors(blk, spec)
        rl, rg = torch.ops.ffc.ffc_bn_act(xl, xg, p, b, [], [], [], False, spec)[:2]
    assert torch.equal(ol, rl) and torch.equal(og, rg)


def test_two_models_same_structure_do_not_share_packed_weights():
    """the layer ops' packed-weight caches are keyed by the weight tensor object (rt.weight_key): two
    generators of one structure, built and freed in turn, never see each other's packs"""
    import fastfourierconvolution_amd as F
    z = torch.randn(16, 100, 1, 1, device=DEV)
    outs = []
    for seed in (1, 2, 1):
        torch.manual_seed(seed)
        g = _quiet(F.FFCGenerator, 100, 3, 32).to(DEV).eval()
        with torch.no_grad():
            outs.append(g(z).clone())
        del g
        torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[2]) and not torch.equal(outs[0], outs[1])


# --------------------------------------------------------------------------- round 5: ADVICE r04 regressions
def test_noise_wgrad_strided_noise():
    """ffc::noise_inject saves the caller's noise; a strided view (a channel slice of a wider tensor)
    must give the same weight gradient as its dense copy (noise_wgrad assumed dense)"""
    from fastfourierconvolution_amd.layers_misc import NoiseInjection
    mod = NoiseInjection(8).to(DEV)
    with torch.no_grad():
        mod.weight.copy_(torch.randn_like(mod.weight))
    x = torch.randn(4, 8, 16, 16, device=DEV)
    wide = torch.randn(4, 3, 16, 16, device=DEV)
    g = torch.randn(4, 8, 16, 16, device=DEV)
    grads = []
    for n in (wide[:, 1:2], wide[:, 1:2].contiguous()):
        mod.weight.grad = None
        xs = x.clone().requires_grad_()
        y = torch.ops.ffc.noise_inject(xs, mod.weight, n)
        (y * g).sum().backward()
        grads.append(mod.weight.grad.clone())
    assert not wide[:, 1:2].is_contiguous()
    assert torch.equal(grads[0], grads[1])
    ref = (g * wide[:, 1:2]).sum(dim=(0, 2, 3)).view_as(grads[0])
    torch.testing.assert_close(grads[0], ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("op", ["bn_act", "se_scale"])
def test_backward_channels_last_input(op):
    """ffc::bn_act / ffc::se_scale called directly with a channels_last x: dx and the parameter
    gradients equal those of the same values in NCHW (the backward read the saved raw x)"""
    x0 = torch.randn(4, 32, 8, 8, device=DEV)
    dy = torch.randn(4, 32, 8, 8, device=DEV)
    w_se = (0.3 * torch.randn(2, 32, device=DEV), 0.3 * torch.randn(32, 2, device=DEV))
    res = []
    for x in (x0.clone(), x0.clone().to(memory_format=torch.channels_last)):
        x.requires_grad_()
        if op == "bn_act":
            gm = torch.ones(32, device=DEV).requires_grad_()
            bt = torch.zeros(32, device=DEV).requires_grad_()
            y = torch.ops.ffc.bn_act(x, gm, bt, None, None, True, 1e-5, 2, 0.1)[0]
            params = (gm, bt)
        else:
            gm, bt = (w.clone().requires_grad_() for w in w_se)
            y = torch.ops.ffc.se_scale(x, gm, bt)
            params = (gm, bt)
        (y * dy).sum().backward()
        res.append([x.grad.contiguous()] + [p.grad.clone() for p in params])
    for a, b in zip(res[0], res[1]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


# --------------------------------------------------------------------------- round 5: threaded callers
def test_threaded_replicas_bitwise_equal_serial():
    """SURVEY.md §8b "Threading": nn.DataParallel runs module replicas concurrently, one thread each
    (/root/reference/train_cond.py:66-68).  Two threads, each with its own FFCGenerator replica and
    its own stream on cuda:0, run forwards concurrently: every output is bitwise equal to the same
    replica's serial run, and the two threads held different template instances (ops._TemplatePool:
    no plan cache or packed-weight buffer is shared across threads)."""
    import threading
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import ops
    reps, zs = [], []
    for seed in (11, 12):
        torch.manual_seed(seed)
        g = _quiet(F.FFCGenerator, 100, 3, 32).to(DEV).train()
        reps.append(g)
        zs.append(torch.randn(24, 100, 1, 1, device=DEV))
    n_iter = 6
    # serial references: a fresh copy of each replica's state (train-mode BN moves the running stats)
    init = [{k: v.clone() for k, v in g.state_dict().items()} for g in reps]
    serial = []
    with torch.no_grad():
        for g, z in zip(reps, zs):
            serial.append([g(z).clone() for _ in range(n_iter)])
    torch.cuda.synchronize()
    after_serial = [{k: v.clone() for k, v in g.state_dict().items()} for g in reps]
    for g, sd in zip(reps, init):
        g.load_state_dict(sd)
    torch.cuda.synchronize()
    from fastfourierconvolution_amd import _runtime as rt
    held, used, clash = set(), {}, []
    lock = threading.Lock()
    orig_take, orig_give = rt.StreamPool.take, rt.StreamPool.give

    def spy_take(self):
        obj = orig_take(self)
        if isinstance(obj, ops._Template):
            with lock:
                if id(obj) in held:
                    clash.append(id(obj))   # checked out twice at once
                held.add(id(obj))
                used.setdefault(threading.get_ident(), set()).add(id(obj))
        return obj

    def spy_give(self, obj):
        if isinstance(obj, ops._Template):
            with lock:
                held.discard(id(obj))
        orig_give(self, obj)
    rt.StreamPool.take, rt.StreamPool.give = spy_take, spy_give
    outs = [[None] * n_iter for _ in reps]
    errors = []
    bar = threading.Barrier(2)

    def worker(k):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s), torch.no_grad():
                bar.wait()
                for i in range(n_iter):
                    outs[k][i] = reps[k](zs[k]).clone()
            s.synchronize()
        except Exception as e:   # reported by the main thread
            errors.append(e)
    try:
        ths = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=120)
    finally:
        rt.StreamPool.take, rt.StreamPool.give = orig_take, orig_give
    torch.cuda.synchronize()
    assert not errors, errors
    for k in range(2):
        for i in range(n_iter):
            assert torch.equal(outs[k][i], serial[k][i]), (k, i)
        for key, v in reps[k].state_dict().items():
            assert torch.equal(v, after_serial[k][key]), key
    assert not clash, "a template instance was held by two callers at once"
    assert len(used) == 2, used.keys()
    insts = {ops.template(ops.layer_spec(m)).instances for m in reps[0].modules() if hasattr(m, "_ffc_ctor")}
    print(f"template instances per spec after the threaded run: {sorted(insts)}")


def test_capture_takes_templates_last_used_by_another_thread():
    """a pooled template last held by another thread (on its own stream) handed to a
    thread that is capturing a hipGraph.  The hand-over must not wait on an event recorded outside
    the capture (that invalidates it); the capture succeeds and the replay equals the other
    thread's eager output."""
    import threading
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import graphs
    torch.manual_seed(21)
    g = _quiet(F.FFCGenerator, 100, 3, 32).to(DEV).eval()
    z = torch.randn(16, 100, 1, 1, device=DEV)
    got, errors = [], []

    def worker():
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s), torch.no_grad():
                got.append(g(z).clone())
            s.synchronize()
        except Exception as e:   # reported by the main thread
            errors.append(e)
    th = threading.Thread(target=worker)
    th.start()
    th.join(timeout=120)
    assert not errors, errors

    def step():
        with torch.no_grad():
            return g(z)
    graph = graphs.capture_step(step, warmup=0)   # the first take happens inside the capture
    assert graph is not None, "capture failed"
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(graph.ffc_output, got[0])
