"""The custom-op boundary on CPU (no GPU): every torch.ops.ffc.* op is registered with a fake
implementation, and the drop-in modules trace -- under FakeTensor, on fake HIP tensors -- to graphs
whose compute is ffc:: ops only (the hot path is reached through custom ops).
Numerics of the ops are the GPU suites' job (tests/test_gpu_ops.py: torch.library.opcheck)."""
import contextlib
import io
from collections import Counter

import pytest
import torch
import torch.nn as nn
from torch._subclasses.fake_tensor import FakeTensorMode
from torch.fx.experimental.proxy_tensor import make_fx

import fastfourierconvolution_amd as F

OPS = ["conv_layer", "conv_layer_backward", "bn_act", "bn_act_backward", "bn_update_running", "se_scale",
       "se_scale_backward", "pool2", "up2", "rfft2", "irfft2", "noise_inject", "noise_wgrad", "linear", "quantize_u8",
       "ffc_bn_act", "spectral_transform", "fourier_unit"]
# what a traced forward may contain besides ffc:: ops: tuple indexing, parameter detach (make_fx),
# and the RNG of NoiseInjection's noise (drawn by torch, as in the reference)
ALLOWED = {"<built-in function getitem>", "aten.detach.default", "aten.empty.memory_format", "aten.new_empty.default",
           "aten.normal.default", "aten.normal_.default", "aten.view.default"}


def _quiet(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


def _trace(mod, fn, *shapes, grad=False, train=True):
    """make_fx trace of fn(mod, *inputs) on fake HIP tensors -> Counter of called targets, outputs"""
    mode = FakeTensorMode(allow_non_fake_inputs=True)
    with mode:
        mod = mod.to("cuda").train(train)
        ins = [torch.empty(s, device="cuda") for s in shapes]
        ctx = contextlib.nullcontext() if grad else torch.no_grad()

        def f(*xs):
            with ctx:
                return fn(mod, *xs)
        g = make_fx(f, tracing_mode="real")(*ins)
        outs = f(*ins)
    return Counter(str(n.target) for n in g.graph.nodes if n.op == "call_function"), outs


def _only_ffc(cnt):
    bad = {k: v for k, v in cnt.items() if not k.startswith("ffc.") and k not in ALLOWED}
    assert not bad, f"non-ffc compute on the hot path: {bad}"


def test_every_op_registered_with_fake():
    for name in OPS:
        op = getattr(torch.ops.ffc, name).default
        assert op.name() == f"ffc::{name}"
        from torch._library.simple_registry import singleton   # where register_fake puts the kernel
        assert singleton.find(op.name()).fake_impl.kernel is not None, name


@pytest.mark.parametrize("train", [True, False])
def test_block_inference_is_one_layer_op(train):
    """BASELINE configs[0] block: one ffc::ffc_bn_act per forward, outputs of the reference's shapes"""
    blk = _quiet(F.FFC_BN_ACT, 32, 32, 3, 0.5, 0.5, 1, 1, norm_layer=nn.BatchNorm2d, activation_layer=nn.ReLU)
    cnt, (ol, og) = _trace(blk, lambda m, a, b: m((a, b)), (16, 16, 32, 32), (16, 16, 32, 32), train=train)
    _only_ffc(cnt)
    assert cnt["ffc.ffc_bn_act.default"] == 1
    assert tuple(ol.shape) == (16, 16, 32, 32) and tuple(og.shape) == (16, 16, 32, 32)


def test_generator_inference_ops_and_shapes():
    """FFCGenerator (models/ffc_generator.py): five ffc::ffc_bn_act, (B, nc, 64, 64) out"""
    g = _quiet(F.FFCGenerator, 100, 3, 64)
    cnt, out = _trace(g, lambda m, z: m(z), (8, 100, 1, 1))
    _only_ffc(cnt)
    assert cnt["ffc.ffc_bn_act.default"] == 5
    assert tuple(out.shape) == (8, 3, 64, 64)


@pytest.mark.parametrize("train", [True, False])
def test_generator_training_path_ops(train):
    """with autograd recording, the per-op training ops (each with a registered backward op)"""
    g = _quiet(F.FFCGenerator, 100, 3, 64)
    cnt, out = _trace(g, lambda m, z: m(z), (8, 100, 1, 1), grad=True, train=train)
    _only_ffc(cnt)
    for op, n in (("conv_layer", 11), ("bn_act", 6), ("rfft2", 3), ("irfft2", 3), ("se_scale", 3), ("up2", 3)):
        assert cnt[f"ffc.{op}.default"] == n, (op, cnt)
    assert cnt["ffc.bn_update_running.default"] == (6 if train else 0)
    assert tuple(out.shape) == (8, 3, 64, 64)


def test_discriminator_ops():
    cnt, out = _trace(_quiet(F.FFCDiscriminator, 3, 64), lambda m, x: m(x), (4, 3, 64, 64))
    _only_ffc(cnt)
    assert cnt["ffc.ffc_bn_act.default"] == 5 and tuple(out.shape) == (4, 1, 1, 1)
    cnt, out = _trace(_quiet(F.FFCDiscriminator, 3, 64), lambda m, x: m(x), (4, 3, 64, 64), grad=True)
    _only_ffc(cnt)
    assert cnt["ffc.pool2.default"] == 3 and tuple(out.shape) == (4, 1, 1, 1)


@pytest.mark.parametrize("train", [True, False])
def test_fgan128_ops(train):
    """fgan128 FGenerator: Linear, six layer ops (conv6 deferred into the 3x3 head), uint8 in eval"""
    g = _quiet(F.FGenerator, 128)
    cnt, out = _trace(g, lambda m, z: m(z), (4, 128), train=train)
    _only_ffc(cnt)
    assert cnt["ffc.linear.default"] == 1 and cnt["ffc.ffc_bn_act.default"] == 6
    assert cnt["ffc.quantize_u8.default"] == (0 if train else 1)
    assert tuple(out.shape) == (4, 3, 128, 128)


def test_spectral_transform_and_fourier_unit_ops():
    st = _quiet(F.SpectralTransform, 64, 64, 2, upsample=True)
    cnt, out = _trace(st, lambda m, x: m(x), (4, 64, 8, 8))
    _only_ffc(cnt)
    assert cnt["ffc.spectral_transform.default"] == 1 and tuple(out.shape) == (4, 64, 16, 16)
    cnt, out = _trace(F.FourierUnitSN(16, 16), lambda m, x: m(x), (4, 16, 32, 32))
    assert cnt["ffc.fourier_unit.default"] == 1 and tuple(out.shape) == (4, 16, 32, 32)
    cnt, out = _trace(F.FourierUnitSN(16, 16), lambda m, x: m(x), (4, 16, 32, 32), grad=True)
    _only_ffc(cnt)
    assert cnt["ffc.rfft2.default"] == 1 and cnt["ffc.irfft2.default"] == 1


def test_backward_op_fakes():
    """the backward ops' fake implementations give gradients of their inputs' shapes"""
    from fastfourierconvolution_amd import _autograd as ag
    from fastfourierconvolution_amd import _plan
    with FakeTensorMode():
        x = torch.empty(4, 16, 8, 8, device="cuda")
        w = torch.empty(16, 32, 4, 4, device="cuda")      # ConvTranspose2d(16, 32, 4, 2, 1)
        b = torch.empty(32, device="cuda")
        spec = ag.conv_spec([(32, 2, 0.1)], [(0, 0, _plan.Seg("convT", 16, 8, 8, 4, 2, 1), 1, 0)])
        (y,) = torch.ops.ffc.conv_layer([x], [w], [b], spec)
        assert tuple(y.shape) == (4, 32, 16, 16)
        dx, dw, db = torch.ops.ffc.conv_layer_backward([x], [w], [y], [y], [True, True, True], spec)
        assert dx.shape == x.shape and dw.shape == w.shape and tuple(db.shape) == (32,)
        y2, sc, sh, st = torch.ops.ffc.bn_act(y, b, b, b, b, True, 1e-5, 1, 0.0)
        assert st.dtype == torch.float64 and tuple(st.shape) == (32, 3)
        dx, dg, dbeta = torch.ops.ffc.bn_act_backward(y, y2, sc, sh, st, b, True, False, 1e-5, 1, 0.0, True, True, True)
        assert dx.shape == y.shape and tuple(dg.shape) == (32,)
        Z = torch.ops.ffc.rfft2(x, 1.0)
        assert tuple(Z.shape) == (4, 32, 8, 5)
        assert torch.ops.ffc.irfft2(Z, 8, 8, 1.0, None).shape == x.shape
        w1, w2 = torch.empty(1, 16, device="cuda"), torch.empty(16, 1, device="cuda")
        r = torch.ops.ffc.se_scale_backward(x, x, w1, w2)
        assert [t.shape for t in r] == [x.shape, w1.shape, w2.shape]
        assert tuple(torch.ops.ffc.noise_wgrad(x, x[:, :1]).shape) == (1, 16, 1, 1)


def test_layer_spec_round_trip():
    """the template built from a module's spec has the module's structure and tensor slots"""
    from fastfourierconvolution_amd import ops
    blk = _quiet(F.FFC_BN_ACT, 64, 128, 4, 0.5, 0.5, 2, 1, activation_layer=nn.LeakyReLU, upsampling=True)
    spec = ops.layer_spec(blk)
    tpl = ops.template(spec)
    params, buffers = ops.layer_tensors(blk, spec)
    assert [n for n, _ in blk.named_parameters()] == tpl.param_names
    assert len(buffers) == len(tpl.buffer_names)
    assert all(p.device.type == "meta" for p in tpl.module.parameters())
    assert isinstance(tpl.module.act_l, nn.LeakyReLU) and tpl.module.act_l.negative_slope == 0.1
    blk.eval()
    assert ops.layer_spec(blk) != spec     # the modes are part of the spec


def test_ops_fail_loudly_on_cpu_tensors():
    """no CPU fallback: a CPU tensor reaching an op raises"""
    from fastfourierconvolution_amd._lib import FFCError
    with pytest.raises((FFCError, TypeError)):
        torch.ops.ffc.pool2(torch.randn(1, 1, 4, 4), 0.25)
