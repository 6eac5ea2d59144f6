"""Training path parity (BASELINE config 3, fwd + bwd custom-op autograd) on the GPU, through the
C ABI: gradients of the drop-in modules vs the gradients the REFERENCE computes with autograd
(tests/golden/gen_golden_grad.py fixtures), and at model size vs the fp64 oracle (autograd through
oracle/ffc_oracle.py, itself pinned by tests/test_oracle_grad.py).

Tolerance: normwise max|d| / max|ref| <= 1e-4 per output / gradient tensor."""
import contextlib
import io

import numpy as np
import pytest
import torch

from conftest import build_dropin, grad_arrays, grad_cases, load_case
from oracle.ffc_oracle import ffc_discriminator, ffc_generator, normwise_err

pytestmark = pytest.mark.gpu
CASES = grad_cases()
TOL = 1e-4


def _run(case, mod, inputs, cots):
    tin = {k: torch.from_numpy(v).cuda().requires_grad_(True) for k, v in inputs.items()}
    if case["kind"] == "FFC_BN_ACT":
        x = (tin["x_l"], tin["x_g"]) if "x_l" in tin else tin["x"]
        ol, og = mod(x)
        outs = {k: v for k, v in (("out_l", ol), ("out_g", og)) if isinstance(v, torch.Tensor)}
    else:
        outs = {"out": mod(next(iter(tin.values())))}
    loss = sum((v * torch.from_numpy(cots[k]).cuda()).sum() for k, v in outs.items())
    loss.backward()
    return outs, tin


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_grad_golden(case):
    state, inputs, data = load_case(case)
    mod = build_dropin(case, state)
    outs, tin = _run(case, mod, inputs, grad_arrays(data, "cot."))
    for k, v in outs.items():
        assert normwise_err(v.detach().cpu(), torch.from_numpy(data["ref." + k])) < TOL, k
    params = dict(mod.named_parameters())
    for k in case["grads"]:
        if k.startswith("gin."):
            g = tin[k[4:]].grad
        else:
            g = params[k[5:]].grad
        assert g is not None, k
        err = normwise_err(g.cpu(), torch.from_numpy(data[k]))
        assert err < TOL, (k, err)
    # train mode: running statistics move exactly as nn.BatchNorm2d's
    if case["mode"] == "train":
        for mname, m in mod.named_modules():
            if isinstance(m, torch.nn.BatchNorm2d) and ".lfu." not in "." + mname:   # lfu never runs
                assert int(m.num_batches_tracked) == 1, mname


def _randomize(mod, gen):
    with torch.no_grad():
        for k, v in mod.state_dict().items():
            if v.is_floating_point() and not k.endswith(("running_mean", "running_var")):
                fan = v[0].numel() if v.dim() > 1 else 1
                base = 1.0 if (v.dim() == 1 and k.endswith("weight")) else 0.0
                v.copy_(base + torch.randn(v.shape, generator=gen) / max(1, fan) ** 0.5 * (0.1 if v.dim() == 1 else 1))


class _KinkF:
    """stand-in for torch.nn.functional inside the oracle: ReLU / LeakyReLU take their active set
    from the HIP path's own outputs (x * mask), so the oracle differentiates the same piece of the
    piecewise-linear network; every other function is torch's"""

    def __init__(self, relu_outs, lrelu_outs):
        self.relu_outs, self.lrelu_outs = list(relu_outs), list(lrelu_outs)

    def __getattr__(self, name):
        return getattr(torch.nn.functional, name)

    def relu(self, x):
        if self.relu_outs and tuple(self.relu_outs[0].shape) == tuple(x.shape):
            return x * (self.relu_outs.pop(0) > 0).to(x.dtype)
        return torch.nn.functional.relu(x)

    def leaky_relu(self, x, slope):
        if self.lrelu_outs and tuple(self.lrelu_outs[0].shape) == tuple(x.shape):
            y = self.lrelu_outs.pop(0)
            return x * torch.where(y > 0, torch.ones_like(x), torch.full_like(x, slope))
        return torch.nn.functional.leaky_relu(x, slope)


def _layer_checks(train: bool, B: int = 8, fp32_ref: bool = True, check_loss: bool = False):
    """config 3 architecture at full width (G nz=100 nc=3 ngf=64, D nc=3 ndf=64), loss =
    mean(D(G(z))), fwd + bwd on the HIP path, checked LAYER BY LAYER: for every FFC_BN_ACT, the
    oracle's vector-Jacobian product at the HIP path's own layer input and output gradient, with
    ReLU / LeakyReLU active sets taken from the HIP path's outputs (_KinkF), must match the HIP
    path's gradients of that layer's input and parameters.  The network is piecewise linear: with
    ~1e5 activations per layer some sit within fp32 rounding of a kink (|y| down to 4e-7 max|y|
    measured here), and one flipped LeakyReLU moves a weight gradient by 5e-2 normwise -- that
    would test the kinks, not the kernels (a 1e-6 relative change of D's input moves D's input
    gradient by 5e-3 in fp64).  Each layer also runs in fp32 on the CPU (the reference's own arithmetic) for the
    train-mode conditioning bound (``fp32_ref``).  ``check_loss``: the scalar loss against the fp64
    oracle's end-to-end forward (<= 1e-4 relative).
    -> [(name, err vs fp64, fp32-reference err vs fp64 or nan)]"""
    import fastfourierconvolution_amd as F
    from oracle.ffc_oracle import discriminator_layers, ffc_bn_act, generator_layers
    gen = torch.Generator().manual_seed(3)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FFCGenerator(100, 3, 64)
        D = F.FFCDiscriminator(3, 64)
    _randomize(G, gen)
    _randomize(D, gen)
    z = torch.randn(B, 100, 1, 1, generator=gen)
    sds = {"G": {k: v.detach().clone() for k, v in G.state_dict().items()},
           "D": {k: v.detach().clone() for k, v in D.state_dict().items()}}
    G, D = G.cuda().train(train), D.cuda().train(train)
    trace = {"G": [], "D": []}

    from fastfourierconvolution_amd import _autograd as ag
    import oracle.ffc_oracle as O

    def run(name, model, x):
        for i in range(5):
            layer = getattr(model, f"ffc{i}")
            ag.RECORD = []
            y = layer(x)
            recorded = [t.cpu() for t in ag.RECORD]
            ag.RECORD = None
            for t in y:
                if isinstance(t, torch.Tensor):
                    t.retain_grad()
            trace[name].append((x, y, recorded))
            x = y
        return model.resizer(x)

    zc = z.detach().cuda().requires_grad_(True)
    out = run("D", D, run("G", G, zc)).mean()
    out.backward()
    if check_loss:
        with torch.no_grad():
            sd64 = {n: {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in sds[n].items()}
                    for n in ("G", "D")}
            ref_loss = ffc_discriminator(ffc_generator(z.double(), sd64["G"], 100, 3, 64, train), sd64["D"], 3, 64,
                                         train).mean().item()
        rel = abs(out.item() - ref_loss) / abs(ref_loss)
        print(f"loss {out.item():.8f} vs fp64 oracle {ref_loss:.8f}: rel {rel:.2e}")
        assert rel <= TOL, rel
    cfgs = {"G": generator_layers(100, 3, 64), "D": discriminator_layers(3, 64)}
    mods = {"G": G, "D": D}
    res = []
    for name in ("G", "D"):
        for i, ((x, y, recorded), cfg) in enumerate(zip(trace[name], cfgs[name])):
            xs = x if type(x) is tuple else (x,)
            params = {k: p for k, p in mods[name].named_parameters() if k.startswith(f"ffc{i}.") and p.grad is not None}
            ref = {}
            for bits, dt in ((64, torch.float64), (32, torch.float32))[:2 if fp32_ref else 1]:
                sd = {k: (v.to(dt).clone().requires_grad_(k in params)) if v.is_floating_point() else v.clone()
                      for k, v in sds[name].items()}
                xin = [t.detach().cpu().to(dt).requires_grad_(True) if isinstance(t, torch.Tensor) else t for t in xs]
                old = O.F
                O.F = _KinkF(recorded, [t.detach().cpu() for t in y if isinstance(t, torch.Tensor)])
                try:
                    o = ffc_bn_act(tuple(xin) if len(xin) == 2 else xin[0], sd, f"ffc{i}.", cfg, train, fft="torch")
                finally:
                    O.F = old
                loss = sum((ot * yt.grad.cpu().to(dt)).sum() for ot, yt in zip(o, y)
                           if isinstance(yt, torch.Tensor) and yt.grad is not None)
                loss.backward()
                ref[bits] = {f"in{j}": t.grad for j, t in enumerate(xin) if isinstance(t, torch.Tensor) and
                             t.grad is not None}
                ref[bits].update({k: sd[k].grad for k in params})
            mine = {f"in{j}": t.grad.cpu() for j, t in enumerate(xs) if isinstance(t, torch.Tensor) and
                    t.grad is not None}
            mine.update({k: p.grad.cpu() for k, p in params.items()})
            assert set(ref[64]) == set(mine), (name, i, set(ref[64]) ^ set(mine))
            for k in ref[64]:
                res.append((f"{name}.{k}" if k.startswith("ffc") else f"{name}.ffc{i}.{k}",
                            normwise_err(mine[k], ref[64][k]),
                            normwise_err(ref[32][k], ref[64][k]) if fp32_ref else float("nan")))
    return res


def test_config3_gen_disc_eval_vs_oracle():
    """eval-mode BN: every layer's input and parameter gradients within 1e-4 of the fp64 oracle"""
    res = _layer_checks(False)
    print(f"config-3 eval: {len(res)} gradients, worst normwise error {max(e for _, e, _ in res):.2e}")
    bad = sorted(((e, k) for k, e, _ in res if not e < TOL), reverse=True)
    assert not bad, bad[:12]


def test_config3_gen_disc_train_vs_oracle():
    """train-mode BN (batch statistics, B=8): every layer's gradients within 1e-4 of the fp64 oracle"""
    res = _layer_checks(True)
    print(f"config-3 train: {len(res)} gradients, worst normwise error {max(e for _, e, _ in res):.2e} "
          f"(reference fp32 autograd: {max(r for _, _, r in res):.2e})")
    bad = sorted(((e, k) for k, e, _ in res if not e < TOL), reverse=True)
    assert not bad, bad[:12]


def test_no_grad_uses_inference_path_and_matches_train_path():
    """the same module under no_grad (fused inference kernels) and with autograd (training path)
    produce the same forward"""
    import fastfourierconvolution_amd as F
    gen = torch.Generator().manual_seed(5)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FFCGenerator(100, 3, 64)
    _randomize(G, gen)
    G = G.cuda().eval()
    z = torch.randn(16, 100, 1, 1, generator=gen).cuda()
    with torch.no_grad():
        a = G(z)
    b = G(z)
    assert b.requires_grad
    assert normwise_err(b.detach().cpu(), a.cpu()) < 1e-5


def test_train_step_optimizer_repacks_weights():
    """an optimizer step changes the weights in place; the next forward must use them (packed
    weights are cached by tensor version)"""
    import fastfourierconvolution_amd as F
    gen = torch.Generator().manual_seed(9)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FFCGenerator(100, 3, 64)
    _randomize(G, gen)
    sd = {k: v.detach().double().clone() if v.is_floating_point() else v.clone() for k, v in G.state_dict().items()}
    G = G.cuda().train()
    opt = torch.optim.SGD(G.parameters(), lr=0.05)
    z = torch.randn(4, 100, 1, 1, generator=gen)
    for _ in range(2):
        opt.zero_grad()
        G(z.cuda()).square().mean().backward()
        opt.step()
    # replay the same two steps on the oracle
    for _ in range(2):
        p = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and
                 not k.endswith(("running_mean", "running_var")) else v) for k, v in sd.items()}
        ffc_generator(z.double(), p, 100, 3, 64, True, fft="torch").square().mean().backward()
        with torch.no_grad():
            for k, v in p.items():
                if isinstance(v, torch.Tensor) and v.requires_grad and v.grad is not None:
                    sd[k] = (v - 0.05 * v.grad).detach()
                else:
                    sd[k] = v
    for k, v in G.state_dict().items():
        if v.is_floating_point():
            assert normwise_err(v.cpu(), sd[k]) < 1e-4, k


def test_train_step_graph_capture_bit_identical():
    """the whole training step (forward, custom-op backward, optimizer) captured into one hipGraph
    and replayed gives bit-identical weights and BN buffers to eager steps (deterministic kernels;
    re-packs of the optimizer-updated weights are captured with the step)"""
    import fastfourierconvolution_amd as F

    def make():
        torch.manual_seed(0)
        with contextlib.redirect_stdout(io.StringIO()):
            G, D = F.FFCGenerator(100, 3, 64), F.FFCDiscriminator(3, 64)
        return G.cuda().train(), D.cuda().train()

    z = torch.randn(16, 100, 1, 1, generator=torch.Generator().manual_seed(1)).cuda()
    res = []
    for graph in (False, True):
        G, D = make()
        opt = torch.optim.SGD(list(G.parameters()) + list(D.parameters()), lr=0.05)

        def step():
            opt.zero_grad(set_to_none=True)
            D(G(z)).mean().backward()
            opt.step()
        if graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                step()
                step()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            for _ in range(2):
                g.replay()
        else:
            for _ in range(4):
                step()
        torch.cuda.synchronize()
        res.append({n + k: v.detach().cpu().clone() for n, m in (("G.", G), ("D.", D))
                    for k, v in m.state_dict().items()})
    for k in res[0]:
        assert torch.equal(res[0][k], res[1][k]), k
