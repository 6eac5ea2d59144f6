"""Per-layer timing of the fgan128 Discriminator's convs on the training path at B (default 64):
forward (conv + bias + LeakyReLU), data gradient alone, weight gradient alone (ffc_conv_wgrad),
HIP events over repeated calls, with each one's TFLOP/s.  Diagnostic only.
usage: dtrain_probe.py [B]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fastfourierconvolution_amd as F  # noqa: E402
from fastfourierconvolution_amd import _autograd as ag, _plan  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
D = F.Discriminator().to(dev).train()


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def spec_cache_items(cache):
    for k, v in cache.items():
        if isinstance(k, tuple) and k and k[0] == "spec":
            for k2, v2 in v.cache.items():
                if isinstance(v2, tuple) and len(v2) == 2 and hasattr(v2[0], "kind"):
                    yield k2, v2[0]
        elif isinstance(v, tuple) and len(v) == 2 and hasattr(v[0], "kind"):
            yield k, v[0]


side = 128
tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
print(f"B={B}  layer  C->M  k s  in  |  fwd ms TF/s | dgrad ms TF/s | wgrad ms TF/s")
for i, (cin, cout, k, s) in enumerate(F.Discriminator.CONVS, 1):
    conv = getattr(D, f"conv{i}")
    x = torch.randn(B, cin, side, side, device=dev)
    sg = _plan.Seg("conv", cin, side, side, k, s, 1)
    OH = side // s
    fl = 2.0 * B * cout * cin * k * k * OH * OH
    cache = {}
    conv.requires_grad_(False)

    def fwd():
        return ag.conv_layer(cache, B, [(cout, 2, 0.1)], [(0, 0, sg, conv)], [x])[0]
    t_f = timeit(fwd)
    xg = x.clone().requires_grad_(True)
    g = torch.randn(B, cout, OH, OH, device=dev)
    (y,) = ag.conv_layer(cache, B, [(cout, 2, 0.1)], [(0, 0, sg, conv)], [xg])

    def dgrad():
        torch.autograd.grad(y, xg, g, retain_graph=True)
    t_d = timeit(dgrad) if i > 1 else 0.0
    W = conv.weight.detach()

    def wgrad():
        ag.conv_wgrad(g, x, k, s, 1, 1, tuple(W.shape))
    t_w = timeit(wgrad)
    tot["fwd"] += t_f
    tot["dgrad"] += t_d
    tot["wgrad"] += t_w
    print(f"conv{i} {cin:4d}->{cout:4d} {k} {s} {side:4d} | {t_f:7.3f} {fl / t_f / 1e9:6.1f} | "
          f"{t_d:7.3f} {fl / max(t_d, 1e-9) / 1e9:6.1f} | {t_w:7.3f} {fl / t_w / 1e9:6.1f}")
    for key, v in spec_cache_items(cache):
        print(f"    {key[0]}: kind={v.kind} launch={v.launch_key} ksplit={getattr(v.plan, 'ksplit', None)}")
    side = OH
print("totals ms:", {k: round(v, 3) for k, v in tot.items()})
print("iteration estimate ms (3 fwd + 3 dgrad + 2 wgrad):",
      round(3 * tot["fwd"] + 3 * tot["dgrad"] + 2 * tot["wgrad"], 2))
