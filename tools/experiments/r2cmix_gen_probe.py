"""Debug probe: gen64 generator at B = 86 / 64, FFC_FU2D_R2CMIX on vs off: per-module output differences."""
import contextlib
import copy
import io
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import fastfourierconvolution_amd as F
from fastfourierconvolution_amd import _runtime as rt

def _weights_init(m):
    name = m.__class__.__name__
    if name.find("Conv") != -1:
        torch.nn.init.normal_(m.weight.data, 0.0, 0.02)
    elif name.find("BatchNorm") != -1:
        torch.nn.init.normal_(m.weight.data, 1.0, 0.02)
        torch.nn.init.constant_(m.bias.data, 0)


for B in (86, 64, 32):
    torch.manual_seed(1234)
    with contextlib.redirect_stdout(io.StringIO()):
        G0 = F.FFCGenerator(100, 3, 64)
    G0.apply(_weights_init)
    G0 = G0.cuda().train()
    z = torch.randn((B, 100, 1, 1), generator=torch.Generator().manual_seed(B)).cuda()
    res = []
    for flag in (False, True):
        rt.FU2D_R2CMIX = flag
        G = copy.deepcopy(G0)
        acts = {}

        def hook(name):
            def f(mod, inp, out):
                o = out if isinstance(out, tuple) else (out,)
                acts[name] = [t.detach().clone() if isinstance(t, torch.Tensor) else None for t in o]
            return f
        for n, m in G.named_modules():
            if n and n.count(".") <= 3:
                m.register_forward_hook(hook(n))
        with torch.no_grad():
            out = G(z).clone()
        torch.cuda.synchronize()
        res.append((out, acts, {k: v.clone() for k, v in G.state_dict().items()}))
    (o0, a0, s0), (o1, a1, s1) = res
    print(f"B={B} out max|d|={(o0 - o1).abs().max().item():.3e}", flush=True)
    for n in a0:
        for i, (x, y) in enumerate(zip(a0[n], a1[n])):
            if x is not None and y is not None and x.shape == y.shape:
                d = (x - y).abs().max().item()
                if d > 1e-4 * max(1.0, x.abs().max().item()):
                    print(f"  {n}[{i}] {tuple(x.shape)} max|d|={d:.3e} |x|max={x.abs().max().item():.3e}", flush=True)
    for k in s0:
        if s0[k].dtype.is_floating_point:
            d = (s0[k] - s1[k]).abs().max().item()
            if d > 1e-5:
                print(f"  state {k} max|d|={d:.3e}", flush=True)
        elif not torch.equal(s0[k], s1[k]):
            print(f"  state {k}: {s0[k].item()} vs {s1[k].item()}", flush=True)
