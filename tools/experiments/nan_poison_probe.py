"""Debug probe: every torch.empty allocation filled with NaN (a read of memory no kernel wrote shows
up as NaN), gen64 generator train forward at the strong-scaling shard sizes, FFC_FU2D_R2CMIX on / off:
the first module whose output holds a non-finite value."""
import contextlib
import io
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
_empty = torch.empty


def poisoned(*a, **k):
    t = _empty(*a, **k)
    if t.is_floating_point() and t.numel():
        t.fill_(float("nan"))
    return t


torch.empty = poisoned
import fastfourierconvolution_amd as F
from fastfourierconvolution_amd import _runtime as rt


def _weights_init(m):
    name = m.__class__.__name__
    if name.find("Conv") != -1:
        torch.nn.init.normal_(m.weight.data, 0.0, 0.02)
    elif name.find("BatchNorm") != -1:
        torch.nn.init.normal_(m.weight.data, 1.0, 0.02)
        torch.nn.init.constant_(m.bias.data, 0)


for flag in (True, False):
    rt.FU2D_R2CMIX = flag
    for B in (128, 86, 64, 32):
        torch.manual_seed(1234)
        with contextlib.redirect_stdout(io.StringIO()):
            G = F.FFCGenerator(100, 3, 64)
        G.apply(_weights_init)
        G = G.cuda().train()
        bad = []

        def hook(name):
            def f(mod, inp, out):
                for i, t in enumerate(out if isinstance(out, tuple) else (out,)):
                    if isinstance(t, torch.Tensor) and not torch.isfinite(t).all():
                        bad.append(f"{name}[{i}] {tuple(t.shape)} nonfinite={int((~torch.isfinite(t)).sum())}")
            return f
        for n, m in G.named_modules():
            if n:
                m.register_forward_hook(hook(n))
        z = torch.randn((B, 100, 1, 1), generator=torch.Generator().manual_seed(B)).cuda()
        with torch.no_grad():
            out = G(z)
        torch.cuda.synchronize()
        print(f"R2CMIX={flag} B={B} finite={bool(torch.isfinite(out).all())} first bad: {bad[:4]}", flush=True)
