"""Debug probe: determinism of gen64 train forward at B = 86 over repeated calls (fresh generator each
time, same weights and z), FFC_FU2D_R2CMIX on / off; reports how many runs differ from the first and
the normwise error against the CPU oracle of a differing run."""
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


torch.manual_seed(1234)
with contextlib.redirect_stdout(io.StringIO()):
    G0 = F.FFCGenerator(100, 3, 64)
G0.apply(_weights_init)
G0 = G0.cuda().train()
for flag in (True, False):
    rt.FU2D_R2CMIX = flag
    for B in (86, 64):
        z = torch.randn((B, 100, 1, 1), generator=torch.Generator().manual_seed(B)).cuda()
        outs = []
        for rep in range(30):
            G = copy.deepcopy(G0)
            with torch.no_grad():
                outs.append(G(z).clone())
        torch.cuda.synchronize()
        diff = [i for i, o in enumerate(outs) if not torch.equal(o, outs[0])]
        md = max(((o - outs[0]).abs().max().item() for o in outs), default=0.0)
        print(f"R2CMIX={flag} B={B}: {len(diff)} of 30 differ from run 0 (max|d| {md:.3e}) at {diff[:10]}", flush=True)
