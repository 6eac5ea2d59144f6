"""Debug probe: which run is wrong -- fresh process, gen64 train forward at B = 86 (R2CMIX on), runs
0..3 compared with each other and with the fp64 CPU oracle; then the same after a B = 64 warm-up."""
import contextlib
import copy
import io
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import fastfourierconvolution_amd as F
from fastfourierconvolution_amd import _runtime as rt
from oracle.ffc_oracle import ffc_generator, normwise_err


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
sd = {k: (v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu().clone())
      for k, v in G0.state_dict().items()}
G0 = G0.cuda().train()
mode = sys.argv[1] if len(sys.argv) > 1 else "fresh"
if mode == "warm64":
    z = torch.randn((64, 100, 1, 1)).cuda()
    with torch.no_grad():
        copy.deepcopy(G0)(z)
B = 86
z = torch.randn((B, 100, 1, 1), generator=torch.Generator().manual_seed(B))
ref = ffc_generator(z.double(), sd, 100, 3, 64, True)
outs = []
for rep in range(4):
    G = copy.deepcopy(G0)
    with torch.no_grad():
        outs.append(G(z.cuda()).cpu())
for i, o in enumerate(outs):
    print(f"{mode} run {i}: err vs oracle {normwise_err(o, ref):.2e}; equal to run 0: {torch.equal(o, outs[0])}, "
          f"to run 1: {torch.equal(o, outs[1])}", flush=True)
