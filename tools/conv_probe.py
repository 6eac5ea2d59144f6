"""Every implicit-GEMM conv launch (ffc_convp_forward / ffc_conv_forward) of one config-3 train step
(G + D fwd + bwd, B = 256) or one gen64 forward: kernel kind / cfg, segments, HIP-event time and
TFLOP/s.  Diagnostic only (not part of the product path).   usage: conv_probe.py [train|gen64]"""
import contextlib
import io
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import fastfourierconvolution_amd as F  # noqa: E402
from fastfourierconvolution_amd import _runtime as rt  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "train"
B = 256
dev = torch.device("cuda", 0)
torch.manual_seed(1234)
with contextlib.redirect_stdout(io.StringIO()):
    G = F.FFCGenerator(100, 3, 64)
    D = F.FFCDiscriminator(3, 64)
G.apply(bench.weights_init)
D.apply(bench.weights_init)
G, D = G.to(dev).train(), D.to(dev).train()
z = torch.randn((B, 100, 1, 1), device=dev)


def step():
    if mode == "train":
        D(G(z)).mean().backward()
    else:
        with torch.no_grad():
            G(z)


step()
torch.cuda.synchronize()
recs = []
orig = rt.LaunchPlan.launch


def launch(self, jobs, stream, flops=0.0):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    orig(self, jobs, stream, flops)
    e1.record()
    desc = []
    for j in jobs:
        segs = []
        for s in range(j.nseg) if hasattr(j, "nseg") else []:
            sg = j.seg[s]
            segs.append(f"{sg.C}@{sg.IH}x{sg.IW}")
        desc.append(f"M{j.M}->{j.OH}x{j.OW}[{','.join(segs)}]")
    recs.append((self.key, self.ntiles, " ".join(desc), flops, e0, e1))


rt.LaunchPlan.launch = launch
step()
torch.cuda.synchronize()
tot = fl = 0.0
for key, nt, desc, flops, e0, e1 in recs:
    us = e0.elapsed_time(e1) * 1e3
    tot += us
    fl += flops
    print(f"{str(key):14s} tiles={nt:5d} {us:8.1f} us {flops / us / 1e6 if us else 0:6.1f} TF  {desc}")
print(f"total {tot:.0f} us, {fl / tot / 1e6:.1f} TF over {len(recs)} launches")
