"""Weight-gradient launches of one config-3 train step (G + D fwd + bwd, B = 256; or with argv[2] =
fgan128train the fgan128 G + D iteration at B = 64): shape, split count, HIP-event time and TFLOP/s of
every ffc_conv_wgrad call on the split-once kernel and on the former split-per-use kernel
(FFC_WGRAD_KERNEL=old), and the same call at other split counts.  Diagnostic only."""
import contextlib
import io
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import fastfourierconvolution_amd as F  # noqa: E402
from fastfourierconvolution_amd import _autograd as ag  # noqa: E402
from fastfourierconvolution_amd import _runtime as rt  # noqa: E402
from fastfourierconvolution_amd._lib import ptr  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
MODEL = sys.argv[2] if len(sys.argv) > 2 else "gan64train"
dev = torch.device("cuda", 0)
torch.manual_seed(1234)
with contextlib.redirect_stdout(io.StringIO()):
    if MODEL == "fgan128train":
        G = F.FGenerator(128)
        D = F.Discriminator()
    else:
        G = F.FFCGenerator(100, 3, 64)
        D = F.FFCDiscriminator(3, 64)
G.apply(bench.weights_init)
D.apply(bench.weights_init)
G, D = G.to(dev).train(), D.to(dev).train()
z = torch.randn((B, 128) if MODEL == "fgan128train" else (B, 100, 1, 1), device=dev)

calls = []
orig = ag.conv_wgrad


def rec(U, V, k, s, p, d, dW_shape):
    calls.append((U.detach().clone(), V.detach().clone(), k, s, p, d, dW_shape))
    return orig(U, V, k, s, p, d, dW_shape)


ag.conv_wgrad = rec
if MODEL == "fgan128train":
    from fastfourierconvolution_amd.training import discriminator_step, generator_step
    oG = torch.optim.AdamW(G.parameters(), lr=0.0)
    oD = torch.optim.AdamW(D.parameters(), lr=0.0)
    generator_step(G, D, oG, oD, z)
    discriminator_step(G, D, oG, oD, z, torch.rand((B, 3, 128, 128), device=dev) * 2 - 1)
else:
    D(G(z)).mean().backward()
torch.cuda.synchronize()
ag.conv_wgrad = orig
L = rt.lib()


def timed(U, V, k, s, p, d, dW_shape, S, reps=10, old=False):
    if old:
        os.environ["FFC_WGRAD_KERNEL"] = "old"
    else:
        os.environ.pop("FFC_WGRAD_KERNEL", None)
    Bq, Mu, PH, PW = U.shape
    _, Nv, VH, VW = V.shape
    NT = Nv * k * k
    dW = torch.empty(dW_shape, device=dev)
    ws = torch.empty(S * Mu * NT, device=dev) if S > 1 else None
    st = torch.cuda.current_stream().cuda_stream

    def go():
        L.ffc_conv_wgrad(ptr(U), Mu, PH, PW, ptr(V), Nv, VH, VW, Bq, k, s, p, d, S, ptr(ws), ptr(dW), 0, st)
    go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        go()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


tot = tot_old = 0.0
tot_fl = 0.0
maxerr = 0.0
for (U, V, k, s, p, d, shp) in calls:
    Bq, Mu, PH, PW = U.shape
    Nv = V.shape[1]
    NT = Nv * k * k
    S0 = ag.wgrad_splits(Bq, Mu, NT, PH * PW, L.ffc_conv_wgrad_tile(Mu, NT))
    fl = 2.0 * Bq * Mu * NT * PH * PW
    t0 = timed(U, V, k, s, p, d, shp, S0)
    t_old = timed(U, V, k, s, p, d, shp, S0, old=True)
    tot += t0
    tot_old += t_old
    try:
        ref = torch.nn.grad.conv2d_weight(V.double(), (Mu, Nv, k, k), U.double(), stride=s, padding=p, dilation=d)
        got = ag.conv_wgrad(U, V, k, s, p, d, shp).double().reshape(ref.shape)
        err = ((got - ref).norm() / ref.norm().clamp_min(1e-30)).item()
    except RuntimeError:
        err = float("nan")
    maxerr = max(maxerr, err)
    tot_fl += fl
    alts = []
    for S in sorted({max(1, S0 // 4), max(1, S0 // 2), S0 * 2, S0 * 4}):
        if S != S0 and S <= Bq * PH * PW // 64:
            alts.append(f"S={S}:{timed(U, V, k, s, p, d, shp, S):.0f}")
    print(f"U{tuple(U.shape)} V{tuple(V.shape)} k{k}s{s}p{p} Mu={Mu} NT={NT} K={Bq * PH * PW} S={S0} "
          f"tile={L.ffc_conv_wgrad_tile(Mu, NT)}: {t0:7.1f} us {fl / t0 / 1e6:6.1f} TF (old {t_old:7.1f} us) "
          f"err {err:.1e} | " + " ".join(alts), flush=True)
print(f"total {tot:.0f} us ({tot_fl / tot / 1e6:.1f} TF), old kernel {tot_old:.0f} us, over {len(calls)} calls; "
      f"max normwise err vs fp64 {maxerr:.1e}")
