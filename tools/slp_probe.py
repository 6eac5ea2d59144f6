"""Per-layer parity probe of the B = 8 FFC-DCGAN generator (the smoke test's job) for one library
build (FFC_LIB_PATH): every FFC_BN_ACT layer, and the SpectralTransform of ffc1-ffc3 on its own,
run on the HIP path's own layer input and compared with the fp64 oracle on that same input.
Names the layer / op of a build-flag-dependent miscompare.

    FFC_LIB_PATH=fastfourierconvolution_amd/libffc_amd_<v>.so python tools/slp_probe.py [B]
"""
import contextlib
import io
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import fastfourierconvolution_amd as F  # noqa: E402
from oracle.ffc_oracle import ffc_bn_act, generator_layers, normwise_err, spectral_transform  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda:0")
    gen = torch.Generator().manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        g = F.FFCGenerator(100, 3, 64)
    with torch.no_grad():     # the smoke test's randomisation (same seed stream)
        for k, v in g.state_dict().items():
            if v.is_floating_point() and not k.endswith(("running_mean", "running_var")):
                fan = v[0].numel() if v.dim() > 1 else 1
                base = 1.0 if (v.dim() == 1 and k.endswith("weight")) else 0.0
                v.copy_(base + torch.randn(v.shape, generator=gen) / max(1, fan) ** 0.5 * (0.1 if v.dim() == 1 else 1))
    sd = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in g.state_dict().items()}
    z = torch.randn(B, 100, 1, 1, generator=gen)
    g = g.to(dev).train()
    cfgs = generator_layers(100, 3, 64)
    x = z.to(dev)
    worst = 0.0
    with torch.no_grad():
        for i, cfg in enumerate(cfgs):
            layer = getattr(g, f"ffc{i}")
            xin = x
            out = layer(xin)
            xd = tuple(t.double().cpu() if isinstance(t, torch.Tensor) else t for t in xin) \
                if isinstance(xin, tuple) else xin.double().cpu()
            ref = ffc_bn_act(xd, sd, f"ffc{i}.", cfg, True)
            outs = out if isinstance(out, tuple) else (out,)
            refs = ref if isinstance(ref, tuple) else (ref,)
            errs = [normwise_err(o.cpu(), r) for o, r in zip(outs, refs) if isinstance(o, torch.Tensor)]
            line = f"ffc{i}: " + " ".join(f"{e:.2e}" for e in errs)
            st = layer.ffc.convg2g
            if isinstance(xin, tuple) and isinstance(xin[1], torch.Tensor) and not isinstance(st, nn.Identity):
                v = st(xin[1]).cpu()
                vr = spectral_transform(xin[1].double().cpu(), sd, f"ffc{i}.ffc.convg2g.", 2, True, True)
                e = normwise_err(v, vr)
                line += f" | st {e:.2e}"
                errs.append(e)
            worst = max([worst] + errs)
            print(line, flush=True)
            x = out
    print(f"probe B={B} lib={os.environ.get('FFC_LIB_PATH', 'default')} worst {worst:.2e}")


if __name__ == "__main__":
    main()
