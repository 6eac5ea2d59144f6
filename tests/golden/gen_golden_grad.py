"""Generate the GRADIENT golden fixtures (BASELINE config 3: fwd + bwd) by running the REFERENCE
itself with torch autograd.  Run here only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_grad.py

The reference is imported exactly as gen_golden.py does (namespace-module bypass, SURVEY.md
§8c).  Per case: weights from fixture_weights (seed, key), inputs and cotangents from
input_array, forward in train / eval mode, loss = sum_k <out_k, cot_k>, backward.  Stored:
``in.*`` inputs, ``cot.*`` cotangents, ``ref.*`` outputs, ``gin.*`` input gradients,
``gpar.<state_dict key>`` parameter gradients, ``before.*`` running stats (eval cases).
Manifest: manifest_grad.json.
"""
from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gen_golden as G  # noqa: E402
from fixture_weights import input_array  # noqa: E402

CASES = []


def case(name, kind, ctor, inputs, mode="train", seed=4321, note=""):
    CASES.append(dict(name=name, kind=kind, ctor=ctor, inputs=inputs, mode=mode, seed=seed, note=note))


def build_cases():
    T = dict(kernel_size=4, stride=2, padding=1)
    case("grad_fba_transpose_lrelu", "FFC_BN_ACT",
         dict(in_channels=32, out_channels=32, ratio_gin=0.5, ratio_gout=0.5, activation_layer="LeakyReLU",
              upsampling=True, **T),
         {"x_l": [2, 16, 4, 4], "x_g": [2, 16, 4, 4]}, note="FFCGenerator ffc1-3 family (ConvT + ST upsample)")
    case("grad_fba_conv_pool_lrelu", "FFC_BN_ACT",
         dict(in_channels=64, out_channels=64, ratio_gin=0.5, ratio_gout=0.5, activation_layer="LeakyReLU", **T),
         {"x_l": [2, 32, 16, 16], "x_g": [2, 32, 16, 16]},
         note="FFCDiscriminator ffc1-3 family (strided conv + ST avg-pool, SE hidden 2)")
    case("grad_fba_first_convT", "FFC_BN_ACT",
         dict(in_channels=16, out_channels=32, kernel_size=4, ratio_gin=0.0, ratio_gout=0.5, stride=1, padding=0,
              activation_layer="LeakyReLU", upsampling=True),
         {"x": [2, 16, 1, 1]}, note="FFCGenerator ffc0 (ConvT on the 1x1 noise)")
    case("grad_fba_first_conv", "FFC_BN_ACT",
         dict(in_channels=3, out_channels=16, ratio_gin=0.0, ratio_gout=0.5, activation_layer="LeakyReLU", **T),
         {"x": [2, 3, 16, 16]}, note="FFCDiscriminator ffc0")
    case("grad_fba_last_tanh", "FFC_BN_ACT",
         dict(in_channels=16, out_channels=3, ratio_gin=0.5, ratio_gout=0.0, activation_layer="Tanh",
              upsampling=True, **T),
         {"x_l": [2, 8, 8, 8], "x_g": [2, 8, 8, 8]}, note="FFCGenerator ffc4")
    case("grad_fba_disc_sigmoid", "FFC_BN_ACT",
         dict(in_channels=32, out_channels=1, kernel_size=4, ratio_gin=0.5, ratio_gout=0.0, stride=1, padding=0,
              activation_layer="Sigmoid"),
         {"x_l": [2, 16, 4, 4], "x_g": [2, 16, 4, 4]}, note="FFCDiscriminator ffc4")
    case("grad_fba_config1", "FFC_BN_ACT",
         dict(in_channels=32, out_channels=32, kernel_size=3, ratio_gin=0.5, ratio_gout=0.5, stride=1, padding=1,
              norm_layer="BatchNorm2d", activation_layer="ReLU"),
         {"x_l": [2, 16, 16, 16], "x_g": [2, 16, 16, 16]}, note="BASELINE config 1 block, train-mode BN")
    case("grad_fba_config1_eval", "FFC_BN_ACT",
         dict(in_channels=32, out_channels=32, kernel_size=3, ratio_gin=0.5, ratio_gout=0.5, stride=1, padding=1,
              norm_layer="BatchNorm2d", activation_layer="ReLU"),
         {"x_l": [2, 16, 16, 16], "x_g": [2, 16, 16, 16]}, mode="eval", note="running statistics")
    case("grad_fba_transpose_bn_gelu", "FFC_BN_ACT",
         dict(in_channels=32, out_channels=32, ratio_gin=0.5, ratio_gout=0.5, activation_layer="GELU",
              norm_layer="BatchNorm2d", upsampling=True, **T),
         {"x_l": [2, 16, 8, 8], "x_g": [2, 16, 8, 8]}, note="fgan128 conv3-6 family")
    case("grad_gen_nc3", "FFCGenerator", dict(nz=16, nc=3, ngf=8), {"z": [2, 16, 1, 1]},
         note="models/ffc_generator.py at ngf=8 (FU planes 8, 16, 32)")
    case("grad_disc_nc3", "FFCDiscriminator", dict(nc=3, ndf=8), {"x": [2, 3, 64, 64]},
         note="models/ffc_discriminator.py at ndf=8 (FU planes 16, 8, 4)")


def run_case(ref, c):
    torch.manual_seed(0)
    mod = G.construct(ref, c)
    specs = G.weight_specs(mod)
    G.load_specs(mod, c["seed"], specs)
    seed = c["seed"]
    inputs = {k: input_array(seed, k, shp) for k, shp in c["inputs"].items()}
    arrays = {"in." + k: v for k, v in inputs.items()}

    def call(t):
        if c["kind"] == "FFC_BN_ACT" and "x_l" in t:
            return mod((t["x_l"], t["x_g"]))
        return mod(next(iter(t.values())))

    if c["mode"] == "eval":
        warm = {k: torch.from_numpy(input_array(seed + 7, k, shp)) for k, shp in c["inputs"].items()}
        G.set_momentum(mod, 1.0)
        mod.train()
        with torch.no_grad():
            call(warm)
        G.set_momentum(mod, 0.1)
        for k, v in G.bn_buffers(mod).items():
            arrays["before." + k] = v
        mod.eval()
    else:
        mod.train()
    tin = {k: torch.from_numpy(v).requires_grad_(True) for k, v in inputs.items()}
    out = call(tin)
    outs = {}
    if isinstance(out, tuple):
        for name, v in zip(("out_l", "out_g"), out):
            if isinstance(v, torch.Tensor):
                outs[name] = v
    else:
        outs["out"] = out
    loss = 0.0
    for k, v in outs.items():
        cot = input_array(seed + 11, "cot:" + k, list(v.shape))
        arrays["cot." + k] = cot
        arrays["ref." + k] = v.detach().numpy()
        loss = loss + (v * torch.from_numpy(cot)).sum()
    loss.backward()
    for k, t in tin.items():
        arrays["gin." + k] = t.grad.numpy()
    for k, p in mod.named_parameters():
        if p.grad is not None:
            arrays["gpar." + k] = p.grad.numpy()
    return specs, arrays


def main():
    ref = G.load_reference()
    build_cases()
    manifest = {"generator": "tests/golden/gen_golden_grad.py", "torch": torch.__version__,
                "numpy": np.__version__, "cases": []}
    total = 0
    for c in CASES:
        specs, arrays = run_case(ref, c)
        path = os.path.join(HERE, c["name"] + ".npz")
        np.savez_compressed(path, **arrays)
        total += os.path.getsize(path)
        entry = dict(c)
        entry["specs"] = specs
        entry["outputs"] = sorted(k for k in arrays if k.startswith("ref."))
        entry["grads"] = sorted(k for k in arrays if k.startswith(("gin.", "gpar.")))
        manifest["cases"].append(entry)
        print(f"{c['name']:30s} {os.path.getsize(path)/1024:8.1f} KiB  grads={len(entry['grads'])}")
    with open(os.path.join(HERE, "manifest_grad.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"total {total/1024/1024:.2f} MiB")


if __name__ == "__main__":
    main()
