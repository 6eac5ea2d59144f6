"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run here only (the reference tree does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

How the reference is imported: ``import layers`` fails with an
ordinary ModuleNotFoundError (torchvision) via layers/__init__.py ->
layers/gaussian_noise.py -> util/data_loader.py, so the script registers
namespace modules ``layers`` / ``models`` whose ``__path__`` points into
/root/reference (their ``__init__.py`` files are not executed) plus a stub
``util`` exposing ``torch``/``os``.  ``FFCModel.__init__`` takes no
``inplanes`` (models/ffcmodel.py:17) although FFCGenerator/FFCDiscriminator
pass it (models/ffc_generator.py:22, models/ffc_discriminator.py:24); the
shim accepts and ignores it.  Nothing is written into /root/reference
(bytecode writing is disabled).

Outputs: manifest.json (case list: constructor args, input shapes, weight
specs) and one ``<case>.npz`` per case (inputs, outputs, BN buffers).
Weights are regenerated from (seed, key) by fixture_weights.make_state.
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from fixture_weights import input_array, make_state  # noqa: E402


def load_reference():
    sys.path.insert(0, REF)  # for the top-level ``config`` package
    util = types.ModuleType("util")
    util.torch = torch
    util.os = os
    sys.modules["util"] = util
    layers = types.ModuleType("layers")
    layers.__path__ = [REF + "/layers"]
    sys.modules["layers"] = layers
    import layers.ffc.ffc_bn_act as fba
    import layers.ffc.fourier_unity as fu
    import layers.ffc.spectral_transform as st
    import layers.noise_injection as ni
    import layers.print_layer as pl
    import layers.resizer as rs
    import layers.snffc.snffc as snf
    for mod in (fba, fu, st, ni, pl, rs):
        for name in dir(mod):
            if not name.startswith("_"):
                setattr(layers, name, getattr(mod, name))
    models = types.ModuleType("models")
    models.__path__ = [REF + "/models"]
    sys.modules["models"] = models
    import models.ffcmodel as fm
    orig_init = fm.FFCModel.__init__

    def shim_init(self, *args, inplanes=None, **kw):  # accept the kwarg the callers pass
        orig_init(self, *args, **kw)

    fm.FFCModel.__init__ = shim_init
    import models.ffc_discriminator as fd
    import models.ffc_generator as fg
    return types.SimpleNamespace(
        FourierUnitSN=fu.FourierUnitSN, SpectralTransform=st.SpectralTransform,
        FFC_BN_ACT=fba.FFC_BN_ACT, FFCGenerator=fg.FFCGenerator,
        FFCDiscriminator=fd.FFCDiscriminator, Resizer=rs.Resizer, NoiseInjection=ni.NoiseInjection,
        FFCModel=fm.FFCModel, SNFFC=snf.SNFFC)


def fgenerator_class(ref):
    """fgan128_complete.py:442-522 FGenerator, rebuilt from the reference's own layers (the script
    runs main() at import and needs torchvision/tensorboard/torch_fidelity).  Same
    module names and state_dict keys; forward takes the train-mode NoiseInjection noise explicitly
    (the reference draws it with normal_(), layers/noise_injection.py:26-28) and returns the float
    output (the eval-mode uint8 quantization of :516-521 is checked separately)."""
    class FGenerator(ref.FFCModel):
        def __init__(self, z_size=128, mg=4):
            super().__init__()
            self.z_size, self.ngf, self.mg = z_size, 128, mg
            ngf, g = self.ngf, 0.5
            self.noise_to_feature = nn.Sequential(nn.Linear(z_size, (mg * mg) * ngf * 8))
            T = dict(activation_layer=nn.GELU, norm_layer=nn.BatchNorm2d, upsampling=True, uses_noise=True,
                     uses_sn=True)
            self.conv2 = ref.FFC_BN_ACT(ngf * 8, ngf * 4, 4, 0.0, g, stride=2, padding=1, **T)
            self.lcl_noise2 = ref.NoiseInjection(int(ngf * 4 * (1 - g)))
            self.glb_noise2 = ref.NoiseInjection(int(ngf * 4 * g))
            self.conv3 = ref.FFC_BN_ACT(ngf * 4, ngf * 2, 4, g, g, stride=2, padding=1, **T)
            self.lcl_noise3 = ref.NoiseInjection(int(ngf * 2 * (1 - g)))
            self.glb_noise3 = ref.NoiseInjection(int(ngf * 2 * g))
            self.conv4 = ref.FFC_BN_ACT(ngf * 2, ngf, 4, g, g, stride=2, padding=1, **T)
            self.lcl_noise4 = ref.NoiseInjection(int(ngf * (1 - g)))
            self.glb_noise4 = ref.NoiseInjection(int(ngf * g))
            self.conv5 = ref.FFC_BN_ACT(ngf, ngf, 4, g, g, stride=2, padding=1, **T)
            self.lcl_noise5 = ref.NoiseInjection(int(ngf * (1 - g)))
            self.glb_noise5 = ref.NoiseInjection(int(ngf * g))
            self.conv6 = ref.FFC_BN_ACT(ngf, ngf, 4, g, g, stride=2, padding=1, **T)
            self.lcl_noise6 = ref.NoiseInjection(int(ngf * (1 - g)))
            self.glb_noise6 = ref.NoiseInjection(int(ngf * g))
            self.conv7 = ref.FFC_BN_ACT(ngf, 3, 3, g, 0.0, stride=1, padding=1, activation_layer=nn.Tanh,
                                        norm_layer=nn.Identity, upsampling=False, uses_noise=True, uses_sn=True)

        def forward(self, z, noises=None):
            fake = self.noise_to_feature(z)
            fake = fake.reshape(fake.size(0), -1, self.mg, self.mg)
            for i, n in enumerate((2, 3, 4, 5, 6)):
                fake = getattr(self, f"conv{n}")(fake)
                if self.training:
                    fake = (getattr(self, f"lcl_noise{n}")(fake[0], noises[i][0]),
                            getattr(self, f"glb_noise{n}")(fake[1], noises[i][1]))
            fake = self.conv7(fake)
            return self.resizer(fake)
    return FGenerator


def weight_specs(module: nn.Module) -> dict:
    """Per state_dict key: [shape, dist, a, b, dtype].  Fan-in scaled so signals stay O(1)."""
    specs = {}
    for mname, m in module.named_modules():
        pre = (mname + ".") if mname else ""
        if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)) and hasattr(m, "weight_orig"):
            # torch.nn.utils.spectral_norm: weight_orig + power-iteration vectors u (rows) / v (cols)
            w = m.weight_orig
            fan = w[0].numel()
            specs[pre + "weight_orig"] = [list(w.shape), "normal", 0.0, fan ** -0.5, "float32"]
            specs[pre + "weight_u"] = [list(m.weight_u.shape), "normal", 0.0, 1.0, "float32"]
            specs[pre + "weight_v"] = [list(m.weight_v.shape), "normal", 0.0, 1.0, "float32"]
            if m.bias is not None:
                specs[pre + "bias"] = [list(m.bias.shape), "normal", 0.0, 0.1, "float32"]
        elif isinstance(m, nn.ConvTranspose2d):
            i, o, kh, kw = m.weight.shape
            fan = max(1.0, i * kh * kw / float(m.stride[0] * m.stride[1]))
            specs[pre + "weight"] = [list(m.weight.shape), "normal", 0.0, fan ** -0.5, "float32"]
            if m.bias is not None:
                specs[pre + "bias"] = [list(m.bias.shape), "normal", 0.0, 0.1, "float32"]
        elif isinstance(m, nn.Conv2d):
            o, i, kh, kw = m.weight.shape
            specs[pre + "weight"] = [list(m.weight.shape), "normal", 0.0, (i * kh * kw) ** -0.5, "float32"]
            if m.bias is not None:
                specs[pre + "bias"] = [list(m.bias.shape), "normal", 0.0, 0.1, "float32"]
        elif isinstance(m, nn.Linear):
            fan = max(1, m.weight.shape[1])
            specs[pre + "weight"] = [list(m.weight.shape), "normal", 0.0, fan ** -0.5, "float32"]
            if m.bias is not None:
                specs[pre + "bias"] = [list(m.bias.shape), "normal", 0.0, 0.1, "float32"]
        elif type(m).__name__ == "NoiseInjection":
            specs[pre + "weight"] = [list(m.weight.shape), "normal", 0.0, 0.2, "float32"]
        elif isinstance(m, nn.BatchNorm2d):
            c = m.num_features
            specs[pre + "weight"] = [[c], "normal", 1.0, 0.1, "float32"]
            specs[pre + "bias"] = [[c], "normal", 0.0, 0.1, "float32"]
            specs[pre + "running_mean"] = [[c], "const", 0.0, 0.0, "float32"]
            specs[pre + "running_var"] = [[c], "const", 1.0, 0.0, "float32"]
            specs[pre + "num_batches_tracked"] = [[], "const", 0, 0, "int64"]
    sd = module.state_dict()
    missing = set(sd) - set(specs)
    assert not missing, missing
    return specs


def load_specs(module, seed, specs):
    arrays = make_state(seed, specs)
    module.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in arrays.items()})


def bn_buffers(module):
    out = {}
    for k, v in module.state_dict().items():
        if k.endswith(("running_mean", "running_var", "num_batches_tracked", "weight_u", "weight_v")):
            out[k] = v.detach().cpu().numpy()
    return out


def set_momentum(module, mom):
    for m in module.modules():
        if isinstance(m, nn.BatchNorm2d):
            m.momentum = mom


def as_pair(out):
    """Flatten the (x_l, x_g) tuple protocol: int 0 branches are recorded as absent."""
    if isinstance(out, tuple):
        res = {}
        for name, v in zip(("out_l", "out_g"), out):
            if isinstance(v, torch.Tensor):
                res[name] = v.detach().numpy()
        return res
    return {"out": out.detach().numpy()}


CASES = []


def case(name, kind, ctor, inputs, mode="train", seed=1234, note=""):
    CASES.append(dict(name=name, kind=kind, ctor=ctor, inputs=inputs, mode=mode, seed=seed, note=note))


def build_cases():
    # --- FourierUnitSN (layers/ffc/fourier_unity.py) at every FU shape of the named models
    for c, h, w, b in [(64, 8, 8, 2), (32, 16, 16, 2), (16, 32, 32, 2),   # FFCGenerator ffc1-3
                       (64, 16, 16, 2), (128, 8, 8, 2), (256, 4, 4, 2),   # FFCDiscriminator ffc1-3
                       (8, 32, 32, 3), (4, 16, 8, 2), (3, 4, 4, 3)]:       # config-1 block, non-square, odd c
        case(f"fu_c{c}_{h}x{w}", "FourierUnitSN", dict(in_channels=c, out_channels=c),
             {"x": [b, c, h, w]})
    for c, h, w in [(32, 16, 16), (16, 32, 32)]:
        case(f"fu_c{c}_{h}x{w}_eval", "FourierUnitSN", dict(in_channels=c, out_channels=c),
             {"x": [2, c, h, w]}, mode="eval")
    # --- SpectralTransform (layers/ffc/spectral_transform.py)
    case("st_gen_ffc1", "SpectralTransform", dict(in_channels=256, out_channels=128, stride=2, upsample=True),
         {"x": [2, 256, 4, 4]})
    case("st_gen_ffc3", "SpectralTransform", dict(in_channels=64, out_channels=32, stride=2, upsample=True),
         {"x": [2, 64, 16, 16]})
    case("st_disc_ffc1", "SpectralTransform", dict(in_channels=64, out_channels=128, stride=2, upsample=False),
         {"x": [2, 64, 32, 32]})
    case("st_block", "SpectralTransform", dict(in_channels=16, out_channels=16, stride=1),
         {"x": [2, 16, 32, 32]})
    case("st_se_hidden0", "SpectralTransform", dict(in_channels=8, out_channels=8, stride=1),
         {"x": [2, 8, 16, 16]})
    case("st_gen_ffc2_eval", "SpectralTransform", dict(in_channels=128, out_channels=64, stride=2, upsample=True),
         {"x": [2, 128, 8, 8]}, mode="eval")
    # --- FFC_BN_ACT (layers/ffc/ffc_bn_act.py)
    case("fba_config1", "FFC_BN_ACT",
         dict(in_channels=32, out_channels=32, kernel_size=3, ratio_gin=0.5, ratio_gout=0.5, stride=1, padding=1,
              norm_layer="BatchNorm2d", activation_layer="ReLU"),
         {"x_l": [4, 16, 32, 32], "x_g": [4, 16, 32, 32]}, note="BASELINE config 1 at B=4")
    case("fba_config1_eval", "FFC_BN_ACT",
         dict(in_channels=32, out_channels=32, kernel_size=3, ratio_gin=0.5, ratio_gout=0.5, stride=1, padding=1,
              norm_layer="BatchNorm2d", activation_layer="ReLU"),
         {"x_l": [2, 16, 32, 32], "x_g": [2, 16, 32, 32]}, mode="eval")
    case("fba_first_tensor_in", "FFC_BN_ACT",
         dict(in_channels=3, out_channels=32, kernel_size=4, ratio_gin=0.0, ratio_gout=0.5, stride=2, padding=1,
              activation_layer="LeakyReLU"),
         {"x": [2, 3, 32, 32]})
    case("fba_transpose_lrelu", "FFC_BN_ACT",
         dict(in_channels=64, out_channels=32, kernel_size=4, ratio_gin=0.5, ratio_gout=0.5, stride=2, padding=1,
              activation_layer="LeakyReLU", upsampling=True),
         {"x_l": [2, 32, 8, 8], "x_g": [2, 32, 8, 8]})
    case("fba_transpose_bn_gelu", "FFC_BN_ACT",
         dict(in_channels=64, out_channels=64, kernel_size=4, ratio_gin=0.5, ratio_gout=0.5, stride=2, padding=1,
              activation_layer="GELU", norm_layer="BatchNorm2d", upsampling=True),
         {"x_l": [2, 32, 8, 8], "x_g": [2, 32, 8, 8]}, note="fgan128 conv3-6 layer shape family")
    case("fba_head_3x3_tanh", "FFC_BN_ACT",
         dict(in_channels=32, out_channels=3, kernel_size=3, ratio_gin=0.5, ratio_gout=0.0, stride=1, padding=1,
              activation_layer="Tanh"),
         {"x_l": [2, 16, 32, 32], "x_g": [2, 16, 32, 32]}, note="fgan128 conv7 family")
    case("fba_disc_last_sigmoid", "FFC_BN_ACT",
         dict(in_channels=64, out_channels=1, kernel_size=4, ratio_gin=0.5, ratio_gout=0.0, stride=1, padding=0,
              activation_layer="Sigmoid"),
         {"x_l": [2, 32, 4, 4], "x_g": [2, 32, 4, 4]})
    # --- callers (models/ffc_generator.py, models/ffc_discriminator.py)
    case("gen_nc1", "FFCGenerator", dict(nz=100, nc=1, ngf=64), {"z": [4, 100, 1, 1]}, note="BASELINE config 2 shape")
    case("gen_nc3", "FFCGenerator", dict(nz=100, nc=3, ngf=64), {"z": [4, 100, 1, 1]})
    case("gen_nc3_eval", "FFCGenerator", dict(nz=100, nc=3, ngf=64), {"z": [4, 100, 1, 1]}, mode="eval")
    case("disc_nc3", "FFCDiscriminator", dict(nc=3, ndf=64), {"x": [2, 3, 64, 64]})
    blk = dict(in_channels=32, out_channels=32, kernel_size=3, ratio_gin=0.5, ratio_gout=0.5, stride=1, padding=1)
    case("snffc_block", "SNFFC", blk, {"x_l": [2, 16, 16, 16], "x_g": [2, 16, 16, 16]},
         note="layers/snffc/snffc.py: spectral norm, one power iteration (train)")
    case("snffc_block_eval", "SNFFC", blk, {"x_l": [2, 16, 16, 16], "x_g": [2, 16, 16, 16]}, mode="eval",
         note="layers/snffc/snffc.py: spectral norm with the stored u, v (eval)")
    noise = {f"noise{n}_{br}": [2, 1, 2 ** (n + 1), 2 ** (n + 1)] for n in (2, 3, 4, 5, 6) for br in "lg"}
    case("fgan128_train", "FGenerator", dict(z_size=128), {"z": [2, 128], **noise},
         note="BASELINE config 4 stack (fgan128_complete.py:442-522), train mode, explicit noise")
    case("fgan128_eval", "FGenerator", dict(z_size=128), {"z": [2, 128]}, mode="eval",
         note="BASELINE config 4 stack, eval mode (float output before the uint8 quantization)")


def construct(ref, c):
    if c["kind"] == "FGenerator":
        return fgenerator_class(ref)(**c["ctor"])
    kw = dict(c["ctor"])
    for k in ("norm_layer", "activation_layer"):
        if k in kw:
            kw[k] = getattr(nn, kw[k])
    with contextlib.redirect_stdout(io.StringIO()):  # FFC prints at construction (layers/ffc/ffc.py:38-39)
        return getattr(ref, c["kind"])(**kw)


def shp_b(c):
    return next(iter(c["inputs"].values()))[0]


def run_case(ref, c):
    torch.manual_seed(0)
    mod = construct(ref, c)
    specs = weight_specs(mod)
    load_specs(mod, c["seed"], specs)
    seed = c["seed"]
    inputs = {k: input_array(seed, k, shp) for k, shp in c["inputs"].items()}
    tin = {k: torch.from_numpy(v) for k, v in inputs.items()}

    def call(t):
        if c["kind"] == "FGenerator":
            noises = [(t.get(f"noise{n}_l"), t.get(f"noise{n}_g")) for n in (2, 3, 4, 5, 6)]
            return mod(t["z"], noises)
        if c["kind"] in ("FFC_BN_ACT", "SNFFC") and "x_l" in t:
            return mod((t["x_l"], t["x_g"]))
        return mod(next(iter(t.values())))

    arrays = {"in." + k: v for k, v in inputs.items()}
    if c["mode"] == "eval":
        # give the running stats realistic scales: stats of a different warm-up batch
        warm = {k: torch.from_numpy(input_array(seed + 7, k, shp)) for k, shp in c["inputs"].items()}
        if c["kind"] == "FGenerator":   # the warm-up pass is a train-mode pass: it needs noise
            warm.update({f"noise{n}_{br}": torch.from_numpy(input_array(seed + 7, f"noise{n}_{br}",
                                                                        [shp_b(c), 1, 2 ** (n + 1), 2 ** (n + 1)]))
                         for n in (2, 3, 4, 5, 6) for br in "lg"})
        set_momentum(mod, 1.0)
        mod.train()
        with torch.no_grad():
            call(warm)
        set_momentum(mod, 0.1)
        for k, v in bn_buffers(mod).items():
            arrays["before." + k] = v
        mod.eval()
    else:
        mod.train()
    with torch.no_grad():
        out = call(tin)
    for k, v in as_pair(out).items():
        arrays["ref." + k] = v
    for k, v in bn_buffers(mod).items():
        arrays["after." + k] = v
    return specs, arrays


def main():
    ref = load_reference()
    build_cases()
    manifest = {"generator": "tests/golden/gen_golden.py", "torch": torch.__version__,
                "numpy": np.__version__, "cases": []}
    total = 0
    only = set(sys.argv[1:])     # regenerate only these cases (the manifest keeps the others)
    old = {}
    if only and os.path.exists(os.path.join(HERE, "manifest.json")):
        old = {e["name"]: e for e in json.load(open(os.path.join(HERE, "manifest.json")))["cases"]}
    for c in CASES:
        if only and c["name"] not in only and c["name"] in old:
            manifest["cases"].append(old[c["name"]])
            continue
        specs, arrays = run_case(ref, c)
        path = os.path.join(HERE, c["name"] + ".npz")
        np.savez_compressed(path, **arrays)
        total += os.path.getsize(path)
        entry = dict(c)
        entry["specs"] = specs
        entry["outputs"] = sorted(k for k in arrays if k.startswith("ref."))
        manifest["cases"].append(entry)
        print(f"{c['name']:28s} {os.path.getsize(path)/1024:8.1f} KiB  outputs={entry['outputs']}")
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"total {total/1024/1024:.2f} MiB")


if __name__ == "__main__":
    main()
