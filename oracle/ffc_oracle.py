"""ORACLE — CPU restatement of the reference FFC forward.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product path (``fastfourierconvolution_amd``) never imports it.

It restates, op for op, the reference's forward for the hot path named by
BASELINE.json:north_star (file:line citations into /root/reference):

* Fourier unit      layers/ffc/fourier_unity.py:32-56
* SE gate           layers/ffc/spectral_transform.py:12-28
* spectral transform layers/ffc/spectral_transform.py:36-110
* FFC               layers/ffc/ffc.py:21-99
* FFCTranspose      layers/ffc/ffc_transpose.py:19-110
* FFC_BN_ACT        layers/ffc/ffc_bn_act.py:25-83
* Resizer           layers/resizer.py:15-24
* FFCGenerator      models/ffc_generator.py:21-44
* FFCDiscriminator  models/ffc_discriminator.py:18-58
* NoiseInjection    layers/noise_injection.py:20-32
* fgan128 FGenerator fgan128_complete.py:442-522 (reconstructed: the script runs main() at import)
* SNFFC             layers/snffc/snffc.py:12-33 (torch.nn.utils.spectral_norm restated: sn_materialize)
* fgan128 Discriminator fgan128_complete.py:525-572 (a plain spectral-norm CNN: pinned against torch.nn
  modules built per those lines, tests/test_oracle_fgan_d.py)

The arithmetic itself lives in the un-vendored third-party dependency PyTorch
(pinned torch==1.10.2 at requirements.txt:5).  Its published semantics are
restated here: convolutions / batch norm through torch CPU ops in the dtype
of the inputs (float64 for parity checks), and the 2-D real FFTs through an
independent implementation (numpy's pocketfft, float64) with the same
``norm="ortho"`` scaling and the same C2R rule (inverse C2C over H, then C2R
over W that ignores the imaginary part of the k_w = 0 and k_w = W/2 bins).
``fft="torch"`` switches the FFTs to torch.fft (the reference's own calls), which
is the op-for-op fp32 CPU path timed as bench.py's cpu_baseline.

Pinning: tests/test_oracle_golden.py checks every function here against the
golden vectors in tests/golden/, produced by running the reference itself
(tests/golden/gen_golden.py).  The reference ships no tests of its own.

Parameters are passed as a flat ``state_dict``-style mapping using the
reference's key names (e.g. ``ffc1.ffc.convg2g.fu.conv_layer.weight``); train
mode updates the BatchNorm running buffers in that mapping in place, exactly as
nn.BatchNorm2d does.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

ACTS = ("Identity", "ReLU", "LeakyReLU", "Tanh", "Sigmoid", "GELU")


# ----------------------------------------------------------------------------- primitives
def rfft2_ortho(x: torch.Tensor, fft: str = "numpy") -> torch.Tensor:
    """torch.fft.rfftn(x, dim=(-2,-1), norm="ortho")  (fourier_unity.py:38)."""
    if fft == "torch":
        return torch.fft.rfftn(x, dim=(-2, -1), norm="ortho")
    a = np.fft.rfftn(x.detach().double().numpy(), axes=(-2, -1), norm="ortho")
    return torch.from_numpy(a).to(torch.complex128 if x.dtype == torch.float64 else torch.complex64)


def irfft2_ortho(X: torch.Tensor, s, fft: str = "numpy") -> torch.Tensor:
    """torch.fft.irfftn(X, s=s, dim=(-2,-1), norm="ortho")  (fourier_unity.py:56)."""
    if fft == "torch":
        return torch.fft.irfftn(X, s=s, dim=(-2, -1), norm="ortho")
    a = np.fft.irfftn(X.detach().cdouble().numpy(), s=tuple(s), axes=(-2, -1), norm="ortho")
    return torch.from_numpy(a).to(torch.float64 if X.dtype == torch.complex128 else torch.float32)


def batch_norm(x, sd, prefix, training, momentum=0.1, eps=1e-5):
    """nn.BatchNorm2d forward incl. running-stat update (biased var to normalise,
    unbiased var into running_var, num_batches_tracked += 1)."""
    w, b = sd[prefix + "weight"], sd[prefix + "bias"]
    rm, rv = sd[prefix + "running_mean"], sd[prefix + "running_var"]
    if training:
        dims = [0] + list(range(2, x.dim()))
        n = x.numel() // x.shape[1]
        mean = x.mean(dim=dims)
        var = x.var(dim=dims, unbiased=False)
        y = (x - mean[None, :, None, None]) / torch.sqrt(var[None, :, None, None] + eps)
        with torch.no_grad():
            unb = var * (n / max(n - 1, 1))
            rm.mul_(1 - momentum).add_(momentum * mean.to(rm.dtype))
            rv.mul_(1 - momentum).add_(momentum * unb.to(rv.dtype))
            key = prefix + "num_batches_tracked"
            if key in sd:
                sd[key] += 1
    else:
        y = (x - rm.to(x.dtype)[None, :, None, None]) / torch.sqrt(rv.to(x.dtype)[None, :, None, None] + eps)
    return y * w.to(x.dtype)[None, :, None, None] + b.to(x.dtype)[None, :, None, None]


def activation(x, name):
    """ffc_bn_act.py:63-67 — LeakyReLU is built with slope 0.1; GELU is the exact (erf) form."""
    if isinstance(x, int):
        return x
    if name == "Identity":
        return x
    if name == "ReLU":
        return F.relu(x)
    if name == "LeakyReLU":
        return F.leaky_relu(x, 0.1)
    if name == "Tanh":
        return torch.tanh(x)
    if name == "Sigmoid":
        return torch.sigmoid(x)
    if name == "GELU":
        return F.gelu(x)
    raise ValueError(name)


def _w(sd, key, dtype):
    return sd[key].to(dtype)


# ----------------------------------------------------------------------------- Fourier unit
def fourier_unit(x, sd, prefix, training, fft="numpy"):
    """FourierUnitSN.forward (fourier_unity.py:32-56), y=None path."""
    b, c, h, w = x.shape
    X = rfft2_ortho(x, fft)                                            # :38
    Z = torch.stack((X.real, X.imag), dim=-1)                          # :40
    Z = Z.permute(0, 1, 4, 2, 3).contiguous().view(b, 2 * c, h, -1)    # :41-42 (interleaved Re/Im)
    Y = F.conv2d(Z, _w(sd, prefix + "conv_layer.weight", x.dtype))     # :45 (1x1, groups=1)
    Y = F.relu(batch_norm(Y, sd, prefix + "bn.", training))            # :49
    Y = Y.view(b, -1, 2, h, Y.shape[-1]).permute(0, 1, 3, 4, 2).contiguous()  # :51-52
    Xc = torch.complex(Y[..., 0], Y[..., 1])                           # :53
    return irfft2_ortho(Xc, (h, w), fft)                               # :56


# ----------------------------------------------------------------------------- spectral transform
def se_layer(x, sd, prefix):
    """SELayer.forward (spectral_transform.py:23-28); hidden width C//16 may be 0 -> gate 0.5."""
    b, c = x.shape[:2]
    y = x.mean(dim=(2, 3))
    w1 = _w(sd, prefix + "fc.0.weight", x.dtype)
    w2 = _w(sd, prefix + "fc.2.weight", x.dtype)
    y = torch.sigmoid(F.linear(F.relu(F.linear(y, w1)), w2))
    return x * y.view(b, c, 1, 1)


def spectral_transform(x, sd, prefix, stride, upsample, training, fft="numpy"):
    """SpectralTransform.forward (spectral_transform.py:77-110)."""
    if stride == 2 and upsample:                                        # :44-45
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    elif stride == 2:                                                   # :46-47
        x = F.avg_pool2d(x, 2, 2)
    x = se_layer(x, sd, prefix + "se_block.")                          # :87
    x = F.conv2d(x, _w(sd, prefix + "conv1.weight", x.dtype))          # :89
    x = F.relu(batch_norm(x, sd, prefix + "bn1.", training))
    out = fourier_unit(x, sd, prefix + "fu.", training, fft)           # :91 (lfu never executed :94-105)
    return F.conv2d(x + out, _w(sd, prefix + "conv2.weight", x.dtype))  # :108


# ----------------------------------------------------------------------------- FFC / FFCTranspose
def split_channels(in_ch, out_ch, r_in, r_out):
    """ffc.py:33-36 / ffc_transpose.py:37-40."""
    in_cg = int(in_ch * r_in)
    out_cg = int(out_ch * r_out)
    return in_ch - in_cg, in_cg, out_ch - out_cg, out_cg


def ffc(x, sd, prefix, cfg, training, fft="numpy"):
    """FFC.forward (ffc.py:84-99) when cfg['transpose'] is False, else
    FFCTranspose.forward (ffc_transpose.py:91-110).  Returns (out_l, out_g) with
    int 0 for an absent branch."""
    in_cl, in_cg, out_cl, out_cg = split_channels(cfg["in_channels"], cfg["out_channels"],
                                                  cfg["ratio_gin"], cfg["ratio_gout"])
    k, s, p = cfg["kernel_size"], cfg.get("stride", 1), cfg.get("padding", 0)
    d, op = cfg.get("dilation", 1), cfg.get("out_padding", 0)
    transpose = cfg.get("transpose", False)
    x_l, x_g = x if type(x) is tuple else (x, 0)

    def conv(name, inp, exists):
        if not exists:                         # nn.Identity returns its input (int 0 or tensor)
            return inp
        w = _w(sd, prefix + name + ".weight", inp.dtype)
        bkey = prefix + name + ".bias"
        b = _w(sd, bkey, inp.dtype) if bkey in sd else None
        if transpose:
            return F.conv_transpose2d(inp, w, b, s, p, op, 1, d)
        return F.conv2d(inp, w, b, s, p, d)

    out_l, out_g = 0, 0
    if cfg["ratio_gout"] != 1:
        out_l = conv("convl2l", x_l, not (in_cl == 0 or out_cl == 0)) + \
            conv("convg2l", x_g, not (in_cg == 0 or out_cl == 0))
    if cfg["ratio_gout"] != 0:
        out_g = conv("convl2g", x_l, not (in_cl == 0 or out_cg == 0))
        if not (in_cg == 0 or out_cg == 0):
            out_g = out_g + spectral_transform(x_g, sd, prefix + "convg2g.", s, transpose, training, fft)
    return out_l, out_g


def ffc_bn_act(x, sd, prefix, cfg, training, fft="numpy"):
    """FFC_BN_ACT.forward (ffc_bn_act.py:70-83); cfg['upsampling'] picks FFCTranspose."""
    c2 = dict(cfg)
    c2["transpose"] = cfg.get("upsampling", False)
    x_l, x_g = ffc(x, sd, prefix + "ffc.", c2, training, fft)
    r = cfg["ratio_gout"]
    norm = cfg.get("norm_layer", "Identity")
    act = cfg.get("activation_layer", "Identity")
    if norm == "BatchNorm2d" and r != 1 and not isinstance(x_l, int):
        x_l = batch_norm(x_l, sd, prefix + "bn_l.", training)
    if norm == "BatchNorm2d" and r != 0 and not isinstance(x_g, int):
        x_g = batch_norm(x_g, sd, prefix + "bn_g.", training)
    x_l = activation(x_l, act if r != 1 else "Identity")
    x_g = activation(x_g, act if r != 0 else "Identity")
    return x_l, x_g


def resizer(x):
    """Resizer.forward (resizer.py:15-24)."""
    if type(x) is tuple:
        return x[0] if type(x[1]) is int else torch.cat(list(x), dim=1)
    return x


# ----------------------------------------------------------------------------- callers
def generator_layers(nz, nc, ngf, g=0.5):
    """models/ffc_generator.py:24-28."""
    L = lambda i, o, ri, ro, s, p, act="LeakyReLU": dict(  # noqa: E731
        in_channels=i, out_channels=o, kernel_size=4, ratio_gin=ri, ratio_gout=ro, stride=s, padding=p,
        activation_layer=act, upsampling=True)
    return [L(nz, ngf * 8, 0, g, 1, 0), L(ngf * 8, ngf * 4, g, g, 2, 1), L(ngf * 4, ngf * 2, g, g, 2, 1),
            L(ngf * 2, ngf, g, g, 2, 1), L(ngf, nc, g, 0, 2, 1, "Tanh")]


def discriminator_layers(nc, ndf):
    """models/ffc_discriminator.py:26-31."""
    L = lambda i, o, ri, ro, s, p, act="LeakyReLU": dict(  # noqa: E731
        in_channels=i, out_channels=o, kernel_size=4, ratio_gin=ri, ratio_gout=ro, stride=s, padding=p,
        activation_layer=act)
    return [L(nc, ndf * 2, 0, 0.5, 2, 1), L(ndf * 2, ndf * 4, 0.5, 0.5, 2, 1), L(ndf * 4, ndf * 8, 0.5, 0.5, 2, 1),
            L(ndf * 8, ndf * 16, 0.5, 0.5, 2, 1), L(ndf * 16, 1, 0.5, 0, 1, 0, "Sigmoid")]


def ffc_generator(z, sd, nz, nc, ngf, training, fft="numpy"):
    """FFCGenerator.forward (models/ffc_generator.py:30-44)."""
    x = z
    for i, cfg in enumerate(generator_layers(nz, nc, ngf)):
        x = ffc_bn_act(x, sd, f"ffc{i}.", cfg, training, fft)
    return resizer(x)


def ffc_discriminator(x, sd, nc, ndf, training, fft="numpy"):
    """FFCDiscriminator.forward (models/ffc_discriminator.py:33-58)."""
    for i, cfg in enumerate(discriminator_layers(nc, ndf)):
        x = ffc_bn_act(x, sd, f"ffc{i}.", cfg, training, fft)
    return resizer(x)


def fgan128_layers(ngf=128, g=0.5):
    """fgan128_complete.py:457-485: conv2..conv7 FFC_BN_ACT configs."""
    T = lambda i, o, ri, ro: dict(in_channels=i, out_channels=o, kernel_size=4, ratio_gin=ri,  # noqa: E731
                                  ratio_gout=ro, stride=2, padding=1, activation_layer="GELU",
                                  norm_layer="BatchNorm2d", upsampling=True)
    return [("conv2", T(ngf * 8, ngf * 4, 0.0, g)), ("conv3", T(ngf * 4, ngf * 2, g, g)),
            ("conv4", T(ngf * 2, ngf, g, g)), ("conv5", T(ngf, ngf, g, g)), ("conv6", T(ngf, ngf, g, g)),
            ("conv7", dict(in_channels=ngf, out_channels=3, kernel_size=3, ratio_gin=g, ratio_gout=0.0, stride=1,
                           padding=1, activation_layer="Tanh", norm_layer="Identity", upsampling=False))]


def noise_injection(x, sd, prefix, noise):
    """NoiseInjection.forward(x, noise) (layers/noise_injection.py:25-32): x + weight * noise,
    noise (B, 1, H, W) broadcast over channels."""
    return x + _w(sd, prefix + "weight", x.dtype) * noise


def fgan128_generator(z, sd, training, noises=None, mg=4, ngf=128, fft="numpy"):
    """FGenerator.forward (fgan128_complete.py:489-522) up to (not including) the eval-mode uint8
    quantization.  ``noises``: train-mode NoiseInjection noise, a list of (lcl, glb) pairs for
    conv2..conv6 (the reference draws them with normal_(); parity passes them explicitly)."""
    x = F.linear(z, _w(sd, "noise_to_feature.0.weight", z.dtype), _w(sd, "noise_to_feature.0.bias", z.dtype))
    x = x.reshape(x.size(0), -1, mg, mg)                                        # :494
    for i, (name, cfg) in enumerate(fgan128_layers(ngf)):
        x = ffc_bn_act(x, sd, name + ".", cfg, training, fft)
        if training and name != "conv7":                                        # :498-515
            n = int(name[-1])
            nl, ng = noises[i]
            x = (noise_injection(x[0], sd, f"lcl_noise{n}.", nl), noise_injection(x[1], sd, f"glb_noise{n}.", ng))
    return resizer(x)


def quantize_u8(fake):
    """eval-mode output (fgan128_complete.py:516-521): 255 * (clamp(x, min x, max x) * 0.5 + 0.5) -> uint8.
    The clamp to the tensor's own range is the identity."""
    return (255 * (fake * 0.5 + 0.5)).to(torch.uint8)


def sn_materialize(sd, dims, training, n_power_iterations=1, eps=1e-12):
    """torch.nn.utils.spectral_norm's SpectralNorm.compute_weight (torch/nn/utils/spectral_norm.py,
    the un-vendored dependency the reference's layers/snffc/*.py call) for every ``<m>.weight_orig``
    in ``sd``: sd[<m>.weight] = W / sigma, sigma = u . (W_mat v); in training mode one power
    iteration first updates u and v in place (v = normalize(W_mat^T u), u = normalize(W_mat v)).
    ``dims[m]``: the reshape dim (0 for Conv2d / Linear, 1 for ConvTranspose2d)."""
    for key in [k for k in sd if k.endswith(".weight_orig")]:
        m = key[: -len(".weight_orig")]
        W = sd[key]
        d = dims.get(m, 0)
        Wm = W.permute(d, *[i for i in range(W.dim()) if i != d]).reshape(W.shape[d], -1) if d else \
            W.reshape(W.shape[0], -1)
        u, v = sd[m + ".weight_u"], sd[m + ".weight_v"]
        if training:
            with torch.no_grad():   # u, v are constants of the weight's gradient, as in torch
                for _ in range(n_power_iterations):
                    v = F.normalize(torch.mv(Wm.t(), u), dim=0, eps=eps)
                    u = F.normalize(torch.mv(Wm, v), dim=0, eps=eps)
            sd[m + ".weight_u"], sd[m + ".weight_v"] = u, v
        sigma = torch.dot(u, torch.mv(Wm, v))
        sd[m + ".weight"] = W / sigma
    return sd


FGAN_D_CONVS = ((3, 64, 3, 1), (64, 64, 4, 2), (64, 128, 3, 1), (128, 128, 4, 2), (128, 256, 3, 1),
                (256, 256, 4, 2), (256, 512, 3, 1), (512, 512, 4, 2), (512, 512, 4, 2))


def fgan128_discriminator(x, sd, training, sn=True, mg=4):
    """Discriminator.forward (fgan128_complete.py:525-562): conv1..conv9 (padding 1, bias) each followed
    by LeakyReLU(0.1), fc on the flattened (512, mg, mg) map, no output activation.  With ``sn`` the
    spectral-norm weights are materialized first (sn_materialize: one power iteration in training
    mode, which updates sd's u / v as the reference's module call does)."""
    if sn:
        sn_materialize(sd, {}, training)
    for i, (_, _, k, s) in enumerate(FGAN_D_CONVS, 1):
        x = F.leaky_relu(F.conv2d(x, _w(sd, f"conv{i}.weight", x.dtype), _w(sd, f"conv{i}.bias", x.dtype),
                                  stride=s, padding=1), 0.1)
    x = x.reshape(-1, mg * mg * 512)                                               # :556
    return F.linear(x, _w(sd, "fc.weight", x.dtype), _w(sd, "fc.bias", x.dtype))


def hinge_loss_gen(fake):
    """fgan128_complete.py:581-585"""
    return -fake.mean()


def hinge_loss_dis(fake, real):
    """fgan128_complete.py:566-572"""
    return F.relu(1.0 - real).mean() + F.relu(1.0 + fake).mean()


# ----------------------------------------------------------------------------- fixture driver
def forward_case(case: dict, sd: dict, tin: dict, training: bool, fft="numpy") -> dict:
    """the forward of one golden-manifest case -> {"out" | "out_l" | "out_g": tensor}"""
    kind, ctor = case["kind"], case["ctor"]
    if kind == "FourierUnitSN":
        out = {"out": fourier_unit(tin["x"], sd, "", training, fft)}
    elif kind == "SpectralTransform":
        out = {"out": spectral_transform(tin["x"], sd, "", ctor.get("stride", 1),
                                         ctor.get("upsample", False), training, fft)}
    elif kind == "FFC_BN_ACT":
        x = (tin["x_l"], tin["x_g"]) if "x_l" in tin else tin["x"]
        ol, og = ffc_bn_act(x, sd, "", ctor, training, fft)
        out = {}
        if not isinstance(ol, int):
            out["out_l"] = ol
        if not isinstance(og, int):
            out["out_g"] = og
    elif kind == "FFCGenerator":
        out = {"out": ffc_generator(tin["z"], sd, ctor["nz"], ctor["nc"], ctor["ngf"], training, fft)}
    elif kind == "FFCDiscriminator":
        out = {"out": ffc_discriminator(tin["x"], sd, ctor["nc"], ctor["ndf"], training, fft)}
    elif kind == "SNFFC":
        sn_materialize(sd, {}, training)
        x = (tin["x_l"], tin["x_g"]) if "x_l" in tin else tin["x"]
        ol, og = ffc(x, sd, "", ctor, training, fft)
        out = {}
        if not isinstance(ol, int):
            out["out_l"] = ol
        if not isinstance(og, int):
            out["out_g"] = og
    elif kind == "FGenerator":
        noises = [(tin.get(f"noise{n}_l"), tin.get(f"noise{n}_g")) for n in (2, 3, 4, 5, 6)]
        out = {"out": fgan128_generator(tin["z"], sd, training, noises, fft=fft)}
    else:
        raise ValueError(kind)
    return out


def run_fixture_case(case: dict, state: dict, inputs: dict, dtype=torch.float64, fft="numpy"):
    """Run one golden-manifest case (tests/golden/manifest.json) through the oracle.
    ``state`` maps key -> numpy array (it is converted and updated in place via the
    returned dict).  Returns (outputs dict, state dict of torch tensors)."""
    sd = {k: (torch.from_numpy(np.array(v)).to(dtype) if np.asarray(v).dtype.kind == "f"
              else torch.from_numpy(np.array(v))) for k, v in state.items()}
    tin = {k: torch.from_numpy(v).to(dtype) for k, v in inputs.items()}
    training = case["mode"] == "train"
    with torch.no_grad():
        out = forward_case(case, sd, tin, training, fft)
    return out, sd


PARAM_SUFFIXES = ("running_mean", "running_var", "num_batches_tracked", "weight_u", "weight_v")


def grad_case(case: dict, state: dict, inputs: dict, cots: dict, dtype=torch.float64):
    """Gradients of  loss = sum_k <out_k, cot_k>  for one case, by torch autograd through the
    op-for-op restatement (torch.fft, fp64): the reference differentiates the same ops through
    ATen (config 3, fwd+bwd).  -> (grads of inputs {name: t}, grads of parameters {key: t})."""
    sd = {k: (torch.from_numpy(np.array(v)).to(dtype) if np.asarray(v).dtype.kind == "f"
              else torch.from_numpy(np.array(v))) for k, v in state.items()}
    params = [k for k, v in sd.items() if v.is_floating_point() and not k.endswith(PARAM_SUFFIXES)]
    for k in params:
        sd[k].requires_grad_(True)
    tin = {k: torch.from_numpy(v).to(dtype).requires_grad_(True) for k, v in inputs.items()}
    with torch.enable_grad():
        out = forward_case(case, sd, tin, case["mode"] == "train", fft="torch")
        loss = sum((out[k] * torch.from_numpy(cots[k]).to(dtype)).sum() for k in out)
        names = list(tin) + params
        gs = torch.autograd.grad(loss, [tin[k] for k in tin] + [sd[k] for k in params], allow_unused=True)
    gin = {k: g for k, g in zip(names[:len(tin)], gs[:len(tin)]) if g is not None}
    gpar = {k: g for k, g in zip(params, gs[len(tin):]) if g is not None}
    return gin, gpar


def normwise_err(a, ref) -> float:
    """max|a-ref| / max|ref| — the parity metric of SURVEY.md §8c."""
    a = a.detach().double() if isinstance(a, torch.Tensor) else torch.as_tensor(a).double()
    ref = ref.detach().double() if isinstance(ref, torch.Tensor) else torch.as_tensor(ref).double()
    if ref.numel() == 0:
        return 0.0 if a.numel() == 0 else float("inf")
    den = ref.abs().max().item()
    return (a - ref).abs().max().item() / (den if den > 0 else 1.0)
