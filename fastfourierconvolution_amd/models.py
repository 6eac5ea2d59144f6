"""The reference's callers of the FFC block, restated over the drop-in layers.

FFCModel (models/ffcmodel.py:12-110), FFCGenerator (models/ffc_generator.py:14-44),
FFCDiscriminator (models/ffc_discriminator.py:11-58), the fgan128 FGenerator
(fgan128_complete.py:442-522, BASELINE config 4) and the fgan128 spectral-norm Discriminator it is
trained against (fgan128_complete.py:525-562).  The layer stacks are identical; the
only change is that the ``inplanes=`` keyword the reference callers pass (and its base class
rejects, models/ffcmodel.py:17) is accepted and ignored.
"""
import os

import torch
import torch.nn as nn

from . import _autograd as ag
from . import _runtime as rt
from ._lib import check, ptr
from . import _plan
from .config import Config
from .ffc import FFC_BN_ACT
from .layers_misc import NoiseInjection, Print, Resizer, debug_print

# FGenerator conv6 -> conv7 hand-off with the BN + GELU + noise pass deferred into the head's operand
# staging (FFC_DEFER_HEAD=0: the separate pass, for A/B runs).  The head is VALU-bound, so the
# deferred GELU uses a branch-free erf: B = 512 head 1.36 -> 2.46 ms, BN/act/noise pass 2.36 -> 0.79 ms,
# step 18.11 -> 17.61 ms (with erff the head took 4.05 ms: profiles/r02/ab1, s4)
DEFER_HEAD_INPUT = os.environ.get("FFC_DEFER_HEAD", "1") != "0"


class FFCModel(nn.Module):
    def __init__(self, debug=False, inplanes=None):
        super().__init__()
        self.lfu = True
        self.use_se = False
        self.debug = debug
        self.print_size = Print(debug=Config.shared().DEBUG)
        self.resizer = Resizer()

    def get_lr(self, optimizer):
        for param_group in optimizer.param_groups:
            return param_group["lr"]

    def restore_checkpoint(self, ckpt_file, optimizer=None, scheduler=None):
        """models/ffcmodel.py:31-64 (state_dict keys are the reference's)."""
        if not ckpt_file:
            raise ValueError("No checkpoint file to be restored.")
        ckpt_dict = torch.load(ckpt_file, map_location="cpu", weights_only=True)
        self.load_state_dict(ckpt_dict["model_state_dict"])
        if optimizer:
            optimizer.load_state_dict(ckpt_dict["optimizer_state_dict"])
        if scheduler:
            scheduler.load_state_dict(ckpt_dict["scheduler_state_dict"])
        return ckpt_dict["global_step"]

    def save_checkpoint(self, directory, global_step, optimizer=None, scheduler=None, name=None):
        """models/ffcmodel.py:66-107: '{basename(dir)}_{step}_steps.pth'."""
        os.makedirs(directory, exist_ok=True)
        ckpt_dict = {
            "model_state_dict": self.state_dict(),
            "optimizer_state_dict": optimizer.state_dict() if optimizer is not None else None,
            "scheduler_state_dict": scheduler.state_dict() if scheduler is not None else None,
            "global_step": global_step,
        }
        if name is None:
            name = "{}_{}_steps.pth".format(os.path.basename(directory), global_step)
        torch.save(ckpt_dict, os.path.join(directory, name))

    def forward(self, x):
        pass


class FFCGenerator(FFCModel):
    def __init__(self, nz: int, nc: int, ngf: int, g_factor: float = 0.5, debug: bool = False):
        super().__init__(inplanes=ngf * 8, debug=debug)
        self.ffc0 = FFC_BN_ACT(nz, ngf * 8, 4, 0, g_factor, 1, 0, activation_layer=nn.LeakyReLU, upsampling=True)
        self.ffc1 = FFC_BN_ACT(ngf * 8, ngf * 4, 4, g_factor, g_factor, 2, 1, activation_layer=nn.LeakyReLU,
                               upsampling=True)
        self.ffc2 = FFC_BN_ACT(ngf * 4, ngf * 2, 4, g_factor, g_factor, 2, 1, activation_layer=nn.LeakyReLU,
                               upsampling=True)
        self.ffc3 = FFC_BN_ACT(ngf * 2, ngf * 1, 4, g_factor, g_factor, 2, 1, activation_layer=nn.LeakyReLU,
                               upsampling=True)
        self.ffc4 = FFC_BN_ACT(ngf * 1, nc, 4, g_factor, 0, 2, 1, norm_layer=nn.Identity, activation_layer=nn.Tanh,
                               upsampling=True)

    def forward(self, x):
        debug_print("G --")
        x = self.ffc0(x)
        x = self.print_size(x)
        x = self.ffc1(x)
        x = self.print_size(x)
        x = self.ffc2(x)
        x = self.print_size(x)
        x = self.ffc3(x)
        x = self.print_size(x)
        x = self.ffc4(x)
        x = self.resizer(x)
        debug_print("End G --")
        return x


class FFCDiscriminator(FFCModel):
    def __init__(self, nc: int, ndf: int, debug: bool = False):
        super().__init__(inplanes=ndf, debug=debug)
        self.ffc0 = FFC_BN_ACT(nc, ndf * 2, 4, 0, 0.5, 2, 1, activation_layer=nn.LeakyReLU)
        self.ffc1 = FFC_BN_ACT(ndf * 2, ndf * 4, 4, 0.5, 0.5, 2, 1, activation_layer=nn.LeakyReLU)
        self.ffc2 = FFC_BN_ACT(ndf * 4, ndf * 8, 4, 0.5, 0.5, 2, 1, activation_layer=nn.LeakyReLU)
        self.ffc3 = FFC_BN_ACT(ndf * 8, ndf * 16, 4, 0.5, 0.5, 2, 1, activation_layer=nn.LeakyReLU)
        self.ffc4 = FFC_BN_ACT(ndf * 16, 1, 4, 0.5, 0, 1, 0, norm_layer=nn.Identity, activation_layer=nn.Sigmoid)

    def forward(self, x):
        debug_print("D --")
        x = self.print_size(x)
        x = self.ffc0(x)
        x = self.print_size(x)
        x = self.ffc1(x)
        x = self.print_size(x)
        x = self.ffc2(x)
        x = self.print_size(x)
        x = self.ffc3(x)
        x = self.ffc4(x)
        x = self.resizer(x)
        x = self.print_size(x)
        debug_print("End D --")
        return x


class FGenerator(FFCModel):
    """fgan128_complete.py:442-522: Linear(z, 16*1024) -> (1024, 4, 4) -> five x2 FFC_BN_ACT
    (FFCTranspose, BatchNorm2d + GELU, train-mode NoiseInjection on both branches) -> 3x3 FFC_BN_ACT
    head (Tanh) -> Resizer; eval mode returns the uint8 image of :516-521.

    ``forward(z, noises=None)``: ``noises`` optionally supplies the train-mode noise as
    [(lcl, glb)] * 5 ((B, 1, H, W) each) instead of drawing it (the reference draws it inside
    NoiseInjection with normal_()); the reference's forward(z) is the noises=None call."""

    def __init__(self, z_size, mg: int = 4):
        super().__init__()
        self.z_size = z_size
        self.ngf = 128
        ratio_g = 0.5
        self.mg = mg
        ngf = self.ngf
        self.noise_to_feature = nn.Sequential(nn.Linear(z_size, (self.mg * self.mg) * self.ngf * 8))
        T = dict(activation_layer=nn.GELU, norm_layer=nn.BatchNorm2d, upsampling=True, uses_noise=True,
                 uses_sn=True)
        self.conv2 = FFC_BN_ACT(ngf * 8, ngf * 4, 4, 0.0, ratio_g, stride=2, padding=1, **T)
        self.lcl_noise2 = NoiseInjection(int(ngf * 4 * (1 - ratio_g)))
        self.glb_noise2 = NoiseInjection(int(ngf * 4 * ratio_g))
        self.conv3 = FFC_BN_ACT(ngf * 4, ngf * 2, 4, ratio_g, ratio_g, stride=2, padding=1, **T)
        self.lcl_noise3 = NoiseInjection(int(ngf * 2 * (1 - ratio_g)))
        self.glb_noise3 = NoiseInjection(int(ngf * 2 * ratio_g))
        self.conv4 = FFC_BN_ACT(ngf * 2, ngf, 4, ratio_g, ratio_g, stride=2, padding=1, **T)
        self.lcl_noise4 = NoiseInjection(int(ngf * (1 - ratio_g)))
        self.glb_noise4 = NoiseInjection(int(ngf * ratio_g))
        self.conv5 = FFC_BN_ACT(ngf, ngf, 4, ratio_g, ratio_g, stride=2, padding=1, **T)
        self.lcl_noise5 = NoiseInjection(int(ngf * (1 - ratio_g)))
        self.glb_noise5 = NoiseInjection(int(ngf * ratio_g))
        self.conv6 = FFC_BN_ACT(ngf, ngf, 4, ratio_g, ratio_g, stride=2, padding=1, **T)
        self.lcl_noise6 = NoiseInjection(int(ngf * (1 - ratio_g)))
        self.glb_noise6 = NoiseInjection(int(ngf * ratio_g))
        self.conv7 = FFC_BN_ACT(ngf, 3, 3, ratio_g, 0.0, stride=1, padding=1, activation_layer=nn.Tanh,
                                norm_layer=nn.Identity, upsampling=False, uses_noise=True, uses_sn=True)

    def _noise_to_feature(self, z):
        """nn.Linear(z_size, 16*1024) (fgan128_complete.py:453-455) on the HIP dense GEMM"""
        lin = self.noise_to_feature[0]
        z = rt.require(z, "z")
        if z.dim() != 2 or z.shape[1] != lin.in_features:
            raise RuntimeError(f"FGenerator: z must be (B, {lin.in_features}), got {tuple(z.shape)}")
        B = z.shape[0]
        if ag.wants_grad(self.noise_to_feature, z):   # training path: Linear as a 1x1 conv job with autograd
            return ag.linear(lin, z).view(B, -1, self.mg, self.mg)
        return torch.ops.ffc.linear(z, lin.weight, lin.bias).view(B, -1, self.mg, self.mg)

    def forward_float(self, z, noises=None):
        """FGenerator.forward up to the float image (:491-515): the eval-mode uint8 quantization of
        :516-521 is left out"""
        fake = self._noise_to_feature(z)                                     # :491-494
        grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        for i, n in enumerate((2, 3, 4, 5, 6)):                              # :496-515
            conv = getattr(self, f"conv{n}")
            # conv6 -> conv7: conv6's BN + GELU (+ noise) is applied by the 3x3 head as it stages its
            # input (ffc_conv3x3_smallm_tf), no separate pass over the 128x128 activations
            defer = n == 6 and not grad and DEFER_HEAD_INPUT
            if self.training:   # NoiseInjection fused into conv{n}'s BN + GELU pass
                nl, ng = noises[i] if noises is not None else (None, None)
                nzl, nzg = (getattr(self, f"lcl_noise{n}"), nl), (getattr(self, f"glb_noise{n}"), ng)
                fake = conv.forward_deferred(fake, nzl, nzg) if defer else conv.forward_noise(fake, nzl, nzg)
            else:
                fake = conv.forward_deferred(fake) if defer else conv(fake)
        return self.resizer(self.conv7(fake))

    def forward(self, z, noises=None):
        fake = self.forward_float(z, noises)
        if self.training:
            return fake
        return torch.ops.ffc.quantize_u8(fake)   # :516-521


class Discriminator(FFCModel):
    """fgan128_complete.py:525-562: the plain-CNN critic FGenerator is trained against (:616, :680-703).
    conv1..conv9 (3x3 s1 / 4x4 s2 Conv2d with bias, spectral norm when ``sn``), LeakyReLU(0.1) after
    each, fc = Linear(mg*mg*512, 1) on the flattened 4x4x512 map, no output activation (the reference
    builds ``last_act`` = Sigmoid and leaves it unused, :545-546, :558).  Module names and the
    state_dict are the reference's.

    Every conv is one implicit-GEMM launch of libffc_amd.so with bias + LeakyReLU in its epilogue
    (the ffc::conv_layer op: data / weight / bias gradients on the HIP kernels too); the spectral-norm
    pre-hook runs before each launch as the reference's module call runs it (one power iteration per
    forward in train mode).  Input: (B, 3, 32*mg, 32*mg) fp32 on the GPU."""

    CONVS = ((3, 64, 3, 1), (64, 64, 4, 2), (64, 128, 3, 1), (128, 128, 4, 2), (128, 256, 3, 1),
             (256, 256, 4, 2), (256, 512, 3, 1), (512, 512, 4, 2), (512, 512, 4, 2))

    def __init__(self, sn: bool = True, mg: int = 4):
        super().__init__()
        self.mg = mg
        sn_fn = torch.nn.utils.spectral_norm if sn else (lambda m: m)
        for i, (cin, cout, k, s) in enumerate(self.CONVS, 1):
            setattr(self, f"conv{i}", sn_fn(nn.Conv2d(cin, cout, k, stride=s, padding=(1, 1))))
        self.fc = sn_fn(nn.Linear(self.mg * self.mg * 512, 1))
        self.act = nn.LeakyReLU(0.1)
        self.last_act = nn.Sigmoid()

    def forward(self, x):
        x = rt.require(x, "x")
        side = 32 * self.mg
        if x.dim() != 4 or tuple(x.shape[1:]) != (3, side, side):
            raise RuntimeError(f"Discriminator: x must be (B, 3, {side}, {side}), got {tuple(x.shape)}")
        act, param = rt.act_code(self.act)
        m = x
        for i in range(1, len(self.CONVS) + 1):
            conv = getattr(self, f"conv{i}")
            B, C, H, W = m.shape
            sg = _plan.Seg("conv", C, H, W, conv.kernel_size[0], conv.stride[0], conv.padding[0])
            (m,) = ag.conv_layer(B, [(conv.out_channels, act, param)], [(0, 0, sg, conv)], [m])
        return ag.linear(self.fc, m.reshape(m.shape[0], -1))   # :556


FGanDiscriminator = Discriminator
