"""The reference's callers of the FFC block, restated over the drop-in layers.

FFCModel (models/ffcmodel.py:12-110), FFCGenerator (models/ffc_generator.py:14-44) and
FFCDiscriminator (models/ffc_discriminator.py:11-58).  The layer stacks are identical; the
only change is that the ``inplanes=`` keyword the reference callers pass (and its base class
rejects, models/ffcmodel.py:17) is accepted and ignored.
"""
import os

import torch
import torch.nn as nn

from .config import Config
from .ffc import FFC_BN_ACT
from .layers_misc import Print, Resizer, debug_print


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
