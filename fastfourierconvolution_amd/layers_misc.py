"""Caller helpers of the FFC block: Resizer (layers/resizer.py:10-24), Print / debug_print
(layers/print_layer.py:10-32), NoiseInjection (layers/noise_injection.py:20-32).

Resizer / Print only move tuples around or print shapes.  NoiseInjection's add (fgan128 train
mode) runs in the HIP library (ffc_noise_inject); the noise itself is drawn with torch's device
RNG as the reference draws it with normal_() (or passed explicitly, as in the reference's
``forward(x, noise)``).
"""
import torch
import torch.nn as nn

from .config import Config


def debug_print(*txt):
    if Config.shared().DEBUG:
        print(*txt)


class Print(nn.Module):
    def __init__(self, debug=False):
        super().__init__()
        self.debug = debug

    def forward(self, x):
        if self.debug:
            if type(x) == tuple:
                if type(x[1]) == int:
                    print(x[0].shape, "global = 0")
                else:
                    aux = torch.cat(list(x), dim=1)
                    aux = aux.view(aux.shape[0], -1, *aux.shape[3:])
                    print(aux.shape)
            else:
                print(x.shape)
        return x


class Resizer(nn.Module):
    def __init__(self, debug=False):
        super().__init__()
        self.print_size = Print(debug=debug)

    def forward(self, x):
        output = x
        if type(x) == tuple:
            if type(x[1]) == int:
                output = x[0]
            else:
                output = torch.cat(list(x), dim=1)
                self.print_size(output)
        return output


class NoiseInjection(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(1, channels, 1, 1))

    def forward(self, x, noise=None):
        from . import _runtime as rt
        from ._lib import check, ptr
        x = rt.require(x, "x")
        batch, C, height, width = x.shape
        if noise is None:
            noise = x.new_empty(batch, 1, height, width).normal_()
        noise = rt.require(noise, "noise")
        if tuple(noise.shape) != (batch, 1, height, width) or (height * width) % 4:
            raise NotImplementedError("NoiseInjection: noise must be (B, 1, H, W) with H*W % 4 == 0")
        from . import _autograd as ag
        if ag.wants_grad(self, x):   # training path: weight gradient through ffc_noise_wgrad
            return ag.noise_inject(self, x, noise)
        w = rt.require(self.weight.detach(), "weight")
        out = torch.empty_like(x)
        with rt.observe("noise_inject", bytes=8.0 * x.numel() + 4.0 * noise.numel()):
            check(rt.lib().ffc_noise_inject(ptr(x), ptr(w), ptr(noise), ptr(out), batch, C, height * width,
                                            rt.stream_of(x)), "ffc_noise_inject")
        return out
