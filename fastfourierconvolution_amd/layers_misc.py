"""Caller helpers of the FFC block: Resizer (layers/resizer.py:10-24), Print / debug_print
(layers/print_layer.py:10-32), NoiseInjection (layers/noise_injection.py:20-32).

Resizer / Print only move tuples around or print shapes.  NoiseInjection's add (fgan128 train
mode) runs in the HIP library (the ffc::noise_inject op); the noise itself is drawn with torch's device
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
        """x + weight * noise on the ffc::noise_inject op (its weight gradient on ffc::noise_wgrad)"""
        from . import _autograd as ag
        from . import _runtime as rt
        return ag.noise_inject(self, rt.require(x, "x"), noise)
