"""Drop-in ``FFC_BN_ACT`` (reference: layers/ffc/ffc_bn_act.py:11-83): the model-facing block.

forward runs the ``ffc::ffc_bn_act`` custom op (ops.py; the training ops under autograd).  The
activation is fused into the local-branch GEMM epilogue; with norm_layer=BatchNorm2d the GEMM
epilogue collects BN partials and one BN+activation pass follows.
"""
import torch.nn as nn

from .. import _runtime as rt
from .ffc import FFC, layer_call
from .ffc_transpose import FFCTranspose


class FFC_BN_ACT(nn.Module):
    def __init__(self, in_channels, out_channels,
                 kernel_size, ratio_gin, ratio_gout,
                 stride=1, padding=0, dilation=1, groups=1, bias=False,
                 norm_layer: nn.Module = nn.Identity, activation_layer: nn.Module = nn.Identity,
                 enable_lfu=True, upsampling=False, out_padding=0,
                 uses_noise: bool = False, uses_sn: bool = False, num_classes: int = 1):
        super().__init__()
        self._ffc_ctor = ["FFC_BN_ACT", dict(in_channels=in_channels, out_channels=out_channels,
                                             kernel_size=kernel_size, ratio_gin=ratio_gin, ratio_gout=ratio_gout,
                                             stride=stride, padding=padding, dilation=dilation, groups=groups,
                                             bias=bias, norm_layer=norm_layer.__name__,
                                             activation_layer=activation_layer.__name__, enable_lfu=enable_lfu,
                                             upsampling=upsampling, out_padding=out_padding,
                                             num_classes=num_classes)]
        self.uses_sn = uses_sn
        if upsampling:
            self.ffc = FFCTranspose(in_channels, out_channels, kernel_size, ratio_gin, ratio_gout, stride, padding,
                                    dilation, groups, bias, enable_lfu, out_padding=out_padding,
                                    num_classes=num_classes)
        else:
            self.ffc = FFC(in_channels, out_channels, kernel_size, ratio_gin, ratio_gout, stride, padding,
                           dilation, groups, bias, enable_lfu, num_classes=num_classes)
        out_ch_l = int(out_channels * (1 - ratio_gout))
        out_ch_g = int(out_channels * ratio_gout)
        lnorm = nn.Identity if ratio_gout == 1 else norm_layer
        gnorm = nn.Identity if ratio_gout == 0 else norm_layer
        if num_classes > 1:
            self.bn_l = lnorm(out_ch_l, num_classes)
            self.bn_g = gnorm(out_ch_g, num_classes)
        else:
            self.bn_l = lnorm(out_ch_l)
            self.bn_g = gnorm(out_ch_g)
        lact = nn.Identity if ratio_gout == 1 else activation_layer
        gact = nn.Identity if ratio_gout == 0 else activation_layer
        self.act_l = lact(0.1, inplace=True) if isinstance(lact(), nn.LeakyReLU) else lact()
        self.act_g = gact(0.1, inplace=True) if isinstance(gact(), nn.LeakyReLU) else gact()

    @staticmethod
    def _norm(m):
        if isinstance(m, nn.Identity):
            return None
        if isinstance(m, nn.BatchNorm2d):
            return m
        raise NotImplementedError(f"norm layer {type(m).__name__} has no HIP path")

    def _call(self, x, y=None, noise=None, defer=False):
        bn_l, bn_g = self._norm(self.bn_l), self._norm(self.bn_g)
        if y is not None and (bn_l is not None or bn_g is not None):
            raise TypeError("FFC_BN_ACT: BatchNorm2d.forward() takes no label input (reference ffc_bn_act.py:73-81)")
        return layer_call(self, self.ffc, x, y, rt.act_code(self.act_l), rt.act_code(self.act_g), bn_l, bn_g,
                          noise=noise, defer=defer)

    def forward(self, x, y=None):
        return self._call(x, y)

    def forward_noise(self, x, noise_l, noise_g):
        """forward followed by NoiseInjection on both outputs (fgan128_complete.py:496-515), the noise add
        fused into the BN + activation pass.  noise_*: (NoiseInjection module, noise tensor or None)."""
        return self._call(x, noise={"l": noise_l, "g": noise_g})

    def forward_deferred(self, x, noise_l=None, noise_g=None):
        """forward (plus NoiseInjection when noise_* are given, as forward_noise) whose outputs are
        rt.PendingAct: BN + activation + noise are left to the consuming layer, which applies them
        while it stages its operands (or materializes them).  Not for autograd."""
        noise = {k: v for k, v in (("l", noise_l), ("g", noise_g)) if v is not None}
        return self._call(x, noise=noise or None, defer=True)
