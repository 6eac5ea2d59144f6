"""Drop-in ``FFCTranspose`` (reference: layers/ffc/ffc_transpose.py:10-110).

Local branch: nn.ConvTranspose2d modules (run as phase-decomposed implicit GEMMs);
global branch: SpectralTransform with the x2 nearest upsample (upsample=True).
"""
import torch.nn as nn

from .ffc import _FFCExec, layer_call
from .spectral_transform import SpectralTransform


class FFCTranspose(_FFCExec, nn.Module):
    def __init__(self, in_channels: int, out_channels: int, kernel_size: int,
                 ratio_gin: float, ratio_gout: float, stride: int = 1, padding: int = 0,
                 dilation: int = 1, groups: int = 1, bias: bool = False,
                 enable_lfu: bool = True, out_padding: int = 0, num_classes: int = 1):
        super().__init__()
        assert stride == 1 or stride == 2, "Stride should be 1 or 2."
        self._ffc_ctor = ["FFCTranspose", dict(in_channels=in_channels, out_channels=out_channels,
                                               kernel_size=kernel_size, ratio_gin=ratio_gin, ratio_gout=ratio_gout,
                                               stride=stride, padding=padding, dilation=dilation, groups=groups,
                                               bias=bias, enable_lfu=enable_lfu, out_padding=out_padding,
                                               num_classes=num_classes)]
        self.stride = stride
        in_cg = int(in_channels * ratio_gin)
        in_cl = int(in_channels - in_cg)
        out_cg = int(out_channels * ratio_gout)
        out_cl = int(out_channels - out_cg)
        self.ratio_gin = ratio_gin
        self.ratio_gout = ratio_gout
        self.convl2l = self.convtransp2d(in_cl == 0 or out_cl == 0, in_cl, out_cl, kernel_size, stride, padding,
                                         output_padding=out_padding, groups=groups, bias=bias, dilation=dilation)
        self.convl2g = self.convtransp2d(in_cl == 0 or out_cg == 0, in_cl, out_cg, kernel_size, stride, padding,
                                         output_padding=out_padding, groups=groups, bias=bias, dilation=dilation)
        self.convg2l = self.convtransp2d(in_cg == 0 or out_cl == 0, in_cg, out_cl, kernel_size, stride, padding,
                                         output_padding=out_padding, groups=groups, bias=bias, dilation=dilation)
        module = nn.Identity if in_cg == 0 or out_cg == 0 else SpectralTransform
        self.convg2g = module(in_cg, out_cg, stride, 1 if groups == 1 else groups // 2, enable_lfu, True,
                              num_classes)

    def convtransp2d(self, condition: bool, in_ch: int, out_ch: int, kernel_size: int,
                     stride: int, padding: int, output_padding: int, groups: int, bias: int, dilation: int):
        if condition:
            return nn.Identity(in_ch, out_ch, kernel_size, stride, padding, dilation, groups, bias)
        return nn.ConvTranspose2d(in_ch, out_ch, kernel_size, stride, padding, output_padding=output_padding,
                                  groups=groups, bias=bias, dilation=dilation)

    def forward(self, x, y=None):
        return layer_call(self, self, x, y)
