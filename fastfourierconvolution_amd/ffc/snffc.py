"""Spectral-norm FFC variants (reference: layers/snffc/snffc.py:12-33, snffc_transpose.py:11-35).

``SNFFC`` is FFC with ``torch.nn.utils.spectral_norm`` on convl2l (always), convg2l / convl2g (when
they are Conv2d) and the Conv2d children of the SpectralTransform (conv1, conv2) -- exactly the
reference's wrapping.  The HIP executor refreshes each normalised weight (one power iteration in
training mode, host-driven PyTorch as in the reference) where the reference's forward would call the
module (_runtime.sn_refresh), so the packed GEMM weights always see W / sigma.

``SNFFCTranspose`` reproduces the reference constructor, including its defect: it wraps
``self.convg2gup``, which FFCTranspose never defines (snffc_transpose.py:28), so construction raises
AttributeError exactly as the reference does.  ``spectral_norm_ffc`` applies the wrapping the
reference intended to any FFC / FFCTranspose stack (BASELINE config 5: the fgan128 generator with
spectral norm on l2l / l2g / g2l and the SpectralTransform conv1 / conv2).
"""
import torch.nn as nn
from torch.nn.utils import spectral_norm

from .ffc import FFC
from .ffc_transpose import FFCTranspose


def _wrap_st_children(st):
    if isinstance(st, nn.Identity):
        return
    for name, module in st.named_children():
        if isinstance(module, (nn.Conv2d, nn.ConvTranspose2d)):
            st._modules[name] = spectral_norm(module)


class SNFFC(FFC):
    def __init__(self, in_channels: int, out_channels: int, kernel_size: int,
                 ratio_gin: float, ratio_gout: float, stride: int = 1, padding: int = 0,
                 dilation: int = 1, groups: int = 1, bias: bool = False, enable_lfu: bool = True,
                 attention: bool = False):
        FFC.__init__(self, in_channels, out_channels, kernel_size, ratio_gin, ratio_gout, stride,
                     padding, dilation, groups, bias, enable_lfu, attention)
        self.convl2l = spectral_norm(self.convl2l)
        self.convg2l = spectral_norm(self.convg2l) if isinstance(self.convg2l, nn.Conv2d) else self.convg2l
        self.convl2g = spectral_norm(self.convl2g) if isinstance(self.convl2g, nn.Conv2d) else self.convl2g
        _wrap_st_children(self.convg2g)


class SNFFCTranspose(FFCTranspose):
    def __init__(self, in_channels: int, out_channels: int, kernel_size: int,
                 ratio_gin: float, ratio_gout: float, stride: int = 1, padding: int = 0,
                 dilation: int = 1, groups: int = 1, bias: bool = False,
                 enable_lfu: bool = True, out_padding: int = 0, attention: bool = False):
        # FFCTranspose's 13th positional parameter is num_classes; the reference passes `attention`
        # there (snffc_transpose.py:18-19)
        FFCTranspose.__init__(self, in_channels, out_channels, kernel_size, ratio_gin, ratio_gout, stride,
                              padding, dilation, groups, bias, enable_lfu, out_padding, attention)
        self.convl2l = spectral_norm(self.convl2l)
        if isinstance(self.convg2l, nn.ConvTranspose2d):
            self.convg2l = spectral_norm(self.convg2l)
        if isinstance(self.convl2g, nn.ConvTranspose2d):
            self.convl2g = spectral_norm(self.convl2g)
        self.convg2gup = spectral_norm(self.convg2gup)   # AttributeError, as in the reference (:28)
        _wrap_st_children(self.convg2g)


def spectral_norm_ffc(model: nn.Module) -> nn.Module:
    """Wrap, in every FFC / FFCTranspose of ``model``, convl2l / convl2g / convg2l (Conv2d or
    ConvTranspose2d) and the SpectralTransform's conv1 / conv2 with spectral_norm (what SNFFC does
    and SNFFCTranspose intends).  Returns ``model``."""
    for m in list(model.modules()):
        if isinstance(m, (FFC, FFCTranspose)):
            for name in ("convl2l", "convl2g", "convg2l"):
                mod = getattr(m, name)
                if isinstance(mod, (nn.Conv2d, nn.ConvTranspose2d)) and not hasattr(mod, "weight_orig"):
                    setattr(m, name, spectral_norm(mod))
            if not isinstance(m.convg2g, nn.Identity):
                for name in ("conv1", "conv2"):
                    mod = getattr(m.convg2g, name)
                    if not hasattr(mod, "weight_orig"):
                        m.convg2g._modules[name] = spectral_norm(mod)
    return model


def set_mix_precision(model: nn.Module, precision: str) -> nn.Module:
    """Spectral mix arithmetic of every FourierUnitSN in ``model``: "fp32" (exact, default) or "fp16"
    (fp16 operands, fp32 accumulation on the f16 MFMA; BASELINE config 5).  Returns ``model``."""
    from .fourier_unity import FourierUnitSN
    if precision not in ("fp32", "fp16"):
        raise ValueError(f"mix precision must be 'fp32' or 'fp16', got {precision!r}")
    for m in model.modules():
        if isinstance(m, FourierUnitSN):
            m.mix_precision = precision
    return model
