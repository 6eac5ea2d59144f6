"""MI355X-native Fast Fourier Convolution: drop-in for the reference's ``layers`` FFC surface.

    from fastfourierconvolution_amd import *      # instead of  `from layers import *`

exports FourierUnitSN, SELayer, SpectralTransform, FFC, FFCTranspose, FFC_BN_ACT, SNFFC, SNFFCTranspose
(layers/snffc), Resizer,
Print, debug_print, NoiseInjection (the names layers/__init__.py:2-18 exports for this path)
plus the restated callers FFCModel / FFCGenerator / FFCDiscriminator / FGenerator and Discriminator (fgan128).  All compute runs in
the gfx950 HIP library libffc_amd.so (include/ffc_amd.h); there is no CPU fallback.
"""
from . import ops  # noqa: F401  (registers the torch.ops.ffc.* custom ops)
from .config import Config
from .ffc import (FFC, FFC_BN_ACT, SNFFC, FFCTranspose, FourierUnitSN, SELayer, SNFFCTranspose, SpectralTransform,
                  set_mix_precision, spectral_norm_ffc)
from .layers_misc import NoiseInjection, Print, Resizer, debug_print
from .models import Discriminator, FFCDiscriminator, FFCGenerator, FFCModel, FGanDiscriminator, FGenerator

__all__ = ["FourierUnitSN", "SELayer", "SpectralTransform", "FFC", "FFCTranspose", "FFC_BN_ACT", "SNFFC",
           "SNFFCTranspose", "spectral_norm_ffc", "set_mix_precision", "Resizer",
           "Print", "debug_print", "NoiseInjection", "FFCModel", "FFCGenerator", "FFCDiscriminator", "FGenerator",
           "Discriminator", "FGanDiscriminator", "Config"]
