from .ffc import FFC
from .ffc_bn_act import FFC_BN_ACT
from .ffc_transpose import FFCTranspose
from .fourier_unity import FourierUnitSN
from .snffc import SNFFC, SNFFCTranspose, set_mix_precision, spectral_norm_ffc
from .spectral_transform import SELayer, SpectralTransform

__all__ = ["FFC", "FFC_BN_ACT", "FFCTranspose", "FourierUnitSN", "SELayer", "SpectralTransform", "SNFFC",
           "SNFFCTranspose", "spectral_norm_ffc", "set_mix_precision"]
