from .ffc import FFC
from .ffc_bn_act import FFC_BN_ACT
from .ffc_transpose import FFCTranspose
from .fourier_unity import FourierUnitSN
from .spectral_transform import SELayer, SpectralTransform

__all__ = ["FFC", "FFC_BN_ACT", "FFCTranspose", "FourierUnitSN", "SELayer", "SpectralTransform"]
