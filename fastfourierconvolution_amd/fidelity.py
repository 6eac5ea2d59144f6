"""The evaluation caller of the generators: how torch_fidelity drives a
generator when the reference scripts compute FID / IS (fgan_complete.py:416-418 wraps ``G`` in
``GenerativeModelModuleWrapper(G, z_size, z_type, 0)``).

Only the generator side is restated: sample noise, run the generator batch by batch, hand the
fakes on.  The feature extractor (Inception weights fetched by URL) and the metrics are out of
scope (tier framing: no network, not on the hot path).

  * ``random_normal``      torch_fidelity/noise.py:8-9      (numpy RandomState.randn -> float32)
  * ``GenerativeModelModuleWrapper``  torch_fidelity/generative_model_modulewrapper.py:10-68
                           (argument checks, eval mode, optional .cuda()).  torch_fidelity itself
                           passes the 2-D noise (B, z_size) through unchanged; ``FFCGenerator``
                           takes 4-D noise (B, nz, 1, 1) (models/ffc_generator.py:30), so this
                           wrapper has an explicit ``noise_4d`` argument (default: True exactly
                           for ``FFCGenerator`` instances) -- an extension, not reference behaviour
  * ``generate_batches``   torch_fidelity/utils.py:160-208 without the feature extractor: batches
                           of ``batch_size`` (default 64, defaults.py:5), RandomState(rng_seed)
                           (default 2020, defaults.py:56), ``torch.no_grad()``, the last batch ragged
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

__all__ = ["random_normal", "GenerativeModelModuleWrapper", "generate_batches"]

DEFAULT_BATCH_SIZE = 64     # torch_fidelity/defaults.py:5
DEFAULT_RNG_SEED = 2020     # torch_fidelity/defaults.py:56


def random_normal(rng: np.random.RandomState, shape) -> torch.Tensor:
    """torch_fidelity/noise.py:8-9"""
    return torch.from_numpy(rng.randn(*shape)).float()


NOISE_SOURCES = {"normal": random_normal}


class GenerativeModelModuleWrapper(nn.Module):
    """torch_fidelity/generative_model_modulewrapper.py:10-68 for the FFC generators.  Raises
    ValueError where torch_fidelity's ``vassert`` raises.  Only the "normal" noise source is on the
    reference's path (fgan_complete.py passes ``args.z_type`` = "normal")."""

    def __init__(self, module, z_size, z_type="normal", num_classes=0, make_eval=True, cuda=None, noise_4d=None):
        super().__init__()
        if not isinstance(module, nn.Module):
            raise ValueError("Not an instance of torch.nn.Module")
        if type(z_size) is not int or z_size <= 0:
            raise ValueError("z_size must be a positive integer")
        if z_type not in NOISE_SOURCES:
            raise ValueError(f"z_type={z_type} not implemented")
        if type(num_classes) is not int or num_classes != 0:
            raise ValueError("the FFC generators are unconditional: num_classes must be 0")
        self.module = module
        if make_eval:
            self.module.eval()
        if cuda is not None:
            self.module = self.module.cuda() if cuda else self.module.cpu()
        self.z_size, self.z_type, self.num_classes = z_size, z_type, num_classes
        # FFCGenerator's first layer is a ConvTranspose2d on a 1x1 input: it takes (B, nz, 1, 1);
        # torch_fidelity proper would hand it the 2-D noise unchanged (noise_4d=False)
        if noise_4d is None:
            from .models import FFCGenerator
            noise_4d = isinstance(module, FFCGenerator)
        self._noise_4d = bool(noise_4d)

    def forward(self, z):
        if self._noise_4d and z.dim() == 2:
            z = z.reshape(z.shape[0], z.shape[1], 1, 1)
        return self.module(z)


def generate_batches(gen_model: GenerativeModelModuleWrapper, num_samples: int,
                     batch_size: int = DEFAULT_BATCH_SIZE, cuda: bool = True, rng_seed: int = DEFAULT_RNG_SEED):
    """Yield the generator's fakes batch by batch, as torch_fidelity/utils.py:160-208 feeds them
    to its feature extractor."""
    if not isinstance(gen_model, GenerativeModelModuleWrapper):
        raise ValueError("Input can only be a GenerativeModel instance")
    if batch_size > num_samples:
        batch_size = num_samples
    rng = np.random.RandomState(rng_seed)
    if cuda:
        gen_model.cuda()
    with torch.no_grad():
        for start in range(0, num_samples, batch_size):
            sz = min(start + batch_size, num_samples) - start
            noise = NOISE_SOURCES[gen_model.z_type](rng, (sz, gen_model.z_size))
            if cuda:
                noise = noise.cuda(non_blocking=True)
            yield gen_model(noise)
