"""Deterministic parameter generator shared by ``gen_golden.py`` and the tests.

The golden fixtures do not store weights (the FFC-DCGAN generator alone has
~3M parameters).  Instead ``manifest.json`` records, per ``state_dict`` key, a
shape and a distribution; every consumer regenerates the identical float32
tensor from ``(seed, key)`` with numpy's PCG64, which is bit-stable across
machines for a given numpy major version.

Key names are the reference's own ``state_dict`` names
(/root/reference/layers/ffc/*.py module attribute names), so the same spec
drives the reference (fixture generation), the oracle and the HIP drop-in.
"""
from __future__ import annotations

import zlib

import numpy as np


def key_rng(seed: int, key: str) -> np.random.Generator:
    return np.random.default_rng(np.random.SeedSequence([int(seed), zlib.crc32(key.encode())]))


def make_array(seed: int, key: str, spec) -> np.ndarray:
    """spec = [shape, dist, a, b, dtype]; dist in {normal(mean=a,std=b), uniform(lo=a,hi=b), const(a)}."""
    shape, dist, a, b, dtype = spec
    shape = tuple(int(s) for s in shape)
    if dist == "const":
        arr = np.full(shape, a, dtype=np.float64)
    elif dist == "normal":
        arr = key_rng(seed, key).normal(a, b, size=shape)
    elif dist == "uniform":
        arr = key_rng(seed, key).uniform(a, b, size=shape)
    else:
        raise ValueError(dist)
    return arr.astype(dtype)


def make_state(seed: int, specs: dict) -> dict:
    return {k: make_array(seed, k, s) for k, s in specs.items()}


def input_array(seed: int, name: str, shape) -> np.ndarray:
    return key_rng(seed, "input:" + name).normal(0.0, 1.0, size=tuple(shape)).astype(np.float32)
