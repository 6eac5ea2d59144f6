"""Shared test helpers.  ``-m gpu`` tests need an MI355X; everything else runs on CPU."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def load_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_cases():
    return load_manifest()["cases"]


def load_case(case):
    """-> (state dict of numpy arrays incl. eval-mode running stats, inputs, fixture arrays)."""
    from fixture_weights import make_state
    data = np.load(os.path.join(GOLDEN, case["name"] + ".npz"))
    state = make_state(case["seed"], case["specs"])
    for k in data.files:
        if k.startswith("before."):
            state[k[len("before."):]] = data[k]
    inputs = {k[len("in."):]: data[k] for k in data.files if k.startswith("in.")}
    return state, inputs, data


@pytest.fixture(scope="session")
def manifest():
    return load_manifest()


def build_dropin(case, state, device="cuda"):
    """the drop-in module for a golden case, loaded with the case's state (numpy arrays)."""
    import contextlib
    import io

    import torch
    import torch.nn as nn

    import fastfourierconvolution_amd as F
    kw = dict(case["ctor"])
    for k in ("norm_layer", "activation_layer"):
        if k in kw:
            kw[k] = getattr(nn, kw[k])
    with contextlib.redirect_stdout(io.StringIO()):
        mod = getattr(F, case["kind"])(**kw)
    mod.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    mod = mod.to(device)
    mod.train(case["mode"] == "train")
    return mod


def call_dropin(case, mod, inputs):
    """run a case's forward; -> dict like the fixture outputs (out / out_l / out_g)."""
    import torch
    t = {k: torch.from_numpy(v).cuda() for k, v in inputs.items()}
    with torch.no_grad():
        if case["kind"] == "FGenerator":
            noises = [(t.get(f"noise{n}_l"), t.get(f"noise{n}_g")) for n in (2, 3, 4, 5, 6)]
            return {"out": mod.forward_float(t["z"], noises if mod.training else None)}
        if case["kind"] in ("FFC_BN_ACT", "SNFFC"):
            x = (t["x_l"], t["x_g"]) if "x_l" in t else t["x"]
            ol, og = mod(x)
            res = {}
            if isinstance(ol, torch.Tensor):
                res["out_l"] = ol
            if isinstance(og, torch.Tensor):
                res["out_g"] = og
            return res
        return {"out": mod(next(iter(t.values())))}


def grad_cases():
    """gradient fixtures (tests/golden/gen_golden_grad.py, BASELINE config 3 fwd + bwd)"""
    with open(os.path.join(GOLDEN, "manifest_grad.json")) as f:
        return json.load(f)["cases"]


def grad_arrays(data, prefix):
    return {k[len(prefix):]: data[k] for k in data.files if k.startswith(prefix)}
