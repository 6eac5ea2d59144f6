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
