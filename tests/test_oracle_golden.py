"""Pin the oracle (oracle/ffc_oracle.py) against the golden vectors produced by the
reference itself (tests/golden/gen_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from conftest import golden_cases, load_case
from oracle.ffc_oracle import normwise_err, run_fixture_case

CASES = golden_cases()
IDS = [c["name"] for c in CASES]


@pytest.mark.parametrize("case", CASES, ids=IDS)
@pytest.mark.parametrize("fft", ["numpy", "torch"])
def test_oracle_matches_reference(case, fft):
    state, inputs, data = load_case(case)
    # fp64 restatement with the independent FFT; fp32 op-for-op with torch.fft
    dtype = torch.float64 if fft == "numpy" else torch.float32
    out, sd = run_fixture_case(case, state, inputs, dtype=dtype, fft=fft)
    assert sorted("ref." + k for k in out) == case["outputs"]
    tol = 2e-5
    for k, v in out.items():
        err = normwise_err(v, torch.from_numpy(data["ref." + k]))
        assert err < tol, (k, err)
    # train mode: BN running-stat updates match nn.BatchNorm2d
    for k in data.files:
        if k.startswith("after."):
            key = k[len("after."):]
            ref = data[k]
            got = sd[key].numpy()
            if ref.dtype.kind == "i":
                assert int(got) == int(ref), key
            else:
                np.testing.assert_allclose(got, ref, rtol=2e-4, atol=2e-5, err_msg=key)
