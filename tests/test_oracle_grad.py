"""Pin the oracle's gradients (torch autograd through oracle/ffc_oracle.py in fp64) against the
gradients the REFERENCE computes with autograd (tests/golden/gen_golden_grad.py).  CPU only.
These are the checker for the HIP training path (tests/test_gpu_train.py)."""
import pytest
import torch

from conftest import grad_arrays, grad_cases, load_case
from oracle.ffc_oracle import grad_case, normwise_err

CASES = grad_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_grads_match_reference(case):
    state, inputs, data = load_case(case)
    cots = grad_arrays(data, "cot.")
    gin, gpar = grad_case(case, state, inputs, cots)
    want = set(case["grads"])
    got = {"gin." + k for k in gin} | {"gpar." + k for k in gpar}
    assert want <= got, want - got
    # reference fixtures are fp32 CPU autograd; the oracle runs fp64
    for k in case["grads"]:
        g = gin[k[4:]] if k.startswith("gin.") else gpar[k[5:]]
        err = normwise_err(g, torch.from_numpy(data[k]))
        assert err < 2e-5, (k, err)
