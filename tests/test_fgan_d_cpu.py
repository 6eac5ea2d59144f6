"""CPU checks for the fgan128 Discriminator (fgan128_complete.py:525-562) and the training helpers
(no GPU): the state_dict is the reference's (torch.nn modules built per those lines), every conv's
adjoint (data gradient) and the fc have plans, and the product path refuses CPU tensors (no
fallback)."""
import pytest
import torch
import torch.nn as nn

import fastfourierconvolution_amd as F
from fastfourierconvolution_amd import _plan
from fastfourierconvolution_amd._autograd import adjoint_seg
from fastfourierconvolution_amd._lib import FFCError
from fastfourierconvolution_amd.training import hinge_loss_dis, hinge_loss_gen


def test_state_dict_matches_reference_layout():
    D = F.Discriminator()
    ref = {}
    for i, (cin, cout, k, s) in enumerate(F.Discriminator.CONVS, 1):
        m = nn.utils.spectral_norm(nn.Conv2d(cin, cout, k, stride=s, padding=(1, 1)))
        ref.update({f"conv{i}.{n}": t.shape for n, t in m.state_dict().items()})
    ref.update({f"fc.{n}": t.shape for n, t in nn.utils.spectral_norm(nn.Linear(4 * 4 * 512, 1)).state_dict().items()})
    got = {k: v.shape for k, v in D.state_dict().items()}
    assert got == ref
    plain = {f"conv{i}.{n}" for i in range(1, 10) for n in ("weight", "bias")} | {"fc.weight", "fc.bias"}
    assert set(F.Discriminator(sn=False).state_dict()) == plain
    assert F.FGanDiscriminator is F.Discriminator


def test_every_layer_plans_forward_and_adjoint():
    side = 128
    for cin, cout, k, s in F.Discriminator.CONVS:
        sg = _plan.Seg("conv", cin, side, side, k, s, 1)
        plan = _plan.plan_job(64, cout, (sg,))
        OH, OW = _plan.seg_out(sg)
        assert (plan.OH, plan.OW) == (OH, OW) == (side // s, side // s)
        adj = adjoint_seg(sg, cout, OH, OW)
        assert _plan.seg_out(adj) == (side, side)
        _plan.plan_job(64, cin, (adj,))
        side //= s
    assert side == 4
    _plan.plan_job(64, 1, (_plan.Seg("pw", 8192, 1, 1),))
    _plan.plan_job(64, 8192, (adjoint_seg(_plan.Seg("pw", 8192, 1, 1), 1, 1, 1),))


def test_cpu_tensor_refused():
    D = F.Discriminator()
    with pytest.raises(FFCError):
        D(torch.zeros(1, 3, 128, 128))


def test_hinge_losses_shapes():
    with pytest.raises(AssertionError):
        hinge_loss_dis(torch.zeros(2, 1), torch.zeros(3, 1))
    assert hinge_loss_gen(torch.tensor([[1.0], [3.0]])).item() == -2.0
