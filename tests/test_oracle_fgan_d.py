"""Pins the oracle's fgan128 Discriminator and hinge losses (oracle/ffc_oracle.py) against torch.nn
modules built per fgan128_complete.py:525-585 (Conv2d / Linear wrapped in torch.nn.utils.spectral_norm,
LeakyReLU(0.1), no output activation): forward, one power iteration per train-mode call, and the
gradients of the weight_orig / bias parameters and of the input (fp64, CPU).  The module under
test here is torch itself (the reference's dependency); the script cannot be imported (it runs
main() at import), so this is the pin for the restatement."""
import torch
import torch.nn as nn

from oracle.ffc_oracle import FGAN_D_CONVS, fgan128_discriminator, hinge_loss_dis, hinge_loss_gen, normwise_err


class _TorchD(nn.Module):
    def __init__(self, mg):
        super().__init__()
        self.mg = mg
        for i, (cin, cout, k, s) in enumerate(FGAN_D_CONVS, 1):
            setattr(self, f"conv{i}", nn.utils.spectral_norm(nn.Conv2d(cin, cout, k, stride=s, padding=(1, 1))))
        self.fc = nn.utils.spectral_norm(nn.Linear(mg * mg * 512, 1))
        self.act = nn.LeakyReLU(0.1)

    def forward(self, x):
        m = x
        for i in range(1, 10):
            m = self.act(getattr(self, f"conv{i}")(m))
        return self.fc(m.view(-1, self.mg * self.mg * 512))


def test_oracle_discriminator_matches_torch_modules():
    torch.manual_seed(0)
    mg = 1                                   # 32x32 input: the same layer stack at 1/16 of the pixels
    D = _TorchD(mg).double().train()
    sd = {k: v.clone() for k, v in D.state_dict().items()}
    x = torch.randn(3, 3, 32 * mg, 32 * mg, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    xo = x.clone().requires_grad_(True)
    params = [k for k in sd if k.endswith(("weight_orig", "bias"))]
    for k in params:
        sd[k].requires_grad_(True)
    for step in range(2):                    # two calls: the second starts from the updated u / v
        ref = D(xr)
        got = fgan128_discriminator(xo, sd, True, mg=mg)
        assert normwise_err(got.detach(), ref.detach()) < 1e-12
        for k in sd:
            if k.endswith(("weight_u", "weight_v")):
                assert torch.allclose(sd[k], D.state_dict()[k], rtol=1e-12, atol=1e-14), k
    fake = torch.randn(3, 1, dtype=torch.float64)
    (hinge_loss_gen(ref) + hinge_loss_dis(fake, ref)).backward()
    (hinge_loss_gen(got) + hinge_loss_dis(fake, got)).backward()
    assert normwise_err(xo.grad, xr.grad) < 1e-12
    named = dict(D.named_parameters())
    for k in params:
        assert normwise_err(sd[k].grad, named[k].grad) < 1e-12, k


def test_hinge_losses():
    f = torch.tensor([[0.5], [-2.0], [1.5]])
    r = torch.tensor([[2.0], [0.25], [-1.0]])
    assert torch.isclose(hinge_loss_gen(f), -f.mean())
    exp = torch.tensor([0.0, 0.75, 2.0]).mean() + torch.tensor([1.5, 0.0, 2.5]).mean()
    assert torch.isclose(hinge_loss_dis(f, r), exp)
