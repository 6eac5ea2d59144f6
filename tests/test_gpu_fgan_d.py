"""fgan128 Discriminator (fgan128_complete.py:525-562) and the training iteration it takes part in
(:680-703, fastfourierconvolution_amd/training.py) on the HIP path, against the fp64 oracle
(oracle/ffc_oracle.py fgan128_discriminator / fgan128_generator, pinned by tests/test_oracle_fgan_d.py).

LeakyReLU(0.1) makes D piecewise linear: the oracle's backward takes the active sets from the HIP
path's own layer outputs (_KinkF, as tests/test_gpu_train.py does), so both sides differentiate the
same piece.  Tolerance: normwise 1e-4."""
import contextlib
import io

import pytest
import torch

import oracle.ffc_oracle as O
from oracle.ffc_oracle import (fgan128_discriminator, fgan128_generator, hinge_loss_dis, hinge_loss_gen,
                               normwise_err)

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _d_state64(D):
    sd = {k: v.detach().cpu().double().clone() for k, v in D.state_dict().items()}
    for k in sd:
        if k.endswith(("weight_orig", "bias")):
            sd[k].requires_grad_(True)
    return sd


def _oracle_d(xs, sd, recorded, sn=True):
    """oracle D on each of ``xs`` in order (one power iteration each), active sets from ``recorded``"""
    from test_gpu_train import _KinkF
    old = O.F
    O.F = _KinkF([], [r.double() for r in recorded])
    try:
        return [fgan128_discriminator(x, sd, True, sn=sn) for x in xs]
    finally:
        O.F = old


def _check_d_grads(D, sd, tag):
    errs = {}
    for k, p in D.named_parameters():
        assert p.grad is not None and sd[k].grad is not None, k
        errs[k] = normwise_err(p.grad.cpu(), sd[k].grad)
    print(f"{tag}: {len(errs)} D gradients, worst {max(errs.values()):.2e}")
    assert len(errs) == 20
    bad = {k: e for k, e in errs.items() if not e <= TOL}
    assert not bad, bad


@pytest.mark.parametrize("B", [2, 3])
def test_discriminator_fwd_bwd_vs_oracle(B):
    """D forward, input gradient and every weight_orig / bias gradient (spectral norm, one power
    iteration) vs the fp64 oracle; u / v after the call match the oracle's"""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _autograd as ag
    torch.manual_seed(B)
    D = F.Discriminator().cuda().train()
    sd = _d_state64(D)
    gen = torch.Generator().manual_seed(10 + B)
    x = torch.randn((B, 3, 128, 128), generator=gen)
    c = torch.randn((B, 1), generator=gen)
    xg = x.cuda().requires_grad_(True)
    ag.RECORD = []
    try:
        out = D(xg)
        recorded = [t.cpu() for t in ag.RECORD]
    finally:
        ag.RECORD = None
    assert tuple(out.shape) == (B, 1) and len(recorded) == 9
    (out * c.cuda()).sum().backward()
    xo = x.double().requires_grad_(True)
    (ref,) = _oracle_d([xo], sd, recorded)
    (ref * c.double()).sum().backward()
    e_out = normwise_err(out.detach().cpu(), ref.detach())
    e_in = normwise_err(xg.grad.cpu(), xo.grad)
    print(f"D B={B}: out {e_out:.2e}, input grad {e_in:.2e}")
    assert e_out <= TOL and e_in <= TOL
    for k, v in D.state_dict().items():
        if k.endswith(("weight_u", "weight_v")):
            assert normwise_err(v.cpu(), sd[k]) <= 1e-5, k
    _check_d_grads(D, sd, f"D B={B}")


def test_discriminator_eval_no_sn():
    """sn=False, eval mode, no autograd: the forward alone (the inference path of the same kernels)"""
    import fastfourierconvolution_amd as F
    torch.manual_seed(5)
    D = F.Discriminator(sn=False).cuda().eval()
    sd = {k: v.detach().cpu().double() for k, v in D.state_dict().items()}
    x = torch.randn((4, 3, 128, 128), generator=torch.Generator().manual_seed(6))
    with torch.no_grad():
        out = D(x.cuda()).cpu()
        ref = fgan128_discriminator(x.double(), sd, False, sn=False)
    assert normwise_err(out, ref) <= TOL


def _models(seed):
    import fastfourierconvolution_amd as F
    from test_gpu_fgan_train import _randomize
    torch.manual_seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FGenerator(128)
    _randomize(G, torch.Generator().manual_seed(seed))
    D = F.Discriminator()
    return G, D


def _noises(B, gen):
    return [(torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen),
             torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen)) for n in (2, 3, 4, 5, 6)]


def _cuda(noises):
    return [(a.cuda(), b.cuda()) for a, b in noises]


def _g_state64(G):
    return {k: (v.detach().cpu().double().clone() if v.is_floating_point() else v.detach().cpu().clone())
            for k, v in G.state_dict().items()}


def test_generator_step_vs_oracle():
    """training.generator_step (:680-690): loss_G = hinge_loss_gen(D(G(z))) vs the fp64 oracle; every
    live G parameter gets a finite gradient, D (frozen) none; the step moves G and not D"""
    from fastfourierconvolution_amd.training import generator_step
    G, D = _models(21)
    sdg, sdd = _g_state64(G), _d_state64(D)
    G, D = G.cuda().train(), D.cuda().train()
    gen = torch.Generator().manual_seed(22)
    B = 2
    z = torch.randn((B, 128), generator=gen)
    nz = _noises(B, gen)
    oG = torch.optim.AdamW(G.parameters(), lr=2e-4, betas=(0.5, 0.999))
    oD = torch.optim.AdamW(D.parameters(), lr=2e-4, betas=(0.5, 0.999))
    d0 = {k: v.detach().clone() for k, v in D.state_dict().items() if not k.endswith(("weight_u", "weight_v"))}
    g0 = {k: v.detach().clone() for k, v in G.named_parameters()}
    loss = generator_step(G, D, oG, oD, z.cuda(), _cuda(nz))
    with torch.no_grad():
        fake = fgan128_generator(z.double(), sdg, True, [(a.double(), b.double()) for a, b in nz])
        ref = hinge_loss_gen(fgan128_discriminator(fake, sdd, True))
    rel = abs(loss.item() - ref.item()) / abs(ref.item())
    print(f"generator_step B={B}: loss_G {loss.item():.6f} rel err {rel:.2e}")
    assert rel <= TOL
    assert all(p.grad is None for p in D.parameters())
    live = [k for k, p in G.named_parameters() if ".lfu." not in k]
    bad = [k for k in live if dict(G.named_parameters())[k].grad is None or
           not torch.isfinite(dict(G.named_parameters())[k].grad).all()]
    assert not bad, bad[:5]
    assert any(not torch.equal(g0[k], p) for k, p in G.named_parameters())
    for k, v in d0.items():
        assert torch.equal(v, D.state_dict()[k]), k


def test_discriminator_step_vs_oracle():
    """training.discriminator_step (:692-703): G's no-grad forward (explicit noise) vs the oracle, loss_D
    and every D gradient vs the fp64 oracle run on the HIP path's own fake (two power iterations: D(fake),
    then D(real), in the reference's order); G receives no gradient"""
    from fastfourierconvolution_amd import _autograd as ag
    from fastfourierconvolution_amd.training import discriminator_step
    G, D = _models(31)
    sdg, sdd = _g_state64(G), _d_state64(D)
    G, D = G.cuda().train(), D.cuda().train()
    gen = torch.Generator().manual_seed(32)
    B = 2
    z = torch.randn((B, 128), generator=gen)
    nz = _noises(B, gen)
    real = torch.rand((B, 3, 128, 128), generator=gen) * 2 - 1
    oG = torch.optim.AdamW(G.parameters(), lr=0.0)
    oD = torch.optim.AdamW(D.parameters(), lr=0.0, weight_decay=0.0)
    with torch.no_grad():
        fake_hip = G(z.cuda(), _cuda(nz)).cpu()     # train-mode BN: batch statistics, same output again
        fake_ref = fgan128_generator(z.double(), sdg, True, [(a.double(), b.double()) for a, b in nz])
    e_fake = normwise_err(fake_hip, fake_ref)
    ag.RECORD = []
    try:
        loss = discriminator_step(G, D, oG, oD, z.cuda(), real.cuda(), _cuda(nz))
        recorded = [t.cpu() for t in ag.RECORD[-18:]]
    finally:
        ag.RECORD = None
    dg, dr = _oracle_d([fake_hip.double(), real.double()], sdd, recorded)
    ref = hinge_loss_dis(dg, dr)
    ref.backward()
    rel = abs(loss.item() - ref.item()) / abs(ref.item())
    print(f"discriminator_step B={B}: fake {e_fake:.2e}, loss_D {loss.item():.6f} rel err {rel:.2e}")
    assert e_fake <= TOL and rel <= TOL
    assert all(p.grad is None for p in G.parameters())
    _check_d_grads(D, sdd, "discriminator_step")
