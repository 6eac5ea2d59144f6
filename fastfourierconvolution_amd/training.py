"""The fgan128 training iteration (fgan128_complete.py:666-703) over the HIP layers: the reference's
hinge losses and its generator / discriminator updates, restated as functions so a caller (or a
hipGraph capture, bench.py --workload fgan128train) can run the same step the reference's loop runs.

Every convolution, Fourier unit, BatchNorm, activation, NoiseInjection and Linear of G and D runs
on libffc_amd.so (forward and backward); the hinge losses (a few ops on a (B, 1) tensor), the
spectral-norm power iteration (torch.nn.utils.spectral_norm's own hook, on the GPU) and the
optimizer are torch's, as in the reference."""
import torch
import torch.nn.functional as tF


def hinge_loss_dis(fake, real):
    """fgan128_complete.py:566-572"""
    assert fake.dim() == 2 and fake.shape[1] == 1 and real.shape == fake.shape, f"{fake.shape} {real.shape}"
    return tF.relu(1.0 - real).mean() + tF.relu(1.0 + fake).mean()


def hinge_loss_gen(fake):
    """fgan128_complete.py:581-585"""
    assert fake.dim() == 2 and fake.shape[1] == 1, f"{fake.shape}"
    return -fake.mean()


def generator_step(G, D, optim_G, optim_D, z, noises=None):
    """fgan128_complete.py:680-690: G trainable, D frozen; loss_G = hinge_loss_gen(D(G(z))), backward
    through D into G, optim_G.step().  ``noises``: explicit NoiseInjection noise (FGenerator.forward);
    None draws it on the GPU as the reference does."""
    G.requires_grad_(True)
    D.requires_grad_(False)
    optim_D.zero_grad()
    optim_G.zero_grad()
    fake = G(z, noises)
    loss_G = hinge_loss_gen(D(fake))
    loss_G.backward()
    optim_G.step()
    return loss_G


def discriminator_step(G, D, optim_G, optim_D, z, real, noises=None):
    """fgan128_complete.py:692-703 (one of num_dis_updates): G frozen (its forward takes the
    no-grad inference path), loss_D = hinge_loss_dis(D(G(z)), D(real)) in the reference's call order,
    backward into D, optim_D.step()."""
    G.requires_grad_(False)
    D.requires_grad_(True)
    optim_D.zero_grad()
    optim_G.zero_grad()
    fake = G(z, noises)
    output_dg = D(fake)
    output_dreal = D(real)
    loss_D = hinge_loss_dis(output_dg, output_dreal)
    loss_D.backward()
    optim_D.step()
    return loss_D


def train_iteration(G, D, optim_G, optim_D, z_g, z_d, real, num_dis_updates=1):
    """one iteration of the reference's loop body (:680-703) without its logging / LR schedule:
    a generator update, then ``num_dis_updates`` discriminator updates (z_d: one z per update)"""
    loss_G = generator_step(G, D, optim_G, optim_D, z_g)
    zs = z_d if isinstance(z_d, (list, tuple)) else [z_d]
    assert len(zs) == num_dis_updates
    loss_D = None
    for z in zs:
        loss_D = discriminator_step(G, D, optim_G, optim_D, z, real)
    return loss_G, loss_D
