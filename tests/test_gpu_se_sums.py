"""The SE gate of a SpectralTransform on large planes from the plane sums that the previous
layer's BN-apply pass writes while it stores y (ffc_bn_act_apply_batch plane_sum +
ffc_se_gate_sums), against the second read of y (se_mean_kernel + se_fc_kernel): the fgan128
generator (fgan128_complete.py:440-520; SELayer spectral_transform.py:12-28) in train mode with
NoiseInjection noise.  The two differ only in the order the means are summed (about one ulp of a
mean), which the later layers carry through their batch-statistics BNs (B = 4: 1.3e-6 at the
output): outputs within 1e-5 normwise, and the sums path must actually be taken.  Both paths are
checked against the fp64 oracle layer by layer in test_gpu_timed_shapes.py."""
import pytest
import torch

from oracle.ffc_oracle import normwise_err
from test_gpu_timed_shapes import _fgan, _gpu_layers, _noises

pytestmark = pytest.mark.gpu


def _run(G, z, noises, on, monkeypatch):
    from fastfourierconvolution_amd import _runtime as rt
    used = []
    orig = rt.plane_sums_for

    def spy(x):
        r = orig(x)
        used.append(r is not None)
        return r

    monkeypatch.setattr(rt, "SE_SUMS", on)
    monkeypatch.setattr(rt, "plane_sums_for", spy)
    outs = _gpu_layers(G, z, noises)
    torch.cuda.synchronize()
    monkeypatch.undo()
    return outs, used


@pytest.mark.parametrize("B", [4, 16])
def test_se_gate_from_plane_sums_matches_second_read(B, monkeypatch):
    G = _fgan(False, "fp32").cuda().train()
    gen = torch.Generator().manual_seed(B)
    z = torch.randn((B, 128), generator=gen).cuda()
    noises = [(a.cuda(), b.cuda()) for a, b in _noises(B, gen)]
    ref, used_off = _run(G, z, noises, False, monkeypatch)
    got, used_on = _run(G, z, noises, True, monkeypatch)
    assert not any(used_off)
    assert sum(used_on) >= 2, used_on   # the large-plane layers take their means from the sums
    for g, r in zip(got, ref):
        gs = g if isinstance(g, tuple) else (g,)
        rs = r if isinstance(r, tuple) else (r,)
        for a, b in zip(gs, rs):
            assert normwise_err(a.double().cpu(), b.double().cpu()) <= 1e-5
