"""Sharded training with SyncBN through the HIP training path: a 2-way sample
shard (gloo carries the BN moments and the backward sums; both ranks on cuda:0 -- RCCL needs
one GPU per rank, which the 1-GPU test box does not have) of FFCGenerator's forward + backward
equals the single-process global-batch step: input gradients (concatenated shards), parameter
gradients (summed over the ranks, what a data-parallel wrapper all-reduces), outputs and
running statistics.  torch.nn.SyncBatchNorm semantics: dx from the all-reduced {sum g, sum g*x},
dgamma / dbeta from each rank's own sums (ffc_bn_bwd_sums / _coeff / _apply)."""
import contextlib
import io
import os
import socket

import numpy as np
import pytest
import torch

from oracle.ffc_oracle import normwise_err

pytestmark = pytest.mark.gpu
NZ, NC, NGF, B = 16, 3, 8, 6


def _gen(seed=31):
    import fastfourierconvolution_amd as F
    torch.manual_seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        g = F.FFCGenerator(NZ, NC, NGF)
    for m in g.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    return g


def _inputs():
    gen = torch.Generator().manual_seed(8)
    z = torch.randn((B, NZ, 1, 1), generator=gen)
    cot = torch.randn((B, NC, 64, 64), generator=gen)
    return z, cot


def _step(g, z, cot):
    z = z.cuda().requires_grad_(True)
    out = g(z)
    (out * cot.cuda()).sum().backward()
    torch.cuda.synchronize()
    # parameters outside the path (unused lfu.*, zero-element SE Linear) have no gradient
    return out.detach().cpu(), z.grad.detach().cpu(), {n: p.grad.detach().cpu() for n, p in g.named_parameters()
                                                       if p.grad is not None}


def _worker(rank, port, out_dir):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import fastfourierconvolution_amd.distributed as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    g = _gen().cuda().train()
    D.broadcast_module(g)
    D.enable_sync_bn()
    z, cot = _inputs()
    lo, hi = rank * B // 2, (rank + 1) * B // 2
    out, dz, grads = _step(g, z[lo:hi], cot[lo:hi])
    torch.save({"out": out, "dz": dz, "grads": grads, "sd": {k: v.cpu() for k, v in g.state_dict().items()}},
               os.path.join(out_dir, f"r{rank}.pt"))
    D.disable_sync_bn()
    dist.destroy_process_group()


def test_sharded_syncbn_training_matches_global_batch(tmp_path):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_worker, args=(port, str(tmp_path)), nprocs=2, join=True)
    g = _gen().cuda().train()
    z, cot = _inputs()
    out, dz, grads = _step(g, z, cot)
    rs = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(2)]
    assert normwise_err(torch.cat([r["out"] for r in rs]), out) <= 1e-5
    assert normwise_err(torch.cat([r["dz"] for r in rs]), dz) <= 1e-4
    assert set(grads) == set(rs[0]["grads"]) == set(rs[1]["grads"]) and len(grads) > 10
    for n, v in grads.items():
        got = rs[0]["grads"][n] + rs[1]["grads"][n]
        assert normwise_err(got, v) <= 1e-4, n
    for k, v in g.state_dict().items():
        if "running" in k:
            np.testing.assert_allclose(rs[0]["sd"][k].numpy(), v.cpu().numpy(), rtol=1e-4, atol=1e-6, err_msg=k)
