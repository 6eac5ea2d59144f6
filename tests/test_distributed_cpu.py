"""N > 1 path on CPU: world_size-2 gloo process groups.

The data path's only exchange is the SyncBN moments all-reduce (fastfourierconvolution_amd/
distributed.py).  These tests run it over gloo with two ranks and check the claims the
multi-GPU bench relies on:
  * shard_range / gather_batch partition and reassemble a (ragged) batch exactly;
  * broadcast_module replicates rank 0's parameters and BN buffers;
  * merge_moments of per-shard raw moments equals the global-batch moments;
  * the FFC generator forward, sharded over 2 ranks with SyncBN (the oracle's batch_norm fed
    merged moments), equals the single-process global-batch forward, running statistics
    included — while the naive (unsynchronised) shard does not.
No GPU is touched: the oracle (test infrastructure) stands in for the kernels here; the same
flow through the HIP kernels is tests/test_gpu_parity.py::test_sharded_syncbn_gpu.
"""
from __future__ import annotations

import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from fastfourierconvolution_amd.distributed import shard_range  # noqa: E402

WORLD = 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, port):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=WORLD)


def _spawn(fn, *args):
    port = _free_port()
    mp.spawn(fn, args=(port,) + args, nprocs=WORLD, join=True)


# --------------------------------------------------------------------------- pure host logic
@pytest.mark.parametrize("B,world", [(0, 2), (1, 2), (5, 2), (256, 8), (7, 3), (512, 8)])
def test_shard_range_partitions(B, world):
    spans = [shard_range(B, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == B
    for (a0, b0), (a1, _) in zip(spans, spans[1:]):
        assert b0 == a1
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def test_shard_range_rejects_bad_rank():
    with pytest.raises(ValueError):
        shard_range(8, 2, 2)


# --------------------------------------------------------------------------- gloo workers
def _w_collectives(rank, port, out_dir):
    _init(rank, port)
    from fastfourierconvolution_amd import distributed as D
    res = {}
    # gather_batch: ragged 5 = 3 + 2
    g = torch.arange(5 * 3, dtype=torch.float32).reshape(5, 3)
    mine = D.shard_batch(g)
    res["gather"] = bool(torch.equal(D.gather_batch(mine, 5), g))
    # broadcast_module: BN buffers and weights
    torch.manual_seed(10 + rank)
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3), torch.nn.BatchNorm2d(4))
    m[1].running_mean.normal_()
    m[1].num_batches_tracked += 3 + rank
    D.broadcast_module(m)
    flat = torch.cat([t.detach().double().flatten() for t in list(m.parameters()) + list(m.buffers())])
    ref = flat.clone()
    dist.broadcast(ref, 0)
    res["broadcast"] = bool(torch.equal(flat, ref))
    # merge_moments == global moments
    torch.manual_seed(0)
    X = torch.randn(6, 5, 4, 4, dtype=torch.float64) * 3 + 1
    xs = D.shard_batch(X)
    mom = torch.stack([torch.full((5,), float(xs.numel() // 5), dtype=torch.float64),
                       xs.sum(dim=(0, 2, 3)), (xs * xs).sum(dim=(0, 2, 3))], dim=1)
    D.merge_moments(mom)
    glob = torch.stack([torch.full((5,), float(X.numel() // 5), dtype=torch.float64),
                        X.sum(dim=(0, 2, 3)), (X * X).sum(dim=(0, 2, 3))], dim=1)
    res["moments"] = float((mom - glob).abs().max() / glob.abs().max())
    torch.save(res, os.path.join(out_dir, f"coll{rank}.pt"))
    dist.destroy_process_group()


def test_gloo_collectives(tmp_path):
    _spawn(_w_collectives, str(tmp_path))
    for r in range(WORLD):
        res = torch.load(tmp_path / f"coll{r}.pt", weights_only=True)
        assert res["gather"] and res["broadcast"], res
        assert res["moments"] < 1e-15, res


def _sync_batch_norm_factory(D):
    """oracle.batch_norm with SyncBN semantics: raw moments of the local shard are merged with
    distributed.merge_moments (what _runtime.bn_scale_shift does between ffc_bn_reduce and
    ffc_bn_finalize), then nn.BatchNorm2d's normalise / running-stat update is applied."""
    def batch_norm(x, sd, prefix, training, momentum=0.1, eps=1e-5):
        w, b = sd[prefix + "weight"], sd[prefix + "bias"]
        rm, rv = sd[prefix + "running_mean"], sd[prefix + "running_var"]
        assert training
        C = x.shape[1]
        xd = x.double()
        mom = torch.stack([torch.full((C,), float(x.numel() // C), dtype=torch.float64),
                           xd.sum(dim=(0, 2, 3)), (xd * xd).sum(dim=(0, 2, 3))], dim=1)
        D.merge_moments(mom)
        n = mom[:, 0]
        mean = mom[:, 1] / n
        var = (mom[:, 2] / n - mean * mean).clamp_min(0)
        y = (x - mean.to(x.dtype)[None, :, None, None]) / torch.sqrt(var.to(x.dtype)[None, :, None, None] + eps)
        with torch.no_grad():
            unb = var * (n / (n - 1))
            rm.mul_(1 - momentum).add_(momentum * mean.to(rm.dtype))
            rv.mul_(1 - momentum).add_(momentum * unb.to(rv.dtype))
            key = prefix + "num_batches_tracked"
            if key in sd:
                sd[key] += 1
        return y * w.to(x.dtype)[None, :, None, None] + b.to(x.dtype)[None, :, None, None]
    return batch_norm


def _w_sharded_generator(rank, port, out_dir, sync):
    _init(rank, port)
    from fastfourierconvolution_amd import distributed as D
    import oracle.ffc_oracle as O
    nz, nc, ngf, B = 16, 3, 8, 6
    torch.manual_seed(3)
    z = torch.randn(B, nz, 1, 1, dtype=torch.float64)
    sd = {k: v.clone() for k, v in torch.load(os.path.join(out_dir, "state.pt"), weights_only=True).items()}
    if sync:
        O.batch_norm = _sync_batch_norm_factory(D)
    out = O.ffc_generator(D.shard_batch(z), sd, nz, nc, ngf, True, fft="torch")
    full = D.gather_batch(out.contiguous(), B)
    torch.save({"out": full, "sd": sd}, os.path.join(out_dir, f"gen{rank}.pt"))
    dist.destroy_process_group()


def _generator_state(nz, nc, ngf):
    """fp64 state with the generator's state_dict names (the drop-in module is only constructed,
    never run: construction needs no GPU), weights N(0, 0.02)-ish, BN gamma ~1"""
    import contextlib
    import io
    from fastfourierconvolution_amd import FFCGenerator
    with contextlib.redirect_stdout(io.StringIO()):
        G = FFCGenerator(nz, nc, ngf)
    g = torch.Generator().manual_seed(11)
    sd = {}
    for k, v in G.state_dict().items():
        if k.endswith("num_batches_tracked"):
            sd[k] = v.clone()
        elif k.endswith("running_mean") or k.endswith("running_var"):
            sd[k] = v.double().clone()
        elif v.dim() == 1:   # BN affine
            base = 1.0 if k.endswith("weight") else 0.0
            sd[k] = base + 0.05 * torch.randn(v.shape, generator=g, dtype=torch.float64)
        else:
            fan = v[0].numel() if v.numel() else 1
            sd[k] = torch.randn(v.shape, generator=g, dtype=torch.float64) / max(fan, 1) ** 0.5
    return sd


@pytest.mark.parametrize("sync", [True, False])
def test_sharded_generator_syncbn(tmp_path, sync):
    import oracle.ffc_oracle as O
    nz, nc, ngf, B = 16, 3, 8, 6
    sd0 = _generator_state(nz, nc, ngf)
    torch.save(sd0, tmp_path / "state.pt")
    torch.manual_seed(3)
    z = torch.randn(B, nz, 1, 1, dtype=torch.float64)
    sd_ref = {k: v.clone() for k, v in sd0.items()}
    ref = O.ffc_generator(z, sd_ref, nz, nc, ngf, True, fft="torch")
    _spawn(_w_sharded_generator, str(tmp_path), sync)
    for r in range(WORLD):
        res = torch.load(tmp_path / f"gen{r}.pt", weights_only=True)
        err = O.normwise_err(res["out"], ref)
        if sync:
            assert err < 1e-12, err
            for k, v in sd_ref.items():
                assert torch.allclose(res["sd"][k].double(), v.double(), rtol=0, atol=1e-12), k
        else:
            assert err > 1e-3, err   # naive sharding changes train-mode BN: SyncBN is required
