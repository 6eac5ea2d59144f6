"""The RCCL side of the N > 1 path, as far as a one-GPU box can run it.

RCCL needs one GPU per rank, so the multi-rank RCCL run happens only in the driver's 8-GPU
scaling bench (bench.py --gpus N).  What a single GPU can check is the machinery that run relies
on: a one-rank "nccl" (RCCL) process group, the SyncBN moment all-reduce routed through it
(distributed.enable_sync_bn(even_world1=True) keeps the collective in a one-rank group), eager and
captured inside a hipGraph together with the generator's kernels, replayed to the same output as
the forward without the collective.  The numerics of the exchange itself (shards + merged moments
== global batch) are covered over gloo in tests/test_distributed_cpu.py and, through the HIP
kernels, in tests/test_gpu_parity.py::test_sharded_syncbn_gpu.
"""
import contextlib
import io
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture
def rccl_world1():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        yield
    finally:
        from fastfourierconvolution_amd import distributed as D
        D.disable_sync_bn()
        dist.destroy_process_group()


def test_rccl_moments_all_reduce_in_graph(rccl_world1):
    from fastfourierconvolution_amd import distributed as D
    m = torch.arange(30, dtype=torch.float64, device="cuda").reshape(10, 3)
    ref = m.clone()
    D.merge_moments(m)
    torch.cuda.synchronize()
    assert torch.equal(m, ref)
    from fastfourierconvolution_amd.graphs import capture_step

    def step():
        m.mul_(2.0)
        D.merge_moments(m)
    # warm-up on a side stream, synchronise, thread-local capture, ranks agree (graphs.py): an
    # eager all-reduce right before a global-mode capture is what aborted once in round 2
    g = capture_step(step, warmup=0)
    assert g is not None
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(m, ref * 2)      # capture records without running: one replayed mul + all-reduce
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(m, ref * 4)


@pytest.mark.parametrize("B", [32, 64, 128])
def test_syncbn_generator_graph_over_rccl(rccl_world1, B):
    """train-mode generator forward with every BN's moments all-reduced over RCCL: eager and
    hipGraph-replayed outputs equal the forward without SyncBN, running statistics included
    (B = 32: staged 16² / 32² FUs; 64 / 128: the fused FU over two workgroups per sample)"""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import distributed as D
    from fastfourierconvolution_amd import _runtime as rt
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FFCGenerator(100, 3, 64).cuda().train()
    z = torch.randn(B, 100, 1, 1, device="cuda")
    state = {k: v.clone() for k, v in G.state_dict().items()}
    with torch.no_grad():
        ref = G(z).clone()
        ref_state = {k: v.clone() for k, v in G.state_dict().items()}
        G.load_state_dict(state)
        D.enable_sync_bn(even_world1=True)
        assert rt._sync_group() is not None
        obs = rt.LaunchObserver()
        rt.set_observer(obs)
        eager = G(z).clone()
        rt.set_observer(None)
        assert obs.summary()["bn_stats"]["launches"] == 6      # the 6 SyncBN exchanges of the generator
        # fused reduce+finalize vs reduce / all-reduce / finalize: same fp64 moments, maybe another order
        torch.testing.assert_close(eager, ref, rtol=1e-6, atol=1e-6)
        for k, v in ref_state.items():
            torch.testing.assert_close(G.state_dict()[k], v, rtol=1e-6, atol=1e-7, msg=k)
        from fastfourierconvolution_amd.graphs import capture_step
        res = {}

        def step():
            res["out"] = G(z)
        graph = capture_step(step, warmup=1)
        assert graph is not None
        out = res["out"]
        graph.replay()
        torch.cuda.synchronize()
    torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-6)


def test_paired_syncbn_one_collective(rccl_world1):
    """an FFC layer's bn_l and bn_g under SyncBN share ONE all-reduce (_runtime.bn_scale_shift_many):
    same scale / shift and running statistics, bit for bit, as the per-BN single-rank path -- a small
    slab (one-block-per-channel merge) beside a large one (two-level merge, scratch behind moments)"""
    import torch.nn as nn
    from fastfourierconvolution_amd import _runtime as rt, distributed as D
    g = torch.Generator().manual_seed(5)
    items, twins = [], []
    for C, nrows in ((64, 300), (32, 2000)):
        n = torch.randint(1, 64, (nrows, C), generator=g).float()
        slab = torch.stack([n, torch.randn((nrows, C), generator=g), torch.rand((nrows, C), generator=g) * n,
                            torch.zeros_like(n)], -1).cuda()
        bn = nn.BatchNorm2d(C).cuda().train()
        with torch.no_grad():
            bn.weight.copy_(1 + 0.1 * torch.randn(C, generator=g))
            bn.bias.copy_(0.1 * torch.randn(C, generator=g))
        twin = nn.BatchNorm2d(C).cuda().train()
        twin.load_state_dict(bn.state_dict())
        items.append((bn, C, slab, nrows, 1.0))
        twins.append((twin, C, slab, nrows, 1.0))
    ref = [rt.bn_scale_shift(b, C, s, n, cm, torch.device("cuda"), rt.stream_of(s)) for b, C, s, n, cm in twins]
    calls = []
    orig = D.merge_moments
    D.merge_moments = lambda m, group=None: calls.append(m.shape) or orig(m, group=group)
    try:
        D.enable_sync_bn(even_world1=True)
        got = rt.bn_scale_shift_many(items, torch.device("cuda"), torch.cuda.current_stream().cuda_stream)
    finally:
        D.merge_moments = orig
        D.disable_sync_bn()
    torch.cuda.synchronize()
    assert calls == [torch.Size([96, 3])]
    for (s0, h0), (s1, h1) in zip(ref, got):
        assert torch.equal(s0, s1) and torch.equal(h0, h1)
    for (b, *_), (t, *_) in zip(items, twins):
        for k, v in b.state_dict().items():
            assert torch.equal(v, t.state_dict()[k]), k


@pytest.mark.parametrize("path", ["staged", "fused"])
@pytest.mark.parametrize("B", [32, 64])
def test_syncbn_moments_fold_repeat_bitwise(rccl_world1, path, B):
    """SyncBN with the consumers finalizing from the all-reduced moments (ffc_bn_fold.moments, round
    6): twenty fresh SpectralTransform train forwards (gen64 ffc3 shape) bitwise equal, and within
    1e-6 of the single-rank path (same fp64 moments, another merge / finalize route)"""
    import copy
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import distributed as D
    from fastfourierconvolution_amd import _runtime as rt
    torch.manual_seed(B)
    with contextlib.redirect_stdout(io.StringIO()):
        st = F.SpectralTransform(64, 32, stride=2, upsample=True).cuda().train()
    x = torch.randn((B, 64, 16, 16), generator=torch.Generator().manual_seed(B + 1)).cuda()
    old = rt.FU_PATH
    rt.FU_PATH = path
    try:
        with torch.no_grad():
            ref = copy.deepcopy(st)(x).clone()
            D.enable_sync_bn(even_world1=True)
            outs = [copy.deepcopy(st)(x).clone() for _ in range(20)]
        torch.cuda.synchronize()
    finally:
        rt.FU_PATH = old
        D.disable_sync_bn()
    bad = [i for i, o in enumerate(outs) if not torch.equal(o, outs[0])]
    assert not bad, f"runs {bad} differ from run 0"
    torch.testing.assert_close(outs[0], ref, rtol=1e-6, atol=1e-6)
