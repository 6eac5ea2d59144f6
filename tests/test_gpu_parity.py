"""GPU parity of the HIP path (through the C ABI) against the reference's golden vectors and
the fp64 oracle.  Tolerance (BASELINE.json north_star): normwise
max|got - ref| / max|ref| <= 1e-4 in fp32."""
import contextlib
import io

import numpy as np
import pytest
import torch

from conftest import build_dropin, call_dropin, golden_cases, load_case
from oracle.ffc_oracle import ffc_generator, normwise_err, run_fixture_case

pytestmark = pytest.mark.gpu
TOL = 1e-4
CASES = golden_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden(case, fu_path):
    state, inputs, data = load_case(case)
    mod = build_dropin(case, state)
    out = call_dropin(case, mod, inputs)
    assert sorted("ref." + k for k in out) == case["outputs"]
    torch.cuda.synchronize()
    for k, v in out.items():
        err = normwise_err(v.cpu(), torch.from_numpy(data["ref." + k]))
        assert err <= TOL, (k, err)
    # BN running statistics / num_batches_tracked after the forward
    sd = mod.state_dict()
    for k in data.files:
        if k.startswith("after."):
            key = k[len("after."):]
            got = sd[key].cpu().numpy()
            if data[k].dtype.kind == "i":
                assert int(got) == int(data[k]), key
            else:
                np.testing.assert_allclose(got, data[k], rtol=1e-4, atol=1e-5, err_msg=key)


@pytest.mark.parametrize("case", [c for c in CASES if c["kind"] == "FourierUnitSN"][:4],
                         ids=lambda c: c["name"])
def test_deterministic(case):
    """two runs on the same inputs are bitwise identical (no atomics on the path)"""
    state, inputs, _ = load_case(case)
    a = call_dropin(case, build_dropin(case, state), inputs)["out"]
    b = call_dropin(case, build_dropin(case, state), inputs)["out"]
    assert torch.equal(a, b)


def _gen_state(nz, nc, ngf, seed=5):
    import fastfourierconvolution_amd as F
    with contextlib.redirect_stdout(io.StringIO()):
        g = F.FFCGenerator(nz, nc, ngf)
    gen = torch.Generator().manual_seed(seed)
    sd = {}
    for k, v in g.state_dict().items():
        if k.endswith("num_batches_tracked"):
            sd[k] = v.clone()
        elif k.endswith("running_var"):
            sd[k] = torch.ones_like(v)
        elif k.endswith("running_mean"):
            sd[k] = torch.zeros_like(v)
        elif v.dim() == 1:   # BN affine
            sd[k] = (1.0 if k.endswith("weight") else 0.0) + 0.1 * torch.randn(v.shape, generator=gen)
        else:
            fan = v[0].numel() if v.dim() > 1 else 1
            sd[k] = torch.randn(v.shape, generator=gen) / max(1.0, fan) ** 0.5
    g.load_state_dict(sd)
    return g, sd


@pytest.mark.parametrize("nc,B", [(1, 256), (3, 256), (3, 7)])
def test_generator_full_batch_vs_oracle(nc, B):
    """BASELINE config 2 (nc=1) / metric shape (nc=3) at the full batch, train-mode BN,
    against the fp64 oracle; also running statistics."""
    g, sd = _gen_state(100, nc, 64)
    g = g.cuda().train()
    z = torch.randn((B, 100, 1, 1), generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        out = g(z.cuda()).cpu()
    osd = {k: v.double() if v.is_floating_point() else v.clone() for k, v in sd.items()}
    with torch.no_grad():
        ref = ffc_generator(z.double(), osd, 100, nc, 64, True)
    err = normwise_err(out, ref)
    assert err <= TOL, err
    gsd = g.state_dict()
    for k, v in osd.items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            np.testing.assert_allclose(gsd[k].cpu().double().numpy(), v.numpy(), rtol=2e-4, atol=1e-5, err_msg=k)


def test_generator_eval_matches_oracle():
    g, sd = _gen_state(100, 3, 64, seed=9)
    # realistic running stats: one train step with momentum 1
    for m in g.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.momentum = 1.0
    g = g.cuda().train()
    with torch.no_grad():
        g(torch.randn(16, 100, 1, 1, device="cuda"))
    g.eval()
    z = torch.randn((32, 100, 1, 1), generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        out = g(z.cuda()).cpu()
    osd = {k: (v.detach().cpu().double() if v.is_floating_point() else v.cpu()) for k, v in g.state_dict().items()}
    with torch.no_grad():
        ref = ffc_generator(z.double(), osd, 100, 3, 64, False)
    assert normwise_err(out, ref) <= TOL


@pytest.fixture(params=["fused", "staged"])
def fu_path(request):
    """run a test under each Fourier-unit path (the auto choice depends on the batch size)"""
    from fastfourierconvolution_amd import _runtime as rt
    old = rt.FU_PATH
    rt.FU_PATH = request.param
    yield request.param
    rt.FU_PATH = old


def test_fu_sizes_vs_oracle(fu_path):
    """every supported FU plane size, train + eval, several channel counts, fused and staged paths"""
    import fastfourierconvolution_amd as F
    from oracle.ffc_oracle import fourier_unit
    gen = torch.Generator().manual_seed(11)
    for (c, h, w) in [(1, 4, 4), (5, 8, 32), (24, 32, 8), (96, 8, 8), (40, 16, 16), (2, 32, 32)]:
        for train in (True, False):
            fu = F.FourierUnitSN(c, c)
            with torch.no_grad():
                fu.conv_layer.weight.copy_(torch.randn(fu.conv_layer.weight.shape, generator=gen) / (2 * c) ** 0.5)
                fu.bn.weight.copy_(1 + 0.1 * torch.randn(2 * c, generator=gen))
                fu.bn.bias.copy_(0.1 * torch.randn(2 * c, generator=gen))
                fu.bn.running_mean.copy_(0.1 * torch.randn(2 * c, generator=gen))
                fu.bn.running_var.copy_(1 + torch.rand(2 * c, generator=gen))
            sd = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in fu.state_dict().items()}
            fu = fu.cuda().train(train)
            x = torch.randn((3, c, h, w), generator=gen)
            with torch.no_grad():
                got = fu(x.cuda()).cpu()
                ref = fourier_unit(x.double(), sd, "", train)
            err = normwise_err(got, ref)
            assert err <= TOL, (c, h, w, train, err)


def test_unsupported_plane_raises():
    import fastfourierconvolution_amd as F
    fu = F.FourierUnitSN(4, 4).cuda()
    with torch.no_grad():                                 # the fused inference kernels
        with pytest.raises(NotImplementedError):
            fu(torch.randn(1, 4, 48, 48, device="cuda"))     # not a power of two
        with pytest.raises(NotImplementedError):
            fu(torch.randn(1, 4, 64, 128, device="cuda"))    # staged FU: square planes only
    with pytest.raises(NotImplementedError):             # training path: line FFTs on square planes
        fu(torch.randn(1, 4, 128, 64, device="cuda"))        # up to 128^2, direct DFTs up to 64^2
    y = fu(torch.randn(1, 4, 128, 128, device="cuda"))      # 128^2 trains (tests/test_gpu_fgan_train.py)
    assert y.shape == (1, 4, 128, 128) and y.requires_grad


def test_conditional_path_raises_like_reference():
    import fastfourierconvolution_amd as F
    fu = F.FourierUnitSN(4, 4).cuda()
    with pytest.raises(TypeError):
        fu(torch.randn(1, 4, 8, 8, device="cuda"), torch.zeros(1, dtype=torch.long, device="cuda"))


def test_graph_capture_replays():
    """the whole generator forward captures into one hipGraph and replays to the same result"""
    g, _ = _gen_state(100, 3, 64, seed=2)
    g = g.cuda().eval()
    z = torch.randn(64, 100, 1, 1, device="cuda")
    with torch.no_grad():
        ref = g(z).clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            g(z)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = g(z)
        graph.replay()
        torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("arith", ["f32", "split-presplit"])
@pytest.mark.parametrize("case", [c for c in CASES if c["kind"] in ("FFC_BN_ACT", "FFCGenerator", "FFCDiscriminator")],
                         ids=lambda c: c["name"])
def test_golden_conv_arith_variants(case, arith):
    """the LDS-patch conv's other product paths on the same cases (the default split-bf16 path with
    A split in registers runs in test_golden): the exact f32-input MFMA (FFC_CONV_ARITH=f32) and the
    split with pre-split A planes (FFC_CONVP_PRESPLIT=1, ffc_split_bf16 + ffc_convp_job.A3)"""
    from fastfourierconvolution_amd import _runtime as rt
    old = rt.CONV_ARITH, rt.PRESPLIT_A
    rt.CONV_ARITH, rt.PRESPLIT_A = ("f32", False) if arith == "f32" else ("split", True)
    try:
        state, inputs, data = load_case(case)
        out = call_dropin(case, build_dropin(case, state), inputs)
        for k, v in out.items():
            assert normwise_err(v.cpu(), torch.from_numpy(data["ref." + k])) <= TOL, k
    finally:
        rt.CONV_ARITH, rt.PRESPLIT_A = old


@pytest.mark.parametrize("case", [c for c in CASES if c["kind"] in ("FFC_BN_ACT", "FFCGenerator")],
                         ids=lambda c: c["name"])
def test_golden_generic_conv_kernel(case):
    """the same cases with the LDS-patch kernel disabled (generic phase-GEMM kernel)"""
    from fastfourierconvolution_amd import _runtime as rt
    old = rt.USE_PATCH
    rt.USE_PATCH = False
    try:
        state, inputs, data = load_case(case)
        out = call_dropin(case, build_dropin(case, state), inputs)
        for k, v in out.items():
            assert normwise_err(v.cpu(), torch.from_numpy(data["ref." + k])) <= TOL, k
    finally:
        rt.USE_PATCH = old


@pytest.mark.parametrize("M,H,W,bias", [(1, 5, 7, True), (2, 32, 32, False), (4, 3, 40, True), (3, 64, 16, False)])
def test_smallm_convt_odd_sizes_vs_oracle(M, H, W, bias):
    """direct VALU ConvT k4 s2 p1 path (M <= 4): odd sizes, tiles wider than 32, bias"""
    import fastfourierconvolution_amd as F
    from oracle.ffc_oracle import ffc_bn_act
    cfg = dict(in_channels=40, out_channels=M, kernel_size=4, ratio_gin=0.5, ratio_gout=0.0, stride=2, padding=1,
               bias=bias, activation_layer="Tanh", upsampling=True)
    with contextlib.redirect_stdout(io.StringIO()):
        m = F.FFC_BN_ACT(40, M, 4, 0.5, 0.0, 2, 1, bias=bias, activation_layer=torch.nn.Tanh, upsampling=True)
    gen = torch.Generator().manual_seed(M)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn(p.shape, generator=gen) * 0.2)
    sd = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in m.state_dict().items()}
    xl = torch.randn(3, 20, H, W, generator=gen)
    xg = torch.randn(3, 20, H, W, generator=gen)
    m = m.cuda()
    with torch.no_grad():
        ol, og = m((xl.cuda(), xg.cuda()))
        rl, rg = ffc_bn_act((xl.double(), xg.double()), sd, "", cfg, True)
    assert og == 0 and rg == 0
    assert normwise_err(ol.cpu(), rl) <= TOL


@pytest.mark.parametrize("cin,M,H,W,bias", [(64, 3, 32, 32, False), (64, 1, 32, 32, True), (32, 4, 12, 20, True),
                                              (16, 3, 8, 36, False), (128, 2, 16, 48, False)])
def test_smallm_convt_vs_oracle(cin, M, H, W, bias):
    """ConvT k4 s2 p1 with M <= 4 on the direct small-M kernel (convt_smallm.hip) -- the FFC-DCGAN
    generator's last layer (models/ffc_generator.py:28) and ragged 8 x 32 tiles"""
    import fastfourierconvolution_amd as F
    from oracle.ffc_oracle import ffc_bn_act
    cfg = dict(in_channels=cin, out_channels=M, kernel_size=4, ratio_gin=0.5, ratio_gout=0.0, stride=2, padding=1,
               bias=bias, activation_layer="Tanh", upsampling=True)
    with contextlib.redirect_stdout(io.StringIO()):
        m = F.FFC_BN_ACT(cin, M, 4, 0.5, 0.0, 2, 1, bias=bias, activation_layer=torch.nn.Tanh, upsampling=True)
    gen = torch.Generator().manual_seed(cin + M + H)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn(p.shape, generator=gen) * (2.0 / cin) ** 0.5)
    sd = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in m.state_dict().items()}
    xl = torch.randn(3, cin // 2, H, W, generator=gen)
    xg = torch.randn(3, cin // 2, H, W, generator=gen)
    m = m.cuda()
    with torch.no_grad():
        ol, og = m((xl.cuda(), xg.cuda()))
        rl, rg = ffc_bn_act((xl.double(), xg.double()), sd, "", cfg, True)
    assert og == 0 and rg == 0
    assert normwise_err(ol.cpu(), rl) <= 1e-5


def _w_sharded_gpu(rank, port, out_dir):
    """one rank of a 2-way sample shard on cuda:0 (gloo carries the BN moments; RCCL needs one
    GPU per rank, which the 1-GPU test box does not have)"""
    import os
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import fastfourierconvolution_amd.distributed as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    g, _ = _gen_state(100, 3, 64, seed=21 + rank)   # rank 1 starts from different weights ...
    g = g.cuda().train()
    D.broadcast_module(g)                            # ... and receives rank 0's
    D.enable_sync_bn()
    z = torch.randn((10, 100, 1, 1), generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        out = g(D.shard_batch(z).cuda())
    torch.save({"out": out.cpu(), "sd": {k: v.cpu() for k, v in g.state_dict().items()}},
               os.path.join(out_dir, f"r{rank}.pt"))
    D.disable_sync_bn()
    dist.destroy_process_group()


def test_sharded_syncbn_gpu(tmp_path):
    """N>1 data path through the HIP kernels: a ragged 2-way shard (5+5 of B=10) with SyncBN
    equals the single-process global-batch forward, running statistics included."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_w_sharded_gpu, args=(port, str(tmp_path)), nprocs=2, join=True)
    g, _ = _gen_state(100, 3, 64, seed=21)
    g = g.cuda().train()
    z = torch.randn((10, 100, 1, 1), generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        ref = g(z.cuda()).cpu()
    rs = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(2)]
    got = torch.cat([r["out"] for r in rs], dim=0)
    assert normwise_err(got, ref) <= TOL
    gsd = g.state_dict()
    for r in rs:
        for k, v in gsd.items():
            if "running" in k:
                np.testing.assert_allclose(r["sd"][k].numpy(), v.cpu().numpy(), rtol=1e-4, atol=1e-6, err_msg=k)
            elif k.endswith("num_batches_tracked"):
                assert int(r["sd"][k]) == int(v), k


def test_bn_momentum_none_cumulative():
    """nn.BatchNorm2d(momentum=None): cumulative running average (factor 1/(num_batches_tracked+1)),
    the one case where num_batches_tracked is read by the statistics kernel."""
    import functools
    import oracle.ffc_oracle as O
    g, sd = _gen_state(100, 3, 16, seed=13)
    g = g.cuda().train()
    for m in g.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.momentum = None
    osd = {k: v.double() if v.is_floating_point() else v.clone() for k, v in sd.items()}
    orig = O.batch_norm
    try:
        for step in range(2):
            z = torch.randn((9, 100, 1, 1), generator=torch.Generator().manual_seed(40 + step))
            with torch.no_grad():
                out = g(z.cuda()).cpu()
            O.batch_norm = functools.partial(orig, momentum=1.0 / (step + 1))
            with torch.no_grad():
                ref = O.ffc_generator(z.double(), osd, 100, 3, 16, True)
            assert normwise_err(out, ref) <= TOL
    finally:
        O.batch_norm = orig
    gsd = g.state_dict()
    for k, v in osd.items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            np.testing.assert_allclose(gsd[k].cpu().double().numpy(), v.numpy(), rtol=2e-4, atol=1e-5, err_msg=k)
        elif k.endswith("num_batches_tracked"):
            assert int(gsd[k]) == int(v) == (0 if ".lfu." in k else 2), k


@pytest.mark.parametrize("B,C,M,H", [(4, 100, 4096, 1), (8, 16, 32, 1), (4, 16, 32, 2), (4, 16, 32, 3),
                                     (4, 16, 32, 8), (2, 20, 40, 6), (256, 100, 4096, 1)])
@pytest.mark.parametrize("patch", [True, False])
def test_pointwise_conv_kernels(B, C, M, H, patch):
    """1x1 segments through both conv kernels (LDS-patch incl. its unaligned float staging, and
    the generic GEMM) vs the PyTorch fp32 reference; 1x1 spatial is the outer-product ConvT path."""
    from fastfourierconvolution_amd import _plan, _runtime as rt
    gen = torch.Generator().manual_seed(B * 131 + H)
    x = torch.randn(B, C, H, H, generator=gen).cuda()
    w = torch.randn(M, C, 1, 1, generator=gen).cuda()
    ref = torch.nn.functional.conv2d(x, w)
    old = rt.USE_PATCH
    rt.USE_PATCH = patch
    try:
        ex = rt.ConvExec(B, M, [_plan.Seg("pw", C, H, H)], [(w, 0, 1, 1, None)], x.device)
        lp = rt.LaunchPlan([ex], x.device)
        out = torch.empty(B, M, H, H, device=x.device)
        lp.launch([ex.job([(x, None)], out)], torch.cuda.current_stream().cuda_stream)
    finally:
        rt.USE_PATCH = old
    assert normwise_err(out.cpu(), ref.cpu()) <= TOL



def test_conv3x3_nonfinite_input_halo():
    """Non-finite inputs: a 3x3 stride-1 conv runs as 4x4 taps whose 4th row / column has
    zero weights but reads the real pixel one past the window (_plan.plan_patch_job), and the split-bf16
    products turn an Inf operand into NaN pieces.  So an Inf input pixel P makes every output whose
    padded 4x4 window holds P non-finite -- one row and one column more than the reference's 3x3
    halo -- and leaves every other output finite and equal to the reference."""
    import fastfourierconvolution_amd as F
    from oracle.ffc_oracle import ffc_bn_act
    cfg = dict(in_channels=16, out_channels=16, kernel_size=3, ratio_gin=0.0, ratio_gout=0.0, stride=1, padding=1,
               norm_layer="Identity", activation_layer="Identity")
    with contextlib.redirect_stdout(io.StringIO()):
        m = F.FFC_BN_ACT(16, 16, 3, 0.0, 0.0, 1, 1)
    sd = {k: v.double() for k, v in m.state_dict().items()}
    x = torch.randn(2, 16, 32, 32, generator=torch.Generator().manual_seed(5))
    y0, x0 = 9, 20
    x[1, 3, y0, x0] = float("inf")
    with torch.no_grad():
        out = m.cuda().eval()(x.cuda())[0].cpu()
    ref = ffc_bn_act(x.double(), sd, "", cfg, False)[0]
    pad = torch.zeros(32, 32, dtype=torch.bool)
    pad[max(0, y0 - 2):y0 + 2, max(0, x0 - 2):x0 + 2] = True     # outputs y, x with P in rows y-1..y+2, cols x-1..x+2
    halo = torch.zeros(32, 32, dtype=torch.bool)
    halo[y0 - 1:y0 + 2, x0 - 1:x0 + 2] = True                     # the reference's 3x3 halo
    assert not torch.isfinite(ref[1][:, halo]).any() and torch.isfinite(ref[1][:, ~halo]).all()
    assert not torch.isfinite(out[1][:, pad]).any()
    ok = torch.ones_like(out, dtype=torch.bool)
    ok[1][:, pad] = False
    assert torch.isfinite(out[ok]).all()
    assert normwise_err(torch.where(ok, out, torch.zeros_like(out)), torch.where(ok, ref, torch.zeros_like(ref))) <= TOL
