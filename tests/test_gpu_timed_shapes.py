"""Parity at the shapes bench.py times (VERDICT r1 "parity at the timed shapes").

Kernel choice depends on the batch: the fused per-sample Fourier unit needs B >= 64
(_runtime.FU_FUSED_MIN_BATCH), the patch-conv tile configuration (_plan.pick_patch_cfg), the
1x1 GEMM tiles (_runtime.pick_pw_cfg) and the weight-gradient split (_autograd.wgrad_splits)
depend on B too.  So every per-GPU batch a bench line runs is checked here against the oracle:

  gen64 (FFCGenerator 64x64x3)      strong-scaling shards 256 / 128 / 86 / 64 / 32 (N = 1, 2, 3, 4, 8),
                                    train-mode BN; eval at B = 256
  fgan128 (configs[3])              the N = 8 shard, B = 64, fp32 mix, direct; the N = 1 job, B = 512,
                                    by permuted replicas (below)
  fgan128sn (configs[4], fp16 mix)  the N = 8 shard, B = 128, direct, per-layer errors; the N = 1 job,
                                    B = 1024, by permuted replicas
  gan64train (configs[2])           B = 256: the loss, and every layer's input / parameter gradients of
                                    G and D (layer-wise VJPs, tests/test_gpu_train.py's method)

Permuted replicas: the oracle cannot run a 512- or 1024-sample fgan128 forward in a test's
time, so the big batch is built from 8 distinct samples, each repeated B/8 times in a random
order (noise rows with them).  Train-mode BN statistics of the replicated batch equal those of
the 8 samples (mean and biased variance are invariant under replication), so every output row
must equal the oracle's 8-sample train forward at its source sample: that checks the B = 512 /
1024 kernels (fused FU, tile tables, BN slab rows) row by row, and the random order catches any
sample-indexing error.

Tolerances: 1e-4 normwise (fp32); fp16 mix: 1e-2 for the stack (the gate of
tests/test_gpu_sn_fp16.py), per-layer errors printed.
"""
import contextlib
import io

import pytest
import torch
import torch.nn as nn

from oracle.ffc_oracle import (fgan128_layers, ffc_bn_act, ffc_generator, noise_injection, normwise_err,
                               sn_materialize)

pytestmark = pytest.mark.gpu
TOL = 1e-4
TOL_FP16_STACK = 1e-2


def _weights_init(m):
    """fgan64_complete.py:22-31, as bench.py initialises"""
    name = m.__class__.__name__
    if name.find("Conv") != -1:
        nn.init.normal_(m.weight.data, 0.0, 0.02)
    elif name.find("BatchNorm") != -1:
        nn.init.normal_(m.weight.data, 1.0, 0.02)
        nn.init.constant_(m.bias.data, 0)


def _sd64(mod):
    return {k: (v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu().clone())
            for k, v in mod.state_dict().items()}


def _gen64(seed=1234):
    import fastfourierconvolution_amd as F
    torch.manual_seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FFCGenerator(100, 3, 64)
    G.apply(_weights_init)
    return G


@pytest.mark.parametrize("B", [128, 86, 64, 32])
def test_gen64_strong_scaling_shards_train(B):
    """the per-GPU batches of `bench.py --gpus N` (global 256): train-mode BN, weights_init weights"""
    G = _gen64()
    sd = _sd64(G)
    G = G.cuda().train()
    z = torch.randn((B, 100, 1, 1), generator=torch.Generator().manual_seed(B))
    with torch.no_grad():
        got = G(z.cuda()).cpu()
        ref = ffc_generator(z.double(), sd, 100, 3, 64, True)
    err = normwise_err(got, ref)
    print(f"gen64 train B={B}: {err:.2e}")
    assert err <= TOL, err
    gsd = G.state_dict()
    for k, v in sd.items():    # running statistics moved like nn.BatchNorm2d's
        if k.endswith(("running_mean", "running_var")):
            torch.testing.assert_close(gsd[k].cpu().double(), v, rtol=2e-4, atol=1e-5, msg=k)


def test_gen64_eval_full_batch():
    """eval-mode BN at the metric batch (B = 256) with a warm-up batch's running statistics"""
    G = _gen64(7).cuda().train()
    for m in G.modules():
        if isinstance(m, nn.BatchNorm2d):
            m.momentum = 1.0
    with torch.no_grad():
        G(torch.randn((64, 100, 1, 1), generator=torch.Generator().manual_seed(2)).cuda())
    G.eval()
    sd = _sd64(G)
    z = torch.randn((256, 100, 1, 1), generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        got = G(z.cuda()).cpu()
        ref = ffc_generator(z.double(), sd, 100, 3, 64, False)
    err = normwise_err(got, ref)
    print(f"gen64 eval B=256: {err:.2e}")
    assert err <= TOL, err


# --------------------------------------------------------------------------- fgan128 stacks
def _fgan(sn: bool, mix: str, seed=1234):
    import fastfourierconvolution_amd as F
    torch.manual_seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FGenerator(128)
    G.apply(_weights_init)
    if sn:
        F.spectral_norm_ffc(G)
    F.set_mix_precision(G, mix)
    return G


def _noises(B, gen):
    return [(torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen),
             torch.randn((B, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen)) for n in (2, 3, 4, 5, 6)]


def _gpu_layers(G, z, noises):
    """FGenerator.forward_float in train mode, layer by layer (the same calls), -> [layer outputs]"""
    outs = []
    with torch.no_grad():
        x = G._noise_to_feature(z)
        for i, n in enumerate((2, 3, 4, 5, 6)):
            nl, ng = noises[i]
            x = getattr(G, f"conv{n}").forward_noise(x, (getattr(G, f"lcl_noise{n}"), nl),
                                                     (getattr(G, f"glb_noise{n}"), ng))
            outs.append(x)
        outs.append(G.resizer(G.conv7(x)))
    return outs


def _oracle_layers(z, sd, noises):
    """oracle.fgan128_generator (fgan128_complete.py:489-515) in train mode, -> [layer outputs]"""
    import torch.nn.functional as Fn
    from oracle.ffc_oracle import resizer
    x = Fn.linear(z, sd["noise_to_feature.0.weight"], sd["noise_to_feature.0.bias"]).reshape(z.shape[0], -1, 4, 4)
    outs = []
    for i, (name, cfg) in enumerate(fgan128_layers(128)):
        x = ffc_bn_act(x, sd, name + ".", cfg, True)
        if name != "conv7":
            nl, ng = noises[i]
            x = (noise_injection(x[0], sd, f"lcl_noise{name[-1]}.", nl),
                 noise_injection(x[1], sd, f"glb_noise{name[-1]}.", ng))
        outs.append(x)
    outs[-1] = resizer(outs[-1])
    return outs


def _layer_errs(got, ref):
    errs = []
    for g, r in zip(got, ref):
        gs = g if isinstance(g, tuple) else (g,)
        rs = r if isinstance(r, tuple) else (r,)
        errs.append(max(normwise_err(a.cpu(), b) for a, b in zip(gs, rs) if isinstance(a, torch.Tensor)))
    return errs


def _sd_for_oracle(G, sn):
    sd = _sd64(G)
    if sn:   # one power iteration from the same u / v the GPU forward will start from
        sn_materialize(sd, {n: 1 for n, m in G.named_modules() if isinstance(m, nn.ConvTranspose2d)}, True)
    return sd


@pytest.mark.parametrize("sn,mix,B", [(False, "fp32", 64), (True, "fp16", 128)])
def test_fgan128_shard_direct(sn, mix, B):
    """the N = 8 per-GPU shards of configs[3] (B = 64, fp32 mix) and configs[4] (B = 128, SN + fp16
    mix), train mode with explicit NoiseInjection noise, every layer against the fp64 oracle"""
    G = _fgan(sn, mix)
    sd = _sd_for_oracle(G, sn)
    G = G.cuda().train()
    gen = torch.Generator().manual_seed(B)
    z = torch.randn((B, 128), generator=gen)
    noises = _noises(B, gen)
    got = _gpu_layers(G, z.cuda(), [(a.cuda(), b.cuda()) for a, b in noises])
    ref = _oracle_layers(z.double(), sd, [(a.double(), b.double()) for a, b in noises])
    errs = _layer_errs(got, ref)
    print(f"fgan128{'sn' if sn else ''} {mix} B={B} per-layer normwise errors (conv2..conv7): "
          + ", ".join(f"{e:.2e}" for e in errs))
    assert errs[-1] <= (TOL if mix == "fp32" else TOL_FP16_STACK), errs
    if mix == "fp32":
        assert max(errs) <= TOL, errs


@pytest.mark.parametrize("sn,mix,B", [(False, "fp32", 512), (True, "fp16", 1024)])
def test_fgan128_full_job_permuted_replicas(sn, mix, B):
    """the N = 1 strong-scaling jobs (B = 512 / 1024 on one GPU): 8 distinct samples repeated B/8
    times in a random order; each output row must equal the oracle's 8-sample train forward at its
    source sample (module docstring)"""
    G = _fgan(sn, mix)
    sd = _sd_for_oracle(G, sn)
    G = G.cuda().train()
    gen = torch.Generator().manual_seed(B + 1)
    z8 = torch.randn((8, 128), generator=gen)
    n8 = _noises(8, gen)
    src = torch.randperm(B, generator=gen) % 8
    with torch.no_grad():
        got = G.forward_float(z8[src].cuda(), [(a[src].cuda(), b[src].cuda()) for a, b in n8]).cpu()
    ref = _oracle_layers(z8.double(), sd, [(a.double(), b.double()) for a, b in n8])[-1]
    err = normwise_err(got, ref[src])
    print(f"fgan128{'sn' if sn else ''} {mix} B={B} (permuted replicas of 8): {err:.2e}")
    assert err <= (TOL if mix == "fp32" else TOL_FP16_STACK), err


# --------------------------------------------------------------------------- gan64train B = 256
def test_gan64train_full_batch_layerwise():
    """configs[2] at the timed batch (B = 256, train-mode BN): loss = mean(D(G(z))) against the fp64
    oracle, and every FFC_BN_ACT's input and parameter gradients of G and D against the oracle's
    vector-Jacobian product at the HIP path's own layer input (test_gpu_train._layer_checks)"""
    from test_gpu_train import _layer_checks
    res = _layer_checks(True, B=256, fp32_ref=False, check_loss=True)
    print(f"gan64train B=256: {len(res)} gradients, worst normwise error {max(e for _, e, _ in res):.2e}")
    bad = sorted(((e, k) for k, e, _ in res if not e < TOL), reverse=True)
    assert not bad, bad[:12]


# --------------------------------------------------------------------------- configs[0] (bench --workload block)
BLOCK_CFG = dict(in_channels=32, out_channels=32, kernel_size=3, ratio_gin=0.5, ratio_gout=0.5, stride=1, padding=1,
                 norm_layer="BatchNorm2d", activation_layer="ReLU")


@pytest.mark.parametrize("mode", ["train", "eval"])
def test_block_config0_b16(mode):
    """BASELINE configs[0] at exactly its batch: FFC_BN_ACT(32, 32, 3, 0.5, 0.5, 1, 1, BN, ReLU),
    x = (x_l, x_g) ~ N(0,1)^(16,16,32,32), bench.py's weights; the output pair and (train) the
    updated running statistics against the fp64 oracle (layers/ffc/ffc_bn_act.py:70-83)"""
    import fastfourierconvolution_amd as F
    torch.manual_seed(1234)
    with contextlib.redirect_stdout(io.StringIO()):
        blk = F.FFC_BN_ACT(32, 32, 3, 0.5, 0.5, stride=1, padding=1, norm_layer=nn.BatchNorm2d,
                           activation_layer=nn.ReLU)
    blk.apply(_weights_init)
    if mode == "eval":     # randomised running statistics (untrained eval outputs are tiny)
        g = torch.Generator().manual_seed(3)
        for m in blk.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.running_mean.copy_(0.1 * torch.randn(m.num_features, generator=g))
                m.running_var.copy_(0.5 + torch.rand(m.num_features, generator=g))
    sd = _sd64(blk)
    g = torch.Generator().manual_seed(0)
    x = (torch.randn((16, 16, 32, 32), generator=g), torch.randn((16, 16, 32, 32), generator=g))
    blk = blk.cuda().train(mode == "train")
    with torch.no_grad():
        out = blk(tuple(t.cuda() for t in x))
    torch.cuda.synchronize()
    ref = ffc_bn_act(tuple(t.double() for t in x), sd, "", BLOCK_CFG, mode == "train")
    for o, r in zip(out, ref):
        assert normwise_err(o.cpu(), r) <= TOL
    if mode == "train":    # the oracle's batch_norm updated sd's running stats in place
        for k, v in blk.state_dict().items():
            if k.endswith(("running_mean", "running_var")):
                assert normwise_err(v.cpu(), sd[k]) <= TOL, k


# --------------------------------------------------------------------------- round 5: the timed artifact itself
def test_gen64_train_graph_replays_vs_oracle():
    """bench.py's timed artifact: the train-mode B = 256 generator forward captured into one hipGraph
    (graphs.capture_step, as bench.py captures it: one warm-up on a side stream, then the capture)
    and replayed twice.  The graph's static output after the replays equals the fp64 oracle's train
    forward, and the BN running statistics / num_batches_tracked advanced exactly as three
    nn.BatchNorm2d train steps on the same batch (warm-up + 2 replays; the capture runs nothing):
    the in-graph BN slab resets and folds are checked, not just an eager forward
    (/root/reference/models/ffc_generator.py:30-44)."""
    from fastfourierconvolution_amd.graphs import capture_step
    G = _gen64()
    sd = _sd64(G)
    G = G.cuda().train()
    z = torch.randn((256, 100, 1, 1), generator=torch.Generator().manual_seed(100)).cuda()

    def step():
        with torch.no_grad():
            return G(z)
    graph = capture_step(step, warmup=1)
    assert graph is not None and getattr(graph, "ffc_output", None) is not None
    out = graph.ffc_output
    with torch.no_grad():
        out.fill_(float("nan"))
    graph.replay()
    graph.replay()
    torch.cuda.synchronize()
    got = out.cpu()
    with torch.no_grad():
        for _ in range(3):
            ref = ffc_generator(z.cpu().double(), sd, 100, 3, 64, True)
    err = normwise_err(got, ref)
    print(f"gen64 train B=256 graph replay: {err:.2e}")
    assert err <= TOL, err
    gsd = G.state_dict()
    n_bn = 0
    for k, v in sd.items():
        if k.endswith(("running_mean", "running_var")):
            torch.testing.assert_close(gsd[k].cpu().double(), v, rtol=2e-4, atol=1e-5, msg=k)
            n_bn += ".lfu." not in k
        elif k.endswith("num_batches_tracked"):   # the never-run lfu BNs stay at 0 in both
            assert int(gsd[k]) == int(v) == (0 if ".lfu." in k else 3), k
    assert n_bn == 12   # bn1 + fu.bn of ffc1..ffc3, mean and var each


def test_fgan128_full_job_distinct_samples_eval():
    """configs[3] at B = 512 with 512 DISTINCT samples (the train-mode full-job test replicates 8):
    eval-mode BN makes every row a function of its own sample alone, so rows picked at random are
    checked against the oracle's forward of just those samples -- an indexing error between samples
    of the big batch (tile tables, fused FU rows, head tiles) shows up here"""
    G = _fgan(False, "fp32", seed=4321)
    G = G.cuda().train()
    for m in G.modules():   # realistic running statistics: one train batch with momentum 1
        if isinstance(m, nn.BatchNorm2d):
            m.momentum = 1.0
    gen = torch.Generator().manual_seed(9)
    with torch.no_grad():
        G.forward_float(torch.randn((64, 128), generator=gen).cuda())
    G.eval()
    sd = _sd64(G)
    z = torch.randn((512, 128), generator=gen)
    with torch.no_grad():
        got = G.forward_float(z.cuda()).cpu()
    rows = torch.randperm(512, generator=gen)[:6]
    from oracle.ffc_oracle import fgan128_generator
    with torch.no_grad():
        ref = fgan128_generator(z[rows].double(), sd, False, None)
    err = normwise_err(got[rows], ref)
    print(f"fgan128 eval B=512 distinct samples, rows {rows.tolist()}: {err:.2e}")
    assert err <= TOL, err
