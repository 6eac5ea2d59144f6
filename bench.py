#!/usr/bin/env python3
"""bench.py — FFC-DCGAN generator forward throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload gen64|fgan128|fgan128sn|gan64train|fgan128train|block]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`--gpus N` without a launcher (WORLD_SIZE unset) starts the N ranks itself
(fastfourierconvolution_amd/launch.py: N fresh child processes, one per GPU, before anything
touches the GPU) and exits with their status; fewer than N visible GPUs is an error (exit 3).
Under a launcher WORLD_SIZE must equal --gpus.

Workload (BASELINE.json metric "FFC-generator fwd images/sec @ B=256 64x64x3"):
FFCGenerator(nz=100, nc=3, ngf=64) (models/ffc_generator.py) forward, B=256 per GPU,
train-mode BatchNorm (the modules' default state; SpectralTransform.bn1 and FourierUnitSN.bn
use batch statistics), synthetic z ~ N(0,1), weights from the reference's weights_init
(fgan64_complete.py:22-31: conv N(0, 0.02), BN gamma N(1, 0.02), beta 0).
One step = one generator forward over one batch; inputs resident in HBM.

Scaling (``--scaling``, default strong): the configuration's batch split over the ranks, with the
weak-scaling figure alongside at N > 1.  ``--scaling weak``: every GPU runs the configuration's batch (gen64 256,
fgan128 512 = configs[3], fgan128sn 1024 = configs[4]); the job's global batch is N x that, drawn
once from one seed and sliced per rank, and train-mode BN normalises over ALL of it (SyncBN: the
BN moments are all-reduced over RCCL, so the sharded result equals the global-batch forward; the
strong split does the same over the configuration's batch).  The per-rank shard steps and the
strong-scaling budget are in DESIGN.md §5.  One process per GPU; weights are
broadcast once at init.  The step is hipGraph-captured (thread-local capture, the RCCL
all-reduces inside the graph; graphs.py).  At N > 1 the gen64 line also carries the gathered
global-batch output's parity against the CPU reference.

The JSON line also carries:
  roofline      live per-kernel HIP-event timing of one eager pass (dominant kernel), MFMA f32 peak
  cpu_baseline  the oracle's fp32 op-for-op torch CPU path (oracle/ffc_oracle.py, fft="torch"),
                rank 0 at N=1 only, bounded sample
  parity        normwise max|GPU - CPU reference| / max|CPU reference| for the same z and weights
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from fastfourierconvolution_amd.graphs import capture_step  # noqa: E402  (no GPU touched at import)

METRIC = "FFC-generator fwd images/sec @ B=256 64×64×3; % HBM roofline; max |Δ| vs ref"
PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_32x32x2_f32) dense peak
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 dense MFMA peak (v_mfma_f32_32x32x16_bf16)
SPLIT_PRODUCTS = 6              # bf16 piece products per fp32 product in the split-bf16 kernels


def mfma_roof(dom, achieved):
    """MFMA roofline entry.  `peak` is the dtype's (f32) dense MFMA peak.  The LDS-patch conv and
    weight-gradient kernels compute their fp32 products as six exact bf16 piece products
    (ffc_internal.h split3), so their own instruction ceiling is the bf16 peak / 6: reported
    beside it as `split_peak` / `split_frac` (the other GEMM kernels run the f32 MFMA)."""
    from fastfourierconvolution_amd import _runtime as rt
    r = {"kernel": dom, "bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_F32_MFMA_TFLOPS,
         "unit": "TFLOP/s", "frac": round(achieved / PEAK_F32_MFMA_TFLOPS, 4)}
    if rt.CONV_ARITH == "split":
        sp = PEAK_BF16_MFMA_TFLOPS / SPLIT_PRODUCTS
        r.update({"arith": "split-bf16 x6 (fp32-accurate)", "split_peak": round(sp, 1),
                  "split_frac": round(achieved / sp, 4)})
    return r


def profile_pass(step, n):
    """One instrumented eager pass (rt.LaunchObserver: HIP events around every library launch on its
    stream) of ``n`` steps.  The GPU is held busy (torch.cuda._sleep) while the host enqueues each
    step, so the stream never runs dry inside an event pair: the events then time the kernels alone,
    not the host's op-dispatch gaps between them.  -> (observer summary, last step's output)"""
    from fastfourierconvolution_amd import _runtime as rt
    obs = rt.LaunchObserver()
    out = None
    for _ in range(max(1, n)):
        torch.cuda.synchronize()
        torch.cuda._sleep(100_000_000)    # >= 40 ms of GPU time: the whole step is enqueued behind it
        rt.set_observer(obs)
        out = step()
        rt.set_observer(None)
    return obs.summary(), out


def time_steps(run, steps, world=1):
    """Time EXACTLY ``steps`` calls of ``run`` between a barrier + device synchronise on both sides
    (wall clock, max over ranks), with a HIP event after every step on the launch stream for the
    per-step median (SURVEY.md §8d asks for the median).  -> (elapsed_s, median_ms_per_step)"""
    import torch.distributed as dist
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(steps):
        run()
        evs[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    med = per[len(per) // 2] if steps % 2 else 0.5 * (per[steps // 2 - 1] + per[steps // 2])
    if world > 1:
        t = torch.tensor([elapsed, med], device=torch.device("cuda", torch.cuda.current_device()),
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, med = float(t[0]), float(t[1])
    return elapsed, med


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", choices=["gen64", "fgan128", "fgan128sn", "gan64train", "fgan128train", "block"],
                   default="gen64",
                   help="gen64: FFCGenerator 64x64 (BASELINE metric, configs[1]/[2]); "
                        "fgan128: fgan128 FGenerator 128x128x3 (configs[3]: B 512, split over the GPUs); "
                        "fgan128sn: its spectral-norm variant with the fp16 mix (configs[4]: B 1024, split); "
                        "gan64train: generator + discriminator 64x64x3 fwd+bwd + Adam (configs[2], B=256); "
                        "fgan128train: fgan128 training iteration, G update + D update (fgan128_complete.py:680-703, "
                        "B=64); "
                        "block: one FFC_BN_ACT 32->32 at 32x32, B=16 (configs[0])")
    p.add_argument("--mix", choices=["fp32", "fp16"], default=None,
                   help="spectral mix arithmetic (default: fp16 for fgan128sn, fp32 otherwise)")
    p.add_argument("--gpus", type=int, default=None,
                   help="number of GPUs / ranks (default: WORLD_SIZE, or 1); starts the ranks itself when "
                        "WORLD_SIZE is unset")
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                   help="strong (default): the configuration's batch (gen64 256, fgan128 512, fgan128sn 1024) "
                        "split over the ranks, as BASELINE configs[3]/[4] shard it; at N > 1 the line also "
                        "carries the weak-scaling measurement (every GPU runs the configuration's batch) in "
                        "'weak_scaling'.  weak: only that measurement")
    p.add_argument("--global-batch", type=int, default=None,
                   help="strong scaling global batch (gen64: 256, fgan128: 512, fgan128sn: 1024)")
    p.add_argument("--batch", type=int, default=None, help="weak scaling samples per GPU (gen64: 256, "
                                                           "fgan128: 512, fgan128sn: 1024)")
    p.add_argument("--dry-run", action="store_true",
                   help="launch + shard plan only, over gloo on the CPU (no GPU touched): rank 0 prints the plan")
    p.add_argument("--nz", type=int, default=100)
    p.add_argument("--nc", type=int, default=3)
    p.add_argument("--ngf", type=int, default=64)
    p.add_argument("--bn-mode", choices=["train", "eval"], default="train")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--profile-steps", type=int, default=3)
    p.add_argument("--syncbn-rehearsal", action="store_true",
                   help="N = 1 only: run the SyncBN path of N > 1 (moments reduce -> all_reduce over a one-rank "
                        "RCCL group -> finalize, no in-kernel BN folds) to time a rank's kernels as they run at "
                        "N > 1, without the xGMI latency (DESIGN.md section 5)")
    return p.parse_args()


# kernel-name prefixes behind each observed launch label (for the PMC traffic lookup)
LABEL_KERNELS = {"conv_gemm": ("convq_kernel", "convq_reduce_kernel", "convp_kernel", "conv_gemm_kernel"), "fu_pass0": ("fu_kernel",),
                 "fu_pass1": ("fu_kernel",), "st_prologue": ("st_prologue_kernel",),
                 "convt_smallm": ("convt_smallm_kernel",), "fu2d_r2c": ("fu2d_r2c_kernel", "fu2d_r2c_mix_kernel"),
                 "fu2d_mix0": ("fu2d_mix_kernel",), "fu2d_mix1": ("fu2d_mix_cols_kernel", "fu2d_mix_kernel"),
                 "fu2d_c2r": ("fu2d_c2r",), "conv3_smallm": ("conv3x3_smallm_kernel",),
                 "dense": ("dense_kernel",)}


def pmc_traffic(label, workload="gen64"):
    """HBM bytes per launch of the kernels behind `label`, from the newest committed
    profiles/<round>/pmc_traffic.json (tools/pmc_traffic.sh: FETCH_SIZE / WRITE_SIZE passes,
    corrected per MI355X_MICROARCH.md), or None."""
    import glob
    name = "pmc_traffic.json" if workload == "gen64" else f"pmc_traffic_{workload}.json"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name)))
    if not files or label not in LABEL_KERNELS:
        return None
    kern = json.load(open(files[-1]))["kernels"]
    sel = [v for k, v in kern.items() if k.startswith(LABEL_KERNELS[label])]
    n = sum(v["launches"] for v in sel)
    if n == 0:
        return None
    return {"bytes_per_launch": round(sum(v["bytes_per_launch"] * v["launches"] for v in sel) / n),
            "source": os.path.relpath(files[-1], ROOT)}


def fgan_cpu_baseline(args, G, z_cpu, sn):
    """fgan128: the oracle's fp32 torch-CPU FGenerator on a bounded sample of the batch (train mode
    draws its noise on the CPU); parity of the GPU forward against the fp64 oracle in train mode on
    the same sample with the same explicit NoiseInjection noise (BN batch statistics and, for the SN
    variant, one power iteration from the same u / v on both sides)."""
    import torch.nn as nn
    from oracle.ffc_oracle import fgan128_generator, normwise_err, sn_materialize
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    nb = min(args.batch, 8)
    zs = z_cpu[:nb]
    dims = {n: 1 for n, m in G.named_modules() if isinstance(m, nn.ConvTranspose2d)}
    gen = torch.Generator().manual_seed(7)

    def noises():
        return [(torch.randn((nb, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen),
                 torch.randn((nb, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=gen)) for n in (2, 3, 4, 5, 6)]
    state = {k: v.detach().cpu().clone() for k, v in G.state_dict().items()}
    with torch.no_grad():
        sd = {k: v.clone() for k, v in state.items()}
        if sn:
            sn_materialize(sd, dims, True)
        iters, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds or iters == 0:
            fgan128_generator(zs, sd, True, noises(), fft="torch")
            iters += 1
        el = time.perf_counter() - t0
        nz = noises()
        sd = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in state.items()}
        if sn:
            sn_materialize(sd, dims, True)
        ref = fgan128_generator(zs.double(), sd, True, [(a.double(), b.double()) for a, b in nz])
        G.train()
        dev = next(G.parameters()).device
        got = G.forward_float(zs.to(dev), [(a.to(dev), b.to(dev)) for a, b in nz]).cpu()
        G.train(args.bn_mode == "train")
    cpu = {"value": round(nb * iters / el, 2), "unit": "images/s", "cores": threads, "kind": "port",
           "sample": f"oracle fp32 torch-CPU fgan128 FGenerator{' + spectral norm' if sn else ''} fwd, B={nb} "
                     f"(bounded sample), {iters} iterations in {el:.1f}s, train-mode BN"}
    tol = 1e-2 if args.mix == "fp16" else 1e-4
    parity = {"normwise_err_vs_cpu_ref": normwise_err(got, ref), "mode": f"train, B={nb}, explicit noise, fp64 oracle",
              "mix": args.mix, "tolerance": tol}
    return cpu, parity


def sharded_parity(args, step, cpu_state, z_glob, global_batch, rank, timed_out=None):
    """N > 1 (gen64, train-mode BN; every rank calls it): one more sharded forward on every rank,
    outputs gathered to the global batch (all_gather over RCCL), compared on rank 0 with the fp32
    CPU reference path run on the global z.  This checks the SyncBN all-reduces end to end: a naive
    shard differs from the global-batch forward by ~3e-1 normwise.  (Eval mode
    needs the GPU's running stats and no collective: the caller skips it on every rank.)"""
    from fastfourierconvolution_amd.distributed import gather_batch
    torch.cuda.synchronize()
    mine = timed_out if timed_out is not None else step()   # the graph's output after the timed replays
    out = gather_batch(mine.contiguous(), global_batch)
    if rank != 0:
        return None
    from oracle.ffc_oracle import ffc_generator, normwise_err
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1))
    with torch.no_grad():
        ref = ffc_generator(z_glob, {k: v.clone() for k, v in cpu_state.items()}, args.nz, args.nc, args.ngf,
                            args.bn_mode == "train", fft="torch")
    return {"normwise_err_vs_cpu_ref": normwise_err(out.cpu(), ref), "mode": f"train, global B={global_batch}, "
            "sharded + SyncBN, outputs gathered", "tolerance": 1e-4,
            "checked": "captured hipGraphs' outputs after the timed replays" if timed_out is not None else
            "eager forward"}


def weights_init(m):
    """fgan64_complete.py:22-31"""
    import torch.nn as nn
    name = m.__class__.__name__
    if name.find("Conv") != -1:
        nn.init.normal_(m.weight.data, 0.0, 0.02)
    elif name.find("BatchNorm") != -1:
        nn.init.normal_(m.weight.data, 1.0, 0.02)
        nn.init.constant_(m.bias.data, 0)


def train_main(args):
    """BASELINE configs[2]: FFCGenerator(100, 3, 64) + FFCDiscriminator(3, 64), 64x64x3, B=256, one
    step = z -> G -> D -> loss = mean(D(G(z))) -> backward through D and G (custom-op autograd, every
    forward and backward op a HIP kernel of libffc_amd.so) -> Adam on both parameter sets (the
    reference's fgan64 optimizer, lr 2e-4, betas (0.5, 0.999); torch's foreach Adam).  Train-mode
    BN.  Single GPU (config 3 is 1x MI355X)."""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("gan64train is the single-GPU configs[2] workload")
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FFCGenerator(args.nz, args.nc, args.ngf)
        D = F.FFCDiscriminator(args.nc, args.ngf)
    G.apply(weights_init)
    D.apply(weights_init)
    cpu_state = ({k: v.clone() for k, v in G.state_dict().items()}, {k: v.clone() for k, v in D.state_dict().items()})
    G, D = G.to(dev).train(), D.to(dev).train()
    use_graph = not args.no_graph
    opt = torch.optim.Adam(list(G.parameters()) + list(D.parameters()), lr=2e-4, betas=(0.5, 0.999), foreach=True,
                           capturable=use_graph)
    gen = torch.Generator(device="cpu").manual_seed(100)
    z_cpu = torch.randn((args.batch, args.nz, 1, 1), generator=gen)
    z = z_cpu.to(dev)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = D(G(z)).mean()
        loss.backward()
        opt.step()
        return loss

    run = step
    if use_graph:
        # whole-step capture (forward, custom-op backward, Adam): the library launches allocate
        # nothing and never sync, plans / packed-weight buffers exist after the eager warm-up, and
        # the weight re-packs the optimizer's in-place updates trigger are captured with the step
        graph = capture_step(step, warmup=max(2, args.warmup))
        use_graph = graph is not None
        if use_graph:
            run = graph.replay
    for _ in range(max(1, args.warmup)):
        run()
    elapsed, med = time_steps(run, args.steps)
    value = args.batch * args.steps / elapsed
    summ, _ = profile_pass(step, args.profile_steps)
    nprof = max(1, args.profile_steps)
    kernels = {k: {"launches_per_step": v["launches"] / nprof, "ms_per_step": v["ms"] / nprof,
                   "avg_us": 1e3 * v["ms"] / v["launches"]} for k, v in summ.items()}
    mm = {k: v for k, v in summ.items() if v["flops"] > 0}
    dom = max(mm, key=lambda k: mm[k]["ms"])
    d = summ[dom]
    achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
    roof = mfma_roof(dom, achieved)
    tr = pmc_traffic(dom, args.workload)
    roof["traffic"] = tr["bytes_per_launch"] if tr else None
    cpu = parity = None
    if not args.no_cpu_baseline:
        from oracle.ffc_oracle import ffc_discriminator, ffc_generator
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        torch.set_num_threads(threads)
        nb = min(args.batch, 16)
        zs = z_cpu[:nb]

        def cpu_step(dt, sdg, sdd):
            p = [v for sd in (sdg, sdd) for k, v in sd.items() if v.is_floating_point() and
                 not k.endswith(("running_mean", "running_var"))]
            for t in p:
                t.grad = None
                t.requires_grad_(True)
            loss = ffc_discriminator(ffc_generator(zs.to(dt), sdg, args.nz, args.nc, args.ngf, True, fft="torch"),
                                     sdd, args.nc, args.ngf, True, fft="torch").mean()
            loss.backward()
            return loss.item()
        sdg = {k: v.clone() for k, v in cpu_state[0].items()}
        sdd = {k: v.clone() for k, v in cpu_state[1].items()}
        iters, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds or iters == 0:
            cpu_step(torch.float32, sdg, sdd)
            iters += 1
        el = time.perf_counter() - t0
        cpu = {"value": round(nb * iters / el, 2), "unit": "images/s", "cores": threads, "kind": "port",
               "sample": f"oracle fp32 torch-CPU G+D fwd+bwd (torch autograd through the op-for-op reference "
                         f"path, no optimizer), B={nb}, {iters} iterations in {el:.1f}s, train-mode BN"}
        sd64 = [{k: (v.double() if v.is_floating_point() else v.clone()) for k, v in st.items()} for st in cpu_state]
        ref = cpu_step(torch.float64, *sd64)
        with contextlib.redirect_stdout(io.StringIO()):
            G2 = F.FFCGenerator(args.nz, args.nc, args.ngf)
            D2 = F.FFCDiscriminator(args.nc, args.ngf)
        G2.load_state_dict(cpu_state[0])
        D2.load_state_dict(cpu_state[1])
        got = D2.to(dev).train()(G2.to(dev).train()(zs.to(dev))).mean().item()
        parity = {"loss_rel_err_vs_fp64_oracle": abs(got - ref) / abs(ref), "mode": f"train, B={nb}",
                  "gradients": "layer-wise vs the fp64 oracle in tests/test_gpu_train.py (<= 1e-4 normwise)",
                  "tolerance": 1e-4}
    line = {
        "metric": "FFC-DCGAN G+D fwd+bwd train step images/sec @ B=256 64x64x3 (BASELINE configs[2])",
        "value": round(value, 1), "unit": "images/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4), "ms_per_step_median": round(med, 4),
        "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: z ~ N(0,1); weights per fgan64_complete.py:22-31 weights_init",
        "config": {"workload": f"FFCGenerator(nz={args.nz},nc={args.nc},ngf={args.ngf}) + FFCDiscriminator("
                               f"nc={args.nc},ndf={args.ngf}) fwd+bwd + Adam, loss = mean(D(G(z)))",
                   "global_batch": args.batch, "per_gpu_batch": args.batch, "bn_mode": "train", "hipgraph": use_graph,
                   "parallelism": "dp1"},
        "roofline": roof, "cpu_baseline": cpu, "parity": parity, "kernels": kernels,
    }
    print(json.dumps(line))


def fgan128train_main(args):
    """One iteration of the fgan128 training loop (fgan128_complete.py:680-703, num_dis_updates = 1):
    a generator update (z -> FGenerator -> Discriminator -> hinge_loss_gen -> backward through D into
    G -> AdamW on G, D frozen) then a discriminator update (z -> FGenerator no-grad -> D(fake), D(real)
    -> hinge_loss_dis -> backward -> AdamW on D), at the reference's default batch 64 (:759), AdamW
    lr 2e-4 betas (0.5, 0.999) (:624-625), train-mode BN, spectral-norm D (one power iteration per D
    call), NoiseInjection noise drawn on the GPU.  Both z are redrawn on the GPU every step; the
    "real" batch is a fixed synthetic tensor in [-1, 1] (no dataset).  Every G / D layer, forward and
    backward, is a libffc_amd.so kernel (fastfourierconvolution_amd/training.py); the whole iteration
    is one hipGraph.  Single GPU (the reference's loop is)."""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    from fastfourierconvolution_amd.training import discriminator_step, generator_step
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("fgan128train is a single-GPU workload (the reference's training loop)")
    B = args.batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FGenerator(128)
    D = F.Discriminator()
    G.apply(weights_init)
    D.apply(weights_init)
    cpu_state = ({k: v.clone() for k, v in G.state_dict().items()}, {k: v.clone() for k, v in D.state_dict().items()})
    G, D = G.to(dev).train(), D.to(dev).train()
    use_graph = not args.no_graph
    kw = dict(lr=2e-4, betas=(0.5, 0.999), foreach=True, capturable=use_graph)
    optim_G = torch.optim.AdamW(G.parameters(), **kw)
    optim_D = torch.optim.AdamW(D.parameters(), **kw)
    gen = torch.Generator(device="cpu").manual_seed(100)
    real = (torch.rand((B, 3, 128, 128), generator=gen) * 2 - 1).to(dev)
    z_g = torch.empty((B, 128), device=dev)
    z_d = torch.empty((B, 128), device=dev)

    def step():
        z_g.normal_()
        loss_G = generator_step(G, D, optim_G, optim_D, z_g)
        z_d.normal_()
        loss_D = discriminator_step(G, D, optim_G, optim_D, z_d, real)
        return loss_G, loss_D

    run = step
    if use_graph:
        graph = capture_step(step, warmup=max(2, args.warmup))
        use_graph = graph is not None
        if use_graph:
            run = graph.replay
    for _ in range(max(1, args.warmup)):
        run()
    elapsed, med = time_steps(run, args.steps)
    value = B * args.steps / elapsed
    summ, _ = profile_pass(step, args.profile_steps)
    nprof = max(1, args.profile_steps)
    kernels = {k: {"launches_per_step": v["launches"] / nprof, "ms_per_step": v["ms"] / nprof,
                   "avg_us": 1e3 * v["ms"] / v["launches"]} for k, v in summ.items()}
    mm = {k: v for k, v in summ.items() if v["flops"] > 0}
    dom = max(mm, key=lambda k: mm[k]["ms"])
    achieved = summ[dom]["flops"] / (summ[dom]["ms"] * 1e-3) / 1e12
    roof = mfma_roof(dom, achieved)
    tr = pmc_traffic(dom, args.workload)
    roof["traffic"] = tr["bytes_per_launch"] if tr else None
    cpu = parity = None
    if not args.no_cpu_baseline:
        cpu, parity = fgan128train_cpu(args, cpu_state, dev)
    line = {
        "metric": f"fgan128 G+D training iteration images/sec @ B={B} 128x128x3 (fgan128_complete.py:680-703)",
        "value": round(value, 1), "unit": "images/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4), "ms_per_step_median": round(med, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: z ~ N(0,1) redrawn on the GPU each step, real = fixed U(-1, 1) batch; weights per "
                "fgan128_complete.py:23-32 weights_init",
        "config": {"workload": "FGenerator(z=128) + spectral-norm Discriminator: generator update + 1 discriminator "
                               "update, hinge losses, AdamW", "global_batch": B, "per_gpu_batch": B,
                   "bn_mode": "train", "hipgraph": use_graph, "parallelism": "dp1"},
        "roofline": roof, "cpu_baseline": cpu, "parity": parity, "kernels": kernels,
    }
    print(json.dumps(line))


def fgan128train_cpu(args, cpu_state, dev):
    """cpu_baseline: the oracle's fp32 torch-CPU iteration (G update fwd + bwd through D, D update fwd on
    fake and real + bwd; no optimizer) on a bounded sample; parity: both hinge losses of one HIP iteration
    (explicit noise, same z) vs the fp64 oracle from the same initial state (u / v included)."""
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd.training import discriminator_step, generator_step
    from oracle.ffc_oracle import fgan128_discriminator, fgan128_generator, hinge_loss_dis, hinge_loss_gen
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    nb = 2
    gen = torch.Generator().manual_seed(7)
    zg, zd = torch.randn((nb, 128), generator=gen), torch.randn((nb, 128), generator=gen)
    real = torch.rand((nb, 3, 128, 128), generator=gen) * 2 - 1

    def noises(dt):
        g = torch.Generator().manual_seed(8)
        return [(torch.randn((nb, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=g).to(dt),
                 torch.randn((nb, 1, 2 ** (n + 1), 2 ** (n + 1)), generator=g).to(dt)) for n in (2, 3, 4, 5, 6)]

    def oracle_iter(dt, fft):
        sdg = {k: (v.to(dt) if v.is_floating_point() else v.clone()) for k, v in cpu_state[0].items()}
        sdd = {k: (v.to(dt) if v.is_floating_point() else v.clone()) for k, v in cpu_state[1].items()}
        for k, v in sdg.items():
            if v.is_floating_point() and not k.endswith(("running_mean", "running_var")):
                v.requires_grad_(True)
        lg = hinge_loss_gen(fgan128_discriminator(fgan128_generator(zg.to(dt), sdg, True, noises(dt), fft=fft),
                                                  sdd, True))
        lg.backward()
        for k, v in sdd.items():
            if k.endswith(("weight_orig", "bias")):
                v.requires_grad_(True)
        with torch.no_grad():
            fake = fgan128_generator(zd.to(dt), sdg, True, noises(dt), fft=fft)
        ld = hinge_loss_dis(fgan128_discriminator(fake, sdd, True), fgan128_discriminator(real.to(dt), sdd, True))
        ld.backward()
        return lg.item(), ld.item()
    iters, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds or iters == 0:
        oracle_iter(torch.float32, "torch")
        iters += 1
    el = time.perf_counter() - t0
    cpu = {"value": round(nb * iters / el, 3), "unit": "images/s", "cores": threads, "kind": "port",
           "sample": f"oracle fp32 torch-CPU fgan128 G+D iteration (torch autograd through the op-for-op reference "
                     f"path, no optimizer), B={nb}, {iters} iterations in {el:.1f}s, train-mode BN"}
    ref = oracle_iter(torch.float64, "numpy")
    with contextlib.redirect_stdout(io.StringIO()):
        G2 = F.FGenerator(128)
    D2 = F.Discriminator()
    G2.load_state_dict(cpu_state[0])
    D2.load_state_dict(cpu_state[1])
    G2, D2 = G2.to(dev).train(), D2.to(dev).train()
    oG = torch.optim.AdamW(G2.parameters(), lr=0.0, weight_decay=0.0)
    oD = torch.optim.AdamW(D2.parameters(), lr=0.0, weight_decay=0.0)
    nz = [(a.to(dev), b.to(dev)) for a, b in noises(torch.float32)]
    lg = generator_step(G2, D2, oG, oD, zg.to(dev), nz).item()
    ld = discriminator_step(G2, D2, oG, oD, zd.to(dev), real.to(dev), nz).item()
    parity = {"loss_G_rel_err_vs_fp64_oracle": abs(lg - ref[0]) / abs(ref[0]),
              "loss_D_rel_err_vs_fp64_oracle": abs(ld - ref[1]) / abs(ref[1]), "mode": f"train, B={nb}, explicit noise",
              "gradients": "D layer-wise and G step vs the fp64 oracle in tests/test_gpu_fgan_d.py (<= 1e-4 normwise)",
              "tolerance": 1e-4}
    return cpu, parity


BLOCK_CFG = dict(in_channels=32, out_channels=32, kernel_size=3, ratio_gin=0.5, ratio_gout=0.5, stride=1, padding=1,
                 norm_layer="BatchNorm2d", activation_layer="ReLU")


def block_main(args):
    """BASELINE configs[0]: one FFC_BN_ACT(32, 32, 3, 0.5, 0.5, stride 1, padding 1, BatchNorm2d, ReLU)
    block (layers/ffc/ffc_bn_act.py:25-83), x = (x_l, x_g) ~ N(0,1)^(16,16,32,32) each (SURVEY.md
    §8d cfg1: seed 0), train-mode BN.  One step = one block forward over the batch of 16 samples.
    The reference quotes this configuration on its CPU path; the same CPU restatement is timed
    beside the GPU (cpu_baseline), and the GPU output is checked against it (parity)."""
    import torch.nn as nn
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("block is the single-device configs[0] workload")
    B = args.batch or 16
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    with contextlib.redirect_stdout(io.StringIO()):
        blk = F.FFC_BN_ACT(32, 32, 3, 0.5, 0.5, stride=1, padding=1, norm_layer=nn.BatchNorm2d,
                           activation_layer=nn.ReLU)
    blk.apply(weights_init)
    cpu_state = {k: v.clone() for k, v in blk.state_dict().items()}
    blk = blk.to(dev).train(args.bn_mode == "train")
    g = torch.Generator().manual_seed(0)
    x_cpu = (torch.randn((B, 16, 32, 32), generator=g), torch.randn((B, 16, 32, 32), generator=g))
    x = tuple(t.to(dev) for t in x_cpu)

    def step():
        with torch.no_grad():
            return blk(x)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    use_graph, run = not args.no_graph, step
    if use_graph:
        graph = capture_step(step, warmup=1)
        use_graph = graph is not None
        if use_graph:
            run = graph.replay
    for _ in range(max(1, args.warmup)):
        run()
    elapsed, med = time_steps(run, args.steps)
    value = B * args.steps / elapsed
    summ, _ = profile_pass(step, args.profile_steps)
    nprof = max(1, args.profile_steps)
    kernels = {k: {"launches_per_step": v["launches"] / nprof, "ms_per_step": v["ms"] / nprof,
                   "avg_us": 1e3 * v["ms"] / v["launches"]} for k, v in summ.items()}
    mm = {k: v for k, v in summ.items() if v["flops"] > 0}
    dom = max(mm, key=lambda k: mm[k]["ms"])
    roof = mfma_roof(dom, mm[dom]["flops"] / (mm[dom]["ms"] * 1e-3) / 1e12)
    roof["traffic"] = None
    cpu = parity = None
    if not args.no_cpu_baseline:
        from oracle.ffc_oracle import ffc_bn_act, normwise_err
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        torch.set_num_threads(threads)
        training = args.bn_mode == "train"
        sd = {k: v.clone() for k, v in cpu_state.items()}
        if not training:
            sd = {k: v.detach().cpu().clone() for k, v in blk.state_dict().items()}
        with torch.no_grad():
            ref = ffc_bn_act(x_cpu, sd, "", BLOCK_CFG, training, fft="torch")
            iters, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < args.cpu_seconds or iters == 0:
                ffc_bn_act(x_cpu, sd, "", BLOCK_CFG, training, fft="torch")
                iters += 1
            el = time.perf_counter() - t0
            got = step()
        ref_cat, got_cat = torch.cat(ref, 1), torch.cat([t.cpu() for t in got], 1)
        sd64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in sd.items()}
        ref64 = torch.cat(ffc_bn_act(tuple(t.double() for t in x_cpu), sd64, "", BLOCK_CFG, training), 1)
        parity = {"normwise_err_vs_cpu_ref": normwise_err(got_cat, ref_cat),
                  "normwise_err_vs_fp64_oracle": normwise_err(got_cat, ref64), "tolerance": 1e-4}
        cpu = {"value": round(B * iters / el, 2), "unit": "samples/s", "cores": threads, "kind": "port",
               "sample": f"oracle fp32 torch-CPU FFC_BN_ACT fwd (op-for-op reference path), B={B}, {iters} "
                         f"iterations in {el:.1f}s, {args.bn_mode}-mode BN"}
    print(json.dumps({
        "metric": "FFC_BN_ACT(32->32, k3, 0.5/0.5, BN, ReLU) fwd samples/sec @ B=16 32x32 (BASELINE configs[0])",
        "value": round(value, 1), "unit": "samples/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4), "ms_per_step_median": round(med, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: x ~ N(0,1); weights per fgan64_complete.py:22-31 weights_init",
        "config": {"workload": "FFC_BN_ACT(32,32,3,0.5,0.5,stride=1,padding=1,BatchNorm2d,ReLU) forward 32x32",
                   "global_batch": B, "per_gpu_batch": B, "bn_mode": args.bn_mode, "hipgraph": use_graph,
                   "parallelism": "dp1"},
        "roofline": roof, "cpu_baseline": cpu, "parity": parity, "kernels": kernels}))


GLOBAL_BATCH = {"gen64": 256, "fgan128": 512, "fgan128sn": 1024,   # BASELINE.json configs[1..4]
                "gan64train": 256, "fgan128train": 64, "block": 16}                     # configs[2], configs[0] (one device)
WEAK_BATCH = dict(GLOBAL_BATCH)   # weak scaling: each GPU runs the configuration's whole batch


def ranks_or_launch(args):
    """-> (world, rank, local_rank) of this process.  With WORLD_SIZE unset and --gpus N > 1, start
    the N ranks (fresh child processes; nothing here has touched the GPU) and exit with their
    status.  Fewer visible GPUs than asked for, or a launcher world that disagrees with --gpus, is
    an error (exit 3): a scaling line never silently reports another GPU count."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        n = 1 if args.gpus is None else args.gpus
        if n < 1:
            raise SystemExit("--gpus must be >= 1")
        if n > 1:
            from fastfourierconvolution_amd.launch import spawn_ranks, visible_gpus
            if not args.dry_run and visible_gpus() < n:
                print(f"[bench] --gpus {n} but only {visible_gpus()} GPU(s) visible", file=sys.stderr)
                sys.exit(3)
            sys.exit(spawn_ranks(os.path.abspath(__file__), sys.argv[1:], n))
        return 1, 0, 0
    world = int(env_world)
    if args.gpus is not None and args.gpus != world:
        print(f"[bench] --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(3)
    rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not args.dry_run and local >= torch.cuda.device_count():
        print(f"[bench] rank {rank}: LOCAL_RANK {local} but {torch.cuda.device_count()} GPU(s) visible",
              file=sys.stderr)
        sys.exit(3)
    return world, rank, local


def batch_plan(args, world, rank):
    """-> (global_batch, this rank's [start, stop) of it)"""
    from fastfourierconvolution_amd.distributed import shard_range
    if args.scaling == "strong":
        gb = args.global_batch or GLOBAL_BATCH[args.workload]
        if gb < world:
            raise SystemExit(f"global batch {gb} < {world} ranks")
        return gb, shard_range(gb, rank, world)
    per = args.batch or WEAK_BATCH[args.workload]
    return per * world, (rank * per, (rank + 1) * per)


def dry_run(args, world, rank):
    """The launch and shard plan over gloo on the CPU: every rank reports its batch slice and the
    checksum of its z slice; rank 0 checks they tile the global batch and prints one JSON line."""
    import torch.distributed as dist
    gb, (a, b) = batch_plan(args, world, rank)
    if world > 1:
        dist.init_process_group("gloo")
    fgan = args.workload in ("fgan128", "fgan128sn")
    zg = torch.randn((gb, 128) if fgan else (gb, args.nz, 1, 1), generator=torch.Generator().manual_seed(100))
    mine = torch.tensor([float(a), float(b), float(zg[a:b].double().sum())], dtype=torch.float64)
    parts = [torch.zeros_like(mine) for _ in range(world)]
    if world > 1:
        dist.all_gather(parts, mine)
    else:
        parts = [mine]
    if rank == 0:
        spans = [(int(p[0]), int(p[1])) for p in parts]
        ok = spans[0][0] == 0 and spans[-1][1] == gb and all(x[1] == y[0] for x, y in zip(spans, spans[1:]))
        zsum = sum(float(p[2]) for p in parts)
        print(json.dumps({"dry_run": True, "workload": args.workload, "n_gpus": world, "scaling": args.scaling,
                          "global_batch": gb, "per_gpu_batch": [b - a for a, b in spans], "spans": spans,
                          "tiles_global_batch": bool(ok and abs(zsum - float(zg.double().sum())) < 1e-6),
                          "parallelism": f"dp{world}" + ("+syncbn" if world > 1 and args.bn_mode == "train" else "")}))
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    world, rank, local = ranks_or_launch(args)
    if args.dry_run:
        return dry_run(args, world, rank)
    if args.workload == "block":
        if world > 1:
            raise SystemExit("block is the single-device configs[0] workload")
        return block_main(args)
    if args.workload == "fgan128train":
        if args.batch is None:
            args.batch = 64
        return fgan128train_main(args)
    if args.workload == "gan64train":
        if world > 1:
            raise SystemExit("gan64train is the single-GPU configs[2] workload")
        if args.batch is None:
            args.batch = 256
        return train_main(args)
    fgan = args.workload in ("fgan128", "fgan128sn")
    sn = args.workload == "fgan128sn"
    if args.mix is None:
        args.mix = "fp16" if sn else "fp32"
    global_batch, (b0, b1) = batch_plan(args, world, rank)
    args.batch = b1 - b0              # this rank's samples
    import torch.distributed as dist
    if world > 1:
        import datetime
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                timeout=datetime.timedelta(seconds=300))
    dev = torch.device("cuda", local)

    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt

    torch.manual_seed(1234)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FGenerator(128) if fgan else F.FFCGenerator(args.nz, args.nc, args.ngf)
    G.apply(weights_init)
    if sn:
        F.spectral_norm_ffc(G)          # SNFFC wrapping of l2l / l2g / g2l + ST conv1 / conv2
    F.set_mix_precision(G, args.mix)
    cpu_state = {k: v.clone() for k, v in G.state_dict().items()}
    G = G.to(dev).train(args.bn_mode == "train")
    if world > 1:
        from fastfourierconvolution_amd import distributed as D
        D.broadcast_module(G)           # weights + BN buffers from rank 0, once
        if args.bn_mode == "train":
            D.enable_sync_bn()          # the only data-path exchange: BN moments all-reduce
    elif args.syncbn_rehearsal and args.bn_mode == "train":
        import datetime
        from fastfourierconvolution_amd import distributed as D
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{29500 + os.getpid() % 2000}", rank=0,
                                world_size=1, device_id=torch.device("cuda", local),
                                timeout=datetime.timedelta(seconds=300))
        D.enable_sync_bn(even_world1=True)
    # one global z from one seed (weak or strong), this rank's slice: at N = 1 both modes time the
    # same batch, and at N > 1 the gathered output can be checked against the global-batch forward
    gen = torch.Generator(device="cpu").manual_seed(100)
    z_glob = torch.randn((global_batch, 128) if fgan else (global_batch, args.nz, 1, 1), generator=gen)
    z_cpu = z_glob[b0:b1].clone()
    z = z_cpu.to(dev)

    def step():
        with torch.no_grad():
            return G.forward_float(z) if fgan else G(z)

    for _ in range(max(1, args.warmup)):
        out = step()
    torch.cuda.synchronize()

    use_graph = not args.no_graph
    run = step
    if use_graph:
        # thread-local capture after a synchronise, and every rank agrees on graph vs eager BEFORE
        # the first replay (graphs.py: the RCCL watchdog and the round-2 exit 134)
        graph = capture_step(step, warmup=1)
        use_graph = graph is not None
        if use_graph:
            run = graph.replay

    for _ in range(max(1, args.warmup)):
        run()
    elapsed, med = time_steps(run, args.steps, world)
    value = global_batch * args.steps / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    weak = None
    if world > 1 and args.scaling == "strong":
        # beside the strong split: every GPU runs the configuration's whole batch (SURVEY.md §8e "report
        # weak scaling alongside"), z from the same seed, SyncBN over the N x larger global batch
        per = WEAK_BATCH[args.workload]
        zw = torch.randn((per * world, 128) if fgan else (per * world, args.nz, 1, 1),
                         generator=torch.Generator(device="cpu").manual_seed(100))[rank * per:(rank + 1) * per].to(dev)

        def step_w():
            with torch.no_grad():
                return G.forward_float(zw) if fgan else G(zw)
        for _ in range(max(1, args.warmup)):
            step_w()
        gw = capture_step(step_w, warmup=1) if use_graph else None
        run_w = gw.replay if gw is not None else step_w
        for _ in range(max(1, args.warmup)):
            run_w()
        el_w, med_w = time_steps(run_w, args.steps, world)
        weak = {"value": round(per * world * args.steps / el_w, 1), "unit": "images/s", "per_gpu_batch": per,
                "global_batch": per * world, "ms_per_step": round(el_w * 1e3 / args.steps, 4),
                "ms_per_step_median": round(med_w, 4), "hipgraph": gw is not None}
        del gw

    # ---- live per-kernel roofline: one instrumented eager pass (HIP events on the launch stream)
    summ, out = profile_pass(step, args.profile_steps)
    kernels = {k: {"launches_per_step": v["launches"] / max(1, args.profile_steps),
                   "ms_per_step": v["ms"] / max(1, args.profile_steps),
                   "avg_us": 1e3 * v["ms"] / v["launches"]} for k, v in summ.items()}
    dom = max(summ, key=lambda k: summ[k]["ms"])
    d = summ[dom]
    if d["flops"] > 0:
        achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
        roof = mfma_roof(dom, achieved)
    else:
        achieved = d["bytes"] / (d["ms"] * 1e-3) / 1e9
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4)}
    tr = pmc_traffic(dom, args.workload)
    roof["traffic"] = tr["bytes_per_launch"] if tr else None
    if tr:
        roof["traffic_source"] = tr["source"]
    fu = {k: summ[k] for k in ("fu_pass0", "fu_pass1", "fu2d_r2c", "fu2d_c2r") if k in summ}
    fft_roof = None
    if fu:
        b = sum(v["bytes"] for v in fu.values())
        ms = sum(v["ms"] for v in fu.values())
        mv = sum(v["moved"] for v in fu.values())
        fft_roof = {"kernel": "+".join(fu), "bound": "hbm", "achieved": round(b / (ms * 1e-3) / 1e9, 1),
                    "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(b / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                    "basis": "SURVEY.md §8d algorithmic bytes per launch (fused train FU 12*N_r, R2C 4*N_r + "
                             "8*N_c, C2R 8*N_c + 4*N_r; no spill counted), each capped at the bytes the launch "
                             "moves (the upsample-folded R2C reads t and writes T, 1/4 of the formula)",
                    "algorithmic_bytes_per_step": b / max(1, args.profile_steps),
                    "moved_bytes_per_step": mv / max(1, args.profile_steps),
                    "moved_frac": round(mv / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                    "ms_per_step": round(ms / max(1, args.profile_steps), 4),
                    "per_stage": {k: {"us_per_launch": round(1e3 * v["ms"] / v["launches"], 2),
                                      "frac": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
                                  for k, v in fu.items()}}

    # ---- CPU baseline + parity (rank 0, N=1 only); N > 1: the gathered sharded output (SyncBN)
    cpu = None
    parity = None
    # the timed artifact: the captured graph's static output after the timed replays (train-mode
    # BN: every replay computes the same output from the batch's own statistics)
    timed_out = getattr(graph, "ffc_output", None) if use_graph else None
    if world > 1 and not fgan and args.bn_mode == "train" and not args.no_cpu_baseline:
        parity = sharded_parity(args, step, cpu_state, z_glob, global_batch, rank, timed_out)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and fgan:
        cpu, parity = fgan_cpu_baseline(args, G, z_cpu, sn)
    elif rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.ffc_oracle import ffc_generator, normwise_err
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        torch.set_num_threads(threads)
        sd = {k: v.clone() for k, v in cpu_state.items()}
        training = args.bn_mode == "train"
        if not training:  # eval: use the GPU model's current running stats
            sd = {k: v.detach().cpu().clone() for k, v in G.state_dict().items()}
        with torch.no_grad():
            ref = ffc_generator(z_cpu, sd, args.nz, args.nc, args.ngf, training, fft="torch")
            iters, t0 = 1, time.perf_counter()
            while time.perf_counter() - t0 < args.cpu_seconds:
                ffc_generator(z_cpu, sd, args.nz, args.nc, args.ngf, training, fft="torch")
                iters += 1
            cpu_el = time.perf_counter() - t0
        with torch.no_grad():
            if timed_out is not None and training:
                torch.cuda.synchronize()
                gpu_out, source = timed_out.cpu(), "captured hipGraph's output after the timed replays"
            else:   # eval mode: the profile pass moved nothing, any forward is the timed one
                gpu_out, source = step().cpu(), "eager forward" if timed_out is None else \
                    "eager forward (eval-mode BN: the same kernels and running statistics as the graph)"
        parity = {"normwise_err_vs_cpu_ref": normwise_err(gpu_out, ref),
                  "max_abs_diff": float((gpu_out - ref).abs().max()), "tolerance": 1e-4, "checked": source}
        cpu = {"value": round(args.batch * (iters - 1) / cpu_el, 2), "unit": "images/s", "cores": threads,
               "kind": "port",
               "sample": f"oracle fp32 torch-CPU FFCGenerator fwd (op-for-op reference path), B={args.batch}, "
                         f"{iters - 1} timed iterations in {cpu_el:.1f}s, {args.bn_mode}-mode BN"}

    if rank == 0:
        metric = METRIC if not fgan else (
            f"fgan128 FGenerator{' + spectral norm, fp16 mix' if sn else ''} fwd images/sec @ B={global_batch // world}"
            f" per GPU 128x128x3 (BASELINE configs[{4 if sn else 3}])")
        line = {
            "metric": metric, "value": round(value, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "ms_per_step_median": round(med, 4), "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None,
            "dtype": "f32" if args.mix == "fp32" else "f32 (fp16 spectral mix)",
            "data": "synthetic: z ~ N(0,1); weights per fgan64_complete.py:22-31 weights_init",
            "config": {"workload": (f"fgan128 FGenerator(z=128, ngf=128){' + spectral norm (SNFFC)' if sn else ''} "
                                    "forward 128x128x3 (float output)" if fgan else
                                    f"FFCGenerator(nz={args.nz},nc={args.nc},ngf={args.ngf}) forward 64x64x{args.nc}"),
                       "global_batch": global_batch, "per_gpu_batch": args.batch, "bn_mode": args.bn_mode,
                       "spectral_mix": args.mix,
                       "hipgraph": use_graph, "parallelism": f"dp{world}" + ("+syncbn" if world > 1 and
                                                                          args.bn_mode == "train" else "")
                       + ("+syncbn-rehearsal(1-rank RCCL group)" if world == 1 and args.syncbn_rehearsal else "")},
            "roofline": roof, "fft_roofline": fft_roof, "cpu_baseline": cpu, "parity": parity,
            "kernels": kernels,
        }
        if weak is not None:
            line["weak_scaling"] = weak
        print(json.dumps(line))
    if world > 1 or (args.syncbn_rehearsal and dist.is_initialized()):
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
