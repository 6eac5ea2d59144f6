"""Ordered per-launch timing of one eager forward (HIP events on the launch stream).

    python tools/trace_launches.py [--workload gen64|fgan128] [--batch B] [--eval]

Prints each library launch in issue order with its label, duration, and achieved TF/s or GB/s
on the launch's algorithmic work (the numbers bench.py aggregates per label).
"""
import argparse
import contextlib
import io
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", choices=["gen64", "fgan128"], default="fgan128")
    p.add_argument("--batch", type=int, default=None)
    p.add_argument("--eval", action="store_true")
    a = p.parse_args()
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    from bench import weights_init
    fgan = a.workload == "fgan128"
    B = a.batch or (64 if fgan else 256)
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FGenerator(128) if fgan else F.FFCGenerator(100, 3, 64)
    G.apply(weights_init)
    G = G.cuda().train(not a.eval)
    z = torch.randn((B, 128) if fgan else (B, 100, 1, 1), device="cuda")
    fwd = G.forward_float if fgan else G
    with torch.no_grad():
        for _ in range(3):
            fwd(z)
        torch.cuda.synchronize()
        obs = rt.LaunchObserver()
        rt.set_observer(obs)
        fwd(z)
        rt.set_observer(None)
    torch.cuda.synchronize()
    tot = 0.0
    for label, e0, e1, work in obs.records:
        ms = e0.elapsed_time(e1)
        tot += ms
        rate = ""
        if work.get("flops"):
            rate = f"{work['flops'] / (ms * 1e-3) / 1e12:7.1f} TF/s  ({work['flops'] / 1e9:.2f} GF)"
        elif work.get("bytes"):
            rate = f"{work['bytes'] / (ms * 1e-3) / 1e9:7.0f} GB/s  ({work['bytes'] / 1e6:.1f} MB)"
        print(f"{label:14s} {1e3 * ms:9.1f} us  {rate}")
    print(f"total {1e3 * tot:.1f} us over {len(obs.records)} launches")


if __name__ == "__main__":
    main()
