"""Per-stage timing of the large-plane Fourier unit (fgan128 conv5/conv6 FUs, fgan128_complete.py:474-485).

    python tools/bench_fu2d.py [--batch 64] [--c 32] [--n 128] [--iters 20]

Runs FourierUnitSN's staged path inside SpectralTransform(2c, 2c, stride=2, upsample=True) on a
(B, 2c, n/2, n/2) input and reports, per stage, HIP-event time and achieved GB/s on the bytes the
stage must move (r2c: t + T, mix pass 0: T, mix pass 1: T + Y, c2r: Y + t + out).
"""
import argparse
import contextlib
import io
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--c", type=int, default=32)
    p.add_argument("--n", type=int, default=128)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--eval", action="store_true")
    a = p.parse_args()
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        st = F.SpectralTransform(2 * a.c, 2 * a.c, stride=2, upsample=True).cuda().train(not a.eval)
    x = torch.randn((a.batch, 2 * a.c, a.n // 2, a.n // 2), device="cuda")
    with torch.no_grad():
        for _ in range(3):
            st.spectral(x)
        torch.cuda.synchronize()
        obs = rt.LaunchObserver()
        rt.set_observer(obs)
        for _ in range(a.iters):
            st.spectral(x)
        rt.set_observer(None)
    summ = obs.summary()
    res = {}
    for k, v in summ.items():
        ms = v["ms"] / v["launches"]
        res[k] = {"avg_us": round(1e3 * ms, 2), "GB/s": round(v["bytes"] / v["launches"] / (ms * 1e-3) / 1e9, 1),
                  "frac_hbm": round(v["bytes"] / v["launches"] / (ms * 1e-3) / 8e12, 3),
                  "TF/s": round(v["flops"] / v["launches"] / (ms * 1e-3) / 1e12, 2)}
    print(json.dumps({"B": a.batch, "c": a.c, "n": a.n, "train": not a.eval, "stages": res}, indent=1))


if __name__ == "__main__":
    main()
