#!/usr/bin/env python3
"""Phase timeline of the ST-prologue and Fourier-unit kernels (diagnostic build only).

    VARIANT_FLAGS=-DFFC_TRACE tools/build_variant.sh trace - && \
    FFC_LIB_PATH=fastfourierconvolution_amd/libffc_amd_trace.so python tools/trace_spectral.py

Per launch: span, workgroup duration, and the mean cycles wave 0 spent between the phase
stamps of the kernel (fu_kernels.hip FU_STAMP / st_prologue.hip ST_STAMP).  Shares, not
absolute times: the stamps serialise what the real kernels overlap.
"""
import contextlib
import ctypes
import io
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = {
    "fu0": ["rows R2C", "col FFT", "mix+stats", "-", "merge+slab"],
    "fu0kg": ["bn1 fold", "rows R2C", "col FFT", "mix+stats", "merge+slab"],
    "fu1": ["rows R2C", "col FFT", "mix+BN/ReLU", "inv col FFT", "rows C2R+store"],
    "st": ["load x (+w)", "SE gate", "conv1 MFMA", "slab merge"],
}


def main():
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    torch.manual_seed(1234)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FFCGenerator(100, 3, 64)
    G = G.cuda().train()
    z = torch.randn(int(os.environ.get("TRACE_B", "256")), 100, 1, 1, device="cuda")
    with torch.no_grad():
        for _ in range(3):
            G(z)
    torch.cuda.synchronize()
    L = rt.lib()
    rfu, rst = L.ffc_debug_fu_trace_read, L.ffc_debug_st_trace_read
    for f in (rfu, rst):
        f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    recs = []
    ofu, ost = L.ffc_fu_forward_ex4, L.ffc_st_prologue_ex3

    def fu(*a):   # ffc_fu_forward_ex4: pass a[11], kgroups a[20]
        rc = ofu(*a)
        torch.cuda.synchronize()
        kg = a[20] if a[11] == 0 else 1
        buf = np.zeros((a[1] * kg, 8), dtype=np.uint64)
        assert rfu(buf.ctypes.data, buf.nbytes) == 0
        recs.append((f"fu{a[11]}" + ("kg" if kg > 1 else ""), f"C={a[2]} {a[3]}x{a[4]} up={a[5]}", buf))
        return rc

    def st(*a):
        rc = ost(*a)
        torch.cuda.synchronize()
        B = a[1] * a[12]   # workgroups: samples x split
        buf = np.zeros((B, 8), dtype=np.uint64)
        assert rst(buf.ctypes.data, buf.nbytes) == 0
        recs.append(("st", f"Cin={a[2]} {a[3]}x{a[4]} c={a[11]} split={a[12]}", buf))
        return rc

    L.ffc_fu_forward_ex4, L.ffc_st_prologue_ex3 = fu, st
    with torch.no_grad():
        G(z)
    L.ffc_fu_forward_ex4, L.ffc_st_prologue_ex3 = ofu, ost
    for kind, desc, buf in recs:
        if not buf[:, 0].any():   # a kernel without stamps (the split pass 1)
            continue
        rt0, rt1 = buf[:, 0].astype(np.float64), buf[:, 1].astype(np.float64)
        dur = (rt1 - rt0) / 100.0
        names = PHASES[kind]
        st = buf[:, 2:2 + len(names) + 1].astype(np.float64)
        d = np.diff(st, axis=1)
        d[d < 0] = 0
        tot = st[:, -1] - st[:, 0]
        clk = np.median(tot / np.maximum(rt1 - rt0, 1) * 100e6) / 1e9
        parts = "  ".join(f"{n} {100 * d[:, i].mean() / tot.mean():.0f}%" for i, n in enumerate(names) if n != "-")
        print(f"{kind:4s} {desc:24s} span {(rt1.max() - rt0.min()) / 100:.1f} us  WG mean {dur.mean():.1f} "
              f"max {dur.max():.1f} us  clk {clk:.2f}  | {parts}")


if __name__ == "__main__":
    main()
