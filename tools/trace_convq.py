#!/usr/bin/env python3
"""Where the cycles of ffc_convq_forward go (diagnostic build only).

    VARIANT_FLAGS=-DFFC_TRACE_Q tools/build_variant.sh traceq - && \\
    FFC_LIB_PATH=fastfourierconvolution_amd/libffc_amd_traceq.so python tools/trace_convq.py <layer> <B> <cfg>

Runs one FFCTranspose layer's conv launch (tools/convq_probe.py shapes) and prints, over the
workgroups: launch span, workgroup durations, and the per-section cycles of compute wave 0 and
staging wave 4 (s_memtime stamps; they serialise the sections they bracket, so read shares)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
li, B, cfg = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
model = sys.argv[4] if len(sys.argv) > 4 else "gen64"
sys.argv = [sys.argv[0], str(B), model]
os.environ["FFC_CONVQ_CFG"] = cfg
import convq_probe as P  # noqa: E402

C, IH, M, c = P.LAYERS[li]
us, tf, keys = P.time_layer(P.job_pair(C, IH, M, c), reps=3)
L = P.rt.lib()
read = L.ffc_debug_trace_read_q
read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
read.restype = ctypes.c_int
ntiles = int(keys.split(":")[-2])
buf = np.zeros((ntiles, 16), dtype=np.uint64)
assert read(buf.ctypes.data, buf.nbytes) == 0
rt0, rt1 = buf[:, 0].astype(np.float64), buf[:, 1].astype(np.float64)
span = (rt1.max() - rt0.min()) / 100.0   # realtime counter: 100 MHz
dur = (rt1 - rt0) / 100.0
print(f"layer {li} B={B} cfg {cfg}: {us:.1f} us/launch (events), {ntiles} workgroups, traced span {span:.1f} us, "
      f"workgroup {dur.mean():.2f} us mean / {dur.max():.2f} max")
names = ["barrier", "A issue", "MFMA taps", "direct", "epilogue", "total"]
cw = buf[:, 3:9].astype(np.float64)
print("compute wave 0 (kcycles mean): " + ", ".join(f"{n} {v / 1e3:.2f}" for n, v in zip(names, cw.mean(0))))
sw = buf[:, [9, 10, 11, 14, 12]].astype(np.float64)
print("staging wave 4 (kcycles mean): " + ", ".join(f"{n} {v / 1e3:.2f}" for n, v in
                                                 zip(["loads", "split+store", "barrier", "issue", "total"], sw.mean(0))) +
      f", chunks {buf[:, 13].mean():.1f}")
cu = (buf[:, 2] & 0xF00) >> 8
print(f"workgroups per (XCC, CU): max {np.bincount(((buf[:, 2] >> 32) & 7) * 16 + cu).max()}")
