#!/usr/bin/env python3
"""Per-workgroup timeline of the LDS-patch conv kernel (diagnostic build only).

    VARIANT_FLAGS=-DFFC_TRACE tools/build_variant.sh trace - && \
    FFC_LIB_PATH=fastfourierconvolution_amd/libffc_amd_trace.so python tools/trace_convp.py

Runs the bench workload eagerly, synchronises after every ffc_convp_forward and reads the
per-workgroup stamps (start/end realtime, CU id, wave-0 cycles in barrier / staging issue /
MFMA sections).  Prints, per launch: span, per-job workgroup durations, the load balance over
CUs (busy time of the busiest CU vs the mean) and where wave 0's cycles went.  Read shares,
not absolute times: the stamps serialise what the real kernel overlaps.
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


def main():
    import fastfourierconvolution_amd as F
    from fastfourierconvolution_amd import _runtime as rt
    B = int(os.environ.get("TRACE_BATCH", "256"))
    torch.manual_seed(1234)
    with contextlib.redirect_stdout(io.StringIO()):
        G = F.FFCGenerator(100, 3, 64)
    for m in G.modules():
        if "Conv" in type(m).__name__ and hasattr(m, "weight"):
            torch.nn.init.normal_(m.weight, 0.0, 0.02)
    G = G.cuda().train()
    z = torch.randn(B, 100, 1, 1, device="cuda")
    with torch.no_grad():
        for _ in range(3):
            G(z)
    torch.cuda.synchronize()
    L = rt.lib()
    read = L.ffc_debug_trace_read
    read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    launches = []

    orig_launch = rt.LaunchPlan.launch

    def launch(self, jobs, stream, flops=0.0):
        orig_launch(self, jobs, stream, flops)
        if self.key[0] != "patch":
            return
        torch.cuda.synchronize()
        buf = np.zeros((self.ntiles, 8), dtype=np.uint64)
        assert read(buf.ctypes.data, buf.nbytes) == 0
        launches.append((self.cfg, len(jobs), self.ntiles, buf, self.tiles.cpu().numpy().reshape(-1, 4)))

    rt.LaunchPlan.launch = launch
    with torch.no_grad():
        G(z)
    rt.LaunchPlan.launch = orig_launch
    for i, (cfg, njobs, ntiles, buf, tiles) in enumerate(launches):
        job = tiles[:, 0]   # int4 {job, m0, pixel block, 0} per workgroup
        rt0, rt1 = buf[:, 0].astype(np.float64), buf[:, 1].astype(np.float64)
        span_us = (rt1.max() - rt0.min()) / 100.0        # s_memrealtime: 100 MHz
        dur = (rt1 - rt0) / 100.0
        cyc = buf[:, 6].astype(np.float64)
        clk = np.median(cyc / np.maximum(rt1 - rt0, 1) * 100e6) / 1e9
        hw = buf[:, 2]
        cu = ((hw >> np.uint64(32)) & np.uint64(0xF)) * np.uint64(1 << 16) + ((hw >> np.uint64(8)) & np.uint64(0xFF))
        ucu, inv = np.unique(cu, return_inverse=True)
        busy = np.zeros(len(ucu))
        cnt = np.zeros(len(ucu))
        first = np.full(len(ucu), np.inf)
        last = np.zeros(len(ucu))
        for k in range(ntiles):
            busy[inv[k]] += dur[k]
            cnt[inv[k]] += 1
            first[inv[k]] = min(first[inv[k]], rt0[k])
            last[inv[k]] = max(last[inv[k]], rt1[k])
        print(f"launch {i}: cfg {cfg} jobs {njobs} tiles {ntiles}  span {span_us:.1f} us  clock {clk:.2f} GHz  "
              f"CUs used {len(ucu)}  WGs/CU min {cnt.min():.0f} max {cnt.max():.0f}")
        occ = (last - first) / 100.0
        print(f"   per-CU active span us: mean {occ.mean():.1f} max {occ.max():.1f} min {occ.min():.1f}; "
              f"start skew {(first.max() - first.min()) / 100:.1f} us")
        for j in range(njobs):
            sel = job == j
            if sel.any():
                d = dur[sel]
                f = buf[sel][:, 3:6].astype(np.float64).sum(0) / buf[sel][:, 6].astype(np.float64).sum()
                pe = buf[sel][:, 7]
                tot = buf[sel][:, 6].astype(np.float64).sum()
                pro = (pe & np.uint64(0xFFFFFFFF)).astype(np.float64).sum() / tot
                epi = (pe >> np.uint64(32)).astype(np.float64).sum() / tot
                print(f"   job {j}: {sel.sum()} WGs  dur us mean {d.mean():.1f} min {d.min():.1f} max {d.max():.1f}  "
                      f"wave0 share: prologue {pro:.2f} barrier {f[0]:.2f} stage {f[1]:.2f} mfma {f[2]:.2f} "
                      f"epilogue {epi:.2f}")


if __name__ == "__main__":
    main()
