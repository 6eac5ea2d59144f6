"""DESIGN 10c probe (libffc_amd_chfdump.so: FFC_R2CMIX_CHFOLD + FFC_R2CMIX_DUMP): fu2d_r2c_mix's T plane
(LDS) after the row FFTs and at the end of every workgroup, compared element by element between the
workgroups of one sample (every bin-range split recomputes the same T)."""
import contextlib
import copy
import ctypes
import io
import os
import sys
from collections import Counter

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import fastfourierconvolution_amd as F
from fastfourierconvolution_amd import _runtime as rt

L = rt.lib()
rd = L.ffc_debug_r2cmix_dump
rd.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
B, C, HT, WPT = 64, 16, 16, 9
torch.manual_seed(128)
with contextlib.redirect_stdout(io.StringIO()):
    st = F.SpectralTransform(64, 32, stride=2, upsample=True)
st = st.cuda().train()
x = torch.randn((B, 64, 16, 16)).cuda()
nwg = L.ffc_fu2d_slab_rows(B, C, 32, 32)
nsplit = nwg // B
shown = 0
for rep in range(30):
    m = copy.deepcopy(st)
    with torch.no_grad():
        m(x)
    torch.cuda.synchronize()
    buf = np.zeros((512, 2, 4608), dtype=np.float32)
    assert rd(buf.ctypes.data, buf.nbytes) == 0
    # Tl: float2 [ch][y][k] (row r = ch * HT + y, stride WPT) -> (ch, y, k, re/im)
    T = buf[:nwg].reshape(nsplit, B, 2, C, HT, WPT, 2)
    bad = T != T[0:1]
    if not bad.any():
        continue
    for sp, b in sorted({(int(a), int(c)) for a, c in zip(*np.nonzero(bad.any(axis=(2, 3, 4, 5, 6))))})[:3]:
        for slot, name in ((0, "after rows"), (1, "at end")):
            d = bad[sp, b, slot]
            if not d.any():
                print(f"rep {rep} wg {sp * B + b} (split {sp}, sample {b}) {name}: equal", flush=True)
                continue
            chs = sorted(set(np.nonzero(d)[0].tolist()))
            desc = []
            for ch in chs:
                yk = np.nonzero(d[ch].any(axis=2))
                ys, ks = sorted(set(yk[0].tolist())), sorted(set(yk[1].tolist()))
                desc.append(f"ch {ch}: rows y {ys} cols k {ks} ({int(d[ch].sum())} values)")
            print(f"rep {rep} wg {sp * B + b} (split {sp}, sample {b}) {name}: " + "; ".join(desc), flush=True)
            if slot == 0 and shown < 3:
                ch = chs[0]
                yk = np.nonzero(d[ch].any(axis=2))
                y0 = int(yk[0][0])
                got, want = T[sp, b, 0, ch, y0], T[0, b, 0, ch, y0]
                print(f"   got  ch {ch} y {y0}: {np.round(got[:, 0], 4).tolist()}", flush=True)
                print(f"   want ch {ch} y {y0}: {np.round(want[:, 0], 4).tolist()}", flush=True)
                # where else in this run's dumps does the stale row occur?  (any WG, any slot, ch, y)
                flat = T.reshape(-1, WPT, 2)
                hits = np.nonzero(np.all(np.isclose(flat, got, rtol=0, atol=1e-6), axis=(1, 2)))[0]
                locs = [np.unravel_index(h, (nsplit, B, 2, C, HT)) for h in hits[:6]]
                print(f"   the stale row equals rows at (split, sample, slot, ch, y): {[tuple(int(v) for v in l) for l in locs]}"
                      f" (R2C of other samples?)", flush=True)
                print(f"   stale row all zero: {bool(np.all(got == 0))}", flush=True)
        shown += 1
    if shown >= 12:
        break
print("done", flush=True)
