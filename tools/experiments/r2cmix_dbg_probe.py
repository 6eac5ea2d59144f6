"""DESIGN 10c probe (libffc_amd_chfdbg.so: FFC_R2CMIX_CHFOLD + FFC_R2CMIX_DBG): per-workgroup checksums
of fu2d_r2c_mix's stages -- bn1 scale / shift, the bn1-transformed planes R, T after the row FFTs, T
after the column FFTs -- compared between the workgroups of one sample (the bin-range splits all
recompute the same T) and across repeated runs."""
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
rd = L.ffc_debug_r2cmix_read
rd.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
SLOTS = ["scale", "shift", "sumR", "T_rows|mixM2(end)", "T_cols"]
for B in (64, 86):
    torch.manual_seed(64 + B)
    with contextlib.redirect_stdout(io.StringIO()):
        st = F.SpectralTransform(64, 32, stride=2, upsample=True)
    st = st.cuda().train()
    x = torch.randn((B, 64, 16, 16)).cuda()
    nwg = L.ffc_fu2d_slab_rows(B, 16, 32, 32)
    nsplit = nwg // B
    runs, outs = [], []
    for rep in range(30):
        m = copy.deepcopy(st)
        with torch.no_grad():
            outs.append(m(x).clone())
        torch.cuda.synchronize()
        buf = np.zeros((4096, 5, 32), dtype=np.float32)
        assert rd(buf.ctypes.data, buf.nbytes) == 0
        runs.append(buf[:nwg, :, :16].copy())   # (mix M2 of channels 0..15 in slot 3 for DBGEND)
    ndiff = sum(not torch.equal(o, outs[0]) for o in outs)
    within = Counter()
    wgs = Counter()
    for r in runs:
        a = r.reshape(nsplit, B, 5, 16)
        d = a != a[0:1]
        for sp, b, sl, ch in zip(*np.nonzero(d)):
            within[(SLOTS[sl], int(ch))] += 1
            wgs[int(sp * B + b) >= 256] += 1
    across = Counter()
    for r in runs[1:]:
        d = r != runs[0]
        for wg, sl, ch in zip(*np.nonzero(d)):
            across[SLOTS[sl]] += 1
    print(f"B={B} nsplit={nsplit}: outputs differ in {ndiff}/30 runs; within-run WG mismatches by (stage, ch): "
          f"{sorted(within.items())[:24]}; by blockIdx>=256: {dict(wgs)}; across runs by stage: {dict(across)}",
          flush=True)
