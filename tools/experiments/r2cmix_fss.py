"""Debug probe (libffc_amd_rm5.so): every r2c_mix workgroup's bn1 scale / shift, stored in the stats
slab's 4th slot, compared across workgroups and with the leader's scale_out / shift_out."""
import contextlib
import copy
import io
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import fastfourierconvolution_amd as F
from fastfourierconvolution_amd import _runtime as rt

L = rt.lib()
orig = L.ffc_fu2d_r2c_mix
made = []
_empty = torch.empty
cap = {}


def spy(t, B, C, H, W, up, isc, ish, relu, fold, wmix, slab, Y, stream):
    rc = orig(t, B, C, H, W, up, isc, ish, relu, fold, wmix, slab, Y, stream)
    cap.update(slab=slab, B=B, C=C, rows=L.ffc_fu2d_slab_rows(B, C, H, W))
    return rc


L.ffc_fu2d_r2c_mix = spy


def rec(*a, **k):
    t = _empty(*a, **k)
    made.append(t)
    return t


torch.manual_seed(7)
with contextlib.redirect_stdout(io.StringIO()):
    st = F.SpectralTransform(64, 32, stride=2, upsample=True)
st = st.cuda().train()
B = 64
x = torch.randn((B, 64, 16, 16)).cuda()
for rep in range(12):
    m = copy.deepcopy(st)
    made.clear()
    torch.empty = rec
    try:
        with torch.no_grad():
            m(x)
    finally:
        torch.empty = _empty
    torch.cuda.synchronize()
    slab = {t.data_ptr(): t for t in made}[cap["slab"]].clone().view(cap["rows"], 2 * cap["C"], 4)
    w = slab[:, :, 3]                 # [rows = split * B + b][2C]
    if os.environ.get("PROBE_T"):
        # T checksums: every split of a sample must agree
        Bn = cap["B"]
        ws = w.view(-1, Bn, w.shape[1])      # [split][b][2C]
        bad = (ws != ws[0:1]).any(dim=2)     # [split][b]
        lst = bad.nonzero().tolist()
        Cc = cap["C"]
        det = []
        for sp, b in lst[:6]:
            dR = (ws[sp, b, :Cc] != ws[0, b, :Cc]).nonzero().flatten().tolist()
            dT = (ws[sp, b, Cc:] != ws[0, b, Cc:]).nonzero().flatten().tolist()
            det.append((sp, b, "R ch", dR, "T ch", dT))
        print(f"rep {rep}: {len(lst)} (split, sample) workgroups differing from split 0: {det}", flush=True)
        continue
    ref = w[0]
    bad = (w != ref).any(dim=1).nonzero().flatten().tolist()
    info = [(r, r % cap["B"], r // cap["B"], (w[r] - ref).abs().max().item()) for r in bad[:6]]
    print(f"rep {rep}: {len(bad)} of {w.shape[0]} workgroups with a different bn1 scale/shift: "
          f"(row, sample, split, max|d|) {info}", flush=True)
