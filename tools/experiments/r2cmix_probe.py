"""Debug probe: ffc_fu2d_r2c_mix vs ffc_fu2d_r2c + ffc_fu2d_mix(pass 0, spill) on random inputs through
the C ABI (in_scale / in_shift bn1, no fold): max |dY| and slab differences per (B, C, H)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from fastfourierconvolution_amd import _runtime as rt
from fastfourierconvolution_amd._runtime import ptr

L = rt.lib()
for B, C, H in [(6, 16, 32), (32, 16, 32), (86, 16, 32), (86, 32, 16), (32, 32, 16), (128, 16, 32)]:
    up, h = 2, H // 2
    g = torch.Generator().manual_seed(B + C)
    t = torch.randn((B, C, h, h), generator=g).cuda()
    sc = (torch.rand(C, generator=g) + 0.5).cuda()
    sh = (torch.rand(C, generator=g) - 0.5).cuda()
    C2, Mpad = 2 * C, (2 * C + 31) // 32 * 32
    w = torch.randn((C2, C2), generator=g) / C2 ** 0.5
    wT = torch.zeros((C2, Mpad))
    wT[:, :C2] = w.t()
    wT = wT.cuda().contiguous()
    rows = L.ffc_fu2d_slab_rows(B, C, H, H)
    s = torch.cuda.current_stream().cuda_stream
    T = torch.empty((B, C, h, h // 2 + 1, 2), device="cuda")
    Y1 = torch.zeros((B, C, H, H // 2 + 1, 2), device="cuda")
    Y2 = torch.zeros_like(Y1)
    sl1 = torch.zeros((rows, C2, 4), device="cuda")
    sl2 = torch.zeros_like(sl1)
    assert L.ffc_fu2d_r2c_ex(ptr(t), B, C, h, h, ptr(sc), ptr(sh), 1, None, ptr(T), s) == 0
    assert L.ffc_fu2d_mix(ptr(T), B, C, H, H, up, ptr(wT), 0, ptr(sl1), None, None, ptr(Y1), s) == 0
    assert L.ffc_fu2d_r2c_mix(ptr(t), B, C, H, H, up, ptr(sc), ptr(sh), 1, None, ptr(wT), ptr(sl2), ptr(Y2), s) == 0
    torch.cuda.synchronize()
    dy = (Y1 - Y2).abs().max().item()
    bad = ((Y1 - Y2).abs() > 1e-3 * (Y1.abs().max())).nonzero()
    ds = (sl1 - sl2).abs().max().item()
    print(f"B={B} C={C} H={H} rows={rows} max|dY|={dy:.3e} (|Y|max {Y1.abs().max().item():.3e}) "
          f"max|dslab|={ds:.3e} bad={bad.shape[0]} first={bad[:4].tolist()}", flush=True)

# the SpectralTransform level with the bn1 fold (as tests/test_gpu_bn_fold.py), at B = 86
import copy, contextlib, io
import fastfourierconvolution_amd as F
for cin, cout, hw, B in [(64, 32, 16, 86), (128, 64, 8, 86), (64, 32, 16, 64), (64, 32, 16, 32)]:
    torch.manual_seed(cin + B)
    with contextlib.redirect_stdout(io.StringIO()):
        st = F.SpectralTransform(cin, cout, stride=2, upsample=True)
    st = st.cuda().train()
    x = torch.randn((B, cin, hw, hw)).cuda()
    outs = []
    for flag in (False, True):
        rt.FU2D_R2CMIX = flag
        m = copy.deepcopy(st)
        with torch.no_grad():
            outs.append(m(x).clone())
    torch.cuda.synchronize()
    d = (outs[0] - outs[1]).abs().max().item()
    print(f"ST cin={cin} cout={cout} hw={hw} B={B} split={L.ffc_st_prologue_split(B, cin, hw, hw, 0, cout // 2)} "
          f"max|d|={d:.3e} |out|max={outs[0].abs().max().item():.3e}", flush=True)
