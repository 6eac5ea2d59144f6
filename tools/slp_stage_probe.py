"""Stage-by-stage comparison of the staged Fourier unit (csrc/fu2d_kernels.hip) between two library
builds, on identical inputs: the 32x32 unit of FFCGenerator ffc3 at B = 8 (t: (8, 16, 16, 16),
x2 upsample folded in, bn1 affine + ReLU on load, train-mode BN).  Names the fu2d kernel of a
build-flag-dependent miscompare (tools/slp_probe.py names the layer first).

    FFC_LIB_PATH=<reference build> python tools/slp_stage_probe.py ref <file.pt>
    FFC_LIB_PATH=<suspect build>   python tools/slp_stage_probe.py cmp <file.pt>
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from fastfourierconvolution_amd import _lib  # noqa: E402


def stages(L, d, s):
    """run r2c, mix pass 0 and c2r_bn on the tensors of d; -> their outputs"""
    B, C, h, w, up = 8, 16, 16, 16, 2
    H, W = h * up, w * up
    T = torch.zeros((B, C, h, w // 2 + 1, 2), device="cuda")
    assert L.ffc_fu2d_r2c(d["t"].data_ptr(), B, C, h, w, d["isc"].data_ptr(), d["ish"].data_ptr(), 1, T.data_ptr(),
                          s) == 0, L.ffc_last_error()
    rows = L.ffc_fu2d_slab_rows(B, C, H, W)
    slab = torch.zeros((rows, 2 * C, 4), device="cuda")
    Y = torch.zeros((B, C, H, W // 2 + 1, 2), device="cuda")
    Tin = d.get("T", T)
    assert L.ffc_fu2d_mix(Tin.data_ptr(), B, C, H, W, up, d["mixT"].data_ptr(), 0, slab.data_ptr(), None, None,
                          Y.data_ptr(), s) == 0, L.ffc_last_error()
    out = torch.zeros((B, C, H, W), device="cuda")
    Yin = d.get("Y", Y)
    assert L.ffc_fu2d_c2r_bn(Yin.data_ptr(), B, C, H, W, d["t"].data_ptr(), up, d["isc"].data_ptr(),
                             d["ish"].data_ptr(), 1, 1, d["sc"].data_ptr(), d["sh"].data_ptr(), out.data_ptr(),
                             s) == 0, L.ffc_last_error()
    torch.cuda.synchronize()
    return {"T": T, "slab": slab, "Y": Y, "out": out}


def main():
    mode, path = sys.argv[1], sys.argv[2]
    L = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    if mode == "ref":
        g = torch.Generator().manual_seed(3)
        C = 16
        d = {"t": torch.randn(8, C, 16, 16, generator=g), "isc": 0.5 + torch.rand(C, generator=g),
             "ish": 0.1 * torch.randn(C, generator=g), "sc": 0.5 + torch.rand(2 * C, generator=g),
             "sh": 0.1 * torch.randn(2 * C, generator=g), "w": torch.randn(2 * C, 2 * C, generator=g) / 6}
        d = {k: v.cuda() for k, v in d.items()}
        d["mixT"] = torch.zeros((2 * C, 32), device="cuda")
        assert L.ffc_fu_pack_mix(d["w"].data_ptr(), 2 * C, d["mixT"].data_ptr(), s) == 0
        res = stages(L, d, s)
        torch.save({"in": {k: v.cpu() for k, v in d.items()}, "out": {k: v.cpu() for k, v in res.items()}}, path)
        print("reference stages written", {k: float(v.abs().max()) for k, v in res.items()})
        return
    ref = torch.load(path, weights_only=True)
    d = {k: v.cuda() for k, v in ref["in"].items()}
    # each stage on the reference build's inputs to it (T and Y from the reference), then chained
    iso = stages(L, dict(d, T=ref["out"]["T"].cuda(), Y=ref["out"]["Y"].cuda()), s)
    chain = stages(L, d, s)
    for name, res in (("isolated", iso), ("chained", chain)):
        for k in ("T", "slab", "Y", "out"):
            a, b = res[k].cpu(), ref["out"][k]
            err = float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))
            print(f"{name:9s} {k:5s} normwise {err:.3e}  nan {int(torch.isnan(a).sum())}")


if __name__ == "__main__":
    main()
