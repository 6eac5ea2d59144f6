import sys, torch
sys.path.insert(0, '.')
from fastfourierconvolution_amd import _runtime as rt, _plan
torch.manual_seed(0)
dev = torch.device("cuda")
for (B, C, M, H) in [(4, 100, 4096, 1), (8, 100, 256, 1), (8, 16, 32, 1), (4, 16, 32, 2), (4, 16, 32, 3), (4, 16, 32, 8), (2, 20, 40, 6)]:
    x = torch.randn(B, C, H, H, device=dev)
    w = torch.randn(M, C, 1, 1, device=dev)
    ref = torch.nn.functional.conv2d(x, w)
    for patch in (True, False):
        rt.USE_PATCH = patch
        ex = rt.ConvExec(B, M, [_plan.Seg("pw", C, H, H)], [(w, 0, 1, 1, None)], dev)
        lp = rt.LaunchPlan([ex], dev)
        out = torch.empty(B, M, H, H, device=dev)
        lp.launch([ex.job([(x, None)], out)], torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        extra = f"NS {ex.plan.NS} TR {ex.plan.TR} TC {ex.plan.TC} vec4 {ex.plan.vec4} rowlen {ex.plan.rowlen} prc {ex.plan.prc}" if ex.kind == "patch" else ""
        print(B, C, M, H, ex.kind, "cfg", lp.cfg, "err", float((out - ref).abs().max() / ref.abs().max()), extra, flush=True)
