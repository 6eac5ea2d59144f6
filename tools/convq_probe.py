"""Per-layer timing of the stride-2 ConvT launches (out_l + out_g jobs of one FFCTranspose layer,
conv2 folded in) on ffc_convq_forward for every cfg and on ffc_convp_forward, HIP events over
repeated launches.  Diagnostic only.   usage: convq_probe.py [B] [gen64|fgan128]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fastfourierconvolution_amd import _plan, _runtime as rt  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 256
model = sys.argv[2] if len(sys.argv) > 2 else "gen64"
dev = torch.device("cuda", 0)
# (C_l = C_g in, IH, M_l = M_g out, c of the ST = conv2 input channels)
LAYERS_ALL = {"gen64": [(256, 4, 128, 64), (128, 8, 64, 32), (64, 16, 32, 16)],
              # fgan128 (ngf 128) conv2 (local input only: c = 0) and conv3..conv6: in_cl = in_cg = C,
              # out_l = out_g = M, ST c = M / 2
              "fgan128": [(1024, 4, 256, 0), (256, 8, 128, 64), (128, 16, 64, 32), (64, 32, 64, 32),
                          (64, 64, 64, 32)]}
LAYERS = LAYERS_ALL.get(model, LAYERS_ALL["gen64"])


def job_pair(C, IH, M, c):
    g = torch.Generator().manual_seed(C + IH)
    xl = torch.randn(B, C, IH, IH, generator=g).to(dev)
    xg = torch.randn(B, C, IH, IH, generator=g).to(dev)
    v = torch.randn(B, max(c, 1), 2 * IH, 2 * IH, generator=g).to(dev)
    wl = torch.randn(C, M, 4, 4, generator=g).to(dev) * 0.02
    wg = torch.randn(C, M, 4, 4, generator=g).to(dev) * 0.02
    wlg = torch.randn(C, M, 4, 4, generator=g).to(dev) * 0.02
    w2 = torch.randn(M, max(c, 1), 1, 1, generator=g).to(dev) * 0.02
    segT = _plan.Seg("convT", C, IH, IH, 4, 2, 1)
    if c == 0:   # FFCTranspose with ratio_gin 0: out_l = l2l(x_l), out_g = l2g(x_l)
        return [([segT], [(wl, 1, 4, 4, None)], [xl]), ([segT], [(wlg, 1, 4, 4, None)], [xl])]
    jobs = [([segT, segT], [(wl, 1, 4, 4, None), (wg, 1, 4, 4, None)], [xl, xg]),
            ([segT, _plan.Seg("pw", c, 2 * IH, 2 * IH)], [(wlg, 1, 4, 4, None), (w2, 0, 1, 1, None)], [xl, v])]
    return jobs


def time_layer(jobs, reps=20):
    execs = [rt.ConvExec(B, w[0][0].shape[1] if w[0][1] == 1 else w[0][0].shape[0], segs, w, dev)
             for segs, w, _ in jobs]
    groups = {}
    for e, (segs, w, xs) in zip(execs, jobs):
        groups.setdefault(e.launch_key, []).append((e, xs))
    launches = []
    for key, items in groups.items():
        lp = rt.LaunchPlan([e for e, _ in items], dev)
        outs = [torch.empty(B, e.plan.M, e.plan.OH, e.plan.OW, device=dev) for e, _ in items]
        structs = [e.job([(x, None) for x in xs], o) for (e, xs), o in zip(items, outs)]
        launches.append((lp, structs, sum(e.flops for e, _ in items)))
    s = torch.cuda.current_stream().cuda_stream
    for lp, st, fl in launches:
        lp.launch(st, s, fl)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        for lp, st, fl in launches:
            lp.launch(st, s, fl)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    fl = sum(f for _, _, f in launches)
    keys = "+".join(f"{lp.key}:{lp.ntiles}:k{lp.ksplit}" for lp, _, _ in launches)
    return us, fl / us / 1e6, keys


def sweep_ksplit():
    """every (cfg, ksplit) per layer: FFC_CONVQ_SWEEP=1 convq_probe.py <B>"""
    rt.USE_CONVQ = True
    for C, IH, M, c in LAYERS:
        jobs = job_pair(C, IH, M, c)
        row = [f"B{B} C{C}@{IH}x{IH}->M{M}"]
        for cfg in (0, 1, 2, 3):
            os.environ["FFC_CONVQ_CFG"] = str(cfg)
            for k in (1, 2, 4, 8):
                os.environ["FFC_CONVQ_KSPLIT"] = str(k)
                try:
                    us, tf, keys = time_layer(jobs)
                    row.append(f"c{cfg}k{k} {us:6.1f}")
                except Exception as ex:  # noqa: BLE001
                    row.append(f"c{cfg}k{k} n/a")
        os.environ.pop("FFC_CONVQ_CFG", None)
        os.environ.pop("FFC_CONVQ_KSPLIT", None)
        us, tf, keys = time_layer(jobs)
        row.append(f"auto {us:6.1f} [{keys}]")
        print(" | ".join(row), flush=True)


def main():
  for C, IH, M, c in LAYERS:
    jobs = job_pair(C, IH, M, c)
    row = [f"C{C}@{IH}x{IH}->M{M}"]
    for var in ["convp", 0, 1, 2, 3]:
        if var == "convp":
            rt.USE_CONVQ = rt.CONVQ_FORCE = False
            os.environ.pop("FFC_CONVQ_CFG", None)
        else:
            rt.USE_CONVQ = rt.CONVQ_FORCE = True
            os.environ["FFC_CONVQ_CFG"] = str(var)
        try:
            us, tf, keys = time_layer(jobs)
            row.append(f"{var}: {us:7.1f}us {tf:6.1f}TF [{keys}]")
        except Exception as ex:  # noqa: BLE001
            row.append(f"{var}: n/a ({type(ex).__name__})")
    print(" | ".join(row), flush=True)


if __name__ == "__main__":
    sweep_ksplit() if os.environ.get("FFC_CONVQ_SWEEP") else main()
