"""Debug probe: SpectralTransform (gen64 ffc3 / ffc2 shapes) train forward repeated at B = 86 / 64,
FFC_FU2D_R2CMIX on, bn1 channel fold on / off: how many runs differ from run 0."""
import contextlib
import copy
import io
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import fastfourierconvolution_amd as F
from fastfourierconvolution_amd import _runtime as rt

QUICK = bool(os.environ.get("R2C_PROBE_QUICK"))
for chfold in ((True,) if QUICK else (True, False)):
    rt.BN_CHFOLD = chfold
    for cin, cout, hw, B in ([(64, 32, 16, 86), (64, 32, 16, 64)] if QUICK else [(64, 32, 16, 86), (128, 64, 8, 86), (64, 32, 16, 64)]):
        torch.manual_seed(cin + B)
        with contextlib.redirect_stdout(io.StringIO()):
            st = F.SpectralTransform(cin, cout, stride=2, upsample=True)
        st = st.cuda().train()
        x = torch.randn((B, cin, hw, hw)).cuda()
        outs = []
        for rep in range(40):
            m = copy.deepcopy(st)
            with torch.no_grad():
                outs.append(m(x).clone())
        torch.cuda.synchronize()
        diff = [i for i, o in enumerate(outs) if not torch.equal(o, outs[0])]
        md = max((o - outs[0]).abs().max().item() for o in outs)
        print(f"lib={os.environ.get('FFC_LIB_PATH', '')} chfold={chfold} ST({cin},{cout}) hw={hw} B={B}: {len(diff)}/40 differ (max|d| {md:.3e}) {diff[:8]}",
              flush=True)
