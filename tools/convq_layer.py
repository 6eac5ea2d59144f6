"""Run ONE FFCTranspose layer's conv launch (out_l + out_g jobs) `reps` times: the target of a
rocprofv3 --pmc pass.  Diagnostic only.
usage: convq_layer.py <layer index> <B> <convp|0..3> [reps] [gen64|fgan128]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.argv += [None] * 3
li, B, var = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
reps = int(sys.argv[4] or 10)
model = sys.argv[5] or "gen64"
sys.argv = [sys.argv[0], str(B), model]
import convq_probe as P  # noqa: E402

if var == "convp":
    P.rt.USE_CONVQ = False
else:
    os.environ["FFC_CONVQ_CFG"] = var
C, IH, M, c = P.LAYERS[li]
us, tf, keys = P.time_layer(P.job_pair(C, IH, M, c), reps=reps)
print(f"layer {li} B={B} {var}: {us:.1f} us {tf:.1f} TF {keys}")
