"""Per-kernel MFMA utilisation from a rocprofv3 --pmc pass with SQ_INSTS_MFMA,
SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES (kernel-trace only).
MFMA-busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel duration x 2.4 GHz): the
share of the chip's matrix-pipe cycles the kernel kept busy (a lower bound when the clock runs
below its 2.4 GHz peak).  Averaged per launch.
    python tools/pmc_mfma.py <dir with */run_counter_collection.csv> <out.json>"""
import collections
import csv
import glob
import json
import sys

SIMDS, GHZ = 1024, 2.4
root, out = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(dict)
for f in glob.glob(f"{root}/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        durs[name][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
res = {}
for k, d in vals.items():
    e = {c: sum(v) / len(v) for c, v in d.items()}
    dur = sum(durs[k].values()) / len(durs[k])
    e["launches"] = len(durs[k])
    e["duration_us"] = dur * 1e6
    if "SQ_VALU_MFMA_BUSY_CYCLES" in e and dur > 0:
        e["mfma_busy_frac"] = e["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * dur * GHZ * 1e9)
    res[k] = e
json.dump({"recipe": "rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES "
                     "SQ_WAVE_CYCLES over bench.py --no-graph; per-launch averages; mfma_busy_frac = "
                     "MFMA_BUSY / (1024 SIMDs * duration * 2.4 GHz); durations here are under counter "
                     "collection (slower than the rocprof --stats traces)",
           "kernels": res}, open(out, "w"), indent=1, sort_keys=True)
for k, e in sorted(res.items(), key=lambda kv: -kv[1].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0))[:10]:
    print(f"{e.get('mfma_busy_frac', 0):6.3f} busy  {e['duration_us']:9.1f} us  {e.get('SQ_INSTS_MFMA', 0):10.3g} MFMA  {k[:70]}")
