"""Aggregate rocprofv3 counter_collection.csv files: per kernel name, mean counter value per dispatch."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        key = name.replace("void ", "").replace("(anonymous namespace)::", "", 1).split("(")[0]
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    vals = {c: sum(v) / len(v) for c, v in d.items()}
    print(k[:60])
    print("   " + "  ".join(f"{c}={v:.3g}" for c, v in sorted(vals.items())))
    if "SQ_WAVE_CYCLES" in vals and vals["SQ_WAVE_CYCLES"] > 0:
        w = vals["SQ_WAVE_CYCLES"]
        print(f"   wait_any {vals.get('SQ_WAIT_ANY', 0) / w:.2f}  wait_inst {vals.get('SQ_WAIT_INST_ANY', 0) / w:.2f}"
              f"  active {vals.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "GRBM_GUI_ACTIVE" in vals and vals["GRBM_GUI_ACTIVE"] > 0:
        # MFMA busy is summed over SIMDs (1024); GUI_ACTIVE is summed over 8 XCDs
        gui = vals["GRBM_GUI_ACTIVE"] / 8
        print(f"   mfma_util {vals['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui * 1024):.3f}  (busy cycles / (gui cycles x 1024 SIMDs))")
