"""Per-kernel HBM traffic (bytes per launch) from rocprofv3 FETCH_SIZE / WRITE_SIZE passes."""
import collections
import csv
import glob
import json
import sys

root, out = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, d in vals.items():
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        fetch = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
        write = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
        res[k] = {"fetch_kb": fetch, "write_kb": write, "bytes_per_launch": (2.0 * fetch + write) * 1024.0,
                  "launches": len(d["FETCH_SIZE"])}
json.dump({"recipe": "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch (MI355X_MICROARCH.md HBM)",
           "kernels": res}, open(out, "w"), indent=1, sort_keys=True)
for k, v in sorted(res.items(), key=lambda kv: -kv[1]["bytes_per_launch"]):
    print(f"{v['bytes_per_launch'] / 1e6:10.2f} MB/launch  {k[:90]}")
