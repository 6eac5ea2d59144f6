"""Per-kernel GPU time of one training iteration from a rocprofv3 kernel trace (csv): the iteration is
the span between two step starts, found by the `marker` kernel that occurs `per` times per iteration
(fgan128train: 22 normal_() draws).  usage: trace_iter.py trace.csv [k-th iteration from the end]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
per = int(sys.argv[3]) if len(sys.argv) > 3 else 22


def nm(r):
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:70]


idx = [i for i, r in enumerate(rows) if "distribution_elementwise" in r["Kernel_Name"]]
a, b = idx[-per * back], idx[-per * (back - 1)] if back > 1 else len(rows)
sel = rows[a:b]
span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e6
tot = collections.defaultdict(lambda: [0, 0.0])
for r in sel:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    t = tot[nm(r)]
    t[0] += 1
    t[1] += d
busy = sum(v[1] for v in tot.values())
print(f"iteration: {len(sel)} kernels, span {span:.2f} ms, kernel-busy {busy:.2f} ms")
for k, (c, ms) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{ms:8.3f} ms  x{c:4d}  {k}")
