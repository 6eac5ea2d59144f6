"""Print the JSON bench line(s) of bench.py logs: value, ms/step, rooflines, per-kernel times."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        print(f, d["value"], "ms/step", d["ms_per_step"], "roofline", d["roofline"]["frac"],
              "fft", (d.get("fft_roofline") or {}).get("frac"), "graph", d["config"].get("hipgraph"),
              "parity", d.get("parity"))
        ks = d.get("kernels", {})
        for k, v in sorted(ks.items(), key=lambda kv: -kv[1]["ms_per_step"]):
            print(f"    {k:18s} {v['ms_per_step']:8.3f} ms  {v['avg_us']:8.1f} us x {v['launches_per_step']}")
