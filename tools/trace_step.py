"""Print one generator step's kernel sequence from a rocprofv3 kernel_trace.csv."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tr = list(csv.DictReader(open(path)))
tot = 0
for r in tr[-n:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    print(f"{r['Kernel_Name'][:64]:64s} wg={int(r['Grid_Size_X'])//int(r['Workgroup_Size_X']):6d} "
          f"lds={r['LDS_Block_Size']:>6} vgpr={r['VGPR_Count']:>3} agpr={r['Accum_VGPR_Count']:>3} {d:9.2f} us")
print(f"sum {tot:.1f} us")
