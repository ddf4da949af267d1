"""Group a rocprofv3 kernel_trace.csv by (kernel, grid) and print per-step time (dev tool).

  python tools/trace_by_shape.py <run_kernel_trace.csv> [steps] [top]
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
d = collections.defaultdict(list)
for r in rows:
    grid = f"{r['Grid_Size_X']}x{r['Grid_Size_Y']}"
    d[(r["Kernel_Name"][:80], grid, r["Workgroup_Size_X"])].append(
        int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{sum(v) / steps / 1e6:7.3f} ms/step {len(v) / steps:6.1f}/step avg {sum(v) / len(v) / 1e3:8.1f}us "
          f"grid {k[1]:>10} wg {k[2]:>4} {k[0]}")
print(f"total {tot / steps / 1e6:.2f} ms/step")
