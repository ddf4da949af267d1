"""Host lead per main-stream kernel (dev tool): from a rocprofv3 --kernel-trace --hip-trace run,
for each main-queue kernel of one step, the time between the host's launch call returning and
the kernel's start (negative: the GPU waited for the host). Prints the kernels with the least
lead, grouped by (previous -> this) kernel name.

  python tools/host_lead.py <dir with run_kernel_trace.csv and run_hip_api_trace.csv>"""
import collections
import csv
import os
import sys

d = sys.argv[1]
ks = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
api = list(csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv"))))
by_corr = {r["Correlation_Id"]: r for r in api}
for r in ks:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
ks.sort(key=lambda r: r["s"])
ad = [r for r in ks if "adamw_kernel" in r["Kernel_Name"]]
i = len(ad) // 2
t0, t1 = ad[i - 1]["e"], ad[i]["e"]
win = [r for r in ks if t0 <= r["s"] and r["e"] <= t1]
busy = collections.Counter()
for r in win:
    busy[r["Queue_Id"]] += r["e"] - r["s"]
mq = busy.most_common(1)[0][0]  # the image chain: the busiest queue
main = [r for r in win if r["Queue_Id"] == mq]


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:44]


agg = collections.defaultdict(list)
missing = 0
for j in range(1, len(main)):
    a = by_corr.get(main[j]["Correlation_Id"])
    if a is None:
        missing += 1
        continue
    lead = main[j]["s"] - int(a["End_Timestamp"])  # > 0: call returned before the kernel started
    gap = main[j]["s"] - main[j - 1]["e"]
    agg[(short(main[j - 1]["Kernel_Name"]), short(main[j]["Kernel_Name"]))].append((lead, gap))
print(f"{len(main)} main kernels, {missing} without an API record")
print("count  min-lead-us  avg-lead-us  avg-gap-us  prev -> this")
for k, v in sorted(agg.items(), key=lambda kv: min(x for x, _ in kv[1])):
    print(f"{len(v):5d} {min(x for x, _ in v) / 1e3:11.1f} {sum(x for x, _ in v) / len(v) / 1e3:11.1f} "
          f"{sum(g for _, g in v) / len(v) / 1e3:10.1f}  {k[0]} -> {k[1]}")
