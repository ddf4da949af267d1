"""Per-stream view of one step of a rocprofv3 kernel trace (dev tool): the step window between
two consecutive adamw_kernel dispatches, each stream's busy time, the main stream's idle gaps,
and the main-stream kernels grouped by name with the side-stream time that overlapped them.

  python tools/trace_streams.py <run_kernel_trace.csv> [step index (default: middle)]
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
ad = [r for r in rows if "adamw_kernel" in r["Kernel_Name"]]
i = int(sys.argv[2]) if len(sys.argv) > 2 else len(ad) // 2
t0, t1 = ad[i - 1]["e"], ad[i]["e"]
win = [r for r in rows if r["s"] >= t0 and r["e"] <= t1]
by_q = collections.defaultdict(list)
for r in win:
    by_q[(r["Queue_Id"], r["Stream_Id"])].append(r)
main_key = max(by_q, key=lambda k: sum(r["e"] - r["s"] for r in by_q[k]))
print(f"step window {(t1 - t0) / 1e3:.1f} us, {len(win)} dispatches")
for k, rs in sorted(by_q.items()):
    busy = sum(r["e"] - r["s"] for r in rs)
    print(f"  queue {k[0]} stream {k[1]}: {len(rs)} kernels, busy {busy / 1e3:.1f} us"
          + ("  <- main" if k == main_key else ""))
main = by_q[main_key]
gaps = [(main[j + 1]["s"] - main[j]["e"], main[j]["Kernel_Name"][:60], main[j + 1]["Kernel_Name"][:60])
        for j in range(len(main) - 1)]
print(f"main stream idle between kernels: {sum(max(g, 0) for g, _, _ in gaps) / 1e3:.1f} us; largest:")
for g, a, b in sorted(gaps, reverse=True)[:8]:
    print(f"  {g / 1e3:7.1f} us  after {a}  before {b}")
side = [r for k, rs in by_q.items() if k != main_key for r in rs]
agg = collections.defaultdict(lambda: [0, 0, 0])
for r in main:
    ov = sum(max(0, min(r["e"], s["e"]) - max(r["s"], s["s"])) for s in side)
    key = (r["Kernel_Name"][:70], r["Grid_Size_X"])
    agg[key][0] += 1
    agg[key][1] += r["e"] - r["s"]
    agg[key][2] += ov
print("main-stream kernels: count, total us, avg us, side-stream kernel time overlapping them")
for k, (n, t, ov) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:24]:
    print(f"  {n:3d} {t / 1e3:8.1f} {t / n / 1e3:7.1f}  ovl {ov / 1e3:7.1f}  grid {k[1]:>8} {k[0]}")
print("side-stream kernels: count, total us")
sagg = collections.defaultdict(lambda: [0, 0])
for r in side:
    key = (r["Kernel_Name"][:70], r["Grid_Size_X"], r["Queue_Id"])
    sagg[key][0] += 1
    sagg[key][1] += r["e"] - r["s"]
for k, (n, t) in sorted(sagg.items(), key=lambda kv: -kv[1][1])[:20]:
    print(f"  {n:3d} {t / 1e3:8.1f}  q{k[2]} grid {k[1]:>8} {k[0]}")


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:48]


print("main-stream gaps by (previous kernel -> next kernel): count, total us, avg us")
gagg = collections.defaultdict(lambda: [0, 0])
for j in range(len(main) - 1):
    g = main[j + 1]["s"] - main[j]["e"]
    key = (short(main[j]["Kernel_Name"]), short(main[j + 1]["Kernel_Name"]))
    gagg[key][0] += 1
    gagg[key][1] += max(g, 0)
for k, (n, t) in sorted(gagg.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"  {n:3d} {t / 1e3:8.1f} {t / n / 1e3:7.1f}  {k[0]} -> {k[1]}")
hist = collections.Counter(min(int(max(g, 0) / 1e3 // 2) * 2, 40) for g, _, _ in gaps)
print("gap histogram (us bucket: count):", dict(sorted(hist.items())))
