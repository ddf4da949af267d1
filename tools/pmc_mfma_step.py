"""MFMA-pipe utilisation per kernel family over bench steps, from a rocprofv3 PMC pass with
SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (dev tool; profiles/<round>/mfma_busy.json).

usage: python tools/pmc_mfma_step.py <pmc_dir> <out.json>

busy share of a dispatch = SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs) / (GRBM_GUI_ACTIVE / 8
XCDs) — the fraction of the kernel's cycles in which an average SIMD's MFMA pipe was busy
(rocprofv3 serialises dispatches while it counts, so each figure is the kernel on its own). The
step line weights every dispatch by its duration."""
import collections
import csv
import glob
import json
import os
import sys

d, out = sys.argv[1], sys.argv[2]
per = collections.defaultdict(dict)  # dispatch id -> counters
meta = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = (f, r["Dispatch_Id"])
        per[k][r["Counter_Name"]] = float(r["Counter_Value"])
        name = r["Kernel_Name"]
        name = name.split("(anonymous namespace)::", 1)[1] if "(anonymous namespace)::" in name else name
        name = name.split("(")[0]
        meta[k] = (name, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
fam = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])  # n, us, busy, active
tot = [0.0, 0.0, 0.0]
for k, c in per.items():
    if "SQ_VALU_MFMA_BUSY_CYCLES" not in c or "GRBM_GUI_ACTIVE" not in c:
        continue
    name, us = meta[k]
    busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024.0
    act = c["GRBM_GUI_ACTIVE"] / 8.0
    e = fam[name]
    e[0] += 1
    e[1] += us
    e[2] += busy
    e[3] += act
    tot[0] += us
    tot[1] += busy
    tot[2] += act
rows = sorted(fam.items(), key=lambda kv: -kv[1][1])
res = {"source": d, "counters": ["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],
       "all_kernels": {"us": round(tot[0], 1), "mfma_busy_share": round(tot[1] / max(tot[2], 1), 4)},
       "families": {}}
for name, (n, us, busy, act) in rows:
    res["families"][name] = {"dispatches": n, "us": round(us, 1),
                             "mfma_busy_share": round(busy / max(act, 1), 4)}
    print(f"{us:10.1f} us {n:5d}x  MFMA busy {busy / max(act, 1):6.3f}  {name[:70]}")
print(f"all kernels: {tot[0]:.1f} us, MFMA busy share {tot[1] / max(tot[2], 1):.3f}")
json.dump(res, open(out, "w"), indent=1)
