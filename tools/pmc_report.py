"""Average rocprofv3 PMC counters per kernel over dispatches (dev tool).

usage: python tools/pmc_report.py <substring> <dir> [<dir> ...]
Prints, per kernel whose name contains <substring>, the mean of every counter collected in the given
rocprofv3 output directories, the mean duration and a few derived figures (clock, MFMA busy share,
HBM bytes with the gfx950 FETCH_SIZE x2 correction)."""
import collections
import csv
import glob
import os
import sys

sub, dirs = sys.argv[1], sys.argv[2:]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
for d in dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if sub not in name:
                continue
            base = name.split("(anonymous namespace)::")[-1]
            key = base.split("(")[0][:60] + "|" + r["Grid_Size"]
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for key, cs in vals.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    us = sorted(durs[key])[len(durs[key]) // 2]
    print(f"== {key}  median {us:.1f} us")
    for c in sorted(m):
        print(f"   {c:28s} {m[c]:16.0f}")
    if "GRBM_GUI_ACTIVE" in m:
        print(f"   clock ~ {m['GRBM_GUI_ACTIVE'] / 8 / us / 1e3:.2f} GHz (GRBM/8/t)")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        # MFMA busy summed over 256 CUs x 4 SIMDs; GRBM counts every XCD (8)
        busy = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (256 * 4) / (m["GRBM_GUI_ACTIVE"] / 8)
        print(f"   MFMA busy share ~ {busy:.3f}")
    if "FETCH_SIZE" in m:
        print(f"   HBM read ~ {2 * m['FETCH_SIZE'] * 1024 / 1e6:.1f} MB (FETCH_SIZE x2, KB units), "
              f"write ~ {m.get('WRITE_SIZE', 0) * 1024 / 1e6:.1f} MB")
