"""Per-launch HBM bytes per kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json>

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE is in KiB and on gfx950 reports half the
bytes of a wide coalesced streaming read, so read_bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE (KiB)
is exact for 16-B-per-lane stores. Kernels are keyed by their short name and grid size (one
entry per launch shape); the 'families' section aggregates the 256x256 GEMM launches per kernel
family (gemm8_kernel bf16 = the dominant kernel bench.py reports, its fp8 form, and the older
ping-pong gemm_pp_kernel), every epilogue."""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    """Kernel name without namespace, return type and parameter list (parameter types may
    themselves be namespace-qualified, so cut at the first '(' after the name)."""
    base = name.split("(anonymous namespace)::", 1)[-1] if "::" in name else name
    return base.split("(")[0]


def load(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            acc[(short(r["Kernel_Name"]), int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {"note": "bytes per launch; read = 2*1024*FETCH_SIZE (gfx950 correction), "
                   "write = 1024*WRITE_SIZE", "kernels": {}, "families": {}}
    fam = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for key in sorted(set(fetch) | set(write)):
        f = fetch.get(key, [])
        w = write.get(key, [])
        rd = 2 * 1024 * sum(f) / len(f) if f else None
        wr = 1024 * sum(w) / len(w) if w else None
        name, grid = key
        out["kernels"][f"{name}|grid={grid}"] = {"launches": max(len(f), len(w)), "read_bytes": rd,
                                                 "write_bytes": wr}
        family = None
        if name.startswith("gemm_pp_kernel"):
            family = "gemm_pp_kernel"
        elif name.startswith("gemm8_kernel"):
            family = "gemm8_kernel_fp8" if "true" in name else "gemm8_kernel_bf16"
        if family and rd is not None and wr is not None:
            n = min(len(f), len(w))
            fam[family][0] += n
            fam[family][1] += rd * n
            fam[family][2] += wr * n
    for k, (n, rd, wr) in fam.items():
        out["families"][k] = {"launches": n, "read_bytes_per_launch": rd / n,
                              "write_bytes_per_launch": wr / n,
                              "bytes_per_launch": (rd + wr) / n}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -((kv[1]["read_bytes"] or 0) + (kv[1]["write_bytes"] or 0)) * kv[1]["launches"])[:25]:
        print(f"{k[:70]:70s} n={v['launches']:4d} rd={(v['read_bytes'] or 0) / 1e6:9.2f} MB "
              f"wr={(v['write_bytes'] or 0) / 1e6:9.2f} MB")
    print(json.dumps(out["families"], indent=1))


if __name__ == "__main__":
    main()
