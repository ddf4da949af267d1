"""Instruction census of one kernel in a hipcc -save-temps .s file (dev tool)."""
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
s = open(path).read()
m = re.search(r"^(_Z\S*" + pat + r"\S*):", s, re.M)
i = m.start()
j = s.index(".Lfunc_end", i)
body = s[i:j].split("\n")
cnt = {}
loop = []
for l in body:
    t = l.strip().split()
    if not t or t[0].startswith(";"):
        continue
    op = t[0]
    key = l.strip().split(";")[0].strip() if (op.startswith("s_waitcnt") or op == "s_setprio") else op
    if op.startswith(("s_waitcnt", "s_barrier", "s_setprio", "v_mfma", "global_load", "ds_read", "ds_write",
                      "s_cbranch", "buffer_", "global_store", "scratch")):
        cnt[key] = cnt.get(key, 0) + 1
print(m.group(1)[:120])
for k, v in sorted(cnt.items()):
    print(f"  {v:5d} {k}")
meta = s[j:j + 4000]
for f in ("vgpr_count", "agpr_count", "vgpr_spill_count", "private_segment_fixed_size"):
    mm = re.search(r"\." + f + r":\s+(\d+)", s[j:])
    if mm:
        print(f"  .{f} = {mm.group(1)}")
