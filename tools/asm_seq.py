"""Compressed instruction sequence of one kernel in a hipcc --save-temps .s file: runs of MFMAs,
ds_reads, LDS-DMA, VALU and SALU collapsed, waits / barriers / branches / stores kept verbatim.
    python tools/asm_seq.py file.s kernel_substring [max_lines]"""
import re
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    lim = int(sys.argv[3]) if len(sys.argv) > 3 else 400
    s = open(path).read()
    m = re.search(r"^(_Z\S*" + re.escape(sub) + r"\S*):", s, re.M)
    start = m.start()
    end = s.index(".Lfunc_end", start)
    out, prev, cnt = [], None, 0
    for line in s[start:end].split("\n"):
        t = line.strip()
        if not t or t.startswith(";") or t.startswith("."):
            if t.startswith(".LBB"):
                if prev:
                    out.append(f"{prev} x{cnt}" if cnt > 1 else prev)
                prev, cnt = None, 0
                out.append(t)
            continue
        op = t.split()[0]
        if op.startswith("v_mfma"):
            key = "mfma"
        elif op.startswith("ds_read"):
            key = "ds_read"
        elif op.startswith("global_load_lds"):
            key = "glds"
        elif (op in ("s_barrier", "s_setprio") or op.startswith("s_waitcnt") or op.startswith("s_cbranch")
              or op.startswith("s_branch") or op.startswith("scratch") or op.startswith("ds_write")
              or op.startswith("global_store") or op.startswith("global_load") or op.startswith("buffer")):
            key = t.split(";")[0].strip()
        elif op.startswith("v_"):
            key = "valu"
        elif op.startswith("s_"):
            key = "salu"
        else:
            key = op
        if key == prev:
            cnt += 1
        else:
            if prev:
                out.append(f"{prev} x{cnt}" if cnt > 1 else prev)
            prev, cnt = key, 1
    if prev:
        out.append(f"{prev} x{cnt}" if cnt > 1 else prev)
    print("\n".join(out[:lim]))


if __name__ == "__main__":
    main()
