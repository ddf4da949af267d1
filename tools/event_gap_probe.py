"""Main-stream bubble of a cross-stream dependency (dev tool, run under rocprofv3 --kernel-trace).

Launches pairs of ~20 us torch kernels on the current stream in four forms, 100 pairs each,
separated by a synchronize so the trace can tell them apart:
  plain      k1, k2
  record     k1, event.record(main), k2
  side       k1, side.wait_stream(main) + a small kernel on the side stream, k2
  waitside   k1, main.wait_event(event recorded on an idle side stream), k2
then (tools/trace_gaps_probe below) prints the average k1 -> k2 gap per form."""
import os
import sys
import torch

if len(sys.argv) > 1 and sys.argv[1] == "report":
    import csv
    rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    main = [r for r in rows if "elementwise" in r["Kernel_Name"] or "vectorized" in r["Kernel_Name"]]
    qs = {}
    for r in rows:
        qs.setdefault(r["Queue_Id"], 0)
        qs[r["Queue_Id"]] += 1
    mq = max(qs, key=qs.get)
    main = [r for r in rows if r["Queue_Id"] == mq and "mul" not in r["Kernel_Name"].lower()]
    forms = ["plain", "record", "side", "waitside"]
    # the probe's main-stream kernels come in blocks of 200 (100 pairs) per form, after 20 warmup
    k = main[20:]
    for i, f in enumerate(forms):
        blk = k[i * 200:(i + 1) * 200]
        gaps = [int(blk[j + 1]["Start_Timestamp"]) - int(blk[j]["End_Timestamp"])
                for j in range(0, len(blk) - 1, 2)]
        dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in blk]
        print(f"{f:9s} k1->k2 gap avg {sum(gaps) / len(gaps) / 1e3:6.2f} us  "
              f"max {max(gaps) / 1e3:6.2f}  kernel avg {sum(dur) / len(dur) / 1e3:6.2f} us")
    raise SystemExit(0)

dev = torch.device("cuda:0")
busy = os.environ.get("PROBE_BUSY") == "1"  # a third stream kept busy meanwhile (the text tower)
a = torch.zeros(16 << 20, device=dev)
b = torch.zeros(16 << 20, device=dev)
c = torch.zeros(1024, device=dev)
side = torch.cuda.Stream()
main = torch.cuda.current_stream()
for _ in range(10):
    a.add_(1.0)
    b.add_(1.0)
torch.cuda.synchronize()
third = torch.cuda.Stream()
big = torch.zeros(64 << 20, device=dev)
for form in ("plain", "record", "side", "waitside"):
    if busy:
        with torch.cuda.stream(third):
            for _ in range(60):
                big.mul_(1.0)
    for _ in range(100):
        a.add_(1.0)
        if form == "record":
            torch.cuda.Event().record(main)
        elif form == "side":
            side.wait_stream(main)
            with torch.cuda.stream(side):
                c.add_(1.0)
        elif form == "waitside":
            e = torch.cuda.Event()
            e.record(side)
            main.wait_event(e)
        b.add_(1.0)
    torch.cuda.synchronize()
print("done")
