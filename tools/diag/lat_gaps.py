"""Summarise a rocprofv3 kernel trace of tools/diag/lat_trace.py: per call (one plan-descriptor
kernel starts a call), the span, the sum of kernel durations and the mean duration of the layer
kernels. Usage: python tools/diag/lat_gaps.py kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
calls, cur = [], None
for r in rows:
    name = r["Kernel_Name"]
    if "plan_desc" in name:
        cur = []
        calls.append(cur)
    if cur is not None:
        cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for i, c in enumerate(calls):
    span = (c[-1][2] - c[0][1]) / 1e3
    busy = sum(e - s for _, s, e in c) / 1e3
    lay = [(e - s) / 1e3 for n, s, e in c if "layer" in n]
    gaps = [(c[j + 1][1] - c[j][2]) / 1e3 for j in range(len(c) - 1)]
    first = {n.split("(")[0].split("::")[-1][:28]: round((e - s) / 1e3, 1) for n, s, e in c if "layer" not in n}
    print(f"call {i:2d}: {len(c)} kernels span {span:7.1f} us busy {busy:7.1f} layers mean {sum(lay)/max(len(lay),1):6.2f} "
          f"min {min(lay or [0]):6.2f} max {max(lay or [0]):6.2f} gap mean {sum(gaps)/max(len(gaps),1):5.2f} {first}")
