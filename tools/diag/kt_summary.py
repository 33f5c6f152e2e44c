"""Summarise the last forward of a rocprofv3 kernel trace (diagnostic, here or on the box).

  python tools/diag/kt_summary.py DIR/run_kernel_trace.csv [GAP_US]

The last forward = the kernels after the last host-side gap longer than GAP_US (default 200 us)
between one kernel's end and the next one's start. Prints its span, the sum of kernel times, and per
kernel family (template name): launches, summed us, and the us of the span during which that family
had a kernel running."""
import csv
import re
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    gap = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    start = 0
    end_max = ks[0][1]
    for i in range(1, len(ks)):
        if ks[i][0] - end_max > gap * 1e3:
            start = i
        end_max = max(end_max, ks[i][1])
    last = ks[start:]
    t0 = min(k[0] for k in last)
    t1 = max(k[1] for k in last)
    fam = defaultdict(lambda: [0, 0.0, []])
    for s, e, name in last:
        m = re.search(r"pwg::(?:\(anonymous namespace\)::)?(\w+)(<[^(]*>)?", name)
        key = (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0][:60]
        f = fam[key]
        f[0] += 1
        f[1] += (e - s) / 1e3
        f[2].append((s, e))
    print(f"last forward: {len(last)} kernels, span {(t1 - t0) / 1e3:.1f} us, kernel sum {sum(f[1] for f in fam.values()):.1f} us")
    for key, (n, us, iv) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        iv.sort()
        cover, cs, ce = 0, None, None
        for s, e in iv:
            if cs is None or s > ce:
                if cs is not None:
                    cover += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        cover += ce - cs
        print(f"{n:4d} x  {us:8.1f} us  covers {cover / 1e3:8.1f} us  {key}")


if __name__ == "__main__":
    main()
