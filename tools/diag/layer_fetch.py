"""Summarise tools/diag/layer_fetch.sh: per residual-layer dispatch of the second forward, HBM read
(FETCH_SIZE x 2) and write (WRITE_SIZE) bytes, the algorithmic bytes of that launch (x pairs in /
out, fp32 skip in / out, D rows) and the read over-fetch, grouped by dilation."""
import csv
import glob
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def per_dispatch(d, ctr):
    vals, names = {}, {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if row.get("Counter_Name") != ctr:
                continue
            i = int(row["Dispatch_Id"])
            vals[i] = vals.get(i, 0.0) + float(row["Counter_Value"])
            names[i] = row.get("Kernel_Name", "")
    dur = {}
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            dur[int(row["Dispatch_Id"])] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
    return vals, names, dur


def main():
    out = sys.argv[1]
    from parallelwavegan_amd import synthetic

    lengths = synthetic.libritts_lengths(32, seed=3)
    T = int(lengths.sum()) * 300
    F = int(lengths.sum())
    L = 30
    res = {}
    for spec in sys.argv[2:]:
        v = spec.split("=")[0]
        f, names, dur = per_dispatch(os.path.join(out, v, "FETCH_SIZE"), "FETCH_SIZE")
        w, _, _ = per_dispatch(os.path.join(out, v, "WRITE_SIZE"), "WRITE_SIZE")
        ids = sorted(i for i in f if "pwg_layer_split16_kernel" in names[i])[-L:]
        rows = []
        for l, i in enumerate(ids):
            rd = f[i] * 2048.0
            wr = w.get(i, 0.0) * 1024.0
            alg_rd = T * ((4 if l == 0 else 256) + (0 if l == 0 else 256)) + F * 512
            alg_wr = T * (4 if l == L - 1 else 512)
            rows.append({"layer": l, "dil": 2 ** (l % 10), "read_GB": round(rd / 1e9, 3), "write_GB": round(wr / 1e9, 3),
                         "alg_read_GB": round(alg_rd / 1e9, 3), "alg_write_GB": round(alg_wr / 1e9, 3),
                         "read_over": round(rd / alg_rd, 3), "ms": round(dur.get(i, 0.0), 4)})
        mid = [r for r in rows if 0 < r["layer"] < L - 1]
        by_d = {}
        for r in mid:
            by_d.setdefault(r["dil"], []).append(r)
        summ = {d: {"read_GB": round(float(np.mean([r["read_GB"] for r in rs])), 3),
                    "read_over": round(float(np.mean([r["read_over"] for r in rs])), 3),
                    "ms": round(float(np.mean([r["ms"] for r in rs])), 4)} for d, rs in sorted(by_d.items())}
        res[v] = {"layers": rows, "by_dilation": summ,
                  "mid_read_GB": round(float(np.mean([r["read_GB"] for r in mid])), 3),
                  "mid_write_GB": round(float(np.mean([r["write_GB"] for r in mid])), 3),
                  "mid_ms": round(float(np.mean([r["ms"] for r in mid])), 4)}
        print(v, "middle layers: read", res[v]["mid_read_GB"], "GB, write", res[v]["mid_write_GB"], "GB,",
              res[v]["mid_ms"], "ms (under PMC)")
        for d, s in summ.items():
            print(f"  d={d:4d} read {s['read_GB']:.3f} GB  over {s['read_over']:.3f}  {s['ms']:.4f} ms")
    json.dump(res, open(os.path.join(out, "layer_fetch.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
