"""Join the FETCH_SIZE / WRITE_SIZE / kernel-trace passes of tools/voc_traffic.sh per dispatch of the
second forward: kernel, grid, HBM read (FETCH_SIZE x 2 KB, the gfx950 correction of
MI355X_MICROARCH.md) and write bytes, duration, achieved HBM GB/s. Dispatches are matched by
ordinal (the child runs the same launches in the same order in every pass); names are checked.
Usage: python tools/traffic_summary.py OUT  (prints a table; writes OUT/per_dispatch.json)"""
import csv
import glob
import json
import os
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("pwg::", "").replace("void ", "")
    return n.split("(")[0]


def counters(root, ctr):
    vals = {}
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if row.get("Counter_Name") != ctr:
                continue
            d = int(row["Dispatch_Id"])
            name, v = vals.get(d, (row["Kernel_Name"], 0.0))
            vals[d] = (name, v + float(row["Counter_Value"]))
    return [vals[d] for d in sorted(vals)]


def trace(root):
    rows = []
    for path in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            rows.append((int(row["Dispatch_Id"]), row["Kernel_Name"],
                         (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6,
                         f'{row["Grid_Size_X"]}x{row["Grid_Size_Y"]}x{row["Grid_Size_Z"]}/{row["Workgroup_Size_X"]}'))
    rows.sort()
    return rows


def main(out):
    fetch = counters(os.path.join(out, "fetch"), "FETCH_SIZE")
    write = counters(os.path.join(out, "write"), "WRITE_SIZE")
    kt = [r for r in trace(os.path.join(out, "trace")) if not short(r[1]).startswith("__amd")]
    fetch = [f for f in fetch if not short(f[0]).startswith("__amd")]
    write = [w for w in write if not short(w[0]).startswith("__amd")]
    n = min(len(fetch), len(write), len(kt))
    half = n // 2
    recs = []
    for i in range(half, n):
        (fn, fv), (wn, wv), (_, kn, ms, grid) = fetch[i], write[i], kt[i]
        if not (short(fn) == short(wn) == short(kn)):
            raise SystemExit(f"dispatch {i}: names differ across passes: {short(fn)} / {short(wn)} / {short(kn)}")
        rd, wr = fv * 2048.0, wv * 1024.0
        recs.append(dict(i=i - half, kernel=short(kn), grid=grid, read_GB=rd / 1e9, write_GB=wr / 1e9, ms=ms,
                         GBs=(rd + wr) / 1e9 / (ms * 1e-3) if ms > 0 else 0.0))
    json.dump(recs, open(os.path.join(out, "per_dispatch.json"), "w"), indent=0)
    tot_rd = sum(r["read_GB"] for r in recs)
    tot_wr = sum(r["write_GB"] for r in recs)
    tot_ms = sum(r["ms"] for r in recs)
    print(f"dispatches {len(recs)}  read {tot_rd:.2f} GB  write {tot_wr:.2f} GB  kernel time {tot_ms:.2f} ms  "
          f"mean {(tot_rd + tot_wr) / tot_ms * 1e3:.0f} GB/s")
    agg = {}
    for r in recs:
        a = agg.setdefault(r["kernel"], [0, 0.0, 0.0, 0.0])
        a[0] += 1
        a[1] += r["read_GB"]
        a[2] += r["write_GB"]
        a[3] += r["ms"]
    print(f"\n{'kernel':78s} {'n':>4s} {'read GB':>8s} {'write GB':>8s} {'ms':>7s} {'GB/s':>6s}")
    for k, (c, rd, wr, ms) in sorted(agg.items(), key=lambda kv: -kv[1][3]):
        print(f"{k[:78]:78s} {c:4d} {rd:8.2f} {wr:8.2f} {ms:7.2f} {(rd + wr) / ms * 1e3:6.0f}")
    print(f"\n{'#':>4s} {'kernel':64s} {'grid':>18s} {'read':>7s} {'write':>7s} {'ms':>6s} {'GB/s':>6s}")
    for r in sorted(recs, key=lambda r: -r["ms"])[:40]:
        print(f"{r['i']:4d} {r['kernel'][:64]:64s} {r['grid']:>18s} {r['read_GB']:7.2f} {r['write_GB']:7.2f} "
              f"{r['ms']:6.2f} {r['GBs']:6.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
