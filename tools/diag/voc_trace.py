"""Kernel-trace view of the B = 1 vocoder forward (diagnostic, GPU box).

  rocprofv3 --kernel-trace --output-format csv -d DIR -o kt -- python3 tools/diag/voc_trace.py run CFG T [dma]
  python3 tools/diag/voc_trace.py summarize DIR

`run` does 3 + 20 forwards of CFG at T' = T, B = 1 (engine.run, no checks, no timing events);
`summarize` prints, for the last forward, every launch's GPU duration and its gap after the previous
launch's end, plus totals (busy vs idle time of the forward)."""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

REPS = 20


def run(cfg, T, dma):
    import torch

    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    dev = torch.device("cuda", 0)
    cls, p = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(dev)
    eng = m.engine()
    eng.set_narrow_dma(dma)
    plan = eng.plan([T])
    mel = torch.randn(T * 80, device=dev)
    out = torch.empty(plan.out_rows * eng.out_channels, device=dev)
    eng.run(plan, mel, out)
    for _ in range(3 + REPS):
        eng.run(plan, mel, out, check=False)
    torch.cuda.synchronize()
    print("launches per forward marker", flush=True)


def summarize_concurrent(d, per):
    """The last forward's `per` launches by start time (forwards are serialised by the join), with
    the queue they ran on and the idle time of the forward's span."""
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], q))
    rows.sort()
    last = rows[-per:]
    t0 = last[0][0]
    span = (max(e for _, e, _, _ in last) - t0) * 1e-3
    busy = sum(e - s for s, e, _, _ in last) * 1e-3
    for s, e, name, q in last:
        short = name.split("(")[0].replace("void pwg::(anonymous namespace)::", "")[:60]
        print(f"{(s - t0) * 1e-3:8.1f} .. {(e - t0) * 1e-3:8.1f} us  q{q:>3}  {short}")
    print(f"forward span {span:.1f} us, kernel time {busy:.1f} us (sum over streams)")


def summarize(d):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # the last forward: the launches after the last gap longer than 200 us (the host between
    # forwards is fast, so use the per-forward launch count from the repeating tail instead)
    names = [r[2] for r in rows]
    n = len(names)
    per = None
    for L in range(5, 200):
        if n >= 3 * L and names[n - L:] == names[n - 2 * L:n - L] == names[n - 3 * L:n - 2 * L]:
            per = L
            break
    if per is None:
        print("could not find the per-forward launch count")
        return
    last = rows[n - per:]
    busy = 0.0
    print(f"{per} launches per forward")
    prev_end = None
    for s, e, name in last:
        dur = (e - s) * 1e-3
        gap = (s - prev_end) * 1e-3 if prev_end is not None else 0.0
        busy += dur
        short = name.split("(")[0][-70:]
        print(f"{dur:8.2f} us  gap {gap:6.2f} us  {short}")
        prev_end = e
    span = (last[-1][1] - last[0][0]) * 1e-3
    print(f"forward span {span:.1f} us, kernels {busy:.1f} us, gaps {span - busy:.1f} us")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 1)
    elif sys.argv[1] == "concurrent":
        summarize_concurrent(sys.argv[2], int(sys.argv[3]))
    else:
        summarize(sys.argv[2])
