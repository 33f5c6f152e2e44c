"""Layer pipeline vs per-layer launches under PMC (verdict r02 item 6's negative result).

child mode (run under rocprofv3 by tools/pipe_pmc.sh):
    python tools/diag/pipe_pmc.py child {per_layer|pipeline} {bench|lj512}
  two forwards of the workload (bench: the 32-utterance LibriTTS batch; lj512: LJ v1, B = 1,
  T' = 512), pipeline option 0 or 1 << 24.
summary mode:
    python tools/diag/pipe_pmc.py summary OUT
  per mode and workload, over the SECOND forward's dispatches: residual-layer kernel time, HBM
  read (FETCH_SIZE x 2 KB, gfx950 correction) and write bytes, effective clock
  (GRBM_GUI_ACTIVE / 8 XCDs / wall), matrix-pipe busy (SQ_VALU_MFMA_BUSY_CYCLES over
  GRBM_GUI_ACTIVE / 8 x 256 CUs x 4 SIMDs), wave wait share (SQ_WAIT_ANY / SQ_WAVE_CYCLES)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def child(mode, work):
    import numpy as np
    import torch

    from parallelwavegan_amd import Engine, configs, synthetic

    dev = torch.device("cuda", 0)
    if work == "bench":
        cfg, lengths = "libritts_v1", synthetic.libritts_lengths(32, seed=3).tolist()
    else:
        cfg, lengths = "ljspeech_v1", [512]
    params = configs.generator_params(cfg)
    eng = Engine(params, dev)
    eng.load_state_dict(synthetic.make_state_dict(params, seed=0))
    eng.set_option("pipeline", 0 if mode == "per_layer" else 1 << 24)
    plan = eng.plan(lengths)
    rs = np.random.RandomState(1)
    mel = torch.from_numpy(rs.standard_normal(sum(lengths) * params["aux_channels"]).astype(np.float32)).to(dev)
    noise = torch.from_numpy(rs.standard_normal(plan.total_samples).astype(np.float32)).to(dev)
    out = torch.empty(plan.total_samples, device=dev)
    for _ in range(2):
        eng.run(plan, mel, noise, out, check=False)
    torch.cuda.synchronize()
    eng.run_status(plan)


def load(root):
    """{dispatch: (kernel, dur_ns, {counter: value})} over every counter CSV under root."""
    d = {}
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = (os.path.relpath(path, root).split(os.sep)[0], int(r["Dispatch_Id"]))  # (pass, dispatch)
            e = d.setdefault(k, [r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), defaultdict(float)])
            e[2][r["Counter_Name"]] += float(r["Counter_Value"])
    return d


def summary(out):
    res = {}
    for run in sorted(os.listdir(out)):
        root = os.path.join(out, run)
        if not os.path.isdir(root):
            continue
        d = load(root)
        by_pass = defaultdict(list)
        for (p, disp), e in d.items():
            by_pass[p].append((disp, e))
        agg = defaultdict(float)
        for p, rows in by_pass.items():
            rows.sort(key=lambda x: x[0])
            layer = [e for _, e in rows if "split16_kernel" in e[0]]
            second = layer[len(layer) // 2:]
            for name, dur, ctr in second:
                for c, v in ctr.items():
                    agg[c] += v
                agg["dur_ns_" + p] += dur
                agg["launches_" + p] += 1
        durs = [v for k, v in agg.items() if k.startswith("dur_ns_")]
        dur = sum(durs) / max(len(durs), 1)
        gui = agg.get("GRBM_GUI_ACTIVE", 0.0)
        r = {"launches": int(max(v for k, v in agg.items() if k.startswith("launches_"))),
             "layer_ms": round(dur / 1e6, 4),
             "read_GB": round(agg.get("FETCH_SIZE", 0) * 2048 / 1e9, 3),
             "write_GB": round(agg.get("WRITE_SIZE", 0) * 1024 / 1e9, 3)}
        pd = [k for k in agg if k.startswith("dur_ns_")]
        gui_dur = next((agg[k] for k in pd if "clk" in k), dur)
        if gui:
            r["clock_GHz"] = round(gui / 8 / gui_dur, 3)
            r["mfma_busy"] = round(agg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui / 8 * 256 * 4), 3)
            r["wait_share"] = round(agg.get("SQ_WAIT_ANY", 0) / max(agg.get("SQ_WAVE_CYCLES", 1), 1), 3)
            r["busy_share"] = round(agg.get("SQ_BUSY_CYCLES", 0) / max(gui, 1), 3)
        r["HBM_GBs"] = round((r["read_GB"] + r["write_GB"]) / (dur / 1e9), 1)
        res[run] = r
        print(run, json.dumps(r))
    json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "child":
        child(sys.argv[2], sys.argv[3])
    else:
        summary(sys.argv[2])
