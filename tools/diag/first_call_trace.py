"""The full default bench in one process, with every conv-network inference_batch call of 16
utterances timed by part (plan, concatenation, output allocation, run incl. status read) and
printed to stderr (diagnostic, GPU box): python tools/diag/first_call_trace.py [bench args]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from parallelwavegan_amd import cnet  # noqa: E402

_orig_infer = cnet.CnetEngine.infer


def infer(self, mels, mean=None, scale=None):
    if len(mels) != 16:
        return _orig_infer(self, mels, mean, scale)
    t = {}

    def lap(name, t0):
        torch.cuda.synchronize(self.device)
        t1 = time.perf_counter()
        t[name] = round((t1 - t0) * 1e3, 3)
        return t1

    torch.cuda.synchronize(self.device)
    t0 = time.perf_counter()
    frames = [int(m.shape[0]) for m in mels]
    plan = self.plan(frames)
    t0 = lap("plan", t0)
    mel = torch.cat([m.reshape(-1) for m in mels])
    t0 = lap("cat", t0)
    O = self.out_channels
    out = torch.empty(plan.out_rows * O, dtype=torch.float32, device=self.device)
    t0 = lap("empty", t0)
    ws0 = sum(w.numel() for w in self._workspaces.values())
    self.run(plan, mel, out, mean, scale)
    t0 = lap("run", t0)
    t["ws_MB"] = (round(ws0 / 2**20, 1), round(sum(w.numel() for w in self._workspaces.values()) / 2**20, 1))
    t["frames"] = frames[0]
    t["out_ch"] = O
    print("[first_call_trace]", t, file=sys.stderr, flush=True)
    res, off = [], 0
    for f in frames:
        T = f * self.hop
        res.append(out[off * O:(off + T) * O].view(T, O))
        off += T
    return res


cnet.CnetEngine.infer = infer
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
