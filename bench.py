#!/usr/bin/env python3
"""Throughput benchmark of the PWG generator hot path on MI355X.

Workload (BASELINE.json metric "audio samples/sec/GPU (24 kHz PWG, 80-band mel)", configs[4]):
LibriTTS parallel_wavegan.v1 generator (30 layers, 24 kHz, hop 300), random-init seeded
weights, a batch of synthetic utterances per GPU with T'_i = RandomState(3).randint(80, 1200)
mel frames (1-15 s of audio each). One "step" = one generator forward over the whole batch
(every kernel of the hot path), inputs resident in HBM before the timed region.

Multi-GPU: one process per GPU (torch.distributed.run), utterances are independent so the data
path has no collective; rank 0's packed weights are RCCL-broadcast once at start-up through the
C-ABI (pwg_broadcast_weights). Default: weak scaling, every rank runs the same per-GPU batch shape.
--strong: SURVEY.md sec 8(d)(5), the fixed 512-utterance list LPT-sharded over the ranks.

At N=1 the line also carries the reference's own call pattern (B=1 inference() latency rows, LJ v1,
bin/decode.py:236-268) and a CPU baseline on a bounded sample.

Prints ONE JSON line (rank 0) with the contract fields plus "roofline" and "cpu_baseline".
"""

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from parallelwavegan_amd import Engine, GraphedRun, _lib, configs, synthetic  # noqa: E402
from parallelwavegan_amd.sharding import (  # noqa: E402
    broadcast_packed_weights, broadcast_weights_rccl, lpt_partition, max_over_ranks, shard_loads)

FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: Peak FP32 (matrix) = vector, spec
HBM_PEAK_GBS = 8000.0
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 dense (no sparsity)


def split_layer_bytes_per_sample(params, H, L, fuse_first=False):
    """Algorithmic HBM bytes per sample of the split engine's residual layer, averaged over the L
    launches: x read + write (4 B per channel as an fp16 pair) and skip read + write (fp32); layer 0
    reads no skip (and, with the fused first_conv, the 4-byte noise instead of x), the last layer
    writes neither x nor skip but the output; plus the frame-rate aux rows (GR pairs per frame).
    DESIGN.md sec 3.0."""
    R, S, G, O = (params[k] for k in ("residual_channels", "skip_channels", "gate_channels", "out_channels"))
    mid = 4 * (2 * R + 2 * S)
    first = 4 * (R + S) + 4 if fuse_first else 4 * (2 * R + S)
    last = 4 * (R + S) + 4 * O
    return (first + (L - 2) * mid + last) / L + 4 * G / H


def split_executed_flop_per_block(L, kernel="split16"):
    """f16 MFMA FLOP one 32-sample block executes, averaged over the L launches. split: 144 GEMM-1
    + 12 aux/bias + 48 GEMM-2 v_mfma_f32_32x32x16_f16 (32,768 FLOP each), the last layer 24 GEMM-2;
    split16: 288 + 16 + 96 v_mfma_f32_16x16x32_f16 (16,384 FLOP each), the last layer 48
    GEMM-2. The last layer's head runs as fp32 MFMA (not counted)."""
    if kernel == "split":
        return 32768 * ((L - 1) * 204 + (144 + 12 + 24)) / L
    return 16384 * ((L - 1) * 400 + (288 + 16 + 48)) / L


def layer_flops_per_sample(params):
    """Algorithmic FLOP per output sample of ONE residual layer in the reference formulation
    (SURVEY.md sec 8(a) a10): 2 * (K*R*G + A*G + GH*S + GH*R)."""
    R, G, S, A, K = (params[k] for k in ("residual_channels", "gate_channels", "skip_channels",
                                         "aux_channels", "kernel_size"))
    return 2 * (K * R * G + A * G + (G // 2) * S + (G // 2) * R)


def layer_bytes_per_sample(params):
    """Algorithmic HBM bytes per output sample of one residual layer (fp32, layer-streaming):
    read x (R) + c_up (A) + skip (S), write x (R) + skip (S)."""
    R, S, A = params["residual_channels"], params["skip_channels"], params["aux_channels"]
    return 4 * (2 * R + A + 2 * S)


def model_flops_per_sample(params):
    """Whole-forward algorithmic FLOP per sample (2,591,262 for LibriTTS v1)."""
    L = params["layers"]
    R, S, A, O = params["residual_channels"], params["skip_channels"], params["aux_channels"], params["out_channels"]
    scales = params["upsample_params"]["upsample_scales"]
    H = int(np.prod(scales))
    w = params["aux_context_window"]
    conv_in = A * A * (2 * w + 1) / H
    fir, n = 0.0, 1
    for s in scales:
        n *= s
        fir += A * (2 * s + 1) * n / H
    head = S * S + S * O + R
    return L * layer_flops_per_sample(params) + 2 * (conv_in + fir + head)


def launch_command(n, argv, port):
    """The torch.distributed.run command that starts N ranks of this script with the same
    arguments (the form the driver itself uses for N > 1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, argv):
    """`bench.py --gpus N` started as ONE process (no WORLD_SIZE in the environment): start the N
    ranks as a child torch.distributed.run and return its exit code. The reference's multi-GPU
    entry does the same from one command (parallel_wavegan/distributed/launch.py:117-171).

    Called before this process makes any GPU call; the child is a subprocess, never an exec.
    On the nccl backend (one process per GPU) fewer than N visible devices is an error, so a
    scaling run can never record fewer GPUs than its label; PWG_BENCH_BACKEND=gloo rehearses N
    ranks sharing the devices there are. Rank 0's JSON line reaches our stdout directly (the
    child inherits it; the other ranks print nothing there)."""
    import socket

    backend = os.environ.get("PWG_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if backend == "nccl" and ndev < n:
        print(f"[bench] --gpus {n}: only {ndev} GPU(s) visible; one process per GPU needs {n}", file=sys.stderr)
        return 2
    if backend != "nccl" and ndev < 1:
        print("[bench] no GPU visible", file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(launch_command(n, argv, port), env=env)
    return r.returncode


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # one process per GPU; PWG_BENCH_BACKEND=gloo (with ranks sharing a GPU when there are
        # fewer GPUs than ranks) only rehearses the multi-rank path on a 1-GPU box
        backend = os.environ.get("PWG_BENCH_BACKEND", "nccl")
        ndev = torch.cuda.device_count()
        local = local if backend == "nccl" else local % max(ndev, 1)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        if world != n_gpus:
            print(f"[bench] WORLD_SIZE={world} but --gpus {n_gpus}: reporting {world} ranks", file=sys.stderr)
        return dist.get_rank(), world, dev
    if n_gpus != 1:
        raise RuntimeError(f"--gpus {n_gpus} reached single-process setup (launch_ranks should have run)")
    return 0, 1, torch.device("cuda", 0)


def per_rank_seconds(local_s, world, dev):
    """Every rank's timed-region wall seconds (all_gather; host tensor on gloo)."""
    if world == 1:
        return [local_s]
    gloo = dist.get_backend() == "gloo"
    t = torch.tensor([local_s], dtype=torch.float64, device="cpu" if gloo else dev)
    ts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(ts, t)
    return [float(x.item()) for x in ts]


PMC_PASSES = (("FETCH_SIZE",), ("WRITE_SIZE",), ("GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"))


def _pmc_passes(args):
    """rocprofv3 --pmc passes, one counter group each (FETCH_SIZE and WRITE_SIZE need separate
    passes on gfx950; the third reads the shader clock and the matrix pipes' busy cycles) over a
    child process (`bench.py --pmc-child`, never an exec) that runs two forwards of this workload.
    Returns ({counter: {dispatch_id: (kernel_name, value, duration_ns)}}, None) or (None, failure
    note); a failed clock pass leaves its counters out."""
    import csv
    import glob
    import shutil
    import tempfile

    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    per = {}
    for group in PMC_PASSES:
        optional = "FETCH_SIZE" not in group and "WRITE_SIZE" not in group
        with tempfile.TemporaryDirectory(prefix="pwg_pmc_", dir="/tmp") as d:
            cmd = [prof, "--pmc", *group, "--output-format", "csv", "-d", d, "-o", "pmc", "--", sys.executable,
                   os.path.abspath(__file__), "--pmc-child", "--config", args.config, "--utts", str(args.utts)]
            if args.layer_kernel:
                cmd += ["--layer-kernel", args.layer_kernel]
            env = dict(os.environ, TMPDIR="/tmp")
            for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
                env.pop(k, None)
            try:
                r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=150)
            except subprocess.TimeoutExpired:
                if optional:
                    continue
                return None, f"rocprofv3 --pmc {' '.join(group)} pass timed out"
            if r.returncode != 0:
                if optional:
                    continue
                return None, f"rocprofv3 --pmc {' '.join(group)} pass failed (rc {r.returncode})"
            vals = {c: {} for c in group}
            for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for row in csv.DictReader(open(path)):
                    ctr = row.get("Counter_Name")
                    if ctr not in vals:
                        continue
                    disp = int(row.get("Dispatch_Id") or 0)
                    try:
                        dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                    except (KeyError, TypeError, ValueError):
                        dur = 0
                    name, v, _ = vals[ctr].get(disp, (row.get("Kernel_Name", ""), 0.0, dur))
                    vals[ctr][disp] = (name, v + float(row.get("Counter_Value") or 0), dur)
            if not all(vals.values()):
                if optional:
                    continue
                return None, f"rocprofv3 --pmc {' '.join(group)}: no dispatches recorded"
            per.update(vals)
    return per, None


def _clock_busy(per, pick):
    """Shader clock (GHz: GRBM_GUI_ACTIVE / 8 XCDs / dispatch time, MI355X_MICROARCH.md 'DVFS
    give-back') and matrix-pipe busy fraction (SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 256 CUs x 4
    SIMDs)) over the dispatches `pick(name)` selects, time-weighted; None without the clock pass."""
    g, m = per.get("GRBM_GUI_ACTIVE"), per.get("SQ_VALU_MFMA_BUSY_CYCLES")
    if not g or not m:
        return None
    cyc = busy = ns = 0.0
    n = 0
    for disp, (name, v, dur) in g.items():
        if not pick(name) or dur <= 0 or disp not in m:
            continue
        cyc += v / 8.0
        busy += m[disp][1]
        ns += dur
        n += 1
    if n == 0 or ns <= 0:
        return None
    return {"shader_clock_ghz": round(cyc / ns, 3), "mfma_busy": round(busy / (cyc * 256 * 4), 4),
            "dispatches": n,
            "source": "rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES pass in this run (dispatch "
                      "times of that pass; clock reads high on dispatches under ~0.3 ms)"}


def measure_layer_traffic(args):
    """HBM bytes per middle residual-layer launch of THIS workload, measured in this run (two
    --pmc passes over a child running the same plan, _pmc_passes). FETCH_SIZE is doubled
    (MI355X_MICROARCH.md: gfx950 reports half the bytes of wide coalesced reads), KB -> bytes.
    Runs before this process touches the GPU. Returns (bytes or None, source note, clock/busy)."""
    per, err = _pmc_passes(args)
    if per is None:
        return None, err, None
    kernel = f"pwg_layer_{args.layer_kernel or 'split16'}_kernel<false"
    mean = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = per[ctr]
        # middle layers: not the last (<true...>) and not layer 0 with the fused first_conv
        v = [x for name, x, _ in vals.values() if kernel in name and ", true>" not in name]
        if not v:
            return None, f"rocprofv3 --pmc {ctr}: no {kernel}...> dispatches found", None
        mean[ctr] = (sum(v) / len(v), len(v))
    fetch = mean["FETCH_SIZE"][0] * 1024 * 2
    write = mean["WRITE_SIZE"][0] * 1024
    note = (f"measured in this run: rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) and WRITE_SIZE passes over "
            f"two forwards of this workload in a child process, mean of {mean['FETCH_SIZE'][1]} middle-layer launches; "
            f"read {fetch / 1e9:.3f} GB + write {write / 1e9:.3f} GB")
    clk = _clock_busy(per, lambda name: kernel in name and ", true>" not in name)
    return fetch + write, note, clk


# kernels of a conv-network forward: the executor's own (pwg_cnet_*) and those it launches from
# pwg_mstack.hip / pwg_rstack.hip (fused stack chains, batched stacks, wide-stack conv and 1x1)
_PROG_KERNELS = ("pwg_cnet_", "pwg_mstack_", "pwg_rstack_", "pwg_rconv_", "pwg_r1x1")


def _prog_kernel(name):
    return any(t in name for t in _PROG_KERNELS) and "desc_kernel" not in name


def measure_program_traffic(args):
    """Vocoder configs: HBM bytes of ONE whole forward (every launch of the conv program), measured
    as measure_layer_traffic does, from the second of the child's two forwards (the later half of
    its dispatches). Returns (bytes or None, source note, {kernel: bytes} of the top kernels,
    clock/busy of the whole program and of its top kernels)."""
    per, err = _pmc_passes(args)
    if per is None:
        return None, err, None, None
    tot, by_kernel, n_fwd = {}, {}, 0
    short = lambda name: name.replace("(anonymous namespace)::", "").replace("pwg::", "").split("(")[0].replace("void ", "")  # noqa: E731
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = per[ctr]
        # the conv program's own launches only (module setup runs torch / copy kernels before them)
        ids = sorted(i for i in vals if _prog_kernel(vals[i][0]) or "desc_kernel" in vals[i][0])
        second = ids[len(ids) // 2:]
        n_fwd = len(second)
        scale = 2048.0 if ctr == "FETCH_SIZE" else 1024.0
        tot[ctr] = sum(vals[i][1] for i in second) * scale
        for i in second:
            name = short(vals[i][0])
            by_kernel[name] = by_kernel.get(name, 0.0) + vals[i][1] * scale
    note = (f"measured in this run: rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) and WRITE_SIZE passes over "
            f"two forwards in a child process, the second forward's {n_fwd} conv-program launches; read "
            f"{tot['FETCH_SIZE'] / 1e9:.3f} GB + write {tot['WRITE_SIZE'] / 1e9:.3f} GB per forward")
    top = dict(sorted(((k, round(v / 1e9, 4)) for k, v in by_kernel.items()), key=lambda kv: -kv[1])[:6])
    clk = _clock_busy(per, _prog_kernel)
    if clk is not None:
        # the kernels that take the most time in the clock pass
        dur = {}
        for name, _, d in per["GRBM_GUI_ACTIVE"].values():
            if _prog_kernel(name):
                dur[short(name)] = dur.get(short(name), 0) + d
        slow = sorted(dur, key=lambda k: -dur[k])[:5]
        clk["per_kernel"] = {}
        for k in slow:
            v = _clock_busy(per, lambda name, k=k: short(name) == k) or {}
            v.pop("source", None)
            v["ms_per_forward"] = round(dur[k] / 2e6, 3)
            clk["per_kernel"][k] = v
    return tot["FETCH_SIZE"] + tot["WRITE_SIZE"], note, top, clk


def pmc_child(args):
    """--pmc-child: two forwards of the bench plan (PWG or vocoder), nothing printed (profiled by
    _pmc_passes)."""
    dev = torch.device("cuda", 0)
    if args.config in VOCODERS:
        m, eng, _, _, _ = vocoder_setup(args, dev)
        lengths = synthetic.libritts_lengths(args.utts, seed=3)
        plan = eng.plan(lengths.tolist())
        rs = np.random.RandomState(100)
        mel = torch.from_numpy(rs.standard_normal(int(lengths.sum()) * 80).astype(np.float32)).to(dev)
        out = torch.empty(plan.out_rows * eng.out_channels, dtype=torch.float32, device=dev)
        for _ in range(2):
            eng.run(plan, mel, out, check=False)
        torch.cuda.synchronize(dev)
        return
    params = configs.generator_params(args.config)
    eng = Engine(params, dev)
    eng.set_option("layer_kernel", args.layer_kernel or "split16")
    eng.load_state_dict(synthetic.make_state_dict(params, seed=0))
    lengths = synthetic.libritts_lengths(args.utts, seed=3)
    plan = eng.plan(lengths.tolist())
    rs = np.random.RandomState(100)
    mel = torch.from_numpy(rs.standard_normal(int(lengths.sum()) * params["aux_channels"]).astype(np.float32)).to(dev)
    noise = torch.from_numpy(rs.standard_normal(plan.total_samples).astype(np.float32)).to(dev)
    out = torch.empty(plan.total_samples * params["out_channels"], dtype=torch.float32, device=dev)
    for _ in range(2):
        eng.run(plan, mel, noise, out, check=False)
    torch.cuda.synchronize(dev)


def host_cpus():
    """CPUs this process may use and how that was decided: the scheduler affinity mask capped by a
    cgroup v2 CPU quota when one is set (on the GPU box os.cpu_count() reports the whole host,
    while the job's share is smaller), plus os.cpu_count() and the lscpu model name for the
    record."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        quota = None
    threads = min(aff, quota) if quota else aff
    model = "?"
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        model = next((ln.split(":", 1)[1].strip() for ln in out.splitlines() if ln.startswith("Model name")), "?")
    except (OSError, subprocess.SubprocessError):
        pass
    return threads, {"os_cpu_count": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                     "cpu_model": model}


def cpu_subset(n_total=512, n_pick=16, seed=3):
    """BASELINE.md sec 4's fixed CPU subset of the 512-utterance LibriTTS list
    (RandomState(3).randint(80, 1200)): n_pick utterances at evenly spaced length ranks, so the
    sample spans the length distribution. Returns (indices, lengths)."""
    lengths = synthetic.libritts_lengths(n_total, seed=seed)
    order = np.argsort(lengths, kind="stable")
    idx = [int(order[int((k + 0.5) * n_total / n_pick)]) for k in range(n_pick)]
    return idx, lengths[idx]


def cpu_baseline(params, sd, config, n_utts, reps=1):
    """Time the torch-CPU restatement of the reference (oracle/pwg_torch_cpu.py, the reference's
    aten op sequence; within 2-9 % of the imported reference on the same 8 cores,
    profiles/r02_cpu/cpu_crosscheck.json) on a bounded sample of the workload, B=1 per utterance
    like bin/decode.py, one warm-up call, each utterance timed `reps` times (best kept).
    BASELINE.md sec 4's protocol is the 16-utterance subset, best of 3 (`--cpu-utts 16 --cpu-reps
    3`, ~5 min of CPU); the default bench line times 4 of those utterances once (~25 s) to stay
    within the bench's bounded CPU sample, and says so. Returns the cpu_baseline object."""
    from oracle.pwg_torch_cpu import TorchCPUGenerator

    threads, info = host_cpus()
    torch.set_num_threads(threads)
    gen = TorchCPUGenerator(sd, params)
    A = params["aux_channels"]
    H = int(np.prod(params["upsample_params"]["upsample_scales"]))
    gen.inference(synthetic.make_mel(40, A, seed=99), synthetic.make_noise(40 * H, seed=98))  # warm-up
    idx, lengths = cpu_subset(n_pick=n_utts)
    done, t_total, rates = 0, 0.0, []
    for i, f in zip(idx, lengths):
        mel = synthetic.make_mel(int(f), A, seed=1000 + i)
        noise = synthetic.make_noise(int(f) * H, seed=2000 + i)
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            gen.inference(mel, noise)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        t_total += best
        done += int(f) * H
        rates.append(int(f) * H / best)
    protocol = ("BASELINE.md sec 4 protocol (16-utterance subset, best of 3)" if n_utts >= 16 and reps >= 3 else
                f"BASELINE.md sec 4's 16-utterance subset, best of {reps}" if n_utts >= 16 else
                f"{len(idx)} of BASELINE.md sec 4's 16 subset utterances, best of {reps}")
    desc = (f"{config}: {len(idx)} utterances of the 512-utterance RandomState(3) list at evenly spaced length "
            f"ranks (T' = {', '.join(str(int(f)) for f in lengths)}; {done} samples), B=1 each, torch-CPU aten "
            f"restatement of the reference op sequence, {threads} threads; {protocol}")
    rates.sort()
    spread = {"min": round(rates[0], 1), "median": round(rates[len(rates) // 2], 1), "max": round(rates[-1], 1),
              "unit": "audio samples/s per utterance"}
    return dict({"value": round(done / t_total, 1), "unit": "audio samples/s", "cores": threads, "kind": "port",
                 "sample": desc, "seconds": round(t_total, 2), "per_utterance_spread": spread}, **info)


VOCODERS = ["mb_melgan_v2", "hifigan_v1", "melgan_v1"]


def program_flops_per_frame(P):
    """Algorithmic FLOP per input frame of a conv program (each op: 2 * out * K per output row)."""
    from parallelwavegan_amd import cnet

    fl = 0.0
    for op in P.ops:
        rows = P.rate[op["dst"]]
        if op["kind"] == cnet.CONV:
            k = sum(s["channels"] * s["taps"] for s in op["srcs"])
        elif op["kind"] == cnet.CONVT:
            k = op["srcs"][0]["channels"] * 2
        else:  # PQMF: (taps / S) taps x S bands per output sample
            k = op["padding"]
        fl += 2.0 * op["out_channels"] * k * rows
    return fl


def program_bytes_per_frame(P):
    """Algorithmic HBM bytes per input frame: every op reads its sources / residual once and
    writes its destination once (fp32, unpadded channels)."""
    b = 0.0
    for op in P.ops:
        rows = P.rate[op["dst"]]
        for s in op["srcs"]:
            b += 4.0 * s["channels"] * P.rate[s["buf"]]
        if op["res"] >= 0:
            b += 4.0 * op["out_channels"] * rows
        b += 4.0 * op["out_channels"] * rows * (2 if op["accumulate"] else 1)
    return b


# SURVEY sec. 8(d)(5)'s 512-utterance list (RandomState(3), 80-1199 frames): 97 lengths repeat
REPEAT_LIST = [int(f) for f in synthetic.libritts_lengths(512, seed=3)]


def span_and_overhead(eng, call, timed, reps):
    """Device span and host overhead measured over the SAME calls: timing mode 2 (one event pair
    around each run), per call its wall time (synchronised) and its device span; returns the median
    span and the median of wall - span (clipped at 0: the span lies inside the wall clock)."""
    spans, overs = [], []
    eng.set_timing(2)
    eng.collect_timing()
    for _ in range(max(5, reps // 2)):
        wall = timed(call)
        sp = eng.timing_span()
        eng.collect_timing()
        spans.append(sp)
        overs.append(max(wall - sp, 0.0))
    eng.set_timing(False)
    return float(np.median(spans)), float(np.median(overs))


def decode_loop_row(call, lengths, dev, hop, noise=False):
    """The reference's decode loop (bin/decode.py:236-268): one B = 1 call per utterance, each at its
    own length, every call the first at that length (plan build, workspace growth and graph policy
    included). Mean / median wall ms per call (synchronised), over all utterances and over those of
    at most 512 frames."""
    ms = []
    for i, f in enumerate(lengths):
        args = [torch.from_numpy(synthetic.make_mel(int(f), 80, seed=500 + i)).to(dev)]
        if noise:  # explicit x (PWG), drawn outside the timed call
            args.append(torch.from_numpy(synthetic.make_noise(int(f) * hop, seed=700 + i)).to(dev))
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        call(*args)
        torch.cuda.synchronize(dev)
        ms.append((time.perf_counter() - t0) * 1e3)
    ms = np.array(ms)
    short = ms[np.asarray(lengths) <= 512]
    samples = int(np.sum(lengths)) * hop
    return {"pattern": "decode loop: B=1, one call per utterance, in list order" +
                       (", every length new" if len(set(int(f) for f in lengths)) == len(lengths) else
                        " (lengths repeat: the reference's own list)"),
            "utterances": len(lengths), "distinct_lengths": len(set(int(f) for f in lengths)),
            "frames": f"RandomState(3) LibriTTS list, {int(np.min(lengths))}-{int(np.max(lengths))}",
            "mean_ms_per_call": round(float(ms.mean()), 3), "median_ms_per_call": round(float(np.median(ms)), 3),
            "max_ms_per_call": round(float(ms.max()), 3),
            "short_utterances": int(short.size),
            "mean_ms_per_call_le512_frames": round(float(short.mean()), 3) if short.size else None,
            "samples_per_s": round(samples / (ms.sum() * 1e-3), 1)}


def vocoder_latency_rows(m, dev, reps=10):
    """the drop-in's inference() (B = 1, the reference decode loop) and
    inference_batch (B = 16 equal-length) at T' in {64, 512, 2048}: median wall ms per call with
    device-resident mels (synchronised), and the device span of one call's launches (first start
    to last end over every stream, pwg_cnet_timing_span; kernel_sum_ms adds the per-launch times,
    concurrent launches counted each). First: the decode loop over 32 distinct lengths."""
    rows = []
    eng = m.engine()
    hop = eng.hop
    lengths = synthetic.libritts_lengths(32, seed=3)
    with torch.no_grad():
        m.inference(torch.from_numpy(synthetic.make_mel(7, 80, seed=1)).to(dev))  # engine built, weights packed
        loop = decode_loop_row(lambda mel: m.inference(mel), lengths, dev, hop)
        # the reference's own pattern with its repeats: the first 128 utterances of the 512-utterance
        # RandomState(3) list, in order (10 repeated lengths)
        loop_rep = decode_loop_row(lambda mel: m.inference(mel), REPEAT_LIST[:128], dev, hop)

    def timed(fn):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e3

    with torch.no_grad():
        for F in (64, 512, 2048):
            for B in (1, 16):
                mels = [torch.from_numpy(synthetic.make_mel(F, 80, seed=30 + b)).to(dev) for b in range(B)]
                call = (lambda: m.inference(mels[0])) if B == 1 else (lambda: m.inference_batch(mels))
                first = timed(call)
                for _ in range(2):
                    call()
                ms = sorted(timed(call) for _ in range(reps))
                span, over = span_and_overhead(eng, call, timed, reps)
                eng.set_timing(1)  # per-launch events
                call()
                torch.cuda.synchronize(dev)
                eng.set_timing(False)
                kern = sum(t for _, t, _ in eng.collect_timing())
                med = ms[len(ms) // 2]
                rows.append({"frames": F, "batch": B, "samples_per_call": F * hop * B, "first_call_ms": round(first, 3),
                             "median_ms": round(med, 3), "kernel_span_ms": round(span, 3),
                             "kernel_sum_ms": round(kern, 3), "host_overhead_ms": round(over, 3),
                             "samples_per_s": round(F * hop * B / (med * 1e-3), 1)})
    return {"model": f"{type(m).__name__}.inference / inference_batch (drop-in)", "decode_loop": loop,
            "decode_loop_repeats": loop_rep, "rows": rows,
            "note": "kernel_span_ms: median device span of eager calls (HIP events around the whole run only; "
                    "graph replay is off while timing); host_overhead_ms: median over those same calls of wall "
                    "minus span (>= 0 by construction); median_ms: wall time of the default path (graph replay "
                    "for repeated small HiFiGAN plans); kernel_sum_ms: per-launch event times summed "
                    "(concurrent launches each counted)"}


def vocoder_exact_fp32_leg(eng, plan, out_mel, out, flop_step, samples, steps):
    """The precision-matched vocoder number: the same batch on the exact
    fp32 MFMA kernels (PWG_CNET_OPT_SPLIT_F16 0, v_mfma_f32_32x32x2_f32, no fp16 pairs), one
    warm-up and `steps` timed forwards; roofline on the fp32 MFMA peak with the program's
    algorithmic FLOPs (every product executed once in this mode)."""
    dev = eng.device
    eng.set_split_f16(False)
    try:
        eng.run(plan, out_mel, out, check=False)
        torch.cuda.synchronize(dev)
        eng.set_timing(True)
        eng.collect_timing()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.run(plan, out_mel, out, check=False)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        eng.set_timing(False)
        kern_s = sum(ms for _, ms, _ in eng.collect_timing()) / 1e3 / steps
    finally:
        eng.set_split_f16(True)
    if not torch.isfinite(out).all():
        raise RuntimeError("non-finite exact-fp32 vocoder output")
    tf = flop_step / kern_s / 1e12
    return {"kernel": "conv program on the exact-fp32 MFMA kernels (PWG_CNET_OPT_SPLIT_F16 0)", "dtype": "f32",
            "value": round(samples * steps / wall, 1), "unit": "audio samples/s", "steps": steps,
            "ms_per_step": round(wall / steps * 1e3, 3), "kernel_ms_per_step": round(kern_s * 1e3, 3),
            "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tf / FP32_PEAK_TFLOPS, 4), "flop_per_step": int(flop_step)}}


def vocoder_setup(args, dev):
    """The drop-in module of a vocoder config with seeded weights on `dev` and its engine set up
    as the bench runs it. Returns (module, engine, class name, params, (state dict, PQMF taps))."""
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(args.config)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    sd = synthetic.make_module_state_dict(m, seed=0)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    syn = None
    if args.config in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[args.config])
        syn = m.pqmf.synthesis_taps()
    m = m.to(dev)
    eng = m.engine()
    eng.set_split_f16(not args.cnet_fp32)
    eng.set_fuse_pairs(not args.cnet_nofuse)
    if getattr(args, "cnet_streams", None) is not None:
        eng.set_streams(args.cnet_streams)
    if args.pair_steps:
        eng.set_pair_steps(args.pair_steps)
    return m, eng, cls_name, params, (sd, syn)


def bench_vocoder(args, rank, world, dev, live_traffic=(None, "off", None, None), embedded=False):
    """MelGAN-family generator inference (BASELINE configs[2] multi_band_melgan.v2 and [3]
    hifigan.v1) on the conv-network executor: same ragged-batch workload shape
    as the PWG bench, weak scaling, utterance sharding, RCCL weight broadcast.
    embedded: called from the default PWG line (N = 1): return the result object instead of
    printing it (the line's "vocoders" object)."""
    from oracle.melgan_torch_cpu import TorchCPUVocoder  # cpu_baseline leg only
    from parallelwavegan_amd.engine import fold_weight_norm

    m, eng, cls_name, params, (sd, syn) = vocoder_setup(args, dev)
    if world > 1:
        broadcast_packed_weights(eng.packed, src=0)
    P = eng.program
    hop = eng.hop
    fs = configs.SAMPLING_RATE[args.config]
    lengths = synthetic.libritts_lengths(args.utts, seed=3)
    plan = eng.plan(lengths.tolist())
    rs = np.random.RandomState(100 + rank)
    mel = torch.from_numpy(rs.standard_normal(int(lengths.sum()) * 80).astype(np.float32)).to(dev)
    out = torch.empty(plan.out_rows * eng.out_channels, dtype=torch.float32, device=dev)
    for _ in range(args.warmup):
        eng.run(plan, mel, out, check=False)
    torch.cuda.synchronize(dev)
    # untimed pass with per-op timing on: its events return to the executor's pool, so the timed
    # steps record pooled events instead of creating ~2 per op on the host between launches
    eng.set_timing(True)
    for _ in range(args.steps):
        eng.run(plan, mel, out, check=False)
    torch.cuda.synchronize(dev)
    eng.collect_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run(plan, mel, out, check=False)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    local_elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(local_elapsed, dev)
    rank_seconds = per_rank_seconds(local_elapsed, world, dev) if not embedded else [local_elapsed]
    eng.set_timing(False)
    timing = eng.collect_timing()
    if eng.split_f16:
        eng.run_status(plan)  # split-f16 range flag of the last timed run (raises when set)
    if not torch.isfinite(out).all():
        raise RuntimeError("non-finite generator output")
    samples = int(lengths.sum()) * hop
    value = samples * world * args.steps / elapsed
    if rank != 0:
        if not embedded:
            dist.destroy_process_group()
        return None
    fl_frame = program_flops_per_frame(P)
    by_frame = program_bytes_per_frame(P)
    kern_ms = sum(ms for _, ms, _ in timing) / args.steps
    voc_bytes = live_traffic[0] and int(live_traffic[0])  # HBM bytes of one forward (rocprofv3 --pmc)
    frames = int(lengths.sum())
    achieved = fl_frame * frames / (kern_ms * 1e-3) / 1e12
    top = sorted(timing, key=lambda r: -r[1])[:5]
    cpu = None
    if args.cpu_seconds > 0 and world == 1:
        threads, info = host_cpus()
        torch.set_num_threads(threads)
        gen = TorchCPUVocoder(cls_name, fold_weight_norm(sd), params, syn)
        gen.inference(synthetic.make_mel(40, 80, seed=99))
        done, tt, used = 0, 0.0, 0
        for i, f in enumerate(lengths):
            c = synthetic.make_mel(int(f), 80, seed=1000 + i)
            t1 = time.perf_counter()
            gen.inference(c)
            tt += time.perf_counter() - t1
            done += int(f) * hop
            used += 1
            if tt >= args.cpu_seconds:
                break
        cpu = dict({"value": round(done / tt, 1), "unit": "audio samples/s", "cores": threads, "kind": "port",
                    "sample": f"{args.config}: {used} utterances ({done} samples, first of the bench batch), B=1, "
                              f"torch-CPU restatement of the reference op sequence, {threads} threads"}, **info)
    exact = None
    if world == 1 and not args.cnet_fp32 and not getattr(args, "no_exact", False):
        exact = vocoder_exact_fp32_leg(eng, plan, mel, out, fl_frame * frames, samples, max(2, min(args.steps, 3)))
    lat = None
    if not args.no_latency and world == 1:
        lat = vocoder_latency_rows(m, dev)
    res = {
        "metric": f"audio samples/sec/GPU ({fs / 1000:g} kHz {args.config}, 80-band mel)",
        "value": round(value, 1),
        "unit": "audio samples/s (whole job, all GPUs)",
        "n_gpus": world if os.environ.get("PWG_BENCH_BACKEND", "nccl") == "nccl"
                  else min(world, max(torch.cuda.device_count(), 1)),
        "ranks": world,
        "rank_seconds": [round(x, 4) for x in rank_seconds],
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.cnet_fp32 else "f32 (fp16 hi+lo pair operands, 3 f16 MFMAs per product, fp32 accumulate)",
        "data": "synthetic (seeded N(0,1) mel, seeded N(0, 1/fan_in) weights)",
        "config": {"workload": f"{args.config} generator inference, {args.utts} ragged utterances per GPU per step",
                   "model": cls_name, "sampling_rate": fs, "hop": hop, "global_batch": args.utts * world,
                   "frames_per_gpu": frames, "samples_per_step_per_gpu": samples,
                   "parallelism": f"utterance-sharded x{world}",
                   "fused_conv_pairs": sum(1 for _, _, n in timing if n == 0)},
        "x_realtime_per_gpu": round(value / world / fs, 1),
        "range_check": "ok (pwg_cnet_run_status after the timed steps)" if eng.split_f16 else "n/a (exact fp32)",
        "kernel_ms_per_step": round(kern_ms, 3),
        "top_ops_ms_per_step": {n: round(ms / args.steps, 3) for n, ms, _ in top},
        "roofline": ({"kernel": "all conv ops (fp32 MFMA implicit GEMM), whole program", "bound": "mfma",
                      "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                      "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": voc_bytes,
                      "traffic_source": live_traffic[1], "traffic_top_kernels_GB": live_traffic[2],
                      "hbm_GBs_measured": voc_bytes and round(voc_bytes / (kern_ms * 1e-3) / 1e9, 1),
                      "hbm_frac_measured": voc_bytes and round(voc_bytes / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                      "clock_pmc": live_traffic[3],
                      "flop_per_sample": round(fl_frame / hop, 1),
                      "algorithmic_bytes_per_sample": round(by_frame / hop, 1)} if args.cnet_fp32 else
                     # split-f16: every reference product runs as three f16 MFMA products
                     {"kernel": "all conv ops (split-f16 MFMA implicit GEMM), whole program", "bound": "mfma",
                      "achieved": round(3 * achieved, 3), "peak": F16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                      "frac": round(3 * achieved / F16_MFMA_PEAK_TFLOPS, 4), "traffic": voc_bytes,
                      "traffic_source": live_traffic[1], "traffic_top_kernels_GB": live_traffic[2],
                      "hbm_GBs_measured": voc_bytes and round(voc_bytes / (kern_ms * 1e-3) / 1e9, 1),
                      "hbm_frac_measured": voc_bytes and round(voc_bytes / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                      "reference_tflops": round(achieved, 3),
                      "clock_pmc": live_traffic[3],
                      "flop_per_sample": round(fl_frame / hop, 1),
                      "executed_f16_flop_per_sample": round(3 * fl_frame / hop, 1),
                      "algorithmic_bytes_per_sample": round(by_frame / hop, 1)}),
        "cpu_baseline": cpu,
        "exact_fp32": exact,
        "latency": lat,
    }
    if embedded:
        for k in ("n_gpus", "ranks", "rank_seconds", "higher_is_better", "scaling", "vs_baseline", "data", "warmup"):
            res.pop(k, None)
        res["config"].pop("parallelism", None)
        return res
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


# Vocoder configs carried in the default PWG line (BASELINE.json configs[2] and [3]).
EMBED_VOCODERS = ["mb_melgan_v2", "hifigan_v1"]


def with_config(args, config):
    """A copy of the parsed arguments with another --config (the embedded vocoder runs)."""
    a = argparse.Namespace(**vars(args))
    a.config = config
    a.layer_kernel = None
    return a


def exact_fp32_leg(eng, plan, mel, noise, out, params, steps):
    """The precision-matched number: the same PWG bench batch on the
    exact-fp32 layer kernel (pwg_layer_persistent_kernel, v_mfma_f32_32x32x2_f32, no fp16 pairs),
    one warm-up and `steps` timed forwards, per-launch HIP events. The roofline is the fp32 MFMA
    peak in the reference formulation's FLOPs."""
    dev = eng.device
    kernel = eng.layer_kernel
    eng.set_option("layer_kernel", "persistent")
    try:
        eng.run(plan, mel, noise, out, check=False)
        torch.cuda.synchronize(dev)
        eng.set_timing(True)
        eng.collect_timing()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.run(plan, mel, noise, out, check=False)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        eng.set_timing(False)
        timing = eng.collect_timing()
    finally:
        eng.set_option("layer_kernel", kernel)
    if not torch.isfinite(out).all():
        raise RuntimeError("non-finite exact-fp32 output")
    layer_ms, layer_n = timing["residual_layer"]
    avg_s = layer_ms / 1e3 / max(layer_n, 1)
    flop_launch = layer_flops_per_sample(params) * plan.total_samples
    # executed: the dilated conv and the skip / out 1x1s per sample; the aux 1x1 runs once per frame
    # in pwg_aux_proj_kernel (its rows are interpolated in the layer), so the layer executes
    # 2 (K R G + G/2 (S + R)) FLOP per sample (0.762 of the reference's per LibriTTS v1 layer)
    R, G, S, K = (params[k] for k in ("residual_channels", "gate_channels", "skip_channels", "kernel_size"))
    exec_launch = 2 * (K * R * G + (G // 2) * (S + R)) * plan.total_samples
    tf = exec_launch / avg_s / 1e12
    tf_ref = flop_launch / avg_s / 1e12
    return {"kernel": "pwg_layer_persistent_kernel (exact fp32, v_mfma_f32_32x32x2_f32)", "dtype": "f32",
            "value": round(plan.total_samples * steps / wall, 1), "unit": "audio samples/s",
            "steps": steps, "ms_per_step": round(wall / steps * 1e3, 3),
            "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tf / FP32_PEAK_TFLOPS, 4), "avg_launch_ms": round(avg_s * 1e3, 4),
                         "launches_timed": layer_n, "executed_flop_per_launch": int(exec_launch),
                         "reference_flop_per_launch": int(flop_launch),
                         "reference_formulation_tflops": round(tf_ref, 2),
                         "note": "frac on executed FLOPs (dilated conv + skip/out 1x1s per sample; the aux 1x1 "
                                 "runs at frame rate); reference_formulation_tflops counts the per-sample aux 1x1 "
                                 "the reference executes, and can exceed the fp32 peak"}}


def latency_rows(dev, reps=20):
    """The reference's own call pattern (bin/decode.py:236-268: one utterance per inference()
    call, B=1) through the drop-in module, SURVEY.md sec 8(d)(2): LJ v1 at T' in {64, 512, 2048},
    B=1 and B=16 equal-length (inference_batch). Per call: wall ms of the first call at a new
    length (plan build included), median / min wall ms of repeated calls with device-resident
    inputs (synchronised, range check included), host-to-host ms (numpy mel/noise in, .cpu() out,
    like decode.py), and the device span of the call's launches (first start to last end, HIP
    events). First: the decode loop over 32 distinct lengths (every call at a new length)."""
    from parallelwavegan_amd import ParallelWaveGANGenerator

    params = configs.generator_params("ljspeech_v1")
    m = ParallelWaveGANGenerator(**params)
    m.remove_weight_norm()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(params, seed=0).items()})
    m = m.eval().to(dev)
    H = m.upsample_factor
    rows = []
    lengths = synthetic.libritts_lengths(32, seed=3)
    with torch.no_grad():
        m.inference(torch.from_numpy(synthetic.make_mel(7, 80, seed=1)).to(dev),
                    torch.from_numpy(synthetic.make_noise(7 * H, seed=1)).to(dev))  # engine built, weights packed
        loop = decode_loop_row(lambda mel, x: m.inference(mel, x), lengths, dev, H, noise=True)
        loop_rep = decode_loop_row(lambda mel, x: m.inference(mel, x), REPEAT_LIST[:128], dev, H, noise=True)

    def timed(fn):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e3

    with torch.no_grad():
        for F in (64, 512, 2048):
            for B in (1, 16):
                mels_h = [synthetic.make_mel(F, 80, seed=30 + b) for b in range(B)]
                noises_h = [synthetic.make_noise(F * H, seed=60 + b) for b in range(B)]
                mels = [torch.from_numpy(x).to(dev) for x in mels_h]
                noises = [torch.from_numpy(x).to(dev) for x in noises_h]
                if B == 1:
                    call = lambda: m.inference(mels[0], noises[0])  # noqa: E731
                    call_host = lambda: m.inference(mels_h[0], noises_h[0]).cpu()  # noqa: E731
                else:
                    call = lambda: m.inference_batch(mels, noises)  # noqa: E731
                    call_host = lambda: [y.cpu() for y in m.inference_batch(mels_h, noises_h)]  # noqa: E731
                first = timed(call)
                for _ in range(3):
                    call()
                dev_ms = sorted(timed(call) for _ in range(reps))
                host_ms = sorted(timed(call_host) for _ in range(max(3, reps // 4)))
                eng = m.engine()
                graph_ms = None
                if B == 1:
                    # the same call pattern replayed from a HIP graph (pwg_graph_create): inputs
                    # copied into the graph's buffers, one submission, range check included
                    g = GraphedRun(eng, eng.plan([F]))
                    for _ in range(3):
                        g(mels[0], noises[0])
                    graph_ms = sorted(timed(lambda: g(mels[0], noises[0])) for _ in range(reps))
                    del g
                kern, over = span_and_overhead(eng, call, timed, reps)
                med = dev_ms[len(dev_ms) // 2]
                rows.append({"frames": F, "batch": B, "samples_per_call": F * H * B,
                             "first_call_ms": round(first, 3), "median_ms": round(med, 3),
                             "min_ms": round(dev_ms[0], 3), "host_to_host_median_ms": round(host_ms[len(host_ms) // 2], 3),
                             "kernel_span_ms": round(kern, 3), "host_overhead_ms": round(over, 3),
                             "graph_replay_median_ms": graph_ms and round(graph_ms[len(graph_ms) // 2], 3),
                             "samples_per_s": round(F * H * B / (med * 1e-3), 1)})
    return {"model": "ljspeech_v1 ParallelWaveGANGenerator.inference / inference_batch (drop-in)",
            "decode_loop": loop, "decode_loop_repeats": loop_rep, "rows": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="libritts_v1",
                    choices=["libritts_v1", "ljspeech_v1", "yesno_debug"] + VOCODERS)
    ap.add_argument("--utts", type=int, default=32, help="utterances per GPU per step (weak scaling)")
    ap.add_argument("--strong", action="store_true",
                    help="SURVEY.md sec 8(d)(5): the fixed 512-utterance RandomState(3) list, LPT-sharded over "
                         "the ranks (strong scaling); one step = the whole list")
    ap.add_argument("--cpu-seconds", type=float, default=None, help="0 = skip the CPU baseline (other values: legacy)")
    ap.add_argument("--cpu-utts", type=int, default=16,
                    help="CPU baseline sample: utterances of BASELINE.md sec 4's stratified subset (16 = all of it)")
    ap.add_argument("--cpu-reps", type=int, default=1, help="CPU baseline: timings per utterance, best kept (3 = BASELINE.md)")
    ap.add_argument("--no-latency", action="store_true", help="skip the B=1 / B=16 latency rows")
    ap.add_argument("--no-vocoders", action="store_true",
                    help="PWG line: skip the embedded MB-MelGAN v2 / HiFiGAN v1 runs (configs[2], [3])")
    ap.add_argument("--no-exact", action="store_true", help="PWG line: skip the exact-fp32 leg")
    ap.add_argument("--voc-cpu-seconds", type=float, default=6.0,
                    help="embedded vocoder runs: CPU-baseline budget per vocoder (0 = skip)")
    ap.add_argument("--sub-plans", type=int, default=1,
                    help="experiment: run the per-GPU utterances as this many sequential sub-batches")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "layer_traffic.json"),
                    help="fallback for roofline.traffic when the in-run PMC passes are off or fail")
    ap.add_argument("--pmc", choices=["auto", "off"], default="auto",
                    help="auto: measure roofline.traffic with two rocprofv3 --pmc passes before the run (N=1)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--layer-kernel", default=None, choices=["split", "split16", "persistent", "tiled"],
                    help="default: split where the shape allows, else persistent (the engine default)")
    ap.add_argument("--waves-per-wg", type=int, default=None)
    ap.add_argument("--wg-per-cu", type=int, default=None)
    ap.add_argument("--no-fuse-first", action="store_true", help="split16: standalone first_conv kernel (A/B)")
    ap.add_argument("--cnet-fp32", action="store_true", help="vocoder configs: exact fp32 MFMA instead of split-f16")
    ap.add_argument("--cnet-nofuse", action="store_true", help="vocoder configs: run fusable conv pairs unfused")
    ap.add_argument("--cnet-streams", type=int, default=None, choices=[0, 1, 2],
                    help="vocoder configs: PWG_CNET_OPT_STREAMS (A/B; default: the library's, 1)")
    ap.add_argument("--pair-steps", type=int, default=None, help="vocoder configs: 128-column tiles per fused-pair strip")
    args = ap.parse_args()
    if args.cpu_seconds is None:
        args.cpu_seconds = 12.0
    if args.cpu_seconds == 0:
        args.cpu_utts = 0

    if args.pmc_child:
        return pmc_child(args)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    # measured HBM traffic of the dominant kernel, before this process touches the GPU
    live_traffic = (None, "off", None)
    single = args.pmc == "auto" and int(os.environ.get("WORLD_SIZE", "1")) == 1
    if (single and args.config not in VOCODERS
            and not args.strong and args.sub_plans == 1 and args.layer_kernel in (None, "split16")
            and not args.no_fuse_first and not args.waves_per_wg and not args.wg_per_cu):
        live_traffic = measure_layer_traffic(args)
    voc_traffic = (None, "off", None, None)
    if single and args.config in VOCODERS:
        voc_traffic = measure_program_traffic(args)
    embed = (int(os.environ.get("WORLD_SIZE", "1")) == 1 and args.config not in VOCODERS and not args.strong
             and not args.no_vocoders and args.sub_plans == 1)
    embed_traffic = {}
    if embed:
        for vc in EMBED_VOCODERS:
            embed_traffic[vc] = (measure_program_traffic(with_config(args, vc)) if args.pmc == "auto"
                                 else (None, "off", None, None))
    rank, world, dev = dist_setup(args.gpus)
    _lib.build()
    if args.config in VOCODERS:
        return bench_vocoder(args, rank, world, dev, voc_traffic)
    params = configs.generator_params(args.config)
    fs = configs.SAMPLING_RATE[args.config]
    eng = Engine(params, dev)
    if args.layer_kernel is None:
        try:
            eng.set_option("layer_kernel", "split16")
            args.layer_kernel = "split16"
        except NotImplementedError:
            args.layer_kernel = "persistent"
    eng.set_option("layer_kernel", args.layer_kernel)
    if args.waves_per_wg:
        eng.set_option("waves_per_wg", args.waves_per_wg)
    if args.wg_per_cu:
        eng.set_option("wg_per_cu", args.wg_per_cu)
    fuse_first = args.layer_kernel == "split16" and not args.no_fuse_first and params["layers"] > 1
    eng.set_option("fuse_first_conv", 0 if args.no_fuse_first else 1)
    H = eng.upsample_factor
    A = params["aux_channels"]

    # weights: packed on rank 0 and broadcast to the other ranks, the design's one collective
    # (start-up only): the C-ABI's RCCL path (pwg_broadcast_weights) on the nccl backend
    sd = synthetic.make_state_dict(params, seed=0)
    if rank == 0:
        packed = torch.from_numpy(eng.pack(sd)).to(dev)
    else:
        packed = torch.empty(eng.packed_weight_count, dtype=torch.float32, device=dev)
    broadcast = "none (one process)"
    if world > 1:
        if os.environ.get("PWG_BENCH_BACKEND", "nccl") == "nccl":
            try:
                broadcast_weights_rccl(eng, packed, src=0)
                broadcast = "pwg_broadcast_weights (C-ABI, RCCL over xGMI)"
            except (RuntimeError, OSError, NotImplementedError) as e:
                # the C-ABI broadcast is the design's one collective: a failure ends the run unless
                # a fallback was asked for explicitly (every rank agrees on the outcome first,
                # sharding.broadcast_weights_rccl, so no rank waits on a broken communicator)
                if os.environ.get("PWG_BENCH_BCAST_FALLBACK") != "1":
                    raise
                print(f"[bench] C-ABI RCCL broadcast failed ({e}); PWG_BENCH_BCAST_FALLBACK=1: "
                      "using torch.distributed.broadcast", file=sys.stderr)
                broadcast_packed_weights(packed, src=0)
                broadcast = "torch.distributed.broadcast over RCCL (C-ABI broadcast failed, fallback asked for)"
        else:
            broadcast_packed_weights(packed, src=0)
            broadcast = "torch.distributed.broadcast (gloo rehearsal)"
    eng.set_packed(packed)

    if args.strong:
        all_lengths = synthetic.libritts_lengths(512, seed=3)
        shards = lpt_partition(all_lengths, world)
        mine = shards[rank]
        lengths = all_lengths[mine]
        loads = shard_loads(all_lengths, shards)
        workload = (f"{args.config} generator inference, the fixed 512-utterance RandomState(3) list "
                    f"({int(all_lengths.sum())} frames) LPT-sharded over {world} rank(s); one step = the whole list")
    else:
        # weak scaling: the same lengths on every rank, rank-specific content
        lengths = synthetic.libritts_lengths(args.utts, seed=3)
        workload = f"{args.config} generator inference, {args.utts} ragged utterances per GPU per step"
    plan = eng.plan(lengths.tolist())
    rs = np.random.RandomState(100 + rank)
    mel = torch.from_numpy(rs.standard_normal(int(lengths.sum()) * A).astype(np.float32)).to(dev)
    noise = torch.from_numpy(rs.standard_normal(plan.total_samples).astype(np.float32)).to(dev)
    out = torch.empty(plan.total_samples * params["out_channels"], dtype=torch.float32, device=dev)
    subs = None
    if args.sub_plans > 1:
        # sequential sub-batches of consecutive utterances (views into the same buffers)
        subs, f0 = [], 0
        for part in np.array_split(np.arange(len(lengths)), args.sub_plans):
            fl = [int(lengths[i]) for i in part]
            sp = eng.plan(fl)
            n = sum(fl)
            subs.append((sp, mel[f0 * A:(f0 + n) * A], noise[f0 * H:(f0 + n) * H],
                         out[f0 * H * params["out_channels"]:(f0 + n) * H * params["out_channels"]]))
            f0 += n
    torch.cuda.synchronize(dev)

    def run_step():
        if subs is None:
            eng.run(plan, mel, noise, out, check=False)
        else:
            for sp, m_, n_, o_ in subs:
                eng.run(sp, m_, n_, o_, check=False)

    for _ in range(args.warmup):
        run_step()
    torch.cuda.synchronize(dev)

    # untimed pass with per-launch timing on: its events return to the engine's pool, so the timed
    # steps record pooled events instead of creating them on the host between launches
    eng.set_timing(True)
    for _ in range(args.steps):
        run_step()
    torch.cuda.synchronize(dev)
    eng.collect_timing()  # clear
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    local_elapsed = time.perf_counter() - t0
    eng.set_timing(False)
    timing = eng.collect_timing()
    elapsed = max_over_ranks(local_elapsed, dev)
    # the split-f16 range flag of the last timed run (pwg_run_status; raises on a flagged run)
    if args.layer_kernel in ("split", "split16"):
        eng.run_status(plan)
    if not torch.isfinite(out).all():
        raise RuntimeError("non-finite generator output")
    exact = None
    if (world == 1 and not args.no_exact and not args.strong and subs is None
            and args.layer_kernel in ("split", "split16")):
        exact = exact_fp32_leg(eng, plan, mel, noise, out, params, max(2, min(args.steps, 5)))

    # PCIe-inclusive rate (never `value`): host mel + noise in pinned memory -> H2D -> forward ->
    # D2H of the audio, like inference() called on host arrays (models/parallel_wavegan.py:244-263)
    mel_h, noise_h = mel.cpu().pin_memory(), noise.cpu().pin_memory()
    out_h = torch.empty(out.numel(), dtype=torch.float32).pin_memory()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        mel.copy_(mel_h, non_blocking=True)
        noise.copy_(noise_h, non_blocking=True)
        eng.run(plan, mel, noise, out, check=False)
        out_h.copy_(out, non_blocking=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    e2e = max_over_ranks(time.perf_counter() - t0, dev)

    if args.strong:
        samples_per_step = int(all_lengths.sum()) * H
    else:
        samples_per_step = plan.total_samples * world
    value = samples_per_step * args.steps / elapsed
    per_gpu = value / world
    layer_ms, layer_n = timing["residual_layer"]
    layer_avg_s = layer_ms / 1e3 / max(layer_n, 1)
    flops_launch = layer_flops_per_sample(params) * plan.total_samples
    achieved_tflops = flops_launch / layer_avg_s / 1e12
    traffic = mfma_insts = None
    traffic_source = None
    if live_traffic[0] is not None:
        traffic, traffic_source = live_traffic[:2]
    elif os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if (tj.get("config") == args.config and tj.get("utts") == args.utts and not args.strong
                    and tj.get("layer_kernel", "persistent") == args.layer_kernel):
                traffic = tj.get("hbm_bytes_per_launch")
                mfma_insts = tj.get("mfma_insts_per_launch")
                traffic_source = (f"{os.path.relpath(args.traffic_json, REPO)} (rocprofv3 --pmc FETCH_SIZE x2 + "
                                  f"WRITE_SIZE of this workload, {tj.get('source', 'committed profile')}; "
                                  f"not measured in this run: {live_traffic[1]})")
        except (OSError, ValueError):
            traffic = None
    L = params["layers"]
    if args.layer_kernel in ("split", "split16"):
        # HBM-bound: algorithmic bytes of the engine's layer per launch / launch time
        bytes_launch = split_layer_bytes_per_sample(params, H, L, fuse_first) * plan.total_samples
        n_blocks = int(sum(-(-int(f) * H // 128) * 4 for f in lengths))
        exec_flop = split_executed_flop_per_block(L, args.layer_kernel) * n_blocks
        achieved_gbs = bytes_launch / layer_avg_s / 1e9
        roofline = {
            "kernel": f"residual layer ({args.layer_kernel} persistent kernel, one fused WaveNet residual block)",
            "bound": "hbm",
            "achieved": round(achieved_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_source,
            "algorithmic_bytes_per_launch": int(bytes_launch),
            "avg_launch_ms": round(layer_avg_s * 1e3, 4),
            "launches_timed": layer_n,
            "mfma": {
                "executed_f16_flop_per_launch": int(exec_flop),
                "achieved_tflops": round(exec_flop / layer_avg_s / 1e12, 1),
                "peak_tflops": F16_MFMA_PEAK_TFLOPS,
                "frac": round(exec_flop / layer_avg_s / 1e12 / F16_MFMA_PEAK_TFLOPS, 4),
            },
            # the reference formulation's fp32 FLOPs per launch over the same time
            "reference_flop_per_launch": int(flops_launch),
            "reference_tflops": round(achieved_tflops, 1),
            "hbm_GBs_measured": traffic and round(traffic / layer_avg_s / 1e9, 1),
            # shader clock and matrix-pipe busy of the middle-layer launches (in-run PMC pass): the
            # layer runs power-limited well under the 2.4 GHz max clock
            "clock_pmc": live_traffic[2],
        }
    else:
        roofline = {
            "kernel": f"residual layer ({args.layer_kernel} kernel, one fused WaveNet residual block)",
            "bound": "mfma",
            "achieved": round(achieved_tflops, 3),
            "peak": FP32_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved_tflops / FP32_PEAK_TFLOPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_source,
            "flop_per_launch": int(flops_launch),
            "algorithmic_bytes_per_launch": int(layer_bytes_per_sample(params) * plan.total_samples),
            "avg_launch_ms": round(layer_avg_s * 1e3, 4),
            "launches_timed": layer_n,
            # FLOPs the MFMAs actually execute (rocprofv3 SQ_INSTS_MFMA x 4096 per 32x32x2 f32 MFMA):
            # below the reference count because the aux 1x1 runs at frame rate
            "executed_flop_per_launch": mfma_insts and int(mfma_insts * 4096),
            "executed_frac": mfma_insts and round(mfma_insts * 4096 / layer_avg_s / 1e12 / FP32_PEAK_TFLOPS, 4),
            "hbm_GBs": traffic and round(traffic / layer_avg_s / 1e9, 1),
        }
    # per-rank wall time of the timed steps next to the max (load imbalance of the partition)
    rank_seconds = per_rank_seconds(local_elapsed, world, dev)

    if rank != 0:
        dist.destroy_process_group()
        return

    cpu = None
    if args.cpu_utts > 0 and world == 1:
        cpu = cpu_baseline(params, sd, args.config, args.cpu_utts, args.cpu_reps)
    lat = None
    if not args.no_latency and world == 1:
        lat = latency_rows(dev)

    parallelism = (f"utterance-sharded x{world} (no data-path collective; weights broadcast once: {broadcast})"
                   if world > 1 else "1 process, 1 GPU (no collective)")
    res = {
        "metric": "audio samples/sec/GPU (24 kHz PWG, 80-band mel) + RTF at 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "audio samples/s (whole job, all GPUs)",
        # ranks sharing a device (the gloo rehearsal on a 1-GPU box) count the devices, not ranks
        "n_gpus": world if os.environ.get("PWG_BENCH_BACKEND", "nccl") == "nccl"
                  else min(world, max(torch.cuda.device_count(), 1)),
        "ranks": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "f32 (fp16 hi+lo pair operands, 3 f16 MFMAs per product, fp32 accumulate)"
                 if args.layer_kernel in ("split", "split16") else "f32",
        "data": "synthetic (seeded N(0,1) mel + noise, seeded kaiming-init weights)",
        "config": {
            "workload": workload,
            "model": "ParallelWaveGANGenerator",
            "sampling_rate": fs,
            "hop": H,
            "global_batch": 512 if args.strong else args.utts * world,
            "frames_per_gpu": int(lengths.sum()),
            "samples_per_step_per_gpu": int(plan.total_samples),
            "parallelism": parallelism,
        },
        "value_per_gpu": round(per_gpu, 1),
        "x_realtime_per_gpu": round(per_gpu / fs, 1),
        "rtf_per_gpu": per_gpu and fs / per_gpu,
        "kernel_ms_per_step": {k: round(ms / args.steps, 3) for k, (ms, _) in timing.items()},
        "range_check": "ok (pwg_run_status after the timed steps)" if args.layer_kernel in ("split", "split16")
                       else "n/a (exact fp32)",
        "roofline": roofline,
        "model_flop_per_sample": round(model_flops_per_sample(params), 1),
        "model_tflops": round(value / world * model_flops_per_sample(params) / 1e12, 3),
        "pcie_inclusive_value": round(samples_per_step * args.steps / e2e, 1),
        "cpu_baseline": cpu,
        "latency": lat,
    }
    res["rank_seconds"] = [round(x, 4) for x in rank_seconds]
    res["exact_fp32"] = exact
    if embed:
        vocs = {}
        for vc in EMBED_VOCODERS:
            va = with_config(args, vc)
            va.cpu_seconds = args.voc_cpu_seconds
            vocs[vc] = bench_vocoder(va, 0, 1, dev, embed_traffic[vc], embedded=True)
        res["vocoders"] = vocs
    if args.strong:
        per = rank_seconds
        res["strong"] = {"shard_frames": loads, "frame_imbalance": round(max(loads) / (sum(loads) / world), 4),
                         "rank_seconds": [round(x, 4) for x in per],
                         "time_imbalance": round(max(per) / (sum(per) / world), 4)}
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
