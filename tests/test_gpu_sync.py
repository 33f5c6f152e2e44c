"""Grid-synchronised forward (PWG_OPT_SYNC; csrc/pwg_split16.hip pwg_sync_split16_kernel): residual
layers 0 .. L - 2 of a small plan in ONE launch, one workgroup per CU, a grid barrier between
layers (x and skip handed over with sc1 stores and loads), the last layer as its own launch (and
layer 0 too on whole-block plans with the fused first_conv). Every
layer runs the per-layer kernel's work units through the same block body, so the forward must be
BIT-IDENTICAL to the per-layer launches: ragged batches, utterances shorter than a block, causal
configs, first_conv fused or not, the batched forward() layout, graph replay and the drop-in's
B = 1 call (bin/decode.py:236-268). GPU only; every forward goes through include/pwg.h."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engines(params, dev, seed=0):
    from parallelwavegan_amd import Engine, synthetic

    sd = synthetic.make_state_dict(params, seed=seed)
    engs = []
    for sync in (0, 1 << 30):
        e = Engine(params, dev)
        e.load_state_dict(sd)
        e.set_option("sync", sync)
        assert e.get_option("sync") == sync
        engs.append(e)
    return engs


def _inputs(lengths, hop, dev, seed=5):
    rs = np.random.RandomState(seed)
    mels = [torch.from_numpy(rs.standard_normal((f, 80)).astype(np.float32)).to(dev) for f in lengths]
    noises = [torch.from_numpy(rs.standard_normal((f * hop, 1)).astype(np.float32)).to(dev) for f in lengths]
    return mels, noises


@pytest.mark.parametrize("cfg, lengths, over, fuse", [
    ("ljspeech_v1", [64], {}, 1),
    ("ljspeech_v1", [64], {}, 0),
    ("ljspeech_v1", [128], {}, 1),
    ("ljspeech_v1", [7, 30, 1, 2], {}, 1),
    ("libritts_v1", [43, 17, 1, 20], {}, 1),
    ("libritts_v1", [3, 1, 40], {"use_causal_conv": True}, 1),
    ("ljspeech_v1", [7, 90, 2], {"use_causal_conv": True}, 0),
    # whole-block plans (more blocks than PWG_OPT_HALF_BLOCKS allows): layer 0 runs per-layer when
    # first_conv is fused
    ("ljspeech_v1", [300], {}, 1),
    ("ljspeech_v1", [300], {}, 0),
    ("libritts_v1", [143, 17, 250], {"use_causal_conv": True}, 1),
])
def test_sync_bitwise_equal_to_per_layer(cfg, lengths, over, fuse, built_lib, cuda_device):
    from parallelwavegan_amd import configs

    params = configs.generator_params(cfg, **over)
    per_layer, sync = _engines(params, cuda_device)
    for e in (per_layer, sync):
        e.set_option("fuse_first_conv", fuse)
    hop = per_layer.upsample_factor
    mels, noises = _inputs(lengths, hop, cuda_device)
    ref = [y.cpu().numpy() for y in per_layer.infer(mels, noises)]
    got = [y.cpu().numpy() for y in sync.infer(mels, noises)]
    for a, b in zip(got, ref):
        assert np.isfinite(a).all()
        np.testing.assert_array_equal(a, b)


def test_sync_launch_count_forward_layout_and_graph(built_lib, cuda_device):
    """Two residual launches (the synchronised one and the last layer), the batched forward(z, c)
    layout (models/parallel_wavegan.py:144-173), and graph replay: all bit-identical."""
    from parallelwavegan_amd import GraphedRun, _lib, configs

    params = configs.generator_params("ljspeech_v1")
    per_layer, sync = _engines(params, cuda_device, seed=2)
    mels, noises = _inputs([33], 256, cuda_device, seed=7)
    sync.set_timing(True)
    sync.collect_timing()
    y = sync.infer(mels, noises)[0]
    t = sync.collect_timing()
    sync.set_timing(False)
    assert t["residual_layer"][1] == 2
    assert torch.equal(y, per_layer.infer(mels, noises)[0])

    B, F, w = 2, 9, params["aux_context_window"]
    rs = np.random.RandomState(3)
    c = torch.from_numpy(rs.standard_normal((B, 80, F + 2 * w)).astype(np.float32)).to(cuda_device)
    z = torch.from_numpy(rs.standard_normal((B, 1, F * 256)).astype(np.float32)).to(cuda_device)
    outs = []
    for e in (per_layer, sync):
        plan = e.plan([F] * B, _lib.PWG_LAYOUT_FORWARD)
        out = torch.empty(B, 1, F * 256, device=cuda_device)
        e.run(plan, c, z, out)
        outs.append(out.cpu().numpy())
    np.testing.assert_array_equal(outs[1], outs[0])

    g = GraphedRun(sync, sync.plan([64]))
    for seed in (1, 2):
        mels, noises = _inputs([64], 256, cuda_device, seed=seed)
        y = g(mels[0], noises[0]).clone()
        assert torch.equal(y, per_layer.infer(mels, noises)[0].reshape(-1))
    del g


def test_sync_many_runs_stay_identical(built_lib, cuda_device):
    """The barrier counter is reset by every run (plan-descriptor kernel): 20 back-to-back runs on
    one stream, no synchronisation between them, all bit-identical and none flagged."""
    from parallelwavegan_amd import configs

    params = configs.generator_params("ljspeech_v1")
    per_layer, sync = _engines(params, cuda_device, seed=4)
    mels, noises = _inputs([64, 5], 256, cuda_device, seed=9)
    ref = per_layer.infer(mels, noises)[0].clone()
    plan = sync.plan([64, 5])
    mel = torch.cat([m.reshape(-1) for m in mels])
    noise = torch.cat([n.reshape(-1) for n in noises])
    outs = [torch.empty(plan.total_samples, device=cuda_device) for _ in range(20)]
    for o in outs:
        sync.run(plan, mel, noise, o, check=False)
    sync.run_status(plan)
    for o in outs:
        assert torch.equal(o[: ref.numel()], ref.reshape(-1))


def test_sync_concurrent_streams_complete(built_lib, cuda_device):
    """Two synchronised forwards in flight at once on two streams (each wants every CU): each either
    runs with all its workgroups resident or finds the GPU shared, decides "abort" for all its
    workgroups at once and writes nothing, which pwg_run_status reports as PWG_ERR_RERUN and the
    engine's check redoes on the per-layer launches. No wait may time out, and every output is
    bit-identical to the per-layer forward."""
    from parallelwavegan_amd import configs

    params = configs.generator_params("ljspeech_v1")
    per_layer, sync = _engines(params, cuda_device, seed=6)
    lengths = [200]  # whole-block plan: 1,600 blocks, 6 per CU
    mels, noises = _inputs(lengths, 256, cuda_device, seed=11)
    ref = per_layer.infer(mels, noises)[0].reshape(-1).clone()
    plan = sync.plan(lengths)
    mel = mels[0].reshape(-1).contiguous()
    noise = noises[0].reshape(-1).contiguous()
    streams = [torch.cuda.Stream(cuda_device) for _ in range(2)]
    torch.cuda.synchronize(cuda_device)
    for _ in range(8):
        outs = [torch.empty(plan.total_samples, device=cuda_device) for _ in streams]
        for st, o in zip(streams, outs):
            with torch.cuda.stream(st):
                sync.run(plan, mel, noise, o, stream=st, check=False)
        for st, o in zip(streams, outs):
            with torch.cuda.stream(st):
                sync._range_check(plan, mel, noise, o, None, None, st)
        torch.cuda.synchronize(cuda_device)
        for o in outs:
            assert torch.equal(o, ref)
    print("sync reruns", sync.sync_reruns)


def test_sync_abort_reruns_per_layer(built_lib, cuda_device):
    """The "abort" path itself: a stream kept busy by a long per-layer forward while the
    synchronised one is queued on another stream; whatever the decision, the checked result is
    the per-layer forward's, bit for bit."""
    from parallelwavegan_amd import configs

    params = configs.generator_params("ljspeech_v1")
    per_layer, sync = _engines(params, cuda_device, seed=8)
    mels, noises = _inputs([64], 256, cuda_device, seed=12)
    ref = per_layer.infer(mels, noises)[0].reshape(-1).clone()
    big = [512] * 8
    bm, bn = _inputs(big, 256, cuda_device, seed=13)
    bplan = per_layer.plan(big)
    bmel = torch.cat([m.reshape(-1) for m in bm])
    bnoise = torch.cat([n.reshape(-1) for n in bn])
    bout = torch.empty(bplan.total_samples, device=cuda_device)
    plan = sync.plan([64])
    s1, s2 = torch.cuda.Stream(cuda_device), torch.cuda.Stream(cuda_device)
    torch.cuda.synchronize(cuda_device)
    for _ in range(4):
        with torch.cuda.stream(s1):
            per_layer.run(bplan, bmel, bnoise, bout, stream=s1, check=False)
        o = torch.empty(plan.total_samples, device=cuda_device)
        with torch.cuda.stream(s2):
            sync.run(plan, mels[0].reshape(-1), noises[0].reshape(-1), o, stream=s2)
        torch.cuda.synchronize(cuda_device)
        assert torch.equal(o, ref)
    print("sync reruns", sync.sync_reruns)


def test_sync_abort_path_writes_nothing_and_reruns(built_lib, cuda_device):
    """PWG_OPT_SYNC_ABORT forces the residency exit: the launch writes no x or skip,
    pwg_run_status returns PWG_ERR_RERUN, and Engine.run(check=True) / the drop-in redo the forward
    on the per-layer launches: bit-identical output, one rerun counted per call."""
    from parallelwavegan_amd import ParallelWaveGANGenerator, _lib, configs, synthetic

    params = configs.generator_params("ljspeech_v1")
    per_layer, sync = _engines(params, cuda_device, seed=9)
    sync.set_option("sync_abort", 1)
    mels, noises = _inputs([64, 3], 256, cuda_device, seed=14)
    ref = [y.clone() for y in per_layer.infer(mels, noises)]
    plan = sync.plan([64, 3])
    mel = torch.cat([m.reshape(-1) for m in mels])
    noise = torch.cat([n.reshape(-1) for n in noises])
    out = torch.full((plan.total_samples,), float("nan"), device=cuda_device)
    sync.run(plan, mel, noise, out, check=False)
    with pytest.raises(_lib.RerunError):
        sync.run_status(plan)
    sync.run(plan, mel, noise, out)  # check=True: reruns per-layer
    assert sync.sync_reruns == 1
    assert torch.equal(out, torch.cat([y.reshape(-1) for y in ref]))

    m = ParallelWaveGANGenerator(**params)
    m.remove_weight_norm()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(params, seed=9).items()})
    m = m.eval().to(cuda_device)
    m.engine().set_option("sync_abort", 1)
    with torch.no_grad():
        y = m.inference(mels[0], noises[0])
    assert m.engine().sync_reruns == 1
    assert torch.equal(y.reshape(-1), ref[0].reshape(-1))


@pytest.mark.parametrize("hook", ["sync_abort", "sync_timeout"])
def test_sync_failure_poisons_output_and_sticky_status(hook, built_lib, cuda_device):
    """Both failure exits of the synchronised launch: the residency abort and a
    grid-barrier wait that gives up (PWG_OPT_SYNC_TIMEOUT: every wait gives up at once, so the
    workgroups run ahead on partial planes). Either way
    - the last layer writes NaN audio, never a plausible wrong waveform;
    - pwg_run_status returns PWG_ERR_RERUN, and it does so even when later runs completed, because
      the handle's sticky status word keeps the bit until a status call reads it (a serving loop
      that checks once per batch of runs);
    - Engine.run(check=True) redoes the run on the per-layer launches: bit-identical output, one
      rerun counted."""
    from parallelwavegan_amd import _lib, configs

    params = configs.generator_params("ljspeech_v1")
    per_layer, sync = _engines(params, cuda_device, seed=10)
    mels, noises = _inputs([64, 3], 256, cuda_device, seed=15)
    ref = torch.cat([y.reshape(-1) for y in per_layer.infer(mels, noises)])
    plan = sync.plan([64, 3])
    mel = torch.cat([m.reshape(-1) for m in mels])
    noise = torch.cat([n.reshape(-1) for n in noises])

    sync.set_option(hook, 1)
    out = torch.zeros(plan.total_samples, device=cuda_device)
    sync.run(plan, mel, noise, out, check=False)
    torch.cuda.synchronize(cuda_device)
    assert torch.isnan(out).all()
    with pytest.raises(_lib.RerunError):
        sync.run_status(plan)

    # the failed run first, then three good ones, one status call at the end: still reported
    sync.run(plan, mel, noise, out, check=False)
    sync.set_option(hook, 0)
    good = torch.empty_like(out)
    for _ in range(3):
        sync.run(plan, mel, noise, good, check=False)
    with pytest.raises(_lib.RerunError):
        sync.run_status(plan)
    sync.run_status(plan)  # read and cleared: the next call sees only the last (good) run
    assert torch.equal(good, ref)

    sync.set_option(hook, 1)
    n0 = sync.sync_reruns
    sync.run(plan, mel, noise, out)  # check=True: rerun per-layer
    assert sync.sync_reruns == n0 + 1
    assert torch.equal(out, ref)
    sync.set_option(hook, 0)


def test_engine_suspends_sync_after_repeated_failures(built_lib, cuda_device):
    """on a GPU that is persistently shared every synchronised call would pay the
    failed launch, a synchronisation and a full rerun. After Engine.SYNC_FAIL_STREAK reruns in a
    row the engine stops using the synchronised forward, and tries it again after
    SYNC_RETRY_RUNS runs."""
    from parallelwavegan_amd import configs

    params = configs.generator_params("ljspeech_v1")
    per_layer, sync = _engines(params, cuda_device, seed=11)
    sync.SYNC_RETRY_RUNS = 5
    mels, noises = _inputs([64], 256, cuda_device, seed=16)
    ref = per_layer.infer(mels, noises)[0].clone()
    limit = sync.get_option("sync")
    sync.set_option("sync_abort", 1)
    for i in range(sync.SYNC_FAIL_STREAK):
        assert torch.equal(sync.infer(mels, noises)[0], ref)
    assert sync.sync_reruns == sync.SYNC_FAIL_STREAK
    assert sync.get_option("sync") == 0  # suspended
    for _ in range(4):
        assert torch.equal(sync.infer(mels, noises)[0], ref)
    assert sync.sync_reruns == sync.SYNC_FAIL_STREAK  # per-layer runs: no more reruns
    sync.set_option("sync_abort", 0)
    assert torch.equal(sync.infer(mels, noises)[0], ref)  # the 5th run: sync restored, and it works
    assert sync.get_option("sync") == limit
    assert sync.sync_reruns == sync.SYNC_FAIL_STREAK
