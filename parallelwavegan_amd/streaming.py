"""Chunked and streaming ParallelWaveGAN inference on the HIP engine (SURVEY.md sec 8(e) "single
very long utterance" and sec 8(f) row 3 "causal / streaming PWG").

A generator output sample depends on a bounded window of inputs:
  * the WaveNet stack: +-(receptive_field-1)/2 samples (non-causal) or receptive_field-1 samples
    to the left (causal) (models/parallel_wavegan.py:197-211);
  * the upsampler: conv_in's aux_context_window frames and the FIR chain's few frames
    (layers/upsample.py:112-194).
So an utterance can be cut into chunks that carry ``halo`` extra frames of context: the engine
treats every chunk as its own utterance (edge padding at the chunk ends), and every output sample
farther than the halo from a chunk end is computed by exactly the same arithmetic as in one
whole-utterance run. Outputs are BIT-IDENTICAL to the unchunked inference (tests/test_streaming.py).

  * ``infer_chunked``: one long utterance as a ragged batch of overlapping chunks in ONE engine
    pass (also the unit of multi-GPU splitting of a single long utterance);
  * ``CausalStream``: for ``use_causal_conv=True`` generators, push mel frames as they arrive and
    get the audio of exactly those frames back (left halo only: no look-ahead latency).
"""

import math

import torch


def upsample_reach_frames(scales, causal, bilinear=False):
    """Input frames the FIR chain reaches from one output sample (layers/upsample.py:97-103,
    112-128): stage i filters at rate prod(s_1..s_i) with s_i taps per side (2 s_i to the left,
    causal), i.e. 1 / prod(s_1..s_{i-1}) frames (2x causal). Summed over stages: <= 2 (<= 4).
    A bilinear stretch (Stretch2d interpolate_mode, :43-45) reaches one more input sample of its
    stage on each side."""
    reach, prev = 0.0, 1
    for s in scales:
        reach += (2.0 if causal else 1.0) / prev + (1.0 / prev if bilinear else 0.0)
        prev *= int(s)
    return reach


def _bilinear(engine):
    return int(getattr(engine.config, "interpolate_mode", 0)) == 1


def halo_frames(engine, causal=None):
    """Context frames a chunk needs on each side (left only for causal generators): the WaveNet
    stack's reach in samples (models/parallel_wavegan.py:197-211) over the hop, plus the FIR
    chain's reach (upsample_reach_frames), plus conv_in's aux_context_window, plus one frame for
    the sample's position inside its frame."""
    cfg = engine.config
    causal = bool(cfg.use_causal_conv) if causal is None else causal
    rf = int(engine.receptive_field_size)
    reach = rf - 1 if causal else (rf - 1) // 2
    H = int(engine.upsample_factor)
    scales = [int(cfg.upsample_scales[i]) for i in range(int(cfg.num_scales))]
    up = upsample_reach_frames(scales, causal, _bilinear(engine))
    return int(math.ceil(reach / H + up)) + int(cfg.aux_context_window) + 1


def align_frames(hop, block=32):
    """Chunk starts must be multiples of this many frames for bit-identity. Every layer kernel
    works in 32-sample blocks counted from the utterance start and places a block's aux frames
    (frame = t // hop) in MFMA K slots relative to the block's first frame; a chunk that starts
    off that phase sums the same products in another order (hop 300: every 8 frames)."""
    return block // math.gcd(int(hop), block)


def chunk_ranges(frames, chunk_frames, halo, causal=False, align=1):
    """[(lo, s, e, hi)]: chunk core [s, e) computed from frames [lo, hi); lo is rounded down to a
    multiple of ``align`` (at least ``halo`` frames of left context)."""
    out = []
    for s in range(0, frames, chunk_frames):
        e = min(frames, s + chunk_frames)
        lo = max(0, (s - halo) // align * align)
        hi = e if causal else min(frames, e + halo)
        out.append((lo, s, e, hi))
    return out


def infer_chunked(engine, mel, noise, chunk_frames, halo=None, mean=None, scale=None):
    """One utterance (mel (T', A), noise (T,) or (T, 1), device tensors) -> (T, out_channels),
    computed as overlapping chunks in one ragged engine pass."""
    # a bilinear stretch looks ahead even in a causal generator: right halos then too
    causal = bool(engine.config.use_causal_conv) and not _bilinear(engine)
    halo = halo_frames(engine) if halo is None else int(halo)
    H = int(engine.upsample_factor)
    F = int(mel.shape[0])
    noise = noise.reshape(-1)
    if noise.numel() != F * H:
        raise ValueError("noise must have frames * upsample_factor samples")
    rng = chunk_ranges(F, int(chunk_frames), halo, causal, align_frames(H))
    mels = [mel[lo:hi] for lo, _, _, hi in rng]
    noises = [noise[lo * H:hi * H] for lo, _, _, hi in rng]
    outs = engine.infer(mels, noises, mean, scale)
    parts = [y[(s - lo) * H:(e - lo) * H] for (lo, s, e, _), y in zip(rng, outs)]
    return torch.cat(parts, 0)


class CausalStream:
    """Streaming decode for causal generators: ``push(mel_frames, noise)`` returns the audio of
    exactly the pushed frames, bit-identical to the same frames of one whole-utterance run.
    Keeps ``halo`` frames of mel and noise history; each push runs one engine pass over
    halo + new frames (overlap-save)."""

    def __init__(self, engine, halo=None, mean=None, scale=None):
        if not engine.config.use_causal_conv:
            raise ValueError("CausalStream needs a use_causal_conv=True generator")
        if _bilinear(engine):
            raise ValueError("CausalStream: a bilinear upsampler stretch looks ahead (use infer_chunked)")
        self.engine = engine
        self.halo = halo_frames(engine) if halo is None else int(halo)
        self.H = int(engine.upsample_factor)
        self.align = align_frames(self.H)
        self.mean, self.scale = mean, scale
        self._mel = None
        self._noise = None
        self.frames_out = 0

    def push(self, mel, noise):
        """mel (n, A) and noise (n*H,) device tensors -> (n*H, out_channels)."""
        n = int(mel.shape[0])
        noise = noise.reshape(-1)
        if n == 0:
            return mel.new_zeros((0, int(self.engine.config.out_channels)))
        if noise.numel() != n * self.H:
            raise ValueError("noise must have n * upsample_factor samples")
        if self._mel is None:
            m, z, ctx = mel, noise, 0
        else:
            m = torch.cat([self._mel, mel], 0)
            z = torch.cat([self._noise, noise], 0)
            ctx = int(self._mel.shape[0])
        y = self.engine.infer([m.contiguous()], [z.contiguous()], self.mean, self.scale)[0]
        # keep >= halo frames so that the next pass starts on an aligned frame (align_frames)
        total = self.frames_out + n
        keep = min(self.halo + (total - self.halo) % self.align, int(m.shape[0])) if total > self.halo \
            else int(m.shape[0])
        self._mel = m[-keep:].clone()
        self._noise = z[-keep * self.H:].clone()
        self.frames_out += n
        return y[ctx * self.H:]
