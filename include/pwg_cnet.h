/*
 * pwg_cnet.h — C-ABI of the MI355X conv-network executor behind the MelGAN-family drop-ins
 * (MelGANGenerator incl. multi-band + PQMF synthesis, HiFiGANGenerator).
 *
 * The reference builds these generators as torch.nn.Sequential / ModuleList stacks of
 * Conv1d, ConvTranspose1d, LeakyReLU, ReflectionPad1d, Tanh and residual sums
 * (parallel_wavegan/models/melgan.py:17-257, layers/residual_stack.py:13-85,
 *  models/hifigan.py:23-265, layers/residual_block.py:143-258, layers/pqmf.py:51-149).
 * Here a generator is a PROGRAM of fused conv ops that the Python drop-in builds from its
 * constructor arguments (parallelwavegan_amd/melgan.py, hifigan.py); this library packs the
 * weights for the MFMA kernels, plans ragged utterance batches and runs the program on the
 * caller's HIP stream. Every op is one launch of a generic fp32 MFMA implicit-GEMM kernel:
 *
 *   y[o, t] = post( ( sum_src sum_{i<C_src, k<K_src} W_src[o, i, k] *
 *                     pre_src( x_src[i, t - pad_src + k * dil_src] ) + b[o] + b2[o]
 *                     + res[o, t] + (accumulate ? y_old[o, t] : 0) ) / out_div )
 *
 * pre = optional (x - mean)/scale (first op) then LeakyReLU(pre_slope) (slope 1 = identity);
 * taps outside an utterance read zeros (PWG_PAD_ZERO, Conv1d padding=), the mirrored sample
 * (PWG_PAD_REFLECT, ReflectionPad1d) or the nearest edge sample (PWG_PAD_REPLICATE,
 * ReplicationPad1d); post = none | LeakyReLU | tanh. A causal conv (layers/causal_conv.py:12-40,
 * CausalConv1d: pad (K-1)*dil on the left, keep the first T outputs) is pad = (K-1)*dil.
 * PWG_CNET_CONVT is ConvTranspose1d(kernel 2*stride): split into `stride` output phases, each a
 * 2-tap conv of the input (models/melgan.py:86-100, models/hifigan.py:96-107). With its source's
 * pad_mode = PWG_PAD_REPLICATE and padding = output_padding = 0 it is CausalConvTranspose1d
 * (layers/causal_conv.py:43-78: ReplicationPad1d((1, 0)), ConvTranspose1d, trim stride on both
 * sides), i.e. y[q*s + r] = W[:, :, r] x[q] + W[:, :, r + s] x[max(q - 1, 0)].
 * PWG_CNET_PQMF is PQMF.synthesis (layers/pqmf.py:133-149) with host-supplied filters.
 *
 * Buffers are time-major [rows][ld] fp32 (ld = channels rounded up to 16); buffer b of a plan
 * holds frames[u] * rate[b] rows per utterance u, utterances back to back. Buffer 0 is the input
 * (mel frames-major, exactly inference()'s c), the op writing the last buffer makes the output.
 *
 * Errors: int status codes as in pwg.h (pwg_last_error() gives the message).
 */
#ifndef PWG_CNET_H_
#define PWG_CNET_H_

#include "pwg.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PWG_CNET_ABI_VERSION 1

enum { PWG_CNET_CONV = 0, PWG_CNET_CONVT = 1, PWG_CNET_PQMF = 2 };
enum { PWG_PAD_ZERO = 0, PWG_PAD_REFLECT = 1, PWG_PAD_REPLICATE = 2 };
enum { PWG_ACT_NONE = 0, PWG_ACT_LRELU = 1, PWG_ACT_TANH = 2 };

typedef struct PwgCnetSrc {
  int buf;          /* buffer id; -1 = source unused */
  int channels;     /* input channels (C_src) */
  int taps;         /* kernel size K_src */
  int dilation;
  int pad;          /* tap k reads row t - pad + k*dilation */
  int pad_mode;     /* PWG_PAD_* */
  int normalize;    /* apply (x - mean) / scale from pwg_cnet_run (inference normalize_before) */
  float pre_slope;  /* LeakyReLU negative slope applied on load; 1.0 = identity */
  long long w_off;  /* floats into the reference-order weights: Conv1d (out, C_src, K_src);
                       CONVT: ConvTranspose1d (C_src, out, 2*stride) */
} PwgCnetSrc;

typedef struct PwgCnetOp {
  int kind;           /* PWG_CNET_* */
  int dst;            /* output buffer id */
  int out_channels;
  PwgCnetSrc src[2];  /* CONVT and PQMF use src[0] only */
  long long b_off;    /* bias (out_channels floats) or -1 */
  long long b2_off;   /* second bias summed with the first (two-source ops) or -1 */
  int res;            /* buffer added after the bias, -1 = none */
  int accumulate;     /* add the destination's previous value */
  float out_div;      /* result divided by this (1.0 = none) */
  int post_act;       /* PWG_ACT_* */
  float post_slope;
  int stride;         /* CONVT: stride (rate[dst] = stride * rate[src]); PQMF: subbands */
  int padding;        /* CONVT: padding; PQMF: filter taps (odd, = taps+1 of PQMF) */
  int output_padding; /* CONVT */
} PwgCnetOp;

typedef struct PwgCnet PwgCnet;
typedef struct PwgCnetPlan PwgCnetPlan;

PWG_API int pwg_cnet_abi_version(void);
/* n_bufs buffers with `channels[b]` channels and `rate[b]` rows per input frame. device -1 creates a
 * host-only handle: packing, and plans that are built and checked (pwg_cnet_plan_rows /
 * _workspace_bytes answer) but never uploaded; pwg_cnet_run refuses them. */
PWG_API int pwg_cnet_create(const PwgCnetOp* ops, int n_ops, int n_bufs, const int* channels, const int* rate,
                    long long ref_weight_count, int device, PwgCnet** out);
PWG_API void pwg_cnet_destroy(PwgCnet* n);
PWG_API long long pwg_cnet_packed_weight_count(const PwgCnet* n);
/* Host -> host packing of the reference-order weight vector into the kernel image. */
PWG_API int pwg_cnet_pack_weights(const PwgCnet* n, const float* ref_host, float* packed_host);
/* Plans are host objects: creating one allocates and copies nothing on the GPU (the handle's
 * per-program chunk tables aside, uploaded by its first plan). The plan's block lists live in the
 * caller's workspace and are written by a descriptor kernel at the start of every pwg_cnet_run, so a
 * new utterance length per call (the reference's decode loop, bin/decode.py:236-268) costs host
 * work only, and a captured forward regenerates them on every replay. */
PWG_API int pwg_cnet_plan_create(PwgCnet* n, int n_utts, const long long* frames, PwgCnetPlan** out);
PWG_API void pwg_cnet_plan_destroy(PwgCnetPlan* p);
/* The device-list image pwg_cnet_run writes into the workspace: its byte offset there, its length
 * in ints, and (cap > 0) its first `cap` ints as the host built and checked them. For tests. */
PWG_API int pwg_cnet_plan_image(const PwgCnetPlan* p, long long* offset_bytes, long long* n_ints, int* out,
                                long long cap);
PWG_API long long pwg_cnet_plan_rows(const PwgCnetPlan* p, int buf); /* sum_u frames[u]*rate[buf] */
PWG_API long long pwg_cnet_plan_workspace_bytes(const PwgCnetPlan* p);
/* mel: buffer 0 contents (device, rows x channels[0], frames-major = time-major);
 * out: the last buffer's first channels[last] channels, time-major (device);
 * mean/scale: device or NULL (ops with normalize=1 need them). */
PWG_API int pwg_cnet_run(PwgCnetPlan* p, const float* packed, const float* mel, const float* mean,
                 const float* scale, float* out, void* workspace, void* stream);
/* Split-f16 range status of the last pwg_cnet_run on this workspace (synchronises `stream`):
 * PWG_ERR_RANGE when the program output holds a non-finite value, i.e. some activation left the
 * fp16 pair range upstream (it became (inf, -inf), every later product NaN) or the input was not
 * finite. The caller reruns with PWG_CNET_OPT_SPLIT_F16 = 0 to get the reference's fp32 semantics
 * (parallelwavegan_amd.cnet.CnetEngine.run(check=True) does). Exact-fp32 runs always return PWG_OK.
 * pwg_cnet_pack_weights likewise returns PWG_ERR_RANGE when a weight cannot be carried as an fp16
 * pair; the packed image is still complete for the exact-fp32 mode. */
PWG_API int pwg_cnet_run_status(PwgCnetPlan* p, const void* workspace, void* stream);
/* The launches pwg_cnet_run would make now (host only, no GPU needed; host-only plans too): their
 * count, and for the first `cap` of them the program phase each starts at, the stream it goes to
 * (0 = the caller's, 1-3 = the handle's auxiliary streams, PWG_CNET_OPT_STREAMS) and the enqueue
 * order (order[i] = the launch enqueued i-th). For tests and tools. */
PWG_API int pwg_cnet_plan_schedule(PwgCnetPlan* p, int cap, int* n_launches, int* phase, int* stream, int* order);
/* Options. PWG_CNET_OPT_SPLIT_F16 (default 1): fp32 operands as fp16 hi+lo pairs on the f16
 * MFMA (three products, fp32 accumulate; error class of fp32); 0: fp32 MFMA.
 * PWG_CNET_OPT_FUSE_PAIRS (default 1, split-f16 mode): run "conv A -> t -> conv B" pairs whose
 * intermediate t has no other reader (HiFiGAN ResBlock steps, layers/residual_block.py:231-237)
 * as one kernel with t kept in LDS; bit-identical to the unfused ops. Applies to 32-channel
 * (weights resident in LDS) and 64-channel (weights streamed) zero-padded pairs (HiFiGAN v1's
 * last two stages).
 * The same option fuses MelGAN ResidualStacks (dilated conv + the two-source 1x1, up to 96
 * channels; bit-identical too).
 * PWG_CNET_OPT_PAIR_STEPS (default 16): 128-column tiles per fused-pair workgroup, for plans
 * created afterwards.
 * PWG_CNET_OPT_XTILE (default 1, split-f16 mode): single-source dilated convs (K = 3/5/7/11, 32, 64
 * or >= 128 rows per tile) run channel-block-major with the input tile staged once per 16-channel
 * block (fp32 summation order differs from the tap-major kernel: parity to the oracle, not bit
 * identity). Conv pairs of such convs then run as two of these launches instead of fused (measured
 * faster on HiFiGAN v1); 0 restores the tap-major kernel and the fused pairs.
 * PWG_CNET_OPT_XT_DMA (flags, default 9 = 1 | 8): x-tile kernels that stage their weight
 * fragments by global_load_lds into two LDS buffers, the next tap group's copy running under the
 * current one's MFMAs. 1: the convs where that measured faster (>= 96-row workgroups at k >= 7,
 * k = 3 up to 192 channels); 2: every eligible conv; 4: the fewest tap groups (one workgroup per
 * CU) instead of groups sized for two; these are bit-identical to the register-staged x-tile
 * kernels. 8: the wide (> 64 output channels) ConvTranspose phases on this kernel instead of the
 * tap-major one (channel-block-major summation: parity to the oracle, not bit identity).
 * PWG_CNET_OPT_XCD_ORDER (default 1): launches with several m-groups or ConvTranspose phases per
 * column block deal a block's siblings to one XCD in consecutive rounds, so they share its L2
 * instead of each fetching the block's input rows from HBM (0: grid order; same results).
 * PWG_CNET_OPT_NARROW (default 1, x-tile mode, applies to plans created afterwards): x-tile
 * launches (convs, conv pair / stack halves, ConvTranspose phases) whose 8-wave, 256-column
 * workgroups would number fewer than the device's CUs run narrow workgroups instead: 1-4 waves
 * (32-128 columns) and 1-2 m-tiles each, weights DMA-staged in tap groups, so a short utterance's
 * op spreads over every CU (the B = 1 decode path, bin/decode.py:236-268); a fused pair or stack
 * whose first conv runs narrow runs as its two ops. Bit-identical to the default launches.
 * 0: never; 2: every x-tile launch (tests).
 * PWG_CNET_OPT_NARROW_DMA (default 1, plans created afterwards): narrow launches run the DMA-ring
 * kernel (one m-tile, 1-4 waves per workgroup): every step (a 16-channel block with all its taps,
 * or one chunk of a tap-major op) is staged by global_load_lds a few steps ahead of its MFMAs, the
 * input rows pre-activated LDS -> LDS; also takes the narrow launches of tap-major convs (MelGAN's
 * two-source 1x1s). Bit-identical to 0 (the DMA-staged narrow x-tile kernel and the narrow
 * tap-major kernel, sized as described above), which stays for A/B. Launches whose DMA-ring
 * workgroups would need more than one round over the CUs keep the narrow x-tile kernel (the
 * DMA-ring forms for them measured slower and were removed in round 6).
 * PWG_CNET_OPT_STREAMS (default 1): launches that do not depend on each other (HiFiGAN's parallel
 * residual blocks, models/hifigan.py:159-168) run concurrently on up to 3 auxiliary streams of the
 * handle, forked from and joined back into the caller's stream with events (graph-capturable):
 * 1 for plans with narrow launches (latency-bound small plans), 2 for every plan, 0 never.
 * The accumulated sum's writers stay in program order: bit-identical to one stream.
 * PWG_CNET_OPT_MSTACK (default 1, plans created afterwards, split-f16 x-tile mode with fused ops): a
 * chain of up to 4 ResidualStacks of one MelGAN stage (layers/residual_stack.py:75-85; k = 3 conv +
 * two-source 1x1 each, zero or reflect "same" padding, 32-128 channels) runs as ONE launch: each
 * workgroup takes a block of output columns through every stack with the input tile (+- the summed
 * dilations, recomputed by neighbouring blocks) in LDS and h in registers, instead of two launches per
 * stack. 1: when the chain's first conv runs narrow (small plans, blocks within one round over the
 * CUs, <= 128 channels); 0 never. Bit-identical to the unfused launches. (Large plans run each
 * stack on PWG_CNET_OPT_RSTACK's kernel: the halo recompute costs more than it saves there.)
 * PWG_CNET_OPT_PRESPLIT (default 1, plans created afterwards, split-f16 mode with narrow DMA-ring
 * launches): a buffer that DMA-ring launches read with a LeakyReLU slope gets a pre-split image
 * (its rows pre-activated and split into fp16 hi / lo pairs) written by its last writer's epilogue
 * when that writer is a DMA-ring launch too; the readers then stage those rows as they are instead of
 * converting them in every workgroup and step. Bit-identical (the same conversion, done once).
 * PWG_CNET_OPT_RSTACK (default 1, split-f16 x-tile mode with fused ops): the batched launch of a fused
 * ResidualStack with 32-96 channels (16-channel multiples, no epilogue extras) runs the persistent
 * LDS-ring kernel (weights and input rows streamed by global_load_lds two steps ahead across tiles,
 * h in registers) instead of the x-tile stack kernel; at <= 64 channels its weights stay resident in
 * LDS (only input rows stream). The two-source 1x1 of stacks too wide for it (128-256 channels)
 * runs alone on the same kind of persistent ring kernel (two 16-channel chunks per step where both
 * sources allow it). Bit-identical; 0 for the x-tile stack and the tap-major 1x1, 2 for the
 * streamed-weight form at every width and one chunk per 1x1 step (A/B). */
enum { PWG_CNET_OPT_SPLIT_F16 = 0, PWG_CNET_OPT_FUSE_PAIRS = 1, PWG_CNET_OPT_PAIR_STEPS = 2, PWG_CNET_OPT_XTILE = 3,
       PWG_CNET_OPT_XT_DMA = 4, PWG_CNET_OPT_XCD_ORDER = 5, PWG_CNET_OPT_NARROW = 6, PWG_CNET_OPT_NARROW_DMA = 7,
       PWG_CNET_OPT_STREAMS = 8, PWG_CNET_OPT_MSTACK = 9, PWG_CNET_OPT_PRESPLIT = 10,
       PWG_CNET_OPT_RSTACK = 11 };
PWG_API int pwg_cnet_set_option(PwgCnet* n, int option, long long value);
/* Timing: 0 off, 1 HIP events around every launch (per-bucket / per-op sums), 2 one event pair
 * around each whole run on the caller's stream (its device span only; no events between launches,
 * so the run's launches are timed undisturbed). */
/* Per caller stream the handle keeps a set of 3 auxiliary streams, their cross-stream events and a
 * pinned status word (PWG_CNET_OPT_STREAMS; pwg_cnet_run_status), created on first use and freed by
 * pwg_cnet_destroy. A host that creates and destroys streams per request calls
 * pwg_cnet_release_stream(n, stream) before destroying a stream: it waits for that stream and its
 * auxiliary streams and frees the set (unknown streams and host-only handles: a no-op). */
PWG_API int pwg_cnet_release_stream(PwgCnet* n, void* stream);
PWG_API int pwg_cnet_set_timing(PwgCnet* n, int enable);
/* Adds per-op milliseconds and launch counts (arrays of n_ops) and clears the records. */
PWG_API int pwg_cnet_timing_collect(PwgCnet* n, double* ms, long long* launches);
/* Device span of the timed launches recorded since the last collect: the first launch's start to
 * the last launch's end over every stream (PWG_CNET_OPT_STREAMS), milliseconds. The per-op sums of
 * pwg_cnet_timing_collect add up concurrent launches; this is wall time on the device. Call
 * before pwg_cnet_timing_collect. */
PWG_API int pwg_cnet_timing_span(PwgCnet* n, double* span_ms);

/* Diagnostics of the batched ResidualStack kernel (PWG_CNET_OPT_RSTACK, csrc/pwg_rstack.hip), for
 * tests and tools/diag/rstack_probe.py; not part of the reference's surface.
 * pwg_rstack_debug_launches: launches of that kernel enqueued since the library loaded (tests assert
 * the kernel engaged). pwg_rstack_debug_probe: enable = cs (16-channel blocks) arms a shader-clock
 * timeline of workgroup wg's wave 0 for the following launches of that width, 0 disarms, < 0 leaves
 * it; out != NULL (n >= 4096 words) copies the last timeline. 0 on success. */
PWG_API long long pwg_rstack_debug_launches(void);
PWG_API int pwg_rstack_debug_probe(int enable, int wg, unsigned long long* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* PWG_CNET_H_ */
