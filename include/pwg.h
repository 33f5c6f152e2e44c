/*
 * pwg.h — C-ABI of the MI355X-native Parallel WaveGAN generator inference engine.
 *
 * The reference has no FFI for this path: its "operator API" is the Python class
 * parallel_wavegan.models.ParallelWaveGANGenerator looked up by string
 * (/root/reference/parallel_wavegan/utils/utils.py:317-327). Each entry point
 * below replaces one piece of that class; the Python drop-in
 * (parallelwavegan_amd/models.py) binds them through ctypes
 * (parallelwavegan_amd/_lib.py). Signatures carry only plain pointers, sizes and
 * an opaque stream; no torch types cross this boundary.
 *
 *   pwg_create / PwgConfig      <- ParallelWaveGANGenerator.__init__
 *                                  models/parallel_wavegan.py:24-142 (constructor args)
 *   pwg_ref_weight_count        <- the generator state_dict after remove_weight_norm
 *   pwg_pack_weights            <- remove_weight_norm + parameters, models/parallel_wavegan.py:175-185
 *                                  (the caller folds g*v/||v||; this packs for the kernels)
 *   pwg_plan_create             <- per-call shape logic of inference()/forward()
 *                                  models/parallel_wavegan.py:231-263 and :144-173
 *   pwg_run                     <- ParallelWaveGANGenerator.forward (upsample_net -> first_conv ->
 *                                  30 residual blocks -> skip sum -> last_conv_layers)
 *                                  models/parallel_wavegan.py:144-173,
 *                                  layers/upsample.py:112-128,178-194, layers/residual_block.py:102-140
 *   pwg_receptive_field_size    <- ParallelWaveGANGenerator.receptive_field_size :197-211
 *
 * Error behaviour mirrors the reference: a Python `assert` there maps to
 * PWG_ERR_ASSERT (AssertionError), argument errors to PWG_ERR_INVALID
 * (ValueError), unsupported constructor options to PWG_ERR_UNSUPPORTED
 * (NotImplementedError), HIP failures to PWG_ERR_HIP (RuntimeError).
 * pwg_last_error() returns a thread-local message for the last failure.
 *
 * Threading: a handle/plan is not thread-safe; work is enqueued on the caller's
 * HIP stream (hipStream_t passed as void*); only pwg_run_status and
 * pwg_timing_collect synchronise the host. Plans are host-only objects (no device
 * allocation): pwg_run rebuilds the plan's block descriptors inside the caller's
 * workspace with one small kernel per 48 utterances, so a new utterance length costs
 * no hipMalloc / blocking copy and a run is capturable in a HIP graph.
 */
#ifndef PWG_H_
#define PWG_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PWG_ABI_VERSION 2  /* 2: PwgConfig.interpolate_mode */
#if defined(__GNUC__) || defined(__clang__)
#define PWG_API __attribute__((visibility("default")))
#else
#define PWG_API
#endif
#define PWG_MAX_SCALES 8

enum {
  PWG_OK = 0,
  PWG_ERR_INVALID = 1,     /* ValueError */
  PWG_ERR_ASSERT = 2,      /* AssertionError */
  PWG_ERR_HIP = 3,         /* RuntimeError (HIP runtime failure) */
  PWG_ERR_UNSUPPORTED = 4, /* NotImplementedError */
  PWG_ERR_RANGE = 5,       /* a value left the fp16 pair range of the split-f16 kernels (no reference
                              counterpart: the reference computes in fp32; the drop-in reruns on the
                              exact-fp32 kernel, see pwg_run_status) */
  PWG_ERR_RERUN = 6        /* pwg_run_status: a grid-synchronised (PWG_OPT_SYNC) or layer-pipelined
                              forward did not complete (the GPU was shared, or a bounded wait gave
                              up); its output is invalid (NaN); rerun with PWG_OPT_SYNC 0 and
                              PWG_OPT_PIPELINE 0 (the Python engine does) */
};

/* Input layouts accepted by pwg_plan_create / pwg_run. */
enum {
  /* inference(): per utterance c (T'_u, aux) frames-major, utterances concatenated
   * along frames; optional (c-mean)/scale; ReplicationPad1d(aux_context_window)
   * applied inside the engine (models/parallel_wavegan.py:254-262).
   * noise x: per utterance (T_u, 1) concatenated -> (sum T_u).
   * out: per utterance (T_u, out_channels) concatenated. */
  PWG_LAYOUT_INFERENCE = 0,
  /* forward(z, c): c (B, aux, T' + 2w) channel-major, already context-padded by the
   * caller (models/parallel_wavegan.py:144-158); z (B, 1, T); out (B, out_channels, T).
   * All B items share T' (the reference's batched API is equal-length). */
  PWG_LAYOUT_FORWARD = 1
};

/* Timing buckets reported by pwg_timing_collect. */
enum {
  PWG_KERNEL_CONV_IN = 0,
  PWG_KERNEL_UPSAMPLE = 1,        /* frame-rate aux projection (the upsampler is folded into the layers) */
  PWG_KERNEL_FIRST_CONV = 2,
  PWG_KERNEL_RESIDUAL_LAYER = 3,
  PWG_KERNEL_HEAD = 4,            /* fused into the last residual layer: always 0 launches */
  PWG_NUM_KERNELS = 5
};

/* Mirrors ParallelWaveGANGenerator.__init__ arguments
 * (models/parallel_wavegan.py:24-43). dropout is inference-irrelevant;
 * bias=False is expressed by zero biases in the reference-order weights. */
typedef struct PwgConfig {
  int in_channels;          /* must be 1 */
  int out_channels;
  int kernel_size;          /* odd (non-causal) */
  int layers;
  int stacks;               /* layers % stacks == 0 (AssertionError otherwise) */
  int residual_channels;
  int gate_channels;        /* even */
  int skip_channels;
  int aux_channels;
  int aux_context_window;
  int use_causal_conv;
  int use_conv_in;          /* 1: "ConvInUpsampleNetwork", 0: "UpsampleNetwork" */
  int num_scales;
  int upsample_scales[PWG_MAX_SCALES];
  int interpolate_mode;     /* Stretch2d mode (layers/upsample.py:43-45, 62-128): 0 "nearest" (also
                               "nearest-exact" / "area", the same map at integer scales), 1
                               "bilinear" (linear along time, align_corners=False) */
} PwgConfig;

typedef struct PwgHandle PwgHandle;
typedef struct PwgPlan PwgPlan;

PWG_API int pwg_abi_version(void);
PWG_API const char* pwg_last_error(void);

PWG_API int pwg_create(const PwgConfig* cfg, int device, PwgHandle** out);
PWG_API void pwg_destroy(PwgHandle* h);

/* receptive field (kernel_size-1)*sum(dilations)+1, models/parallel_wavegan.py:197-211 */
PWG_API long long pwg_receptive_field_size(const PwgHandle* h);
PWG_API long long pwg_upsample_factor(const PwgHandle* h);

/* Number of floats in the reference-order flat weight vector (after weight-norm
 * folding), in this order:
 *   first_conv.weight (R,in,1), first_conv.bias (R)
 *   upsample_net.conv_in.weight (A,A,KW)            [only when use_conv_in]
 *   upsample_net.upsample.up_layers.{1,3,..}.weight (2s+1) per scale
 *   per layer l: conv.weight (G,R,K), conv.bias (G), conv1x1_aux.weight (G,A),
 *                conv1x1_skip.weight (S,G/2), conv1x1_skip.bias (S),
 *                conv1x1_out.weight (R,G/2), conv1x1_out.bias (R)
 *   last_conv_layers.1.weight (S,S), .bias (S), last_conv_layers.3.weight (O,S), .bias (O)
 * Missing biases (bias=False) are passed as zeros. */
PWG_API long long pwg_ref_weight_count(const PwgHandle* h);
/* Number of floats of the kernel-ready packed weight image (fp32). */
PWG_API long long pwg_packed_weight_count(const PwgHandle* h);
/* Host -> host: pack reference-order weights into the kernel image. The caller
 * uploads the image to device memory (and may RCCL-broadcast it, pwg_broadcast_weights).
 * Returns PWG_ERR_RANGE (image still fully written) when a weight of the split-f16
 * images exceeds the fp16 range: the image is then valid for the exact-fp32 layer
 * kernels (PWG_OPT_LAYER_KERNEL 0/1) only. */
PWG_API int pwg_pack_weights(const PwgHandle* h, const float* ref_host, float* packed_host);

/* Plan a batch of n_utts utterances with frames[u] mel frames each. */
PWG_API int pwg_plan_create(PwgHandle* h, int n_utts, const long long* frames, int layout, PwgPlan** out);
PWG_API void pwg_plan_destroy(PwgPlan* p);
PWG_API long long pwg_plan_total_samples(const PwgPlan* p);   /* sum_u frames[u]*upsample_factor */
PWG_API long long pwg_plan_padded_samples(const PwgPlan* p);  /* HBM time axis incl. segment padding */
PWG_API long long pwg_plan_workspace_bytes(const PwgPlan* p);

/* Enqueue one generator forward over the planned batch on `stream`.
 *   packed   device, pwg_packed_weight_count floats
 *   mel      device, layout-dependent (see PWG_LAYOUT_*)
 *   noise    device, sum_u T_u floats
 *   mean/scale device (aux floats) or NULL: (c-mean)/scale before padding
 *              (models/parallel_wavegan.py:259-260); PWG_LAYOUT_INFERENCE only
 *   out      device, sum_u T_u * out_channels floats
 *   workspace device, pwg_plan_workspace_bytes bytes, 256-B aligned */
PWG_API int pwg_run(PwgPlan* p, const float* packed, const float* mel, const float* noise,
            const float* mean, const float* scale, float* out, void* workspace, void* stream);

/* Status of the last pwg_run on `workspace`, and of every run of this handle since the previous
 * pwg_run_status call on it (a sticky per-handle word that this call reads and clears):
 * synchronises `stream`, then returns
 *   PWG_ERR_RERUN  a grid-synchronised forward (PWG_OPT_SYNC) found the GPU shared and computed
 *                  nothing (status bit 4), or one of its grid-barrier waits gave up (bit 8), or a
 *                  layer-pipelined forward's dependency wait gave up (bit 2). The output of such a
 *                  run is not valid (after a bit-4 or bit-8 run the last layer writes NaN audio);
 *                  rerun it with PWG_OPT_SYNC 0 (and PWG_OPT_PIPELINE 0), which rebuilds every
 *                  intermediate from the mel and the noise. The Python drop-in does this itself.
 *   PWG_ERR_RANGE  (split-f16 layer kernels, which carry fp32 operands as fp16 hi+lo pairs; bit 1)
 *                  a live column's final skip sum was not finite, i.e. some x / D / first_conv value
 *                  exceeded the fp16 range (|v| >= 65520), or the input itself was not finite; the
 *                  split16 aux projection also flags a D value beyond the pair range, and the last
 *                  layer a scaled skip sum the head cannot split. Rerun with PWG_OPT_LAYER_KERNEL 0
 *                  (exact fp32), as the drop-in does. The exact-fp32 kernels never set it.
 * While PWG_OPT_SYNC is on (the default for small plans) a caller that enqueues runs without
 * checking each one must still call this before trusting any of their outputs: the sticky word
 * makes one call per batch of runs enough to learn that SOME run needs redoing (it does not say
 * which; redo them all, or check after every run as the drop-in does). The sticky word belongs to
 * the handle, not to a stream or workspace: the once-per-batch guarantee holds for a handle driven
 * from ONE stream. A handle serving several streams must check after every run (each check then
 * reads its own run's word exactly, and may also report -- and clear -- another stream's unchecked
 * failure, which only costs a spurious rerun). */
PWG_API int pwg_run_status(PwgPlan* p, const void* workspace, void* stream);

/* HIP graph of one pwg_run with fixed buffers (no reference counterpart: the replay path for
 * repeated shapes, e.g. fixed-size streaming chunks or a serving loop over one batch shape).
 * pwg_graph_create captures pwg_run(p, packed, mel, noise, mean, scale, out, workspace) on
 * `stream` (a created stream, not the legacy null stream; timing must be off) into an executable
 * graph (after one eager, synchronised pwg_run on the same buffers, so that first-launch work
 * stays outside the capture). pwg_graph_launch replays the whole forward (workspace reset, plan descriptors, conv_in,
 * aux projection, L layer launches) as one submission on any stream; the caller refills mel /
 * noise in place between launches and may call pwg_run_status on the same workspace after it.
 * The graph reads the plan's descriptors and options as they were at capture time. */
typedef struct PwgGraph PwgGraph;
PWG_API int pwg_graph_create(PwgPlan* p, const float* packed, const float* mel, const float* noise,
                             const float* mean, const float* scale, float* out, void* workspace, void* stream,
                             PwgGraph** out_graph);
PWG_API int pwg_graph_launch(PwgGraph* g, void* stream);
PWG_API void pwg_graph_destroy(PwgGraph* g);

/* Engine options (pwg_set_option). Defaults are the tuned values; the others exist for A/B
 * measurement (bench.py --layer-kernel ...). */
enum {
  PWG_OPT_LAYER_KERNEL = 0,   /* 0: persistent fp32 MFMA, weights resident in LDS (default for shapes
                                    the split kernel does not cover); 1: tiled fp32; 2: persistent
                                    split-f16 (fp32 operands as fp16 hi+lo pairs, 3 f16 MFMAs per
                                    product) on v_mfma_f32_32x32x16_f16; 3: the same on
                                    v_mfma_f32_16x16x32_f16 (default for R = S = 64, gate 128,
                                    kernel 3) */
  PWG_OPT_WAVES_PER_WG = 1,   /* persistent kernel: waves per workgroup (1..8, default 8) */
  PWG_OPT_WG_PER_CU = 2,      /* persistent kernel: workgroups per CU in the grid (default 1) */
  PWG_OPT_FUSE_FIRST_CONV = 3, /* split16 layer kernel: first_conv evaluated inside layer 0 from the
                                    noise, x0 never stored (default 1; bit-identical to 0) */
  PWG_OPT_PIPELINE = 4,        /* split16: plans with at most this many padded samples run all
                                    residual layers in ONE layer-pipelined launch (each CU keeps one
                                    layer's weights; blocks flow layer to layer through per-block
                                    progress words), bit-identical to the per-layer launches; the
                                    B = 1 decode path of bin/decode.py. 0 = never. Applies to plans
                                    created afterwards (default PWG_PIPE_MAX_DEFAULT). */
  PWG_OPT_HALF_BLOCKS = 5,     /* split16: launches of at most this many 32-sample blocks (every layer
                                    but the last) take half blocks (16 columns) as work units: twice
                                    the waves, half of a block's dependent MFMA chain per wave; the
                                    B = 1 latency path. Bit-identical. 0 = never; default 4 x the
                                    CU count (one unit per wave at 8 waves per CU: LJ T' = 64
                                    0.42 -> 0.35 ms per forward; slower from ~4 blocks per CU on). */
  PWG_OPT_SYNC = 6,            /* split16: plans of at most this many 32-sample blocks run all residual
                                    layers in ONE launch, one workgroup per CU, a grid barrier in place
                                    of each launch boundary (the next layer's weights stage while the
                                    barrier completes); same work units and kernel body as the
                                    per-layer launches, bit-identical. 0 = never; default 64 x the
                                    CU count (LJ B = 1, T' = 64 / 512 / 2048: 0.35 -> 0.33, 1.49 ->
                                    1.19, 4.04 -> 3.93 ms per forward; slower than the per-layer
                                    launches' work queues at 256 blocks per CU). A launch that
                                    finds the GPU shared writes nothing and pwg_run_status returns
                                    PWG_ERR_RERUN. */
  PWG_OPT_SYNC_ABORT = 7,      /* test hook: 1 makes every grid-synchronised launch take its "GPU shared"
                                    exit (no output, PWG_ERR_RERUN from pwg_run_status), so the
                                    caller's rerun path can be tested; default 0 */
  PWG_OPT_SYNC_TIMEOUT = 8     /* test hook: 1 makes every grid-barrier wait of a grid-synchronised
                                    launch give up at once (its workgroups run ahead on partial
                                    planes, status bit 8, NaN audio, PWG_ERR_RERUN from
                                    pwg_run_status); default 0 */
};
#define PWG_PIPE_MAX_DEFAULT 0LL /* off: measured slower than the per-layer launches */
PWG_API int pwg_set_option(PwgHandle* h, int option, long long value);
/* Current value of an option (the layer kernel the handle picked for its shape, ...). */
PWG_API int pwg_get_option(const PwgHandle* h, int option, long long* value);

/* Per-kernel HIP-event timing of pwg_run (off by default). collect synchronises
 * on the recorded events, adds ms and launch counts per PWG_KERNEL_* bucket into
 * the caller's arrays and clears the records. */
/* Timing: 0 off, 1 HIP events around every launch (per-bucket / per-op sums), 2 one event pair
 * around each whole run on the caller's stream (its device span only; no events between launches,
 * so the run's launches are timed undisturbed). */
/* Per caller stream the handle keeps a pinned host word for pwg_run_status (allocated on the first
 * status read on that stream, released by pwg_destroy). A host that creates and destroys streams per
 * request calls pwg_release_stream(h, stream) before destroying a stream: it waits for the stream and
 * frees that word (a recycled stream handle would otherwise reuse it; a no-op for unknown streams). */
PWG_API int pwg_release_stream(PwgHandle* h, void* stream);
PWG_API int pwg_set_timing(PwgHandle* h, int enable);
PWG_API int pwg_timing_collect(PwgHandle* h, double* ms, long long* launches);
/* Device span of the timed launches recorded since the last pwg_timing_collect: the first launch's
 * start to the last launch's end, milliseconds (idle gaps between launches included, unlike the
 * per-bucket sums). Call before pwg_timing_collect, which releases the records. */
PWG_API int pwg_timing_span(PwgHandle* h, double* span_ms);

/* ---- Multi-GPU: the one collective of the design -----------------
 * Utterances shard across GPUs with no data-path exchange; the only collective is a broadcast of
 * the packed weight image from a root rank over RCCL/xGMI at start-up. librccl is resolved at first
 * use (dlopen of librccl.so.1: inside a torch process that is torch's own RCCL); these return
 * PWG_ERR_UNSUPPORTED when it is absent. comm is an ncclComm_t passed as void*. A host that already
 * owns an RCCL communicator passes it straight to pwg_broadcast_weights; one that does not creates
 * one with the two helpers (rank 0 makes the id and ships its 128 bytes to the other ranks by any
 * out-of-band channel, every rank then calls pwg_rccl_comm_create). Replaces the reference's
 * per-process checkpoint load (bin/decode.py:131-155), which each decode process repeats. */
#define PWG_RCCL_UNIQUE_ID_BYTES 128
PWG_API int pwg_rccl_unique_id(void* id_out /* PWG_RCCL_UNIQUE_ID_BYTES */);
PWG_API int pwg_rccl_comm_create(int nranks, const void* id, int rank, int device, void** comm_out);
PWG_API int pwg_rccl_comm_destroy(void* comm);
/* In-place ncclBroadcast of pwg_packed_weight_count(h) floats at `packed` (device) from `root`,
 * enqueued on `stream`. */
PWG_API int pwg_broadcast_weights(const PwgHandle* h, void* comm, int root, float* packed, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PWG_H_ */
