// Shared between the HIP kernels (pwg_kernels.hip) and the host side (pwg_capi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pwg {

// Time tile of one residual-layer workgroup: 4 waves x 32 samples (one 32x32 MFMA column block each).
constexpr int TILE = 128;
// HBM time axis of a planned batch: [gap][utt 0, padded to TILE][gap][utt 1 ...][gap]. The gaps
// are >= the largest dilated-conv tap offset and hold zeros in both residual buffers, and the
// padding columns of every utterance are written as zeros, so the per-layer zero padding at
// utterance edges (residual_block.py:82-89) costs no masking: a shifted tap simply reads zeros.
// K-chunk of the gate GEMM staged per LDS round.
constexpr int KC = 16;
constexpr int MAX_SCALES = 8;
// Composite-upsampler taps per output sample, padded (J = J1 + J2 + 1 <= 8).
constexpr int AUX_J4 = 8;
// Max frames of the per-workgroup frame window of the aux term.
constexpr int AUX_MAX_NFWG = 16;

// One utterance of a planned batch. All offsets in elements.
struct UttDesc {
  long long seg_base;    // first sample of the utterance on the padded HBM time axis
  long long first_tile;  // index of its first work tile
  long long T;           // samples = frames * upsample_factor
  long long frame_base;  // first frame in the compact conv_in output C1 [A][F_total]
  long long frames;      // T'
  long long mel_off;     // element offset of this utterance's mel in the caller's buffer
  long long io_off;      // element offset of this utterance's noise / output
};

struct ConvInArgs {
  const float* mel;      // caller layout
  const float* mean;     // nullable
  const float* scale;    // nullable
  const float* w;        // [A][A][KW]
  const float* wfrag;    // MFMA A fragments [ceil(A*KW/2)][ceil(A/32)][64]: row o, k = i*KW + kk
  float* c1;             // [A][F_total]
  const UttDesc* utts;
  int n_utts;
  long long F_total;
  int A, KW, ctx;        // ctx = aux_context_window
  int layout;            // PWG_LAYOUT_*
  int use_conv_in;       // 0: identity (UpsampleNetwork)
};

// Exact composite of the upsampler (Stretch2d + FIR stages, layers/upsample.py:112-128) as a
// per-output-sample tap table over mel frames: c_up[:, t] = sum_j w_t[j] * C1[:, t/H - J1 + j].
// Rows t in [TL, T-TR) of an utterance with F >= Fmin frames use interior[t % H]; the first TL
// rows use left[t], the last TR rows right[T-1-t]; utterances with F < Fmin use small[] (rows of
// F frames start at H*F*(F-1)/2). Built and verified against the staged upsampler in double on
// the host (pwg_capi.hip, build_aux_tables).
struct AuxTab {
  const float* interior;
  const float* left;
  const float* right;
  const float* small;
  int H, J1, TL, TR, Fmin;
};

// D[l][f][row] = sum_i Waux_l[row][i] * C1[i][f]: the aux 1x1 conv of every layer applied at FRAME
// rate (it commutes with the per-channel linear upsampler), rows in packed gate-row order.
struct AuxProjArgs {
  const float* c1;       // [A][F_total]
  const float* waux;     // A-fragments [L][ceil(A/2)][MT][64] (packed gate rows x aux channels)
  float* d;              // [L][F_total][GR]
  long long F_total;
  int A, GR;
  int split;             // 1: store (hi | lo << 16) fp16 pairs for the split-f16 layer kernel,
                         // rows [0, GR/2) scaled by split_scale_a, the rest by split_scale_b;
                         // 2: the same in the split16 row order (row 16m + c at c * 8 + m)
  float split_scale_a, split_scale_b;
  int* range_flag;       // split modes: set to 1 when a scaled D value leaves the fp16 pair range
                         // (|v| >= 65520 or not finite; pwg_run_status)
  int* sticky;           // the handle's sticky status word (every flag bit is also ORed there)
};
// Pre-scaling of the split kernel's gate rows (pwg_split.hip gate()): tanh rows by -2 log2(e),
// sigmoid rows by -log2(e).
constexpr double SPLIT_GATE_SCALE_TANH = -2.8853900817779268;
constexpr double SPLIT_GATE_SCALE_SIGM = -1.4426950408889634;

// Writes X0 and zeroes everything of X0/X1 the layers read but never write (gaps, padding
// channels). Blocks [0, n_work) are work tiles, the rest gap tiles (gap_col0).
struct FirstConvArgs {
  const float* noise;    // compact
  const float* w;        // [R]
  const float* b;        // [R]
  float* x;              // [Tpad][RS] time-major
  float* x1;             // the other residual buffer
  float* x2;             // split16 layer pipeline: the third residual plane (gap tiles zeroed), or null
  const int* tile_utt;
  const UttDesc* utts;
  const long long* gap_col0;
  long long n_work;
  long long Tpad;
  int R, RS;
};

// Residual stream x and skip sum are TIME-major ([Tpad][RS], [Tpad][SS], RS/SS = R/S rounded up
// to 4): the MFMA accumulator holds 4 consecutive channels of one sample per register quad, so
// the epilogue moves them with one 16-byte access, and a dilation shift moves whole rows.
struct LayerArgs {
  const float* x_in;     // [Tpad][RS]
  float* x_out;          // [Tpad][RS]
  float* skip;           // [Tpad][SS]
  const float* d;        // this layer's frame-rate aux projection [F_total][GR]
  AuxTab tab;
  const float* wg;       // gate GEMM A-fragments [K1/2][MT][64], K1 = KS*RS (tiled kernel)
  const float* wgp;      // the same, grouped for the persistent kernel [K1/8][MT][64][4]
  long long n_blocks;    // 32-sample blocks (4 per tile)
  const float* bg;       // [2*GHPAD]  gate bias, added by an MFMA k-step against a ones row
  const float* w2;       // skip|out GEMM A-fragments incl. a bias k-step, [NQ4][M2T][64][4]
  const int* tile_utt;
  const UttDesc* utts;
  long long Tpad;
  int R, RS, S, SS, KS;  // RS = R rounded up to KC: the row stride of x, channels [R, RS) are zero
  int dil;
  int nka;               // aux k-steps per wave (frames of a 32-sample window / 2)
  int nfwg;              // frames staged per workgroup
  int tap_center;        // (KS-1)/2 non-causal, KS-1 causal
  int first;             // layer 0: skip buffer is written, not accumulated
  // last layer only: the output head (models/parallel_wavegan.py:131-138,166-171) is fused into
  // the epilogue: y = W2h . relu(W1h . relu(skip * sqrt(1/L)) + b1h) + b2h
  const float* hw1;      // W1h A-fragments incl. bias k-step, [NQH4][M3T][64][4]
  const float* hw2;      // W2h per lane half, [O][M3T][2][16]
  const float* hb2;      // [O]
  float* out;
  long long out_stride_t, out_stride_o;  // caller output strides (base io_off * O)
  int O;
  float skip_scale;
};

// Descriptor of one 32-sample block for the persistent layer kernel, with its utterance's fields
// folded in so a wave fetches everything about its next block in ONE 32-byte load issued a whole
// block ahead (32-bit: the plan guarantees every column and frame index fits).
struct BlockDesc {
  int col;         // global column (padded time axis) of the block's first sample
  int t0;          // utterance-local index of the block's first sample
  int T;           // the utterance's samples
  int frames;      // its T'
  int frame_base;  // its first frame in C1 / D
  int io_off;      // its first sample in the caller's noise/output arrays
  int utt;
  int pad;
};

// Slim argument block of the persistent layer kernel (fewer live scalars than LayerArgs).
struct PersistArgs {
  const float* x_in;     // [Tpad][RS]
  float* x_out;
  float* skip;           // [Tpad][SS]
  const float* d;        // this layer's aux projection [F_total][GR]
  const float* tab;      // AuxTab base; the four tables at 32-bit offsets below
  const BlockDesc* blocks;
  const float* wgp;      // [K1/4][MT][64][4]
  const float* w2;       // [NQ4][M2T][64][4]
  const float* bg;       // [GR]
  const float* hw1;      // last layer only
  const float* hw2;
  const float* hb2;
  float* out;
  int tab_left, tab_right, tab_small;  // offsets (floats) from tab; interior at 0
  int H, J1, TL, TR, Fmin, nka;
  int n_blocks;
  int R, RS, S, SS, KS, dil, tap_center, first, O;
  int out_stride_t, out_stride_o;
  float skip_scale;
  int* ctr;                   // this layer's 8 per-XCD work-queue heads, SCHED_CTR_STRIDE ints apart (zeroed per run)
};

// Split-f16 layer kernel (pwg_split.hip), PWG v1 shape: R = S = 64, 128 gate rows, kernel 3.
struct SplitArgs {
  const unsigned* x_in;  // [Tpad][64] fp16-pair slots (pwg_split.hip header)
  unsigned* x_out;
  float* skip;           // [Tpad][64] fp32, slot order
  const float* skip0;    // [2][32]: sum over layers of the skip biases (layer 0's seed)
  const unsigned* d;     // this layer's aux projection [F_total][128] pairs
  const float* tab;      // AuxTab base (interior at 0)
  const BlockDesc* blocks;
  const unsigned* wg;    // the layer's LDS image: gate frags | W2 frags | gate bias | sqrt(.5) b_out
  const float* hw1;      // last layer: head (as the fp32 kernel)
  const float* hw2;
  const float* hb2;
  float* out;
  int tab_left, tab_right, tab_small;
  int H, J1, TL, TR, Fmin;
  int n_blocks, dil, first, O;
  int out_stride_t, out_stride_o;
  float skip_scale;
  int* ctr;
  unsigned long long* trace;  // per-wave timestamps when PWG_TRACE_FILE is set (tools/trace_layer.py), else null
  const float* noise;         // split16 layer 0 with first_conv fused (else null): caller noise
  const float* fw;            // first_conv weight [64] and bias [64]
  const float* fb;
  int* range_flag;            // the run's status word (pwg_run_status): the last layer sets
                              // PWG_STATUS_RANGE when a live column's final skip sum is not finite
                              // (fp16 pair range exceeded somewhere upstream); the pipelined and
                              // synchronised forwards set their wait / abort bits; the last layer
                              // writes NaN audio when a PWG_STATUS_REDO bit is set on entry
  int* sticky;                // the handle's sticky status word: every bit set in range_flag is
                              // also ORed here, so a status check once per batch of runs sees it
  int compute_waves;          // split16: waves per workgroup that take blocks (the rest only stage)
};
// dwords of one layer's split image (SplitSmem in pwg_split.hip without the head)
constexpr int SPLIT_LAYER_DWORDS = 3 * 4 * 4 * 2 * 64 * 4 + 4 * 4 * 2 * 64 * 4 + 32 * 4 + 64;

// Layer-pipelined split16 forward (pwg_split16.hip pwg_pipe_split16_kernel): all L layers in one
// launch, each workgroup serving one layer with its weights resident, blocks handed from layer to
// layer through per-block progress words. `base` holds the fields every layer shares (the layer's
// weights, D rows, planes and dilation are derived per workgroup).
constexpr int PIPE_MAX_LAYERS = 64;
struct PipeArgs {
  SplitArgs base;            // noise non-null: layer 0 builds x0 from the noise (fused first_conv)
  const unsigned* wg0;       // layer 0's split16 LDS image; layer l's at wg0 + l * wg_stride (dwords)
  long long wg_stride;
  const unsigned* d0;        // layer 0's D rows; layer l's at d0 + l * d_stride (dwords)
  long long d_stride;
  unsigned* x[3];            // residual planes: layer l reads x[l % 3], writes x[(l + 1) % 3]
  int* prog;                 // [n_blocks] layers finished per block (zeroed per run)
  int* ctr;                  // layer l's block queue head at ctr[l * SCHED_CTR_STRIDE * 8] (zeroed per run)
  int L;
  int dil[PIPE_MAX_LAYERS];
};

// Grid-synchronised forward (pwg_sync_split16_kernel): all layers in one launch, a grid barrier
// between layers; x ping-pongs between two planes (layer l reads x[l & 1]).
struct SyncArgs {
  SplitArgs base;            // noise non-null: layer 0 builds x0 from the noise (fused first_conv)
  const unsigned* wg0;       // layer l's split16 LDS image at wg0 + l * wg_stride (dwords)
  long long wg_stride;
  const unsigned* d0;        // layer l's D rows at d0 + l * d_stride (dwords)
  long long d_stride;
  unsigned* x[2];
  int* ctr;                  // barrier counter, arrival counter, residency decision, each on a
                             // line of its own (SCHED_CTR_STRIDE ints apart; zeroed per run)
  int l0, L;                 // the launch runs layers l0 .. l0 + L - 1
  int half;                  // half-block work units
  int force_abort;           // test hook (PWG_OPT_SYNC_ABORT): take the "GPU shared" exit
  int force_timeout;         // test hook (PWG_OPT_SYNC_TIMEOUT): every grid-barrier wait gives up
  int waves_mid;             // computing waves per workgroup
  int dil[PIPE_MAX_LAYERS];
};

// Persistent-kernel work queues: one head per XCD, each on its own 128-byte line.
constexpr int SCHED_CTR_STRIDE = 32;

// Sets the message pwg_last_error() returns and passes `code` through (pwg_capi.hip).
int set_error(int code, const char* msg);

// hipFuncSetAttribute(kfn, MaxDynamicSharedMemorySize, lds) once per (device, kernel) and size:
// the launchers call it before every launch, so the host path of a run with dozens of launches
// (the vocoders' B = 1 decode) keeps only the first call (pwg_capi.hip, thread-safe).
hipError_t allow_lds(const void* kfn, int lds);

// Kernel launchers (pwg_kernels.hip).
// Plan descriptors built on the device at the start of every pwg_run, in the caller's workspace
// (no per-plan hipMalloc / blocking hipMemcpy / hipFree; graph-capturable): up to PLAN_CHUNK
// utterances per launch, passed by value.
constexpr int PLAN_CHUNK = 48;
constexpr int GAP_TILES_MAX = 1 << 20;
struct PlanDescArgs {
  UttDesc utts[PLAN_CHUNK];
  int n;          // utterances in this chunk
  int u0;         // plan index of utts[0]
  int gap_tiles;  // zero tiles between segments (gap / TILE)
  UttDesc* d_utts;
  int* tile_utt;
  long long* gap_col0;
  BlockDesc* blocks;
  int* zero;      // first chunk only: the run's work-queue heads + range flag, zeroed here
  int n_zero;
  int* prog;      // layer pipeline: per-block progress words, zeroed with the block descriptors (or null)
  unsigned* zx[3];  // split16 with the fused first_conv: residual planes whose gap tiles are zeroed
                    // here (null: not here; x[2] null without the layer pipeline's third plane)
};
hipError_t launch_plan_desc(const PlanDescArgs& a, long long max_blocks, hipStream_t s);

hipError_t launch_conv_in(const ConvInArgs& a, hipStream_t s);
hipError_t launch_aux_proj(const AuxProjArgs& a, int layers, hipStream_t s);
hipError_t launch_first_conv(const FirstConvArgs& a, long long n_tiles, hipStream_t s);
hipError_t launch_layer(const LayerArgs& a, int mt, int m2t, bool last, long long n_tiles, hipStream_t s);
hipError_t launch_first_conv_split(const FirstConvArgs& a, long long n_tiles, hipStream_t s);
hipError_t launch_first_conv_split16(const FirstConvArgs& a, long long n_tiles, hipStream_t s);
hipError_t launch_layer_split16(const SplitArgs& a, bool last, int tap_center, int waves_per_wg, int n_wg,
                                hipStream_t s, bool half = false);
hipError_t launch_layer_split(const SplitArgs& a, bool last, int tap_center, int waves_per_wg, int n_wg,
                              hipStream_t s);
hipError_t launch_pipe_split16(const PipeArgs& p, int tap_center, int n_wg, hipStream_t s);
hipError_t launch_sync_split16(const SyncArgs& p, int tap_center, int n_wg, hipStream_t s);
hipError_t launch_layer_persistent(const PersistArgs& a, int mt, int m2t, bool last, int waves_per_wg, int n_wg,
                                   hipStream_t s);

// Copy n 16-byte vectors global -> LDS with the workgroup's nthr threads: 8 loads in flight per
// thread before their stores (a plain load/store loop waits one L2 round trip per vector, which
// dominated a layer launch on small plans: 16-64 dependent trips per thread).
template <typename V>
__device__ __forceinline__ void stage_lds(V* dst, const V* src, int n, int tid, int nthr) {
  int i = tid;
  for (; i + 7 * nthr < n; i += 8 * nthr) {
    V r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = src[i + j * nthr];
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[i + j * nthr] = r[j];
  }
  for (; i < n; i += nthr) dst[i] = src[i];
}

// Fused residual-stack chain of a MelGAN stage (pwg_mstack.hip, the conv-network executor's B = 1
// path): NS consecutive ResidualStacks (layers/residual_stack.py:75-85) -- per stack a dilated
// k = 3 conv h = W_A * lrelu(x) + b_A and the two-source 1x1 x' = W_1 lrelu(h) + W_s x + b -- for
// one block of output columns in ONE workgroup, the input tile (columns +- the stacks' summed
// dilations, recomputed by neighbouring blocks) kept in LDS between stacks, h in registers.
constexpr int MS_MAX = 4;         // stacks per fused launch
struct MsStack {
  const float* wA;                // conv A split-f16 fragments [tap * cs + cb][MT][hi/lo][lane][4]
  const float* bA;                // conv A bias (C floats)
  const float* wB;                // 1x1 split-f16 fragments [chunk][MT][hi/lo][lane][4], chunks
                                  // [h cb 0 .. cs-1][x cb 0 .. cs-1] (the executor's chunk order)
  const float* bB;                // 1x1 bias (both biases summed)
  int dil, pad, mode;             // conv A: dilation, pad (tap t reads column c - pad + t dil), edge mode
  float slopeA, slopeH;           // LeakyReLU slope of conv A's input and of h
};
struct MstackArgs {
  const float* x;                 // stage input (stack 0's x), [rows][ld]
  const int* seg_x;               // [n_utts][2] (first row, rows)
  float* y;                       // the last stack's output, [rows][ld]
  const int* seg_y;
  int ld;                         // row stride of x and y (floats)
  const int2* blocks;             // (utterance, q0): oc output columns each
  int ns, oc, halo;               // stacks, output columns per block, summed dilations
  MsStack st[MS_MAX];
};
// cs: 16-channel blocks (2, 3, 4, 6, 8); tpw: column tiles per wave (1, 2). LDS bytes of a launch:
int mstack_lds(int cs, int oc, int halo, int ns);
bool mstack_supported(int cs, int tpw);
hipError_t launch_mstack(const MstackArgs& a, int cs, int tpw, int n_blocks, hipStream_t s);

// Batched ResidualStack (pwg_rstack.hip, the conv-network executor's launch for large plans): one
// stack -- h = W_A * lrelu(x) + b_A (k = 3, dilation dil), y = W_1 lrelu(h) + W_s x + b -- for
// 256-column tiles, persistent workgroups streaming every step's weights and input rows through an
// LDS ring, h in registers. C = 16 cs channels (cs = 2, 3, 4, 6), y rows of exactly C floats.
constexpr int RS_MAX_REACH = 64;  // (k - 1) dil = 2 dil at most
constexpr int RS_MAX_TILES = 64;  // 256-column tiles per workgroup at most
struct RstackArgs {
  const float* x;                 // stack input [rows][ld_x]
  const int* seg_x;               // [n_utts][2] (first row, rows)
  int ld_x, mode_x;               // row stride (floats, multiple of 4); conv A's edge mode
  int dil, off;                   // conv A: dilation, first tap offset (-pad)
  float slope1;                   // conv A's input LeakyReLU slope
  int mode_2;                     // the 1x1's x source: edge mode and LeakyReLU slope
  float slope2;
  float slope_h;                  // the 1x1's LeakyReLU slope of h
  const float* wA;                // conv A split-f16 fragments [tap * cs + cb][MT][hi/lo][lane][4]
  const float* bA;                // conv A bias (C)
  const float* wB;                // 1x1 fragments [chunk][MT][hi/lo][lane][4], chunks [h cb][x cb]
  const float* bB;                // 1x1 bias (both biases summed, C)
  float* y;                       // [rows][C] (no residual, accumulate, division or activation)
  const int* seg_y;
  const int2* blocks;             // (utterance, q0) of each 256-column tile
  const int* ncols;               // output columns per utterance
  int n_blocks;
};
// A two-source 1x1 op (MelGAN's stack 1x1 + skip_layer over [lrelu(h); x]) on its own, 32 MT
// output channels, the executor's chunk order [source 0 blocks][source 1 blocks]
// (pwg_r1x1_kernel, pwg_rstack.hip)
struct R1x1Args {
  const float* src[2];            // [rows][ld]
  const int* seg[2];              // [n_utts][2] (first row, rows)
  int ld[2];                      // row strides (floats, multiples of 4)
  float slope[2];                 // each source's LeakyReLU slope (1: none)
  int nch0, nch;                  // 16-channel chunks of source 0, of both
  const float* w;                 // split-f16 fragments [chunk][MT][hi/lo][lane][4]
  const float* bias;              // (32 MT)
  float* y;                       // [rows][32 MT] (no residual, accumulate, division or activation)
  const int* seg_y;
  const int2* blocks;             // (utterance, q0) of each 256-column tile
  const int* ncols;
  int n_blocks;
};
bool r1x1_supported(int mt);
// pairs: two chunks per step where both sources allow it (PWG_CNET_OPT_RSTACK 1), else one
hipError_t launch_r1x1(const R1x1Args& a, int mt, int n_wg, hipStream_t s, bool pairs);
// a wide stack's k = 3 conv alone (pwg_rconv_kernel, 32 mt channels in and out, y = W lrelu(x) + b
// with RstackArgs' conv-A fields; mt as r1x1_supported)
hipError_t launch_rconv(const RstackArgs& a, int mt, int n_wg, hipStream_t s);
bool rstack_supported(int cs);
int rstack_lds(int cs);
// resident: the weight-resident form where the fragments fit the LDS (<= 64 channels), else streamed
hipError_t launch_rstack(const RstackArgs& a, int cs, int n_wg, hipStream_t s, bool resident = true);

// Run status bits (the per-run word pwg_run_status reads, and the handle's sticky copy).
constexpr int PWG_STATUS_RANGE = 1;         // a value left the fp16 pair range: rerun in exact fp32
constexpr int PWG_STATUS_PIPE_TIMEOUT = 2;  // layer pipeline: a dependency wait gave up
constexpr int PWG_STATUS_SYNC_ABORT = 4;    // grid-synchronised forward: not every workgroup started
constexpr int PWG_STATUS_SYNC_TIMEOUT = 8;  // grid-synchronised forward: a grid-barrier wait gave up
constexpr int PWG_STATUS_REDO = PWG_STATUS_PIPE_TIMEOUT | PWG_STATUS_SYNC_ABORT | PWG_STATUS_SYNC_TIMEOUT;

// OR status bits into the run's word and the handle's sticky word (either may be null).
__device__ __forceinline__ void flag_status(int* flag, int* sticky, int bits) {
  if (flag != nullptr) __hip_atomic_fetch_or(flag, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (sticky != nullptr) __hip_atomic_fetch_or(sticky, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Split-f16 range flag: one vector atomic per wave (from its lowest flagging lane) when any active
// lane saw a value the fp16 pair split cannot carry. Lanes that already exited simply do not vote.
__device__ __forceinline__ void flag_range(int* flag, int* sticky, bool bad, int lane) {
  const unsigned long long m = __ballot(bad ? 1 : 0);
  if (bad && lane == __builtin_ctzll(m)) flag_status(flag, sticky, PWG_STATUS_RANGE);
}

}  // namespace pwg
