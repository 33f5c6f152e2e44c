// Shared between the HIP kernels (pwg_kernels.hip) and the host side (pwg_capi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pwg {

// Time tile of one residual-layer workgroup: 4 waves x 32 samples (one 32x32 MFMA column block each).
constexpr int TILE = 128;
// Utterance segments on the HBM time axis are padded to this multiple so no tile straddles two
// utterances (per-layer zero padding at utterance edges, residual_block.py:82-89, is then a
// per-tile bounds check).
constexpr int SEG = 256;
// K-chunk of the gate GEMM staged per LDS round.
constexpr int KC = 16;
// Upsampler: channels per LDS pass and max staged width per stage.
constexpr int UP_CG = 16;
constexpr int UP_MAXW = 192;
constexpr int MAX_SCALES = 8;

// One utterance of a planned batch. All offsets in elements.
struct UttDesc {
  long long seg_base;    // first sample of the utterance on the padded HBM time axis
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
  float* c1;             // [A][F_total]
  const UttDesc* utts;
  int n_utts;
  long long F_total;
  int A, KW, ctx;        // ctx = aux_context_window
  int layout;            // PWG_LAYOUT_*
  int use_conv_in;       // 0: identity (UpsampleNetwork)
};

struct UpsampleArgs {
  const float* c1;       // [A][F_total]
  float* cup;            // [A][Tpad]
  const float* taps;     // concatenated (2s+1) per stage
  const int* tile_utt;
  const UttDesc* utts;
  long long F_total, Tpad;
  int A;
  int n_scales;
  int scales[MAX_SCALES];
  int causal;
};

struct FirstConvArgs {
  const float* noise;    // compact
  const float* w;        // [R]
  const float* b;        // [R]
  float* x;              // [R][Tpad]
  const int* tile_utt;
  const UttDesc* utts;
  long long Tpad;
  int R;
};

struct LayerArgs {
  const float* x_in;     // [R][Tpad]
  float* x_out;          // [R][Tpad]
  float* skip;           // [S][Tpad]
  const float* cup;      // [A][Tpad]
  const float* wg;       // gate GEMM A-fragments [K1pad/2][MT][64]
  const float* bg;       // [2*GHPAD]
  const float* w2;       // skip|out GEMM A-fragments [GHPAD/2][M2T][64]
  const float* b2;       // [32*M2T]
  const int* tile_utt;
  const UttDesc* utts;
  long long Tpad;
  int R, S, A, KS;
  int K1pad;
  int dil;
  int tap_center;        // (KS-1)/2 non-causal, KS-1 causal
  int first;             // layer 0: skip buffer is written, not accumulated
};

struct HeadArgs {
  const float* skip;     // [S][Tpad]
  const float* w1;       // [S][S]
  const float* b1;       // [S]
  const float* w2;       // [O][S]
  const float* b2;       // [O]
  float* out;
  const int* tile_utt;
  const UttDesc* utts;
  long long Tpad;
  int S, O;
  float skip_scale;      // sqrt(1/L), models/parallel_wavegan.py:166
  // element strides of the caller's output; utterance u starts at io_off*O in both layouts
  // (inference: (T_u, O) time-major -> t*O + o; forward: (B, O, T) -> o*T + t)
  long long out_stride_t, out_stride_o;
};

// Kernel launchers (pwg_kernels.hip).
hipError_t launch_conv_in(const ConvInArgs& a, hipStream_t s);
hipError_t launch_upsample(const UpsampleArgs& a, long long n_tiles, hipStream_t s);
hipError_t launch_first_conv(const FirstConvArgs& a, long long n_tiles, hipStream_t s);
hipError_t launch_layer(const LayerArgs& a, int mt, int m2t, long long n_tiles, hipStream_t s);
hipError_t launch_head(const HeadArgs& a, long long n_tiles, hipStream_t s);

}  // namespace pwg
