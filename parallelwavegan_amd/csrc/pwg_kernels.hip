// HIP kernels of the PWG generator forward for gfx950 (MI355X, CDNA4).
//
// Data layout in HBM (see DESIGN.md "Data layout"): every activation is channel-major
// [channels][Tpad] on one padded time axis that concatenates the batch's utterances, each
// utterance segment padded to a multiple of SEG samples. A time tile of TILE samples therefore
// belongs to exactly one utterance (tile_utt[]), and the per-layer zero padding at utterance
// edges (layers/residual_block.py:82-89) is a bounds check on the staged operand.
//
// Kernels (reference op each one replaces):
//   pwg_conv_in_kernel      ReplicationPad1d + (c-mean)/scale + conv_in (Conv1d A->A, k=2w+1, valid)
//                           models/parallel_wavegan.py:259-262, layers/upsample.py:166-168,192
//   pwg_upsample_kernel     per scale: Stretch2d nearest xs + Conv2d (1,2s+1) FIR, all stages fused
//                           through LDS, layers/upsample.py:43-45,97-103,112-128
//   pwg_first_conv_kernel   first_conv 1x1 (1->R), models/parallel_wavegan.py:81,161
//   pwg_layer_kernel        one WaveNetResidualBlock + skip accumulation, fused:
//                           dilated conv (K taps) + aux 1x1 as ONE fp32 MFMA GEMM, gate
//                           tanh*sigmoid in registers, skip|out 1x1 as a second MFMA GEMM whose
//                           B operand is the gate tile straight out of the accumulators,
//                           residual*sqrt(.5) and skip += in the epilogue.
//                           layers/residual_block.py:102-140, models/parallel_wavegan.py:163-165
//   pwg_head_kernel         skips*sqrt(1/L) -> ReLU -> 1x1 -> ReLU -> 1x1,
//                           models/parallel_wavegan.py:131-138,166-171
#include "pwg_internal.h"
#include "../../include/pwg.h"

namespace pwg {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ long long floordiv(long long a, long long b) {
  long long q = a / b;
  if ((a % b != 0) && (a < 0)) --q;  // b > 0 everywhere here
  return q;
}

// Largest u with utts[u].frame_base <= g (utts sorted by frame_base).
__device__ __forceinline__ int find_utt_by_frame(const UttDesc* utts, int n, long long g) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (utts[mid].frame_base <= g) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// ---------------------------------------------------------------------------------------------
// conv_in at frame rate. grid (ceil(F_total/256), A), one output (channel o, frame g) per thread.
// 2w+1 taps x A inputs = 400 MAC per output at A=80, w=2: 125 MAC per audio sample, <0.1 % of
// the forward; the input gather is served by L1/L2.
__global__ void __launch_bounds__(256) pwg_conv_in_kernel(const ConvInArgs a) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  if (g >= a.F_total) return;
  const int o = blockIdx.y;
  const int u = find_utt_by_frame(a.utts, a.n_utts, g);
  const UttDesc ud = a.utts[u];
  const long long f = g - ud.frame_base;
  const long long Tf = ud.frames;
  const long long Tin = Tf + 2 * a.ctx;  // padded input length (forward layout)

  auto cin = [&](int i, long long fp) -> float {
    float v;
    if (a.layout == PWG_LAYOUT_INFERENCE) {
      long long src = fp - a.ctx;
      src = src < 0 ? 0 : (src >= Tf ? Tf - 1 : src);  // ReplicationPad1d
      v = a.mel[ud.mel_off + src * a.A + i];
      if (a.mean != nullptr) v = (v - a.mean[i]) / a.scale[i];
    } else {
      v = a.mel[ud.mel_off + (long long)i * Tin + fp];
    }
    return v;
  };

  float acc = 0.f;
  if (a.use_conv_in) {
    const float* w = a.w + (size_t)o * a.A * a.KW;
    for (int i = 0; i < a.A; ++i)
      for (int k = 0; k < a.KW; ++k) acc = fmaf(w[i * a.KW + k], cin(i, f + k), acc);
  } else {
    acc = cin(o, f);
  }
  a.c1[(size_t)o * a.F_total + g] = acc;
}

// ---------------------------------------------------------------------------------------------
// Upsample network: all nearest-xs + (2s+1)-tap FIR stages of one TILE of output samples,
// UP_CG channels per LDS pass. Stage i output t reads up[t+k-P], up[v] = in[v//s] for
// 0 <= v < s*n_i else 0 (Conv2d zero padding, upsample.py:97-102), and stage outputs outside
// [0, n_{i+1}) are zero for the next stage. Integer t//s replaces torch's float nearest index
// (identical below 2^24 samples).
__global__ void __launch_bounds__(256) pwg_upsample_kernel(const UpsampleArgs a) {
  __shared__ float buf[2][UP_CG * UP_MAXW];
  const long long tile = blockIdx.x;
  const UttDesc ud = a.utts[a.tile_utt[tile]];
  const long long col0 = tile * TILE;
  const long long t0 = col0 - ud.seg_base;
  const int tid = threadIdx.x;

  if (t0 >= ud.T) {  // pure padding tile
    for (int idx = tid; idx < a.A * TILE; idx += 256) {
      const int c = idx / TILE, j = idx % TILE;
      a.cup[(size_t)c * a.Tpad + col0 + j] = 0.f;
    }
    return;
  }
  const long long t1 = (t0 + TILE < ud.T) ? t0 + TILE : ud.T;
  const int L = a.n_scales;
  long long lo[MAX_SCALES + 1], hi[MAX_SCALES + 1], n[MAX_SCALES + 1];
  lo[L] = t0; hi[L] = t1;
  for (int i = L - 1; i >= 0; --i) {
    const int s = a.scales[i];
    const int P = a.causal ? 2 * s : s;
    lo[i] = floordiv(lo[i + 1] - P, s);
    hi[i] = floordiv(hi[i + 1] - 1 + 2 * s - P, s) + 1;
  }
  n[0] = ud.frames;
  for (int i = 0; i < L; ++i) n[i + 1] = n[i] * a.scales[i];

  for (int cg = 0; cg < a.A; cg += UP_CG) {
    // stage-0 input: conv_in output frames [lo0, hi0), zero outside the utterance
    {
      const int W = (int)(hi[0] - lo[0]);
      for (int idx = tid; idx < UP_CG * W; idx += 256) {
        const int c = idx / W, j = idx % W;
        const long long f = lo[0] + j;
        const int ch = cg + c;
        float v = 0.f;
        if (ch < a.A && f >= 0 && f < ud.frames) v = a.c1[(size_t)ch * a.F_total + ud.frame_base + f];
        buf[0][c * UP_MAXW + j] = v;
      }
    }
    __syncthreads();
    int cur = 0;
    const float* taps = a.taps;
    for (int i = 0; i < L; ++i) {
      const int s = a.scales[i];
      const int P = a.causal ? 2 * s : s;
      const int KT = 2 * s + 1;
      const int W = (int)(hi[i + 1] - lo[i + 1]);
      const long long nin_up = n[i] * s;
      for (int idx = tid; idx < UP_CG * W; idx += 256) {
        const int c = idx / W, j = idx % W;
        const long long t = lo[i + 1] + j;
        float v = 0.f;
        if (t >= 0 && t < n[i + 1]) {
          const float* bin = &buf[cur][c * UP_MAXW];
          for (int k = 0; k < KT; ++k) {
            const long long uu = t + k - P;
            if (uu >= 0 && uu < nin_up) v = fmaf(taps[k], bin[floordiv(uu, s) - lo[i]], v);
          }
        }
        buf[cur ^ 1][c * UP_MAXW + j] = v;
      }
      taps += KT;
      cur ^= 1;
      __syncthreads();
    }
    for (int idx = tid; idx < UP_CG * TILE; idx += 256) {
      const int c = idx / TILE, j = idx % TILE;
      const int ch = cg + c;
      if (ch >= a.A) continue;
      const long long t = t0 + j;
      a.cup[(size_t)ch * a.Tpad + col0 + j] = (t < t1) ? buf[cur][c * UP_MAXW + (int)(t - t0)] : 0.f;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// first_conv (1x1, 1 -> R, bias): writes X0 on the padded axis, zero in segment padding.
__global__ void __launch_bounds__(256) pwg_first_conv_kernel(const FirstConvArgs a) {
  const long long tile = blockIdx.x;
  const UttDesc ud = a.utts[a.tile_utt[tile]];
  const long long col0 = tile * TILE;
  const long long t0 = col0 - ud.seg_base;
  for (int idx = threadIdx.x; idx < a.R * TILE; idx += 256) {
    const int c = idx / TILE, j = idx % TILE;
    const long long t = t0 + j;
    float v = 0.f;
    if (t < ud.T) v = fmaf(a.w[c], a.noise[ud.io_off + t], a.b[c]);
    a.x[(size_t)c * a.Tpad + col0 + j] = v;
  }
}

// ---------------------------------------------------------------------------------------------
// One residual layer over one TILE of 128 samples. 256 threads = 4 waves; wave w owns the
// 32-sample column block [32w, 32w+32) and ALL gate rows, so the gate and both GEMMs stay in
// its registers.
//
// GEMM 1 (gate pre-activation, 32*MT rows): Z = Wcat . [x(t-d); x(t); x(t+d); c_up(t)]
//   K = KS*R + A (272 for LJ/LibriTTS v1), v_mfma_f32_32x32x2_f32, A operand = packed weight
//   fragments (64 floats per (k-step, m-tile), lane-linear), B operand = staged activation
//   column. K is streamed through LDS in chunks of KC.
// gate: g = tanh(Za + ba) * sigmoid(Zb + bb); Za rows [0,GHPAD), Zb rows [GHPAD, 2*GHPAD) —
//   the two halves sit in the same lane/register of m-tiles m and m+MT/2 (MT==1: regs r, r+8).
// GEMM 2 ([skip; out] rows, 32*M2T): the gate accumulator register (m, r) IS the B fragment of
//   one k-step (lane l: channel row(m,r,l>>5), column l&31); the host packs W2 in the matching
//   permuted-k order, so no LDS round trip for g.
// C/D map of the 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
template <int MT, int M2T>
__global__ void __launch_bounds__(256) pwg_layer_kernel(const LayerArgs a) {
  constexpr int GHPAD = (MT == 1) ? 16 : 16 * MT;
  constexpr int NQ = GHPAD / 2;                 // k-steps of GEMM 2
  constexpr int NG = (MT == 1) ? 1 : MT / 2;    // gate register tiles
  constexpr int A_CHUNK = (KC / 2) * MT * 64;   // floats of weight fragments per K chunk
  constexpr int B_CHUNK = KC * TILE;
  constexpr int W2_FLOATS = NQ * M2T * 64;
  constexpr int LDS_FLOATS = (A_CHUNK + B_CHUNK) > W2_FLOATS ? (A_CHUNK + B_CHUNK) : W2_FLOATS;
  __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
  float* As = lds;
  float* Bs = lds + A_CHUNK;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const long long tile = blockIdx.x;
  const UttDesc ud = a.utts[a.tile_utt[tile]];
  const long long col0 = tile * TILE;
  const long long t0 = col0 - ud.seg_base;
  const long long Tu = ud.T;
  const long long P = a.Tpad;
  const int KSR = a.KS * a.R;
  const int K1 = KSR + a.A;

  f32x16 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;

  for (int kc = 0; kc < a.K1pad; kc += KC) {
    {
      const float4* src = reinterpret_cast<const float4*>(a.wg + (size_t)(kc / 2) * MT * 64);
      float4* dst = reinterpret_cast<float4*>(As);
      for (int i = tid; i < A_CHUNK / 4; i += 256) dst[i] = src[i];
    }
#pragma unroll
    for (int i = 0; i < B_CHUNK / 256; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / TILE, c = idx % TILE;
      const int k = kc + row;
      float v = 0.f;
      if (k < KSR) {
        const int tap = k / a.R;
        const int ch = k - tap * a.R;
        const long long src = t0 + c + (long long)(tap - a.tap_center) * a.dil;
        if (src >= 0 && src < Tu) v = a.x_in[(size_t)ch * P + ud.seg_base + src];
      } else if (k < K1) {
        v = a.cup[(size_t)(k - KSR) * P + col0 + c];
      }
      Bs[row * TILE + c] = v;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < KC / 2; ++s) {
      const float b = Bs[(2 * s + hh) * TILE + wave * 32 + cl];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const float av = As[(s * MT + m) * 64 + lane];
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b, acc[m], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // gate: tanh(Za) * sigmoid(Zb)  (residual_block.py:123-132)
  float g[NG][16];
#pragma unroll
  for (int gm = 0; gm < NG; ++gm) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (MT == 1 && r >= 8) { g[gm][r] = 0.f; continue; }
      const int row = 32 * gm + (r & 3) + 8 * (r >> 2) + 4 * hh;
      const float za = acc[gm][r] + a.bg[row];
      const float zb = (MT == 1 ? acc[0][r + 8] : acc[gm + MT / 2][r]) + a.bg[row + GHPAD];
      g[gm][r] = tanhf(za) * (1.0f / (1.0f + expf(-zb)));
    }
  }

  // stage W2 fragments
  {
    const float4* src = reinterpret_cast<const float4*>(a.w2);
    float4* dst = reinterpret_cast<float4*>(lds);
    for (int i = tid; i < W2_FLOATS / 4; i += 256) dst[i] = src[i];
  }
  __syncthreads();

  f32x16 acc2[M2T];
#pragma unroll
  for (int m = 0; m < M2T; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc2[m][r] = 0.f;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const float bq = g[q >> 4][q & 15];
#pragma unroll
    for (int m2 = 0; m2 < M2T; ++m2) {
      const float av = lds[(q * M2T + m2) * 64 + lane];
      acc2[m2] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bq, acc2[m2], 0, 0, 0);
    }
  }

  // epilogue: skip += W_s g + b_s ; x = (W_o g + b_o + x) * sqrt(0.5)   (residual_block.py:135-138)
  const size_t gt = (size_t)(col0 + wave * 32 + cl);
#pragma unroll
  for (int m2 = 0; m2 < M2T; ++m2) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * m2 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      const float v = acc2[m2][r] + a.b2[row];
      if (row < a.S) {
        float* p = a.skip + (size_t)row * P + gt;
        *p = a.first ? v : (*p + v);
      } else if (row < a.S + a.R) {
        const size_t off = (size_t)(row - a.S) * P + gt;
        a.x_out[off] = (v + a.x_in[off]) * 0.70710677f;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Output head, one sample per thread.
template <int SMAX>
__global__ void __launch_bounds__(TILE) pwg_head_kernel(const HeadArgs a) {
  const long long tile = blockIdx.x;
  const UttDesc ud = a.utts[a.tile_utt[tile]];
  const long long col0 = tile * TILE;
  const long long t = col0 - ud.seg_base + threadIdx.x;
  if (t >= ud.T) return;
  const size_t gt = (size_t)(col0 + threadIdx.x);
  float hv[SMAX];
#pragma unroll
  for (int i = 0; i < SMAX; ++i) {
    float v = 0.f;
    if (i < a.S) v = fmaxf(a.skip[(size_t)i * a.Tpad + gt] * a.skip_scale, 0.f);
    hv[i] = v;
  }
  float* out = a.out + ud.io_off * a.O + t * a.out_stride_t;
  for (int oc = 0; oc < a.O; ++oc) {
    float y = a.b2[oc];
    for (int o = 0; o < a.S; ++o) {
      float z = a.b1[o];
      const float* w1 = a.w1 + (size_t)o * a.S;
#pragma unroll
      for (int i = 0; i < SMAX; ++i)
        if (i < a.S) z = fmaf(w1[i], hv[i], z);
      y = fmaf(a.w2[(size_t)oc * a.S + o], fmaxf(z, 0.f), y);
    }
    out[oc * a.out_stride_o] = y;
  }
}

// ---------------------------------------------------------------------------------------------
hipError_t launch_conv_in(const ConvInArgs& a, hipStream_t s) {
  dim3 grid((unsigned)((a.F_total + 255) / 256), (unsigned)a.A);
  hipLaunchKernelGGL(pwg_conv_in_kernel, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_upsample(const UpsampleArgs& a, long long n_tiles, hipStream_t s) {
  hipLaunchKernelGGL(pwg_upsample_kernel, dim3((unsigned)n_tiles), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_first_conv(const FirstConvArgs& a, long long n_tiles, hipStream_t s) {
  hipLaunchKernelGGL(pwg_first_conv_kernel, dim3((unsigned)n_tiles), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_layer(const LayerArgs& a, int mt, int m2t, long long n_tiles, hipStream_t s) {
  const dim3 grid((unsigned)n_tiles), block(256);
#define PWG_LAYER_CASE(MT_, M2T_)                                                   \
  if (mt == MT_ && m2t == M2T_) {                                                   \
    hipLaunchKernelGGL((pwg_layer_kernel<MT_, M2T_>), grid, block, 0, s, a);        \
    return hipGetLastError();                                                       \
  }
  PWG_LAYER_CASE(1, 1) PWG_LAYER_CASE(1, 2) PWG_LAYER_CASE(1, 4)
  PWG_LAYER_CASE(2, 1) PWG_LAYER_CASE(2, 2) PWG_LAYER_CASE(2, 4)
  PWG_LAYER_CASE(4, 1) PWG_LAYER_CASE(4, 2) PWG_LAYER_CASE(4, 4)
#undef PWG_LAYER_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_head(const HeadArgs& a, long long n_tiles, hipStream_t s) {
  const dim3 grid((unsigned)n_tiles), block(TILE);
  if (a.S <= 16) hipLaunchKernelGGL(pwg_head_kernel<16>, grid, block, 0, s, a);
  else if (a.S <= 32) hipLaunchKernelGGL(pwg_head_kernel<32>, grid, block, 0, s, a);
  else if (a.S <= 64) hipLaunchKernelGGL(pwg_head_kernel<64>, grid, block, 0, s, a);
  else if (a.S <= 128) hipLaunchKernelGGL(pwg_head_kernel<128>, grid, block, 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace pwg
