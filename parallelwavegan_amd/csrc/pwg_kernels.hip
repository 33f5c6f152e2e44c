// HIP kernels of the PWG generator forward for gfx950 (MI355X, CDNA4).
//
// Data layout in HBM (see DESIGN.md "Data layout"): the residual stream and the skip sum are
// time-major [Tpad][channels] on one padded time axis that concatenates the batch's utterances,
// each padded to a multiple of TILE and separated by zero gaps wider than any dilated-conv tap
// offset. A time tile belongs to exactly one utterance (tile_utt[]), and the per-layer zero
// padding at utterance edges (layers/residual_block.py:82-89) is free: shifted taps read zeros.
//
// Kernels (reference op each one replaces):
//   pwg_conv_in_kernel      ReplicationPad1d + (c-mean)/scale + conv_in (Conv1d A->A, k=2w+1, valid)
//                           models/parallel_wavegan.py:259-262, layers/upsample.py:166-168,192
//   pwg_aux_proj_kernel     conv1x1_aux of ALL layers at frame rate: D_l = W_aux_l . C1. The aux 1x1
//                           (residual_block.py:93,126-130) is linear per time step and the upsampler
//                           (layers/upsample.py:43-45,97-103,112-128) is linear per channel, so
//                           W_aux . U(C1) == U(W_aux . C1); the layer kernel applies U as an exact
//                           polyphase tap table over <= 8 frames (AuxTab) inside its MFMA GEMM.
//   pwg_first_conv_kernel   first_conv 1x1 (1->R), models/parallel_wavegan.py:81,161
//   pwg_layer_kernel        one WaveNetResidualBlock + skip accumulation, fused:
//                           dilated conv (K taps) + upsampled aux term as ONE fp32 MFMA GEMM, gate
//                           tanh*sigmoid in registers, skip|out 1x1 as a second MFMA GEMM whose
//                           B operand is the gate tile straight out of the accumulators,
//                           residual*sqrt(.5) and skip += in the epilogue.
//                           layers/residual_block.py:102-140, models/parallel_wavegan.py:163-165
//                           The LAST layer's epilogue also runs the output head, skips*sqrt(1/L) ->
//                           ReLU -> 1x1 -> ReLU -> 1x1 (models/parallel_wavegan.py:131-138,166-171),
//                           as a third MFMA GEMM on the skip tile held in registers.
#include "pwg_internal.h"
#include "../../include/pwg.h"

namespace pwg {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));  // native vector: stays in VGPRs (HIP float4 is a struct)

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
// conv_in at frame rate. grid ceil(F_total/64), 256 threads = 4 waves; lane = frame, wave w =
// output channels [w*OG, (w+1)*OG) (OG = ceil(A/4) <= 32): each thread reads its (2w+1)-frame
// input window once and accumulates OG outputs; the weights are wave-uniform (scalar loads).
// 2w+1 taps x A inputs = 400 MAC per output at A=80, w=2: 125 MAC per audio sample.
template <int OGMAX>
__global__ void __launch_bounds__(256) pwg_conv_in_kernel(const ConvInArgs a) {
  const int lane = threadIdx.x & 63;
  const int grp = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long long g0 = (long long)blockIdx.x * 64 + lane;
  const bool valid = g0 < a.F_total;
  const long long g = valid ? g0 : a.F_total - 1;
  const int u = find_utt_by_frame(a.utts, a.n_utts, g);
  const UttDesc ud = a.utts[u];
  const long long f = g - ud.frame_base;
  const long long Tf = ud.frames;
  const long long Tin = Tf + 2 * a.ctx;  // padded input length (forward layout)
  const int OG = (a.A + 3) / 4;
  const int o0 = grp * OG;

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

  float acc[OGMAX];
#pragma unroll
  for (int j = 0; j < OGMAX; ++j) acc[j] = 0.f;
  if (a.use_conv_in) {
    for (int i = 0; i < a.A; ++i) {
      for (int k = 0; k < a.KW; ++k) {
        const float x = cin(i, f + k);
        const float* w = a.w + ((size_t)o0 * a.A + i) * a.KW + k;  // W[o][i][k], o = o0 + j
#pragma unroll
        for (int j = 0; j < OGMAX; ++j)
          if (j < OG && o0 + j < a.A) acc[j] = fmaf(w[(size_t)j * a.A * a.KW], x, acc[j]);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < OGMAX; ++j)
      if (j < OG && o0 + j < a.A) acc[j] = cin(o0 + j, f);
  }
  if (!valid) return;
#pragma unroll
  for (int j = 0; j < OGMAX; ++j)
    if (j < OG && o0 + j < a.A) a.c1[(size_t)(o0 + j) * a.F_total + g] = acc[j];
}

// ---------------------------------------------------------------------------------------------
// conv_in as an fp32 MFMA GEMM: C1[o][f] = sum_k W[o][k] X[k][f], k = i*KW + kk, X[i*KW+kk][f] =
// the (replication-padded, normalized) input channel i at frame f + kk. M = A rows (MT m-tiles),
// N = 32 frames per wave, K = A*KW in k-steps of 2 (lane half h takes k = 2s + h). The B operand
// is one input value per lane and k-step (L1-resident: the mel tile is 5 frames wide).
// conv_in with K split over the workgroup's CONV_IN_WAVES waves (the B = 1 latency path's first
// kernel): grid (ceil(F_total / 32), MT), wave w sums k-steps [w Q, (w + 1) Q) of m-tile
// blockIdx.y for 32 frames (lane layout above), loads double-buffered in groups of 8, the
// partial tiles summed through LDS in wave order. One wave per (32 frames, all of K, all m-tiles)
// made a 64-frame utterance ONE chain of 200 k-steps x 3 MFMAs behind 25 load waits: 94 us; 4
// waves 23 us; 16 waves (13 k-steps, two load groups each) measured below that.
constexpr int CONV_IN_WAVES = 16;
template <int MT>
__global__ void __launch_bounds__(64 * CONV_IN_WAVES) pwg_conv_in_ksplit_kernel(const ConvInArgs a) {
  constexpr int NW = CONV_IN_WAVES;
  __shared__ float s_red[NW][16][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hh = lane >> 5, cl = lane & 31;
  const int m = blockIdx.y;
  const long long g0 = (long long)blockIdx.x * 32 + cl;
  const bool valid = g0 < a.F_total;
  const long long g = valid ? g0 : a.F_total - 1;
  const int u = find_utt_by_frame(a.utts, a.n_utts, g);
  const UttDesc ud = a.utts[u];
  const long long f = g - ud.frame_base;
  const long long Tf = ud.frames;
  const long long Tin = Tf + 2 * a.ctx;
  const int K = a.A * a.KW;
  const int nks = (K + 1) / 2;
  const int Q = (nks + NW - 1) / NW;
  const int s_begin = wave * Q, s_end = min(nks, s_begin + Q);
  const float* wl = a.wfrag + lane;
  auto load = [&](int s0, float (&x)[8], float (&w)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int s = s0 + j;
      const int k = 2 * s + hh;
      const int i = k / a.KW, kk = k - i * a.KW;
      x[j] = 0.f;
      if (s < s_end && i < a.A) {
        const long long fp = f + kk;
        if (a.layout == PWG_LAYOUT_INFERENCE) {
          long long src = fp - a.ctx;
          src = src < 0 ? 0 : (src >= Tf ? Tf - 1 : src);  // ReplicationPad1d
          x[j] = a.mel[ud.mel_off + src * a.A + i];
          if (a.mean != nullptr) x[j] = (x[j] - a.mean[i]) / a.scale[i];
        } else {
          x[j] = a.mel[ud.mel_off + (long long)i * Tin + fp];
        }
      }
      w[j] = s < s_end ? wl[(s * MT + m) * 64] : 0.f;
    }
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float xa[8], wa[8], xb[8], wb[8];
  load(s_begin, xa, wa);
  for (int s0 = s_begin; s0 < s_end; s0 += 16) {
    load(s0 + 8, xb, wb);  // in flight during group s0's MFMAs
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[j], xa[j], acc, 0, 0, 0);
    load(s0 + 16, xa, wa);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wb[j], xb[j], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) s_red[wave][r][lane] = acc[r];
  __syncthreads();
  for (int v = threadIdx.x; v < 16 * 64; v += 64 * NW) {
    const int r = v >> 6, l = v & 63;
    float sum = s_red[0][r][l];
#pragma unroll
    for (int w = 1; w < NW; ++w) sum += s_red[w][r][l];
    const long long gg = (long long)blockIdx.x * 32 + (l & 31);
    const int o = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    if (gg < a.F_total && o < a.A) a.c1[(size_t)o * a.F_total + gg] = sum;
  }
}

// ---------------------------------------------------------------------------------------------
// D[l][f][row] = sum_i Waux_l[row][i] C1[i][f] as an fp32 MFMA GEMM per layer: M = GR gate rows
// (A fragments host-packed like the layer weights), N = 32 frames per wave (B fragment = C1 row
// segment, 2 x 128-B reads), K = A. The accumulator's register quads are 4 consecutive rows of one
// frame -> 16-byte stores into the frame-major D the layer kernel stages.
// grid (ceil(F_total/128), L), 256 threads: wave w owns frames [128*bx + 32w, +32).
template <int MT>
__global__ void __launch_bounds__(256) pwg_aux_proj_kernel(const AuxProjArgs a) {
  constexpr int GR = 32 * MT;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hh = lane >> 5, cl = lane & 31;
  const int l = blockIdx.y;
  const long long f = (long long)blockIdx.x * 128 + wave * 32 + cl;
  const long long fc = f < a.F_total ? f : a.F_total - 1;
  const int nks = (a.A + 1) / 2;
  const float* w = a.waux + (size_t)l * nks * MT * 64 + lane;
  f32x16 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
  // (issuing all 40 k-steps' loads at once measured slower, 14 -> 25 us at LJ T' = 64: past the
  // wave's 63 outstanding vector loads the waits serialise anyway)
  for (int s0 = 0; s0 < nks; s0 += 8) {  // groups of 8 k-steps, loads first (as conv_in)
    float b[8], wv[8][MT];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int s = s0 + j;
      const int i = 2 * s + hh;
      const float bv = a.c1[(size_t)(i < a.A ? i : 0) * a.F_total + fc];
      b[j] = i < a.A ? bv : 0.f;
#pragma unroll
      for (int m = 0; m < MT; ++m) wv[j][m] = s < nks ? w[(s * MT + m) * 64] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[j][m], b[j], acc[m], 0, 0, 0);
  }
  if constexpr (GR == 128) if (a.split == 2) {
    // split16 layout: row r = 16 m16 + c16 of a frame at dword c16 * 8 + m16, so a layer-kernel
    // lane (c16) reads its 8 m-tiles' rows as two 16-byte loads. Transposed through LDS (row
    // stride 129 dwords: conflict-free column writes), then stored as whole 512-byte frame rows.
    __shared__ unsigned s_d[4][32][129];
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    bool bad = false;  // a value the pair split cannot carry (it would become inf / -inf)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const float sc = 32 * m + 8 * j4 < GR / 2 ? a.split_scale_a : a.split_scale_b;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 32 * m + 8 * j4 + 4 * hh + i;
          const float x = acc[m][4 * j4 + i] * sc;
          bad |= !(__builtin_fabsf(x) < 65520.f);
          const _Float16 hi = (_Float16)x;
          s_d[wave][cl][(r & 15) * 8 + (r >> 4)] = __builtin_bit_cast(unsigned, f16x2{hi, (_Float16)(x - (float)hi)});
        }
      }
    flag_range(a.range_flag, a.sticky, bad && f < a.F_total, lane);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done (wave-private rows)
    __builtin_amdgcn_wave_barrier();
    const long long f0 = (long long)blockIdx.x * 128 + wave * 32;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int k = it * 64 + lane, fr = k >> 5, ch = k & 31;
      if (f0 + fr >= a.F_total) continue;
      const unsigned* src = &s_d[wave][fr][4 * ch];
      *reinterpret_cast<u32x4*>(a.d + ((size_t)l * a.F_total + f0 + fr) * GR + 4 * ch) = u32x4{src[0], src[1], src[2], src[3]};
    }
    return;
  }
  if (f >= a.F_total) return;
  float* d = a.d + ((size_t)l * a.F_total + f) * GR;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[m][4 * j4 + i];
      if (a.split) {
        // fp16 pair (hi | lo << 16) per value for the split-f16 layer kernel
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
        u32x4 u;
        const float sc = 32 * m + 8 * j4 < GR / 2 ? a.split_scale_a : a.split_scale_b;
        bool bad = false;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float x = v[i] * sc;
          bad |= !(__builtin_fabsf(x) < 65520.f);
          const _Float16 hi = (_Float16)x;
          u[i] = __builtin_bit_cast(unsigned, f16x2{hi, (_Float16)(x - (float)hi)});
        }
        if (bad && a.range_flag)  // rare; lanes of exited waves never reach here (f < F_total)
          flag_status(a.range_flag, a.sticky, PWG_STATUS_RANGE);
        *reinterpret_cast<u32x4*>(d + 32 * m + 8 * j4 + 4 * hh) = u;
      } else {
        *reinterpret_cast<f32x4*>(d + 32 * m + 8 * j4 + 4 * hh) = v;
      }
    }
}

// ---------------------------------------------------------------------------------------------
// first_conv (1x1, 1 -> R, bias): writes X0 time-major [Tpad][RS] (zero in utterance padding and
// padding channels), zeroes the padding channels of X1 and, in gap blocks, both buffers.
__global__ void __launch_bounds__(256) pwg_first_conv_kernel(const FirstConvArgs a) {
  const long long tile = blockIdx.x;
  if (tile >= a.n_work) {
    const long long col0 = a.gap_col0[tile - a.n_work];
    for (int idx = threadIdx.x; idx < a.RS * TILE; idx += 256) {
      a.x[(size_t)col0 * a.RS + idx] = 0.f;
      a.x1[(size_t)col0 * a.RS + idx] = 0.f;
    }
    return;
  }
  const UttDesc ud = a.utts[a.tile_utt[tile]];
  const long long col0 = ud.seg_base + (tile - ud.first_tile) * TILE;
  const long long t0 = col0 - ud.seg_base;
  // (4-byte stores, 256 contiguous bytes per wave instruction: a 16-byte-per-lane variant measured
  // slower, 0.87 vs 0.65 ms for the LibriTTS batch)
  for (int idx = threadIdx.x; idx < a.RS * TILE; idx += 256) {
    const int j = idx / a.RS, c = idx - j * a.RS;
    const long long t = t0 + j;
    float v = 0.f;
    if (t < ud.T && c < a.R) v = fmaf(a.w[c], a.noise[ud.io_off + t], a.b[c]);
    a.x[(size_t)(col0 + j) * a.RS + c] = v;
    if (c >= a.R) a.x1[(size_t)(col0 + j) * a.RS + c] = 0.f;
  }
}

// ---------------------------------------------------------------------------------------------
// One residual layer over one TILE of 128 samples. 256 threads = 4 waves; wave w owns the
// 32-sample column block [32w, 32w+32) and ALL gate rows, so the gate and both GEMMs stay in
// its registers.
//
// GEMM 1 (gate pre-activation, GR = 32*MT packed rows):
//   Z = Wdil . [x(t+(0-c)d); x(t+(1-c)d); ...]   K = KS*RS, streamed through LDS in KC=16 chunks,
//       one chunk = 16 channels of ONE tap (uniform time shift), double-buffered: the global
//       loads of chunk i+1 are in flight while chunk i's MFMAs run, one barrier per chunk;
//     + U(D_l)                                   the aux term at sample rate from frame-rate
//       projections: a K = 2*nka GEMM whose A operand is the staged D tile [frame][row] and whose
//       B operand (frame f, sample t) is the composite upsampler tap w_t[f - t/H + J1], from the
//       AuxTab row of the lane's sample;
//     + bias                                     one k-step: A = [bg; 0], B = [1; 0].
//   v_mfma_f32_32x32x2_f32 throughout; A fragments are host-packed lane-linear (64 floats per
//   (k-step, m-tile)); the activation chunk sits time-major in LDS ([t][KC+1], conflict-free
//   B-fragment reads).
// gate: g = tanh(Za) * sigmoid(Zb) on v_exp/v_rcp; Za rows [0,GHPAD), Zb rows [GHPAD, 2*GHPAD)
//   sit in the same lane/register of m-tiles m and m+MT/2 (MT==1: registers r and r+8).
// GEMM 2 ([skip; out] rows, 32*M2T): the gate accumulator register (m, r) IS the B fragment of
//   one k-step (lane l: channel row(m,r,l>>5), column l&31); the host packs W2 in that permuted-k
//   order, 4 k-steps per 16-byte load, plus one bias k-step against a ones row. W2 is read from
//   global memory (L1/L2-resident, 33 KB per layer).
// C/D map of the 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5): registers
//   4j..4j+3 are 4 consecutive channels of one sample -> one 16-byte access in the time-major
//   epilogue.
template <int MT>
struct LayerSmem {
  static constexpr int GR = 32 * MT;
  static constexpr int BSTR = KC + 1;                 // time-major B row stride (floats)
  static constexpr int A_CHUNK = (KC / 2) * MT * 64;  // floats of weight fragments per K chunk
  static constexpr int B_CHUNK = TILE * BSTR;         // floats of activations per K chunk
  static constexpr int BUF = A_CHUNK + B_CHUNK;
  static constexpr int FLOATS = 2 * BUF + (AUX_MAX_NFWG + 2) * GR;
};

// Registers carrying one K chunk from global memory to LDS (named fields, native vectors: an
// array or struct-typed load is spilled to scratch by hipcc).
struct ChunkRegs {
  f32x4 a0, a1, b0, b1;
};

// Chunk c = 16 consecutive K rows of ONE tap: A fragments (contiguous in the packed image) and
// the activation rows x[col0 + off + t][ch0 .. ch0+15], t in [0, 128). Thread -> (t = tid/4 + 64 i,
// channel quad q = tid%4): lanes 4t..4t+3 read one 64-byte row piece. No masks or clamps: the
// zero gaps / padding make every shifted read either valid data or the reference's zero pad.
template <int MT>
__device__ __forceinline__ void layer_load_chunk(const LayerArgs& a, int c, const float* xcol, int tid,
                                                 ChunkRegs& r) {
  constexpr int NA4 = LayerSmem<MT>::A_CHUNK / 4;
  const f32x4* wsrc = reinterpret_cast<const f32x4*>(a.wg + (size_t)c * LayerSmem<MT>::A_CHUNK);
  r.a0 = wsrc[NA4 >= 256 ? tid : (tid < NA4 ? tid : 0)];
  r.a1 = NA4 > 256 ? wsrc[tid + 256] : r.a0;
  const int k0 = c * KC;
  const int tap = k0 / a.RS;                 // uniform
  const int ch0 = k0 - tap * a.RS;
  const long long off = (long long)(tap - a.tap_center) * a.dil;
  const float* p = xcol + (off * a.RS + ch0);
  r.b0 = *reinterpret_cast<const f32x4*>(p);
  r.b1 = *reinterpret_cast<const f32x4*>(p + 64 * a.RS);
}

template <int MT>
__device__ __forceinline__ void layer_store_chunk(float* buf, int tid, const ChunkRegs& r) {
  constexpr int NA4 = LayerSmem<MT>::A_CHUNK / 4;
  constexpr int BSTR = LayerSmem<MT>::BSTR;
  f32x4* as = reinterpret_cast<f32x4*>(buf);
  if (NA4 >= 256 || tid < NA4) as[tid] = r.a0;
  if (NA4 > 256) as[tid + 256] = r.a1;
  float* bs = buf + LayerSmem<MT>::A_CHUNK + (tid >> 2) * BSTR + 4 * (tid & 3);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bs[j] = r.b0[j];
    bs[64 * BSTR + j] = r.b1[j];
  }
}

// tanh(x) = 2 sigmoid(2x) - 1 and sigmoid(x) = 1 / (1 + e^-x) on v_exp_f32 / v_rcp_f32
// (~1e-7 absolute error; the reference uses torch.tanh / torch.sigmoid, residual_block.py:132).
__device__ __forceinline__ float fast_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float fast_tanh(float x) { return 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)) - 1.f; }

// M3T = 0: a middle layer. M3T = ceil(S/32) > 0: the last layer, with the output head fused.
template <int MT, int M2T, int M3T>
__global__ void __launch_bounds__(256, 2) pwg_layer_kernel(const LayerArgs a) {
  constexpr bool LAST = M3T > 0;
  using SM = LayerSmem<MT>;
  constexpr int GHPAD = (MT == 1) ? 16 : 16 * MT;
  constexpr int GR = SM::GR;
  constexpr int BSTR = SM::BSTR;
  constexpr int NQ = GHPAD / 2;                 // k-steps of GEMM 2 (+1 bias step)
  constexpr int NQ4 = (NQ + 1 + 3) / 4;         // 16-byte W2 fragment groups
  constexpr int NG = (MT == 1) ? 1 : MT / 2;    // gate register tiles
  static_assert(SM::A_CHUNK / 4 <= 512, "A chunk staged by at most two float4 per thread");
  __shared__ __attribute__((aligned(16))) float lds[SM::FLOATS];
  float* ds = lds + 2 * SM::BUF;                // aux D tile [nfwg][GR], then bias rows [bg; 0]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const long long tile = blockIdx.x;
  const UttDesc ud = a.utts[a.tile_utt[tile]];
  const long long t0 = (tile - ud.first_tile) * TILE;  // local sample index of the tile start
  const long long col0 = ud.seg_base + t0;
  const long long Tu = ud.T;
  const int NC = a.KS * a.RS / KC;
  const float* xcol = a.x_in + (size_t)(col0 + (tid >> 2)) * a.RS + 4 * (tid & 3);
  const int H = a.tab.H;

  // ---- prologue: chunk 0 in flight, aux D tile + gate bias to LDS
  ChunkRegs cr;
  layer_load_chunk<MT>(a, 0, xcol, tid, cr);
  const long long fwg0 = t0 / H - a.tab.J1;     // first staged frame (utterance-local)
  for (int idx = tid; idx < a.nfwg * GR; idx += 256) {
    const int fi = idx / GR, row = idx - fi * GR;
    const long long f = fwg0 + fi;
    const long long fc = f < 0 ? 0 : (f >= ud.frames ? ud.frames - 1 : f);
    const float v = a.d[(size_t)(ud.frame_base + fc) * GR + row];
    ds[idx] = (f >= 0 && f < ud.frames) ? v : 0.f;
  }
  if (tid < GR) {
    ds[a.nfwg * GR + tid] = a.bg[tid];
    ds[(a.nfwg + 1) * GR + tid] = 0.f;
  }
  layer_store_chunk<MT>(lds, tid, cr);
  __syncthreads();

  f32x16 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;

  // ---- GEMM 1 main loop
  for (int c = 0; c < NC; ++c) {
    if (c + 1 < NC) layer_load_chunk<MT>(a, c + 1, xcol, tid, cr);
    const float* buf = lds + (c & 1) * SM::BUF;
    const float* As = buf;
    const float* Bs = buf + SM::A_CHUNK + (wave * 32 + cl) * BSTR + hh;
#pragma unroll
    for (int s = 0; s < KC / 2; ++s) {
      const float b = Bs[2 * s];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const float av = As[(s * MT + m) * 64 + lane];
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b, acc[m], 0, 0, 0);
      }
    }
    if (c + 1 < NC) layer_store_chunk<MT>(lds + ((c + 1) & 1) * SM::BUF, tid, cr);
    __syncthreads();
  }

  // ---- aux term: + sum_f D[f][row] * w_t[f - t/H + J1]  and the gate bias
  {
    const long long t = t0 + wave * 32 + cl;
    float wt[AUX_J4];
    {
      const long long tc = t < Tu ? t : Tu - 1;  // padding columns: load a valid row, zero it below
      const float* row;
      const long long F = ud.frames;
      if (F < a.tab.Fmin) row = a.tab.small + ((long long)H * F * (F - 1) / 2 + tc) * AUX_J4;
      else if (tc < a.tab.TL) row = a.tab.left + tc * AUX_J4;
      else if (tc >= Tu - a.tab.TR) row = a.tab.right + (Tu - 1 - tc) * AUX_J4;
      else row = a.tab.interior + (tc % H) * AUX_J4;
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(row);
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(row + 4);
      const bool ok = t < Tu;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        wt[j] = ok ? w0[j] : 0.f;
        wt[j + 4] = ok ? w1[j] : 0.f;
      }
    }
    const long long fb = t / H - a.tab.J1;                       // frame of wt[0]
    const long long fw0 = (t0 + wave * 32) / H - a.tab.J1;      // wave window start (uniform)
    const int fo = (int)(fw0 - fwg0);
    for (int s = 0; s < a.nka; ++s) {
      const int j = (int)(fw0 + 2 * s + hh - fb);
      float bw = 0.f;
#pragma unroll
      for (int q = 0; q < AUX_J4; ++q) bw = (j == q) ? wt[q] : bw;
      const float* drow = ds + (fo + 2 * s + hh) * GR + cl;
#pragma unroll
      for (int m = 0; m < MT; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(drow[32 * m], bw, acc[m], 0, 0, 0);
    }
    const float* brow = ds + (a.nfwg + hh) * GR + cl;
    const float one = hh == 0 ? 1.f : 0.f;
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(brow[32 * m], one, acc[m], 0, 0, 0);
  }

  // ---- gate: tanh(Za) * sigmoid(Zb)  (residual_block.py:123-132)
  float g[NG][16];
#pragma unroll
  for (int gm = 0; gm < NG; ++gm) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (MT == 1 && r >= 8) { g[gm][r] = 0.f; continue; }
      const float za = acc[gm][r];
      const float zb = MT == 1 ? acc[0][r + 8] : acc[gm + MT / 2][r];
      g[gm][r] = fast_tanh(za) * fast_sigmoid(zb);
    }
  }

  // ---- GEMM 2: [skip; out] = W2 . g + b2 (bias = k-step NQ against a ones row)
  f32x16 acc2[M2T];
#pragma unroll
  for (int m = 0; m < M2T; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc2[m][r] = 0.f;
  const f32x4* w2 = reinterpret_cast<const f32x4*>(a.w2) + lane;
#pragma unroll
  for (int q4 = 0; q4 < NQ4; ++q4) {
#pragma unroll
    for (int m2 = 0; m2 < M2T; ++m2) {
      const f32x4 wv = w2[(q4 * M2T + m2) * 64];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = 4 * q4 + i;
        if (q > NQ) continue;
        const float bq = q < NQ ? g[q >> 4][q & 15] : (hh == 0 ? 1.f : 0.f);
        acc2[m2] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[i], bq, acc2[m2], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: skip += W_s g + b_s ; x = (W_o g + b_o + x) * sqrt(0.5)   (residual_block.py:135-138)
  const size_t gt = (size_t)(col0 + wave * 32 + cl);
  const bool live = t0 + wave * 32 + cl < Tu;
  if (!LAST) {
#pragma unroll
    for (int m2 = 0; m2 < M2T; ++m2) {
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const int rowu = 32 * m2 + 8 * j4;  // S, R multiples of 8: wave-uniform branch
        const int row = rowu + 4 * hh;       // 4 consecutive channels row..row+3
        f32x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc2[m2][4 * j4 + i];
        if (rowu < a.S) {
          f32x4* p = reinterpret_cast<f32x4*>(a.skip + gt * a.SS + row);
          *p = a.first ? v : (*p + v);
        } else if (rowu < a.S + a.R) {
          const size_t off = gt * a.RS + (row - a.S);
          const f32x4 xin = *reinterpret_cast<const f32x4*>(a.x_in + off);
          const f32x4 z = {0.f, 0.f, 0.f, 0.f};
          // padding columns stay zero: they are the next layers' right-edge zero pad
          *reinterpret_cast<f32x4*>(a.x_out + off) = live ? (v + xin) * 0.70710677f : z;
        }
      }
    }
    return;
  }

  // ---- last layer: output head on the final skip sum, no x / skip stores
  //   hs = relu(skip * sqrt(1/L)) stays in the accumulator layout and is the B operand of
  //   h1 = W1h . hs + b1h (M3T = ceil(S/32) tiles); y = W2h . relu(h1) + b2h is a per-lane dot
  //   over the lane's 32 rows plus the partner half (lane ^ 32) of the same sample.
  float hs[M2T][16];
#pragma unroll
  for (int m2 = 0; m2 < M2T; ++m2) {
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      const int rowu = 32 * m2 + 8 * j4;
      const int row = rowu + 4 * hh;
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc2[m2][4 * j4 + i];
      if (rowu < a.S) {
        if (!a.first) v += *reinterpret_cast<const f32x4*>(a.skip + gt * a.SS + row);
#pragma unroll
        for (int i = 0; i < 4; ++i) hs[m2][4 * j4 + i] = fmaxf(v[i] * a.skip_scale, 0.f);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) hs[m2][4 * j4 + i] = 0.f;
      }
    }
  }
  constexpr int NQH = 16 * (LAST ? M3T : 1);  // k-steps over skip rows [0, 32*M3T)
  constexpr int NQH4 = (NQH + 1 + 3) / 4;
  constexpr int M3 = LAST ? M3T : 1;
  f32x16 acc3[M3];
#pragma unroll
  for (int m = 0; m < M3; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc3[m][r] = 0.f;
  const f32x4* hw1 = reinterpret_cast<const f32x4*>(a.hw1) + lane;
#pragma unroll
  for (int q4 = 0; q4 < NQH4; ++q4) {
#pragma unroll
    for (int m3 = 0; m3 < M3; ++m3) {
      const f32x4 wv = hw1[(q4 * M3 + m3) * 64];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = 4 * q4 + i;
        if (q > NQH) continue;
        const float bq = q < NQH ? hs[q >> 4][q & 15] : (hh == 0 ? 1.f : 0.f);
        acc3[m3] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[i], bq, acc3[m3], 0, 0, 0);
      }
    }
  }
  const long long t = t0 + wave * 32 + cl;
  float* out = a.out + ud.io_off * a.O + t * a.out_stride_t;
  for (int oc = 0; oc < a.O; ++oc) {
    float part = 0.f;
#pragma unroll
    for (int m3 = 0; m3 < M3; ++m3) {
      const f32x4* w = reinterpret_cast<const f32x4*>(a.hw2 + ((size_t)(oc * M3 + m3) * 2 + hh) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 wq = w[q];
#pragma unroll
        for (int i = 0; i < 4; ++i) part = fmaf(wq[i], fmaxf(acc3[m3][4 * q + i], 0.f), part);
      }
    }
    const float y = part + __shfl_xor(part, 32) + a.hb2[oc];
    if (hh == 0 && t < Tu) out[oc * a.out_stride_o] = y;
  }
}

// ---------------------------------------------------------------------------------------------
// Persistent residual layer: the layer's weights live in LDS for the whole launch, every wave
// streams its own 32-sample blocks from HBM/L2 with register prefetch, no barrier after the
// one-time weight load.
//
// LDS (floats): gate fragments [K1/4][MT][64][4] (96 KB for PWG v1) | W2 fragments (incl. bias)
// [NQ4][M2T][64][4] (36 KB) | gate bias [GR] | last layer: head W1 fragments [NQH4][M3T][64][4].
// GEMM 1 runs in groups of GK k-steps = 2*GK channels of one tap: lane (t, h) loads
// x[t+off][c0 + GK*h .. c0 + GK*h + GK-1] (GK*4 contiguous bytes; the two lane halves read one
// whole 128-byte line per row when GK = 16), the B operand of all GK k-steps (k-step i pairs
// channels c0+i and c0+GK+i; the host packs the weights in that order). One ds_read_b128 per
// m-tile gives 4 k-steps of A. Blocks are assigned statically: block b -> wave (b mod waves).
template <int MT, int M2T, int M3T>
struct PersistSmem {
  static constexpr int GR = 32 * MT;
  static constexpr int GHPAD = (MT == 1) ? 16 : 16 * MT;
  static constexpr int NQ4 = (GHPAD / 2 + 1 + 3) / 4;
  static constexpr int NQH4 = (16 * (M3T > 0 ? M3T : 1) + 1 + 3) / 4;
  static constexpr int W2 = NQ4 * M2T * 256;
  static constexpr int HW1 = M3T > 0 ? NQH4 * M3T * 256 : 0;
  __host__ __device__ static constexpr int floats(int k1) { return k1 / 8 * MT * 256 + W2 + GR + HW1; }
};

// tanh(a) * sigmoid(b) with 2 v_exp + 1 v_rcp: (1 - e^-2a) / ((1 + e^-2a)(1 + e^-b)). Inputs are
// clamped where the result is already saturated in fp32 (|a| > 15: tanh = +-1; b < -30: sigmoid
// < 1e-13) so no intermediate overflows.
__device__ __forceinline__ float fast_gate(float a, float b) {
  a = __builtin_amdgcn_fmed3f(a, -15.f, 15.f);
  b = __builtin_amdgcn_fmed3f(b, -30.f, 88.f);
  const float e1 = __builtin_amdgcn_exp2f(a * -2.8853900817779268f);  // e^{-2a}
  const float e2 = __builtin_amdgcn_exp2f(b * -1.4426950408889634f);  // e^{-b}
  return (1.f - e1) * __builtin_amdgcn_rcpf((1.f + e1) * (1.f + e2));
}

// Stores of the streamed outputs (x_out, skip): plain stores. Write-through sc1 stores (which drop
// the line from the XCD's L2) measured 11 % slower on the LibriTTS bench (4.55 vs 4.10 ms per
// layer). That variant and the other rejected A/B builds of this kernel (B-ring unrolling, A
// prefetch, s_setprio, late aux / early skip loads, sequential GEMM-2 passes, the PWG_TRACE build)
// are in git history before round 4.
__device__ __forceinline__ void store_stream(float* wave_base, int byte_off, f32x4 v) {
  *reinterpret_cast<f32x4*>(reinterpret_cast<char*>(wave_base) + byte_off) = v;
}

constexpr int PWG_PERSIST_THREADS = 512;
// RC / SC: compile-time residual / skip channels for the production shapes (0 = runtime).
// 8 waves per CU (2 per SIMD): measured faster than 12 with the XCD-local schedule (L2 footprint).
template <int MT, int M2T, int M3T, int GK, int RC, int SC, int KSC>
__global__ void __launch_bounds__(PWG_PERSIST_THREADS, 1) pwg_layer_persistent_kernel(const PersistArgs a) {
  using SM = PersistSmem<MT, M2T, M3T>;
  constexpr int NB = GK / 4;                                   // 4-k-step slices per group
  typedef float bvec __attribute__((ext_vector_type(GK)));   // one lane's B operands of a group
  constexpr bool LAST = M3T > 0;
  constexpr int GHPAD = SM::GHPAD;
  constexpr int GR = SM::GR;
  constexpr int NQ = GHPAD / 2;
  constexpr int NQ4 = SM::NQ4;
  constexpr int NG = (MT == 1) ? 1 : MT / 2;
  constexpr int NP = M2T >= 2 ? 2 : 1;       // GEMM-2 passes (pass 0: skip rows for PWG v1)
  constexpr int MP = M2T / NP;
  constexpr int NPASS = LAST ? 1 : NP;       // the last layer needs the skip rows only (S <= 32*MP)
  const int R = RC ? RC : a.R;
  const int S = SC ? SC : a.S;
  const int RS = RC ? (RC + KC - 1) / KC * KC : a.RS;
  const int SS = SC ? (SC + 3) / 4 * 4 : a.SS;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int KS = KSC ? KSC : a.KS;
  const int K1 = KS * RS;
  const int NGRP = K1 / (2 * GK);
  float* s_wg = smem;
  float* s_w2 = s_wg + K1 / 8 * MT * 256;
  float* s_bg = s_w2 + SM::W2;
  float* s_hw1 = s_bg + GR;

  // ---- one-time: this layer's weights into LDS
  {
    const int nthr = blockDim.x, tid = (int)threadIdx.x;
    stage_lds(reinterpret_cast<f32x4*>(s_wg), reinterpret_cast<const f32x4*>(a.wgp), K1 / 8 * MT * 64, tid, nthr);
    stage_lds(reinterpret_cast<f32x4*>(s_w2), reinterpret_cast<const f32x4*>(a.w2), SM::W2 / 4, tid, nthr);
    for (int i = tid; i < GR; i += nthr) s_bg[i] = a.bg[i];
    if (LAST) stage_lds(reinterpret_cast<f32x4*>(s_hw1), reinterpret_cast<const f32x4*>(a.hw1), SM::HW1 / 4, tid, nthr);
    __syncthreads();
  }

  const int lane = threadIdx.x & 63;
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const int nw = blockDim.x >> 6;
  // XCD-local work queues (speed only, never correctness): workgroups are dealt round-robin over
  // the 8 XCDs, so workgroup i runs on XCD i % 8. XCD x owns the x-th contiguous eighth of the
  // blocks; its waves take rounds 0 and 1 statically and then claim blocks in order from the XCD's
  // queue head, so all waves of an XCD sweep its range side by side and the dilated taps of a block
  // re-read rows that neighbouring waves just loaded into the same 4 MB L2. Dynamic claiming
  // balances the two waves sharing a SIMD (arbitration makes one of them up to 30 % slower) and
  // the XCDs (a wave whose own range is drained steals from the next XCDs' queues). Claims run two
  // blocks ahead so the atomic's latency hides behind a whole block.
  const int xcd = blockIdx.x & 7;
  const int wave = threadIdx.x >> 6;
  auto xcd_waves = [&](int y) { return (((int)gridDim.x - y + 7) >> 3) * nw; };
  auto xcd_first = [&](int y) { return (int)((long long)a.n_blocks * y / 8); };
  const int x_first = xcd_first(xcd), x_end = xcd_first(xcd + 1), x_waves = xcd_waves(xcd);
  int victim = 0;  // XCD offset being claimed from: 0 = own queue
  auto ticket_issue = [&]() -> int {  // non-blocking claim on the own queue (lane 0's value)
    int v = 0;
    if (victim == 0 && lane == 0)
      v = __hip_atomic_fetch_add(a.ctr + xcd * SCHED_CTR_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
  };
  auto ticket_resolve = [&](int v) -> int {  // block index of an issued ticket, or steal, or -1
    if (victim == 0) {
      const int i = x_first + 2 * x_waves + __builtin_amdgcn_readfirstlane(v);
      if (i < x_end) return i;
      victim = 1;
    }
    for (; victim < 8; ++victim) {
      const int y = (xcd + victim) & 7;
      int tk = 0;
      if (lane == 0)
        tk = __hip_atomic_fetch_add(a.ctr + y * SCHED_CTR_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int i = xcd_first(y) + 2 * xcd_waves(y) + __builtin_amdgcn_readfirstlane(tk);
      if (i < xcd_first(y + 1)) return i;
    }
    return -1;
  };
  const int gpt = RS / (2 * GK);  // groups per tap
  const f32x4* wgl = reinterpret_cast<const f32x4*>(s_wg) + lane;
  const f32x4* w2l = reinterpret_cast<const f32x4*>(s_w2) + lane;

  // lane's B operand (GK channels) of group g for the block starting at column c
  auto bload = [&](int c, int g) -> bvec {
    const int tap = g / gpt;
    const int c0 = (g - tap * gpt) * 2 * GK;
    const int off = (tap - a.tap_center) * a.dil;
    return *reinterpret_cast<const bvec*>(a.x_in + (size_t)(c + cl + off) * RS + c0 + GK * hh);
  };
  // 4*GK-byte group of k-steps: 16 MFMAs per 4-k-step slice, A from LDS
  auto group_mfma = [&](f32x16 (&acc)[MT], const bvec& b, int g) {
#pragma unroll
    for (int sub = 0; sub < NB; ++sub) {
      f32x4 av[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) av[m] = wgl[((g * NB + sub) * MT + m) * 64];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int m = 0; m < MT; ++m)
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m][i], b[4 * sub + i], acc[m], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  int blk = x_first + (blockIdx.x >> 3) * nw + wave;  // static round 0
  int nblk = blk + x_waves;                           // static round 1
  if (blk >= x_end) blk = -1;
  if (nblk >= x_end) nblk = -1;
  if (blk < 0) return;
  BlockDesc bdn = a.blocks[blk];  // descriptor of the block processed next (loaded a block ahead)
  bvec b0 = bload(bdn.col, 0);     // B operand of the next group (prefetched, across blocks)

  while (true) {
    const BlockDesc bd = bdn;
    bdn = a.blocks[nblk >= 0 ? nblk : blk];  // unconditional: a branch here would force a wait
    const BlockDesc& ui = bd;
    const int col = bd.col + cl;  // this lane's column
    const int t = bd.t0 + cl;     // this lane's utterance-local sample
    const bool live = t < ui.T;
    const int col_next = nblk >= 0 ? bdn.col : bd.col;

    // aux inputs, in flight during GEMM 1: B weights bw[s] = w_t[f - t/H + J1] of frame
    // f = fw0 + 2s + h (a table load per k-step), A = D rows of those frames
    float bw[4];
    float dv[4][MT];
    const int fw0 = bd.t0 / a.H - a.J1;  // wave window (uniform)
    auto load_dv = [&]() {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int f = fw0 + 2 * s + hh;
        const int fc = f < 0 ? 0 : (f >= ui.frames ? ui.frames - 1 : f);  // weight 0 outside
        const float* drow = a.d + (size_t)(ui.frame_base + fc) * GR + cl;
#pragma unroll
        for (int m = 0; m < MT; ++m) dv[s][m] = drow[32 * m];
      }
    };
    {
      const int tc = live ? t : ui.T - 1;
      int roff;
      if (ui.frames < a.Fmin) roff = a.tab_small + (a.H * ui.frames * (ui.frames - 1) / 2 + tc) * AUX_J4;
      else if (tc < a.TL) roff = a.tab_left + tc * AUX_J4;
      else if (tc >= ui.T - a.TR) roff = a.tab_right + (ui.T - 1 - tc) * AUX_J4;
      else roff = (tc % a.H) * AUX_J4;
      const int fb = t / a.H - a.J1;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int f = fw0 + 2 * s + hh;
        const int j = f - fb;
        const bool ok = live && j >= 0 && j < AUX_J4 && s < a.nka;
        const float w = a.tab[roff + (j < 0 ? 0 : (j >= AUX_J4 ? AUX_J4 - 1 : j))];
        bw[s] = ok ? w : 0.f;
      }
    }
    load_dv();  // in flight during GEMM 1

    // ---- GEMM 2 accumulators seeded with [skip_old; x_in]: the MFMA performs the skip sum and
    //      the residual add (residual_block.py:138, parallel_wavegan.py:164); pass-0 loads in flight
    //      during aux + gate, pass-1 loads during pass 0.
    auto init_pass = [&](int pass, f32x16 (&acc2)[MP]) {
#pragma unroll
      for (int mm = 0; mm < MP; ++mm)
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const int rowu = 32 * (pass * MP + mm) + 8 * j4;  // S, R multiples of 8: wave-uniform branch
          const int row = rowu + 4 * hh;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (rowu < S) {
            // unconditional load + select: a branch around the load would make its join wait for it
            v = *reinterpret_cast<const f32x4*>(a.skip + (size_t)col * SS + row);
            if (a.first) v = f32x4{0.f, 0.f, 0.f, 0.f};  // layer 0: no skip sum yet (buffer unset)
          } else if (rowu < S + R) {
            v = *reinterpret_cast<const f32x4*>(a.x_in + (size_t)col * RS + (row - S));
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) acc2[mm][4 * j4 + i] = v[i];
        }
    };
    int ticket = 0;  // claim for the block after next, issued once GEMM 1's loads are out
    f32x16 accp0[MP], accp1[MP];
    // ---- GEMM 1. acc starts from the gate bias (k-step against a ones row, zero C), B operands
    //      ping-pong between two register groups, the last group prefetching the next block's first
    f32x16 acc[MT];
    {
      const float one = hh == 0 ? 1.f : 0.f;
      const f32x16 zero = {};
      float bgv[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) bgv[m] = s_bg[32 * m + cl];  // all reads in flight, one wait
#pragma unroll
      for (int m = 0; m < MT; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(hh == 0 ? bgv[m] : 0.f, one, zero, 0, 0, 0);
    }
    for (int g = 0; g < NGRP; g += 2) {
      const bvec b1 = bload(bd.col, g + 1 < NGRP ? g + 1 : g);
      group_mfma(acc, b0, g);
      if (g + 1 >= NGRP) {  // odd group count: b0 takes the next block's first group
        b0 = bload(col_next, 0);
        break;
      }
      b0 = g + 2 < NGRP ? bload(bd.col, g + 2) : bload(col_next, 0);
      group_mfma(acc, b1, g + 1);
    }

    init_pass(0, accp0);
    if (nblk >= 0) ticket = ticket_issue();

    // ---- aux term: + sum_f D[f][row] * w_t[f - t/H + J1]
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s >= a.nka) break;
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(dv[s][m], bw[s], acc[m], 0, 0, 0);
    }

    // ---- gate: tanh(Za) * sigmoid(Zb)  (residual_block.py:123-132)
    float gt[NG][16];
#pragma unroll
    for (int gm = 0; gm < NG; ++gm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (MT == 1 && r >= 8) { gt[gm][r] = 0.f; continue; }
        gt[gm][r] = fast_gate(acc[gm][r], MT == 1 ? acc[0][r + 8] : acc[gm + MT / 2][r]);
      }
    if (NPASS > 1) init_pass(1, accp1);

    auto gemm2_pass = [&](int pass, f32x16 (&acc2)[MP]) {
#pragma unroll
      for (int q4 = 0; q4 < NQ4; ++q4) {
#pragma unroll
        for (int mm = 0; mm < MP; ++mm) {
          const f32x4 wv = w2l[(q4 * M2T + pass * MP + mm) * 64];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int q = 4 * q4 + i;
            if (q > NQ) continue;
            const float bq = q < NQ ? gt[q >> 4][q & 15] : (hh == 0 ? 1.f : 0.f);
            acc2[mm] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[i], bq, acc2[mm], 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // keep LDS fragment reads next to their MFMAs
      }
    };
    auto store_pass = [&](int pass, const f32x16 (&acc2)[MP]) {
#pragma unroll
      for (int mm = 0; mm < MP; ++mm)
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const int rowu = 32 * (pass * MP + mm) + 8 * j4;
          const int row = rowu + 4 * hh;
          f32x4 v;
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = acc2[mm][4 * j4 + i];
          if (rowu < S) {
            store_stream(a.skip + (size_t)bd.col * SS, (cl * SS + row) * 4, v);
          } else if (rowu < S + R) {
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            // padding columns stay zero: they are the next layers' right-edge zero pad
            store_stream(a.x_out + (size_t)bd.col * RS, (cl * RS + row - S) * 4, live ? v * 0.70710677f : z);
          }
        }
    };

    gemm2_pass(0, accp0);
    if (!LAST) {
      store_pass(0, accp0);
      if (NPASS > 1) {
        gemm2_pass(1, accp1);
        store_pass(1, accp1);
      }
    } else {
      // ---- last layer: fused output head (models/parallel_wavegan.py:131-138,166-171) on the
      //      final skip sum: h1 = W1h . relu(skip * sqrt(1/L)) + b1h as a third MFMA GEMM whose B
      //      operand is the skip tile in registers; y = W2h . relu(h1) + b2h as a per-lane dot
      //      plus the partner lane half.
      constexpr int M3 = LAST ? M3T : 1;
      constexpr int NQH = 16 * M3;
      constexpr int NQH4 = SM::NQH4;
      float hs[MP][16];
#pragma unroll
      for (int mm = 0; mm < MP; ++mm)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 32 * mm + (r & 3) + 8 * (r >> 2) + 4 * hh;
          hs[mm][r] = row < S ? fmaxf(accp0[mm][r] * a.skip_scale, 0.f) : 0.f;
        }
      f32x16 acc3[M3];
#pragma unroll
      for (int m = 0; m < M3; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc3[m][r] = 0.f;
      const f32x4* hw1 = reinterpret_cast<const f32x4*>(s_hw1) + lane;
#pragma unroll
      for (int q4 = 0; q4 < NQH4; ++q4)
#pragma unroll
        for (int m3 = 0; m3 < M3; ++m3) {
          const f32x4 wv = hw1[(q4 * M3 + m3) * 64];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int q = 4 * q4 + i;
            if (q > NQH || (q < NQH && (q >> 4) >= MP)) continue;
            const float bq = q < NQH ? hs[q >> 4][q & 15] : (hh == 0 ? 1.f : 0.f);
            acc3[m3] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[i], bq, acc3[m3], 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      float* out = a.out + (size_t)ui.io_off * a.O + (size_t)t * a.out_stride_t;
      for (int oc = 0; oc < a.O; ++oc) {
        float part = 0.f;
#pragma unroll
        for (int m3 = 0; m3 < M3; ++m3) {
          const f32x4* w = reinterpret_cast<const f32x4*>(a.hw2 + ((size_t)(oc * M3 + m3) * 2 + hh) * 16);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 wq = w[q];
#pragma unroll
            for (int i = 0; i < 4; ++i) part = fmaf(wq[i], fmaxf(acc3[m3][4 * q + i], 0.f), part);
          }
        }
        const float y = part + __shfl_xor(part, 32) + a.hb2[oc];
        if (hh == 0 && live) out[(size_t)oc * a.out_stride_o] = y;
      }
    }

    if (nblk < 0) break;
    blk = nblk;
    nblk = ticket_resolve(ticket);
  }
}

// ---------------------------------------------------------------------------------------------
// One thread per 32-sample block of utterance blockIdx.y of the chunk: its BlockDesc, the
// tile -> utterance map, the utterance's trailing gap tiles (chunk 0 also the leading ones) and
// the UttDesc itself (same values pwg_plan_create computed on the host).
__global__ void __launch_bounds__(256) pwg_plan_desc_kernel(const PlanDescArgs a) {
  const int y = blockIdx.y;
  const UttDesc& d = a.utts[y];
  const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long nb = (d.T + TILE - 1) / TILE * (TILE / 32);
  if (j < nb) {
    BlockDesc b;
    b.t0 = (int)(32 * j);
    b.col = (int)(d.seg_base + b.t0);
    b.T = (int)d.T;
    b.frames = (int)d.frames;
    b.frame_base = (int)d.frame_base;
    b.io_off = (int)d.io_off;
    b.utt = a.u0 + y;
    b.pad = 0;
    a.blocks[d.first_tile * (TILE / 32) + j] = b;
    if (a.prog != nullptr) a.prog[d.first_tile * (TILE / 32) + j] = 0;
    if ((j & (TILE / 32 - 1)) == 0) a.tile_utt[d.first_tile + j / (TILE / 32)] = a.u0 + y;
  }
  if (j < a.gap_tiles) {
    const long long seg_end = d.seg_base + (d.T + TILE - 1) / TILE * TILE;
    a.gap_col0[(long long)(a.u0 + y + 1) * a.gap_tiles + j] = seg_end + j * TILE;
    if (a.u0 == 0 && y == 0) a.gap_col0[j] = j * TILE;
  }
  if (j == 0) a.d_utts[a.u0 + y] = d;
  // the run's work-queue heads and range flag start at zero (a kernel, not hipMemsetAsync: a
  // memset captured into a HIP graph did not reset them on every replay)
  if (a.zero != nullptr && blockIdx.x == 0 && y == 0)
    for (int i = threadIdx.x; i < a.n_zero; i += 256) a.zero[i] = 0;
  // gap tiles of the residual planes (the layers read them as the zero padding of the dilated
  // taps): the gap after this utterance, and chunk 0's leading gap (saves the B = 1 path a launch)
  if (a.zx[0] != nullptr && blockIdx.x == 0) {
    const long long seg_end = d.seg_base + (d.T + TILE - 1) / TILE * TILE;
    const int lead = a.u0 == 0 && y == 0 ? a.gap_tiles : 0;
    const int n4 = 64 * TILE / 4;  // 16-byte stores per tile per plane
    typedef unsigned u32x4z __attribute__((ext_vector_type(4)));
    for (int t = 0; t < a.gap_tiles + lead; ++t) {
      const long long col0 = t < a.gap_tiles ? seg_end + (long long)t * TILE : (long long)(t - a.gap_tiles) * TILE;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        if (a.zx[pl] == nullptr) continue;
        u32x4z* z = reinterpret_cast<u32x4z*>(a.zx[pl] + (size_t)col0 * 64);
        for (int i = threadIdx.x; i < n4; i += 256) z[i] = u32x4z{0u, 0u, 0u, 0u};
      }
    }
  }
}

hipError_t launch_plan_desc(const PlanDescArgs& a, long long max_blocks, hipStream_t s) {
  const long long m = max_blocks > a.gap_tiles ? max_blocks : a.gap_tiles;
  const long long nx = m > 0 ? (m + 255) / 256 : 1;
  hipLaunchKernelGGL(pwg_plan_desc_kernel, dim3((unsigned)nx, (unsigned)a.n), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_conv_in(const ConvInArgs& a, hipStream_t s) {
  if (a.use_conv_in && a.A <= 128) {
    const int mt = (a.A + 31) / 32;
    const dim3 grid((unsigned)((a.F_total + 31) / 32), (unsigned)mt);
    switch (mt) {
      case 1: hipLaunchKernelGGL(pwg_conv_in_ksplit_kernel<1>, grid, dim3(64 * CONV_IN_WAVES), 0, s, a); break;
      case 2: hipLaunchKernelGGL(pwg_conv_in_ksplit_kernel<2>, grid, dim3(64 * CONV_IN_WAVES), 0, s, a); break;
      case 3: hipLaunchKernelGGL(pwg_conv_in_ksplit_kernel<3>, grid, dim3(64 * CONV_IN_WAVES), 0, s, a); break;
      default: hipLaunchKernelGGL(pwg_conv_in_ksplit_kernel<4>, grid, dim3(64 * CONV_IN_WAVES), 0, s, a); break;
    }
    return hipGetLastError();
  }
  const dim3 grid((unsigned)((a.F_total + 63) / 64));
  const int og = (a.A + 3) / 4;
  if (og <= 8) hipLaunchKernelGGL(pwg_conv_in_kernel<8>, grid, dim3(256), 0, s, a);
  else if (og <= 20) hipLaunchKernelGGL(pwg_conv_in_kernel<20>, grid, dim3(256), 0, s, a);
  else if (og <= 32) hipLaunchKernelGGL(pwg_conv_in_kernel<32>, grid, dim3(256), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_aux_proj(const AuxProjArgs& a, int layers, hipStream_t s) {
  const dim3 grid((unsigned)((a.F_total + 127) / 128), (unsigned)layers), block(256);
  if (a.GR == 32) hipLaunchKernelGGL(pwg_aux_proj_kernel<1>, grid, block, 0, s, a);
  else if (a.GR == 64) hipLaunchKernelGGL(pwg_aux_proj_kernel<2>, grid, block, 0, s, a);
  else if (a.GR == 128) hipLaunchKernelGGL(pwg_aux_proj_kernel<4>, grid, block, 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_first_conv(const FirstConvArgs& a, long long n_tiles, hipStream_t s) {
  hipLaunchKernelGGL(pwg_first_conv_kernel, dim3((unsigned)n_tiles), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_layer(const LayerArgs& a, int mt, int m2t, bool last, long long n_tiles, hipStream_t s) {
  const dim3 grid((unsigned)n_tiles), block(256);
  const int m3t = (a.S + 31) / 32;
#define PWG_LAYER_CASE(MT_, M2T_)                                                                  \
  if (mt == MT_ && m2t == M2T_) {                                                                  \
    if (!last) hipLaunchKernelGGL((pwg_layer_kernel<MT_, M2T_, 0>), grid, block, 0, s, a);          \
    else if (m3t == 1) hipLaunchKernelGGL((pwg_layer_kernel<MT_, M2T_, 1>), grid, block, 0, s, a);  \
    else if (m3t == 2 && M2T_ >= 2) hipLaunchKernelGGL((pwg_layer_kernel<MT_, M2T_, (M2T_ >= 2 ? 2 : 1)>), grid, block, 0, s, a); \
    else if (M2T_ >= 4) hipLaunchKernelGGL((pwg_layer_kernel<MT_, M2T_, (M2T_ >= 4 ? 4 : 1)>), grid, block, 0, s, a); \
    else return hipErrorInvalidValue;                                                              \
    return hipGetLastError();                                                                      \
  }
  PWG_LAYER_CASE(1, 1) PWG_LAYER_CASE(1, 2) PWG_LAYER_CASE(1, 4)
  PWG_LAYER_CASE(2, 1) PWG_LAYER_CASE(2, 2) PWG_LAYER_CASE(2, 4)
  PWG_LAYER_CASE(4, 1) PWG_LAYER_CASE(4, 2) PWG_LAYER_CASE(4, 4)
#undef PWG_LAYER_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_layer_persistent(const PersistArgs& a, int mt, int m2t, bool last, int waves_per_wg, int n_wg,
                                   hipStream_t s) {
  if (waves_per_wg > PWG_PERSIST_THREADS / 64) waves_per_wg = PWG_PERSIST_THREADS / 64;
  const dim3 grid((unsigned)n_wg), block((unsigned)(64 * waves_per_wg));
  const int k1 = a.KS * a.RS;
  const int m3t = (a.S + 31) / 32;
  const bool gk16 = a.RS % 32 == 0;  // 32-channel groups when every tap block holds whole groups
#define PWG_PERS_LAUNCH3(MT_, M2T_, M3T_, GK_, RC_, SC_, KSC_)                                             \
  {                                                                                                        \
    const size_t lds = sizeof(float) * PersistSmem<MT_, M2T_, M3T_>::floats(k1);                           \
    if (lds > 160 * 1024) return hipErrorInvalidValue;                                                     \
    auto kfn = &pwg_layer_persistent_kernel<MT_, M2T_, M3T_, GK_, RC_, SC_, KSC_>;                         \
    hipError_t e_ = allow_lds(reinterpret_cast<const void*>(kfn), (int)lds);              \
    if (e_ != hipSuccess) return e_;                                                                       \
    hipLaunchKernelGGL(kfn, grid, block, lds, s, a);                                                       \
    return hipGetLastError();                                                                              \
  }
// PWG v1 (R = S = 64) gets compile-time channel counts; other shapes the runtime kernel.
#define PWG_PERS_LAUNCH2(MT_, M2T_, M3T_, GK_)                                          \
  {                                                                                     \
    if (MT_ == 4 && M2T_ == 4 && a.R == 64 && a.S == 64 && a.KS == 3)                   \
      PWG_PERS_LAUNCH3(MT_, M2T_, M3T_, GK_, 64, 64, 3)                                 \
    else PWG_PERS_LAUNCH3(MT_, M2T_, M3T_, GK_, 0, 0, 0)                                \
  }
#define PWG_PERS_LAUNCH(MT_, M2T_, M3T_) \
  { if (gk16) PWG_PERS_LAUNCH2(MT_, M2T_, M3T_, 16) else PWG_PERS_LAUNCH2(MT_, M2T_, M3T_, 8) }
#define PWG_PERS_CASE(MT_, M2T_)                                                    \
  if (mt == MT_ && m2t == M2T_) {                                                   \
    if (!last) PWG_PERS_LAUNCH(MT_, M2T_, 0)                                        \
    if (m3t == 1) PWG_PERS_LAUNCH(MT_, M2T_, 1)                                     \
    if (m3t == 2 && M2T_ >= 2) PWG_PERS_LAUNCH(MT_, M2T_, (M2T_ >= 2 ? 2 : 1))      \
    if (M2T_ >= 4) PWG_PERS_LAUNCH(MT_, M2T_, (M2T_ >= 4 ? 4 : 1))                  \
    return hipErrorInvalidValue;                                                    \
  }
  PWG_PERS_CASE(1, 1) PWG_PERS_CASE(1, 2) PWG_PERS_CASE(1, 4)
  PWG_PERS_CASE(2, 1) PWG_PERS_CASE(2, 2) PWG_PERS_CASE(2, 4)
  PWG_PERS_CASE(4, 1) PWG_PERS_CASE(4, 2) PWG_PERS_CASE(4, 4)
#undef PWG_PERS_CASE
#undef PWG_PERS_LAUNCH
#undef PWG_PERS_LAUNCH2
#undef PWG_PERS_LAUNCH3
  return hipErrorInvalidValue;
}

}  // namespace pwg
