// Conv-network executor (include/pwg_cnet.h): the MelGAN / multi-band MelGAN + PQMF / HiFiGAN
// generators as programs of fused fp32 MFMA implicit-GEMM conv ops, for gfx950.
//
// One op = one launch of pwg_cnet_conv_kernel<MT>:
//   * workgroup = 4 waves x 32 output columns (one 128-column block of ONE utterance) x 32*MT
//     output rows; grid = (blocks, row tiles);
//   * K = sum over sources, taps and 16-channel chunks; a chunk is 8 k-steps of
//     v_mfma_f32_32x32x2_f32 in which k-step i pairs channels c0+i (lane half 0) and c0+8+i (lane
//     half 1), so a lane's B operand of a chunk is 8 contiguous channels (32 bytes) of one
//     time-major row, loaded with the op's pre-activation (normalize, LeakyReLU) and edge mode
//     (zero / reflect) applied, one chunk ahead in registers;
//   * the chunk's A fragments (host-packed lane-linear, MT x 2 KB) are staged in LDS by the whole
//     workgroup, double-buffered, one barrier per chunk;
//   * epilogue: + bias (+ second bias) + residual (+ old value) then / out_div then post
//     activation, 16-byte stores of 4 consecutive channels of one time row.
// Split-f16 mode (pwg_cnet_set_option PWG_CNET_OPT_SPLIT_F16, default on): the same kernel with
// every operand an fp16 pair v = hi + lo and ONE v_mfma_f32_32x32x16_f16 k-step per chunk run
// three times (hi*hi, hi*lo, lo*hi), fp32 accumulate, as the PWG layer: a lane's
// 8 channels of a chunk are exactly its 32x32x16 B fragment (k = 8*hh + j), and the A fragments
// ([chunk][m][hi/lo][lane][8 halves]) take the fp32 fragments' bytes.
// ConvTranspose1d(kernel 2s, stride s) runs as s phase launches: outputs t = q*s + r are a 2-tap
// conv of input rows q + floor((r+p)/s) - {0, 1} with taps k_a = (r+p) mod s and k_a + s.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/pwg_cnet.h"
#include "pwg_internal.h"

namespace pwg {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef float f32x8v __attribute__((ext_vector_type(8)));

constexpr int CN_COLS = 128;       // output columns per workgroup (4 waves x 32)
constexpr int CN_CHUNK = 16;       // input channels per K chunk
constexpr int CN_MAX_CHUNKS = 4096;
// Tuned choices (round 2, same-box A/B; the rejected alternatives are in git history before
// round 3: two chunks per barrier, two column tiles per wave, 512-column x-tile workgroups, 2/4
// channel blocks per staging step, two-deep load rings, explicit waves-per-SIMD requests).
constexpr int CN_G = 1;                    // 16-channel chunks staged per barrier (2: 9 % slower)
constexpr int CN_NARROW_G = 4;             // ... in narrow tap-major launches (small plans: fewer, longer
                                           // steps between barriers; same product order)
constexpr int CNET_NW8_MT = 4;             // conv ops with MT >= this run 8-wave workgroups (256 columns)
constexpr int CNET_XTILE_LDS = 150 * 1024; // LDS budget of one x-tile workgroup
constexpr int CNET_XPAIR_MAXK = 11;        // largest kernel size fused into an x-tile pair
// x-tile ConvTranspose phases launched together too (A/B: -DCNET_CT_ZMERGE=0)
#ifndef CNET_CT_ZMERGE
#define CNET_CT_ZMERGE 1
#endif
constexpr int CNET_XTILE_CONVT = 2;        // ConvTranspose phases of <= this many m-tiles on the x-tile
                                           // kernel: faster up to 64 output channels, slower at 128-256
                                           // (stride 8; profiles/r02_ct)
// PWG_CNET_OPT_XT_DMA flags (include/pwg_cnet.h)
constexpr int CNET_DMA_RULE = 1, CNET_DMA_ALL = 2, CNET_DMA_FEWEST = 4, CNET_DMA_CONVT = 8;
constexpr int CNET_XT_MT2_MAXK = 7;        // >= 256-row convs with <= this many taps: 2 m-tiles per workgroup

struct ChunkDesc {   // one K chunk of an op (uniform per launch)
  int src;           // 0 / 1
  int row_off;       // -pad + tap*dil
  int c0;            // first input channel
  int pad;
};

struct CnSrc {
  const float* x;
  const int* seg;    // [n_utts][2]: first row, rows of this buffer
  int ld;
  int pad_mode;
  int normalize;
  float slope;
  int taps, nc;      // thin kernel: taps, 16-channel blocks
  int chunk_base;    // first chunk of this source (chunks: tap-major, then channel block)
  int off_min;       // smallest tap row offset
  int span;          // rows a 128-column block reads: 128 + off_max - off_min
};

struct CnConvArgs {
  CnSrc src[2];
  const ChunkDesc* chunks;
  int n_chunks;
  const float* wfrag;     // [chunk][MTtot][2][64][4]
  int mt_total;
  const float* bias;      // MTtot*32 floats (both biases summed host-side, zero padded)
  const float* res;
  const int* seg_res;
  int ld_res;
  float* y;
  const int* seg_dst;
  int ld_dst;
  int M;
  int accumulate;
  float out_div;
  int post_act;
  float post_slope;
  const int2* blocks;     // (utt, q0)
  const int* ncols;       // [n_utts] columns of this phase
  int ostride, ophase;
  const float* mean;
  const float* scale;
  // ConvTranspose1d in ONE launch: blockIdx.z = output phase r (phase 0 = the fields above);
  // phases share the block list (every phase has T / stride columns per utterance)
  const ChunkDesc* z_chunks[8];
  const float* z_wfrag[8];
  const float* z_bias[8];
  int* range_flag;        // thin kernel writing the program output (split-f16 mode): set to 1 on a
                          // non-finite output value (pwg_cnet_run_status), else null
  int xcd_order;          // 1: XCD-aware tile order (xcd_tile), PWG_CNET_OPT_XCD_ORDER
  // pre-split images of the output rows written by the x-tile kernels' epilogue (cn_store_col's
  // quad path; PWG_CNET_OPT_PRESPLIT): n_oimg of them, each with its readers' LeakyReLU slope,
  // [row][16-channel block][hi 16 f16 | lo 16 f16], oimg_rowb = channels x 4 B
  unsigned char* oimg[2];
  float oslope[2];
  int n_oimg, oimg_rowb;
};

// 16 zero bytes (64 allocated): the DMA source of a pre-split row outside a zero-padded utterance
__device__ __attribute__((aligned(64))) unsigned g_cn_zero16[16];

// 4 output channels row .. row + 3 of image row irow: the readers' LeakyReLU (as their staging
// applies it) and the fp16 pair split of the values just stored
__device__ __forceinline__ void cn_img4(unsigned char* img, long long irow, int rowb, int row, const float (&v)[4],
                                        float slope) {
  _Float16 hv[4], lv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float x = v[i];
    if (slope != 1.f) x = x > 0.f ? x : x * slope;
    hv[i] = (_Float16)x;
    lv[i] = (_Float16)(x - (float)hv[i]);
  }
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  unsigned char* const d = img + irow * rowb + (row >> 4) * 64 + (row & 15) * 2;
  *reinterpret_cast<h4*>(d) = h4{hv[0], hv[1], hv[2], hv[3]};
  *reinterpret_cast<h4*>(d + 32) = h4{lv[0], lv[1], lv[2], lv[3]};
}

// Workgroup -> (column block, m-group, ConvTranspose phase). Workgroup ids are dispatched x-fastest
// and dealt round-robin over the 8 XCDs, each with its own L2: in grid order the m-groups and phases
// of one column block (which stage the same input rows) land on different XCDs, nx dispatches apart,
// and each re-fetches those rows from HBM. The XCD-aware order deals the ny x nz siblings of a
// column block to ONE XCD in consecutive rounds (ids L, L + 8, ...), where the later ones find the
// rows in L2. A bijection over the grid (the last partial group of 8 column blocks keeps a plain
// order); the tiles, and so the results, are the same.
struct TileId { int x, y, z; };
__device__ __forceinline__ TileId xcd_tile(int enable) {
  const int nx = gridDim.x, ns = gridDim.y * gridDim.z;
  if (!enable || ns == 1) return {(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
  const long long L = blockIdx.x + (long long)nx * (blockIdx.y + (long long)gridDim.y * blockIdx.z);
  const long long G = 8LL * ns, full = nx / 8;
  const long long g = L / G;
  int x, sib;
  if (g < full) {
    const int r = (int)(L - g * G);
    x = (int)(g * 8) + (r & 7);
    sib = r >> 3;
  } else {
    const int tail = nx - (int)(full * 8);
    const int r = (int)(L - full * G);
    x = (int)(full * 8) + r % tail;
    sib = r / tail;
  }
  return {x, sib % (int)gridDim.y, sib / (int)gridDim.y};
}

__device__ __forceinline__ int reflect_row(int p, int T) {
  p = p < 0 ? -p : p;
  p = p >= T ? 2 * (T - 1) - p : p;
  return p < 0 ? 0 : (p >= T ? T - 1 : p);  // masked columns / tiny T: stay in bounds
}

// Row p of a T-row utterance under the source's edge mode, clamped in bounds; false: the tap reads
// zero (PWG_PAD_ZERO outside the utterance). REFLECT mirrors (ReflectionPad1d), REPLICATE takes
// the edge row (ReplicationPad1d: CausalConvTranspose1d's left pad).
__device__ __forceinline__ bool edge_row(int& p, int T, int mode) {
  if (mode == PWG_PAD_REFLECT) {
    p = reflect_row(p, T);
    return true;
  }
  const bool inside = p >= 0 && p < T;
  p = p < 0 ? 0 : (p >= T ? T - 1 : p);
  return inside || mode == PWG_PAD_REPLICATE;
}

typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8v __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x4v __attribute__((ext_vector_type(4)));

// 8 fp32 -> fp16 pairs: hi = rne16(v), lo = rne16(v - hi)
__device__ __forceinline__ void cn_split8(const f32x8v& v, u32x4v& hi, u32x4v& lo) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const _Float16 h0 = (_Float16)v[2 * d], h1 = (_Float16)v[2 * d + 1];
    hi[d] = __builtin_bit_cast(unsigned, f16x2v{h0, h1});
    lo[d] = __builtin_bit_cast(unsigned, f16x2v{(_Float16)(v[2 * d] - (float)h0), (_Float16)(v[2 * d + 1] - (float)h1)});
  }
}

template <int MT, int NT, int G, bool SPLIT = false, int NW = 4>
__global__ void __launch_bounds__(64 * NW) pwg_cnet_conv_kernel(const CnConvArgs a) {
  constexpr int NTH = 64 * NW;                      // threads: NW waves x 32 * NT columns each
  constexpr int AQ = (MT * 128 + NTH - 1) / NTH;    // A-fragment 16-B vectors per thread and chunk
  __shared__ __attribute__((aligned(16))) float s_a[2][G * MT * 512];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const TileId tid = xcd_tile(a.xcd_order);
  const int2 blk = a.blocks[tid.x];
  const int u = blk.x;
  const int qb = blk.y + wave * 32 * NT + cl;  // this lane's column in n-tile 0 (phase index space)
  const int nq = a.ncols[u];
  const int m0 = tid.y * MT;                   // first m-tile of this workgroup
  // ConvTranspose phase of this workgroup (all phases in one launch; 0 for plain convs)
  const int zp = tid.z;
  const ChunkDesc* const chunks_ = zp == 0 ? a.chunks : a.z_chunks[zp];
  const float* const wfrag_ = zp == 0 ? a.wfrag : a.z_wfrag[zp];
  const float* const bias_ = zp == 0 ? a.bias : a.z_bias[zp];
  const int ophase_ = a.ophase + zp;

  // B operands of chunk c for the NT column tiles: 8 channels of one input row each. The load
  // (braw) and the pre-activation (bprep) are split so the raw loads of chunk c+1 stay in flight
  // during chunk c's MFMAs: processing them right after issue would wait for them there.
  struct BRaw {
    f32x8v v[NT];
    bool ok[NT];
    int c;
  };
  auto braw = [&](int c, BRaw& r) {
    const ChunkDesc cd = chunks_[c];
    const CnSrc& s = a.src[cd.src];
    const int2 sg = *reinterpret_cast<const int2*>(s.seg + 2 * u);
    const int ch = cd.c0 + 8 * hh;
    r.c = c;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      int p = qb + 32 * n + cd.row_off;
      const bool ok = edge_row(p, sg.y, s.pad_mode);
      r.v[n] = *reinterpret_cast<const f32x8v*>(s.x + (size_t)(sg.x + p) * s.ld + ch);
      r.ok[n] = ok;
    }
  };
  auto bprep = [&](const BRaw& r, f32x8v (&v)[NT]) {
    const ChunkDesc cd = chunks_[r.c];
    const CnSrc& s = a.src[cd.src];
    const int ch = cd.c0 + 8 * hh;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      f32x8v x = r.v[n];
      if (s.normalize) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = (x[i] - a.mean[ch + i]) / a.scale[ch + i];
      }
      if (s.slope != 1.f) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = x[i] > 0.f ? x[i] : x[i] * s.slope;
      }
      v[n] = r.ok[n] ? x : f32x8v{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    }
  };
  // (G chunks are staged per barrier; the host pads the chunk list to a multiple of G with
  // zero-weight chunks)
  // (narrow launches, G > 1: the last group may be partial; its missing chunks load nothing and
  // run no MFMAs, so every accumulator sees the same product sequence as with G = 1)
  auto aload = [&](int cg, f32x4v (&r)[G][AQ]) {
#pragma unroll
    for (int g2 = 0; g2 < G; ++g2) {
      const bool live = G == 1 || cg * G + g2 < a.n_chunks;
      const f32x4v* gp = reinterpret_cast<const f32x4v*>(wfrag_ + ((size_t)(live ? cg * G + g2 : 0) * a.mt_total + m0) * 512);
#pragma unroll
      for (int i = 0; i < AQ; ++i) {
        const int idx = threadIdx.x + NTH * i;
        r[g2][i] = idx < MT * 128 && live ? gp[idx] : f32x4v{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto astore = [&](int buf, const f32x4v (&r)[G][AQ]) {
#pragma unroll
    for (int g2 = 0; g2 < G; ++g2) {
      f32x4v* d = reinterpret_cast<f32x4v*>(s_a[buf] + g2 * MT * 512);
#pragma unroll
      for (int i = 0; i < AQ; ++i) {
        const int idx = threadIdx.x + NTH * i;
        if (idx < MT * 128) d[idx] = r[g2][i];
      }
    }
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;

  // one chunk group's MFMAs from LDS buffer buf and the prepared B operands
  auto compute = [&](int buf, const f32x8v (&bc)[G][NT], int n_live) {
#pragma unroll
    for (int g2 = 0; g2 < G; ++g2) {
      if (G > 1 && g2 >= n_live) break;
      if constexpr (SPLIT) {
        const u32x4v* sa = reinterpret_cast<const u32x4v*>(s_a[buf] + g2 * MT * 512) + lane;
        u32x4v bh[NT], bl[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) cn_split8(bc[g2][n], bh[n], bl[n]);
        u32x4v ah[MT], al[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          ah[m] = sa[(m * 2) * 64];
          al[m] = sa[(m * 2 + 1) * 64];
        }
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah[m]),
                                                               __builtin_bit_cast(f16x8v, bh[n]), acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah[m]),
                                                               __builtin_bit_cast(f16x8v, bl[n]), acc[m][n], 0, 0, 0);
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, al[m]),
                                                               __builtin_bit_cast(f16x8v, bh[n]), acc[m][n], 0, 0, 0);
          }
      } else {
        const f32x4v* sa = reinterpret_cast<const f32x4v*>(s_a[buf] + g2 * MT * 512) + lane;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          f32x4v av[MT];
#pragma unroll
          for (int m = 0; m < MT; ++m) av[m] = sa[(m * 2 + sub) * 64];
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
              for (int n = 0; n < NT; ++n)
                acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m][e], bc[g2][n][4 * sub + e], acc[m][n], 0, 0, 0);
        }
      }
    }
  };

  const int n_groups = (a.n_chunks + G - 1) / G;
  auto cmin = [&](int c) { return c < a.n_chunks ? c : a.n_chunks - 1; };  // partial group: in-bounds reads
  f32x8v bcur[G][NT];
  f32x4v ar[G][AQ];
  aload(0, ar);
  astore(0, ar);
  BRaw bnext[G];
#pragma unroll
  for (int g2 = 0; g2 < G; ++g2) {
    braw(cmin(g2), bnext[g2]);
    bprep(bnext[g2], bcur[g2]);
  }
  __syncthreads();
  for (int cg = 0; cg < n_groups; ++cg) {
    const bool more = cg + 1 < n_groups;
    if (more) {
      aload(cg + 1, ar);
#pragma unroll
      for (int g2 = 0; g2 < G; ++g2) braw(cmin((cg + 1) * G + g2), bnext[g2]);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the loads issued before the MFMAs below
    compute(cg & 1, bcur, a.n_chunks - cg * G);
    __builtin_amdgcn_sched_barrier(0);  // ... and their consumers after them
    if (more) astore((cg + 1) & 1, ar);
    __syncthreads();
    if (more) {
#pragma unroll
      for (int g2 = 0; g2 < G; ++g2) bprep(bnext[g2], bcur[g2]);
    }
  }

  // epilogue
  const int2 sd = *reinterpret_cast<const int2*>(a.seg_dst + 2 * u);
  const int2 sr = a.res ? *reinterpret_cast<const int2*>(a.seg_res + 2 * u) : make_int2(0, 0);
  const bool quad = (a.ld_dst & 3) == 0;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int q = qb + 32 * n;
    if (q >= nq) continue;
    const int t = q * a.ostride + ophase_;
    float* yrow = a.y + (size_t)(sd.x + t) * a.ld_dst;
    const float* rrow = a.res ? a.res + (size_t)(sr.x + t) * a.ld_res : nullptr;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const int row = 32 * (m0 + m) + 8 * j4 + 4 * hh;
        if (row >= a.M) {
          // padding channels of a padded buffer are written as zeros: later ops read whole chunks
          if (quad && row < a.ld_dst) *reinterpret_cast<f32x4v*>(yrow + row) = f32x4v{0.f, 0.f, 0.f, 0.f};
          continue;
        }
        const f32x4v b = *reinterpret_cast<const f32x4v*>(bias_ + row);
        f32x4v v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[m][n][4 * j4 + i] + b[i];
        if (quad) {
          if (rrow) v += *reinterpret_cast<const f32x4v*>(rrow + row);
          if (a.accumulate) v = *reinterpret_cast<const f32x4v*>(yrow + row) + v;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (row + i >= a.M) continue;
            if (rrow) v[i] += rrow[row + i];
            if (a.accumulate) v[i] = yrow[row + i] + v[i];
          }
        }
        if (a.out_div != 1.f) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = v[i] / a.out_div;
        }
        if (a.post_act == PWG_ACT_LRELU) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = v[i] > 0.f ? v[i] : v[i] * a.post_slope;
        } else if (a.post_act == PWG_ACT_TANH) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = tanhf(v[i]);
        }
        if (quad) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (row + i >= a.M) v[i] = 0.f;
          *reinterpret_cast<f32x4v*>(yrow + row) = v;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (row + i < a.M) yrow[row + i] = v[i];
        }
      }
  }
}

// Wide dilated convs (split-f16, >= 128 output rows per tile, K taps > 1): channel-block-major
// variant of pwg_cnet_conv_kernel with the input tile staged ONCE per 16-channel block.
// pwg_cnet_conv_kernel walks chunks tap-major and loads every tap's B rows from L2 again (k loads
// of each input column) while staging one 16-channel A chunk per barrier; on HiFiGAN's 128/256-
// channel convs that is ~30-40 B per CU-cycle of L2 -> CU traffic, the kernel's limit. Here a
// workgroup (8 waves x 32 columns = 256 output columns, MT m-tiles of rows) stages, per 16-channel
// block cb:
//   * the A fragments of ALL K taps of cb (K x MT x 2 KB), and
//   * the block's input rows [q0 - pad, q0 + 256 - pad + (K-1) dil) x 16 channels, pre-activated
//     (normalize, LeakyReLU, edge mode) and pair-split once, [row][hi 16 | lo 16 halves | pad],
// then every wave runs K x MT x 3 MFMAs with A and B from LDS; the next block's loads are in
// flight meanwhile (registers), two barriers per block. Same products and pair splits as the
// tap-major kernel, summed channel-block-major (fp32 rounding order differs; parity vs the oracle).
// ConvTranspose1d phases run here too (K = 2 taps at rows q + off_a - 1, q + off_a, dilation 1;
// rev: tap t uses the phase's weight chunk K-1-t; blockIdx.z = phase as in pwg_cnet_conv_kernel).
struct CnXtileArgs {
  int K, dil, off_min;    // taps, dilation, first tap's row offset (-pad)
  int cs;                 // 16-channel blocks of the source
  int span;               // input rows per block: 256 + (K-1) dil
  int rev;                // 1: tap t multiplies weight chunk K-1-t (ConvTranspose phases)
  int z_off[8];           // ConvTranspose: off_min of phase blockIdx.z (z_off[0] = off_min)
  const unsigned char* simg;  // PRE (narrow DMA-staged launches): the source's pre-split image
  int simg_rowb;              // ... its row bytes (channels x 4)
};
__host__ __device__ constexpr bool xtile_supported(int k) { return k == 3 || k == 5 || k == 7 || k == 11; }
constexpr int XT_COLS = 256;
constexpr int NARROW_HALO = 64;  // narrow x-tile launches: (K - 1) dil at most this (register budget)
constexpr int XT_ROWB = 80;  // bytes per staged input row: 16 hi + 16 lo halves + 16 B pad

// One lane's column of MT m-tiles: + bias [+ residual] [+ y_old] [/ div] [act] -> y (the conv
// kernels' epilogue arithmetic). With quad-aligned rows every bias / residual / y_old load is issued
// before the first store: the stores may alias the later loads for the compiler, which otherwise
// serialises one load round trip per 4 rows (MT x 4 of them, ~1 us each at B = 1).
// IMG: also the pre-split images a.oimg (narrow launches only: the wide kernels keep their epilogue)
// GM: m-tiles per load group (3 x 4 quads each in flight); 1 in kernels held to 128 VGPRs (the
// DMA-staged and synchronous x-tile kernels: at MT 2 a group of 2 spilled 42-55 VGPRs to scratch)
template <int MT, bool IMG = false, int GM = (MT <= 2 ? MT : 1)>
__device__ __forceinline__ void cn_store_col(const CnConvArgs& a, const f32x16 (&acc)[MT], const float* bias_, int m0,
                                             int hh, float* yrow, const float* rrow, long long irow = 0) {
  auto finish = [&](f32x4v v) {
    if (a.out_div != 1.f) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = v[i] / a.out_div;
    }
    if (a.post_act == PWG_ACT_LRELU) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = v[i] > 0.f ? v[i] : v[i] * a.post_slope;
    } else if (a.post_act == PWG_ACT_TANH) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = tanhf(v[i]);
    }
    return v;
  };
  if ((a.ld_dst & 3) == 0) {
#pragma unroll
    for (int mg = 0; mg < MT; mg += GM) {
      f32x4v bv[GM][4], rv[GM][4], yv[GM][4];
#pragma unroll
      for (int m = 0; m < GM; ++m)
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const int row = 32 * (m0 + mg + m) + 8 * j4 + 4 * hh;
          const bool live = row < a.M;
          const f32x4v z = {0.f, 0.f, 0.f, 0.f};
          bv[m][j4] = live ? *reinterpret_cast<const f32x4v*>(bias_ + row) : z;
          rv[m][j4] = live && rrow ? *reinterpret_cast<const f32x4v*>(rrow + row) : z;
          yv[m][j4] = live && a.accumulate ? *reinterpret_cast<const f32x4v*>(yrow + row) : z;
        }
#pragma unroll
      for (int m = 0; m < GM; ++m)
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const int row = 32 * (m0 + mg + m) + 8 * j4 + 4 * hh;
          if (row >= a.M) {
            if (row < a.ld_dst) *reinterpret_cast<f32x4v*>(yrow + row) = f32x4v{0.f, 0.f, 0.f, 0.f};
            continue;
          }
          f32x4v v;
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = acc[mg + m][4 * j4 + i] + bv[m][j4][i];
          if (rrow) v += rv[m][j4];
          if (a.accumulate) v = yv[m][j4] + v;
          v = finish(v);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (row + i >= a.M) v[i] = 0.f;
          *reinterpret_cast<f32x4v*>(yrow + row) = v;
          if constexpr (IMG) {
            const float vv[4] = {v[0], v[1], v[2], v[3]};
            for (int j = 0; j < a.n_oimg; ++j) cn_img4(a.oimg[j], irow, a.oimg_rowb, row, vv, a.oslope[j]);
          }
        }
    }
    return;
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      const int row = 32 * (m0 + m) + 8 * j4 + 4 * hh;
      if (row >= a.M) continue;
      const f32x4v b = *reinterpret_cast<const f32x4v*>(bias_ + row);
      f32x4v v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[m][4 * j4 + i] + b[i];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (row + i >= a.M) continue;
        if (rrow) v[i] += rrow[row + i];
        if (a.accumulate) v[i] = yrow[row + i] + v[i];
      }
      v = finish(v);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (row + i < a.M) yrow[row + i] = v[i];
    }
}

// SY (synchronous staging): no register prefetch of the next channel block; the kernel is held to
// 128 VGPRs (4 waves per SIMD) so two workgroups share a CU and one's staging overlaps the other's
// MFMAs. Same arithmetic and order: bit-identical.
template <int MT, int K, int CB, bool SY = false, bool DB = false>
constexpr int xt_wpe() {
  return SY || DB ? 4 : 1;  // DB: also held to 128 VGPRs, two workgroups per CU when LDS allows
}
// NC column tiles of 256 per workgroup (wave w: columns 256 nc + 32 w + [0, 32)); the engine runs
// NC = 1 (NC = 2 measured no faster, profiles/r02_nc).
// KS (SY only): taps whose A fragments are staged per step; KS < K stages a channel block's taps in
// ceil(K / KS) steps (same MFMA order) so the A region fits two workgroups per CU (k = 11, MT 4).
// DB (double-buffered DMA staging): the A fragments of the next tap group go global -> LDS by
// global_load_lds (no registers) into the second of two A buffers while the waves run the MFMAs of
// the current one; the next channel block's input rows are loaded to registers over the last tap
// group's MFMAs and converted into the (single) row buffer after it. KS < K: two tap groups per
// channel block, [0, KS) always in buffer 0 and [KS, K) in buffer 1; KS == K: the buffers alternate
// per block. Same products in the same order as the other variants: bit-identical.
// PRE (narrow DMA-staged launches, PWG_CNET_OPT_PRESPLIT): the input rows come pre-activated and
// pair-split from the source's image (its writer's epilogue), DMA'd straight into one of two row
// buffers during the previous block's last tap group -- no register prefetch, no conversion, one
// barrier per block end instead of two. Rows are 64 B with piece q of row r at slot q ^ ((r >> 2) & 3).
template <int MT, int K, int CB, int NC = 1, bool SY = false, int KS = K, bool DB = false, int NWV = 8, bool PRE = false>
__global__ void __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(xt_wpe<MT, K, CB, SY, DB>())))
pwg_cnet_xtile_kernel(const CnConvArgs a, const CnXtileArgs xt) {
  static_assert(KS == K || SY || DB, "tap-split staging is a synchronous-staging or DMA variant");
  static_assert(!PRE || (DB && NWV < 8), "pre-split rows: the narrow DMA-staged variant");
  static_assert(!DB || (CB == 1 && NC == 1 && !SY), "DMA staging: one block, one column tile");
  static_assert(NWV == 8 || (DB && NC == 1), "narrow workgroups: the DMA-staged variant");
  constexpr int NTH = 64 * NWV;
  constexpr int XC = 32 * NWV;  // output columns per column tile (256 at 8 waves)
  constexpr int AV = CB * K * MT * 128;                // A vectors (16 B) per group of CB channel blocks
  constexpr int AQ = DB ? 1 : (AV + NTH - 1) / NTH;
  constexpr int A_BYTES = CB * KS * MT * 2048;
  extern __shared__ __attribute__((aligned(16))) unsigned char xt_smem[];
  f32x4v* s_a = reinterpret_cast<f32x4v*>(xt_smem);                          // [CB][K][MT][2][64] x 16 B
  f32x4v* s_a1 = reinterpret_cast<f32x4v*>(xt_smem + (DB ? A_BYTES : 0));   // DB: second A buffer
  unsigned char* s_x = xt_smem + (size_t)(DB ? 2 : 1) * A_BYTES;              // [CB][span][XT_ROWB]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const TileId tid = xcd_tile(a.xcd_order);
  const int2 blk = a.blocks[tid.x];
  const int u = blk.x;
  const int q0 = blk.y;
  const int nq = a.ncols[u];
  const int m0 = tid.y * MT;
  const int zp = tid.z;  // ConvTranspose phase (0 for convs)
  // column tiles holding live columns (uniform over the workgroup)
  const int nc_live = NC == 1 ? 1 : (nq - q0 > XC ? NC : 1);
  const float* const wfrag_ = zp == 0 ? a.wfrag : a.z_wfrag[zp];
  const float* const bias_ = zp == 0 ? a.bias : a.z_bias[zp];
  const int ophase_ = a.ophase + zp;
  const int off_min = xt.z_off[zp];
  const CnSrc& sx = a.src[0];
  const int2 sg = *reinterpret_cast<const int2*>(sx.seg + 2 * u);
  const int xv = CB * xt.span * 4;                     // input quads (4 channels) per group
  constexpr int XQ_MAX = (CB * (NC * XC + (NWV == 8 ? 192 : NARROW_HALO)) * 4 + NTH - 1) / NTH;
  // PRE: rows per buffer (the span, rounded to the 16 rows of a DMA instruction), instructions
  constexpr int XRP = (XC + (K == 2 ? 16 : NARROW_HALO) + 15) / 16 * 16;
  constexpr int NXI = XRP / 16, DXI = (NXI + NWV - 1) / NWV;
  long long pxo[PRE ? DXI : 1];  // each lane's (row, piece) byte offset in the image's block 0, -1: zero
  if constexpr (PRE) {
#pragma unroll
    for (int k = 0; k < DXI; ++k) {
      const int i = wave + NWV * k;
      const int r = 16 * i + (lane >> 2), q = (lane & 3) ^ ((r >> 2) & 3);
      int p = q0 + off_min + r;
      const bool ok = i < NXI && r < xt.span && edge_row(p, sg.y, sx.pad_mode);
      pxo[k] = ok ? (long long)(sg.x + p) * xt.simg_rowb + q * 16 : -1;
    }
  }
  const unsigned char* s_xcur = s_x;  // PRE: the row buffer of the block being computed

  f32x4v ar[AQ];
  f32x4v xr[XQ_MAX];
  bool xok[XQ_MAX];
  // group g = channel blocks [CB g, CB g + CB): global -> registers
  auto aload = [&](int grp) {
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      const int idx = threadIdx.x + NTH * i;  // [c][tap][m][128 vectors]
      const int c = idx / (K * MT * 128), rem1 = idx - c * (K * MT * 128);
      const int tap = rem1 / (MT * 128), rem = rem1 - tap * (MT * 128);
      const int wt = xt.rev ? K - 1 - tap : tap;
      ar[i] = idx < AV ? reinterpret_cast<const f32x4v*>(
                             wfrag_ + ((size_t)(wt * xt.cs + CB * grp + c) * a.mt_total + m0) * 512)[rem]
                       : f32x4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto xload = [&](int grp) {
#pragma unroll
    for (int i = 0; i < XQ_MAX; ++i) {
      const int idx = threadIdx.x + NTH * i;  // [c][row][quad]
      const bool in = idx < xv;
      const int c = in ? idx / (xt.span * 4) : 0;
      const int r = in ? (idx >> 2) - c * xt.span : 0, qd = idx & 3;
      int p = q0 + off_min + r;
      xok[i] = edge_row(p, sg.y, sx.pad_mode) && in;
      xr[i] = in ? *reinterpret_cast<const f32x4v*>(sx.x + (size_t)(sg.x + p) * sx.ld + 16 * (CB * grp + c) + 4 * qd)
                 : f32x4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto load = [&](int grp) {
    aload(grp);
    xload(grp);
  };
  // registers -> LDS (x pre-activated and pair-split on the way)
  auto astore = [&]() {
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      const int idx = threadIdx.x + NTH * i;
      if (idx < AV) s_a[idx] = ar[i];
    }
  };
  auto xstore = [&](int grp) {
#pragma unroll
    for (int i = 0; i < XQ_MAX; ++i) {
      const int idx = threadIdx.x + NTH * i;
      if (idx >= xv) continue;
      const int c = idx / (xt.span * 4);
      const int r = (idx >> 2) - c * xt.span, qd = idx & 3;
      f32x4v v = xr[i];
      const int ch = 16 * (CB * grp + c) + 4 * qd;
      if (sx.normalize) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (v[e] - a.mean[ch + e]) / a.scale[ch + e];
      }
      if (sx.slope != 1.f) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * sx.slope;
      }
      if (!xok[i]) v = f32x4v{0.f, 0.f, 0.f, 0.f};
      _Float16 hv[4], lv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hv[e] = (_Float16)v[e];
        lv[e] = (_Float16)(v[e] - (float)hv[e]);
      }
      unsigned char* row = s_x + ((size_t)c * xt.span + r) * XT_ROWB;
      *reinterpret_cast<f16x4v*>(row + 8 * qd) = f16x4v{hv[0], hv[1], hv[2], hv[3]};
      *reinterpret_cast<f16x4v*>(row + 32 + 8 * qd) = f16x4v{lv[0], lv[1], lv[2], lv[3]};
    }
  };
  auto store = [&](int grp) {
    astore();
    xstore(grp);
  };
  // DB: A fragments of taps [t0, t0 + nt) of channel block grp, global -> LDS buffer dst by DMA
  // (1 KB per wave-instruction: 64 lanes x 16 B of one (tap, m, hi|lo) fragment, lane-linear)
  auto dma = [&](int grp, int t0, int nt, f32x4v* dst) {
    typedef __attribute__((address_space(1))) void* gptr_t;
    typedef __attribute__((address_space(3))) void* lptr_t;
    for (int i = wave; i < nt * MT * 2; i += NTH / 64) {
      const int tl = i / (MT * 2), j = i - tl * (MT * 2);
      const int tap = t0 + tl, wt = xt.rev ? K - 1 - tap : tap;
      const float* src = wfrag_ + ((size_t)(wt * xt.cs + grp) * a.mt_total + m0) * 512 + j * 256 + lane * 4;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + (size_t)i * 64), 16, 0, 0);
    }
  };
  // PRE: channel block grp's pre-split rows -> row buffer b
  auto rdma = [&](int grp, int b) {
    typedef __attribute__((address_space(1))) void* gptr_t;
    typedef __attribute__((address_space(3))) void* lptr_t;
    unsigned char* const dst = s_x + (size_t)b * XRP * 64;
    const unsigned char* const src0 = xt.simg + 64 * grp;
#pragma unroll
    for (int k = 0; k < (PRE ? DXI : 0); ++k) {
      const int i = wave + NWV * k;
      if (i >= NXI) break;
      const void* src = pxo[k] >= 0 ? (const void*)(src0 + pxo[k]) : (const void*)g_cn_zero16;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + (size_t)i * 1024), 16, 0, 0);
    }
  };

  // SY: each vector goes global -> LDS on its own (the compiler batches them within 128 VGPRs)
  constexpr int AVS = CB * KS * MT * 128, AQS = (AVS + NTH - 1) / NTH;
  auto stage_sync = [&](int grp, int th) {  // A fragments of taps [th KS, th KS + KS); x rows at th 0
#pragma unroll
    for (int i = 0; i < AQS; ++i) {
      const int idx = threadIdx.x + NTH * i;
      if (idx >= AVS) continue;
      const int c = idx / (KS * MT * 128), rem1 = idx - c * (KS * MT * 128);
      const int tap = th * KS + rem1 / (MT * 128), rem = rem1 - (rem1 / (MT * 128)) * (MT * 128);
      if (tap >= K) continue;
      const int wt = xt.rev ? K - 1 - tap : tap;
      s_a[idx] = reinterpret_cast<const f32x4v*>(wfrag_ + ((size_t)(wt * xt.cs + CB * grp + c) * a.mt_total + m0) * 512)[rem];
    }
    if (th != 0) return;
#pragma unroll
    for (int i = 0; i < XQ_MAX; ++i) {
      const int idx = threadIdx.x + NTH * i;
      if (idx >= xv) continue;
      const int c = idx / (xt.span * 4);
      const int r = (idx >> 2) - c * xt.span, qd = idx & 3;
      int p = q0 + off_min + r;
      const bool ok = edge_row(p, sg.y, sx.pad_mode);
      f32x4v v = *reinterpret_cast<const f32x4v*>(sx.x + (size_t)(sg.x + p) * sx.ld + 16 * (CB * grp + c) + 4 * qd);
      const int ch = 16 * (CB * grp + c) + 4 * qd;
      if (sx.normalize) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (v[e] - a.mean[ch + e]) / a.scale[ch + e];
      }
      if (sx.slope != 1.f) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * sx.slope;
      }
      if (!ok) v = f32x4v{0.f, 0.f, 0.f, 0.f};
      _Float16 hv[4], lv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hv[e] = (_Float16)v[e];
        lv[e] = (_Float16)(v[e] - (float)hv[e]);
      }
      unsigned char* row = s_x + ((size_t)c * xt.span + r) * XT_ROWB;
      *reinterpret_cast<f16x4v*>(row + 8 * qd) = f16x4v{hv[0], hv[1], hv[2], hv[3]};
      *reinterpret_cast<f16x4v*>(row + 32 + 8 * qd) = f16x4v{lv[0], lv[1], lv[2], lv[3]};
    }
  };

  f32x16 acc[NC][MT];
#pragma unroll
  for (int nc = 0; nc < NC; ++nc)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[nc][m][r] = 0.f;

  const int ngrp = xt.cs / CB;
  // taps [T0, T1) of the staged channel blocks (A fragments of tap t at slot t - T0)
  auto mma_taps = [&](auto t0c, auto t1c, const f32x4v* abase) {
    constexpr int T0 = decltype(t0c)::value, T1 = decltype(t1c)::value;
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int tap = T0; tap < T1; ++tap) {
        const u32x4v* sa = reinterpret_cast<const u32x4v*>(abase) + (size_t)(c * KS + tap - T0) * MT * 128 + lane;
        u32x4v bh[NC], bl[NC];
#pragma unroll
        for (int nc = 0; nc < NC; ++nc) {
          if constexpr (PRE) {
            const int R = wave * 32 + cl + tap * xt.dil, sw = (R >> 2) & 3;
            const unsigned char* row = s_xcur + (size_t)R * 64;
            bh[nc] = *reinterpret_cast<const u32x4v*>(row + 16 * (hh ^ sw));
            bl[nc] = *reinterpret_cast<const u32x4v*>(row + 16 * ((2 + hh) ^ sw));
          } else {
            const unsigned char* row =
                s_x + ((size_t)c * xt.span + nc * XC + wave * 32 + cl + tap * xt.dil) * XT_ROWB;
            bh[nc] = *reinterpret_cast<const u32x4v*>(row + 16 * hh);
            bl[nc] = *reinterpret_cast<const u32x4v*>(row + 32 + 16 * hh);
          }
        }
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const u32x4v ah = sa[(m * 2) * 64], al = sa[(m * 2 + 1) * 64];
#pragma unroll
          for (int nc = 0; nc < NC; ++nc) {
            if (nc > 0 && nc >= nc_live) continue;
            f32x16& ac = acc[nc][m];
            ac = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah), __builtin_bit_cast(f16x8v, bh[nc]),
                                                        ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah), __builtin_bit_cast(f16x8v, bl[nc]),
                                                        ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, al), __builtin_bit_cast(f16x8v, bh[nc]),
                                                        ac, 0, 0, 0);
          }
        }
      }
  };
  if constexpr (DB) {
    // tap groups h = 0 .. NH-1 of KS taps ([h KS, min(K, h KS + KS))); global group g = grp NH + h
    // computes from buffer g & 1 while the DMA of group g + 1 fills the other buffer
    constexpr int NH = (K + KS - 1) / KS;
    dma(0, 0, KS, s_a);
    if constexpr (PRE) {
      rdma(0, 0);
    } else {
      xload(0);
      xstore(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int grp = 0; grp < ngrp; ++grp) {
      const bool more = grp + 1 < ngrp;
      if constexpr (PRE) s_xcur = s_x + (size_t)(grp & 1) * XRP * 64;
      auto stage = [&](auto hc) {
        constexpr int h = decltype(hc)::value;
        constexpr int T0 = h * KS, T1 = (h + 1) * KS < K ? (h + 1) * KS : K;
        const int g = grp * NH + h;
        f32x4v* const cur = (g & 1) ? s_a1 : s_a;
        f32x4v* const nxt = (g & 1) ? s_a : s_a1;  // read last by group g - 1, before the barrier
        if constexpr (h + 1 < NH) {
          constexpr int T2 = (h + 2) * KS < K ? (h + 2) * KS : K;
          dma(grp, T1, T2 - T1, nxt);
        } else if (more) {
          dma(grp + 1, 0, KS, nxt);
          if constexpr (PRE) rdma(grp + 1, (grp + 1) & 1);  // (its buffer's last reader: block grp - 1)
          else if constexpr (MT < 4) xload(grp + 1);  // MT 4: after the MFMAs (128 VGPRs hold no prefetch)
        }
        mma_taps(std::integral_constant<int, T0>{}, std::integral_constant<int, T1>{}, cur);
        if constexpr (h + 1 < NH) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
        } else if (more) {
          if constexpr (PRE) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
          } else {
            __syncthreads();  // every wave is done with this block's input rows
            if constexpr (MT >= 4) xload(grp + 1);
            xstore(grp + 1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
          }
        }
      };
      stage(std::integral_constant<int, 0>{});
      if constexpr (NH > 1) stage(std::integral_constant<int, (NH > 1 ? 1 : 0)>{});
      if constexpr (NH > 2) stage(std::integral_constant<int, (NH > 2 ? 2 : 0)>{});
      if constexpr (NH > 3) stage(std::integral_constant<int, (NH > 3 ? 3 : 0)>{});
      static_assert(NH <= 4, "at most four tap groups");
    }
  } else if constexpr (SY) {
    constexpr int NH = (K + KS - 1) / KS;
    stage_sync(0, 0);
    __syncthreads();
    for (int grp = 0; grp < ngrp; ++grp) {
      const bool more = grp + 1 < ngrp;
      mma_taps(std::integral_constant<int, 0>{}, std::integral_constant<int, KS < K ? KS : K>{}, s_a);
      if constexpr (NH > 1) {
        __syncthreads();
        stage_sync(grp, 1);
        __syncthreads();
        mma_taps(std::integral_constant<int, KS>{}, std::integral_constant<int, K>{}, s_a);
      }
      if (!more) break;
      __syncthreads();
      stage_sync(grp + 1, 0);
      __syncthreads();
    }
  } else {
    load(0);
    store(0);
    __syncthreads();
    for (int grp = 0; grp < ngrp; ++grp) {
      const bool more = grp + 1 < ngrp;
      if (more) load(grp + 1);
      __builtin_amdgcn_sched_barrier(0);
      mma_taps(std::integral_constant<int, 0>{}, std::integral_constant<int, K>{}, s_a);
      __builtin_amdgcn_sched_barrier(0);
      if (!more) break;
      __syncthreads();
      store(grp + 1);
      __syncthreads();
    }
  }

  // epilogue (pwg_cnet_conv_kernel's arithmetic)
  const int2 sd = *reinterpret_cast<const int2*>(a.seg_dst + 2 * u);
  const int2 sr = a.res ? *reinterpret_cast<const int2*>(a.seg_res + 2 * u) : make_int2(0, 0);
#pragma unroll
  for (int nc = 0; nc < NC; ++nc) {
    const int qb = q0 + nc * XC + wave * 32 + cl;
    if (qb >= nq) break;
    const int t = qb * a.ostride + ophase_;
    float* yrow = a.y + (size_t)(sd.x + t) * a.ld_dst;
    const float* rrow = a.res ? a.res + (size_t)(sr.x + t) * a.ld_res : nullptr;
    cn_store_col<MT, DB && NWV < 8, (DB || SY || MT > 2 ? 1 : MT)>(a, acc[nc], bias_, m0, hh, yrow, rrow, (long long)(sd.x + t));
  }
}

template <int MT, int K, int CB, int NC = 1, bool SY = false, int KS = K, bool DB = false>
hipError_t xtile_launch_k(dim3 grid, int lds, hipStream_t s, const CnConvArgs& a, const CnXtileArgs& xt) {
  const hipError_t e = allow_lds(reinterpret_cast<const void*>(pwg_cnet_xtile_kernel<MT, K, CB, NC, SY, KS, DB>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((pwg_cnet_xtile_kernel<MT, K, CB, NC, SY, KS, DB>), grid, dim3(512), (size_t)lds, s, a, xt);
  return hipGetLastError();
}
template <int MT>
hipError_t xtile_launch_sync(int k, int ks, dim3 grid, int lds, hipStream_t s, const CnConvArgs& a,
                             const CnXtileArgs& xt) {
  if (ks != k) {  // tap-split staging: k = 11 in steps of 6 taps
    if constexpr (MT == 4)
      if (k == 11 && ks == 6) return xtile_launch_k<MT, 11, 1, 1, true, 6>(grid, lds, s, a, xt);
    return hipErrorInvalidValue;
  }
  switch (k) {
    case 3: return xtile_launch_k<MT, 3, 1, 1, true>(grid, lds, s, a, xt);
    case 5: return xtile_launch_k<MT, 5, 1, 1, true>(grid, lds, s, a, xt);
    case 7: return xtile_launch_k<MT, 7, 1, 1, true>(grid, lds, s, a, xt);
    case 11: return xtile_launch_k<MT, 11, 1, 1, true>(grid, lds, s, a, xt);
    default: return hipErrorInvalidValue;
  }
}
template <int MT, int CB>
hipError_t xtile_launch_mt(int k, dim3 grid, int lds, hipStream_t s, const CnConvArgs& a, const CnXtileArgs& xt) {
  switch (k) {
    case 2: return xtile_launch_k<MT, 2, CB>(grid, lds, s, a, xt);
    case 3: return xtile_launch_k<MT, 3, CB>(grid, lds, s, a, xt);
    case 5: return xtile_launch_k<MT, 5, CB>(grid, lds, s, a, xt);
    case 7: return xtile_launch_k<MT, 7, CB>(grid, lds, s, a, xt);
    case 11: return xtile_launch_k<MT, 11, CB>(grid, lds, s, a, xt);
    default: return hipErrorInvalidValue;
  }
}
// DMA-staged launches: KS = K, or tap groups of ceil(K / NH) for NH = 2..4 at >= 64 rows
template <int MT, int K, int KS>
hipError_t xtile_launch_db_ks(dim3 grid, int lds, hipStream_t s, const CnConvArgs& a, const CnXtileArgs& xt) {
  return xtile_launch_k<MT, K, 1, 1, false, KS, true>(grid, lds, s, a, xt);
}
template <int MT>
hipError_t xtile_launch_db(int k, int ks, dim3 grid, int lds, hipStream_t s, const CnConvArgs& a,
                           const CnXtileArgs& xt) {
  if (ks == k) {
    switch (k) {
      case 2: return xtile_launch_db_ks<MT, 2, 2>(grid, lds, s, a, xt);  // ConvTranspose phases
      case 3: return xtile_launch_db_ks<MT, 3, 3>(grid, lds, s, a, xt);
      case 5: return xtile_launch_db_ks<MT, 5, 5>(grid, lds, s, a, xt);
      case 7: return xtile_launch_db_ks<MT, 7, 7>(grid, lds, s, a, xt);
      case 11: return xtile_launch_db_ks<MT, 11, 11>(grid, lds, s, a, xt);
      default: return hipErrorInvalidValue;
    }
  }
  if constexpr (MT >= 2) {
    if (k == 3 && ks == 2) return xtile_launch_db_ks<MT, 3, 2>(grid, lds, s, a, xt);
    if (k == 5 && ks == 3) return xtile_launch_db_ks<MT, 5, 3>(grid, lds, s, a, xt);
    if (k == 7 && ks == 4) return xtile_launch_db_ks<MT, 7, 4>(grid, lds, s, a, xt);
    if (k == 7 && ks == 3) return xtile_launch_db_ks<MT, 7, 3>(grid, lds, s, a, xt);
    if (k == 11 && ks == 6) return xtile_launch_db_ks<MT, 11, 6>(grid, lds, s, a, xt);
    if (k == 11 && ks == 4) return xtile_launch_db_ks<MT, 11, 4>(grid, lds, s, a, xt);
    if (k == 11 && ks == 3) return xtile_launch_db_ks<MT, 11, 3>(grid, lds, s, a, xt);
  }
  return hipErrorInvalidValue;
}
// the tap-group sizes xtile_launch_db instantiates for kernel size k (ks == k first)
inline int db_ks_options(int k, int mt, int* out) {
  int n = 0;
  out[n++] = k;
  if (mt < 2) return n;
  switch (k) {
    case 3: out[n++] = 2; break;
    case 5: out[n++] = 3; break;
    case 7: out[n++] = 4; out[n++] = 3; break;
    case 11: out[n++] = 6; out[n++] = 4; out[n++] = 3; break;
    default: break;
  }
  return n;
}
hipError_t xtile_launch(int mt, int k, bool sync, int ks, dim3 grid, int lds, hipStream_t s, const CnConvArgs& a,
                        const CnXtileArgs& xt, bool db = false) {
  if (db) {
    switch (mt) {
      case 1: return xtile_launch_db<1>(k, ks, grid, lds, s, a, xt);
      case 2: return xtile_launch_db<2>(k, ks, grid, lds, s, a, xt);
      case 3: return xtile_launch_db<3>(k, ks, grid, lds, s, a, xt);
      case 4: return xtile_launch_db<4>(k, ks, grid, lds, s, a, xt);
      default: return hipErrorInvalidValue;
    }
  }
  if (sync) {
    switch (mt) {
      case 2: return xtile_launch_sync<2>(k, ks, grid, lds, s, a, xt);
      case 3: return xtile_launch_sync<3>(k, ks, grid, lds, s, a, xt);
      case 4: return xtile_launch_sync<4>(k, ks, grid, lds, s, a, xt);
      default: return hipErrorInvalidValue;
    }
  }
  switch (mt) {
    case 1: return xtile_launch_mt<1, 1>(k, grid, lds, s, a, xt);
    case 2: return xtile_launch_mt<2, 1>(k, grid, lds, s, a, xt);
    case 3: return xtile_launch_mt<3, 1>(k, grid, lds, s, a, xt);
    case 4: return xtile_launch_mt<4, 1>(k, grid, lds, s, a, xt);
    default: return hipErrorInvalidValue;
  }
}

// Narrow x-tile launches (PWG_CNET_OPT_NARROW, small plans: the B = 1 decode path of
// bin/decode.py:236-268): NWV waves (32 NWV output columns) and MT m-tiles per workgroup, the A
// fragments DMA-staged in tap groups of narrow_ks(K) taps, so an op whose 8-wave launch would
// occupy a few dozen CUs spreads over all of them. Every column sums the same products in the same
// order as on the 8-wave kernels: bit-identical.
constexpr int narrow_ks(int k) { return k <= 3 ? k : (k == 5 ? 3 : 4); }
template <int MT, int NWV, bool PRE>
hipError_t xtile_launch_narrow_mt(int k, dim3 grid, int lds, hipStream_t s, const CnConvArgs& a, const CnXtileArgs& xt) {
  auto go = [&](auto kfn, int ks) -> hipError_t {
    // PRE: two row buffers of the rounded span (64 B rows) after the two A buffers
    const int l = PRE ? 2 * ks * MT * 2048 + 2 * ((32 * NWV + (k == 2 ? 16 : NARROW_HALO) + 15) / 16 * 16) * 64 : lds;
    const hipError_t e = allow_lds(reinterpret_cast<const void*>(kfn), l);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kfn, grid, dim3(64 * NWV), (size_t)l, s, a, xt);
    return hipGetLastError();
  };
  switch (k) {
    case 2: return go(pwg_cnet_xtile_kernel<MT, 2, 1, 1, false, narrow_ks(2), true, NWV, PRE>, narrow_ks(2));
    case 3: return go(pwg_cnet_xtile_kernel<MT, 3, 1, 1, false, narrow_ks(3), true, NWV, PRE>, narrow_ks(3));
    case 5: return go(pwg_cnet_xtile_kernel<MT, 5, 1, 1, false, narrow_ks(5), true, NWV, PRE>, narrow_ks(5));
    case 7: return go(pwg_cnet_xtile_kernel<MT, 7, 1, 1, false, narrow_ks(7), true, NWV, PRE>, narrow_ks(7));
    case 11: return go(pwg_cnet_xtile_kernel<MT, 11, 1, 1, false, narrow_ks(11), true, NWV, PRE>, narrow_ks(11));
    default: return hipErrorInvalidValue;
  }
}
// pre: the input rows from the source's pre-split image (xt.simg)
hipError_t xtile_launch_narrow(int mt, int nwv, int k, bool pre, dim3 grid, int lds, hipStream_t s, const CnConvArgs& a,
                               const CnXtileArgs& xt) {
  if (pre) {
    if (mt == 1 && nwv == 1) return xtile_launch_narrow_mt<1, 1, true>(k, grid, lds, s, a, xt);
    if (mt == 1 && nwv == 2) return xtile_launch_narrow_mt<1, 2, true>(k, grid, lds, s, a, xt);
    if (mt == 1 && nwv == 4) return xtile_launch_narrow_mt<1, 4, true>(k, grid, lds, s, a, xt);
    if (mt == 2 && nwv == 1) return xtile_launch_narrow_mt<2, 1, true>(k, grid, lds, s, a, xt);
    if (mt == 2 && nwv == 2) return xtile_launch_narrow_mt<2, 2, true>(k, grid, lds, s, a, xt);
    if (mt == 2 && nwv == 4) return xtile_launch_narrow_mt<2, 4, true>(k, grid, lds, s, a, xt);
    return hipErrorInvalidValue;
  }
  if (mt == 1 && nwv == 1) return xtile_launch_narrow_mt<1, 1, false>(k, grid, lds, s, a, xt);
  if (mt == 1 && nwv == 2) return xtile_launch_narrow_mt<1, 2, false>(k, grid, lds, s, a, xt);
  if (mt == 1 && nwv == 4) return xtile_launch_narrow_mt<1, 4, false>(k, grid, lds, s, a, xt);
  if (mt == 2 && nwv == 1) return xtile_launch_narrow_mt<2, 1, false>(k, grid, lds, s, a, xt);
  if (mt == 2 && nwv == 2) return xtile_launch_narrow_mt<2, 2, false>(k, grid, lds, s, a, xt);
  if (mt == 2 && nwv == 4) return xtile_launch_narrow_mt<2, 4, false>(k, grid, lds, s, a, xt);
  return hipErrorInvalidValue;
}

// Narrow DMA-ring launches (PWG_CNET_OPT_NARROW_DMA, default): the tiles of the narrow launches
// above (NWV waves x 32 columns, MT m-tiles), with every byte a step needs staged by
// global_load_lds into a ring of P slots and the steps issued P - 1 ahead of the MFMAs. A step is
// one 16-channel block with all K taps (x-tile family: K > 1, or ConvTranspose phases, K = 2 rev)
// or one chunk of the tap-major chunk list (K = 1 mode: any op, each chunk at its own row offset and
// source). A slot holds the step's raw input rows (16 rows x 64 B per DMA instruction, edge rows
// clamped) and its A fragments (1 KB per instruction); the raw rows of step g + 1 are pre-activated
// (normalize, LeakyReLU, edge mask) and pair-split LDS -> LDS into one of two row buffers while the
// MFMAs of step g run. At B = 1 a workgroup sums 2-16 steps of a few dozen MFMAs each; the narrow
// x-tile kernel waited out the L2/HBM round trip of every step (~1.2 us each, HiFiGAN's 256-channel
// convs 35-59 us), here it is paid about once per launch.
// Per column the products and their order are those of pwg_cnet_xtile_kernel (channel block, tap,
// hi.hi / hi.lo / lo.hi) or, in K = 1 mode, of pwg_cnet_conv_kernel (chunk order): bit-identical.
struct CnXdmaArgs {
  int dil;        // K > 1: dilation
  int cs;         // K > 1: 16-channel blocks (weight chunk of tap t, block c: t cs + c)
  int n_steps;    // K > 1: cs; K = 1: chunks of the op (pwg_cnet_conv_kernel's list)
  int rev;        // ConvTranspose phases: tap t multiplies weight chunk K-1-t
  int z_off[8];   // K > 1: row offset of tap 0 for phase blockIdx.z
  int probe_slot; // PWG_XDMA_PROBE builds only (timeline of workgroup 0, tools/diag/xdma_probe.py)
  const int2* bfr;  // per block: (first frame, frames) of its utterance
  int rate[2], rate_dst, rate_res;  // rows per frame of the sources', destination and residual buffers
  // Pre-split activation images (PWG_CNET_OPT_PRESPLIT): a buffer's rows as [16-channel block][hi 16
  // f16 | lo 16 f16] (64 B per block, row = channels x 4 B), the consumer's LeakyReLU applied before
  // the pair split. PRE launches DMA their B rows from simg (no per-step conversion); any launch
  // writes n_oimg images of its output rows beside the fp32 store (quad epilogue path).
  const unsigned char* simg[2];
  int simg_rowb[2];
  unsigned char* oimg[2];
  float oslope[2];
  int n_oimg, oimg_rowb;
  int row0[2];    // PRE, K = 1: the row offset every chunk of source s shares, or INT_MIN (1x1s: 0)
  int k1_n0;      // K = 1: n0 >= 0 when the chunk list is [source 0 blocks 0..n0-1][source 1 blocks],
                  // row offset 0 (every 1x1): descriptors by arithmetic, no table; else -1
};

constexpr int XDMA_CHUNKS_MAX = 256;  // K = 1 mode: chunks per op (the table sits in LDS)
#ifndef PWG_XDMA_K1_G
#define PWG_XDMA_K1_G 4
#endif
#ifndef PWG_XDMA_RING_CAP
#define PWG_XDMA_RING_CAP 4
#endif
constexpr int XDMA_K1_G = PWG_XDMA_K1_G;          // K = 1 mode: chunks per step
constexpr int XDMA_RING_CAP = PWG_XDMA_RING_CAP;  // ring slots at most (see XdmaShape::ring)
#ifdef PWG_XDMA_PROBE
constexpr int XDMA_PROBE_SLOTS = 128, XDMA_PROBE_N = 96;
__device__ unsigned long long g_xdma_probe[XDMA_PROBE_SLOTS][XDMA_PROBE_N];
#endif
template <int K, int MT, int NWV, bool PRE = false>
struct XdmaShape {
  static constexpr int XC = 32 * NWV;
  // raw input rows per step: the tile + the taps' reach (ConvTranspose phases, K = 2: one row)
  static constexpr int XR = XC + (K == 1 ? 0 : (K == 2 ? 16 : NARROW_HALO));
  // K = 1 mode stages G chunks per step (each its own source rows), so a step's barrier and DMA
  // round trip cover G chunks' few MFMAs
  static constexpr int G = K == 1 ? XDMA_K1_G : 1;
  static constexpr int KT = K == 1 ? G : K;                    // A fragments (taps / chunks) per step
  // PRE: a step's rows arrive converted, 64 B each (hi 16 f16, lo 16 f16 as four 16-B pieces, piece
  // q of row r at slot q ^ ((r >> 2) & 3): every 16-lane group of a ds_read_b128 of 16 consecutive
  // rows then covers all 16 slots of a bank row, conflict-free, without the 16-B pad). Instruction j
  // of a row block holds rows 16 j .. 16 j + 15, lane l row 16 j + l / 4, slot l & 3.
  static constexpr int CHI = XC / 16;                          // PRE, K = 1: instructions per chunk
  static constexpr int NA = KT * MT * 2;                       // 1-KB DMA instructions per step
  static constexpr int NX = PRE ? (K == 1 ? G * CHI : XR / 16) : G * XR / 16;
  // PRE, K = 1: wave w copies instructions w, w + NWV, .. of every chunk (JW = 2 per chunk):
  // compile-time chunk indices
  static constexpr int JW = (CHI + NWV - 1) / NWV;
  static constexpr int DA = (NA + NWV - 1) / NWV, DX = PRE && K == 1 ? G * JW : (NX + NWV - 1) / NWV;  // ... per wave
  static constexpr int D = DA + DX;
  static constexpr int SLOT = (NX + NA) * 1024;                // rows, then A fragments
  // K > 1: two converted-row buffers (not PRE); K = 1: none (B split in registers) but the chunk table
  static constexpr int CBUF = (K == 1 || PRE) ? 0 : XR * XT_ROWB;
  static constexpr int CHT = K == 1 ? XDMA_CHUNKS_MAX * (int)sizeof(ChunkDesc) : 0;
  // deepest ring (<= XDMA_RING_CAP slots) whose wait counts fit vmcnt (63) and LDS 159 KB
  static constexpr int ring(int p) {
    return p <= 2 ? 2 : (((p - 2) * D <= 63 && p * SLOT + 2 * CBUF + CHT <= 159 * 1024) ? p : ring(p - 1));
  }
  // at most 4 slots: the prologue issues P - 1 steps before the first MFMA, and deeper rings
  // measured slower at B = 1 (MB-MelGAN v2 T' = 64: 16 slots 0.507 ms, 8: 0.508, 4: 0.478;
  // HiFiGAN v1 0.973 / 0.989 / 0.954; profiles/r04_h); 3 slots measured the same as 4 and 2 slots
  // slower (MB-MelGAN 0.442 / 0.441 / 0.491 ms), K = 1 with 2 chunks per step no faster
  // (profiles/r04_p; -DPWG_XDMA_RING_CAP / -DPWG_XDMA_K1_G build those variants)
  static constexpr int P = ring(XDMA_RING_CAP);
  static constexpr int LDS = P * SLOT + 2 * CBUF + CHT;
  static_assert(LDS <= 160 * 1024, "DMA-ring shape");
};
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt vmcnt(BASE + min(r, R) * D)
template <int BASE, int D, int R>
__device__ __forceinline__ void vm_wait_steps(int r) {
  if constexpr (R > 0) {
    if (r >= R) {
      vm_wait<BASE + R * D>();
      return;
    }
    vm_wait_steps<BASE, D, R - 1>(r);
  } else {
    vm_wait<BASE>();
  }
}

template <int K, int MT, int NWV, bool PRE>
__global__ void __launch_bounds__(64 * NWV) pwg_cnet_xdma_kernel(const CnConvArgs a, const CnXdmaArgs xd) {
  using S = XdmaShape<K, MT, NWV, PRE>;
  constexpr int NTH = 64 * NWV, P = S::P;
  constexpr int NQ = (S::XR * 4 + NTH - 1) / NTH;  // raw 16-B quads converted per thread and step
  extern __shared__ __attribute__((aligned(16))) unsigned char xt_smem[];
  unsigned char* const s_cb = xt_smem + (size_t)P * S::SLOT;  // [2][XR][XT_ROWB]
  typedef __attribute__((address_space(1))) void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const TileId tid = xcd_tile(a.xcd_order);
  // The block and its utterance's (first frame, frames): with the buffers' rates that gives every
  // row range and the column count without a dependent second load. Every global value the loop
  // needs is read here, before the first DMA: while an LDS-DMA is outstanding the compiler waits
  // vmcnt(0) at the next use of any ordinary global load (and at __syncthreads()), which would drain
  // the ring (cdna_hip_programming.md, "Pipelining across barriers"); the loop's barriers are raw.
  const int2 blk = a.blocks[tid.x];
  const int2 fr = xd.bfr[tid.x];
  const int q0 = blk.y;
  const int m0 = tid.y * MT;
  const int zp = tid.z;
  const float* const wfrag_ = zp == 0 ? a.wfrag : a.z_wfrag[zp];
  const float* const bias_ = zp == 0 ? a.bias : a.z_bias[zp];
  const ChunkDesc* const chunks_ = zp == 0 ? a.chunks : a.z_chunks[zp];
  const int nch = xd.n_steps;                               // K > 1: channel blocks; K = 1: chunks
  const int ns = K == 1 ? (nch + S::G - 1) / S::G : nch;     // steps
  const int span = K == 1 ? S::XC : S::XC + (K - 1) * xd.dil;
  const int sgx0 = fr.x * xd.rate[0], sgy0 = fr.y * xd.rate[0];
  const int sgx1 = fr.x * xd.rate[1], sgy1 = fr.y * xd.rate[1];
  auto barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  // epilogue operands (bias, residual, y_old) in flight from the start (pwg_cnet_conv_kernel's
  // epilogue arithmetic; quad-aligned destinations, else loaded at the end)
  const int nq = (fr.y * xd.rate_dst - a.ophase + a.ostride - 1) / a.ostride;
  const int qb = q0 + wave * 32 + cl;
  const int t_out = qb * a.ostride + a.ophase + zp;
  float* const yrow = a.y + (size_t)(fr.x * xd.rate_dst + t_out) * a.ld_dst;
  const float* const rrow = a.res ? a.res + (size_t)(fr.x * xd.rate_res + t_out) * a.ld_res : nullptr;
  const bool quad = (a.ld_dst & 3) == 0;
  f32x4v bv[MT][4], rv[MT][4], yv[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      const int row = 32 * (m0 + m) + 8 * j4 + 4 * hh;
      const bool live = quad && qb < nq && row < a.M;
      const f32x4v z = {0.f, 0.f, 0.f, 0.f};
      bv[m][j4] = live ? *reinterpret_cast<const f32x4v*>(bias_ + row) : z;
      rv[m][j4] = live && rrow ? *reinterpret_cast<const f32x4v*>(rrow + row) : z;
      yv[m][j4] = live && a.accumulate ? *reinterpret_cast<const f32x4v*>(yrow + row) : z;
    }

  // K > 1: the rows every step stages are the same (only the channel block moves): per-lane row
  // offsets of this wave's raw-row DMA instructions and the edge mask of its converted quads, once
  const CnSrc& s0 = a.src[0];
  const int off0 = xd.z_off[zp];
  int xoff[S::DX];
  unsigned okm = 0;
  // PRE, K > 1: each lane's 16 B of instruction k is (tile row r, piece q) of the swizzled 64-B rows;
  // the image byte offset of that piece in channel block 0, or -1 (the zero page) for a zero-padded
  // row or one past the span
  long long pxo[PRE && K > 1 ? S::DX : 1];
  int prow[PRE && K == 1 ? S::JW : 1], pq16[PRE && K == 1 ? S::JW : 1];  // PRE, K = 1: (row, piece x 16) per jj
  // ... and, for a source whose chunks share one row offset, each instruction's image byte offset
  // (-1: zero page), once: the per-step issue is then a base + offset per instruction
  long long pk1[2][PRE && K == 1 ? S::JW : 1];
  if constexpr (PRE && K == 1) {
#pragma unroll
    for (int jj = 0; jj < S::JW; ++jj) {
      const int j = wave + NWV * jj < S::CHI ? wave + NWV * jj : S::CHI - 1;
      const int r = 16 * j + (lane >> 2);
      prow[jj] = r;
      pq16[jj] = ((lane & 3) ^ ((r >> 2) & 3)) * 16;
#pragma unroll
      for (int si = 0; si < 2; ++si) {
        int p = q0 + (xd.row0[si] == INT_MIN ? 0 : xd.row0[si]) + prow[jj];
        const bool ok = edge_row(p, si ? sgy1 : sgy0, a.src[si].pad_mode);
        pk1[si][jj] = ok ? (long long)((si ? sgx1 : sgx0) + p) * xd.simg_rowb[si] + pq16[jj] : -1;
      }
    }
  }
  if constexpr (PRE && K > 1) {
#pragma unroll
    for (int k = 0; k < S::DX; ++k) {
      const int i = wave + NWV * k < S::NX ? wave + NWV * k : S::NX - 1;
      const int r = 16 * i + (lane >> 2), q = (lane & 3) ^ ((r >> 2) & 3);
      int p = q0 + off0 + r;
      const bool ok = edge_row(p, sgy0, s0.pad_mode) && r < span;
      pxo[k] = ok ? (long long)(sgx0 + p) * xd.simg_rowb[0] + q * 16 : -1;
    }
  } else if constexpr (K > 1) {
#pragma unroll
    for (int k = 0; k < S::DX; ++k) {
      const int i = wave + NWV * k < S::NX ? wave + NWV * k : S::NX - 1;
      int p = q0 + off0 + 16 * i + (lane >> 2);
      (void)edge_row(p, sgy0, s0.pad_mode);
      xoff[k] = (sgx0 + p) * s0.ld + 4 * (lane & 3);
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int r = (int)(threadIdx.x + NTH * i) >> 2;
      int p = q0 + off0 + r;
      if (r < span && edge_row(p, sgy0, s0.pad_mode)) okm |= 1u << i;
    }
  }

  // K = 1: the op's chunk list, staged in LDS before the first DMA (one ordinary load round trip)
  // (a 1x1's list is arithmetic: no table, so no global round trip and barrier before the first DMA)
  ChunkDesc* const s_ch = reinterpret_cast<ChunkDesc*>(xt_smem + (size_t)P * S::SLOT + 2 * S::CBUF);
  const int k1n0 = xd.k1_n0;
  if constexpr (K == 1) {
    if (k1n0 < 0) {
      for (int c = threadIdx.x; c < nch; c += NTH) s_ch[c] = chunks_[c];
      __syncthreads();
    }
  }
  auto chunk_at = [&](int i) -> ChunkDesc {
    if (k1n0 >= 0) {
      ChunkDesc c;
      c.src = i >= k1n0 ? 1 : 0;
      c.row_off = 0;
      c.c0 = 16 * (i - (c.src ? k1n0 : 0));
      c.pad = 0;
      return c;
    }
    return s_ch[i];
  };
  auto chunk = [&](int s) -> ChunkDesc {
    ChunkDesc c = chunk_at(s);
    c.src = __builtin_amdgcn_readfirstlane(c.src);
    c.row_off = __builtin_amdgcn_readfirstlane(c.row_off);
    c.c0 = __builtin_amdgcn_readfirstlane(c.c0);
    return c;
  };

  // step s -> slot s % P: DA A-fragment then DX raw-row instructions per wave (uniform counts: the
  // last instruction of a kind is repeated by waves past the end, same bytes to the same place), so
  // a wait for a step's rows covers its A fragments too. Addresses: a scalar base + the lane's offset.
  auto issue = [&](int s) {
    unsigned char* const slot = xt_smem + (size_t)(s % P) * S::SLOT;
#pragma unroll
    for (int k = 0; k < S::DA; ++k) {
      const int i = wave + NWV * k < S::NA ? wave + NWV * k : S::NA - 1;
      const int tl = i / (MT * 2), j = i - tl * (MT * 2);
      const int wt = xd.rev ? K - 1 - tl : tl;
      const int chunk = K == 1 ? min(s * S::G + tl, nch - 1) : wt * xd.cs + s;
      const float* src = wfrag_ + ((size_t)chunk * a.mt_total + m0) * 512 + j * 256;
      __builtin_amdgcn_global_load_lds((gptr_t)(src + lane * 4), (lptr_t)(slot + (S::NX + i) * 1024), 16, 0, 0);
    }
    if constexpr (PRE && K > 1) {
      const unsigned char* const xs = xd.simg[0] + 64 * s;
#pragma unroll
      for (int k = 0; k < S::DX; ++k) {
        const int i = wave + NWV * k < S::NX ? wave + NWV * k : S::NX - 1;
        const void* src = pxo[k] >= 0 ? (const void*)(xs + pxo[k]) : (const void*)g_cn_zero16;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(slot + i * 1024), 16, 0, 0);
      }
    } else if constexpr (PRE) {
      // K = 1: chunk t's XC rows are instructions t CHI .. + CHI - 1, each lane's 16 B a (row,
      // piece) of the XT_ROWB-strided rows, read from its source's image at the chunk's channels
      // the step's chunk descriptors: every LDS read first, one wait
      ChunkDesc cdr[S::G];
#pragma unroll
      for (int t = 0; t < S::G; ++t) cdr[t] = chunk_at(min(s * S::G + t, nch - 1));
#pragma unroll
      for (int t = 0; t < S::G; ++t) {
        const int csrc = __builtin_amdgcn_readfirstlane(cdr[t].src);
        const int crow = __builtin_amdgcn_readfirstlane(cdr[t].row_off);
        const int cc0 = __builtin_amdgcn_readfirstlane(cdr[t].c0);
        const bool s1 = csrc != 0;  // (uniform: scalar selects, no indexed source array)
        const unsigned char* const img = (s1 ? xd.simg[1] : xd.simg[0]) + cc0 * 4;
        const bool common = crow == (s1 ? xd.row0[1] : xd.row0[0]);
        const int rowb = s1 ? xd.simg_rowb[1] : xd.simg_rowb[0];
        const int sgx = s1 ? sgx1 : sgx0, sgy = s1 ? sgy1 : sgy0;
        const int pm = s1 ? a.src[1].pad_mode : a.src[0].pad_mode;
#pragma unroll
        for (int jj = 0; jj < S::JW; ++jj) {
          const int j = wave + NWV * jj < S::CHI ? wave + NWV * jj : S::CHI - 1;
          long long off;
          if (common) {
            off = s1 ? pk1[1][jj] : pk1[0][jj];
          } else {
            int p = q0 + crow + prow[jj];
            off = edge_row(p, sgy, pm) ? (long long)(sgx + p) * rowb + pq16[jj] : -1;
          }
          const void* src = off >= 0 ? (const void*)(img + off) : (const void*)g_cn_zero16;
          __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(slot + (t * S::CHI + j) * 1024), 16, 0, 0);
        }
      }
    } else if constexpr (K > 1) {
      const float* const xs = s0.x + 16 * s;
#pragma unroll
      for (int k = 0; k < S::DX; ++k) {
        const int i = wave + NWV * k < S::NX ? wave + NWV * k : S::NX - 1;
        __builtin_amdgcn_global_load_lds((gptr_t)(xs + xoff[k]), (lptr_t)(slot + i * 1024), 16, 0, 0);
      }
    } else {
      // a chunk's XC rows are 2 NWV instructions: wave w's k-th is chunk k / 2, row group
      // w + NWV (k & 1) (DX = 2 G, no clamping); the step's chunk descriptors are read once
      static_assert(S::DX == 2 * S::G && S::NX == 2 * NWV * S::G, "K = 1 DMA layout");
      ChunkDesc cds[S::G];
#pragma unroll
      for (int t = 0; t < S::G; ++t) cds[t] = chunk(min(s * S::G + t, nch - 1));
#pragma unroll
      for (int k = 0; k < S::DX; ++k) {
        const int t = k >> 1, ii = wave + NWV * (k & 1);
        const int i = t * 2 * NWV + ii;
        const ChunkDesc& cd = cds[t];
        const CnSrc& sx = a.src[cd.src];
        const int sgx = cd.src ? sgx1 : sgx0, sgy = cd.src ? sgy1 : sgy0;
        int p = q0 + cd.row_off + 16 * ii + (lane >> 2);
        (void)edge_row(p, sgy, sx.pad_mode);
        const float* src = sx.x + (size_t)(sgx + p) * sx.ld + cd.c0 + 4 * (lane & 3);
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(slot + i * 1024), 16, 0, 0);
      }
    }
  };
  // raw rows of step s -> converted-row buffer s & 1 (pwg_cnet_xtile_kernel's xstore arithmetic):
  // every read first, then the stores (they may alias the reads for the compiler)
  auto convert = [&](int s) {
    const unsigned char* const raw = xt_smem + (size_t)(s % P) * S::SLOT;
    unsigned char* const cb = s_cb + (size_t)(s & 1) * S::CBUF;
    const float slope = s0.slope;
    const unsigned ok = okm;
    f32x4v v[NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int idx = threadIdx.x + NTH * i;
      v[i] = (idx >> 2) < span ? *reinterpret_cast<const f32x4v*>(raw + (idx >> 2) * 64 + (idx & 3) * 16)
                               : f32x4v{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int idx = threadIdx.x + NTH * i;
      const int r = idx >> 2, qd = idx & 3;
      if (r >= span) continue;
      f32x4v x = v[i];
      // (no normalize: ops that normalize their input run the narrow x-tile kernel)
      if (slope != 1.f) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = x[e] > 0.f ? x[e] : x[e] * slope;
      }
      if (!((ok >> i) & 1u)) x = f32x4v{0.f, 0.f, 0.f, 0.f};
      _Float16 hv[4], lv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hv[e] = (_Float16)x[e];
        lv[e] = (_Float16)(x[e] - (float)hv[e]);
      }
      unsigned char* row = cb + (size_t)r * XT_ROWB;
      *reinterpret_cast<f16x4v*>(row + 8 * qd) = f16x4v{hv[0], hv[1], hv[2], hv[3]};
      *reinterpret_cast<f16x4v*>(row + 32 + 8 * qd) = f16x4v{lv[0], lv[1], lv[2], lv[3]};
    }
  };

  f32x16 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
  // one step's MFMAs: every operand read first, then the MFMAs in pwg_cnet_xtile_kernel's order
  auto mma = [&](int g) {
    const unsigned char* const cb = s_cb + (size_t)(g & 1) * S::CBUF;
    const u32x4v* const sa =
        reinterpret_cast<const u32x4v*>(xt_smem + (size_t)(g % P) * S::SLOT + S::NX * 1024) + lane;
    constexpr int KT = S::KT;
    u32x4v bh[KT], bl[KT], ah[KT][MT], al[KT][MT];
    ChunkDesc cds[S::G];
    if constexpr (K == 1 && !PRE) {
#pragma unroll
      for (int t = 0; t < S::G; ++t) cds[t] = chunk(min(g * S::G + t, nch - 1));
    }
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      if constexpr (PRE) {
        // converted rows straight from the step's slot (K = 1: chunk t's rows; K > 1: tap t's row),
        // pieces hh (hi) and 2 + hh (lo) at their swizzled slots
        const int R = K == 1 ? wave * 32 + cl : wave * 32 + cl + t * xd.dil;
        const int sw = (R >> 2) & 3;
        const unsigned char* row = xt_smem + (size_t)(g % P) * S::SLOT + (K == 1 ? t * S::CHI * 1024 : 0) + R * 64;
        bh[t] = *reinterpret_cast<const u32x4v*>(row + 16 * (hh ^ sw));
        bl[t] = *reinterpret_cast<const u32x4v*>(row + 16 * ((2 + hh) ^ sw));
      } else if constexpr (K == 1) {
        // chunk g G + t: the lane's 8 channels of its raw row, pre-activated and pair-split in
        // registers (pwg_cnet_conv_kernel's bprep + cn_split8)
        const ChunkDesc& cd = cds[t];
        const CnSrc& sx = a.src[cd.src];
        const int r = wave * 32 + cl;
        int p = q0 + cd.row_off + r;
        const bool okr = edge_row(p, cd.src ? sgy1 : sgy0, sx.pad_mode);
        const unsigned char* const raw = xt_smem + (size_t)(g % P) * S::SLOT + (t * S::XC + r) * 64 + 32 * hh;
        const f32x4v v0 = *reinterpret_cast<const f32x4v*>(raw), v1 = *reinterpret_cast<const f32x4v*>(raw + 16);
        f32x8v x = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        if (sx.slope != 1.f) {
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = x[e] > 0.f ? x[e] : x[e] * sx.slope;
        }
        if (!okr) x = f32x8v{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        cn_split8(x, bh[t], bl[t]);
      } else {
        const unsigned char* row = cb + (size_t)(wave * 32 + cl + t * xd.dil) * XT_ROWB;
        bh[t] = *reinterpret_cast<const u32x4v*>(row + 16 * hh);
        bl[t] = *reinterpret_cast<const u32x4v*>(row + 32 + 16 * hh);
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        ah[t][m] = sa[(t * MT * 2 + m * 2) * 64];
        al[t][m] = sa[(t * MT * 2 + m * 2 + 1) * 64];
      }
    }
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      if (K == 1 && g * S::G + t >= nch) break;  // the last step's missing chunks: no products
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah[t][m]),
                                                        __builtin_bit_cast(f16x8v, bh[t]), acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah[t][m]),
                                                        __builtin_bit_cast(f16x8v, bl[t]), acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, al[t][m]),
                                                        __builtin_bit_cast(f16x8v, bh[t]), acc[m], 0, 0, 0);
      }
    }
  };

#ifdef PWG_XDMA_PROBE
  // shader-clock stamps of workgroup (0, 0, 0), wave 0, kept in the LDS tail (no stores in flight)
  unsigned long long* const s_probe = reinterpret_cast<unsigned long long*>(xt_smem + S::LDS);
  const bool probe = xd.probe_slot >= 0 && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0;
  int np = 0;
  auto stamp = [&] {
    if (probe && np < XDMA_PROBE_N - 1) s_probe[np++] = __builtin_readcyclecounter();
  };
#else
  auto stamp = [] {};
#endif
  stamp();
  // steps 0 .. P-2 in flight; wait for step 0 (the later steps may still land)
  for (int s = 0; s < P - 1; ++s)
    if (s < ns) issue(s);
  stamp();
  if constexpr (K == 1 || PRE) {
    stamp();  // (probe builds: keep the K > 1 timeline's column layout)
    stamp();
    // one barrier per step: after it every wave is done with step g - 1's slot, which the issue of
    // step g + P - 1 refills
    for (int g = 0; g < ns; ++g) {
      vm_wait_steps<0, S::D, P - 2>(ns - 1 - g);
      barrier();
      stamp();
      if (g + P - 1 < ns) issue(g + P - 1);
      stamp();
      mma(g);
      stamp();
      stamp();
    }
  } else {
  vm_wait_steps<0, S::D, P - 2>(ns - 1);
  barrier();
  stamp();
  convert(0);
  barrier();
  stamp();
  for (int g = 0; g < ns; ++g) {
    // slot (g - 1) % P: read by step g - 1's MFMAs and conversion, both before the last barrier
    if (g + P - 1 < ns) issue(g + P - 1);
    stamp();
    // step g + 1 landed (step g did before the last barrier)
    if (g + 1 < ns) {
      vm_wait_steps<0, S::D, P - 2>(ns - 2 - g);
      barrier();
    }
    stamp();
    mma(g);
    stamp();
    if (g + 1 < ns) convert(g + 1);  // into the buffer step g - 1's MFMAs read
    barrier();
    stamp();
  }
  }

  // epilogue
  if (qb < nq) {
    if (quad) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const int row = 32 * (m0 + m) + 8 * j4 + 4 * hh;
          if (row >= a.M) {
            if (row < a.ld_dst) *reinterpret_cast<f32x4v*>(yrow + row) = f32x4v{0.f, 0.f, 0.f, 0.f};
            continue;
          }
          f32x4v v;
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = acc[m][4 * j4 + i] + bv[m][j4][i];
          if (rrow) v += rv[m][j4];
          if (a.accumulate) v = yv[m][j4] + v;
          if (a.out_div != 1.f) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = v[i] / a.out_div;
          }
          if (a.post_act == PWG_ACT_LRELU) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = v[i] > 0.f ? v[i] : v[i] * a.post_slope;
          } else if (a.post_act == PWG_ACT_TANH) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = tanhf(v[i]);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (row + i >= a.M) v[i] = 0.f;
          *reinterpret_cast<f32x4v*>(yrow + row) = v;
          // pre-split images of these 4 channels for the consumers (the conversion those consumers'
          // own staging would apply to the stored values: bit-identical)
          const float vv[4] = {v[0], v[1], v[2], v[3]};
          for (int j = 0; j < xd.n_oimg; ++j)
            cn_img4(xd.oimg[j], (long long)(fr.x * xd.rate_dst + t_out), xd.oimg_rowb, row, vv, xd.oslope[j]);
        }
    } else {
      cn_store_col<MT>(a, acc, bias_, m0, hh, yrow, rrow);
    }
  }
#ifdef PWG_XDMA_PROBE
  if (probe) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp();
    unsigned long long* dst = g_xdma_probe[xd.probe_slot % XDMA_PROBE_SLOTS];
    dst[0] = (unsigned long long)np | ((unsigned long long)K << 16) | ((unsigned long long)MT << 24) |
             ((unsigned long long)NWV << 32) | ((unsigned long long)ns << 40) | ((unsigned long long)P << 56);
    for (int i = 0; i < np; ++i) dst[1 + i] = s_probe[i];
  }
#endif
}

template <int K, int MT, int NWV, bool PRE>
hipError_t xdma_go(dim3 grid, hipStream_t s, const CnConvArgs& a, const CnXdmaArgs& xd) {
#ifdef PWG_XDMA_PROBE
  constexpr int lds = XdmaShape<K, MT, NWV, PRE>::LDS + XDMA_PROBE_N * 8;
#else
  constexpr int lds = XdmaShape<K, MT, NWV, PRE>::LDS;
#endif
  const hipError_t e = allow_lds(reinterpret_cast<const void*>(pwg_cnet_xdma_kernel<K, MT, NWV, PRE>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((pwg_cnet_xdma_kernel<K, MT, NWV, PRE>), grid, dim3(64 * NWV), (size_t)lds, s, a, xd);
  return hipGetLastError();
}
template <int NWV, bool PRE>
hipError_t xdma_launch_k(int k, dim3 grid, hipStream_t s, const CnConvArgs& a, const CnXdmaArgs& xd) {
  switch (k) {
    case 1: return xdma_go<1, 1, NWV, PRE>(grid, s, a, xd);
    case 2: return xdma_go<2, 1, NWV, PRE>(grid, s, a, xd);
    case 3: return xdma_go<3, 1, NWV, PRE>(grid, s, a, xd);
    case 5: return xdma_go<5, 1, NWV, PRE>(grid, s, a, xd);
    case 7: return xdma_go<7, 1, NWV, PRE>(grid, s, a, xd);
    case 11: return xdma_go<11, 1, NWV, PRE>(grid, s, a, xd);
    default: return hipErrorInvalidValue;
  }
}
// k = 1: K = 1 mode (steps = the tap-major chunk list); pre: B rows from the sources' pre-split
// images (xd.simg). One m-tile per workgroup (the plan's only DMA-ring form)
hipError_t xdma_launch(int mt, int nwv, int k, bool pre, dim3 grid, hipStream_t s, const CnConvArgs& a,
                       const CnXdmaArgs& xd) {
  if (mt != 1) return hipErrorInvalidValue;
  if (pre) {
    if (nwv == 1) return xdma_launch_k<1, true>(k, grid, s, a, xd);
    if (nwv == 2) return xdma_launch_k<2, true>(k, grid, s, a, xd);
    if (nwv == 4) return xdma_launch_k<4, true>(k, grid, s, a, xd);
  } else {
    if (nwv == 1) return xdma_launch_k<1, false>(k, grid, s, a, xd);
    if (nwv == 2) return xdma_launch_k<2, false>(k, grid, s, a, xd);
    if (nwv == 4) return xdma_launch_k<4, false>(k, grid, s, a, xd);
  }
  return hipErrorInvalidValue;
}

// Fused conv pair on the x-tile scheme (split-f16; HiFiGAN ResBlock step x = c2(lrelu(c1(lrelu(x)))) + x,
// layers/residual_block.py:231-237, 32 or 64 channels, 128 at k = 3): one workgroup = 8 waves, 224 output columns.
//   stage 1: h over the 256 columns [q0 - 16, q0 + 240) (wave w: 32 of them), channel-block-major
//            exactly as pwg_cnet_xtile_kernel runs conv 1 (A fragments of all taps of a 16-channel
//            block + the block's pre-activated, pair-split input rows staged once per block);
//   h + b1, conv 2's LeakyReLU, zero outside the utterance (conv 2's zero padding), pair split ->
//            an LDS tile [256 rows][hi C | lo C | 16 B];
//   stage 2: waves 0..6 compute the 7 output tiles from the h tile (conv 2's taps reach within
//            +-16 columns), channel-block-major as the x-tile kernel runs conv 2; conv 2's
//            epilogue (+ b2 + residual [+ y_old] [/ div]).
// Same arithmetic and order as two pwg_cnet_xtile_kernel launches: bit-identical to them. h never
// leaves the chip: per pair x is read once (+ the L2-hot residual rows), y written once.
struct CnXpairArgs {
  int K1, dil1, off1;     // conv 1 taps, dilation, first tap's row offset (-pad)
  int K2, off2;           // conv 2 taps (dilation 1), first tap's offset
  int cs;                 // 16-channel blocks (C / 16)
  int span1;              // conv-1 input rows per block: 256 + (K1-1) dil1
  float slope_h;          // conv 2's pre-activation
  const float* w2;        // conv 2 split fragments [tap * cs + cb][MT][hi/lo][lane][4 dwords]
  const float* b2;
};
constexpr int XP_OUT = 224;   // output columns per workgroup (7 tiles; h covers 8)

template <int MT, int K1, int K2>
__global__ void __launch_bounds__(512) pwg_cnet_xpair_kernel(const CnConvArgs a, const CnXpairArgs xp) {
  constexpr int NTH = 512;
  constexpr int C = 32 * MT;
  constexpr int HROWB = 4 * C + 16;                     // h tile row: hi C halves | lo C halves | pad
  constexpr int AV1 = K1 * MT * 128, AQ1 = (AV1 + NTH - 1) / NTH;
  constexpr int AV2 = K2 * MT * 128, AQ2 = (AV2 + NTH - 1) / NTH;
  constexpr int AQ = AQ1 > AQ2 ? AQ1 : AQ2;
  constexpr int XQ_MAX = ((XT_COLS + 192) * 4 + NTH - 1) / NTH;
  extern __shared__ __attribute__((aligned(16))) unsigned char xp_smem[];
  f32x4v* s_a = reinterpret_cast<f32x4v*>(xp_smem);                                   // A of one block
  unsigned char* s_x = xp_smem + (size_t)(K1 > K2 ? K1 : K2) * MT * 2048;              // [span1][80 B]
  // [256][HROWB]: after stage 1, over the input rows (dead by then)
  unsigned char* s_h = s_x;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const int2 blk = a.blocks[blockIdx.x];
  const int u = blk.x;
  const int q0 = blk.y;                 // first output column
  const int h0 = q0 - 16;               // first h column
  const int nq = a.ncols[u];
  const CnSrc& sx = a.src[0];
  const int2 sg = *reinterpret_cast<const int2*>(sx.seg + 2 * u);
  const int xv = xp.span1 * 4;

  f32x4v ar[AQ];
  f32x4v xr[XQ_MAX];
  bool xok[XQ_MAX];
  auto aload = [&](const float* w, int K, int cb) {
    const int av = K * MT * 128;
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      const int idx = threadIdx.x + NTH * i;  // [tap][m][128 vectors]
      const int tap = idx / (MT * 128), rem = idx - tap * (MT * 128);
      ar[i] = idx < av ? reinterpret_cast<const f32x4v*>(w + ((size_t)(tap * xp.cs + cb) * MT) * 512)[rem]
                       : f32x4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto astore = [&](int K) {
    const int av = K * MT * 128;
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      const int idx = threadIdx.x + NTH * i;
      if (idx < av) s_a[idx] = ar[i];
    }
  };
  auto xload = [&](int cb) {
#pragma unroll
    for (int i = 0; i < XQ_MAX; ++i) {
      const int idx = threadIdx.x + NTH * i;
      const bool in = idx < xv;
      const int r = in ? idx >> 2 : 0, qd = idx & 3;
      int p = h0 + xp.off1 + r;
      xok[i] = edge_row(p, sg.y, sx.pad_mode) && in;
      xr[i] = in ? *reinterpret_cast<const f32x4v*>(sx.x + (size_t)(sg.x + p) * sx.ld + 16 * cb + 4 * qd)
                 : f32x4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto xstore = [&](int cb) {
#pragma unroll
    for (int i = 0; i < XQ_MAX; ++i) {
      const int idx = threadIdx.x + NTH * i;
      if (idx >= xv) continue;
      const int r = idx >> 2, qd = idx & 3;
      f32x4v v = xr[i];
      const int ch = 16 * cb + 4 * qd;
      if (sx.normalize) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (v[e] - a.mean[ch + e]) / a.scale[ch + e];
      }
      if (sx.slope != 1.f) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * sx.slope;
      }
      if (!xok[i]) v = f32x4v{0.f, 0.f, 0.f, 0.f};
      _Float16 hv[4], lv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hv[e] = (_Float16)v[e];
        lv[e] = (_Float16)(v[e] - (float)hv[e]);
      }
      unsigned char* row = s_x + (size_t)r * XT_ROWB;
      *reinterpret_cast<f16x4v*>(row + 8 * qd) = f16x4v{hv[0], hv[1], hv[2], hv[3]};
      *reinterpret_cast<f16x4v*>(row + 32 + 8 * qd) = f16x4v{lv[0], lv[1], lv[2], lv[3]};
    }
  };
  f32x16 acc[MT];
  auto mma3 = [&](int m, const u32x4v ah, const u32x4v al, const u32x4v bh, const u32x4v bl) {
    acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah), __builtin_bit_cast(f16x8v, bh),
                                                    acc[m], 0, 0, 0);
    acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah), __builtin_bit_cast(f16x8v, bl),
                                                    acc[m], 0, 0, 0);
    acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, al), __builtin_bit_cast(f16x8v, bh),
                                                    acc[m], 0, 0, 0);
  };

  // ---- stage 1: h (conv 1) for h columns h0 + 32 wave + cl
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
  aload(a.wfrag, K1, 0);
  xload(0);
  astore(K1);
  xstore(0);
  __syncthreads();
  for (int cb = 0; cb < xp.cs; ++cb) {
    const bool more = cb + 1 < xp.cs;
    if (more) {
      aload(a.wfrag, K1, cb + 1);
      xload(cb + 1);
    } else {
      aload(xp.w2, K2, 0);  // stage 2's first block, in flight during the last stage-1 block
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int tap = 0; tap < K1; ++tap) {
      const unsigned char* row = s_x + (size_t)(wave * 32 + cl + tap * xp.dil1) * XT_ROWB;
      const u32x4v bh = *reinterpret_cast<const u32x4v*>(row + 16 * hh);
      const u32x4v bl = *reinterpret_cast<const u32x4v*>(row + 32 + 16 * hh);
      const u32x4v* sa = reinterpret_cast<const u32x4v*>(s_a) + (size_t)tap * MT * 128 + lane;
#pragma unroll
      for (int m = 0; m < MT; ++m) mma3(m, sa[(m * 2) * 64], sa[(m * 2 + 1) * 64], bh, bl);
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    if (more) {
      astore(K1);
      xstore(cb + 1);
      __syncthreads();
    }
  }
  // h + b1, conv 2's LeakyReLU, zero outside the utterance, pair split -> h tile row (wave 32 + cl)
  {
    const int hcol = h0 + wave * 32 + cl;
    const bool inside = hcol >= 0 && hcol < nq;
    unsigned char* hrow = s_h + (size_t)(wave * 32 + cl) * HROWB;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const int row = 32 * m + 8 * j4 + 4 * hh;
        const f32x4v b = *reinterpret_cast<const f32x4v*>(a.bias + row);
        _Float16 hv[4], lv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = acc[m][4 * j4 + i] + b[i];
          v = v > 0.f ? v : v * xp.slope_h;
          v = inside ? v : 0.f;
          hv[i] = (_Float16)v;
          lv[i] = (_Float16)(v - (float)hv[i]);
        }
        *reinterpret_cast<f16x4v*>(hrow + 2 * row) = f16x4v{hv[0], hv[1], hv[2], hv[3]};
        *reinterpret_cast<f16x4v*>(hrow + 2 * C + 2 * row) = f16x4v{lv[0], lv[1], lv[2], lv[3]};
      }
  }
  astore(K2);
  __syncthreads();

  // ---- stage 2: output tile wave (columns q0 + 32 wave + cl), waves 0..6
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
  for (int cb = 0; cb < xp.cs; ++cb) {
    const bool more = cb + 1 < xp.cs;
    if (more) aload(xp.w2, K2, cb + 1);
    __builtin_amdgcn_sched_barrier(0);
    if (wave < XP_OUT / 32) {
#pragma unroll
      for (int tap = 0; tap < K2; ++tap) {
        // output column q0 + 32 wave + cl reads h column + off2 + tap = h row 16 + 32 wave + cl + off2 + tap
        const unsigned char* hrow = s_h + (size_t)(16 + wave * 32 + cl + xp.off2 + tap) * HROWB;
        const u32x4v bh = *reinterpret_cast<const u32x4v*>(hrow + 2 * (16 * cb + 8 * hh));
        const u32x4v bl = *reinterpret_cast<const u32x4v*>(hrow + 2 * C + 2 * (16 * cb + 8 * hh));
        const u32x4v* sa = reinterpret_cast<const u32x4v*>(s_a) + (size_t)tap * MT * 128 + lane;
#pragma unroll
        for (int m = 0; m < MT; ++m) mma3(m, sa[(m * 2) * 64], sa[(m * 2 + 1) * 64], bh, bl);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (!more) break;
    __syncthreads();
    astore(K2);
    __syncthreads();
  }

  // ---- conv 2's epilogue (pwg_cnet_conv_kernel's)
  const int qb = q0 + wave * 32 + cl;
  if (wave >= XP_OUT / 32 || qb >= nq || qb >= q0 + XP_OUT) return;
  const int2 sd = *reinterpret_cast<const int2*>(a.seg_dst + 2 * u);
  const int2 sr = a.res ? *reinterpret_cast<const int2*>(a.seg_res + 2 * u) : make_int2(0, 0);
  const bool quad = (a.ld_dst & 3) == 0;
  float* yrow = a.y + (size_t)(sd.x + qb) * a.ld_dst;
  const float* rrow = a.res ? a.res + (size_t)(sr.x + qb) * a.ld_res : nullptr;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      const int row = 32 * m + 8 * j4 + 4 * hh;
      if (row >= a.M) {
        if (quad && row < a.ld_dst) *reinterpret_cast<f32x4v*>(yrow + row) = f32x4v{0.f, 0.f, 0.f, 0.f};
        continue;
      }
      const f32x4v b = *reinterpret_cast<const f32x4v*>(xp.b2 + row);
      f32x4v v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[m][4 * j4 + i] + b[i];
      if (quad) {
        if (rrow) v += *reinterpret_cast<const f32x4v*>(rrow + row);
        if (a.accumulate) v = *reinterpret_cast<const f32x4v*>(yrow + row) + v;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (row + i >= a.M) continue;
          if (rrow) v[i] += rrow[row + i];
          if (a.accumulate) v[i] = yrow[row + i] + v[i];
        }
      }
      if (a.out_div != 1.f) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] / a.out_div;
      }
      if (a.post_act == PWG_ACT_LRELU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] > 0.f ? v[i] : v[i] * a.post_slope;
      } else if (a.post_act == PWG_ACT_TANH) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = tanhf(v[i]);
      }
      if (quad) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (row + i >= a.M) v[i] = 0.f;
        *reinterpret_cast<f32x4v*>(yrow + row) = v;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (row + i < a.M) yrow[row + i] = v[i];
      }
    }
}

template <int MT, int K1, int K2>
hipError_t xpair_launch_k(dim3 grid, int lds, hipStream_t s, const CnConvArgs& a, const CnXpairArgs& xp) {
  const hipError_t e = allow_lds(reinterpret_cast<const void*>(pwg_cnet_xpair_kernel<MT, K1, K2>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((pwg_cnet_xpair_kernel<MT, K1, K2>), grid, dim3(512), (size_t)lds, s, a, xp);
  return hipGetLastError();
}
template <int MT>
hipError_t xpair_launch_mt(int k, dim3 grid, int lds, hipStream_t s, const CnConvArgs& a, const CnXpairArgs& xp) {
  switch (k) {  // HiFiGAN ResBlocks: conv 1 and conv 2 share the kernel size
    case 3: return xpair_launch_k<MT, 3, 3>(grid, lds, s, a, xp);
    case 5: return xpair_launch_k<MT, 5, 5>(grid, lds, s, a, xp);
    case 7: return xpair_launch_k<MT, 7, 7>(grid, lds, s, a, xp);
    case 11: return xpair_launch_k<MT, 11, 11>(grid, lds, s, a, xp);
    default: return hipErrorInvalidValue;
  }
}
hipError_t xpair_launch(int mt, int k, dim3 grid, int lds, hipStream_t s, const CnConvArgs& a, const CnXpairArgs& xp) {
  if (mt == 1) return xpair_launch_mt<1>(k, grid, lds, s, a, xp);
  if (mt == 2) return xpair_launch_mt<2>(k, grid, lds, s, a, xp);
  // 128 channels: only k = 3 fits (A of one block 24 KB + the h tile 256 x 528 B = 159.7 KB)
  if (mt == 4 && k == 3) return xpair_launch_k<4, 3, 3>(grid, lds, s, a, xp);
  return hipErrorInvalidValue;
}
__host__ __device__ constexpr int xpair_lds(int mt, int k, int span1) {
  return k * mt * 2048 + (span1 * XT_ROWB > 256 * (4 * 32 * mt + 16) ? span1 * XT_ROWB : 256 * (4 * 32 * mt + 16));
}

// Fused MelGAN ResidualStack (split-f16 mode; layers/residual_stack.py:75-85 stack(c) + skip_layer(c)):
// op A  h = conv_k(pre_A(x)) + b1             (dilated, zero / reflection / replication edges)
// op B  y = post(W2 pre_B(h) + W3 x + b2 + b3 [+ res] [+ y_old]) / div   (the two-source 1x1)
// as ONE launch in which h never leaves the chip. Workgroup = 4 waves x 32 columns (one 128-column
// block of one utterance), every output row (MT m-tiles of 32 cover all C channels):
//   * stage 1: op A's chunks exactly as pwg_cnet_conv_kernel runs them (A fragments staged in LDS,
//     double-buffered; B rows from HBM one chunk ahead, pre-activated and pair-split);
//   * h + b1, op B's pre-activation and the fp16 pair split go to a wave-private LDS tile
//     [32 columns][C + 8 halves] (hi and lo images);
//   * stage 2: op B's chunks in its own order (h chunks read from LDS, x chunks from HBM / L2 again,
//     raw), then op B's epilogue.
// Chunk order, pair split, fp32 accumulation and epilogue order are the two unfused ops' exactly:
// the result is bit-identical to running op A then op B in split mode. HBM traffic per stack: x read
// once (+ its L2-hot center re-read) and y written, instead of x, h written, h and x read, y written.
struct CnStackArgs {
  CnSrc x1;               // op A's source (its taps come from the chunk list)
  CnSrc x2;               // op B's second source: the same buffer, op B's pre-activation
  const ChunkDesc* ch1;
  int n1;
  const float* w1;        // split-f16 fragments [chunk][MT][hi/lo][lane][4 dwords]
  const float* b1;
  float slope_h;          // op B's pre-activation of h
  int ldh;                // h channels (C rounded up to 16)
  const ChunkDesc* ch2;   // op B: src 0 chunks (h) then src 1 chunks (x)
  int n2;
  const float* w2;
  const float* b2;        // both biases of op B, summed host-side
  const float* res;
  const int* seg_res;
  int ld_res;
  float* y;
  const int* seg_y;
  int ld_y;
  int M;                  // op B's output channels
  int accumulate;
  float out_div;
  int post_act;
  float post_slope;
  const int2* blocks;     // (utt, q0)
  const int* ncols;
  const float* mean;
  const float* scale;
};

template <int MT>
__global__ void __launch_bounds__(256) pwg_cnet_stack_kernel(const CnStackArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char st_smem[];
  float* s_a = reinterpret_cast<float*>(st_smem);                      // [2][MT * 512] A staging
  const int hrow = a.ldh + 8;                                          // halves per h column (+16 B pad)
  _Float16* s_h = reinterpret_cast<_Float16*>(st_smem + 2 * MT * 512 * sizeof(float));
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const int2 blk = a.blocks[blockIdx.x];
  const int u = blk.x;
  const int qb = blk.y + wave * 32 + cl;
  const int nq = a.ncols[u];
  _Float16* h_hi = s_h + (size_t)(wave * 32 + cl) * 2 * hrow;          // this lane's column: [hi][lo]
  _Float16* h_lo = h_hi + hrow;

  // B row of chunk cd from source s (column qb + row_off), raw: loaded one chunk ahead
  auto braw = [&](const CnSrc& s, const ChunkDesc& cd, f32x8v& v, bool& ok) {
    const int2 sg = *reinterpret_cast<const int2*>(s.seg + 2 * u);
    int p = qb + cd.row_off;
    ok = edge_row(p, sg.y, s.pad_mode);
    v = *reinterpret_cast<const f32x8v*>(s.x + (size_t)(sg.x + p) * s.ld + cd.c0 + 8 * hh);
  };
  auto bprep = [&](const CnSrc& s, const ChunkDesc& cd, f32x8v x, bool ok, u32x4v& bh, u32x4v& bl) {
    const int ch = cd.c0 + 8 * hh;
    if (s.normalize) {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = (x[i] - a.mean[ch + i]) / a.scale[ch + i];
    }
    if (s.slope != 1.f) {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = x[i] > 0.f ? x[i] : x[i] * s.slope;
    }
    if (!ok) x = f32x8v{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    cn_split8(x, bh, bl);
  };
  auto aload = [&](const float* w, int c, f32x4v (&r)[(MT + 1) / 2]) {
    const f32x4v* gp = reinterpret_cast<const f32x4v*>(w + (size_t)c * MT * 512);
#pragma unroll
    for (int i = 0; i < (MT + 1) / 2; ++i) {
      const int idx = threadIdx.x + 256 * i;
      r[i] = idx < MT * 128 ? gp[idx] : f32x4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto astore = [&](int buf, const f32x4v (&r)[(MT + 1) / 2]) {
    f32x4v* d = reinterpret_cast<f32x4v*>(s_a + buf * MT * 512);
#pragma unroll
    for (int i = 0; i < (MT + 1) / 2; ++i) {
      const int idx = threadIdx.x + 256 * i;
      if (idx < MT * 128) d[idx] = r[i];
    }
  };
  f32x16 acc[MT];
  auto compute = [&](int buf, const u32x4v bh, const u32x4v bl) {
    const u32x4v* sa = reinterpret_cast<const u32x4v*>(s_a + buf * MT * 512) + lane;
    u32x4v ah[MT], al[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      ah[m] = sa[(m * 2) * 64];
      al[m] = sa[(m * 2 + 1) * 64];
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah[m]), __builtin_bit_cast(f16x8v, bh),
                                                      acc[m], 0, 0, 0);
      acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah[m]), __builtin_bit_cast(f16x8v, bl),
                                                      acc[m], 0, 0, 0);
      acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, al[m]), __builtin_bit_cast(f16x8v, bh),
                                                      acc[m], 0, 0, 0);
    }
  };
  // one GEMM over n chunks: A fragments double-buffered through LDS (one barrier per chunk), the
  // B operand of chunk c from src (global, one chunk ahead) or, for stage-2 chunks of source 0,
  // from the wave's h tile
  auto gemm = [&](const ChunkDesc* chunks, int n, const float* w, auto stage2_c) {
    constexpr bool stage2 = decltype(stage2_c)::value;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
    auto src_of = [&](const ChunkDesc&) -> const CnSrc& { return stage2 ? a.x2 : a.x1; };
    auto from_h = [&](const ChunkDesc& cd) { return stage2 && cd.src == 0; };
    auto hread = [&](const ChunkDesc& cd, u32x4v& bh, u32x4v& bl) {
      bh = *reinterpret_cast<const u32x4v*>(h_hi + cd.c0 + 8 * hh);
      bl = *reinterpret_cast<const u32x4v*>(h_lo + cd.c0 + 8 * hh);
    };
    f32x4v ar[(MT + 1) / 2];
    aload(w, 0, ar);
    astore(0, ar);
    ChunkDesc cd = chunks[0];
    u32x4v bh, bl;
    f32x8v xr;
    bool ok;
    if (from_h(cd)) {
      hread(cd, bh, bl);
    } else {
      braw(src_of(cd), cd, xr, ok);
      bprep(src_of(cd), cd, xr, ok, bh, bl);
    }
    __syncthreads();
    for (int c = 0; c < n; ++c) {
      const bool more = c + 1 < n;
      ChunkDesc cn = cd;
      if (more) {
        cn = chunks[c + 1];
        aload(w, c + 1, ar);
        if (!from_h(cn)) braw(src_of(cn), cn, xr, ok);
      }
      __builtin_amdgcn_sched_barrier(0);
      compute(c & 1, bh, bl);
      __builtin_amdgcn_sched_barrier(0);
      if (more) astore((c + 1) & 1, ar);
      __syncthreads();
      if (more) {
        if (from_h(cn)) hread(cn, bh, bl);
        else bprep(src_of(cn), cn, xr, ok, bh, bl);
      }
      cd = cn;
    }
  };

  // ---- stage 1: h = op A
  gemm(a.ch1, a.n1, a.w1, std::false_type{});
  // h + b1, op B's pre-activation, pair split -> this lane's LDS column (rows >= ldh: padding)
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      const int row = 32 * m + 8 * j4 + 4 * hh;
      if (row >= a.ldh) continue;
      const f32x4v b = *reinterpret_cast<const f32x4v*>(a.b1 + row);
      _Float16 hv[4], lv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = acc[m][4 * j4 + i] + b[i];
        v = v > 0.f ? v : v * a.slope_h;
        hv[i] = (_Float16)v;
        lv[i] = (_Float16)(v - (float)hv[i]);
      }
      *reinterpret_cast<f16x4v*>(h_hi + row) = f16x4v{hv[0], hv[1], hv[2], hv[3]};
      *reinterpret_cast<f16x4v*>(h_lo + row) = f16x4v{lv[0], lv[1], lv[2], lv[3]};
    }
  // (the h tile is wave-private: the barrier inside stage 2's prologue orders these writes)

  // ---- stage 2: y = op B over [pre_B(h); x]
  gemm(a.ch2, a.n2, a.w2, std::true_type{});
  if (qb >= nq) return;
  const int2 sd = *reinterpret_cast<const int2*>(a.seg_y + 2 * u);
  const int2 sr = a.res ? *reinterpret_cast<const int2*>(a.seg_res + 2 * u) : make_int2(0, 0);
  float* yrow = a.y + (size_t)(sd.x + qb) * a.ld_y;
  const float* rrow = a.res ? a.res + (size_t)(sr.x + qb) * a.ld_res : nullptr;
  const bool quad = (a.ld_y & 3) == 0;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      const int row = 32 * m + 8 * j4 + 4 * hh;
      if (row >= a.M) {
        if (quad && row < a.ld_y) *reinterpret_cast<f32x4v*>(yrow + row) = f32x4v{0.f, 0.f, 0.f, 0.f};
        continue;
      }
      const f32x4v b = *reinterpret_cast<const f32x4v*>(a.b2 + row);
      f32x4v v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[m][4 * j4 + i] + b[i];
      if (quad) {
        if (rrow) v += *reinterpret_cast<const f32x4v*>(rrow + row);
        if (a.accumulate) v = *reinterpret_cast<const f32x4v*>(yrow + row) + v;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (row + i >= a.M) continue;
          if (rrow) v[i] += rrow[row + i];
          if (a.accumulate) v[i] = yrow[row + i] + v[i];
        }
      }
      if (a.out_div != 1.f) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] / a.out_div;
      }
      if (a.post_act == PWG_ACT_LRELU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] > 0.f ? v[i] : v[i] * a.post_slope;
      } else if (a.post_act == PWG_ACT_TANH) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = tanhf(v[i]);
      }
      if (quad) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (row + i >= a.M) v[i] = 0.f;
        *reinterpret_cast<f32x4v*>(yrow + row) = v;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (row + i < a.M) yrow[row + i] = v[i];
      }
    }
}

// ResidualStack on the x-tile scheme (split-f16; default with x-tile + fuse-pairs): 8 waves x 32
// columns = 256 columns per workgroup. Stage 1 is the dilated conv exactly as pwg_cnet_xtile_kernel
// runs it (per 16-channel block: A fragments of all taps + the block's pre-activated, pair-split
// input rows staged once); h + b1, the 1x1's LeakyReLU and the pair split go to an LDS tile
// [256][4 ldh + 16 B] that reuses the input-row space; stage 2 is the two-source 1x1 in op B's
// chunk order (h chunks from the tile, x chunks from L2, raw) with its A fragments staged g2
// chunks at a time where stage 1's were. LDS = max(A) + max(input rows, h tile): <= 80 KB (two
// workgroups per CU) up to 64 channels. Bit-identical to the x-tile conv + the tap-major 1x1.
constexpr int XS_G2MAX = 12;  // stage-2 chunks per staged group, at most
struct CnXstackArgs {
  int K1, dil1, off1, cs1, span1;  // stage 1: taps, dilation, first offset, input blocks, rows
  int g2;                          // stage-2 chunks staged per group
  int x_off;                       // LDS byte offset of the input rows / h tile region
};

template <int MT, int K1>
__global__ void __launch_bounds__(512) pwg_cnet_xstack_kernel(const CnStackArgs a, const CnXstackArgs xs) {
  constexpr int NTH = 512;
  constexpr int AV1 = K1 * MT * 128, AQ1 = (AV1 + NTH - 1) / NTH;
  constexpr int XQ_MAX = ((XT_COLS + 192) * 4 + NTH - 1) / NTH;
  constexpr int AQ2 = (XS_G2MAX * MT * 128 + NTH - 1) / NTH;
  extern __shared__ __attribute__((aligned(16))) unsigned char xs_smem[];
  f32x4v* s_a = reinterpret_cast<f32x4v*>(xs_smem);
  unsigned char* s_x = xs_smem + xs.x_off;
  unsigned char* s_h = s_x;  // after stage 1
  const int hrowb = 4 * a.ldh + 16;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const int2 blk = a.blocks[blockIdx.x];
  const int u = blk.x;
  const int q0 = blk.y;
  const int qb = q0 + wave * 32 + cl;
  const int nq = a.ncols[u];
  const CnSrc& sx = a.x1;
  const int2 sg = *reinterpret_cast<const int2*>(sx.seg + 2 * u);
  const int xv = xs.span1 * 4;

  f32x4v ar[AQ1 > AQ2 ? AQ1 : AQ2];
  f32x4v xr[XQ_MAX];
  bool xok[XQ_MAX];
  f32x16 acc[MT];
  auto mma3 = [&](int m, const u32x4v ah, const u32x4v al, const u32x4v bh, const u32x4v bl) {
    acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah), __builtin_bit_cast(f16x8v, bh),
                                                    acc[m], 0, 0, 0);
    acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah), __builtin_bit_cast(f16x8v, bl),
                                                    acc[m], 0, 0, 0);
    acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, al), __builtin_bit_cast(f16x8v, bh),
                                                    acc[m], 0, 0, 0);
  };
  // stage 1 block cb: A fragments of all taps + input rows, global -> registers -> LDS
  auto load1 = [&](int cb) {
#pragma unroll
    for (int i = 0; i < AQ1; ++i) {
      const int idx = threadIdx.x + NTH * i;
      const int tap = idx / (MT * 128), rem = idx - tap * (MT * 128);
      ar[i] = idx < AV1 ? reinterpret_cast<const f32x4v*>(a.w1 + ((size_t)(tap * xs.cs1 + cb) * MT) * 512)[rem]
                        : f32x4v{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < XQ_MAX; ++i) {
      const int idx = threadIdx.x + NTH * i;
      const bool in = idx < xv;
      const int r = in ? idx >> 2 : 0, qd = idx & 3;
      int p = q0 + xs.off1 + r;
      xok[i] = edge_row(p, sg.y, sx.pad_mode) && in;
      xr[i] = in ? *reinterpret_cast<const f32x4v*>(sx.x + (size_t)(sg.x + p) * sx.ld + 16 * cb + 4 * qd)
                 : f32x4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store1 = [&](int cb) {
#pragma unroll
    for (int i = 0; i < AQ1; ++i) {
      const int idx = threadIdx.x + NTH * i;
      if (idx < AV1) s_a[idx] = ar[i];
    }
#pragma unroll
    for (int i = 0; i < XQ_MAX; ++i) {
      const int idx = threadIdx.x + NTH * i;
      if (idx >= xv) continue;
      const int r = idx >> 2, qd = idx & 3;
      f32x4v v = xr[i];
      const int ch = 16 * cb + 4 * qd;
      if (sx.normalize) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (v[e] - a.mean[ch + e]) / a.scale[ch + e];
      }
      if (sx.slope != 1.f) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * sx.slope;
      }
      if (!xok[i]) v = f32x4v{0.f, 0.f, 0.f, 0.f};
      _Float16 hv[4], lv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hv[e] = (_Float16)v[e];
        lv[e] = (_Float16)(v[e] - (float)hv[e]);
      }
      unsigned char* row = s_x + (size_t)r * XT_ROWB;
      *reinterpret_cast<f16x4v*>(row + 8 * qd) = f16x4v{hv[0], hv[1], hv[2], hv[3]};
      *reinterpret_cast<f16x4v*>(row + 32 + 8 * qd) = f16x4v{lv[0], lv[1], lv[2], lv[3]};
    }
  };
  // stage 2 group g: op B's chunk fragments [g2 chunks][MT][2][64] x 16 B
  auto load2 = [&](int grp) {
    const int av = xs.g2 * MT * 128;
#pragma unroll
    for (int i = 0; i < AQ2; ++i) {
      const int idx = threadIdx.x + NTH * i;
      ar[i] = idx < av ? reinterpret_cast<const f32x4v*>(a.w2 + (size_t)grp * xs.g2 * MT * 512)[idx]
                       : f32x4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store2 = [&]() {
    const int av = xs.g2 * MT * 128;
#pragma unroll
    for (int i = 0; i < AQ2; ++i) {
      const int idx = threadIdx.x + NTH * i;
      if (idx < av) s_a[idx] = ar[i];
    }
  };

  // ---- stage 1: h for columns qb
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
  load1(0);
  store1(0);
  __syncthreads();
  for (int cb = 0; cb < xs.cs1; ++cb) {
    const bool more = cb + 1 < xs.cs1;
    if (more) load1(cb + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int tap = 0; tap < K1; ++tap) {
      const unsigned char* row = s_x + (size_t)(wave * 32 + cl + tap * xs.dil1) * XT_ROWB;
      const u32x4v bh = *reinterpret_cast<const u32x4v*>(row + 16 * hh);
      const u32x4v bl = *reinterpret_cast<const u32x4v*>(row + 32 + 16 * hh);
      const u32x4v* sa = reinterpret_cast<const u32x4v*>(s_a) + (size_t)tap * MT * 128 + lane;
#pragma unroll
      for (int m = 0; m < MT; ++m) mma3(m, sa[(m * 2) * 64], sa[(m * 2 + 1) * 64], bh, bl);
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    if (more) {
      store1(cb + 1);
      __syncthreads();
    }
  }
  // ---- stage 2: op B's chunks over [pre_B(h); x]
  const unsigned char* hrow = s_h + (size_t)(wave * 32 + cl) * hrowb;
  const CnSrc& s2 = a.x2;
  const int2 sg2 = *reinterpret_cast<const int2*>(s2.seg + 2 * u);
  const int ngrp = a.n2 / xs.g2;
  // x chunks' B rows (raw, from L2) one chunk ahead
  f32x8v xr2;
  bool ok2 = true;
  auto braw2 = [&](const ChunkDesc& d) {
    if (d.src == 0) return;
    int p = qb + d.row_off;
    ok2 = edge_row(p, sg2.y, s2.pad_mode);
    xr2 = *reinterpret_cast<const f32x8v*>(s2.x + (size_t)(sg2.x + p) * s2.ld + d.c0 + 8 * hh);
  };
  ChunkDesc cd = a.ch2[0];
  braw2(cd);
  load2(0);
  __syncthreads();  // stage 1's last block is done with the staging space
  store2();
  // h + b1, the 1x1's LeakyReLU, pair split -> h tile row (wave 32 + cl); rows >= ldh: padding
  {
    unsigned char* hw = s_h + (size_t)(wave * 32 + cl) * hrowb;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const int row = 32 * m + 8 * j4 + 4 * hh;
        if (row >= a.ldh) continue;
        const f32x4v b = *reinterpret_cast<const f32x4v*>(a.b1 + row);
        _Float16 hv[4], lv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = acc[m][4 * j4 + i] + b[i];
          v = v > 0.f ? v : v * a.slope_h;
          hv[i] = (_Float16)v;
          lv[i] = (_Float16)(v - (float)hv[i]);
        }
        *reinterpret_cast<f16x4v*>(hw + 2 * row) = f16x4v{hv[0], hv[1], hv[2], hv[3]};
        *reinterpret_cast<f16x4v*>(hw + 2 * a.ldh + 2 * row) = f16x4v{lv[0], lv[1], lv[2], lv[3]};
      }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
  __syncthreads();
  for (int grp = 0; grp < ngrp; ++grp) {
    const bool more = grp + 1 < ngrp;
    if (more) load2(grp + 1);
    for (int c = 0; c < xs.g2; ++c) {
      const int ci = grp * xs.g2 + c;
      u32x4v bh, bl;
      if (cd.src == 0) {
        bh = *reinterpret_cast<const u32x4v*>(hrow + 2 * (cd.c0 + 8 * hh));
        bl = *reinterpret_cast<const u32x4v*>(hrow + 2 * a.ldh + 2 * (cd.c0 + 8 * hh));
      } else {
        f32x8v x = xr2;
        const int ch = cd.c0 + 8 * hh;
        if (s2.normalize) {
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = (x[i] - a.mean[ch + i]) / a.scale[ch + i];
        }
        if (s2.slope != 1.f) {
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = x[i] > 0.f ? x[i] : x[i] * s2.slope;
        }
        if (!ok2) x = f32x8v{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        cn_split8(x, bh, bl);
      }
      const ChunkDesc cn = ci + 1 < a.n2 ? a.ch2[ci + 1] : cd;
      if (ci + 1 < a.n2) braw2(cn);
      const u32x4v* sa = reinterpret_cast<const u32x4v*>(s_a) + (size_t)c * MT * 128 + lane;
#pragma unroll
      for (int m = 0; m < MT; ++m) mma3(m, sa[(m * 2) * 64], sa[(m * 2 + 1) * 64], bh, bl);
      cd = cn;
    }
    if (!more) break;
    __syncthreads();
    store2();
    __syncthreads();
  }

  // ---- op B's epilogue
  if (qb >= nq) return;
  const int2 sd = *reinterpret_cast<const int2*>(a.seg_y + 2 * u);
  const int2 sr = a.res ? *reinterpret_cast<const int2*>(a.seg_res + 2 * u) : make_int2(0, 0);
  float* yrow = a.y + (size_t)(sd.x + qb) * a.ld_y;
  const float* rrow = a.res ? a.res + (size_t)(sr.x + qb) * a.ld_res : nullptr;
  const bool quad = (a.ld_y & 3) == 0;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      const int row = 32 * m + 8 * j4 + 4 * hh;
      if (row >= a.M) {
        if (quad && row < a.ld_y) *reinterpret_cast<f32x4v*>(yrow + row) = f32x4v{0.f, 0.f, 0.f, 0.f};
        continue;
      }
      const f32x4v b = *reinterpret_cast<const f32x4v*>(a.b2 + row);
      f32x4v v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[m][4 * j4 + i] + b[i];
      if (quad) {
        if (rrow) v += *reinterpret_cast<const f32x4v*>(rrow + row);
        if (a.accumulate) v = *reinterpret_cast<const f32x4v*>(yrow + row) + v;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (row + i >= a.M) continue;
          if (rrow) v[i] += rrow[row + i];
          if (a.accumulate) v[i] = yrow[row + i] + v[i];
        }
      }
      if (a.out_div != 1.f) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] / a.out_div;
      }
      if (a.post_act == PWG_ACT_LRELU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] > 0.f ? v[i] : v[i] * a.post_slope;
      } else if (a.post_act == PWG_ACT_TANH) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = tanhf(v[i]);
      }
      if (quad) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (row + i >= a.M) v[i] = 0.f;
        *reinterpret_cast<f32x4v*>(yrow + row) = v;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (row + i < a.M) yrow[row + i] = v[i];
      }
    }
}

template <int MT, int K1>
hipError_t xstack_launch_k(dim3 grid, int lds, hipStream_t s, const CnStackArgs& a, const CnXstackArgs& xs) {
  const hipError_t e = allow_lds(reinterpret_cast<const void*>(pwg_cnet_xstack_kernel<MT, K1>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((pwg_cnet_xstack_kernel<MT, K1>), grid, dim3(512), (size_t)lds, s, a, xs);
  return hipGetLastError();
}
hipError_t xstack_launch(int mt, int k, dim3 grid, int lds, hipStream_t s, const CnStackArgs& a, const CnXstackArgs& xs) {
  if (k != 3) return hipErrorInvalidValue;  // MelGAN ResidualStack kernel size
  switch (mt) {
    case 1: return xstack_launch_k<1, 3>(grid, lds, s, a, xs);
    case 2: return xstack_launch_k<2, 3>(grid, lds, s, a, xs);
    case 3: return xstack_launch_k<3, 3>(grid, lds, s, a, xs);
    default: return hipErrorInvalidValue;
  }
}

// Fused conv pair (split-f16 mode): y = post((conv2(pre2(conv1(pre1(x)) + b1)) + b2 + res [+ y_old]) / div)
// with conv2's intermediate never leaving the chip. This is HiFiGAN's ResBlock step
// (layers/residual_block.py:231-237: xt = c1(lrelu(x)); xt = c2(lrelu(xt)); x = xt + x) and any other
// program pair "op A writes t, op B is the only reader of t" (PwgCnet::pair_of).
//   * one workgroup = 4 waves sweeping a STRIP of `steps` 128-column tiles of one utterance;
//   * step s: stage 1 computes the intermediate h (C channels) for columns [base + 128s - 16,
//     base + 128s + 112) (wave w: 32 of them) into LDS slot s & 1, with conv2's pre-activation
//     applied, zeros outside the utterance (conv2's zero padding), split into fp16 hi/lo;
//     stage 2 computes output columns [base + 128(s-1), base + 128s), whose conv2 taps (offsets
//     within +-16) read slots (s-1) & 1 and s & 1. Each h column is computed once per strip
//     (plus one 128-column tile of warm-up per strip).
//   * A fragments of both convs stream through the same double-buffered LDS staging as
//     pwg_cnet_conv_kernel (one barrier per 16-channel chunk); stage-1 B rows come from HBM one
//     chunk ahead, stage-2 B rows from LDS.
// The arithmetic (chunk order, pair split, fp32 accumulate, epilogue order) is the unfused ops'
// exactly, so the fused result is bit-identical to running op A then op B in split mode.
constexpr int CNET_STACK_MAX_MT = 3;  // ResidualStack fusion up to 3 m-tiles (96 channels; 192: slower)
constexpr int PR_HALO = 16;
constexpr int PR_MAX_XS = 128 + 2 * 64;        // x tile columns (stage-1 tap reach +-64 - PR_HALO)
constexpr int PR_XQ = PR_MAX_XS * 8 / 256;     // 16-byte x quads per thread
constexpr int PR_MAX_LDS = 160 * 1024;
constexpr int CNET_PAIR_STREAM_C = 64;  // channels of the streamed-weight pair kernel (x-tile off)
struct CnPairArgs {
  const float* x;
  const int* seg_x;
  int ld_x;
  float slope1, slope2;
  const ChunkDesc* ch1;
  int n1;
  const float* w1;        // split-f16 fragments [chunk][MT][hi/lo][lane][4 dwords]
  const float* b1;
  const ChunkDesc* ch2;
  int n2;
  const float* w2;
  const float* b2;
  const float* res;
  const int* seg_res;
  int ld_res;
  float* y;
  const int* seg_y;
  int ld_y;
  int accumulate;
  float out_div;
  int post_act;
  float post_slope;
  const int2* strips;     // (utt, first output column)
  const int* ncols;       // [n_utts]
  int steps;              // 128-column tiles per strip
  int x_min_off, xs;      // stage-1 x tile: first column offset (vs the h tile start) and width
  int off1, dil1, off2, dil2;  // chunk c reads row offset off + (c >> 1) * dil (2 chunks per tap)
};

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global loads/stores in flight (__syncthreads' release fence would drain those too).
__device__ __forceinline__ void pr_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// C = 32 channels (MT = 1). Dynamic LDS: [A fragments of all n1 + n2 chunks, 2 KB each]
// [x tile: xs columns x HROW halves] [h ring: 2 x 128 columns x HROW halves].
__global__ void __launch_bounds__(256) pwg_cnet_pair_kernel(const CnPairArgs a) {
  constexpr int C = 32;
  constexpr int HROW = 2 * C + 8;  // halves per LDS column: [hi C][lo C][16 B pad]
  extern __shared__ __attribute__((aligned(16))) unsigned char pr_smem[];
  const int n1 = a.n1, n2 = a.n2;
  unsigned* s_w = reinterpret_cast<unsigned*>(pr_smem);                      // [(n1+n2)][2][64][4]
  _Float16* s_x = reinterpret_cast<_Float16*>(pr_smem + (size_t)(n1 + n2) * 2048);
  _Float16* s_h = s_x + (size_t)a.xs * HROW;                                    // [2][128][HROW]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const int2 st = a.strips[blockIdx.x];
  const int u = st.x, base = st.y;
  const int T = a.ncols[u];
  const int nsteps = min(a.steps, (T - base + 127) / 128);
  const int2 sx = *reinterpret_cast<const int2*>(a.seg_x + 2 * u);
  const int sd_x = a.seg_y[2 * u];
  const int sr_x = a.res ? a.seg_res[2 * u] : 0;

  // weights of both convs, resident for the whole strip
  {
    const u32x4v* g1 = reinterpret_cast<const u32x4v*>(a.w1);
    const u32x4v* g2 = reinterpret_cast<const u32x4v*>(a.w2);
    u32x4v* d = reinterpret_cast<u32x4v*>(s_w);
    for (int i = threadIdx.x; i < n1 * 128; i += 256) d[i] = g1[i];
    for (int i = threadIdx.x; i < n2 * 128; i += 256) d[n1 * 128 + i] = g2[i];
  }
  // x tile of step s: columns x0(s) + [0, xs), x0(s) = base + 128 s - PR_HALO + x_min_off; each
  // thread moves up to PR_XQ 16-byte quads (column = q >> 3, channels 4 (q & 7) .. +3)
  f32x4v xq[PR_XQ];
  auto xfetch = [&](int s) {
    const int x0 = base + 128 * s - PR_HALO + a.x_min_off;
#pragma unroll
    for (int i = 0; i < PR_XQ; ++i) {
      // unconditional (clamped) loads: a predicated load makes the compiler wait for the
      // previous ones first
      const int q = threadIdx.x + 256 * i;
      int p = x0 + (q >> 3);
      p = p < 0 ? 0 : (p >= T ? T - 1 : p);
      xq[i] = *reinterpret_cast<const f32x4v*>(a.x + (size_t)(sx.x + p) * a.ld_x + 4 * (q & 7));
    }
  };
  auto xstore = [&](int s) {  // LeakyReLU(slope1), zeros outside the utterance, fp16 pair split
    const int x0 = base + 128 * s - PR_HALO + a.x_min_off;
#pragma unroll
    for (int i = 0; i < PR_XQ; ++i) {
      const int q = threadIdx.x + 256 * i;
      if (q >= a.xs * 8) continue;
      const int p = x0 + (q >> 3);
      f32x4v v = xq[i];
      if (a.slope1 != 1.f) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * a.slope1;
      }
      if (p < 0 || p >= T) v = f32x4v{0.f, 0.f, 0.f, 0.f};
      f16x4v vh, vl;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        vh[e] = (_Float16)v[e];
        vl[e] = (_Float16)(v[e] - (float)vh[e]);
      }
      _Float16* r = s_x + (q >> 3) * HROW + 4 * (q & 7);
      *reinterpret_cast<f16x4v*>(r) = vh;
      *reinterpret_cast<f16x4v*>(r + C) = vl;
    }
  };
  auto mfma3 = [&](const u32x4v& ah, const u32x4v& al, const u32x4v& bh, const u32x4v& bl, f32x16& acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah), __builtin_bit_cast(f16x8v, bh), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah), __builtin_bit_cast(f16x8v, bl), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, al), __builtin_bit_cast(f16x8v, bh), acc, 0, 0, 0);
  };
  struct Ops { u32x4v ah, al, bh, bl; };
  // stage-1 operands of chunk c: A from s_w, B = x tile column (32 wave + cl + row_off - x_min_off)
  auto op1 = [&](int c, Ops& o) {
    const u32x4v* w = reinterpret_cast<const u32x4v*>(s_w) + (size_t)c * 128 + lane;
    o.ah = w[0];
    o.al = w[64];
    // chunk c = (tap c >> 1, channels 16 (c & 1) ..): the op's chunk order (pwg_cnet_create)
    const int row_off = a.off1 + (c >> 1) * a.dil1;
    const _Float16* r = s_x + (32 * wave + cl + row_off - a.x_min_off) * HROW + 16 * (c & 1) + 8 * hh;
    o.bh = *reinterpret_cast<const u32x4v*>(r);
    o.bl = *reinterpret_cast<const u32x4v*>(r + C);
  };
  // stage-2 operands of chunk c at step s: B = h columns of tiles s-1 / s
  auto op2 = [&](int s, int c, Ops& o) {
    const u32x4v* w = reinterpret_cast<const u32x4v*>(s_w) + (size_t)(n1 + c) * 128 + lane;
    o.ah = w[0];
    o.al = w[64];
    const int p = 32 * wave + cl + PR_HALO + a.off2 + (c >> 1) * a.dil2;  // 0 .. 159 within tiles s-1, s
    const _Float16* r = s_h + ((p < 128 ? ((s - 1) & 1) : (s & 1)) * 128 + (p & 127)) * HROW + 16 * (c & 1) + 8 * hh;
    o.bh = *reinterpret_cast<const u32x4v*>(r);
    o.bl = *reinterpret_cast<const u32x4v*>(r + C);
  };

  f32x4v rb1[4], rb2[4];  // biases of this lane's rows 8 j4 + 4 hh .. +3 (read once)
#pragma unroll
  for (int j4 = 0; j4 < 4; ++j4) {
    rb1[j4] = *reinterpret_cast<const f32x4v*>(a.b1 + 8 * j4 + 4 * hh);
    rb2[j4] = *reinterpret_cast<const f32x4v*>(a.b2 + 8 * j4 + 4 * hh);
  }
  // Output rows are stored one step late (after the next stage 1): a store's data registers
  // cannot be rewritten before the store completes, and the next step's first LDS reads would
  // otherwise wait for that at once.
  f32x4v pend[4];
  float* pend_row = nullptr;
  auto flush = [&]() {
    if (pend_row) {
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) *reinterpret_cast<f32x4v*>(pend_row + 8 * j4 + 4 * hh) = pend[j4];
    }
  };
  xfetch(0);
  xstore(0);
  pr_barrier();
  for (int s = 0; s <= nsteps; ++s) {
    // ---------------- stage 1: h columns j of tile s
    const int j = base + 128 * s - PR_HALO + 32 * wave + cl;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    {
      Ops cur, nxt;
      op1(0, cur);
      for (int c = 0; c < n1; ++c) {
        if (c + 1 < n1) op1(c + 1, nxt);
        mfma3(cur.ah, cur.al, cur.bh, cur.bl, acc);
        cur = nxt;
      }
    }
    flush();
    pend_row = nullptr;
    // x tile s+1: in flight during epilogue 1 and stage 2, stored to LDS after stage 2 (issued
    // after stage 1 so that no wait of stage 1 covers it)
    if (s < nsteps) xfetch(s + 1);
    // epilogue 1: + b1, conv2's pre-activation, zero outside [0, T), fp16 pair split -> h slot s & 1
    // (its previous tile was last read by stage 2 of step s-1, before the barrier ending that step)
    {
      _Float16* hrow = s_h + ((s & 1) * 128 + 32 * wave + cl) * HROW;
      const bool inside = j >= 0 && j < T;
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const int row = 8 * j4 + 4 * hh;
        const f32x4v b = rb1[j4];
        f16x4v vh, vl;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[4 * j4 + e] + b[e];
          if (a.slope2 != 1.f) v = v > 0.f ? v : v * a.slope2;
          v = inside ? v : 0.f;
          vh[e] = (_Float16)v;
          vl[e] = (_Float16)(v - (float)vh[e]);
        }
        *reinterpret_cast<f16x4v*>(hrow + row) = vh;
        *reinterpret_cast<f16x4v*>(hrow + C + row) = vl;
      }
    }
    pr_barrier();  // h tile s visible; every wave is done with x tile s
    if (s >= 1) {
      // ---------------- stage 2: output columns q of tile s-1
      const int q = base + 128 * (s - 1) + 32 * wave + cl;
      const bool live = q < T;
      const int qc = live ? q : 0;
      float* yrow = a.y + (size_t)(sd_x + qc) * a.ld_y;
      // residual and old value, loaded unconditionally (a predicated load waits for all earlier
      // ones) before the MFMAs; without a residual buffer the y row stands in and is not used
      const float* rrow = a.res ? a.res + (size_t)(sr_x + qc) * a.ld_res : yrow;
      f32x4v rv[4], ov[4];
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const int row = 8 * j4 + 4 * hh;
        rv[j4] = *reinterpret_cast<const f32x4v*>(rrow + row);
        ov[j4] = *reinterpret_cast<const f32x4v*>(yrow + row);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      {
        Ops cur, nxt;
        op2(s, 0, cur);
        for (int c = 0; c < n2; ++c) {
          if (c + 1 < n2) op2(s, c + 1, nxt);
          mfma3(cur.ah, cur.al, cur.bh, cur.bl, acc);
          cur = nxt;
        }
      }
      if (live) {
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const f32x4v b = rb2[j4];
          f32x4v v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[4 * j4 + e] + b[e];
          if (a.res) v += rv[j4];
          if (a.accumulate) v = ov[j4] + v;
          if (a.out_div != 1.f) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = v[e] / a.out_div;
          }
          if (a.post_act == PWG_ACT_LRELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * a.post_slope;
          } else if (a.post_act == PWG_ACT_TANH) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = tanhf(v[e]);
          }
          pend[j4] = v;
        }
        pend_row = yrow;
      }
    }
    if (s < nsteps) xstore(s + 1);
    pr_barrier();  // x tile s+1 visible; h slot (s+1) & 1 free
  }
  flush();
}

// C = 32 MT channels with the weights STREAMED (they do not fit in LDS next to the tiles, e.g.
// HiFiGAN's 64-channel stage): same strip / x tile / h ring scheme as pwg_cnet_pair_kernel, the A
// fragments of PR_SG chunks at a time staged in a double-buffered LDS area, the next group's
// loaded into registers while the current group computes (across stage and step boundaries).
// Dynamic LDS: [x tile: xs x HROW halves] [h ring: 2 x 128 x HROW] [A: 2 x PR_SG x MT x 2 KB].
// WN waves along time: a step covers STEP = 32 WN columns; wave w owns column tile w % WN and the
// MTW = MT WN / 4 m-tiles of group w / WN (C = 64: WN 4, all 2 m-tiles per wave, 128-column
// steps; C = 128: WN 2, 2 of the 4 m-tiles per wave, 64-column steps so the tiles fit in LDS).
constexpr int PR_SG = 4;
template <int MT, int WN, int SG>
__global__ void __launch_bounds__(256) pwg_cnet_pair_stream_kernel(const CnPairArgs a) {
  constexpr int C = 32 * MT;
  constexpr int CS = C / 16;        // 16-channel chunks per tap
  constexpr int HROW = 2 * C + 8;   // halves per LDS column: [hi C][lo C][16 B pad]
  constexpr int STEP = 32 * WN;     // columns per step
  constexpr int MTW = MT * WN / 4;  // m-tiles per wave
  constexpr int AQ = SG * MT * 128 / 256;  // 16-byte A quads per thread per group
  constexpr int XQ = (STEP + PR_MAX_XS - 128) * (C / 4) / 256;  // x tile <= STEP + 128 columns
  extern __shared__ __attribute__((aligned(16))) unsigned char pr_smem[];
  const int n1 = a.n1, n2 = a.n2;   // multiples of SG (host check)
  _Float16* s_x = reinterpret_cast<_Float16*>(pr_smem);
  _Float16* s_h = s_x + (size_t)a.xs * HROW;
  u32x4v* s_a = reinterpret_cast<u32x4v*>(s_h + 2 * STEP * HROW);  // [2][SG][MT][2][64]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const int nt = wave % WN;          // column tile
  const int m0 = (wave / WN) * MTW;  // first m-tile
  const int2 st = a.strips[blockIdx.x];
  const int u = st.x, base = st.y;
  const int T = a.ncols[u];
  const int nsteps = min(a.steps, (T - base + STEP - 1) / STEP);
  const int2 sx = *reinterpret_cast<const int2*>(a.seg_x + 2 * u);
  const int sd_x = a.seg_y[2 * u];
  const int sr_x = a.res ? a.seg_res[2 * u] : 0;

  f32x4v rb1[MTW][4], rb2[MTW][4];
#pragma unroll
  for (int m = 0; m < MTW; ++m)
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      rb1[m][j4] = *reinterpret_cast<const f32x4v*>(a.b1 + 32 * (m0 + m) + 8 * j4 + 4 * hh);
      rb2[m][j4] = *reinterpret_cast<const f32x4v*>(a.b2 + 32 * (m0 + m) + 8 * j4 + 4 * hh);
    }
  // A group (stage st, first chunk c0): SG chunks x MT x 2 KB, contiguous in the packed image
  u32x4v aq[AQ];
  auto agload = [&](int stg, int c0) {
    const u32x4v* g = reinterpret_cast<const u32x4v*>(stg == 0 ? a.w1 : a.w2) + (size_t)c0 * MT * 128;
#pragma unroll
    for (int i = 0; i < AQ; ++i) aq[i] = g[threadIdx.x + 256 * i];
  };
  auto agstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AQ; ++i) s_a[(size_t)buf * SG * MT * 128 + threadIdx.x + 256 * i] = aq[i];
  };
  f32x4v xq[XQ];
  auto xfetch = [&](int s) {
    const int x0 = base + STEP * s - PR_HALO + a.x_min_off;
#pragma unroll
    for (int i = 0; i < XQ; ++i) {
      const int q = threadIdx.x + 256 * i;
      int p = x0 + q / (C / 4);
      p = p < 0 ? 0 : (p >= T ? T - 1 : p);
      xq[i] = *reinterpret_cast<const f32x4v*>(a.x + (size_t)(sx.x + p) * a.ld_x + 4 * (q % (C / 4)));
    }
  };
  auto xstore = [&](int s) {
    const int x0 = base + STEP * s - PR_HALO + a.x_min_off;
#pragma unroll
    for (int i = 0; i < XQ; ++i) {
      const int q = threadIdx.x + 256 * i;
      if (q >= a.xs * (C / 4)) continue;
      const int col = q / (C / 4), ch = 4 * (q % (C / 4));
      const int p = x0 + col;
      f32x4v v = xq[i];
      if (a.slope1 != 1.f) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * a.slope1;
      }
      if (p < 0 || p >= T) v = f32x4v{0.f, 0.f, 0.f, 0.f};
      f16x4v vh, vl;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        vh[e] = (_Float16)v[e];
        vl[e] = (_Float16)(v[e] - (float)vh[e]);
      }
      _Float16* r = s_x + col * HROW + ch;
      *reinterpret_cast<f16x4v*>(r) = vh;
      *reinterpret_cast<f16x4v*>(r + C) = vl;
    }
  };
  f32x16 acc[MTW];
  auto zero_acc = [&]() {
#pragma unroll
    for (int m = 0; m < MTW; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
  };
  // one chunk: A of group slot k from s_a[buf], B = 8 channels (hi, lo) of an LDS column row
  auto chunk = [&](int buf, int k, const _Float16* brow) {
    const u32x4v bh = *reinterpret_cast<const u32x4v*>(brow);
    const u32x4v bl = *reinterpret_cast<const u32x4v*>(brow + C);
    const u32x4v* sa = s_a + ((size_t)buf * SG + k) * MT * 128 + lane;
#pragma unroll
    for (int m = 0; m < MTW; ++m) {
      const u32x4v ah = sa[((m0 + m) * 2) * 64], al = sa[((m0 + m) * 2 + 1) * 64];
      acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah), __builtin_bit_cast(f16x8v, bh), acc[m], 0, 0, 0);
      acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, ah), __builtin_bit_cast(f16x8v, bl), acc[m], 0, 0, 0);
      acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, al), __builtin_bit_cast(f16x8v, bh), acc[m], 0, 0, 0);
    }
  };
  f32x4v pend[MTW][4];
  float* pend_row = nullptr;
  auto flush = [&]() {
    if (pend_row) {
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) *reinterpret_cast<f32x4v*>(pend_row + 32 * (m0 + m) + 8 * j4 + 4 * hh) = pend[m][j4];
    }
  };

  int buf = 0;
  agload(0, 0);
  agstore(0);
  xfetch(0);
  xstore(0);
  pr_barrier();
  for (int s = 0; s <= nsteps; ++s) {
    // ---------------- stage 1: h columns j of tile s
    const int j = base + STEP * s - PR_HALO + 32 * nt + cl;
    zero_acc();
    for (int c0 = 0; c0 < n1; c0 += SG) {
      // next group: stage 1's, else stage 2's first (s >= 1) or the next step's stage 1 (s == 0)
      if (c0 + SG < n1) agload(0, c0 + SG);
      else agload(s >= 1 ? 1 : 0, 0);
#pragma unroll
      for (int k = 0; k < SG; ++k) {
        const int c = c0 + k;
        const int row_off = a.off1 + (c / CS) * a.dil1;
        chunk(buf, k, s_x + (32 * nt + cl + row_off - a.x_min_off) * HROW + 16 * (c % CS) + 8 * hh);
      }
      agstore(buf ^ 1);
      pr_barrier();
      buf ^= 1;
    }
    flush();
    pend_row = nullptr;
    if (s < nsteps) xfetch(s + 1);
    {
      _Float16* hrow = s_h + ((s & 1) * STEP + 32 * nt + cl) * HROW;
      const bool inside = j >= 0 && j < T;
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const int row = 32 * (m0 + m) + 8 * j4 + 4 * hh;
          f16x4v vh, vl;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = acc[m][4 * j4 + e] + rb1[m][j4][e];
            if (a.slope2 != 1.f) v = v > 0.f ? v : v * a.slope2;
            v = inside ? v : 0.f;
            vh[e] = (_Float16)v;
            vl[e] = (_Float16)(v - (float)vh[e]);
          }
          *reinterpret_cast<f16x4v*>(hrow + row) = vh;
          *reinterpret_cast<f16x4v*>(hrow + C + row) = vl;
        }
    }
    pr_barrier();  // h tile s visible; every wave is done with x tile s
    if (s < nsteps) xstore(s + 1);  // visible after stage 2's first group barrier (or below)
    if (s >= 1) {
      // ---------------- stage 2: output columns q of tile s-1
      const int q = base + STEP * (s - 1) + 32 * nt + cl;
      const bool live = q < T;
      const int qc = live ? q : 0;
      float* yrow = a.y + (size_t)(sd_x + qc) * a.ld_y;
      const float* rrow = a.res ? a.res + (size_t)(sr_x + qc) * a.ld_res : yrow;
      f32x4v rv[MTW][4], ov[MTW][4];
#pragma unroll
      for (int m = 0; m < MTW; ++m)
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const int row = 32 * (m0 + m) + 8 * j4 + 4 * hh;
          rv[m][j4] = *reinterpret_cast<const f32x4v*>(rrow + row);
          ov[m][j4] = *reinterpret_cast<const f32x4v*>(yrow + row);
        }
      zero_acc();
      for (int c0 = 0; c0 < n2; c0 += SG) {
        const bool last = c0 + SG >= n2 && s == nsteps;
        if (c0 + SG < n2) agload(1, c0 + SG);
        else if (!last) agload(0, 0);
#pragma unroll
        for (int k = 0; k < SG; ++k) {
          const int c = c0 + k;
          const int p = 32 * nt + cl + PR_HALO + a.off2 + (c / CS) * a.dil2;  // 0 .. STEP + 31
          chunk(buf, k, s_h + ((p < STEP ? ((s - 1) & 1) : (s & 1)) * STEP + (p < STEP ? p : p - STEP)) * HROW + 16 * (c % CS) + 8 * hh);
        }
        if (!last) agstore(buf ^ 1);
        pr_barrier();
        buf ^= 1;
      }
      if (live) {
#pragma unroll
        for (int m = 0; m < MTW; ++m)
#pragma unroll
          for (int j4 = 0; j4 < 4; ++j4) {
            f32x4v v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[m][4 * j4 + e] + rb2[m][j4][e];
            if (a.res) v += rv[m][j4];
            if (a.accumulate) v = ov[m][j4] + v;
            if (a.out_div != 1.f) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = v[e] / a.out_div;
            }
            if (a.post_act == PWG_ACT_LRELU) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * a.post_slope;
            } else if (a.post_act == PWG_ACT_TANH) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = tanhf(v[e]);
            }
            pend[m][j4] = v;
          }
        pend_row = yrow;
      }
    }
    pr_barrier();  // x tile s+1 visible; h slot (s+1) & 1 free
  }
  flush();
}

// Thin outputs (M <= 8: the last conv of a generator, 1 or 4 channels). A 32-row MFMA tile would
// be >= 75 % zero rows, so one THREAD computes all M outputs of one column on the VALU: per K
// chunk it loads its 16 input channels (pre-activation and edge mode as in the MFMA kernel) and
// FMAs them with the M x 16 weights, which are wave-uniform scalar loads from the same packed
// fragments (chunk c, m-tile 0: output o / channel c0+8h+i sit at lane o+32h, k-step i).
// The staged tile is dynamic LDS sized by the phase's span (a fixed 640-row array held 40 KB per
// 2-wave workgroup: 4 workgroups per CU).
constexpr int THIN_MAX_SPAN = 128 + 512;
// staged row stride in floats: 16 channels + 4 of pad. At 16 (64 B) the per-lane row reads
// (ds_read_b128, lane i at 64 i + 16 j bytes) hit the same banks every 4 lanes (69 % of LDS cycles
// were bank conflicts, r02_voc_pmc); 80-B rows put 16 lanes on 16 disjoint 4-bank groups
constexpr int THIN_ROW = 20;
template <int M>
__global__ void __launch_bounds__(128) pwg_cnet_thin_kernel(const CnConvArgs a, int nsrc) {
  extern __shared__ __attribute__((aligned(16))) float s_x[];  // [span][THIN_ROW]
  const int2 blk = a.blocks[blockIdx.x];
  const int u = blk.x;
  const int q = blk.y + threadIdx.x;
  const bool live = q < a.ncols[u];
  float acc[M];
#pragma unroll
  for (int o = 0; o < M; ++o) acc[o] = 0.f;
  for (int si = 0; si < nsrc; ++si) {
    const CnSrc& s = a.src[si];
    const int2 sg = *reinterpret_cast<const int2*>(s.seg + 2 * u);
    for (int cb = 0; cb < s.nc; ++cb) {
      // stage rows [q0 + off_min, q0 + off_min + span) x 16 channels, pre-activation applied once
      __syncthreads();
      for (int i = threadIdx.x; i < s.span * 4; i += 128) {
        const int r = i >> 2, qd = i & 3;
        int p = blk.y + s.off_min + r;
        const bool ok = edge_row(p, sg.y, s.pad_mode);
        const int ch = 16 * cb + 4 * qd;
        f32x4v v = *reinterpret_cast<const f32x4v*>(s.x + (size_t)(sg.x + p) * s.ld + ch);
        if (s.normalize) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (v[e] - a.mean[ch + e]) / a.scale[ch + e];
        }
        if (s.slope != 1.f) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * s.slope;
        }
        *reinterpret_cast<f32x4v*>(s_x + THIN_ROW * r + 4 * qd) = ok ? v : f32x4v{0.f, 0.f, 0.f, 0.f};
      }
      __syncthreads();
      for (int k = 0; k < s.taps; ++k) {
        const int c = s.chunk_base + k * s.nc + cb;
        const int r = threadIdx.x + a.chunks[c].row_off - s.off_min;
        const float* xr = s_x + THIN_ROW * r;
        const float* wf = a.wfrag + (size_t)c * a.mt_total * 512;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4v x0 = *reinterpret_cast<const f32x4v*>(xr + 8 * h);
          const f32x4v x1 = *reinterpret_cast<const f32x4v*>(xr + 8 * h + 4);
#pragma unroll
          for (int o = 0; o < M; ++o) {
            // k-step i = 4 sub + e of lane o + 32 h: W[o][16 cb + 8 h + i][k]
            const f32x4v w0 = *reinterpret_cast<const f32x4v*>(wf + (o + 32 * h) * 4);
            const f32x4v w1 = *reinterpret_cast<const f32x4v*>(wf + 256 + (o + 32 * h) * 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[o] = fmaf(w0[e], x0[e], acc[o]);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[o] = fmaf(w1[e], x1[e], acc[o]);
          }
        }
      }
    }
  }
  if (!live) return;
  const int t = q * a.ostride + a.ophase;
  const int2 sd = *reinterpret_cast<const int2*>(a.seg_dst + 2 * u);
  float* yrow = a.y + (size_t)(sd.x + t) * a.ld_dst;
  const float* rrow = nullptr;
  if (a.res) {
    const int2 sr = *reinterpret_cast<const int2*>(a.seg_res + 2 * u);
    rrow = a.res + (size_t)(sr.x + t) * a.ld_res;
  }
  bool bad = false;
#pragma unroll
  for (int o = 0; o < M; ++o) {
    if (o >= a.M) break;
    float v = acc[o] + a.bias[o];
    if (rrow) v += rrow[o];
    if (a.accumulate) v = yrow[o] + v;
    if (a.out_div != 1.f) v = v / a.out_div;
    if (a.post_act == PWG_ACT_LRELU) v = v > 0.f ? v : v * a.post_slope;
    else if (a.post_act == PWG_ACT_TANH) v = tanhf(v);
    bad |= !__builtin_isfinite(v);
    yrow[o] = v;
  }
  for (int o = a.M; o < a.ld_dst; ++o) yrow[o] = 0.f;  // padding channels stay zero
  // program output in split-f16 mode: a value beyond the fp16 pair range anywhere upstream became
  // (inf, -inf), every later product NaN, and nothing on the way (LeakyReLU, tanh, sums) clears it
  if (a.range_flag) flag_range(a.range_flag, nullptr, bad, (int)(threadIdx.x & 63));
}

// One-pass form of pwg_cnet_thin_kernel (the ops whose whole staged input fits THIN1_LDS): the
// input rows of EVERY 16-channel block of every source and the op's M x 16 weights of every chunk
// are staged up front, 8 loads per thread in flight per batch, behind one barrier; then the same
// FMAs in the same order (bit-identical). The per-block form pays a load round trip per block and
// per 128-quad slice of it plus a scalar weight load per tap (HiFiGAN / MB-MelGAN output convs at
// B = 1: 17-26 us for a few us of FMAs).
constexpr int THIN1_LDS = 64 * 1024;
// Stage the input rows of every 16-channel block of every source (pre-activated, edge rows
// resolved) into LDS [src][cb][span][THIN_ROW], 8 loads per thread in flight per batch (NT threads).
template <int NT>
__device__ __forceinline__ void thin_stage_rows(const CnConvArgs& a, int nsrc, float* s_x, int xf0, int2 blk, int u) {
  constexpr int B = 8;
  for (int si = 0; si < nsrc; ++si) {
    const CnSrc& s = a.src[si];
    const int2 sg = *reinterpret_cast<const int2*>(s.seg + 2 * u);
    float* const sx = s_x + (si ? xf0 : 0);
    const int total = s.nc * s.span * 4;  // quads: [cb][row][quad]
    for (int b0 = 0; b0 < total; b0 += NT * B) {
      f32x4v v[B];
      bool ok[B];
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const int i = b0 + threadIdx.x + NT * j;
        const int ii = i < total ? i : total - 1;
        const int cb = ii / (s.span * 4), rq = ii - cb * (s.span * 4);
        int p = blk.y + s.off_min + (rq >> 2);
        ok[j] = edge_row(p, sg.y, s.pad_mode);
        v[j] = *reinterpret_cast<const f32x4v*>(s.x + (size_t)(sg.x + p) * s.ld + 16 * cb + 4 * (rq & 3));
      }
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const int i = b0 + threadIdx.x + NT * j;
        if (i >= total) break;
        const int cb = i / (s.span * 4), rq = i - cb * (s.span * 4);
        const int ch = 16 * cb + 4 * (rq & 3);
        f32x4v x = v[j];
        if (s.normalize) {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = (x[e] - a.mean[ch + e]) / a.scale[ch + e];
        }
        if (s.slope != 1.f) {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = x[e] > 0.f ? x[e] : x[e] * s.slope;
        }
        *reinterpret_cast<f32x4v*>(sx + THIN_ROW * (cb * s.span + (rq >> 2)) + 4 * (rq & 3)) =
            ok[j] ? x : f32x4v{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
}

// TPC threads per column, each summing the outputs o = sub, sub + TPC, ... (same per-output FMA
// order): M = 4 / 8 outputs no longer serialise on one thread (MB-MelGAN's 4-band output conv).
template <int M, int TPC>
__global__ void __launch_bounds__(128 * TPC) pwg_cnet_thin1_kernel(const CnConvArgs a, int nsrc) {
  constexpr int NT = 128 * TPC, MO = M / TPC;
  static_assert(M % TPC == 0, "outputs split evenly over a column's threads");
  const int col = threadIdx.x / TPC, sub = threadIdx.x - col * TPC;
  extern __shared__ __attribute__((aligned(16))) float s_x[];  // [src][cb][span][THIN_ROW], then [chunk][h][M][8]
  const int2 blk = a.blocks[blockIdx.x];
  const int u = blk.x;
  const int q = blk.y + col;
  const bool live = q < a.ncols[u];
  const int xf0 = a.src[0].nc * a.src[0].span * THIN_ROW;
  const int xf = xf0 + (nsrc > 1 ? a.src[1].nc * a.src[1].span * THIN_ROW : 0);
  float* const s_w = s_x + xf;
  thin_stage_rows<NT>(a, nsrc, s_x, xf0, blk, u);
  constexpr int B = 8;
  // weights: chunk c, h, output o -> 8 floats (k-steps 8 h + [0, 8)): sub 0 then sub 1 of lane o + 32 h
  {
    const int total = a.n_chunks * 2 * M * 2;  // quads: [chunk][h][o][sub]
    for (int b0 = 0; b0 < total; b0 += NT * B) {
      f32x4v v[B];
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const int i = b0 + threadIdx.x + NT * j;
        const int ii = i < total ? i : total - 1;
        const int sub = ii & 1, o = (ii >> 1) % M, h = ((ii >> 1) / M) & 1, c = (ii >> 1) / M >> 1;
        v[j] = *reinterpret_cast<const f32x4v*>(a.wfrag + (size_t)c * a.mt_total * 512 + 256 * sub + (o + 32 * h) * 4);
      }
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const int i = b0 + threadIdx.x + NT * j;
        if (i < total) *reinterpret_cast<f32x4v*>(s_w + 4 * i) = v[j];
      }
    }
  }
  __syncthreads();
  float acc[MO];
#pragma unroll
  for (int o = 0; o < MO; ++o) acc[o] = 0.f;
  for (int si = 0; si < nsrc; ++si) {
    const CnSrc& s = a.src[si];
    const float* const sx = s_x + (si ? xf0 : 0);
    for (int cb = 0; cb < s.nc; ++cb) {
      for (int k = 0; k < s.taps; ++k) {
        const int c = s.chunk_base + k * s.nc + cb;
        const int r = col + a.chunks[c].row_off - s.off_min;
        const float* xr = sx + THIN_ROW * (cb * s.span + r);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4v x0 = *reinterpret_cast<const f32x4v*>(xr + 8 * h);
          const f32x4v x1 = *reinterpret_cast<const f32x4v*>(xr + 8 * h + 4);
#pragma unroll
          for (int o = 0; o < MO; ++o) {
            const int oo = sub + TPC * o;
            const f32x4v w0 = *reinterpret_cast<const f32x4v*>(s_w + ((c * 2 + h) * M + oo) * 8);
            const f32x4v w1 = *reinterpret_cast<const f32x4v*>(s_w + ((c * 2 + h) * M + oo) * 8 + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[o] = fmaf(w0[e], x0[e], acc[o]);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[o] = fmaf(w1[e], x1[e], acc[o]);
          }
        }
      }
    }
  }
  if (!live) return;
  const int t = q * a.ostride + a.ophase;
  const int2 sd = *reinterpret_cast<const int2*>(a.seg_dst + 2 * u);
  float* yrow = a.y + (size_t)(sd.x + t) * a.ld_dst;
  const float* rrow = nullptr;
  if (a.res) {
    const int2 sr = *reinterpret_cast<const int2*>(a.seg_res + 2 * u);
    rrow = a.res + (size_t)(sr.x + t) * a.ld_res;
  }
  bool bad = false;
#pragma unroll
  for (int o = 0; o < MO; ++o) {
    const int oo = sub + TPC * o;
    if (oo >= a.M) break;
    float v = acc[o] + a.bias[oo];
    if (rrow) v += rrow[oo];
    if (a.accumulate) v = yrow[oo] + v;
    if (a.out_div != 1.f) v = v / a.out_div;
    if (a.post_act == PWG_ACT_LRELU) v = v > 0.f ? v : v * a.post_slope;
    else if (a.post_act == PWG_ACT_TANH) v = tanhf(v);
    bad |= !__builtin_isfinite(v);
    yrow[oo] = v;
  }
  for (int o = a.M + sub; o < a.ld_dst; o += TPC) yrow[o] = 0.f;
  if (a.range_flag) flag_range(a.range_flag, nullptr, bad, (int)(threadIdx.x & 63));
}

// PQMF synthesis (layers/pqmf.py:133-149): y[t] = sum_m sum_k h[m][k] * S * x[(t+k-P)/S][m] over
// the k with (t+k-P) divisible by S and inside the utterance. One thread per output sample.
struct CnPqmfArgs {
  const float* x;
  const int* seg_src;
  int ld_src;
  const float* h;     // [S][NT] synthesis filters
  float* y;
  const int* seg_dst;
  int ld_dst;
  const int2* blocks; // (utt, first output sample) per 256-sample block
  int S, NT;
  int* range_flag;    // as CnConvArgs::range_flag
};

// One workgroup = 256 consecutive output samples of one utterance. The subband rows it needs
// (256/S + NT/S + 1 rows x S bands) and the S x NT filter bank are staged in LDS once; each thread
// then sums its ~NT/S taps x S bands from LDS.
constexpr int PQ_MAX_S = 8, PQ_MAX_NT = 128, PQ_ROWS = 256 + PQ_MAX_NT;
__global__ void __launch_bounds__(256) pwg_cnet_pqmf_kernel(const CnPqmfArgs a) {
  __shared__ __attribute__((aligned(16))) float s_x[PQ_ROWS * PQ_MAX_S];
  __shared__ __attribute__((aligned(16))) float s_h[PQ_MAX_S * PQ_MAX_NT];  // [tap][band]
  const int2 blk = a.blocks[blockIdx.x];
  const int u = blk.x;
  const int2 sd = *reinterpret_cast<const int2*>(a.seg_dst + 2 * u);
  const int2 ss = *reinterpret_cast<const int2*>(a.seg_src + 2 * u);
  const int S = a.S, NT = a.NT, P = NT / 2;
  const int t0 = blk.y;
  // subband rows j with S*j in [t0 - P, t0 + 255 + NT - 1 - P]
  const int j0 = (t0 - P) >= 0 ? (t0 - P) / S : -((P - t0 + S - 1) / S);
  const int nrow = (t0 + 255 + NT - 1 - P) / S - j0 + 1;
  // every load in flight before the first store (the block's only global round trip): rows
  // nrow * S <= 256 + NT + 2 S <= 2 x 256, filters S * NT <= 4 x 256
  constexpr int XB = 2, HB = (PQ_MAX_S * PQ_MAX_NT + 255) / 256;
  float xv[XB], hv[HB];
#pragma unroll
  for (int k = 0; k < XB; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int r = i / S, m = i - r * S;
    const int j = j0 + r;
    xv[k] = (i < nrow * S && j >= 0 && j < ss.y) ? (float)S * a.x[(size_t)(ss.x + j) * a.ld_src + m] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < HB; ++k) {
    const int i = threadIdx.x + 256 * k;
    hv[k] = i < S * NT ? a.h[i] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < XB; ++k)
    if (threadIdx.x + 256 * k < nrow * S) s_x[threadIdx.x + 256 * k] = xv[k];
#pragma unroll
  for (int k = 0; k < HB; ++k) {
    const int i = threadIdx.x + 256 * k, m = i / NT;
    if (i < S * NT) s_h[(i - m * NT) * S + m] = hv[k];  // filter m, tap k -> [k][m]
  }
  for (int i = threadIdx.x + 256 * XB; i < nrow * S; i += 256) {  // (not reached within the limits)
    const int r = i / S, m = i - r * S;
    const int j = j0 + r;
    s_x[i] = (j >= 0 && j < ss.y) ? (float)S * a.x[(size_t)(ss.x + j) * a.ld_src + m] : 0.f;
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= sd.y) return;
  float acc = 0.f;
  const int r0 = ((P - t) % S + S) % S;  // first tap k with (t + k - P) % S == 0
  // row of tap r0 (exact division); each later tap (k += S) is the next row: one division per
  // thread instead of one per tap (S is a run-time value: ~30 instructions each)
  const int rr0 = (t + r0 - P) / S - j0;
  if (S == 4) {  // multi-band MelGAN: a row's 4 bands and a tap's 4 filters as one 16-B LDS read each
    const f32x4v* x4 = reinterpret_cast<const f32x4v*>(s_x) + rr0;
    const f32x4v* h4 = reinterpret_cast<const f32x4v*>(s_h) + r0;
    for (int k = r0; k < NT; k += 4, ++x4, h4 += 4) {
      const f32x4v xv = *x4, hw = *h4;
#pragma unroll
      for (int m = 0; m < 4; ++m) acc = fmaf(hw[m], xv[m], acc);
    }
  } else {
    int rr = rr0;
    for (int k = r0; k < NT; k += S, ++rr)
      for (int m = 0; m < S; ++m) acc = fmaf(s_h[k * S + m], s_x[rr * S + m], acc);
  }
  a.y[(size_t)(sd.x + t) * a.ld_dst] = acc;
  if (a.range_flag) flag_range(a.range_flag, nullptr, !__builtin_isfinite(acc), (int)(threadIdx.x & 63));
}

// Non-finite check of the program output when its last op is not a thin or PQMF launch (split-f16
// range flag, pwg_cnet_run_status): rows x ld floats, grid-stride.
__global__ void __launch_bounds__(256) pwg_cnet_finite_kernel(const float* y, long long n, int* flag) {
  bool bad = false;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    bad |= !__builtin_isfinite(y[i]);
  flag_range(flag, nullptr, bad, (int)(threadIdx.x & 63));
}

// ---------------------------------------------------------------------------------------------
// A plan's device lists (segments, block lists, columns per utterance, fused-pair strips, x-tile
// and narrow blocks with their frame ranges) live in the caller's workspace and are written at the
// start of every run by pwg_cnet_desc_kernel from the utterance lengths carried in its arguments:
// a new plan costs host work only (no per-plan allocation or copy), and a captured forward
// regenerates them itself. Every list is one enumeration over the plan's utterances:
//   CN_L_SEG   per utterance: (first row, rows) of a buffer of `rate` rows per frame;
//   CN_L_NCOL  per utterance: its columns n_u = ceil((frames * rate - ophase) / ostride);
//   CN_L_BLK   per utterance, q0 = 0, step, .. < n_u: (utterance, q0);
//   CN_L_NFR   same enumeration as CN_L_BLK: (first frame, frames) of the utterance.
// The host builds the same image (pwg_cnet_plan_image) and checks it against the lists it
// validated, so the kernel's output is the checked image.
enum { CN_L_SEG = 0, CN_L_NCOL = 1, CN_L_BLK = 2, CN_L_NFR = 3 };
constexpr int CN_DESC_UTTS = 64;   // utterances per descriptor launch
// lists per descriptor launch: every list of a vocoder plan in one launch (MB-MelGAN v2 77, HiFiGAN
// v1 ~100) -- each launch sits on the B = 1 forward's critical path before its first op
constexpr int CN_DESC_SPECS = 96;
struct CnDescSpec {
  int kind, rate, ostride, ophase, step;
  int off;              // ints into the image
  int base_idx;         // entries of the utterances before this launch's first (< 2^30: the image)
  int base_row;         // CN_L_SEG: rows of the utterances before this launch's first (< 2^31)
};
struct CnDescArgs {
  int* img;
  int* flag;            // first launch: the run's range flag, zeroed here (null otherwise)
  int n_utts, u0, f0, n_specs;
  int last;             // covers the plan's last utterances: also writes each odd-length CN_L_NCOL
                        // list's pad int (0) before the next 8-byte-aligned list
  int frames[CN_DESC_UTTS];
  CnDescSpec specs[CN_DESC_SPECS];
};
static_assert(sizeof(CnDescArgs) <= 3584, "descriptor launch arguments within the 4 KB kernel-argument block");

__host__ __device__ inline long long cn_list_cols(int kind, long long frames, int rate, int ostride, int ophase) {
  const long long T = frames * rate;
  return kind == CN_L_SEG ? T : (T - ophase + ostride - 1) / ostride;
}
__host__ __device__ inline long long cn_list_count(int kind, long long cols, int step) {
  return (kind == CN_L_SEG || kind == CN_L_NCOL) ? 1 : (cols + step - 1) / step;
}

// one workgroup per list: per-utterance entry counts, their prefix (thread 0; <= 64 utterances),
// then the entries, 8-byte stores
__global__ void __launch_bounds__(256) pwg_cnet_desc_kernel(const CnDescArgs a) {
  const CnDescSpec& sp = a.specs[blockIdx.x];
  __shared__ long long start[CN_DESC_UTTS + 1], row0[CN_DESC_UTTS + 1], frame0[CN_DESC_UTTS + 1];
  if (threadIdx.x == 0) {
    long long e = sp.base_idx, r = sp.base_row, f = a.f0;
    for (int u = 0; u < a.n_utts; ++u) {
      start[u] = e; row0[u] = r; frame0[u] = f;
      const long long cols = cn_list_cols(sp.kind, a.frames[u], sp.rate, sp.ostride, sp.ophase);
      e += cn_list_count(sp.kind, cols, sp.step);
      r += (long long)a.frames[u] * sp.rate;
      f += a.frames[u];
    }
    start[a.n_utts] = e;
  }
  if (a.flag != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *a.flag = 0;
  __syncthreads();
  if (a.last && sp.kind == CN_L_NCOL && threadIdx.x == 0 && (start[a.n_utts] & 1)) a.img[sp.off + start[a.n_utts]] = 0;
  for (int u = 0; u < a.n_utts; ++u) {
    const long long cols = cn_list_cols(sp.kind, a.frames[u], sp.rate, sp.ostride, sp.ophase);
    const long long n = start[u + 1] - start[u];
    for (long long j = threadIdx.x; j < n; j += 256) {
      const long long at = start[u] + j;
      if (sp.kind == CN_L_NCOL) {
        a.img[sp.off + at] = (int)cols;
      } else {
        int2 v;
        if (sp.kind == CN_L_SEG) v = make_int2((int)row0[u], (int)((long long)a.frames[u] * sp.rate));
        else if (sp.kind == CN_L_BLK) v = make_int2(a.u0 + u, (int)(j * sp.step));
        else v = make_int2((int)frame0[u], a.frames[u]);
        reinterpret_cast<int2*>(a.img + sp.off)[at] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
struct OpPhase {          // one launch
  int op = 0;
  int phase = 0;          // CONVT phase r, else 0
  int MT = 0, mt_total = 0;
  long long frag_off = 0; // floats into the packed image
  long long frag16_off = -1;  // split-f16 A fragments (same size), MFMA phases only
  long long bias_off = -1;
  std::vector<ChunkDesc> chunks;
  ChunkDesc* d_chunks = nullptr;
  int ostride = 1, ophase = 0;
  int k_a = 0, off_a = 0; // CONVT
  int NW = 4;             // waves per workgroup of pwg_cnet_conv_kernel
  bool xtile = false;     // split mode runs pwg_cnet_xtile_kernel (channel-block-major, staged input tile)
  int xt_lds = 0;
  bool xt_sync = false;   // synchronous staging at 128 VGPRs (two workgroups per CU)
  int xt_ks = 0;          // with xt_sync: taps staged per step (the kernel size unless split)
  bool xt_db = false;     // PWG_CNET_OPT_XT_DMA applies: double-buffered DMA staging of the A fragments
  bool xt_db_pick = false; // ... and the measured rule picks it (option value 1)
  bool xt_convt_db = false;  // wide ConvTranspose phase (> 2 m-tiles): tap-major kernel, or the DMA
                             // x-tile kernel over 256-column blocks (d_xblocks) when PWG_CNET_OPT_XT_DMA
  int xt_db_ks[2] = {0, 0}, xt_db_lds[2] = {0, 0};  // taps per tap group and LDS bytes: [0] the fewest
                                                     // groups within 80 KB (two workgroups per CU), [1] within 160 KB
  int z_phases = 1;       // CONVT phase 0: phases launched together (gridDim.z); others: 0 (merged)
  int xpair_b = -1;       // x-tile conv pair: phase index of conv 2 (pwg_cnet_xpair_kernel)
  int xpair_lds = 0;
  int n_real_chunks = 0;  // chunks before padding to a multiple of CN_G (the rest pack as zeros)
  bool thin = false;      // M <= 8: VALU kernel with an LDS-staged input tile
  int thin_taps[2] = {0, 0}, thin_nc[2] = {0, 0}, thin_base[2] = {0, 0}, thin_off_min[2] = {0, 0},
      thin_span[2] = {0, 0};
  int pair_b = -1;        // phase index of the op this one fuses with (pwg_cnet_pair_kernel), -1 = none
  int pair_xmin = 0, pair_xs = 0, pair_lds = 0;  // its x tile offset / width and dynamic LDS bytes
  bool pair_resident = true;  // weights resident (pwg_cnet_pair_kernel) or streamed (_stream_kernel)
  int pair_step = 128;        // columns per kernel step (streamed 128-channel pairs: 64)
  int stack_b = -1;           // phase index of the two-source 1x1 fused with this conv (pwg_cnet_stack_kernel)
  int stack_lds = 0;          // its dynamic LDS bytes
  int xstack_lds = 0;         // > 0: with x-tile on, the stack runs pwg_cnet_xstack_kernel (256-column blocks)
  int xstack_g2 = 0;          // its stage-2 chunks per staged group
  int xstack_xoff = 0;        // its input-row / h-tile region offset
  int rstack_cs = 0;          // > 0: the stack also fits pwg_rstack.hip (16-channel blocks; PWG_CNET_OPT_RSTACK)
  int r1x1_mt = 0;            // > 0: a two-source 1x1 of 32 r1x1_mt outputs that pwg_r1x1_kernel runs alone
  int rconv_mt = 0;           // > 0: a k = 3 x-tile conv of 32 rconv_mt channels that pwg_rconv_kernel runs
  int ms_n = 0;               // > 0: head of a chain of this many fusable ResidualStacks (pwg_mstack.hip)
  int ms_halo = 0;            // ... their summed dilations
};

}  // namespace
}  // namespace pwg

using namespace pwg;

struct PwgCnet {
  int device = 0;
  int split_f16 = 1;  // PWG_CNET_OPT_SPLIT_F16
  int fuse_pairs = 1; // PWG_CNET_OPT_FUSE_PAIRS (split-f16 mode only)
  int pair_steps = 16; // PWG_CNET_OPT_PAIR_STEPS: 128-column tiles per fused-pair strip (plan time)
  int xtile = 1;       // PWG_CNET_OPT_XTILE
  int xt_dma = 9;      // PWG_CNET_OPT_XT_DMA flags (CNET_DMA_RULE | CNET_DMA_CONVT)
  int xcd_order = 1;   // PWG_CNET_OPT_XCD_ORDER
  int narrow = 1;      // PWG_CNET_OPT_NARROW (plan time): 0 off, 1 small launches, 2 every x-tile phase
  int narrow_dma = 1;  // PWG_CNET_OPT_NARROW_DMA: narrow launches on the DMA-ring kernel where its
                       // one-m-tile workgroups fit one round (0: the narrow x-tile / tap-major kernels)
  int mstack = 1;      // PWG_CNET_OPT_MSTACK (plan time): 0 off, 1 fused stack chains in plans whose first
                       // conv of the chain runs narrow
  int rstack = 1;      // PWG_CNET_OPT_RSTACK: batched ResidualStacks on pwg_rstack.hip, 1 weights resident in
                       // LDS where they fit (<= 64 channels), 2 always streamed (A/B); 0 the x-tile stack
  int presplit = 1;    // PWG_CNET_OPT_PRESPLIT (plan time): DMA-ring launches write / read pre-split images
  int streams = 1;     // PWG_CNET_OPT_STREAMS: 0 one stream, 1 independent launches of plans with narrow
                       // launches run on auxiliary streams, 2 every plan
  static constexpr int N_AUX = 3;
  // Auxiliary streams and cross-stream dependency events, one set per caller stream: a forward
  // being captured on one caller stream forks into aux streams no other caller's run uses, and
  // runs of one plan (or of two plans) on two caller streams never record into each other's events.
  // Events are re-recorded every run (a wait binds the record made before it). Guarded by mu.
  struct CallerSet {
    hipStream_t aux[N_AUX] = {nullptr, nullptr, nullptr};
    std::vector<hipEvent_t> ev;
    int* hflag = nullptr;  // pinned host word pwg_cnet_run_status copies the range flag into
  };
  std::map<hipStream_t, CallerSet> callers;
  std::mutex mu;       // `callers` (concurrent runs from host threads)
  int n_cu = 0;        // CUs of the device (queried once; plan-time launch sizing)
  bool pair_attr_set = false;
  std::vector<PwgCnetOp> ops;
  std::vector<int> channels, rate, ld;
  long long ref_count = 0;
  std::vector<OpPhase> phases;
  long long packed_count = 0;
  int timing = 0;  // pwg_cnet_set_timing: 1 per-launch events, 2 one event pair around each run
  struct Rec { int op; hipEvent_t a, b; };
  std::vector<Rec> records;
  std::vector<hipEvent_t> pool;
};

struct CnSchedule {
  std::vector<std::pair<int, int>> launches;  // (phase, second op fused into the launch or -1)
  bool conc = false;
  std::vector<int> stream, event;              // per launch: stream (0 = caller's), event slot or -1
  std::vector<std::vector<int>> waits;         // per launch: launches on other streams it waits for
  std::vector<size_t> order;                   // enqueue order
  bool used[1 + PwgCnet::N_AUX] = {true, false, false, false};
  int n_events = 0;
};

struct PwgCnetPlan {
  PwgCnet* n = nullptr;
  // the run's launch schedule (cnet_schedule), cached for the options it was built under
  // (sched_key; ~15-30 us of host work per eager run otherwise)
  CnSchedule sched;
  int sched_key = -1;
  int n_utts = 0;
  std::vector<long long> frames;
  std::vector<long long> rows;               // per buffer
  std::vector<size_t> buf_off;               // workspace offsets (SIZE_MAX: external)
  size_t ws_bytes = 0;
  size_t ws_flag = 0;                        // split-f16 range flag (one int) in the workspace
  size_t ws_img = 0;                         // the device lists (pwg_cnet_desc_kernel) in the workspace
  // Device lists as int offsets into that image (-1 = none); see CnDescSpec. The host image `img`
  // is what the descriptor kernel writes (built and checked here, never uploaded).
  std::vector<int> img;
  std::vector<CnDescSpec> specs;
  std::vector<CnDescArgs> desc;              // the descriptor launches' arguments (image / flag set per run)
  std::vector<int> o_seg;                   // per buffer: [n_utts][2] (first row, rows)
  std::vector<int> o_blocks;                 // per phase
  std::vector<int> n_blocks;
  std::vector<int> o_ncols;                  // per phase
  std::vector<int> o_strips;                 // per phase: fused-pair strips (utt, q0)
  std::vector<int> n_strips;
  std::vector<int> o_xblocks;                // per phase: x-tile pair blocks (utt, q0 step XP_OUT)
  std::vector<int> n_xblocks;
  int pair_steps = 16;
  bool host_only = false;                    // a handle created for device -1: built and checked, not uploaded
  int n_cu = 0;                              // CUs of the device (plan-time launch sizing)
  // per phase: narrow x-tile launch (PWG_CNET_OPT_NARROW), 0 waves = the phase's default launch
  std::vector<int> nar_nwv, nar_mt, nar_lds, n_nblocks;
  std::vector<char> nar_tap;                 // ... on the tap-major kernel (not the x-tile family)
  std::vector<char> nar_xdma;                // ... on the DMA-ring kernel (tap-major phases: K = 1 mode)
  std::vector<int> o_nblocks;                // its blocks (utt, q0 step 32 nar_nwv)
  std::vector<int> o_nfr;                    // ... and their utterances' (first frame, frames)
  // per phase: fused stack chain launch (pwg_mstack.hip) when > 0 output columns per block
  std::vector<int> ms_oc, o_msblocks, n_msblocks;
  bool has_narrow = false;                   // some phase runs narrow (PWG_CNET_OPT_STREAMS 1)
  // pre-split activation images (PWG_CNET_OPT_PRESPLIT): per image its buffer, the consumers'
  // LeakyReLU slope and workspace offset; per phase (2 pi + k) the images its sources read and its
  // launch writes (-1 none)
  std::vector<int> simg_buf;
  std::vector<float> simg_slope;
  std::vector<size_t> simg_off;
  std::vector<int> ph_simg, ph_oimg;
};

namespace {

int fail(int code, const std::string& m) { return set_error(code, m.c_str()); }
int hipf(hipError_t e, const char* what) {
  return fail(PWG_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct Guard {
  int prev = -1;
  bool ok = true;
  explicit Guard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) { ok = false; return; }
    if (prev != dev && hipSetDevice(dev) != hipSuccess) ok = false;
  }
  ~Guard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// host fp16 round-to-nearest-even and its exact inverse (split-f16 packing)
uint16_t cn_f2h(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u, ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return (uint16_t)(sign | (ax > 0x7f800000u ? 0x7e00u : 0x7c00u));
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);
  if (ax < 0x38800000u) {
    float v;
    std::memcpy(&v, &ax, 4);
    return (uint16_t)(sign | (uint32_t)std::nearbyint(v * 16777216.0f));
  }
  uint32_t h = (((ax >> 23) - 112u) << 10) | ((ax & 0x7fffffu) >> 13);
  const uint32_t rem = ax & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
  return (uint16_t)(sign | h);
}
float cn_h2f(uint16_t h) {
  const uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  float v;
  if (e == 0) v = std::ldexp((float)m, -24);
  else if (e == 31) v = m ? NAN : INFINITY;
  else v = std::ldexp((float)(m | 0x400u), (int)e - 25);
  return (h & 0x8000u) ? -v : v;
}

// The launches of one run and, with PWG_CNET_OPT_STREAMS, their streams, cross-stream waits and
// enqueue order (host only: pwg_cnet_run and pwg_cnet_plan_schedule).
// phase pi heads a fused stack chain this run launches as one pwg_mstack_kernel (split-f16 x-tile
// mode with fused ops, and the plan picked a block width for it)
bool cnet_mstack_on(const PwgCnetPlan* p, size_t pi) {
  const PwgCnet* n = p->n;
  return n->split_f16 && n->xtile && n->fuse_pairs && pi < p->ms_oc.size() && p->ms_oc[pi] > 0;
}
int cnet_schedule(PwgCnetPlan* p, CnSchedule& sc) {
  PwgCnet* n = p->n;
  const int nb = (int)n->channels.size();
  const bool fuse = n->fuse_pairs && n->split_f16;
  const bool xt = n->xtile && n->split_f16;
  auto pair_fused = [&](const OpPhase& q) { return fuse && q.pair_b >= 0 && !(xt && q.xtile); };
  auto narrow = [&](size_t i) { return xt && p->nar_nwv[i] > 0 && !p->nar_tap[i]; };
  // phases inside a fused stack chain (pwg_mstack.hip) that runs as its head's launch
  std::vector<char> in_chain(n->phases.size(), 0);
  for (size_t pi = 0; pi < n->phases.size(); ++pi)
    if (cnet_mstack_on(p, pi))
      for (int k = 1; k < 2 * n->phases[pi].ms_n; ++k) in_chain[pi + k] = 1;
  // the launches of this run: (phase, second op fused into it or -1)
  auto skipped = [&](size_t pi) {
    const OpPhase& ph = n->phases[pi];
    if (in_chain[pi]) return true;
    return (pi > 0 && ((pair_fused(n->phases[pi - 1]) && n->phases[pi - 1].pair_b == (int)pi) ||
                       (fuse && n->phases[pi - 1].stack_b == (int)pi && !narrow(pi - 1)))) ||
           ph.z_phases == 0 || (xt && fuse && pi > 0 && n->phases[pi - 1].xpair_b == (int)pi && !narrow(pi - 1));
  };
  std::vector<std::pair<int, int>>& launches = sc.launches;
  for (size_t pi = 0; pi < n->phases.size(); ++pi) {
    if (skipped(pi)) continue;
    const OpPhase& ph = n->phases[pi];
    int second = -1;
    if (cnet_mstack_on(p, pi)) second = n->phases[pi + 2 * ph.ms_n - 1].op;  // the chain's output op
    else if (pair_fused(ph)) second = n->phases[ph.pair_b].op;
    else if (fuse && ph.stack_b >= 0 && !narrow(pi)) second = n->phases[ph.stack_b].op;
    else if (xt && fuse && ph.xpair_b >= 0 && !narrow(pi)) second = n->phases[ph.xpair_b].op;
    launches.push_back({(int)pi, second});
  }
  // Concurrent launches (PWG_CNET_OPT_STREAMS): a small plan's launches are each a few dozen
  // workgroups and latency-bound, and a generator's parallel branches (HiFiGAN's multi-receptive-
  // field blocks, models/hifigan.py:159-168) are independent until their sum: each launch follows
  // the launch it depends on latest on that launch's stream when it is that stream's last, else
  // takes the least recently used stream, and waits on an event for every dependency on another
  // stream. Buffers are written once per run except an accumulated sum, whose writers stay in
  // program order: same launches, same arithmetic, bit-identical to one stream.
  const int NS = 1 + PwgCnet::N_AUX;
  const bool conc = sc.conc = n->streams == 2 || (n->streams == 1 && p->has_narrow);
  std::vector<int>& l_stream = sc.stream;
  std::vector<int>& l_event = sc.event;
  std::vector<std::vector<int>>& l_waits = sc.waits;
  l_stream.assign(launches.size(), 0);
  l_event.assign(launches.size(), -1);
  l_waits.assign(launches.size(), {});
  bool* const stream_used = sc.used;
  if (conc) {
    // dependencies by storage, not buffer id: buffers of a plan built for one stream share slots
    std::vector<int> mem(nb);
    for (int b = 0; b < nb; ++b) {
      mem[b] = b;
      if (b > 0 && b < nb - 1)
        for (int c = 1; c < b; ++c)
          if (p->buf_off[c] == p->buf_off[b]) { mem[b] = mem[c]; break; }
    }
    std::vector<int> last_writer(nb, -1);
    std::vector<std::vector<int>> readers(nb);
    int tail[1 + PwgCnet::N_AUX] = {-1, -1, -1, -1}, used_at[1 + PwgCnet::N_AUX] = {-1, -1, -1, -1};
    for (size_t L = 0; L < launches.size(); ++L) {
      std::vector<int> deps;
      auto op_deps = [&](int oi) {
        const PwgCnetOp& o = n->ops[oi];
        auto rd = [&](int b) {
          if (b >= 0 && last_writer[mem[b]] >= 0) deps.push_back(last_writer[mem[b]]);
        };
        rd(o.src[0].buf);
        if (o.kind == PWG_CNET_CONV) rd(o.src[1].buf);
        rd(o.res);
        if (o.accumulate) rd(o.dst);
        if (last_writer[mem[o.dst]] >= 0) deps.push_back(last_writer[mem[o.dst]]);  // WAW
        for (int r : readers[mem[o.dst]]) deps.push_back(r);                          // WAR
      };
      op_deps(n->phases[launches[L].first].op);
      if (launches[L].second >= 0) op_deps(launches[L].second);
      int best = -1;  // the latest dependency that is its stream's tail
      for (int d : deps)
        if (tail[l_stream[d]] == d && (best < 0 || d > best)) best = d;
      int st;
      if (best >= 0) {
        st = l_stream[best];
      } else if (deps.empty()) {
        st = 0;
      } else {
        st = 0;
        for (int k = 1; k < NS; ++k)
          if (used_at[k] < used_at[st]) st = k;
      }
      l_stream[L] = st;
      for (int d : deps)
        if (l_stream[d] != st && std::find(l_waits[L].begin(), l_waits[L].end(), d) == l_waits[L].end())
          l_waits[L].push_back(d);
      tail[st] = (int)L;
      used_at[st] = (int)L;
      stream_used[st] = true;
      auto note = [&](int oi) {
        const PwgCnetOp& o = n->ops[oi];
        for (int b : {o.src[0].buf, o.kind == PWG_CNET_CONV ? o.src[1].buf : -1, o.res, o.accumulate ? o.dst : -1})
          if (b >= 0) readers[mem[b]].push_back((int)L);
      };
      note(n->phases[launches[L].first].op);
      if (launches[L].second >= 0) note(launches[L].second);
      auto wrote = [&](int oi) {
        const int b = mem[n->ops[oi].dst];
        last_writer[b] = (int)L;
        readers[b].clear();
      };
      wrote(n->phases[launches[L].first].op);
      if (launches[L].second >= 0) wrote(launches[L].second);
    }
    // events: after every launch some launch on another stream waits for, and each aux stream's tail
    int ne = 0;
    for (size_t L = 0; L < launches.size(); ++L)
      for (int d : l_waits[L])
        if (l_event[d] < 0) l_event[d] = ne++;
    for (int k = 1; k < NS; ++k)
      if (stream_used[k] && tail[k] >= 0 && l_event[tail[k]] < 0) l_event[tail[k]] = ne++;
    sc.n_events = ne;
  }
  // Enqueue order: program order on one stream; with concurrency, breadth-first over the streams
  // (round robin, a launch once every launch it waits for is enqueued -- its event then recorded),
  // so each branch's first launches reach the GPU before the host has enqueued a whole other branch
  // (~5-10 us of host time per launch: in program order HiFiGAN's second and third residual chains
  // started 60 and 140 us after the first, profiles/r04_m). Per stream the order is program order.
  std::vector<size_t>& order = sc.order;
  order.clear();
  order.reserve(launches.size());
  if (!conc) {
    for (size_t L = 0; L < launches.size(); ++L) order.push_back(L);
  } else {
    std::vector<std::vector<size_t>> per(NS);
    for (size_t L = 0; L < launches.size(); ++L) per[l_stream[L]].push_back(L);
    std::vector<size_t> head(NS, 0);
    std::vector<char> done(launches.size(), 0);
    while (order.size() < launches.size()) {
      bool progress = false;
      for (int k = 0; k < NS; ++k) {
        if (head[k] >= per[k].size()) continue;
        const size_t L = per[k][head[k]];
        bool ready = true;
        for (int d : l_waits[L]) ready = ready && done[d];
        if (!ready) continue;
        order.push_back(L);
        done[L] = 1;
        ++head[k];
        progress = true;
      }
      if (!progress) return fail(PWG_ERR_ASSERT, "internal: no enqueue order for the concurrent launches");
    }
  }
  return PWG_OK;
}

int pick_mt(int mt_total) {
  if (mt_total <= 4) return mt_total;
  if (mt_total % 4 == 0) return 4;
  if (mt_total % 3 == 0) return 3;
  if (mt_total % 2 == 0) return 2;
  return 4;
}

// weight of (op, phase) at (output o, source s, channel i, tap k) in reference order, 0 outside
float ref_weight(const PwgCnetOp& op, const OpPhase& ph, const float* ref, int s, int o, int i, int k) {
  const PwgCnetSrc& src = op.src[s];
  if (o >= op.out_channels || i >= src.channels) return 0.f;
  if (op.kind == PWG_CNET_CONVT) {
    // ConvTranspose1d weight (C_in, C_out, 2*stride); phase tap k=0 -> k_a, k=1 -> k_a + stride
    const int kk = ph.k_a + k * op.stride;
    return ref[src.w_off + ((long long)i * op.out_channels + o) * (2 * op.stride) + kk];
  }
  return ref[src.w_off + ((long long)o * src.channels + i) * src.taps + k];
}

}  // namespace

extern "C" {

int pwg_cnet_abi_version(void) { return PWG_CNET_ABI_VERSION; }

int pwg_cnet_create(const PwgCnetOp* ops, int n_ops, int n_bufs, const int* channels, const int* rate,
                    long long ref_weight_count, int device, PwgCnet** out) {
  if (!ops || n_ops < 1 || n_bufs < 2 || !channels || !rate || !out) return fail(PWG_ERR_INVALID, "bad arguments");
  *out = nullptr;
  PwgCnet* n = new PwgCnet();
  n->device = device;
  n->ops.assign(ops, ops + n_ops);
  n->channels.assign(channels, channels + n_bufs);
  n->rate.assign(rate, rate + n_bufs);
  n->ref_count = ref_weight_count;
  for (int b = 0; b < n_bufs; ++b) {
    if (channels[b] < 1 || rate[b] < 1) { delete n; return fail(PWG_ERR_INVALID, "buffer channels/rate must be >= 1"); }
    n->ld.push_back(b == n_bufs - 1 ? channels[b] : (channels[b] + 15) / 16 * 16);
  }
  if (n->ld[0] != channels[0] || channels[0] % 16) {
    delete n;
    return fail(PWG_ERR_UNSUPPORTED, "input channels must be a multiple of 16");
  }
  long long off = 0;
  auto check_w = [&](long long o, long long cnt) { return o >= 0 && o + cnt <= ref_weight_count; };
  for (int oi = 0; oi < n_ops; ++oi) {
    const PwgCnetOp& op = n->ops[oi];
    std::string where = "op " + std::to_string(oi) + ": ";
    if (op.dst < 1 || op.dst >= n_bufs) { delete n; return fail(PWG_ERR_INVALID, where + "bad dst"); }
    if (op.out_channels != channels[op.dst]) { delete n; return fail(PWG_ERR_INVALID, where + "out_channels != dst channels"); }
    if (op.kind == PWG_CNET_PQMF) {
      const PwgCnetSrc& s = op.src[0];
      if (s.buf < 0 || s.buf >= n_bufs || op.stride < 1 || channels[s.buf] < op.stride ||
          rate[op.dst] != op.stride * rate[s.buf] || op.out_channels != 1 || op.padding < 1 || op.padding % 2 == 0 ||
          op.stride > PQ_MAX_S || op.padding > PQ_MAX_NT ||
          !check_w(s.w_off, (long long)op.stride * op.padding)) {
        delete n;
        return fail(PWG_ERR_INVALID, where + "bad PQMF op");
      }
      OpPhase ph;
      ph.op = oi; ph.phase = 0; ph.MT = 0; ph.mt_total = 0; ph.frag_off = off; ph.bias_off = -1;
      ph.ostride = 1; ph.ophase = 0;
      off += (long long)op.stride * op.padding;
      n->phases.push_back(ph);
      continue;
    }
    if (op.kind != PWG_CNET_CONV && op.kind != PWG_CNET_CONVT) { delete n; return fail(PWG_ERR_INVALID, where + "bad kind"); }
    const int nsrc = (op.src[1].buf >= 0 && op.kind == PWG_CNET_CONV) ? 2 : 1;
    for (int s = 0; s < nsrc; ++s) {
      const PwgCnetSrc& src = op.src[s];
      if (src.buf < 0 || src.buf >= n_bufs || src.channels < 1 || src.channels > channels[src.buf] || src.taps < 1 ||
          (op.kind == PWG_CNET_CONV && src.dilation < 1)) {
        delete n;
        return fail(PWG_ERR_INVALID, where + "bad source");
      }
      if (src.buf == n_bufs - 1) { delete n; return fail(PWG_ERR_INVALID, where + "the output buffer cannot be read"); }
      if (op.kind == PWG_CNET_CONV && rate[src.buf] != rate[op.dst]) {
        delete n;
        return fail(PWG_ERR_INVALID, where + "conv source and destination rates differ");
      }
      if (src.normalize && src.buf != 0) { delete n; return fail(PWG_ERR_INVALID, where + "normalize on a non-input buffer"); }
      if (src.pad_mode < PWG_PAD_ZERO || src.pad_mode > PWG_PAD_REPLICATE) {
        delete n;
        return fail(PWG_ERR_INVALID, where + "bad pad_mode");
      }
    }
    if (op.res >= 0 && (op.res >= n_bufs || rate[op.res] != rate[op.dst] || channels[op.res] < op.out_channels ||
                        op.res == n_bufs - 1)) {
      delete n;
      return fail(PWG_ERR_INVALID, where + "bad residual buffer");
    }
    if (op.out_div == 0.f) { delete n; return fail(PWG_ERR_INVALID, where + "out_div must be non-zero"); }
    const int mt_total0 = (op.out_channels + 31) / 32;
    int MT = pick_mt(mt_total0);
    // >= 256-row single-source convs with <= 7 taps run 2 m-tiles per x-tile workgroup (half the A
    // staging, more workgroups in flight): HiFiGAN v1's 256-channel k = 3 / 7 convs -10 / -12 %;
    // slower at k = 11 and at 128 rows (profiles/r02_mt2)
    if (op.kind == PWG_CNET_CONV && op.src[1].buf < 0 && MT == 4 && mt_total0 >= 8 &&
        op.src[0].taps <= CNET_XT_MT2_MAXK)
      MT = 2;
    const int mt_total = (mt_total0 + MT - 1) / MT * MT;
    int n_phase = 1;
    if (op.kind == PWG_CNET_CONVT) {
      const int s = op.stride;
      // causal (CausalConvTranspose1d): replicate-padded source, no padding, T -> stride*T after the trim
      const bool causal = op.src[0].pad_mode == PWG_PAD_REPLICATE;
      if (s < 1 || rate[op.dst] != s * rate[op.src[0].buf] ||
          (causal ? op.padding != 0 || op.output_padding != 0 : s - 2 * op.padding + op.output_padding != 0)) {
        delete n;
        return fail(PWG_ERR_UNSUPPORTED, where + "ConvTranspose1d must map T -> stride*T (kernel 2*stride)");
      }
      if (op.src[0].pad_mode == PWG_PAD_REFLECT) {
        delete n;
        return fail(PWG_ERR_UNSUPPORTED, where + "reflection padding on a ConvTranspose1d");
      }
      if (!check_w(op.src[0].w_off, (long long)op.src[0].channels * op.out_channels * 2 * s)) {
        delete n;
        return fail(PWG_ERR_INVALID, where + "weights out of range");
      }
      n_phase = s;
    } else {
      for (int s = 0; s < nsrc; ++s)
        if (!check_w(op.src[s].w_off, (long long)op.out_channels * op.src[s].channels * op.src[s].taps)) {
          delete n;
          return fail(PWG_ERR_INVALID, where + "weights out of range");
        }
    }
    if ((op.b_off >= 0 && !check_w(op.b_off, op.out_channels)) || (op.b2_off >= 0 && !check_w(op.b2_off, op.out_channels))) {
      delete n;
      return fail(PWG_ERR_INVALID, where + "bias out of range");
    }
    for (int r = 0; r < n_phase; ++r) {
      OpPhase ph;
      ph.op = oi; ph.phase = r; ph.MT = MT; ph.mt_total = mt_total;
      // 8 waves (256 columns) share each staged A chunk of the wide ops
      if (MT >= CNET_NW8_MT && op.kind == PWG_CNET_CONV) ph.NW = 8;
      // wide dilated single-source convs: the staged-input-tile kernel (split mode)
      // (ConvTranspose phases: 2 taps of dilation 1, CNET_XTILE_CONVT)
      const bool convt = op.kind == PWG_CNET_CONVT;
      const int xk = convt ? 2 : op.src[0].taps, xd = convt ? 1 : op.src[0].dilation;
      if ((op.kind == PWG_CNET_CONV || (convt && mt_total <= CNET_XTILE_CONVT)) && nsrc == 1 &&
          (MT == 1 || MT == 2 || MT == 3 || MT == 4) && mt_total % MT == 0 &&
          (convt || xtile_supported(xk)) && (xk - 1) * xd <= 191 && op.src[0].channels % 16 == 0) {
        ph.xtile = true;
        ph.NW = 8;  // 256-column blocks
        // one 16-channel block per staging step (2 or 4 measured 1 % slower, r02_xt5)
        const int span = XT_COLS + (xk - 1) * xd;
        ph.xt_lds = xk * MT * 2048 + span * XT_ROWB;
        // ConvTranspose phases of 2 m-tiles: the DMA-staged form (128 VGPRs, two workgroups per CU)
        // on the measured rule (CNET_DMA_RULE): MB-MelGAN v2's 96 -> 48 0.376 -> 0.296 ms, HiFiGAN
        // v1's 128 -> 64 0.869 -> 0.695 ms; at 1 m-tile it lost (HiFiGAN 64 -> 32 0.576 -> 0.601 ms;
        // profiles/r06_ab/ct_*)
        if (convt) {
          ph.xt_db = true;
          ph.xt_db_pick = MT == 2;
          ph.xt_db_ks[0] = ph.xt_db_ks[1] = 2;
          ph.xt_db_lds[0] = ph.xt_db_lds[1] = 2 * 2 * MT * 2048 + span * XT_ROWB;
        }
      } else if (convt && nsrc == 1 && (MT == 3 || MT == 4) && mt_total % MT == 0 && op.src[0].channels % 16 == 0) {
        ph.xt_convt_db = true;  // 2 taps: both tap groups' A (2 x MT x 4 KB) + 257 input rows, <= 53 KB
        ph.xt_db = ph.xt_db_pick = true;
        ph.xt_db_ks[0] = ph.xt_db_ks[1] = 2;
        ph.xt_db_lds[0] = ph.xt_db_lds[1] = 2 * 2 * MT * 2048 + (XT_COLS + 1) * XT_ROWB;
      }
      ph.ostride = op.kind == PWG_CNET_CONVT ? op.stride : 1;
      ph.ophase = r;
      if (op.kind == PWG_CNET_CONVT) {
        ph.k_a = (r + op.padding) % op.stride;
        ph.off_a = (r + op.padding) / op.stride;
        const int cs = (op.src[0].channels + CN_CHUNK - 1) / CN_CHUNK;
        for (int k = 0; k < 2; ++k)
          for (int c = 0; c < cs; ++c) ph.chunks.push_back({0, ph.off_a - k, c * CN_CHUNK, 0});
      } else {
        ph.k_a = ph.off_a = 0;
        for (int s = 0; s < nsrc; ++s) {
          const PwgCnetSrc& src = op.src[s];
          const int cs = (src.channels + CN_CHUNK - 1) / CN_CHUNK;
          for (int k = 0; k < src.taps; ++k)
            for (int c = 0; c < cs; ++c) ph.chunks.push_back({s, -src.pad + k * src.dilation, c * CN_CHUNK, 0});
        }
      }
      ph.n_real_chunks = (int)ph.chunks.size();
      while (ph.chunks.size() % CN_G) ph.chunks.push_back(ph.chunks.back());  // zero-weight padding
      if (ph.chunks.size() > (size_t)CN_MAX_CHUNKS) { delete n; return fail(PWG_ERR_UNSUPPORTED, where + "K too large"); }
      if (op.kind == PWG_CNET_CONV && op.out_channels <= 8 && n->ld[op.dst] <= 16) {
        ph.thin = true;
        int base = 0;
        for (int s2 = 0; s2 < nsrc; ++s2) {
          const PwgCnetSrc& src = op.src[s2];
          const int lo = std::min(-src.pad, -src.pad + (src.taps - 1) * src.dilation);
          const int hi = std::max(-src.pad, -src.pad + (src.taps - 1) * src.dilation);
          ph.thin_taps[s2] = src.taps;
          ph.thin_nc[s2] = (src.channels + CN_CHUNK - 1) / CN_CHUNK;
          ph.thin_base[s2] = base;
          ph.thin_off_min[s2] = lo;
          ph.thin_span[s2] = CN_COLS + hi - lo;
          base += src.taps * ph.thin_nc[s2];
          if (ph.thin_span[s2] > THIN_MAX_SPAN) ph.thin = false;
        }
      }
      for (const ChunkDesc& cd : ph.chunks)
        if (cd.c0 + CN_CHUNK > n->ld[op.src[cd.src].buf]) {
          delete n;
          return fail(PWG_ERR_UNSUPPORTED, where + "source channel padding too small");
        }
      ph.frag_off = off;
      off += (long long)ph.chunks.size() * mt_total * 512;
      ph.frag16_off = off;
      off += (long long)ph.chunks.size() * mt_total * 512;
      ph.bias_off = off;
      off += (long long)mt_total * 32;
      n->phases.push_back(ph);
    }
  }
  n->packed_count = off;
  // ConvTranspose phases run as ONE launch (gridDim.z = stride) on the tap-major kernel: a launch
  // per phase left most of the chip idle (MB-MelGAN's x8 upsample: 8 launches of ~380 workgroups)
  for (size_t i = 0; i < n->phases.size(); ++i) {
    OpPhase& ph = n->phases[i];
    const PwgCnetOp& op = n->ops[ph.op];
    if (op.kind != PWG_CNET_CONVT || ph.phase != 0) continue;
    const int s2 = op.stride;
    bool ok = s2 <= 8 && i + s2 <= n->phases.size() && !ph.thin && (!ph.xtile || CNET_CT_ZMERGE);
    for (int r = 1; ok && r < s2; ++r) {
      const OpPhase& q = n->phases[i + r];
      ok = q.op == ph.op && q.phase == r && q.MT == ph.MT && q.NW == ph.NW && !q.thin &&
           q.chunks.size() == ph.chunks.size() && q.mt_total == ph.mt_total;
    }
    if (!ok) continue;
    ph.z_phases = s2;
    for (int r = 1; r < s2; ++r) n->phases[i + r].z_phases = 0;
  }
  // Fusable pairs (pwg_cnet_pair_kernel): op A = single-source zero-padded conv C_in -> C writing t
  // with no residual / accumulate / division / post activation; the next op B = single-source
  // zero-padded conv C -> C reading t, taps within +-PR_HALO; nobody else reads t.
  for (size_t i = 0; i + 1 < n->phases.size(); ++i) {
    const OpPhase& pa = n->phases[i];
    const OpPhase& pb = n->phases[i + 1];
    if (pb.op != pa.op + 1) continue;
    const PwgCnetOp& A = n->ops[pa.op];
    const PwgCnetOp& B = n->ops[pb.op];
    const int C = A.out_channels;
    if (A.kind != PWG_CNET_CONV || B.kind != PWG_CNET_CONV || pa.thin || pb.thin) continue;
    if (A.src[1].buf >= 0 || B.src[1].buf >= 0 || B.src[0].buf != A.dst) continue;
    if (A.res >= 0 || A.accumulate || A.out_div != 1.f || A.post_act != PWG_ACT_NONE) continue;
    if (A.src[0].pad_mode != PWG_PAD_ZERO || A.src[0].normalize || B.src[0].pad_mode != PWG_PAD_ZERO) continue;
    // 32 channels: both convs' weights resident in LDS; 64: weights streamed in PR_SG-chunk groups
    if ((C != 32 && C != CNET_PAIR_STREAM_C) || A.src[0].channels != C ||
        n->ld[A.src[0].buf] != C || B.out_channels != C || B.src[0].channels != C || n->ld[A.dst] != C)
      continue;
    const int MT = C / 32, cs = C / 16;
    const bool resident = C == 32;
    const int step = C == 128 ? 64 : 128, sg = C == 128 ? 2 : PR_SG;  // streamed kernel geometry
    if (pa.mt_total != MT || pb.mt_total != MT || pa.MT != MT || pb.MT != MT) continue;
    bool ok = true;
    int mn = 1 << 30, mx = -(1 << 30);
    for (const ChunkDesc& cd : pa.chunks) { mn = std::min(mn, cd.row_off); mx = std::max(mx, cd.row_off); }
    for (size_t c = 0; c < pa.chunks.size(); ++c)
      ok = ok && pa.chunks[c].row_off == -A.src[0].pad + (int)(c / cs) * A.src[0].dilation && pa.chunks[c].c0 == 16 * (int)(c % cs);
    for (size_t c = 0; c < pb.chunks.size(); ++c)
      ok = ok && pb.chunks[c].row_off == -B.src[0].pad + (int)(c / cs) * B.src[0].dilation && pb.chunks[c].c0 == 16 * (int)(c % cs);
    if (!resident) ok = ok && pa.chunks.size() % sg == 0 && pb.chunks.size() % sg == 0;
    const int xs = step + mx - mn;
    const long long tiles = (long long)(xs + 2 * step) * (2 * C + 8) * 2;
    const long long lds = resident ? (long long)(pa.chunks.size() + pb.chunks.size()) * 2048 + tiles
                                   : tiles + 2LL * sg * MT * 2048;
    if (xs - step > PR_MAX_XS - 128 || lds > PR_MAX_LDS) continue;
    if (B.dst != n_bufs - 1 && n->ld[B.dst] != C) continue;
    ok = ok && n->ld[B.dst] % 4 == 0 && (B.res < 0 || n->ld[B.res] % 4 == 0);
    for (const ChunkDesc& cd : pb.chunks) ok = ok && cd.row_off >= -PR_HALO && cd.row_off <= PR_HALO;
    for (int k = 0; k < n_ops && ok; ++k) {
      if (k == pb.op) continue;
      const PwgCnetOp& o2 = n->ops[k];
      ok = o2.src[0].buf != A.dst && o2.src[1].buf != A.dst && o2.res != A.dst && (k == pa.op || o2.dst != A.dst);
    }
    if (ok) {
      n->phases[i].pair_b = (int)i + 1;
      n->phases[i].pair_xmin = mn;
      n->phases[i].pair_xs = xs;
      n->phases[i].pair_lds = (int)lds;
      n->phases[i].pair_resident = resident;
      n->phases[i].pair_step = step;
    }
  }
  // Fusable ResidualStacks (pwg_cnet_stack_kernel): op A = single-source conv X -> H with no
  // residual / accumulate / division / post activation; the next op B = 1x1 over [H; X] (taps 1,
  // no padding); nobody else reads H; both ops have the same rows (<= 7 m-tiles: the fused kernel
// covers all of them) and the h tile fits LDS.
  for (size_t i = 0; i + 1 < n->phases.size(); ++i) {
    OpPhase& pa = n->phases[i];
    const OpPhase& pb = n->phases[i + 1];
    if (pa.pair_b >= 0 || pb.op != pa.op + 1) continue;
    const PwgCnetOp& A = n->ops[pa.op];
    const PwgCnetOp& B = n->ops[pb.op];
    if (A.kind != PWG_CNET_CONV || B.kind != PWG_CNET_CONV || pa.thin || pb.thin ||
        (pa.NW != 4 && !pa.xtile))
      continue;
    if (A.src[1].buf >= 0 || A.res >= 0 || A.accumulate || A.out_div != 1.f || A.post_act != PWG_ACT_NONE) continue;
    const PwgCnetSrc& b0 = B.src[0];
    const PwgCnetSrc& b1 = B.src[1];
    if (b0.buf != A.dst || b1.buf != A.src[0].buf || b0.taps != 1 || b1.taps != 1 || b0.pad != 0 || b1.pad != 0) continue;
    if (b0.channels != A.out_channels || b1.channels != A.src[0].channels || b0.normalize) continue;
    // the fused kernel covers every row in one workgroup: measured faster than the two ops up to
    // 96 channels (MB-MelGAN v2: 48 ch 0.49 -> 0.31 ms, 96 ch 0.535 -> 0.50 ms per stack) and
    // slower at 192 (0.43 -> 0.61 ms: one 126 KB-LDS workgroup per CU), profiles/r02_stack
    if (pa.mt_total != pb.mt_total || pa.mt_total > CNET_STACK_MAX_MT) continue;
    if (B.dst != n_bufs - 1 && n->ld[B.dst] % 4 != 0) continue;
    bool ok = true;
    for (int k = 0; k < n_ops && ok; ++k) {
      if (k == pb.op || k == pa.op) continue;
      const PwgCnetOp& o2 = n->ops[k];
      ok = o2.src[0].buf != A.dst && o2.src[1].buf != A.dst && o2.res != A.dst && o2.dst != A.dst;
    }
    const long long lds = 2LL * pa.mt_total * 512 * 4 + 128LL * 2 * (n->ld[A.dst] + 8) * 2;
    if (!ok || lds > PR_MAX_LDS) continue;
    pa.stack_b = (int)i + 1;
    pa.stack_lds = (int)lds;
    pa.NW = 4;  // the tap-major stack kernel's 128-column blocks (d_blocks)
    // x-tile on: the stack on the x-tile scheme (k = 3, all rows in one tile, h tile + staging in LDS);
    // op A unfused runs the x-tile kernel over the same 256-column blocks (d_xblocks)
    if (pa.xtile && A.src[0].taps == 3 && pa.MT == pa.mt_total) {
      // LDS = A region (stage 1: all taps of one block; stage 2: g2 chunks) + max(input rows, h
      // tile); g2 = the largest divisor of op B's chunks that keeps the smallest layout's
      // occupancy (two workgroups per CU when it fits 80 KB)
      const int span = XT_COLS + 2 * A.src[0].dilation;
      const int region = std::max(span * XT_ROWB, 256 * (4 * n->ld[A.dst] + 16));
      const int a1 = 3 * pa.MT * 2048;
      const int n2 = (int)pb.chunks.size();
      const int budget = a1 + region <= PR_MAX_LDS / 2 ? PR_MAX_LDS / 2 : PR_MAX_LDS;
      int g2 = 0;
      for (int g = 1; g <= std::min(n2, XS_G2MAX); ++g)
        if (n2 % g == 0 && std::max(a1, g * pa.MT * 2048) + region <= budget) g2 = g;
      if (g2 > 0) {
        pa.xstack_g2 = g2;
        pa.xstack_xoff = std::max(a1, g2 * pa.MT * 2048);
        pa.xstack_lds = pa.xstack_xoff + region;
      }
    }
    if (pa.xstack_lds == 0) pa.xtile = false;
    // the batched stack kernel (pwg_rstack.hip): C = 16 cs channels in and out of both ops, y rows of
    // exactly C floats, op B with the executor's chunk order [h blocks][x blocks] and no epilogue
    // extras, conv A's taps within the kernel's row window
    if (pa.xtile && pa.xstack_lds > 0) {
      const int C = A.out_channels, cs = C / 16;
      const PwgCnetSrc& xa = A.src[0];
      bool rs = C % 16 == 0 && rstack_supported(cs) && xa.channels == C && B.out_channels == C &&
                pa.MT == (cs + 1) / 2 && n->ld[B.dst] == C && n->ld[xa.buf] % 4 == 0 && n->ld[xa.buf] >= C &&
                !xa.normalize && !b1.normalize && B.res < 0 && !B.accumulate && B.out_div == 1.f &&
                B.post_act == PWG_ACT_NONE && xa.dilation >= 1 && 2 * xa.dilation <= RS_MAX_REACH &&
                xa.pad >= 0 && xa.pad <= 2 * xa.dilation && (int)pb.chunks.size() == 2 * cs;
      for (int c = 0; rs && c < 2 * cs; ++c) {
        const ChunkDesc& cd = pb.chunks[c];
        rs = cd.src == (c < cs ? 0 : 1) && cd.row_off == 0 && cd.c0 == 16 * (c % cs);
      }
      if (rs) pa.rstack_cs = cs;
    }
  }
  // Two-source 1x1s run alone (MelGAN stacks too wide for the fused kernels: 128 / 192 / 256
  // channels) on pwg_r1x1_kernel (PWG_CNET_OPT_RSTACK): [source 0 chunks][source 1 chunks] in the
  // executor's order, each source 16-channel blocks of rows at the op's own rate, y rows of exactly
  // the op's channels, no epilogue extras, LeakyReLU slopes in [0, 1]
  for (size_t i = 0; i < n->phases.size(); ++i) {
    OpPhase& ph = n->phases[i];
    const PwgCnetOp& op = n->ops[ph.op];
    if (op.kind != PWG_CNET_CONV || ph.thin || ph.z_phases != 1 || op.src[1].buf < 0) continue;
    if (i > 0 && n->phases[i - 1].stack_b == (int)i) continue;
    const PwgCnetSrc& s0 = op.src[0];
    const PwgCnetSrc& s1 = op.src[1];
    const int mt = ph.mt_total;
    bool ok = r1x1_supported(mt) && op.out_channels == 32 * mt && n->ld[op.dst] == op.out_channels &&
              op.res < 0 && !op.accumulate && op.out_div == 1.f && op.post_act == PWG_ACT_NONE &&
              op.dst != n_bufs - 1 && ph.ostride == 1 && ph.ophase == 0;
    for (const PwgCnetSrc* sp : {&s0, &s1})
      ok = ok && sp->taps == 1 && sp->pad == 0 && !sp->normalize && sp->channels % 16 == 0 &&
           n->ld[sp->buf] % 4 == 0 && n->ld[sp->buf] >= sp->channels && sp->pre_slope >= 0.f && sp->pre_slope <= 1.f &&
           n->rate[sp->buf] == n->rate[op.dst];
    const int n0 = s0.channels / 16, n1 = s1.channels / 16;
    ok = ok && (int)ph.chunks.size() == n0 + n1;
    for (int c = 0; ok && c < n0 + n1; ++c) {
      const ChunkDesc& cd = ph.chunks[c];
      ok = cd.src == (c < n0 ? 0 : 1) && cd.row_off == 0 && cd.c0 == 16 * (c < n0 ? c : c - n0);
    }
    if (ok) ph.r1x1_mt = mt;
  }
  // k = 3 convs of wide stacks on pwg_rconv_kernel (PWG_CNET_OPT_RSTACK): single source, C in = C
  // out = 32 mt, x rows of >= C floats (multiple of 4), y rows of exactly C, taps within the row window
  for (size_t i = 0; i < n->phases.size(); ++i) {
    OpPhase& ph = n->phases[i];
    const PwgCnetOp& op = n->ops[ph.op];
    if (op.kind != PWG_CNET_CONV || !ph.xtile || ph.thin || ph.z_phases != 1 || op.src[1].buf >= 0) continue;
    if (ph.stack_b >= 0 || ph.xpair_b >= 0 || (i > 0 && n->phases[i - 1].xpair_b == (int)i)) continue;
    const PwgCnetSrc& x = op.src[0];
    const int mt = ph.mt_total;
    const bool ok = r1x1_supported(mt) && op.out_channels == 32 * mt && x.channels == op.out_channels &&
                    n->ld[op.dst] == op.out_channels && n->ld[x.buf] % 4 == 0 && n->ld[x.buf] >= x.channels &&
                    x.taps == 3 && x.dilation >= 1 && 2 * x.dilation <= RS_MAX_REACH && x.pad >= 0 &&
                    x.pad <= 2 * x.dilation && !x.normalize && x.pre_slope >= 0.f && x.pre_slope <= 1.f &&
                    op.res < 0 && !op.accumulate && op.out_div == 1.f && op.post_act == PWG_ACT_NONE &&
                    op.dst != n_bufs - 1 && ph.ostride == 1 && ph.ophase == 0 && n->rate[x.buf] == n->rate[op.dst];
    bool canon = ok && (int)ph.chunks.size() == 3 * mt * 2;
    // chunk order tap-major over blocks: (k, cb) -> k cs + cb, row offset -pad + k dil
    for (int c = 0; canon && c < (int)ph.chunks.size(); ++c) {
      const ChunkDesc& cd = ph.chunks[c];
      const int k = c / (2 * mt), cb = c % (2 * mt);
      canon = cd.src == 0 && cd.c0 == 16 * cb && cd.row_off == -x.pad + k * x.dilation;
    }
    if (canon) ph.rconv_mt = mt;
  }
  // x-tile conv pairs (pwg_cnet_xpair_kernel): both convs on the x-tile kernel, 32 or 64 channels
  // (128 at k = 3) in one row tile, conv 1 single-source zero-padded with no epilogue extras, conv 2 the only
  // reader of its output, same kernel size, dilation 1 and taps within +-16 columns.
  for (size_t i = 0; i + 1 < n->phases.size(); ++i) {
    OpPhase& pa = n->phases[i];
    const OpPhase& pb = n->phases[i + 1];
    if (pb.op != pa.op + 1 || !pa.xtile || !pb.xtile || pa.stack_b >= 0) continue;
    const PwgCnetOp& A = n->ops[pa.op];
    const PwgCnetOp& B = n->ops[pb.op];
    const int C = A.out_channels;
    const bool c128 = C == 128 && A.src[0].taps == 3;
    if ((C != 32 && C != 64 && !c128) || pa.MT != C / 32 || pa.mt_total != pa.MT || pb.MT != pa.MT || pb.mt_total != pb.MT) continue;
    if (A.src[1].buf >= 0 || B.src[1].buf >= 0 || B.src[0].buf != A.dst || A.src[0].channels != C ||
        B.src[0].channels != C || B.out_channels != C || n->ld[A.dst] != C || n->ld[A.src[0].buf] != C)
      continue;
    if (A.res >= 0 || A.accumulate || A.out_div != 1.f || A.post_act != PWG_ACT_NONE) continue;
    if (A.src[0].pad_mode != PWG_PAD_ZERO || B.src[0].pad_mode != PWG_PAD_ZERO || A.src[0].normalize) continue;
    const int K = A.src[0].taps;
    if (B.src[0].taps != K || B.src[0].dilation != 1 || -B.src[0].pad < -16 || -B.src[0].pad + K - 1 > 16) continue;
    if ((K - 1) * A.src[0].dilation > 192 || K > CNET_XPAIR_MAXK) continue;
    if (B.dst != n_bufs - 1 && n->ld[B.dst] % 4 != 0) continue;
    bool ok = true;
    for (int k = 0; k < n_ops && ok; ++k) {
      if (k == pb.op || k == pa.op) continue;
      const PwgCnetOp& o2 = n->ops[k];
      ok = o2.src[0].buf != A.dst && o2.src[1].buf != A.dst && o2.res != A.dst && o2.dst != A.dst;
    }
    const int lds = xpair_lds(pa.MT, K, XT_COLS + (K - 1) * A.src[0].dilation);
    if (!ok || lds > PR_MAX_LDS) continue;
    pa.xpair_b = (int)i + 1;
    pa.xpair_lds = lds;
  }
  // unfused x-tile convs whose prefetching kernel needs > 128 VGPRs (MT >= 3, or MT 2 at k = 11:
  // one workgroup per CU) but whose LDS fits two workgroups per CU: synchronous staging
  for (size_t i = 0; i < n->phases.size(); ++i) {
    OpPhase& ph = n->phases[i];
    const PwgCnetOp& op = n->ops[ph.op];
    if (!ph.xtile || op.kind != PWG_CNET_CONV ||
        ph.stack_b >= 0 || ph.xpair_b >= 0 || (i > 0 && n->phases[i - 1].xpair_b == (int)i) ||
        !xtile_supported(op.src[0].taps))
      continue;
    const int K = op.src[0].taps;
    const int span = XT_COLS + (K - 1) * op.src[0].dilation;
    // DMA-staged variant: two A buffers of one tap group each + the input rows; the fewest tap
    // groups that fit two workgroups per CU (80 KB), else one workgroup per CU
    {
      int opts[4];
      const int nopt = db_ks_options(K, ph.MT, opts);
      for (int pass = 1; pass >= 0; --pass)
        for (int oi2 = 0; oi2 < nopt; ++oi2) {
          const int lds = 2 * opts[oi2] * ph.MT * 2048 + span * XT_ROWB;
          if (lds > (pass == 0 ? 80 * 1024 : 160 * 1024)) continue;
          ph.xt_db = true;
          ph.xt_db_ks[pass] = opts[oi2];
          ph.xt_db_lds[pass] = lds;
          break;
        }
      if (ph.xt_db && ph.xt_db_ks[0] == 0) {  // nothing fits 80 KB: the 160 KB choice for both
        ph.xt_db_ks[0] = ph.xt_db_ks[1];
        ph.xt_db_lds[0] = ph.xt_db_lds[1];
      }
      // measured (r03_dma, same box, bit-identical): DMA staging wins at >= 96 rows per workgroup
      // for k >= 7 (HiFiGAN's 128/256-ch k = 7/11: -3..9 %) and for k = 3 up to 192 channels
      // (MB-MelGAN 192-ch -13..19 %, MelGAN 128-ch -3..13 %); it loses at 256-ch k = 3 (+4..8 %)
      // and at 64-row workgroups
      ph.xt_db_pick = ph.xt_db && ph.MT >= 3 && (K >= 7 || ph.mt_total <= 6);
    }
    if (!(ph.MT >= 3 || (ph.MT == 2 && op.src[0].taps >= 11))) continue;
    if (2 * ph.xt_lds <= 160 * 1024) {
      ph.xt_sync = true;
      ph.xt_ks = K;
    } else if (ph.MT == 4 && K == 11 && 2 * (6 * 4 * 2048 + span * XT_ROWB) <= 160 * 1024) {
      ph.xt_sync = true;
      ph.xt_ks = 6;
      ph.xt_lds = 6 * 4 * 2048 + span * XT_ROWB;
    }
  }
  // Fused residual-stack chains (pwg_mstack.hip, PWG_CNET_OPT_MSTACK): runs of ResidualStacks, each
  // conv A (single-source k = 3 x-tile conv, "same" padding pad = dilation, zero or reflect edges, no
  // epilogue extras) followed by its two-source 1x1 B over [h; x] (B's x source not pre-activated),
  // C a multiple of 16 with every fragment image at C / 32 rounded-up m-tiles, h and every
  // intermediate x read by nobody else, the next stack's conv reading this stack's output.
  auto only_readers = [&](int buf, int op_a, int op_b, int writer) {
    for (int k = 0; k < n_ops; ++k) {
      if (k == op_a || k == op_b || k == writer) continue;
      const PwgCnetOp& o2 = n->ops[k];
      if (o2.src[0].buf == buf || o2.src[1].buf == buf || o2.res == buf || o2.dst == buf) return false;
    }
    return true;
  };
  auto stack_ok = [&](size_t i) {
    if (i + 1 >= n->phases.size()) return false;
    const OpPhase& pa = n->phases[i];
    const OpPhase& pb = n->phases[i + 1];
    if (pb.op != pa.op + 1 || !pa.xtile || pa.thin || pb.thin || pa.z_phases != 1 || pb.z_phases != 1) return false;
    const PwgCnetOp& A = n->ops[pa.op];
    const PwgCnetOp& B = n->ops[pb.op];
    const PwgCnetSrc& a0 = A.src[0];
    const int C = A.out_channels, cs = C / 16, mt = (cs + 1) / 2;
    if (A.kind != PWG_CNET_CONV || B.kind != PWG_CNET_CONV || A.src[1].buf >= 0 || C % 16 != 0 ||
        !mstack_supported(cs, 1))
      return false;
    if (a0.taps != 3 || a0.pad != a0.dilation || a0.channels != C || a0.normalize ||
        (a0.pad_mode != PWG_PAD_ZERO && a0.pad_mode != PWG_PAD_REFLECT))
      return false;
    if (A.res >= 0 || A.accumulate || A.out_div != 1.f || A.post_act != PWG_ACT_NONE) return false;
    const PwgCnetSrc& b0 = B.src[0];
    const PwgCnetSrc& b1 = B.src[1];
    if (b0.buf != A.dst || b1.buf != a0.buf || b0.taps != 1 || b1.taps != 1 || b0.pad != 0 || b1.pad != 0 ||
        b0.channels != C || b1.channels != C || B.out_channels != C || b0.normalize || b1.normalize ||
        b1.pre_slope != 1.f)
      return false;
    if (B.res >= 0 || B.accumulate || B.out_div != 1.f || B.post_act != PWG_ACT_NONE) return false;
    if (n->ld[a0.buf] != C || n->ld[A.dst] != C || n->ld[B.dst] != C || B.dst == n_bufs - 1) return false;
    if (pa.mt_total != mt || pb.mt_total != mt || (int)pb.chunks.size() != 2 * cs) return false;
    for (int c = 0; c < 2 * cs; ++c)  // [h blocks][x blocks], the kernel's fixed chunk order
      if (pb.chunks[c].src != (c >= cs) || pb.chunks[c].c0 != 16 * (c % cs) || pb.chunks[c].row_off != 0) return false;
    return only_readers(A.dst, pa.op, pb.op, pa.op);
  };
  for (size_t i = 0; i < n->phases.size();) {
    if (!stack_ok(i)) {
      ++i;
      continue;
    }
    const int C = n->ops[n->phases[i].op].out_channels;
    int k = 1;  // stacks in the chain
    while (k < MS_MAX && stack_ok(i + 2 * k)) {
      const PwgCnetOp& prevB = n->ops[n->phases[i + 2 * k - 1].op];
      const PwgCnetOp& nextA = n->ops[n->phases[i + 2 * k].op];
      if (nextA.src[0].buf != prevB.dst || nextA.out_channels != C ||
          !only_readers(prevB.dst, n->phases[i + 2 * k].op, n->phases[i + 2 * k + 1].op,
                        n->phases[i + 2 * k - 1].op))
        break;
      ++k;
    }
    OpPhase& head = n->phases[i];
    head.ms_n = k;
    head.ms_halo = 0;
    for (int s = 0; s < k; ++s) head.ms_halo += n->ops[n->phases[i + 2 * s].op].src[0].dilation;
    i += 2 * k;
  }
  *out = n;  // device tables are uploaded by the first plan: packing needs no GPU
  return PWG_OK;
}

void pwg_cnet_destroy(PwgCnet* n) {
  if (!n) return;
  Guard g(n->device);
  for (OpPhase& ph : n->phases)
    if (ph.d_chunks) (void)hipFree(ph.d_chunks);
  for (auto& r : n->records) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
  for (hipEvent_t e : n->pool) (void)hipEventDestroy(e);
  for (auto& kv : n->callers) {
    for (hipStream_t x : kv.second.aux)
      if (x) (void)hipStreamDestroy(x);
    for (hipEvent_t e : kv.second.ev) (void)hipEventDestroy(e);
    if (kv.second.hflag) (void)hipHostFree(kv.second.hflag);
  }
  delete n;
}

long long pwg_cnet_packed_weight_count(const PwgCnet* n) { return n ? n->packed_count : -1; }

int pwg_cnet_pack_weights(const PwgCnet* n, const float* ref, float* packed) {
  if (!n || !ref || !packed) return fail(PWG_ERR_INVALID, "null argument");
  std::memset(packed, 0, sizeof(float) * n->packed_count);
  long long overflow = 0;  // split-f16 weights whose pair would be (inf, -inf)
  for (const OpPhase& ph : n->phases) {
    const PwgCnetOp& op = n->ops[ph.op];
    if (op.kind == PWG_CNET_PQMF) {
      std::memcpy(packed + ph.frag_off, ref + op.src[0].w_off, sizeof(float) * op.stride * op.padding);
      continue;
    }
    // A fragments: [chunk][m][sub][lane][e], k-step i = 4 sub + e pairs channels c0+i / c0+8+i
    for (size_t c = 0; c < (size_t)ph.n_real_chunks; ++c) {
      const ChunkDesc& cd = ph.chunks[c];
      const PwgCnetSrc& src = op.src[cd.src];
      const int tap = op.kind == PWG_CNET_CONVT ? ph.off_a - cd.row_off   // 0 or 1
                                                : (cd.row_off + src.pad) / src.dilation;
      for (int m = 0; m < ph.mt_total; ++m)
        for (int sub = 0; sub < 2; ++sub)
          for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 4; ++e) {
              const int i = 4 * sub + e;
              const int o = 32 * m + (l & 31);
              const int ch = cd.c0 + i + 8 * (l >> 5);
              packed[ph.frag_off + (((size_t)c * ph.mt_total + m) * 2 + sub) * 256 + l * 4 + e] =
                  ref_weight(op, ph, ref, cd.src, o, ch, tap);
            }
      // split-f16 fragments: [chunk][m][hi/lo][lane][4 dwords], lane (cl, hh) dword d = halves of
      // channels c0 + 8hh + 2d, +1 of output row 32m + cl
      uint32_t* p16 = reinterpret_cast<uint32_t*>(packed + ph.frag16_off);
      for (int m = 0; m < ph.mt_total; ++m)
        for (int l = 0; l < 64; ++l)
          for (int d = 0; d < 4; ++d) {
            uint32_t hv = 0, lv = 0;
            for (int e2 = 0; e2 < 2; ++e2) {
              const int o = 32 * m + (l & 31);
              const int ch = cd.c0 + 8 * (l >> 5) + 2 * d + e2;
              const float w = ref_weight(op, ph, ref, cd.src, o, ch, tap);
              overflow += !ph.thin && !(std::fabs(w) < 65520.f);  // the thin kernel reads fp32
              const uint16_t h = cn_f2h(w);
              const uint16_t lo = cn_f2h(w - cn_h2f(h));
              hv |= (uint32_t)h << (16 * e2);
              lv |= (uint32_t)lo << (16 * e2);
            }
            const size_t base = (((size_t)c * ph.mt_total + m) * 2) * 256 + (size_t)l * 4 + d;
            p16[base] = hv;
            p16[base + 256] = lv;
          }
    }
    for (int o = 0; o < op.out_channels; ++o) {
      float b = op.b_off >= 0 ? ref[op.b_off + o] : 0.f;
      if (op.b2_off >= 0) b += ref[op.b2_off + o];
      packed[ph.bias_off + o] = b;
    }
  }
  if (overflow)
    return fail(PWG_ERR_RANGE, std::to_string(overflow) +
                                   " weight(s) beyond the fp16 pair range (|w| >= 65520 or not finite): the image "
                                   "is complete for the exact-fp32 mode only (PWG_CNET_OPT_SPLIT_F16 0)");
  return PWG_OK;
}

int pwg_cnet_plan_create(PwgCnet* n, int n_utts, const long long* frames, PwgCnetPlan** out) {
  if (!n || n_utts < 1 || !frames || !out) return fail(PWG_ERR_INVALID, "bad arguments");
  *out = nullptr;
  const int nb = (int)n->channels.size();
  PwgCnetPlan* p = new PwgCnetPlan();
  p->n = n;
  p->n_utts = n_utts;
  p->pair_steps = n->pair_steps;
  p->frames.assign(frames, frames + n_utts);
  p->rows.assign(nb, 0);
  for (int b = 0; b < nb; ++b) {
    long long base = 0;
    for (int u = 0; u < n_utts; ++u) {
      if (frames[u] < 1) { delete p; return fail(PWG_ERR_INVALID, "every utterance needs >= 1 frame"); }
      base += frames[u] * n->rate[b];
    }
    if (base >= (1LL << 31) / std::max(1, n->ld[b])) { delete p; return fail(PWG_ERR_UNSUPPORTED, "batch too large for one plan"); }
    p->rows[b] = base;
  }
  // reflect padding needs pad < T (torch.nn.ReflectionPad1d raises otherwise)
  for (const PwgCnetOp& op : n->ops)
    for (int s = 0; s < 2; ++s) {
      const PwgCnetSrc& src = op.src[s];
      if (src.buf < 0 || op.kind != PWG_CNET_CONV || src.pad_mode != PWG_PAD_REFLECT) continue;
      const long long reach = std::max<long long>(src.pad, (long long)(src.taps - 1) * src.dilation - src.pad);
      for (int u = 0; u < n_utts; ++u)
        if (reach >= frames[u] * n->rate[src.buf]) {
          delete p;
          return fail(PWG_ERR_INVALID, "reflection padding wider than an utterance (ReflectionPad1d)");
        }
    }
  // Workspace: internal buffers (1 .. nb-2) share storage slots when their live ranges (first
  // write .. last read, in op order) do not overlap and their sizes match; an op never gets a
  // destination that aliases one of its own inputs.
  const int nops = (int)n->ops.size();
  std::vector<int> first_def(nb, nops), last_use(nb, -1);
  for (int oi = 0; oi < nops; ++oi) {
    const PwgCnetOp& op = n->ops[oi];
    first_def[op.dst] = std::min(first_def[op.dst], oi);
    last_use[op.dst] = std::max(last_use[op.dst], oi);
    for (int s2 = 0; s2 < 2; ++s2)
      if (op.src[s2].buf >= 0) last_use[op.src[s2].buf] = std::max(last_use[op.src[s2].buf], oi);
    if (op.res >= 0) last_use[op.res] = std::max(last_use[op.res], oi);
  }
  // (reuse = false: every buffer its own slot, for plans whose independent launches run
  // concurrently -- a shared slot would order them; PWG_CNET_OPT_STREAMS, set below)
  auto assign_slots = [&](bool reuse) {
    struct Slot { size_t off, bytes; int free_after; };
    std::vector<Slot> slots;
    size_t o = 0;
    p->buf_off.assign(nb, SIZE_MAX);
    std::vector<int> order;
    for (int b = 1; b < nb - 1; ++b) order.push_back(b);
    std::sort(order.begin(), order.end(), [&](int x, int y) { return first_def[x] < first_def[y]; });
    for (int b : order) {
      const size_t bytes = ((size_t)p->rows[b] * n->ld[b] * sizeof(float) + 255) / 256 * 256;
      int pick = -1;
      for (size_t si = 0; reuse && si < slots.size(); ++si)
        if (slots[si].bytes == bytes && slots[si].free_after < first_def[b]) { pick = (int)si; break; }
      if (pick < 0) {
        slots.push_back({o, bytes, -1});
        o += bytes;
        pick = (int)slots.size() - 1;
      }
      p->buf_off[b] = slots[pick].off;
      slots[pick].free_after = std::max(last_use[b], first_def[b]);
    }
    p->ws_flag = o;  // after the buffer slots (256-byte aligned)
    p->ws_bytes = o + 256;
  };
  assign_slots(true);
  // Per phase: its columns per utterance, the entry counts of its lists (block list, fused-pair
  // strips, x-tile blocks, narrow blocks) and its launch sizing. The lists themselves are
  // enumerations the descriptor kernel writes into the workspace (CnDescSpec), registered once per
  // distinct (kind, rate, stride, phase, step) -- phases of one rate share them -- and checked below
  // before the plan can run: a bad list (a step or stride that was never set, an entry outside its
  // utterance) fails with PWG_ERR_ASSERT instead of turning into an illegal address in a kernel
  // (round 3's fault: an uninitialised OpPhase field).
  const size_t nph = n->phases.size();
  p->nar_nwv.assign(nph, 0);
  p->nar_mt.assign(nph, 0);
  p->nar_lds.assign(nph, 0);
  p->nar_tap.assign(nph, 0);
  p->nar_xdma.assign(nph, 0);
  p->n_cu = 256;  // host-only handles size for an MI355X
  if (n->device >= 0) {
    if (n->n_cu < 1) {
      int cu = 0;
      if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, n->device) != hipSuccess || cu < 1) {
        delete p;
        return fail(PWG_ERR_HIP, "cannot query the CU count");
      }
      n->n_cu = cu;
    }
    p->n_cu = n->n_cu;
  }
  // DMA-ring launches (PWG_CNET_OPT_NARROW_DMA): one m-tile and 4 waves (128 columns) per workgroup
  // when the utterances are that long. A step's serial cost per wave -- DMA issue (~40 cycles per
  // 1-KB instruction) and the pre-activation / pair split (~180 cycles per 16-B quad) -- shrinks with
  // the waves sharing it while the MFMAs per wave stay; measured per step on HiFiGAN v1's 256-channel
  // k = 11 convs at B = 1 (tools/diag/xdma_probe.py): 1 wave ~4,400 cycles.
  auto xdma_waves = [&](const std::vector<int>& nc) {
    int mx = 0;
    for (int c : nc) mx = std::max(mx, c);
    return mx >= 96 ? 4 : (mx >= 48 ? 2 : 1);
  };
  // ... used while its workgroups fit one round over the CUs; past that (T' = 512: HiFiGAN's
  // 128-channel stage, 1,024 of them) the narrow x-tile kernel's 2-m-tile workgroups reuse each
  // staged input row twice as often and measured faster
  auto xdma_fits = [&](const std::vector<int>& nc, int w, long long mt_groups) {
    long long nwg = 0;
    for (int c : nc) nwg += (c + 32 * w - 1) / (32 * w);
    return nwg * mt_groups <= p->n_cu;
  };
  auto bad_list = [&](size_t pi, const char* what) {
    delete p;
    return fail(PWG_ERR_ASSERT, "internal: plan phase " + std::to_string(pi) + ": " + what);
  };
  long long img_ints = 0;
  auto list = [&](int kind, int rate, int ostride, int ophase, int step) -> int {
    for (const CnDescSpec& sp : p->specs)  // a few dozen distinct lists
      if (sp.kind == kind && sp.rate == rate && sp.ostride == ostride && sp.ophase == ophase && sp.step == step)
        return sp.off;
    long long cnt = 0;
    for (int u = 0; u < n_utts; ++u)
      cnt += cn_list_count(kind, cn_list_cols(kind, frames[u], rate, ostride, ophase), step);
    img_ints = (img_ints + 1) / 2 * 2;  // int2 lists 8-byte aligned
    CnDescSpec sp{kind, rate, ostride, ophase, step, (int)img_ints, 0, 0};
    img_ints += cnt * (kind == CN_L_NCOL ? 1 : 2);
    p->specs.push_back(sp);
    return sp.off;
  };
  for (int b = 0; b < nb; ++b) p->o_seg.push_back(list(CN_L_SEG, n->rate[b], 1, 0, 1));
  std::vector<int> ncols(n_utts, 0);
  auto count = [&](int step) {
    long long c = 0;
    for (int u = 0; u < n_utts; ++u) c += (ncols[u] + step - 1) / step;
    return c;
  };
  for (size_t pi = 0; pi < nph; ++pi) {
    const OpPhase& ph = n->phases[pi];
    const PwgCnetOp& op = n->ops[ph.op];
    const int rate = n->rate[op.dst];
    const bool pq = op.kind == PWG_CNET_PQMF;
    if (!pq && (ph.ostride < 1 || ph.ophase < 0 || ph.ophase >= ph.ostride)) return bad_list(pi, "output stride / phase");
    if (!pq && ph.NW != 4 && ph.NW != 8) return bad_list(pi, "waves per workgroup");
    const int os = pq ? 1 : ph.ostride, oph = pq ? 0 : ph.ophase;
    for (int u = 0; u < n_utts; ++u) ncols[u] = (int)cn_list_cols(CN_L_NCOL, frames[u], rate, os, oph);
    const int blk_step = pq ? 256 : (ph.thin ? CN_COLS : 32 * ph.NW);
    const long long n_blk = count(blk_step);
    if (n_blk > (long long)INT32_MAX / 2) return bad_list(pi, "block count");
    p->o_blocks.push_back(list(CN_L_BLK, rate, os, oph, blk_step));
    p->n_blocks.push_back((int)n_blk);
    p->o_ncols.push_back(pq ? -1 : list(CN_L_NCOL, rate, os, oph, 1));
    if (ph.pair_b >= 0) {
      if (p->pair_steps < 1) return bad_list(pi, "pair strip steps");
      p->o_strips.push_back(list(CN_L_BLK, rate, os, oph, 128 * p->pair_steps));
      p->n_strips.push_back((int)count(128 * p->pair_steps));
    } else {
      p->o_strips.push_back(-1);
      p->n_strips.push_back(0);
    }
    if (ph.xpair_b >= 0 || (ph.stack_b >= 0 && ph.xtile) || ph.xt_convt_db || ph.r1x1_mt > 0) {
      const int step = ph.xpair_b >= 0 ? XP_OUT : XT_COLS;
      p->o_xblocks.push_back(list(CN_L_BLK, rate, os, oph, step));
      p->n_xblocks.push_back((int)count(step));
    } else {
      p->o_xblocks.push_back(-1);
      p->n_xblocks.push_back(0);
    }
    // narrow x-tile launch: phases of the x-tile family (plain x-tile convs, x-tile pair / stack
    // halves, ConvTranspose phases) whose default launch has fewer workgroups than CUs (or all of
    // them with PWG_CNET_OPT_NARROW 2): the widest tile (waves, m-tiles) that gives every CU one
    // workgroup, else the narrowest
    const bool xt_family = !ph.thin && !pq && (ph.xtile || ph.xt_convt_db) && ph.z_phases > 0 && ph.MT >= 1;
    const bool convt = op.kind == PWG_CNET_CONVT;
    // narrow tap-major launch (split-f16 convs outside the x-tile family, e.g. MelGAN's two-source
    // 1x1s; not the fused tap-major pairs / stacks): 1-2 waves, 1-2 m-tiles, CN_NARROW_G chunks per
    // barrier
    const bool tap_family = !xt_family && !ph.thin && !pq && ph.z_phases > 0 && ph.pair_b < 0 &&
                            !(pi > 0 && n->phases[pi - 1].pair_b == (int)pi) && ph.stack_b < 0 && !ph.xt_convt_db;
    const long long zn = ph.z_phases;
    int pick_w = 0, pick_m = 1;
    if (n->narrow && xt_family && (convt || (op.src[0].taps - 1) * op.src[0].dilation <= NARROW_HALO)) {
      const int xk = convt ? 2 : op.src[0].taps, xd = convt ? 1 : op.src[0].dilation;
      long long base = 0;
      if (ph.xpair_b >= 0 || (ph.stack_b >= 0 && ph.xtile)) base = p->n_xblocks[pi];
      else if (ph.xt_convt_db) base = (long long)p->n_xblocks[pi] * (ph.mt_total / ph.MT) * zn;
      else base = n_blk * (ph.mt_total / ph.MT) * zn;
      if (n->narrow == 2 || base < p->n_cu) {
        pick_w = 1;
        // the DMA-ring kernel while its one-m-tile workgroups fit one round over the CUs; past that
        // the narrow x-tile kernel's 2-m-tile workgroups were faster than every DMA-ring form tried
        // (every narrow launch on it: HiFiGAN v1 T' = 512 1.67 -> 1.80 ms; two m-tiles per DMA-ring
        // workgroup: T' = 256 1.23 -> 1.33 ms; profiles/r05_narrow_dma2.json, r05_mt2.json)
        const bool fit1 = xdma_fits(ncols, xdma_waves(ncols), (long long)ph.mt_total * zn);
        if (n->narrow_dma && fit1) {
          pick_w = xdma_waves(ncols);
          pick_m = 1;
          p->nar_xdma[pi] = 1;
        } else {
          bool found = false;
          for (int w : {4, 2, 1}) {
            for (int mtn : {2, 1}) {
              if (mtn == 2 && ph.mt_total % 2 != 0) continue;
              if (count(32 * w) * (ph.mt_total / mtn) * zn >= p->n_cu) {
                pick_w = w;
                pick_m = mtn;
                found = true;
                break;
              }
            }
            if (found) break;
          }
        }
        const int span = 32 * pick_w + (xk - 1) * xd;
        p->nar_lds[pi] = 2 * narrow_ks(xk) * pick_m * 2048 + span * XT_ROWB;
      }
    } else if (n->narrow && tap_family) {
      const long long base = n_blk * (ph.mt_total / ph.MT) * zn;
      if (n->narrow == 2 || base < p->n_cu) {
        pick_w = 1;
        // the DMA-ring kernel (K = 1 mode) unless a source normalizes (the narrow tap-major kernel
        // then runs it, 1-2 waves)
        if (n->narrow_dma && !op.src[0].normalize && !(op.src[1].buf >= 0 && op.src[1].normalize) &&
            ph.chunks.size() <= (size_t)XDMA_CHUNKS_MAX &&
            xdma_fits(ncols, std::min(2, xdma_waves(ncols)), (long long)ph.mt_total * zn)) {
          pick_w = std::min(2, xdma_waves(ncols));  // K = 1 mode: 2 waves keep a 4-chunk step's ring 6 deep
          p->nar_xdma[pi] = 1;
        } else {
          bool found = false;
          for (int w : {2, 1}) {
            for (int mtn : {2, 1}) {
              if (mtn == 2 && ph.mt_total % 2 != 0) continue;
              if (count(32 * w) * (ph.mt_total / mtn) * zn >= p->n_cu) {
                pick_w = w;
                pick_m = mtn;
                found = true;
                break;
              }
            }
            if (found) break;
          }
        }
        p->nar_tap[pi] = 1;
      }
    }
    p->nar_nwv[pi] = pick_w;
    p->nar_mt[pi] = pick_w > 0 ? pick_m : 0;
    p->o_nblocks.push_back(pick_w > 0 ? list(CN_L_BLK, rate, os, oph, 32 * pick_w) : -1);
    p->o_nfr.push_back(pick_w > 0 ? list(CN_L_NFR, rate, os, oph, 32 * pick_w) : -1);
    p->n_nblocks.push_back(pick_w > 0 ? (int)count(32 * pick_w) : 0);
  }
  // fused stack chains (PWG_CNET_OPT_MSTACK): the widest block (a multiple of 32 columns, at most
  // 128) whose first stack's output -- the block plus the later stacks' halos -- is at most one
  // 32-column tile per wave and whose tile, ring and biases fit the LDS. Mode 1 takes a chain when
  // its blocks fit one round over the CUs (the halo recompute costs more than the launches it saves
  // once the blocks queue: MB-MelGAN v2 T' = 512 0.54 -> 0.62 ms) and it has at most 128 channels
  // (the 192-channel chain, one fragment unit per step, measured 0.23 ms against 0.15 ms for its
  // 8 launches at T' = 64; profiles/r05_e)
  p->ms_oc.assign(nph, 0);
  p->o_msblocks.assign(nph, -1);
  p->n_msblocks.assign(nph, 0);
  for (size_t pi = 0; pi < nph; ++pi) {
    const OpPhase& ph = n->phases[pi];
    if (ph.ms_n == 0 || n->mstack == 0 || p->nar_nwv[pi] == 0) continue;
    const PwgCnetOp& A = n->ops[ph.op];
    const int cs = A.out_channels / 16, d0 = A.src[0].dilation, rate = n->rate[A.dst];
    int oc = 0;
    for (int o = 32; o <= 128; o += 32)
      if ((o + 2 * (ph.ms_halo - d0) + 31) / 32 <= 4 && mstack_lds(cs, o, ph.ms_halo, ph.ms_n) <= PR_MAX_LDS) oc = o;
    if (oc == 0 || cs > 8) continue;
    for (int u = 0; u < n_utts; ++u) ncols[u] = (int)(frames[u] * rate);
    if (count(oc) > p->n_cu) continue;
    p->ms_oc[pi] = oc;
    p->o_msblocks[pi] = list(CN_L_BLK, rate, 1, 0, oc);
    p->n_msblocks[pi] = (int)count(oc);
  }
  // A chain's one launch reads its stage input (and, through the halos, neighbouring blocks' columns)
  // for the whole launch while other workgroups write the chain's output: every buffer the chain's
  // ops touch stays live until its last op, or slot reuse could place the output on the input's
  // storage (per-op liveness would free the input after stack 0's 1x1)
  bool chains = false;
  for (size_t pi = 0; pi < nph; ++pi) {
    if (p->ms_oc[pi] == 0) continue;
    chains = true;
    const int last_op = n->phases[pi + 2 * n->phases[pi].ms_n - 1].op;
    for (int k = 0; k < 2 * n->phases[pi].ms_n; ++k) {
      const PwgCnetOp& o2 = n->ops[n->phases[pi + k].op];
      for (int b : {o2.dst, o2.src[0].buf, o2.src[1].buf, o2.res})
        if (b >= 0) last_use[b] = std::max(last_use[b], last_op);
    }
  }
  if (chains) assign_slots(true);
  // Pre-split images: a buffer read by a DMA-ring launch (not inside a fused stack chain) with a
  // LeakyReLU slope gets an image of its rows pre-activated with that slope and pair-split, written
  // by its last writer's epilogue when that writer runs on the DMA-ring kernel too (run time decides:
  // a consumer reads an image only once every launch of the last writer wrote it). At B = 1 every
  // one of a column block's m-tile workgroups converted the same rows each step (~1k of a step's
  // ~2.4k cycles, tools/diag/xdma_probe.py). Two images per buffer at most (MelGAN's x_j: conv A's
  // slope and the 1x1's skip source, slope 1).
  p->ph_simg.assign(2 * nph, -1);
  p->ph_oimg.assign(2 * nph, -1);
  if (n->presplit && n->split_f16 && n->narrow_dma) {
    std::vector<char> in_chain(nph, 0);
    for (size_t pi = 0; pi < nph; ++pi)
      if (cnet_mstack_on(p, pi))
        for (int k = 0; k < 2 * n->phases[pi].ms_n; ++k) in_chain[pi + k] = 1;
    std::vector<int> last_wr(nb, -1);
    for (int oi = 0; oi < nops; ++oi) last_wr[n->ops[oi].dst] = oi;
    auto xdma_phase = [&](size_t q) { return p->nar_xdma[q] && p->nar_nwv[q] > 0 && !in_chain[q]; };
    // narrow x-tile launches (the DMA-staged x-tile kernel) read and, in their epilogue, write images
    // too; whether a phase ends up on those kernels is decided per run (fused pairs / stacks,
    // options), which the run-time image state follows
    auto xtile_reader = [&](size_t q) {
      return n->xtile && p->nar_nwv[q] > 0 && !p->nar_tap[q] && !p->nar_xdma[q] && !in_chain[q];
    };
    auto img_writer = [&](size_t q) { return xdma_phase(q) || xtile_reader(q); };  // (narrow launches)
    for (size_t pi = 0; pi < nph; ++pi) {
      if (!xdma_phase(pi) && !xtile_reader(pi)) continue;
      const PwgCnetOp& op = n->ops[n->phases[pi].op];
      const int nsrc = p->nar_tap[pi] && op.src[1].buf >= 0 && op.kind == PWG_CNET_CONV ? 2 : 1;
      for (int si = 0; si < nsrc; ++si) {
        const PwgCnetSrc& src = op.src[si];
        const int b = src.buf;
        if (b <= 0 || b >= nb - 1 || src.normalize || n->channels[b] % 16 != 0 || last_wr[b] < 0) continue;
        bool writer_dma = false;
        for (size_t q = 0; q < nph; ++q) writer_dma |= n->phases[q].op == last_wr[b] && img_writer(q);
        if (!writer_dma) continue;
        int k = -1, per_buf = 0;
        for (size_t j = 0; j < p->simg_buf.size(); ++j)
          if (p->simg_buf[j] == b) {
            ++per_buf;
            if (p->simg_slope[j] == src.pre_slope) k = (int)j;
          }
        if (k < 0) {
          if (per_buf >= 2) continue;
          k = (int)p->simg_buf.size();
          p->simg_buf.push_back(b);
          p->simg_slope.push_back(src.pre_slope);
          for (size_t q = 0; q < nph; ++q)
            if (n->phases[q].op == last_wr[b]) p->ph_oimg[2 * q + (p->ph_oimg[2 * q] < 0 ? 0 : 1)] = k;
        }
        p->ph_simg[2 * pi + si] = k;
      }
    }
  }
  for (size_t pi = 0; pi < nph; ++pi) p->has_narrow |= p->nar_nwv[pi] > 0;
  if (n->streams == 2 || (n->streams == 1 && p->has_narrow)) assign_slots(false);
  img_ints = (img_ints + 1) / 2 * 2;  // room for a last odd NCOL list's pad int
  if (img_ints >= (1LL << 30)) { delete p; return fail(PWG_ERR_UNSUPPORTED, "batch too large for one plan"); }
  // host image (the descriptor kernel's algorithm), every entry checked: utterance in the batch,
  // first column inside it, frame range and segment rows consistent with the plan
  p->img.assign((size_t)img_ints, 0);
  for (size_t si = 0; si < p->specs.size(); ++si) {
    const CnDescSpec& sp = p->specs[si];
    if (sp.kind < CN_L_SEG || sp.kind > CN_L_NFR || sp.rate < 1 || sp.ostride < 1 || sp.ophase < 0 ||
        sp.ophase >= sp.ostride || sp.step < 1)
      return bad_list(si, "device list with an unset step / stride");
    long long at = 0, row = 0, f = 0;
    for (int u = 0; u < n_utts; ++u) {
      const long long cols = cn_list_cols(sp.kind, frames[u], sp.rate, sp.ostride, sp.ophase);
      const long long cnt = cn_list_count(sp.kind, cols, sp.step);
      for (long long j = 0; j < cnt; ++j, ++at) {
        int* e = p->img.data() + sp.off;
        if (sp.kind == CN_L_NCOL) { e[at] = (int)cols; continue; }
        e += 2 * at;
        if (sp.kind == CN_L_SEG) { e[0] = (int)row; e[1] = (int)(frames[u] * sp.rate); }
        else if (sp.kind == CN_L_BLK) { e[0] = u; e[1] = (int)(j * sp.step); }
        else { e[0] = (int)f; e[1] = (int)frames[u]; }
        if (sp.kind == CN_L_BLK && (e[1] < 0 || e[1] >= cols)) return bad_list(si, "block past its utterance");
      }
      row += frames[u] * sp.rate;
      f += frames[u];
    }
    if ((size_t)sp.off + (size_t)at * (sp.kind == CN_L_NCOL ? 1 : 2) > p->img.size())
      return bad_list(si, "device list outside the image");
  }
  // descriptor launches: CN_DESC_UTTS utterances x CN_DESC_SPECS lists each, argument blocks
  // prebuilt here (pwg_cnet_run patches the image and flag pointers)
  for (int u0 = 0; u0 < n_utts; u0 += CN_DESC_UTTS) {
    const int nu = std::min(CN_DESC_UTTS, n_utts - u0);
    long long f0 = 0;
    for (int u = 0; u < u0; ++u) f0 += frames[u];
    for (size_t s0 = 0; s0 < p->specs.size(); s0 += CN_DESC_SPECS) {
      CnDescArgs a;
      std::memset(&a, 0, sizeof(a));
      a.n_utts = nu;
      a.u0 = u0;
      a.last = u0 + nu == n_utts;
      a.f0 = (int)f0;
      for (int u = 0; u < nu; ++u) a.frames[u] = (int)frames[u0 + u];
      a.n_specs = (int)std::min<size_t>(CN_DESC_SPECS, p->specs.size() - s0);
      for (int k = 0; k < a.n_specs; ++k) {
        CnDescSpec sp = p->specs[s0 + k];
        for (int u = 0; u < u0; ++u) {
          sp.base_idx += (int)cn_list_count(sp.kind, cn_list_cols(sp.kind, frames[u], sp.rate, sp.ostride, sp.ophase), sp.step);
          sp.base_row += (int)(frames[u] * sp.rate);
        }
        a.specs[k] = sp;
      }
      p->desc.push_back(a);
    }
  }
  p->ws_img = p->ws_bytes;  // after the buffer slots and the flag (256-byte aligned)
  p->ws_bytes = p->ws_img + ((size_t)img_ints * sizeof(int) + 255) / 256 * 256;
  // the pre-split images, each its own region (live from its writer to its last reader: small
  // plans only, the DMA-ring kernel runs where its workgroups fit one round over the CUs)
  for (size_t k = 0; k < p->simg_buf.size(); ++k) {
    const int b = p->simg_buf[k];
    p->simg_off.push_back(p->ws_bytes);
    p->ws_bytes += ((size_t)p->rows[b] * n->channels[b] * 4 + 255) / 256 * 256;
  }
  if (n->device < 0) {  // host-only handle: sizes and lists checked (cannot run)
    p->host_only = true;
    *out = p;
    return PWG_OK;
  }
  // the handle's chunk tables (first plan only: they depend on the program, not the utterances)
  Guard g(n->device);
  if (!g.ok) { delete p; return fail(PWG_ERR_HIP, "hipSetDevice failed"); }
  for (OpPhase& ph : n->phases) {
    if (ph.chunks.empty() || ph.d_chunks) continue;
    hipError_t e = hipMalloc(&ph.d_chunks, sizeof(ChunkDesc) * ph.chunks.size());
    if (e == hipSuccess)
      e = hipMemcpy(ph.d_chunks, ph.chunks.data(), sizeof(ChunkDesc) * ph.chunks.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      if (ph.d_chunks) (void)hipFree(ph.d_chunks);
      ph.d_chunks = nullptr;
      delete p;
      return hipf(e, "chunk table upload");
    }
  }
  *out = p;
  return PWG_OK;
}

void pwg_cnet_plan_destroy(PwgCnetPlan* p) { delete p; }  // host memory only

int pwg_cnet_plan_image(const PwgCnetPlan* p, long long* offset_bytes, long long* n_ints, int* out, long long cap) {
  if (!p || !offset_bytes || !n_ints || (cap > 0 && !out)) return fail(PWG_ERR_INVALID, "null argument");
  *offset_bytes = (long long)p->ws_img;
  *n_ints = (long long)p->img.size();
  if (cap > 0) std::memcpy(out, p->img.data(), sizeof(int) * (size_t)std::min<long long>(cap, (long long)p->img.size()));
  return PWG_OK;
}

long long pwg_cnet_plan_rows(const PwgCnetPlan* p, int buf) {
  if (!p || buf < 0 || buf >= (int)p->rows.size()) return -1;
  return p->rows[buf];
}

long long pwg_cnet_plan_workspace_bytes(const PwgCnetPlan* p) { return p ? (long long)p->ws_bytes : -1; }

int pwg_cnet_run(PwgCnetPlan* p, const float* packed, const float* mel, const float* mean, const float* scale,
                 float* out, void* workspace, void* stream) {
  if (!p || !packed || !mel || !out || !workspace) return fail(PWG_ERR_INVALID, "null argument");
  if (p->host_only) return fail(PWG_ERR_INVALID, "a plan of a host-only handle (device -1) cannot run");
  PwgCnet* n = p->n;
  const int nb = (int)n->channels.size();
  Guard g(n->device);
  if (!g.ok) return fail(PWG_ERR_HIP, "hipSetDevice failed");
  hipStream_t const s_main = (hipStream_t)stream;
  std::vector<float*> bufs(nb);
  bufs[0] = const_cast<float*>(mel);
  bufs[nb - 1] = out;
  for (int b = 1; b < nb - 1; ++b) bufs[b] = (float*)((char*)workspace + p->buf_off[b]);
  int* const img = (int*)((char*)workspace + p->ws_img);
  auto i2 = [&](int off) -> const int2* { return off < 0 ? nullptr : reinterpret_cast<const int2*>(img + off); };
  auto i1 = [&](int off) -> const int* { return off < 0 ? nullptr : img + off; };
  auto seg_of = [&](int b) -> const int* { return img + p->o_seg[b]; };
  const bool fuse = n->fuse_pairs && n->split_f16;
  const bool xt = n->xtile && n->split_f16;
  // split-f16 range flag: zeroed every run (exact-fp32 runs leave it clear), set by the launch that
  // writes the program output
  int* const flag_word = (int*)((char*)workspace + p->ws_flag);
  int* rflag = n->split_f16 ? flag_word : nullptr;
  bool out_checked = false;
  // timing mode 2: one event pair around the whole run on the caller's stream (after the join)
  hipEvent_t run_a = nullptr;
  // (an early return hands the event back to the pool instead of leaking it)
  struct PoolBack {
    std::vector<hipEvent_t>& pool;
    hipEvent_t* e;
    ~PoolBack() {
      if (*e) pool.push_back(*e);
    }
  } run_a_back{n->pool, &run_a};
  if (n->timing == 2) {
    if (!n->pool.empty()) { run_a = n->pool.back(); n->pool.pop_back(); }
    else if (hipEventCreate(&run_a) != hipSuccess) return fail(PWG_ERR_HIP, "event create");
    if (hipEventRecord(run_a, s_main) != hipSuccess) return fail(PWG_ERR_HIP, "timing event");
  }
  // the plan's device lists, and the flag reset (a kernel: graph replays redo it)
  for (size_t k = 0; k < p->desc.size(); ++k) {
    CnDescArgs da = p->desc[k];
    da.img = img;
    da.flag = k == 0 ? flag_word : nullptr;
    hipLaunchKernelGGL(pwg_cnet_desc_kernel, dim3((unsigned)da.n_specs), dim3(256), 0, s_main, da);
    const hipError_t ez = hipGetLastError();
    if (ez != hipSuccess) return hipf(ez, "descriptor kernel launch");
  }
  // a conv pair runs fused unless its convs run on the x-tile kernel (measured faster unfused)
  auto pair_fused = [&](const OpPhase& q) { return fuse && q.pair_b >= 0 && !(xt && q.xtile); };
  // narrow x-tile launch of phase i (plan time; x-tile mode only): an x-tile pair or stack whose
  // first conv runs narrow runs unfused (its second op as its own launch)
  auto narrow = [&](size_t i) { return xt && p->nar_nwv[i] > 0 && !p->nar_tap[i]; };
  auto narrow_tap = [&](size_t i) { return n->split_f16 && p->nar_nwv[i] > 0 && p->nar_tap[i]; };
  // the DMA-ring kernel's row ranges: per-block frames and the buffers' rows per frame
  auto xdma_rows = [&](CnXdmaArgs& xd, size_t i) {
    const PwgCnetOp& o = n->ops[n->phases[i].op];
    xd.bfr = i2(p->o_nfr[i]);
    xd.rate[0] = n->rate[o.src[0].buf];
    xd.rate[1] = o.src[1].buf >= 0 && o.kind == PWG_CNET_CONV ? n->rate[o.src[1].buf] : xd.rate[0];
    xd.rate_dst = n->rate[o.dst];
    xd.rate_res = o.res >= 0 ? n->rate[o.res] : 0;
  };
  // pre-split images: -1 not yet written this run, 1 written by every launch of the buffer's last
  // writer so far, 0 some launch did not (its consumers then stage the fp32 rows)
  std::vector<signed char> img_state(p->simg_buf.size(), -1);
  auto img_ptr = [&](int k) { return (unsigned char*)workspace + p->simg_off[k]; };
  // a DMA-ring launch of phase i: the images it writes; whether its nsrc sources' images are ready
  auto xdma_images = [&](CnXdmaArgs& xd, size_t i, int nsrc) -> bool {
    const PwgCnetOp& o = n->ops[n->phases[i].op];
    xd.n_oimg = 0;
    xd.oimg_rowb = n->channels[o.dst] * 4;
    if ((n->ld[o.dst] & 3) == 0)
      for (int j = 0; j < 2; ++j) {
        const int k = p->ph_oimg[2 * i + j];
        if (k < 0) continue;
        xd.oimg[xd.n_oimg] = img_ptr(k);
        xd.oslope[xd.n_oimg] = p->simg_slope[k];
        ++xd.n_oimg;
      }
    bool pre = n->presplit != 0;
    for (int si = 0; si < 2; ++si) {
      const int k = si < nsrc ? p->ph_simg[2 * i + si] : -1;
      pre &= si >= nsrc || (k >= 0 && img_state[k] == 1);
      xd.simg[si] = k >= 0 ? img_ptr(k) : nullptr;
      xd.simg_rowb[si] = k >= 0 ? n->channels[p->simg_buf[k]] * 4 : 0;
    }
    return pre;
  };
#ifdef PWG_XDMA_PROBE
  auto probe_slot = [](size_t i) { return (int)i; };  // phase index (tools/diag/xdma_probe.py)
#else
  auto probe_slot = [](size_t) { return -1; };
#endif
  const int NS = 1 + PwgCnet::N_AUX;
  {
    const int key = (n->fuse_pairs ? 1 : 0) | (n->split_f16 ? 2 : 0) | (n->xtile ? 4 : 0) | (n->streams << 3);
    std::lock_guard<std::mutex> lk(n->mu);
    if (p->sched_key != key) {
      p->sched = CnSchedule{};
      p->sched_key = -1;
      const int rc = cnet_schedule(p, p->sched);
      if (rc != PWG_OK) return rc;
      p->sched_key = key;
    }
  }
  const CnSchedule& sc = p->sched;
  const std::vector<std::pair<int, int>>& launches = sc.launches;
  const bool conc = sc.conc;
  const std::vector<int>& l_stream = sc.stream;
  const std::vector<int>& l_event = sc.event;
  const std::vector<std::vector<int>>& l_waits = sc.waits;
  const std::vector<size_t>& order = sc.order;
  std::unique_lock<std::mutex> lock(n->mu, std::defer_lock);
  if (conc) lock.lock();  // held for the whole enqueue: the aux streams are the handle's
  std::vector<hipEvent_t>* xev_run = nullptr;
  hipStream_t* aux = nullptr;
  if (conc) {
    const int ne = sc.n_events + 1;  // + the fork event (s_main after the descriptor launch)
    PwgCnet::CallerSet& cs = n->callers[s_main];
    aux = cs.aux;
    std::vector<hipEvent_t>& xev = cs.ev;
    xev_run = &xev;
    while ((int)xev.size() < ne) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail(PWG_ERR_HIP, "event create");
      xev.push_back(e);
    }
    for (int k = 1; k < NS; ++k)
      if (sc.used[k] && !aux[k - 1] && hipStreamCreateWithFlags(&aux[k - 1], hipStreamNonBlocking) != hipSuccess)
        return fail(PWG_ERR_HIP, "auxiliary stream create");
    // fork: the aux streams start after everything queued on the caller's stream so far
    hipEvent_t fork = xev[ne - 1];
    if (hipEventRecord(fork, s_main) != hipSuccess) return fail(PWG_ERR_HIP, "fork event");
    for (int k = 1; k < NS; ++k)
      if (sc.used[k] && hipStreamWaitEvent(aux[k - 1], fork, 0) != hipSuccess)
        return fail(PWG_ERR_HIP, "fork wait");
  }
  auto stream_of = [&](int k) { return k == 0 ? s_main : aux[k - 1]; };
  for (size_t oi = 0; oi < order.size(); ++oi) {
    const size_t L = order[oi];
    const size_t pi = (size_t)launches[L].first;
    const OpPhase& ph = n->phases[pi];
    const PwgCnetOp& op = n->ops[ph.op];
    hipStream_t const s = stream_of(l_stream[L]);
    for (int d : l_waits[L])
      if (hipStreamWaitEvent(s, (*xev_run)[l_event[d]], 0) != hipSuccess) return fail(PWG_ERR_HIP, "dependency wait");
    bool wrote_img = false;  // this launch wrote its phase's pre-split images
    hipEvent_t ea = nullptr, eb = nullptr;
    if (n->timing == 1) {
      for (hipEvent_t* ev : {&ea, &eb}) {
        if (!n->pool.empty()) { *ev = n->pool.back(); n->pool.pop_back(); }
        else if (hipEventCreate(ev) != hipSuccess) return fail(PWG_ERR_HIP, "event create");
      }
      (void)hipEventRecord(ea, s);
    }
    if (cnet_mstack_on(p, pi)) {
      // a fused chain of ph.ms_n ResidualStacks (phases pi .. pi + 2 ms_n - 1) in one launch
      const PwgCnetOp& Bn = n->ops[n->phases[pi + 2 * ph.ms_n - 1].op];
      MstackArgs ma;
      ma.x = bufs[op.src[0].buf]; ma.seg_x = seg_of(op.src[0].buf);
      ma.y = bufs[Bn.dst]; ma.seg_y = seg_of(Bn.dst); ma.ld = n->ld[Bn.dst];
      ma.blocks = i2(p->o_msblocks[pi]); ma.ns = ph.ms_n; ma.oc = p->ms_oc[pi]; ma.halo = ph.ms_halo;
      for (int k = 0; k < MS_MAX; ++k) {
        const int kk = k < ph.ms_n ? k : 0;  // (unused entries: copies of the first)
        const OpPhase& pa = n->phases[pi + 2 * kk];
        const OpPhase& pb = n->phases[pi + 2 * kk + 1];
        const PwgCnetOp& A = n->ops[pa.op];
        const PwgCnetOp& B = n->ops[pb.op];
        MsStack& st = ma.st[k];
        st.wA = packed + pa.frag16_off; st.bA = packed + pa.bias_off;
        st.wB = packed + pb.frag16_off; st.bB = packed + pb.bias_off;
        st.dil = A.src[0].dilation; st.pad = A.src[0].pad; st.mode = A.src[0].pad_mode;
        st.slopeA = A.src[0].pre_slope; st.slopeH = B.src[0].pre_slope;
      }
      if (p->n_msblocks[pi] > 0) {
        const hipError_t ea2 = launch_mstack(ma, op.out_channels / 16, 1, p->n_msblocks[pi], s);
        if (ea2 != hipSuccess) return hipf(ea2, "fused stack chain launch");
      }
    } else if (pair_fused(ph)) {
      if (p->n_strips[pi] > 0) {
        const OpPhase& pb = n->phases[ph.pair_b];
        const PwgCnetOp& opb = n->ops[pb.op];
        CnPairArgs a;
        a.x = bufs[op.src[0].buf]; a.seg_x = seg_of(op.src[0].buf); a.ld_x = n->ld[op.src[0].buf];
        a.slope1 = op.src[0].pre_slope; a.slope2 = opb.src[0].pre_slope;
        a.ch1 = ph.d_chunks; a.n1 = (int)ph.chunks.size(); a.w1 = packed + ph.frag16_off; a.b1 = packed + ph.bias_off;
        a.ch2 = pb.d_chunks; a.n2 = (int)pb.chunks.size(); a.w2 = packed + pb.frag16_off; a.b2 = packed + pb.bias_off;
        a.res = opb.res >= 0 ? bufs[opb.res] : nullptr; a.seg_res = opb.res >= 0 ? seg_of(opb.res) : nullptr;
        a.ld_res = opb.res >= 0 ? n->ld[opb.res] : 0;
        a.y = bufs[opb.dst]; a.seg_y = seg_of(opb.dst); a.ld_y = n->ld[opb.dst];
        a.accumulate = opb.accumulate; a.out_div = opb.out_div; a.post_act = opb.post_act; a.post_slope = opb.post_slope;
        a.strips = i2(p->o_strips[pi]); a.ncols = i1(p->o_ncols[pi]); a.steps = p->pair_steps * 128 / ph.pair_step;
        a.x_min_off = ph.pair_xmin; a.xs = ph.pair_xs;
        a.off1 = -op.src[0].pad; a.dil1 = op.src[0].dilation; a.off2 = -opb.src[0].pad; a.dil2 = opb.src[0].dilation;
        if (!n->pair_attr_set) {
          for (const void* kf : {reinterpret_cast<const void*>(pwg_cnet_pair_kernel),
                                 reinterpret_cast<const void*>(pwg_cnet_pair_stream_kernel<1, 4, PR_SG>),
                                 reinterpret_cast<const void*>(pwg_cnet_pair_stream_kernel<2, 4, PR_SG>),
                                 reinterpret_cast<const void*>(pwg_cnet_pair_stream_kernel<4, 2, 2>)}) {
            const hipError_t ea2 = allow_lds(kf, PR_MAX_LDS);
            if (ea2 != hipSuccess) return hipf(ea2, "pair kernel LDS attribute");
          }
          n->pair_attr_set = true;
        }
        const dim3 pgrid((unsigned)p->n_strips[pi]);
        if (ph.pair_resident)
          hipLaunchKernelGGL(pwg_cnet_pair_kernel, pgrid, dim3(256), (size_t)ph.pair_lds, s, a);
        else if (ph.mt_total == 1)
          hipLaunchKernelGGL((pwg_cnet_pair_stream_kernel<1, 4, PR_SG>), pgrid, dim3(256), (size_t)ph.pair_lds, s, a);
        else if (ph.mt_total == 2)
          hipLaunchKernelGGL((pwg_cnet_pair_stream_kernel<2, 4, PR_SG>), pgrid, dim3(256), (size_t)ph.pair_lds, s, a);
        else
          hipLaunchKernelGGL((pwg_cnet_pair_stream_kernel<4, 2, 2>), pgrid, dim3(256), (size_t)ph.pair_lds, s, a);
      }
    } else if (fuse && ph.stack_b >= 0 && !narrow(pi)) {
      if (p->n_blocks[pi] > 0) {
        const bool xs_on = xt && ph.xtile;
        const OpPhase& pb = n->phases[ph.stack_b];
        const PwgCnetOp& opb = n->ops[pb.op];
        CnStackArgs a;
        auto src_args = [&](const PwgCnetSrc& src, CnSrc& d) {
          d = CnSrc{};
          d.x = bufs[src.buf]; d.seg = seg_of(src.buf); d.ld = n->ld[src.buf];
          d.pad_mode = src.pad_mode;
          d.normalize = src.normalize && mean && scale;
          d.slope = src.pre_slope;
        };
        src_args(op.src[0], a.x1);
        src_args(opb.src[1], a.x2);
        a.ch1 = ph.d_chunks; a.n1 = (int)ph.chunks.size(); a.w1 = packed + ph.frag16_off; a.b1 = packed + ph.bias_off;
        a.slope_h = opb.src[0].pre_slope; a.ldh = n->ld[op.dst];
        a.ch2 = pb.d_chunks; a.n2 = (int)pb.chunks.size(); a.w2 = packed + pb.frag16_off; a.b2 = packed + pb.bias_off;
        a.res = opb.res >= 0 ? bufs[opb.res] : nullptr; a.seg_res = opb.res >= 0 ? seg_of(opb.res) : nullptr;
        a.ld_res = opb.res >= 0 ? n->ld[opb.res] : 0;
        a.y = bufs[opb.dst]; a.seg_y = seg_of(opb.dst); a.ld_y = n->ld[opb.dst]; a.M = opb.out_channels;
        a.accumulate = opb.accumulate; a.out_div = opb.out_div; a.post_act = opb.post_act; a.post_slope = opb.post_slope;
        a.blocks = xs_on ? i2(p->o_xblocks[pi]) : i2(p->o_blocks[pi]); a.ncols = i1(p->o_ncols[pi]);
        a.mean = mean; a.scale = scale;
        if (xs_on) {
          CnXstackArgs xs;
          xs.K1 = op.src[0].taps; xs.dil1 = op.src[0].dilation; xs.off1 = -op.src[0].pad;
          xs.cs1 = op.src[0].channels / 16; xs.span1 = XT_COLS + (xs.K1 - 1) * xs.dil1; xs.g2 = ph.xstack_g2;
          xs.x_off = ph.xstack_xoff;
          if (n->rstack && ph.rstack_cs > 0) {
            RstackArgs r;
            r.x = a.x1.x; r.seg_x = a.x1.seg; r.ld_x = a.x1.ld; r.mode_x = a.x1.pad_mode;
            r.dil = xs.dil1; r.off = xs.off1; r.slope1 = a.x1.slope;
            r.mode_2 = a.x2.pad_mode; r.slope2 = a.x2.slope; r.slope_h = a.slope_h;
            r.wA = a.w1; r.bA = a.b1; r.wB = a.w2; r.bB = a.b2;
            r.y = a.y; r.seg_y = a.seg_y;
            r.blocks = a.blocks; r.ncols = a.ncols; r.n_blocks = p->n_xblocks[pi];
            // persistent workgroups, one per CU (the ring fills the LDS), each a contiguous range
            const int n_wg = std::max(std::min(r.n_blocks, std::max(p->n_cu, 1)), (r.n_blocks + RS_MAX_TILES - 1) / RS_MAX_TILES);
            const hipError_t ea2 = launch_rstack(r, ph.rstack_cs, n_wg, s, n->rstack == 1);
            if (ea2 != hipSuccess) return hipf(ea2, "rstack kernel launch");
          } else {
            const hipError_t ea2 =
                xstack_launch(ph.MT, xs.K1, dim3((unsigned)p->n_xblocks[pi]), ph.xstack_lds, s, a, xs);
            if (ea2 != hipSuccess) return hipf(ea2, "xstack kernel launch");
          }
        } else {
        const void* kf = nullptr;
        switch (ph.mt_total) {
          case 1: kf = reinterpret_cast<const void*>(pwg_cnet_stack_kernel<1>); break;
          case 2: kf = reinterpret_cast<const void*>(pwg_cnet_stack_kernel<2>); break;
          case 3: kf = reinterpret_cast<const void*>(pwg_cnet_stack_kernel<3>); break;
          case 4: kf = reinterpret_cast<const void*>(pwg_cnet_stack_kernel<4>); break;
          case 5: kf = reinterpret_cast<const void*>(pwg_cnet_stack_kernel<5>); break;
          case 6: kf = reinterpret_cast<const void*>(pwg_cnet_stack_kernel<6>); break;
          default: kf = reinterpret_cast<const void*>(pwg_cnet_stack_kernel<7>); break;
        }
        const hipError_t ea2 = allow_lds(kf, ph.stack_lds);
        if (ea2 != hipSuccess) return hipf(ea2, "stack kernel LDS attribute");
        const dim3 sgrid((unsigned)p->n_blocks[pi]);
        switch (ph.mt_total) {
          case 1: hipLaunchKernelGGL(pwg_cnet_stack_kernel<1>, sgrid, dim3(256), (size_t)ph.stack_lds, s, a); break;
          case 2: hipLaunchKernelGGL(pwg_cnet_stack_kernel<2>, sgrid, dim3(256), (size_t)ph.stack_lds, s, a); break;
          case 3: hipLaunchKernelGGL(pwg_cnet_stack_kernel<3>, sgrid, dim3(256), (size_t)ph.stack_lds, s, a); break;
          case 4: hipLaunchKernelGGL(pwg_cnet_stack_kernel<4>, sgrid, dim3(256), (size_t)ph.stack_lds, s, a); break;
          case 5: hipLaunchKernelGGL(pwg_cnet_stack_kernel<5>, sgrid, dim3(256), (size_t)ph.stack_lds, s, a); break;
          case 6: hipLaunchKernelGGL(pwg_cnet_stack_kernel<6>, sgrid, dim3(256), (size_t)ph.stack_lds, s, a); break;
          default: hipLaunchKernelGGL(pwg_cnet_stack_kernel<7>, sgrid, dim3(256), (size_t)ph.stack_lds, s, a); break;
        }
        }
      }
    } else if (op.kind == PWG_CNET_PQMF) {
      CnPqmfArgs a;
      a.x = bufs[op.src[0].buf]; a.seg_src = seg_of(op.src[0].buf); a.ld_src = n->ld[op.src[0].buf];
      a.h = packed + ph.frag_off; a.y = bufs[op.dst]; a.seg_dst = seg_of(op.dst); a.ld_dst = n->ld[op.dst];
      a.blocks = i2(p->o_blocks[pi]); a.S = op.stride; a.NT = op.padding;
      a.range_flag = op.dst == nb - 1 ? rflag : nullptr;
      out_checked |= op.dst == nb - 1;
      hipLaunchKernelGGL(pwg_cnet_pqmf_kernel, dim3((unsigned)p->n_blocks[pi]), dim3(256), 0, s, a);
    } else if (p->n_blocks[pi] > 0) {
      CnConvArgs a;
      a.range_flag = nullptr;
      a.xcd_order = n->xcd_order;
      a.n_oimg = 0;
      a.oimg_rowb = n->channels[op.dst] * 4;
      const int nsrc = (op.src[1].buf >= 0 && op.kind == PWG_CNET_CONV) ? 2 : 1;
      for (int si = 0; si < 2; ++si) {
        const PwgCnetSrc& src = op.src[si];
        CnSrc& d = a.src[si];
        if (si < nsrc) {
          d.x = bufs[src.buf]; d.seg = seg_of(src.buf); d.ld = n->ld[src.buf];
          d.pad_mode = src.pad_mode;  // CONVT: ZERO, or REPLICATE for the causal form
          d.normalize = src.normalize && mean && scale;  // normalize_before: caller passes stats
          d.slope = src.pre_slope;
          d.taps = ph.thin_taps[si]; d.nc = ph.thin_nc[si]; d.chunk_base = ph.thin_base[si];
          d.off_min = ph.thin_off_min[si]; d.span = ph.thin_span[si];
        } else {
          d = a.src[0];
        }
      }
      a.chunks = ph.d_chunks; a.n_chunks = (int)ph.chunks.size();
      const bool split = n->split_f16 && !ph.thin;
      a.wfrag = packed + (split ? ph.frag16_off : ph.frag_off); a.mt_total = ph.mt_total; a.bias = packed + ph.bias_off;
      a.res = op.res >= 0 ? bufs[op.res] : nullptr; a.seg_res = op.res >= 0 ? seg_of(op.res) : nullptr;
      a.ld_res = op.res >= 0 ? n->ld[op.res] : 0;
      a.y = bufs[op.dst]; a.seg_dst = seg_of(op.dst); a.ld_dst = n->ld[op.dst]; a.M = op.out_channels;
      a.accumulate = op.accumulate; a.out_div = op.out_div; a.post_act = op.post_act; a.post_slope = op.post_slope;
      a.blocks = i2(p->o_blocks[pi]); a.ncols = i1(p->o_ncols[pi]); a.ostride = ph.ostride; a.ophase = ph.ophase;
      a.mean = mean; a.scale = scale;
      for (int r = 0; r < 8; ++r) {
        const OpPhase& q = n->phases[pi + (r < ph.z_phases ? r : 0)];
        a.z_chunks[r] = q.d_chunks;
        a.z_wfrag[r] = packed + (split ? q.frag16_off : q.frag_off);
        a.z_bias[r] = packed + q.bias_off;
      }
      const dim3 grid((unsigned)p->n_blocks[pi], (unsigned)(ph.mt_total / ph.MT), (unsigned)ph.z_phases), block(256);
      if (ph.thin) {
        const dim3 tgrid((unsigned)p->n_blocks[pi]), tblock(CN_COLS);
        const size_t tl = (size_t)std::max(ph.thin_span[0], ph.thin_span[1]) * THIN_ROW * sizeof(float);
        a.range_flag = op.dst == nb - 1 ? rflag : nullptr;
        out_checked |= op.dst == nb - 1;
        const int mt_ = op.out_channels <= 1 ? 1 : (op.out_channels <= 4 ? 4 : 8);
        size_t tl1 = (size_t)a.n_chunks * 2 * mt_ * 8 * sizeof(float);
        for (int si = 0; si < nsrc; ++si) tl1 += (size_t)ph.thin_nc[si] * ph.thin_span[si] * THIN_ROW * sizeof(float);
        if (tl1 <= (size_t)THIN1_LDS) {
          auto go = [&](auto kfn, int tpc) -> hipError_t {
            const hipError_t e1 = allow_lds(reinterpret_cast<const void*>(kfn), (int)tl1);
            if (e1 != hipSuccess) return e1;
            hipLaunchKernelGGL(kfn, tgrid, dim3(CN_COLS * tpc), tl1, s, a, nsrc);
            return hipGetLastError();
          };
          const hipError_t e1 = mt_ == 1 ? go(pwg_cnet_thin1_kernel<1, 1>, 1)
                                : mt_ == 4 ? go(pwg_cnet_thin1_kernel<4, 4>, 4) : go(pwg_cnet_thin1_kernel<8, 4>, 4);
          if (e1 != hipSuccess) return hipf(e1, "thin kernel launch");
        } else if (op.out_channels <= 1) hipLaunchKernelGGL(pwg_cnet_thin_kernel<1>, tgrid, tblock, tl, s, a, nsrc);
        else if (op.out_channels <= 4) hipLaunchKernelGGL(pwg_cnet_thin_kernel<4>, tgrid, tblock, tl, s, a, nsrc);
        else hipLaunchKernelGGL(pwg_cnet_thin_kernel<8>, tgrid, tblock, tl, s, a, nsrc);
      } else
      if (xt && fuse && ph.xpair_b >= 0 && !narrow(pi)) {
        const OpPhase& pb = n->phases[ph.xpair_b];
        const PwgCnetOp& opb = n->ops[pb.op];
        CnXpairArgs xp;
        xp.K1 = op.src[0].taps; xp.dil1 = op.src[0].dilation; xp.off1 = -op.src[0].pad;
        xp.K2 = opb.src[0].taps; xp.off2 = -opb.src[0].pad; xp.cs = op.out_channels / 16;
        xp.span1 = XT_COLS + (xp.K1 - 1) * xp.dil1; xp.slope_h = opb.src[0].pre_slope;
        xp.w2 = packed + pb.frag16_off; xp.b2 = packed + pb.bias_off;
        // conv 2's epilogue fields in a
        a.res = opb.res >= 0 ? bufs[opb.res] : nullptr; a.seg_res = opb.res >= 0 ? seg_of(opb.res) : nullptr;
        a.ld_res = opb.res >= 0 ? n->ld[opb.res] : 0;
        a.y = bufs[opb.dst]; a.seg_dst = seg_of(opb.dst); a.ld_dst = n->ld[opb.dst]; a.M = opb.out_channels;
        a.accumulate = opb.accumulate; a.out_div = opb.out_div; a.post_act = opb.post_act; a.post_slope = opb.post_slope;
        a.blocks = i2(p->o_xblocks[pi]);
        if (p->n_xblocks[pi] > 0) {
          const hipError_t ea2 = xpair_launch(ph.MT, xp.K1, dim3((unsigned)p->n_xblocks[pi]), ph.xpair_lds, s, a, xp);
          if (ea2 != hipSuccess) return hipf(ea2, "xpair kernel launch");
        }
      } else if (xt && (ph.xtile || (ph.xt_convt_db && (n->xt_dma & CNET_DMA_CONVT)))) {
        CnXtileArgs xt;
        xt.simg = nullptr;
        xt.simg_rowb = 0;
        const bool convt = op.kind == PWG_CNET_CONVT;
        xt.K = convt ? 2 : op.src[0].taps; xt.dil = convt ? 1 : op.src[0].dilation;
        xt.off_min = convt ? ph.off_a - 1 : -op.src[0].pad;
        xt.cs = op.src[0].channels / 16; xt.span = XT_COLS + (xt.K - 1) * xt.dil;
        xt.rev = convt ? 1 : 0;
        for (int r = 0; r < 8; ++r)
          xt.z_off[r] = convt && r < ph.z_phases ? n->phases[pi + r].off_a - 1 : xt.off_min;
        dim3 xgrid = grid;
        // stack op A / wide ConvTranspose: 128-column d_blocks belong to the tap-major kernels
        if (ph.stack_b >= 0 || ph.xt_convt_db) {
          a.blocks = i2(p->o_xblocks[pi]);
          xgrid.x = (unsigned)p->n_xblocks[pi];
        }
        hipError_t ea2;
        // pre-split images of a narrow x-tile launch's output (its epilogue; the DMA-ring launches
        // below set their own)
        auto xtile_images = [&]() {
          a.n_oimg = 0;
          if ((n->ld[op.dst] & 3) != 0) return;
          for (int j = 0; j < 2; ++j) {
            const int k = p->ph_oimg[2 * pi + j];
            if (k < 0) continue;
            a.oimg[a.n_oimg] = img_ptr(k);
            a.oslope[a.n_oimg] = p->simg_slope[k];
            ++a.n_oimg;
          }
        };
        if (narrow(pi)) {
          const int nw = p->nar_nwv[pi], mtn = p->nar_mt[pi];
          xt.span = 32 * nw + (xt.K - 1) * xt.dil;
          a.blocks = i2(p->o_nblocks[pi]);
          const dim3 ngrid((unsigned)p->n_nblocks[pi], (unsigned)(ph.mt_total / mtn), (unsigned)ph.z_phases);
          if (p->n_nblocks[pi] == 0) {
            ea2 = hipSuccess;
          } else if (p->nar_xdma[pi] && !a.src[0].normalize) {
            CnXdmaArgs xd;
            xd.dil = xt.dil; xd.cs = xt.cs; xd.n_steps = xt.cs; xd.rev = xt.rev;
            xd.probe_slot = probe_slot(pi);
            xdma_rows(xd, pi);
            for (int r = 0; r < 8; ++r) xd.z_off[r] = xt.z_off[r];
            xd.row0[0] = xd.row0[1] = INT_MIN;
            xd.k1_n0 = -1;
            const bool pre = xdma_images(xd, pi, 1);
            wrote_img = xd.n_oimg > 0;
            ea2 = xdma_launch(mtn, nw, xt.K, pre, ngrid, s, a, xd);
          } else {
            xtile_images();
            wrote_img = a.n_oimg > 0;
            const int k0 = p->ph_simg[2 * pi];
            const bool pre = n->presplit && !a.src[0].normalize && k0 >= 0 && img_state[k0] == 1;
            xt.simg = pre ? img_ptr(k0) : nullptr;
            xt.simg_rowb = pre ? n->channels[p->simg_buf[k0]] * 4 : 0;
            ea2 = xtile_launch_narrow(mtn, nw, xt.K, pre, ngrid, p->nar_lds[pi], s, a, xt);
            a.n_oimg = 0;
          }
        } else if (n->rstack && ph.rconv_mt > 0 && !a.src[0].normalize) {
          RstackArgs r;
          r.x = a.src[0].x; r.seg_x = a.src[0].seg; r.ld_x = a.src[0].ld; r.mode_x = a.src[0].pad_mode;
          r.dil = xt.dil; r.off = xt.off_min; r.slope1 = a.src[0].slope;
          r.mode_2 = 0; r.slope2 = 1.f; r.slope_h = 1.f;
          r.wA = packed + ph.frag16_off; r.bA = packed + ph.bias_off; r.wB = nullptr; r.bB = nullptr;
          r.y = bufs[op.dst]; r.seg_y = seg_of(op.dst);
          r.blocks = a.blocks; r.ncols = a.ncols; r.n_blocks = (int)grid.x;
          const int n_wg = std::max(std::min(r.n_blocks, std::max(p->n_cu, 1)), (r.n_blocks + RS_MAX_TILES - 1) / RS_MAX_TILES);
          ea2 = launch_rconv(r, ph.rconv_mt, n_wg, s);
        } else {
          const bool db = ph.xt_convt_db ||
                          (ph.xt_db && ((n->xt_dma & CNET_DMA_ALL) || ((n->xt_dma & CNET_DMA_RULE) && ph.xt_db_pick)));
          const int dv = (n->xt_dma & CNET_DMA_FEWEST) ? 1 : 0;
          ea2 = db ? xtile_launch(ph.MT, xt.K, false, ph.xt_db_ks[dv], xgrid, ph.xt_db_lds[dv], s, a, xt, true)
                   : xtile_launch(ph.MT, xt.K, ph.xt_sync, ph.xt_ks, xgrid, ph.xt_lds, s, a, xt);
        }
        if (ea2 != hipSuccess) return hipf(ea2, "xtile kernel launch");
      } else if (split && narrow_tap(pi)) {
        a.blocks = i2(p->o_nblocks[pi]);
        const int nw = p->nar_nwv[pi], mtn = p->nar_mt[pi];
        const dim3 ngrid((unsigned)p->n_nblocks[pi], (unsigned)(ph.mt_total / mtn), (unsigned)ph.z_phases);
        if (p->nar_xdma[pi]) {
          CnXdmaArgs xd;  // K = 1 mode: the chunk list, each chunk at its own source and row offset
          xd.dil = 1; xd.cs = 0; xd.n_steps = a.n_chunks; xd.rev = 0;
          xd.probe_slot = probe_slot(pi);
          xdma_rows(xd, pi);
          for (int r = 0; r < 8; ++r) xd.z_off[r] = 0;
          for (int si = 0; si < 2; ++si) {  // the row offset all of source si's chunks share
            int r0 = INT_MIN;
            bool same = true;
            for (const ChunkDesc& c : ph.chunks)
              if (c.src == si) {
                if (r0 == INT_MIN) r0 = c.row_off;
                same &= c.row_off == r0;
              }
            xd.row0[si] = same ? r0 : INT_MIN;
          }
          {  // canonical 1x1 list: [source 0 blocks 0..n0-1][source 1 blocks 0..], row offset 0
            const int nc = (int)ph.chunks.size();
            int n0 = 0;
            while (n0 < nc && ph.chunks[n0].src == 0) ++n0;
            bool canon = true;
            for (int i = 0; i < nc && canon; ++i) {
              const ChunkDesc& c = ph.chunks[i];
              const int src = i >= n0 ? 1 : 0;
              canon = c.src == src && c.row_off == 0 && c.c0 == 16 * (i - (src ? n0 : 0));
            }
            xd.k1_n0 = canon ? n0 : -1;
          }
          const bool pre = xdma_images(xd, pi, nsrc);
          wrote_img = xd.n_oimg > 0 && p->n_nblocks[pi] > 0;
          const hipError_t ea2 = p->n_nblocks[pi] > 0 ? xdma_launch(mtn, nw, 1, pre, ngrid, s, a, xd) : hipSuccess;
          if (ea2 != hipSuccess) return hipf(ea2, "xdma kernel launch");
        } else if (mtn == 1 && nw == 1) hipLaunchKernelGGL((pwg_cnet_conv_kernel<1, 1, CN_NARROW_G, true, 1>), ngrid, dim3(64), 0, s, a);
        else if (mtn == 1) hipLaunchKernelGGL((pwg_cnet_conv_kernel<1, 1, CN_NARROW_G, true, 2>), ngrid, dim3(128), 0, s, a);
        else if (nw == 1) hipLaunchKernelGGL((pwg_cnet_conv_kernel<2, 1, CN_NARROW_G, true, 1>), ngrid, dim3(64), 0, s, a);
        else hipLaunchKernelGGL((pwg_cnet_conv_kernel<2, 1, CN_NARROW_G, true, 2>), ngrid, dim3(128), 0, s, a);
      } else if (split && n->rstack && ph.r1x1_mt > 0 && p->n_xblocks[pi] > 0) {
        R1x1Args r;
        for (int si = 0; si < 2; ++si) {
          const PwgCnetSrc& src = op.src[si];
          r.src[si] = bufs[src.buf]; r.seg[si] = seg_of(src.buf); r.ld[si] = n->ld[src.buf]; r.slope[si] = src.pre_slope;
        }
        r.nch0 = op.src[0].channels / 16; r.nch = r.nch0 + op.src[1].channels / 16;
        r.w = packed + ph.frag16_off; r.bias = packed + ph.bias_off;
        r.y = bufs[op.dst]; r.seg_y = seg_of(op.dst);
        r.blocks = i2(p->o_xblocks[pi]); r.ncols = i1(p->o_ncols[pi]); r.n_blocks = p->n_xblocks[pi];
        const int n_wg = std::max(std::min(r.n_blocks, std::max(p->n_cu, 1)), (r.n_blocks + RS_MAX_TILES - 1) / RS_MAX_TILES);
        const hipError_t ea2 = launch_r1x1(r, ph.r1x1_mt, n_wg, s, n->rstack == 1);
        if (ea2 != hipSuccess) return hipf(ea2, "r1x1 kernel launch");
      } else if (split) {
        switch (ph.MT) {
          case 1:
            if (ph.NW == 8) hipLaunchKernelGGL((pwg_cnet_conv_kernel<1, 1, CN_G, true, 8>), grid, dim3(512), 0, s, a);
            else hipLaunchKernelGGL((pwg_cnet_conv_kernel<1, 1, CN_G, true>), grid, block, 0, s, a);
            break;
          case 2:
            if (ph.NW == 8) hipLaunchKernelGGL((pwg_cnet_conv_kernel<2, 1, CN_G, true, 8>), grid, dim3(512), 0, s, a);
            else hipLaunchKernelGGL((pwg_cnet_conv_kernel<2, 1, CN_G, true>), grid, block, 0, s, a);
            break;
          case 3:
            if (ph.NW == 8) hipLaunchKernelGGL((pwg_cnet_conv_kernel<3, 1, CN_G, true, 8>), grid, dim3(512), 0, s, a);
            else hipLaunchKernelGGL((pwg_cnet_conv_kernel<3, 1, CN_G, true>), grid, block, 0, s, a);
            break;
          default:
            if (ph.NW == 8)
              hipLaunchKernelGGL((pwg_cnet_conv_kernel<4, 1, CN_G, true, 8>), grid, dim3(512), 0, s, a);
            else hipLaunchKernelGGL((pwg_cnet_conv_kernel<4, 1, CN_G, true>), grid, block, 0, s, a);
            break;
        }
      } else {
        // (x-tile phases use 256-column blocks: their exact-fp32 form runs 8-wave workgroups)
        switch (ph.MT) {
          case 1:
            if (ph.NW == 8) hipLaunchKernelGGL((pwg_cnet_conv_kernel<1, 1, CN_G, false, 8>), grid, dim3(512), 0, s, a);
            else hipLaunchKernelGGL((pwg_cnet_conv_kernel<1, 1, CN_G>), grid, block, 0, s, a);
            break;
          case 2:
            if (ph.NW == 8) hipLaunchKernelGGL((pwg_cnet_conv_kernel<2, 1, CN_G, false, 8>), grid, dim3(512), 0, s, a);
            else hipLaunchKernelGGL((pwg_cnet_conv_kernel<2, 1, CN_G>), grid, block, 0, s, a);
            break;
          case 3:
            if (ph.NW == 8) hipLaunchKernelGGL((pwg_cnet_conv_kernel<3, 1, CN_G, false, 8>), grid, dim3(512), 0, s, a);
            else hipLaunchKernelGGL((pwg_cnet_conv_kernel<3, 1, CN_G>), grid, block, 0, s, a);
            break;
          default:
            if (ph.NW == 8) hipLaunchKernelGGL((pwg_cnet_conv_kernel<4, 1, CN_G, false, 8>), grid, dim3(512), 0, s, a);
            else hipLaunchKernelGGL((pwg_cnet_conv_kernel<4, 1, CN_G>), grid, block, 0, s, a);
            break;
        }
      }
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hipf(e, "cnet op launch");
    for (int j = 0; j < 2; ++j) {
      const int k = p->ph_oimg[2 * pi + j];
      if (k >= 0) img_state[k] = wrote_img && img_state[k] != 0 ? 1 : 0;
    }
    if (n->timing == 1) {
      (void)hipEventRecord(eb, s);
      n->records.push_back({ph.op, ea, eb});
    }
    if (l_event[L] >= 0 && hipEventRecord((*xev_run)[l_event[L]], s) != hipSuccess)
      return fail(PWG_ERR_HIP, "dependency event");
  }
  // join: the caller's stream waits for every auxiliary stream's last launch
  if (conc) {
    int tail_of[1 + PwgCnet::N_AUX] = {-1, -1, -1, -1};
    for (size_t L = 0; L < launches.size(); ++L) tail_of[l_stream[L]] = (int)L;
    for (int k = 1; k < NS; ++k)
      if (tail_of[k] >= 0 && hipStreamWaitEvent(s_main, (*xev_run)[l_event[tail_of[k]]], 0) != hipSuccess)
        return fail(PWG_ERR_HIP, "join wait");
  }
  hipStream_t const s = s_main;
  if (rflag && !out_checked && p->rows[nb - 1] > 0) {
    const long long cnt = p->rows[nb - 1] * n->ld[nb - 1];
    const long long nblk = std::min<long long>((cnt + 255) / 256, 4096);
    hipLaunchKernelGGL(pwg_cnet_finite_kernel, dim3((unsigned)nblk), dim3(256), 0, s, (const float*)out, cnt, rflag);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hipf(e, "output range check launch");
  }
  if (run_a != nullptr) {
    hipEvent_t run_b = nullptr;
    if (!n->pool.empty()) { run_b = n->pool.back(); n->pool.pop_back(); }
    else if (hipEventCreate(&run_b) != hipSuccess) return fail(PWG_ERR_HIP, "event create");
    if (hipEventRecord(run_b, s) != hipSuccess) {
      n->pool.push_back(run_b);
      return fail(PWG_ERR_HIP, "timing event");
    }
    n->records.push_back({-1, run_a, run_b});
    run_a = nullptr;  // (recorded: no longer the guard's)
  }
  return PWG_OK;
}

int pwg_cnet_plan_schedule(PwgCnetPlan* p, int cap, int* n_launches, int* phase, int* stream, int* order) {
  if (!p || !n_launches || (cap > 0 && (!phase || !stream || !order))) return fail(PWG_ERR_INVALID, "null argument");
  CnSchedule sc;
  const int rc = cnet_schedule(p, sc);
  if (rc != PWG_OK) return rc;
  *n_launches = (int)sc.launches.size();
  for (int L = 0; L < (int)sc.launches.size() && L < cap; ++L) {
    phase[L] = sc.launches[L].first;
    stream[L] = sc.stream[L];
    order[L] = (int)sc.order[L];
  }
  return PWG_OK;
}

int pwg_cnet_run_status(PwgCnetPlan* p, const void* workspace, void* stream) {
  if (!p || !workspace) return fail(PWG_ERR_INVALID, "null argument");
  Guard g(p->n->device);
  if (!g.ok) return fail(PWG_ERR_HIP, "hipSetDevice failed");
  hipStream_t s = (hipStream_t)stream;
  // a pinned word per caller stream (a copy into pageable memory takes HIP's staged path: ~20-30 us
  // of a B = 1 call, tools/diag/host_overhead.py)
  int* hf = nullptr;
  {
    std::lock_guard<std::mutex> lk(p->n->mu);
    PwgCnet::CallerSet& cs = p->n->callers[s];
    if (!cs.hflag && hipHostMalloc(reinterpret_cast<void**>(&cs.hflag), sizeof(int), hipHostMallocDefault) != hipSuccess) {
      cs.hflag = nullptr;
      return fail(PWG_ERR_HIP, "pinned status word");
    }
    hf = cs.hflag;
  }
  hipError_t e = hipMemcpyAsync(hf, (const char*)workspace + p->ws_flag, sizeof(int), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hipf(e, "cnet run status");
  const int flag = *hf;
  if (flag != 0)
    return fail(PWG_ERR_RANGE,
                "non-finite program output in split-f16 mode: a value left the fp16 pair range upstream (or the "
                "input is not finite); rerun with PWG_CNET_OPT_SPLIT_F16 0 (exact fp32)");
  return PWG_OK;
}

int pwg_cnet_set_option(PwgCnet* n, int option, long long value) {
  if (!n) return fail(PWG_ERR_INVALID, "null handle");
  if (option == PWG_CNET_OPT_PAIR_STEPS) {
    if (value < 1 || value > 4096) return fail(PWG_ERR_INVALID, "pair_steps must be in [1, 4096]");
    n->pair_steps = (int)value;
    return PWG_OK;
  }
  if (option == PWG_CNET_OPT_NARROW) {
    if (value < 0 || value > 2) return fail(PWG_ERR_INVALID, "narrow must be 0, 1 or 2");
    n->narrow = (int)value;
    return PWG_OK;
  }
  int* slot = option == PWG_CNET_OPT_SPLIT_F16   ? &n->split_f16
              : option == PWG_CNET_OPT_FUSE_PAIRS ? &n->fuse_pairs
              : option == PWG_CNET_OPT_XTILE      ? &n->xtile
              : option == PWG_CNET_OPT_XT_DMA     ? &n->xt_dma
              : option == PWG_CNET_OPT_XCD_ORDER  ? &n->xcd_order
              : option == PWG_CNET_OPT_NARROW_DMA ? &n->narrow_dma
              : option == PWG_CNET_OPT_PRESPLIT   ? &n->presplit
                                                  : nullptr;
  if (option == PWG_CNET_OPT_MSTACK) {
    if (value < 0 || value > 1) return fail(PWG_ERR_INVALID, "mstack must be 0 or 1");
    n->mstack = (int)value;
    return PWG_OK;
  }
  if (option == PWG_CNET_OPT_RSTACK) {
    if (value < 0 || value > 2) return fail(PWG_ERR_INVALID, "rstack must be 0, 1 or 2");
    n->rstack = (int)value;
    return PWG_OK;
  }
  if (option == PWG_CNET_OPT_STREAMS) {
    if (value < 0 || value > 2) return fail(PWG_ERR_INVALID, "streams must be 0, 1 or 2");
    n->streams = (int)value;
    return PWG_OK;
  }
  if (!slot) return fail(PWG_ERR_INVALID, "unknown option");
  if (value != 0 && value != 1 && !(option == PWG_CNET_OPT_XT_DMA && value >= 0 && value <= 15))
    return fail(PWG_ERR_INVALID, "option value must be 0 or 1 (PWG_CNET_OPT_XT_DMA: flags 0 - 15)");
  *slot = (int)value;
  return PWG_OK;
}

int pwg_cnet_release_stream(PwgCnet* n, void* stream) {
  if (!n) return fail(PWG_ERR_INVALID, "null handle");
  if (n->device < 0) return PWG_OK;  // host-only handle: nothing per stream
  Guard g(n->device);
  if (!g.ok) return fail(PWG_ERR_HIP, "hipSetDevice failed");
  std::lock_guard<std::mutex> lk(n->mu);
  auto it = n->callers.find((hipStream_t)stream);
  if (it == n->callers.end()) return PWG_OK;
  PwgCnet::CallerSet& cs = it->second;
  // the caller's stream and the set's auxiliary streams drain first (a run may still use them)
  if (stream && hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return fail(PWG_ERR_HIP, "stream synchronize");
  for (hipStream_t x : cs.aux)
    if (x && hipStreamSynchronize(x) != hipSuccess) return fail(PWG_ERR_HIP, "stream synchronize");
  for (hipStream_t x : cs.aux)
    if (x) (void)hipStreamDestroy(x);
  for (hipEvent_t e : cs.ev) (void)hipEventDestroy(e);
  if (cs.hflag) (void)hipHostFree(cs.hflag);
  n->callers.erase(it);
  return PWG_OK;
}

int pwg_cnet_set_timing(PwgCnet* n, int enable) {
  if (!n) return fail(PWG_ERR_INVALID, "null handle");
  if (enable < 0 || enable > 2) return fail(PWG_ERR_INVALID, "timing mode must be 0, 1 or 2");
  n->timing = enable;
  return PWG_OK;
}

int pwg_cnet_timing_collect(PwgCnet* n, double* ms, long long* launches) {
  if (!n || !ms || !launches) return fail(PWG_ERR_INVALID, "null argument");
  Guard g(n->device);
  for (auto& r : n->records) {
    hipError_t e = hipEventSynchronize(r.b);
    float t = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, r.a, r.b);
    if (e != hipSuccess) return hipf(e, "cnet timing");
    if (r.op >= 0) {  // (-1: a whole-run span record of timing mode 2)
      ms[r.op] += t;
      launches[r.op] += 1;
    }
    n->pool.push_back(r.a);
    n->pool.push_back(r.b);
  }
  n->records.clear();
  return PWG_OK;
}

int pwg_cnet_timing_span(PwgCnet* n, double* span_ms) {
  if (!n || !span_ms) return fail(PWG_ERR_INVALID, "null argument");
  *span_ms = 0.0;
  if (n->records.empty()) return PWG_OK;
  Guard g(n->device);
  // every launch of a run starts after the first one's start event (the auxiliary streams' launches
  // all depend on some earlier launch), so offsets from it are >= 0
  hipEvent_t ref = n->records[0].a;
  double lo = 0.0, hi = 0.0;
  for (auto& r : n->records) {
    hipError_t e = hipEventSynchronize(r.b);
    float ta = 0.f, tb = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ta, ref, r.a);
    if (e == hipSuccess) e = hipEventElapsedTime(&tb, ref, r.b);
    if (e != hipSuccess) return hipf(e, "cnet timing span");
    lo = std::min(lo, (double)ta);
    hi = std::max(hi, (double)tb);
  }
  *span_ms = hi - lo;
  return PWG_OK;
}

}  // extern "C"

#ifdef PWG_XDMA_PROBE
// probe builds only: the DMA-ring kernels' workgroup-0 timelines, [slot][XDMA_PROBE_N] words
extern "C" PWG_API int pwg_cnet_debug_probe(unsigned long long* out, int n_words) {
  const int total = XDMA_PROBE_SLOTS * XDMA_PROBE_N;
  if (!out || n_words < total) return PWG_ERR_INVALID;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_xdma_probe), sizeof(unsigned long long) * total) == hipSuccess
             ? PWG_OK : PWG_ERR_HIP;
}
#endif
