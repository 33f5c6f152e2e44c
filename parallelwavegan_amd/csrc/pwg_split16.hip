// Split-f16 residual layer on v_mfma_f32_16x16x32_f16 (PWG_OPT_LAYER_KERNEL = 3).
//
// Same arithmetic as pwg_split.hip (fp32 operands as fp16 hi+lo pairs, three MFMAs per product,
// fp32 accumulate) on the 16x16x32 shape: per wave a 128-row x 32-column block is
// 8 m-tiles x 2 n-tiles of 16x16. On this power-limited chip the 16x16x32 loop delivered 11 % more
// f16 FLOP/s than the 32x32x16 loop at the same tile (tools/mfma_f16_peak.hip, kind 3 vs 1), and
// its K = 32 packs the whole aux term (three products of two frames plus the bias) into one MFMA.
//
// Lane l: c = l & 15 (A row / B column inside a 16-tile), g = l >> 4 (k group: k = 8g + j).
// Accumulator: column c, rows 4g + i.
// Channel of k element (k-step ks, group g, element j), for x (GEMM-1 B) and for the gate values
// (GEMM-2 B) alike:  chan16(ks, g, j) = 16 (2ks + (j >> 2)) + 4g + (j & 3)
// which is exactly the accumulator position (m-tile 2ks + (j >> 2), register j & 3) of lane
// group g: a lane's x pieces are its GEMM-2 out rows and its gate values its GEMM-2 B operand.
//
// Tiled layout (32 columns, 8 KB per tile, 16-B pieces, lane (c, g) of n-tile nt):
//   x     [nt 2][ks 2][hi/lo 2][g 4][c 16][16 B]   piece = 8 fp16 halves of chan16(ks, g, 0..7)
//   skip  [nt 2][ms 4][g 4][c 16][16 B]           piece = fp32 rows 16ms + 4g + 0..3
// so one wave-instruction reads or writes 1 KB contiguous.
// Reference: layers/residual_block.py:102-140, models/parallel_wavegan.py:131-138,160-171.
#include "pwg_internal.h"


namespace pwg {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mma16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

// rows pre-scaled into exp2 arguments (see pwg_split.hip gate())
__device__ __forceinline__ float gate16(float u, float v) {
  u = fminf(u, 64.f);
  const float e1 = __builtin_amdgcn_exp2f(u);
  const float e2 = __builtin_amdgcn_exp2f(v);
  return (1.f - e1) * __builtin_amdgcn_rcpf((1.f + e1) * (1.f + e2));
}

// 8 values -> 4 hi dwords + 4 lo dwords (v_cvt_pk_f16_f32 + v_fma_mix{lo,hi}_f16). NOPS leading
// wait states for MFMA-fresh inputs, trailing s_nop 1 for MFMA consumers (cdna_hip_programming.md
// 5.7 item 2).
template <int NOPS>
__device__ __forceinline__ void split8x(const float (&v)[8], u32x4& hi, u32x4& lo) {
  unsigned h0, h1, h2, h3, l0, l1, l2, l3;
  asm volatile(
      "s_nop %16\n\t"
      "v_cvt_pk_f16_f32 %0, %8, %9\n\t"
      "v_cvt_pk_f16_f32 %1, %10, %11\n\t"
      "v_cvt_pk_f16_f32 %2, %12, %13\n\t"
      "v_cvt_pk_f16_f32 %3, %14, %15\n\t"
      "v_fma_mixlo_f16 %4, %0, -1.0, %8 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %5, %1, -1.0, %10 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %6, %2, -1.0, %12 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %7, %3, -1.0, %14 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %4, %0, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %5, %1, -1.0, %11 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %6, %2, -1.0, %13 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %7, %3, -1.0, %15 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "s_nop 1"
      : "=&v"(h0), "=&v"(h1), "=&v"(h2), "=&v"(h3), "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]), "i"(NOPS));
  hi = u32x4{h0, h1, h2, h3};
  lo = u32x4{l0, l1, l2, l3};
}

// c * (hi + lo) + b for the 8 fp16 pairs of one piece pair, two v_fma_mix_f32 each; trailing
// s_nop 1: the results seed MFMA accumulators.
__device__ __forceinline__ void seed8x(const u32x4 h, const u32x4 l, const f32x4 b0, const f32x4 b1, float c,
                                       float (&o)[8]) {
  asm volatile(
      "v_fma_mix_f32 %0, %8, %16, %12 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %1, %8, %16, %13 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %2, %9, %16, %14 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %3, %9, %16, %15 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %4, %10, %16, %17 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %5, %10, %16, %18 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %6, %11, %16, %19 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %7, %11, %16, %20 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %0, %21, %16, %0 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %1, %21, %16, %1 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %2, %22, %16, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %3, %22, %16, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %4, %23, %16, %4 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %5, %23, %16, %5 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %6, %24, %16, %6 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %7, %24, %16, %7 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "s_nop 1"
      : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]), "=&v"(o[7])
      : "v"(l[0]), "v"(l[1]), "v"(l[2]), "v"(l[3]), "v"(b0[0]), "v"(b0[1]), "v"(b0[2]), "v"(b0[3]), "v"(c),
        "v"(b1[0]), "v"(b1[1]), "v"(b1[2]), "v"(b1[3]), "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]));
}

struct Pair16 {
  unsigned hi, lo;
};
__device__ __forceinline__ Pair16 split_pair16(float v0, float v1) {
  typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
  const _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
  const _Float16 l0 = (_Float16)(v0 - (float)h0), l1 = (_Float16)(v1 - (float)h1);
  return {__builtin_bit_cast(unsigned, f16x2{h0, h1}), __builtin_bit_cast(unsigned, f16x2{l0, l1})};
}

}  // namespace

// dword offset of piece q of column c (n-tile from c) for lane group g; pieces of one n-tile are
// 256 dwords (1 KB) apart
__device__ __forceinline__ size_t row16(int c, int g) {
  return (size_t)(c >> 5) * 2048 + (size_t)((c >> 4) & 1) * 1024 + (size_t)g * 64 + (size_t)(c & 15) * 4;
}

// byte offset of piece q of column c for lane group g (row16 in bytes)
__device__ __forceinline__ unsigned row16_bytes(int c, int g) { return (unsigned)row16(c, g) * 4u; }

// buffer resource over a wave-uniform base (num_records 2 GB: the pipelined path's planes are smaller)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc16(const void* base) {
  const unsigned long long b = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b), hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, 0x7fffffff, 0x00020000);
}
// sc1 (write-through / L1-bypassing) 16-byte accesses: the pipelined kernel's hand-off bytes
// (cdna_hip_programming.md Guideline 16: every store and every load of a handed-off byte is sc1)
constexpr int AUX_SC1 = 16;
__device__ __forceinline__ u32x4 ld16_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX_SC1));
}
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, AUX_SC1);
}

// LDS image of one layer (dwords): GEMM-1 A fragments [tap 3][ks 2][m 8][hi/lo 2][lane 64][4]
// | GEMM-2 [ks 2][m 8][hi/lo 2][lane 64][4] | gate bias pairs [m 8][c 16] | sqrt(.5) b_out [g 4][16]
// | last layer: head W1 [ms 4][m3 4][lane 64][4] fp32 + b1 [g 4][16]; layer 0 with the fused
// first_conv: w[64] | b[64] after that.
struct Split16Smem {
  static constexpr int WG = 3 * 2 * 8 * 2 * 64 * 4;
  static constexpr int W2 = 2 * 8 * 2 * 64 * 4;
  static constexpr int BG = 8 * 16;
  static constexpr int BO = 64;
  static constexpr int HW1 = 4 * 4 * 64 * 4 + 64;
  static constexpr int dwords(bool last) { return WG + W2 + BG + BO + (last ? HW1 : 0); }
};
static_assert(Split16Smem::WG + Split16Smem::W2 + Split16Smem::BG + Split16Smem::BO == SPLIT_LAYER_DWORDS,
              "split16 layer image size");

// Stage one layer's image (and the head / first_conv constants of its role) into LDS; every
// thread of the workgroup calls it, a __syncthreads() follows.
template <bool LAST, bool FIRST>
__device__ __forceinline__ void s16_stage(const SplitArgs& a, unsigned* smem16) {
  const int nthr = blockDim.x;
  stage_lds(reinterpret_cast<u32x4*>(smem16), reinterpret_cast<const u32x4*>(a.wg), SPLIT_LAYER_DWORDS / 4,
            (int)threadIdx.x, nthr);
  if (LAST)
    stage_lds(reinterpret_cast<u32x4*>(smem16 + SPLIT_LAYER_DWORDS), reinterpret_cast<const u32x4*>(a.hw1),
              Split16Smem::HW1 / 4, (int)threadIdx.x, nthr);
  if (FIRST) {
    float* s_fwb = reinterpret_cast<float*>(smem16 + Split16Smem::dwords(LAST));
    for (int i = threadIdx.x; i < 128; i += nthr) s_fwb[i] = i < 64 ? a.fw[i] : a.fb[i - 64];
  }
}

// A lane's tap row pieces of one block for its NTN n-tiles from column h16 on (NTN = 2: both, h16 =
// 0; NTN = 1: one half block): b[nt*4 + ks*2 + hl]. FIRST (layer 0 with
// PWG_OPT_FUSE_FIRST_CONV): first_conv (models/parallel_wavegan.py:81,161, x0 = w z + b, zero
// outside the utterance) is evaluated from the 4-byte noise with the same fmaf and pair split as
// pwg_first_conv_split16_kernel (bit-identical), so x0 never touches HBM. PIPE: sc1 loads.
template <int TC, bool FIRST, bool PIPE, int NTN = 2>
__device__ __forceinline__ void s16_bload(const SplitArgs& a, const float* s_fwb, const BlockDesc& d, int tap,
                                          u32x4 (&b)[8], int g, int c, int h16 = 0) {
  if constexpr (FIRST) {
    const f32x4* fw4 = reinterpret_cast<const f32x4*>(s_fwb) + g;
    const f32x4* fb4 = reinterpret_cast<const f32x4*>(s_fwb + 64) + g;
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) {
      const int t = d.t0 + h16 + 16 * nt + c + (tap - TC) * a.dil;
      const bool inside = t >= 0 && t < d.T;
      const float z = a.noise[d.io_off + (t < 0 ? 0 : (t >= d.T ? d.T - 1 : t))];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float v[8];
#pragma unroll
        for (int jh = 0; jh < 2; ++jh) {
          const f32x4 w = fw4[4 * (2 * ks + jh)], bb = fb4[4 * (2 * ks + jh)];
#pragma unroll
          for (int i = 0; i < 4; ++i) v[4 * jh + i] = inside ? fmaf(w[i], z, bb[i]) : 0.f;
        }
        split8x<0>(v, b[nt * 4 + ks * 2], b[nt * 4 + ks * 2 + 1]);
      }
    }
  } else if constexpr (PIPE) {
    const __amdgpu_buffer_rsrc_t r = rsrc16(a.x_in);
    const int cc = d.col + h16 + (tap - TC) * a.dil;
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) {
      const unsigned off = row16_bytes(cc + 16 * nt + c, g);
#pragma unroll
      for (int q = 0; q < 4; ++q) b[nt * 4 + q] = ld16_sc1(r, off + q * 1024u);
    }
  } else {
    const int cc = d.col + h16 + (tap - TC) * a.dil;
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) {
      const u32x4* p = reinterpret_cast<const u32x4*>(a.x_in + row16(cc + 16 * nt + c, g));
#pragma unroll
      for (int q = 0; q < 4; ++q) b[nt * 4 + q] = p[q * 64];
    }
  }
}

// D rows of a block's aux window: lane group g covers window frames fw0 + 2g, fw0 + 2g + 1 of the
// frame-rate aux projection, in the split16 layout [c 16][m 8] (pwg_aux_proj_kernel, split == 2).
__device__ __forceinline__ void s16_load_dv(const SplitArgs& a, const BlockDesc& bd, unsigned (&dv)[2][8], int g,
                                            int c) {
  const int fw0 = bd.t0 / a.H - a.J1;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int f = fw0 + 2 * g + j;
    const int fc = f < 0 ? 0 : (f >= bd.frames ? bd.frames - 1 : f);  // weight 0 there
    const u32x4* drow = reinterpret_cast<const u32x4*>(a.d + (size_t)(bd.frame_base + fc) * 128 + 8 * c);
    const u32x4 d0 = drow[0], d1 = drow[1];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      dv[j][m] = d0[m];
      dv[j][m + 4] = d1[m];
    }
  }
}

// The old skip sum of a block as GEMM-2 seeds sk[ms][nt] (skip rows 16 ms + 4 g + i of column
// bd.col + 16 nt + c). Layer 0: the sum of all layers' skip biases.
template <bool PIPE, int NTN = 2>
__device__ __forceinline__ void s16_load_skip(const SplitArgs& a, const BlockDesc& bd, f32x4 (&sk)[4][2], int g,
                                              int c, int h16 = 0) {
  [[maybe_unused]] __amdgpu_buffer_rsrc_t rs;
  if constexpr (PIPE) rs = rsrc16(a.skip);
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
    for (int ms = 0; ms < 4; ++ms) {
      if (a.first) {
        sk[ms][nt] = reinterpret_cast<const f32x4*>(a.skip0 + 16 * g)[ms];
      } else if constexpr (PIPE) {
        sk[ms][nt] = __builtin_bit_cast(f32x4, ld16_sc1(rs, row16_bytes(bd.col + h16 + 16 * nt + c, g) + ms * 1024u));
      } else {
        const f32x4* sp = reinterpret_cast<const f32x4*>(a.skip + row16(bd.col + h16 + 16 * nt + c, g));
        sk[ms][nt] = __builtin_nontemporal_load(sp + ms * 64);
      }
    }
}

// One 32-sample block of one WaveNet residual block (layers/residual_block.py:102-140) with the
// skip accumulation (models/parallel_wavegan.py:163-165) and, on the LAST layer, the output head.
// On entry b0 holds tap 0 of `bd`; the other taps, the D rows and the skip seeds load inside the
// block one step ahead of use; with has_next, tap 0 of the next block `bdn` loads into b1 during
// the center tap's MFMAs (the per-layer kernel's cross-block prefetch). `mid` runs once after
// GEMM 1 (the caller issues its next work-queue claim there). PIPE: sc1 skip loads and sc1
// stores of x and skip (hand-off bytes of the pipelined kernel).
// NTN = 1 (half blocks, the small-plan latency path): only n-tile h16 / 16 of `bd` (columns
// bd.col + h16 + [0, 16)); the next unit's half is h16n. Every column's accumulators sum the same
// products in the same order as with NTN = 2, and the aux K slots stay anchored at the 32-sample
// block's first frame: bit-identical per column.
// poison (LAST): the run's earlier layers did not complete (a PWG_STATUS_REDO bit was set when the
// launch started), so the block writes NaN audio instead of a plausible-looking wrong result.
template <bool LAST, int TC, bool FIRST, bool PIPE, int NTN = 2, typename Mid>
__device__ __forceinline__ void s16_block(const SplitArgs& a, const unsigned* smem16, const BlockDesc& bd,
                                          const BlockDesc& bdn, bool has_next, u32x4 (&b0)[8], u32x4 (&b1)[8],
                                          bool& nonfinite, Mid&& mid, int h16 = 0, int h16n = 0,
                                          bool poison = false) {
  static_assert(NTN == 2 || !LAST, "half blocks: middle layers");
  const unsigned* s_wg = smem16;
  const unsigned* s_w2 = s_wg + Split16Smem::WG;
  const unsigned* s_bg = s_w2 + Split16Smem::W2;
  const float* s_bo = reinterpret_cast<const float*>(s_bg + Split16Smem::BG);
  const float* s_hw1 = s_bo + Split16Smem::BO;
  const float* s_fwb = reinterpret_cast<const float*>(smem16 + Split16Smem::dwords(LAST));
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int c = lane & 15;
  constexpr int T1 = TC == 1 ? 2 : 1;  // the non-center tap after tap 0
  const bool full = bd.t0 + h16 + 16 * NTN <= bd.T;

  // aux operands: K slots [Dh0 Dh1 Dl0 Dl1 Dh0 Dh1 bh bl] x [wh0 wh1 wh0 wh1 wl0 wl1 1 1] (bias in
  // group 0 only); bw = the composite upsampler weights of the lane's two window frames
  unsigned dv[2][8];  // [frame][m], loaded during GEMM 1
  float bw[2][2];  // [nt][frame]
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt) {
    const int t = bd.t0 + h16 + 16 * nt + c;
    const bool live = t < bd.T;
    const int tc = live ? t : bd.T - 1;
    int roff;
    if (bd.frames < a.Fmin) roff = a.tab_small + (a.H * bd.frames * (bd.frames - 1) / 2 + tc) * AUX_J4;
    else if (tc < a.TL) roff = a.tab_left + tc * AUX_J4;
    else if (tc >= bd.T - a.TR) roff = a.tab_right + (bd.T - 1 - tc) * AUX_J4;
    else roff = (tc % a.H) * AUX_J4;
    const int shift = t / a.H - bd.t0 / a.H;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int idx = 2 * g + j - shift;
      const bool ok = live && idx >= 0 && idx < AUX_J4;
      const float w = a.tab[roff + (idx < 0 ? 0 : (idx >= AUX_J4 ? AUX_J4 - 1 : idx))];
      bw[nt][j] = ok ? w : 0.f;
    }
  }
  const u32x4* wgl = reinterpret_cast<const u32x4*>(s_wg) + lane;
  auto mma_tap = [&](f32x4 (&acc)[8][2], const u32x4 (&b)[8], int tap) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int mh = 0; mh < 2; ++mh) {  // 4 m-tiles per group: their A fragments read ahead
        u32x4 ah[4], al[4];
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
          const int m = 4 * mh + mm;
          ah[mm] = wgl[(((tap * 2 + ks) * 8 + m) * 2) * 64];
          al[mm] = wgl[(((tap * 2 + ks) * 8 + m) * 2 + 1) * 64];
        }
#pragma unroll
        for (int mm = 0; mm < 4; ++mm)
#pragma unroll
          for (int nt = 0; nt < NTN; ++nt) {
            f32x4& ac = acc[4 * mh + mm][nt];
            ac = mma16(ah[mm], b[nt * 4 + ks * 2], ac);
            ac = mma16(ah[mm], b[nt * 4 + ks * 2 + 1], ac);
            ac = mma16(al[mm], b[nt * 4 + ks * 2], ac);
          }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  // ---- GEMM 1: taps 0, other, center (the center row becomes the GEMM-2 seeds at the end)
  f32x4 acc[8][2];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) acc[m][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc2[8][2];
  s16_bload<TC, FIRST, PIPE, NTN>(a, s_fwb, bd, T1, b1, g, c, h16);
  mma_tap(acc, b0, 0);
  s16_load_dv(a, bd, dv, g, c);
  s16_bload<TC, FIRST, PIPE, NTN>(a, s_fwb, bd, TC, b0, g, c, h16);
  mma_tap(acc, b1, T1);
  mma_tap(acc, b0, TC);
  if (!LAST) {
    // GEMM-2 out-row seeds sqrt(.5)(x + b_out) from the center tap: acc2[4 + 2ks + (j>>2)][nt][j&3]
    const f32x4* bo_l = reinterpret_cast<const f32x4*>(s_bo + 16 * g);
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float o[8];
        seed8x(b0[nt * 4 + ks * 2], b0[nt * 4 + ks * 2 + 1], bo_l[2 * ks], bo_l[2 * ks + 1], 0.70710677f, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc2[4 + 2 * ks + (j >> 2)][nt][j & 3] = o[j];
      }
  }
  mid();

  {
    // skip seeds: old skip sum, in flight during the aux term and the gate
    f32x4 sk[4][2];
    s16_load_skip<PIPE, NTN>(a, bd, sk, g, c, h16);
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
      for (int ms = 0; ms < 4; ++ms) acc2[ms][nt] = sk[ms][nt];
  }

  // ---- aux term + gate bias: one MFMA per (m, nt)
  {
    const Pair16 bias_one = split_pair16(g == 0 ? 1.f : 0.f, g == 0 ? 1.f : 0.f);
    u32x4 bB[2];
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) {
      const Pair16 w = split_pair16(bw[nt][0], bw[nt][1]);
      bB[nt] = u32x4{w.hi, w.hi, w.lo, bias_one.hi};  // [wh0 wh1 | wh0 wh1 | wl0 wl1 | 1 1]
    }
    const unsigned* bgl = s_bg + c;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const unsigned bgp = g == 0 ? bgl[16 * m] : 0u;  // (bias hi | bias lo << 16)
      const unsigned dh = __builtin_amdgcn_perm(dv[1][m], dv[0][m], 0x05040100u);
      const unsigned dl = __builtin_amdgcn_perm(dv[1][m], dv[0][m], 0x07060302u);
      const u32x4 aA = {dh, dl, dh, bgp};  // [Dh0 Dh1 | Dl0 Dl1 | Dh0 Dh1 | bh bl]
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt) acc[m][nt] = mma16(aA, bB[nt], acc[m][nt]);
    }
  }

  // ---- gate -> GEMM-2 B pairs: k-step ks element j = channel chan16(ks, g, j) = acc row
  u32x4 gh[2][2], gl[2][2];  // [nt][ks]
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      float gv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = 2 * ks + (j >> 2), i = j & 3;
        gv[j] = gate16(acc[m][nt][i], acc[m + 4][nt][i]);
      }
      split8x<0>(gv, gh[nt][ks], gl[nt][ks]);
    }

  // the next work unit's tap-0 row, into b0 (dead since the seeds): loaded here, just before
  // GEMM 2, its rows are still in L2 (round 4 per-layer PMC: loading it during the center tap's
  // MFMAs, ~0.7 unit-times earlier, re-read 1.30-1.38x the algorithmic bytes from HBM, here
  // 1.02-1.13x; tools/diag/layer_fetch.sh)
  if (has_next) s16_bload<TC, FIRST, PIPE, NTN>(a, s_fwb, bdn, 0, b0, g, c, h16n);
  // ---- GEMM 2: [skip; out] rows, 8 m-tiles (last layer: the 4 skip tiles)
  constexpr int M2 = LAST ? 4 : 8;
  const u32x4* w2l = reinterpret_cast<const u32x4*>(s_w2) + lane;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int mh = 0; mh < M2 / 4; ++mh) {
      u32x4 ah[4], al[4];
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) {
        ah[mm] = w2l[((ks * 8 + 4 * mh + mm) * 2) * 64];
        al[mm] = w2l[((ks * 8 + 4 * mh + mm) * 2 + 1) * 64];
      }
#pragma unroll
      for (int mm = 0; mm < 4; ++mm)
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt) {
          f32x4& ac = acc2[4 * mh + mm][nt];
          ac = mma16(ah[mm], gh[nt][ks], ac);
          ac = mma16(ah[mm], gl[nt][ks], ac);
          ac = mma16(al[mm], gh[nt][ks], ac);
        }
      __builtin_amdgcn_sched_barrier(0);
    }

  if (!LAST) {
    [[maybe_unused]] __amdgpu_buffer_rsrc_t rsk, rx;
    if constexpr (PIPE) {
      rsk = rsrc16(a.skip);
      rx = rsrc16(a.x_out);
    }
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) {
      const int col = bd.col + h16 + 16 * nt + c;
      const bool live = bd.t0 + h16 + 16 * nt + c < bd.T;
#pragma unroll
      for (int ms = 0; ms < 4; ++ms) {
        if constexpr (PIPE)
          st16_sc1(rsk, row16_bytes(col, g) + ms * 1024u, __builtin_bit_cast(u32x4, acc2[ms][nt]));
        else
          __builtin_nontemporal_store(acc2[ms][nt], reinterpret_cast<f32x4*>(a.skip + row16(col, g)) + ms * 64);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = acc2[4 + 2 * ks + (j >> 2)][nt][j & 3];
        u32x4 vh, vl;
        split8x<11>(v, vh, vl);  // inputs straight from the GEMM-2 MFMAs
        if (!full) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            vh[k] = live ? vh[k] : 0u;
            vl[k] = live ? vl[k] : 0u;
          }
        }
        if constexpr (PIPE) {
          st16_sc1(rx, row16_bytes(col, g) + (ks * 2) * 1024u, vh);
          st16_sc1(rx, row16_bytes(col, g) + (ks * 2 + 1) * 1024u, vl);
        } else {
          u32x4* xp = reinterpret_cast<u32x4*>(a.x_out + row16(col, g));
          __builtin_nontemporal_store(vh, xp + (ks * 2) * 64);
          __builtin_nontemporal_store(vl, xp + (ks * 2 + 1) * 64);
        }
      }
    }
  } else {
    // ---- fused output head (models/parallel_wavegan.py:131-138,166-171), split-f16 on
    //      v_mfma_f32_16x16x32_f16 like the layer: h1 = W1h . relu(skip * sqrt(1/L)) + b1h with
    //      k-step ks element j = skip row chan16(ks, g, j) = acc2[2ks + (j >> 2)][nt][j & 3]
    //      (the W1h image is packed in that k order); then y = W2h . relu(h1) + b2h across the 4
    //      lane groups. (The fp32 v_mfma_f32_16x16x4f32 head took 128 MFMAs of twice the cycles.)
    const u32x4* hw1 = reinterpret_cast<const u32x4*>(s_hw1) + lane;
    const f32x4* hb1 = reinterpret_cast<const f32x4*>(s_hw1 + 4 * 4 * 64 * 4 + 16 * g);
    f32x4 acc3[4][2];
#pragma unroll
    for (int m3 = 0; m3 < 4; ++m3)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc3[m3][nt] = hb1[m3];
    u32x4 sh[2][2], sl[2][2];  // [nt][ks]
    // range check: an x, D or first_conv value beyond the fp16 pair range became (inf, -inf) and
    // every later product NaN, which every skip sum downstream carries (the ReLU's fmaxf below
    // would hide it), so the final skip sums cover every layer; and the scaled skip itself must
    // fit the head's pair split
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      float sum = 0.f;
#pragma unroll
      for (int ms = 0; ms < 4; ++ms)
#pragma unroll
        for (int i = 0; i < 4; ++i) sum += acc2[ms][nt][i];
      nonfinite |= bd.t0 + 16 * nt + c < bd.T && !__builtin_isfinite(sum);
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float hv[8];
        float hmax = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          hv[j] = fmaxf(acc2[2 * ks + (j >> 2)][nt][j & 3] * a.skip_scale, 0.f);
          hmax = fmaxf(hmax, hv[j]);
        }
        nonfinite |= bd.t0 + 16 * nt + c < bd.T && hmax >= 65520.f;
        split8x<0>(hv, sh[nt][ks], sl[nt][ks]);
      }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int m3 = 0; m3 < 4; ++m3) {
        const u32x4 ah = hw1[((ks * 4 + m3) * 2) * 64], al = hw1[((ks * 4 + m3) * 2 + 1) * 64];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          acc3[m3][nt] = mma16(ah, sh[nt][ks], acc3[m3][nt]);
          acc3[m3][nt] = mma16(ah, sl[nt][ks], acc3[m3][nt]);
          acc3[m3][nt] = mma16(al, sh[nt][ks], acc3[m3][nt]);
        }
      }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int t = bd.t0 + 16 * nt + c;
      const bool live = t < bd.T;
      float* out = a.out + (size_t)bd.io_off * a.O + (size_t)t * a.out_stride_t;
      for (int oc = 0; oc < a.O; ++oc) {
        const f32x4* w = reinterpret_cast<const f32x4*>(a.hw2 + ((size_t)oc * 4 + g) * 16);
        float part = 0.f;
#pragma unroll
        for (int m3 = 0; m3 < 4; ++m3) {
          const f32x4 wq = w[m3];
#pragma unroll
          for (int i = 0; i < 4; ++i) part = fmaf(wq[i], fmaxf(acc3[m3][nt][i], 0.f), part);
        }
        part += __shfl_xor(part, 16);
        part += __shfl_xor(part, 32);
        if (g == 0 && live) out[(size_t)oc * a.out_stride_o] = poison ? __builtin_nanf("") : part + a.hb2[oc];
      }
    }
  }
}

// One launch = one residual layer over the whole padded time axis (the default path).
// XCD-local work queues with stealing: workgroup i runs on XCD i mod 8, XCD x owns
// the x-th eighth of the blocks; rounds 0 and 1 are static, then a wave claims its next-but-one
// block from its XCD's queue head one block ahead of use; a wave whose XCD range is drained steals
// from the next XCDs'.
// Small plans launch fewer computing waves per workgroup (a.compute_waves, spreading the blocks
// over every CU) but still all the workgroup's waves stage the layer image (8 loads in flight per
// thread over every thread).
// a.trace (diagnostic, PWG_TRACE_FILE): per wave [start, staged, first block done, end, blocks,
// shader clock at start, at end, XCC id], real time at 100 MHz.
// NTN = 1 (small plans, the B = 1 latency path): the work unit is half a block (one 16-column
// n-tile; unit u = block u / 2, columns 16 (u % 2) + [0, 16)), so twice the waves share a layer and
// each wave's dependent chain runs half the MFMAs; bit-identical to whole blocks.
template <bool LAST, int TC, bool FIRST, int NTN = 2>
__global__ void __launch_bounds__(512, 1) pwg_layer_split16_kernel(const SplitArgs a) {
  constexpr int UB = NTN == 1 ? 1 : 0;  // log2(units per block)
  const int n_units = a.n_blocks << UB;
  extern __shared__ __attribute__((aligned(16))) unsigned smem16[];
  const bool tr = a.trace != nullptr;
  unsigned long long t_start = 0, c_start = 0, t_staged = 0, t_first = 0;
  if (tr) {
    t_start = __builtin_amdgcn_s_memrealtime();
    c_start = __builtin_amdgcn_s_memtime();
  }
  const int lane = threadIdx.x & 63;
  const int nw = a.compute_waves;
  const int xcd = blockIdx.x & 7;
  const int wave = threadIdx.x >> 6;
  // the wave's first block (a static round) is known before the image is staged: its descriptor
  // and tap-0 rows load while the workgroup stages (layer 0 with the fused first_conv builds tap 0
  // from the first_conv weights in LDS, after the barrier)
  const int blk0 = wave < nw ? (int)((long long)n_units * xcd / 8) + (blockIdx.x >> 3) * nw + wave : -1;
  // LAST: the run's status on entry (a grid-synchronised or pipelined launch before this one that
  // aborted or timed out leaves stale planes: poison the output, pwg_run_status reports the redo)
  bool poison = false;
  if constexpr (LAST)
    if (a.range_flag != nullptr)
      poison = (__hip_atomic_load(a.range_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & PWG_STATUS_REDO) != 0;
  const bool has0 = blk0 >= 0 && blk0 < (int)((long long)n_units * (xcd + 1) / 8);
  BlockDesc bdn;
  int h16n = 0;
  u32x4 b0[8], b1[8];
  if (has0) {
    bdn = a.blocks[blk0 >> UB];
    h16n = NTN == 1 ? 16 * (blk0 & 1) : 0;
    if constexpr (!FIRST) s16_bload<TC, false, false, NTN>(a, nullptr, bdn, 0, b0, lane >> 4, lane & 15, h16n);
  }
  s16_stage<LAST, FIRST>(a, smem16);
  __syncthreads();
  int n_done = 0;
  auto trace_out = [&]() {
    if (tr && lane == 0) {
      unsigned long long* r = a.trace + ((size_t)blockIdx.x * (blockDim.x >> 6) + wave) * 8;
      const unsigned long long t_end = __builtin_amdgcn_s_memrealtime(), c_end = __builtin_amdgcn_s_memtime();
      r[0] = t_start; r[1] = t_staged; r[2] = t_first; r[3] = t_end; r[4] = (unsigned long long)n_done;
      r[5] = c_start; r[6] = c_end; r[7] = (unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));
    }
  };
  if (tr) t_staged = __builtin_amdgcn_s_memrealtime();
  if (wave >= nw) {
    trace_out();
    return;
  }
  auto xcd_waves = [&](int y) { return (((int)gridDim.x - y + 7) >> 3) * nw; };
  auto xcd_first = [&](int y) { return (int)((long long)n_units * y / 8); };
  const int x_first = xcd_first(xcd), x_end = xcd_first(xcd + 1), x_waves = xcd_waves(xcd);
  int victim = 0;
  auto ticket_issue = [&]() -> int {
    int v = 0;
    if (victim == 0 && lane == 0)
      v = __hip_atomic_fetch_add(a.ctr + xcd * SCHED_CTR_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
  };
  auto ticket_resolve = [&](int v) -> int {
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

  int blk = x_first + (blockIdx.x >> 3) * nw + wave;
  int nblk = blk + x_waves;
  if (blk >= x_end) blk = -1;
  if (nblk >= x_end) nblk = -1;
  if (blk < 0) {
    trace_out();
    return;
  }
  const float* s_fwb = reinterpret_cast<const float*>(smem16 + Split16Smem::dwords(LAST));
  if constexpr (FIRST) s16_bload<TC, true, false, NTN>(a, s_fwb, bdn, 0, b0, lane >> 4, lane & 15, h16n);
  bool nonfinite = false;  // LAST: range flag (pwg_run_status)
  while (true) {
    const BlockDesc bd = bdn;
    const int h16 = h16n;
    const int pf = nblk >= 0 ? nblk : blk;  // prefetch target (this unit itself when there is none)
    bdn = a.blocks[pf >> UB];
    h16n = NTN == 1 ? 16 * (pf & 1) : 0;
    int ticket = 0;
    s16_block<LAST, TC, FIRST, false, NTN>(a, smem16, bd, bdn, true, b0, b1, nonfinite, [&]() {
      if (nblk >= 0) ticket = ticket_issue();
    }, h16, h16n, poison);
    if (tr && n_done++ == 0) t_first = __builtin_amdgcn_s_memrealtime();
    if (nblk < 0) break;
    blk = nblk;
    nblk = ticket_resolve(ticket);
  }
  if (LAST && nonfinite && a.range_flag) flag_status(a.range_flag, a.sticky, PWG_STATUS_RANGE);
  trace_out();
}

// ---------------------------------------------------------------------------------------------
// Layer-pipelined forward (all L residual layers in ONE launch): workgroup w (one per CU) keeps
// layer l(w)'s weights resident in LDS for the whole forward and its waves take that layer's
// blocks in order from a per-layer queue; a block of layer l starts once layer l - 1 has finished
// the blocks its dilated taps read (RAW on x) and layer l - 2 the blocks whose columns this write
// overwrites (x lives in 3 rotating planes: layer l reads plane l % 3, writes (l + 1) % 3; skip is
// updated in place). prog[b] = layers finished on block b. Hand-off bytes (x, skip) are stored and
// loaded sc1, each storing wave drains its stores (s_waitcnt vmcnt(0)) before it publishes
// prog[b] with an sc1 atomic store; consumers poll prog relaxed (Guideline 16, R1 with sc1 loads).
// Every spin is bounded: a wait that gives up sets PWG_STATUS_PIPE_TIMEOUT (pwg_run_status reports
// PWG_ERR_RERUN) and the grid still drains. Requires every workgroup resident: grid <= CUs, one
// 512-thread workgroup per CU (the LDS image holds that).
constexpr int PIPE_SPIN_LIMIT = 1 << 20;

template <bool LAST, int TC, bool FIRST>
__device__ __forceinline__ void pipe_layer(const PipeArgs& p, int l, unsigned* smem16) {
  SplitArgs a = p.base;
  a.wg = p.wg0 + (size_t)l * p.wg_stride;
  a.d = p.d0 + (size_t)l * p.d_stride;
  a.x_in = p.x[l % 3];
  a.x_out = p.x[(l + 1) % 3];
  a.dil = p.dil[l];
  a.first = l == 0;
  if (!FIRST) a.noise = nullptr;
  s16_stage<LAST, FIRST>(a, smem16);
  __syncthreads();

  const int lane = threadIdx.x & 63;
  int* const queue = p.ctr + l * SCHED_CTR_STRIDE * 8;
  // waits, in blocks around b: layer l - 1 done on [b - rl1, b + rr1] (what this layer's taps read:
  // TC * dil to the left, (2 - TC) * dil to the right), layer l - 2 done on [b - rr2, b + rl2] (the
  // blocks whose taps read the columns of b in the plane this layer overwrites)
  const int rl1 = (TC * a.dil + 31) / 32, rr1 = ((2 - TC) * a.dil + 31) / 32;
  const int rl2 = l >= 2 ? (TC * p.dil[l - 2] + 31) / 32 : 0, rr2 = l >= 2 ? ((2 - TC) * p.dil[l - 2] + 31) / 32 : 0;
  const int left = rl1 > rr2 ? rl1 : rr2, right = rr1 > rl2 ? rr1 : rl2;  // left + right < 64 (plan check)
  auto ticket = [&]() -> int {
    int v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(queue, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(v);
  };
  auto wait_deps = [&](int b) {
    if (l == 0) return;
    const int i = lane - left, bb = b + i;
    const bool need = lane <= left + right && bb >= 0 && bb < a.n_blocks;
    const int thr = (i >= -rl1 && i <= rr1) ? l : l - 1;
    for (int spins = 0;; ++spins) {
      const int v = need ? __hip_atomic_load(p.prog + (need ? bb : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : 0x7fffffff;
      if (__all(v >= thr)) break;
      if (spins >= PIPE_SPIN_LIMIT) {
        if (lane == 0) flag_status(p.base.range_flag, p.base.sticky, PWG_STATUS_PIPE_TIMEOUT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the sc1 loads below the poll
  };

  bool nonfinite = false;
  const float* s_fwb = reinterpret_cast<const float*>(smem16 + Split16Smem::dwords(LAST));
  int blk = ticket();
  u32x4 b0[8], b1[8];
  while (blk < a.n_blocks) {
    const BlockDesc bd = a.blocks[blk];
    wait_deps(blk);
    s16_bload<TC, FIRST, true>(a, s_fwb, bd, 0, b0, lane >> 4, lane & 15);
    int next = 0;
    s16_block<LAST, TC, FIRST, true>(a, smem16, bd, bd, false, b0, b1, nonfinite, [&]() { next = ticket(); });
    if (!LAST) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores have landed
      if (lane == 0) __hip_atomic_store(p.prog + blk, l + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    blk = next;
  }
  if (LAST && nonfinite && a.range_flag) flag_status(a.range_flag, a.sticky, PWG_STATUS_RANGE);
}

template <int TC>
__global__ void __launch_bounds__(512, 1) pwg_pipe_split16_kernel(const PipeArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned smem16[];
  // layers laid out over the XCDs in order (workgroup i runs on XCD i mod 8 in practice: consecutive
  // layers then share an L2; placement is a speed heuristic only, correctness does not depend on it)
  const int nwg = gridDim.x;
  const int lin = (blockIdx.x & 7) * (nwg >> 3) + (blockIdx.x >> 3);
  const int l = (int)((long long)lin * p.L / nwg);
  if (l == p.L - 1) pipe_layer<true, TC, false>(p, l, smem16);
  else if (l == 0 && p.base.noise != nullptr) pipe_layer<false, TC, true>(p, l, smem16);
  else pipe_layer<false, TC, false>(p, l, smem16);
}

// ---------------------------------------------------------------------------------------------
// Grid-synchronised forward (residual layers l0 .. l0 + L - 1 in ONE launch, one workgroup per CU;
// the B = 1 decode path; the last layer, with the output head, runs as its own per-layer launch,
// and so does layer 0 with the fused first_conv on whole-block plans). Each layer runs the
// per-layer launch's work units (its static rounds: XCD x takes the x-th eighth of the units, wave
// w of workgroup b every x_waves-th unit from (b >> 3) nw + w) through the same block body, so the
// forward is bit-identical; a grid barrier replaces each launch boundary, and a workgroup stages
// the next layer's LDS image while the barrier completes (the per-layer path pays ~2.2 us of launch
// gap plus ~1.9 us of staging per layer after the previous layer's tail).
// Residency: the static split needs every workgroup on the GPU at once, which a second stream or
// process holding CUs can prevent. So every workgroup first counts itself in, and the first one to
// see either the full count or its bounded wait expire decides for all (one CAS): "run" (every
// workgroup had started, so all are resident) or "abort" (every workgroup exits at once, no x or skip
// written, PWG_STATUS_SYNC_ABORT: pwg_run_status returns PWG_ERR_RERUN, the last layer writes NaN
// audio, and the engine reruns on the per-layer launches).
// Measured: claiming units dynamically instead (one queue per layer, deadlock-free without the
// check) cost 0.35 -> 0.89 ms at LJ T' = 64: the claims serialise on the queue head.
// Hand-off (cdna_hip_programming.md Guideline 16; MI355X_MICROARCH.md hand-off table, row 1): every
// store and every load of x and skip is sc1 (the PIPE forms of s16_block), every storing wave
// drains (s_waitcnt vmcnt(0)) before a workgroup barrier, then one lane adds to the barrier counter
// (agent-scope atomic); one lane polls it with sc1 loads and a workgroup barrier follows. Bounded
// spins: a wait that gives up sets PWG_STATUS_SYNC_TIMEOUT (pwg_run_status returns PWG_ERR_RERUN,
// the last layer writes NaN audio, and the engine reruns on the per-layer launches, which rebuild
// every plane from the mel and the noise). The grid needs at least 8 workgroups (one per XCD
// eighth of the work units; launch_sync_split16 checks).
template <int TC, bool FIRST, int NTN>
__device__ __forceinline__ void sync_layer(const SplitArgs& a, const unsigned* smem16) {
  constexpr int UB = NTN == 1 ? 1 : 0;
  const int n_units = a.n_blocks << UB;
  const int nw = a.compute_waves;
  const int wave = threadIdx.x >> 6;
  if (wave >= nw) return;
  const int lane = threadIdx.x & 63;
  const int xcd = blockIdx.x & 7;
  const int x_first = (int)((long long)n_units * xcd / 8), x_end = (int)((long long)n_units * (xcd + 1) / 8);
  const int x_waves = (((int)gridDim.x - xcd + 7) >> 3) * nw;
  int u = x_first + (blockIdx.x >> 3) * nw + wave;
  if (u >= x_end) return;
  const float* s_fwb = reinterpret_cast<const float*>(smem16 + Split16Smem::dwords(false));
  bool nonfinite = false;  // (middle layers never set it)
  BlockDesc bd = a.blocks[u >> UB];
  int h16 = NTN == 1 ? 16 * (u & 1) : 0;
  u32x4 b0[8], b1[8];
  s16_bload<TC, FIRST, true, NTN>(a, s_fwb, bd, 0, b0, lane >> 4, lane & 15, h16);
  while (true) {
    const int un = u + x_waves;
    const bool has_next = un < x_end;
    const BlockDesc bdn = a.blocks[(has_next ? un : u) >> UB];
    const int h16n = NTN == 1 ? 16 * ((has_next ? un : u) & 1) : 0;
    s16_block<false, TC, FIRST, true, NTN>(a, smem16, bd, bdn, has_next, b0, b1, nonfinite, []() {}, h16, h16n);
    if (!has_next) break;
    u = un;
    bd = bdn;
    h16 = h16n;
  }
}

constexpr int SYNC_RESIDENCY_SPINS = 512;  // bounded wait for every workgroup to start (~0.5 ms)

template <int TC, int NTN>
__global__ void __launch_bounds__(512, 1) pwg_sync_split16_kernel(const SyncArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned smem16[];
  __shared__ int s_decision;
  const int nwg = gridDim.x;
  int* const bar = p.ctr;
  int* const arrive = p.ctr + SCHED_CTR_STRIDE;
  int* const decision = p.ctr + 2 * SCHED_CTR_STRIDE;
  if (threadIdx.x == 0) __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  auto layer_args = [&](int l) {
    SplitArgs a = p.base;
    a.wg = p.wg0 + (size_t)l * p.wg_stride;
    a.d = p.d0 + (size_t)l * p.d_stride;
    a.x_in = p.x[l & 1];
    a.x_out = p.x[(l + 1) & 1];
    a.dil = p.dil[l];
    a.first = l == 0;
    a.compute_waves = p.waves_mid;
    if (l != 0) a.noise = nullptr;
    return a;
  };
  // layer 0 with the fused first_conv: half-block launches only (whole-block launches start at
  // layer 1; the register budget holds one block body per kernel there)
  const bool fused = NTN == 1 && p.base.noise != nullptr;
  auto stage = [&](int l) {
    const SplitArgs a = layer_args(l);
    if (l == 0 && fused) s16_stage<false, true>(a, smem16);
    else s16_stage<false, false>(a, smem16);
  };
  const int l_end = p.l0 + p.L;
  stage(p.l0);
  if (threadIdx.x == 0) {
    int d = 0;
    for (int spins = 0;; ++spins) {
      d = __hip_atomic_load(decision, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d != 0) break;
      int want = 0;
      if (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= nwg)
        __hip_atomic_compare_exchange_strong(decision, &want, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      else if (spins >= SYNC_RESIDENCY_SPINS)
        __hip_atomic_compare_exchange_strong(decision, &want, 2, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      else
        __builtin_amdgcn_s_sleep(1);
    }
    s_decision = d;
  }
  __syncthreads();
  if (s_decision != 1 || p.force_abort) {
    if (threadIdx.x == 0) flag_status(p.base.range_flag, p.base.sticky, PWG_STATUS_SYNC_ABORT);
    return;
  }
  bool timed_out = false;
  for (int l = p.l0; l < l_end; ++l) {
    const SplitArgs a = layer_args(l);
    if constexpr (NTN == 1) {
      if (l == 0 && fused) sync_layer<TC, true, NTN>(a, smem16);
      else sync_layer<TC, false, NTN>(a, smem16);
    } else {
      sync_layer<TC, false, NTN>(a, smem16);
    }
    if (l == l_end - 1) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores have landed
    __syncthreads();                                   // ... and every wave's; LDS image free
    if (threadIdx.x == 0) __hip_atomic_fetch_add(bar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    stage(l + 1);
    if (threadIdx.x == 0) {
      const int target = (l - p.l0 + 1) * nwg;
      for (int spins = 0;; ++spins) {
        if (p.force_timeout) {  // test hook: give up without waiting
          timed_out = true;
          break;
        }
        if (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
        if (spins >= PIPE_SPIN_LIMIT) {
          timed_out = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
  }
  if (timed_out) flag_status(p.base.range_flag, p.base.sticky, PWG_STATUS_SYNC_TIMEOUT);
}

// first_conv (1x1, 1 -> 64, bias) into the split16 x layout; gap tiles zero every residual plane.
__global__ void __launch_bounds__(256) pwg_first_conv_split16_kernel(const FirstConvArgs a) {
  const long long tile = blockIdx.x;
  unsigned* x = reinterpret_cast<unsigned*>(a.x);
  unsigned* x1 = reinterpret_cast<unsigned*>(a.x1);
  unsigned* x2 = reinterpret_cast<unsigned*>(a.x2);
  if (tile >= a.n_work) {
    const long long col0 = a.gap_col0[tile - a.n_work];
    for (int idx = threadIdx.x; idx < 64 * TILE; idx += 256) {
      x[(size_t)col0 * 64 + idx] = 0u;
      x1[(size_t)col0 * 64 + idx] = 0u;
      if (x2 != nullptr) x2[(size_t)col0 * 64 + idx] = 0u;
    }
    return;
  }
  const UttDesc ud = a.utts[a.tile_utt[tile]];
  const long long col0 = ud.seg_base + (tile - ud.first_tile) * TILE;
  const long long t0 = col0 - ud.seg_base;
  // 128 columns = 4 tiles of 2048 dwords, walked in memory order:
  // [sub 4][nt 2][ks 2][hl 2][g 4][c 16][dw 4]
  for (int idx = threadIdx.x; idx < 64 * TILE; idx += 256) {
    const int sub = idx >> 11, rem = idx & 2047;
    const int nt = rem >> 10, ks = (rem >> 9) & 1, hl = (rem >> 8) & 1, g = (rem >> 6) & 3, cc = (rem >> 2) & 15,
              dw = rem & 3;
    const int jcol = 32 * sub + 16 * nt + cc;
    const long long t = t0 + jcol;
    unsigned v = 0u;
    if (t < ud.T) {
      const float z = a.noise[ud.io_off + t];
      float y[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = 2 * dw + e;
        const int ch = 16 * (2 * ks + (j >> 2)) + 4 * g + (j & 3);
        y[e] = fmaf(a.w[ch], z, a.b[ch]);
      }
      const Pair16 pr = split_pair16(y[0], y[1]);
      v = hl ? pr.lo : pr.hi;
    }
    x[(size_t)col0 * 64 + idx] = v;
  }
}

hipError_t launch_first_conv_split16(const FirstConvArgs& a, long long n_tiles, hipStream_t s) {
  hipLaunchKernelGGL(pwg_first_conv_split16_kernel, dim3((unsigned)n_tiles), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_layer_split16(const SplitArgs& a, bool last, int tap_center, int waves_per_wg, int n_wg,
                                hipStream_t s, bool half) {
  if (waves_per_wg > 8) waves_per_wg = 8;
  if (a.compute_waves < 1 || a.compute_waves > waves_per_wg) return hipErrorInvalidValue;
  if (half && last) return hipErrorInvalidValue;  // the head needs both n-tiles of a block
  const dim3 grid((unsigned)n_wg), block((unsigned)(64 * waves_per_wg));
#define PWG_SPLIT16_LAUNCH(LAST_, TC_, FIRST_, NTN_)                                                    \
  {                                                                                                     \
    const size_t lds = sizeof(unsigned) * (Split16Smem::dwords(LAST_) + (FIRST_ ? 128 : 0));            \
    auto kfn = &pwg_layer_split16_kernel<LAST_, TC_, FIRST_, NTN_>;                                     \
    hipError_t e_ = allow_lds(reinterpret_cast<const void*>(kfn), (int)lds);                           \
    if (e_ != hipSuccess) return e_;                                                                    \
    hipLaunchKernelGGL(kfn, grid, block, lds, s, a);                                                    \
    return hipGetLastError();                                                                           \
  }
  const bool first = a.noise != nullptr;  // fused first_conv (never together with last: L > 1)
  if (first && last) return hipErrorInvalidValue;
  if (tap_center == 1) {
    if (half) {
      if (first) PWG_SPLIT16_LAUNCH(false, 1, true, 1) else PWG_SPLIT16_LAUNCH(false, 1, false, 1)
    }
    if (first) PWG_SPLIT16_LAUNCH(false, 1, true, 2)
    if (last) PWG_SPLIT16_LAUNCH(true, 1, false, 2) else PWG_SPLIT16_LAUNCH(false, 1, false, 2)
  } else if (tap_center == 2) {
    if (half) {
      if (first) PWG_SPLIT16_LAUNCH(false, 2, true, 1) else PWG_SPLIT16_LAUNCH(false, 2, false, 1)
    }
    if (first) PWG_SPLIT16_LAUNCH(false, 2, true, 2)
    if (last) PWG_SPLIT16_LAUNCH(true, 2, false, 2) else PWG_SPLIT16_LAUNCH(false, 2, false, 2)
  }
#undef PWG_SPLIT16_LAUNCH
  return hipErrorInvalidValue;
}

hipError_t launch_sync_split16(const SyncArgs& p, int tap_center, int n_wg, hipStream_t s) {
  const size_t lds = sizeof(unsigned) * (Split16Smem::dwords(false) + 128);
  if (p.L < 1 || p.L > PIPE_MAX_LAYERS || p.waves_mid < 1 || p.waves_mid > 8) return hipErrorInvalidValue;
  if (n_wg < 8) return hipErrorInvalidValue;  // sync_layer deals the units to 8 eighths by blockIdx & 7
  auto kfn = tap_center == 1 ? (p.half ? &pwg_sync_split16_kernel<1, 1> : &pwg_sync_split16_kernel<1, 2>)
             : tap_center == 2 ? (p.half ? &pwg_sync_split16_kernel<2, 1> : &pwg_sync_split16_kernel<2, 2>)
                               : nullptr;
  if (kfn == nullptr) return hipErrorInvalidValue;
  const hipError_t e = allow_lds(reinterpret_cast<const void*>(kfn), (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kfn, dim3((unsigned)n_wg), dim3(512), lds, s, p);
  return hipGetLastError();
}

hipError_t launch_pipe_split16(const PipeArgs& p, int tap_center, int n_wg, hipStream_t s) {
  const size_t lds = sizeof(unsigned) * (Split16Smem::dwords(true) > Split16Smem::dwords(false) + 128
                                             ? Split16Smem::dwords(true) : Split16Smem::dwords(false) + 128);
  if (n_wg < p.L || n_wg % 8 != 0) return hipErrorInvalidValue;
  auto kfn = tap_center == 1 ? &pwg_pipe_split16_kernel<1> : tap_center == 2 ? &pwg_pipe_split16_kernel<2> : nullptr;
  if (kfn == nullptr) return hipErrorInvalidValue;
  const hipError_t e = allow_lds(reinterpret_cast<const void*>(kfn), (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kfn, dim3((unsigned)n_wg), dim3(512), lds, s, p);
  return hipGetLastError();
}

}  // namespace pwg
