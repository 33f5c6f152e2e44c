// Split-f16 residual layer for gfx950: the PWG v1 shape (R = S = 64, 128 gate rows, kernel 3)
// on the f16 MFMA pipe at fp32 accuracy.
//
// Why: the layer is a dense contraction (86 kFLOP per sample per layer); on
// v_mfma_f32_32x32x2_f32 it is compute-bound at 1/16 of the f16 matrix rate. Every fp32 operand
// v is carried as an fp16 pair v = hi + lo (hi = rne16(v), lo = rne16(v - hi)) and a product as
//   a*b ~= ah*bh + ah*bl + al*bh            (three v_mfma_f32_32x32x16_f16, fp32 accumulate)
// The dropped al*bl and the pair's own rounding are ~2^-22 relative per product (fp32 rounding is
// 2^-24), so this runs at 16/3 = 5.3x the fp32 MFMA rate. The tolerance it must meet is the
// reference's |d| < 1e-4 (BASELINE north star); measured end to end it stays at the plain-fp32
// engine's error level (tests/test_gpu_parity.py).
//
// Data layout (256 B per padded time column, as the fp32 engine, but TILED): columns are grouped
// in 32-column tiles of 8 KB, [hh 2][piece 8][column 32][16 B]. Piece i < 4 of half hh holds the hi
// halves of slots 8i..8i+7, piece 4 + i their lo halves. So the 32 lanes of one half reading piece
// i of 32 consecutive columns read 512 contiguous bytes: a wave's 16-byte load touches 8 cache
// lines, not 64 (1.83 vs 2.67 ms per layer with per-column rows).
//   x   lane half hh owns 32 channel SLOTS p = 0..31 (16 dwords of hi halves, 16 of lo). Slot p of half hh holds channel
//           chan(s = p>>3, hh, j = p&7) = 32(s>>1) + 16(s&1) + 8(j>>2) + 4hh + (j&3)
//       which is at once (a) k-element j of k-step s of the GEMM-1 B operand of lane half hh
//       (B[k = 8hh + j][col]) and (b) accumulator register r = 16(s>>1)... of the GEMM-2 out rows:
//       acc[2+mo][r] holds channel 32mo + 8(r>>2) + 4hh + (r&3) = slot 16mo + r. So a lane's
//       128 contiguous bytes per tap row ARE its MFMA operand, and its epilogue writes exactly the
//       bytes it will read as the next layer's center tap.
//   skip the same tiles and slot order, fp32 (it is never an MFMA operand): piece i of half hh =
//       slots 4i..4i+3.
//   D    [F][128 dwords]: the aux projection of this layer at frame rate as (hi | lo << 16).
//
// Per block of 32 samples (one wave): GEMM 1 = 3 taps x 4 k-steps x 4 m-tiles x 3 = 144 MFMA,
// aux + gate bias = 12 MFMA (K slots: 8 frames of the block's window + the bias against a ones
// row), gate in fp32, GEMM 2 = 4 k-steps x 4 m-tiles x 3 = 48 MFMA (skip rows seeded with the
// old skip sum, out rows with sqrt(.5)*(x_in + b_out) and W_out pre-scaled by sqrt(.5)).
// Reference: layers/residual_block.py:102-140, models/parallel_wavegan.py:160-171.
#include "pwg_internal.h"

namespace pwg {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ f16x8 h8(u32x4 v) { return __builtin_bit_cast(f16x8, v); }

// two values -> {hi halves, lo halves} dwords (v = hi + lo, hi = rne16(v), lo = rne16(v - hi))
struct Pair2 {
  unsigned hi, lo;
};
__device__ __forceinline__ Pair2 split2(float v0, float v1) {
  const _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
  // v - hi as one v_fma_mix_f32 each (f16 source widened inside the FMA)
  const _Float16 l0 = (_Float16)__builtin_fmaf((float)h0, -1.f, v0), l1 = (_Float16)__builtin_fmaf((float)h1, -1.f, v1);
  return {__builtin_bit_cast(unsigned, f16x2{h0, h1}), __builtin_bit_cast(unsigned, f16x2{l0, l1})};
}


__device__ __forceinline__ f32x16 mma(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(h8(a), h8(b), c, 0, 0, 0);
}

// tanh(a) * sigmoid(b) = (1 - e^-2a) / ((1 + e^-2a)(1 + e^-b)) with 2 v_exp + 1 v_rcp. The gate
// rows arrive PRE-SCALED (host packing and the aux projection): u = -2 log2(e) a, v = -log2(e) b,
// so e^-2a = 2^u and e^-b = 2^v. Clamps where fp32 is already saturated (|a| > 15: tanh = +-1;
// b < -30: sigmoid < 1e-13) keep every intermediate finite.
constexpr float GATE_SCALE_TANH = -2.8853900817779268f;  // -2 log2(e)
constexpr float GATE_SCALE_SIGM = -1.4426950408889634f;  // -log2(e)
// Only u needs a clamp: 2^u must stay finite (u <= 64: tanh is -1 to fp32 precision long
// before). 2^v may overflow to +inf: rcp(inf) = 0 gives the sigmoid's limit 0, and 2^v -> 0 its 1.
__device__ __forceinline__ float gate(float u, float v) {
  u = fminf(u, 64.f);
  const float e1 = __builtin_amdgcn_exp2f(u);
  const float e2 = __builtin_amdgcn_exp2f(v);
  return (1.f - e1) * __builtin_amdgcn_rcpf((1.f + e1) * (1.f + e2));
}

// Four split pairs in one statement: hi = cvt_pk (RNE), lo = rne16(v - hi) by v_fma_mix{lo,hi}
// (one instruction per value; the compiler's own form is 2 conversions + a packed f32 add).
// The trailing s_nop 1 covers a VALU write -> MFMA operand read; NOPS leading wait states cover
// inputs fresh from an MFMA (12 for an 8-pass 32x32x16; cdna_hip_programming.md 5.7 item 2).
template <int NOPS>
__device__ __forceinline__ void split8(const float (&v)[8], unsigned (&hi)[4], unsigned (&lo)[4]) {
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
      : "=&v"(hi[0]), "=&v"(hi[1]), "=&v"(hi[2]), "=&v"(hi[3]), "=&v"(lo[0]), "=&v"(lo[1]), "=&v"(lo[2]),
        "=&v"(lo[3])
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]), "i"(NOPS));
}

// GEMM-2 out-row seeds of 8 slots: c * (hi + lo) + b for the fp16 pairs of one k-step (hi halves
// in dwords h, lo halves in l), two v_fma_mix_f32 per value; trailing s_nop 1: the results are
// MFMA accumulator inputs.
__device__ __forceinline__ void seed8(const u32x4 h, const u32x4 l, const f32x4 b0, const f32x4 b1, float c,
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

}  // namespace

// LDS image of one layer (dwords): GEMM-1 A fragments [tap 3][kstep 4][m 4][hi/lo 2][lane 64][4]
// | GEMM-2 A fragments [kstep 4][m 4][hi/lo 2][lane 64][4] | gate bias pairs [lane 32][m 4]
// | sqrt(.5)*b_out [hh 2][slot 32] (float) | last layer: head W1 fp32 fragments [9][2][64][4].
struct SplitSmem {
  static constexpr int WG = 3 * 4 * 4 * 2 * 64 * 4;
  static constexpr int W2 = 4 * 4 * 2 * 64 * 4;
  static constexpr int BG = 32 * 4;
  static constexpr int BO = 64;
  static constexpr int HW1 = 9 * 2 * 256;
  static constexpr int dwords(bool last) { return WG + W2 + BG + BO + (last ? HW1 : 0); }
};

// dword offset of piece 0 of column c, lane half hh, in the tiled x / skip layout (header);
// piece i is PWG_PIECE dwords further
#define PWG_ROW(c, hh) ((size_t)((c) >> 5) * 2048 + (size_t)(hh) * 1024 + (size_t)((c) & 31) * 4)
#define PWG_PIECE 128

// Cache policy of the streams that are touched once per layer (skip sum in, skip sum and x out):
// non-temporal, so the XCD's L2 keeps the x rows that the three dilated taps of neighbouring
// blocks re-read (1.825 -> 1.747 ms per layer). The A/B variants (cached streams, diagnostic
// builds) are in git history before round 4.
#define PWG_ST_STREAM(p, v) __builtin_nontemporal_store((v), (p))
#define PWG_LD_SKIP(p) __builtin_nontemporal_load(p)

template <bool LAST, int TC>
__global__ void __launch_bounds__(512, 1) pwg_layer_split_kernel(const SplitArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned smem_u[];
  unsigned* s_wg = smem_u;
  unsigned* s_w2 = s_wg + SplitSmem::WG;
  unsigned* s_bg = s_w2 + SplitSmem::W2;
  float* s_bo = reinterpret_cast<float*>(s_bg + SplitSmem::BG);
  float* s_hw1 = s_bo + SplitSmem::BO;
  {
    const int nthr = blockDim.x;
    // the four sections are contiguous in the packed image too
    stage_lds(reinterpret_cast<u32x4*>(s_wg), reinterpret_cast<const u32x4*>(a.wg),
              (SplitSmem::WG + SplitSmem::W2 + SplitSmem::BG + SplitSmem::BO) / 4, (int)threadIdx.x, nthr);
    if (LAST)
      stage_lds(reinterpret_cast<u32x4*>(s_hw1), reinterpret_cast<const u32x4*>(a.hw1), SplitSmem::HW1 / 4,
                (int)threadIdx.x, nthr);
    __syncthreads();
  }

  const int lane = threadIdx.x & 63;
  const int hh = lane >> 5;
  const int cl = lane & 31;
  const int nw = blockDim.x >> 6;
  // XCD-local work queues with stealing (the fp32 persistent kernel's scheduler, pwg_kernels.hip)
  const int xcd = blockIdx.x & 7;
  const int wave = threadIdx.x >> 6;
  auto xcd_waves = [&](int y) { return (((int)gridDim.x - y + 7) >> 3) * nw; };
  auto xcd_first = [&](int y) { return (int)((long long)a.n_blocks * y / 8); };
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

  // a lane's 128 B of tap row (block column c + lane column + tap offset): [0..3] hi k-steps,
  // [4..7] lo k-steps
  auto bload = [&](int c, int tap, u32x4 (&b)[8]) {
    const u32x4* p = reinterpret_cast<const u32x4*>(a.x_in + PWG_ROW(c + cl + (tap - TC) * a.dil, hh));
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = p[i * (PWG_PIECE / 4)];
  };
  const u32x4* wgl = reinterpret_cast<const u32x4*>(s_wg) + lane;
  auto mma_tap = [&](f32x16 (&acc)[4], const u32x4 (&b)[8], int tap) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u32x4 ah[4], al[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        ah[m] = wgl[(((tap * 4 + s) * 4 + m) * 2) * 64];
        al[m] = wgl[(((tap * 4 + s) * 4 + m) * 2 + 1) * 64];
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = mma(ah[m], b[s], acc[m]);
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = mma(ah[m], b[4 + s], acc[m]);
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = mma(al[m], b[s], acc[m]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // out-row seeds of GEMM 2 from the center tap: sqrt(.5) * (x_in + b_out), slot 16mo + r
  auto x_seed = [&](const u32x4 (&b)[8], f32x16 (&seed)[2]) {
    const f32x4* bo = reinterpret_cast<const f32x4*>(s_bo + 32 * hh);
#pragma unroll
    for (int s = 0; s < 4; ++s) {  // k-step s = slots 8s..8s+7 = seed[s >> 1][8(s & 1) + 0..7]
      float o[8];
      seed8(b[s], b[4 + s], bo[2 * s], bo[2 * s + 1], 0.70710677f, o);
#pragma unroll
      for (int j = 0; j < 8; ++j) seed[s >> 1][8 * (s & 1) + j] = o[j];
    }
  };

  int blk = x_first + (blockIdx.x >> 3) * nw + wave;
  int nblk = blk + x_waves;
  if (blk >= x_end) blk = -1;
  if (nblk >= x_end) nblk = -1;
  if (blk < 0) return;
  BlockDesc bdn = a.blocks[blk];
  u32x4 b0[8], b1[8];
  bload(bdn.col, 0, b0);
  bool nonfinite = false;  // LAST: a live column's final skip sum is not finite

  while (true) {
    const BlockDesc bd = bdn;
    bdn = a.blocks[nblk >= 0 ? nblk : blk];
    const int t = bd.t0 + cl;
    const bool live = t < bd.T;
    const bool full = bd.t0 + 32 <= bd.T;  // wave-uniform: no padding column in this block
    const int col_next = nblk >= 0 ? bdn.col : bd.col;

    // aux operands, in flight during GEMM 1. Window frames fw0 + 4hh + j (j < 4) hold K slots
    // 8hh + j; slot 4 of half 0 is the gate bias against a ones row; the rest are zero.
    const int fw0 = bd.t0 / a.H - a.J1;
    unsigned dv[4][4];
    auto load_dv = [&]() {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int f = fw0 + 4 * hh + j;
      const int fc = f < 0 ? 0 : (f >= bd.frames ? bd.frames - 1 : f);  // its weight is 0
      const unsigned* drow = a.d + (size_t)(bd.frame_base + fc) * 128 + cl;
#pragma unroll
      for (int m = 0; m < 4; ++m) dv[j][m] = drow[32 * m];
    }
    };
    float bw[4];
    {
      const int tc = live ? t : bd.T - 1;
      int roff;
      if (bd.frames < a.Fmin) roff = a.tab_small + (a.H * bd.frames * (bd.frames - 1) / 2 + tc) * AUX_J4;
      else if (tc < a.TL) roff = a.tab_left + tc * AUX_J4;
      else if (tc >= bd.T - a.TR) roff = a.tab_right + (bd.T - 1 - tc) * AUX_J4;
      else roff = (tc % a.H) * AUX_J4;
      const int shift = t / a.H - bd.t0 / a.H;  // lane row's first frame - window's first frame
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int idx = 4 * hh + j - shift;
        const bool ok = live && idx >= 0 && idx < AUX_J4;
        const float w = a.tab[roff + (idx < 0 ? 0 : (idx >= AUX_J4 ? AUX_J4 - 1 : idx))];
        bw[j] = ok ? w : 0.f;
      }
    }

    // ---- GEMM 1 over the three taps; B rows ping-pong b0/b1, the last tap prefetching the next
    //      block's first
    f32x16 acc[4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
    f32x16 seed[2];
    // taps in the order 0, the other, the center: the center row is in registers at the end of
    // GEMM 1 and becomes the GEMM-2 out-row seeds right there (re-loading it later missed L2 for
    // ~half the blocks: +1.05 GB of HBM reads per launch)
    constexpr int T1 = TC == 1 ? 2 : 1;
    bload(bd.col, T1, b1);
    mma_tap(acc, b0, 0);
    load_dv();  // in flight during the other two taps
    bload(bd.col, TC, b0);
    mma_tap(acc, b1, T1);
    bload(col_next, 0, b1);
    mma_tap(acc, b0, TC);
    x_seed(b0, seed);

    int ticket = 0;
    if (nblk >= 0) ticket = ticket_issue();
    // skip seeds (old skip sum; layer 0: the sum of all layers' skip biases)
    f32x16 acc2[4];
    {
      const f32x4* sp = reinterpret_cast<const f32x4*>(
          a.first ? a.skip0 + 32 * hh : a.skip + PWG_ROW(bd.col + cl, hh));
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const f32x4 v = PWG_LD_SKIP(sp + (a.first ? k : k * (PWG_PIECE / 4)));
#pragma unroll
        for (int i = 0; i < 4; ++i) acc2[k >> 2][4 * (k & 3) + i] = v[i];
      }
    }

    // ---- aux term + gate bias (one K = 16 k-step per m-tile)
    {
      u32x4 bh, bl;
      {
        const float one = hh == 0 ? 1.f : 0.f;
        const Pair2 p0 = split2(bw[0], bw[1]), p1 = split2(bw[2], bw[3]), p2 = split2(one, 0.f);
        bh[0] = p0.hi; bl[0] = p0.lo;
        bh[1] = p1.hi; bl[1] = p1.lo;
        bh[2] = p2.hi; bl[2] = p2.lo;
        bh[3] = 0u;
        bl[3] = 0u;
      }
      const u32x4 bgv = reinterpret_cast<const u32x4*>(s_bg)[cl];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        u32x4 ah, al;
        ah[0] = __builtin_amdgcn_perm(dv[1][m], dv[0][m], 0x05040100u);
        al[0] = __builtin_amdgcn_perm(dv[1][m], dv[0][m], 0x07060302u);
        ah[1] = __builtin_amdgcn_perm(dv[3][m], dv[2][m], 0x05040100u);
        al[1] = __builtin_amdgcn_perm(dv[3][m], dv[2][m], 0x07060302u);
        ah[2] = hh == 0 ? (bgv[m] & 0xffffu) : 0u;
        al[2] = hh == 0 ? (bgv[m] >> 16) : 0u;
        ah[3] = 0u;
        al[3] = 0u;
        acc[m] = mma(ah, bh, acc[m]);
        acc[m] = mma(ah, bl, acc[m]);
        acc[m] = mma(al, bh, acc[m]);
      }
    }

    // ---- gate (residual_block.py:123-132) -> GEMM-2 B operand pairs: k-step s = 2gm + (r >> 3),
    //      element r & 7
    u32x4 gh[4], gl[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int gm = s >> 1, r0 = 8 * (s & 1);
      float gv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) gv[k] = gate(acc[gm][r0 + k], acc[gm + 2][r0 + k]);
      unsigned hv[4], lv[4];
      split8<0>(gv, hv, lv);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        gh[s][k] = hv[k];
        gl[s][k] = lv[k];
      }
    }
    if (!LAST) {
      acc2[2] = seed[0];
      acc2[3] = seed[1];
    }

    // ---- GEMM 2: [skip; out] rows
    constexpr int M2 = LAST ? 2 : 4;
    const u32x4* w2l = reinterpret_cast<const u32x4*>(s_w2) + lane;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u32x4 ah[M2], al[M2];
#pragma unroll
      for (int m = 0; m < M2; ++m) {
        ah[m] = w2l[((s * 4 + m) * 2) * 64];
        al[m] = w2l[((s * 4 + m) * 2 + 1) * 64];
      }
#pragma unroll
      for (int m = 0; m < M2; ++m) acc2[m] = mma(ah[m], gh[s], acc2[m]);
#pragma unroll
      for (int m = 0; m < M2; ++m) acc2[m] = mma(ah[m], gl[s], acc2[m]);
#pragma unroll
      for (int m = 0; m < M2; ++m) acc2[m] = mma(al[m], gh[s], acc2[m]);
      __builtin_amdgcn_sched_barrier(0);
    }

    if (!LAST) {
      // skip sum (fp32) and the next residual stream (fp16 pairs; padding columns stay zero)
      f32x4* sp = reinterpret_cast<f32x4*>(a.skip + PWG_ROW(bd.col + cl, hh));
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        f32x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc2[k >> 2][4 * (k & 3) + i];
        PWG_ST_STREAM(sp + k * (PWG_PIECE / 4), v);
      }
      u32x4* xp = reinterpret_cast<u32x4*>(a.x_out + PWG_ROW(bd.col + cl, hh));
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {  // k-step k4 = slots 8k4..8k4+7 = acc2[2 + (k4 >> 1)][8(k4 & 1) + j]
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = acc2[2 + (k4 >> 1)][8 * (k4 & 1) + j];
        unsigned hv[4], lv[4];
        split8<11>(v, hv, lv);  // inputs straight from the GEMM-2 MFMAs
        u32x4 vh = {hv[0], hv[1], hv[2], hv[3]}, vl = {lv[0], lv[1], lv[2], lv[3]};
        if (!full) {  // wave-uniform: only a block holding padding columns masks (they stay zero)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            vh[k] = live ? vh[k] : 0u;
            vl[k] = live ? vl[k] : 0u;
          }
        }
        PWG_ST_STREAM(xp + k4 * (PWG_PIECE / 4), vh);
        PWG_ST_STREAM(xp + (4 + k4) * (PWG_PIECE / 4), vl);
      }
    } else {
      // ---- fused output head on the final skip sum (models/parallel_wavegan.py:131-138,166-171):
      //      fp32 MFMA GEMM (S -> S, bias k-step) on relu(skip * sqrt(1/L)), then relu and the
      //      S -> O dot product across the two lane halves
      constexpr int M3 = 2, NQH = 32, NQH4 = 9;
      float hs[2][16];
      {
        float sum = 0.f;  // range check of the final skip sum (see pwg_split16.hip)
#pragma unroll
        for (int mm = 0; mm < 2; ++mm)
#pragma unroll
          for (int r = 0; r < 16; ++r) sum += acc2[mm][r];
        nonfinite |= live && !__builtin_isfinite(sum);
      }
#pragma unroll
      for (int mm = 0; mm < 2; ++mm)
#pragma unroll
        for (int r = 0; r < 16; ++r) hs[mm][r] = fmaxf(acc2[mm][r] * a.skip_scale, 0.f);
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
            if (q > NQH) continue;
            const float bq = q < NQH ? hs[q >> 4][q & 15] : (hh == 0 ? 1.f : 0.f);
            acc3[m3] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[i], bq, acc3[m3], 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      float* out = a.out + (size_t)bd.io_off * a.O + (size_t)t * a.out_stride_t;
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
#pragma unroll
    for (int i = 0; i < 8; ++i) b0[i] = b1[i];
  }
  if (LAST && nonfinite && a.range_flag) flag_status(a.range_flag, a.sticky, PWG_STATUS_RANGE);
}

// first_conv (1x1, 1 -> 64, bias) into the split x layout; gap tiles zero both buffers.
__global__ void __launch_bounds__(256) pwg_first_conv_split_kernel(const FirstConvArgs a) {
  const long long tile = blockIdx.x;
  unsigned* x = reinterpret_cast<unsigned*>(a.x);
  unsigned* x1 = reinterpret_cast<unsigned*>(a.x1);
  if (tile >= a.n_work) {
    const long long col0 = a.gap_col0[tile - a.n_work];
    for (int idx = threadIdx.x; idx < 64 * TILE; idx += 256) {
      x[(size_t)col0 * 64 + idx] = 0u;
      x1[(size_t)col0 * 64 + idx] = 0u;
    }
    return;
  }
  const UttDesc ud = a.utts[a.tile_utt[tile]];
  const long long col0 = ud.seg_base + (tile - ud.first_tile) * TILE;
  const long long t0 = col0 - ud.seg_base;
  // the 128 columns are 4 whole 32-column tiles = 8192 contiguous dwords: idx walks them in
  // memory order (coalesced stores)
  for (int idx = threadIdx.x; idx < 64 * TILE; idx += 256) {
    const int sub = idx >> 11, rem = idx & 2047;
    const int hh = rem >> 10, piece = (rem >> 7) & 7, jc = (rem >> 2) & 31, dw = rem & 3;
    const int jcol = 32 * sub + jc;
    const int s = piece & 3, p = 8 * s + 2 * dw;  // slots p, p+1
    const long long t = t0 + jcol;
    unsigned v = 0u;
    if (t < ud.T) {
      const float z = a.noise[ud.io_off + t];
      float y[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = (p + e) & 7;
        const int c = 32 * (s >> 1) + 16 * (s & 1) + 8 * (j >> 2) + 4 * hh + (j & 3);
        y[e] = fmaf(a.w[c], z, a.b[c]);
      }
      const Pair2 pr = split2(y[0], y[1]);
      v = piece >= 4 ? pr.lo : pr.hi;
    }
    x[(size_t)col0 * 64 + idx] = v;
  }
}

hipError_t launch_first_conv_split(const FirstConvArgs& a, long long n_tiles, hipStream_t s) {
  hipLaunchKernelGGL(pwg_first_conv_split_kernel, dim3((unsigned)n_tiles), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_layer_split(const SplitArgs& a, bool last, int tap_center, int waves_per_wg, int n_wg,
                              hipStream_t s) {
  if (waves_per_wg > 8) waves_per_wg = 8;
  const dim3 grid((unsigned)n_wg), block((unsigned)(64 * waves_per_wg));
#define PWG_SPLIT_LAUNCH(LAST_, TC_)                                                                    \
  {                                                                                                     \
    const size_t lds = sizeof(unsigned) * SplitSmem::dwords(LAST_);                                     \
    auto kfn = &pwg_layer_split_kernel<LAST_, TC_>;                                                     \
    hipError_t e_ = allow_lds(reinterpret_cast<const void*>(kfn), (int)lds);           \
    if (e_ != hipSuccess) return e_;                                                                    \
    hipLaunchKernelGGL(kfn, grid, block, lds, s, a);                                                    \
    return hipGetLastError();                                                                           \
  }
  if (tap_center == 1) {
    if (last) PWG_SPLIT_LAUNCH(true, 1) else PWG_SPLIT_LAUNCH(false, 1)
  } else if (tap_center == 2) {
    if (last) PWG_SPLIT_LAUNCH(true, 2) else PWG_SPLIT_LAUNCH(false, 2)
  }
#undef PWG_SPLIT_LAUNCH
  return hipErrorInvalidValue;
}

}  // namespace pwg
