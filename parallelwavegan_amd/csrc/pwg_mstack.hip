// Fused residual-stack chain of one MelGAN / multi-band MelGAN upsampling stage (split-f16 MFMA,
// gfx950): the conv-network executor's B = 1 path for MelGANGenerator's ResidualStacks
// (layers/residual_stack.py:75-85, models/melgan.py:117-130).
//
// A stage ends with NS ResidualStacks on C channels; stack j computes
//   h     = W_A * lrelu(x_j)  + b_A      (k = 3, dilation d_j, ReflectionPad1d(d_j) or zero pad)
//   x_j+1 = W_1 lrelu(h) + W_s x_j + b    (the stack's 1x1 and skip_layer as ONE two-source op)
// The executor runs each of those as its own launch (2 NS dependent launches per stage, each a few
// dozen workgroups at B = 1: latency-bound, ~8-16 us apiece on MB-MelGAN v2, profiles/r04_o). Here
// ONE workgroup takes a block of `oc` output columns of one utterance through all NS stacks:
//   * the stage input over [q0 - H, q0 + oc + H) (H = sum of the dilations: what the chain's taps
//     reach) is copied into an LDS tile once (global_load_lds), and every stack rewrites it in place;
//     stack j computes its output over [q0 - H_j, q0 + oc + H_j), H_j = sum of the later dilations,
//     so neighbouring blocks recompute the halos instead of exchanging them;
//   * h stays in registers: conv A's accumulators (+ b_A, lrelu) become the 1x1's B operands by a
//     cross-half exchange per 16 channels (the 32x32 MFMA's C layout holds rows 8 j + 4 hh + i, the
//     B layout channels 8 hh + i);
//   * the weight fragments stream through an LDS ring (3-6 slots by channel count) by
//     global_load_lds, a few steps ahead (a step = one 16-channel block of conv A with its 3 taps,
//     or 3 chunks of the 1x1), across stack boundaries;
//   * conv A's B operands of a channel block are pre-activated and pair-split once per workgroup
//     into one of two converted blocks, two steps ahead, and read by every tap and wave; the 1x1's
//     operands (h from the accumulators, x_j's own columns) are prepared per wave, each step's
//     during the previous step's MFMAs.
// Every output column sums the same products in the same order as the executor's launches (conv A
// channel-block-major with taps inner, pwg_cnet_xtile_kernel / the DMA-ring kernel; the 1x1 in its
// chunk order [h blocks][x blocks], pwg_cnet_conv_kernel), with the same pre-activations, pair
// splits and epilogues (h = acc + b_A rounded to fp32 before the lrelu, exactly the value the
// executor stores and reloads): bit-identical (tests/test_gpu_vocoders.py::test_fused_stack_chain).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/pwg_cnet.h"
#include "pwg_internal.h"

namespace pwg {
namespace {

typedef float ms_f32x16 __attribute__((ext_vector_type(16)));
typedef float ms_f32x4 __attribute__((ext_vector_type(4)));
typedef float ms_f32x8 __attribute__((ext_vector_type(8)));
typedef unsigned ms_u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 ms_f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 ms_f16x2 __attribute__((ext_vector_type(2)));

constexpr int MS_NWV = 4, MS_NTH = 64 * MS_NWV;  // waves / threads per workgroup
constexpr int MS_CROW = 80;  // bytes per converted tile row (32 hi + 32 lo + pad: lanes on other banks)
// weight ring slots: P - 1 steps in flight. A step's MFMAs (~0.4 us) are far shorter than a
// fragment copy's round trip, so the ring runs deep: 3 slots measured 2.85 us per step on
// MB-MelGAN v2's 96-channel chain (the copy latency,
// profiles/r05_c); deepest that fits the LDS beside a 32-column block's tile and converted blocks
__host__ __device__ constexpr int ms_ring(int mt) { return mt <= 2 ? 6 : mt == 3 ? 5 : 3; }
// fragment units per step (taps of one conv-A channel block, or 1x1 chunks): 3, or 1 at 6 m-tiles
// (192 channels), whose 3-unit slots would not fit the LDS beside the 192-channel input tile
__host__ __device__ constexpr int ms_units(int mt) { return mt <= 4 ? 3 : 1; }

// row p of a T-row utterance under the edge mode (the executor's edge_row)
__device__ __forceinline__ bool ms_edge(int& p, int T, int mode) {
  if (mode == PWG_PAD_REFLECT) {
    p = p < 0 ? -p : p;
    p = p >= T ? 2 * (T - 1) - p : p;
    p = p < 0 ? 0 : (p >= T ? T - 1 : p);
    return true;
  }
  const bool inside = p >= 0 && p < T;
  p = p < 0 ? 0 : (p >= T ? T - 1 : p);
  return inside || mode == PWG_PAD_REPLICATE;
}

// 8 fp32 -> fp16 pairs hi = rne16(v), lo = rne16(v - hi) (the executor's cn_split8)
__device__ __forceinline__ void ms_split8(const ms_f32x8& v, ms_u32x4& hi, ms_u32x4& lo) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const _Float16 h0 = (_Float16)v[2 * d], h1 = (_Float16)v[2 * d + 1];
    hi[d] = __builtin_bit_cast(unsigned, ms_f16x2{h0, h1});
    lo[d] = __builtin_bit_cast(unsigned, ms_f16x2{(_Float16)(v[2 * d] - (float)h0), (_Float16)(v[2 * d + 1] - (float)h1)});
  }
}

__device__ __forceinline__ ms_f32x16 ms_mma3(const ms_u32x4& ah, const ms_u32x4& al, const ms_u32x4& bh,
                                              const ms_u32x4& bl, ms_f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(ms_f16x8, ah), __builtin_bit_cast(ms_f16x8, bh), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(ms_f16x8, ah), __builtin_bit_cast(ms_f16x8, bl), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(ms_f16x8, al), __builtin_bit_cast(ms_f16x8, bh), acc, 0, 0, 0);
  return acc;
}

// Keep a prepared operand where it is computed: without it the compiler sinks the preparation past
// the next step's wait and barrier, next to the MFMAs that use it, and nothing overlaps
__device__ __forceinline__ void ms_pin(ms_u32x4& v) { asm volatile("" : "+v"(v)); }

// LeakyReLU exactly as the executor computes it, unconditionally (slope 1: x either way), so the
// preparation has no branch. (x * (x > 0 ? 1 : slope) would let the compiler contract the product
// into the pair split's subtraction, an fma: other bits.)
__device__ __forceinline__ float ms_lrelu(float x, float slope) { return x > 0.f ? x : x * slope; }

template <int N>
__device__ __forceinline__ void ms_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt vmcnt(min(r, R) * D): wait for a step while the r steps issued after it may still land
template <int D, int R>
__device__ __forceinline__ void ms_vm_wait_steps(int r) {
  if constexpr (R > 0) {
    if (r >= R) {
      ms_vm_wait<R * D>();
      return;
    }
    ms_vm_wait_steps<D, R - 1>(r);
  } else {
    ms_vm_wait<0>();
  }
}

// f(integral_constant<int, i>) for i = B .. E - 1, unrolled at compile time (indices into
// accumulator arrays must be constants, or the compiler selects registers by runtime compares)
template <int B, int E, typename F>
__device__ __forceinline__ void ms_static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    ms_static_for<B + 1, E>(f);
  }
}

template <int CS>
struct MsShape {
  static constexpr int MT = (CS + 1) / 2;   // 32-row m-tiles (C rounded up to 32)
  static constexpr int C = 16 * CS;
  static constexpr int LDX = C + 4;          // floats per LDS tile row (16-B pad: lanes on other banks)
  static constexpr int G = ms_units(MT);     // units per step
  static constexpr int NI = G * MT * 2;      // 1-KB fragment copies per step (G taps or chunks, hi + lo)
  static constexpr int D = (NI + MS_NWV - 1) / MS_NWV;  // ... per wave (uniform: the last one repeats)
  static constexpr int SLOT = NI * 1024;
  static constexpr int SA = CS * (3 / G);           // conv-A steps per stack (block-major, taps inner)
  static constexpr int SB = (2 * CS + G - 1) / G;   // 1x1 steps per stack
  static constexpr int SPS = SA + SB;               // steps per stack
  static constexpr int P = ms_ring(MT);
};

#ifdef PWG_MSTACK_PROBE
// probe builds only: shader-clock stamps of workgroup 0, wave 0 (tools/diag/mstack_probe.py)
constexpr int MS_PROBE_N = 512;
__device__ unsigned long long g_ms_probe[MS_PROBE_N];
#endif

template <int CS, int TPW>
__global__ void __launch_bounds__(MS_NTH) pwg_mstack_kernel(const MstackArgs a) {
  using S = MsShape<CS>;
  constexpr int MT = S::MT, C = S::C, LDX = S::LDX;
  typedef __attribute__((address_space(1))) void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char ms_smem[];
  unsigned char* const ring = ms_smem;
  constexpr int P = S::P;
  float* const sx = reinterpret_cast<float*>(ms_smem + P * S::SLOT);
  const int xw = a.oc + 2 * a.halo;           // tile rows: utterance columns c0col .. c0col + xw - 1
  // conv A's B operands of one channel block, pre-activated and pair-split ONCE per workgroup for
  // all taps and waves: [2 blocks][xw rows][hi 16 f16 | lo 16 f16 | 16-B pad]
  unsigned char* const cbuf = reinterpret_cast<unsigned char*>(sx + (size_t)xw * LDX);
  float* const sb = reinterpret_cast<float*>(cbuf + (size_t)2 * xw * MS_CROW);  // [stack][b_A | b]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int hh = lane >> 5, cl = lane & 31;
  const int2 blk = a.blocks[blockIdx.x];
  const int2 sgx = *reinterpret_cast<const int2*>(a.seg_x + 2 * blk.x);
  const int2 sgy = *reinterpret_cast<const int2*>(a.seg_y + 2 * blk.x);
  const int T = sgx.y;
  const int c0col = blk.y - a.halo;
  const int ns = a.ns;
  int hout[MS_MAX];  // columns each side stack j still has to produce for the later ones
  {
    int h = 0;
#pragma unroll
    for (int j = MS_MAX - 1; j >= 0; --j) {
      hout[j] = h;
      if (j < ns) h += a.st[j].dil;
    }
  }
  // biases (ordinary loads, all landed before the first fragment copy)
  for (int i = threadIdx.x; i < ns * 2 * C; i += MS_NTH) {
    const int j = i / (2 * C), r = i - j * 2 * C;
    sb[i] = r < C ? a.st[j].bA[r] : a.st[j].bB[r - C];
  }
  // step s -> ring slot s % P: stack s / SPS, then SA conv-A steps (channel block r / (3 / G), its
  // taps G (r % (3 / G)) .. + G - 1) and SB 1x1 steps (chunks G (r - SA) .. + G - 1)
  const int n_steps = ns * S::SPS;
  // every per-stack value the loop needs, in registers before the first barrier: the barriers'
  // and waits' memory clobbers would otherwise reload them from the kernel arguments (a scalar
  // load round trip) in every step
  const float* wA_[MS_MAX];
  const float* wB_[MS_MAX];
#pragma unroll
  for (int k = 0; k < MS_MAX; ++k) {
    wA_[k] = a.st[k].wA;
    wB_[k] = a.st[k].wB;
  }
  auto issue = [&](int s) {
    const int j = s / S::SPS, r = s - j * S::SPS;
    unsigned char* const slot = ring + (size_t)(s % P) * S::SLOT;
    const float* const wa = j == 0 ? wA_[0] : j == 1 ? wA_[1] : j == 2 ? wA_[2] : wA_[3];
    const float* const wb = j == 0 ? wB_[0] : j == 1 ? wB_[1] : j == 2 ? wB_[2] : wB_[3];
#pragma unroll
    for (int k = 0; k < S::D; ++k) {
      const int i = wave + MS_NWV * k < S::NI ? wave + MS_NWV * k : S::NI - 1;
      const int g = i / (2 * MT), rem = i - g * 2 * MT, m = rem >> 1, hl = rem & 1;
      const float* src;
      if (r < S::SA) {
        const int cb = r / (3 / S::G), t = S::G * (r - cb * (3 / S::G)) + g;
        src = wa + ((size_t)(t * CS + cb) * MT + m) * 512 + hl * 256;
      } else {
        const int ch = min(S::G * (r - S::SA) + g, 2 * CS - 1);
        src = wb + ((size_t)ch * MT + m) * 512 + hl * 256;
      }
      __builtin_amdgcn_global_load_lds((gptr_t)(src + lane * 4), (lptr_t)(slot + i * 1024), 16, 0, 0);
    }
  };
  auto barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  ms_f32x16 accA[TPW][MT], accB[TPW][MT];
#ifdef PWG_MSTACK_PROBE
  const bool probe = blockIdx.x == 0 && threadIdx.x == 0;
  int np = 1;
  auto stamp = [&] {
    if (probe && np < MS_PROBE_N) g_ms_probe[np++] = __builtin_readcyclecounter();
  };
#else
  auto stamp = [] {};
#endif
  stamp();
  __syncthreads();  // biases in LDS (ordinary loads and stores, done before the first LDS copy)
  // the input tile: 1-KB copies of consecutive LDS bytes, each lane's 16 B from its row / quad
  // (pad quads and rows outside the utterance copy a harmless in-bounds quad)
  {
    const int bytes = xw * LDX * 4;
    const int n_ins = (bytes + 1023) / 1024;
    for (int k = wave; k < n_ins; k += MS_NWV) {
      const int o = k * 1024 + lane * 16;
      const int r = o / (LDX * 4), q = (o - r * LDX * 4) >> 4;
      int c = c0col + r;
      c = c < 0 ? 0 : (c >= T ? T - 1 : c);
      const float* src = a.x + (size_t)(sgx.x + c) * a.ld + 4 * (q < C / 4 ? q : 0);
      if (o < bytes)
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(reinterpret_cast<unsigned char*>(sx) + k * 1024), 16, 0, 0);
    }
  }

  // Software-pipelined steps: the operands of step s + 1 (A fragments and B rows from LDS,
  // pre-activation, pair split) are prepared while step s's MFMAs run, so one wave per SIMD keeps
  // its matrix pipe fed (a step's MFMAs are ~0.6k cycles, its operand work ~1.5k, and serially they
  // took ~2.5k cycles per step, tools/diag/mstack_probe.py). Step s + 1's fragments must therefore
  // be visible before step s computes: the ring holds P steps, step s + P issues once every wave has
  // prepared step s.
  for (int s0 = 0; s0 < P && s0 < n_steps; ++s0) issue(s0);
  int s = 0;
  // step s + 1 landed and visible (the steps issued after it may still be in flight); every wave
  // has prepared step s, so step s's slot takes step s + P
  auto advance = [&]() {
    stamp();  // (probe: previous step's work issued)
    if (s + 1 < n_steps) ms_vm_wait_steps<S::D, P - 2>(n_steps - 2 - s);
    stamp();
    barrier();
    stamp();
    if (s + P < n_steps) issue(s + P);
  };
  constexpr int G = S::G;
  int dil_[MS_MAX], pad_[MS_MAX], mode_[MS_MAX];
  float slopeA_[MS_MAX], slopeH_[MS_MAX];
#pragma unroll
  for (int k = 0; k < MS_MAX; ++k) {
    dil_[k] = a.st[k].dil;
    pad_[k] = a.st[k].pad;
    mode_[k] = a.st[k].mode;
    slopeA_[k] = a.st[k].slopeA;
    slopeH_[k] = a.st[k].slopeH;
  }
  // one step's operands: A fragments of its G units, B (hi, lo) per tile and unit
  ms_u32x4 ah[G][MT], al[G][MT], bh[TPW][G], bl[TPW][G];
  auto load_a = [&](int step) {
    const ms_u32x4* const sa = reinterpret_cast<const ms_u32x4*>(ring + (size_t)(step % P) * S::SLOT) + lane;
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        ah[g][m] = sa[(g * MT * 2 + m * 2) * 64];
        al[g][m] = sa[(g * MT * 2 + m * 2 + 1) * 64];
      }
  };
  auto pin_ops = [&]() {
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        ms_pin(ah[g][m]);
        ms_pin(al[g][m]);
      }
#pragma unroll
      for (int n = 0; n < TPW; ++n) {
        ms_pin(bh[n][g]);
        ms_pin(bl[n][g]);
      }
    }
  };
  int trow[TPW][3];  // conv A's tap rows of this lane's tiles in a converted block (x MS_CROW)
  int i0 = 0, nt = 0, dil = 1, pad = 0, mode = 0;
  float slopeA = 1.f, slopeH = 1.f;
  auto stack_setup = [&](int j) {
    auto pick = [&](const auto& arr) { return j == 0 ? arr[0] : j == 1 ? arr[1] : j == 2 ? arr[2] : arr[3]; };
    dil = pick(dil_); pad = pick(pad_); mode = pick(mode_);
    slopeA = pick(slopeA_); slopeH = pick(slopeH_);
    i0 = a.halo - hout[j];                // first tile row stack j produces
    nt = (a.oc + 2 * hout[j] + 31) >> 5;  // its 32-column tiles
#pragma unroll
    for (int n = 0; n < TPW; ++n)
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        // a zero-padded tap outside the utterance reads its own (converted-to-zero) tile row: the
        // taps of every stored column stay inside the tile (the halo); later tiles are garbage
        const int pu = c0col + i0 + 32 * (wave + MS_NWV * n) + cl - pad + t * dil;
        int p = pu;
        const int ir = (ms_edge(p, T, mode) ? p : pu) - c0col;
        trow[n][t] = (ir < 0 ? 0 : (ir >= xw ? xw - 1 : ir)) * MS_CROW;
      }
#pragma unroll
    for (int n = 0; n < TPW; ++n)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int e = 0; e < 16; ++e) accA[n][m][e] = accB[n][m][e] = 0.f;
  };
  // channel block cb of x_j for conv A, every tile row: lrelu (or 0 for a zero-padded row outside
  // the utterance: the executor's masked tap) and the pair split, into converted block cb & 1
  auto convert = [&](int cb) {
    unsigned char* const cv = cbuf + (size_t)(cb & 1) * xw * MS_CROW;
    for (int k = threadIdx.x; k < 2 * xw; k += MS_NTH) {
      const int i = k >> 1, hf = k & 1;
      const float* xr = sx + (size_t)i * LDX + 16 * cb + 8 * hf;
      const ms_f32x4 v0 = *reinterpret_cast<const ms_f32x4*>(xr), v1 = *reinterpret_cast<const ms_f32x4*>(xr + 4);
      ms_f32x8 x = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      const int c = c0col + i;
      const bool z = mode == PWG_PAD_ZERO && (c < 0 || c >= T);
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = z ? 0.f : ms_lrelu(x[e], slopeA);
      ms_u32x4 h, l;
      ms_split8(x, h, l);
      *reinterpret_cast<ms_u32x4*>(cv + (size_t)i * MS_CROW + 16 * hf) = h;
      *reinterpret_cast<ms_u32x4*>(cv + (size_t)i * MS_CROW + 32 + 16 * hf) = l;
    }
  };
  // conv A step r: channel block cb, taps t0 .. t0 + G - 1 (pwg_cnet_xtile_kernel's order), B read
  // straight from the converted block. Tiles past the stack's range compute garbage that is never
  // stored (no branch: the loads and the MFMAs stay one scheduling region)
  auto load_conv = [&](int step, int r) {
    load_a(step);
    const int cb = r / (3 / G), t0 = G * (r - cb * (3 / G));
    const unsigned char* const cv = cbuf + (size_t)(cb & 1) * xw * MS_CROW + 16 * hh;
#pragma unroll
    for (int n = 0; n < TPW; ++n)
#pragma unroll
      for (int t = 0; t < G; ++t) {
        const int tr = G == 3 ? trow[n][t] : (t0 == 0 ? trow[n][0] : t0 == 1 ? trow[n][1] : trow[n][2]);
        bh[n][t] = *reinterpret_cast<const ms_u32x4*>(cv + tr);
        bl[n][t] = *reinterpret_cast<const ms_u32x4*>(cv + tr + 32);
      }
    pin_ops();
  };
  auto mma_conv = [&]() {
#pragma unroll
    for (int n = 0; n < TPW; ++n)
#pragma unroll
      for (int t = 0; t < G; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m) accA[n][m] = ms_mma3(ah[t][m], al[t][m], bh[n][t], bl[n][t], accA[n][m]);
  };
  // the 1x1 over [lrelu(h); x_j], step kg: chunks G kg .. + G - 1 of [h blocks][x blocks], compile-
  // time (h's accumulator registers are indexed statically)
  auto prep_mm1 = [&](int step, int j, auto kgc) {
    constexpr int kg = decltype(kgc)::value;
    load_a(step);
    const float* const bA = sb + (size_t)j * 2 * C;
    ms_static_for<0, G>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      constexpr int ch = G * kg + g;
      if constexpr (ch < 2 * CS) {
#pragma unroll
        for (int n = 0; n < TPW; ++n) {
          ms_f32x8 x;
          if constexpr (ch < CS) {
            // h channels 16 ch .. + 15 from conv A's accumulators: lane half hh needs rows
            // 8 (J0 + hh) + 0..7, i.e. rows 8 (J0 + hh) + 0..3 (j4 = J0 + hh of half 0) and + 4..7
            // (the same j4 of half 1). With A = acc[j4 = J0], B = acc[j4 = J0 + 1] (rows + 4 hh):
            // half 0 takes (A, A of half 1), half 1 (B of half 0, B): one cross-half exchange of
            // each (the selects pick between two values, never between accumulator registers)
            constexpr int mh = ch >> 1, J0 = (ch & 1) * 2;
            const float* bb = bA + 16 * ch + 8 * hh;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float va = accA[n][mh][4 * J0 + e], vb = accA[n][mh][4 * (J0 + 1) + e];
              const float xa = __shfl_xor(va, 32), xb = __shfl_xor(vb, 32);
              x[e] = (hh ? xb : va) + bb[e];
              x[4 + e] = (hh ? vb : xa) + bb[4 + e];
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = ms_lrelu(x[e], slopeH);
          } else {
            const int i = i0 + 32 * (wave + MS_NWV * n) + cl;
            const int ir = i < xw ? i : xw - 1;
            const float* xr = sx + (size_t)ir * LDX + 16 * (ch - CS) + 8 * hh;
            const ms_f32x4 v0 = *reinterpret_cast<const ms_f32x4*>(xr), v1 = *reinterpret_cast<const ms_f32x4*>(xr + 4);
            x = ms_f32x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
          }
          ms_split8(x, bh[n][g], bl[n][g]);
        }
      }
    });
    pin_ops();
  };
  auto mma_mm1 = [&](auto kgc) {
    constexpr int kg = decltype(kgc)::value;
    ms_static_for<0, G>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      if constexpr (G * kg + g < 2 * CS) {
#pragma unroll
        for (int n = 0; n < TPW; ++n)
#pragma unroll
          for (int m = 0; m < MT; ++m) accB[n][m] = ms_mma3(ah[g][m], al[g][m], bh[n][g], bl[n][g], accB[n][m]);
      }
    });
  };

  // a stack starts once x_j is in the tile (a barrier): its first two channel blocks converted,
  // then step s's operands
  auto begin_stack = [&](int j) {
    stack_setup(j);
    convert(0);
    if constexpr (G == 3) convert(1);
    barrier();
    load_conv(s, 0);
  };
  // prologue: step 0 (and the input tile) landed
  ms_vm_wait_steps<S::D, P - 1>(n_steps - 1);
  barrier();
  begin_stack(0);
  for (int j = 0; j < ns; ++j) {
    // step r: its MFMAs, then step r + 1's operands and step r + 2's channel block (into the
    // converted block step r read from, free once every wave passed this step's barrier). No
    // branch between a step's MFMAs and the next step's loads: one scheduling region
    for (int r = 0; r + 2 < S::SA; ++r, ++s) {
      advance();
      mma_conv();
      load_conv(s + 1, r + 1);
      if constexpr (G == 3) {
        convert(r + 2);
      } else {
        if ((r + 2) % 3 == 0) convert((r + 2) / 3);
      }
    }
    advance();
    mma_conv();
    load_conv(s + 1, S::SA - 1);
    ++s;
    advance();
    mma_conv();
    prep_mm1(s + 1, j, std::integral_constant<int, 0>{});  // waits for conv A's last MFMAs
    ++s;
    ms_static_for<0, S::SB>([&](auto kgc) {
      constexpr int kg = decltype(kgc)::value;
      advance();
      mma_mm1(kgc);
      if constexpr (kg + 1 < S::SB) prep_mm1(s + 1, j, std::integral_constant<int, kg + 1>{});
      ++s;
    });
    // ---- epilogue of stack j: x_j+1 = acc + b into the tile (own columns), or, for the last
    // stack, y; then every wave's tile rows are visible before the next stack's first operands
    const float* const bB = sb + (size_t)j * 2 * C + C;
    const bool last = j == ns - 1;
#pragma unroll
    for (int n = 0; n < TPW; ++n) {
      const int tile = wave + MS_NWV * n;
      if (tile >= nt) break;
      const int i = i0 + 32 * tile + cl;
      const int c = c0col + i;
      const bool live = last ? (i >= a.halo && i < a.halo + a.oc && c < T) : i < xw;
      if (!live) continue;
      float* const dst = last ? a.y + (size_t)(sgy.x + c) * a.ld : sx + (size_t)i * LDX;
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const int row = 32 * m + 8 * j4 + 4 * hh;
          if (row >= C) continue;
          ms_f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = accB[n][m][4 * j4 + e] + bB[row + e];
          *reinterpret_cast<ms_f32x4*>(dst + row) = v;
        }
    }
    if (j + 1 < ns) {
      barrier();
      begin_stack(j + 1);
    }
  }
#ifdef PWG_MSTACK_PROBE
  stamp();
  if (probe) g_ms_probe[0] = (unsigned long long)np | ((unsigned long long)n_steps << 16) | ((unsigned long long)CS << 32);
#endif
}

template <int CS, int TPW>
hipError_t ms_go(const MstackArgs& a, int n_blocks, hipStream_t s) {
  const int lds = mstack_lds(CS, a.oc, a.halo, a.ns);
  const hipError_t e = allow_lds(reinterpret_cast<const void*>(pwg_mstack_kernel<CS, TPW>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((pwg_mstack_kernel<CS, TPW>), dim3((unsigned)n_blocks), dim3(MS_NTH), (size_t)lds, s, a);
  return hipGetLastError();
}

}  // namespace

int mstack_lds(int cs, int oc, int halo, int ns) {
  const int mt = (cs + 1) / 2;
  return ms_ring(mt) * ms_units(mt) * mt * 2 * 1024 + (oc + 2 * halo) * ((16 * cs + 4) * 4 + 2 * MS_CROW) +
         ns * 2 * 16 * cs * 4;
}

// accumulators: 2 x TPW x MT x 16 VGPRs; TPW x MT <= 4 (or one tile of 192 channels, one fragment unit
// per step) keeps the kernel within one wave per SIMD's registers without spills
bool mstack_supported(int cs, int tpw) {
  const int mt = (cs + 1) / 2;
  return ((cs == 2 || cs == 3 || cs == 4 || cs == 6 || cs == 8) && (tpw == 1 || tpw == 2) && tpw * mt <= 4) ||
         (cs == 12 && tpw == 1);
}

hipError_t launch_mstack(const MstackArgs& a, int cs, int tpw, int n_blocks, hipStream_t s) {
  if (!mstack_supported(cs, tpw) || a.ns < 1 || a.ns > MS_MAX || n_blocks < 1) return hipErrorInvalidValue;
  if (tpw == 1) {
    switch (cs) {
      case 2: return ms_go<2, 1>(a, n_blocks, s);
      case 3: return ms_go<3, 1>(a, n_blocks, s);
      case 4: return ms_go<4, 1>(a, n_blocks, s);
      case 6: return ms_go<6, 1>(a, n_blocks, s);
      case 8: return ms_go<8, 1>(a, n_blocks, s);
      case 12: return ms_go<12, 1>(a, n_blocks, s);
    }
  } else {
    switch (cs) {
      case 2: return ms_go<2, 2>(a, n_blocks, s);
      case 3: return ms_go<3, 2>(a, n_blocks, s);
      case 4: return ms_go<4, 2>(a, n_blocks, s);
    }
  }
  return hipErrorInvalidValue;
}

}  // namespace pwg

#ifdef PWG_MSTACK_PROBE
extern "C" __attribute__((visibility("default"))) int pwg_mstack_debug_probe(unsigned long long* out, int n) {
  if (!out || n < pwg::MS_PROBE_N) return 1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(pwg::g_ms_probe), sizeof(unsigned long long) * pwg::MS_PROBE_N) == hipSuccess ? 0 : 3;
}
#endif
