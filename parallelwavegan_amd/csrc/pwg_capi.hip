// C-ABI of the engine (include/pwg.h): config validation, weight packing, batch planning,
// launch sequencing and HIP-event timing. Kernels live in pwg_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/pwg.h"
#include "pwg_internal.h"

#ifndef PWG_SMALL_SPREAD
#define PWG_SMALL_SPREAD 1  // small plans: fewer waves per workgroup, every CU (A/B: 0)
#endif

using namespace pwg;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(PWG_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

size_t align64(size_t n) { return (n + 63) / 64 * 64; }
size_t align_bytes(size_t n) { return (n + 255) / 256 * 256; }

struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) { ok = false; return; }
    if (prev != dev && hipSetDevice(dev) != hipSuccess) ok = false;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// fp16 round-to-nearest-even on the host (split-f16 weight packing); h2f is its exact inverse.
uint16_t f2h(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u, ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return (uint16_t)(sign | (ax > 0x7f800000u ? 0x7e00u : 0x7c00u));
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds to infinity
  if (ax < 0x38800000u) {                                     // half subnormal: units of 2^-24
    float v;
    std::memcpy(&v, &ax, 4);
    return (uint16_t)(sign | (uint32_t)std::nearbyint(v * 16777216.0f));
  }
  uint32_t h = (((ax >> 23) - 112u) << 10) | ((ax & 0x7fffffu) >> 13);
  const uint32_t rem = ax & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
  return (uint16_t)(sign | h);
}

float h2f(uint16_t h) {
  const uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  float v;
  if (e == 0) v = std::ldexp((float)m, -24);
  else if (e == 31) v = m ? NAN : INFINITY;
  else v = std::ldexp((float)(m | 0x400u), (int)e - 25);
  return (h & 0x8000u) ? -v : v;
}

// Values pwg_pack_weights split into fp16 pairs that left the fp16 range (|v| >= 65520 rounds
// to inf): such an image is refused for the split-f16 kernels (PWG_ERR_RANGE).
thread_local long long g_split_overflow = 0;

// v ~= hi + lo as fp16 (hi = rne(v), lo = rne(v - hi)); returns hi | lo << 16
uint32_t split_pair(float v) {
  const uint16_t hi = f2h(v);
  if ((hi & 0x7c00u) == 0x7c00u) ++g_split_overflow;
  const uint16_t lo = f2h(v - h2f(hi));
  return (uint32_t)hi | ((uint32_t)lo << 16);
}

// Channel held by slot p = 8s + j of lane half hh in the split layout (pwg_split.hip header).
int split_chan(int s, int hh, int j) { return 32 * (s >> 1) + 16 * (s & 1) + 8 * (j >> 2) + 4 * hh + (j & 3); }

struct TimingRecord {
  int bucket;
  hipEvent_t start, stop;
};

// ---------------------------------------------------------------------------------------------
// Composite upsampler tables (AuxTab). The reference upsampler (layers/upsample.py:112-128) is,
// per channel, a linear map from T' frames to T = T'*H samples: U[t][f]. Rows whose dependency
// cone never meets a zero-padded boundary equal the periodic interior kernel; the first TL / last
// TR rows see the left / right boundary only and depend on t / T-1-t alone once F >= Fmin; shorter
// utterances get their full matrices. Everything is computed by running the staged upsampler on
// unit impulses in double precision and then VERIFIED row by row against the exact matrix.

struct AuxStruct {
  long long H = 1;
  int J1 = 0, J2 = 0, J = 1, TL = 0, TR = 0, Fmin = 1;
  int nka = 1, nfwg = 1;
};

// One stage: Stretch2d (nearest: out[t] = in[t / s]; bilinear along time, align_corners=False as
// aten's upsample_bilinear2d: src = max((t + 0.5) / s - 0.5, 0), i0 = floor(src), i1 = min(i0 + 1,
// n - 1), out[t] = (1 - l) in[i0] + l in[i1], l = src - i0), then the (2s+1)-tap FIR with zero
// padding s (causal: 2s, trimmed).
void up_stage(const std::vector<double>& in, int s, const double* h, bool causal, int mode,
              std::vector<double>& out) {
  const long long n_in = (long long)in.size(), n = n_in * s;
  std::vector<double> st((size_t)n);
  for (long long t = 0; t < n; ++t) {
    if (mode == 0) {
      st[t] = in[t / s];
    } else {  // src = (2t + 1 - s) / 2s in exact integers: the same weight for every period
      const long long num = std::max(2 * t + 1 - s, 0LL);
      const long long i0 = num / (2 * s);
      const long long i1 = std::min(i0 + 1, n_in - 1);
      const double l = (double)(num % (2 * s)) / (double)(2 * s);
      st[t] = (1.0 - l) * in[i0] + l * in[i1];
    }
  }
  const int P = causal ? 2 * s : s;
  out.assign(n, 0.0);
  for (long long t = 0; t < n; ++t) {
    double v = 0.0;
    for (int k = 0; k < 2 * s + 1; ++k) {
      const long long u = t + k - P;
      if (u >= 0 && u < n) v += h[k] * st[u];
    }
    out[t] = v;
  }
}

// Exact U for F frames, row-major [F*H][F].
std::vector<double> upsample_matrix(const PwgConfig& c, const std::vector<std::vector<double>>& taps, int F,
                                    long long H) {
  std::vector<double> M((size_t)(F * H) * F, 0.0), a, b;
  for (int f = 0; f < F; ++f) {
    a.assign(F, 0.0);
    a[f] = 1.0;
    for (int i = 0; i < c.num_scales; ++i) {
      up_stage(a, c.upsample_scales[i], taps[i].data(), c.use_causal_conv != 0, c.interpolate_mode, b);
      a.swap(b);
    }
    for (long long t = 0; t < F * H; ++t) M[(size_t)t * F + f] = a[t];
  }
  return M;
}

long long floordiv_h(long long a, long long b) {
  long long q = a / b;
  if ((a % b != 0) && (a < 0)) --q;
  return q;
}

// Frame window [t/H - J1, t/H + J2] of every output row, from the stage dependency ranges.
void aux_window(const PwgConfig& c, long long H, int* J1, int* J2) {
  const long long fm = 64;
  int j1 = 0, j2 = 0;
  for (long long p = 0; p < H; ++p) {
    long long lo = fm * H + p, hi = lo + 1;
    for (int i = c.num_scales - 1; i >= 0; --i) {
      const int s = c.upsample_scales[i];
      const int P = c.use_causal_conv ? 2 * s : s;
      lo = floordiv_h(lo - P, s);
      hi = floordiv_h(hi - 1 + 2 * s - P, s) + 1;
    }
    j1 = std::max(j1, (int)(fm - lo));
    j2 = std::max(j2, (int)(hi - 1 - fm));
  }
  *J1 = j1;
  *J2 = j2;
}

// The same window for any stretch mode, from the exact matrix of positive generic taps: the
// interior rows' nonzero frames relative to t / H (bilinear stretch reaches one more input
// sample per stage than nearest).
int aux_window_numeric(const PwgConfig& c, long long H, const std::vector<std::vector<double>>& taps, int* J1,
                       int* J2);

// Row weights as the layer kernel selects them (w has AUX_J4 entries).
void decomposed_row(const AuxStruct& st, const std::vector<float>& interior, const std::vector<float>& left,
                    const std::vector<float>& right, const std::vector<float>& small, long long F, long long t,
                    float* w) {
  const long long T = F * st.H;
  const float* row;
  if (F < st.Fmin) row = small.data() + (st.H * F * (F - 1) / 2 + t) * AUX_J4;
  else if (t < st.TL) row = left.data() + t * AUX_J4;
  else if (t >= T - st.TR) row = right.data() + (T - 1 - t) * AUX_J4;
  else row = interior.data() + (t % st.H) * AUX_J4;
  for (int j = 0; j < AUX_J4; ++j) w[j] = row[j];
}

void exact_row(const AuxStruct& st, const std::vector<double>& M, long long F, long long t, double* w) {
  for (int j = 0; j < AUX_J4; ++j) {
    const long long f = t / st.H - st.J1 + j;
    w[j] = (j < st.J && f >= 0 && f < F) ? M[(size_t)t * F + f] : 0.0;
  }
}

int aux_window_numeric(const PwgConfig& c, long long H, const std::vector<std::vector<double>>& taps, int* J1,
                       int* J2) {
  const int Fb = 24;
  const long long fm = Fb / 2;
  const std::vector<double> M = upsample_matrix(c, taps, Fb, H);
  int j1 = 0, j2 = 0;
  for (long long p = 0; p < H; ++p) {
    const long long t = fm * H + p;
    for (int f = 0; f < Fb; ++f) {
      if (M[(size_t)t * Fb + f] == 0.0) continue;
      j1 = std::max(j1, (int)(fm - f));
      j2 = std::max(j2, (int)(f - fm));
    }
  }
  if (j1 >= fm - 2 || j2 >= fm - 2) return fail(PWG_ERR_UNSUPPORTED, "composite upsampler window too wide");
  *J1 = j1;
  *J2 = j2;
  return PWG_OK;
}

// Structure (TL, TR, Fmin, window sizes) from generic taps; tables from the real taps.
int aux_structure(const PwgConfig& c, AuxStruct* st) {
  long long H = 1;
  for (int i = 0; i < c.num_scales; ++i) H *= c.upsample_scales[i];
  st->H = H;
  if (H < 2 || H > 4096) return fail(PWG_ERR_UNSUPPORTED, "upsample factor must be in [2, 4096]");
  if (c.interpolate_mode != 0 && c.interpolate_mode != 1)
    return fail(PWG_ERR_UNSUPPORTED, "interpolate_mode must be 0 (nearest) or 1 (bilinear)");
  // bilinear: the reference's source index (t + 0.5) / s - 0.5 is fp32 (aten opmath), exact for
  // power-of-two scales; at other scales its rounding grows with t (~t 2^-24 / s: 3e-3 of a weight
  // at a million samples), which no periodic table reproduces, so those are refused
  if (c.interpolate_mode == 1)
    for (int i = 0; i < c.num_scales; ++i)
      if ((c.upsample_scales[i] & (c.upsample_scales[i] - 1)) != 0)
        return fail(PWG_ERR_UNSUPPORTED, "interpolate_mode bilinear needs power-of-two upsample scales");
  // generic taps: the unclean row set is structural (boundary truncation), not value-dependent
  std::vector<std::vector<double>> taps(c.num_scales);
  uint64_t x = 0x9E3779B97F4A7C15ULL;
  for (int i = 0; i < c.num_scales; ++i)
    for (int k = 0; k < 2 * c.upsample_scales[i] + 1; ++k) {
      x = x * 6364136223846793005ULL + 1442695040888963407ULL;
      taps[i].push_back(0.5 + (double)(x >> 11) / (double)(1ULL << 53));
    }
  if (c.interpolate_mode == 0) {
    aux_window(c, H, &st->J1, &st->J2);
  } else {
    const int rc = aux_window_numeric(c, H, taps, &st->J1, &st->J2);
    if (rc != PWG_OK) return rc;
  }
  st->J = st->J1 + st->J2 + 1;
  if (st->J > AUX_J4) return fail(PWG_ERR_UNSUPPORTED, "composite upsampler spans more than 8 frames");
  const int Fb = 24;
  const std::vector<double> M = upsample_matrix(c, taps, Fb, H);
  const long long T = Fb * H, fm = Fb / 2;
  int TL = 0, TR = 0;
  for (long long t = 0; t < T; ++t) {
    double w[AUX_J4];
    exact_row(*st, M, Fb, t, w);
    bool clean = true;
    for (int j = 0; j < st->J; ++j)
      if (std::fabs(w[j] - M[(size_t)(fm * H + t % H) * Fb + fm - st->J1 + j]) > 1e-13) clean = false;
    if (!clean) {
      if (t < T / 2) TL = std::max(TL, (int)(t + 1));
      else TR = std::max(TR, (int)(T - t));
    }
  }
  st->TL = TL;
  st->TR = TR;
  st->Fmin = (int)((TL + TR + H - 1) / H) + 1;
  if (st->Fmin + 4 > Fb) return fail(PWG_ERR_UNSUPPORTED, "upsampler edge region too wide");
  // aux k-steps per 32-sample wave window and frames per 128-sample workgroup window
  int cnt = 0, nfwg = 0;
  for (long long t0 = 0; t0 < 128 * H; t0 += 32)
    cnt = std::max(cnt, (int)((t0 + 31) / H - t0 / H) + st->J);
  st->nka = (cnt + 1) / 2;
  for (long long t0 = 0; t0 < 128 * H; t0 += TILE)
    for (int w = 0; w < 4; ++w)
      nfwg = std::max(nfwg, (int)((t0 + 32 * w) / H - t0 / H) + 2 * st->nka);
  st->nfwg = nfwg;
  if (nfwg > AUX_MAX_NFWG) return fail(PWG_ERR_UNSUPPORTED, "upsample factor too small for the aux frame window");
  return PWG_OK;
}

int aux_tables(const PwgConfig& c, const AuxStruct& st, const std::vector<std::vector<double>>& taps,
               std::vector<float>& interior, std::vector<float>& left, std::vector<float>& right,
               std::vector<float>& small) {
  const long long H = st.H;
  const int Fb = 24;
  const long long fm = Fb / 2;
  const std::vector<double> Mb = upsample_matrix(c, taps, Fb, H);
  const long long Tb = Fb * H;
  interior.assign((size_t)H * AUX_J4, 0.f);
  left.assign((size_t)std::max(st.TL, 1) * AUX_J4, 0.f);
  right.assign((size_t)std::max(st.TR, 1) * AUX_J4, 0.f);
  small.assign((size_t)std::max<long long>(H * st.Fmin * (st.Fmin - 1) / 2, 1) * AUX_J4, 0.f);
  double w[AUX_J4];
  for (long long p = 0; p < H; ++p) {
    exact_row(st, Mb, Fb, fm * H + p, w);
    for (int j = 0; j < AUX_J4; ++j) interior[p * AUX_J4 + j] = (float)w[j];
  }
  for (long long t = 0; t < st.TL; ++t) {
    exact_row(st, Mb, Fb, t, w);
    for (int j = 0; j < AUX_J4; ++j) left[t * AUX_J4 + j] = (float)w[j];
  }
  for (long long q = 0; q < st.TR; ++q) {
    exact_row(st, Mb, Fb, Tb - 1 - q, w);
    for (int j = 0; j < AUX_J4; ++j) right[q * AUX_J4 + j] = (float)w[j];
  }
  for (int F = 1; F < st.Fmin; ++F) {
    const std::vector<double> M = upsample_matrix(c, taps, F, H);
    for (long long t = 0; t < F * H; ++t) {
      exact_row(st, M, F, t, w);
      for (int j = 0; j < AUX_J4; ++j) small[(H * F * (F - 1) / 2 + t) * AUX_J4 + j] = (float)w[j];
    }
  }
  // verify the decomposition against exact matrices (every row, every frame)
  double scale = 0.0;
  for (double v : Mb) scale = std::max(scale, std::fabs(v));
  const double tol = 1e-6 * std::max(scale, 1e-30);  // fp32 storage of the weights
  std::vector<int> Fs;
  for (int F = 1; F < st.Fmin + 4; ++F) Fs.push_back(F);
  Fs.push_back(Fb);
  for (int F : Fs) {
    const std::vector<double> M = F == Fb ? Mb : upsample_matrix(c, taps, F, H);
    for (long long t = 0; t < F * H; ++t) {
      float wd[AUX_J4];
      decomposed_row(st, interior, left, right, small, F, t, wd);
      for (int f = 0; f < F; ++f) {
        const long long j = f - (t / H - st.J1);
        const double got = (j >= 0 && j < AUX_J4) ? (double)wd[j] : 0.0;
        if (std::fabs(got - M[(size_t)t * F + f]) > tol)
          return fail(PWG_ERR_INVALID, "internal: composite upsampler table does not reproduce the reference upsampler");
      }
    }
  }
  return PWG_OK;
}

}  // namespace

struct PwgHandle {
  PwgConfig cfg;
  int device;
  // derived shapes
  int R, RS, G, GH, GHPAD, GR, MT, S, SS, M2T, A, KS, KW, O, L, lps, K1, NQ, NQ4;
  long long gap;  // zero columns between utterance segments (>= the largest tap offset)
  std::vector<int> dil;
  AuxStruct aux;
  // packed image offsets (floats)
  size_t off_first_w, off_first_b, off_conv_in, off_conv_in_frag, off_waux;
  size_t off_tab_interior, off_tab_left, off_tab_right, off_tab_small;
  size_t off_layers, layer_stride, lo_wg, lo_bg, lo_w2;
  size_t off_head_w1, off_head_w2, off_head_b2, packed_total;
  int M3T;
  long long ref_total;
  size_t lo_wgp;
  // split-f16 layer kernel (R = S = 64, 128 gate rows, kernel 3): per-layer image + skip-bias sum
  int split_ok = 0;
  size_t lo_split = 0, off_skip0 = 0;
  // 16x16x32 variant (pwg_split16.hip): its own layer image, skip-bias sum and head
  size_t lo_split16 = 0, off_skip0_16 = 0, off_head16_w1 = 0, off_head16_w2 = 0;
  // options
  int layer_kernel = 0, waves_per_wg = 8, wg_per_cu = 1;
  int fuse_first = 1;  // PWG_OPT_FUSE_FIRST_CONV
  long long pipe_max = PWG_PIPE_MAX_DEFAULT;  // PWG_OPT_PIPELINE: largest padded plan on the layer pipeline
  int sync_abort = 0;       // PWG_OPT_SYNC_ABORT (test hook)
  int sync_timeout = 0;     // PWG_OPT_SYNC_TIMEOUT (test hook)
  long long sync_max = -1;  // PWG_OPT_SYNC: most 32-sample blocks on the grid-synchronised forward (-1: 64 x n_cu)
  long long half_max = -1;  // PWG_OPT_HALF_BLOCKS: most blocks of a half-block launch (-1: 4 x n_cu)
  int n_cu = 0;
  // sticky run status (device, one int on its own 256-B allocation, zeroed once): every status bit a
  // run sets is also ORed here, pwg_run_status reports and clears it (allocated by the first pwg_run)
  int* d_status = nullptr;
  // diagnostic per-wave timeline of the split16 layer launches (PWG_TRACE_FILE, read once at
  // pwg_create; tools/trace_layer.py): this handle's device buffer, grown to the largest run
  std::string trace_fn;
  unsigned long long* d_trace = nullptr;
  size_t trace_words = 0;
  // timing
  int timing = 0;  // pwg_set_timing: 1 per-launch events, 2 one event pair around each run
  std::vector<TimingRecord> records;
  std::vector<hipEvent_t> event_pool;
  // pinned host words pwg_run_status copies the run's and the sticky status into, per caller stream
  // (a copy into pageable memory takes HIP's staged path, ~10-20 us of a B = 1 call)
  std::map<hipStream_t, int*> hstatus;
  std::mutex hstatus_mu;
};

struct PwgPlan {
  PwgHandle* h;
  int layout;
  int n_utts;
  std::vector<UttDesc> utts;
  long long n_tiles, n_gap_tiles, Tpad, F_total, T_total;
  // workspace offsets (bytes); the descriptor arrays (utts, tile_utt, gap_col0, blocks) are
  // written by pwg_plan_desc_kernel at the start of every pwg_run
  size_t ws_x0, ws_x1, ws_skip, ws_c1, ws_d, ws_ctr, ws_flag;
  size_t ws_utts, ws_tile_utt, ws_gap, ws_blocks, ws_total;
  // layer pipeline (split16, plans whose residual plane fits 2 GB): third plane + progress words
  bool pipe_ok = false;
  size_t ws_x2 = 0, ws_prog = 0;
  long long max_blocks_per_utt = 0;
};

extern "C" {

int pwg_abi_version(void) { return PWG_ABI_VERSION; }
const char* pwg_last_error(void) { return g_err.c_str(); }

int pwg_create(const PwgConfig* cfg, int device, PwgHandle** out) {
  if (!cfg || !out) return fail(PWG_ERR_INVALID, "null argument");
  const PwgConfig& c = *cfg;
  if (c.in_channels != 1) return fail(PWG_ERR_UNSUPPORTED, "in_channels != 1 is not supported");
  if (c.out_channels < 1) return fail(PWG_ERR_INVALID, "out_channels must be >= 1");
  if (c.layers < 1 || c.stacks < 1) return fail(PWG_ERR_INVALID, "layers and stacks must be >= 1");
  if (c.layers % c.stacks != 0) return fail(PWG_ERR_ASSERT, "layers % stacks == 0");
  if (c.kernel_size < 1) return fail(PWG_ERR_INVALID, "kernel_size must be >= 1");
  if (!c.use_causal_conv && (c.kernel_size - 1) % 2 != 0)
    return fail(PWG_ERR_ASSERT, "Not support even number kernel size.");
  if (c.gate_channels < 2 || c.gate_channels % 2 != 0)
    return fail(PWG_ERR_INVALID, "gate_channels must be even (split into tanh/sigmoid halves)");
  if (c.residual_channels < 1 || c.skip_channels < 1 || c.aux_channels < 1)
    return fail(PWG_ERR_UNSUPPORTED, "residual/skip/aux channels must be >= 1");
  if (c.residual_channels % 8 != 0 || c.skip_channels % 8 != 0)
    return fail(PWG_ERR_UNSUPPORTED, "residual_channels and skip_channels must be multiples of 8");
  if (c.aux_context_window < 0) return fail(PWG_ERR_INVALID, "aux_context_window must be >= 0");
  if (c.num_scales < 1 || c.num_scales > PWG_MAX_SCALES)
    return fail(PWG_ERR_UNSUPPORTED, "1..8 upsample scales supported");
  for (int i = 0; i < c.num_scales; ++i)
    if (c.upsample_scales[i] < 1) return fail(PWG_ERR_INVALID, "upsample scales must be >= 1");

  PwgHandle* h = new PwgHandle();
  if (const char* tf = getenv("PWG_TRACE_FILE")) h->trace_fn = tf;
  h->cfg = c;
  h->device = device;
  h->R = c.residual_channels;
  h->G = c.gate_channels;
  h->GH = c.gate_channels / 2;
  h->S = c.skip_channels;
  h->A = c.aux_channels;
  h->KS = c.kernel_size;
  h->O = c.out_channels;
  h->L = c.layers;
  h->lps = c.layers / c.stacks;
  h->KW = c.use_conv_in ? (c.use_causal_conv ? c.aux_context_window + 1 : 2 * c.aux_context_window + 1) : 1;
  h->GHPAD = h->GH <= 16 ? 16 : (h->GH + 31) / 32 * 32;
  h->MT = h->GHPAD <= 16 ? 1 : h->GHPAD / 16;
  h->NQ = h->GHPAD / 2;
  h->GR = 32 * h->MT;
  h->M2T = (h->S + h->R + 31) / 32;
  h->RS = (h->R + KC - 1) / KC * KC;
  h->SS = (h->S + 3) / 4 * 4;
  h->NQ4 = (h->NQ + 1 + 3) / 4;
  h->K1 = h->KS * h->RS;
  if (!(h->MT == 1 || h->MT == 2 || h->MT == 4) || !(h->M2T == 1 || h->M2T == 2 || h->M2T == 4)) {
    delete h;
    return fail(PWG_ERR_UNSUPPORTED, "gate_channels <= 128 and skip+residual <= 128 supported");
  }
  if (h->S > 128) { delete h; return fail(PWG_ERR_UNSUPPORTED, "skip_channels <= 128 supported"); }
  if (h->A > 128) { delete h; return fail(PWG_ERR_UNSUPPORTED, "aux_channels <= 128 supported"); }
  long long dmax = 1;
  for (int l = 0; l < h->L; ++l) {
    long long d = 1LL << (l % h->lps);
    if (d > (1LL << 20)) { delete h; return fail(PWG_ERR_UNSUPPORTED, "dilation too large"); }
    h->dil.push_back((int)d);
    dmax = std::max(dmax, d);
  }
  {
    const long long center = c.use_causal_conv ? h->KS - 1 : (h->KS - 1) / 2;
    const long long halo = std::max(center, (long long)h->KS - 1 - center) * dmax;
    h->gap = (halo + TILE - 1) / TILE * TILE;
  }
  {
    const int rc = aux_structure(c, &h->aux);
    if (rc != PWG_OK) { delete h; return rc; }
  }
  // packed image layout
  size_t o = 0;
  h->off_first_w = o; o += align64(h->R);
  h->off_first_b = o; o += align64(h->R);
  h->off_conv_in = o; o += align64((size_t)h->A * h->A * h->KW);
  h->off_conv_in_frag = o; o += align64((size_t)(h->A * h->KW + 1) / 2 * ((h->A + 31) / 32) * 64);
  h->off_waux = o; o += align64((size_t)h->L * ((h->A + 1) / 2) * h->MT * 64);
  h->off_tab_interior = o; o += align64((size_t)h->aux.H * AUX_J4);
  h->off_tab_left = o; o += align64((size_t)std::max(h->aux.TL, 1) * AUX_J4);
  h->off_tab_right = o; o += align64((size_t)std::max(h->aux.TR, 1) * AUX_J4);
  h->off_tab_small = o;
  o += align64((size_t)std::max<long long>(h->aux.H * h->aux.Fmin * (h->aux.Fmin - 1) / 2, 1) * AUX_J4);
  h->lo_wg = 0;
  h->lo_wgp = h->lo_wg + align64((size_t)(h->K1 / 2) * h->MT * 64);
  h->lo_bg = h->lo_wgp + align64((size_t)(h->K1 / 2) * h->MT * 64);
  h->lo_w2 = h->lo_bg + align64(2 * h->GHPAD);
  h->lo_split = h->lo_w2 + align64((size_t)h->NQ4 * h->M2T * 64 * 4);
  h->split_ok = h->R == 64 && h->S == 64 && h->G == 128 && h->KS == 3 && h->aux.nka <= 4;
  h->layer_kernel = h->split_ok ? 3 : 0;  // split16: 4 % faster than split (32x32x16) on the bench
  h->lo_split16 = h->lo_split + (h->split_ok ? align64(SPLIT_LAYER_DWORDS) : 0);
  h->layer_stride = h->lo_split16 + (h->split_ok ? align64(SPLIT_LAYER_DWORDS) : 0);
  h->off_layers = o; o += h->layer_stride * h->L;
  h->M3T = (h->S + 31) / 32;
  h->off_head_w1 = o; o += align64((size_t)(16 * h->M3T + 1 + 3) / 4 * h->M3T * 64 * 4);
  h->off_head_w2 = o; o += align64((size_t)h->O * h->M3T * 32);
  h->off_head_b2 = o; o += align64(h->O);
  h->off_skip0 = o; o += align64(64);
  h->off_skip0_16 = o; o += align64(64);
  h->off_head16_w1 = o; o += align64(4 * 4 * 64 * 4 + 64);
  h->off_head16_w2 = o; o += align64((size_t)h->O * 64);
  h->packed_total = o;

  long long rt = 0;
  rt += h->R + h->R;
  if (c.use_conv_in) rt += (long long)h->A * h->A * h->KW;
  for (int i = 0; i < c.num_scales; ++i) rt += 2 * c.upsample_scales[i] + 1;
  rt += (long long)h->L * ((long long)h->G * h->R * h->KS + h->G + (long long)h->G * h->A +
                           (long long)h->S * h->GH + h->S + (long long)h->R * h->GH + h->R);
  rt += (long long)h->S * h->S + h->S + (long long)h->O * h->S + h->O;
  h->ref_total = rt;
  *out = h;
  return PWG_OK;
}

void pwg_destroy(PwgHandle* h) {
  if (!h) return;
  {
    DeviceGuard g(h->device);
    for (auto& r : h->records) { (void)hipEventDestroy(r.start); (void)hipEventDestroy(r.stop); }
    for (auto e : h->event_pool) (void)hipEventDestroy(e);
    if (h->d_status) (void)hipFree(h->d_status);
    if (h->d_trace) (void)hipFree(h->d_trace);
    for (auto& kv : h->hstatus) (void)hipHostFree(kv.second);
  }
  delete h;
}

long long pwg_receptive_field_size(const PwgHandle* h) {
  long long s = 0;
  for (int d : h->dil) s += d;
  return (long long)(h->KS - 1) * s + 1;
}

long long pwg_upsample_factor(const PwgHandle* h) {
  long long f = 1;
  for (int i = 0; i < h->cfg.num_scales; ++i) f *= h->cfg.upsample_scales[i];
  return f;
}

long long pwg_ref_weight_count(const PwgHandle* h) { return h->ref_total; }
long long pwg_packed_weight_count(const PwgHandle* h) { return (long long)h->packed_total; }

int pwg_pack_weights(const PwgHandle* h, const float* ref, float* pk) {
  if (!h || !ref || !pk) return fail(PWG_ERR_INVALID, "null argument");
  std::memset(pk, 0, sizeof(float) * h->packed_total);
  g_split_overflow = 0;
  const PwgConfig& c = h->cfg;
  const int R = h->R, G = h->G, GH = h->GH, GHPAD = h->GHPAD, MT = h->MT, S = h->S, M2T = h->M2T;
  const int A = h->A, KS = h->KS, KW = h->KW, O = h->O;
  const float* p = ref;
  for (int i = 0; i < R; ++i) pk[h->off_first_w + i] = *p++;
  for (int i = 0; i < R; ++i) pk[h->off_first_b + i] = *p++;
  if (c.use_conv_in) {
    for (size_t i = 0; i < (size_t)A * A * KW; ++i) pk[h->off_conv_in + i] = p[i];
    // MFMA fragments: k-step s, lane l -> W[o = 32 m + (l & 31)][k = 2 s + (l >> 5)], k = i*KW + kk
    const int nks = (A * KW + 1) / 2, mti = (A + 31) / 32;
    for (int s2 = 0; s2 < nks; ++s2)
      for (int m = 0; m < mti; ++m)
        for (int l = 0; l < 64; ++l) {
          const int o2 = 32 * m + (l & 31), k = 2 * s2 + (l >> 5);
          pk[h->off_conv_in_frag + ((size_t)s2 * mti + m) * 64 + l] =
              (o2 < A && k < A * KW) ? p[(size_t)o2 * A * KW + k] : 0.f;
        }
    p += (size_t)A * A * KW;
  } else {
    pk[h->off_conv_in] = 1.f;  // unused (identity path)
  }
  {
    std::vector<std::vector<double>> taps(c.num_scales);
    for (int i = 0; i < c.num_scales; ++i)
      for (int k = 0; k < 2 * c.upsample_scales[i] + 1; ++k) taps[i].push_back((double)*p++);
    std::vector<float> ti, tl, tr, ts;
    const int rc = aux_tables(c, h->aux, taps, ti, tl, tr, ts);
    if (rc != PWG_OK) return rc;
    std::copy(ti.begin(), ti.end(), pk + h->off_tab_interior);
    std::copy(tl.begin(), tl.end(), pk + h->off_tab_left);
    std::copy(tr.begin(), tr.end(), pk + h->off_tab_right);
    std::copy(ts.begin(), ts.end(), pk + h->off_tab_small);
  }
  for (int l = 0; l < h->L; ++l) {
    const float* wd = p; p += (size_t)G * R * KS;   // conv.weight [G][R][KS]
    const float* bd = p; p += G;                      // conv.bias
    const float* wa = p; p += (size_t)G * A;          // conv1x1_aux.weight [G][A]
    const float* ws = p; p += (size_t)S * GH;         // conv1x1_skip.weight [S][GH]
    const float* bs = p; p += S;
    const float* wo = p; p += (size_t)R * GH;         // conv1x1_out.weight [R][GH]
    const float* bo = p; p += R;
    float* L0 = pk + h->off_layers + h->layer_stride * l;
    // packed gate row -> reference gate row (or -1 for zero padding rows)
    auto gate_row = [&](int prow) -> int {
      if (prow < GHPAD) return prow < GH ? prow : -1;
      const int q = prow - GHPAD;
      return q < GH ? GH + q : -1;
    };
    const int RS = h->RS;
    auto wcat = [&](int grow, int k) -> float {
      if (grow < 0) return 0.f;
      const int tap = k / RS, ch = k % RS;
      return ch < R ? wd[((size_t)grow * R + ch) * KS + tap] : 0.f;
    };
    float* wg = L0 + h->lo_wg;
    for (int s = 0; s < h->K1 / 2; ++s)
      for (int m = 0; m < MT; ++m)
        for (int lane = 0; lane < 64; ++lane)
          wg[((size_t)s * MT + m) * 64 + lane] = wcat(gate_row(32 * m + (lane & 31)), 2 * s + (lane >> 5));
    // persistent-kernel grouping: group g = 2*GK channels c0.. of one tap (GK = 16 when RS % 32 == 0,
    // else 8); k-step i of the group pairs channels c0+i (lane half 0) and c0+GK+i (lane half 1).
    // Stored in 4-k-step slices: [g][i/4][m][lane][i%4].
    float* wgp = L0 + h->lo_wgp;
    {
      const int GK = RS % 32 == 0 ? 16 : 8;
      const int NB = GK / 4;
      for (int g = 0; g < h->K1 / (2 * GK); ++g) {
        const int tap = (2 * GK * g) / RS, c0 = (2 * GK * g) % RS;
        for (int i = 0; i < GK; ++i)
          for (int m = 0; m < MT; ++m)
            for (int lane = 0; lane < 64; ++lane) {
              const int grow = gate_row(32 * m + (lane & 31));
              const int ch = c0 + i + GK * (lane >> 5);
              wgp[((((size_t)g * NB + i / 4) * MT + m) * 64 + lane) * 4 + (i % 4)] =
                  (grow < 0 || ch >= R) ? 0.f : wd[((size_t)grow * R + ch) * KS + tap];
            }
      }
    }
    float* bg = L0 + h->lo_bg;
    for (int prow = 0; prow < 2 * GHPAD; ++prow) {
      const int gr = gate_row(prow);
      bg[prow] = gr < 0 ? 0.f : bd[gr];
    }
    // aux projection A-fragments: (k-step s, m-tile m, lane) -> Waux[gate_row(32m + lane%32)][2s + lane/32]
    const int nks = (A + 1) / 2;
    float* waux = pk + h->off_waux + (size_t)l * nks * MT * 64;
    for (int s = 0; s < nks; ++s)
      for (int m = 0; m < MT; ++m)
        for (int lane = 0; lane < 64; ++lane) {
          const int gr = gate_row(32 * m + (lane & 31));
          const int i = 2 * s + (lane >> 5);
          waux[((size_t)s * MT + m) * 64 + lane] = (gr < 0 || i >= A) ? 0.f : wa[(size_t)gr * A + i];
        }
    // GEMM 2 A fragments, 4 k-steps per 16-byte lane load: [q/4][m2][lane][q%4]; k-step NQ is
    // the bias (A[i][0] = b2[row i], B = ones row).
    float* w2 = L0 + h->lo_w2;
    for (int q = 0; q < 4 * h->NQ4; ++q)
      for (int m2 = 0; m2 < M2T; ++m2)
        for (int lane = 0; lane < 64; ++lane) {
          const int row2 = 32 * m2 + (lane & 31);
          float v = 0.f;
          if (q < h->NQ) {
            const int r = q & 15, gm = q >> 4;
            const int ch = 32 * gm + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            if (ch < GH) {
              if (row2 < S) v = ws[(size_t)row2 * GH + ch];
              else if (row2 < S + R) v = wo[(size_t)(row2 - S) * GH + ch];
            }
          } else if (q == h->NQ && lane < 32) {
            v = row2 < S ? bs[row2] : (row2 < S + R ? bo[row2 - S] : 0.f);
          }
          w2[(((size_t)(q / 4) * M2T + m2) * 64 + lane) * 4 + (q % 4)] = v;
        }
    if (h->split_ok) {
      // split-f16 image (pwg_split.hip SplitSmem): gate A fragments [tap][s][m][hi/lo][lane][4]
      // (row gate_row(32m + lane%32), k = 8hh + j <-> x channel split_chan(s, hh, j)), GEMM-2 A
      // fragments [s][m][hi/lo][lane][4] (rows: skip 0..63, then out 0..63 pre-scaled by sqrt(.5);
      // k <-> gate channel split_chan(s, hh, j)), gate-bias pairs [lane 32][m 4], sqrt(.5) b_out
      // [hh][slot].
      uint32_t* sp = reinterpret_cast<uint32_t*>(L0 + h->lo_split);
      const double rh = std::sqrt(0.5);
      for (int tap = 0; tap < 3; ++tap)
        for (int s4 = 0; s4 < 4; ++s4)
          for (int m = 0; m < 4; ++m)
            for (int lane = 0; lane < 64; ++lane)
              for (int j = 0; j < 8; j += 2) {
                const int grow = gate_row(32 * m + (lane & 31));
                const double gsc = m < 2 ? SPLIT_GATE_SCALE_TANH : SPLIT_GATE_SCALE_SIGM;
                uint32_t hv = 0, lv = 0;
                for (int e = 0; e < 2; ++e) {
                  const int ch = split_chan(s4, lane >> 5, j + e);
                  const uint32_t pr =
                      grow < 0 ? 0u : split_pair((float)(gsc * wd[((size_t)grow * R + ch) * KS + tap]));
                  hv |= (pr & 0xffffu) << (16 * e);
                  lv |= (pr >> 16) << (16 * e);
                }
                const size_t base = ((((size_t)tap * 4 + s4) * 4 + m) * 2) * 256 + (size_t)lane * 4 + j / 2;
                sp[base] = hv;
                sp[base + 256] = lv;
              }
      uint32_t* s2 = sp + 3 * 4 * 4 * 2 * 256;
      for (int s4 = 0; s4 < 4; ++s4)
        for (int m = 0; m < 4; ++m)
          for (int lane = 0; lane < 64; ++lane)
            for (int j = 0; j < 8; j += 2) {
              const int row = 32 * (m & 1) + (lane & 31);
              uint32_t hv = 0, lv = 0;
              for (int e = 0; e < 2; ++e) {
                const int ch = split_chan(s4, lane >> 5, j + e);
                const float v = m < 2 ? ws[(size_t)row * GH + ch] : (float)(rh * wo[(size_t)row * GH + ch]);
                const uint32_t pr = split_pair(v);
                hv |= (pr & 0xffffu) << (16 * e);
                lv |= (pr >> 16) << (16 * e);
              }
              const size_t base = (((size_t)s4 * 4 + m) * 2) * 256 + (size_t)lane * 4 + j / 2;
              s2[base] = hv;
              s2[base + 256] = lv;
            }
      uint32_t* sbg = s2 + 4 * 4 * 2 * 256;
      for (int cl = 0; cl < 32; ++cl)
        for (int m = 0; m < 4; ++m) {
          const int gr = gate_row(32 * m + cl);
          const double gsc = m < 2 ? SPLIT_GATE_SCALE_TANH : SPLIT_GATE_SCALE_SIGM;
          sbg[cl * 4 + m] = gr < 0 ? 0u : split_pair((float)(gsc * bd[gr]));
        }
      float* sbo = reinterpret_cast<float*>(sbg + 128);
      for (int hh = 0; hh < 2; ++hh)
        for (int p2 = 0; p2 < 32; ++p2) sbo[hh * 32 + p2] = (float)(rh * bo[split_chan(p2 >> 3, hh, p2 & 7)]);
      float* s0 = pk + h->off_skip0;
      for (int hh = 0; hh < 2; ++hh)
        for (int p2 = 0; p2 < 32; ++p2) s0[hh * 32 + p2] += bs[split_chan(p2 >> 3, hh, p2 & 7)];

      // 16x16x32 image (pwg_split16.hip Split16Smem): lane = (c, g), k = 8g + j <->
      // chan16(ks, g, j) = 16(2ks + (j >> 2)) + 4g + (j & 3)
      auto chan16 = [](int ks, int g, int j) { return 16 * (2 * ks + (j >> 2)) + 4 * g + (j & 3); };
      uint32_t* q = reinterpret_cast<uint32_t*>(L0 + h->lo_split16);
      for (int tap = 0; tap < 3; ++tap)
        for (int ks = 0; ks < 2; ++ks)
          for (int m = 0; m < 8; ++m)
            for (int lane = 0; lane < 64; ++lane)
              for (int j = 0; j < 8; j += 2) {
                const int grow = gate_row(16 * m + (lane & 15));
                const double gsc = m < 4 ? SPLIT_GATE_SCALE_TANH : SPLIT_GATE_SCALE_SIGM;
                uint32_t hv = 0, lv = 0;
                for (int e = 0; e < 2; ++e) {
                  const int ch = chan16(ks, lane >> 4, j + e);
                  const uint32_t pr =
                      grow < 0 ? 0u : split_pair((float)(gsc * wd[((size_t)grow * R + ch) * KS + tap]));
                  hv |= (pr & 0xffffu) << (16 * e);
                  lv |= (pr >> 16) << (16 * e);
                }
                const size_t base = ((((size_t)tap * 2 + ks) * 8 + m) * 2) * 256 + (size_t)lane * 4 + j / 2;
                q[base] = hv;
                q[base + 256] = lv;
              }
      uint32_t* q2 = q + 3 * 2 * 8 * 2 * 256;
      for (int ks = 0; ks < 2; ++ks)
        for (int m = 0; m < 8; ++m)
          for (int lane = 0; lane < 64; ++lane)
            for (int j = 0; j < 8; j += 2) {
              const int row = 16 * (m & 3) + (lane & 15);
              uint32_t hv = 0, lv = 0;
              for (int e = 0; e < 2; ++e) {
                const int ch = chan16(ks, lane >> 4, j + e);
                const float v = m < 4 ? ws[(size_t)row * GH + ch] : (float)(rh * wo[(size_t)row * GH + ch]);
                const uint32_t pr = split_pair(v);
                hv |= (pr & 0xffffu) << (16 * e);
                lv |= (pr >> 16) << (16 * e);
              }
              const size_t base = (((size_t)ks * 8 + m) * 2) * 256 + (size_t)lane * 4 + j / 2;
              q2[base] = hv;
              q2[base + 256] = lv;
            }
      uint32_t* qbg = q2 + 2 * 8 * 2 * 256;
      for (int m = 0; m < 8; ++m)
        for (int c = 0; c < 16; ++c) {
          const int gr = gate_row(16 * m + c);
          const double gsc = m < 4 ? SPLIT_GATE_SCALE_TANH : SPLIT_GATE_SCALE_SIGM;
          qbg[m * 16 + c] = gr < 0 ? 0u : split_pair((float)(gsc * bd[gr]));
        }
      float* qbo = reinterpret_cast<float*>(qbg + 128);
      for (int g = 0; g < 4; ++g)
        for (int ks = 0; ks < 2; ++ks)
          for (int j = 0; j < 8; ++j) qbo[16 * g + 8 * ks + j] = (float)(rh * bo[chan16(ks, g, j)]);
      float* s16 = pk + h->off_skip0_16;
      for (int g = 0; g < 4; ++g)
        for (int ms = 0; ms < 4; ++ms)
          for (int i = 0; i < 4; ++i) s16[16 * g + 4 * ms + i] += bs[16 * ms + 4 * g + i];
    }
  }
  // output head (fused into the last layer): W1h A-fragments over skip channels in the same
  // permuted-k order as GEMM 2, bias as k-step NQH; W2h per lane half in accumulator row order.
  {
    const float* w1 = p; p += (size_t)S * S;
    const float* b1 = p; p += S;
    const float* w2h = p; p += (size_t)O * S;
    const float* b2h = p; p += O;
    const int M3T = h->M3T, NQH = 16 * M3T, NQH4 = (NQH + 1 + 3) / 4;
    float* hw1 = pk + h->off_head_w1;
    for (int q = 0; q < 4 * NQH4; ++q)
      for (int m3 = 0; m3 < M3T; ++m3)
        for (int lane = 0; lane < 64; ++lane) {
          const int row = 32 * m3 + (lane & 31);
          float v = 0.f;
          if (row < S) {
            if (q < NQH) {
              const int r = q & 15, gm = q >> 4;
              const int ch = 32 * gm + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
              if (ch < S) v = w1[(size_t)row * S + ch];
            } else if (q == NQH && lane < 32) {
              v = b1[row];
            }
          }
          hw1[(((size_t)(q / 4) * M3T + m3) * 64 + lane) * 4 + (q % 4)] = v;
        }
    float* hw2 = pk + h->off_head_w2;
    for (int oc = 0; oc < O; ++oc)
      for (int m3 = 0; m3 < M3T; ++m3)
        for (int half = 0; half < 2; ++half)
          for (int r = 0; r < 16; ++r) {
            const int row = 32 * m3 + (r & 3) + 8 * (r >> 2) + 4 * half;
            hw2[(((size_t)oc * M3T + m3) * 2 + half) * 16 + r] = row < S ? w2h[(size_t)oc * S + row] : 0.f;
          }
    for (int i = 0; i < O; ++i) pk[h->off_head_b2 + i] = b2h[i];
    if (h->split_ok) {
      // split-f16 head of the split16 kernel (v_mfma_f32_16x16x32_f16, 3 products): W1h pairs
      // [ks 2][m3 4][hi/lo 2][lane (c, g) 64][4 dwords], lane's k = 8g + j <-> skip row
      // chan16(ks, g, j) (its accumulator rows), A row 16m3 + c; then b1 [g][4m3 + i] =
      // b1[16m3 + 4g + i]; W2h [oc][g][4m3 + i] = W2h[oc][16m3 + 4g + i]
      float* w16 = pk + h->off_head16_w1;
      uint32_t* w16u = reinterpret_cast<uint32_t*>(w16);
      auto hchan = [](int ks, int g, int j) { return 16 * (2 * ks + (j >> 2)) + 4 * g + (j & 3); };
      for (int ks = 0; ks < 2; ++ks)
        for (int m3 = 0; m3 < 4; ++m3)
          for (int lane = 0; lane < 64; ++lane)
            for (int j = 0; j < 8; j += 2) {
              uint32_t hv = 0, lv = 0;
              for (int e = 0; e < 2; ++e) {
                const uint32_t pr = split_pair(w1[(size_t)(16 * m3 + (lane & 15)) * S + hchan(ks, lane >> 4, j + e)]);
                hv |= (pr & 0xffffu) << (16 * e);
                lv |= (pr >> 16) << (16 * e);
              }
              const size_t base = (((size_t)ks * 4 + m3) * 2) * 256 + (size_t)lane * 4 + j / 2;
              w16u[base] = hv;
              w16u[base + 256] = lv;
            }
      for (int g = 0; g < 4; ++g)
        for (int m3 = 0; m3 < 4; ++m3)
          for (int i = 0; i < 4; ++i) w16[4096 + 16 * g + 4 * m3 + i] = b1[16 * m3 + 4 * g + i];
      float* v16 = pk + h->off_head16_w2;
      for (int oc = 0; oc < O; ++oc)
        for (int g = 0; g < 4; ++g)
          for (int m3 = 0; m3 < 4; ++m3)
            for (int i = 0; i < 4; ++i) v16[(size_t)oc * 64 + 16 * g + 4 * m3 + i] = w2h[(size_t)oc * S + 16 * m3 + 4 * g + i];
    }
  }
  if ((long long)(p - ref) != h->ref_total) return fail(PWG_ERR_INVALID, "internal: weight count mismatch");
  if (g_split_overflow > 0)
    return fail(PWG_ERR_RANGE, std::to_string(g_split_overflow) +
                                   " weights exceed the fp16 pair range of the split-f16 layer kernels; the "
                                   "image is complete for PWG_OPT_LAYER_KERNEL 0/1 (exact fp32) only");
  return PWG_OK;
}

int pwg_plan_create(PwgHandle* h, int n_utts, const long long* frames, int layout, PwgPlan** out) {
  if (!h || !out || (n_utts > 0 && !frames)) return fail(PWG_ERR_INVALID, "null argument");
  if (n_utts < 1) return fail(PWG_ERR_INVALID, "n_utts must be >= 1");
  if (layout != PWG_LAYOUT_INFERENCE && layout != PWG_LAYOUT_FORWARD)
    return fail(PWG_ERR_INVALID, "unknown input layout");
  if (!h->cfg.use_conv_in && h->cfg.aux_context_window != 0)
    return fail(PWG_ERR_ASSERT, "c.size(-1) == z.size(-1): UpsampleNetwork needs aux_context_window == 0");
  const long long H = pwg_upsample_factor(h);
  const int w = h->cfg.aux_context_window;
  PwgPlan* p = new PwgPlan();
  p->h = h;
  p->layout = layout;
  p->n_utts = n_utts;
  // time axis: [gap][utt 0 padded to TILE][gap][utt 1]...[gap]
  long long seg = h->gap, fb = 0, io = 0, mel = 0, tiles = 0;
  std::vector<long long> gap_col0;
  for (long long c0 = 0; c0 < h->gap; c0 += TILE) gap_col0.push_back(c0);
  for (int u = 0; u < n_utts; ++u) {
    const long long f = frames[u];
    if (f < 1) { delete p; return fail(PWG_ERR_INVALID, "every utterance needs >= 1 mel frame"); }
    if (layout == PWG_LAYOUT_FORWARD && f != frames[0]) {
      delete p;
      return fail(PWG_ERR_INVALID, "forward layout needs equal-length batch items");
    }
    UttDesc d;
    d.seg_base = seg;
    d.first_tile = tiles;
    d.T = f * H;
    d.frame_base = fb;
    d.frames = f;
    d.mel_off = mel;
    d.io_off = io;
    p->utts.push_back(d);
    const long long padded = (d.T + TILE - 1) / TILE * TILE;
    tiles += padded / TILE;
    seg += padded;
    for (long long c0 = 0; c0 < h->gap; c0 += TILE) gap_col0.push_back(seg + c0);
    seg += h->gap;
    fb += f;
    io += d.T;
    mel += layout == PWG_LAYOUT_INFERENCE ? f * h->A : (f + 2 * w) * h->A;
  }
  p->Tpad = seg;
  p->F_total = fb;
  p->T_total = io;
  p->n_tiles = tiles;
  p->n_gap_tiles = (long long)gap_col0.size();
  if (p->Tpad + h->gap >= (1LL << 31) || p->F_total >= (1LL << 31) || p->T_total * h->O >= (1LL << 31)) {
    delete p;
    return fail(PWG_ERR_UNSUPPORTED, "batch too large for one plan (2^31 samples); split it");
  }
  for (const UttDesc& d : p->utts)
    p->max_blocks_per_utt = std::max(p->max_blocks_per_utt, (d.T + TILE - 1) / TILE * (TILE / 32));
  if ((long long)gap_col0.size() != (long long)(n_utts + 1) * (h->gap / TILE)) {
    delete p;
    return fail(PWG_ERR_INVALID, "internal: gap tile count");
  }
  size_t o = 0;
  p->ws_x0 = o; o += align_bytes(sizeof(float) * h->RS * p->Tpad);
  p->ws_x1 = o; o += align_bytes(sizeof(float) * h->RS * p->Tpad);
  p->ws_skip = o; o += align_bytes(sizeof(float) * h->SS * p->Tpad);
  p->ws_c1 = o; o += align_bytes(sizeof(float) * h->A * p->F_total);
  p->ws_d = o; o += align_bytes(sizeof(float) * h->L * h->GR * p->F_total);
  p->ws_ctr = o; o += align_bytes(sizeof(int) * h->L * SCHED_CTR_STRIDE * 8);
  p->ws_flag = o; o += align_bytes(sizeof(int));  // split-f16 range flag (pwg_run_status)
  p->ws_utts = o; o += align_bytes(sizeof(UttDesc) * n_utts);
  p->ws_tile_utt = o; o += align_bytes(sizeof(int) * p->n_tiles);
  p->ws_gap = o; o += align_bytes(sizeof(long long) * std::max<long long>(p->n_gap_tiles, 1));
  p->ws_blocks = o; o += align_bytes(sizeof(BlockDesc) * p->n_tiles * (TILE / 32));
  // the layer pipeline addresses a plane with 32-bit buffer offsets (< 2 GB) and polls the blocks
  // its dependencies span with one wave (<= 64); its extra plane is only allocated when it can run
  const int tc = h->cfg.use_causal_conv ? h->KS - 1 : (h->KS - 1) / 2;
  auto reach = [](long long taps, int d) { return (int)((taps * d + 31) / 32); };
  bool lanes_ok = h->KS == 3;
  for (int l = 0; l < h->L && lanes_ok; ++l) {
    const int rl1 = reach(tc, h->dil[l]), rr1 = reach(h->KS - 1 - tc, h->dil[l]);
    const int rl2 = l >= 2 ? reach(tc, h->dil[l - 2]) : 0, rr2 = l >= 2 ? reach(h->KS - 1 - tc, h->dil[l - 2]) : 0;
    lanes_ok = std::max(rl1, rr2) + std::max(rr1, rl2) + 1 <= 64;
  }
  p->pipe_ok = h->split_ok && h->L >= 2 && h->L <= PIPE_MAX_LAYERS && lanes_ok &&
               (long long)h->RS * 4 * (p->Tpad + h->gap) < (1LL << 31) && p->Tpad <= h->pipe_max;
  if (p->pipe_ok) {
    p->ws_x2 = o; o += align_bytes(sizeof(float) * h->RS * p->Tpad);
    p->ws_prog = o; o += align_bytes(sizeof(int) * p->n_tiles * (TILE / 32));
  }
  p->ws_total = o;
  *out = p;
  return PWG_OK;
}

void pwg_plan_destroy(PwgPlan* p) { delete p; }

long long pwg_plan_total_samples(const PwgPlan* p) { return p->T_total; }
long long pwg_plan_padded_samples(const PwgPlan* p) { return p->Tpad; }
long long pwg_plan_workspace_bytes(const PwgPlan* p) { return (long long)p->ws_total; }

static hipEvent_t pool_get(PwgHandle* h) {
  if (!h->event_pool.empty()) {
    hipEvent_t e = h->event_pool.back();
    h->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

static int pwg_run_impl(PwgPlan* p, const float* packed, const float* mel, const float* noise, const float* mean,
                        const float* scale, float* out, void* workspace, void* stream);

int pwg_run(PwgPlan* p, const float* packed, const float* mel, const float* noise, const float* mean,
            const float* scale, float* out, void* workspace, void* stream) {
  // timing mode 2: one event pair around the whole run (its device span, pwg_timing_span)
  if (!p || p->h->timing != 2) return pwg_run_impl(p, packed, mel, noise, mean, scale, out, workspace, stream);
  PwgHandle* h = p->h;
  DeviceGuard g(h->device);
  hipStream_t s = (hipStream_t)stream;
  hipEvent_t a = pool_get(h), b = pool_get(h);
  auto give_back = [&] {  // (a failed record returns both events to the pool instead of leaking them)
    if (a) h->event_pool.push_back(a);
    if (b) h->event_pool.push_back(b);
  };
  if (!a || !b || hipEventRecord(a, s) != hipSuccess) {
    give_back();
    return fail(PWG_ERR_HIP, "timing event");
  }
  const int rc = pwg_run_impl(p, packed, mel, noise, mean, scale, out, workspace, stream);
  if (hipEventRecord(b, s) != hipSuccess) {
    give_back();
    return fail(PWG_ERR_HIP, "timing event");
  }
  h->records.push_back({-1, a, b});
  return rc;
}

static int pwg_run_impl(PwgPlan* p, const float* packed, const float* mel, const float* noise, const float* mean,
                        const float* scale, float* out, void* workspace, void* stream) {
  if (!p || !packed || !mel || !noise || !out || !workspace) return fail(PWG_ERR_INVALID, "null argument");
  if (((uintptr_t)workspace & 255) != 0) return fail(PWG_ERR_INVALID, "workspace must be 256-byte aligned");
  if ((mean == nullptr) != (scale == nullptr)) return fail(PWG_ERR_INVALID, "mean and scale go together");
  if (mean != nullptr && p->layout != PWG_LAYOUT_INFERENCE)
    return fail(PWG_ERR_INVALID, "normalize_before is an inference() option");
  PwgHandle* h = p->h;
  DeviceGuard g(h->device);
  if (!g.ok) return fail(PWG_ERR_HIP, "hipSetDevice failed");
  if (h->n_cu == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || n < 1)
      return fail(PWG_ERR_HIP, "cannot query the CU count");
    h->n_cu = n;
  }
  if (h->d_status == nullptr) {  // once per handle (pwg_graph_create runs eagerly before capturing)
    if (hipMalloc((void**)&h->d_status, 256) != hipSuccess) return fail(PWG_ERR_HIP, "status word allocation");
    if (hipMemset(h->d_status, 0, 256) != hipSuccess) return fail(PWG_ERR_HIP, "status word reset");
  }
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  float* x0 = (float*)(ws + p->ws_x0);
  float* x1 = (float*)(ws + p->ws_x1);
  float* skip = (float*)(ws + p->ws_skip);
  float* c1 = (float*)(ws + p->ws_c1);
  float* dproj = (float*)(ws + p->ws_d);
  int* sched_ctr = (int*)(ws + p->ws_ctr);

  auto timed = [&](int bucket, auto&& launch) -> hipError_t {
    if (h->timing != 1) return launch();
    hipEvent_t a = pool_get(h), b = pool_get(h);
    auto give_back = [&] {
      if (a) h->event_pool.push_back(a);
      if (b) h->event_pool.push_back(b);
    };
    if (!a || !b) {
      give_back();
      return hipErrorOutOfMemory;
    }
    hipError_t e = hipEventRecord(a, s);
    if (e != hipSuccess) {
      give_back();
      return e;
    }
    e = launch();
    if (e == hipSuccess) e = hipEventRecord(b, s);
    if (e != hipSuccess) {
      give_back();
      return e;
    }
    h->records.push_back({bucket, a, b});
    return e;
  };

  int* range_flag = (int*)(ws + p->ws_flag);
  hipError_t e = hipSuccess;
  // all residual layers in ONE layer-pipelined launch (split16, small plans); the
  // grid needs one workgroup per CU for every layer and a multiple of 8 workgroups
  const int pipe_wg = h->n_cu / 8 * 8;
  const bool use_pipe = p->pipe_ok && h->layer_kernel == 3 && p->Tpad <= h->pipe_max && pipe_wg >= h->L;
  const bool split = h->layer_kernel == 2 || h->layer_kernel == 3;
  const bool split16 = h->layer_kernel == 3;
  const bool fuse_first = split16 && h->fuse_first && h->L > 1;
  UttDesc* d_utts = (UttDesc*)(ws + p->ws_utts);
  int* d_tile_utt = (int*)(ws + p->ws_tile_utt);
  long long* d_gap_col0 = (long long*)(ws + p->ws_gap);
  BlockDesc* d_blocks = (BlockDesc*)(ws + p->ws_blocks);
  for (int u0 = 0; u0 < p->n_utts; u0 += PLAN_CHUNK) {
    PlanDescArgs da;
    da.n = std::min(PLAN_CHUNK, p->n_utts - u0);
    da.u0 = u0;
    da.gap_tiles = (int)(h->gap / TILE);
    for (int i = 0; i < da.n; ++i) da.utts[i] = p->utts[u0 + i];
    da.d_utts = d_utts; da.tile_utt = d_tile_utt; da.gap_col0 = d_gap_col0; da.blocks = d_blocks;
    // work-queue heads and the range flag (adjacent) start at zero every run
    da.zero = u0 == 0 ? sched_ctr : nullptr;
    da.n_zero = (int)((p->ws_flag + sizeof(int) - p->ws_ctr) / sizeof(int));
    da.prog = use_pipe ? (int*)(ws + p->ws_prog) : nullptr;
    // split16 with the fused first_conv: the gap tiles are zeroed here, not by a first_conv launch
    da.zx[0] = fuse_first ? reinterpret_cast<unsigned*>(x0) : nullptr;
    da.zx[1] = fuse_first ? reinterpret_cast<unsigned*>(x1) : nullptr;
    da.zx[2] = fuse_first && use_pipe ? reinterpret_cast<unsigned*>(ws + p->ws_x2) : nullptr;
    e = launch_plan_desc(da, p->max_blocks_per_utt, s);
    if (e != hipSuccess) return hip_fail(e, "plan descriptor launch");
  }
  ConvInArgs ca;
  ca.mel = mel; ca.mean = mean; ca.scale = scale; ca.w = packed + h->off_conv_in; ca.c1 = c1;
  ca.wfrag = packed + h->off_conv_in_frag;
  ca.utts = d_utts; ca.n_utts = p->n_utts; ca.F_total = p->F_total; ca.A = h->A; ca.KW = h->KW;
  ca.ctx = h->cfg.aux_context_window; ca.layout = p->layout; ca.use_conv_in = h->cfg.use_conv_in;
  e = timed(PWG_KERNEL_CONV_IN, [&] { return launch_conv_in(ca, s); });
  if (e != hipSuccess) return hip_fail(e, "conv_in launch");

  AuxProjArgs pa;
  pa.c1 = c1; pa.waux = packed + h->off_waux; pa.d = dproj; pa.F_total = p->F_total; pa.A = h->A; pa.GR = h->GR;
  pa.split = split16 ? 2 : split ? 1 : 0;
  pa.split_scale_a = (float)SPLIT_GATE_SCALE_TANH;
  pa.split_scale_b = (float)SPLIT_GATE_SCALE_SIGM;
  pa.range_flag = split ? range_flag : nullptr;
  pa.sticky = split ? h->d_status : nullptr;
  e = timed(PWG_KERNEL_UPSAMPLE, [&] { return launch_aux_proj(pa, h->L, s); });
  if (e != hipSuccess) return hip_fail(e, "aux projection launch");

  FirstConvArgs fa;
  fa.noise = noise; fa.w = packed + h->off_first_w; fa.b = packed + h->off_first_b; fa.x = x0; fa.x1 = x1;
  fa.tile_utt = d_tile_utt; fa.utts = d_utts; fa.gap_col0 = d_gap_col0; fa.n_work = p->n_tiles;
  fa.Tpad = p->Tpad; fa.R = h->R; fa.RS = h->RS;
  fa.x2 = use_pipe ? (float*)(ws + p->ws_x2) : nullptr;
  // split16 with the fused first_conv: layer 0 builds x0 itself; only the gap tiles of both
  // residual buffers are zeroed here (the work-tile branch is skipped: n_work = 0)
  if (fuse_first) fa.n_work = 0;
  e = timed(PWG_KERNEL_FIRST_CONV, [&] {
    if (fuse_first) return hipSuccess;  // gap tiles zeroed by the plan-descriptor kernel
    return split16 ? launch_first_conv_split16(fa, p->n_tiles + p->n_gap_tiles, s)
           : split ? launch_first_conv_split(fa, p->n_tiles + p->n_gap_tiles, s)
                   : launch_first_conv(fa, p->n_tiles + p->n_gap_tiles, s);
  });
  if (e != hipSuccess) return hip_fail(e, "first_conv launch");

  if (use_pipe) {
    PipeArgs pp;
    SplitArgs& sa = pp.base;
    sa.x_in = nullptr; sa.x_out = nullptr;
    sa.skip = skip; sa.skip0 = packed + h->off_skip0_16;
    sa.d = nullptr;
    sa.tab = packed + h->off_tab_interior;
    sa.tab_left = (int)(h->off_tab_left - h->off_tab_interior);
    sa.tab_right = (int)(h->off_tab_right - h->off_tab_interior);
    sa.tab_small = (int)(h->off_tab_small - h->off_tab_interior);
    sa.blocks = d_blocks;
    sa.wg = nullptr;
    sa.hw1 = packed + h->off_head16_w1; sa.hw2 = packed + h->off_head16_w2; sa.hb2 = packed + h->off_head_b2;
    sa.out = out;
    sa.H = (int)h->aux.H; sa.J1 = h->aux.J1; sa.TL = h->aux.TL; sa.TR = h->aux.TR; sa.Fmin = h->aux.Fmin;
    sa.n_blocks = (int)(p->n_tiles * (TILE / 32)); sa.dil = 1; sa.first = 0; sa.O = h->O;
    if (p->layout == PWG_LAYOUT_INFERENCE) { sa.out_stride_t = h->O; sa.out_stride_o = 1; }
    else { sa.out_stride_t = 1; sa.out_stride_o = (int)p->utts[0].T; }
    sa.skip_scale = (float)std::sqrt(1.0 / h->L);
    sa.ctr = nullptr; sa.trace = nullptr; sa.compute_waves = 8;
    sa.noise = fuse_first ? noise : nullptr;
    sa.fw = packed + h->off_first_w; sa.fb = packed + h->off_first_b;
    sa.range_flag = range_flag;
    sa.sticky = h->d_status;
    pp.wg0 = reinterpret_cast<const unsigned*>(packed + h->off_layers + h->lo_split16);
    pp.wg_stride = (long long)h->layer_stride;
    pp.d0 = reinterpret_cast<const unsigned*>(dproj);
    pp.d_stride = p->F_total * h->GR;
    pp.x[0] = reinterpret_cast<unsigned*>(x0);
    pp.x[1] = reinterpret_cast<unsigned*>(x1);
    pp.x[2] = reinterpret_cast<unsigned*>(ws + p->ws_x2);
    pp.prog = (int*)(ws + p->ws_prog);
    pp.ctr = sched_ctr;
    pp.L = h->L;
    for (int l = 0; l < PIPE_MAX_LAYERS; ++l) pp.dil[l] = l < h->L ? h->dil[l] : 1;
    const int tc = h->cfg.use_causal_conv ? h->KS - 1 : (h->KS - 1) / 2;
    e = timed(PWG_KERNEL_RESIDUAL_LAYER, [&] { return launch_pipe_split16(pp, tc, pipe_wg, s); });
    if (e != hipSuccess) return hip_fail(e, "layer-pipelined forward launch");
    return PWG_OK;
  }
  // the residual layers but the last in ONE grid-synchronised launch (split16, PWG_OPT_SYNC: the
  // B = 1 decode path)
  const long long n_blocks_all = p->n_tiles * (TILE / 32);
  const long long half_max_all = h->half_max >= 0 ? h->half_max : 4LL * h->n_cu;
  // (the grid deals its units to 8 XCD eighths: it needs at least 8 workgroups, one per CU)
  const bool use_sync = split16 && h->split_ok && h->n_cu >= 8 && h->L >= 2 && h->L <= PIPE_MAX_LAYERS && h->KS == 3 &&
                        n_blocks_all <= (h->sync_max >= 0 ? h->sync_max : 64LL * h->n_cu) &&
                        (long long)h->RS * 4 * (p->Tpad + h->gap) < (1LL << 31);
  // the layers it covers: 0 .. L - 2 (from 1 on whole-block plans with the fused first_conv)
  SyncArgs sy;
  int sync_begin = h->L, sync_end = h->L;
  if (use_sync) {
    SplitArgs& sa = sy.base;
    sa.x_in = nullptr; sa.x_out = nullptr;
    sa.skip = skip; sa.skip0 = packed + h->off_skip0_16;
    sa.d = nullptr;
    sa.tab = packed + h->off_tab_interior;
    sa.tab_left = (int)(h->off_tab_left - h->off_tab_interior);
    sa.tab_right = (int)(h->off_tab_right - h->off_tab_interior);
    sa.tab_small = (int)(h->off_tab_small - h->off_tab_interior);
    sa.blocks = d_blocks;
    sa.wg = nullptr;
    sa.hw1 = packed + h->off_head16_w1; sa.hw2 = packed + h->off_head16_w2; sa.hb2 = packed + h->off_head_b2;
    sa.out = out;
    sa.H = (int)h->aux.H; sa.J1 = h->aux.J1; sa.TL = h->aux.TL; sa.TR = h->aux.TR; sa.Fmin = h->aux.Fmin;
    sa.n_blocks = (int)n_blocks_all; sa.dil = 1; sa.first = 0; sa.O = h->O;
    if (p->layout == PWG_LAYOUT_INFERENCE) { sa.out_stride_t = h->O; sa.out_stride_o = 1; }
    else { sa.out_stride_t = 1; sa.out_stride_o = (int)p->utts[0].T; }
    sa.skip_scale = (float)std::sqrt(1.0 / h->L);
    sa.ctr = nullptr; sa.trace = nullptr; sa.compute_waves = 8;
    sa.noise = fuse_first ? noise : nullptr;
    sa.fw = packed + h->off_first_w; sa.fb = packed + h->off_first_b;
    sa.range_flag = range_flag;
    sa.sticky = h->d_status;
    sy.wg0 = reinterpret_cast<const unsigned*>(packed + h->off_layers + h->lo_split16);
    sy.wg_stride = (long long)h->layer_stride;
    sy.d0 = reinterpret_cast<const unsigned*>(dproj);
    sy.d_stride = p->F_total * h->GR;
    sy.x[0] = reinterpret_cast<unsigned*>(x0);
    sy.x[1] = reinterpret_cast<unsigned*>(x1);
    sy.half = n_blocks_all <= half_max_all;
    sy.force_abort = h->sync_abort;
    sy.force_timeout = h->sync_timeout;
    sync_begin = (!sy.half && fuse_first) ? 1 : 0;
    sync_end = h->L - 1;
    sy.l0 = sync_begin;
    // its counters: the work-queue heads of the first layer it covers (no per-layer launch uses
    // them; zeroed by the plan-descriptor kernel every run)
    sy.ctr = sched_ctr + (size_t)sync_begin * SCHED_CTR_STRIDE * 8;
    sy.L = sync_end - sync_begin;
    for (int l = 0; l < PIPE_MAX_LAYERS; ++l) sy.dil[l] = l < h->L ? h->dil[l] : 1;
    // the per-layer launch's work-unit rules (below), at one workgroup per CU, without its 4-wave
    // cap for 8-32 units per CU (that cap answers the work queues' issue-arbitration imbalance;
    // with the static split 8 waves measured faster: LJ T' = 768 1.65 -> 1.57 ms, T' = 1024
    // 2.15 -> 1.92 ms, `profiles/r03_sync/cap8_*.jsonl`)
    const long long nwg = h->n_cu;
    auto waves = [&](long long units) {
      int w = std::min(8, h->waves_per_wg);
      if (PWG_SMALL_SPREAD && units < nwg * w) w = (int)std::max(1LL, (units + nwg - 1) / nwg);
      return w;
    };
    sy.waves_mid = waves(sy.half ? 2 * n_blocks_all : n_blocks_all);
  }
  // the per-layer launches; the grid-synchronised launch takes the place of layers
  // [sync_begin, sync_end)
  float* xin = x0;
  float* xout = x1;
  for (int l = 0; l < h->L; ++l) {
    if (l == sync_begin && sync_begin < sync_end) {
      const int tc = h->cfg.use_causal_conv ? h->KS - 1 : (h->KS - 1) / 2;
      e = timed(PWG_KERNEL_RESIDUAL_LAYER, [&] { return launch_sync_split16(sy, tc, h->n_cu, s); });
      if (e != hipSuccess) return hip_fail(e, "grid-synchronised forward launch");
    }
    if (l >= sync_begin && l < sync_end) {
      std::swap(xin, xout);
      continue;
    }
    const float* L0 = packed + h->off_layers + h->layer_stride * l;
    LayerArgs la;
    la.x_in = xin; la.x_out = xout; la.skip = skip;
    la.d = dproj + (size_t)l * p->F_total * h->GR;
    la.tab.interior = packed + h->off_tab_interior; la.tab.left = packed + h->off_tab_left;
    la.tab.right = packed + h->off_tab_right; la.tab.small = packed + h->off_tab_small;
    la.tab.H = (int)h->aux.H; la.tab.J1 = h->aux.J1; la.tab.TL = h->aux.TL; la.tab.TR = h->aux.TR;
    la.tab.Fmin = h->aux.Fmin; la.nka = h->aux.nka; la.nfwg = h->aux.nfwg;
    la.wg = L0 + h->lo_wg; la.wgp = L0 + h->lo_wgp; la.bg = L0 + h->lo_bg; la.w2 = L0 + h->lo_w2;
    la.n_blocks = p->n_tiles * (TILE / 32);
    // Small plans (the B = 1 latency path): at most one 32-sample block per wave, spread over every
    // CU with fewer waves per workgroup, rather than crowding the blocks into the first workgroups
    // of each XCD at 8 waves per CU.
    const long long nwg_all = (long long)h->n_cu * h->wg_per_cu;
    // small plans on split16: half-block work units (PWG_OPT_HALF_BLOCKS), every layer but the last
    const long long half_max = h->half_max >= 0 ? h->half_max : 4LL * h->n_cu;
    const bool half = h->layer_kernel == 3 && l != h->L - 1 && la.n_blocks <= half_max;
    const long long units = half ? 2 * la.n_blocks : la.n_blocks;
    int wpw = h->waves_per_wg;
    if (PWG_SMALL_SPREAD && units < nwg_all * wpw) wpw = (int)std::max(1LL, (units + nwg_all - 1) / nwg_all);
    la.tile_utt = d_tile_utt; la.utts = d_utts; la.Tpad = p->Tpad;
    la.R = h->R; la.RS = h->RS; la.S = h->S; la.SS = h->SS; la.KS = h->KS; la.dil = h->dil[l];
    la.tap_center = h->cfg.use_causal_conv ? h->KS - 1 : (h->KS - 1) / 2;
    la.first = l == 0;
    const bool last = l == h->L - 1;
    la.hw1 = packed + h->off_head_w1; la.hw2 = packed + h->off_head_w2; la.hb2 = packed + h->off_head_b2;
    la.out = out; la.O = h->O; la.skip_scale = (float)std::sqrt(1.0 / h->L);
    if (p->layout == PWG_LAYOUT_INFERENCE) { la.out_stride_t = h->O; la.out_stride_o = 1; }
    else { la.out_stride_t = 1; la.out_stride_o = p->utts[0].T; }
    if (split) {
      SplitArgs sa;
      sa.x_in = reinterpret_cast<const unsigned*>(xin); sa.x_out = reinterpret_cast<unsigned*>(xout);
      sa.skip = skip; sa.skip0 = packed + h->off_skip0;
      sa.d = reinterpret_cast<const unsigned*>(la.d);
      sa.tab = packed + h->off_tab_interior;
      sa.tab_left = (int)(h->off_tab_left - h->off_tab_interior);
      sa.tab_right = (int)(h->off_tab_right - h->off_tab_interior);
      sa.tab_small = (int)(h->off_tab_small - h->off_tab_interior);
      sa.blocks = d_blocks;
      sa.wg = reinterpret_cast<const unsigned*>(L0 + (split16 ? h->lo_split16 : h->lo_split));
      sa.hw1 = la.hw1; sa.hw2 = la.hw2; sa.hb2 = la.hb2; sa.out = out;
      if (split16) {
        sa.skip0 = packed + h->off_skip0_16;
        sa.hw1 = packed + h->off_head16_w1;
        sa.hw2 = packed + h->off_head16_w2;
      }
      sa.H = (int)h->aux.H; sa.J1 = h->aux.J1; sa.TL = h->aux.TL; sa.TR = h->aux.TR; sa.Fmin = h->aux.Fmin;
      sa.n_blocks = (int)la.n_blocks; sa.dil = h->dil[l]; sa.first = la.first; sa.O = h->O;
      sa.out_stride_t = (int)la.out_stride_t; sa.out_stride_o = (int)la.out_stride_o;
      sa.skip_scale = la.skip_scale;
      sa.ctr = sched_ctr + (size_t)l * SCHED_CTR_STRIDE * 8;
      const int nwg = h->n_cu * h->wg_per_cu;
      sa.trace = nullptr;
      sa.noise = nullptr; sa.fw = sa.fb = nullptr;
      sa.range_flag = last ? range_flag : nullptr;
      sa.sticky = last ? h->d_status : nullptr;
      if (fuse_first && l == 0) {
        sa.noise = noise; sa.fw = packed + h->off_first_w; sa.fb = packed + h->off_first_b;
      }
      // split16: all of a launch's waves stage the image, wpw of them take blocks. Mid-size plans
      // (8-32 blocks per CU) run 4 computing waves, one per SIMD: with two per SIMD and two or three
      // blocks each, the SIMD's issue arbitration lets one wave finish a block-time before its
      // partner and the launch waits for the later one (LJ T' = 512: 1.58 -> 1.47 ms per forward)
      const int launch_w = split16 ? std::min(8, h->waves_per_wg) : wpw;
      if (split16 && units > 8LL * h->n_cu && units <= 32LL * h->n_cu) wpw = std::min(wpw, 4);
      sa.compute_waves = std::min(wpw, launch_w);
      // diagnostic per-wave timeline (PWG_TRACE_FILE set at pwg_create; split16): every layer's
      // records in the handle's buffer, dumped after the last layer of the run (tools/trace_layer.py)
      const bool trace_on = split16 && !h->trace_fn.empty();
      const size_t per_layer_s = (size_t)nwg * launch_w * 8;
      if (trace_on) {
        const size_t need = per_layer_s * 64;
        if (need > h->trace_words) {  // (re)allocate for this launch's grid: every layer slot fits
          if (h->d_trace) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(h->d_trace);
            h->d_trace = nullptr;
            h->trace_words = 0;
          }
          if (hipMalloc((void**)&h->d_trace, need * sizeof(unsigned long long)) != hipSuccess)
            return fail(PWG_ERR_HIP, "trace buffer");
          h->trace_words = need;
        }
        sa.trace = h->d_trace + per_layer_s * (l % 64);
      }
      e = timed(PWG_KERNEL_RESIDUAL_LAYER, [&] {
        return split16 ? launch_layer_split16(sa, last, la.tap_center, launch_w, nwg, s, half)
                       : launch_layer_split(sa, last, la.tap_center, wpw, nwg, s);
      });
      if (e == hipSuccess && last && trace_on) {
        std::vector<unsigned long long> host(per_layer_s * std::min(h->L, 64));
        e = hipStreamSynchronize(s);
        if (e == hipSuccess) e = hipMemcpy(host.data(), h->d_trace, host.size() * 8, hipMemcpyDeviceToHost);
        FILE* f = e == hipSuccess ? fopen(h->trace_fn.c_str(), "wb") : nullptr;
        if (f) {
          const long long hdr[4] = {std::min(h->L, 64), nwg, launch_w, 8};
          fwrite(hdr, sizeof(hdr), 1, f);
          fwrite(host.data(), 8, host.size(), f);
          fclose(f);
        }
      }
    } else if (h->layer_kernel == 0 && h->aux.nka <= 4) {
      PersistArgs pa2;
      pa2.x_in = xin; pa2.x_out = xout; pa2.skip = skip; pa2.d = la.d;
      pa2.tab = packed + h->off_tab_interior;
      pa2.tab_left = (int)(h->off_tab_left - h->off_tab_interior);
      pa2.tab_right = (int)(h->off_tab_right - h->off_tab_interior);
      pa2.tab_small = (int)(h->off_tab_small - h->off_tab_interior);
      pa2.blocks = d_blocks;
      pa2.wgp = la.wgp; pa2.w2 = la.w2; pa2.bg = la.bg;
      pa2.hw1 = la.hw1; pa2.hw2 = la.hw2; pa2.hb2 = la.hb2; pa2.out = out;
      pa2.H = (int)h->aux.H; pa2.J1 = h->aux.J1; pa2.TL = h->aux.TL; pa2.TR = h->aux.TR;
      pa2.Fmin = h->aux.Fmin; pa2.nka = h->aux.nka;
      pa2.n_blocks = (int)la.n_blocks;
      pa2.R = h->R; pa2.RS = h->RS; pa2.S = h->S; pa2.SS = h->SS; pa2.KS = h->KS; pa2.dil = h->dil[l];
      pa2.tap_center = la.tap_center; pa2.first = la.first; pa2.O = h->O;
      pa2.out_stride_t = (int)la.out_stride_t; pa2.out_stride_o = (int)la.out_stride_o;
      pa2.skip_scale = la.skip_scale;
      const int nwg = h->n_cu * h->wg_per_cu;
      pa2.ctr = sched_ctr + (size_t)l * SCHED_CTR_STRIDE * 8;
      e = timed(PWG_KERNEL_RESIDUAL_LAYER, [&] {
        return launch_layer_persistent(pa2, h->MT, h->M2T, last, wpw, nwg, s);
      });
    } else {
      e = timed(PWG_KERNEL_RESIDUAL_LAYER,
                [&] { return launch_layer(la, h->MT, h->M2T, last, p->n_tiles, s); });
    }
    if (e != hipSuccess) return hip_fail(e, "residual layer launch");
    std::swap(xin, xout);
  }
  return PWG_OK;
}

int pwg_run_status(PwgPlan* p, const void* workspace, void* stream) {
  if (!p || !workspace) return fail(PWG_ERR_INVALID, "null argument");
  DeviceGuard g(p->h->device);
  if (!g.ok) return fail(PWG_ERR_HIP, "hipSetDevice failed");
  hipStream_t s = (hipStream_t)stream;
  int* flag = nullptr;
  {
    std::lock_guard<std::mutex> lk(p->h->hstatus_mu);
    int*& w = p->h->hstatus[s];
    if (!w && hipHostMalloc(reinterpret_cast<void**>(&w), 2 * sizeof(int), hipHostMallocDefault) != hipSuccess) {
      w = nullptr;
      return fail(PWG_ERR_HIP, "pinned status words");
    }
    flag = w;
  }
  flag[0] = flag[1] = 0;
  hipError_t e = hipMemcpyAsync(&flag[0], (const char*)workspace + p->ws_flag, sizeof(int), hipMemcpyDeviceToHost, s);
  // the handle's sticky word: every flag any run of this handle set since the previous status call
  // (a serving loop that checks once per batch of runs still sees an earlier run's abort); cleared
  // here, in stream order
  if (e == hipSuccess && p->h->d_status != nullptr) {
    e = hipMemcpyAsync(&flag[1], p->h->d_status, sizeof(int), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemsetAsync(p->h->d_status, 0, sizeof(int), s);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "run status");
  const int st = flag[0] | flag[1];
  if (st & PWG_STATUS_SYNC_ABORT)
    return fail(PWG_ERR_RERUN, "grid-synchronised forward: not every workgroup could start (the GPU is shared "
                               "with other work), so it computed nothing and the output is NaN; rerun with "
                               "PWG_OPT_SYNC 0");
  if (st & PWG_STATUS_SYNC_TIMEOUT)
    return fail(PWG_ERR_RERUN, "grid-synchronised forward: a grid-barrier wait gave up (a workgroup was "
                               "descheduled?), so the output is NaN; rerun with PWG_OPT_SYNC 0");
  if (st & PWG_STATUS_PIPE_TIMEOUT)
    return fail(PWG_ERR_RERUN, "layer-pipelined forward: a dependency wait gave up, so the output is invalid; "
                               "rerun with PWG_OPT_PIPELINE 0");
  if (st != 0)
    return fail(PWG_ERR_RANGE,
                "split-f16 range flag: a value left the fp16 pair range (an aux projection row, the "
                "scaled final skip sum, or upstream x / first_conv values making a skip sum non-finite; or the "
                "input is not finite); rerun with PWG_OPT_LAYER_KERNEL 0 (exact fp32)");
  return PWG_OK;
}

struct PwgGraph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  int device = 0;
};

int pwg_graph_create(PwgPlan* p, const float* packed, const float* mel, const float* noise, const float* mean,
                     const float* scale, float* out, void* workspace, void* stream, PwgGraph** out_graph) {
  if (!p || !out_graph) return fail(PWG_ERR_INVALID, "null argument");
  *out_graph = nullptr;
  if (stream == nullptr) return fail(PWG_ERR_INVALID, "graph capture needs a created stream, not the null stream");
  PwgHandle* h = p->h;
  if (h->timing) return fail(PWG_ERR_INVALID, "disable timing (pwg_set_timing) before capturing a graph");
  DeviceGuard g(h->device);
  if (!g.ok) return fail(PWG_ERR_HIP, "hipSetDevice failed");
  if (h->n_cu == 0) {  // pwg_run queries it on first use; not inside the capture
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || n < 1)
      return fail(PWG_ERR_HIP, "cannot query the CU count");
    h->n_cu = n;
  }
  hipStream_t s = (hipStream_t)stream;
  // one eager run first, so that the kernels' first-launch work (code-object load, LDS size
  // attribute) happens outside the capture
  int rc0 = pwg_run(p, packed, mel, noise, mean, scale, out, workspace, stream);
  if (rc0 != PWG_OK) return rc0;
  hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "graph warm-up run");
  e = hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
  if (e != hipSuccess) return hip_fail(e, "hipStreamBeginCapture");
  const int rc = pwg_run(p, packed, mel, noise, mean, scale, out, workspace, stream);
  hipGraph_t graph = nullptr;
  e = hipStreamEndCapture(s, &graph);
  if (rc != PWG_OK) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc;  // pwg_run's message stands
  }
  if (e != hipSuccess || !graph) return hip_fail(e != hipSuccess ? e : hipErrorUnknown, "hipStreamEndCapture");
  hipGraphExec_t exec = nullptr;
  e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    (void)hipGraphDestroy(graph);
    return hip_fail(e, "hipGraphInstantiate");
  }
  PwgGraph* gr = new PwgGraph();
  gr->graph = graph;
  gr->exec = exec;
  gr->device = h->device;
  *out_graph = gr;
  return PWG_OK;
}

int pwg_graph_launch(PwgGraph* gr, void* stream) {
  if (!gr) return fail(PWG_ERR_INVALID, "null graph");
  DeviceGuard g(gr->device);
  if (!g.ok) return fail(PWG_ERR_HIP, "hipSetDevice failed");
  const hipError_t e = hipGraphLaunch(gr->exec, (hipStream_t)stream);
  return e == hipSuccess ? PWG_OK : hip_fail(e, "hipGraphLaunch");
}

void pwg_graph_destroy(PwgGraph* gr) {
  if (!gr) return;
  DeviceGuard g(gr->device);
  if (gr->exec) (void)hipGraphExecDestroy(gr->exec);
  if (gr->graph) (void)hipGraphDestroy(gr->graph);
  delete gr;
}

int pwg_set_option(PwgHandle* h, int option, long long value) {
  if (!h) return fail(PWG_ERR_INVALID, "null handle");
  switch (option) {
    case PWG_OPT_LAYER_KERNEL:
      if (value < 0 || value > 3) return fail(PWG_ERR_INVALID, "layer kernel must be 0, 1, 2 or 3");
      if (value >= 2 && !h->split_ok)
        return fail(PWG_ERR_UNSUPPORTED, "split-f16 layer kernel needs R = S = 64, gate_channels = 128, kernel_size = 3");
      h->layer_kernel = (int)value;
      return PWG_OK;
    case PWG_OPT_WAVES_PER_WG:
      if (value < 1 || value > 16) return fail(PWG_ERR_INVALID, "waves per workgroup must be in [1, 16]");
      h->waves_per_wg = (int)value;
      return PWG_OK;
    case PWG_OPT_FUSE_FIRST_CONV:
      if (value != 0 && value != 1) return fail(PWG_ERR_INVALID, "fuse_first_conv must be 0 or 1");
      h->fuse_first = (int)value;
      return PWG_OK;
    case PWG_OPT_WG_PER_CU:
      if (value < 1 || value > 64) return fail(PWG_ERR_INVALID, "workgroups per CU must be in [1, 64]");
      h->wg_per_cu = (int)value;
      return PWG_OK;
    case PWG_OPT_PIPELINE:
      if (value < 0) return fail(PWG_ERR_INVALID, "pipeline plan limit must be >= 0");
      h->pipe_max = value;
      return PWG_OK;
    case PWG_OPT_HALF_BLOCKS:
      if (value < 0) return fail(PWG_ERR_INVALID, "half-block limit must be >= 0");
      h->half_max = value;
      return PWG_OK;
    case PWG_OPT_SYNC:
      if (value < 0) return fail(PWG_ERR_INVALID, "grid-synchronised plan limit must be >= 0");
      h->sync_max = value;
      return PWG_OK;
    case PWG_OPT_SYNC_ABORT:
      if (value != 0 && value != 1) return fail(PWG_ERR_INVALID, "sync_abort must be 0 or 1");
      h->sync_abort = (int)value;
      return PWG_OK;
    case PWG_OPT_SYNC_TIMEOUT:
      if (value != 0 && value != 1) return fail(PWG_ERR_INVALID, "sync_timeout must be 0 or 1");
      h->sync_timeout = (int)value;
      return PWG_OK;

    default:
      return fail(PWG_ERR_INVALID, "unknown option");
  }
}

int pwg_get_option(const PwgHandle* h, int option, long long* value) {
  if (!h || !value) return fail(PWG_ERR_INVALID, "null argument");
  switch (option) {
    case PWG_OPT_LAYER_KERNEL: *value = h->layer_kernel; return PWG_OK;
    case PWG_OPT_WAVES_PER_WG: *value = h->waves_per_wg; return PWG_OK;
    case PWG_OPT_FUSE_FIRST_CONV: *value = h->fuse_first; return PWG_OK;
    case PWG_OPT_WG_PER_CU: *value = h->wg_per_cu; return PWG_OK;
    case PWG_OPT_PIPELINE: *value = h->pipe_max; return PWG_OK;
    case PWG_OPT_HALF_BLOCKS: *value = h->half_max >= 0 ? h->half_max : 4LL * h->n_cu; return PWG_OK;
    case PWG_OPT_SYNC: *value = h->sync_max >= 0 ? h->sync_max : 64LL * h->n_cu; return PWG_OK;
    case PWG_OPT_SYNC_ABORT: *value = h->sync_abort; return PWG_OK;
    case PWG_OPT_SYNC_TIMEOUT: *value = h->sync_timeout; return PWG_OK;

    default: return fail(PWG_ERR_INVALID, "unknown option");
  }
}

int pwg_release_stream(PwgHandle* h, void* stream) {
  if (!h) return fail(PWG_ERR_INVALID, "null handle");
  std::lock_guard<std::mutex> lk(h->hstatus_mu);
  auto it = h->hstatus.find((hipStream_t)stream);
  if (it == h->hstatus.end()) return PWG_OK;
  DeviceGuard g(h->device);
  // the pinned word's copy is queued on that stream: let it land before the word is freed
  if (stream && hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return fail(PWG_ERR_HIP, "stream synchronize");
  (void)hipHostFree(it->second);
  h->hstatus.erase(it);
  return PWG_OK;
}

int pwg_set_timing(PwgHandle* h, int enable) {
  if (!h) return fail(PWG_ERR_INVALID, "null handle");
  if (enable < 0 || enable > 2) return fail(PWG_ERR_INVALID, "timing mode must be 0, 1 or 2");
  h->timing = enable;
  return PWG_OK;
}

int pwg_timing_collect(PwgHandle* h, double* ms, long long* launches) {
  if (!h || !ms || !launches) return fail(PWG_ERR_INVALID, "null argument");
  DeviceGuard g(h->device);
  for (auto& r : h->records) {
    hipError_t e = hipEventSynchronize(r.stop);
    float t = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, r.start, r.stop);
    if (e != hipSuccess) return hip_fail(e, "timing collect");
    if (r.bucket >= 0) {  // (-1: a whole-run span record of timing mode 2)
      ms[r.bucket] += t;
      launches[r.bucket] += 1;
    }
    h->event_pool.push_back(r.start);
    h->event_pool.push_back(r.stop);
  }
  h->records.clear();
  return PWG_OK;
}

int pwg_timing_span(PwgHandle* h, double* span_ms) {
  if (!h || !span_ms) return fail(PWG_ERR_INVALID, "null argument");
  *span_ms = 0.0;
  if (h->records.empty()) return PWG_OK;
  DeviceGuard g(h->device);
  hipEvent_t ref = h->records[0].start;  // one stream: every later record is later
  double hi = 0.0;
  for (auto& r : h->records) {
    hipError_t e = hipEventSynchronize(r.stop);
    float t = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, ref, r.stop);
    if (e != hipSuccess) return hip_fail(e, "timing span");
    hi = std::max(hi, (double)t);
  }
  *span_ms = hi;
  return PWG_OK;
}

}  // extern "C"

namespace pwg {
// shared with pwg_cnet.hip: one thread-local last-error message for the whole library
int set_error(int code, const char* msg) { return fail(code, msg); }

hipError_t allow_lds(const void* kfn, int lds) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, int> done;  // (device, kernel) -> largest size allowed
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = done.find({dev, kfn});
    if (it != done.end() && it->second >= lds) return hipSuccess;
  }
  const hipError_t e = hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e == hipSuccess) {
    std::lock_guard<std::mutex> lk(mu);
    int& v = done[{dev, kfn}];
    v = std::max(v, lds);
  }
  return e;
}
}  // namespace pwg
