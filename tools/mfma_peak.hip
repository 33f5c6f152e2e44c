// Calibration microbenchmark (not part of the engine): sustained v_mfma_f32_32x32x2_f32 rate on
// this MI355X, (a) register-only with 4 independent accumulators per wave, (b) A operands read
// from LDS with ds_read_b128 every 4 k-steps and B from registers -- the shape of the persistent
// layer kernel's GEMM-1 loop. Random operands (DVFS depends on data, MI355X_MICROARCH.md).
//   hipcc --offload-arch=gfx950 -O3 -o mfma_peak tools/mfma_peak.hip && ./mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int ITERS>
__global__ void __launch_bounds__(768) mfma_regs(const float* in, float* out) {
  const int lane = threadIdx.x & 63;
  float a0 = in[lane], a1 = in[lane + 64], b0 = in[lane + 128], b1 = in[lane + 192];
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int it = 0; it < ITERS; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int ITERS>
__global__ void __launch_bounds__(768) mfma_lds(const float* in, float* out) {
  __shared__ f32x4 lds[64 * 4 * 16];  // 16 slices x 4 m-tiles x 64 lanes
  for (int i = threadIdx.x; i < 64 * 4 * 16; i += blockDim.x) {
    f32x4 v = {in[i & 255], in[(i + 1) & 255], in[(i + 2) & 255], in[(i + 3) & 255]};
    lds[i] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  f32x4 b = {in[lane], in[lane + 64], in[lane + 128], in[lane + 192]};
  f32x16 acc[4] = {};
  for (int it = 0; it < ITERS; ++it) {
    const int sl = it & 15;
    f32x4 av[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) av[m] = lds[(sl * 4 + m) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m][i], b[i], acc[m], 0, 0, 0);
  }
  float s = 0.f;
  for (int m = 0; m < 4; ++m)
    for (int r = 0; r < 16; ++r) s += acc[m][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int dev = 0, ncu = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<float> h(256);
  unsigned x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (float)(x >> 8) / (1 << 24) - 0.5f; }
  float *in, *out;
  CHECK(hipMalloc(&in, 256 * sizeof(float)));
  CHECK(hipMalloc(&out, (size_t)ncu * 4 * 768 * sizeof(float)));
  CHECK(hipMemcpy(in, h.data(), 256 * sizeof(float), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  constexpr int IT = 20000;
  for (int waves : {4, 8, 12}) {
    for (int kind = 0; kind < 2; ++kind) {
      const dim3 grid(ncu), block(64 * waves);
      for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(e0));
        if (kind == 0) hipLaunchKernelGGL(mfma_regs<IT>, grid, block, 0, 0, in, out);
        else hipLaunchKernelGGL(mfma_lds<IT / 4>, grid, block, 0, 0, in, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double mfmas = (double)ncu * waves * IT * 4;
        const double tf = mfmas * 32 * 32 * 2 * 2 / (ms * 1e-3) / 1e12;
        if (rep == 2)
          printf("%s waves/CU=%2d: %.3f ms  %.1f TFLOP/s  (%.2f GHz-equivalent at 100%% pipe)\n",
                 kind == 0 ? "regs" : "lds ", waves, ms, tf, tf * 1e12 / (ncu * 4 * 64.0) / 1e9);
      }
    }
  }
  return 0;
}
