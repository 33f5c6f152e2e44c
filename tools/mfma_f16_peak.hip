// Calibration microbenchmark (not part of the engine): the split-f16 layer kernel's GEMM-1 inner
// loop shape on v_mfma_f32_32x32x16_f16 -- 4 accumulators (m-tiles), per k-step 8 ds_read_b128
// (A hi/lo of 4 m-tiles) and 12 MFMAs (hi*hi, hi*lo, lo*hi) with B in registers.
//   kind 0: operands in registers only
//   kind 1: A from LDS, read at the top of each k-step (the kernel as first written)
//   kind 2: A from LDS, read one k-step ahead (double-buffered fragments)
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_f16 tools/mfma_f16_peak.hip && /tmp/mfma_f16
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ f32x16 mma(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

template <int KIND>
__global__ void __launch_bounds__(512, 1) kern(const unsigned* in, float* out, int iters) {
  extern __shared__ u32x4 lds[];  // 16 k-steps x 4 m x 2 x 64 lanes = 128 KB
  for (int i = threadIdx.x; i < 16 * 8 * 64; i += blockDim.x) {
    u32x4 v = {in[i & 255], in[(i + 7) & 255], in[(i + 13) & 255], in[(i + 29) & 255]};
    lds[i] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  u32x4 b[8];
  for (int i = 0; i < 8; ++i) b[i] = u32x4{in[lane], in[lane + 64], in[lane + 128], in[(lane + 192 + i) & 255]};
  f32x16 acc[4] = {};
  const u32x4* al = lds + lane;
  u32x4 ah[4], alo[4];
  if (KIND == 0 || KIND == 2)
    for (int m = 0; m < 4; ++m) { ah[m] = al[(m * 2) * 64]; alo[m] = al[(m * 2 + 1) * 64]; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ks = (it * 4 + s) & 15;
      u32x4 nh[4], nl[4];
      if (KIND == 1) {
#pragma unroll
        for (int m = 0; m < 4; ++m) { ah[m] = al[((ks * 4 + m) * 2) * 64]; alo[m] = al[((ks * 4 + m) * 2 + 1) * 64]; }
      } else if (KIND == 2) {
        const int kn = (ks + 1) & 15;
#pragma unroll
        for (int m = 0; m < 4; ++m) { nh[m] = al[((kn * 4 + m) * 2) * 64]; nl[m] = al[((kn * 4 + m) * 2 + 1) * 64]; }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = mma(ah[m], b[s], acc[m]);
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = mma(ah[m], b[4 + s], acc[m]);
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = mma(alo[m], b[s], acc[m]);
      if (KIND == 2) {
#pragma unroll
        for (int m = 0; m < 4; ++m) { ah[m] = nh[m]; alo[m] = nl[m]; }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float sum = 0.f;
  for (int m = 0; m < 4; ++m)
    for (int r = 0; r < 16; ++r) sum += acc[m][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = sum;
}

// kind 3: the same work on v_mfma_f32_16x16x32_f16 -- 8 m-tiles x 2 n-tiles of 16x16 per wave (the
// same 128 x 32 output tile), per k-step 16 ds_read_b128 (A hi/lo) and 48 MFMAs
__device__ __forceinline__ f32x4 mma16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
__global__ void __launch_bounds__(512, 1) kern16(const unsigned* in, float* out, int iters) {
  extern __shared__ u32x4 lds[];
  for (int i = threadIdx.x; i < 16 * 8 * 64; i += blockDim.x) {
    u32x4 v = {in[i & 255], in[(i + 7) & 255], in[(i + 13) & 255], in[(i + 29) & 255]};
    lds[i] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  u32x4 b[2][2];
  for (int n = 0; n < 2; ++n)
    for (int h = 0; h < 2; ++h) b[n][h] = u32x4{in[lane], in[lane + 64 + n], in[lane + 128 + h], in[(lane + 192) & 255]};
  f32x4 acc[8][2] = {};
  const u32x4* al = lds + lane;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ks = (it * 4 + s) & 7;
      u32x4 ah[8], alo[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) { ah[m] = al[((ks * 8 + m) * 2) * 64]; alo[m] = al[((ks * 8 + m) * 2 + 1) * 64]; }
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          acc[m][n] = mma16(ah[m], b[n][0], acc[m][n]);
          acc[m][n] = mma16(ah[m], b[n][1], acc[m][n]);
          acc[m][n] = mma16(alo[m], b[n][0], acc[m][n]);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float sum = 0.f;
  for (int m = 0; m < 8; ++m)
    for (int n = 0; n < 2; ++n)
      for (int r = 0; r < 4; ++r) sum += acc[m][n][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = sum;
}

int main() {
  int dev = 0, ncu = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<unsigned> h(256);
  unsigned x = 12345;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    const unsigned a = 0x3000u + ((x >> 8) & 0x7ffu), c = 0x3000u + ((x >> 20) & 0x7ffu);  // fp16 ~[0.125, 0.5)
    v = a | (c << 16);
  }
  unsigned* in;
  float* out;
  CHECK(hipMalloc(&in, 256 * sizeof(unsigned)));
  CHECK(hipMalloc(&out, (size_t)ncu * 512 * sizeof(float)));
  CHECK(hipMemcpy(in, h.data(), 256 * sizeof(unsigned), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int iters = 4000;
  const size_t lds = 16 * 8 * 64 * 16;
  CHECK(hipFuncSetAttribute((const void*)kern<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CHECK(hipFuncSetAttribute((const void*)kern<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CHECK(hipFuncSetAttribute((const void*)kern<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CHECK(hipFuncSetAttribute((const void*)kern16, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int waves : {4, 8}) {
    for (int kind = 0; kind < 4; ++kind) {
      const dim3 grid(ncu), block(64 * waves);
      for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(e0));
        if (kind == 0) hipLaunchKernelGGL(kern<0>, grid, block, lds, 0, in, out, iters);
        else if (kind == 1) hipLaunchKernelGGL(kern<1>, grid, block, lds, 0, in, out, iters);
        else if (kind == 2) hipLaunchKernelGGL(kern<2>, grid, block, lds, 0, in, out, iters);
        else hipLaunchKernelGGL(kern16, grid, block, lds, 0, in, out, iters);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double mfmas = (double)ncu * waves * iters * 4 * 12;
        const double tf = mfmas * 32 * 32 * 16 * 2 * (kind == 3 ? 2 : 1) / (ms * 1e-3) / 1e12;  // kind 3: K=32 steps
        if (rep == 2)
          printf("kind %d waves/CU=%d: %.3f ms  %.1f TFLOP/s f16  (%.1f cyc/MFMA/SIMD at 2.4 GHz)\n", kind, waves, ms, tf,
                 ms * 1e-3 * 2.4e9 / (mfmas / (ncu * 4)));
      }
    }
  }
  return 0;
}
