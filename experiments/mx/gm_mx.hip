// gm_mx.hip — gfx950 block-scaled (MX) MFMA probes (fp8 e4m3 / fp4 e2m1 with E8M0 scales).
// Moved out of the gpumounter-amd probe library in round 5: the post-attach validation needs
// only the liveness kernel; these stay as a stand-alone experiment (README.md). Built with
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I../../native/hip
#include "gm_mx.h"

#include <hip/hip_runtime.h>

#include "gm_probe_common.h"

namespace {

// ------------------------------------------------------------------ MX (block-scaled) MFMA
// gfx950's v_mfma_scale_f32_16x16x128_f8f6f4: one instruction = a 16x16 f32 tile += A[16x128]·
// B[128x16] with A/B in fp8 (e4m3, fmt 0), bf8 (e5m2, 1), fp6 (2/3) or fp4 (e2m1, 4), each lane's
// K-block of 32 scaled by an E8M0 exponent (127 = 1.0). MI355X runs fp8 at 2× and fp6/fp4 at 4×
// the bf16 MFMA rate (MI355X_MICROARCH.md "FP8/FP6/FP4"), so this is the pipe inference kernels
// use and the bf16 probe does not exercise. A/B operands are 8 dwords per lane (fp4 uses 4).
typedef int i32x8 __attribute__((ext_vector_type(8)));

template <int FMT>
__device__ __forceinline__ f32x4 mx_mfma(const i32x8& a, const i32x8& b, f32x4 c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, FMT, FMT, 0, sa, 0, sb);
}

// Register-resident MX-MFMA peak: 8 independent accumulators per wave, deterministic inputs, the
// wave's sums written out so two runs (or two GPUs) can be compared bit for bit.
template <int FMT>
__global__ __launch_bounds__(256) void k_mx_peak(float* out, int iters, uint32_t seed) {
  i32x8 a, b;
  for (int j = 0; j < 8; ++j) {
    // small finite values in every format: clear each byte's top exponent bit (no NaN/inf)
    a[j] = (int)((seed * (threadIdx.x * 8 + j + 1) * 2654435761u) & 0x3b3b3b3bu);
    b[j] = (int)((seed * (blockIdx.x * 8 + j + 7) * 40503u) & 0x3b3b3b3bu);
  }
  const int sa = 127 - (int)(threadIdx.x & 3), sb = 126;   // 2^0 … 2^-3, 2^-1
  f32x4 c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0}, c4 = {0}, c5 = {0}, c6 = {0}, c7 = {0};
  for (int i = 0; i < iters; ++i) {
    c0 = mx_mfma<FMT>(a, b, c0, sa, sb);
    c1 = mx_mfma<FMT>(b, a, c1, sa, sb);
    c2 = mx_mfma<FMT>(a, a, c2, sa, sb);
    c3 = mx_mfma<FMT>(b, b, c3, sa, sb);
    c4 = mx_mfma<FMT>(a, b, c4, sb, sa);
    c5 = mx_mfma<FMT>(b, a, c5, sb, sa);
    c6 = mx_mfma<FMT>(a, a, c6, sb, sa);
    c7 = mx_mfma<FMT>(b, b, c7, sb, sa);
  }
  float s = 0.f;
  for (int j = 0; j < 4; ++j) s += c0[j] + c1[j] + c2[j] + c3[j] + c4[j] + c5[j] + c6[j] + c7[j];
  // one value per wave: blockIdx.x * 4 + wave
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

// 32x32x64 form: the same MX pipe on a 32x32 tile (16 accumulator registers per chain).
template <int FMT, int CHAINS>
__global__ __launch_bounds__(256) void k_mx_peak32(float* out, int iters, uint32_t seed) {
  i32x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (int)((seed * (threadIdx.x * 8 + j + 1) * 2654435761u) & 0x3b3b3b3bu);
    b[j] = (int)((seed * (blockIdx.x * 8 + j + 7) * 40503u) & 0x3b3b3b3bu);
  }
  const int sa = 127 - (int)(threadIdx.x & 3), sb = 126;
  f32x16 c[CHAINS];
  for (int q = 0; q < CHAINS; ++q) c[q] = (f32x16){0};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int q = 0; q < CHAINS; ++q)
      c[q] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4((q & 1) ? b : a, (q & 2) ? b : a,
                                                             c[q], FMT, FMT, 0, sa, 0, sb);
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < CHAINS; ++q)
    for (int j = 0; j < 16; ++j) s += c[q][j];
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

// One MX-MFMA on caller-given per-lane register images (numerics check; the lane→(row, k) map is
// the test's business): afrag/bfrag = 64 lanes × 32 bytes, sa/sb = 64 E8M0 bytes, c = 64 × 4 f32.
template <int FMT>
__global__ __launch_bounds__(64) void k_mx_tile(const i32x8* afrag, const i32x8* bfrag,
                                                const uint8_t* sa, const uint8_t* sb, f32x4* c) {
  const int l = threadIdx.x;
  f32x4 acc = {0};
  acc = mx_mfma<FMT>(afrag[l], bfrag[l], acc, sa[l], sb[l]);
  c[l] = acc;
}

}  // namespace

// Default = the measured-best form per format on MI355X (profiles/r3_mx/sweep.json, best of 3):
// 32x32x64 × 4 chains for fp8 (5.02 PF/s vs 4.91 for 16x16x128 × 8), × 8 chains for fp4
// (9.37 PF/s vs 7.21).
int gm_mx_peak(int dev, int fmt, int iters, int blocks_per_cu, float* sums, int nsums,
                     double* tflops) {
  return gm_mx_peak_variant(dev, fmt, fmt == 4 ? 2 : 1, iters, blocks_per_cu, sums, nsums,
                                  tflops);
}

int gm_mx_peak_variant(int dev, int fmt, int variant, int iters, int blocks_per_cu,
                             float* sums, int nsums, double* tflops) {
  *tflops = 0;
  if ((fmt != 0 && fmt != 4) || variant < 0 || variant > 2) return (int)hipErrorInvalidValue;
  DeviceGuard g(dev);
  if (!g.ok) return (int)hipErrorInvalidDevice;
  hipDeviceProp_t p;
  GM_CHECK(hipGetDeviceProperties(&p, dev));
  const int blocks = p.multiProcessorCount * blocks_per_cu;
  if (sums != nullptr && nsums < blocks * 4) return (int)hipErrorInvalidValue;
  float* out = nullptr;
  GM_CHECK(hipMalloc(&out, (size_t)blocks * 4 * sizeof(float)));
  const uint32_t seed = 0x9e3779b9u;
  auto launch = [&](int it) {
    const dim3 g(blocks), t(256);
    if (variant == 1) {
      if (fmt == 4) hipLaunchKernelGGL((k_mx_peak32<4, 4>), g, t, 0, 0, out, it, seed);
      else hipLaunchKernelGGL((k_mx_peak32<0, 4>), g, t, 0, 0, out, it, seed);
    } else if (variant == 2) {
      if (fmt == 4) hipLaunchKernelGGL((k_mx_peak32<4, 8>), g, t, 0, 0, out, it, seed);
      else hipLaunchKernelGGL((k_mx_peak32<0, 8>), g, t, 0, 0, out, it, seed);
    } else {
      if (fmt == 4) hipLaunchKernelGGL(k_mx_peak<4>, g, t, 0, 0, out, it, seed);
      else hipLaunchKernelGGL(k_mx_peak<0>, g, t, 0, 0, out, it, seed);
    }
  };
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch(iters);  // warm-up as long as the timed run (DVFS)
  (void)hipEventRecord(a, 0);
  launch(iters);
  (void)hipEventRecord(b, 0);
  hipError_t e = hipEventSynchronize(b);
  float ms = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
  const double per_wave_iter = variant == 0 ? 2.0 * 16 * 16 * 128 * 8
                                              : 2.0 * 32 * 32 * 64 * (variant == 1 ? 4 : 8);
  const double flops = per_wave_iter * iters * (double)blocks * 4;
  if (e == hipSuccess && ms > 0) *tflops = flops / (ms * 1e-3) / 1e12;
  if (e == hipSuccess && sums != nullptr)
    e = hipMemcpy(sums, out, (size_t)blocks * 4 * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(out);
  return (int)e;
}

int gm_mx_tile(int dev, int fmt, const uint8_t* afrag, const uint8_t* bfrag,
                     const uint8_t* sa, const uint8_t* sb, float* c) {
  if (fmt != 0 && fmt != 4) return (int)hipErrorInvalidValue;
  DeviceGuard g(dev);
  if (!g.ok) return (int)hipErrorInvalidDevice;
  uint8_t* d = nullptr;   // afrag 2048 | bfrag 2048 | sa 64 | sb 64 | c 1024
  GM_CHECK(hipMalloc(&d, 2048 + 2048 + 64 + 64 + 1024));
  hipError_t e = hipMemcpy(d, afrag, 2048, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d + 2048, bfrag, 2048, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d + 4096, sa, 64, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d + 4160, sb, 64, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    auto* af = reinterpret_cast<const i32x8*>(d);
    auto* bf = reinterpret_cast<const i32x8*>(d + 2048);
    auto* cf = reinterpret_cast<f32x4*>(d + 4224);
    if (fmt == 4)
      hipLaunchKernelGGL(k_mx_tile<4>, dim3(1), dim3(64), 0, 0, af, bf, d + 4096, d + 4160, cf);
    else
      hipLaunchKernelGGL(k_mx_tile<0>, dim3(1), dim3(64), 0, 0, af, bf, d + 4096, d + 4160, cf);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(c, d + 4224, 1024, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  return (int)e;
}

const char* gm_mx_strerror(int err) { return hipGetErrorString((hipError_t)err); }
