// gm_probe.hip — CDNA4 (gfx950) post-attach validation kernels. Built with
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC
// Design notes (MI355X-first):
//   * every kernel is written for 64-lane waves (lane = threadIdx.x & 63, 64-bit ballots);
//   * the HBM probe streams 16 B/lane (global_load_dwordx4) with a grid of 8 blocks per CU so all
//     256 CUs / 8 XCDs are busy; blockIdx is remapped so consecutive tiles land on one XCD's L2;
//   * the MFMA probes use __builtin_amdgcn_mfma_f32_32x32x16_bf16 with the gfx950 lane maps
//     (A[r][8h+j], B[8h+j][r], C row=(i&3)+8(i>>2)+4h, col=r) — see cdna_hip_programming.md §3.
#include "gm_probe.h"

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <strings.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <mutex>
#include <random>
#include <vector>

#include "gm_probe_common.h"

namespace {

// ------------------------------------------------------------------ liveness
__global__ __launch_bounds__(64) void k_quick(uint32_t* out, uint32_t salt) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t v = lane * 2654435761u ^ salt;
  out[lane] = v;
  // wave-wide reduction through 64-lane shuffles: the checksum lands in lane 0
  uint32_t s = v;
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, kWave);
  const unsigned long long ballot = __ballot(1);
  if (lane == 0) {
    out[64] = s;
    out[65] = (uint32_t)__popcll(ballot);  // 64 on a wave64 machine
  }
}

// ------------------------------------------------------------------ HBM stream
// XCD-aware remap: the dispatcher round-robins consecutive block ids over the 8 XCDs; giving each
// XCD a contiguous slab keeps its L2 prefetch streams independent.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nblocks) {
  const uint32_t per = nblocks / 8;
  if (per == 0 || nblocks % 8) return bid;
  return (bid % 8) * per + (bid / 8);
}

__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ src,
                                              float4* __restrict__ dst, size_t n) {
  const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)b * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

// Contiguous chunk per block, 4 independent 16-B loads in flight per lane before the stores:
// more bytes outstanding per wave and DRAM-page-friendly streams.
typedef float v4f __attribute__((ext_vector_type(4)));

template <int kChunk, bool kNonTemporal>
__global__ __launch_bounds__(256) void k_copy_chunk(const float4* __restrict__ src_,
                                                    float4* __restrict__ dst_, size_t n,
                                                    size_t per_block) {
  const v4f* __restrict__ src = reinterpret_cast<const v4f*>(src_);
  v4f* __restrict__ dst = reinterpret_cast<v4f*>(dst_);
  const size_t begin = (size_t)blockIdx.x * per_block;
  const size_t end = begin + per_block < n ? begin + per_block : n;
  size_t i = begin + threadIdx.x;
  for (; i + (kChunk - 1) * 256 < end; i += kChunk * 256) {
    v4f r[kChunk];
#pragma unroll
    for (int c = 0; c < kChunk; ++c) {  // all loads issued before the first store
      if constexpr (kNonTemporal)
        r[c] = __builtin_nontemporal_load(&src[i + c * 256]);
      else
        r[c] = src[i + c * 256];
    }
#pragma unroll
    for (int c = 0; c < kChunk; ++c) {
      if constexpr (kNonTemporal)
        __builtin_nontemporal_store(r[c], &dst[i + c * 256]);
      else
        dst[i + c * 256] = r[c];
    }
  }
  for (; i < end; i += 256) dst[i] = src[i];
}

// Read-only stream: each block walks its contiguous chunk with kChunk 16-B nontemporal loads in
// flight per lane and folds them into one XOR per lane (written once, so nothing is dead code).
template <int kChunk>
__global__ __launch_bounds__(256) void k_read_chunk(const float4* __restrict__ src_,
                                                    uint32_t* __restrict__ sink, size_t n,
                                                    size_t per_block) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u* __restrict__ src = reinterpret_cast<const v4u*>(src_);
  const size_t begin = (size_t)blockIdx.x * per_block;
  const size_t end = begin + per_block < n ? begin + per_block : n;
  v4u acc = {0, 0, 0, 0};
  size_t i = begin + threadIdx.x;
  for (; i + (kChunk - 1) * 256 < end; i += kChunk * 256) {
    v4u r[kChunk];
#pragma unroll
    for (int c = 0; c < kChunk; ++c) r[c] = __builtin_nontemporal_load(&src[i + c * 256]);
#pragma unroll
    for (int c = 0; c < kChunk; ++c) acc ^= r[c];
  }
  for (; i < end; i += 256) acc ^= src[i];
  const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9e3779b9u) sink[blockIdx.x & 1023] = x;  // practically never taken, keeps the loads
}

// Software-pipelined variant: the next chunk's loads are issued before the current chunk's
// stores, so a wave always has kChunk reads outstanding while its writes drain.
template <int kChunk>
__global__ __launch_bounds__(256) void k_copy_pipe(const float4* __restrict__ src_,
                                                   float4* __restrict__ dst_, size_t n,
                                                   size_t per_block) {
  const v4f* __restrict__ src = reinterpret_cast<const v4f*>(src_);
  v4f* __restrict__ dst = reinterpret_cast<v4f*>(dst_);
  const size_t begin = (size_t)blockIdx.x * per_block;
  const size_t end = begin + per_block < n ? begin + per_block : n;
  constexpr size_t kStep = (size_t)kChunk * 256;
  size_t i = begin + threadIdx.x;
  if (i + (kChunk - 1) * 256 < end) {
    v4f cur[kChunk];
#pragma unroll
    for (int c = 0; c < kChunk; ++c) cur[c] = __builtin_nontemporal_load(&src[i + c * 256]);
    for (; i + kStep + (kChunk - 1) * 256 < end; i += kStep) {
      v4f nxt[kChunk];
#pragma unroll
      for (int c = 0; c < kChunk; ++c)
        nxt[c] = __builtin_nontemporal_load(&src[i + kStep + c * 256]);
#pragma unroll
      for (int c = 0; c < kChunk; ++c) __builtin_nontemporal_store(cur[c], &dst[i + c * 256]);
#pragma unroll
      for (int c = 0; c < kChunk; ++c) cur[c] = nxt[c];
    }
#pragma unroll
    for (int c = 0; c < kChunk; ++c) __builtin_nontemporal_store(cur[c], &dst[i + c * 256]);
    i += kStep;
  }
  for (; i < end; i += 256) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void k_fill(float4* dst, size_t n, float v) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
}

// ------------------------------------------------------------------ MFMA peak
// 4 independent 32x32 accumulators per wave hide the dependent-MFMA latency; operands stay in
// registers so the loop measures the matrix pipe alone.
__global__ __launch_bounds__(256) void k_mfma_peak(float* out, int iters, float seed) {
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(seed * (float)(threadIdx.x + j));
    b[j] = (__bf16)(seed * (float)(j + 1));
  }
  f32x16 c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, b, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int j = 0; j < 16; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
  if (s == 1234.5678f) out[0] = s;  // keeps the loop alive without a store per thread
  if (threadIdx.x == 0 && blockIdx.x == 0) out[1] = s;
}

// 16x16x32 form: ≈1.15× the FLOP/s of 32x32x16 under DVFS on random data (MI355X_MICROARCH
// "DVFS give-back" item 7); 4 independent accumulators per wave.
// dst tied to srcC in AGPRs. With the builtin, hipcc (ROCm 7.2) fails to coalesce the
// loop-carried 16x16x32 accumulators and emits 4-20 v_accvgpr moves per iteration (the
// 32x32x16 builtin is clean). Dependent MFMAs are ≥4 instructions apart here, so no hazard nops
// are needed inside the loop.
#define GM_MFMA16(c, x, y) \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(x), "v"(y))

__global__ __launch_bounds__(256) void k_mfma_peak16(float* out, int iters, float seed) {
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(seed * (float)(threadIdx.x * 7 + j));
    b[j] = (__bf16)(seed * (float)(j * 3 + 1 + blockIdx.x));
  }
  f32x4 c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  for (int i = 0; i < iters; ++i) {
    GM_MFMA16(c0, a, b);
    GM_MFMA16(c1, b, a);
    GM_MFMA16(c2, a, a);
    GM_MFMA16(c3, b, b);
  }
  float s = 0.f;
  for (int j = 0; j < 4; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
  if (s == 1234.5678f) out[0] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) out[1] = s;
}

// 8 independent 16x16x32 chains: twice the MFMAs in flight per wave of k_mfma_peak16.
__global__ __launch_bounds__(256) void k_mfma_peak16x8(float* out, int iters, float seed) {
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(seed * (float)(threadIdx.x * 7 + j));
    b[j] = (__bf16)(seed * (float)(j * 3 + 1 + blockIdx.x));
  }
  f32x4 c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0}, c4 = {0}, c5 = {0}, c6 = {0}, c7 = {0};
  for (int i = 0; i < iters; ++i) {
    GM_MFMA16(c0, a, b);
    GM_MFMA16(c1, b, a);
    GM_MFMA16(c2, a, a);
    GM_MFMA16(c3, b, b);
    GM_MFMA16(c4, a, b);
    GM_MFMA16(c5, b, a);
    GM_MFMA16(c6, a, a);
    GM_MFMA16(c7, b, b);
  }
  float s = 0.f;
  for (int j = 0; j < 4; ++j) s += c0[j] + c1[j] + c2[j] + c3[j] + c4[j] + c5[j] + c6[j] + c7[j];
  if (s == 1234.5678f) out[0] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) out[1] = s;
}

// ------------------------------------------------------------------ MFMA bf16 GEMM
// Block 256 threads = 4 waves in a 2x2 layout, block tile 64x64, K-tile 32 (two k16 MFMA steps).
// A tile staged row-major in LDS, B tile staged transposed (Bt[n][k]) so both fragments are one
// contiguous 16-byte LDS read per lane. Rows padded by 8 bf16 to stagger banks.
constexpr int BM = 64, BN = 64, BK = 32, PAD = 8;

__global__ __launch_bounds__(256) void k_gemm_bf16(const __bf16* __restrict__ A,
                                                   const __bf16* __restrict__ B,
                                                   float* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) __bf16 As[BM][BK + PAD];
  __shared__ __attribute__((aligned(16))) __bf16 Bt[BN][BK + PAD];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  const int bm = blockIdx.y, bn = blockIdx.x;

  // global→LDS assignment: each thread moves 8 bf16 (16 B) of A and of B per K-tile
  const int a_row = tid >> 2, a_col = (tid & 3) * 8;  // 64 rows × 4 chunks
  const int b_row = tid >> 3, b_col = (tid & 7) * 8;  // 32 rows × 8 chunks

  f32x16 acc = {0};
  for (int k0 = 0; k0 < K; k0 += BK) {
    const uint4 av =
        *reinterpret_cast<const uint4*>(A + (size_t)(bm * BM + a_row) * K + k0 + a_col);
    *reinterpret_cast<uint4*>(&As[a_row][a_col]) = av;
    const uint4 bv =
        *reinterpret_cast<const uint4*>(B + (size_t)(k0 + b_row) * N + bn * BN + b_col);
    const __bf16* bp = reinterpret_cast<const __bf16*>(&bv);
#pragma unroll
    for (int j = 0; j < 8; ++j) Bt[b_col + j][b_row] = bp[j];
    __syncthreads();
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(&As[wm * 32 + r][16 * s + 8 * h]);
      const bf16x8 bf = *reinterpret_cast<const bf16x8*>(&Bt[wn * 32 + r][16 * s + 8 * h]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc, 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    C[(size_t)(bm * BM + wm * 32 + row) * N + bn * BN + wn * 32 + r] = acc[i];
  }
}

// ------------------------------------------------------------------ scratch cache
struct Scratch {
  uint32_t* quick = nullptr;
  uint32_t* quick_host = nullptr;
};
std::mutex g_mu;
std::vector<Scratch> g_scratch;

Scratch* scratch(int dev) {
  std::lock_guard<std::mutex> lk(g_mu);
  if ((int)g_scratch.size() <= dev) g_scratch.resize(dev + 1);
  Scratch& s = g_scratch[dev];
  if (!s.quick) {
    if (hipMalloc(&s.quick, 128 * sizeof(uint32_t)) != hipSuccess) return nullptr;
    if (hipHostMalloc(&s.quick_host, 128 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess)
      return nullptr;
  }
  return &s;
}

uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint32_t rounding = 0x7fff + ((u >> 16) & 1);  // round-to-nearest-even
  return (uint16_t)((u + rounding) >> 16);
}
float bf2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

}  // namespace

extern "C" {

int gm_probe_device_count(int* n) { return (int)hipGetDeviceCount(n); }

int gm_probe_props(int dev, gm_probe_props_t* out) {
  memset(out, 0, sizeof(*out));
  hipDeviceProp_t p;
  GM_CHECK(hipGetDeviceProperties(&p, dev));
  snprintf(out->name, sizeof(out->name), "%s", p.name);
  snprintf(out->gcn_arch, sizeof(out->gcn_arch), "%s", p.gcnArchName);
  GM_CHECK(hipDeviceGetPCIBusId(out->pci_bus_id, sizeof(out->pci_bus_id), dev));
  out->cu_count = p.multiProcessorCount;
  out->warp_size = p.warpSize;
  out->total_mem = p.totalGlobalMem;
  out->lds_per_block = p.sharedMemPerBlock;
  out->clock_khz = p.clockRate;
  out->mem_clock_khz = p.memoryClockRate;
  return 0;
}

int gm_probe_find_device(const char* bdf, int* dev) {
  *dev = -1;
  int n = 0;
  GM_CHECK(hipGetDeviceCount(&n));
  for (int i = 0; i < n; ++i) {
    char id[32] = {0};
    if (hipDeviceGetPCIBusId(id, sizeof(id), i) != hipSuccess) continue;
    if (strcasecmp(id, bdf) == 0) {
      *dev = i;
      return 0;
    }
  }
  return 0;
}

int gm_probe_quick(int dev, int* ok, double* elapsed_us) {
  *ok = 0;
  DeviceGuard g(dev);
  if (!g.ok) return (int)hipErrorInvalidDevice;
  Scratch* s = scratch(dev);
  if (!s) return (int)hipErrorOutOfMemory;
  const auto t0 = std::chrono::steady_clock::now();
  const uint32_t salt = 0x9e3779b9u ^ (uint32_t)dev;
  hipLaunchKernelGGL(k_quick, dim3(1), dim3(64), 0, 0, s->quick, salt);
  GM_CHECK(hipGetLastError());
  GM_CHECK(hipMemcpy(s->quick_host, s->quick, 66 * sizeof(uint32_t), hipMemcpyDeviceToHost));
  const auto t1 = std::chrono::steady_clock::now();
  uint32_t sum = 0;
  bool good = true;
  for (uint32_t l = 0; l < 64; ++l) {
    const uint32_t v = l * 2654435761u ^ salt;
    good &= s->quick_host[l] == v;
    sum += v;
  }
  good &= s->quick_host[64] == sum && s->quick_host[65] == 64;
  *ok = good ? 1 : 0;
  *elapsed_us = std::chrono::duration<double, std::micro>(t1 - t0).count();
  return 0;
}

int gm_probe_hbm_copy_variant(int dev, int variant, uint64_t bytes, int iters,
                              int blocks_per_cu, double* gbps) {
  *gbps = 0;
  DeviceGuard g(dev);
  if (!g.ok) return (int)hipErrorInvalidDevice;
  bytes &= ~(uint64_t)15;
  if (bytes == 0 || iters <= 0 || blocks_per_cu <= 0) return (int)hipErrorInvalidValue;
  hipDeviceProp_t p;
  GM_CHECK(hipGetDeviceProperties(&p, dev));
  float4 *src = nullptr, *dst = nullptr;
  GM_CHECK(hipMalloc(&src, bytes));
  hipError_t e = hipMalloc(&dst, bytes);
  if (e != hipSuccess) {
    (void)hipFree(src);
    return (int)e;
  }
  const size_t n = bytes / sizeof(float4);
  const int blocks = p.multiProcessorCount * blocks_per_cu;
  const size_t per_block = ((n + blocks - 1) / blocks + 1023) / 1024 * 1024;
  auto launch = [&]() {
    switch (variant) {
      case 0: hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, 0, src, dst, n); break;
      case 1:
        hipLaunchKernelGGL((k_copy_chunk<4, false>), dim3(blocks), dim3(256), 0, 0, src, dst,
                           n, per_block);
        break;
      case 3:
        hipLaunchKernelGGL((k_copy_chunk<8, true>), dim3(blocks), dim3(256), 0, 0, src, dst,
                           n, per_block);
        break;
      case 4:
        hipLaunchKernelGGL((k_copy_chunk<8, false>), dim3(blocks), dim3(256), 0, 0, src, dst,
                           n, per_block);
        break;
      case 5:
        hipLaunchKernelGGL((k_copy_pipe<4>), dim3(blocks), dim3(256), 0, 0, src, dst, n,
                           per_block);
        break;
      case 6:
        hipLaunchKernelGGL((k_copy_pipe<2>), dim3(blocks), dim3(256), 0, 0, src, dst, n,
                           per_block);
        break;
      default:
        hipLaunchKernelGGL((k_copy_chunk<4, true>), dim3(blocks), dim3(256), 0, 0, src, dst,
                           n, per_block);
    }
  };
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, 0, src, n, 1.0f);
  launch();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(b, 0);
  e = hipEventSynchronize(b);
  float ms = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
  if (e == hipSuccess && ms > 0) *gbps = 2.0 * (double)bytes * iters / (ms * 1e-3) / 1e9;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(src);
  (void)hipFree(dst);
  return (int)e;
}

int gm_probe_hbm_read(int dev, uint64_t bytes, int iters, int blocks_per_cu, double* gbps) {
  *gbps = 0;
  DeviceGuard g(dev);
  if (!g.ok) return (int)hipErrorInvalidDevice;
  bytes &= ~(uint64_t)15;
  if (bytes == 0 || iters <= 0 || blocks_per_cu <= 0) return (int)hipErrorInvalidValue;
  hipDeviceProp_t p;
  GM_CHECK(hipGetDeviceProperties(&p, dev));
  float4* src = nullptr;
  uint32_t* sink = nullptr;
  GM_CHECK(hipMalloc(&src, bytes));
  hipError_t e = hipMalloc(&sink, 1024 * sizeof(uint32_t));
  if (e != hipSuccess) {
    (void)hipFree(src);
    return (int)e;
  }
  const size_t n = bytes / sizeof(float4);
  const int blocks = p.multiProcessorCount * blocks_per_cu;
  const size_t per_block = ((n + blocks - 1) / blocks + 2047) / 2048 * 2048;
  auto launch = [&]() {
    hipLaunchKernelGGL((k_read_chunk<8>), dim3(blocks), dim3(256), 0, 0, src, sink, n, per_block);
  };
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, 0, src, n, 1.0f);
  launch();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(b, 0);
  e = hipEventSynchronize(b);
  float ms = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
  if (e == hipSuccess && ms > 0) *gbps = (double)bytes * iters / (ms * 1e-3) / 1e9;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(src);
  (void)hipFree(sink);
  return (int)e;
}

int gm_probe_mfma_peak_variant(int dev, int variant, int iters, int blocks_per_cu,
                               double* tflops) {
  *tflops = 0;
  DeviceGuard g(dev);
  if (!g.ok) return (int)hipErrorInvalidDevice;
  hipDeviceProp_t p;
  GM_CHECK(hipGetDeviceProperties(&p, dev));
  float* out = nullptr;
  GM_CHECK(hipMalloc(&out, 2 * sizeof(float)));
  const int blocks = p.multiProcessorCount * blocks_per_cu;
  auto launch = [&](int it) {
    if (variant == 1)
      hipLaunchKernelGGL(k_mfma_peak16, dim3(blocks), dim3(256), 0, 0, out, it, 1e-3f);
    else if (variant == 2)
      hipLaunchKernelGGL(k_mfma_peak16x8, dim3(blocks), dim3(256), 0, 0, out, it, 1e-3f);
    else
      hipLaunchKernelGGL(k_mfma_peak, dim3(blocks), dim3(256), 0, 0, out, it, 1e-3f);
  };
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch(iters);  // warm-up as long as the timed run: clocks ramp before timing (DVFS)
  (void)hipEventRecord(a, 0);
  launch(iters);
  (void)hipEventRecord(b, 0);
  hipError_t e = hipEventSynchronize(b);
  float ms = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
  const double per = variant ? 2.0 * 16 * 16 * 32 : 2.0 * 32 * 32 * 16;
  const double chains = variant == 2 ? 8.0 : 4.0;
  const double flops = per * chains * iters * (double)blocks * 4 /* waves */;
  if (e == hipSuccess && ms > 0) *tflops = flops / (ms * 1e-3) / 1e12;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(out);
  return (int)e;
}

// Default HBM stream = the measured-best variant on MI355X (profiles/history/r1_probe_sweep: chunked,
// nontemporal, 8 blocks/CU → 5.57-5.65 TB/s vs 5.0-5.5 TB/s grid-stride).
int gm_probe_hbm_copy(int dev, uint64_t bytes, int iters, double* gbps) {
  return gm_probe_hbm_copy_variant(dev, 2, bytes, iters, 8, gbps);
}

// Default MFMA peak = the measured-best form on MI355X (profiles/history/r1_gpu_b/probe_sweep.json):
// v_mfma_f32_16x16x32_bf16, 8 dst-tied chains per wave, 8 blocks/CU → 2.45 PF/s
// (≈98 % of the 2.5 PF/s dense bf16 peak) vs 2.0-2.16 PF/s for 32x32x16 × 4 chains.
int gm_probe_mfma_peak(int dev, int iters, double* tflops) {
  return gm_probe_mfma_peak_variant(dev, 2, iters, 8, tflops);
}

int gm_probe_gemm_bf16(const void* A, const void* B, float* C, int M, int N, int K,
                       void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gemm_bf16, dim3(N / BN, M / BM), dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)A, (const __bf16*)B, C, M, N, K);
  return (int)hipGetLastError();
}

int gm_probe_gemm_check(int dev, int M, int N, int K, double* max_abs_err, double* ref_scale) {
  *max_abs_err = -1;
  *ref_scale = 0;
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK) return (int)hipErrorInvalidValue;
  DeviceGuard g(dev);
  if (!g.ok) return (int)hipErrorInvalidDevice;
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  std::vector<uint16_t> ha((size_t)M * K), hb((size_t)K * N);
  std::vector<float> fa(ha.size()), fb(hb.size());
  for (size_t i = 0; i < ha.size(); ++i) {
    ha[i] = f2bf(U(rng));
    fa[i] = bf2f(ha[i]);
  }
  for (size_t i = 0; i < hb.size(); ++i) {
    hb[i] = f2bf(U(rng));
    fb[i] = bf2f(hb[i]);
  }
  void *da = nullptr, *db = nullptr;
  float* dc = nullptr;
  GM_CHECK(hipMalloc(&da, ha.size() * 2));
  GM_CHECK(hipMalloc(&db, hb.size() * 2));
  GM_CHECK(hipMalloc(&dc, (size_t)M * N * 4));
  GM_CHECK(hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
  GM_CHECK(hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
  int e = gm_probe_gemm_bf16(da, db, dc, M, N, K, nullptr);
  std::vector<float> hc((size_t)M * N);
  if (e == 0) e = (int)hipMemcpy(hc.data(), dc, hc.size() * 4, hipMemcpyDeviceToHost);
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dc);
  if (e != 0) return e;
  double maxerr = 0, scale = 0;
  std::vector<float> row(N);
  for (int i = 0; i < M; ++i) {
    std::fill(row.begin(), row.end(), 0.f);
    for (int k = 0; k < K; ++k) {
      const float a = fa[(size_t)i * K + k];
      const float* bp = &fb[(size_t)k * N];
      for (int j = 0; j < N; ++j) row[j] += a * bp[j];
    }
    for (int j = 0; j < N; ++j) {
      maxerr = std::max(maxerr, (double)std::fabs(row[j] - hc[(size_t)i * N + j]));
      scale = std::max(scale, (double)std::fabs(row[j]));
    }
  }
  *max_abs_err = maxerr;
  *ref_scale = scale;
  return 0;
}

int gm_probe_p2p(int dev_a, int dev_b, uint64_t bytes, int iters, int* can_access, double* gbps) {
  *can_access = 0;
  *gbps = 0;
  if (iters <= 0 || bytes == 0) return (int)hipErrorInvalidValue;
  GM_CHECK(hipDeviceCanAccessPeer(can_access, dev_a, dev_b));
  DeviceGuard g(dev_a);
  if (!g.ok) return (int)hipErrorInvalidDevice;
  if (*can_access) {
    hipError_t pe = hipDeviceEnablePeerAccess(dev_b, 0);
    if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) return (int)pe;
    (void)hipGetLastError();
  }
  void *src = nullptr, *dst = nullptr;
  GM_CHECK(hipMalloc(&src, bytes));
  {
    DeviceGuard gb(dev_b);
    if (!gb.ok) return (int)hipErrorInvalidDevice;
    GM_CHECK(hipMalloc(&dst, bytes));
  }
  hipStream_t st;
  GM_CHECK(hipStreamCreate(&st));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipError_t e = hipMemcpyPeerAsync(dst, dev_b, src, dev_a, bytes, st);  // warm
  (void)hipEventRecord(a, st);
  for (int i = 0; i < iters && e == hipSuccess; ++i)
    e = hipMemcpyPeerAsync(dst, dev_b, src, dev_a, bytes, st);
  (void)hipEventRecord(b, st);
  if (e == hipSuccess) e = hipEventSynchronize(b);
  float ms = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
  if (e == hipSuccess && ms > 0) *gbps = (double)bytes * iters / (ms * 1e-3) / 1e9;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipStreamDestroy(st);
  (void)hipFree(src);
  {
    DeviceGuard gb(dev_b);
    (void)hipFree(dst);
  }
  return (int)e;
}

const char* gm_probe_strerror(int err) { return hipGetErrorString((hipError_t)err); }

}  // extern "C"
