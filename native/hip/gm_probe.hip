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

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;

struct DeviceGuard {
  int prev = 0;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && hipSetDevice(dev) == hipSuccess) ok = true;
  }
  ~DeviceGuard() {
    if (ok) (void)hipSetDevice(prev);
  }
};

#define GM_CHECK(x)                        \
  do {                                     \
    hipError_t e__ = (x);                  \
    if (e__ != hipSuccess) return (int)e__; \
  } while (0)

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
typedef float f32x4 __attribute__((ext_vector_type(4)));
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

// ------------------------------------------------------------------ MFMA bf16 GEMM, 256² tile
// Throughput form of the burn-in GEMM: C[M,N] (bf16) = A[M,K] · Bt[N,K]ᵀ, both operands K-major
// (the layout global_load_lds can stage without a transpose). Design (cdna_hip_programming.md §5):
//   * 256×256 output tile, BK=64, 512 threads = 8 waves as 2(M)×4(N); each wave owns 128×64 as
//     8×4 v_mfma_f32_16x16x32_bf16 accumulators (128 VGPRs), ~1 block per CU;
//   * operands go HBM→LDS with global_load_lds_dwordx4 (no VGPR round trip), two LDS stages of
//     64 KiB, the next stage's DMA issued before the current stage's MFMAs;
//   * LDS image lane-linear (one 1 KiB wave instruction = 8 rows × 128 B); bank conflicts of the
//     16-row ds_read_b128 fragment reads are removed by an XOR swizzle of the 16-B chunk index
//     with (row>>1)&7, applied to the per-lane GLOBAL source address and to the LDS read address;
//   * blockIdx remapped bijectively so each XCD runs a contiguous range of tiles, grouped 8 tile
//     rows deep, so concurrently running blocks of one XCD share A/B panels in that XCD's L2.
namespace g256 {
constexpr int TM = 256, TN = 256, TK = 64, kThreads = 512, kGroupM = 8;
constexpr int kTileBytes = TM * TK * 2;       // 32 KiB: one operand, one stage
constexpr int kStageBytes = 2 * kTileBytes;   // A + Bt
constexpr int kLdsBytes = 2 * kStageBytes;    // two stages: 128 KiB of the 160 KiB LDS
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;
}  // namespace g256
constexpr int kGemmNtDefault = 5;  // profiles/r1_gemm: V5 +2.9 % over V1 at 4096³, +0.9 % at 8192³

// XCD-aware block → output tile: bijective for any grid size (the dispatcher deals block ids
// round-robin over the 8 XCDs, so ids ≡ x mod 8 share XCD x's L2 and get a contiguous range of
// tiles), then a GROUP_M-deep raster so co-resident tiles share A rows and B columns.
__device__ __forceinline__ void gemm_tile_of(int M, int N, int& tm, int& tn) {
  using namespace g256;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg >> 3, r8 = nwg & 7, xcd = orig & 7;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
  const int ntm = M / TM, ntn = N / TN;
  const int per_group = kGroupM * ntn;
  const int first_m = (wgid / per_group) * kGroupM;
  const int gsize = min(ntm - first_m, kGroupM);
  tm = first_m + (wgid % per_group) % gsize;
  tn = (wgid % per_group) / gsize;
}

// V = 0: per 32-deep k-step, 12 fragment reads → wait → 32 MFMAs.
// V = 1: all 24 fragment reads of the 64-deep K-tile issued up front, so the second k-step's
//        reads overlap the first step's MFMAs (+48 VGPRs).
// V = 3: V1's schedule on v_mfma_f32_32x32x16_bf16 (same 128×64 per wave: 4×2 32² blocks).
template <int V>
__global__ __launch_bounds__(512) void k_gemm_nt256(const __bf16* __restrict__ A,
                                                    const __bf16* __restrict__ Bt,
                                                    __bf16* __restrict__ C, int M, int N, int K) {
  using namespace g256;
  __shared__ __attribute__((aligned(1024))) char lds[kLdsBytes];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  int tm, tn;
  gemm_tile_of(M, N, tm, tn);

  // Staging: wave w moves 1 KiB chunks c = w + 8i (i = 0..3) of each operand's 256×64 tile.
  // Lane l writes LDS byte c*1024 + l*16 = row 8c + (l>>3), slot l&7, which holds logical
  // 16-B chunk (l&7) ^ ((row>>1)&7). (row>>1)&7 is the same for all i (rows differ by 64).
  const int srow = 8 * wave + (lane >> 3);
  const int schunk = (lane & 7) ^ ((srow >> 1) & 7);
  const __bf16* a_src = A + (size_t)(tm * TM + srow) * K + schunk * 8;
  const __bf16* b_src = Bt + (size_t)(tn * TN + srow) * K + schunk * 8;
  const size_t row64 = (size_t)64 * K;

  auto stage = [&](int buf, int k0) {
    char* base = lds + buf * kStageBytes + wave * 1024;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_global_load_lds((gbl_void*)(a_src + i * row64 + k0),
                                       (lds_void*)(base + i * 8192), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_void*)(b_src + i * row64 + k0),
                                       (lds_void*)(base + kTileBytes + i * 8192), 16, 0, 0);
    }
  };

  // Fragment reads: lane l reads row (l&15) of a 16-row block at logical chunk 4kk + (l>>4).
  const int frow = lane & 15;
  const int foff0 = frow * 128 + (((lane >> 4) ^ (frow >> 1)) << 4);  // kk = 0; kk = 1: ^ 64
  const int a_off = wm * 128 * 128 + foff0;
  const int b_off = kTileBytes + wn * 64 * 128 + foff0;

  f32x4 acc[V == 3 ? 1 : 8][4];
  f32x16 acc32[V == 3 ? 4 : 1][2];
  if constexpr (V == 3) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc32[i][j][r] = 0.f;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int r32 = lane & 31, h32 = lane >> 5, sw32 = (r32 >> 1) & 7;
  const int a32_off = wm * 128 * 128 + r32 * 128;
  const int b32_off = kTileBytes + wn * 64 * 128 + r32 * 128;

  const int nt = K / TK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) stage(cur ^ 1, (t + 1) * TK);
    const char* sb = lds + cur * kStageBytes;
    if constexpr (V == 0) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[8], bfr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(sb + ((b_off + j * 16 * 128) ^ (kk << 6)));
#pragma unroll
        for (int i = 0; i < 8; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(sb + ((a_off + i * 16 * 128) ^ (kk << 6)));
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    } else if constexpr (V == 3) {
      // 32x32x16 shape, same per-wave 128×64 tile: 4×2 blocks, 4 k16-steps per K-tile.
      // Lane l reads row (l&31) of a 32-row block at logical chunk 2s + (l>>5).
      bf16x8 af[4][4], bfr[4][2];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[st][j] = *reinterpret_cast<const bf16x8*>(sb + b32_off + j * 32 * 128 +
                                                        ((((st * 2 + h32) ^ sw32)) << 4));
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[st][i] = *reinterpret_cast<const bf16x8*>(sb + a32_off + i * 32 * 128 +
                                                       ((((st * 2 + h32) ^ sw32)) << 4));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[st][i], bfr[st][j],
                                                                  acc32[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    } else {
      bf16x8 af[2][8], bfr[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          bfr[kk][j] =
              *reinterpret_cast<const bf16x8*>(sb + ((b_off + j * 16 * 128) ^ (kk << 6)));
#pragma unroll
        for (int i = 0; i < 8; ++i)
          af[kk][i] =
              *reinterpret_cast<const bf16x8*>(sb + ((a_off + i * 16 * 128) ^ (kk << 6)));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j],
                                                                acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if constexpr (V == 3) {
    // C/D map of 32x32x16: col = l&31, row = (reg&3) + 8(reg>>2) + 4(l>>5).
    const int crow = tm * TM + wm * 128 + 4 * h32;
    const int ccol = tn * TN + wn * 64 + r32;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          C[(size_t)(crow + i * 32 + (r & 3) + 8 * (r >> 2)) * N + ccol + j * 32] =
              (__bf16)acc32[i][j][r];
    return;
  }
  // Epilogue: C/D map of 16x16x32: col = l&15, row = 4(l>>4) + reg.
  const int crow = tm * TM + wm * 128 + 4 * (lane >> 4);
  const int ccol = tn * TN + wn * 64 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(size_t)(crow + i * 16 + r) * N + ccol + j * 16] = (__bf16)acc[i][j][r];
}

// V2 — quadrant phases with half-tile staging (same LDS budget, deeper pipeline). Measured
// 7-8 % slower than V1 on MI355X (profiles/r1_gemm): kept as the tested counter-example.
// Each stage's A and B tiles are split into row halves (lo = rows 0-127, hi = 128-255) of 16 KiB,
// giving 8 half-tile slots in the 128 KiB. Wave (wm, wn) owns A rows {wm*64 + [0,64)} of both
// halves and B rows {wn*32 + [0,32)} of both, i.e. four 64×32 output quadrants. A K-tile runs
// as 4 phases, one quadrant each, in the order (Alo,Blo) (Alo,Bhi) (Ahi,Bhi) (Ahi,Blo). Operands
// are carried in registers between neighbouring phases, so each half-tile is read from LDS in
// exactly one phase.
// Half-tiles are loaded in consumption order L[m] (m = 4t + {Alo, Blo, Bhi, Ahi}) into slot m%8.
// Phase p issues L[p+6] and ends with a counted vmcnt that retires only what phase p+1 reads,
// then a raw s_barrier. So 4-5 half-tiles (2 glds each) stay in flight across every barrier,
// where V0/V1 drain to vmcnt(0) once per K-tile.
// WAR: L[m+8] overwrites L[m]'s slot. It is issued in phase m+2, and L[m] was last read in
// phase ≤ m, with a barrier between.
__device__ __forceinline__ void vm_wait_glds(int n) {  // n = glds allowed in flight (uniform)
  switch (n) {
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <int Q>
struct QPhase {
  static constexpr int value = Q;
};

__global__ __launch_bounds__(512) void k_gemm_nt256q(const __bf16* __restrict__ A,
                                                     const __bf16* __restrict__ Bt,
                                                     __bf16* __restrict__ C, int M, int N,
                                                     int K) {
  using namespace g256;
  constexpr int kHalf = 16384, kAhead = 6;
  __shared__ __attribute__((aligned(1024))) char lds[kLdsBytes];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int tm, tn;
  gemm_tile_of(M, N, tm, tn);

  // Half-tile staging: wave w moves 1 KiB chunks w and w+8 (rows 8c + (l>>3) of the half).
  const int srow = 8 * wave + (lane >> 3);
  const int schunk = (lane & 7) ^ ((srow >> 1) & 7);
  const __bf16* a_src = A + (size_t)(tm * TM + srow) * K + schunk * 8;
  const __bf16* b_src = Bt + (size_t)(tn * TN + srow) * K + schunk * 8;
  const size_t row64 = (size_t)64 * K, row128 = (size_t)128 * K;
  const int nt = K / TK, last = 4 * nt - 1;

  auto issue = [&](int m) {  // L[m]: kind m&3 = 0 Alo, 1 Blo, 2 Bhi, 3 Ahi; tile m>>2
    const int kind = m & 3;
    const __bf16* src = ((kind == 0 || kind == 3) ? a_src : b_src) +
                        (kind >= 2 ? row128 : (size_t)0) + (m >> 2) * TK;
    char* dst = lds + (m & 7) * kHalf + wave * 1024;
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)dst, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void*)(src + row64), (lds_void*)(dst + 8192), 16, 0,
                                     0);
  };

  const int frow = lane & 15;
  const int foff0 = frow * 128 + (((lane >> 4) ^ (frow >> 1)) << 4);
  const int a_off = wm * 64 * 128 + foff0;
  const int b_off = wn * 32 * 128 + foff0;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[x][y][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[2][4], fbl[2][2], fbh[2][2];

  auto read_a = [&](const char* base) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[kk][i] = *reinterpret_cast<const bf16x8*>(base + ((a_off + i * 2048) ^ (kk << 6)));
  };
  auto read_b = [&](const char* base, bf16x8 (&fb)[2][2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[kk][j] = *reinterpret_cast<const bf16x8*>(base + ((b_off + j * 2048) ^ (kk << 6)));
  };
  auto mma = [&](f32x4 (&c)[4][2], bf16x8 (&fb)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][i], fb[kk][j], c[i][j], 0, 0,
                                                            0);
    __builtin_amdgcn_s_setprio(0);
  };

  auto phase = [&](auto qc, int t) {
    constexpr int q = decltype(qc)::value;
    const int p = 4 * t + q;
    const char* slot = lds + ((4 * t) & 7) * kHalf;  // Alo of tile t; +1..3 halves follow
    if constexpr (q == 0) {
      read_b(slot + 1 * kHalf, fbl);
      read_a(slot + 0 * kHalf);
    } else if constexpr (q == 1) {
      read_b(slot + 2 * kHalf, fbh);
    } else if constexpr (q == 2) {
      read_a(slot + 3 * kHalf);
    }
    if (p + kAhead <= last) issue(p + kAhead);
    if constexpr (q == 0) mma(acc[0][0], fbl);
    if constexpr (q == 1) mma(acc[0][1], fbh);
    if constexpr (q == 2) mma(acc[1][1], fbh);
    if constexpr (q == 3) mma(acc[1][0], fbl);
    if (p < last) {
      // phase p+1 reads up to L[need]: Bhi(t) after q0, Ahi(t) after q1/q2, Blo(t+1) after q3
      constexpr int need_rel = q == 0 ? 2 : (q == 3 ? 5 : 3);
      const int issued = min(p + kAhead, last);
      vm_wait_glds(2 * (issued - (4 * t + need_rel)));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  };

  // Prologue: L[0..6] in flight; retire L[0], L[1] (Alo, Blo of tile 0).
  const int pre = min(kAhead, last);
  for (int m = 0; m <= pre; ++m) issue(m);
  vm_wait_glds(2 * (pre - 1));
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int t = 0; t < nt; ++t) {
    phase(QPhase<0>{}, t);
    phase(QPhase<1>{}, t);
    phase(QPhase<2>{}, t);
    phase(QPhase<3>{}, t);
  }

  const int crow = tm * TM + wm * 64 + 4 * (lane >> 4);
  const int ccol = tn * TN + wn * 32 + (lane & 15);
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            C[(size_t)(crow + x * 128 + i * 16 + r) * N + ccol + y * 128 + j * 16] =
                (__bf16)acc[x][y][i][j][r];
}

// V4 — measured 7-13 % slower than V1 on MI355X (profiles/r1_gemm).
// 4 waves (2×2), each 128×128 = 8×8 16x16x32 accumulators (256 fp32/lane: the MFMA
// destinations live in AGPRs, 1 wave per SIMD). A fragment read feeds 8 MFMAs instead of 4,
// so LDS read traffic per K-tile drops by a third against V1; latency hiding is then
// up to the single wave's own schedule: all 32 fragment reads of the K-tile are issued
// before its 128 MFMAs.
__global__ __launch_bounds__(256) void k_gemm_nt256w4(const __bf16* __restrict__ A,
                                                      const __bf16* __restrict__ Bt,
                                                      __bf16* __restrict__ C, int M, int N,
                                                      int K) {
  using namespace g256;
  __shared__ __attribute__((aligned(1024))) char lds[kLdsBytes];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int tm, tn;
  gemm_tile_of(M, N, tm, tn);

  // Staging: wave w moves chunks c = w + 4i (i = 0..7), rows 8c + (l>>3): rows differ by 32
  // between i, so (row>>1)&7 is again the same for all of a lane's chunks.
  const int srow = 8 * wave + (lane >> 3);
  const int schunk = (lane & 7) ^ ((srow >> 1) & 7);
  const __bf16* a_src = A + (size_t)(tm * TM + srow) * K + schunk * 8;
  const __bf16* b_src = Bt + (size_t)(tn * TN + srow) * K + schunk * 8;
  const size_t row32 = (size_t)32 * K;
  auto stage = [&](int buf, int k0) {
    char* base = lds + buf * kStageBytes + wave * 1024;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_global_load_lds((gbl_void*)(a_src + i * row32 + k0),
                                       (lds_void*)(base + i * 4096), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_void*)(b_src + i * row32 + k0),
                                       (lds_void*)(base + kTileBytes + i * 4096), 16, 0, 0);
    }
  };
  const int frow = lane & 15;
  const int foff0 = frow * 128 + (((lane >> 4) ^ (frow >> 1)) << 4);
  const int a_off = wm * 128 * 128 + foff0;
  const int b_off = kTileBytes + wn * 128 * 128 + foff0;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = K / TK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) stage(cur ^ 1, (t + 1) * TK);
    const char* sb = lds + cur * kStageBytes;
    bf16x8 af[2][8], bfr[2][8];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        bfr[kk][j] = *reinterpret_cast<const bf16x8*>(sb + ((b_off + j * 2048) ^ (kk << 6)));
#pragma unroll
      for (int i = 0; i < 8; ++i)
        af[kk][i] = *reinterpret_cast<const bf16x8*>(sb + ((a_off + i * 2048) ^ (kk << 6)));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  const int crow = tm * TM + wm * 128 + 4 * (lane >> 4);
  const int ccol = tn * TN + wn * 128 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(size_t)(crow + i * 16 + r) * N + ccol + j * 16] = (__bf16)acc[i][j][r];
}

// Buffer-resource LDS DMA (buffer_load_dwordx4 … lds): gfx9-family resource word 3 =
// 0x00020000 (raw, untyped), stride 0, num_records = size in bytes (range-checked).
typedef __attribute__((address_space(3))) void lds_any;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                           0x00020000);
}

// V5 — V1's geometry with a local-read prefetch across the barrier. The second k-step's MFMAs
// of tile t are deferred past the barrier, so they run while the first k-step fragments of
// tile t+1 are read. Every fragment-read batch then overlaps 32 MFMAs of the same wave, and
// register use stays at two fragment sets (like V1). The barrier sits mid-tile, so the next
// tile's DMA is issued right after it.
template <bool kBufDma>
__global__ __launch_bounds__(512) void k_gemm_nt256p(const __bf16* __restrict__ A,
                                                     const __bf16* __restrict__ Bt,
                                                     __bf16* __restrict__ C, int M, int N,
                                                     int K) {
  using namespace g256;
  __shared__ __attribute__((aligned(1024))) char lds[kLdsBytes];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int tm, tn;
  gemm_tile_of(M, N, tm, tn);
  const int srow = 8 * wave + (lane >> 3);
  const int schunk = (lane & 7) ^ ((srow >> 1) & 7);
  const __bf16* a_src = A + (size_t)(tm * TM + srow) * K + schunk * 8;
  const __bf16* b_src = Bt + (size_t)(tn * TN + srow) * K + schunk * 8;
  const size_t row64 = (size_t)64 * K;
  // kBufDma (V7): the same DMA as buffer_load … lds from SGPR resources plus one 32-bit
  // per-lane offset, instead of eight per-lane 64-bit source pointers.
  const __amdgpu_buffer_rsrc_t a_rsrc = make_rsrc(A + (size_t)tm * TM * K, (uint32_t)TM * K * 2);
  const __amdgpu_buffer_rsrc_t b_rsrc =
      make_rsrc(Bt + (size_t)tn * TN * K, (uint32_t)TN * K * 2);
  const int lane_off = (srow * K + schunk * 8) * 2;
  auto stage = [&](int buf, int k0) {
    char* base = lds + buf * kStageBytes + wave * 1024;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (kBufDma) {
        const int soff = __builtin_amdgcn_readfirstlane((i * 64 * K + k0) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_any*)(base + i * 8192), 16,
                                                 lane_off, soff, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, (lds_any*)(base + kTileBytes + i * 8192),
                                                 16, lane_off, soff, 0, 0);
      } else {
        __builtin_amdgcn_global_load_lds((gbl_void*)(a_src + i * row64 + k0),
                                         (lds_void*)(base + i * 8192), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gbl_void*)(b_src + i * row64 + k0),
                                         (lds_void*)(base + kTileBytes + i * 8192), 16, 0, 0);
      }
    }
  };
  const int frow = lane & 15;
  const int foff0 = frow * 128 + (((lane >> 4) ^ (frow >> 1)) << 4);
  const int a_off = wm * 128 * 128 + foff0;
  const int b_off = kTileBytes + wn * 64 * 128 + foff0;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a0[8], b0[4], a1[8], b1[4];
  auto read = [&](const char* sb, int kk, bf16x8 (&af)[8], bf16x8 (&bf)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bf[j] = *reinterpret_cast<const bf16x8*>(sb + ((b_off + j * 2048) ^ (kk << 6)));
#pragma unroll
    for (int i = 0; i < 8; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(sb + ((a_off + i * 2048) ^ (kk << 6)));
  };
  auto mma = [&](bf16x8 (&af)[8], bf16x8 (&bf)[4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nt = K / TK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // Waits go through __builtin_amdgcn_s_waitcnt (gfx9 simm16: vmcnt[3:0]|expcnt[6:4]|
  // lgkmcnt[11:8]|vmcnt[5:4]<<14), not inline asm, so the compiler's own wait insertion knows
  // the counters are clear and adds no lgkmcnt(0) in front of the MFMAs.
  constexpr int kWaitLgkm0 = 0xC07F, kWaitVm0Lgkm0 = 0x0070;
  // Tile t+1's DMA is issued right after the barrier that frees its buffer (mid-tile t-1), so
  // it has a whole tile of MFMAs (64 per wave) to land before the vmcnt(0) that retires it.
  if (nt > 1) stage(1, TK);
  read(lds, 0, a0, b0);
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const char* sb = lds + cur * kStageBytes;
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);  // a0/b0 (read behind the last 32 MFMAs) are in
    read(sb, 1, a1, b1);
    mma(a0, b0);
    __builtin_amdgcn_s_waitcnt(kWaitVm0Lgkm0);  // tile t+1 landed; our reads of `cur` done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < nt) stage(cur, (t + 2) * TK);   // every wave is past its reads of `cur`
    if (t + 1 < nt) read(lds + (cur ^ 1) * kStageBytes, 0, a0, b0);
    mma(a1, b1);
  }

  const int crow = tm * TM + wm * 128 + 4 * (lane >> 4);
  const int ccol = tn * TN + wn * 64 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(size_t)(crow + i * 16 + r) * N + ccol + j * 16] = (__bf16)acc[i][j][r];
}

// V6 — V4's geometry (4 waves × 128², AGPR accumulators) on V5's schedule.
// (V5:) V1's geometry with a local-read prefetch across the barrier. The second k-step's MFMAs
// of tile t are deferred past the barrier, so they run while the first k-step fragments of
// tile t+1 are read. Every fragment-read batch then overlaps 32 MFMAs of the same wave, and
// register use stays at two fragment sets (like V1). The barrier sits mid-tile, so the next
// tile's DMA is issued right after it.
__global__ __launch_bounds__(256) void k_gemm_nt256w4p(const __bf16* __restrict__ A,
                                                     const __bf16* __restrict__ Bt,
                                                     __bf16* __restrict__ C, int M, int N,
                                                     int K) {
  using namespace g256;
  __shared__ __attribute__((aligned(1024))) char lds[kLdsBytes];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int tm, tn;
  gemm_tile_of(M, N, tm, tn);
  const int srow = 8 * wave + (lane >> 3);
  const int schunk = (lane & 7) ^ ((srow >> 1) & 7);
  // buffer_load … lds: the block's A/B panels as buffer resources (SGPRs), one 32-bit per-lane
  // byte offset, the per-load row/k offset in soffset (SGPR). Two VGPRs of addressing instead
  // of sixteen 64-bit pointers (which spilled), and range-checked: an out-of-panel read
  // returns zeros instead of faulting.
  const __amdgpu_buffer_rsrc_t a_rsrc = make_rsrc(A + (size_t)tm * TM * K, (uint32_t)TM * K * 2);
  const __amdgpu_buffer_rsrc_t b_rsrc =
      make_rsrc(Bt + (size_t)tn * TN * K, (uint32_t)TN * K * 2);
  const int lane_off = (srow * K + schunk * 8) * 2;
  auto stage = [&](int buf, int k0) {
    char* base = lds + buf * kStageBytes + wave * 1024;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int soff = __builtin_amdgcn_readfirstlane((i * 32 * K + k0) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_any*)(base + i * 4096), 16, lane_off,
                                               soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, (lds_any*)(base + kTileBytes + i * 4096),
                                               16, lane_off, soff, 0, 0);
    }
  };
  const int frow = lane & 15;
  const int foff0 = frow * 128 + (((lane >> 4) ^ (frow >> 1)) << 4);
  const int a_off = wm * 128 * 128 + foff0;
  const int b_off = kTileBytes + wn * 128 * 128 + foff0;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  auto read = [&](const char* sb, int kk, bf16x8 (&af)[8], bf16x8 (&bf)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      bf[j] = *reinterpret_cast<const bf16x8*>(sb + ((b_off + j * 2048) ^ (kk << 6)));
#pragma unroll
    for (int i = 0; i < 8; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(sb + ((a_off + i * 2048) ^ (kk << 6)));
  };
  auto mma = [&](bf16x8 (&af)[8], bf16x8 (&bf)[8]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nt = K / TK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // Waits go through __builtin_amdgcn_s_waitcnt (gfx9 simm16: vmcnt[3:0]|expcnt[6:4]|
  // lgkmcnt[11:8]|vmcnt[5:4]<<14), not inline asm, so the compiler's own wait insertion knows
  // the counters are clear and adds no lgkmcnt(0) in front of the MFMAs.
  constexpr int kWaitLgkm0 = 0xC07F, kWaitVm0Lgkm0 = 0x0070;
  // Tile t+1's DMA is issued right after the barrier that frees its buffer (mid-tile t-1), so
  // it has a whole tile of MFMAs (64 per wave) to land before the vmcnt(0) that retires it.
  if (nt > 1) stage(1, TK);
  read(lds, 0, a0, b0);
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const char* sb = lds + cur * kStageBytes;
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);  // a0/b0 (read behind the last 32 MFMAs) are in
    read(sb, 1, a1, b1);
    mma(a0, b0);
    __builtin_amdgcn_s_waitcnt(kWaitVm0Lgkm0);  // tile t+1 landed; our reads of `cur` done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < nt) stage(cur, (t + 2) * TK);   // every wave is past its reads of `cur`
    if (t + 1 < nt) read(lds + (cur ^ 1) * kStageBytes, 0, a0, b0);
    mma(a1, b1);
  }

  const int crow = tm * TM + wm * 128 + 4 * (lane >> 4);
  const int ccol = tn * TN + wn * 128 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(size_t)(crow + i * 16 + r) * N + ccol + j * 16] = (__bf16)acc[i][j][r];
}

// Deterministic uniform [-1, 1) bf16 fill (random operands: zero-filled ones overstate a GEMM).
__global__ __launch_bounds__(256) void k_fill_bf16(__bf16* dst, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    dst[i] = (__bf16)((float)(h >> 8) * (2.0f / 16777216.0f) - 1.0f);
  }
}

// Owning device buffer / event pair for the host entry points (freed on every return path).
struct DevBuf {
  void* p = nullptr;
  hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes); }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};
struct Events {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipError_t create() {
    hipError_t e = hipEventCreate(&e0);
    return e != hipSuccess ? e : hipEventCreate(&e1);
  }
  ~Events() {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  }
};

// Number of 16-B words that differ between a and b: one ballot + popcount per wave, one
// atomic per wave.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_count_diff(const u32x4* __restrict__ a,
                                                    const u32x4* __restrict__ b, size_t n,
                                                    unsigned long long* count) {
  unsigned long long local = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 x = __builtin_nontemporal_load(&a[i]), y = __builtin_nontemporal_load(&b[i]);
    local += (x.x != y.x) | (x.y != y.y) | (x.z != y.z) | (x.w != y.w);
  }
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, kWave);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(count, local);
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

// Default HBM stream = the measured-best variant on MI355X (profiles/r1_probe_sweep: chunked,
// nontemporal, 8 blocks/CU → 5.57-5.65 TB/s vs 5.0-5.5 TB/s grid-stride).
int gm_probe_hbm_copy(int dev, uint64_t bytes, int iters, double* gbps) {
  return gm_probe_hbm_copy_variant(dev, 2, bytes, iters, 8, gbps);
}

// Default MFMA peak = the measured-best form on MI355X (profiles/r1_gpu_b/probe_sweep.json):
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

int gm_probe_gemm_nt_variant(int variant, const void* A, const void* Bt, void* C, int M, int N,
                             int K, void* stream) {
  using namespace g256;
  if (M <= 0 || N <= 0 || K <= 0 || M % TM || N % TN || K % TK) return (int)hipErrorInvalidValue;
  const dim3 grid((M / TM) * (N / TN)), block(kThreads);
  switch (variant) {
    case 0:
      hipLaunchKernelGGL(k_gemm_nt256<0>, grid, block, 0, (hipStream_t)stream,
                         (const __bf16*)A, (const __bf16*)Bt, (__bf16*)C, M, N, K);
      break;
    case 1:
      hipLaunchKernelGGL(k_gemm_nt256<1>, grid, block, 0, (hipStream_t)stream,
                         (const __bf16*)A, (const __bf16*)Bt, (__bf16*)C, M, N, K);
      break;
    case 3:
      hipLaunchKernelGGL(k_gemm_nt256<3>, grid, block, 0, (hipStream_t)stream,
                         (const __bf16*)A, (const __bf16*)Bt, (__bf16*)C, M, N, K);
      break;
    case 5:
      hipLaunchKernelGGL(k_gemm_nt256p<false>, grid, block, 0, (hipStream_t)stream,
                         (const __bf16*)A, (const __bf16*)Bt, (__bf16*)C, M, N, K);
      break;
    case 7:
      hipLaunchKernelGGL(k_gemm_nt256p<true>, grid, block, 0, (hipStream_t)stream,
                         (const __bf16*)A, (const __bf16*)Bt, (__bf16*)C, M, N, K);
      break;
    case 6:
      hipLaunchKernelGGL(k_gemm_nt256w4p, grid, dim3(256), 0, (hipStream_t)stream,
                         (const __bf16*)A, (const __bf16*)Bt, (__bf16*)C, M, N, K);
      break;
    case 4:
      hipLaunchKernelGGL(k_gemm_nt256w4, grid, dim3(256), 0, (hipStream_t)stream,
                         (const __bf16*)A, (const __bf16*)Bt, (__bf16*)C, M, N, K);
      break;
    case 2:
      hipLaunchKernelGGL(k_gemm_nt256q, grid, block, 0, (hipStream_t)stream,
                         (const __bf16*)A, (const __bf16*)Bt, (__bf16*)C, M, N, K);
      break;
    default:
      return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

int gm_probe_gemm_nt(const void* A, const void* Bt, void* C, int M, int N, int K,
                     void* stream) {
  return gm_probe_gemm_nt_variant(kGemmNtDefault, A, Bt, C, M, N, K, stream);
}

int gm_probe_gemm_nt_tflops(int dev, int M, int N, int K, int iters, double* tflops) {
  using namespace g256;
  *tflops = 0;
  if (iters <= 0 || M <= 0 || N <= 0 || K <= 0 || M % TM || N % TN || K % TK)
    return (int)hipErrorInvalidValue;
  DeviceGuard g(dev);
  if (!g.ok) return (int)hipErrorInvalidDevice;
  DevBuf da, db, dc;
  GM_CHECK(da.alloc((size_t)M * K * 2));
  GM_CHECK(db.alloc((size_t)N * K * 2));
  GM_CHECK(dc.alloc((size_t)M * N * 2));
  hipLaunchKernelGGL(k_fill_bf16, dim3(4096), dim3(256), 0, 0, (__bf16*)da.p, (size_t)M * K,
                     0x1234u);
  hipLaunchKernelGGL(k_fill_bf16, dim3(4096), dim3(256), 0, 0, (__bf16*)db.p, (size_t)N * K,
                     0x9876u);
  Events ev;
  GM_CHECK(ev.create());
  int e = gm_probe_gemm_nt(da.p, db.p, dc.p, M, N, K, nullptr);  // warm-up
  if (!e) e = (int)hipEventRecord(ev.e0, nullptr);
  for (int i = 0; i < iters && !e; ++i) e = gm_probe_gemm_nt(da.p, db.p, dc.p, M, N, K, nullptr);
  if (!e) e = (int)hipEventRecord(ev.e1, nullptr);
  if (!e) e = (int)hipEventSynchronize(ev.e1);
  float ms = 0;
  if (!e) e = (int)hipEventElapsedTime(&ms, ev.e0, ev.e1);
  if (!e && ms > 0) *tflops = 2.0 * M * N * (double)K * iters / (ms * 1e-3) / 1e12;
  return e;
}

int gm_probe_burn_in(int dev, int n, double seconds, double* tflops, uint64_t* mismatches,
                     int* iters) {
  using namespace g256;
  *tflops = 0;
  *mismatches = 0;
  *iters = 0;
  if (n <= 0 || n % TM || seconds <= 0) return (int)hipErrorInvalidValue;
  DeviceGuard g(dev);
  if (!g.ok) return (int)hipErrorInvalidDevice;
  const size_t elems = (size_t)n * n;
  DevBuf da, db, dref, dc, dcount;
  GM_CHECK(da.alloc(elems * 2));
  GM_CHECK(db.alloc(elems * 2));
  GM_CHECK(dref.alloc(elems * 2));
  GM_CHECK(dc.alloc(elems * 2));
  GM_CHECK(dcount.alloc(sizeof(unsigned long long)));
  GM_CHECK(hipMemset(dcount.p, 0, sizeof(unsigned long long)));
  hipLaunchKernelGGL(k_fill_bf16, dim3(4096), dim3(256), 0, 0, (__bf16*)da.p, elems, 0x5151u);
  hipLaunchKernelGGL(k_fill_bf16, dim3(4096), dim3(256), 0, 0, (__bf16*)db.p, elems, 0xa3a3u);
  int e = gm_probe_gemm_nt(da.p, db.p, dref.p, n, n, n, nullptr);  // the reference result
  if (e) return e;
  Events ev;
  GM_CHECK(ev.create());
  GM_CHECK(hipEventRecord(ev.e0, nullptr));
  const auto t0 = std::chrono::steady_clock::now();
  const size_t vec = elems / 8;  // 16-B compares
  int done = 0;
  // Batches of 8 GEMMs, each result compared bit-for-bit with the first one: the kernel is
  // deterministic (fixed reduction order, no atomics), so any difference is a hardware fault.
  while (!e) {
    for (int i = 0; i < 8 && !e; ++i) {
      e = gm_probe_gemm_nt(da.p, db.p, dc.p, n, n, n, nullptr);
      if (!e) {
        hipLaunchKernelGGL(k_count_diff, dim3(2048), dim3(256), 0, 0,
                           (const u32x4*)dc.p, (const u32x4*)dref.p, vec,
                           (unsigned long long*)dcount.p);
        e = (int)hipGetLastError();
      }
      ++done;
    }
    if (!e) e = (int)hipDeviceSynchronize();
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el >= seconds) break;
  }
  if (!e) e = (int)hipEventRecord(ev.e1, nullptr);
  if (!e) e = (int)hipEventSynchronize(ev.e1);
  float ms = 0;
  if (!e) e = (int)hipEventElapsedTime(&ms, ev.e0, ev.e1);
  unsigned long long bad = 0;
  if (!e) e = (int)hipMemcpy(&bad, dcount.p, sizeof(bad), hipMemcpyDeviceToHost);
  if (e) return e;
  *iters = done;
  *mismatches = bad;
  // compare kernels are included in the wall time; they move 2 × n² × 2 B per GEMM (< 1 %)
  if (ms > 0) *tflops = 2.0 * n * (double)n * n * done / (ms * 1e-3) / 1e12;
  return 0;
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
