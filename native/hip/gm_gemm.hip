// gm_gemm.hip — the 256²-tile bf16 burn-in GEMM (schedule V5, with V1 as its reference point)
// and the bit-exact burn-in loop. Part of libgm_probe.so (built with gm_probe.hip).
// Measurements: profiles/history/r1_gemm/ (round 1 also timed eight other schedules, V0 V2-V4 V6-V9;
// none beat V5, and they were removed: the GEMM is a burn-in load, not a product kernel).
#include <chrono>

#include "gm_probe.h"
#include "gm_probe_common.h"

namespace {

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
constexpr int kGemmNtDefault = 5;  // profiles/history/r1_gemm: V5 +2.9 % over V1 at 4096³, +0.9 % at 8192³

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

// V1 — the plain schedule, kept as the reference point for V5: all 24 fragment reads of the
// 64-deep K-tile are issued up front, so the second k-step's reads overlap the first step's
// MFMAs, then one vmcnt(0) + barrier per K-tile.
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

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = K / TK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) stage(cur ^ 1, (t + 1) * TK);
    const char* sb = lds + cur * kStageBytes;
    {
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

// V5 — V1's geometry with a local-read prefetch across the barrier. The second k-step's MFMAs
// of tile t are deferred past the barrier, so they run while the first k-step fragments of
// tile t+1 are read. Every fragment-read batch then overlaps 32 MFMAs of the same wave, and
// register use stays at two fragment sets (like V1). The barrier sits mid-tile, so the next
// tile's DMA is issued right after it.
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

}  // namespace

extern "C" {

int gm_probe_gemm_nt_variant(int variant, const void* A, const void* Bt, void* C, int M, int N,
                             int K, void* stream) {
  using namespace g256;
  if (M <= 0 || N <= 0 || K <= 0 || M % TM || N % TN || K % TK) return (int)hipErrorInvalidValue;
  const dim3 grid((M / TM) * (N / TN)), block(kThreads);
  switch (variant) {
    case 1:
      hipLaunchKernelGGL(k_gemm_nt256, grid, block, 0, (hipStream_t)stream,
                         (const __bf16*)A, (const __bf16*)Bt, (__bf16*)C, M, N, K);
      break;
    case 5:
      hipLaunchKernelGGL(k_gemm_nt256p, grid, block, 0, (hipStream_t)stream,
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

}  // extern "C"
