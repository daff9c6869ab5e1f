// gm_probe.h — post-attach device validation for MI355X (gfx950), C ABI over HIP.
//
// The reference has no post-mount check at all: success means "mknod returned 0"
// (reference: pkg/util/util.go:64-70). gpumounter-amd proves an attached GPU is actually usable
// from the tenant side by running real CDNA4 kernels on it (wave64 liveness, HBM3E stream,
// MFMA bf16 peak and numerics) and, for multi-GPU attaches, by timing xGMI peer copies.
// All functions return hipError_t values (0 = success).
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gm_probe_props {
  char name[128];
  char gcn_arch[64];
  char pci_bus_id[32];   // "0000:05:00.0"
  int32_t cu_count;
  int32_t warp_size;
  uint64_t total_mem;
  uint64_t lds_per_block;
  int32_t clock_khz;
  int32_t mem_clock_khz;
} gm_probe_props_t;

int gm_probe_device_count(int* n);
int gm_probe_props(int dev, gm_probe_props_t* out);
// HIP device index whose PCI bus id matches `bdf` (case-insensitive "dddd:bb:dd.f"), -1 if none.
int gm_probe_find_device(const char* bdf, int* dev);
// Liveness: launches one wave64 kernel that writes lane ids and a checksum; verifies on host.
// *elapsed_us = launch→readback wall time.
int gm_probe_quick(int dev, int* ok, double* elapsed_us);
// HBM3E stream: float4 copy of `bytes` for `iters`; *gbps = (read+write) bytes / time.
int gm_probe_hbm_copy(int dev, uint64_t bytes, int iters, double* gbps);
// Read-only HBM stream over `bytes` (8 nontemporal 16-B loads in flight per lane); GB/s read.
int gm_probe_hbm_read(int dev, uint64_t bytes, int iters, int blocks_per_cu, double* gbps);
// Tuning variants: 0 grid-stride, 1 chunked 4×16B/lane, 2 chunked 4 + nontemporal,
// 3 chunked 8 + nontemporal, 4 chunked 8, 5/6 software-pipelined 4/2 (next loads before
// current stores), nontemporal.
int gm_probe_hbm_copy_variant(int dev, int variant, uint64_t bytes, int iters,
                              int blocks_per_cu, double* gbps);
// variant 0: v_mfma_f32_32x32x16_bf16 × 4 chains, 1: v_mfma_f32_16x16x32_bf16 × 4 chains,
// 2: 16x16x32 × 8 chains.
int gm_probe_mfma_peak_variant(int dev, int variant, int iters, int blocks_per_cu,
                               double* tflops);
// MFMA bf16 register-resident peak (best measured form: 16x16x32 × 8 chains); *tflops dense.
int gm_probe_mfma_peak(int dev, int iters, double* tflops);
// C[M,N] (fp32) = A[M,K] (bf16, row-major) · B[K,N] (bf16, row-major) on MFMA.
// Requires M%64 == 0, N%64 == 0, K%32 == 0 (checked). Device pointers; stream may be NULL.
int gm_probe_gemm_bf16(const void* A, const void* B, float* C, int M, int N, int K, void* stream);
// C[M,N] (bf16) = A[M,K] · Bt[N,K]ᵀ (bf16, both K-major), fp32 accumulate: the 256²-tile
// global_load_lds throughput GEMM. Requires M%256 == 0, N%256 == 0, K%64 == 0 (checked).
int gm_probe_gemm_nt(const void* A, const void* Bt, void* C, int M, int N, int K, void* stream);
// Schedule variants of the same kernel (A/B measurements; bench/gemm_sweep.py).
int gm_probe_gemm_nt_variant(int variant, const void* A, const void* Bt, void* C, int M, int N,
                             int K, void* stream);
// Dense bf16 TF/s of gm_probe_gemm_nt on uniform [-1,1) operands, `iters` back-to-back launches.
int gm_probe_gemm_nt_tflops(int dev, int M, int N, int K, int iters, double* tflops);
// Burn-in: back-to-back n³ GEMMs (gm_probe_gemm_nt) for `seconds` on uniform [-1,1) operands;
// every result is compared bit-for-bit with the first (the kernel is deterministic), so
// *mismatches > 0 (16-B words that differ, summed over iterations) means silent data
// corruption. *tflops includes the compare kernels. n % 256 == 0.
int gm_probe_burn_in(int dev, int n, double seconds, double* tflops, uint64_t* mismatches,
                     int* iters);
// Self-contained numerics check of gm_probe_gemm_bf16 against a host fp32 reference.
int gm_probe_gemm_check(int dev, int M, int N, int K, double* max_abs_err, double* ref_scale);
// xGMI / PCIe peer copy a→b; *can_access from hipDeviceCanAccessPeer.
int gm_probe_p2p(int dev_a, int dev_b, uint64_t bytes, int iters, int* can_access, double* gbps);
const char* gm_probe_strerror(int err);

#ifdef __cplusplus
}
#endif
