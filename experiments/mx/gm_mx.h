// gm_mx.h — block-scaled (MX) MFMA probes for gfx950, C ABI over HIP (experiment, not part of
// gpumounter-amd: nothing on the attach path or in the package uses them; see README.md).
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Block-scaled (MX) MFMA register-resident peak in the measured-best form per format
// (v_mfma_scale_f32_32x32x64_f8f6f4, 4 chains for fp8, 8 for fp4): fmt 0 = fp8 e4m3 (OCP),
// 4 = fp4 e2m1. *tflops dense. `sums` (may be NULL) receives one f32 per
// wave (blocks_per_cu × CUs × 4 of them, nsums ≥ that): deterministic, so two runs or two GPUs
// must agree bit for bit.
int gm_mx_peak(int dev, int fmt, int iters, int blocks_per_cu, float* sums, int nsums,
                     double* tflops);
// variant 0: 16x16x128 × 8 chains (gm_mx_peak), 1: 32x32x64 × 4, 2: 32x32x64 × 8.
int gm_mx_peak_variant(int dev, int fmt, int variant, int iters, int blocks_per_cu,
                             float* sums, int nsums, double* tflops);
// One MX-MFMA 16x16x128 on host-given per-lane register images: afrag/bfrag 64 × 32 bytes,
// sa/sb 64 E8M0 bytes (one per lane), c 64 × 4 f32 (lane-major). Numerics tests map lanes.
int gm_mx_tile(int dev, int fmt, const uint8_t* afrag, const uint8_t* bfrag,
                     const uint8_t* sa, const uint8_t* sb, float* c);
const char* gm_mx_strerror(int err);

#ifdef __cplusplus
}
#endif
