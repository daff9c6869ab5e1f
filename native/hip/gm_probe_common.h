// gm_probe_common.h — shared by the gfx950 probe translation units (gm_probe.hip, gm_gemm.hip):
// vector types, device selection guard, error macro, owning device buffer / event pair.
// Everything is in an anonymous namespace: each translation unit gets its own copy.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

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
typedef float f32x4 __attribute__((ext_vector_type(4)));

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

}  // namespace
