// gm_smi.cpp — hand-written dlopen binding to libamd_smi (no NVML header, no vendor shim).
//
// Reference parity: the NVML cgo binding dlopen()s libnvidia-ml.so.1 and resolves the versioned
// init through a C trampoline (reference: pkg/util/gpu/collector/nvml/nvml_dl.go:11-36) and then
// makes one cgo round trip per attribute (nvml.go:17-119). Here every symbol is resolved once at
// gm_smi_open(); the handles are cached for the lifetime of the worker (the reference re-inits NVML
// on every process query, nvidia.go:59-63 — SURVEY §2.6 defect 11), and Python receives one
// packed record per GPU.
//
// Only the amdsmi types come from the ROCm header; every entry point is called through a pointer
// obtained with dlsym, so this library links against nothing but libdl and works with the real
// libamd_smi.so or with the mock (native/src/amdsmi_mock.cpp) that exports the same symbols.
#include "gm_smi.h"

#include <amd_smi/amdsmi.h>
#include <dlfcn.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

namespace {

#define GM_SYM(name) decltype(&::name) name = nullptr

struct Api {
  void* dl = nullptr;
  std::string path;
  // required
  GM_SYM(amdsmi_init);
  GM_SYM(amdsmi_shut_down);
  GM_SYM(amdsmi_get_socket_handles);
  GM_SYM(amdsmi_get_processor_handles);
  // optional (feature-probed; absent → field left at its "unknown" value)
  GM_SYM(amdsmi_get_processor_type);
  GM_SYM(amdsmi_get_gpu_device_uuid);
  GM_SYM(amdsmi_get_gpu_device_bdf);
  GM_SYM(amdsmi_get_gpu_enumeration_info);
  GM_SYM(amdsmi_get_gpu_kfd_info);
  GM_SYM(amdsmi_get_xgmi_info);
  GM_SYM(amdsmi_topo_get_numa_node_number);
  GM_SYM(amdsmi_topo_get_link_type);
  GM_SYM(amdsmi_topo_get_link_weight);
  GM_SYM(amdsmi_get_gpu_process_list);
  GM_SYM(amdsmi_status_code_to_string);
  GM_SYM(amdsmi_get_gpu_asic_info);
  GM_SYM(amdsmi_get_gpu_vram_info);
  GM_SYM(amdsmi_get_gpu_compute_partition);
  GM_SYM(amdsmi_get_gpu_memory_partition);
  GM_SYM(amdsmi_get_gpu_total_ecc_count);
};

Api g_api;
std::vector<amdsmi_processor_handle> g_gpus;
std::mutex g_mu;  // amdsmi is documented thread-safe; the cache and open/close are not.
bool g_open = false;

template <typename F>
void resolve(void* dl, F& fn, const char* name) {
  fn = reinterpret_cast<F>(dlsym(dl, name));
}

void copy_str(char* dst, size_t cap, const char* src) {
  if (!src) {
    dst[0] = 0;
    return;
  }
  snprintf(dst, cap, "%s", src);
}

int enumerate_locked() {
  g_gpus.clear();
  uint32_t nsock = 0;
  amdsmi_status_t st = g_api.amdsmi_get_socket_handles(&nsock, nullptr);
  if (st != AMDSMI_STATUS_SUCCESS) return st;
  std::vector<amdsmi_socket_handle> socks(nsock);
  st = g_api.amdsmi_get_socket_handles(&nsock, socks.data());
  if (st != AMDSMI_STATUS_SUCCESS) return st;
  for (uint32_t s = 0; s < nsock; ++s) {
    uint32_t np = 0;
    st = g_api.amdsmi_get_processor_handles(socks[s], &np, nullptr);
    if (st != AMDSMI_STATUS_SUCCESS) return st;
    std::vector<amdsmi_processor_handle> ph(np);
    st = g_api.amdsmi_get_processor_handles(socks[s], &np, ph.data());
    if (st != AMDSMI_STATUS_SUCCESS) return st;
    for (uint32_t p = 0; p < np; ++p) {
      if (g_api.amdsmi_get_processor_type) {
        processor_type_t t = AMDSMI_PROCESSOR_TYPE_UNKNOWN;
        if (g_api.amdsmi_get_processor_type(ph[p], &t) == AMDSMI_STATUS_SUCCESS &&
            t != AMDSMI_PROCESSOR_TYPE_AMD_GPU)
          continue;
      }
      g_gpus.push_back(ph[p]);
    }
  }
  return AMDSMI_STATUS_SUCCESS;
}

uint64_t pack_bdf(const amdsmi_bdf_t& b) {
  return (uint64_t(b.domain_number) << 32) | (uint64_t(b.bus_number) << 8) |
         (uint64_t(b.device_number) << 3) | uint64_t(b.function_number);
}

int fill_info(uint32_t index, gm_gpu_info_t* out) {
  memset(out, 0, sizeof(*out));
  amdsmi_processor_handle h = g_gpus[index];
  out->index = index;
  out->render_minor = 0xFFFFFFFFu;
  out->card_minor = 0xFFFFFFFFu;
  out->hsa_id = 0xFFFFFFFFu;
  out->hip_id = 0xFFFFFFFFu;
  out->kfd_node_id = 0xFFFFFFFFu;
  out->kfd_gpu_id = ~0ull;
  out->numa_node = -1;

  if (g_api.amdsmi_get_gpu_device_uuid) {
    unsigned int len = sizeof(out->uuid);
    if (g_api.amdsmi_get_gpu_device_uuid(h, &len, out->uuid) != AMDSMI_STATUS_SUCCESS)
      out->uuid[0] = 0;
    out->uuid[sizeof(out->uuid) - 1] = 0;
  }
  if (g_api.amdsmi_get_gpu_device_bdf) {
    amdsmi_bdf_t b;
    memset(&b, 0, sizeof(b));
    if (g_api.amdsmi_get_gpu_device_bdf(h, &b) == AMDSMI_STATUS_SUCCESS) {
      out->bdf_id = pack_bdf(b);
      snprintf(out->bdf, sizeof(out->bdf), "%04llx:%02x:%02x.%x",
               (unsigned long long)b.domain_number, (unsigned)b.bus_number,
               (unsigned)b.device_number, (unsigned)b.function_number);
    }
  }
  if (g_api.amdsmi_get_gpu_enumeration_info) {
    amdsmi_enumeration_info_t e;
    memset(&e, 0, sizeof(e));
    if (g_api.amdsmi_get_gpu_enumeration_info(h, &e) == AMDSMI_STATUS_SUCCESS) {
      out->render_minor = e.drm_render;
      out->card_minor = e.drm_card;
      out->hsa_id = e.hsa_id;
      out->hip_id = e.hip_id;
    }
  }
  if (g_api.amdsmi_get_gpu_kfd_info) {
    amdsmi_kfd_info_t k;
    memset(&k, 0, sizeof(k));
    if (g_api.amdsmi_get_gpu_kfd_info(h, &k) == AMDSMI_STATUS_SUCCESS) {
      out->kfd_gpu_id = k.kfd_id;
      out->kfd_node_id = k.node_id;
      out->partition_id = k.current_partition_id == 0xFFFFFFFFu ? 0 : k.current_partition_id;
    }
  }
  if (g_api.amdsmi_get_xgmi_info) {
    amdsmi_xgmi_info_t x;
    memset(&x, 0, sizeof(x));
    if (g_api.amdsmi_get_xgmi_info(h, &x) == AMDSMI_STATUS_SUCCESS) {
      out->xgmi_lanes = x.xgmi_lanes;
      out->xgmi_hive_id = x.xgmi_hive_id;
      out->xgmi_node_id = x.xgmi_node_id;
    }
  }
  if (g_api.amdsmi_topo_get_numa_node_number) {
    uint32_t numa = 0;
    if (g_api.amdsmi_topo_get_numa_node_number(h, &numa) == AMDSMI_STATUS_SUCCESS)
      out->numa_node = (int32_t)numa;
  }
  if (g_api.amdsmi_get_gpu_asic_info) {
    amdsmi_asic_info_t a;
    memset(&a, 0, sizeof(a));
    if (g_api.amdsmi_get_gpu_asic_info(h, &a) == AMDSMI_STATUS_SUCCESS) {
      copy_str(out->market_name, sizeof(out->market_name), a.market_name);
      out->device_id = a.device_id;
      out->num_cu = a.num_of_compute_units == 0xFFFFFFFFu ? 0 : a.num_of_compute_units;
      if (a.target_graphics_version != ~0ull && a.target_graphics_version != 0)
        snprintf(out->gfx_target, sizeof(out->gfx_target), "gfx%llx",
                 (unsigned long long)a.target_graphics_version);
    }
  }
  if (g_api.amdsmi_get_gpu_vram_info) {
    amdsmi_vram_info_t v;
    memset(&v, 0, sizeof(v));
    if (g_api.amdsmi_get_gpu_vram_info(h, &v) == AMDSMI_STATUS_SUCCESS)
      out->vram_bytes = v.vram_size * 1024ull * 1024ull;  // reported in MB
  }
  if (g_api.amdsmi_get_gpu_compute_partition) {
    char buf[32] = {0};
    if (g_api.amdsmi_get_gpu_compute_partition(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS)
      copy_str(out->compute_partition, sizeof(out->compute_partition), buf);
  }
  if (g_api.amdsmi_get_gpu_memory_partition) {
    char buf[32] = {0};
    if (g_api.amdsmi_get_gpu_memory_partition(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS)
      copy_str(out->memory_partition, sizeof(out->memory_partition), buf);
  }
  return GM_SMI_OK;
}

int link_locked(uint32_t src, uint32_t dst, gm_link_info_t* out) {
  memset(out, 0, sizeof(*out));
  out->link_type = AMDSMI_LINK_TYPE_UNKNOWN;
  if (src == dst) {
    out->link_type = AMDSMI_LINK_TYPE_INTERNAL;
    return GM_SMI_OK;
  }
  if (g_api.amdsmi_topo_get_link_type) {
    uint64_t hops = 0;
    amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
    if (g_api.amdsmi_topo_get_link_type(g_gpus[src], g_gpus[dst], &hops, &t) ==
        AMDSMI_STATUS_SUCCESS) {
      out->link_type = (uint32_t)t;
      out->hops = hops;
    }
  }
  if (g_api.amdsmi_topo_get_link_weight) {
    uint64_t w = 0;
    if (g_api.amdsmi_topo_get_link_weight(g_gpus[src], g_gpus[dst], &w) == AMDSMI_STATUS_SUCCESS)
      out->weight = w;
  }
  return GM_SMI_OK;
}

}  // namespace

extern "C" {

int gm_smi_abi_version(void) { return GM_SMI_ABI_VERSION; }

int gm_smi_open(const char* lib_path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_open) return GM_SMI_OK;
  const char* candidates[] = {lib_path, "libamd_smi.so", "libamd_smi.so.26",
                              "/opt/rocm/lib/libamd_smi.so"};
  void* dl = nullptr;
  for (const char* c : candidates) {
    if (!c || !*c) continue;
    dl = dlopen(c, RTLD_NOW | RTLD_LOCAL);
    if (dl) {
      g_api.path = c;
      break;
    }
    if (lib_path && c == lib_path) break;  // explicit path: do not silently fall back
  }
  if (!dl) return GM_SMI_ERR_DLOPEN;
  g_api.dl = dl;
  resolve(dl, g_api.amdsmi_init, "amdsmi_init");
  resolve(dl, g_api.amdsmi_shut_down, "amdsmi_shut_down");
  resolve(dl, g_api.amdsmi_get_socket_handles, "amdsmi_get_socket_handles");
  resolve(dl, g_api.amdsmi_get_processor_handles, "amdsmi_get_processor_handles");
  if (!g_api.amdsmi_init || !g_api.amdsmi_shut_down || !g_api.amdsmi_get_socket_handles ||
      !g_api.amdsmi_get_processor_handles) {
    dlclose(dl);
    g_api = Api();
    return GM_SMI_ERR_DLSYM;
  }
  resolve(dl, g_api.amdsmi_get_processor_type, "amdsmi_get_processor_type");
  resolve(dl, g_api.amdsmi_get_gpu_device_uuid, "amdsmi_get_gpu_device_uuid");
  resolve(dl, g_api.amdsmi_get_gpu_device_bdf, "amdsmi_get_gpu_device_bdf");
  resolve(dl, g_api.amdsmi_get_gpu_enumeration_info, "amdsmi_get_gpu_enumeration_info");
  resolve(dl, g_api.amdsmi_get_gpu_kfd_info, "amdsmi_get_gpu_kfd_info");
  resolve(dl, g_api.amdsmi_get_xgmi_info, "amdsmi_get_xgmi_info");
  resolve(dl, g_api.amdsmi_topo_get_numa_node_number, "amdsmi_topo_get_numa_node_number");
  resolve(dl, g_api.amdsmi_topo_get_link_type, "amdsmi_topo_get_link_type");
  resolve(dl, g_api.amdsmi_topo_get_link_weight, "amdsmi_topo_get_link_weight");
  resolve(dl, g_api.amdsmi_get_gpu_process_list, "amdsmi_get_gpu_process_list");
  resolve(dl, g_api.amdsmi_status_code_to_string, "amdsmi_status_code_to_string");
  resolve(dl, g_api.amdsmi_get_gpu_asic_info, "amdsmi_get_gpu_asic_info");
  resolve(dl, g_api.amdsmi_get_gpu_vram_info, "amdsmi_get_gpu_vram_info");
  resolve(dl, g_api.amdsmi_get_gpu_compute_partition, "amdsmi_get_gpu_compute_partition");
  resolve(dl, g_api.amdsmi_get_gpu_memory_partition, "amdsmi_get_gpu_memory_partition");
  resolve(dl, g_api.amdsmi_get_gpu_total_ecc_count, "amdsmi_get_gpu_total_ecc_count");

  amdsmi_status_t st = g_api.amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    dlclose(dl);
    g_api = Api();
    return (int)st;
  }
  int e = enumerate_locked();
  if (e != AMDSMI_STATUS_SUCCESS) {
    g_api.amdsmi_shut_down();
    dlclose(dl);
    g_api = Api();
    return e;
  }
  g_open = true;
  return GM_SMI_OK;
}

int gm_smi_close(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_open) return GM_SMI_OK;
  g_api.amdsmi_shut_down();
  dlclose(g_api.dl);
  g_api = Api();
  g_gpus.clear();
  g_open = false;
  return GM_SMI_OK;
}

int gm_smi_is_open(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_open ? 1 : 0;
}

const char* gm_smi_lib_path(void) { return g_api.path.c_str(); }

int gm_smi_count(uint32_t* n) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_open) return GM_SMI_ERR_NOT_OPEN;
  *n = (uint32_t)g_gpus.size();
  return GM_SMI_OK;
}

int gm_smi_gpu_info(uint32_t index, gm_gpu_info_t* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_open) return GM_SMI_ERR_NOT_OPEN;
  if (index >= g_gpus.size()) return GM_SMI_ERR_RANGE;
  return fill_info(index, out);
}

int gm_smi_all_gpu_info(gm_gpu_info_t* out, uint32_t cap, uint32_t* n) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_open) return GM_SMI_ERR_NOT_OPEN;
  *n = (uint32_t)g_gpus.size();
  for (uint32_t i = 0; i < g_gpus.size() && i < cap; ++i) fill_info(i, &out[i]);
  return g_gpus.size() > cap ? GM_SMI_MORE_DATA : GM_SMI_OK;
}

int gm_smi_link(uint32_t src, uint32_t dst, gm_link_info_t* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_open) return GM_SMI_ERR_NOT_OPEN;
  if (src >= g_gpus.size() || dst >= g_gpus.size()) return GM_SMI_ERR_RANGE;
  return link_locked(src, dst, out);
}

int gm_smi_link_matrix(gm_link_info_t* out, uint32_t cap) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_open) return GM_SMI_ERR_NOT_OPEN;
  const uint32_t n = (uint32_t)g_gpus.size();
  if ((uint64_t)n * n > cap) return GM_SMI_ERR_RANGE;
  for (uint32_t i = 0; i < n; ++i)
    for (uint32_t j = 0; j < n; ++j) link_locked(i, j, &out[i * n + j]);
  return GM_SMI_OK;
}

int gm_smi_process_list(uint32_t index, gm_proc_info_t* out, uint32_t cap, uint32_t* n) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_open) return GM_SMI_ERR_NOT_OPEN;
  if (index >= g_gpus.size()) return GM_SMI_ERR_RANGE;
  *n = 0;
  if (!g_api.amdsmi_get_gpu_process_list) return AMDSMI_STATUS_NOT_SUPPORTED;
  // amdsmi reports the true count through max_processes when the buffer is too small.
  uint32_t want = cap > 0 ? cap : 1;
  std::vector<amdsmi_proc_info_t> buf(want);
  uint32_t got = want;
  amdsmi_status_t st = g_api.amdsmi_get_gpu_process_list(g_gpus[index], &got, buf.data());
  if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES &&
      st != AMDSMI_STATUS_MORE_DATA)
    return (int)st;
  *n = got;
  const uint32_t fill = got < cap ? got : cap;
  for (uint32_t i = 0; i < fill; ++i) {
    memset(&out[i], 0, sizeof(out[i]));
    out[i].pid = buf[i].pid;
    out[i].cu_occupancy = buf[i].cu_occupancy;
    out[i].vram_bytes = buf[i].memory_usage.vram_mem;
    out[i].gtt_bytes = buf[i].memory_usage.gtt_mem;
    copy_str(out[i].name, sizeof(out[i].name), buf[i].name);
  }
  return got > cap ? GM_SMI_MORE_DATA : GM_SMI_OK;
}

int gm_smi_ecc(uint32_t index, uint64_t* correctable, uint64_t* uncorrectable,
               uint64_t* deferred) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_open) return GM_SMI_ERR_NOT_OPEN;
  if (index >= g_gpus.size()) return GM_SMI_ERR_RANGE;
  *correctable = *uncorrectable = *deferred = 0;
  if (!g_api.amdsmi_get_gpu_total_ecc_count) return AMDSMI_STATUS_NOT_SUPPORTED;
  amdsmi_error_count_t ec;
  memset(&ec, 0, sizeof(ec));
  amdsmi_status_t st = g_api.amdsmi_get_gpu_total_ecc_count(g_gpus[index], &ec);
  if (st != AMDSMI_STATUS_SUCCESS) return (int)st;
  *correctable = ec.correctable_count;
  *uncorrectable = ec.uncorrectable_count;
  *deferred = ec.deferred_count;
  return GM_SMI_OK;
}

const char* gm_smi_strerror(int status) {
  switch (status) {
    case GM_SMI_ERR_NOT_OPEN: return "gm_smi: library not opened";
    case GM_SMI_ERR_DLOPEN: return "gm_smi: dlopen(libamd_smi) failed";
    case GM_SMI_ERR_DLSYM: return "gm_smi: required amdsmi symbol missing";
    case GM_SMI_ERR_RANGE: return "gm_smi: index out of range";
    default: break;
  }
  if (g_api.amdsmi_status_code_to_string) {
    const char* s = nullptr;
    if (g_api.amdsmi_status_code_to_string((amdsmi_status_t)status, &s) ==
            AMDSMI_STATUS_SUCCESS &&
        s)
      return s;
  }
  // The library may be unloaded (failed open): fall back to the header's names.
  switch (status) {
    case AMDSMI_STATUS_INVAL: return "AMDSMI_STATUS_INVAL";
    case AMDSMI_STATUS_NOT_SUPPORTED: return "AMDSMI_STATUS_NOT_SUPPORTED";
    case AMDSMI_STATUS_FAIL_LOAD_MODULE: return "AMDSMI_STATUS_FAIL_LOAD_MODULE";
    case AMDSMI_STATUS_NO_PERM: return "AMDSMI_STATUS_NO_PERM";
    case AMDSMI_STATUS_INIT_ERROR: return "AMDSMI_STATUS_INIT_ERROR";
    case AMDSMI_STATUS_NOT_FOUND: return "AMDSMI_STATUS_NOT_FOUND";
    case AMDSMI_STATUS_NOT_INIT: return "AMDSMI_STATUS_NOT_INIT";
    case AMDSMI_STATUS_DRIVER_NOT_LOADED: return "AMDSMI_STATUS_DRIVER_NOT_LOADED";
    case AMDSMI_STATUS_FILE_ERROR: return "AMDSMI_STATUS_FILE_ERROR";
    default: return "amdsmi: unknown status";
  }
}

}  // extern "C"
