// gm_smi.h — flat C ABI of the gpumounter-amd device-inventory shim over libamd_smi.
//
// Replaces the reference's CGo NVML binding (reference: pkg/util/gpu/collector/nvml/
// nvml_dl.go:11-53, bindings.go:19-61, nvml.go:17-119). Instead of a vendored vendor header and
// one cgo call per attribute, the shim dlopen()s libamd_smi once, walks every GPU once, and hands
// Python one fixed-layout record per GPU (render/card minors, KFD ids, xGMI hive, NUMA, BDF …)
// plus an N×N link matrix. The record layout is mirrored by ctypes in gpumounter_amd/_native.py;
// change both together.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GM_SMI_ABI_VERSION 1

typedef struct gm_gpu_info {
  uint32_t index;            // enumeration order of the shim (socket-major)
  uint32_t render_minor;     // /dev/dri/renderD<render_minor> (0xFFFFFFFF if unknown)
  uint32_t card_minor;       // /dev/dri/card<card_minor>      (0xFFFFFFFF if unknown)
  uint32_t hsa_id;
  uint32_t hip_id;
  uint32_t kfd_node_id;
  uint32_t partition_id;     // current compute partition id (0 on SPX)
  uint32_t xgmi_lanes;
  int32_t numa_node;         // -1 if unknown
  uint32_t num_cu;
  uint64_t bdf_id;           // packed BDF (domain<<32 | bus<<8 | dev<<3 | fn)
  uint64_t kfd_gpu_id;
  uint64_t xgmi_hive_id;     // 0 if not in a hive
  uint64_t xgmi_node_id;
  uint64_t vram_bytes;
  uint64_t device_id;        // PCI device id
  char uuid[64];
  char bdf[32];              // "0000:05:00.0"
  char market_name[128];
  char gfx_target[32];       // "gfx950"
  char compute_partition[16];// "SPX"/"CPX"/...
  char memory_partition[16]; // "NPS1"/...
} gm_gpu_info_t;

typedef struct gm_proc_info {
  uint32_t pid;
  uint32_t cu_occupancy;
  uint64_t vram_bytes;
  uint64_t gtt_bytes;
  char name[64];
} gm_proc_info_t;

typedef struct gm_link_info {
  uint32_t link_type;        // amdsmi_link_type_t: 0 internal, 1 PCIe, 2 xGMI, 3 n/a, 4 unknown
  uint32_t reserved;
  uint64_t hops;
  uint64_t weight;
} gm_link_info_t;

// Loads `lib_path` (NULL → "libamd_smi.so", then /opt/rocm/lib/libamd_smi.so) and calls
// amdsmi_init(AMDSMI_INIT_AMD_GPUS). Enumerates and caches processor handles.
// Returns 0 or an amdsmi status code / negative errno-style shim code.
int gm_smi_open(const char* lib_path);
int gm_smi_close(void);
int gm_smi_is_open(void);
int gm_smi_abi_version(void);
// Path of the library actually loaded (for diagnostics).
const char* gm_smi_lib_path(void);
int gm_smi_count(uint32_t* n);
int gm_smi_gpu_info(uint32_t index, gm_gpu_info_t* out);
// Bulk fetch: fills out[0..min(cap,count)); *n = count.
int gm_smi_all_gpu_info(gm_gpu_info_t* out, uint32_t cap, uint32_t* n);
int gm_smi_link(uint32_t src, uint32_t dst, gm_link_info_t* out);
// Row-major count×count link matrix (count = gm_smi_count).
int gm_smi_link_matrix(gm_link_info_t* out, uint32_t cap);
// Processes that currently hold a context on GPU `index`. *n is set to the total number even
// if it exceeds cap (then return value is GM_SMI_MORE_DATA).
int gm_smi_process_list(uint32_t index, gm_proc_info_t* out, uint32_t cap, uint32_t* n);
// Accumulated ECC error counts of GPU `index` (amdsmi_get_gpu_total_ecc_count); an amdsmi status
// such as AMDSMI_STATUS_NOT_SUPPORTED when the driver/firmware does not report them.
int gm_smi_ecc(uint32_t index, uint64_t* correctable, uint64_t* uncorrectable,
               uint64_t* deferred);
const char* gm_smi_strerror(int status);

#define GM_SMI_OK 0
#define GM_SMI_MORE_DATA 39
#define GM_SMI_ERR_NOT_OPEN -1
#define GM_SMI_ERR_DLOPEN -2
#define GM_SMI_ERR_DLSYM -3
#define GM_SMI_ERR_RANGE -4

#ifdef __cplusplus
}
#endif
