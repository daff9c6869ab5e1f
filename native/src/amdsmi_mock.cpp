// amdsmi_mock.cpp — a stand-in libamd_smi for hosts without an AMD GPU (CPU CI, the build sandbox).
//
// Exports the subset of the amdsmi C API that gm_smi.cpp resolves, with the exact prototypes from
// /opt/rocm/include/amd_smi/amdsmi.h, so the *same* shim code path runs against the mock and the
// real library. The reference had no such seam: its NVML tests needed ≥3 physical GPUs
// (reference: pkg/util/gpu/collector/nvml/nvml_test.go:58,71) — SURVEY §4.
//
// Configuration (read at amdsmi_init):
//   GM_AMDSMI_MOCK_CONFIG=<file.json>   topology/inventory (default: one 8×MI355X xGMI hive)
//   GM_AMDSMI_MOCK_PROCS=<file>         live process table, re-read on every process-list call;
//                                       lines "<gpu_index> <pid> <vram_bytes> [name]"
// JSON schema: {"gpus":[{"uuid","bdf","render","card","numa","hive","xgmi_node","kfd_id",
//   "kfd_node","partition","market_name","gfx","cu","vram_mb","compute_partition",
//   "memory_partition","socket"}...], "links": {"default":"xgmi"|"pcie",
//   "overrides":[{"a":0,"b":1,"type":1,"hops":2,"weight":40}]}, "fail_init": <status>,
//   "procs_file": "<path>"}
#include <amd_smi/amdsmi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "mini_json.h"

namespace {

struct MockGpu {
  std::string uuid, bdf, market = "AMD Instinct MI355X", cpart = "SPX", mpart = "NPS1";
  uint32_t render = 128, card = 0, numa = 0, kfd_node = 0, partition = 0, cu = 256, hsa = 0,
           hip = 0, socket = 0;
  uint64_t hive = 0, xnode = 0, kfd_id = 0, gfx = 0x950, vram_mb = 294896;
  uint64_t ecc_ce = 0, ecc_ue = 0;
  amdsmi_bdf_t bdfv{};
};

struct MockLink {
  amdsmi_link_type_t type;
  uint64_t hops, weight;
};

struct MockSocket {
  std::vector<uint32_t> gpus;
};

std::mutex g_mu;
bool g_init = false;
int g_init_calls = 0;
std::vector<MockGpu> g_gpus;
std::vector<MockSocket> g_sockets;
std::map<std::pair<uint32_t, uint32_t>, MockLink> g_link_over;
amdsmi_link_type_t g_default_link = AMDSMI_LINK_TYPE_XGMI;
std::string g_procs_file;

bool parse_bdf(const std::string& s, amdsmi_bdf_t* b) {
  unsigned dom = 0, bus = 0, dev = 0, fn = 0;
  if (sscanf(s.c_str(), "%x:%x:%x.%x", &dom, &bus, &dev, &fn) != 4) return false;
  b->as_uint = 0;
  b->domain_number = dom;
  b->bus_number = bus;
  b->device_number = dev;
  b->function_number = fn;
  return true;
}

void default_inventory() {
  // One 8-GPU MI355X OAM platform: two NUMA sockets × 4 GPUs, one xGMI hive, fully connected.
  static const char* kBus[8] = {"05", "15", "65", "75", "85", "95", "e5", "f5"};
  g_gpus.clear();
  for (uint32_t i = 0; i < 8; ++i) {
    MockGpu g;
    char buf[64];
    snprintf(buf, sizeof(buf), "0000:%s:00.0", kBus[i]);
    g.bdf = buf;
    snprintf(buf, sizeof(buf), "a5ff74a1-0000-1000-80%02x-%012x", i, 0x355000 + i);
    g.uuid = buf;
    g.render = 128 + i;
    g.card = i;
    g.numa = i < 4 ? 0 : 1;
    g.hive = 0x5f3a9c2e11d40001ull;
    g.xnode = 0x1000 + i;
    g.kfd_id = 50000 + 1111 * i;
    g.kfd_node = i + 2;  // KFD nodes 0/1 are the CPUs
    g.hsa = i + 2;
    g.hip = i;
    g.socket = i;
    g_gpus.push_back(g);
  }
}

bool load_config(const char* path) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  gmjson::Value root;
  if (!gmjson::parse(ss.str(), root)) return false;
  if (const gmjson::Value* fi = root.get("fail_init"))
    if (fi->kind == gmjson::Value::Number) return false;
  const gmjson::Value* gpus = root.get("gpus");
  if (gpus && gpus->kind == gmjson::Value::Array) {
    g_gpus.clear();
    uint32_t i = 0;
    for (const auto& gv : gpus->arr) {
      MockGpu g;
      char buf[64];
      snprintf(buf, sizeof(buf), "0000:%02x:00.0", 0x10 * (i + 1));
      g.bdf = gv.str_or("bdf", buf);
      snprintf(buf, sizeof(buf), "mock-uuid-%04u", i);
      g.uuid = gv.str_or("uuid", buf);
      g.render = (uint32_t)gv.num_or("render", 128 + i);
      g.card = (uint32_t)gv.num_or("card", i);
      g.numa = (uint32_t)gv.num_or("numa", 0);
      g.hive = (uint64_t)gv.num_or("hive", 0);
      g.xnode = (uint64_t)gv.num_or("xgmi_node", 0x1000 + i);
      g.kfd_id = (uint64_t)gv.num_or("kfd_id", 50000 + i);
      g.kfd_node = (uint32_t)gv.num_or("kfd_node", i + 1);
      g.partition = (uint32_t)gv.num_or("partition", 0);
      g.market = gv.str_or("market_name", g.market);
      g.gfx = (uint64_t)gv.num_or("gfx", 0x950);
      g.cu = (uint32_t)gv.num_or("cu", 256);
      g.vram_mb = (uint64_t)gv.num_or("vram_mb", 294896);
      g.cpart = gv.str_or("compute_partition", g.cpart);
      g.mpart = gv.str_or("memory_partition", g.mpart);
      g.hsa = (uint32_t)gv.num_or("hsa_id", i + 1);
      g.hip = (uint32_t)gv.num_or("hip_id", i);
      g.socket = (uint32_t)gv.num_or("socket", i);
      g.ecc_ce = (uint64_t)gv.num_or("ecc_correctable", 0);
      g.ecc_ue = (uint64_t)gv.num_or("ecc_uncorrectable", 0);
      g_gpus.push_back(g);
      ++i;
    }
  }
  if (const gmjson::Value* links = root.get("links")) {
    if (links->str_or("default", "xgmi") == "pcie") g_default_link = AMDSMI_LINK_TYPE_PCIE;
    if (const gmjson::Value* ov = links->get("overrides")) {
      for (const auto& o : ov->arr) {
        uint32_t a = (uint32_t)o.num_or("a", 0), b = (uint32_t)o.num_or("b", 0);
        MockLink l{(amdsmi_link_type_t)(int)o.num_or("type", 2), (uint64_t)o.num_or("hops", 1),
                   (uint64_t)o.num_or("weight", 15)};
        g_link_over[{a, b}] = l;
        g_link_over[{b, a}] = l;
      }
    }
  }
  g_procs_file = root.str_or("procs_file", "");
  return true;
}

void build_sockets() {
  g_sockets.clear();
  std::map<uint32_t, size_t> idx;
  for (uint32_t i = 0; i < g_gpus.size(); ++i) {
    parse_bdf(g_gpus[i].bdf, &g_gpus[i].bdfv);
    auto it = idx.find(g_gpus[i].socket);
    if (it == idx.end()) {
      idx[g_gpus[i].socket] = g_sockets.size();
      g_sockets.push_back(MockSocket{});
      it = idx.find(g_gpus[i].socket);
    }
    g_sockets[it->second].gpus.push_back(i);
  }
}

// Handles are 1-based encoded integers so a NULL handle is never valid.
inline amdsmi_processor_handle gpu_handle(uint32_t i) {
  return reinterpret_cast<amdsmi_processor_handle>(uintptr_t(0x6d000000u + i + 1));
}
inline amdsmi_socket_handle sock_handle(uint32_t i) {
  return reinterpret_cast<amdsmi_socket_handle>(uintptr_t(0x5c000000u + i + 1));
}
inline bool gpu_index(amdsmi_processor_handle h, uint32_t* out) {
  uintptr_t v = reinterpret_cast<uintptr_t>(h);
  if (v <= 0x6d000000u || v > 0x6d000000u + g_gpus.size()) return false;
  *out = (uint32_t)(v - 0x6d000000u - 1);
  return true;
}
inline bool sock_index(amdsmi_socket_handle h, uint32_t* out) {
  uintptr_t v = reinterpret_cast<uintptr_t>(h);
  if (v <= 0x5c000000u || v > 0x5c000000u + g_sockets.size()) return false;
  *out = (uint32_t)(v - 0x5c000000u - 1);
  return true;
}

#define MOCK_GPU(h, i)                                 \
  std::lock_guard<std::mutex> lk(g_mu);                \
  if (!g_init) return AMDSMI_STATUS_NOT_INIT;          \
  uint32_t i = 0;                                      \
  if (!gpu_index(h, &i)) return AMDSMI_STATUS_INVAL;

}  // namespace

extern "C" {

amdsmi_status_t amdsmi_init(uint64_t init_flags) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!(init_flags & AMDSMI_INIT_AMD_GPUS)) return AMDSMI_STATUS_NOT_SUPPORTED;
  ++g_init_calls;
  if (g_init) return AMDSMI_STATUS_SUCCESS;
  g_link_over.clear();
  g_default_link = AMDSMI_LINK_TYPE_XGMI;
  g_procs_file.clear();
  default_inventory();
  const char* cfg = getenv("GM_AMDSMI_MOCK_CONFIG");
  if (cfg && *cfg) {
    if (!load_config(cfg)) return AMDSMI_STATUS_DRIVER_NOT_LOADED;
  }
  const char* pf = getenv("GM_AMDSMI_MOCK_PROCS");
  if (pf && *pf) g_procs_file = pf;
  build_sockets();
  g_init = true;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_shut_down(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_init = false;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_socket_handles(uint32_t* socket_count,
                                          amdsmi_socket_handle* socket_handles) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_init) return AMDSMI_STATUS_NOT_INIT;
  if (!socket_count) return AMDSMI_STATUS_INVAL;
  if (!socket_handles) {
    *socket_count = (uint32_t)g_sockets.size();
    return AMDSMI_STATUS_SUCCESS;
  }
  uint32_t n = *socket_count < g_sockets.size() ? *socket_count : (uint32_t)g_sockets.size();
  for (uint32_t i = 0; i < n; ++i) socket_handles[i] = sock_handle(i);
  *socket_count = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle socket_handle,
                                             uint32_t* processor_count,
                                             amdsmi_processor_handle* processor_handles) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_init) return AMDSMI_STATUS_NOT_INIT;
  uint32_t s = 0;
  if (!processor_count || !sock_index(socket_handle, &s)) return AMDSMI_STATUS_INVAL;
  const auto& gs = g_sockets[s].gpus;
  if (!processor_handles) {
    *processor_count = (uint32_t)gs.size();
    return AMDSMI_STATUS_SUCCESS;
  }
  uint32_t n = *processor_count < gs.size() ? *processor_count : (uint32_t)gs.size();
  for (uint32_t i = 0; i < n; ++i) processor_handles[i] = gpu_handle(gs[i]);
  *processor_count = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_type(amdsmi_processor_handle h, processor_type_t* t) {
  MOCK_GPU(h, i);
  (void)i;
  *t = AMDSMI_PROCESSOR_TYPE_AMD_GPU;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_handle_from_bdf(amdsmi_bdf_t bdf,
                                                      amdsmi_processor_handle* h) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_init) return AMDSMI_STATUS_NOT_INIT;
  for (uint32_t i = 0; i < g_gpus.size(); ++i)
    if (g_gpus[i].bdfv.as_uint == bdf.as_uint) {
      *h = gpu_handle(i);
      return AMDSMI_STATUS_SUCCESS;
    }
  return AMDSMI_STATUS_NOT_FOUND;
}

amdsmi_status_t amdsmi_get_gpu_device_uuid(amdsmi_processor_handle h, unsigned int* len,
                                           char* uuid) {
  MOCK_GPU(h, i);
  const std::string& u = g_gpus[i].uuid;
  if (*len < u.size() + 1) {
    *len = (unsigned)u.size() + 1;
    return AMDSMI_STATUS_INSUFFICIENT_SIZE;
  }
  memcpy(uuid, u.c_str(), u.size() + 1);
  *len = (unsigned)u.size() + 1;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_bdf(amdsmi_processor_handle h, amdsmi_bdf_t* bdf) {
  MOCK_GPU(h, i);
  *bdf = g_gpus[i].bdfv;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_bdf_id(amdsmi_processor_handle h, uint64_t* id) {
  MOCK_GPU(h, i);
  const amdsmi_bdf_t& b = g_gpus[i].bdfv;
  *id = (uint64_t(b.domain_number) << 32) | (uint64_t(b.bus_number) << 8) |
        (uint64_t(b.device_number) << 3) | uint64_t(b.function_number);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_enumeration_info(amdsmi_processor_handle h,
                                                amdsmi_enumeration_info_t* info) {
  MOCK_GPU(h, i);
  memset(info, 0, sizeof(*info));
  info->drm_render = g_gpus[i].render;
  info->drm_card = g_gpus[i].card;
  info->hsa_id = g_gpus[i].hsa;
  info->hip_id = g_gpus[i].hip;
  snprintf(info->hip_uuid, sizeof(info->hip_uuid), "GPU-%s", g_gpus[i].uuid.c_str());
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_kfd_info(amdsmi_processor_handle h, amdsmi_kfd_info_t* info) {
  MOCK_GPU(h, i);
  memset(info, 0, sizeof(*info));
  info->kfd_id = g_gpus[i].kfd_id;
  info->node_id = g_gpus[i].kfd_node;
  info->current_partition_id = g_gpus[i].partition;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_xgmi_info(amdsmi_processor_handle h, amdsmi_xgmi_info_t* info) {
  MOCK_GPU(h, i);
  memset(info, 0, sizeof(*info));
  if (g_gpus[i].hive == 0) return AMDSMI_STATUS_NOT_SUPPORTED;
  info->xgmi_lanes = 16;
  info->xgmi_hive_id = g_gpus[i].hive;
  info->xgmi_node_id = g_gpus[i].xnode;
  info->index = i;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_topo_get_numa_node_number(amdsmi_processor_handle h, uint32_t* numa) {
  MOCK_GPU(h, i);
  *numa = g_gpus[i].numa;
  return AMDSMI_STATUS_SUCCESS;
}

static MockLink mock_link(uint32_t a, uint32_t b) {
  auto it = g_link_over.find({a, b});
  if (it != g_link_over.end()) return it->second;
  if (a == b) return MockLink{AMDSMI_LINK_TYPE_INTERNAL, 0, 0};
  const bool same_hive = g_gpus[a].hive != 0 && g_gpus[a].hive == g_gpus[b].hive;
  if (same_hive && g_default_link == AMDSMI_LINK_TYPE_XGMI)
    return MockLink{AMDSMI_LINK_TYPE_XGMI, 1, 15};
  // PCIe through the root complex; crossing sockets costs more.
  const bool same_numa = g_gpus[a].numa == g_gpus[b].numa;
  return MockLink{AMDSMI_LINK_TYPE_PCIE, same_numa ? 2u : 3u, same_numa ? 40u : 72u};
}

amdsmi_status_t amdsmi_topo_get_link_type(amdsmi_processor_handle s, amdsmi_processor_handle d,
                                          uint64_t* hops, amdsmi_link_type_t* type) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_init) return AMDSMI_STATUS_NOT_INIT;
  uint32_t a = 0, b = 0;
  if (!gpu_index(s, &a) || !gpu_index(d, &b)) return AMDSMI_STATUS_INVAL;
  MockLink l = mock_link(a, b);
  *hops = l.hops;
  *type = l.type;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_topo_get_link_weight(amdsmi_processor_handle s, amdsmi_processor_handle d,
                                            uint64_t* weight) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_init) return AMDSMI_STATUS_NOT_INIT;
  uint32_t a = 0, b = 0;
  if (!gpu_index(s, &a) || !gpu_index(d, &b)) return AMDSMI_STATUS_INVAL;
  *weight = mock_link(a, b).weight;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_process_list(amdsmi_processor_handle h, uint32_t* max_processes,
                                            amdsmi_proc_info_t* list) {
  MOCK_GPU(h, idx);
  if (!max_processes) return AMDSMI_STATUS_INVAL;
  std::vector<amdsmi_proc_info_t> found;
  if (!g_procs_file.empty()) {
    std::ifstream f(g_procs_file);
    std::string line;
    while (std::getline(f, line)) {
      std::istringstream ls(line);
      unsigned gi = 0, pid = 0;
      unsigned long long vram = 0;
      std::string name;
      if (!(ls >> gi >> pid)) continue;
      ls >> vram >> name;
      if (gi != idx) continue;
      amdsmi_proc_info_t p;
      memset(&p, 0, sizeof(p));
      p.pid = pid;
      p.mem = vram;
      p.memory_usage.vram_mem = vram;
      snprintf(p.name, sizeof(p.name), "%s", name.empty() ? "mockproc" : name.c_str());
      p.cu_occupancy = 0;
      found.push_back(p);
    }
  }
  const uint32_t cap = *max_processes;
  const uint32_t n = (uint32_t)found.size();
  for (uint32_t i = 0; i < n && i < cap && list; ++i) list[i] = found[i];
  *max_processes = n;
  return n > cap ? AMDSMI_STATUS_OUT_OF_RESOURCES : AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_asic_info(amdsmi_processor_handle h, amdsmi_asic_info_t* info) {
  MOCK_GPU(h, i);
  memset(info, 0, sizeof(*info));
  snprintf(info->market_name, sizeof(info->market_name), "%s", g_gpus[i].market.c_str());
  info->vendor_id = 0x1002;
  snprintf(info->vendor_name, sizeof(info->vendor_name), "Advanced Micro Devices Inc. [AMD/ATI]");
  info->device_id = 0x75a3;
  info->oam_id = i;
  info->num_of_compute_units = g_gpus[i].cu;
  info->target_graphics_version = g_gpus[i].gfx;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_vram_info(amdsmi_processor_handle h, amdsmi_vram_info_t* info) {
  MOCK_GPU(h, i);
  memset(info, 0, sizeof(*info));
  info->vram_size = g_gpus[i].vram_mb;
  info->vram_bit_width = 8192;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_compute_partition(amdsmi_processor_handle h, char* buf,
                                                 uint32_t len) {
  MOCK_GPU(h, i);
  snprintf(buf, len, "%s", g_gpus[i].cpart.c_str());
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_partition(amdsmi_processor_handle h, char* buf,
                                                uint32_t len) {
  MOCK_GPU(h, i);
  snprintf(buf, len, "%s", g_gpus[i].mpart.c_str());
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_total_ecc_count(amdsmi_processor_handle h,
                                               amdsmi_error_count_t* ec) {
  MOCK_GPU(h, i);
  if (!ec) return AMDSMI_STATUS_INVAL;
  memset(ec, 0, sizeof(*ec));
  ec->correctable_count = g_gpus[i].ecc_ce;
  ec->uncorrectable_count = g_gpus[i].ecc_ue;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_status_code_to_string(amdsmi_status_t status, const char** s) {
  switch (status) {
    case AMDSMI_STATUS_SUCCESS: *s = "AMDSMI_STATUS_SUCCESS: Call succeeded"; break;
    case AMDSMI_STATUS_NOT_INIT: *s = "AMDSMI_STATUS_NOT_INIT: Processor not initialized"; break;
    case AMDSMI_STATUS_DRIVER_NOT_LOADED:
      *s = "AMDSMI_STATUS_DRIVER_NOT_LOADED: Processor driver not loaded";
      break;
    case AMDSMI_STATUS_INVAL: *s = "AMDSMI_STATUS_INVAL: Invalid parameters"; break;
    default: *s = "AMDSMI_STATUS (mock): other"; break;
  }
  return AMDSMI_STATUS_SUCCESS;
}

// Test hook: point the live process table at another file ("" disables).
void gm_mock_set_procs_file(const char* path) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_procs_file = path ? path : "";
}

// Test hook: set a GPU's accumulated ECC counts (simulates a memory error showing up).
int gm_mock_set_ecc(uint32_t index, uint64_t correctable, uint64_t uncorrectable) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (index >= g_gpus.size()) return -1;
  g_gpus[index].ecc_ce = correctable;
  g_gpus[index].ecc_ue = uncorrectable;
  return 0;
}

// Test hook: number of amdsmi_init() calls since load (proves the shim does not re-init per query).
int gm_mock_init_calls(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_init_calls;
}

}  // extern "C"
