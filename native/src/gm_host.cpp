// gm_host.cpp — in-process implementation of the node agent's privileged operations.
// See gm_host.h for the contract; reference parity notes are inline.
#include "gm_host.h"

#include <dirent.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <linux/bpf.h>
#include <sched.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mount.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/sysmacros.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr const char* kProgName = "gm_devallow";

// ------------------------------------------------------------------ small fd helpers
struct Fd {
  int fd = -1;
  Fd() = default;
  explicit Fd(int f) : fd(f) {}
  Fd(const Fd&) = delete;
  Fd& operator=(const Fd&) = delete;
  Fd(Fd&& o) noexcept : fd(o.fd) { o.fd = -1; }
  Fd& operator=(Fd&& o) noexcept {
    if (this != &o) {
      reset();
      fd = o.fd;
      o.fd = -1;
    }
    return *this;
  }
  ~Fd() { reset(); }
  void reset() {
    if (fd >= 0) close(fd);
    fd = -1;
  }
  bool ok() const { return fd >= 0; }
};

int write_all(int fd, const char* buf, size_t len) {
  while (len > 0) {
    ssize_t w = write(fd, buf, len);
    if (w < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    buf += w;
    len -= (size_t)w;
  }
  return 0;
}

// ------------------------------------------------------------------ bpf(2)
long sys_bpf(int cmd, union bpf_attr* attr, unsigned size) {
  return syscall(__NR_bpf, cmd, attr, size);
}

inline uint64_t ptr_u64(const void* p) { return (uint64_t)(uintptr_t)p; }

// struct bpf_insn packed into a uint64 in host (little-endian) order.
uint64_t insn(uint8_t code, uint8_t dst, uint8_t src, int16_t off, int32_t imm) {
  struct bpf_insn i;
  memset(&i, 0, sizeof(i));
  i.code = code;
  i.dst_reg = dst & 0xf;
  i.src_reg = src & 0xf;
  i.off = off;
  i.imm = imm;
  uint64_t v;
  static_assert(sizeof(i) == sizeof(v), "bpf_insn is 8 bytes");
  memcpy(&v, &i, sizeof(v));
  return v;
}

// Opcodes used by the device filter.
constexpr uint8_t LDX_W = BPF_LDX | BPF_MEM | BPF_W;
constexpr uint8_t MOV64_X = BPF_ALU64 | BPF_MOV | BPF_X;
constexpr uint8_t MOV64_K = BPF_ALU64 | BPF_MOV | BPF_K;
constexpr uint8_t AND64_K = BPF_ALU64 | BPF_AND | BPF_K;
constexpr uint8_t RSH64_K = BPF_ALU64 | BPF_RSH | BPF_K;
constexpr uint8_t JNE_K = BPF_JMP | BPF_JNE | BPF_K;
constexpr uint8_t CALL = BPF_JMP | BPF_CALL;
constexpr uint8_t EXIT = BPF_JMP | BPF_EXIT;
constexpr uint8_t LD_IMM64 = BPF_LD | BPF_DW | BPF_IMM;
constexpr uint8_t STX_W = BPF_STX | BPF_MEM | BPF_W;
constexpr uint8_t ADD64_K = BPF_ALU64 | BPF_ADD | BPF_K;
constexpr uint8_t XOR64_K = BPF_ALU64 | BPF_XOR | BPF_K;
constexpr uint8_t JEQ_K = BPF_JMP | BPF_JEQ | BPF_K;

// r2 = access_type; r3 = r2 & 0xffff (dev type); r2 >>= 16 (access); r4 = major; r5 = minor,
// from the context in r1. Returns the next index.
int emit_ctx_load(uint64_t* out, int k) {
  out[k++] = insn(LDX_W, 2, 1, 0, 0);
  out[k++] = insn(MOV64_X, 3, 2, 0, 0);
  out[k++] = insn(AND64_K, 3, 0, 0, 0xffff);
  out[k++] = insn(RSH64_K, 2, 0, 0, 16);
  out[k++] = insn(LDX_W, 4, 1, 4, 0);
  out[k++] = insn(LDX_W, 5, 1, 8, 0);
  return k;
}

int rule_block_len(const gm_dev_rule_t& r);

// One block per rule (first match wins): matching → return allow/deny, else fall through to
// the next block. Expects emit_ctx_load's registers. Returns the next index or -EINVAL.
int emit_rule_blocks(const gm_dev_rule_t* rules, int n, uint64_t* out, int k) {
  for (int i = 0; i < n; ++i) {
    const gm_dev_rule_t& r = rules[i];
    const int start = k;
    const int end = start + rule_block_len(r);  // index of first insn after this block
    auto jne = [&](int reg, int32_t imm) {
      int16_t off = (int16_t)(end - (k + 1));
      out[k] = insn(JNE_K, (uint8_t)reg, 0, off, imm);
      ++k;
    };
    if (r.type != 'a') jne(3, r.type == 'c' ? BPF_DEVCG_DEV_CHAR : BPF_DEVCG_DEV_BLOCK);
    if ((r.access & 7) != 7) {
      // requested access must be a subset of the rule's: (req & ~rule) == 0
      out[k++] = insn(MOV64_X, 0, 2, 0, 0);
      out[k++] = insn(AND64_K, 0, 0, 0, (int32_t)(~r.access & 7));
      // jne r0, 0 → next rule
      int16_t off = (int16_t)(end - (k + 1));
      out[k] = insn(JNE_K, 0, 0, off, 0);
      ++k;
    }
    if (r.major >= 0) jne(4, r.major);
    if (r.minor >= 0) jne(5, r.minor);
    out[k++] = insn(MOV64_K, 0, 0, 0, r.allow ? 1 : 0);
    out[k++] = insn(EXIT, 0, 0, 0, 0);
    if (k != end) return -EINVAL;  // layout bug guard (see rule_block_len)
  }
  return k;
}

int rule_block_len(const gm_dev_rule_t& r) {
  int n = 2;  // mov r0, allow; exit
  if (r.type != 'a') n += 1;
  if ((r.access & 7) != 7) n += 3;  // mov r0,r2; and r0,~acc; jne r0,0
  if (r.major >= 0) n += 1;
  if (r.minor >= 0) n += 1;
  return n;
}

int get_prog_fd_by_id(uint32_t id) {
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.prog_id = id;
  long fd = sys_bpf(BPF_PROG_GET_FD_BY_ID, &a, sizeof(a));
  return fd < 0 ? -errno : (int)fd;
}

int prog_info(int fd, struct bpf_prog_info* info, uint32_t* map_ids, uint32_t map_cap) {
  memset(info, 0, sizeof(*info));
  info->nr_map_ids = map_cap;
  info->map_ids = ptr_u64(map_ids);
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.info.bpf_fd = (uint32_t)fd;
  a.info.info_len = sizeof(*info);
  a.info.info = ptr_u64(info);
  return sys_bpf(BPF_OBJ_GET_INFO_BY_FD, &a, sizeof(a)) < 0 ? -errno : 0;
}

int map_fd_by_id(uint32_t id) {
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.map_id = id;
  long fd = sys_bpf(BPF_MAP_GET_FD_BY_ID, &a, sizeof(a));
  return fd < 0 ? -errno : (int)fd;
}

// Prog id stored in slot 0 of a PROG_ARRAY (user-space lookups return ids, not fds).
int prog_array_slot0(int map_fd, uint32_t* prog_id) {
  uint32_t key = 0, val = 0;
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.map_fd = (uint32_t)map_fd;
  a.key = ptr_u64(&key);
  a.value = ptr_u64(&val);
  if (sys_bpf(BPF_MAP_LOOKUP_ELEM, &a, sizeof(a)) < 0) return -errno;
  *prog_id = val;
  return 0;
}

int make_chain_map(int target_prog_fd) {
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.map_type = BPF_MAP_TYPE_PROG_ARRAY;
  a.key_size = 4;
  a.value_size = 4;
  a.max_entries = 1;
  snprintf(a.map_name, sizeof(a.map_name), "gm_devchain");
  long mfd = sys_bpf(BPF_MAP_CREATE, &a, sizeof(a));
  if (mfd < 0) return -errno;
  uint32_t key = 0, val = (uint32_t)target_prog_fd;
  memset(&a, 0, sizeof(a));
  a.map_fd = (uint32_t)mfd;
  a.key = ptr_u64(&key);
  a.value = ptr_u64(&val);
  a.flags = BPF_ANY;
  if (sys_bpf(BPF_MAP_UPDATE_ELEM, &a, sizeof(a)) < 0) {
    int e = -errno;
    close((int)mfd);
    return e;
  }
  return (int)mfd;
}

// ---- tail-call map lifetime (see gm_host.h: PROG_ARRAY slots die with the last user ref)
// One map per wrapped program, keyed by (cgroup inode, id of the program it chains to).
std::mutex g_keep_mu;
std::map<std::pair<uint64_t, uint32_t>, int> g_kept_maps;  // map fds kept open (no bpffs)

uint64_t cgroup_ino(int cgfd) {
  struct stat st;
  return fstat(cgfd, &st) == 0 ? (uint64_t)st.st_ino : 0;
}

std::string pin_prefix(uint64_t ino) { return "gm_" + std::to_string(ino); }

std::string pin_path(const char* pin_dir, uint64_t ino, uint32_t chain) {
  return std::string(pin_dir) + "/" + pin_prefix(ino) + "_" + std::to_string(chain);
}

int obj_pin(int fd, const std::string& path) {
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.pathname = ptr_u64(path.c_str());
  a.bpf_fd = (uint32_t)fd;
  return sys_bpf(BPF_OBJ_PIN, &a, sizeof(a)) < 0 ? -errno : 0;
}

// Makes `map_fd` survive this call: pin (atomically replacing the previous pin) or keep the fd.
int keep_map(const char* pin_dir, uint64_t ino, uint32_t chain, int map_fd) {
  if (pin_dir && *pin_dir) {
    const std::string final_path = pin_path(pin_dir, ino, chain);
    const std::string tmp = final_path + "_new";  // bpffs rejects "." in names
    unlink(tmp.c_str());
    int e = obj_pin(map_fd, tmp);
    if (e < 0) return e;
    if (rename(tmp.c_str(), final_path.c_str()) < 0) {
      unlink(final_path.c_str());
      unlink(tmp.c_str());
      return obj_pin(map_fd, final_path);
    }
    return 0;
  }
  int dupfd = fcntl(map_fd, F_DUPFD_CLOEXEC, 0);
  if (dupfd < 0) return -errno;
  std::lock_guard<std::mutex> lk(g_keep_mu);
  auto key = std::make_pair(ino, chain);
  auto it = g_kept_maps.find(key);
  if (it != g_kept_maps.end()) close(it->second);
  g_kept_maps[key] = dupfd;
  return 0;
}

// Drops every kept/pinned map of the cgroup whose chain target is not in `keep`
// (also the single-map pin name "gm_<ino>" of ABI 1).
void drop_maps_except(const char* pin_dir, uint64_t ino, const std::vector<uint32_t>& keep) {
  auto kept = [&](uint32_t c) {
    for (uint32_t k : keep)
      if (k == c) return true;
    return false;
  };
  if (pin_dir && *pin_dir) {
    const std::string pre = pin_prefix(ino);
    unlink((std::string(pin_dir) + "/" + pre).c_str());
    if (DIR* d = opendir(pin_dir)) {
      while (struct dirent* de = readdir(d)) {
        const char* nm = de->d_name;
        if (strncmp(nm, pre.c_str(), pre.size()) != 0 || nm[pre.size()] != '_') continue;
        char* end = nullptr;
        unsigned long c = strtoul(nm + pre.size() + 1, &end, 10);
        if (end && *end == 0 && kept((uint32_t)c)) continue;
        unlinkat(dirfd(d), nm, 0);
      }
      closedir(d);
    }
  }
  std::lock_guard<std::mutex> lk(g_keep_mu);
  for (auto it = g_kept_maps.begin(); it != g_kept_maps.end();) {
    if (it->first.first == ino && !kept(it->first.second)) {
      close(it->second);
      it = g_kept_maps.erase(it);
    } else {
      ++it;
    }
  }
}

struct Attached {
  std::vector<uint32_t> ids;
  uint32_t flags = 0;
};

int query(int cgfd, Attached* out) {
  uint32_t ids[64];
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.query.target_fd = (uint32_t)cgfd;
  a.query.attach_type = BPF_CGROUP_DEVICE;
  a.query.prog_ids = ptr_u64(ids);
  a.query.prog_cnt = 64;
  if (sys_bpf(BPF_PROG_QUERY, &a, sizeof(a)) < 0) return -errno;
  out->flags = a.query.attach_flags;
  out->ids.assign(ids, ids + (a.query.prog_cnt < 64 ? a.query.prog_cnt : 64));
  return 0;
}

int attach(int cgfd, int prog_fd, int replace_fd, uint32_t existing_flags) {
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.target_fd = (uint32_t)cgfd;
  a.attach_bpf_fd = (uint32_t)prog_fd;
  a.attach_type = BPF_CGROUP_DEVICE;
  if (existing_flags & BPF_F_ALLOW_MULTI) {
    a.attach_flags = BPF_F_ALLOW_MULTI;
    if (replace_fd >= 0) {
      a.attach_flags |= BPF_F_REPLACE;
      a.replace_bpf_fd = (uint32_t)replace_fd;
    }
  } else {
    // Single-program mode (flags 0 / ALLOW_OVERRIDE): attaching again replaces the program.
    a.attach_flags = existing_flags & BPF_F_ALLOW_OVERRIDE;
  }
  return sys_bpf(BPF_PROG_ATTACH, &a, sizeof(a)) < 0 ? -errno : 0;
}

int map_info(int fd, struct bpf_map_info* info) {
  memset(info, 0, sizeof(*info));
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.info.bpf_fd = (uint32_t)fd;
  a.info.info_len = sizeof(*info);
  a.info.info = ptr_u64(info);
  return sys_bpf(BPF_OBJ_GET_INFO_BY_FD, &a, sizeof(a)) < 0 ? -errno : 0;
}

// Ours = named kProgName. *chained_id: the program in slot 0 of its PROG_ARRAY (0 if none);
// *set_map_id: its allow-set HASH map (set-mode program, see gm_bpf_dev_build_set), 0 for a
// straight-line program.
bool is_ours(uint32_t id, uint32_t* chained_id, uint32_t* set_map_id = nullptr,
             bool* has_chain_map = nullptr) {
  Fd pfd(get_prog_fd_by_id(id));
  if (!pfd.ok()) return false;
  struct bpf_prog_info info;
  uint32_t maps[4] = {0};
  if (prog_info(pfd.fd, &info, maps, 4) != 0) return false;
  if (strncmp(info.name, kProgName, sizeof(info.name)) != 0) return false;
  if (chained_id) *chained_id = 0;
  if (set_map_id) *set_map_id = 0;
  if (has_chain_map) *has_chain_map = false;
  if (!chained_id && !set_map_id && !has_chain_map) return true;
  for (uint32_t i = 0; i < info.nr_map_ids && i < 4; ++i) {
    Fd mfd(map_fd_by_id(maps[i]));
    struct bpf_map_info mi;
    if (!mfd.ok() || map_info(mfd.fd, &mi) != 0) continue;
    if (mi.type == BPF_MAP_TYPE_PROG_ARRAY) {
      if (has_chain_map) *has_chain_map = true;
      uint32_t pid = 0;
      if (chained_id && prog_array_slot0(mfd.fd, &pid) == 0) *chained_id = pid;
    } else if (mi.type == BPF_MAP_TYPE_HASH && set_map_id) {
      *set_map_id = mi.id;
    }
  }
  return true;
}

// ---- allow-set map (set-mode programs) --------------------------------------------------------
// key = {dev type (BPF_DEVCG_DEV_*), major, minor}, value = allowed access bits (GM_ACC_*).
struct SetKey {
  uint32_t type, major, minor;
};
constexpr uint32_t kSetMax = 512;

int make_set_map() {
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.map_type = BPF_MAP_TYPE_HASH;
  a.key_size = sizeof(SetKey);
  a.value_size = 4;
  a.max_entries = kSetMax;
  snprintf(a.map_name, sizeof(a.map_name), "gm_devset");
  long fd = sys_bpf(BPF_MAP_CREATE, &a, sizeof(a));
  return fd < 0 ? -errno : (int)fd;
}

int set_keys(int map_fd, std::vector<SetKey>* keys) {
  keys->clear();
  SetKey cur{}, next{};
  bool first = true;
  for (uint32_t guard = 0; guard <= kSetMax; ++guard) {
    union bpf_attr a;
    memset(&a, 0, sizeof(a));
    a.map_fd = (uint32_t)map_fd;
    a.key = first ? 0 : ptr_u64(&cur);
    a.next_key = ptr_u64(&next);
    if (sys_bpf(BPF_MAP_GET_NEXT_KEY, &a, sizeof(a)) < 0) return errno == ENOENT ? 0 : -errno;
    keys->push_back(next);
    cur = next;
    first = false;
  }
  return -E2BIG;
}

// Every {key, value} of the set: one BPF_MAP_LOOKUP_BATCH (≥ 5.6) per kSetMax entries, or a
// GET_NEXT_KEY + LOOKUP walk on kernels without batch ops.
int set_entries(int map_fd, std::vector<std::pair<SetKey, uint32_t>>* out) {
  out->clear();
  std::vector<SetKey> keys(kSetMax);
  std::vector<uint32_t> vals(kSetMax);
  uint32_t token = 0;
  bool first = true;
  for (;;) {
    union bpf_attr a;
    memset(&a, 0, sizeof(a));
    a.batch.map_fd = (uint32_t)map_fd;
    a.batch.in_batch = first ? 0 : ptr_u64(&token);
    a.batch.out_batch = ptr_u64(&token);
    a.batch.keys = ptr_u64(keys.data());
    a.batch.values = ptr_u64(vals.data());
    a.batch.count = kSetMax;
    long rc = sys_bpf(BPF_MAP_LOOKUP_BATCH, &a, sizeof(a));
    int err = rc < 0 ? errno : 0;
    if (rc < 0 && err != ENOENT) {
      if (!first || (err != EINVAL && err != ENOTSUP && err != 524 /* ENOTSUPP */)) return -err;
      break;  // no batch ops here: walk instead
    }
    for (uint32_t i = 0; i < a.batch.count; ++i) out->emplace_back(keys[i], vals[i]);
    if (err == ENOENT || a.batch.count == 0) return 0;
    first = false;
  }
  std::vector<SetKey> ks;
  int e = set_keys(map_fd, &ks);
  if (e < 0) return e;
  for (const SetKey& k : ks) {
    uint32_t acc = 0;
    union bpf_attr a;
    memset(&a, 0, sizeof(a));
    a.map_fd = (uint32_t)map_fd;
    a.key = ptr_u64(&k);
    a.value = ptr_u64(&acc);
    if (sys_bpf(BPF_MAP_LOOKUP_ELEM, &a, sizeof(a)) == 0) out->emplace_back(k, acc);
  }
  return 0;
}

int set_op(int cmd, int map_fd, const SetKey& k, uint32_t* value) {
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.map_fd = (uint32_t)map_fd;
  a.key = ptr_u64(&k);
  if (value) a.value = ptr_u64(value);
  if (cmd == BPF_MAP_UPDATE_ELEM) a.flags = BPF_ANY;
  return sys_bpf(cmd, &a, sizeof(a)) < 0 ? -errno : 0;
}

SetKey key_of(const gm_dev_rule_t& r) {
  return SetKey{r.type == 'b' ? (uint32_t)BPF_DEVCG_DEV_BLOCK : (uint32_t)BPF_DEVCG_DEV_CHAR,
                (uint32_t)r.major, (uint32_t)r.minor};
}

// Exact allow rules only (no wildcards, no denies): what a set-mode program can hold.
bool set_eligible(const gm_dev_rule_t* rules, int n) {
  for (int i = 0; i < n; ++i) {
    const gm_dev_rule_t& r = rules[i];
    if (!r.allow || (r.type != 'c' && r.type != 'b') || r.major < 0 || r.minor < 0) return false;
  }
  return n <= (int)kSetMax;
}

// Makes the map hold exactly `rules`: new and changed entries first, then stale ones deleted,
// so a device granted before and after is never denied in between.
int sync_set(int map_fd, const gm_dev_rule_t* rules, int n) {
  std::vector<SetKey> have;
  int e = set_keys(map_fd, &have);
  if (e < 0) return e;
  for (int i = 0; i < n; ++i) {
    uint32_t acc = rules[i].access & 7;
    if ((e = set_op(BPF_MAP_UPDATE_ELEM, map_fd, key_of(rules[i]), &acc)) < 0) return e;
  }
  for (const SetKey& k : have) {
    bool keep = false;
    for (int i = 0; i < n && !keep; ++i) {
      SetKey w = key_of(rules[i]);
      keep = w.type == k.type && w.major == k.major && w.minor == k.minor;
    }
    if (!keep && (e = set_op(BPF_MAP_DELETE_ELEM, map_fd, k, nullptr)) < 0 && e != -ENOENT)
      return e;
  }
  return 0;
}

// ------------------------------------------------------------------ device nodes
constexpr const char* kMarker = "gm-chr";

// Directories that are the host's own /dev (and /dev/dri) as seen from the worker: a container
// whose /dev is a bind of them (hostPath /dev, privileged runtimes) shares the host's nodes, so
// gpumounter must neither create nor unlink anything there. Set once at worker start-up.
struct DirId {
  std::atomic<uint64_t> dev{0}, ino{0};
};
DirId g_guard[2];

bool guarded_dir(int dirfd) {
  struct stat st;
  if (fstat(dirfd, &st) < 0) return false;
  for (auto& g : g_guard) {
    uint64_t ino = g.ino.load(std::memory_order_acquire);
    if (ino && ino == (uint64_t)st.st_ino && g.dev.load(std::memory_order_relaxed) == st.st_dev)
      return true;
  }
  return false;
}

int open_root(int pid, const char* root) {
  if (root && *root) {
    int fd = open(root, O_PATH | O_DIRECTORY | O_CLOEXEC);
    return fd < 0 ? -errno : fd;
  }
  char p[64];
  snprintf(p, sizeof(p), "/proc/%d/root", pid);
  int fd = open(p, O_PATH | O_DIRECTORY | O_CLOEXEC);
  return fd < 0 ? -errno : fd;
}

constexpr int kSharedHost = 2;  // result: the directory is the host's; left untouched

// Walks `path` (relative, '/'-separated) below rootfd without following symlinks, creating
// missing directories when `create`. Returns the parent dir fd and the leaf name.
int walk_parent(int rootfd, const char* path, bool create, Fd* parent, std::string* leaf) {
  std::string p(path);
  while (!p.empty() && p[0] == '/') p.erase(0, 1);
  std::vector<std::string> comps;
  size_t start = 0;
  while (start <= p.size()) {
    size_t e = p.find('/', start);
    if (e == std::string::npos) e = p.size();
    std::string c = p.substr(start, e - start);
    if (!c.empty() && c != ".") {
      if (c == "..") return -EINVAL;  // never climb out of the container root
      comps.push_back(c);
    }
    start = e + 1;
  }
  if (comps.empty()) return -EINVAL;
  int cur = dup(rootfd);
  if (cur < 0) return -errno;
  Fd curfd(cur);
  for (size_t i = 0; i + 1 < comps.size(); ++i) {
    int nfd = openat(curfd.fd, comps[i].c_str(), O_PATH | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC);
    if (nfd < 0 && errno == ENOENT && create) {
      if (guarded_dir(curfd.fd)) return kSharedHost;  // never mkdir inside the host's /dev
      if (mkdirat(curfd.fd, comps[i].c_str(), 0755) < 0 && errno != EEXIST) return -errno;
      nfd = openat(curfd.fd, comps[i].c_str(), O_PATH | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC);
    }
    if (nfd < 0) return -errno;
    curfd = Fd(nfd);
  }
  *leaf = comps.back();
  *parent = std::move(curfd);
  return 0;
}

// walk_parent with the directory fds of one call kept: the nodes of an attach share dev/ and
// dev/dri/, so 8 GPUs (17 nodes) walk two directories once instead of 17 times.
struct Walker {
  int rootfd;
  bool mknod_denied = false;  // emulate mode: mknodat already refused with EPERM in this call
  std::map<std::string, Fd> dirs;
  explicit Walker(int r) : rootfd(r) {}
  // *dirfd stays owned by the walker. Same results as walk_parent.
  int parent(const char* path, bool create, int* dirfd, std::string* leaf) {
    std::string p(path);
    size_t cut = p.rfind('/');
    std::string dir = cut == std::string::npos ? std::string() : p.substr(0, cut);
    auto it = dirs.find(dir);
    if (it != dirs.end()) {
      *leaf = p.substr(cut + 1);
      if (leaf->empty() || *leaf == "." || *leaf == "..") return -EINVAL;
      *dirfd = it->second.fd;
      return 0;
    }
    Fd fd;
    int e = walk_parent(rootfd, path, create, &fd, leaf);
    if (e != 0) return e;
    *dirfd = fd.fd;
    dirs.emplace(dir, std::move(fd));
    return 0;
  }
};

// kind: 0 absent, 1 char dev, 2 emulated marker, 3 other.
int stat_leaf(int dirfd, const std::string& leaf, int* kind, uint32_t* maj, uint32_t* min,
              uint32_t* mode) {
  struct stat st;
  *kind = 0;
  *maj = *min = *mode = 0;
  if (fstatat(dirfd, leaf.c_str(), &st, AT_SYMLINK_NOFOLLOW) < 0) {
    if (errno == ENOENT) return 0;
    return -errno;
  }
  *mode = st.st_mode & 07777;
  if (S_ISCHR(st.st_mode)) {
    *kind = 1;
    *maj = major(st.st_rdev);
    *min = minor(st.st_rdev);
    return 0;
  }
  *kind = 3;
  if (S_ISREG(st.st_mode) && st.st_size < 64) {
    int fd = openat(dirfd, leaf.c_str(), O_RDONLY | O_NOFOLLOW | O_CLOEXEC);
    if (fd >= 0) {
      char buf[64] = {0};
      ssize_t r = read(fd, buf, sizeof(buf) - 1);
      close(fd);
      unsigned a = 0, b = 0;
      char tag[16] = {0};
      if (r > 0 && sscanf(buf, "%15s %u:%u", tag, &a, &b) == 3 && strcmp(tag, kMarker) == 0) {
        *kind = 2;
        *maj = a;
        *min = b;
      }
    }
  }
  return 0;
}

int create_one(Walker& w, const gm_dev_node_t& n, int flags) {
  int pfd;
  std::string leaf;
  int e = w.parent(n.path, true, &pfd, &leaf);
  if (e != 0) return e;
  if (guarded_dir(pfd)) return kSharedHost;
  int kind;
  uint32_t maj, min, mode;
  e = stat_leaf(pfd, leaf, &kind, &maj, &min, &mode);
  if (e < 0) return e;
  if (kind == 1 || kind == 2) {
    if (maj == n.major && min == n.minor) {
      if (kind == 1 && mode != (n.mode & 07777))
        if (fchmodat(pfd, leaf.c_str(), n.mode & 07777, 0) < 0) return -errno;
      return 1;  // idempotent re-attach
    }
    if (!(flags & GM_DEV_REPLACE)) return -EEXIST;
    if (unlinkat(pfd, leaf.c_str(), 0) < 0) return -errno;
  } else if (kind == 3) {
    return -EEXIST;  // refuse to clobber an unrelated file
  }
  const bool try_mknod = !w.mknod_denied;
  if (!try_mknod ||
      mknodat(pfd, leaf.c_str(), S_IFCHR | (n.mode & 07777), makedev(n.major, n.minor)) < 0) {
    int err = try_mknod ? errno : EPERM;
    if (!(err == EPERM && (flags & GM_DEV_EMULATE))) return -err;
    w.mknod_denied = true;  // unprivileged: the rest of this call goes straight to markers
    // The marker appears whole or not at all: written under a hidden temporary name, then
    // linked into place. Created in place, a worker killed between the create and the write
    // left an empty file, which reads as "something else lives there": never replaced, never
    // removed, the node missing for good (chaos on an unprivileged GPU box).
    const std::string tmp = "." + leaf + ".gm-" + std::to_string(getpid());
    unlinkat(pfd, tmp.c_str(), 0);
    int fd = openat(pfd, tmp.c_str(), O_CREAT | O_EXCL | O_WRONLY | O_NOFOLLOW | O_CLOEXEC,
                    n.mode & 07777);
    if (fd < 0) return -errno;
    char buf[48];
    int len = snprintf(buf, sizeof(buf), "%s %u:%u\n", kMarker, n.major, n.minor);
    int wr = write_all(fd, buf, (size_t)len);
    if (wr == 0 && fchmod(fd, n.mode & 07777) < 0) wr = -errno;  // exact mode despite umask
    close(fd);
    if (wr == 0 && linkat(pfd, tmp.c_str(), pfd, leaf.c_str(), 0) < 0) {
      wr = -errno;
      // a filesystem without hard links: a rename that will not replace does the same
      if ((wr == -EPERM || wr == -EOPNOTSUPP) &&
          syscall(SYS_renameat2, pfd, tmp.c_str(), pfd, leaf.c_str(), 1 /* NOREPLACE */) == 0)
        wr = 0;
    }
    unlinkat(pfd, tmp.c_str(), 0);
    if (wr < 0) return wr;
  } else if (fchmodat(pfd, leaf.c_str(), n.mode & 07777, 0) < 0) {
    // mknod honours the umask; set the exact mode the tenant needs (reference used -m 666,
    // namespace.go:168).
    return -errno;
  }
  if (n.uid >= 0 || n.gid >= 0) {
    if (fchownat(pfd, leaf.c_str(), (uid_t)n.uid, (gid_t)n.gid, AT_SYMLINK_NOFOLLOW) < 0 &&
        errno != EPERM)
      return -errno;
  }
  return 0;
}

int remove_one(Walker& w, const gm_dev_node_t& n) {
  int pfd;
  std::string leaf;
  int e = w.parent(n.path, false, &pfd, &leaf);
  if (e == -ENOENT) return 1;
  if (e != 0) return e;
  if (guarded_dir(pfd)) return kSharedHost;
  int kind;
  uint32_t maj, min, mode;
  e = stat_leaf(pfd, leaf, &kind, &maj, &min, &mode);
  if (e < 0) return e;
  if (kind == 0) return 1;
  if ((kind == 1 || kind == 2) && maj == n.major && min == n.minor) {
    if (unlinkat(pfd, leaf.c_str(), 0) < 0) return -errno;
    return 0;
  }
  return -EEXIST;  // something else lives there: never delete it
}

// Runs fn(rootfd) either through /proc/<pid>/root (or a test root) or, with GM_DEV_VIA_SETNS,
// on a helper thread that privatises its fs context and joins the target's mount namespace
// (setns(CLONE_NEWNS) is refused for threads that share CLONE_FS, hence unshare first).
// GM_DEV_BIND always runs on such a thread: mounts are made from inside the target namespace
// (an explicit test root is in ours already) and unmounting changes the thread's cwd.
template <typename F>
int with_root(int pid, const char* root, int flags, F fn) {
  const bool explicit_root = root && *root;
  if (!(flags & GM_DEV_BIND) && (!(flags & GM_DEV_VIA_SETNS) || explicit_root)) {
    int rfd = open_root(pid, root);
    if (rfd < 0) return rfd;
    Fd r(rfd);
    return fn(r.fd);
  }
  int result = 0;
  std::thread t([&]() {
    if (unshare(CLONE_FS) < 0) {
      result = -errno;
      return;
    }
    if (explicit_root) {
      int rfd = open_root(pid, root);
      if (rfd < 0) {
        result = rfd;
        return;
      }
      Fd r(rfd);
      result = fn(r.fd);
      return;
    }
    char p[64];
    snprintf(p, sizeof(p), "/proc/%d/ns/mnt", pid);
    Fd ns(open(p, O_RDONLY | O_CLOEXEC));
    if (!ns.ok()) {
      result = -errno;
      return;
    }
    if (setns(ns.fd, CLONE_NEWNS) < 0) {
      result = -errno;
      return;
    }
    Fd r(open("/", O_PATH | O_DIRECTORY | O_CLOEXEC));
    if (!r.ok()) {
      result = -errno;
      return;
    }
    result = fn(r.fd);
  });
  t.join();
  return result;
}

// ---- bind mode (containers in their own user namespace, see GM_DEV_BIND) -----------------------
#ifndef OPEN_TREE_CLONE
#define OPEN_TREE_CLONE 1
#endif
#ifndef MOVE_MOUNT_F_EMPTY_PATH
#define MOVE_MOUNT_F_EMPTY_PATH 0x00000004
#endif
#ifndef STATX_ATTR_MOUNT_ROOT
#define STATX_ATTR_MOUNT_ROOT 0x00002000
#endif
#ifndef SYS_open_tree
#define SYS_open_tree 428
#endif
#ifndef SYS_move_mount
#define SYS_move_mount 429
#endif

std::atomic<bool> g_straight_line{false};  // gm_bpf_dev_straight_line: set mode off

std::mutex g_stage_mu;
int g_stage_fd = -1;  // O_PATH dir fd of the staging directory (in the worker's mount namespace)

// 1 if dirfd/leaf is the root of a mount (a bind-mounted node), 0 if not, -errno.
int is_mount_leaf(int dirfd, const std::string& leaf) {
  struct statx sx;
  if (statx(dirfd, leaf.c_str(), AT_SYMLINK_NOFOLLOW | AT_NO_AUTOMOUNT, STATX_BASIC_STATS, &sx) <
      0)
    return -errno;
  if (sx.stx_attributes_mask & STATX_ATTR_MOUNT_ROOT)
    return (sx.stx_attributes & STATX_ATTR_MOUNT_ROOT) ? 1 : 0;
  struct stat dir;  // pre-5.8 kernels: a different filesystem than the directory's
  if (fstat(dirfd, &dir) < 0) return -errno;
  return makedev(sx.stx_dev_major, sx.stx_dev_minor) != dir.st_dev ? 1 : 0;
}

// A detached clone (open_tree) of the staged node for `n`, creating the staged node on first use.
// Must run in the worker's own mount namespace, i.e. before any setns.
int staged_tree(const gm_dev_node_t& n) {
  std::lock_guard<std::mutex> lk(g_stage_mu);
  if (g_stage_fd < 0) return -ENOTCONN;
  char name[96];
  snprintf(name, sizeof(name), "c%u_%u_%o_%d_%d", n.major, n.minor, n.mode & 07777, n.uid, n.gid);
  struct stat st;
  bool ok = fstatat(g_stage_fd, name, &st, AT_SYMLINK_NOFOLLOW) == 0 && S_ISCHR(st.st_mode) &&
            st.st_rdev == makedev(n.major, n.minor) && (st.st_mode & 07777) == (n.mode & 07777);
  if (!ok) {
    if (unlinkat(g_stage_fd, name, 0) < 0 && errno != ENOENT) return -errno;
    // the staging dir is an O_PATH fd: mknodat/fchmodat need a real directory fd
    Fd dir(openat(g_stage_fd, ".", O_RDONLY | O_DIRECTORY | O_CLOEXEC));
    if (!dir.ok()) return -errno;
    if (mknodat(dir.fd, name, S_IFCHR | (n.mode & 07777), makedev(n.major, n.minor)) < 0)
      return -errno;
    if (fchmodat(dir.fd, name, n.mode & 07777, 0) < 0) return -errno;
    if ((n.uid >= 0 || n.gid >= 0) &&
        fchownat(dir.fd, name, (uid_t)n.uid, (gid_t)n.gid, AT_SYMLINK_NOFOLLOW) < 0)
      return -errno;
  }
  long fd = syscall(SYS_open_tree, g_stage_fd, name, OPEN_TREE_CLONE | O_CLOEXEC |
                                                          AT_SYMLINK_NOFOLLOW);
  return fd < 0 ? -errno : (int)fd;
}

// Detaches every mount stacked on dirfd/leaf (the thread's cwd becomes dirfd). 0 or -errno.
int unmount_leaf(int dirfd, const std::string& leaf) {
  if (fchdir(dirfd) < 0) return -errno;
  for (int i = 0; i < 8; ++i) {
    int m = is_mount_leaf(dirfd, leaf);
    if (m <= 0) return m;
    if (umount2(leaf.c_str(), MNT_DETACH | UMOUNT_NOFOLLOW) < 0) return -errno;
  }
  return -EBUSY;
}

// The placeholder a bind mount sits on: an empty regular file.
bool is_placeholder(int dirfd, const std::string& leaf) {
  struct stat st;
  return fstatat(dirfd, leaf.c_str(), &st, AT_SYMLINK_NOFOLLOW) == 0 && S_ISREG(st.st_mode) &&
         st.st_size == 0;
}

int create_bound(Walker& w, const gm_dev_node_t& n, int tree_fd, int flags) {
  int pfd;
  std::string leaf;
  int e = w.parent(n.path, true, &pfd, &leaf);
  if (e != 0) return e;
  if (guarded_dir(pfd)) return kSharedHost;
  int kind;
  uint32_t maj, min, mode;
  e = stat_leaf(pfd, leaf, &kind, &maj, &min, &mode);
  if (e < 0) return e;
  int mounted = kind ? is_mount_leaf(pfd, leaf) : 0;
  if (mounted < 0) return mounted;
  bool same = (kind == 1 || kind == 2) && maj == n.major && min == n.minor;
  if (same && mounted) return 1;  // idempotent re-attach
  if (kind != 0) {
    if (!same && (kind == 1 || kind == 2) && !(flags & GM_DEV_REPLACE)) return -EEXIST;
    if (kind == 3 && (mounted || !is_placeholder(pfd, leaf))) return -EEXIST;
    // a node of ours that cannot be opened (mknod'ed on the nodev /dev), an older mount, or a
    // placeholder left by an interrupted attach: clear it and bind over a fresh placeholder
    if (mounted && (e = unmount_leaf(pfd, leaf)) < 0) return e;
    if (!is_placeholder(pfd, leaf) && unlinkat(pfd, leaf.c_str(), 0) < 0)
      return -errno;
  }
  if (!is_placeholder(pfd, leaf)) {
    int fd = openat(pfd, leaf.c_str(), O_CREAT | O_EXCL | O_WRONLY | O_NOFOLLOW | O_CLOEXEC,
                    0);
    if (fd < 0) return -errno;
    close(fd);
  }
  if (syscall(SYS_move_mount, tree_fd, "", pfd, leaf.c_str(), MOVE_MOUNT_F_EMPTY_PATH) < 0) {
    int err = errno;
    unlinkat(pfd, leaf.c_str(), 0);
    return -err;
  }
  return 0;
}

// Removal that also handles bind-mounted nodes: unmount (if ours), then unlink the placeholder.
int remove_bound(Walker& w, const gm_dev_node_t& n) {
  int pfd;
  std::string leaf;
  int e = w.parent(n.path, false, &pfd, &leaf);
  if (e == -ENOENT) return 1;
  if (e != 0) return e;
  if (guarded_dir(pfd)) return kSharedHost;
  int kind;
  uint32_t maj, min, mode;
  e = stat_leaf(pfd, leaf, &kind, &maj, &min, &mode);
  if (e < 0) return e;
  if (kind == 0) return 1;
  int mounted = is_mount_leaf(pfd, leaf);
  if (mounted < 0) return mounted;
  if (!mounted) {
    if (kind == 3 && is_placeholder(pfd, leaf)) {  // interrupted attach
      if (unlinkat(pfd, leaf.c_str(), 0) < 0) return -errno;
      return 0;
    }
    return remove_one(w, n);
  }
  if (!(kind == 1 && maj == n.major && min == n.minor)) return -EEXIST;
  if ((e = unmount_leaf(pfd, leaf)) < 0) return e;
  if (is_placeholder(pfd, leaf) && unlinkat(pfd, leaf.c_str(), 0) < 0) return -errno;
  return 0;
}

// ------------------------------------------------------------------ roctx
struct Roctx {
  std::once_flag once;
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
  uint64_t (*start)(const char*) = nullptr;
  void (*stop)(uint64_t) = nullptr;
};
Roctx g_roctx;

void roctx_init() {
  std::call_once(g_roctx.once, []() {
    const char* env = getenv("GM_ROCTX");
    if (env && strcmp(env, "0") == 0) return;
    const char* libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                          "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"};
    void* dl = nullptr;
    for (const char* l : libs) {
      dl = dlopen(l, RTLD_NOW | RTLD_GLOBAL);
      if (dl) break;
    }
    if (!dl) return;
    g_roctx.push = reinterpret_cast<int (*)(const char*)>(dlsym(dl, "roctxRangePushA"));
    g_roctx.pop = reinterpret_cast<int (*)()>(dlsym(dl, "roctxRangePop"));
    g_roctx.mark = reinterpret_cast<void (*)(const char*)>(dlsym(dl, "roctxMarkA"));
    g_roctx.start = reinterpret_cast<uint64_t (*)(const char*)>(dlsym(dl, "roctxRangeStartA"));
    g_roctx.stop = reinterpret_cast<void (*)(uint64_t)>(dlsym(dl, "roctxRangeStop"));
  });
}

}  // namespace

extern "C" {

int gm_host_abi_version(void) { return GM_HOST_ABI_VERSION; }

// ------------------------------------------------------------------ cgroup v1
int gm_cg1_format_rule(const gm_dev_rule_t* r, char* out, int cap) {
  char acc[4] = {0};
  int k = 0;
  if (r->access & GM_ACC_READ) acc[k++] = 'r';
  if (r->access & GM_ACC_WRITE) acc[k++] = 'w';
  if (r->access & GM_ACC_MKNOD) acc[k++] = 'm';
  char maj[16], min[16];
  if (r->major < 0) snprintf(maj, sizeof(maj), "*");
  else snprintf(maj, sizeof(maj), "%d", r->major);
  if (r->minor < 0) snprintf(min, sizeof(min), "*");
  else snprintf(min, sizeof(min), "%d", r->minor);
  if (r->type == 'a') return snprintf(out, (size_t)cap, "a");
  return snprintf(out, (size_t)cap, "%c %s:%s %s", r->type, maj, min, acc);
}

int gm_cg1_apply(const char* cgdir, const gm_dev_rule_t* rules, int n) {
  // One open per target file, one write(2) per rule: the kernel parses exactly one rule per write.
  Fd allow_fd, deny_fd;
  std::string base(cgdir);
  for (int i = 0; i < n; ++i) {
    Fd& f = rules[i].allow ? allow_fd : deny_fd;
    if (!f.ok()) {
      std::string p = base + (rules[i].allow ? "/devices.allow" : "/devices.deny");
      int fd = open(p.c_str(), O_WRONLY | O_APPEND | O_CLOEXEC);
      if (fd < 0) return -errno;
      f = Fd(fd);
    }
    char line[64];
    int len = gm_cg1_format_rule(&rules[i], line, sizeof(line) - 1);
    line[len++] = '\n';
    int e = write_all(f.fd, line, (size_t)len);
    if (e < 0) return e;
  }
  return n;
}

// ------------------------------------------------------------------ cgroup v2 eBPF
int gm_bpf_dev_build(const gm_dev_rule_t* rules, int n, int default_allow, int chain_map_fd,
                     uint64_t* out, int cap) {
  if (n < 0 || (n > 0 && !rules)) return -EINVAL;
  int need = 6;  // prologue
  for (int i = 0; i < n; ++i) {
    if (rules[i].type != 'a' && rules[i].type != 'c' && rules[i].type != 'b') return -EINVAL;
    need += rule_block_len(rules[i]);
  }
  if (chain_map_fd != -1) need += 4;  // ld_imm64 (2) + mov r3 + call
  need += 2;                          // default: mov r0 + exit
  if (!out || cap < need) return -need;

  int k = emit_ctx_load(out, 0);
  k = emit_rule_blocks(rules, n, out, k);
  if (k < 0) return k;
  if (chain_map_fd != -1) {
    // r1 still holds ctx. r2 = &prog_array (pseudo map fd), r3 = 0, call bpf_tail_call.
    const int32_t mfd = chain_map_fd >= 0 ? chain_map_fd : 0;
    out[k++] = insn(LD_IMM64, 2, BPF_PSEUDO_MAP_FD, 0, mfd);
    out[k++] = insn(0, 0, 0, 0, 0);
    out[k++] = insn(MOV64_K, 3, 0, 0, 0);
    out[k++] = insn(CALL, 0, 0, 0, BPF_FUNC_tail_call);
  }
  out[k++] = insn(MOV64_K, 0, 0, 0, default_allow ? 1 : 0);
  out[k++] = insn(EXIT, 0, 0, 0, 0);
  return k;
}

int gm_bpf_dev_build_set(int set_map_fd, const gm_dev_rule_t* base, int nbase, int default_allow,
                         int chain_map_fd, uint64_t* out, int cap) {
  if (nbase < 0 || (nbase > 0 && !base)) return -EINVAL;
  int need = 23 + 1;  // lookup + verdict, then r1 = ctx at the miss label
  if (nbase > 0) {
    need += 6;
    for (int i = 0; i < nbase; ++i) need += rule_block_len(base[i]);
  }
  if (chain_map_fd != -1) need += 4;
  need += 2;
  if (!out || cap < need) return -need;
  int k = 0;
  const int32_t smfd = set_map_fd >= 0 ? set_map_fd : 0;
  out[k++] = insn(MOV64_X, 6, 1, 0, 0);           // r6 = ctx (callee-saved)
  out[k++] = insn(LDX_W, 2, 6, 0, 0);             // r2 = access_type
  out[k++] = insn(MOV64_X, 3, 2, 0, 0);
  out[k++] = insn(AND64_K, 3, 0, 0, 0xffff);      // r3 = dev type
  out[k++] = insn(MOV64_X, 7, 2, 0, 0);
  out[k++] = insn(RSH64_K, 7, 0, 0, 16);          // r7 = requested access
  out[k++] = insn(STX_W, 10, 3, -12, 0);          // key.type
  out[k++] = insn(LDX_W, 4, 6, 4, 0);
  out[k++] = insn(STX_W, 10, 4, -8, 0);           // key.major
  out[k++] = insn(LDX_W, 5, 6, 8, 0);
  out[k++] = insn(STX_W, 10, 5, -4, 0);           // key.minor
  out[k++] = insn(LD_IMM64, 1, BPF_PSEUDO_MAP_FD, 0, smfd);
  out[k++] = insn(0, 0, 0, 0, 0);
  out[k++] = insn(MOV64_X, 2, 10, 0, 0);
  out[k++] = insn(ADD64_K, 2, 0, 0, -12);         // r2 = &key
  out[k++] = insn(CALL, 0, 0, 0, BPF_FUNC_map_lookup_elem);
  const int miss = 23;
  out[k] = insn(JEQ_K, 0, 0, (int16_t)(miss - (k + 1)), 0);  // not in the set
  ++k;
  out[k++] = insn(LDX_W, 1, 0, 0, 0);             // r1 = allowed access
  out[k++] = insn(XOR64_K, 1, 0, 0, -1);
  out[k++] = insn(BPF_ALU64 | BPF_AND | BPF_X, 1, 7, 0, 0);  // requested & ~allowed
  out[k] = insn(JNE_K, 1, 0, (int16_t)(miss - (k + 1)), 0);
  ++k;
  out[k++] = insn(MOV64_K, 0, 0, 0, 1);
  out[k++] = insn(EXIT, 0, 0, 0, 0);
  if (k != miss) return -EINVAL;
  out[k++] = insn(MOV64_X, 1, 6, 0, 0);           // r1 = ctx again
  if (nbase > 0) {  // chain lost: the runtime's default list, compiled in
    k = emit_ctx_load(out, k);
    k = emit_rule_blocks(base, nbase, out, k);
    if (k < 0) return k;
  }
  if (chain_map_fd != -1) {
    const int32_t mfd = chain_map_fd >= 0 ? chain_map_fd : 0;
    out[k++] = insn(LD_IMM64, 2, BPF_PSEUDO_MAP_FD, 0, mfd);
    out[k++] = insn(0, 0, 0, 0, 0);
    out[k++] = insn(MOV64_K, 3, 0, 0, 0);
    out[k++] = insn(CALL, 0, 0, 0, BPF_FUNC_tail_call);
  }
  out[k++] = insn(MOV64_K, 0, 0, 0, default_allow ? 1 : 0);
  out[k++] = insn(EXIT, 0, 0, 0, 0);
  return k;
}

int gm_bpf_dev_load(const uint64_t* insns, int n, const char* name, char* log, int logcap) {
  union bpf_attr a;
  memset(&a, 0, sizeof(a));
  a.prog_type = BPF_PROG_TYPE_CGROUP_DEVICE;
  a.expected_attach_type = BPF_CGROUP_DEVICE;
  a.insns = ptr_u64(insns);
  a.insn_cnt = (uint32_t)n;
  a.license = ptr_u64("Apache-2.0");
  snprintf(a.prog_name, sizeof(a.prog_name), "%s", name && *name ? name : kProgName);
  if (log && logcap > 0) {
    log[0] = 0;
    a.log_buf = ptr_u64(log);
    a.log_size = (uint32_t)logcap;
    a.log_level = 1;
  }
  long fd = sys_bpf(BPF_PROG_LOAD, &a, sizeof(a));
  if (fd < 0 && log && logcap > 0 && errno != EINVAL && errno != EACCES) {
    // retry without a log buffer (some kernels reject small logs with ENOSPC)
    a.log_buf = 0;
    a.log_size = 0;
    a.log_level = 0;
    fd = sys_bpf(BPF_PROG_LOAD, &a, sizeof(a));
  }
  return fd < 0 ? -errno : (int)fd;
}

int gm_bpf_dev_query(const char* cgroup_path, uint32_t* ids, uint32_t cap, uint32_t* n,
                     uint32_t* attach_flags) {
  Fd cg(open(cgroup_path, O_RDONLY | O_DIRECTORY | O_CLOEXEC));
  if (!cg.ok()) return -errno;
  Attached at;
  int e = query(cg.fd, &at);
  if (e < 0) return e;
  *n = (uint32_t)at.ids.size();
  if (attach_flags) *attach_flags = at.flags;
  for (uint32_t i = 0; i < at.ids.size() && i < cap; ++i) ids[i] = at.ids[i];
  return 0;
}

int gm_bpf_prog_name(uint32_t id, char* name, int cap) {
  Fd pfd(get_prog_fd_by_id(id));
  if (!pfd.ok()) return pfd.fd;
  struct bpf_prog_info info;
  uint32_t maps[1];
  int e = prog_info(pfd.fd, &info, maps, 0);
  if (e < 0) return e;
  snprintf(name, (size_t)cap, "%.*s", (int)sizeof(info.name), info.name);
  return 0;
}

int gm_bpf_dev_program_at(const char* cgroup_path, uint32_t index, int foreign_only,
                          uint64_t* insns, uint32_t cap, uint32_t* n, uint32_t* prog_id,
                          uint32_t* foreign) {
  *n = 0;
  if (prog_id) *prog_id = 0;
  if (foreign) *foreign = 0;
  Fd cg(open(cgroup_path, O_RDONLY | O_DIRECTORY | O_CLOEXEC));
  if (!cg.ok()) return -errno;
  Attached at;
  int e = query(cg.fd, &at);
  if (e < 0) return e;
  uint32_t k = 0;
  int found = -1;
  for (uint32_t id : at.ids) {
    const bool ours = is_ours(id, nullptr);
    if (!ours && foreign) ++*foreign;
    if (ours == (foreign_only != 0)) continue;
    if (k++ == index && found < 0) found = (int)id;
  }
  if (found < 0) return 0;
  const uint32_t id = (uint32_t)found;
  Fd pfd(get_prog_fd_by_id(id));
  if (!pfd.ok()) return pfd.fd;
  struct bpf_prog_info info;
  union bpf_attr a;
  memset(&info, 0, sizeof(info));
  memset(&a, 0, sizeof(a));
  a.info.bpf_fd = (uint32_t)pfd.fd;
  a.info.info_len = sizeof(info);
  a.info.info = ptr_u64(&info);
  if (sys_bpf(BPF_OBJ_GET_INFO_BY_FD, &a, sizeof(a)) < 0) return -errno;
  if (prog_id) *prog_id = id;
  const uint32_t need = info.xlated_prog_len / 8;
  if (need == 0) return -EPERM;  // !bpf_capable(): the kernel reports no instructions
  *n = need;
  if (need > cap || insns == nullptr) return -ENOSPC;
  memset(&info, 0, sizeof(info));
  info.xlated_prog_len = need * 8;
  info.xlated_prog_insns = ptr_u64(insns);
  memset(&a, 0, sizeof(a));
  a.info.bpf_fd = (uint32_t)pfd.fd;
  a.info.info_len = sizeof(info);
  a.info.info = ptr_u64(&info);
  if (sys_bpf(BPF_OBJ_GET_INFO_BY_FD, &a, sizeof(a)) < 0) return -errno;
  return 0;
}

int gm_bpf_dev_program(const char* cgroup_path, uint64_t* insns, uint32_t cap, uint32_t* n,
                       uint32_t* prog_id) {
  return gm_bpf_dev_program_at(cgroup_path, 0, 0, insns, cap, n, prog_id, nullptr);
}

namespace {
thread_local gm_bpf_timing_t t_bpf_timing;
uint64_t mono_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
}  // namespace

void gm_bpf_dev_last_timing(gm_bpf_timing_t* out) {
  if (out) *out = t_bpf_timing;
}

int gm_bpf_dev_install(const char* cgroup_path, const gm_dev_rule_t* rules, int n,
                       const gm_dev_rule_t* base, int nbase, const char* pin_dir,
                       uint32_t* prog_id, uint32_t* chained_id) {
  gm_bpf_timing_t& tm = t_bpf_timing;
  tm = gm_bpf_timing_t{};
  uint64_t t0 = mono_ns();
  Fd cg(open(cgroup_path, O_RDONLY | O_DIRECTORY | O_CLOEXEC));
  if (!cg.ok()) return -errno;
  const uint64_t ino = cgroup_ino(cg.fd);
  Attached at;
  int e = query(cg.fd, &at);
  if (e < 0) return e;
  uint64_t t1 = mono_ns();
  tm.query_ns += t1 - t0;

  // One slot per attached program. Under BPF_F_ALLOW_MULTI every program must allow an access,
  // so each one is wrapped: ours (rules → allow, else tail-call the original). With nothing
  // attached, one slot with default-allow (the cgroup was unrestricted).
  //
  // Set mode (exact allow rules, the attach path): the rules live in a HASH map the program
  // looks up, shared by every wrapper of the cgroup. Once wrapped, an attach or detach is a
  // map update — no program load, verification or attach — and the verifier sees the same
  // short program whatever the number of GPUs. A straight-line program of ours (older worker,
  // or rules a set cannot hold) is replaced.
  const bool set_mode = set_eligible(rules, n) && !g_straight_line.load(std::memory_order_relaxed);
  struct Slot {
    uint32_t replace_id = 0, chain_id = 0, set_id = 0;
    bool ours = false, ours_without_chain = false, chain_lost = false;
  };
  std::vector<Slot> slots;
  for (uint32_t id : at.ids) {
    Slot sl;
    uint32_t c = 0, m = 0;
    bool has_chain = false;
    sl.replace_id = id;
    if (is_ours(id, &c, &m, &has_chain)) {
      sl.ours = true;
      sl.chain_id = c;
      sl.set_id = m;
      sl.ours_without_chain = (c == 0);
      // its PROG_ARRAY slot is empty: the map was neither pinned nor held open (a restart
      // without bpffs), so the tail call to the runtime's program now falls through
      sl.chain_lost = has_chain && c == 0;
    } else {
      sl.chain_id = id;
    }
    slots.push_back(sl);
  }
  if (slots.empty()) slots.push_back(Slot{});
  if (slots.size() > 1 && !(at.flags & BPF_F_ALLOW_MULTI)) return -EINVAL;  // impossible state

  std::vector<uint32_t> chains;
  Fd set_map;
  if (set_mode) {
    // the cgroup's set: the one our programs already look up (a later one would be a leftover
    // of a partial install and is re-synced too), else a new one
    for (const Slot& sl : slots)
      if (sl.set_id && !set_map.ok()) set_map = Fd(map_fd_by_id(sl.set_id));
    if (!set_map.ok()) set_map = Fd(make_set_map());
    if (!set_map.ok()) return set_map.fd;
    if ((e = sync_set(set_map.fd, rules, n)) < 0) return e;
    struct bpf_map_info mi;
    const uint32_t chosen = map_info(set_map.fd, &mi) == 0 ? mi.id : 0;
    for (const Slot& sl : slots) {
      if (sl.set_id && sl.set_id != chosen) {
        Fd other(map_fd_by_id(sl.set_id));
        if (other.ok() && (e = sync_set(other.fd, rules, n)) < 0) return e;
      }
    }
  }
  uint64_t t2 = mono_ns();
  tm.map_ns += t2 - t1;

  uint32_t first_prog = 0;
  for (const Slot& sl : slots) {
    if (set_mode && sl.set_id && !sl.chain_lost) {  // a set-mode wrapper: the sync installed
      if (sl.chain_id) chains.push_back(sl.chain_id);
      if (!first_prog) first_prog = sl.replace_id;
      continue;
    }
    Fd chain_prog, chain_map, replace_fd;
    t0 = mono_ns();
    if (sl.chain_id) {
      chain_prog = Fd(get_prog_fd_by_id(sl.chain_id));
      if (!chain_prog.ok()) return chain_prog.fd;
      chain_map = Fd(make_chain_map(chain_prog.fd));
      if (!chain_map.ok()) return chain_map.fd;
    }
    if (sl.replace_id) {
      replace_fd = Fd(get_prog_fd_by_id(sl.replace_id));
      if (!replace_fd.ok()) return replace_fd.fd;
    }
    // With a chained original (or a compiled-in base list) the fall-through is deny; with
    // neither the cgroup was unrestricted, so default-allow keeps that behaviour.
    const int default_allow = (sl.chain_id || sl.ours_without_chain) ? 0 : 1;
    const gm_dev_rule_t* b = sl.ours_without_chain ? base : nullptr;
    const int nb = sl.ours_without_chain && base ? nbase : 0;
    t1 = mono_ns();
    tm.map_ns += t1 - t0;
    std::vector<uint64_t> prog(48 + (n + nb) * 12);
    int cnt;
    if (set_mode) {
      cnt = gm_bpf_dev_build_set(set_map.fd, b, nb, default_allow,
                                 chain_map.ok() ? chain_map.fd : -1, prog.data(), (int)prog.size());
    } else {
      // rules = ours, then (chain lost) the runtime's default list compiled in
      std::vector<gm_dev_rule_t> all(rules, rules + n);
      if (nb) all.insert(all.end(), b, b + nb);
      cnt = gm_bpf_dev_build(all.data(), (int)all.size(), default_allow,
                             chain_map.ok() ? chain_map.fd : -1, prog.data(), (int)prog.size());
    }
    if (cnt < 0) return -EINVAL;
    t2 = mono_ns();
    tm.build_ns += t2 - t1;
    // No verifier log on the hot path: log_level 1 makes the verifier print every instruction
    // of every explored path, which costs more than the verification itself. The program is
    // generated, so a rejection is a bug; gm_bpf_dev_load with a log buffer reproduces it.
    Fd pfd(gm_bpf_dev_load(prog.data(), cnt, kProgName, nullptr, 0));
    if (!pfd.ok()) return pfd.fd;
    uint64_t t3 = mono_ns();
    tm.load_ns += t3 - t2;
    tm.insns += (uint32_t)cnt;
    if (chain_map.ok()) {
      e = keep_map(pin_dir, ino, sl.chain_id, chain_map.fd);
      if (e < 0) return e;
      chains.push_back(sl.chain_id);
    }
    uint64_t t4 = mono_ns();
    tm.map_ns += t4 - t3;
    e = attach(cg.fd, pfd.fd, replace_fd.ok() ? replace_fd.fd : -1,
               at.ids.empty() ? BPF_F_ALLOW_MULTI : at.flags);
    if (e < 0) return e;
    tm.attach_ns += mono_ns() - t4;
    ++tm.programs;
    if (!first_prog) {
      struct bpf_prog_info info;
      uint32_t maps[1];
      first_prog = prog_info(pfd.fd, &info, maps, 0) == 0 ? info.id : 0;
    }
  }
  drop_maps_except(pin_dir, ino, chains);
  if (prog_id) *prog_id = first_prog;
  if (chained_id) *chained_id = slots[0].chain_id;
  return (int)slots.size();
}

void gm_bpf_dev_straight_line(int on) { g_straight_line.store(on != 0); }

int gm_bpf_dev_probe_set(void) {
  Fd m(make_set_map());
  if (!m.ok()) return m.fd;
  uint64_t prog[64];
  int cnt = gm_bpf_dev_build_set(m.fd, nullptr, 0, 1, -1, prog, 64);
  if (cnt < 0) return -EINVAL;
  Fd p(gm_bpf_dev_load(prog, cnt, "gm_doctor", nullptr, 0));
  return p.ok() ? 0 : p.fd;
}

int gm_bpf_dev_set_at(const char* cgroup_path, uint32_t index, uint32_t* entries, uint32_t cap,
                      uint32_t* n, uint32_t* prog_id) {
  *n = 0;
  if (prog_id) *prog_id = 0;
  Fd cg(open(cgroup_path, O_RDONLY | O_DIRECTORY | O_CLOEXEC));
  if (!cg.ok()) return -errno;
  Attached at;
  int e = query(cg.fd, &at);
  if (e < 0) return e;
  uint32_t k = 0;
  for (uint32_t id : at.ids) {
    uint32_t set_id = 0;
    if (!is_ours(id, nullptr, &set_id)) continue;
    if (k++ != index) continue;
    if (prog_id) *prog_id = id;
    if (!set_id) return 0;  // a straight-line program: read its xlated code instead
    Fd m(map_fd_by_id(set_id));
    if (!m.ok()) return m.fd;
    std::vector<std::pair<SetKey, uint32_t>> all;
    if ((e = set_entries(m.fd, &all)) < 0) return e;
    uint32_t out = 0;
    for (const auto& kv : all) {
      if (out < cap && entries) {
        entries[out * 4 + 0] = kv.first.type;
        entries[out * 4 + 1] = kv.first.major;
        entries[out * 4 + 2] = kv.first.minor;
        entries[out * 4 + 3] = kv.second;
      }
      ++out;
    }
    *n = out;
    return out > cap ? -ENOSPC : 1;
  }
  return -ENOENT;
}

int gm_bpf_dev_restore(const char* cgroup_path, const char* pin_dir) {
  Fd cg(open(cgroup_path, O_RDONLY | O_DIRECTORY | O_CLOEXEC));
  if (!cg.ok()) return -errno;
  const uint64_t ino = cgroup_ino(cg.fd);
  Attached at;
  int e = query(cg.fd, &at);
  if (e < 0) return e;
  int restored = 0;
  for (uint32_t id : at.ids) {
    uint32_t chain = 0;
    if (!is_ours(id, &chain)) continue;
    Fd ours(get_prog_fd_by_id(id));
    if (!ours.ok()) return ours.fd;
    if (chain) {
      Fd orig(get_prog_fd_by_id(chain));
      if (!orig.ok()) return orig.fd;
      e = attach(cg.fd, orig.fd, ours.fd, at.flags);
    } else {
      union bpf_attr a;
      memset(&a, 0, sizeof(a));
      a.target_fd = (uint32_t)cg.fd;
      a.attach_bpf_fd = (uint32_t)ours.fd;
      a.attach_type = BPF_CGROUP_DEVICE;
      e = sys_bpf(BPF_PROG_DETACH, &a, sizeof(a)) < 0 ? -errno : 0;
    }
    if (e < 0) return e;
    ++restored;
  }
  drop_maps_except(pin_dir, ino, {});
  return restored;
}

// ------------------------------------------------------------------ device nodes
int gm_devnodes_guard(const char* host_dev) {
  for (auto& g : g_guard) g.ino.store(0, std::memory_order_release);
  if (!host_dev || !*host_dev) return 0;
  int set = 0;
  const std::string base(host_dev);
  const std::string dirs[2] = {base, base + "/dri"};
  for (int i = 0; i < 2; ++i) {
    struct stat st;
    if (stat(dirs[i].c_str(), &st) < 0 || !S_ISDIR(st.st_mode)) {
      if (i == 0) return -(errno ? errno : ENOTDIR);
      continue;  // a host without /dev/dri (no GPU driver loaded) guards /dev alone
    }
    g_guard[i].dev.store(st.st_dev, std::memory_order_relaxed);
    g_guard[i].ino.store(st.st_ino, std::memory_order_release);
    ++set;
  }
  return set;
}

int gm_devnodes_bind_probe(void) {
  long fd = syscall(SYS_open_tree, AT_FDCWD, "/", OPEN_TREE_CLONE | O_CLOEXEC);
  if (fd < 0) return -errno;
  close((int)fd);
  return 0;
}

int gm_devnodes_stage(const char* dir, int mount_tmpfs) {
  std::lock_guard<std::mutex> lk(g_stage_mu);
  if (g_stage_fd >= 0) close(g_stage_fd);
  g_stage_fd = -1;
  if (!dir || !*dir) return 0;
  if (mkdir(dir, 0711) < 0 && errno != EEXIST) return -errno;
  if (mount_tmpfs) {
    Fd d(open(dir, O_PATH | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC));
    if (!d.ok()) return -errno;
    std::string up = std::string(dir) + "/..";
    struct stat self, parent;
    if (fstat(d.fd, &self) < 0 || stat(up.c_str(), &parent) < 0) return -errno;
    if (self.st_dev == parent.st_dev &&  // not mounted yet (a restarted worker reuses its own)
        mount("gm-devstage", dir, "tmpfs", MS_NOSUID | MS_NOEXEC, "mode=0711") < 0)
      return -errno;
  }
  int fd = open(dir, O_PATH | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC);
  if (fd < 0) return -errno;
  g_stage_fd = fd;
  return 0;
}

int gm_devnodes_create(int pid, const char* root, const gm_dev_node_t* nodes, int n, int flags,
                       int* results) {
  int failures = 0;
  std::vector<Fd> trees;
  if (flags & GM_DEV_BIND) {  // clone the staged nodes while still in our own mount namespace
    for (int i = 0; i < n; ++i) {
      int t = staged_tree(nodes[i]);
      if (t < 0) {
        for (int j = 0; j < n; ++j) results[j] = t;
        return n;
      }
      trees.emplace_back(t);
    }
  }
  int e = with_root(pid, root, flags, [&](int rootfd) {
    Walker w(rootfd);
    for (int i = 0; i < n; ++i) {
      results[i] = (flags & GM_DEV_BIND) ? create_bound(w, nodes[i], trees[i].fd, flags)
                                         : create_one(w, nodes[i], flags);
      if (results[i] < 0) ++failures;
    }
    return 0;
  });
  if (e < 0) {
    for (int i = 0; i < n; ++i) results[i] = e;
    return n;
  }
  return failures;
}

int gm_devnodes_remove(int pid, const char* root, const gm_dev_node_t* nodes, int n, int flags,
                       int* results) {
  int failures = 0;
  int e = with_root(pid, root, flags, [&](int rootfd) {
    Walker w(rootfd);
    for (int i = 0; i < n; ++i) {
      results[i] = (flags & GM_DEV_BIND) ? remove_bound(w, nodes[i]) : remove_one(w, nodes[i]);
      if (results[i] < 0) ++failures;
    }
    return 0;
  });
  if (e < 0) {
    for (int i = 0; i < n; ++i) results[i] = e;
    return n;
  }
  return failures;
}

int gm_devnode_stat(int pid, const char* root, const char* path, int flags, int* kind,
                    uint32_t* maj, uint32_t* min, uint32_t* mode) {
  return with_root(pid, root, flags, [&](int rootfd) {
    Fd parent;
    std::string leaf;
    int e = walk_parent(rootfd, path, false, &parent, &leaf);
    if (e == -ENOENT) {
      *kind = 0;
      *maj = *min = *mode = 0;
      return 0;
    }
    if (e < 0) return e;
    return stat_leaf(parent.fd, leaf, kind, maj, min, mode);
  });
}

int gm_devnodes_present(int pid, const char* root, const gm_dev_node_t* nodes, int n, int flags,
                        uint8_t* present) {
  int count = 0;
  int e = with_root(pid, root, flags, [&](int rootfd) {
    Walker wk(rootfd);
    for (int i = 0; i < n; ++i) {
      present[i] = 0;
      int pfd;
      std::string leaf;
      int w = wk.parent(nodes[i].path, false, &pfd, &leaf);
      if (w == -ENOENT) {
        // a missing directory inside the host's /dev is one create_one would not make either
        std::string dir(nodes[i].path);
        const size_t cut = dir.rfind('/');
        dir = cut == std::string::npos ? std::string() : dir.substr(0, cut);
        Fd d2;
        std::string l2;
        if (!dir.empty() && walk_parent(rootfd, dir.c_str(), false, &d2, &l2) == 0 &&
            guarded_dir(d2.fd)) {
          present[i] = kSharedHost;
          ++count;
        }
        continue;
      }
      if (w < 0) continue;
      if (guarded_dir(pfd)) {  // the host's own /dev: not gpumounter's to provide
        present[i] = kSharedHost;
        ++count;
        continue;
      }
      int kind = 0;
      uint32_t ma = 0, mi = 0, mode = 0;
      if (stat_leaf(pfd, leaf, &kind, &ma, &mi, &mode) < 0) continue;
      if ((kind == 1 || kind == 2) && ma == nodes[i].major && mi == nodes[i].minor &&
          (!(flags & GM_DEV_BIND) || is_mount_leaf(pfd, leaf) == 1)) {
        present[i] = 1;
        ++count;
      }
    }
    return 0;
  });
  return e < 0 ? e : count;
}

// ------------------------------------------------------------------ processes
namespace {
bool pid_uses_dev(long pid, dev_t want) {
  char p[64];
  snprintf(p, sizeof(p), "/proc/%ld/fd", pid);
  int dfd = open(p, O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (dfd < 0) return false;
  DIR* fds = fdopendir(dfd);
  if (!fds) {
    close(dfd);
    return false;
  }
  struct dirent* fe;
  bool hit = false;
  while (!hit && (fe = readdir(fds)) != nullptr) {
    if (fe->d_name[0] == '.') continue;
    struct stat st;
    if (fstatat(dirfd(fds), fe->d_name, &st, 0) == 0 && S_ISCHR(st.st_mode) && st.st_rdev == want)
      hit = true;
  }
  closedir(fds);
  return hit;
}
// 1 = fd table read, 0 = process gone, -1 = not readable (permission).
int pid_scan_devs(long pid, const dev_t* want, int ndev, uint8_t* hits) {
  char p[64];
  snprintf(p, sizeof(p), "/proc/%ld/fd", pid);
  int dfd = open(p, O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (dfd < 0) return errno == ENOENT || errno == ESRCH ? 0 : -1;
  DIR* fds = fdopendir(dfd);
  if (!fds) {
    close(dfd);
    return -1;
  }
  struct dirent* fe;
  while ((fe = readdir(fds)) != nullptr) {
    if (fe->d_name[0] == '.') continue;
    struct stat st;
    if (fstatat(dirfd(fds), fe->d_name, &st, 0) != 0 || !S_ISCHR(st.st_mode)) continue;
    for (int j = 0; j < ndev; ++j)
      if (st.st_rdev == want[j]) hits[j] = 1;
  }
  closedir(fds);
  return 1;
}
}  // namespace

int gm_proc_scan_devs(const int32_t* pids, int n, const uint32_t* majmin, int ndev,
                      uint8_t* hits, int32_t* unreadable) {
  if (n < 0 || ndev < 0 || ndev > 256) return -EINVAL;
  dev_t want[256];
  for (int j = 0; j < ndev; ++j) want[j] = makedev(majmin[2 * j], majmin[2 * j + 1]);
  memset(hits, 0, (size_t)n * (size_t)ndev);
  int bad = 0;
  for (int i = 0; i < n; ++i)
    if (pid_scan_devs(pids[i], want, ndev, hits + (size_t)i * ndev) < 0) unreadable[bad++] = pids[i];
  return bad;
}

int gm_proc_filter_dev_users(const int32_t* pids, int n, uint32_t maj, uint32_t min,
                             int32_t* out) {
  const dev_t want = makedev(maj, min);
  int k = 0;
  for (int i = 0; i < n; ++i)
    if (pid_uses_dev(pids[i], want)) out[k++] = pids[i];
  return k;
}

int gm_proc_dev_users(uint32_t maj, uint32_t min, int32_t* pids, int cap, int* n) {
  *n = 0;
  DIR* proc = opendir("/proc");
  if (!proc) return -errno;
  const dev_t want = makedev(maj, min);
  struct dirent* de;
  while ((de = readdir(proc)) != nullptr) {
    char* endp = nullptr;
    long pid = strtol(de->d_name, &endp, 10);
    if (!endp || *endp != 0 || pid <= 0) continue;
    const bool hit = pid_uses_dev(pid, want);
    if (hit) {
      if (*n < cap) pids[*n] = (int32_t)pid;
      ++*n;
    }
  }
  closedir(proc);
  return 0;
}

int gm_proc_read_pids(const char* path, int32_t* pids, int cap, int* n) {
  *n = 0;
  FILE* f = fopen(path, "re");
  if (!f) return -errno;
  long v;
  while (fscanf(f, "%ld", &v) == 1) {
    if (*n < cap) pids[*n] = (int32_t)v;
    ++*n;
  }
  fclose(f);
  return 0;
}

// ------------------------------------------------------------------ tracing
int gm_roctx_available(void) {
  roctx_init();
  return g_roctx.push != nullptr;
}
void gm_roctx_push(const char* name) {
  roctx_init();
  if (g_roctx.push) g_roctx.push(name);
}
void gm_roctx_pop(void) {
  roctx_init();
  if (g_roctx.pop) g_roctx.pop();
}
uint64_t gm_roctx_start(const char* name) {
  roctx_init();
  return g_roctx.start ? g_roctx.start(name) : 0;
}
void gm_roctx_stop(uint64_t id) {
  roctx_init();
  if (g_roctx.stop && id) g_roctx.stop(id);
}
void gm_roctx_mark(const char* name) {
  roctx_init();
  if (g_roctx.mark) g_roctx.mark(name);
}
uint64_t gm_now_ns(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

}  // extern "C"
