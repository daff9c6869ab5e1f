// test_native.cpp — host-side unit tests for gm_host / gm_smi, built with ASan+UBSan
// (native/Makefile `make check`; driven from tests/test_native_sanitized.py).
// Covers: rule formatting, eBPF program layout (block lengths, jump targets), device-node
// create/idempotence/remove/refuse-to-clobber under a temp root, pid-file parsing, and the amdsmi
// shim against the mock library (GM_MOCK_LIB).
#include <errno.h>
#include <linux/bpf.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "gm_host.h"
#include "gm_smi.h"

static int g_fail = 0;
#define EXPECT(c)                                                 \
  do {                                                            \
    if (!(c)) {                                                   \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                   \
    }                                                             \
  } while (0)

static void test_format() {
  gm_dev_rule_t r{'c', GM_ACC_READ | GM_ACC_WRITE, 1, 0, 226, 128};
  char buf[64];
  gm_cg1_format_rule(&r, buf, sizeof(buf));
  EXPECT(std::string(buf) == "c 226:128 rw");
  gm_dev_rule_t w{'c', GM_ACC_MKNOD, 1, 0, -1, -1};
  gm_cg1_format_rule(&w, buf, sizeof(buf));
  EXPECT(std::string(buf) == "c *:* m");
}

static void test_bpf_layout() {
  gm_dev_rule_t rules[3] = {{'c', GM_ACC_READ | GM_ACC_WRITE, 1, 0, 226, 128},
                            {'c', 7, 1, 0, 511, 0},
                            {'a', GM_ACC_MKNOD, 1, 0, -1, -1}};
  int need = gm_bpf_dev_build(rules, 3, 0, -2, nullptr, 0);
  EXPECT(need < 0);
  std::vector<uint64_t> prog(-need);
  int n = gm_bpf_dev_build(rules, 3, 0, -2, prog.data(), (int)prog.size());
  EXPECT(n == -need);
  // every jump must land inside the program
  for (int i = 0; i < n; ++i) {
    struct bpf_insn in;
    memcpy(&in, &prog[i], 8);
    if ((in.code & 0x07) == BPF_JMP && (in.code & 0xf0) == BPF_JNE) {
      const int tgt = i + 1 + in.off;
      EXPECT(tgt > i && tgt < n);
    }
  }
  struct bpf_insn last;
  memcpy(&last, &prog[n - 1], 8);
  EXPECT(last.code == (BPF_JMP | BPF_EXIT));
  EXPECT(gm_bpf_dev_build(rules, -1, 0, -1, prog.data(), (int)prog.size()) == -EINVAL);
}

static void test_devnodes() {
  char tmpl[] = "/tmp/gm_native_XXXXXX";
  char* root = mkdtemp(tmpl);
  EXPECT(root != nullptr);
  gm_dev_node_t nodes[2];
  memset(nodes, 0, sizeof(nodes));
  snprintf(nodes[0].path, sizeof(nodes[0].path), "dev/kfd");
  nodes[0].major = 511;
  nodes[0].minor = 0;
  nodes[0].mode = 0666;
  nodes[0].uid = nodes[0].gid = -1;
  snprintf(nodes[1].path, sizeof(nodes[1].path), "dev/dri/renderD128");
  nodes[1].major = 226;
  nodes[1].minor = 128;
  nodes[1].mode = 0666;
  nodes[1].uid = nodes[1].gid = -1;
  int res[2] = {9, 9};
  EXPECT(gm_devnodes_create(0, root, nodes, 2, GM_DEV_EMULATE, res) == 0);
  EXPECT(res[0] == 0 && res[1] == 0);
  EXPECT(gm_devnodes_create(0, root, nodes, 2, GM_DEV_EMULATE, res) == 0);
  EXPECT(res[0] == 1 && res[1] == 1);  // idempotent
  int kind = -1;
  uint32_t ma = 0, mi = 0, mode = 0;
  EXPECT(gm_devnode_stat(0, root, "dev/dri/renderD128", 0, &kind, &ma, &mi, &mode) == 0);
  EXPECT((kind == 1 || kind == 2) && ma == 226 && mi == 128 && mode == 0666);
  // batch read-back: both present; a wrong minor or a missing node reads as absent
  gm_dev_node_t probe[4] = {nodes[0], nodes[1], nodes[1], nodes[1]};
  probe[2].minor = 200;
  snprintf(probe[3].path, sizeof(probe[3].path), "dev/dri/renderD200");
  uint8_t present[4] = {9, 9, 9, 9};
  EXPECT(gm_devnodes_present(0, root, probe, 4, GM_DEV_EMULATE, present) == 2);
  EXPECT(present[0] == 1 && present[1] == 1 && present[2] == 0 && present[3] == 0);
  EXPECT(gm_devnodes_present(0, "/nonexistent/gm/root", probe, 1, 0, present) == -ENOENT);
  // path escape attempts are refused
  gm_dev_node_t bad = nodes[0];
  snprintf(bad.path, sizeof(bad.path), "dev/../../etc/evil");
  int rb = 0;
  gm_devnodes_create(0, root, &bad, 1, GM_DEV_EMULATE, &rb);
  EXPECT(rb == -EINVAL);
  // a different device at the same path is not clobbered without GM_DEV_REPLACE
  gm_dev_node_t other = nodes[1];
  other.minor = 129;
  int ro = 0;
  gm_devnodes_create(0, root, &other, 1, GM_DEV_EMULATE, &ro);
  EXPECT(ro == -EEXIST);
  int rr = 0;
  gm_devnodes_remove(0, root, &other, 1, 0, &rr);
  EXPECT(rr == -EEXIST);  // removal refuses a mismatching node
  EXPECT(gm_devnodes_remove(0, root, nodes, 2, 0, res) == 0);
  EXPECT(res[0] == 0 && res[1] == 0);
  EXPECT(gm_devnodes_remove(0, root, nodes, 2, 0, res) == 0);
  EXPECT(res[0] == 1 && res[1] == 1);
  std::string cmd = std::string("rm -rf ") + root;
  EXPECT(system(cmd.c_str()) == 0);
}

// A root whose dev/ is the registered host /dev: nothing is created or unlinked there (result 2),
// including under a missing dev/dri (no mkdir inside the host's /dev).
static void test_devnodes_guard() {
  char tmpl[] = "/tmp/gm_guard_XXXXXX";
  char* root = mkdtemp(tmpl);
  EXPECT(root != nullptr);
  std::string dev = std::string(root) + "/dev";
  EXPECT(mkdir(dev.c_str(), 0755) == 0);
  EXPECT(gm_devnodes_guard(dev.c_str()) == 1);  // no dri/ yet: /dev alone
  gm_dev_node_t n[2];
  memset(n, 0, sizeof(n));
  snprintf(n[0].path, sizeof(n[0].path), "dev/kfd");
  n[0].major = 511;
  n[0].mode = 0666;
  n[0].uid = n[0].gid = -1;
  snprintf(n[1].path, sizeof(n[1].path), "dev/dri/renderD129");
  n[1].major = 226;
  n[1].minor = 129;
  n[1].mode = 0666;
  n[1].uid = n[1].gid = -1;
  int res[2] = {9, 9};
  EXPECT(gm_devnodes_create(0, root, n, 2, GM_DEV_EMULATE, res) == 0);
  EXPECT(res[0] == 2 && res[1] == 2);
  uint8_t present[2] = {9, 9};  // the host's /dev is not ours to provide: reads as shared
  EXPECT(gm_devnodes_present(0, root, n, 2, GM_DEV_EMULATE, present) == 2);
  EXPECT(present[0] == 2 && present[1] == 2);
  struct stat st;
  EXPECT(stat((dev + "/kfd").c_str(), &st) < 0 && stat((dev + "/dri").c_str(), &st) < 0);
  // nodes that exist in the host dir are never unlinked through a container sharing it
  EXPECT(gm_devnodes_guard(nullptr) == 0);
  EXPECT(gm_devnodes_create(0, root, n, 2, GM_DEV_EMULATE, res) == 0);
  EXPECT(res[0] == 0 && res[1] == 0);
  EXPECT(gm_devnodes_guard(dev.c_str()) == 2);  // now /dev and /dev/dri
  EXPECT(gm_devnodes_remove(0, root, n, 2, 0, res) == 0);
  EXPECT(res[0] == 2 && res[1] == 2);
  EXPECT(stat((dev + "/kfd").c_str(), &st) == 0 && stat((dev + "/dri/renderD129").c_str(), &st) == 0);
  EXPECT(gm_devnodes_guard("/nonexistent/gm/dev") == -ENOENT);
  EXPECT(gm_devnodes_guard("") == 0);
  EXPECT(gm_devnodes_remove(0, root, n, 2, 0, res) == 0);
  EXPECT(res[0] == 0 && res[1] == 0);
  std::string cmd = std::string("rm -rf ") + root;
  EXPECT(system(cmd.c_str()) == 0);
}

static void test_pids() {
  char path[] = "/tmp/gm_pids_XXXXXX";
  int fd = mkstemp(path);
  EXPECT(fd >= 0);
  const char* body = "12\n345\n6789\n";
  EXPECT(write(fd, body, strlen(body)) == (ssize_t)strlen(body));
  close(fd);
  int32_t pids[2];
  int n = 0;
  EXPECT(gm_proc_read_pids(path, pids, 2, &n) == 0);
  EXPECT(n == 3 && pids[0] == 12 && pids[1] == 345);
  unlink(path);
}

static void test_smi_mock() {
  const char* lib = getenv("GM_MOCK_LIB");
  if (!lib) {
    fprintf(stderr, "skip smi: GM_MOCK_LIB unset\n");
    return;
  }
  EXPECT(gm_smi_open(lib) == 0);
  uint32_t n = 0;
  EXPECT(gm_smi_count(&n) == 0 && n == 8);
  gm_gpu_info_t info;
  EXPECT(gm_smi_gpu_info(3, &info) == 0);
  EXPECT(info.render_minor == 131 && info.numa_node == 0 && info.xgmi_hive_id != 0);
  EXPECT(std::string(info.gfx_target) == "gfx950");
  gm_link_info_t l;
  EXPECT(gm_smi_link(0, 7, &l) == 0 && l.link_type == 2);
  std::vector<gm_link_info_t> m(64);
  EXPECT(gm_smi_link_matrix(m.data(), 64) == 0 && m[0].link_type == 0);
  gm_proc_info_t procs[4];
  uint32_t np = 99;
  EXPECT(gm_smi_process_list(0, procs, 4, &np) == 0 && np == 0);
  EXPECT(gm_smi_gpu_info(99, &info) == GM_SMI_ERR_RANGE);
  EXPECT(gm_smi_close() == 0);
  EXPECT(gm_smi_count(&n) == GM_SMI_ERR_NOT_OPEN);
}

// Set-mode program: fixed length whatever the device count, every jump inside the program,
// exactly one map lookup, the chain's tail call last before the default verdict; base rules
// (chain lost) add their blocks after the miss label.
static void test_bpf_set_layout() {
  int need = gm_bpf_dev_build_set(-2, nullptr, 0, 0, -2, nullptr, 0);
  EXPECT(need < 0);
  std::vector<uint64_t> prog(-need);
  int n = gm_bpf_dev_build_set(-2, nullptr, 0, 0, -2, prog.data(), (int)prog.size());
  EXPECT(n == -need && n == 30);
  int lookups = 0, tail_calls = 0;
  for (int i = 0; i < n; ++i) {
    struct bpf_insn in;
    memcpy(&in, &prog[i], 8);
    if (in.code == (BPF_JMP | BPF_CALL)) {
      lookups += in.imm == BPF_FUNC_map_lookup_elem;
      tail_calls += in.imm == BPF_FUNC_tail_call;
    }
    if ((in.code & 0x07) == BPF_JMP && ((in.code & 0xf0) == BPF_JNE || (in.code & 0xf0) == BPF_JEQ)) {
      const int tgt = i + 1 + in.off;
      EXPECT(tgt > i && tgt < n);
    }
  }
  EXPECT(lookups == 1 && tail_calls == 1);
  gm_dev_rule_t base[2] = {{'c', 7, 1, 0, 1, 3}, {'c', GM_ACC_MKNOD, 1, 0, -1, -1}};
  int need2 = gm_bpf_dev_build_set(-2, base, 2, 0, -1, nullptr, 0);
  std::vector<uint64_t> prog2(-need2);
  int n2 = gm_bpf_dev_build_set(-2, base, 2, 0, -1, prog2.data(), (int)prog2.size());
  EXPECT(n2 == -need2 && n2 > n - 4);  // no chain (-4) but two rule blocks and a ctx reload
  EXPECT(gm_bpf_dev_build_set(-2, nullptr, -1, 0, -1, prog2.data(), n2) == -EINVAL);
  EXPECT(gm_bpf_dev_build_set(-2, nullptr, 0, 0, -2, prog.data(), 3) < 0);  // too small
}

int main() {
  test_format();
  test_bpf_layout();
  test_bpf_set_layout();
  test_devnodes();
  test_devnodes_guard();
  test_pids();
  test_smi_mock();
  if (g_fail) {
    fprintf(stderr, "%d failure(s)\n", g_fail);
    return 1;
  }
  printf("native tests OK\n");
  return 0;
}
