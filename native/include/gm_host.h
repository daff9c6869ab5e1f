// gm_host.h — privileged host operations of the gpumounter-amd node agent, as a flat C ABI.
//
// Replaces the reference's fork/exec shell pipeline (reference: pkg/util/cgroup/cgroup.go:143-169
// `sh -c "echo 'c 195:N rw' > devices.allow"`, pkg/util/namespace/namespace.go:167-201
// `nsenter --mount sh -c "mknod|rm|kill"`) with in-process syscalls:
//   * cgroup v1: one write(2) per rule into devices.allow / devices.deny
//   * cgroup v2: a BPF_PROG_TYPE_CGROUP_DEVICE allow-list generated here, loaded with bpf(2) and
//     swapped in atomically (BPF_F_REPLACE); the container runtime's own program is preserved by
//     tail-calling into it from ours, so its rules never need to be reverse-engineered
//   * device nodes: mknodat/unlinkat through /proc/<pid>/root of the target container (or a
//     setns(CLONE_NEWNS) helper thread) — no mknod binary in the tenant image (reference FAQ.md:3-4)
//   * processes: pidfd_send_signal by PID (the worker pins PIDs with long-lived pidfds itself:
//     gpumounter_amd/node/procs.py Pinned), /proc/*/fd scan for device users
//   * roctx range markers around attach/detach for rocprofv3 --marker-trace timelines
// All functions return 0 / a count on success and -errno on failure unless stated otherwise.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GM_HOST_ABI_VERSION 6

// Access bits follow BPF_DEVCG_ACC_* so the same rule feeds both cgroup versions.
#define GM_ACC_MKNOD 1
#define GM_ACC_READ 2
#define GM_ACC_WRITE 4

typedef struct gm_dev_rule {
  char type;        // 'c' char, 'b' block, 'a' all
  uint8_t access;   // GM_ACC_* bitmask
  uint8_t allow;    // 1 allow, 0 deny
  uint8_t pad;
  int32_t major;    // -1 = wildcard
  int32_t minor;    // -1 = wildcard
} gm_dev_rule_t;

// ---- cgroup v1 ------------------------------------------------------------------------------
// Writes each rule ("c 226:128 rw") to <cgdir>/devices.allow (rule.allow=1) or devices.deny.
// Returns number of rules written or -errno of the first failure.
int gm_cg1_apply(const char* cgdir, const gm_dev_rule_t* rules, int n);
// Formats a rule the way the v1 devices controller expects it; returns length.
int gm_cg1_format_rule(const gm_dev_rule_t* rule, char* out, int cap);

// ---- cgroup v2 (device eBPF) ----------------------------------------------------------------
// Encodes the allow-list program into `out` (each entry one struct bpf_insn as uint64).
// First matching rule wins. After the rules: if chain_map_fd >= 0 the program tail-calls slot 0
// of that BPF_MAP_TYPE_PROG_ARRAY (the runtime's original program); if the tail call fails or no
// map is given, it returns `default_allow`. chain_map_fd == -2 emits the tail-call sequence with a
// placeholder fd (for offline inspection / interpretation in tests).
// Returns instruction count, or -(needed) if cap is too small, or -EINVAL.
int gm_bpf_dev_build(const gm_dev_rule_t* rules, int n, int default_allow, int chain_map_fd,
                     uint64_t* out, int cap);
// Set-mode program: allows an access if {dev type, major, minor} is in the HASH map
// `set_map_fd` (key 3×u32: BPF_DEVCG_DEV_*, major, minor; value: u32 GM_ACC_* bits that are
// allowed) with every requested access bit; otherwise it evaluates `base` rules (the runtime's
// default list when the chain is lost), tail-calls the chain map like gm_bpf_dev_build and
// finally returns `default_allow`. The program does not grow with the number of devices. -2 for
// either fd emits placeholders (offline inspection). Returns the count, -(needed) or -EINVAL.
int gm_bpf_dev_build_set(int set_map_fd, const gm_dev_rule_t* base, int nbase, int default_allow,
                         int chain_map_fd, uint64_t* out, int cap);
// Loads instructions as a CGROUP_DEVICE program named `name`. Returns prog fd or -errno;
// verifier log (if any) is copied to `log`.
int gm_bpf_dev_load(const uint64_t* insns, int n, const char* name, char* log, int logcap);
// Lists program ids attached to the cgroup-v2 directory for BPF_CGROUP_DEVICE.
int gm_bpf_dev_query(const char* cgroup_path, uint32_t* ids, uint32_t cap, uint32_t* n,
                     uint32_t* attach_flags);
// Name of a loaded program (by id). Returns 0 or -errno.
int gm_bpf_prog_name(uint32_t id, char* name, int cap);
// Verifier-translated ("xlated") instructions of the gpumounter program attached to the cgroup, so
// audits check what the kernel actually enforces. *n = 0 and *prog_id = 0 if none of ours is
// attached; -ENOSPC (with *n = needed) if cap is too small; -EPERM if the kernel hides xlated code.
int gm_bpf_dev_program(const char* cgroup_path, uint64_t* insns, uint32_t cap, uint32_t* n,
                       uint32_t* prog_id);
// Same for the index-th gpumounter program (several when several programs were wrapped), or with
// foreign_only=1 the index-th program that is not ours (each can veto an access under
// BPF_F_ALLOW_MULTI); *n = 0 past the last one. *foreign = number of programs not ours.
int gm_bpf_dev_program_at(const char* cgroup_path, uint32_t index, int foreign_only,
                          uint64_t* insns, uint32_t cap, uint32_t* n, uint32_t* prog_id,
                          uint32_t* foreign);
// Installs (or updates) the gpumounter allow-list on a cgroup-v2 directory. Exact allow rules
// (every hot-mount) use set mode: the rules go into a HASH map shared by the cgroup's
// gpumounter programs (gm_bpf_dev_build_set), so once a cgroup is wrapped an update is a map
// sync without loading or attaching anything; other rule lists compile a straight-line
// program (gm_bpf_dev_build). Every attached
// program is wrapped, because under BPF_F_ALLOW_MULTI each one must allow an access (runc and
// systemd both attach one on systemd-driver hosts):
//   * a program of ours → replaced, chaining to the same original program;
//   * a foreign program → ours replaces it (BPF_F_REPLACE) and tail-calls into it;
//   * nothing attached → ours is attached with default-allow (deny rules only matter then).
// The tail-call maps must outlive this process (the kernel clears PROG_ARRAY slots when the last
// user reference goes away), so each is pinned at <pin_dir>/gm_<cgroup inode>_<original prog id>
// on a bpffs; with pin_dir NULL/"" the map fds are kept open in this process instead. If our
// program is attached but its chain slot is empty (unpinned map after a restart), `base` rules
// (the runtime's default device list) are compiled in instead of the tail call.
// Returns the number of programs installed; *prog_id is the first of ours and *chained_id the
// original it preserves (0 if none).
// Where the last gm_bpf_dev_install on this thread spent its time (ns): query = open cgroup +
// BPF_PROG_QUERY; map = chain-map create/pin + fd lookups; build = program generation;
// load = BPF_PROG_LOAD including the verifier; attach = BPF_PROG_ATTACH (BPF_F_REPLACE).
typedef struct gm_bpf_timing {
  uint64_t query_ns, map_ns, build_ns, load_ns, attach_ns;
  uint32_t programs, insns;
} gm_bpf_timing_t;
void gm_bpf_dev_last_timing(gm_bpf_timing_t* out);
int gm_bpf_dev_install(const char* cgroup_path, const gm_dev_rule_t* rules, int n,
                       const gm_dev_rule_t* base, int nbase, const char* pin_dir,
                       uint32_t* prog_id, uint32_t* chained_id);
// Process-wide switch: 1 = always compile straight-line programs (set mode off; a kill switch
// and the baseline for measurements), 0 = set mode for exact allow rules (default).
void gm_bpf_dev_straight_line(int on);
// 0 if a set-mode program (HASH map + lookup) loads here, else -errno (node preflight).
int gm_bpf_dev_probe_set(void);
// The allow set of the index-th gpumounter program on the cgroup, as entries of 4 u32 (type,
// major, minor, access bits). Returns 1 (set-mode program, *n entries), 0 (a straight-line
// program: read it with gm_bpf_dev_program_at), -ENOENT past the last one, -ENOSPC (*n =
// needed) or -errno.
int gm_bpf_dev_set_at(const char* cgroup_path, uint32_t index, uint32_t* entries, uint32_t cap,
                      uint32_t* n, uint32_t* prog_id);
// Removes our programs, re-attaching each chained original in its place (if any), and unpins.
// Returns how many were removed.
int gm_bpf_dev_restore(const char* cgroup_path, const char* pin_dir);

// ---- device nodes ---------------------------------------------------------------------------
typedef struct gm_dev_node {
  char path[112];   // path inside the container root, e.g. "dev/dri/renderD128"
  uint32_t major;
  uint32_t minor;
  uint32_t mode;    // permission bits, e.g. 0666
  int32_t uid;      // -1 = leave
  int32_t gid;      // -1 = leave
} gm_dev_node_t;

#define GM_DEV_EMULATE 1    // mknod EPERM → regular marker file "gm-chr MAJ:MIN" (unprivileged tests)
#define GM_DEV_VIA_SETNS 2  // enter the mount namespace with a helper thread instead of /proc/pid/root
#define GM_DEV_REPLACE 4    // replace an existing node with different major:minor
// Bind mode, for containers in their own user namespace (Kubernetes `hostUsers: false`): their
// /dev is a tmpfs mounted inside that namespace, so the kernel treats it as nodev and a node
// mknod'ed there exists but cannot be opened. Instead each node is made once in the staging
// directory (gm_devnodes_stage), cloned with open_tree(OPEN_TREE_CLONE) and attached over an
// empty placeholder file in the container with move_mount; removal detaches the mount and
// unlinks the placeholder. Implies the setns helper (the mount must be made from inside the
// container's mount namespace) unless `root` is given. In bind mode a node counts as present
// only if it is such a mount: an mknod'ed node on a nodev /dev is reported absent.
#define GM_DEV_BIND 8

// Registers the host's /dev (and its dri/) as seen from the caller, e.g. "/proc/1/root/dev". From
// then on create/remove leave any node whose directory *is* one of them alone (result 2): a
// container that bind-mounts the host's /dev shares the host's nodes. NULL/"" clears the guard.
// Returns how many directories are guarded, or -errno if host_dev cannot be read.
int gm_devnodes_guard(const char* host_dev);
// Sets the staging directory of bind mode (process-wide). With `mount_tmpfs` a private tmpfs is
// mounted there first (nosuid, noexec, mode 0711), so the staged nodes live on a filesystem
// mounted in the caller's (initial) user namespace. Returns 0 or -errno. NULL/"" unsets it.
int gm_devnodes_stage(const char* dir, int mount_tmpfs);
// 0 if bind mode can work here (open_tree(OPEN_TREE_CLONE) allowed), else -errno.
int gm_devnodes_bind_probe(void);
// Creates nodes inside the target's root: `root` if non-NULL (test prefix), else /proc/<pid>/root.
// results[i] = 0 created, 1 already present (idempotent), 2 directory is the host's (skipped), or
// -errno. Returns #failures.
int gm_devnodes_create(int pid, const char* root, const gm_dev_node_t* nodes, int n, int flags,
                       int* results);
// Removes nodes (only if they are the expected device). results[i] = 0 removed, 1 absent,
// 2 directory is the host's (left alone), -errno.
int gm_devnodes_remove(int pid, const char* root, const gm_dev_node_t* nodes, int n, int flags,
                       int* results);
// Describes a node: *kind = 0 absent, 1 char device, 2 emulated marker, 3 other file.
int gm_devnode_stat(int pid, const char* root, const char* path, int flags, int* kind,
                    uint32_t* major, uint32_t* minor, uint32_t* mode);
// Read-back of a whole node set in one root resolution (the attach verify step):
// present[i] = 1 if nodes[i].path is a char device (or emulated marker) with exactly
// nodes[i].major:minor, 2 if its directory is the host's guarded /dev (shared, never ours to
// create), else 0. Returns the number present, or -errno if the root is unreachable.
int gm_devnodes_present(int pid, const char* root, const gm_dev_node_t* nodes, int n, int flags,
                        uint8_t* present);

// ---- processes ------------------------------------------------------------------------------
// PIDs with an open fd on char device major:minor (scans /proc/*/fd). *n = total found.
int gm_proc_dev_users(uint32_t major, uint32_t minor, int32_t* pids, int cap, int* n);
// Of `pids`, those holding an fd on char device major:minor (scans only /proc/<pid>/fd of the
// given PIDs — cheap and exact for one container). Returns the count written to `out`.
// One pass over each PID's fd table for up to 256 char devices (majmin = [maj0,min0,maj1,...]):
// hits[i*ndev + j] = 1 if pids[i] holds devs[j] open. Returns how many PIDs' fd tables could
// not be read (listed in `unreadable`, capacity n); exited PIDs count as holding nothing.
int gm_proc_scan_devs(const int32_t* pids, int n, const uint32_t* majmin, int ndev,
                      uint8_t* hits, int32_t* unreadable);
int gm_proc_filter_dev_users(const int32_t* pids, int n, uint32_t major, uint32_t minor,
                             int32_t* out);
// Parses a cgroup.procs-style file. *n = total.
int gm_proc_read_pids(const char* path, int32_t* pids, int cap, int* n);

// ---- systemd unit device policy (D-Bus; native/src/gm_sdbus.cpp) ------------------------------
// bus_path: systemd's private socket (/run/systemd/private, peer-to-peer) or the system bus
// socket (/run/dbus/system_bus_socket: Hello, destination org.freedesktop.systemd1). -EPROTO means
// a D-Bus error; its name and message are copied to `err`.
// The unit's DeviceAllow= as "path\tperm\n" lines in `out`; returns the length or -errno.
int gm_sd_get_device_allow(const char* bus_path, const char* unit, char* out, int cap, char* err,
                           int errcap);
// SetUnitProperties(unit, runtime=true, DeviceAllow=...): appends the entries, or with reset=1
// replaces the whole list by them (an empty list first, then the entries, in one call).
int gm_sd_set_device_allow(const char* bus_path, const char* unit, const char* const* paths,
                           const char* const* perms, int n, int reset, char* err, int errcap);
// D-Bus object path of a unit (sd_bus_path_encode). Returns the length or -(needed).
int gm_sd_unit_path(const char* unit, char* out, int cap);

// ---- tracing --------------------------------------------------------------------------------
int gm_roctx_available(void);
void gm_roctx_push(const char* name);
void gm_roctx_pop(void);
void gm_roctx_mark(const char* name);
// Start/stop ranges (not a per-thread stack): correct for spans of interleaved asyncio tasks.
uint64_t gm_roctx_start(const char* name);
void gm_roctx_stop(uint64_t id);
uint64_t gm_now_ns(void);

int gm_host_abi_version(void);

#ifdef __cplusplus
}
#endif
