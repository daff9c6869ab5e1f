// libgm_tenant_view.so — a tenant process's view of the GPU device nodes, for unprivileged hosts.
//
// On a real node gpumounter injects /dev/kfd and /dev/dri/renderD*/card* into the tenant's own
// mount namespace and grants them in its device cgroup (reference: util.go:37-67
// did the same for /dev/nvidiaN). The GPU box that runs this repository's GPU tests allows
// neither namespaces nor cgroup writes, so the worker runs its node operations in emulation
// there: device nodes are marker files under the container's rootfs directory
// ("gm-chr <major>:<minor>") and the cgroup-v2 program plus its allow set are recorded in
// <cgroup>/gm.bpf.json instead of being loaded.
//
// Preloaded into a tenant-side process (LD_PRELOAD), this library makes the ROCm stack in that
// process open the GPU device nodes *through that emulated state*, exactly as the kernel would
// resolve them in a real container:
//   * open("/dev/kfd" | "/dev/dri/...") looks the path up under $GM_TENANT_ROOT: no node there →
//     ENOENT (the tenant has no such node); a marker → the host node with that major:minor;
//   * the (major, minor) must be in the recorded allow set of $GM_TENANT_CGROUP (if set) with
//     read+write access, else EPERM — the device cgroup's verdict.
// Every other path goes straight to libc. A HIP process started with it before an attach sees
// no GPU; after the attach it sees exactly the attached ones; after the detach none again.
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/sysmacros.h>
#include <unistd.h>

namespace {

using open_fn = int (*)(const char*, int, ...);
using openat_fn = int (*)(int, const char*, int, ...);
using access_fn = int (*)(const char*, int);

template <typename F>
F next(const char* name) {
  return reinterpret_cast<F>(dlsym(RTLD_NEXT, name));
}

bool is_gpu_path(const char* p) {
  return p && (strcmp(p, "/dev/kfd") == 0 || strncmp(p, "/dev/dri/", 9) == 0);
}

// Reads the marker at $GM_TENANT_ROOT<path>. 1 = marker (major/minor set), 0 = absent,
// -errno otherwise.
int tenant_node(const char* path, unsigned* ma, unsigned* mi) {
  const char* root = getenv("GM_TENANT_ROOT");
  if (!root || !*root) return -EACCES;  // misconfigured: refuse rather than leak host nodes
  char full[4096];
  if (snprintf(full, sizeof(full), "%s%s", root, path) >= (int)sizeof(full)) return -ENAMETOOLONG;
  int fd = next<open_fn>("open")(full, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return errno == ENOENT || errno == ENOTDIR ? 0 : -errno;
  char buf[64] = {0};
  ssize_t n = read(fd, buf, sizeof(buf) - 1);
  close(fd);
  if (n <= 0 || sscanf(buf, "gm-chr %u:%u", ma, mi) != 2) return -EINVAL;
  return 1;
}

// Is (major, minor) granted rw in the recorded allow set? No cgroup configured → yes.
bool granted(unsigned ma, unsigned mi) {
  const char* cg = getenv("GM_TENANT_CGROUP");
  if (!cg || !*cg) return true;
  char full[4096];
  if (snprintf(full, sizeof(full), "%s/gm.bpf.json", cg) >= (int)sizeof(full)) return false;
  int fd = next<open_fn>("open")(full, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;  // no program of ours: the runtime's default list has no GPU
  static char blob[1 << 16];
  ssize_t n = read(fd, blob, sizeof(blob) - 1);
  close(fd);
  if (n <= 0) return false;
  blob[n] = 0;
  const char* s = strstr(blob, "\"set\"");
  if (!s) return false;
  s = strchr(s, '[');
  if (!s) return false;
  ++s;
  // entries: [type, major, minor, access]; char type = 2, access rw = 2|4
  for (;;) {
    const char* e = strchr(s, '[');
    const char* end = strchr(s, ']');
    if (!e || (end && end < e)) break;  // the closing bracket of the set itself
    unsigned t, a, b, acc;
    if (sscanf(e, "[%u, %u, %u, %u]", &t, &a, &b, &acc) == 4 ||
        sscanf(e, "[%u,%u,%u,%u]", &t, &a, &b, &acc) == 4) {
      if (t == 2 && a == ma && b == mi && (acc & 6u) == 6u) return true;
    }
    s = strchr(e, ']');
    if (!s) break;
    ++s;
  }
  return false;
}

// The host node with that major:minor (the one a real mknod in the tenant would reach).
bool host_path(unsigned ma, unsigned mi, char* out, size_t cap) {
  struct stat st;
  if (stat("/dev/kfd", &st) == 0 && major(st.st_rdev) == ma && minor(st.st_rdev) == mi) {
    snprintf(out, cap, "/dev/kfd");
    return true;
  }
  if (ma != 226) return false;
  snprintf(out, cap, mi >= 128 ? "/dev/dri/renderD%u" : "/dev/dri/card%u", mi);
  return stat(out, &st) == 0 && S_ISCHR(st.st_mode) && st.st_rdev == makedev(ma, mi);
}

// Resolves a GPU path for the tenant: 0 and `out` set, or -errno.
int resolve(const char* path, char* out, size_t cap) {
  unsigned ma = 0, mi = 0;
  int r = tenant_node(path, &ma, &mi);
  if (r < 0) return r;
  if (r == 0) return -ENOENT;
  if (!granted(ma, mi)) return -EPERM;
  if (!host_path(ma, mi, out, cap)) return -ENXIO;
  return 0;
}

int open_via(const char* path, int flags, mode_t mode) {
  char host[256];
  int r = resolve(path, host, sizeof(host));
  if (r < 0) {
    errno = -r;
    return -1;
  }
  return next<open_fn>("open")(host, flags, mode);
}

mode_t mode_arg(int flags, va_list ap) {
  return (flags & O_CREAT) || (flags & O_TMPFILE) == O_TMPFILE ? (mode_t)va_arg(ap, int) : 0;
}

}  // namespace

extern "C" {

int open(const char* path, int flags, ...) {
  va_list ap;
  va_start(ap, flags);
  mode_t mode = mode_arg(flags, ap);
  va_end(ap);
  if (is_gpu_path(path)) return open_via(path, flags, mode);
  return next<open_fn>("open")(path, flags, mode);
}

int open64(const char* path, int flags, ...) {
  va_list ap;
  va_start(ap, flags);
  mode_t mode = mode_arg(flags, ap);
  va_end(ap);
  if (is_gpu_path(path)) return open_via(path, flags, mode);
  return next<open_fn>("open64")(path, flags, mode);
}

int __open_2(const char* path, int flags) {
  if (is_gpu_path(path)) return open_via(path, flags, 0);
  return next<open_fn>("open")(path, flags);
}

int __open64_2(const char* path, int flags) {
  if (is_gpu_path(path)) return open_via(path, flags, 0);
  return next<open_fn>("open64")(path, flags);
}

int openat(int dirfd, const char* path, int flags, ...) {
  va_list ap;
  va_start(ap, flags);
  mode_t mode = mode_arg(flags, ap);
  va_end(ap);
  if (is_gpu_path(path)) return open_via(path, flags, mode);
  return next<openat_fn>("openat")(dirfd, path, flags, mode);
}

int openat64(int dirfd, const char* path, int flags, ...) {
  va_list ap;
  va_start(ap, flags);
  mode_t mode = mode_arg(flags, ap);
  va_end(ap);
  if (is_gpu_path(path)) return open_via(path, flags, mode);
  return next<openat_fn>("openat64")(dirfd, path, flags, mode);
}

int access(const char* path, int amode) {
  if (is_gpu_path(path)) {
    char host[256];
    int r = resolve(path, host, sizeof(host));
    if (r < 0) {
      errno = -r;
      return -1;
    }
    return next<access_fn>("access")(host, amode);
  }
  return next<access_fn>("access")(path, amode);
}

}  // extern "C"
