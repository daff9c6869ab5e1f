"""Real-kernel node sandbox: the production node path against the running kernel (root only).

The hermetic harness stands in for the kernel with a JSON-recording cgroup backend and marker
files for device nodes. This sandbox gives the same :class:`LocalCluster` a real node instead:

* a private **cgroup2** mount (the tenant's container cgroup is a real cgroup with a runc-style
  ``BPF_PROG_TYPE_CGROUP_DEVICE`` program attached, as a container runtime leaves it), so every
  attach loads, verifies and ``BPF_F_REPLACE``-attaches a real device program;
* a private **bpffs** for the pinned tail-call maps;
* a **tenant process in its own mount namespace** with a private tmpfs ``/dev``, so device nodes
  are created with ``mknodat`` through ``/proc/<pid>/root`` exactly as on a node.

The reference's equivalent per-GPU work is a forked ``sh -c "echo … > devices.allow"`` and a forked
``nsenter … mknod`` (reference: pkg/util/cgroup/cgroup.go:143-155,
pkg/util/namespace/namespace.go:167-177, ordered at pkg/util/util.go:37-67). Used by
``bench.py --node-ops real`` and tests/priv_e2e_driver.py.
"""
from __future__ import annotations

import ctypes as C
import ctypes.util
import os
import shutil
import subprocess
import tempfile
import uuid
from typing import Optional

from gpumounter_amd import _native

_BPF_PROG_ATTACH = 8
_BPF_CGROUP_DEVICE = 6
_BPF_F_ALLOW_MULTI = 2
_SYS_BPF = 321  # x86_64


def available() -> Optional[str]:
    """None if the sandbox can run here, else why not."""
    if os.geteuid() != 0:
        return "needs root (mount, mknod, bpf)"
    for tool in ("mount", "umount", "unshare", "sleep"):
        if shutil.which(tool) is None:
            return f"{tool} not found"
    return None


def attach_runtime_program(cg: str) -> None:
    """A runc-style device program (/dev/null rw + mknod only) attached with BPF_F_ALLOW_MULTI,
    as the container runtime leaves it on a cgroup2 container."""
    rules = (_native.DevRule * 1)(_native.DevRule(b"c", 7, 1, 0, 1, 3))
    lib = _native.host()
    need = -lib.gm_bpf_dev_build(rules, 1, 0, -1, None, 0)
    buf = (C.c_uint64 * need)()
    n = lib.gm_bpf_dev_build(rules, 1, 0, -1, buf, need)
    fd = lib.gm_bpf_dev_load(buf, n, b"runc_devices", None, 0)
    if fd < 0:
        raise OSError(-fd, f"BPF_PROG_LOAD runc_devices: {os.strerror(-fd)}")
    libc = C.CDLL(ctypes.util.find_library("c"), use_errno=True)
    cgfd = os.open(cg, os.O_RDONLY | os.O_DIRECTORY)
    try:
        attr = (C.c_uint8 * 128)()
        C.memmove(attr, (C.c_uint32 * 4)(cgfd, fd, _BPF_CGROUP_DEVICE, _BPF_F_ALLOW_MULTI), 16)
        if libc.syscall(_SYS_BPF, _BPF_PROG_ATTACH, attr, 128) != 0:
            err = C.get_errno()
            raise OSError(err, f"BPF_PROG_ATTACH: {os.strerror(err)}")
    finally:
        os.close(cgfd)
        os.close(fd)


class RealNodeSandbox:
    """``with RealNodeSandbox() as sb:`` → ``sb.cgroup_root`` (a real cgroup2 mount, node dirs
    go below ``sb.cgroup_root``), ``sb.bpffs``, ``sb.tenant_pid`` (a process in its own mount
    namespace with a private tmpfs /dev)."""

    def __init__(self) -> None:
        self.mnt = ""
        self.bpffs = ""
        self.cgroup_root = ""
        self.tenants: list = []

    @property
    def tenant_pid(self) -> int:
        return self.tenants[0].pid

    def spawn_tenant(self, setup: str = "mount -t tmpfs tmpfs /dev") -> int:
        p = subprocess.Popen(["unshare", "-m", "--propagation", "private", "sh", "-c",
                              f"set -e; {setup}; echo ok; exec sleep 3600"],
                             stdout=subprocess.PIPE, text=True)
        if p.stdout.readline().strip() != "ok":
            p.kill()
            p.wait()
            raise RuntimeError("tenant mount namespace setup failed")
        self.tenants.append(p)
        return p.pid

    def __enter__(self) -> "RealNodeSandbox":
        why = available()
        if why:
            raise RuntimeError(f"real node sandbox unavailable: {why}")
        self.mnt = tempfile.mkdtemp(prefix="gm-real-cg2-")
        self.bpffs = tempfile.mkdtemp(prefix="gm-real-bpffs-")
        subprocess.run(["mount", "-t", "cgroup2", "none", self.mnt], check=True)
        subprocess.run(["mount", "-t", "bpf", "bpf", self.bpffs], check=True)
        self.cgroup_root = os.path.join(self.mnt, "gm-real-" + uuid.uuid4().hex[:8])
        try:
            self.spawn_tenant()
        except Exception:
            self.__exit__(None, None, None)
            raise
        return self

    def __exit__(self, *exc) -> None:
        for p in self.tenants:
            p.kill()
            p.wait()
        self.tenants.clear()
        if self.cgroup_root and os.path.isdir(self.cgroup_root):
            # tear the real cgroup tree down bottom-up (its processes are gone)
            for dirpath, _, _ in sorted(os.walk(self.cgroup_root),
                                        key=lambda t: -t[0].count("/")):
                try:
                    os.rmdir(dirpath)
                except OSError:
                    pass
        if self.bpffs:
            subprocess.run(["umount", self.bpffs], check=False)
            shutil.rmtree(self.bpffs, ignore_errors=True)
        if self.mnt:
            subprocess.run(["umount", self.mnt], check=False)
            try:
                os.rmdir(self.mnt)
            except OSError:
                pass
