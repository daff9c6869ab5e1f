"""ctypes bindings to the in-tree native libraries (built by ``native/Makefile`` into ``_lib/``).

* ``libgm_smi.so``      — amdsmi inventory shim        (native/include/gm_smi.h)
* ``libamd_smi_mock.so``— amdsmi stand-in for CPU hosts (native/src/amdsmi_mock.cpp)
* ``libgm_host.so``     — cgroup v1/v2, device nodes, processes, roctx (native/include/gm_host.h)
* ``libgm_probe.so``    — gfx950 HIP validation kernels (native/include/gm_probe.h)

Nothing here falls back silently: a missing library raises :class:`NativeError` with the build
command to run. The struct layouts below must match the C headers field-for-field.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading
from typing import Optional

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
NATIVE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "native")

_lock = threading.Lock()
_libs: dict = {}


class NativeError(RuntimeError):
    pass


def lib_path(name: str) -> str:
    return os.path.join(LIB_DIR, name)


def build(target: str = "all", quiet: bool = True) -> None:
    """Run the native Makefile (``host`` needs only g++; ``all`` also needs hipcc). Processes
    that autobuild at the same time (daemons started together in a fresh tree) take turns on
    a lock file; the Makefile renames each library into place whole."""
    import fcntl
    cmd = ["make", "-C", NATIVE_DIR, target, f"-j{min(8, os.cpu_count() or 1)}"]
    os.makedirs(LIB_DIR, exist_ok=True)
    with open(os.path.join(LIB_DIR, ".build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        res = subprocess.run(cmd, capture_output=quiet, text=True)
    if res.returncode != 0:
        raise NativeError(f"native build failed ({' '.join(cmd)}):\n{res.stdout}\n{res.stderr}")


def _load(name: str, autobuild_target: Optional[str]) -> C.CDLL:
    with _lock:
        if name in _libs:
            return _libs[name]
        path = lib_path(name)
        if not os.path.exists(path) and autobuild_target and os.environ.get("GM_NO_AUTOBUILD") != "1":
            build(autobuild_target)
        if not os.path.exists(path):
            raise NativeError(f"{path} missing — run `make -C native` (or __graft_entry__.build())")
        lib = C.CDLL(path, mode=C.RTLD_GLOBAL if name == "libamd_smi_mock.so" else C.RTLD_LOCAL)
        _libs[name] = lib
        return lib


# ------------------------------------------------------------------------------ gm_smi
class GpuInfo(C.Structure):
    _fields_ = [
        ("index", C.c_uint32), ("render_minor", C.c_uint32), ("card_minor", C.c_uint32),
        ("hsa_id", C.c_uint32), ("hip_id", C.c_uint32), ("kfd_node_id", C.c_uint32),
        ("partition_id", C.c_uint32), ("xgmi_lanes", C.c_uint32), ("numa_node", C.c_int32),
        ("num_cu", C.c_uint32), ("bdf_id", C.c_uint64), ("kfd_gpu_id", C.c_uint64),
        ("xgmi_hive_id", C.c_uint64), ("xgmi_node_id", C.c_uint64), ("vram_bytes", C.c_uint64),
        ("device_id", C.c_uint64), ("uuid", C.c_char * 64), ("bdf", C.c_char * 32),
        ("market_name", C.c_char * 128), ("gfx_target", C.c_char * 32),
        ("compute_partition", C.c_char * 16), ("memory_partition", C.c_char * 16),
    ]


class ProcInfo(C.Structure):
    _fields_ = [("pid", C.c_uint32), ("cu_occupancy", C.c_uint32), ("vram_bytes", C.c_uint64),
                ("gtt_bytes", C.c_uint64), ("name", C.c_char * 64)]


class LinkInfo(C.Structure):
    _fields_ = [("link_type", C.c_uint32), ("reserved", C.c_uint32), ("hops", C.c_uint64),
                ("weight", C.c_uint64)]


def smi() -> C.CDLL:
    lib = _load("libgm_smi.so", "host")
    if not getattr(lib, "_gm_typed", False):
        lib.gm_smi_open.argtypes = [C.c_char_p]
        lib.gm_smi_count.argtypes = [C.POINTER(C.c_uint32)]
        lib.gm_smi_gpu_info.argtypes = [C.c_uint32, C.POINTER(GpuInfo)]
        lib.gm_smi_all_gpu_info.argtypes = [C.POINTER(GpuInfo), C.c_uint32, C.POINTER(C.c_uint32)]
        lib.gm_smi_link.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(LinkInfo)]
        lib.gm_smi_link_matrix.argtypes = [C.POINTER(LinkInfo), C.c_uint32]
        lib.gm_smi_process_list.argtypes = [C.c_uint32, C.POINTER(ProcInfo), C.c_uint32,
                                            C.POINTER(C.c_uint32)]
        lib.gm_smi_ecc.argtypes = [C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_uint64)]
        lib.gm_smi_strerror.argtypes = [C.c_int]
        lib.gm_smi_strerror.restype = C.c_char_p
        lib.gm_smi_lib_path.restype = C.c_char_p
        lib._gm_typed = True
    return lib


def mock_smi_path() -> str:
    _load("libamd_smi_mock.so", "host")
    return lib_path("libamd_smi_mock.so")


def mock_smi() -> C.CDLL:
    lib = _load("libamd_smi_mock.so", "host")
    lib.gm_mock_set_procs_file.argtypes = [C.c_char_p]
    lib.gm_mock_set_ecc.argtypes = [C.c_uint32, C.c_uint64, C.c_uint64]
    return lib


# ------------------------------------------------------------------------------ gm_host
class DevRule(C.Structure):
    _fields_ = [("type", C.c_char), ("access", C.c_uint8), ("allow", C.c_uint8),
                ("pad", C.c_uint8), ("major", C.c_int32), ("minor", C.c_int32)]


class DevNode(C.Structure):
    _fields_ = [("path", C.c_char * 112), ("major", C.c_uint32), ("minor", C.c_uint32),
                ("mode", C.c_uint32), ("uid", C.c_int32), ("gid", C.c_int32)]


class BpfTiming(C.Structure):
    _fields_ = [("query_ns", C.c_uint64), ("map_ns", C.c_uint64), ("build_ns", C.c_uint64),
                ("load_ns", C.c_uint64), ("attach_ns", C.c_uint64), ("programs", C.c_uint32),
                ("insns", C.c_uint32)]


HOST_ABI_VERSION = 6          # native/include/gm_host.h GM_HOST_ABI_VERSION
GM_ACC_MKNOD, GM_ACC_READ, GM_ACC_WRITE = 1, 2, 4
GM_DEV_EMULATE, GM_DEV_VIA_SETNS, GM_DEV_REPLACE, GM_DEV_BIND = 1, 2, 4, 8


def host() -> C.CDLL:
    lib = _load("libgm_host.so", "host")
    if not getattr(lib, "_gm_typed", False):
        abi = lib.gm_host_abi_version()
        if abi != HOST_ABI_VERSION:
            raise RuntimeError(f"libgm_host.so ABI {abi} != {HOST_ABI_VERSION} expected: stale "
                               f"build, run `make -C native`")
        lib.gm_cg1_apply.argtypes = [C.c_char_p, C.POINTER(DevRule), C.c_int]
        lib.gm_cg1_format_rule.argtypes = [C.POINTER(DevRule), C.c_char_p, C.c_int]
        lib.gm_bpf_dev_build.argtypes = [C.POINTER(DevRule), C.c_int, C.c_int, C.c_int,
                                         C.POINTER(C.c_uint64), C.c_int]
        lib.gm_bpf_dev_load.argtypes = [C.POINTER(C.c_uint64), C.c_int, C.c_char_p, C.c_char_p,
                                        C.c_int]
        lib.gm_bpf_dev_query.argtypes = [C.c_char_p, C.POINTER(C.c_uint32), C.c_uint32,
                                         C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        lib.gm_bpf_prog_name.argtypes = [C.c_uint32, C.c_char_p, C.c_int]
        lib.gm_bpf_dev_program.argtypes = [C.c_char_p, C.POINTER(C.c_uint64), C.c_uint32,
                                           C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        lib.gm_bpf_dev_program_at.argtypes = [C.c_char_p, C.c_uint32, C.c_int,
                                              C.POINTER(C.c_uint64),
                                              C.c_uint32, C.POINTER(C.c_uint32),
                                              C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        lib.gm_bpf_dev_install.argtypes = [C.c_char_p, C.POINTER(DevRule), C.c_int,
                                           C.POINTER(DevRule), C.c_int, C.c_char_p,
                                           C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        lib.gm_bpf_dev_restore.argtypes = [C.c_char_p, C.c_char_p]
        lib.gm_bpf_dev_build_set.argtypes = [C.c_int, C.POINTER(DevRule), C.c_int, C.c_int,
                                             C.c_int, C.POINTER(C.c_uint64), C.c_int]
        lib.gm_bpf_dev_probe_set.argtypes = []
        lib.gm_devnodes_bind_probe.argtypes = []
        lib.gm_bpf_dev_straight_line.argtypes = [C.c_int]
        lib.gm_bpf_dev_straight_line.restype = None
        lib.gm_bpf_dev_set_at.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_uint32),
                                          C.c_uint32, C.POINTER(C.c_uint32),
                                          C.POINTER(C.c_uint32)]
        lib.gm_bpf_dev_last_timing.argtypes = [C.POINTER(BpfTiming)]
        lib.gm_bpf_dev_last_timing.restype = None
        lib.gm_devnodes_create.argtypes = [C.c_int, C.c_char_p, C.POINTER(DevNode), C.c_int,
                                           C.c_int, C.POINTER(C.c_int)]
        lib.gm_devnodes_remove.argtypes = lib.gm_devnodes_create.argtypes
        lib.gm_devnodes_guard.argtypes = [C.c_char_p]
        lib.gm_devnodes_stage.argtypes = [C.c_char_p, C.c_int]
        lib.gm_devnode_stat.argtypes = [C.c_int, C.c_char_p, C.c_char_p, C.c_int,
                                        C.POINTER(C.c_int), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        lib.gm_devnodes_present.argtypes = [C.c_int, C.c_char_p, C.POINTER(DevNode), C.c_int,
                                            C.c_int, C.POINTER(C.c_uint8)]
        lib.gm_proc_dev_users.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_int32), C.c_int,
                                          C.POINTER(C.c_int)]
        lib.gm_proc_scan_devs.argtypes = [C.POINTER(C.c_int32), C.c_int, C.POINTER(C.c_uint32),
                                          C.c_int, C.POINTER(C.c_uint8), C.POINTER(C.c_int32)]
        lib.gm_proc_filter_dev_users.argtypes = [C.POINTER(C.c_int32), C.c_int, C.c_uint32,
                                                 C.c_uint32, C.POINTER(C.c_int32)]
        lib.gm_proc_read_pids.argtypes = [C.c_char_p, C.POINTER(C.c_int32), C.c_int,
                                          C.POINTER(C.c_int)]
        lib.gm_sd_get_device_allow.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int,
                                               C.c_char_p, C.c_int]
        lib.gm_sd_set_device_allow.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_char_p),
                                               C.POINTER(C.c_char_p), C.c_int, C.c_int,
                                               C.c_char_p, C.c_int]
        lib.gm_sd_unit_path.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
        lib.gm_roctx_push.argtypes = [C.c_char_p]
        lib.gm_roctx_mark.argtypes = [C.c_char_p]
        lib.gm_roctx_start.argtypes = [C.c_char_p]
        lib.gm_roctx_start.restype = C.c_uint64
        lib.gm_roctx_stop.argtypes = [C.c_uint64]
        lib.gm_roctx_stop.restype = None
        lib.gm_now_ns.restype = C.c_uint64
        lib._gm_typed = True
    return lib


# ------------------------------------------------------------------------------ gm_probe
class ProbeProps(C.Structure):
    _fields_ = [("name", C.c_char * 128), ("gcn_arch", C.c_char * 64),
                ("pci_bus_id", C.c_char * 32), ("cu_count", C.c_int32), ("warp_size", C.c_int32),
                ("total_mem", C.c_uint64), ("lds_per_block", C.c_uint64),
                ("clock_khz", C.c_int32), ("mem_clock_khz", C.c_int32)]


def _prefer_torch_hip_runtime() -> None:
    """A process can hold only one HIP runtime, and ``libamdhip64.so.7`` is resolved by soname:
    whichever copy is loaded first (ROCm's /opt/rocm/lib or the one PyTorch bundles) serves
    every later user. PyTorch does not work on a newer runtime than it was built for, so when it
    is installed its bundled runtime is loaded first (by path, without importing torch) and the
    probe binds to it — the probe then works whether torch is imported before or after."""
    if "libgm_probe.so" in _libs or os.environ.get("GM_PROBE_SYSTEM_HIP") == "1":
        return
    import importlib.util

    spec = importlib.util.find_spec("torch")
    for loc in (spec.submodule_search_locations or []) if spec else []:
        hip = os.path.join(loc, "lib", "libamdhip64.so")
        if os.path.exists(hip):
            try:
                C.CDLL(hip, mode=C.RTLD_GLOBAL)
            except OSError:
                pass
            return


def probe() -> C.CDLL:
    _prefer_torch_hip_runtime()
    lib = _load("libgm_probe.so", "hip")
    if not getattr(lib, "_gm_typed", False):
        lib.gm_probe_device_count.argtypes = [C.POINTER(C.c_int)]
        lib.gm_probe_props.argtypes = [C.c_int, C.POINTER(ProbeProps)]
        lib.gm_probe_find_device.argtypes = [C.c_char_p, C.POINTER(C.c_int)]
        lib.gm_probe_quick.argtypes = [C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_double)]
        lib.gm_probe_hbm_copy.argtypes = [C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_double)]
        lib.gm_probe_hbm_read.argtypes = [C.c_int, C.c_uint64, C.c_int, C.c_int,
                                          C.POINTER(C.c_double)]
        lib.gm_probe_mfma_peak.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_double)]
        lib.gm_probe_gemm_bf16.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                           C.c_int, C.c_void_p]
        lib.gm_probe_gemm_nt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                         C.c_int, C.c_void_p]
        lib.gm_probe_gemm_nt_variant.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                                 C.c_int, C.c_int, C.c_int, C.c_void_p]
        lib.gm_probe_gemm_nt_tflops.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                                C.POINTER(C.c_double)]
        lib.gm_probe_burn_in.argtypes = [C.c_int, C.c_int, C.c_double, C.POINTER(C.c_double),
                                         C.POINTER(C.c_uint64), C.POINTER(C.c_int)]
        lib.gm_probe_gemm_check.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int,
                                            C.POINTER(C.c_double), C.POINTER(C.c_double)]
        lib.gm_probe_p2p.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_int),
                                     C.POINTER(C.c_double)]
        lib.gm_probe_strerror.argtypes = [C.c_int]
        lib.gm_probe_strerror.restype = C.c_char_p
        lib._gm_typed = True
    return lib


def loaded_libraries() -> list:
    """Paths of native libraries loaded into this process (for diagnostics/tests)."""
    return sorted(lib_path(n) for n in _libs)


def mapped_in_tree() -> list:
    """In-tree shared objects this process has mapped (``/proc/self/maps``): what the driver's
    round-end check observes. Used by ``GM_RECORD_MAPS`` in tests/conftest.py and smoke()."""
    root = os.path.dirname(LIB_DIR.rstrip("/"))
    root = os.path.dirname(root)
    seen = set()
    try:
        with open("/proc/self/maps") as fh:
            for ln in fh:
                path = ln.rstrip("\n").split(None, 5)[-1] if ln.count(" ") >= 5 else ""
                if path.startswith(root) and ".so" in os.path.basename(path):
                    seen.add(path)
    except OSError:
        pass
    return sorted(seen)


def record_maps(dest: Optional[str] = None) -> None:
    dest = dest or os.environ.get("GM_RECORD_MAPS")
    if not dest:
        return
    with open(dest, "a") as fh:
        for p in mapped_in_tree():
            fh.write(f"{os.getpid()} {p}\n")
