"""Node GPU inventory via the native amdsmi shim.

Reference: ``GPUCollector.GetGPUInfo`` inits NVML, walks handles by index for minor+UUID and shuts
NVML down again (reference: pkg/util/gpu/collector/collector.go:40-79), and
``NvidiaGPU.GetRunningProcess`` re-inits NVML for every process query (pkg/device/nvidia.go:58-87).
Here the shim is opened once per process; enumeration (including the xGMI link matrix) is cached,
and only the process table is queried live.
"""
from __future__ import annotations

import copy
import ctypes as C
import os
import threading
from dataclasses import dataclass
from typing import Dict, List, Optional, Set, Tuple

from gpumounter_amd import _native
from gpumounter_amd.models.device import (DEFAULT_KFD_MAJOR, AmdGpu, LinkMatrix, find_gpu,
                                          gpus_by_key)
from gpumounter_amd.utils import log

_log = log.get("hw.inventory")


class InventoryError(RuntimeError):
    pass


@dataclass
class GpuProcess:
    pid: int
    vram_bytes: int
    gtt_bytes: int
    cu_occupancy: int
    name: str


_open_lock = threading.Lock()
_open_path: Optional[str] = None  # the shim is process-global (one amdsmi session per process)


def resolve_lib(lib: str) -> str:
    if lib == "mock":
        return _native.mock_smi_path()
    return lib


def open_shim(lib: str = "") -> str:
    """Open the process-wide amdsmi session; returns the library path actually loaded."""
    global _open_path
    path = resolve_lib(lib)
    with _open_lock:
        smi = _native.smi()
        if smi.gm_smi_is_open():
            if path and _open_path and os.path.abspath(path) != os.path.abspath(_open_path):
                raise InventoryError(f"amdsmi already open with {_open_path}, requested {path}")
            return _open_path or smi.gm_smi_lib_path().decode()
        st = smi.gm_smi_open(path.encode() if path else None)
        if st != 0:
            raise InventoryError(f"amdsmi open({path or 'libamd_smi.so'}) failed: "
                                 f"{st} {smi.gm_smi_strerror(st).decode()}")
        _open_path = smi.gm_smi_lib_path().decode()
        return _open_path


def close_shim() -> None:
    global _open_path
    with _open_lock:
        _native.smi().gm_smi_close()
        _open_path = None


def read_kfd_major(path: str = "/sys/class/kfd/kfd/dev", default: int = DEFAULT_KFD_MAJOR) -> int:
    try:
        with open(path, "r", encoding="ascii") as fh:
            return int(fh.read().strip().split(":")[0])
    except (OSError, ValueError):
        return default


class Inventory:
    def __init__(self, lib: str = "", kfd_major: int = 0,
                 kfd_dev_path: str = "/sys/class/kfd/kfd/dev") -> None:
        self.lib_path = open_shim(lib)
        self.kfd_major = kfd_major or read_kfd_major(kfd_dev_path)
        self._lock = threading.Lock()
        self._gpus: List[AmdGpu] = []
        self._links: Optional[LinkMatrix] = None
        self._keys = None
        self.ecc_policy = "new"                 # off | new | any (see healthy())
        self._ecc_base: Dict[int, int] = {}
        self._ecc_failed: Set[int] = set()
        self.refresh()

    # ---------------------------------------------------------------------------------- static
    def refresh(self) -> None:
        smi = _native.smi()
        n = C.c_uint32(0)
        st = smi.gm_smi_count(C.byref(n))
        if st != 0:
            raise InventoryError(f"gm_smi_count: {smi.gm_smi_strerror(st).decode()}")
        count = n.value
        arr = (_native.GpuInfo * max(count, 1))()
        st = smi.gm_smi_all_gpu_info(arr, count, C.byref(n))
        if st != 0:
            raise InventoryError(f"gm_smi_all_gpu_info: {smi.gm_smi_strerror(st).decode()}")
        gpus = []
        for i in range(count):
            g = arr[i]
            u32 = lambda v: -1 if v == 0xFFFFFFFF else int(v)  # noqa: E731
            gpus.append(AmdGpu(
                index=int(g.index), uuid=g.uuid.decode(errors="replace"),
                bdf=g.bdf.decode().lower(), render_minor=u32(g.render_minor),
                card_minor=u32(g.card_minor),
                kfd_gpu_id=0 if g.kfd_gpu_id == 0xFFFFFFFFFFFFFFFF else int(g.kfd_gpu_id),
                kfd_node_id=u32(g.kfd_node_id), hip_id=u32(g.hip_id),
                xgmi_hive_id=int(g.xgmi_hive_id), xgmi_node_id=int(g.xgmi_node_id),
                numa_node=int(g.numa_node), partition_id=int(g.partition_id),
                compute_partition=g.compute_partition.decode(errors="replace"),
                memory_partition=g.memory_partition.decode(errors="replace"),
                market_name=g.market_name.decode(errors="replace"),
                gfx_target=g.gfx_target.decode(errors="replace"), num_cu=int(g.num_cu),
                vram_bytes=int(g.vram_bytes)))
        links = LinkMatrix(n=count)
        if count:
            mat = (_native.LinkInfo * (count * count))()
            st = smi.gm_smi_link_matrix(mat, count * count)
            if st != 0:
                raise InventoryError(f"gm_smi_link_matrix: {smi.gm_smi_strerror(st).decode()}")
            links.types = [[int(mat[i * count + j].link_type) for j in range(count)]
                           for i in range(count)]
            links.hops = [[int(mat[i * count + j].hops) for j in range(count)]
                          for i in range(count)]
            links.weights = [[int(mat[i * count + j].weight) for j in range(count)]
                             for i in range(count)]
        with self._lock:
            self._gpus = gpus
            self._links = links
        _log.info("inventory: %d GPU(s) via %s, kfd major %d", count, self.lib_path,
                  self.kfd_major)

    @property
    def is_mock(self) -> bool:
        """The mock amdsmi library: its GPUs and process table are synthetic, not this node's."""
        return os.path.abspath(self.lib_path) == os.path.abspath(_native.mock_smi_path())

    def gpus(self) -> List[AmdGpu]:
        """Fresh copies (callers mutate ledger fields)."""
        with self._lock:
            return [copy.copy(g) for g in self._gpus]

    def by_key(self) -> Dict[str, AmdGpu]:
        """Device-ID spelling → GPU, cached per inventory snapshot. Read-only for callers (the
        identity fields used for lookups; take :meth:`gpus` copies to record ledger state)."""
        with self._lock:
            if self._keys is None or self._keys[0] is not self._gpus:
                self._keys = (self._gpus, gpus_by_key(self._gpus))
            return self._keys[1]

    @property
    def count(self) -> int:
        return len(self._gpus)

    def links(self) -> LinkMatrix:
        assert self._links is not None
        return self._links

    def by_device_id(self, device_id: str) -> Optional[AmdGpu]:
        with self._lock:
            return find_gpu(self._gpus, device_id)

    # ---------------------------------------------------------------------------------- live
    def processes(self, index: int, cap: int = 1024) -> List[GpuProcess]:
        """Processes holding a context on GPU ``index`` (cap 1024 as in reference nvidia.go:69-76)."""
        smi = _native.smi()
        buf = (_native.ProcInfo * cap)()
        n = C.c_uint32(0)
        st = smi.gm_smi_process_list(index, buf, cap, C.byref(n))
        if st == 2:  # AMDSMI_STATUS_NOT_SUPPORTED: caller falls back to /proc fd scan
            raise NotImplementedError("amdsmi process list not supported")
        if st not in (0, 39):
            raise InventoryError(f"process list gpu {index}: {smi.gm_smi_strerror(st).decode()}")
        return [GpuProcess(int(buf[i].pid), int(buf[i].vram_bytes), int(buf[i].gtt_bytes),
                           int(buf[i].cu_occupancy), buf[i].name.decode(errors="replace"))
                for i in range(min(n.value, cap))]

    def ecc(self, index: int) -> Optional[Tuple[int, int, int]]:
        """(correctable, uncorrectable, deferred) accumulated ECC errors, or None when the
        driver does not report them."""
        ce, ue, de = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        st = _native.smi().gm_smi_ecc(index, C.byref(ce), C.byref(ue), C.byref(de))
        if st != 0:
            return None
        return ce.value, ue.value, de.value

    def healthy(self) -> Dict[int, bool]:
        """Per-GPU health for placement and the device plugin:

        * liveness — the device still answers amdsmi queries with the identity it was enumerated
          with (a GPU that fell off the bus or was reset into another partition mode fails);
        * memory errors, by ``ecc_policy``: ``new`` (default) fails a GPU whose uncorrectable
          ECC count rose since this process first looked (a fresh hardware fault), ``any``
          fails every GPU with an uncorrectable error on record, ``off`` ignores ECC.
        A GPU never recovers from an ECC failure within the process (drain it, then restart
        the worker after repair)."""
        smi = _native.smi()
        out: Dict[int, bool] = {}
        for g in self.gpus():
            info = _native.GpuInfo()
            st = smi.gm_smi_gpu_info(g.index, C.byref(info))
            ok = st == 0 and info.bdf.decode().lower() == g.bdf
            if ok and self.ecc_policy != "off":
                counts = self.ecc(g.index)
                if counts is not None:
                    ue = counts[1]
                    base = self._ecc_base.setdefault(g.index, ue)
                    if (self.ecc_policy == "any" and ue > 0) or ue > base:
                        self._ecc_failed.add(g.index)
            out[g.index] = ok and g.index not in self._ecc_failed
        return out

    def summary(self) -> Dict:
        gs = self.gpus()
        return {"lib": self.lib_path, "kfd_major": self.kfd_major, "count": len(gs),
                "gpus": [g.to_dict() for g in gs], "links": self.links().to_dict()}
