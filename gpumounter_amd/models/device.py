"""Device model for AMD Instinct GPUs.

Reference: ``NvidiaGPU{MinorNumber, DeviceFilePath, UUID, State, PodName, Namespace}`` with a single
device file ``/dev/nvidia<minor>`` of fixed major 195 (reference: pkg/device/nvidia.go:10-41).
An AMD GPU is reached through *several* nodes: the shared ``/dev/kfd`` (dynamic major, compute
queues) plus a per-GPU DRM render node ``/dev/dri/renderD<N>`` (major 226; KFD checks the device
cgroup against it) and, for tools such as rocm-smi, ``/dev/dri/card<N>``.
"""
from __future__ import annotations

import enum
import json
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional, Tuple

DRM_MAJOR = 226
DEFAULT_KFD_MAJOR = 511  # typical; the real value is read from /sys/class/kfd/kfd/dev


class GpuState(str, enum.Enum):
    FREE = "GPU_FREE_STATE"            # reference nvidia.go:20-21
    ALLOCATED = "GPU_ALLOCATED_STATE"


@dataclass(frozen=True)
class DeviceNode:
    """A character device to expose inside a container."""

    path: str          # absolute path inside the container, e.g. "/dev/dri/renderD128"
    major: int
    minor: int
    mode: int = 0o666

    def cgroup_rule(self, access: str = "rw") -> str:
        return f"c {self.major}:{self.minor} {access}"


@dataclass
class AmdGpu:
    index: int
    uuid: str
    bdf: str
    render_minor: int
    card_minor: int
    kfd_gpu_id: int = 0
    kfd_node_id: int = -1
    hip_id: int = -1
    xgmi_hive_id: int = 0
    xgmi_node_id: int = 0
    numa_node: int = -1
    partition_id: int = 0
    compute_partition: str = ""
    memory_partition: str = ""
    market_name: str = ""
    gfx_target: str = ""
    num_cu: int = 0
    vram_bytes: int = 0
    # ledger view (reference: State/PodName/Namespace, nvidia.go:14-16)
    state: GpuState = GpuState.FREE
    pod_name: str = ""
    namespace: str = ""
    container: str = ""

    # -------------------------------------------------------------------------------------
    @property
    def render_path(self) -> str:
        return f"/dev/dri/renderD{self.render_minor}"

    @property
    def card_path(self) -> str:
        return f"/dev/dri/card{self.card_minor}"

    @property
    def physical_id(self) -> str:
        """Physical package key: partitions of one OAM share domain:bus (CPX/NPS modes)."""
        return self.bdf.rsplit(":", 1)[0] if self.bdf else str(self.index)

    def device_nodes(self, drm_major: int = DRM_MAJOR, include_card: bool = True,
                     mode: int = 0o666) -> List[DeviceNode]:
        nodes = [DeviceNode(self.render_path, drm_major, self.render_minor, mode)]
        if include_card and self.card_minor >= 0:
            nodes.append(DeviceNode(self.card_path, drm_major, self.card_minor, mode))
        return nodes

    def ledger_keys(self) -> Tuple[str, ...]:
        """Every spelling a device plugin may use as this GPU's device ID.

        ROCm/k8s-device-plugin advertises PCI addresses; other plugins use UUIDs or node names.
        The join is done on all of them (lower-cased), see :func:`normalize_device_id`.
        Memoised on the identity fields (they never change for a GPU).
        """
        ident = (self.uuid, self.bdf, self.render_minor, self.card_minor)
        memo = self.__dict__.get("_keys_memo")
        if memo is not None and memo[0] == ident:
            return memo[1]
        keys = {self.uuid, self.bdf, self.bdf.split(":", 1)[-1] if self.bdf else "",
                f"renderD{self.render_minor}", f"card{self.card_minor}",
                f"GPU-{self.uuid}" if self.uuid else ""}
        out = tuple(sorted(normalize_device_id(k) for k in keys if k))
        self.__dict__["_keys_memo"] = (ident, out)
        return out

    def reset_state(self) -> None:
        self.state = GpuState.FREE
        self.pod_name = self.namespace = self.container = ""

    def to_dict(self) -> Dict:
        d = asdict(self)
        d["state"] = self.state.value
        # 64-bit ids as decimal strings, as the gRPC schema's JSON mapping renders uint64
        # (Device.xgmi_hive_id): a JSON number that large loses digits in JS and jq
        d["xgmi_hive_id"] = str(self.xgmi_hive_id)
        d["xgmi_node_id"] = str(self.xgmi_node_id)
        return d

    def __str__(self) -> str:  # mirrors the reference's JSON String() (nvidia.go:43-50)
        return json.dumps({"index": self.index, "uuid": self.uuid, "bdf": self.bdf,
                           "render": self.render_path, "state": self.state.value,
                           "pod": self.pod_name, "namespace": self.namespace})


def normalize_device_id(s: str) -> str:
    return s.strip().lower()


def kfd_node(major: int) -> DeviceNode:
    return DeviceNode("/dev/kfd", major, 0, 0o666)


@dataclass
class LinkMatrix:
    """Pairwise GPU links from amdsmi (type: 0 internal, 1 PCIe, 2 xGMI, 3 n/a, 4 unknown)."""

    n: int
    types: List[List[int]] = field(default_factory=list)
    hops: List[List[int]] = field(default_factory=list)
    weights: List[List[int]] = field(default_factory=list)

    XGMI = 2
    PCIE = 1

    def is_xgmi(self, a: int, b: int) -> bool:
        return self.types[a][b] == self.XGMI

    def to_dict(self) -> Dict:
        return {"n": self.n, "types": self.types, "hops": self.hops, "weights": self.weights}


def gpus_by_key(gpus: List[AmdGpu]) -> Dict[str, AmdGpu]:
    out: Dict[str, AmdGpu] = {}
    for g in gpus:
        for k in g.ledger_keys():
            out.setdefault(k, g)
    return out


def find_gpu(gpus: List[AmdGpu], device_id: str) -> Optional[AmdGpu]:
    return gpus_by_key(gpus).get(normalize_device_id(device_id))
