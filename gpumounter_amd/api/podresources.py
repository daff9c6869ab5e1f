"""kubelet PodResources API (v1 and v1alpha1), built at runtime.

Reference: the worker imports ``k8s.io/kubernetes/pkg/kubelet/apis/podresources/v1alpha1`` and only
calls ``List`` (reference: pkg/util/gpu/collector/collector.go:16,182-194). v1alpha1 was removed
from kubelet 1.2x; v1 adds ``GetAllocatableResources`` (which devices the plugin exposes) and
``Get`` (one pod). Both are defined here with the upstream field numbers so a real kubelet socket
and the hermetic FakeKubelet speak the same wire format.
"""
from __future__ import annotations

from gpumounter_amd.api.protodef import ProtoFile, method_path


def _define(package: str, v1: bool):
    pf = ProtoFile(f"podresources/{package}/api.proto", package)
    p = f".{package}."
    pf.message("ListPodResourcesRequest")
    pf.message("ListPodResourcesResponse", [("pod_resources", 1, f"msg:{p}PodResources", "rep")])
    pf.message("PodResources", [
        ("name", 1, "string", "opt"),
        ("namespace", 2, "string", "opt"),
        ("containers", 3, f"msg:{p}ContainerResources", "rep"),
    ])
    cr = [("name", 1, "string", "opt"), ("devices", 2, f"msg:{p}ContainerDevices", "rep")]
    cd = [("resource_name", 1, "string", "opt"), ("device_ids", 2, "string", "rep")]
    if v1:
        cr += [("cpu_ids", 3, "int64", "rep"), ("memory", 4, f"msg:{p}ContainerMemory", "rep")]
        cd += [("topology", 3, f"msg:{p}TopologyInfo", "opt")]
        pf.message("TopologyInfo", [("nodes", 1, f"msg:{p}NUMANode", "rep")])
        pf.message("NUMANode", [("ID", 1, "int64", "opt")])
        pf.message("ContainerMemory", [
            ("memory_type", 1, "string", "opt"),
            ("size", 2, "uint64", "opt"),
            ("topology", 3, f"msg:{p}TopologyInfo", "opt"),
        ])
        pf.message("AllocatableResourcesRequest")
        pf.message("AllocatableResourcesResponse", [
            ("devices", 1, f"msg:{p}ContainerDevices", "rep"),
            ("cpu_ids", 2, "int64", "rep"),
            ("memory", 3, f"msg:{p}ContainerMemory", "rep"),
        ])
        pf.message("GetPodResourcesRequest", [("pod_name", 1, "string", "opt"),
                                              ("pod_namespace", 2, "string", "opt")])
        pf.message("GetPodResourcesResponse", [("pod_resources", 1, f"msg:{p}PodResources", "opt")])
    pf.message("ContainerResources", cr)
    pf.message("ContainerDevices", cd)
    methods = [("List", "ListPodResourcesRequest", "ListPodResourcesResponse")]
    if v1:
        methods += [("GetAllocatableResources", "AllocatableResourcesRequest",
                     "AllocatableResourcesResponse"),
                    ("Get", "GetPodResourcesRequest", "GetPodResourcesResponse")]
    pf.service("PodResourcesLister", methods)
    return pf.build()


class _Api:
    def __init__(self, package: str, v1: bool):
        self.package = package
        self.msgs = _define(package, v1)
        for k, v in self.msgs.items():
            setattr(self, k, v)
        self.LIST = method_path(package, "PodResourcesLister", "List")
        self.ALLOCATABLE = method_path(package, "PodResourcesLister", "GetAllocatableResources")
        self.GET = method_path(package, "PodResourcesLister", "Get")
        self.has_allocatable = v1


V1 = _Api("v1", True)
V1ALPHA1 = _Api("v1alpha1", False)
