"""Kubernetes device-plugin API ``v1beta1`` (k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1).

Not part of the reference — it relies on NVIDIA's device plugin to hand slave pods their GPUs and
cannot influence *which* GPUs (reference: pkg/util/gpu/allocator/allocator.go:214-231, SURVEY
§2.4). gpumounter-amd can serve ``amd.com/gpu`` itself (gpumounter_amd/deviceplugin) so that
``GetPreferredAllocation`` steers every placeholder to the xGMI/NUMA-chosen set. Field numbers
follow the upstream api.proto, so the kubelet talks to it like to any other plugin.
"""
from __future__ import annotations

from gpumounter_amd.api.protodef import ProtoFile, method_path

PACKAGE = "v1beta1"
VERSION = "v1beta1"
KUBELET_SOCKET = "kubelet.sock"
DEVICE_PLUGIN_DIR = "/var/lib/kubelet/device-plugins"
HEALTHY, UNHEALTHY = "Healthy", "Unhealthy"

_pf = ProtoFile("gpumounter_amd/deviceplugin_v1beta1.proto", PACKAGE)
_p = f".{PACKAGE}."
_pf.message("DevicePluginOptions", [
    ("pre_start_required", 1, "bool", "opt"),
    ("get_preferred_allocation_available", 2, "bool", "opt"),
])
_pf.message("RegisterRequest", [
    ("version", 1, "string", "opt"),
    ("endpoint", 2, "string", "opt"),
    ("resource_name", 3, "string", "opt"),
    ("options", 4, f"msg:{_p}DevicePluginOptions", "opt"),
])
_pf.message("Empty")
_pf.message("NUMANode", [("ID", 1, "int64", "opt")])
_pf.message("TopologyInfo", [("nodes", 1, f"msg:{_p}NUMANode", "rep")])
_pf.message("Device", [
    ("ID", 1, "string", "opt"),
    ("health", 2, "string", "opt"),
    ("topology", 3, f"msg:{_p}TopologyInfo", "opt"),
])
_pf.message("ListAndWatchResponse", [("devices", 1, f"msg:{_p}Device", "rep")])
_pf.message("PreStartContainerRequest", [("devices_ids", 1, "string", "rep")])
_pf.message("PreStartContainerResponse")
_pf.message("ContainerPreferredAllocationRequest", [
    ("available_deviceIDs", 1, "string", "rep"),
    ("must_include_deviceIDs", 2, "string", "rep"),
    ("allocation_size", 3, "int32", "opt"),
])
_pf.message("PreferredAllocationRequest", [
    ("container_requests", 1, f"msg:{_p}ContainerPreferredAllocationRequest", "rep")])
_pf.message("ContainerPreferredAllocationResponse", [("deviceIDs", 1, "string", "rep")])
_pf.message("PreferredAllocationResponse", [
    ("container_responses", 1, f"msg:{_p}ContainerPreferredAllocationResponse", "rep")])
_pf.message("ContainerAllocateRequest", [("devices_ids", 1, "string", "rep")])
_pf.message("AllocateRequest", [
    ("container_requests", 1, f"msg:{_p}ContainerAllocateRequest", "rep")])
_pf.message("Mount", [
    ("container_path", 1, "string", "opt"),
    ("host_path", 2, "string", "opt"),
    ("read_only", 3, "bool", "opt"),
])
_pf.message("DeviceSpec", [
    ("container_path", 1, "string", "opt"),
    ("host_path", 2, "string", "opt"),
    ("permissions", 3, "string", "opt"),
])
_pf.message("CDIDevice", [("name", 1, "string", "opt")])
_pf.message("ContainerAllocateResponse", [
    ("envs", 1, "map:string,string", "rep"),
    ("mounts", 2, f"msg:{_p}Mount", "rep"),
    ("devices", 3, f"msg:{_p}DeviceSpec", "rep"),
    ("annotations", 4, "map:string,string", "rep"),
    ("cdi_devices", 5, f"msg:{_p}CDIDevice", "rep"),
])
_pf.message("AllocateResponse", [
    ("container_responses", 1, f"msg:{_p}ContainerAllocateResponse", "rep")])
_pf.service("Registration", [("Register", "RegisterRequest", "Empty")])
_pf.service("DevicePlugin", [
    ("GetDevicePluginOptions", "Empty", "DevicePluginOptions"),
    ("ListAndWatch", "Empty", "ListAndWatchResponse"),
    ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse"),
    ("Allocate", "AllocateRequest", "AllocateResponse"),
    ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse"),
])
_c = _pf.build()
globals().update(_c)

REGISTER = method_path(PACKAGE, "Registration", "Register")
GET_OPTIONS = method_path(PACKAGE, "DevicePlugin", "GetDevicePluginOptions")
LIST_AND_WATCH = method_path(PACKAGE, "DevicePlugin", "ListAndWatch")
GET_PREFERRED = method_path(PACKAGE, "DevicePlugin", "GetPreferredAllocation")
ALLOCATE = method_path(PACKAGE, "DevicePlugin", "Allocate")
PRE_START = method_path(PACKAGE, "DevicePlugin", "PreStartContainer")
