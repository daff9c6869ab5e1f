"""``gpu_mount`` RPC schema — wire-compatible with the reference's api.proto.

Reference: pkg/api/gpu-mount/api.proto:1-45 (package ``gpu_mount``; services ``AddGPUService`` and
``RemoveGPUService``; full method names api.pb.go:356,428). Field numbers and enum values below are
identical, so a reference Go master can call this worker and vice versa. Fields numbered ≥5 in
requests and ≥2 in responses are additive extensions (ignored by the reference) that carry the
attached devices, per-stage timings and a human-readable message. ``NodeService`` is new.
The canonical text form lives in ``gpumounter_amd/api/gpu_mount.proto``.
"""
from __future__ import annotations

from gpumounter_amd.api.protodef import ProtoFile, method_path

PACKAGE = "gpu_mount"

_pf = ProtoFile("gpu_mount/api.proto", PACKAGE)
_pf.message("AddGPURequest", [
    ("pod_name", 1, "string", "opt"),
    ("namespace", 2, "string", "opt"),
    ("gpu_num", 3, "int32", "opt"),
    ("is_entire_mount", 4, "bool", "opt"),
    # --- extensions
    ("container", 5, "string", "opt"),          # target container (default: all containers)
    ("request_id", 6, "string", "opt"),
    ("idempotency_key", 7, "string", "opt"),    # client retry key: same key → same attach
    ("requested_by", 8, "string", "opt"),       # caller identity from the master's authn (audit)
    ("lease_s", 9, "double", "opt"),            # > 0: detach automatically after this long
])
_pf.message("Device", [
    ("uuid", 1, "string", "opt"),
    ("bdf", 2, "string", "opt"),
    ("index", 3, "int32", "opt"),
    ("render_minor", 4, "int32", "opt"),
    ("card_minor", 5, "int32", "opt"),
    ("numa_node", 6, "int32", "opt"),
    ("xgmi_hive_id", 7, "uint64", "opt"),
    ("placeholder", 8, "string", "opt"),
])
_pf.message("StageTiming", [("name", 1, "string", "opt"), ("ms", 2, "double", "opt")])
_pf.message("AddGPUResponse", [
    ("add_gpu_result", 1, "enum:.gpu_mount.AddGPUResponse.AddGPUResult", "opt"),
    ("devices", 2, "msg:.gpu_mount.Device", "rep"),
    ("message", 3, "string", "opt"),
    ("timings", 4, "msg:.gpu_mount.StageTiming", "rep"),
    ("total_ms", 5, "double", "opt"),
], enums={"AddGPUResult": [("Success", 0), ("InsufficientGPU", 1), ("PodNotFound", 2)]})
_pf.message("RemoveGPURequest", [
    ("pod_name", 1, "string", "opt"),
    ("namespace", 2, "string", "opt"),
    ("uuids", 3, "string", "rep"),
    ("force", 4, "bool", "opt"),
    ("container", 5, "string", "opt"),
    ("request_id", 6, "string", "opt"),
    ("requested_by", 7, "string", "opt"),
])
_pf.message("RemoveGPUResponse", [
    ("remove_gpu_result", 1, "enum:.gpu_mount.RemoveGPUResponse.RemoveGPUResult", "opt"),
    ("devices", 2, "msg:.gpu_mount.Device", "rep"),
    ("message", 3, "string", "opt"),
    ("timings", 4, "msg:.gpu_mount.StageTiming", "rep"),
    ("total_ms", 5, "double", "opt"),
    ("killed_pids", 6, "int32", "rep"),
], enums={"RemoveGPUResult": [("Success", 0), ("GPUBusy", 1), ("PodNotFound", 2),
                              ("GPUNotFound", 4)]})  # 3 is skipped in the reference too
_pf.message("NodeStatusRequest", [("include_processes", 1, "bool", "opt")])
_pf.message("NodeStatusResponse", [("json", 1, "string", "opt")])
_pf.service("AddGPUService", [("AddGPU", "AddGPURequest", "AddGPUResponse")])
_pf.service("RemoveGPUService", [("RemoveGPU", "RemoveGPURequest", "RemoveGPUResponse")])
_pf.service("NodeService", [("GetNodeStatus", "NodeStatusRequest", "NodeStatusResponse")])
_classes = _pf.build()

AddGPURequest = _classes["AddGPURequest"]
AddGPUResponse = _classes["AddGPUResponse"]
RemoveGPURequest = _classes["RemoveGPURequest"]
RemoveGPUResponse = _classes["RemoveGPUResponse"]
Device = _classes["Device"]
StageTiming = _classes["StageTiming"]
NodeStatusRequest = _classes["NodeStatusRequest"]
NodeStatusResponse = _classes["NodeStatusResponse"]

ADD_SUCCESS = AddGPUResponse.Success
ADD_INSUFFICIENT = AddGPUResponse.InsufficientGPU
ADD_POD_NOT_FOUND = AddGPUResponse.PodNotFound
REMOVE_SUCCESS = RemoveGPUResponse.Success
REMOVE_BUSY = RemoveGPUResponse.GPUBusy
REMOVE_POD_NOT_FOUND = RemoveGPUResponse.PodNotFound
REMOVE_GPU_NOT_FOUND = RemoveGPUResponse.GPUNotFound

ADD_GPU = method_path(PACKAGE, "AddGPUService", "AddGPU")
REMOVE_GPU = method_path(PACKAGE, "RemoveGPUService", "RemoveGPU")
NODE_STATUS = method_path(PACKAGE, "NodeService", "GetNodeStatus")
