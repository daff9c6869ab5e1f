"""Shared enums and constants (reference: pkg/util/gpu/types.go:5-28)."""
from __future__ import annotations

import enum


class MountType(str, enum.Enum):
    """How a pod currently holds hot-mounted GPUs (reference types.go:21-28)."""

    ENTIRE = "entire-mount"
    SINGLE = "single-mount"
    NONE = "no-mount"
    UNKNOWN = "unknown-mount"


class AllocStatus(str, enum.Enum):
    """Placeholder lifecycle outcomes (reference types.go:12-16)."""

    INSUFFICIENT = "InsufficientGPU"
    CREATED = "SuccessfullyCreated"
    FAILED_CREATE = "FailedCreated"
    DELETED = "SuccessfullyDeleted"
    FAILED_DELETE = "FailedDeleted"


# Labels / annotations stamped on placeholder pods. The reference used only ``app: gpu-pool``
# and the name convention ``<owner>-slave-pod-<6 hex>`` (allocator.go:197-201); the owner is
# matched by *substring* (collector.go:158, SURVEY defect 3). Here the owner is an exact label
# pair plus the owner UID, and the name convention is kept for operator familiarity.
LABEL_APP = "app"
LABEL_APP_VALUE = "gpu-pool"
LABEL_OWNER = "gpumounter.amd.com/owner"
LABEL_OWNER_NS = "gpumounter.amd.com/owner-namespace"
ANN_OWNER_UID = "gpumounter.amd.com/owner-uid"
ANN_MOUNT_MODE = "gpumounter.amd.com/mount-mode"
ANN_PREFERRED = "gpumounter.amd.com/preferred-devices"
ANN_ATTACH_ID = "gpumounter.amd.com/attach-id"
# the worker process that created a placeholder (random per start): a never-admitted placeholder
# from another incarnation belongs to an attach whose worker died, so nothing waits for it
ANN_INCARNATION = "gpumounter.amd.com/worker-incarnation"
ANN_CONTAINER = "gpumounter.amd.com/container"
ANN_DEVICES = "gpumounter.amd.com/devices"
ANN_OWNER_NAME = "gpumounter.amd.com/owner-name"
ANN_IDEMPOTENCY = "gpumounter.amd.com/idempotency-key"
ANN_GROUP = "gpumounter.amd.com/group"      # entire-mount group made of pooled placeholders
# a ?lease= attach's expiry (Unix seconds) on its placeholders (worker/lease.py)
ANN_LEASE = "gpumounter.amd.com/lease-expires"
MODE_STANDBY = "standby"
# set on the 1-GPU placeholders a trim or placement correction holds while it picks; cleared on
# the kept ones before they are mounted. A worker that dies mid-pick leaves only candidates
# behind, which nothing mounts and the reconciler releases.
ANN_CANDIDATE = "gpumounter.amd.com/candidate"
# a force-removed GPU whose killed processes have not exited yet (worker/drain.py)
MODE_DRAINING = "draining"
ANN_DRAIN_PIDS = "gpumounter.amd.com/drain-pids"      # pid:starttime,... waited on
ANN_DRAIN_OWNER = "gpumounter.amd.com/drained-from"   # ns/name of the pod it was removed from
FINALIZER = "gpumounter.amd.com/release"
SLAVE_SUFFIX = "-slave-pod-"

# Error strings carried in gRPC status details (master maps them to HTTP bodies).
ERR_POLICY = "MountPolicyDenied"
ERR_QUOTA = "QuotaExceeded"
ERR_INTERNAL = "Service Internal Error"
