"""gpumounter_amd — MI355X-native Kubernetes GPU hot-mount controller.

Adds/removes AMD Instinct GPUs (gfx950) to/from running Pods without restarting them, with the
HTTP API of jason-gideon/GPUMounter (reference: cmd/GPUMounter-master/main.go:231-234) and a
scheduler-consistent placeholder-pod ledger (reference: pkg/util/gpu/allocator/allocator.go).

Layers (bottom → top): ``_native`` (C++/HIP libraries) → ``hw`` (amdsmi inventory, xGMI topology)
→ ``node`` (cgroup v1/v2, device nodes, PodResources ledger, hot-mount transactions) →
``cluster`` (kube REST client, placeholder pods) → ``worker`` (gRPC service, reconciler) →
``master`` (HTTP API). ``ops``/``parallel`` hold the gfx950 validation kernels and the RCCL/xGMI
post-attach checks; ``fakes`` hold the hermetic apiserver/kubelet/cgroupfs used by tests and bench.
"""
import os as _os

# grpc core logs GOAWAY/shutdown chatter at INFO unless told otherwise
_os.environ.setdefault("GRPC_VERBOSITY", "ERROR")

__version__ = "0.1.0"
