"""Single configuration object for master, worker, fakes and bench.

The reference hard-codes nearly everything: ports (reference: cmd/GPUMounter-master/main.go:237,
cmd/GPUMounter-worker/main.go:24, master dial main.go:82), namespaces (pkg/util/gpu/types.go:18,
main.go:255-257), the kubelet socket (types.go:6-7), the slave image (allocator.go:218), the
resource name (types.go:10, allocator.go:223) and a placeholder kubeconfig path
(pkg/config/config.go:20); only ``CGROUP_DRIVER`` is read from the environment (cgroup.go:79).

Here every knob lives in :class:`Config`, resolved in order
``defaults → YAML file (GM_CONFIG) → environment (GM_<FIELD>) → explicit overrides``.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, Mapping, Optional

import yaml


@dataclass
class Config:
    # --- network ---------------------------------------------------------------------------
    master_host: str = "0.0.0.0"       # master HTTP API bind address
    master_port: int = 8080            # master HTTP API (reference: main.go:237)
    worker_host: str = "0.0.0.0"       # worker gRPC bind address
    worker_port: int = 1200            # worker gRPC (reference: worker main.go:24)
    # worker gm-wire port (api/wire.py): the gpu_mount messages for gpumounter's own master on
    # one persistent (m)TLS connection, next to the reference-compatible gRPC port; -1 = off
    wire_port: int = 1201
    # how the master calls a worker: auto = gm-wire when the worker pod advertises its port
    # (annotation gpumounter.amd.com/wire-port), else gRPC; grpc = always gRPC
    master_transport: str = "auto"
    metrics_port: int = 9400           # worker /metrics and /healthz
    # after start-up the daemon writes the ports it actually bound ({"grpc_port", "http_port"}
    # or {"port"}) here, atomically; with ports 0 (ephemeral) that is how a supervisor finds
    # them without racing another process for a pre-picked free port. "" = off
    ready_file: str = ""
    # --- kubernetes ------------------------------------------------------------------------
    kube_api: str = ""                 # "" → in-cluster; else http(s)://host:port (fake in tests)
    kubeconfig: str = ""               # kubeconfig file (out-of-cluster runs)
    kube_token: str = ""               # bearer token for kube_api ("" = service account)
    kube_ca: str = ""                  # CA bundle for kube_api ("" = service account CA)
    kube_insecure: bool = False        # skip apiserver certificate checks (labs only)
    node_name: str = ""                # worker's node (downward API NODE_NAME)
    pod_name: str = ""                 # worker's own pod (downward API POD_NAME): never a target
    pod_namespace: str = ""            # (downward API POD_NAMESPACE)
    worker_namespace: str = "kube-system"  # where the master looks for workers
    worker_label: str = "app=gpu-mounter-worker"  # label selector of the worker pods
    pool_namespace: str = "gpu-pool"   # placeholder namespace in "pool" mode
    # "pool": placeholders in pool_namespace (reference layout, allocator.go:198);
    # "tenant": placeholders next to the tenant pod, so the ownerReference is same-namespace and
    # Kubernetes ≥1.20 GC cleans them up (SURVEY §2.6 defect 4).
    placeholder_namespace_mode: str = "pool"
    resource_name: str = "amd.com/gpu"  # extended resource placeholders request
    # how the cluster hands out GPUs: "device-plugin" (the amd.com/gpu extended resource of the
    # ROCm device plugin; the reference's model) or "dra" (a DRA driver publishes them in
    # ResourceSlices; placeholders then hold ResourceClaims pinned to the chosen devices)
    gpu_allocation: str = "device-plugin"
    dra_driver: str = "gpu.amd.com"    # DRA driver name in ResourceSlices
    dra_device_class: str = "gpu.amd.com"  # DeviceClass placeholder claims request
    dra_bdf_attribute: str = "pciAddr"    # ResourceSlice device attribute holding the PCI BDF
    placeholder_image: str = "registry.k8s.io/pause:3.9"  # placeholder container image
    placeholder_pull_policy: str = "IfNotPresent"  # no registry round trip per attach
    # How placeholders reach the node: "scheduler" = a nodeSelector, kube-scheduler binds them
    # (the reference: allocator.go:189-234); "direct" = spec.nodeName set at creation, so the
    # kubelet admits them without a scheduling cycle and bind write. Direct binding bypasses the
    # scheduler: its nominations for preemptors and a Pod it binds to the node at the same
    # moment (which the kubelet may then reject, OutOfamd.com/gpu). Not with gpu_allocation=dra
    # (the scheduler allocates ResourceClaims)
    placeholder_binding: str = "scheduler"
    # The floor PriorityClass of placeholders (deploy/placeholder-priority.yaml: value 1000000,
    # preemptionPolicy Never). A placeholder backs a GPU its tenant is using, so it must never
    # rank below that tenant: it gets this class, or the tenant's own class when the tenant
    # ranks higher (placeholder_priority_inherit). If the class does not exist in the cluster
    # the tenant's class is used ("" = no floor: always the tenant's class). The reference sets
    # no priority (allocator.go:189-234): any higher-priority amd.com/gpu Pod could preempt a
    # slave pod and take a GPU out from under its running tenant.
    placeholder_priority_class: str = "gpumounter-placeholder"
    placeholder_priority_inherit: bool = True  # tenants above the floor: their own class
    # The floor class's value when the worker may not read PriorityClasses (RBAC) — it reads it
    # from the apiserver otherwise
    placeholder_priority_value: int = 1000000
    # Warm pool: standby placeholders that keep this many GPUs per node pre-admitted for
    # hot-mount (0 = off, the reference's behaviour). Claiming is a metadata patch, so attach
    # latency no longer includes scheduling + kubelet admission; the price is reserved capacity.
    warm_pool_size: int = 0
    # PriorityClass of standby placeholders ("" = placeholder_priority_class: standbys are not
    # preemptible and a claim keeps the pool's latency). A lower class (gpumounter-standby,
    # value -10) lets higher-priority Pods preempt idle standbys; because Pod priority is
    # immutable, an attach then cannot keep a low standby: it yields it (DELETE) and books the
    # GPU with a placeholder at tenant priority — the cold path's latency (docs/CONFIG.md)
    pool_priority_class: str = ""
    # --- kubelet PodResources --------------------------------------------------------------
    kubelet_socket: str = "/var/lib/kubelet/pod-resources/kubelet.sock"  # PodResources API
    kubelet_timeout_s: float = 10.0    # per PodResources call (reference: types.go:7)
    podresources_api: str = "auto"     # auto | v1 | v1alpha1
    # client-side pacing of PodResources calls, under the kubelet's own limiter (100 qps,
    # burst 10, RESOURCE_EXHAUSTED beyond it) which other node agents share; 0 = unpaced
    kubelet_qps: float = 50.0
    # where admission reads a placeholder's GPUs: "auto" = the device manager's checkpoint file
    # (by pod UID, inotify-woken, no RPC: node/checkpoint.py) with PodResources as fallback and
    # authority; "podresources" = always the RPC
    ledger_source: str = "auto"
    # the device manager's checkpoint file that ledger_source=auto reads
    kubelet_checkpoint: str = "/var/lib/kubelet/device-plugins/kubelet_internal_checkpoint"
    kubelet_burst: int = 8             # burst of the client-side PodResources pacing
    # --- device & isolation ----------------------------------------------------------------
    amdsmi_lib: str = ""               # "" → libamd_smi.so from ROCm; "mock" → bundled mock
    cgroup_root: str = "/sys/fs/cgroup"  # host cgroup mount as the worker sees it
    cgroup_mode: str = "auto"          # auto | v1 | v2
    cgroup_driver: str = "auto"        # auto | cgroupfs | systemd
    # record hot-mounted nodes in the container scope's DeviceAllow= so systemd keeps them when
    # it re-realises the unit: auto (systemd-named cgroup + bus socket present) | on | off
    systemd_device_allow: str = "auto"
    systemd_bus: str = ""              # "" = /run/systemd/private, then the system bus socket
    bpf_pin_dir: str = "/sys/fs/bpf/gpumounter"  # bpffs dir for v2 tail-call maps ("" = keep fd)
    # cgroup v2: allow-set map looked up by a fixed program (grants/revokes are map updates);
    # false = one straight-line program per update (the previous scheme; a kill switch)
    bpf_set_mode: bool = True
    devnode_mode: str = "procroot"     # procroot | setns | emulate
    # containers in their own user namespace (hostUsers: false) get bind-mounted nodes, because
    # mknod'ed ones on their nodev /dev cannot be opened: auto (detect per container) | bind
    # (every container) | off (always mknod)
    devnode_userns: str = "auto"
    devnode_stage_dir: str = "/run/gpumounter/devstage"  # worker-private tmpfs for bind mode
    proc_root: str = "/proc"           # host /proc (the DaemonSet runs with hostPID)
    # For hermetic runs: containers' rootfs live at <container_root_prefix>/<container-id>/ and
    # device-node writes go there instead of /proc/<pid>/root.
    container_root_prefix: str = ""
    # node-local injection journal (what gpumounter put into which container; node/journal.py).
    # The DaemonSet mounts it from the host so it outlives worker restarts; "" = in memory only
    state_dir: str = "/var/lib/gpumounter"
    # the host's /dev as the worker sees it (hostPID: /proc/1/root/dev). mknod/unlink are refused
    # in any container directory that *is* this /dev or its dri/ (hostPath or privileged /dev);
    # "" = no guard
    host_dev_path: str = "/proc/1/root/dev"
    drm_major: int = 226               # /dev/dri/* character-device major
    kfd_major: int = 0                 # 0 → read /sys/class/kfd/kfd/dev (fallback 511)
    kfd_dev_path: str = "/sys/class/kfd/kfd/dev"  # sysfs file holding the KFD major:minor
    # KFD's process table (<host pid>/vram_<gpu_id>): busy detection's source for PIDs whose
    # fd table is unreadable, before amdsmi; "" = amdsmi only
    kfd_proc_path: str = "/sys/class/kfd/kfd/proc"
    inject_card_nodes: bool = True     # also inject /dev/dri/card<N> (rocm-smi reads it)
    device_file_mode: int = 0o666      # reference: nvidia.go:39 "666"
    # --- policy ----------------------------------------------------------------------------
    topology_policy: str = "xgmi"      # xgmi | first-fit
    # auto: exact where the cluster offers a way (gpumounter's own device plugin, a DRA CEL
    #   selector); otherwise take what the device plugin admits and, if it is worse-placed than
    #   the topology choice, hold the other free GPUs and keep the best (one extra round only
    #   when the plugin chose badly);
    # trim: always hold every free GPU with 1-GPU placeholders, keep the topology-chosen ones
    #   (SURVEY §7.4.3);
    # hint: the preferred set is only an annotation (no shipped device plugin reads it).
    # Default auto since round 3 (before: hint, the reference's topology-blind behaviour). A
    # correction holds one 1-GPU placeholder per free GPU for a moment under the node's
    # exclusive reservation gate (other attaches on the node wait for it), and in tenant
    # placeholder-namespace mode those holds count against the tenant's quota;
    # gm_placement_corrections_total counts them
    placement_enforce: str = "auto"
    # which worse placement auto corrects: numa = any worse score (hive split, non-xGMI pair or
    # a NUMA split); xgmi = only a hive split or a non-xGMI pair (fewer corrections on nodes
    # whose GPUs all share one hive, at the cost of NUMA-split sets)
    placement_correct_on: str = "numa"
    ledger_get: bool = True            # read admitted placeholders with PodResources v1 Get
    reconcile_on_events: bool = True   # react to placeholder/tenant deletes at once
    # auto: fd scan of the container's PIDs, the KFD/amdsmi process table only for PIDs whose
    # fd table is unreadable; both: always union with the table. The tables name host-namespace
    # PIDs, so the worker consults them only when it runs with hostPID: true
    busy_detection: str = "auto"
    gc_tune: bool = True               # gc.freeze() after startup + larger young-gen threshold
    # pin the daemon to these CPUs at start ("2-3,8", cpuset list format; "" = unpinned): on a
    # node whose kubelet runs the static CPU manager, give the DaemonSet a Guaranteed CPU and
    # the same list here, so request wake-ups land on a core nothing else uses
    cpu_affinity: str = ""
    emit_events: bool = True           # core/v1 Events on the tenant pod (kubectl describe)
    annotate_tenant: bool = False      # keep gpumounter.amd.com/devices on the tenant pod current
    # Events/annotations are sent once the worker has had no attach/detach in flight for
    # notify_idle_ms (so they never compete with a request), but at most notify_max_delay_ms late
    notify_idle_ms: float = 2.0
    notify_max_delay_ms: float = 1000.0  # upper bound on that delay
    # serve amd.com/gpu ourselves (replaces the ROCm device plugin on the node) so
    # GetPreferredAllocation steers placeholders to the topology-chosen GPUs
    device_plugin: bool = False
    device_plugin_dir: str = "/var/lib/kubelet/device-plugins"  # kubelet registration dir
    device_plugin_inject: bool = True     # False: no device specs (kind / mock inventory)
    device_plugin_health_s: float = 5.0   # react to foreign placeholder / owner deletes at once
    max_gpus_per_request: int = 64     # addgpu gpuNum upper bound
    # GPUs with uncorrectable memory errors are left out of placement and reported Unhealthy by
    # the device plugin: new (errors since the worker started) | any (any on record) | off
    ecc_policy: str = "new"
    health_period_s: float = 5.0       # liveness + ECC re-check period
    # leases (?lease=<s> on addgpu): detach at expiry; GPUs still in use are kept and retried
    # unless lease_force, which signals their processes like force=1
    lease_force: bool = False
    lease_retry_s: float = 30.0        # retry period for an expired lease whose GPUs are busy
    # read the device rules and nodes back after each attach (span "verify": one native
    # read-back of every node plus the kernel's rule set per container) and roll back if
    # anything did not take effect; off = rely on the reconciler's periodic audit
    attach_verify: bool = True
    # pool-namespace placeholders are invisible to the tenant namespace's ResourceQuota; enforce
    # requests.<resource_name> quotas for hot-mounted GPUs ourselves (cluster/quota.py) | off
    quota_mode: str = "enforce"
    kill_signal: int = 15              # SIGTERM like the reference's `kill` (namespace.go:192)
    kill_grace_s: float = 5.0          # then SIGKILL
    # after SIGKILL, wait this long for the processes to exit before answering; the GPU stays
    # booked (draining placeholder) until they have, however long that takes
    kill_reap_s: float = 2.0
    # --- timeouts / loops ------------------------------------------------------------------
    attach_timeout_s: float = 120.0    # placeholder admission deadline
    rpc_timeout_s: float = 180.0       # master→worker gRPC deadline (reference: none)
    reconcile_period_s: float = 30.0   # full reconciler sweep period
    # every this many seconds, compare each hot container's device-control state (v2: the
    # attached BPF program ids; v1: devices.list) with what gpumounter last installed, and
    # repair at once when the runtime, runc update or systemd replaced it (0 = only the sweep)
    device_guard_period_s: float = 1.0
    watch_resync_s: float = 300.0      # server-side timeout of one watch request
    api_token: str = ""                # if set, add/remove require "Authorization: Bearer <token>"
    # kube: the caller's own token, TokenReview + SubjectAccessReview on pods/gpumount (default);
    # none: open like the reference (SURVEY defect 13) unless api_token is set — opt-in only
    authz_mode: str = "kube"
    # how long a TokenReview / SubjectAccessReview answer is reused. A decision used after half
    # its lifetime is refreshed in the background; once expired, the next request re-runs the
    # TokenReview and, for a token seen before, the SubjectAccessReview at the same time (one
    # apiserver round trip instead of two)
    authz_token_ttl_s: float = 60.0
    authz_sar_ttl_s: float = 30.0      # the same for SubjectAccessReview answers
    # a token seen for the first time: its TokenReview and a SelfSubjectAccessReview made with
    # the caller's own token go out together (one round trip instead of two where the
    # apiserver's round trip is network-bound; falls back to a SubjectAccessReview where the
    # self-review is not served). Off by default: against the single-process fake apiserver
    # the two concurrent reviews cost 0.2 ms more than two serial ones (profiles/r5_cold/).
    # Only when the master talks to the apiserver with a bearer token: with a client
    # certificate the apiserver would review the master
    authz_self_review: bool = False
    # the master keeps a slim list+watch index of every Pod (name → uid, node, phase) so an
    # attach needs no Pod GET; off: a GET on a miss, answers cached for 30 s
    master_pod_index: bool = True
    # master⇄worker gRPC TLS (reference: insecure, main.go:82). cert+key on the worker enable TLS;
    # a CA on the worker requires client certs (mTLS). The master uses the same three files.
    tls_cert: str = ""
    tls_key: str = ""                  # private key of tls_cert
    tls_ca: str = ""                   # CA that signs peers (worker: requires client certs)
    tls_server_name: str = "gpu-mounter-worker"  # SAN the worker certificate carries
    # identities (certificate SAN DNS names or CN) the worker accepts RPCs from under mTLS;
    # "" = any certificate the CA signed
    tls_client_names: str = "gpu-mounter-master"
    # the worker refuses to serve its gRPC API (which can kill tenant processes) without mTLS
    # unless this is set explicitly (hermetic tests, lab clusters)
    worker_insecure: bool = False
    # HTTPS on the master's API port: callers send bearer tokens (authz_mode=kube), which must
    # not cross the pod network in clear. cert+key set = TLS only on master_port (the shipped
    # deploy sets both; the reference served plain HTTP, main.go:235-240)
    master_tls_cert: str = ""
    master_tls_key: str = ""           # private key of master_tls_cert
    # who may read the worker's /status (every Pod's GPUs on the node) and /audit/{ns}/{pod}:
    # auto = authz_mode (kube: "get" on nodes/gpumount resp. pods/gpumount, as the master's
    # read routes ask); none = open. /healthz, /readyz and /metrics stay open for probes
    status_authz: str = "auto"
    metrics_period_s: float = 15.0     # refresh of the per-GPU process and ledger gauges
    # serve /debug/tasks (every asyncio task's stack) on the worker's metrics port; it has no
    # authentication and that port binds worker_host, so it is off unless asked for
    debug_endpoints: bool = False
    # --- observability ---------------------------------------------------------------------
    log_level: str = "INFO"            # DEBUG | INFO | WARNING | ERROR
    log_file: str = ""                 # also log to this file, rotated ("" = stderr only)
    log_json: bool = True              # one JSON object per line, with request ids
    # roctx ranges per stage (rocprofv3 --marker-trace): emitted when a profiler is attached
    # (its preloaded tool library) or GM_ROCTX=on; without one they are pure cost
    roctx: bool = True
    fault: str = ""                    # fault injection: "stage:prob[,stage:prob]"
    extra: Dict[str, Any] = field(default_factory=dict)

    # -------------------------------------------------------------------------------------
    @classmethod
    def load(cls, path: Optional[str] = None, env: Optional[Mapping[str, str]] = None,
             **overrides: Any) -> "Config":
        env = os.environ if env is None else env
        cfg = cls()
        path = path or env.get("GM_CONFIG", "")
        if path:
            with open(path, "r", encoding="utf-8") as fh:
                data = yaml.safe_load(fh) or {}
            if not isinstance(data, dict):
                raise ValueError(f"config file {path} must hold a mapping")
            cfg.update(data)
        env_vals: Dict[str, Any] = {}
        for f in fields(cls):
            key = "GM_" + f.name.upper()
            if key in env:
                env_vals[f.name] = env[key]
        # compatibility with the reference's only env knob (cgroup.go:79)
        if "cgroup_driver" not in env_vals and env.get("CGROUP_DRIVER"):
            env_vals["cgroup_driver"] = env["CGROUP_DRIVER"]
        for f, k in (("node_name", "NODE_NAME"), ("pod_name", "POD_NAME"),
                     ("pod_namespace", "POD_NAMESPACE")):
            if f not in env_vals and env.get(k):
                env_vals[f] = env[k]
        cfg.update(env_vals)
        cfg.update({k: v for k, v in overrides.items() if v is not None})
        cfg.validate()
        return cfg

    def update(self, values: Mapping[str, Any]) -> None:
        known = {f.name: f for f in fields(self)}
        for k, v in values.items():
            if k not in known:
                self.extra[k] = v
                continue
            setattr(self, k, _coerce(known[k], v))

    def replace(self, **kw: Any) -> "Config":
        c = dataclasses.replace(self, extra=dict(self.extra))
        c.update(kw)
        c.validate()
        return c

    def validate(self) -> None:
        _choice("cgroup_mode", self.cgroup_mode, ("auto", "v1", "v2"))
        _choice("cgroup_driver", self.cgroup_driver, ("auto", "cgroupfs", "systemd"))
        _choice("systemd_device_allow", self.systemd_device_allow, ("auto", "on", "off"))
        _choice("quota_mode", self.quota_mode, ("enforce", "off"))
        _choice("ecc_policy", self.ecc_policy, ("new", "any", "off"))
        _choice("devnode_mode", self.devnode_mode, ("procroot", "setns", "emulate"))
        _choice("devnode_userns", self.devnode_userns, ("auto", "bind", "off"))
        _choice("topology_policy", self.topology_policy, ("xgmi", "first-fit"))
        _choice("placement_enforce", self.placement_enforce, ("auto", "hint", "trim"))
        _choice("placement_correct_on", self.placement_correct_on, ("numa", "xgmi"))
        _choice("busy_detection", self.busy_detection, ("auto", "both"))
        _choice("authz_mode", self.authz_mode, ("none", "kube"))
        _choice("status_authz", self.status_authz, ("auto", "none", "kube"))
        if bool(self.master_tls_cert) != bool(self.master_tls_key):
            raise ValueError("master_tls_cert and master_tls_key go together")
        _choice("placeholder_namespace_mode", self.placeholder_namespace_mode, ("pool", "tenant"))
        _choice("podresources_api", self.podresources_api, ("auto", "v1", "v1alpha1"))
        _choice("ledger_source", self.ledger_source, ("auto", "podresources"))
        _choice("gpu_allocation", self.gpu_allocation, ("device-plugin", "dra"))
        _choice("master_transport", self.master_transport, ("auto", "grpc"))
        _choice("placeholder_binding", self.placeholder_binding, ("scheduler", "direct"))
        if self.gpu_allocation == "dra" and self.placeholder_binding == "direct":
            raise ValueError("placeholder_binding=direct: with gpu_allocation=dra the scheduler "
                             "must allocate the placeholders' ResourceClaims")
        if self.gpu_allocation == "dra" and self.device_plugin:
            raise ValueError("device_plugin serves the extended resource; with "
                             "gpu_allocation=dra the GPUs belong to the DRA driver")
        if not (0 <= self.worker_port < 65536 and 0 <= self.master_port < 65536 and
                -1 <= self.wire_port < 65536):
            raise ValueError("ports out of range")

    def as_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


def _choice(name: str, value: str, allowed) -> None:
    if value not in allowed:
        raise ValueError(f"{name}={value!r} not in {allowed}")


def _coerce(f: dataclasses.Field, v: Any) -> Any:
    t = f.type if isinstance(f.type, str) else getattr(f.type, "__name__", str(f.type))
    if isinstance(v, str):
        if t == "bool":
            low = v.strip().lower()
            if low in ("1", "t", "true", "yes", "on"):
                return True
            if low in ("0", "f", "false", "no", "off", ""):
                return False
            raise ValueError(f"bad boolean for {f.name}: {v!r}")
        if t == "int":
            return int(v, 0)
        if t == "float":
            return float(v)
    if t == "int" and isinstance(v, bool):
        raise ValueError(f"bad int for {f.name}: {v!r}")
    if t == "int":
        return int(v)
    if t == "float":
        return float(v)
    return v
