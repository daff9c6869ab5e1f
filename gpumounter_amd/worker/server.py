"""Worker daemon: wires inventory, ledger, cgroup/devnode backends, informers, the gRPC services and
the reconciler together.

Reference: ``main`` inits the logger, builds ``GPUMountImpl`` (NVML enumeration + one PodResources
read) and serves ``AddGPUService``/``RemoveGPUService`` on ``:1200`` — logging but *continuing
past* a listen failure (reference: cmd/GPUMounter-worker/main.go:11-39 — SURVEY defect 13). Here a
bind failure is fatal, and the worker also serves ``NodeService`` plus ``/healthz``, ``/readyz``
and ``/metrics`` over HTTP.
"""
from __future__ import annotations

import asyncio
import json
import os
import signal
import time
from typing import Optional

import grpc

from gpumounter_amd.api import gpu_mount as api
from gpumounter_amd.api import wire
from gpumounter_amd.cluster.informer import ClaimInformer, PodInformer, QuotaInformer
from gpumounter_amd.cluster.kube import KubeClient
from gpumounter_amd.cluster.placeholder import LABEL_NODE, PlaceholderManager
from gpumounter_amd.cluster.pool import WarmPool
from gpumounter_amd.hw.inventory import Inventory
from gpumounter_amd.models import pod as podu
from gpumounter_amd.node import procs, systemd
from gpumounter_amd.node.cgroup import CgroupError, CgroupResolver, make_backend
from gpumounter_amd.node.checkpoint import DeviceCheckpoint
from gpumounter_amd.node.devnodes import DevNodeWriter
from gpumounter_amd.node.dra import DraLedger
from gpumounter_amd.node.hotmount import HotMount
from gpumounter_amd.node.journal import InjectionJournal
from gpumounter_amd.node.ledger import LedgerClient
from gpumounter_amd.utils import calls, httpd, log, runtime
from gpumounter_amd.utils.faults import FaultInjector
from gpumounter_amd.utils.metrics import Metrics
from gpumounter_amd.worker.reconciler import Reconciler
from gpumounter_amd.worker.service import GpuMountService, RpcError

_log = log.get("worker")


def _calls_window(q) -> list:
    return calls.since(float(q.get("since", "0")), float(q.get("until", "inf")))


def _ser(m) -> bytes:
    return m.SerializeToString()


def _read(path: str) -> bytes:
    with open(path, "rb") as fh:
        return fh.read()


class Worker:
    # SIGTERM: how long operations already running may take to finish (the DaemonSet's
    # terminationGracePeriodSeconds is 30)
    OPS_DRAIN_S = 20.0

    def __init__(self, cfg, kube: Optional[KubeClient] = None,
                 inventory: Optional[Inventory] = None) -> None:
        if not cfg.node_name:
            raise ValueError("worker needs node_name (env NODE_NAME / GM_NODE_NAME)")
        self.cfg = cfg
        self.kube = kube or KubeClient.from_config(cfg)
        self.inv = inventory or Inventory(cfg.amdsmi_lib, cfg.kfd_major, cfg.kfd_dev_path)
        self.inv.ecc_policy = cfg.ecc_policy
        self.metrics = Metrics()
        # /status and /audit list other tenants' Pods and GPUs: the master's read-route rights
        from gpumounter_amd.master.authz import Authorizer
        self.status_authz = Authorizer(cfg, self.kube)
        mode = getattr(cfg, "status_authz", "auto")
        self.status_authz.mode = cfg.authz_mode if mode == "auto" else mode
        if cfg.gpu_allocation == "dra":
            # GPUs come from a DRA driver: the allocations are in ResourceClaims, not in the
            # kubelet's device manager
            self.ledger = DraLedger(self.kube, cfg.node_name, cfg.dra_driver,
                                    cfg.dra_device_class, cfg.dra_bdf_attribute)
        else:
            self.ledger = LedgerClient(cfg.kubelet_socket, cfg.resource_name,
                                       cfg.kubelet_timeout_s, cfg.podresources_api,
                                       cfg.kubelet_qps, cfg.kubelet_burst)
        self.resolver = CgroupResolver(cfg.cgroup_root, cfg.cgroup_mode, cfg.cgroup_driver,
                                       cfg.proc_root)
        emulate = cfg.devnode_mode == "emulate" or os.environ.get("GM_BPF_EMULATE") == "1"
        self.backend = make_backend(self.resolver.mode, emulate, cfg.bpf_pin_dir,
                                    cfg.bpf_set_mode)
        sd_mode = cfg.systemd_device_allow
        if emulate and sd_mode == "auto" and not cfg.systemd_bus:
            sd_mode = "off"          # hermetic runs never talk to the host's systemd by accident
        self.backend = systemd.maybe_wrap(self.backend, sd_mode, cfg.systemd_bus,
                                          self.resolver.driver)
        self.writer = DevNodeWriter(cfg.devnode_mode, cfg.host_dev_path, cfg.devnode_userns,
                                    cfg.devnode_stage_dir, cfg.proc_root)
        self.faults = FaultInjector(cfg.fault)
        self.journal = InjectionJournal(os.path.join(cfg.state_dir, "journal")
                                        if cfg.state_dir else "")
        self.hotmount = HotMount(cfg, self.inv, self.resolver, self.backend, self.writer,
                                 self.faults, self.journal)
        ph_ns = None if cfg.placeholder_namespace_mode == "tenant" else cfg.pool_namespace
        self.ph_informer = PodInformer(self.kube, ph_ns,
                                       PlaceholderManager.selector_for_node(cfg.node_name),
                                       resync_s=cfg.watch_resync_s)
        # every pod of this node except the placeholders, which ph_informer watches already:
        # their events (≈5 per attach/detach cycle) would be parsed twice for nothing
        self.node_informer = PodInformer(self.kube, None, f"!{LABEL_NODE}",
                                         f"spec.nodeName={cfg.node_name}",
                                         resync_s=cfg.watch_resync_s)
        self.placeholders = PlaceholderManager(cfg, self.kube, self.ledger, self.ph_informer,
                                               cfg.node_name, self.faults)
        self.claim_informer = None
        if isinstance(self.ledger, DraLedger):
            self.ledger.pod_lookup = lambda ns, name: (self.ph_informer.cache.get((ns, name))
                                                       or self.node_informer.cache.get((ns, name)))
            # the placeholders' claims: their allocation arrives with the watch (no GET)
            self.claim_informer = ClaimInformer(
                self.kube, ph_ns, PlaceholderManager.selector_for_node(cfg.node_name),
                resync_s=cfg.watch_resync_s)
            self.ledger.claims = self.claim_informer
        self.checkpoint = None
        if cfg.ledger_source == "auto" and cfg.kubelet_checkpoint and \
                cfg.gpu_allocation != "dra":
            self.checkpoint = DeviceCheckpoint(cfg.kubelet_checkpoint, cfg.resource_name)
            self.placeholders.checkpoint = self.checkpoint
        self.service = GpuMountService(cfg, self.kube, self.inv, self.ledger, self.placeholders,
                                       self.hotmount, self.node_informer, self.metrics,
                                       self.faults)
        # ResourceQuotas for the namespace GPU quota check, from a watch (no LIST per attach)
        self.quota_informer = QuotaInformer(self.kube, None, resync_s=cfg.watch_resync_s) \
            if self.service.quota.active else None
        self.pool = WarmPool(cfg, self.placeholders, self.inv, self.metrics)
        self.pool.quiet = self.service.notify.quiet
        self.pool.live_uids = self._live_uids
        self.service.pool = self.pool
        self.plugin = None
        if cfg.device_plugin:
            from gpumounter_amd.deviceplugin.plugin import AmdGpuDevicePlugin
            self.plugin = AmdGpuDevicePlugin(
                self.inv, cfg.resource_name, cfg.device_plugin_dir,
                inject_devices=cfg.device_plugin_inject,
                health_period_s=cfg.device_plugin_health_s, policy=cfg.topology_policy,
                metrics=self.metrics)
            self.service.plugin = self.plugin
        self.reconciler = Reconciler(self.service, cfg.reconcile_period_s)
        self.service.followup = self.reconciler.follow_up
        if cfg.reconcile_on_events:
            self.reconciler.watch_events()
        self.grpc_server: Optional[grpc.aio.Server] = None
        self.wire_server: Optional[wire.WireServer] = None
        self.wire_port = 0
        self._ops: set = set()          # RPC operations running (see run_op)
        self.http: Optional[httpd.HttpServer] = None
        self.grpc_port = 0
        self.http_port = 0
        self.ready = False

    # ------------------------------------------------------------------------ gRPC glue

    def _live_uids(self) -> set:
        """UIDs of the Pods on this node the apiserver still has (placeholders not released by
        us included): the kubelet's checkpoint can still list deleted ones."""
        tomb = self.placeholders.tombstones
        out = {podu.uid_of(p) for p in self.node_informer.cache.values()}
        out.update(u for u in (podu.uid_of(p) for p in self.ph_informer.cache.values()
                               if not p["metadata"].get("deletionTimestamp")) if u not in tomb)
        return out
    def _peer_allowed(self, context) -> bool:
        """Under mTLS, only the configured client identities (the master's certificate) may call:
        a certificate from the same CA for another component is not enough."""
        names = {n.strip() for n in self.cfg.tls_client_names.split(",") if n.strip()}
        if not self.cfg.tls_ca or not names:
            return True
        auth = context.auth_context() or {}
        got = {v.decode() if isinstance(v, bytes) else str(v)
               for k in ("x509_subject_alternative_name", "x509_common_name")
               for v in auth.get(k, [])}
        return bool(got & names)

    async def run_op(self, fn, request, t_in: float):
        """Run one AddGPU/RemoveGPU/GetNodeStatus for either transport (gRPC or gm-wire).
        Failures leave as :class:`RpcError`; ``t_in`` is when the transport handed it over.

        An attach or detach, once started, runs to its end (done, or rolled back) even if the
        caller goes away: a master killed or a deadline passed mid-request cancels the
        transport's handler, and a cancellation landing between two steps would leave a
        placeholder created but never admitted or mounted, or rules without nodes."""
        t0 = time.perf_counter()
        op = asyncio.ensure_future(self._timed(fn, request))
        self._ops.add(op)
        op.add_done_callback(self._ops.discard)
        try:
            resp, t1, t2 = await asyncio.shield(op)
        except asyncio.CancelledError:
            op.add_done_callback(self._orphan_done)     # its outcome reaches no caller
            raise
        except RpcError:
            raise
        except Exception as e:  # noqa: BLE001
            _log.exception("rpc failed")
            raise RpcError(grpc.StatusCode.INTERNAL, f"Service Internal Error: {e}") from e
        if hasattr(resp, "timings"):
            # the handler around the operation: rpc_queue = until the operation's task ran,
            # rpc_tail = from its end until the handler resumed. What is left of the master's
            # RPC time is transport (client, server, TLS)
            resp.timings.add(name="rpc_queue", ms=(t1 - t0) * 1e3)
            t_out = time.perf_counter()
            resp.timings.add(name="rpc_tail", ms=(t_out - t2) * 1e3)
            resp.timings.add(name="rpc_peer_check", ms=(t0 - t_in) * 1e3)
            # when the handler started and returned on the host's monotonic clock
            # (CLOCK_MONOTONIC: the same in every process of the host): a master on the same
            # host splits the hop into its request and response legs
            resp.timings.add(name="clock.in", ms=t_in * 1e3)
            resp.timings.add(name="clock.out", ms=t_out * 1e3)
        return resp

    def _wrap(self, fn):
        """gRPC adapter of :meth:`run_op` (peer identity checked per call)."""
        async def handler(request, context):
            t_in = time.perf_counter()
            if not self._peer_allowed(context):
                await context.abort(grpc.StatusCode.PERMISSION_DENIED,
                                    "client certificate is not an allowed gpumounter identity")
            try:
                return await self.run_op(fn, request, t_in)
            except RpcError as e:
                await context.abort(e.code, e.msg)
        return handler

    def _wire(self, fn):
        """gm-wire adapter of :meth:`run_op` (peer identity checked per connection)."""
        async def handler(request):
            try:
                return await self.run_op(fn, request, time.perf_counter())
            except RpcError as e:
                raise wire.WireStatus(e.code, e.msg) from None
        return handler

    @staticmethod
    async def _timed(fn, request):
        t1 = time.perf_counter()
        return await fn(request), t1, time.perf_counter()

    @staticmethod
    def _orphan_done(op: asyncio.Future) -> None:
        """An operation whose caller went away has ended: log how (and retrieve its exception,
        which nobody else will)."""
        if op.cancelled():
            _log.warning("operation cancelled after its caller left")
        elif op.exception() is not None:
            _log.warning("operation failed after its caller left (rolled back): %s",
                         op.exception())
        else:
            _log.info("operation completed after its caller left")

    async def _status(self, req):
        st = await self.service.node_status(req.include_processes)
        return api.NodeStatusResponse(json=json.dumps(st))

    def handlers(self):
        return (
            grpc.method_handlers_generic_handler("gpu_mount.AddGPUService", {
                "AddGPU": grpc.unary_unary_rpc_method_handler(
                    self._wrap(lambda r: self.service.add_gpu(r)), api.AddGPURequest.FromString,
                    _ser)}),
            grpc.method_handlers_generic_handler("gpu_mount.RemoveGPUService", {
                "RemoveGPU": grpc.unary_unary_rpc_method_handler(
                    self._wrap(lambda r: self.service.remove_gpu(r)),
                    api.RemoveGPURequest.FromString, _ser)}),
            grpc.method_handlers_generic_handler("gpu_mount.NodeService", {
                "GetNodeStatus": grpc.unary_unary_rpc_method_handler(
                    self._wrap(self._status), api.NodeStatusRequest.FromString, _ser)}),
        )

    def wire_handlers(self):
        return {wire.METHOD_ADD: (api.AddGPURequest.FromString,
                                  self._wire(lambda r: self.service.add_gpu(r))),
                wire.METHOD_REMOVE: (api.RemoveGPURequest.FromString,
                                     self._wire(lambda r: self.service.remove_gpu(r))),
                wire.METHOD_STATUS: (api.NodeStatusRequest.FromString, self._wire(self._status))}

    # ------------------------------------------------------------------------ lifecycle
    async def start(self, grpc_port: Optional[int] = None, http_port: Optional[int] = None,
                    reconcile: bool = True, wire_port: Optional[int] = None) -> None:
        await self.ph_informer.start()
        await self.node_informer.start()
        if self.quota_informer is not None:
            try:
                await self.quota_informer.start()
                self.service.quota.informer = self.quota_informer
            except Exception as e:  # noqa: BLE001 - no list/watch grant: per-attach reads
                _log.warning("ResourceQuota watch unavailable (%s); quotas are read per attach",
                             e)
                await self.quota_informer.stop()
                self.quota_informer = None
        if self.claim_informer is not None:
            await self.claim_informer.start()
            # a claim allocated for a placeholder can complete its admission
            self.claim_informer.handlers.append(
                lambda et, c: asyncio.ensure_future(self.ph_informer.poke()))
        # warm the ledger channel (fails fast if the kubelet socket is wrong); the authoritative
        # read also cross-checks the device-manager checkpoint before admission relies on it
        led = await self.service.read_ledger(authoritative=True)
        self.service.prime(led)
        try:   # grants from before the journal existed become revocable (node/hotmount.py adopt)
            await self.service.adopt_existing()
        except Exception as e:  # noqa: BLE001 - the reconciler retries
            _log.error("journal adoption at startup: %s", e)
        if self.checkpoint is not None:
            watched = self.checkpoint.watch(
                lambda: asyncio.ensure_future(self.ph_informer.poke()))
            _log.info("device-manager checkpoint %s: %s, inotify %s", self.checkpoint.path,
                      "present" if self.checkpoint.snapshot() is not None else "absent",
                      "on" if watched else "off")
        # lease timers from the placeholders' annotations, and draining marks a previous worker
        # could not write, before the first request is served
        await self.service.lease.sweep(expire_due=False)
        await self.service.drain.resume()
        if not (self.cfg.tls_cert and self.cfg.tls_key and self.cfg.tls_ca) and \
                not self.cfg.worker_insecure:
            raise ValueError("worker refuses to serve gRPC without mTLS: set GM_TLS_CERT, "
                             "GM_TLS_KEY and GM_TLS_CA (deploy.sh creates them), or "
                             "GM_WORKER_INSECURE=1 to opt out explicitly")
        if self.cfg.worker_insecure and not self.cfg.tls_ca:
            _log.warning("worker gRPC is UNAUTHENTICATED (worker_insecure=1): anyone who can "
                         "reach :%d can attach GPUs or kill tenant GPU processes",
                         self.cfg.worker_port)
        if not self.inv.is_mock and not procs.host_pid_ns():
            _log.warning("not in the host PID namespace: busy detection uses the render-fd scan "
                         "only, since the KFD/amdsmi process tables name host PIDs (the "
                         "DaemonSet runs with hostPID: true)")
        self.grpc_server = grpc.aio.server(options=[("grpc.so_reuseport", 0)])
        self.grpc_server.add_generic_rpc_handlers(self.handlers())
        port = self.cfg.worker_port if grpc_port is None else grpc_port
        addr = f"{self.cfg.worker_host}:{port}"
        if self.cfg.tls_cert and self.cfg.tls_key:
            creds = grpc.ssl_server_credentials(
                [(_read(self.cfg.tls_key), _read(self.cfg.tls_cert))],
                root_certificates=_read(self.cfg.tls_ca) if self.cfg.tls_ca else None,
                require_client_auth=bool(self.cfg.tls_ca))
        try:
            if self.cfg.tls_cert and self.cfg.tls_key:
                self.grpc_port = self.grpc_server.add_secure_port(addr, creds)
            else:
                self.grpc_port = self.grpc_server.add_insecure_port(addr)
        except RuntimeError as e:        # grpcio reports a failed bind this way
            raise OSError(f"cannot bind gRPC {addr}: {e}") from e
        if self.grpc_port == 0:
            raise OSError(f"cannot bind gRPC {self.cfg.worker_host}:{port}")
        await self.grpc_server.start()
        if self.cfg.wire_port >= 0:
            # gm-wire (api/wire.py): the same messages for gpumounter's own master, on one
            # persistent connection; the same certificates and client identities as gRPC
            ctx = wire.server_context(self.cfg.tls_cert, self.cfg.tls_key, self.cfg.tls_ca) \
                if self.cfg.tls_cert and self.cfg.tls_key else None
            names = [n.strip() for n in self.cfg.tls_client_names.split(",")] \
                if self.cfg.tls_ca else []
            self.wire_server = wire.WireServer(self.wire_handlers(), ctx, names)
            wp = self.cfg.wire_port if wire_port is None else wire_port
            try:
                self.wire_port = await self.wire_server.start(self.cfg.worker_host, wp)
            except OSError as e:
                raise OSError(f"cannot bind gm-wire {self.cfg.worker_host}:{wp}: {e}") from e
        hp = self.cfg.metrics_port if http_port is None else http_port
        if hp is not None and hp >= 0:
            r = httpd.Router()
            r.add_get("/healthz", self._healthz)
            r.add_get("/readyz", self._readyz)
            r.add_get("/metrics", self._metrics)
            r.add_get("/status", self._http_status)
            r.add_get("/audit/{namespace}/{pod}", self._http_audit)
            if self.cfg.debug_endpoints:    # stacks of every task: not for the open port
                r.add_get("/debug/tasks", self._debug_tasks)
                r.add_get("/debug/calls", self._debug_calls)
            self.http = httpd.HttpServer(r)
            self.http_port = await self.http.start(self.cfg.worker_host, hp)
        if reconcile and self.cfg.reconcile_period_s > 0:
            await self.reconciler.start()
        else:
            self.reconciler.start_guard()
        if self.plugin is not None:
            await self.plugin.start()
        await self.placeholders.resolve_priority()
        await self.pool.start()
        if self.cfg.metrics_period_s > 0:
            self._collector = asyncio.ensure_future(self._collect_loop())
        await self.check_health()          # ECC baseline before the first attach
        await self.service.lease.sweep()   # re-arm (or expire) leases from before a restart
        if self.cfg.health_period_s > 0:
            self._health_task = asyncio.ensure_future(self._health_loop())
        try:
            await self.service.warm_up()
        except Exception as e:  # noqa: BLE001 - only a head start; the first attach pays it
            _log.warning("attach path warm-up: %s", e)
        if self.cfg.gc_tune:
            runtime.tune_gc()
            runtime.watch_gc_pauses(5.0, _log)
        self.ready = True
        runtime.write_ready_file(self.cfg.ready_file, {"grpc_port": self.grpc_port,
                                                       "http_port": self.http_port,
                                                       "wire_port": self.wire_port})
        _log.info("worker %s serving gRPC :%d gm-wire :%d http :%d (cgroup %s/%s, devnodes %s, "
                  "ledger %s)",
                  self.cfg.node_name, self.grpc_port, self.wire_port, self.http_port,
                  self.resolver.mode,
                  self.backend.name, self.cfg.devnode_mode, self.ledger.api_version)

    async def _healthz(self, request):
        return httpd.text("ok")

    async def _metrics(self, request):
        return httpd.Response(self.metrics.render(), 200,
                              "text/plain; version=0.0.4; charset=utf-8")

    async def _debug_tasks(self, request):
        """Every asyncio task of the worker with the stack it is suspended in — what a stuck
        attach, reaction or sweep is waiting for (the goroutine dump of a Go daemon)."""
        out = []
        for t in sorted(asyncio.all_tasks(), key=lambda t: t.get_name()):
            out.append(f"{t.get_name()} {t.get_coro()!r}")
            for f in t.get_stack():
                out.append(f"    {f.f_code.co_filename}:{f.f_lineno} {f.f_code.co_name}")
        return httpd.text("\n".join(out) + "\n")

    async def _debug_calls(self, request):
        """Outbound control-plane calls that started in [since, until] (monotonic seconds):
        utils/calls.py, for the bench's per-operation call accounting."""
        return httpd.json_response(_calls_window(request.query))

    async def _readyz(self, request):
        return httpd.text("ready" if self.ready else "starting", 200 if self.ready else 503)

    async def _status_denied(self, request, ns: str = "", name: str = ""):
        """None if the caller may read this (``status_authz``), else its 401/403/503."""
        if ns:
            d = await self.status_authz.check(request.headers, "get", ns, name=name)
        else:
            d = await self.status_authz.check(request.headers, "get", resource="nodes",
                                              name=self.cfg.node_name)
        if d.allowed:
            return None
        return httpd.json_response({"error": d.reason}, status=d.status)

    async def _http_status(self, request):
        denied = await self._status_denied(request)
        if denied is not None:
            return denied
        st = await self.service.node_status(request.query.get("processes") == "1")
        return httpd.json_response(st)

    async def _http_audit(self, request):
        """Ledger-vs-node consistency of one pod: [] when its cgroup rules and device nodes are
        exactly what its placeholders hold (the check the reconciler runs)."""
        ns, name = request.match_info["namespace"], request.match_info["pod"]
        bad = podu.name_error(ns, name)
        if bad is not None:
            return httpd.json_response({"error": bad}, status=400)
        denied = await self._status_denied(request, ns, name)
        if denied is not None:
            return denied
        for attempt in range(3):
            pod = await self.service.get_pod(ns, name, fresh=True)
            if pod is None:
                return httpd.json_response({"error": "pod not found"}, status=404)
            st = await self.service.pod_state(pod, fresh=True)
            try:
                issues = self.service.hm.audit(pod, st.hot, st.own)
                break
            except CgroupError as e:
                # a container restarted between the read and the audit: read the pod again
                if attempt == 2:
                    return httpd.json_response({"error": f"pod changing: {e}"}, status=409)
                await asyncio.sleep(0.05)
        return httpd.json_response({"pod": f"{ns}/{name}", "consistent": not issues,
                                  "issues": [vars(i) for i in issues]})

    async def check_health(self) -> None:
        """Refresh GPU health (liveness + ECC policy, hw/inventory.py) off the request path; the
        attach path only reads the cached set of unhealthy GPUs."""
        h = await asyncio.get_running_loop().run_in_executor(None, self.inv.healthy)
        bad = {i for i, ok in h.items() if not ok}
        if bad != self.service.unhealthy:
            by_index = {g.index: g.bdf for g in self.inv.gpus()}
            _log.warning("GPU health changed: unhealthy now %s",
                         sorted(by_index.get(i, str(i)) for i in bad))
            self.service.unhealthy = bad
            if self.plugin is not None:
                for i, ok in h.items():
                    self.plugin.health[i] = ok
                self.plugin._notify()  # noqa: SLF001 - re-send ListAndWatch
        for g in self.inv.gpus():
            self.metrics.gpu_healthy.labels(gpu=g.bdf).set(0 if g.index in bad else 1)

    async def _health_loop(self) -> None:
        while True:
            await asyncio.sleep(self.cfg.health_period_s)
            try:
                await self.check_health()
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001
                _log.warning("health check failed: %s", e)

    async def _collect_loop(self) -> None:
        """Per-GPU process gauges + ledger state gauges."""
        while True:
            try:
                await self.collect_metrics()
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001
                _log.debug("metrics collection failed: %s", e)
            await asyncio.sleep(self.cfg.metrics_period_s)

    async def collect_metrics(self) -> None:
        if self.plugin is not None:
            self.metrics.plugin_healthy.set(sum(1 for v in self.plugin.health.values() if v))
        def counts():
            out = {}
            for g in self.inv.gpus():
                try:
                    out[g.bdf] = len(self.inv.processes(g.index))
                except Exception:  # noqa: BLE001 - not supported / no permission
                    continue
            return out

        # amdsmi walks the KFD process table per GPU: milliseconds each on a busy node, so off
        # the event loop (attaches in flight would otherwise wait for all of them)
        for bdf, n in (await asyncio.to_thread(counts)).items():
            self.metrics.gpu_busy.labels(gpu=bdf).set(n)
        await self.service.node_status(False)  # refreshes gm_ledger_gpus{state}

    async def stop(self) -> None:
        self.ready = False
        if getattr(self, "_collector", None) is not None:
            self._collector.cancel()
        if getattr(self, "_health_task", None) is not None:
            self._health_task.cancel()
        # no new RPCs; the ones running finish (or roll back) while the keepers they hand work
        # to (reconciler follow-ups, leases, drains, notifications) still run
        if self.wire_server is not None:
            await self.wire_server.stop()
        if self.grpc_server is not None:
            await self.grpc_server.stop(0.5)
        if self._ops:
            await asyncio.wait(list(self._ops), timeout=self.OPS_DRAIN_S)
        await self.pool.stop()
        await self.reconciler.stop()
        await self.service.lease.stop()
        await self.service.drain.stop()
        await self.service.notify.stop()
        if isinstance(self.backend, systemd.SystemdPersistingBackend):
            self.backend.sync.stop()
        if self.plugin is not None:
            await self.plugin.stop()
        if self.http is not None:
            await self.http.stop()
        await self.status_authz.stop()
        await self.ph_informer.stop()
        await self.node_informer.stop()
        if self.claim_informer is not None:
            await self.claim_informer.stop()
        if self.quota_informer is not None:
            await self.quota_informer.stop()
        if self.checkpoint is not None:
            self.checkpoint.close()
        await self.ledger.close()
        await self.kube.close()


async def serve(cfg) -> None:
    """Run until SIGTERM/SIGINT, then shut down cleanly (the kubelet sends SIGTERM on pod
    deletion; the reference's daemons just died — reference: cmd/*/main.go)."""
    w = Worker(cfg)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    # a failed start still stops what it started: no gRPC server or executor thread left
    # behind keeps a half-started daemon alive
    try:
        await w.start()
        await stop.wait()
    finally:
        await w.stop()
