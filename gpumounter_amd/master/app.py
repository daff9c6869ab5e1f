"""Master HTTP API — reference-compatible routes, status codes and bodies, plus JSON extensions.

Reference: cmd/GPUMounter-master/main.go (httprouter on ``:8080``):
``GET /`` (19-22), ``GET /addgpu/namespace/:namespace/pod/:pod/gpu/:gpuNum/isEntireMount/
:isEntireMount`` (24-117) and ``POST /removegpu/namespace/:namespace/pod/:pod/force/:force`` with a
repeated ``uuids`` form field (119-225). For every request the reference GETs the pod, LISTs all
worker pods (``findAllWorker``, 248-268) and dials a fresh insecure gRPC connection without a
deadline (82-96, 185-199). Here worker endpoints come from a watch cache, gRPC channels are pooled
per worker with a deadline, and the response is plain text exactly as the reference wrote it unless
the client sends ``Accept: application/json`` (then: result, devices, per-stage timings).

Extensions: ``GET /api/v1/namespaces/{ns}/pods/{pod}/gpus`` (a pod's GPUs),
``GET /api/v1/nodes/{node}/gpus`` (worker NodeService), ``/healthz``, ``/metrics``.
"""
from __future__ import annotations

import asyncio
import json
import signal
import ssl
import time
from typing import Dict, Optional, Tuple

import grpc

from gpumounter_amd.api import gpu_mount as api
from gpumounter_amd.api import protodef, wire
from gpumounter_amd.cluster.informer import PodInformer, SlimPodInformer
from gpumounter_amd.cluster.kube import ApiError, KubeClient, NotFound
from gpumounter_amd.cluster.placeholder import LABEL_NODE
from gpumounter_amd.models import pod as podu
from gpumounter_amd.utils import httpd
from gpumounter_amd.master.authz import Authorizer
from gpumounter_amd.utils.httpd import Request, Response
from gpumounter_amd.utils import calls, log, runtime, trace
from gpumounter_amd.utils.metrics import Metrics

_log = log.get("master")

ANN_WORKER_PORT = "gpumounter.amd.com/grpc-port"
ANN_WIRE_PORT = "gpumounter.amd.com/wire-port"     # the worker serves gm-wire (api/wire.py)
_TRUE = {"1", "t", "T", "TRUE", "true", "True"}
_FALSE = {"0", "f", "F", "FALSE", "false", "False"}


def parse_go_bool(s: str) -> Optional[bool]:
    """Go ``strconv.ParseBool`` (reference main.go:38,140)."""
    if s in _TRUE:
        return True
    if s in _FALSE:
        return False
    return None


def parse_go_int32(s: str) -> Optional[int]:
    """Go ``strconv.ParseInt(s, 10, 32)`` (reference main.go:31)."""
    if not s or s.strip() != s:
        return None
    body = s[1:] if s[0] in "+-" else s
    if not body.isdigit() or not body.isascii():
        return None
    v = int(s)
    if not -(2 ** 31) <= v < 2 ** 31:
        return None
    return v


def parse_lease(v: str) -> Optional[float]:
    """``?lease=<seconds>``: "" → 0.0 (no lease), a positive finite number → it, else None."""
    if v in ("", None):
        return 0.0
    try:
        f = float(v)
    except ValueError:
        return None
    return f if 0 < f < 10 * 365 * 86400 else None


def _text(body: str, status: int = 200) -> Response:
    # Go's http.Error / fmt.Fprintf write text/plain with a trailing newline
    return httpd.text(body if body.endswith("\n") else body + "\n", status)


# AddGPU is retried when the worker answers UNAVAILABLE (restarting, draining). That is safe
# because every AddGPU carries an idempotency key (the caller's Idempotency-Key header or the
# request id): a retry of an attach that did happen replays it instead of adding more GPUs.
# RemoveGPU is not retried (a repeated remove of removed GPUs reads as GPUNotFound).
_SERVICE_CONFIG = json.dumps({"methodConfig": [{
    "name": [{"service": f"{api.PACKAGE}.AddGPUService", "method": "AddGPU"}],
    "retryPolicy": {"maxAttempts": 4, "initialBackoff": "0.05s", "maxBackoff": "1s",
                    "backoffMultiplier": 2, "retryableStatusCodes": ["UNAVAILABLE"]}}]})


USER_KEY = "gm_user"       # the caller's identity, set by _denied()


# method → (gRPC path, request class, response class, gm-wire method id)
_METHODS = {
    "add": (api.ADD_GPU, api.AddGPURequest, api.AddGPUResponse, wire.METHOD_ADD),
    "remove": (api.REMOVE_GPU, api.RemoveGPURequest, api.RemoveGPUResponse, wire.METHOD_REMOVE),
    "status": (api.NODE_STATUS, api.NodeStatusRequest, api.NodeStatusResponse,
               wire.METHOD_STATUS),
}
# what a failed worker call raises, whichever transport carried it (both have code()/details())
RPC_ERRORS = (grpc.aio.AioRpcError, wire.WireError)


class WorkerDirectory:
    """node name → worker endpoint, from a watch on the worker DaemonSet pods; pooled channels.

    A worker pod that advertises a gm-wire port (``ANN_WIRE_PORT``) is called over gm-wire
    (api/wire.py) unless ``master_transport=grpc``; one whose gm-wire port cannot be reached is
    called over gRPC for the next ``WIRE_RETRY_S`` seconds. gRPC is the reference's transport
    (main.go:82-96, a new insecure connection per request); here the channel is kept."""

    WIRE_RETRY_S = 10.0
    ADD_ATTEMPTS = 4           # AddGPU on UNAVAILABLE, as the gRPC retry policy (_SERVICE_CONFIG)

    def __init__(self, kube: KubeClient, namespace: str, label: str, default_port: int,
                 cfg=None) -> None:
        self.informer = PodInformer(kube, namespace, label)
        self.default_port = default_port
        self.cfg = cfg
        self._channels: Dict[str, grpc.aio.Channel] = {}
        self._stubs: Dict[Tuple[str, str], object] = {}
        self._wires: Dict[str, wire.WireChannel] = {}
        self._wire_of: Dict[str, Optional[str]] = {}     # gRPC target → gm-wire target
        self._wire_down: Dict[str, float] = {}           # gm-wire target → retry after
        self._loop = None
        self._targets: Dict[str, Optional[str]] = {}

    async def start(self) -> None:
        await self.informer.start()
        self.informer.handlers.append(lambda etype, pod: self.warm())
        self.warm()

    def warm(self) -> None:
        """Open the channel to every running worker ahead of its first request: the TCP
        connect and the TLS handshake then happen in the background, not in an attach
        (reference: a new insecure connection per request, main.go:82)."""
        targets = {podu.node_of(p): self.target(podu.node_of(p))
                   for p in self.informer.cache.values()}
        if targets != self._targets:
            _log.debug("worker targets: %s", targets)
            self._targets = targets
        for t in set(targets.values()):
            if t is None:
                continue
            try:
                self.channel(t).get_state(try_to_connect=True)
                wt = self._wire_of.get(t)
                if wt is not None:
                    self.wire_channel(wt).warm()
            except RuntimeError:         # no running loop (stopping)
                return

    async def stop(self) -> None:
        await self.informer.stop()
        for ch in self._channels.values():
            await ch.close()
        for w in self._wires.values():
            await w.close()
        self._channels.clear()
        self._stubs.clear()
        self._wires.clear()

    def target(self, node: str) -> Optional[str]:
        best = None
        wire_port = None
        for p in self.informer.cache.values():
            if podu.node_of(p) != node or podu.is_terminating(p):
                continue
            ip = p.get("status", {}).get("podIP")
            if not ip or podu.phase_of(p) != "Running":
                continue
            ann = p["metadata"].get("annotations") or {}
            port = ann.get(ANN_WORKER_PORT, str(self.default_port))
            best = f"{ip}:{port}"
            wire_port = ann.get(ANN_WIRE_PORT)
            wire_port = f"{ip}:{wire_port}" if wire_port and self._wire_enabled() else None
        if best is not None:
            self._wire_of[best] = wire_port
        return best

    def _wire_enabled(self) -> bool:
        return getattr(self.cfg, "master_transport", "auto") == "auto"

    def _check_loop(self) -> None:
        loop = asyncio.get_running_loop()
        if self._loop is not loop:
            self._channels, self._stubs, self._wires = {}, {}, {}
            self._loop = loop

    def channel(self, target: str) -> grpc.aio.Channel:
        self._check_loop()
        ch = self._channels.get(target)
        if ch is None:
            opts = [("grpc.keepalive_time_ms", 30000), ("grpc.enable_retries", 1),
                    ("grpc.service_config", _SERVICE_CONFIG)]
            cfg = self.cfg
            if cfg is not None and cfg.tls_ca:
                creds = grpc.ssl_channel_credentials(
                    root_certificates=_read(cfg.tls_ca),
                    private_key=_read(cfg.tls_key) if cfg.tls_key else None,
                    certificate_chain=_read(cfg.tls_cert) if cfg.tls_cert else None)
                opts.append(("grpc.ssl_target_name_override", cfg.tls_server_name))
                ch = grpc.aio.secure_channel(target, creds, options=opts)
            else:
                ch = grpc.aio.insecure_channel(target, options=opts)
            self._channels[target] = ch
        return ch

    def wire_channel(self, target: str) -> wire.WireChannel:
        self._check_loop()
        ch = self._wires.get(target)
        if ch is None:
            host, port = target.rsplit(":", 1)
            cfg = self.cfg
            ctx = wire.client_context(cfg.tls_ca, cfg.tls_cert, cfg.tls_key) \
                if cfg is not None and cfg.tls_ca else None
            ch = self._wires[target] = wire.WireChannel(
                host, int(port), ctx, cfg.tls_server_name if ctx is not None else "")
        return ch

    def _stub(self, target: str, method: str):
        """The gRPC multicallable, built once per channel and method."""
        self._check_loop()
        stub = self._stubs.get((target, method))
        if stub is None:
            path, req_cls, resp_cls, _ = _METHODS[method]
            stub = self._stubs[(target, method)] = self.channel(target).unary_unary(
                path, request_serializer=req_cls.SerializeToString,
                response_deserializer=resp_cls.FromString)
        return stub

    async def unary(self, target: str, method: str, req, timeout: float):
        """One worker call over gm-wire when the worker offers it, else gRPC. Failures raise
        one of :data:`RPC_ERRORS`."""
        wt = self._wire_of.get(target)
        # one deadline for every attempt, as gRPC's retry policy keeps one for the call
        deadline = time.monotonic() + timeout
        if wt is not None and self._wire_down.get(wt, 0.0) <= time.monotonic():
            _, _, resp_cls, mid = _METHODS[method]
            ch = self.wire_channel(wt)
            payload = req.SerializeToString()
            attempts = self.ADD_ATTEMPTS if method == "add" else 1
            for i in range(attempts):
                left = deadline - time.monotonic()
                if left <= 0:
                    raise wire.WireError(grpc.StatusCode.DEADLINE_EXCEEDED,
                                         f"no answer from {wt} within {timeout:g}s")
                try:
                    return resp_cls.FromString(await ch.call(mid, payload, left))
                except wire.WireError as e:
                    if e.code() != grpc.StatusCode.UNAVAILABLE:
                        raise
                    if not e.sent:
                        # never reached the worker: gRPC instead, for a while
                        _log.warning("gm-wire to %s unavailable (%s); using gRPC for %gs",
                                     wt, e.details(), self.WIRE_RETRY_S)
                        self._wire_down[wt] = time.monotonic() + self.WIRE_RETRY_S
                        break
                    if i == attempts - 1:
                        raise
                    # the idempotency key makes a repeated AddGPU replay the first one
                    await asyncio.sleep(min(0.05 * 2 ** i, 1.0,
                                            max(deadline - time.monotonic(), 0.0)))
        left = deadline - time.monotonic()
        if left <= 0:
            raise wire.WireError(grpc.StatusCode.DEADLINE_EXCEEDED,
                                 f"no answer from {target} within {timeout:g}s")
        return await self._stub(target, method)(req, timeout=left)


def _read(path: str) -> bytes:
    with open(path, "rb") as fh:
        return fh.read()


class Master:
    POD_CACHE_TTL_S = 30.0
    POD_CACHE_MAX = 4096
    POD_INDEX_WAIT_S = 10.0

    def __init__(self, cfg, kube: Optional[KubeClient] = None) -> None:
        self.cfg = cfg
        self.kube = kube or KubeClient.from_config(cfg)
        self.workers = WorkerDirectory(self.kube, cfg.worker_namespace, cfg.worker_label,
                                       cfg.worker_port, cfg)
        self.metrics = Metrics()
        self.authz = Authorizer(cfg, self.kube)
        self.http: Optional[httpd.HttpServer] = None
        self.port = 0
        self._pod_nodes: Dict[Tuple[str, str], Tuple[str, str, float]] = {}
        # pod → node without a GET per request (the reference GETs the pod every time,
        # main.go:52); until its first LIST is in, requests fall back to a GET
        # (placeholders excluded: never an attach target, and every attach creates and deletes
        # some — their events would land on the master's loop while it waits for the worker)
        self.pods: Optional[SlimPodInformer] = SlimPodInformer(
            self.kube, label_selector=f"!{LABEL_NODE}", resync_s=cfg.watch_resync_s) \
            if getattr(cfg, "master_pod_index", True) else None
        self._pods_task: Optional[asyncio.Task] = None

    # ------------------------------------------------------------------------ app
    def router(self) -> httpd.Router:
        r = httpd.Router()
        r.add_get("/", self.index)
        r.add_get("/addgpu/namespace/{namespace}/pod/{pod}/gpu/{gpuNum}/isEntireMount/"
                  "{isEntireMount}", self.add_gpu)
        r.add_post("/removegpu/namespace/{namespace}/pod/{pod}/force/{force}", self.remove_gpu)
        r.add_post("/api/v1/batch", self.batch)
        r.add_get("/api/v1/namespaces/{namespace}/pods/{pod}/gpus", self.pod_gpus)
        r.add_get("/api/v1/nodes/{node}/gpus", self.node_gpus)
        r.add_get("/healthz", self.healthz)
        r.add_get("/metrics", self.metrics_handler)
        if getattr(self.cfg, "debug_endpoints", False):
            r.add_get("/debug/calls", self.debug_calls)
            r.add_post("/debug/authz-expire", self.debug_authz_expire)
        return r

    async def debug_authz_expire(self, request: Request) -> Response:
        """Age the authz caches as a long idle period would (bench: cold attaches interleaved
        with warm ones on the same master process). ``?age=0``: the same request, nothing aged
        (the control cycles send it too, so both kinds wake the master alike)."""
        if request.query.get("age") == "0":
            return httpd.json_response({"aged": 0})
        return httpd.json_response({"aged": self.authz.expire()})

    async def debug_calls(self, request: Request) -> Response:
        """Outbound control-plane calls (utils/calls.py) that started in [since, until]."""
        q = request.query
        return httpd.json_response(calls.since(float(q.get("since", "0")),
                                               float(q.get("until", "inf"))))

    async def start(self, port: Optional[int] = None) -> None:
        await self.workers.start()
        if self.pods is not None:
            # serve once the index has synced (as a controller waits for its caches), but not
            # longer than a few seconds: until then a lookup GETs the pod
            self._pods_task = asyncio.ensure_future(self._start_pod_index())
            await asyncio.wait([self._pods_task], timeout=self.POD_INDEX_WAIT_S)
        self.http = httpd.HttpServer(self.router())
        tls = self.server_tls()
        self.port = await self.http.start(self.cfg.master_host,
                                          self.cfg.master_port if port is None else port,
                                          ssl=tls)
        if tls is None and self.authz.mode == "kube":
            _log.warning("master API is plain HTTP and callers send Kubernetes bearer tokens "
                         "(authz_mode=kube): set master_tls_cert/master_tls_key")
        try:
            self.warm_up()
            await self._warm_http()
            await asyncio.wait_for(self.authz.warm_up(), 2.0)
        except Exception as e:  # noqa: BLE001 - only a head start
            _log.warning("request path warm-up: %s", e)
        if self.cfg.gc_tune:
            runtime.tune_gc()
            runtime.watch_gc_pauses(5.0, _log)
        runtime.write_ready_file(self.cfg.ready_file, {"port": self.port})
        _log.info("master serving HTTP :%d", self.port)

    def warm_up(self) -> None:
        """The request path's in-process work once before the first request: the roctx library,
        a worker reply through the payload and JSON reply code, the metric children of the
        add/remove routes. Nothing leaves the process."""
        trace._roctx_lib()                                       # noqa: SLF001
        with trace.span("master_addgpu") as root:
            with trace.span("master_rpc"):
                resp = api.AddGPUResponse.FromString(api.AddGPUResponse(
                    devices=[api.Device(uuid="warm-up", bdf="0000:00:00.0")], message="warm-up",
                    timings=[api.StageTiming(name="warm-up", ms=0.0)]).SerializeToString())
        payload = self._stamp(self._payload(resp, time.perf_counter()), root)
        httpd.json_response(dict(payload, message="warm-up", code=200))
        for req in (api.AddGPURequest(pod_name="warm-up", namespace="default", gpu_num=1),
                    api.RemoveGPURequest(pod_name="warm-up", namespace="default",
                                         uuids=["warm-up"])):
            req.SerializeToString()
        for route in ("addgpu", "removegpu"):
            for code in ("200", "400", "500"):
                self.metrics.http_requests.labels(route=route, code=code)

    def server_tls(self) -> Optional[ssl.SSLContext]:
        """The API port's TLS context (None: plain HTTP)."""
        if not getattr(self.cfg, "master_tls_cert", ""):
            return None
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ctx.load_cert_chain(self.cfg.master_tls_cert, self.cfg.master_tls_key)
        return ctx

    async def _warm_http(self) -> None:
        """One request through the HTTP server over loopback (accept, parse, route, reply):
        the server half of a client's first request is then not cold code."""
        host = "127.0.0.1" if self.cfg.master_host in ("", "0.0.0.0", "::") else \
            self.cfg.master_host
        ctx = None
        if self.http is not None and self.http.tls:
            ctx = ssl.create_default_context()     # our own loopback: nothing to verify
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        r, w = await asyncio.wait_for(asyncio.open_connection(host, self.port, ssl=ctx), 2.0)
        try:
            w.write(b"GET /healthz HTTP/1.1\r\nHost: warm-up\r\nConnection: close\r\n\r\n")
            await asyncio.wait_for(r.read(), 2.0)
        finally:
            w.close()

    async def _start_pod_index(self) -> None:
        try:
            await self.pods.start()
            _log.info("pod index synced: %d pods", len(self.pods.cache))
        except asyncio.CancelledError:
            raise
        except Exception as e:  # noqa: BLE001 - requests GET the pod meanwhile
            _log.warning("pod index not synced (%s); pod lookups GET the pod", e)

    async def stop(self) -> None:
        if self.http is not None:
            await self.http.stop()
        if self._pods_task is not None:
            self._pods_task.cancel()
        if self.pods is not None:
            await self.pods.stop()
        await self.authz.stop()
        await self.workers.stop()
        await self.kube.close()

    # ------------------------------------------------------------------------ handlers
    async def healthz(self, request: Request) -> Response:
        return httpd.text("ok")

    async def metrics_handler(self, request: Request) -> Response:
        return Response(self.metrics.render(), content_type="text/plain; version=0.0.4")

    async def index(self, request: Request) -> Response:
        return _text("This is gpu mounter api!")

    @staticmethod
    def _wants_json(request: Request) -> bool:
        return "application/json" in request.headers.get("Accept", "")

    async def _denied(self, request: Request, route: str, verb: str, ns: str = "",
                      resource: str = "pods", name: str = "") -> Optional[Response]:
        """None if allowed, else the 401/403/503 reply (master/authz.py; the reference has no
        authn/authz at all: SURVEY defect 13)."""
        d = await self.authz.check(request.headers, verb, ns, resource, name)
        if d.allowed:
            request[USER_KEY] = self._identity(request, d)
            return None
        return self._reply(request, route, d.status, d.reason, {})

    def _identity(self, request: Request, d) -> str:
        """Who asked, for the audit trail (Events, logs): the authenticated Kubernetes user, the
        shared-token holder, or the anonymous caller's address."""
        if d.user:
            return d.user
        if self.cfg.api_token:
            return "api-token"
        return f"anonymous@{request.remote or '?'}"

    def _reply(self, request, route: str, status: int, text: str, payload: dict) -> Response:
        self.metrics.http_requests.labels(route=route, code=str(status)).inc()
        if self._wants_json(request):
            payload = dict(payload)
            if payload.get("message") and payload["message"] != text.rstrip("\n"):
                payload["detail"] = payload["message"]
            payload["message"] = text.rstrip("\n")
            payload["code"] = status
            return httpd.json_response(payload, status=status)
        return _text(text, status)

    def _stale(self, cached: str, pod: dict) -> bool:
        """The worker found no such pod although the lookup did: worth one fresh try (a GET)
        if the answer came from the 30 s cache or from the index, whose watch may not have
        delivered the deletion or the re-creation yet. The GET then answers as the reference
        does on every request (main.go:52): 404 for a pod that is gone. Only this failure path
        pays for the GET."""
        if cached == "ttl":
            self._pod_nodes.pop((podu.ns_of(pod), podu.name_of(pod)), None)
            return True
        return cached == "index"

    async def _locate(self, ns: str, name: str, fresh: bool = False):
        """Pod → node → worker target. Returns (pod, target, error, cached) where error is a
        (status, text, payload) triple and cached where the pod came from ("index", "ttl" or
        "" for a GET). The pod comes from the master's pod index (a watch of
        every Pod) or, with the index off or not yet synced, from a small 30 s cache; a pod not
        found there is read with a GET. A stale answer (the pod was recreated on another node)
        is detected by the worker and retried fresh."""
        key = (ns, name)
        now = time.monotonic()
        indexed = self.pods is not None and self.pods._synced is not None and \
            self.pods._synced.is_set()  # noqa: SLF001
        hit = None if fresh or indexed else self._pod_nodes.get(key)
        idx = self.pods.get(ns, name) if indexed and not fresh else None
        if idx is not None and podu.node_of(idx) and not podu.is_terminating(idx):
            pod, cached = idx, "index"
        elif hit is not None and now - hit[2] < self.POD_CACHE_TTL_S:
            pod = {"metadata": {"name": name, "namespace": ns, "uid": hit[1]},
                   "spec": {"nodeName": hit[0]}}
            cached = "ttl"
        else:
            try:
                pod = await self.kube.get_pod(ns, name)
            except NotFound:
                self._pod_nodes.pop(key, None)
                return None, None, (404, f"No pod: {name} in namespace: {ns}", {}), ""
            except ApiError as e:
                return None, None, (500, str(e), {}), False
            cached = ""
            if podu.node_of(pod):
                self._pod_nodes[key] = (podu.node_of(pod), podu.uid_of(pod), now)
                if len(self._pod_nodes) > self.POD_CACHE_MAX:
                    self._pod_nodes.pop(next(iter(self._pod_nodes)))
        node = podu.node_of(pod)
        target = self.workers.target(node)
        if target is None:
            _log.error("no gpu mounter worker on node %r", node)
            return pod, None, (500, "Service Internal Error",
                               {"error": f"no worker on node {node!r}"}), cached
        return pod, target, None, cached

    # ------------------------------------------------------------------------ operations
    async def _add(self, ns: str, name: str, n: int, entire: bool, container: str = "",
                   rid: str = "", key: str = "", user: str = "", lease_s: float = 0.0):
        """AddGPU through the pod's worker → (status, text, payload) as the reference maps it
        (reference main.go:103-116)."""
        t0 = time.perf_counter()
        for fresh in (False, True):
            with trace.span("master_locate"):
                pod, target, err, cached = await self._locate(ns, name, fresh)
            if err is not None:
                return err
            try:
                with trace.span("master_rpc"):
                    t_send = time.perf_counter()
                    resp = await self.workers.unary(target, "add", api.AddGPURequest(
                        pod_name=name, namespace=ns, gpu_num=n, is_entire_mount=entire,
                        request_id=rid, container=container, idempotency_key=key,
                        requested_by=user, lease_s=lease_s), self.cfg.rpc_timeout_s)
                    self._legs(resp, t_send, time.perf_counter())
            except RPC_ERRORS as e:
                if cached and e.code() == grpc.StatusCode.FAILED_PRECONDITION and \
                        "this worker serves" in (e.details() or ""):
                    self._pod_nodes.pop((ns, name), None)   # pod was recreated elsewhere
                    continue
                if e.code() == grpc.StatusCode.RESOURCE_EXHAUSTED:   # namespace GPU quota
                    _log.info("AddGPU %s/%s refused: %s", ns, name, e.details())
                    return 403, e.details(), {"error": e.details()}
                _log.error("AddGPU rpc to %s failed: %s %s", target, e.code().name, e.details())
                code = 400 if e.code() == grpc.StatusCode.INVALID_ARGUMENT else 500
                body = "Service Internal Error" if code == 500 else e.details()
                return code, body, {"error": e.details()}
            if resp.add_gpu_result == api.ADD_POD_NOT_FOUND and self._stale(cached, pod):
                continue                                    # re-check with a fresh GET
            break
        payload = self._payload(resp, t0)
        node = podu.node_of(pod)
        if resp.add_gpu_result == api.ADD_SUCCESS:
            return 200, "Add GPU Success", payload
        if resp.add_gpu_result == api.ADD_INSUFFICIENT:
            return 500, f"Insufficient GPU on Node: {node}", payload
        if resp.add_gpu_result == api.ADD_POD_NOT_FOUND:
            return 400, f"No Pod{name} on Node: {node}", payload
        return 500, "Service Internal Error", payload

    async def _remove(self, ns: str, name: str, uuids, force: bool, container: str = "",
                      rid: str = "", user: str = ""):
        """RemoveGPU through the pod's worker (reference main.go:206-224 mapping)."""
        t0 = time.perf_counter()
        for fresh in (False, True):
            with trace.span("master_locate"):
                pod, target, err, cached = await self._locate(ns, name, fresh)
            if err is not None:
                return err
            try:
                with trace.span("master_rpc"):
                    t_send = time.perf_counter()
                    resp = await self.workers.unary(target, "remove", api.RemoveGPURequest(
                        pod_name=name, namespace=ns, uuids=uuids, force=force,
                        request_id=rid, container=container, requested_by=user),
                        self.cfg.rpc_timeout_s)
                    self._legs(resp, t_send, time.perf_counter())
            except RPC_ERRORS as e:
                _log.error("RemoveGPU rpc to %s failed: %s %s", target, e.code().name,
                           e.details())
                return 500, "Service Internal Error", {"error": e.details()}
            if resp.remove_gpu_result == api.REMOVE_POD_NOT_FOUND and self._stale(cached, pod):
                continue
            break
        payload = self._payload(resp, t0)
        node = podu.node_of(pod)
        r = resp.remove_gpu_result
        if r == api.REMOVE_SUCCESS:
            return 200, "Remove GPU Success", payload
        if r == api.REMOVE_POD_NOT_FOUND:
            return 400, f"No Pod{name} on Node: {node}", payload
        if r == api.REMOVE_BUSY:
            return 400, f"Pod: {name} has running processes on GPU: {', '.join(uuids)}", payload
        if r == api.REMOVE_GPU_NOT_FOUND:
            return 400, f"Invalid UUIDs: {', '.join(uuids)}", payload
        return 500, "Service Internal Error", payload

    # ------------------------------------------------------------------------ HTTP routes
    async def add_gpu(self, request: Request) -> Response:
        # gm:master_* roctx ranges; the stage split is returned as ``master_timings``
        with trace.span("master_addgpu") as root:
            return await self._add_gpu(request, root)

    async def _add_gpu(self, request: Request, root: trace.Span) -> Response:
        route = "addgpu"
        mi = request.match_info
        ns, name = mi["namespace"], mi["pod"]
        bad = podu.name_error(ns, name)
        if bad is not None:
            return self._reply(request, route, 400, bad, {})
        with trace.span("master_authz"):
            denied = await self._denied(request, route, "create", ns, name=name)
        if denied is not None:
            return denied
        rid = log.new_request_id("add")
        n = parse_go_int32(mi["gpuNum"])
        if n is None:
            return self._reply(request, route, 400, f"Invalid param gpuNum: {mi['gpuNum']}", {})
        entire = parse_go_bool(mi["isEntireMount"])
        if entire is None:
            return self._reply(request, route, 400,
                               f"Invalid param isEntireMount: {mi['isEntireMount']}"
                               "(should be true or false)", {})
        if n <= 0:
            # the reference forwarded 0 and the worker divided by zero (SURVEY defect 6)
            return self._reply(request, route, 400, f"Invalid param gpuNum: {mi['gpuNum']}", {})
        lease_s = parse_lease(request.query.get("lease", ""))
        if lease_s is None:
            return self._reply(request, route, 400,
                               f"Invalid param lease: {request.query.get('lease')}"
                               "(should be a positive number of seconds)", {})
        status, text, payload = await self._add(
            ns, name, n, entire, request.query.get("container", ""), rid,
            request.headers.get("Idempotency-Key", "") or rid, request.get(USER_KEY, ""),
            lease_s)
        return self._reply(request, route, status, text, self._stamp(payload, root, request))

    async def remove_gpu(self, request: Request) -> Response:
        with trace.span("master_removegpu") as root:
            return await self._remove_gpu(request, root)

    async def _remove_gpu(self, request: Request, root: trace.Span) -> Response:
        route = "removegpu"
        mi = request.match_info
        ns, name = mi["namespace"], mi["pod"]
        bad = podu.name_error(ns, name)
        if bad is not None:
            return self._reply(request, route, 400, bad, {})
        with trace.span("master_authz"):
            denied = await self._denied(request, route, "delete", ns, name=name)
        if denied is not None:
            return denied
        rid = log.new_request_id("rm")
        try:
            form = await request.post()
        except Exception:  # noqa: BLE001
            return self._reply(request, route, 500, "Service Internal Error", {})
        uuids = list(form.getall("uuids", [])) + list(request.query.getall("uuids", []))
        if not uuids:
            return self._reply(request, route, 400, "Invalid parameter", {})
        force = parse_go_bool(mi["force"])
        if force is None:
            return self._reply(request, route, 400,
                               f"Invalid parameter force: {mi['force']}(should be true or false)",
                               {})
        status, text, payload = await self._remove(ns, name, uuids, force,
                                                   request.query.get("container", ""), rid,
                                                   request.get(USER_KEY, ""))
        return self._reply(request, route, status, text, self._stamp(payload, root, request))

    @staticmethod
    def _legs(resp, t_send: float, t_recv: float) -> None:
        """The worker stamps when its handler started and returned (``clock.in``/``clock.out``,
        host monotonic ms). On one host that splits the gRPC call into its request leg (master
        send → worker handler) and response leg (handler return → master receive), recorded as
        stages of the master's trace; the stamps themselves are dropped from the reply."""
        stamps = {t.name: t.ms for t in resp.timings if t.name.startswith("clock.")}
        if not stamps:
            return
        keep = [t for t in resp.timings if not t.name.startswith("clock.")]
        del resp.timings[:]
        resp.timings.extend(keep)
        t_in, t_out = stamps.get("clock.in"), stamps.get("clock.out")
        if t_in is None or t_out is None or not t_send * 1e3 <= t_in <= t_out <= t_recv * 1e3:
            return                     # another host's clock: the legs are not measurable
        trace.record("grpc_request", int((t_in - t_send * 1e3) * 1e6))
        trace.record("grpc_response", int((t_recv * 1e3 - t_out) * 1e6))

    @staticmethod
    def _stamp(payload: dict, root: trace.Span, request: Optional[Request] = None) -> dict:
        """The master's own stage split so far (authz, locate, rpc, payload), for the JSON
        reply; the text reply ignores it. ``master_clock``: CLOCK_MONOTONIC when the request
        began to arrive and when its reply is encoded, so a client on the same host can split
        its own round trip (bench.py ``first_attach_stages_ms``)."""
        if payload:
            payload["master_timings"] = [{"name": k, "ms": round(v, 4)}
                                         for k, v in root.flat().items()]
            if request is not None and request.t_in:
                payload["master_clock"] = {"in": request.t_in, "out": time.monotonic()}
        return payload

    async def batch(self, request: Request) -> Response:
        """``POST /api/v1/batch`` {"operations": [{"op": "add", "namespace", "pod", "gpus",
        "entire", "container", "idempotency_key"} | {"op": "remove", "namespace", "pod",
        "uuids", "force", "container"}]} → results in order; operations run concurrently
        (operations on one pod still serialize on the worker's per-pod lock)."""
        route = "batch"
        if self.authz.mode != "kube":   # shared-token mode: one check for the whole batch
            denied = await self._denied(request, route, "create")
            if denied is not None:
                return denied
        try:
            body = await request.json()
            ops = body["operations"]
            assert isinstance(ops, list)
        except Exception:  # noqa: BLE001
            return httpd.json_response({"error": "body must be {\"operations\": [...]}"},
                                     status=400)

        async def one(op):
            try:
                kind = op["op"]
                ns, name = op.get("namespace", "default"), op["pod"]
                bad = podu.name_error(ns, name) if isinstance(ns, str) and \
                    isinstance(name, str) else "namespace and pod must be strings"
                if bad is not None:
                    return 400, bad, {}
                user = request.get(USER_KEY, "")
                if self.authz.mode == "kube":   # per operation: namespaces may differ
                    d = await self.authz.check(request.headers,
                                               "create" if kind == "add" else "delete", ns,
                                               name=name)
                    if not d.allowed:
                        return d.status, d.reason, {}
                    user = self._identity(request, d)
                if kind == "add":
                    n = int(op["gpus"])
                    if n <= 0:
                        return 400, f"Invalid param gpuNum: {n}", {}
                    rid = log.new_request_id("add")
                    lease_s = parse_lease(str(op.get("lease_s", "")))
                    if lease_s is None:
                        return 400, f"Invalid param lease_s: {op.get('lease_s')}", {}
                    return await self._add(ns, name, n, bool(op.get("entire", False)),
                                           op.get("container", ""), rid,
                                           op.get("idempotency_key", "") or rid, user, lease_s)
                if kind == "remove":
                    uuids = list(op["uuids"])
                    if not uuids:
                        return 400, "Invalid parameter", {}
                    return await self._remove(ns, name, uuids, bool(op.get("force", False)),
                                              op.get("container", ""), log.new_request_id("rm"),
                                              user)
                return 400, f"unknown op {kind!r}", {}
            except (KeyError, TypeError, ValueError) as e:
                return 400, f"bad operation: {e}", {}

        results = await asyncio.gather(*[one(op) for op in ops])
        out = []
        for status, text, payload in results:
            d = dict(payload)
            d.update(code=status, message=text)
            out.append(d)
            self.metrics.http_requests.labels(route=route, code=str(status)).inc()
        return httpd.json_response({"results": out})

    @staticmethod
    def _payload(resp, t0: float) -> dict:
        with trace.span("master_payload"):
            d = protodef.to_dict(resp)
        d["master_ms"] = (time.perf_counter() - t0) * 1e3
        return d

    async def node_gpus(self, request: Request) -> Response:
        node = request.match_info["node"]
        if not podu.is_dns1123_subdomain(node):
            return httpd.json_response({"error": f"invalid node name {node!r}"}, status=400)
        denied = await self._denied(request, "nodegpus", "get", resource="nodes", name=node)
        if denied is not None:
            return denied
        target = self.workers.target(node)
        if target is None:
            return httpd.json_response({"error": f"no worker on node {node}"}, status=404)
        try:
            resp = await self.workers.unary(target, "status", api.NodeStatusRequest(
                include_processes=request.query.get("processes") == "1"), 30.0)
        except RPC_ERRORS as e:
            return httpd.json_response({"error": f"worker on {node}: {e.code().name} "
                                               f"{e.details()}"}, status=502)
        return httpd.json_response(json.loads(resp.json))

    async def pod_gpus(self, request: Request) -> Response:
        ns, name = request.match_info["namespace"], request.match_info["pod"]
        bad = podu.name_error(ns, name)
        if bad is not None:
            return httpd.json_response({"error": bad}, status=400)
        denied = await self._denied(request, "podgpus", "get", ns, name=name)
        if denied is not None:
            return denied
        try:
            pod = await self.kube.get_pod(ns, name)
        except NotFound:
            return httpd.json_response({"error": "pod not found"}, status=404)
        except ApiError as e:
            return httpd.json_response({"error": str(e)}, status=500)
        target = self.workers.target(podu.node_of(pod))
        if target is None:
            return httpd.json_response({"error": "no worker"}, status=500)
        try:
            st = json.loads((await self.workers.unary(target, "status", api.NodeStatusRequest(),
                                                      30.0)).json)
        except RPC_ERRORS as e:
            return httpd.json_response({"error": f"worker on {podu.node_of(pod)}: "
                                               f"{e.code().name} {e.details()}"}, status=502)
        uid = podu.uid_of(pod)
        held = {(p["namespace"], p["name"]): p.get("lease_expires")
                for p in st.get("placeholders", [])
                if p["owner"] == name and p["owner_namespace"] == ns and p["owner_uid"] == uid
                and not p.get("releasing")}
        hot = [dict(g, source="hot-mount",
                    lease_expires=held[(g.get("namespace"), g.get("pod_name"))])
               for g in st["gpus"] if (g.get("namespace"), g.get("pod_name")) in held]
        own = [dict(g, source="pod-spec") for g in st["gpus"]
               if (g.get("namespace"), g.get("pod_name")) == (ns, name)]
        return httpd.json_response({"pod": f"{ns}/{name}", "node": podu.node_of(pod),
                                  "gpus": own + hot})


async def serve(cfg) -> None:
    """Run until SIGTERM/SIGINT, then shut down cleanly (the kubelet sends SIGTERM on pod
    deletion; the reference's daemons just died — reference: cmd/*/main.go)."""
    m = Master(cfg)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    # a failed start still stops what it started: no gRPC server or executor thread left
    # behind keeps a half-started daemon alive
    try:
        await m.start()
        await stop.wait()
    finally:
        await m.stop()
