"""Minimal async Kubernetes REST client (pods + watch) on a lean HTTP/1.1 client
(``cluster/http1.py``).

Reference: client-go clientset singleton, always in-cluster, panicking on error, with a
placeholder out-of-cluster kubeconfig path (reference: pkg/config/config.go:11-45). Only
Pods Get/List/Create/Delete are used there, and readiness is found by busy-polling Get
(allocator.go:246-316). This client adds: in-cluster / kubeconfig / explicit-URL config, one
keep-alive session, typed errors, JSON merge-patch, and **watch streams** (the replacement for
busy-polling).
"""
from __future__ import annotations

import asyncio
import base64
import json
import os
import ssl
import tempfile
from typing import Any, AsyncIterator, Dict, List, Optional, Tuple
from urllib.parse import quote

import yaml

from gpumounter_amd.cluster import http1
from gpumounter_amd.utils import calls, log

_log = log.get("kube")
_RESOURCES = {"pods", "events", "resourceclaims", "resourceslices", "resourcequotas",
              "tokenreviews", "subjectaccessreviews", "selfsubjectaccessreviews", "nodes",
              "priorityclasses"}


def _kind(method: str, path: str) -> str:
    """``apiserver POST pods`` for the call log (utils/calls.py)."""
    for part in reversed(path.split("/")):
        if part in _RESOURCES:
            return f"apiserver {method} {part}"
    return f"apiserver {method}"

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


def seg(s: str) -> str:
    """One path segment of an apiserver URL: percent-quoted, so a name can never add a
    segment ("/"), walk up one ("..") or end the path ("?", "#"). Names the apiserver could
    not hold (empty, "." or "..") raise ValueError before anything is sent."""
    if not s or s in (".", ".."):
        raise ValueError(f"invalid object name {s!r}")
    return quote(s, safe="")


class ApiError(Exception):
    def __init__(self, status: int, reason: str, body: Any = None):
        super().__init__(f"{status} {reason}")
        self.status = status
        self.reason = reason
        self.body = body


class NotFound(ApiError):
    pass


class Conflict(ApiError):
    pass


class KubeClient:
    def __init__(self, base_url: str, token: str = "", ca_file: str = "",
                 client_cert: Optional[Tuple[str, str]] = None, insecure: bool = False,
                 timeout_s: float = 30.0) -> None:
        self.base = base_url.rstrip("/")
        self.token = token
        self.timeout_s = timeout_s
        self._ssl: Any = None
        if self.base.startswith("https"):
            if insecure:
                self._ssl = False
            else:
                ctx = ssl.create_default_context(cafile=ca_file or None)
                if client_cert:
                    ctx.load_cert_chain(*client_cert)
                self._ssl = ctx
        self._pool: Optional[http1.Pool] = None
        self._pool_loop = None
        # a request may carry another bearer token (a self-review as the caller) only when the
        # apiserver authenticates this client by its token, not by a TLS client certificate
        self.bearer_only = client_cert is None

    # ------------------------------------------------------------------------- construction
    @classmethod
    def from_config(cls, cfg) -> "KubeClient":
        if cfg.kube_api:
            return cls(cfg.kube_api, token=cfg.kube_token, ca_file=cfg.kube_ca,
                       insecure=cfg.kube_insecure)
        if cfg.kubeconfig:
            return cls.from_kubeconfig(cfg.kubeconfig)
        return cls.in_cluster()

    @classmethod
    def in_cluster(cls) -> "KubeClient":
        host = os.environ.get("KUBERNETES_SERVICE_HOST")
        port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        if not host:
            raise RuntimeError("not in a cluster (KUBERNETES_SERVICE_HOST unset) and no "
                               "kube_api/kubeconfig configured")
        with open(os.path.join(SA_DIR, "token"), encoding="utf-8") as fh:
            token = fh.read().strip()
        if ":" in host and not host.startswith("["):
            host = f"[{host}]"
        return cls(f"https://{host}:{port}", token=token, ca_file=os.path.join(SA_DIR, "ca.crt"))

    @classmethod
    def from_kubeconfig(cls, path: str, context: str = "") -> "KubeClient":
        with open(path, encoding="utf-8") as fh:
            kc = yaml.safe_load(fh)
        ctx_name = context or kc.get("current-context")
        ctx = next(c["context"] for c in kc["contexts"] if c["name"] == ctx_name)
        cluster = next(c["cluster"] for c in kc["clusters"] if c["name"] == ctx["cluster"])
        user = next((u["user"] for u in kc.get("users", []) if u["name"] == ctx.get("user")), {})

        def materialize(data_key: str, file_key: str, src: dict) -> str:
            if src.get(file_key):
                return src[file_key]
            if src.get(data_key):
                fd, p = tempfile.mkstemp(prefix="gm-kc-")
                with os.fdopen(fd, "wb") as out:
                    out.write(base64.b64decode(src[data_key]))
                return p
            return ""

        ca = materialize("certificate-authority-data", "certificate-authority", cluster)
        cert = materialize("client-certificate-data", "client-certificate", user)
        key = materialize("client-key-data", "client-key", user)
        return cls(cluster["server"], token=user.get("token", ""), ca_file=ca,
                   client_cert=(cert, key) if cert and key else None,
                   insecure=bool(cluster.get("insecure-skip-tls-verify")))

    # ------------------------------------------------------------------------- plumbing
    def _http(self) -> http1.Pool:
        loop = asyncio.get_running_loop()
        if self._pool is None or self._pool_loop is not loop:
            headers = {"Accept": "application/json"}
            if self.token:
                headers["Authorization"] = f"Bearer {self.token}"
            # idle keep-alive connections live a minute, so requests a minute apart (an
            # operator's attaches, the reviews of an expired authz answer) connect nothing
            self._pool = http1.Pool(self.base, self._ssl, headers, keepalive_s=60.0,
                                    timeout_s=self.timeout_s)
            self._pool_loop = loop
        return self._pool

    async def close(self) -> None:
        if self._pool is not None:
            await self._pool.close()
        self._pool = None

    # transient apiserver trouble (a control-plane node restarting, an overloaded apiserver
    # shedding load with 429/5xx): retried with backoff for requests that are safe to repeat
    RETRY_STATUS = (429, 500, 502, 503, 504)
    retries = 0     # requests retried (per instance once one happened)
    RETRY_DELAYS = (0.01, 0.05, 0.2, 0.5)

    async def _req(self, method: str, path: str, params: Optional[dict] = None,
                   body: Any = None, content_type: str = "application/json",
                   idempotent: Optional[bool] = None, as_token: str = "") -> Any:
        """One API request. GET/PATCH/DELETE (and POSTs the caller marks ``idempotent``) are
        retried on 429/5xx and transport errors; a transport failure surfaces as
        ``ApiError(503)`` so callers handle one exception type."""
        retry = idempotent if idempotent is not None else method in ("GET", "PATCH", "DELETE")
        delays = self.RETRY_DELAYS if retry else ()
        for attempt in range(len(delays) + 1):
            try:
                return await self._req_once(method, path, params, body, content_type,
                                            as_token, replayable=retry)
            except ApiError as e:
                if e.status not in self.RETRY_STATUS or attempt == len(delays):
                    raise
                why = f"HTTP {e.status}"
            except (asyncio.TimeoutError, OSError) as e:
                if attempt == len(delays):
                    raise ApiError(503, f"apiserver unreachable: {e!r}") from e
                why = repr(e)
            self.retries += 1
            _log.warning("%s %s: %s; retry %d in %.0f ms", method, path, why, attempt + 1,
                         delays[attempt] * 1e3)
            await asyncio.sleep(delays[attempt])
        raise AssertionError("unreachable")

    async def _req_once(self, method: str, path: str, params: Optional[dict], body: Any,
                        content_type: str, as_token: str = "", replayable: bool = False) -> Any:
        """``replayable``: the transport may resend the request on a fresh connection when a
        kept-alive one turns out closed (only requests ``_req`` would retry anyway: a POST
        that may have been processed is never sent twice behind the caller's back)."""
        pool = self._http()
        data = None
        headers = {"Authorization": f"Bearer {as_token}"} if as_token else {}
        if body is not None:
            data = json.dumps(body).encode()
            headers["Content-Type"] = content_type
        with calls.span(_kind(method, path)):
            status, _, raw = await pool.request(method, pool.target(path, params),
                                                headers or None, data, replayable=replayable)
        if status >= 400:
            text = raw.decode("utf-8", "replace")
            try:
                payload = json.loads(text)
            except ValueError:
                payload = text
            reason = payload.get("message", text) if isinstance(payload, dict) else text
            if status == 404:
                raise NotFound(404, reason, payload)
            if status == 409:
                raise Conflict(409, reason, payload)
            raise ApiError(status, reason, payload)
        return json.loads(raw) if raw else None

    @staticmethod
    def _pods_path(ns: Optional[str], name: str = "") -> str:
        base = f"/api/v1/namespaces/{seg(ns)}/pods" if ns else "/api/v1/pods"
        return f"{base}/{seg(name)}" if name else base

    # ------------------------------------------------------------------------- pods
    async def get_pod(self, ns: str, name: str) -> dict:
        return await self._req("GET", self._pods_path(ns, name))

    async def list_pods(self, ns: Optional[str] = None, label_selector: str = "",
                        field_selector: str = "", limit: int = 0) -> Tuple[List[dict], str]:
        """All matching Pods and the list's resourceVersion, read in pages of ``limit``
        (``PAGE`` by default) so no single response holds the whole collection."""
        items: List[dict] = []
        rv = ""
        async for page, rv in self.list_pages(self._pods_path(ns), label_selector,
                                              field_selector, limit):
            if page is None:            # the list restarted: earlier pages are stale
                items = []
                continue
            items.extend(page)
        return items, rv

    # page size of every LIST (client-go's reflector pages by 500 too)
    PAGE = 500
    # a continue token that expired mid-list (410) restarts the list this many times before
    # the error is raised to the caller (a watch-based caller relists on its own schedule)
    PAGE_RESTARTS = 3

    async def list_pages(self, path: str, label_selector: str = "", field_selector: str = "",
                         limit: int = 0) -> AsyncIterator[Tuple[List[dict], str]]:
        """Yield ``(items, resourceVersion)`` page by page (``limit`` + ``continue``). The
        resourceVersion is the list's, the same on every page of one consistent snapshot.
        A continue token that the apiserver no longer serves (410 Expired, the snapshot was
        compacted) restarts the list from the first page; the caller sees a ``None`` page
        first, meaning: drop what the earlier pages gave you."""
        limit = limit or self.PAGE
        restarts = 0
        cont = ""
        while True:
            params = {"limit": str(limit)}
            if label_selector:
                params["labelSelector"] = label_selector
            if field_selector:
                params["fieldSelector"] = field_selector
            if cont:
                params["continue"] = cont
            try:
                out = await self._req("GET", path, params=params)
            except ApiError as e:
                if e.status != 410 or not cont or restarts >= self.PAGE_RESTARTS:
                    raise
                restarts += 1
                _log.info("LIST %s: continue token expired; restarting the list", path)
                cont = ""
                yield None, ""          # type: ignore[misc]
                continue
            md = out.get("metadata", {}) or {}
            yield out.get("items", []) or [], md.get("resourceVersion", "")
            cont = md.get("continue") or ""
            if not cont:
                return

    async def get_priority_class(self, name: str) -> dict:
        return await self._req("GET", f"/apis/scheduling.k8s.io/v1/priorityclasses/{seg(name)}")

    async def create_pod(self, ns: str, pod: dict, dry_run: bool = False) -> dict:
        """Create; retried on transient errors when the name is explicit (a retry that finds
        the pod already created by the lost first attempt returns that pod). ``dry_run``: the
        apiserver validates and admits it but stores nothing (``?dryRun=All``)."""
        name = (pod.get("metadata") or {}).get("name", "")
        if dry_run:
            return await self._req("POST", self._pods_path(ns), params={"dryRun": "All"},
                                   body=pod, idempotent=True)
        try:
            return await self._req("POST", self._pods_path(ns), body=pod, idempotent=bool(name))
        except Conflict:
            if not name:
                raise
            cur = await self.get_pod(ns, name)
            mine = (pod.get("metadata") or {}).get("annotations") or {}
            theirs = (cur.get("metadata") or {}).get("annotations") or {}
            if mine and all(theirs.get(k) == v for k, v in mine.items()):
                return cur                  # our own create went through before the error
            raise

    async def delete_pod(self, ns: str, name: str, grace_period_s: Optional[int] = None,
                         uid: str = "", resource_version: str = "") -> Optional[dict]:
        body: Dict[str, Any] = {"kind": "DeleteOptions", "apiVersion": "v1"}
        if grace_period_s is not None:
            body["gracePeriodSeconds"] = int(grace_period_s)
        pre = {k: v for k, v in (("uid", uid), ("resourceVersion", resource_version)) if v}
        if pre:
            body["preconditions"] = pre
        return await self._req("DELETE", self._pods_path(ns, name), body=body)

    # ---- resource.k8s.io/v1 (DRA): ResourceClaims and ResourceSlices -----------------------
    _DRA = "/apis/resource.k8s.io/v1"

    async def create_claim(self, ns: str, claim: dict) -> dict:
        name = (claim.get("metadata") or {}).get("name", "")
        try:
            return await self._req("POST", f"{self._DRA}/namespaces/{seg(ns)}/resourceclaims",
                                   body=claim, idempotent=bool(name))
        except Conflict:
            cur = await self.get_claim(ns, name)
            mine = (claim.get("metadata") or {}).get("labels") or {}
            theirs = (cur.get("metadata") or {}).get("labels") or {}
            if mine and all(theirs.get(k) == v for k, v in mine.items()):
                return cur                  # our own create went through before the error
            raise

    async def get_claim(self, ns: str, name: str) -> dict:
        return await self._req("GET", f"{self._DRA}/namespaces/{seg(ns)}/resourceclaims/{seg(name)}")

    async def delete_claim(self, ns: str, name: str) -> Optional[dict]:
        return await self._req("DELETE", f"{self._DRA}/namespaces/{seg(ns)}/resourceclaims/{seg(name)}")

    async def list_claims(self, ns: str = "", label_selector: str = "") -> List[dict]:
        return (await self.list_claims_rv(ns, label_selector))[0]

    async def list_slices(self, node: str = "") -> List[dict]:
        params = {"fieldSelector": f"spec.nodeName={node}"} if node else None
        return (await self._req("GET", f"{self._DRA}/resourceslices", params=params)).get(
            "items", [])

    async def patch_pod(self, ns: str, name: str, patch: dict) -> dict:
        return await self._req("PATCH", self._pods_path(ns, name), body=patch,
                               content_type="application/merge-patch+json")

    async def token_review(self, token: str) -> dict:
        out = await self._req("POST", "/apis/authentication.k8s.io/v1/tokenreviews", body={
            "apiVersion": "authentication.k8s.io/v1", "kind": "TokenReview",
            "spec": {"token": token}})
        return (out or {}).get("status") or {}

    async def subject_access_review(self, user: dict, resource_attributes: dict) -> dict:
        out = await self._req("POST", "/apis/authorization.k8s.io/v1/subjectaccessreviews",
                              body={"apiVersion": "authorization.k8s.io/v1",
                                    "kind": "SubjectAccessReview",
                                    "spec": {"user": user.get("username", ""),
                                             "uid": user.get("uid", ""),
                                             "groups": user.get("groups", []),
                                             "extra": user.get("extra", {}),
                                             "resourceAttributes": resource_attributes}})
        return (out or {}).get("status") or {}

    async def self_subject_access_review(self, token: str, resource_attributes: dict) -> dict:
        """A SelfSubjectAccessReview sent with the caller's ``token``: the apiserver
        authenticates the token and answers for that user (allowed to every authenticated user
        by the default ``system:basic-user`` role)."""
        out = await self._req("POST", "/apis/authorization.k8s.io/v1/selfsubjectaccessreviews",
                              body={"apiVersion": "authorization.k8s.io/v1",
                                    "kind": "SelfSubjectAccessReview",
                                    "spec": {"resourceAttributes": resource_attributes}},
                              idempotent=True, as_token=token)
        return (out or {}).get("status") or {}

    async def list_resource_quotas(self, ns: str) -> List[dict]:
        return (await self._list_all(f"/api/v1/namespaces/{seg(ns)}/resourcequotas"))[0]

    @staticmethod
    def _quotas_path(ns: Optional[str]) -> str:
        return f"/api/v1/namespaces/{seg(ns)}/resourcequotas" if ns else "/api/v1/resourcequotas"

    async def list_quotas_rv(self, ns: Optional[str] = None, label_selector: str = ""
                             ) -> Tuple[List[dict], str]:
        return await self._list_all(self._quotas_path(ns), label_selector)

    async def _list_all(self, path: str, label_selector: str = "", field_selector: str = ""
                        ) -> Tuple[List[dict], str]:
        items: List[dict] = []
        rv = ""
        async for page, rv in self.list_pages(path, label_selector, field_selector):
            if page is None:
                items = []
                continue
            items.extend(page)
        return items, rv

    async def get_quota(self, ns: str, name: str) -> dict:
        return await self._req("GET", f"{self._quotas_path(ns)}/{seg(name)}")

    async def watch_quotas(self, ns: Optional[str] = None, label_selector: str = "",
                           field_selector: str = "", resource_version: str = "",
                           timeout_s: int = 300) -> AsyncIterator[Tuple[str, dict]]:
        async for ev in self.watch(self._quotas_path(ns), label_selector, field_selector,
                                   resource_version, timeout_s):
            yield ev

    async def create_event(self, ns: str, event: dict) -> dict:
        return await self._req("POST", f"/api/v1/namespaces/{seg(ns)}/events", body=event)

    async def watch_pods(self, ns: Optional[str] = None, label_selector: str = "",
                         field_selector: str = "", resource_version: str = "",
                         timeout_s: int = 300) -> AsyncIterator[Tuple[str, dict]]:
        """Yield ``(type, pod)`` events (ADDED/MODIFIED/DELETED/BOOKMARK/ERROR)."""
        async for ev in self.watch(self._pods_path(ns), label_selector, field_selector,
                                   resource_version, timeout_s):
            yield ev

    def _claims_path(self, ns: Optional[str]) -> str:
        return f"{self._DRA}/namespaces/{seg(ns)}/resourceclaims" if ns else \
            f"{self._DRA}/resourceclaims"

    async def list_claims_rv(self, ns: Optional[str] = None, label_selector: str = ""
                             ) -> Tuple[List[dict], str]:
        return await self._list_all(self._claims_path(ns), label_selector)

    async def watch_claims(self, ns: Optional[str] = None, label_selector: str = "",
                           field_selector: str = "", resource_version: str = "",
                           timeout_s: int = 300) -> AsyncIterator[Tuple[str, dict]]:
        async for ev in self.watch(self._claims_path(ns), label_selector, field_selector,
                                   resource_version, timeout_s):
            yield ev

    async def watch(self, path: str, label_selector: str = "", field_selector: str = "",
                    resource_version: str = "", timeout_s: int = 300
                    ) -> AsyncIterator[Tuple[str, dict]]:
        """Yield ``(type, object)`` watch events of a collection path."""
        params = {"watch": "true", "timeoutSeconds": str(timeout_s),
                  "allowWatchBookmarks": "true"}
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        if resource_version:
            params["resourceVersion"] = resource_version
        pool = self._http()
        status, _, lines = await pool.stream("GET", pool.target(path, params),
                                             read_timeout_s=timeout_s + 30)
        try:
            if status >= 400:
                raise ApiError(status, b"\n".join([ln async for ln in lines]).decode(
                    "utf-8", "replace"))
            async for line in lines:
                ev = json.loads(line)
                yield ev.get("type", ""), ev.get("object", {})
        finally:
            lines.close()
