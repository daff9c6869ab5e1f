"""Who may hot-mount GPUs into which namespace.

The reference authenticates and authorizes nobody (SURVEY §2.6 defect 13): anyone who reaches the
master can attach GPUs to, or force-kill processes in, any pod. Modes (``GM_AUTHZ_MODE``):

* ``none``  — open, as the reference; if ``api_token`` is set, a single shared bearer token.
* ``kube``  — the caller's own Kubernetes bearer token. It is authenticated with a TokenReview,
  then a SubjectAccessReview asks the cluster's authorizer (RBAC) whether that user may perform
  the operation on the virtual subresource ``pods/gpumount`` in the target namespace:
  ``create`` to attach, ``delete`` to detach, ``get`` to read a pod's GPUs. Node status needs
  ``get`` on ``nodes/gpumount``. Admins grant hot-mount rights with plain RBAC, for example
  ``deploy/rbac-tenant-example.yaml``.

Decisions are cached briefly (TokenReview 60 s, SubjectAccessReview 30 s) so a burst of requests
costs one review round trip, not one per request.
"""
from __future__ import annotations

import hashlib
import hmac
import time
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

from gpumounter_amd.utils import log

_log = log.get("master.authz")
RESOURCE_SUB = "gpumount"


@dataclass
class Decision:
    allowed: bool
    status: int = 200          # 401 unauthenticated, 403 forbidden, 503 review failed
    reason: str = ""
    user: str = ""


class Authorizer:
    def __init__(self, cfg, kube, token_ttl_s: float = 60.0, sar_ttl_s: float = 30.0) -> None:
        self.cfg = cfg
        self.kube = kube
        self.mode = cfg.authz_mode
        self.token_ttl_s = token_ttl_s
        self.sar_ttl_s = sar_ttl_s
        self._tokens: Dict[str, Tuple[float, Optional[dict]]] = {}
        self._sar: Dict[tuple, Tuple[float, bool]] = {}
        self.reviews = {"token": 0, "sar": 0}

    @staticmethod
    def _bearer(headers) -> str:
        got = headers.get("Authorization", "")
        return got[7:].strip() if got.startswith("Bearer ") else ""

    async def check(self, headers, verb: str, namespace: str = "", resource: str = "pods",
                    name: str = "") -> Decision:
        if self.mode != "kube":
            if not self.cfg.api_token:
                return Decision(True)
            got = headers.get("Authorization", "")
            if hmac.compare_digest(got, f"Bearer {self.cfg.api_token}"):
                return Decision(True)
            return Decision(False, 401, "Unauthorized")
        token = self._bearer(headers)
        if not token:
            return Decision(False, 401, "Unauthorized: bearer token required")
        try:
            user = await self._authenticate(token)
        except Exception as e:  # noqa: BLE001
            _log.error("TokenReview failed: %s", e)
            return Decision(False, 503, "authentication unavailable")
        if user is None:
            return Decision(False, 401, "Unauthorized: token not accepted")
        try:
            ok = await self._authorize(user, verb, namespace, resource, name)
        except Exception as e:  # noqa: BLE001
            _log.error("SubjectAccessReview failed: %s", e)
            return Decision(False, 503, "authorization unavailable", user["username"])
        if not ok:
            where = f" in namespace {namespace}" if namespace else ""
            return Decision(False, 403, f"Forbidden: {user['username']} cannot {verb} "
                                        f"{resource}/{RESOURCE_SUB}{where}", user["username"])
        return Decision(True, 200, "", user["username"])

    async def _authenticate(self, token: str) -> Optional[dict]:
        key = hashlib.sha256(token.encode()).hexdigest()
        now = time.monotonic()
        hit = self._tokens.get(key)
        if hit and now - hit[0] < self.token_ttl_s:
            return hit[1]
        self.reviews["token"] += 1
        st = await self.kube.token_review(token)
        user = None
        if st.get("authenticated"):
            u = st.get("user") or {}
            user = {"username": u.get("username", ""), "uid": u.get("uid", ""),
                    "groups": list(u.get("groups") or []), "extra": u.get("extra") or {}}
        if len(self._tokens) > 4096:
            self._tokens.clear()
        self._tokens[key] = (now, user)
        return user

    async def _authorize(self, user: dict, verb: str, namespace: str, resource: str,
                         name: str) -> bool:
        key = (user["username"], tuple(user["groups"]), verb, namespace, resource, name)
        now = time.monotonic()
        hit = self._sar.get(key)
        if hit and now - hit[0] < self.sar_ttl_s:
            return hit[1]
        self.reviews["sar"] += 1
        attrs = {"verb": verb, "resource": resource, "subresource": RESOURCE_SUB,
                 "group": "", "version": "v1"}
        if namespace:
            attrs["namespace"] = namespace
        if name:
            attrs["name"] = name
        st = await self.kube.subject_access_review(user, attrs)
        ok = bool(st.get("allowed")) and not st.get("denied")
        if len(self._sar) > 16384:
            self._sar.clear()
        self._sar[key] = (now, ok)
        return ok
