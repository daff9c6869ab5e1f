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

Decisions are cached briefly (``authz_token_ttl_s`` 60 s, ``authz_sar_ttl_s`` 30 s) so a burst of
requests costs no review round trip. The path stays warm and cheap beyond that:

* a cached answer used after half its lifetime is refreshed in the background (single flight),
  so a caller who keeps working never meets an expired entry;
* once an entry has expired, a token seen before has its TokenReview and its
  SubjectAccessReview — asked for the identity the token had last time — sent together: one
  round trip instead of two. The SAR answer counts only if the TokenReview confirms that same
  identity; otherwise the SAR is asked again for the new one;
* with ``authz_self_review`` (off by default), a token seen for the first time has its
  TokenReview and a SelfSubjectAccessReview made with the token itself sent together: the
  apiserver answers for whoever the token authenticates as, so no identity has to be guessed.
  Where the self-review is not served (or not allowed), the SubjectAccessReview follows the
  TokenReview as before.
"""
from __future__ import annotations

import asyncio
import hashlib
import hmac
import time
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

from gpumounter_amd.utils import log

_log = log.get("master.authz")
RESOURCE_SUB = "gpumount"


def _drop(task: Optional[asyncio.Future]) -> None:
    """Abandon a speculative review: cancel it, and retrieve its outcome once it is done (a SAR
    that already failed would otherwise log "Task exception was never retrieved")."""
    if task is None:
        return
    task.cancel()
    task.add_done_callback(lambda f: f.cancelled() or f.exception())


@dataclass
class Decision:
    allowed: bool
    status: int = 200          # 401 unauthenticated, 403 forbidden, 503 review failed
    reason: str = ""
    user: str = ""


class Authorizer:
    def __init__(self, cfg, kube, token_ttl_s: Optional[float] = None,
                 sar_ttl_s: Optional[float] = None) -> None:
        self.cfg = cfg
        self.kube = kube
        self.mode = cfg.authz_mode
        self.token_ttl_s = token_ttl_s if token_ttl_s is not None else \
            getattr(cfg, "authz_token_ttl_s", 60.0)
        self.sar_ttl_s = sar_ttl_s if sar_ttl_s is not None else \
            getattr(cfg, "authz_sar_ttl_s", 30.0)
        self._tokens: Dict[str, Tuple[float, Optional[dict]]] = {}
        self._sar: Dict[tuple, Tuple[float, bool]] = {}
        # token hash → the identity its last TokenReview returned (outlives the TTL: it is only
        # a guess that lets the SAR start early, never a decision)
        self._last_user: Dict[str, dict] = {}
        self._refreshing: set = set()
        self._bg: set = set()
        self.reviews = {"token": 0, "sar": 0, "speculative": 0, "refresh": 0, "self": 0}
        self.self_review = bool(getattr(cfg, "authz_self_review", False)) and \
            bool(getattr(kube, "bearer_only", False))

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
        key = hashlib.sha256(token.encode()).hexdigest()
        guess = None if self._fresh(self._tokens.get(key), self.token_ttl_s) else \
            self._last_user.get(key)
        spec = own = None
        if guess is not None:
            # expired token entry: the SAR for the identity it had goes out with the TokenReview
            self.reviews["speculative"] += 1
            spec = asyncio.ensure_future(self._authorize(guess, verb, namespace, resource, name))
        elif self.self_review and key not in self._tokens:
            # a token never seen: the apiserver reviews it as itself, alongside the TokenReview
            self.reviews["self"] += 1
            own = asyncio.ensure_future(self._self_review(token, verb, namespace, resource, name))
        try:
            user = await self._authenticate(token, key)
        except Exception as e:  # noqa: BLE001
            _drop(spec)
            _drop(own)
            _log.error("TokenReview failed: %s", e)
            return Decision(False, 503, "authentication unavailable")
        if user is None:
            _drop(spec)
            _drop(own)
            return Decision(False, 401, "Unauthorized: token not accepted")
        try:
            ok = await self._own_answer(own)
            if ok is not None:
                self._remember(user, verb, namespace, resource, name, ok)
            elif spec is not None and self._same(user, guess):
                ok = await spec
            else:
                _drop(spec)
                ok = await self._authorize(user, verb, namespace, resource, name)
        except Exception as e:  # noqa: BLE001
            _log.error("SubjectAccessReview failed: %s", e)
            return Decision(False, 503, "authorization unavailable", user["username"])
        if not ok:
            where = f" in namespace {namespace}" if namespace else ""
            return Decision(False, 403, f"Forbidden: {user['username']} cannot {verb} "
                                        f"{resource}/{RESOURCE_SUB}{where}", user["username"])
        return Decision(True, 200, "", user["username"])

    def expire(self) -> int:
        """Age every cached TokenReview and SubjectAccessReview answer past its TTL, as a long
        idle period would (the identities a token had stay known, as they do then). For the
        bench's cold-attach phase: the same process, caches expired. Returns the entries aged."""
        old = time.monotonic() - max(self.token_ttl_s, self.sar_ttl_s) - 1.0
        self._tokens = {k: (old, v) for k, (_, v) in self._tokens.items()}
        self._sar = {k: (old, v) for k, (_, v) in self._sar.items()}
        return len(self._tokens) + len(self._sar)

    @staticmethod
    def _fresh(hit, ttl: float) -> bool:
        return bool(hit) and time.monotonic() - hit[0] < ttl

    @staticmethod
    def _same(a: dict, b: dict) -> bool:
        return (a["username"], a["uid"], sorted(a["groups"]), a["extra"]) == \
            (b["username"], b["uid"], sorted(b["groups"]), b["extra"])

    def _refresh_ahead(self, what: tuple, hit, ttl: float, coro_fn) -> None:
        """A cached answer past half its lifetime: renew it in the background (single flight)
        so the next request still finds a fresh one."""
        if hit is None or time.monotonic() - hit[0] < ttl / 2 or what in self._refreshing:
            return
        self._refreshing.add(what)
        self.reviews["refresh"] += 1

        async def run():
            try:
                await coro_fn()
            except Exception as e:  # noqa: BLE001 - the entry simply expires
                _log.debug("background review refresh failed: %s", e)
            finally:
                self._refreshing.discard(what)
        t = asyncio.ensure_future(run())
        self._bg.add(t)
        t.add_done_callback(self._bg.discard)

    async def _authenticate(self, token: str, key: str = "", force: bool = False
                            ) -> Optional[dict]:
        key = key or hashlib.sha256(token.encode()).hexdigest()
        hit = self._tokens.get(key)
        if not force and self._fresh(hit, self.token_ttl_s):
            self._refresh_ahead(("token", key), hit, self.token_ttl_s,
                                lambda: self._authenticate(token, key, force=True))
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
            self._last_user.clear()
        self._tokens[key] = (time.monotonic(), user)
        if user is not None:
            self._last_user[key] = user
        else:
            self._last_user.pop(key, None)
        return user

    @staticmethod
    def _attrs(verb: str, namespace: str, resource: str, name: str) -> dict:
        attrs = {"verb": verb, "resource": resource, "subresource": RESOURCE_SUB,
                 "group": "", "version": "v1"}
        if namespace:
            attrs["namespace"] = namespace
        if name:
            attrs["name"] = name
        return attrs

    @staticmethod
    async def _own_answer(own: Optional[asyncio.Future]) -> Optional[bool]:
        """The self-review's answer; None if there was none or it failed (the API not served,
        the self-review not allowed to this user): a SubjectAccessReview decides instead."""
        if own is None:
            return None
        try:
            return await own
        except Exception as e:  # noqa: BLE001
            _log.debug("SelfSubjectAccessReview: %s; SubjectAccessReview instead", e)
            return None

    async def _self_review(self, token: str, verb: str, namespace: str, resource: str,
                           name: str) -> bool:
        st = await self.kube.self_subject_access_review(
            token, self._attrs(verb, namespace, resource, name))
        return bool(st.get("allowed")) and not st.get("denied")

    def _remember(self, user: dict, verb: str, namespace: str, resource: str, name: str,
                  ok: bool) -> None:
        if len(self._sar) > 16384:
            self._sar.clear()
        self._sar[(user["username"], tuple(user["groups"]), verb, namespace, resource, name)] = \
            (time.monotonic(), ok)

    async def _authorize(self, user: dict, verb: str, namespace: str, resource: str,
                         name: str, force: bool = False) -> bool:
        key = (user["username"], tuple(user["groups"]), verb, namespace, resource, name)
        hit = self._sar.get(key)
        if not force and self._fresh(hit, self.sar_ttl_s):
            self._refresh_ahead(("sar",) + key, hit, self.sar_ttl_s,
                                lambda: self._authorize(user, verb, namespace, resource, name,
                                                        force=True))
            return hit[1]
        self.reviews["sar"] += 1
        st = await self.kube.subject_access_review(
            user, self._attrs(verb, namespace, resource, name))
        ok = bool(st.get("allowed")) and not st.get("denied")
        self._remember(user, verb, namespace, resource, name, ok)
        return ok

    async def warm_up(self) -> None:
        """Open as many keep-alive connections to the apiserver as a first request's reviews
        run at once (two with the self-review), with TokenReviews of a token nobody holds:
        the reviews of the first request then connect nothing."""
        if self.mode != "kube":
            return
        n = 2 if self.self_review else 1
        await asyncio.gather(*(self.kube.token_review("gm-warm-up-not-a-token")
                               for _ in range(n)))

    async def stop(self) -> None:
        for t in list(self._bg):
            t.cancel()
