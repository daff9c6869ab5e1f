"""List+watch pod cache with awaitable predicates.

Replaces the reference's readiness loops, which call ``Pods.Get`` for every slave pod in a tight
loop with no sleep and no timeout (reference: pkg/util/gpu/allocator/allocator.go:236-317 —
SURVEY §2.6 defect 1). One watch stream per selector feeds a cache; callers ``await`` a predicate
and are woken by the next matching event instead of polling the apiserver.
"""
from __future__ import annotations

import asyncio
from collections import OrderedDict, deque
from typing import Callable, Dict, List, Optional, Tuple

from gpumounter_amd.cluster.kube import ApiError, KubeClient, NotFound
from gpumounter_amd.models.pod import jcopy
from gpumounter_amd.utils import calls, log

_log = log.get("cluster.informer")

Key = Tuple[str, str]
DELETED_KEEP = 65536


class PodInformer:
    # a re-read after a relist (``_resolve``) gives up after this long; below the worker's
    # SETTLE_WAIT_S, so a stalled GET delays pod views by at most this, never fails them
    RESOLVE_TIMEOUT_S = 1.5

    def __init__(self, kube: KubeClient, namespace: Optional[str] = None, label_selector: str = "",
                 field_selector: str = "", resync_s: float = 300.0) -> None:
        self.kube = kube
        self.namespace = namespace
        self.label_selector = label_selector
        self.field_selector = field_selector
        self.resync_s = resync_s
        self.cache: Dict[Key, dict] = {}
        # key → uid of the last deleted instance, for write-throughs that arrive after the
        # DELETED event (an in-flight request's window); the oldest entries are dropped, so a
        # worker that sees every placeholder ever created does not keep them all
        self.deleted: "OrderedDict[Key, str]" = OrderedDict()
        self._cond: Optional[asyncio.Condition] = None
        self._task: Optional[asyncio.Task] = None
        self._synced: Optional[asyncio.Event] = None
        self.rv = ""
        self.events = 0
        self.relists = 0
        self.resumes = 0
        self._seen: Dict[Key, deque] = {}    # resourceVersions the watch/list delivered per key
        # bumped by every relist: a write whose request went out in an earlier epoch may be
        # older than what the list delivered (see upsert)
        self.epoch = 0
        # key → resourceVersion of a write-through the watch has not delivered yet: until it
        # does, the watch's events for that key are older than the cached object
        self._pending: Dict[Key, str] = {}
        self.resolved = 0        # objects re-read with a GET after a relist (see _relist)
        self._bg: set = set()
        # keys whose write-through a relist overtook, being re-read (see upsert): until then
        # the cache may show them older than this process's own acknowledged writes
        self._resolving: Dict[Key, int] = {}
        # a relist replaces the cache with its list, which can be older than writes of ours
        # acknowledged while it was in flight (a create the list does not hold at all): those
        # are kept here and re-read once the relist is installed (see _relist)
        self._relisting = False
        self._written: Dict[Key, dict] = {}
        # per key, how many write-throughs were acknowledged: a GET sent before one of them
        # may answer with an older version, which must not replace it (see _resolve_once)
        self._writes: Dict[Key, int] = {}
        self.handlers: List[Callable[[str, dict], None]] = []

    async def start(self) -> None:
        self._cond = asyncio.Condition()
        self._synced = asyncio.Event()
        self._task = asyncio.ensure_future(self._run())
        await asyncio.wait_for(self._synced.wait(), timeout=30)

    async def stop(self) -> None:
        for t in list(self._bg):
            t.cancel()
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
            self._task = None

    def _list(self):
        return self.kube.list_pods(self.namespace, self.label_selector, self.field_selector)

    def _watch(self, timeout_s: int):
        return self.kube.watch_pods(self.namespace, self.label_selector, self.field_selector,
                                    self.rv, timeout_s=timeout_s)

    def _get(self, ns: str, name: str):
        return self.kube.get_pod(ns, name)

    async def _fetch(self, key: Key) -> Optional[dict]:
        """The object as the apiserver has it now (None: deleted)."""
        try:
            return await self._get(*key)
        except NotFound:
            return None

    async def _relist(self) -> None:
        self._relisting, self._written = True, {}
        try:
            written = await self._relist_once()
        finally:
            self._relisting, self._written = False, {}
        # a write acknowledged while the relist was in flight may be older or newer than the
        # list (or, a create, missing from it): a GET, newer than both, settles it. Queued
        # before the RELIST handlers run, so whatever they trigger waits for it (``settled``)
        for k in written:
            self._resolve_soon(k)
        await self._notify("RELIST", {})

    async def _relist_once(self) -> List[Key]:
        items, rv = await self._list()
        fresh = {(p["metadata"]["namespace"], p["metadata"]["name"]): p for p in items}
        # our acknowledged writes the watch had not echoed yet: where the list holds another
        # version, it may be older than the write (the list was served before it) or newer —
        # resourceVersions do not say which, a GET issued now does (it is newer than both)
        suspects = [k for k, prv in self._pending.items()
                    if k in fresh and fresh[k]["metadata"].get("resourceVersion") != prv]
        if suspects:
            got = await asyncio.gather(*[self._fetch(k) for k in suspects],
                                       return_exceptions=True)
            pending = {}
            for k, obj in zip(suspects, got):
                if isinstance(obj, BaseException):
                    continue            # keep the listed version; the watch still converges
                if obj is None:
                    fresh.pop(k, None)
                    continue
                listed = fresh[k]["metadata"].get("resourceVersion", "")
                fresh[k] = obj
                grv = obj["metadata"].get("resourceVersion", "")
                if grv != listed:
                    # changed after the list's snapshot: the watch, resumed from the list's
                    # version, will deliver it — older replays wait for it. (Equal: the list
                    # was already current, and no event for it is coming to wait for.)
                    pending[k] = grv
            self.resolved += len(suspects)
        else:
            pending = {}
        # our writes acknowledged meanwhile stand in for what the list lacks until re-read
        written = dict(self._written)
        self._seen = {k: self._seen[k] for k in fresh if k in self._seen}
        for k, p in fresh.items():
            self._note(k, p["metadata"].get("resourceVersion", ""))
        for k, p in written.items():
            fresh.setdefault(k, p)
        for k in set(self.cache) - set(fresh):
            self._forget(k, self.cache[k]["metadata"].get("uid", ""))
        self.cache = fresh
        self.rv = rv
        self.epoch += 1
        # a fetched version is newer than the list: the resumed watch's older events for
        # that key are skipped until it delivers this version (see _run)
        self._pending = {k: v for k, v in pending.items() if v}
        return list(written)

    async def _notify(self, etype: str, pod: dict) -> None:
        for h in list(self.handlers):
            try:
                h(etype, pod)
            except Exception:  # noqa: BLE001
                _log.exception("informer handler failed")
        async with self._cond:
            self._cond.notify_all()

    async def _run(self, initial_list: bool = True) -> None:
        """LIST once, then WATCH from the list's resourceVersion. A watch that ends cleanly (the
        server's timeoutSeconds) is resumed from the last resourceVersion seen — events, and
        the BOOKMARKs the server sends while idle, keep it current — so there is no relist per
        resync period. Only an error relists: 410 Gone (the version left the server's history)
        at once, anything else after a backoff."""
        calls.mark_background()
        backoff = 0.05
        need_list = initial_list
        while True:
            try:
                if need_list:
                    await self._relist()
                    self._synced.set()
                    need_list = False
                    self.relists += 1
                async for etype, pod in self._watch(int(self.resync_s)):
                    backoff = 0.05
                    md = pod.get("metadata", {})
                    if etype == "ERROR":
                        raise ApiError(int(pod.get("code", 500)), pod.get("message", ""))
                    if md.get("resourceVersion"):
                        self.rv = md["resourceVersion"]
                    if etype == "BOOKMARK":
                        continue
                    key = (md.get("namespace", ""), md.get("name", ""))
                    self.events += 1
                    if etype != "DELETED":
                        self._note(key, md.get("resourceVersion", ""))
                    if etype == "DELETED":
                        self.cache.pop(key, None)
                        self._seen.pop(key, None)   # stale upserts: caught by `deleted`
                        self._pending.pop(key, None)
                        self._forget(key, md.get("uid", ""))
                    elif key in self._pending and \
                            self._pending[key] != md.get("resourceVersion", ""):
                        pass        # older than our write-through: the cache is newer
                    else:
                        self._pending.pop(key, None)
                        self.cache[key] = pod
                        self.deleted.pop(key, None)
                    await self._notify(etype, pod)
                self.resumes += 1            # clean end of stream: watch again from self.rv
            except asyncio.CancelledError:
                raise
            except ApiError as e:
                need_list = True
                if e.status == 410:          # expired version: relist now, no backoff
                    _log.info("watch %s/%s: resourceVersion expired; relisting",
                              self.namespace, self.label_selector)
                    continue
                _log.warning("watch %s/%s failed: %s; relisting in %.2fs", self.namespace,
                             self.label_selector, e, backoff)
                await asyncio.sleep(backoff)
                backoff = min(backoff * 2, 5.0)
            except Exception as e:  # noqa: BLE001
                need_list = True
                _log.warning("watch %s/%s failed: %s; relisting in %.2fs", self.namespace,
                             self.label_selector, e, backoff)
                await asyncio.sleep(backoff)
                backoff = min(backoff * 2, 5.0)

    def _forget(self, key: Key, uid: str) -> None:
        self._writes.pop(key, None)
        self.deleted.pop(key, None)
        self.deleted[key] = uid
        while len(self.deleted) > DELETED_KEEP:
            self.deleted.popitem(last=False)

    def _note(self, key: Key, rv: str) -> None:
        if rv:
            seen = self._seen.get(key)
            if seen is None:
                seen = self._seen[key] = deque(maxlen=16)
            seen.append(rv)

    def upsert(self, pod: dict, epoch: Optional[int] = None) -> None:
        """Write-through from our own API responses (create/patch) so readers do not wait for
        the watch echo. resourceVersions are opaque (only equality is meaningful), so ordering
        comes from the watch itself: one object's events arrive in order, so if the watch has
        already delivered this response's version, the cache is at least as new and is kept;
        if not, the watch has not reached our write yet and the response is newer.

        ``epoch``: :attr:`epoch` when the request was sent. A relist since then breaks the
        argument above — the list may hold a *newer* version (someone wrote after us) that the
        watch will never deliver again — so for an object the list holds, the response is
        dropped: the list is either newer, or older and then the watch, resumed from the list's
        version, still delivers our write."""
        md = pod.get("metadata", {})
        key = (md.get("namespace", ""), md.get("name", ""))
        rv = md.get("resourceVersion", "")
        if rv and rv in self._seen.get(key, ()):
            return
        self._writes[key] = self._writes.get(key, 0) + 1
        if epoch is not None and epoch != self.epoch:
            cur = self.cache.get(key)
            if cur is not None and cur["metadata"].get("uid") == md.get("uid"):
                # the relist holds this object in some version, older or newer than our
                # write: a GET decides (until it answers, readers see the listed version)
                self._resolve_soon(key)
                return
        if key in self.deleted and self.deleted[key] == md.get("uid"):
            return
        self.cache[key] = pod
        if rv:
            self._pending[key] = rv
        if self._relisting:
            self._written[key] = pod

    def _resolve_soon(self, key: Key) -> None:
        try:
            loop = asyncio.get_running_loop()
        except RuntimeError:
            return
        self._resolving[key] = self._resolving.get(key, 0) + 1
        t = loop.create_task(self._resolve(key))
        self._bg.add(t)
        t.add_done_callback(self._bg.discard)

    @property
    def settled(self) -> bool:
        """No write-through of ours is waiting to be re-read after a relist: the cache holds
        every write this process has had acknowledged."""
        return not self._resolving

    async def _resolve(self, key: Key, tries: int = 3) -> None:
        calls.mark_background()
        try:
            await self._resolve_once(key, tries)
        finally:
            n = self._resolving.get(key, 0) - 1
            if n > 0:
                self._resolving[key] = n
            else:
                self._resolving.pop(key, None)
            if self._cond is not None:
                async with self._cond:
                    self._cond.notify_all()

    async def _resolve_once(self, key: Key, tries: int) -> None:
        """Replace the cached ``key`` with a fresh GET, unless another relist overtook the GET
        (then the GET may be older than that list: try again)."""
        for _ in range(tries):
            epoch, writes = self.epoch, self._writes.get(key, 0)
            try:
                # bounded well below the kube client's 30 s: while any re-read is out the view
                # is not ``settled``, and every pod view on the node waits for that (worker
                # service pod_state, up to its SETTLE_WAIT_S). One slow GET must not hold up
                # the node's attaches and detaches for half a minute
                obj = await asyncio.wait_for(self._fetch(key), self.RESOLVE_TIMEOUT_S)
            except Exception:  # noqa: BLE001 - the watch still converges; this only shortens it
                return
            if epoch != self.epoch or writes != self._writes.get(key, 0):
                continue        # a relist or a write of ours overtook the GET: maybe older
            self.resolved += 1
            if obj is not None and obj["metadata"].get("resourceVersion", "") in \
                    self._seen.get(key, ()):
                return      # the watch delivered this version meanwhile: the cache is as new
            if obj is None:
                cur = self.cache.pop(key, None)
                if cur is not None:
                    self._forget(key, cur["metadata"].get("uid", ""))
                    await self._notify("DELETED", cur)
                return
            self.cache[key] = obj
            rv = obj["metadata"].get("resourceVersion", "")
            if rv:
                self._pending[key] = rv
            await self._notify("MODIFIED", obj)
            return

    # ------------------------------------------------------------------------ queries
    def get(self, ns: str, name: str) -> Optional[dict]:
        """The cached object itself — read-only for callers. Entries are replaced wholesale on
        every event (never mutated in place), so a reader's reference stays a consistent
        snapshot; callers that need to modify use :meth:`get_copy`."""
        return self.cache.get((ns, name))

    def get_copy(self, ns: str, name: str) -> Optional[dict]:
        p = self.cache.get((ns, name))
        return jcopy(p) if p is not None else None

    def list(self, pred: Callable[[dict], bool] = lambda p: True) -> List[dict]:
        return [p for p in self.cache.values() if pred(p)]

    async def wait_for(self, pred: Callable[[], Optional[object]], timeout: float):
        """Await until ``pred()`` returns a truthy value (re-evaluated on every event)."""
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout
        async with self._cond:
            while True:
                v = pred()
                if v:
                    return v
                left = deadline - loop.time()
                if left <= 0:
                    raise asyncio.TimeoutError()
                try:
                    await asyncio.wait_for(self._cond.wait(), timeout=left)
                except asyncio.TimeoutError:
                    v = pred()
                    if v:
                        return v
                    raise

    async def poke(self) -> None:
        """Wake waiters (used when a non-watch signal, e.g. the kubelet ledger, changed)."""
        async with self._cond:
            self._cond.notify_all()


class ClaimInformer(PodInformer):
    """The same list+watch cache over ``resource.k8s.io/v1`` ResourceClaims (DRA mode: the
    placeholders' claims, whose allocation then arrives with the watch instead of a GET)."""

    def _list(self):
        return self.kube.list_claims_rv(self.namespace, self.label_selector)

    def _get(self, ns: str, name: str):
        return self.kube.get_claim(ns, name)

    def _watch(self, timeout_s: int):
        return self.kube.watch_claims(self.namespace, self.label_selector, self.field_selector,
                                      self.rv, timeout_s=timeout_s)


class QuotaInformer(PodInformer):
    """List+watch of ResourceQuotas (cluster-wide): the namespace GPU quota check reads
    ``spec.hard`` and the quota controller's ``status.used`` from here instead of a LIST per
    attach (cluster/quota.py)."""

    def _list(self):
        return self.kube.list_quotas_rv(self.namespace, self.label_selector)

    def _get(self, ns: str, name: str):
        return self.kube.get_quota(ns, name)

    def _watch(self, timeout_s: int):
        return self.kube.watch_quotas(self.namespace, self.label_selector, self.field_selector,
                                      self.rv, timeout_s=timeout_s)


def slim_pod(p: dict) -> dict:
    """What the master needs of a Pod to route a request: identity, node, phase."""
    md = p.get("metadata", {})
    out = {"metadata": {k: md[k] for k in ("name", "namespace", "uid", "resourceVersion",
                                           "deletionTimestamp") if k in md},
           "spec": {"nodeName": (p.get("spec") or {}).get("nodeName", "")},
           "status": {"phase": (p.get("status") or {}).get("phase", "")}}
    return out


class SlimPodInformer(PodInformer):
    """List+watch of every Pod, cached as :func:`slim_pod` projections (~300 bytes each instead
    of the whole object: 100k Pods ≈ 30 MB). The master's pod → node index."""

    async def _list(self):
        # page by page: only the projections are kept, never a whole cluster's Pods at once
        items, rv = [], ""
        async for page, rv in self.kube.list_pages(self.kube._pods_path(self.namespace),  # noqa: SLF001
                                                   self.label_selector, self.field_selector):
            if page is None:          # the list restarted (continue token expired)
                items = []
                continue
            items.extend(slim_pod(p) for p in page)
        return items, rv

    async def _get(self, ns: str, name: str):
        return slim_pod(await super()._get(ns, name))

    async def _watch(self, timeout_s: int):
        async for etype, obj in super()._watch(timeout_s):
            yield etype, (slim_pod(obj) if etype not in ("ERROR", "BOOKMARK") else obj)
