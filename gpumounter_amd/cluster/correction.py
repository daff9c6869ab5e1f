"""Placement correction: swap a worse-placed device-plugin choice for the best free set.

The reference takes whatever GPUs the device plugin hands its slave pods (reference:
pkg/util/gpu/allocator/allocator.go:40-99, no topology input at all). A stock AMD plugin never
sees gpumounter's preferred set either, so when the set it admitted scores worse (hive split ≫
non-xGMI pair ≫ NUMA split, hw/topology.py) than the best set the free GPUs allow, the worker
holds every other free GPU with a 1-GPU placeholder, keeps the best ``n`` and releases the rest.

This is the one place where placeholders are created, confirmed and deleted in several rounds
inside one attach, and every apiserver call in it can fail before or after taking effect (a
lost reply). It is therefore an explicit state machine over the placeholders it touches, each in
exactly one :class:`Book` state::

    ADMITTED ──let go──▶ RELEASING ──ack──▶ RELEASED
       │                    (no ack: may or may not exist; never kept, handed to the follow-up)
       └──confirm──▶ KEPT
    HELD ─────confirm──▶ KEPT          HELD / ADMITTED / RELEASING left at the end ▶ released

and :meth:`Correction.settle` derives the outcome from the states alone:

* every GPU of the returned reservation is booked by a placeholder in ``KEPT`` (a confirmed pick)
  or, when the correction gives up, by the untouched ``ADMITTED`` one (the plugin's own choice,
  only if no DELETE was ever sent for it);
* every other placeholder it created or let go is released, or — if that fails — handed to the
  reconciler's follow-up, which deletes it when it still exists (worker/reconciler.py).

Both properties are checked by ``tests/test_correction.py`` against a fake whose every POST,
PATCH and DELETE can fail before or after taking effect.
"""
from __future__ import annotations

import asyncio
import contextlib
import enum
from typing import Callable, List, Optional, Sequence

from gpumounter_amd.cluster.placeholder import (InsufficientGPU, Placeholder, Reservation,
                                                ReserveError)
from gpumounter_amd.cluster.quota import QuotaExceeded
from gpumounter_amd.hw import topology
from gpumounter_amd.models.device import AmdGpu, normalize_device_id
from gpumounter_amd.utils import log, trace
from gpumounter_amd.utils.faults import InjectedFault

_log = log.get("cluster.correction")

# failures after which the correction gives up (keeping the plugin's choice when it can)
GIVE_UP = (ReserveError, InsufficientGPU, QuotaExceeded, asyncio.TimeoutError, InjectedFault)


class ReserveGate:
    """Reservations on one node: ordinary ones run concurrently (shared); the ones that hold
    every free GPU for a moment (trim, placement correction) and device-plugin intents, which
    carry no pod identity, run alone (exclusive)."""

    def __init__(self) -> None:
        self._cond = asyncio.Condition()
        self._shared = 0
        self._exclusive = False
        self._waiting_exclusive = 0

    @contextlib.asynccontextmanager
    async def shared(self):
        async with self._cond:
            if self._exclusive or self._waiting_exclusive:
                with trace.span("reserve_gate_wait"):
                    await self._cond.wait_for(lambda: not self._exclusive and
                                              not self._waiting_exclusive)
            self._shared += 1
        try:
            yield
        finally:
            async with self._cond:
                self._shared -= 1
                self._cond.notify_all()

    @contextlib.asynccontextmanager
    async def exclusive(self):
        async with self._cond:
            self._waiting_exclusive += 1
            try:
                if self._exclusive or self._shared:
                    with trace.span("reserve_gate_wait"):
                        await self._cond.wait_for(lambda: not self._exclusive and
                                                  not self._shared)
            finally:
                self._waiting_exclusive -= 1
            self._exclusive = True
        try:
            yield
        finally:
            async with self._cond:
                self._exclusive = False
                self._cond.notify_all()


def placement_worse(inv, attached: Sequence[AmdGpu], got: Sequence[str],
                    want: Sequence[str], on: str = "numa") -> bool:
    """The admitted set ``got`` scores worse together with the pod's ``attached`` GPUs than the
    preferred set ``want`` would have; ``on="xgmi"``: worse by at least a non-xGMI pair or a
    hive split (a NUMA split alone does not count)."""
    if not want or len(want) != len(got):
        return False
    keys = inv.by_key()
    try:
        g = [keys[normalize_device_id(d)].index for d in got]
        w = [keys[normalize_device_id(d)].index for d in want]
    except KeyError:
        return False
    if sorted(g) == sorted(w):
        return False
    table = {x.index: x for x in inv.gpus()}
    att = [x.index for x in attached]
    links = inv.links()
    margin = topology.W_NON_XGMI - 1e-6 if on == "xgmi" else 1e-6
    return topology.score_set(table, links, att + g)[0] > \
        topology.score_set(table, links, att + w)[0] + margin


class Book(enum.Enum):
    ADMITTED = "admitted"     # the plugin's choice: a complete, valid reservation on its own
    HELD = "held"             # an extra 1-GPU candidate, held for the pick
    RELEASING = "releasing"   # DELETE sent, not acknowledged: may or may not still exist
    RELEASED = "released"     # DELETE acknowledged: gone from the scheduler's books
    KEPT = "kept"             # picked and confirmed: part of the reservation returned


class Correction:
    """One correction of one attach (runs under the node's exclusive reserve gate and the
    pod's lock). ``ph`` is the PlaceholderManager; ``release_quiet(phs)`` releases leftovers,
    handing what it cannot delete to the reconciler's follow-up."""

    # second round: how long to wait for the released placeholders' DELETED echo, then the
    # re-hold attempts while the scheduler and the kubelet catch up (a real cluster's kubelet
    # frees the devices when it has seen the deletion, tens to hundreds of ms later)
    ECHO_WAIT_S = 1.0
    REHOLD_DELAYS_S = (0.0, 0.05, 0.2, 0.5, 1.0)

    def __init__(self, ph, inv, free: Sequence[AmdGpu], attached: Sequence[AmdGpu], owner: dict,
                 n: int, entire: bool, group: str, attach_id: str, container: str,
                 idempotency_key: str, policy: str, faults,
                 release_quiet: Callable[[Sequence[Placeholder]], "asyncio.Future"],
                 lease_expires: float = 0.0) -> None:
        self.ph, self.inv, self.faults = ph, inv, faults
        self.free, self.attached, self.owner = list(free), list(attached), owner
        self.n, self.entire, self.group = n, entire, group
        self.attach_id, self.container, self.key = attach_id, container, idempotency_key
        self.policy = policy
        self.lease_expires = lease_expires      # the attach's lease, on every hold it makes
        self.release_quiet = release_quiet
        self.entries: List[List] = []            # [placeholder, Book]
        self.corrected = False
        self.error: Optional[BaseException] = None  # why the correction gave up, if it did
        self._keys = inv.by_key()
        self._links = inv.links()
        self._table = {g.index: g for g in inv.gpus()}

    # ------------------------------------------------------------------------ book keeping
    def _add(self, phs: Sequence[Placeholder], state: Book) -> None:
        for p in phs:
            self.entries.append([p, state])

    def _set(self, phs: Sequence[Placeholder], state: Book) -> None:
        ids = {id(p) for p in phs}
        for e in self.entries:
            if id(e[0]) in ids:
                e[1] = state

    def of(self, *states: Book) -> List[Placeholder]:
        return [p for p, s in self.entries if s in states]

    @staticmethod
    def _gpus(phs: Sequence[Placeholder]) -> int:
        return sum(len(p.device_ids) for p in phs)

    # ------------------------------------------------------------------------ scoring
    def best_of(self, ids: Sequence[str], fallback: Sequence[str]) -> List[str]:
        by = {self._keys[normalize_device_id(d)].index: d for d in ids
              if normalize_device_id(d) in self._keys}
        plc = topology.choose([self._table[i] for i in by], self.n, self._links,
                              attached=self.attached, policy=self.policy) \
            if len(by) >= self.n else None
        return [by[i] for i in plc.chosen] if plc else list(fallback)

    def score(self, ids: Sequence[str]) -> float:
        return topology.score_set(self._table, self._links,
                                  [g.index for g in self.attached] +
                                  [self._keys[normalize_device_id(d)].index for d in ids])[0]

    # ------------------------------------------------------------------------ transitions
    async def _hold(self, width: int) -> List[Placeholder]:
        got = await self.ph.hold_singles(self.owner, width, self.entire, self.group,
                                         self.attach_id, self.container, self.key,
                                         self.lease_expires)
        self._add(got, Book.HELD)
        return got

    async def _let_go(self, phs: Sequence[Placeholder]) -> None:
        # RELEASING before the DELETE is sent: one that takes effect and then fails (a lost
        # reply) must never be counted as a kept reservation again
        self._set(phs, Book.RELEASING)
        await self.ph.release(list(phs))
        self._set(phs, Book.RELEASED)

    async def _observed_gone(self, phs: Sequence[Placeholder]) -> None:
        """Wait (at most ``ECHO_WAIT_S``) until the watch has delivered the DELETED events of
        ``phs``: the scheduler and the kubelet act on the same deletion, so a re-hold sent
        before the echo mostly finds the GPUs still booked. The apiserver answered the DELETEs
        already; the echo only paces the second round."""
        uids = {p.uid for p in phs if p.uid}
        informer = getattr(self.ph, "informer", None)
        if not uids or informer is None:
            return
        try:
            await informer.wait_for(
                lambda: not uids & set(getattr(self.ph, "tombstones", ())), self.ECHO_WAIT_S)
        except asyncio.TimeoutError:
            _log.info("correction: DELETED echo of %d placeholder(s) not seen within %.1fs",
                      len(uids), self.ECHO_WAIT_S)

    async def _keep(self, phs: Sequence[Placeholder]) -> None:
        await self.ph.confirm(phs)        # clears the candidate mark of the HELD ones
        self._set(phs, Book.KEPT)

    # ------------------------------------------------------------------------ run
    async def run(self, res: Reservation) -> Reservation:
        mine = {normalize_device_id(d) for d in res.device_ids}
        free = [g for g in self.free if not mine.intersection(g.ledger_keys())]
        if not free:
            return res
        self._add(res.placeholders, Book.ADMITTED)
        error: Optional[BaseException] = None
        try:
            with trace.span("placement_correct", held=len(free)):
                self.faults.check("placement_correct")
                await self._hold(len(free))
                pick = self._choose(res)
                if pick is None:
                    # the best set needs part of the admitted n-GPU placeholder, which can only be
                    # kept whole: a second round takes its GPUs back as 1-GPU placeholders
                    let_go = self.of(Book.ADMITTED)
                    await self._let_go(let_go)
                    await self._observed_gone(let_go)
                    want_n, got = len(mine), 0
                    for delay in self.REHOLD_DELAYS_S:   # while the kubelet frees them
                        if delay:
                            await asyncio.sleep(delay)
                        got += len(await self._hold(want_n - got))
                        if got >= want_n:
                            break
                    pick = lambda ids: self.best_of(ids, res.device_ids)   # noqa: E731
                new, _ = self.ph.keep_picked(self.of(Book.ADMITTED, Book.HELD), self.n, pick)
                self.faults.check("placement_correct", "after")
                if self._gpus(new.placeholders) == self.n:
                    await self._keep(new.placeholders)
        except GIVE_UP as e:
            error = e
        return await self.settle(res, error)

    def _choose(self, res: Reservation) -> Optional[Callable[[List[str]], Sequence[str]]]:
        """The pick over ADMITTED ∪ HELD, or None when it needs a second round."""
        pick = lambda ids: self.best_of(ids, res.device_ids)   # noqa: E731
        if not self.entire:
            return pick
        mine = {normalize_device_id(d) for d in res.device_ids}
        best = self.best_of([d for p in self.of(Book.ADMITTED, Book.HELD)
                             for d in p.device_ids], res.device_ids)
        want = {normalize_device_id(d) for d in best}
        if not (want & mine) or mine <= want:
            return pick
        new_ids = [d for p in self.of(Book.HELD) for d in p.device_ids]
        alt = self.best_of(new_ids, ()) if len(new_ids) >= self.n else []
        if alt and self.score(alt) <= self.score(best) + 1e-6:
            return lambda ids: alt                 # as good from the new ones alone
        return None

    async def settle(self, res: Reservation, error: Optional[BaseException]) -> Reservation:
        """The outcome, from the book states alone."""
        self.error = error
        kept = self.of(Book.KEPT)
        if error is None and self._gpus(kept) == self.n:
            out, self.corrected = Reservation(kept), True
        elif all(s is Book.ADMITTED or s is Book.KEPT
                 for p, s in self.entries if any(p is q for q in res.placeholders)):
            # no DELETE was ever sent for the plugin's choice: it is still a valid reservation
            if error is not None:
                _log.warning("placement correction failed, keeping the plugin's choice: %s",
                             error)
            out = res
        else:
            out = None
        keep_ids = {id(p) for p in out.placeholders} if out is not None else set()
        booked = {id(p) for p, s in self.entries if s in (Book.KEPT, Book.ADMITTED)}
        if not keep_ids <= booked:      # never reached: the guard of the invariant above
            raise ReserveError("placement correction would mount an unbooked placeholder")
        leftovers = [p for p, s in self.entries
                     if id(p) not in keep_ids and s is not Book.RELEASED]
        if leftovers:
            with trace.span("placement_release", placeholders=len(leftovers)):
                await self.release_quiet(leftovers)
        if out is None:
            if error is not None:
                raise error
            raise InsufficientGPU(f"placement correction could not hold {self.n} GPUs")
        if self.corrected:
            out.preferred = out.device_ids
        return out

