"""Fault injection for attach/detach stages (config ``fault`` / env ``GM_FAULT``).

Spec: ``stage:prob[:mode][,stage:prob[:mode]...]`` where ``stage`` is one of
``pod_lookup, ledger_read, ledger_reserve, placeholder_wait, cgroup_rule, devnodes, busy_check,
unmount, ledger_release`` (the span names of :mod:`gpumounter_amd.utils.trace`), ``prob`` in
[0, 1], and ``mode`` ``raise`` (default), ``after`` (fail *after* the stage's side effect, the
hard case for rollback) or ``exit`` (the process dies at once, before the stage, as under a
SIGKILL: exit status 137, nothing cleaned up). The reference has no such hooks; the
test suite uses them to prove every failure path restores a consistent ledger and leaves no
orphaned rules or nodes.
"""
from __future__ import annotations

import os
import random
import threading
from dataclasses import dataclass
from typing import Dict, Optional


class InjectedFault(RuntimeError):
    pass


@dataclass
class Rule:
    prob: float
    mode: str = "raise"
    hits: int = 0


class FaultInjector:
    def __init__(self, spec: str = "", seed: Optional[int] = None) -> None:
        self.rules: Dict[str, Rule] = {}
        self._rnd = random.Random(seed)
        self._lock = threading.Lock()
        for part in filter(None, (p.strip() for p in spec.split(","))):
            bits = part.split(":")
            if len(bits) < 2:
                raise ValueError(f"bad fault spec {part!r} (want stage:prob[:mode])")
            mode = bits[2] if len(bits) > 2 else "raise"
            if mode not in ("raise", "after", "exit"):
                raise ValueError(f"bad fault mode {mode!r}")
            self.rules[bits[0]] = Rule(float(bits[1]), mode)

    def __bool__(self) -> bool:
        return bool(self.rules)

    def check(self, stage: str, when: str = "raise") -> None:
        """Raise :class:`InjectedFault` if ``stage`` is armed for this phase (``raise`` = before
        the side effect, ``after`` = after it)."""
        r = self.rules.get(stage)
        if r is None or (r.mode != when and not (r.mode == "exit" and when == "raise")):
            return
        with self._lock:
            fire = self._rnd.random() < r.prob
            if fire:
                r.hits += 1
        if fire:
            if r.mode == "exit":
                os._exit(137)            # a SIGKILL at this point: no finally, no cleanup
            raise InjectedFault(f"injected fault at {stage} ({when})")


NONE = FaultInjector("")
