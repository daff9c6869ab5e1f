"""xGMI-hive / NUMA / partition-aware GPU placement.

The reference has no topology awareness: a slave pod gets whatever the device plugin hands out
(reference: pkg/util/gpu/allocator/allocator.go:214-231). On an 8×MI355X node every
GPU has 7 point-to-point xGMI links (≈153 GB/s each) into one hive, so any subset is directly
linked — but a tenant that later runs RCCL still cares about (a) staying inside one hive when the
node has several, (b) not crossing the CPU socket (NUMA) for host staging, and (c) in CPX/NPS
partition modes, keeping logical GPUs of one OAM package together. This module scores candidate
sets on exactly those terms, in that priority, and picks the best one deterministically.

The same policy backs (1) the worker's preferred-device hint on placeholder pods, (2) the attach
order when a pod is grown one GPU at a time (the next GPU is the one best connected to what the
pod already has), and (3) the hermetic fake device plugin's ``GetPreferredAllocation``.
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence

from gpumounter_amd.models.device import AmdGpu, LinkMatrix

# Penalty weights, strictly ordered: hive split ≫ non-xGMI pair ≫ NUMA split ≫ package split.
W_HIVE = 1_000_000
W_NON_XGMI = 10_000
W_NUMA = 100
W_PACKAGE = 10
EXHAUSTIVE_LIMIT = 20_000


@dataclass
class Placement:
    chosen: List[int]          # GPU indices in attach order
    score: float
    hives: int
    numa_nodes: int
    non_xgmi_pairs: int

    def to_dict(self) -> Dict:
        return {"chosen": self.chosen, "score": self.score, "hives": self.hives,
                "numa_nodes": self.numa_nodes, "non_xgmi_pairs": self.non_xgmi_pairs}


def _pair_cost(links: Optional[LinkMatrix], a: int, b: int) -> float:
    if links is None or not links.types:
        return 0.0
    t = links.types[a][b]
    if t == LinkMatrix.XGMI:
        # among xGMI pairs prefer the lower amdsmi weight / fewer hops (1 on a full mesh)
        return links.hops[a][b] + links.weights[a][b] * 1e-3
    return W_NON_XGMI + links.weights[a][b] + 10 * links.hops[a][b]


def score_set(gpus: Dict[int, AmdGpu], links: Optional[LinkMatrix], members: Sequence[int]) -> tuple:
    hives = {gpus[i].xgmi_hive_id for i in members if gpus[i].xgmi_hive_id}
    n_hives = max(len(hives), 1 if members else 0)
    numa = {gpus[i].numa_node for i in members}
    packages = {gpus[i].physical_id for i in members}
    non_xgmi = 0
    pair = 0.0
    for a, b in itertools.combinations(members, 2):
        c = _pair_cost(links, a, b)
        if c >= W_NON_XGMI:
            non_xgmi += 1
        pair += c
    score = (W_HIVE * max(n_hives - 1, 0) + pair + W_NUMA * max(len(numa) - 1, 0)
             + W_PACKAGE * max(len(packages) - 1, 0))
    return score, n_hives, len(numa), non_xgmi


def choose(candidates: Iterable[AmdGpu], n: int, links: Optional[LinkMatrix] = None,
           attached: Iterable[AmdGpu] = (), policy: str = "xgmi",
           prefer: Iterable[int] = ()) -> Optional[Placement]:
    """Pick ``n`` GPUs out of ``candidates`` that best extend ``attached``.

    Returns ``None`` if fewer than ``n`` candidates exist. ``policy="first-fit"`` reproduces the
    topology-blind behaviour (lowest indices first). Among equally scored sets the one with the
    most ``prefer`` indices wins (warm-pool GPUs: same placement quality, lower latency).
    """
    pref = set(prefer)
    cand = sorted({g.index: g for g in candidates}.values(), key=lambda g: g.index)
    att = sorted({g.index: g for g in attached}.values(), key=lambda g: g.index)
    if n <= 0:
        return Placement([], 0.0, 0, 0, 0)
    if len(cand) < n:
        return None
    table = {g.index: g for g in cand}
    table.update({g.index: g for g in att})
    att_ids = [g.index for g in att]
    if policy == "first-fit":
        chosen = [g.index for g in cand[:n]]
        s, h, nn, nx = score_set(table, links, att_ids + chosen)
        return Placement(chosen, s, h, nn, nx)

    ids = [g.index for g in cand]
    best = None
    if math.comb(len(ids), n) <= EXHAUSTIVE_LIMIT:
        for combo in itertools.combinations(ids, n):
            s = score_set(table, links, att_ids + list(combo))
            key = (s[0], -len(pref.intersection(combo)), combo)
            if best is None or key < best[0]:
                best = (key, list(combo), s)
        chosen, s = best[1], best[2]
    else:
        # greedy growth from the best-connected seed; O(n · |cand|²)
        chosen = []
        for _ in range(n):
            pick = None
            for i in ids:
                if i in chosen:
                    continue
                s = score_set(table, links, att_ids + chosen + [i])
                key = (s[0], i not in pref, i)
                if pick is None or key < pick[0]:
                    pick = (key, i)
            chosen.append(pick[1])
        s = score_set(table, links, att_ids + chosen)
    chosen = order_for_attach(table, links, att_ids, chosen)
    return Placement(chosen, s[0], s[1], s[2], s[3])


def order_for_attach(gpus: Dict[int, AmdGpu], links: Optional[LinkMatrix], attached: List[int],
                     chosen: List[int]) -> List[int]:
    """Order a chosen set so each next GPU is the best-connected to everything before it."""
    order: List[int] = []
    rest = list(chosen)
    base = list(attached)
    while rest:
        nxt = min(rest, key=lambda i: (score_set(gpus, links, base + order + [i])[0], i))
        order.append(nxt)
        rest.remove(nxt)
    return order


def describe(gpus: Sequence[AmdGpu], links: Optional[LinkMatrix]) -> Dict:
    """Human-readable topology summary (hives, NUMA split, all-pairs xGMI check)."""
    table = {g.index: g for g in gpus}
    ids = sorted(table)
    s, h, nn, nx = score_set(table, links, ids)
    hives: Dict[str, List[int]] = {}
    for g in gpus:
        hives.setdefault(hex(g.xgmi_hive_id), []).append(g.index)
    return {"gpus": ids, "hives": hives, "numa_nodes": nn, "non_xgmi_pairs": nx,
            "all_pairs_xgmi": nx == 0 and len(ids) > 1}
