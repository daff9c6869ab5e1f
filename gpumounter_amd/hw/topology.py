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
from collections import OrderedDict
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


class _Scorer:
    """``score_set`` with the pairwise link costs and per-GPU keys computed once per call of
    :func:`choose` (the exhaustive search scores up to C(8,4)=70 sets, the attach ordering
    O(n²) prefixes; recomputing pair costs from the link matrix each time dominated)."""

    def __init__(self, gpus: Dict[int, AmdGpu], links: Optional[LinkMatrix]) -> None:
        ids = sorted(gpus)
        self.hive = {i: gpus[i].xgmi_hive_id for i in ids}
        self.numa = {i: gpus[i].numa_node for i in ids}
        self.pkg = {i: gpus[i].physical_id for i in ids}
        self.links = links
        self.pc: Dict[int, Dict[int, float]] = {}

    def _row(self, a: int) -> Dict[int, float]:
        row = self.pc.get(a)
        if row is None:
            row = self.pc[a] = {b: _pair_cost(self.links, a, b) for b in self.hive if b != a}
        return row

    def score(self, members: Sequence[int]) -> tuple:
        hives = {self.hive[i] for i in members if self.hive[i]}
        n_hives = max(len(hives), 1 if members else 0)
        numa = {self.numa[i] for i in members}
        packages = {self.pkg[i] for i in members}
        non_xgmi = 0
        pair = 0.0
        m = list(members)
        for k, a in enumerate(m):
            row = self._row(a)
            for b in m[k + 1:]:
                c = row[b]
                if c >= W_NON_XGMI:
                    non_xgmi += 1
                pair += c
        score = (W_HIVE * max(n_hives - 1, 0) + pair + W_NUMA * max(len(numa) - 1, 0)
                 + W_PACKAGE * max(len(packages) - 1, 0))
        return score, n_hives, len(numa), non_xgmi


def score_set(gpus: Dict[int, AmdGpu], links: Optional[LinkMatrix], members: Sequence[int]) -> tuple:
    """(score, hives, NUMA nodes, non-xGMI pairs) of a GPU set; lower score is better."""
    return _Scorer({i: gpus[i] for i in members}, links).score(members)


_CACHE: "OrderedDict[tuple, Optional[Placement]]" = OrderedDict()
_CACHE_MAX = 1024


def _gkey(gs: Iterable[AmdGpu]) -> tuple:
    return tuple(sorted((g.index, g.xgmi_hive_id, g.numa_node, g.physical_id) for g in gs))


def choose(candidates: Iterable[AmdGpu], n: int, links: Optional[LinkMatrix] = None,
           attached: Iterable[AmdGpu] = (), policy: str = "xgmi",
           prefer: Iterable[int] = ()) -> Optional[Placement]:
    """Pick ``n`` GPUs out of ``candidates`` that best extend ``attached``.

    Returns ``None`` if fewer than ``n`` candidates exist. ``policy="first-fit"`` reproduces the
    topology-blind behaviour (lowest indices first). Among equally scored sets the one with the
    most ``prefer`` indices wins (warm-pool GPUs: same placement quality, lower latency).
    The answer is a pure function of its inputs, and a node only ever sees a few hundred distinct
    (free set, n, attached set) questions, so answers are memoised (LRU).
    """
    cand = list(candidates)
    att = list(attached)
    pref = set(prefer)
    key = (_gkey(cand), n, _gkey(att), policy, tuple(sorted(pref)), _lkey(links))
    hit = _CACHE.get(key, _MISS)
    if hit is not _MISS:
        _CACHE.move_to_end(key)
        return None if hit is None else Placement(list(hit.chosen), hit.score, hit.hives,
                                                  hit.numa_nodes, hit.non_xgmi_pairs)
    res = _choose(cand, n, links, att, policy, pref)
    _CACHE[key] = res
    if len(_CACHE) > _CACHE_MAX:
        _CACHE.popitem(last=False)
    return None if res is None else Placement(list(res.chosen), res.score, res.hives,
                                              res.numa_nodes, res.non_xgmi_pairs)


_MISS = object()


def _lkey(links: Optional[LinkMatrix]) -> tuple:
    """Content key of a link matrix (the matrix is immutable once read from amdsmi)."""
    if links is None:
        return ()
    return (links.n, tuple(map(tuple, links.types)), tuple(map(tuple, links.hops)),
            tuple(map(tuple, links.weights)))


def _choose(candidates: List[AmdGpu], n: int, links: Optional[LinkMatrix],
            attached: List[AmdGpu], policy: str, pref: set) -> Optional[Placement]:
    cand = sorted({g.index: g for g in candidates}.values(), key=lambda g: g.index)
    att = sorted({g.index: g for g in attached}.values(), key=lambda g: g.index)
    if n <= 0:
        return Placement([], 0.0, 0, 0, 0)
    if len(cand) < n:
        return None
    table = {g.index: g for g in cand}
    table.update({g.index: g for g in att})
    sc = _Scorer(table, links)
    att_ids = [g.index for g in att]
    if policy == "first-fit":
        chosen = [g.index for g in cand[:n]]
        s, h, nn, nx = sc.score(att_ids + chosen)
        return Placement(chosen, s, h, nn, nx)

    ids = [g.index for g in cand]
    best = None
    if len(ids) == n:
        chosen = list(ids)
        s = sc.score(att_ids + chosen)
    elif math.comb(len(ids), n) <= EXHAUSTIVE_LIMIT:
        for combo in itertools.combinations(ids, n):
            s = sc.score(att_ids + list(combo))
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
                s = sc.score(att_ids + chosen + [i])
                key = (s[0], i not in pref, i)
                if pick is None or key < pick[0]:
                    pick = (key, i)
            chosen.append(pick[1])
        s = sc.score(att_ids + chosen)
    chosen = order_for_attach(table, links, att_ids, chosen, sc)
    return Placement(chosen, s[0], s[1], s[2], s[3])


def order_for_attach(gpus: Dict[int, AmdGpu], links: Optional[LinkMatrix], attached: List[int],
                     chosen: List[int], scorer: Optional[_Scorer] = None) -> List[int]:
    """Order a chosen set so each next GPU is the best-connected to everything before it."""
    sc = scorer or _Scorer(gpus, links)
    order: List[int] = []
    rest = list(chosen)
    base = list(attached)
    while rest:
        nxt = min(rest, key=lambda i: (sc.score(base + order + [i])[0], i))
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
