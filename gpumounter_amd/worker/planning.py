"""Where an attach's GPUs come from and which GPUs a removal names: pure functions of the
inventory, the ledger view and the policy, kept apart from the RPC service (worker/service.py).

* :func:`free_gpus` — GPUs free in the last ledger view, minus placeholders created since and
  GPUs out of placement (ECC, liveness).
* :func:`preferred` — the xGMI/NUMA-best ``n`` of them (hw/topology.py), as device IDs.
* :func:`plan_with_pool` — the same choice over warm-pool standby ∪ free GPUs: which standby
  placeholders to claim, which GPUs to create placeholders for. The pool saves latency; it does
  not decide placement.
* :func:`select_removal` — the reference's removal rule (allocator.go:101-126): only
  hot-mounted GPUs, an entire mount as a whole, any unknown id invalidates the request.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

from gpumounter_amd.hw import topology
from gpumounter_amd.models.device import AmdGpu, normalize_device_id
from gpumounter_amd.models.types import MountType


def free_gpus(inv, ph, unhealthy, st) -> List[AmdGpu]:
    """GPUs free in the last ledger view (minus placeholders we created since)."""
    allocated = {normalize_device_id(d) for ids in st.ledger.values() for d in ids}
    allocated.update(normalize_device_id(d) for uid, ids in ph.device_ids.items()
                     if uid not in ph.tombstones for d in ids)
    return [g for g in inv.gpus() if not allocated.intersection(g.ledger_keys())
            and g.index not in unhealthy]


def preferred(inv, policy: str, n: int, st, free: Sequence[AmdGpu]) -> List[str]:
    """xGMI/NUMA-aware preferred device IDs among ``free``. BDFs: the device plugin's own
    spelling of the ID is unknown here; BDF is what the ROCm plugin advertises, and the fake
    node honours any ledger key."""
    plc = topology.choose(list(free), n, inv.links(), attached=st.hot + st.own, policy=policy)
    if plc is None:
        return []
    by_index = {g.index: g for g in inv.gpus()}
    return [by_index[i].bdf for i in plc.chosen]


def plan_with_pool(inv, policy: str, standby_phs, n: int, st, free: Sequence[AmdGpu]
                   ) -> Optional[Tuple[List[int], List[str]]]:
    """Place over standby ∪ free GPUs together: (standby GPU indices to claim, device IDs to
    create placeholders for), or None when nothing fits."""
    keys = inv.by_key()
    standby: Dict[int, AmdGpu] = {}
    for ph in standby_phs:
        g = keys.get(normalize_device_id(ph.device_ids[0])) if ph.device_ids else None
        if g is not None:
            standby[g.index] = g
    cands = list(standby.values()) + [g for g in free if g.index not in standby]
    plc = topology.choose(cands, n, inv.links(), attached=st.hot + st.own, policy=policy,
                          prefer=standby)
    if plc is None:
        return None
    by_index = {g.index: g for g in cands}
    return ([i for i in plc.chosen if i in standby],
            [by_index[i].bdf for i in plc.chosen if i not in standby])


def select_removal(st, ids: List[str]) -> List[AmdGpu]:
    """Reference allocator.go:101-126: only hot-mounted GPUs are removable; entire mounts are
    removed as a whole; any unmatched id makes the whole request invalid (empty result)."""
    if not ids:
        return []
    want = {normalize_device_id(i) for i in ids}
    if len(want) != len(ids):
        return []
    if st.mount_type == MountType.ENTIRE:
        candidates = list(st.hot)
        matched = {k for g in candidates for k in g.ledger_keys()}
        if len(want) != len(candidates) or not want <= matched:
            return []
        return candidates
    selected = [g for g in st.hot if want.intersection(g.ledger_keys())]
    if len(selected) != len(want):
        return []
    return selected
