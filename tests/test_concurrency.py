"""Concurrency and ledger invariants (BASELINE config "4 Pods contending for 8 MI355X"; the
reference had no locks at all — SURVEY §2.6 defect 7).

Invariants checked after every operation:
  I1  no device ID is held by two pods in the kubelet ledger;
  I2  every hot-mounted GPU of a pod is backed by exactly one live placeholder of that pod;
  I3  cgroup rules + /dev nodes of every tenant equal its ledger view (audit is empty);
  I4  free + held == capacity.
"""
import asyncio
import random

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gpumounter_amd.fakes.harness import LocalCluster


async def check_invariants(lc, tenants):
    node = lc.nodes["node-0"].node
    held = list(node.allocated)
    assert len(held) == len(set(held))                                   # I1
    svc = lc.nodes["node-0"].worker.service
    total_hot = 0
    for t in tenants:
        pod = lc.cluster.get("default", t)
        st_ = await svc.pod_state(pod)
        total_hot += len(st_.hot)
        for ph in st_.placeholders:                                        # I2
            assert lc.cluster.get(ph.namespace, ph.name) is not None
        assert not svc.hm.audit(pod, st_.hot, st_.own), t                 # I3
    assert len(node.free_ids()) + len(node.allocated) == node.capacity   # I4
    # warm-pool capacity: GPUs held by standby placeholders (a standby the refill created while
    # concurrent attaches filled the node is Pending and holds nothing)
    standby_names = {p["metadata"]["name"] for p in lc.cluster.placeholders()
                     if (p["metadata"].get("annotations") or {}).get(
                         "gpumounter.amd.com/mount-mode") == "standby"
                     and not p["metadata"].get("deletionTimestamp")}
    standby = sum(1 for _, pod, _ in node.allocated.values() if pod in standby_names)
    assert total_hot + standby == len(node.allocated)


def test_four_pods_contending_for_eight_gpus():
    async def main():
        async with LocalCluster() as lc:
            tenants = [f"t{i}" for i in range(4)]
            for t in tenants:
                lc.tenant(t)
            # 4 pods ask for 3 GPUs each at once: 12 > 8, so some must fail cleanly
            res = await asyncio.gather(*[lc.add("default", t, 3) for t in tenants])
            codes = [c for c, _ in res]
            assert codes.count(200) == 2 and set(codes) == {200, 500}  # 3+3 fit, 12 do not
            await asyncio.sleep(0.05)
            await check_invariants(lc, tenants)
            # the losers can still get the 2 leftover GPUs
            losers = [t for t, (c, _) in zip(tenants, res) if c != 200]
            c1, _ = await lc.add("default", losers[0], 2)
            assert c1 == 200
            await check_invariants(lc, tenants)
            # concurrent adds to the SAME pod serialize (per-pod lock) and never double-mount
            for t, (c, b) in zip(tenants, res):
                if c == 200:
                    await lc.remove("default", t, [d["uuid"] for d in b["devices"]])
            same = await asyncio.gather(*[lc.add("default", "t3", 1) for _ in range(6)])
            assert all(c == 200 for c, _ in same)
            await check_invariants(lc, tenants)
    asyncio.run(main())


ops = st.lists(st.tuples(st.sampled_from(["add", "add_entire", "remove", "remove_force"]),
                         st.integers(0, 3), st.integers(1, 4)), min_size=4, max_size=14)


@settings(max_examples=12, deadline=None, suppress_health_check=list(HealthCheck))
@given(ops, st.integers(0, 2 ** 16))
def test_random_operation_sequences_keep_ledger_consistent(seq, seed):
    rnd = random.Random(seed)

    async def main():
        async with LocalCluster() as lc:
            tenants = [f"p{i}" for i in range(4)]
            for t in tenants:
                lc.tenant(t)
            svc = lc.nodes["node-0"].worker.service
            for op, ti, n in seq:
                t = tenants[ti]
                if op.startswith("add"):
                    code, _ = await lc.add("default", t, n, entire=op == "add_entire")
                    assert code in (200, 500)
                else:
                    st_ = await svc.pod_state(lc.cluster.get("default", t))
                    if not st_.hot:
                        continue
                    if st_.mount_type.value == "entire-mount":
                        ids = [g.uuid for g in st_.hot]
                    else:
                        ids = [g.uuid for g in rnd.sample(st_.hot, min(n, len(st_.hot)))]
                    code, _ = await lc.remove("default", t, ids, force=op == "remove_force")
                    assert code == 200
                await asyncio.sleep(0.01)
                await check_invariants(lc, tenants)
    asyncio.run(main())


def test_1000_attach_detach_cycles_leave_no_orphans():
    """BASELINE config: 1000 cycles across 8 GPUs, zero orphaned cgroup entries / nodes."""
    async def main():
        async with LocalCluster() as lc:
            for i in range(2):
                lc.tenant(f"c{i}")
            lat = []
            for k in range(1000):
                t = f"c{k % 2}"
                n = (k % 4) + 1
                code, b = await lc.add("default", t, n, entire=bool(k % 3 == 0))
                assert code == 200, b
                lat.append(b["total_ms"])
                code, _ = await lc.remove("default", t, [d["uuid"] for d in b["devices"]])
                assert code == 200
            await check_invariants(lc, ["c0", "c1"])
            node = lc.nodes["node-0"].node
            for cid in lc.container_ids("default", "c0") + lc.container_ids("default", "c1"):
                assert node.container_devices(cid) == []
            assert lc.cluster.placeholders() == []
            lat.sort()
            assert lat[int(0.99 * len(lat))] < 1000   # generous bound on the CPU sandbox
    asyncio.run(main())


import pytest  # noqa: E402


@pytest.mark.parametrize("mode", ["auto", "auto_random", "trim", "device_plugin", "warm_pool"])
def test_contention_under_each_placement_mode(mode):
    """The 4-pods-for-8-GPUs contract holds whatever enforces the placement."""
    kw = {"auto": dict(alloc_policy="first-free"),
          "auto_random": dict(alloc_policy="random"),
          "trim": dict(alloc_policy="first-free", worker_overrides={"placement_enforce": "trim"}),
          "device_plugin": dict(device_plugin=True),
          "warm_pool": dict(worker_overrides={"warm_pool_size": 4})}[mode]

    async def main():
        async with LocalCluster(**kw) as lc:
            tenants = [f"t{i}" for i in range(4)]
            for t in tenants:
                lc.tenant(t)
            if mode == "warm_pool":
                pool = lc.nodes["node-0"].worker.pool
                for _ in range(500):
                    if len(pool.standby()) >= 4:
                        break
                    await asyncio.sleep(0.01)
            res = await asyncio.gather(*[lc.add("default", t, 3) for t in tenants])
            codes = [c for c, _ in res]
            assert codes.count(200) == 2 and set(codes) == {200, 500}, codes
            await asyncio.sleep(0.05)
            await check_invariants(lc, tenants)
            for t, (c, b) in zip(tenants, res):
                if c == 200:
                    assert len({d["numa_node"] for d in b["devices"]}) == 1, b["devices"]
                    assert (await lc.remove("default", t, [d["uuid"] for d in b["devices"]]))[0] \
                        == 200
            await asyncio.sleep(0.05)
            await check_invariants(lc, tenants)
    asyncio.run(main())
