"""Injected failures at every attach/detach stage (before and after the stage's side effect) never
leave orphaned cgroup rules, device nodes or placeholders: each request either fully happens or
leaves the pod exactly as the ledger describes it (reference defect 12)."""
import asyncio

import pytest

from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.utils.faults import FaultInjector, InjectedFault, Rule

ATTACH_STAGES = ["pod_lookup", "ledger_read", "ledger_reserve", "placeholder_wait",
                 "cgroup_rule", "devnodes"]
DETACH_STAGES = ["pod_lookup", "busy_check", "unmount", "ledger_release"]


def test_fault_spec_parsing():
    f = FaultInjector("devnodes:1,ledger_release:0.5:after", seed=1)
    assert f.rules["devnodes"].mode == "raise" and f.rules["ledger_release"].prob == 0.5
    with pytest.raises(InjectedFault):
        f.check("devnodes")
    f.check("devnodes", "after")       # armed only for "raise"
    f.check("unknown")
    with pytest.raises(ValueError):
        FaultInjector("devnodes")
    with pytest.raises(ValueError):
        FaultInjector("devnodes:1:sometimes")


async def _consistent(lc, pod, only_tenant=True):
    await asyncio.sleep(0.05)
    assert not await lc.audit("default", pod)
    svc = lc.nodes["node-0"].worker.service
    st = await svc.pod_state(lc.cluster.get("default", pod), fresh=True)
    node = lc.nodes["node-0"].node
    if only_tenant:
        assert len(st.hot) == len(node.allocated)   # every held GPU is this pod's hot mount
    return st


@pytest.mark.parametrize("stage", ATTACH_STAGES)
@pytest.mark.parametrize("mode", ["raise", "after"])
def test_attach_fault_leaves_consistent_state(stage, mode):
    async def main():
        async with LocalCluster() as lc:
            lc.tenant("f")
            w = lc.nodes["node-0"].worker
            _, b0 = await lc.add("default", "f", 1)       # pre-existing hot GPU must survive
            w.faults.rules = {stage: Rule(1.0, mode)}
            code, body = await lc.add("default", "f", 2)
            w.faults.rules = {}
            if stage in ("ledger_read", "pod_lookup") and mode == "after":
                assert code == 200      # read-only stages have no side effect to fail after
            else:
                assert code == 500, body
            st = await _consistent(lc, "f")
            held = {g.uuid for g in st.hot}
            assert b0["devices"][0]["uuid"] in held
            code, _ = await lc.add("default", "f", 1)     # and the node keeps working
            assert code == 200
            await _consistent(lc, "f")
    asyncio.run(main())


@pytest.mark.parametrize("stage", DETACH_STAGES)
@pytest.mark.parametrize("mode", ["raise", "after"])
def test_detach_fault_leaves_consistent_state(stage, mode):
    async def main():
        async with LocalCluster() as lc:
            lc.tenant("d")
            w = lc.nodes["node-0"].worker
            _, b = await lc.add("default", "d", 2)
            ids = [d["uuid"] for d in b["devices"]]
            w.faults.rules = {stage: Rule(1.0, mode)}
            code, body = await lc.remove("default", "d", ids[:1])
            w.faults.rules = {}
            st = await _consistent(lc, "d")
            held = {g.uuid for g in st.hot}
            if code == 200:
                assert held == {ids[1]}
            else:
                # failure before the ledger release: still attached; after it: detached
                assert held in ({ids[0], ids[1]}, {ids[1]})
            code, _ = await lc.remove("default", "d", sorted(held))
            assert code == 200
            st = await _consistent(lc, "d")
            assert st.hot == [] and lc.cluster.placeholders() == []
    asyncio.run(main())


def test_random_fault_storm_then_reconcile():
    async def main():
        async with LocalCluster() as lc:
            for t in ("a", "b"):
                lc.tenant(t)
            w = lc.nodes["node-0"].worker
            w.faults = FaultInjector(",".join(f"{s}:0.15" for s in ATTACH_STAGES + DETACH_STAGES)
                                     + ",devnodes:0.1:after,ledger_release:0.1:after", seed=7)
            w.service.faults = w.hotmount.faults = w.placeholders.faults = w.faults
            for k in range(60):
                t = "ab"[k % 2]
                code, b = await lc.add("default", t, 1 + k % 3)
                if code == 200:
                    await lc.remove("default", t, [d["uuid"] for d in b["devices"]])
            w.faults.rules = {}
            await w.reconciler.run_once()
            held = 0
            for t in ("a", "b"):
                st = await _consistent(lc, t, only_tenant=False)
                held += len(st.hot)
            assert held == len(lc.nodes["node-0"].node.allocated)  # no leaked reservation
            for t in ("a", "b"):
                st = await _consistent(lc, t, only_tenant=False)
                if st.hot:
                    ids = [g.uuid for g in st.hot]
                    assert (await lc.remove("default", t, ids))[0] == 200
            await asyncio.sleep(0.05)
            assert lc.cluster.placeholders() == [] and lc.nodes["node-0"].node.allocated == {}
            assert sum(r.hits for r in w.faults.rules.values()) == 0
    asyncio.run(main())


@pytest.mark.parametrize("mode", ["raise", "after"])
def test_placement_correction_fault_keeps_a_valid_attach(mode):
    """A failure inside the placement correction (before it holds anything, or after its pick)
    leaves the attach with the plugin's valid, worse-placed choice and nothing else held."""
    async def main():
        async with LocalCluster(alloc_policy="first-free") as lc:
            lc.tenant("other")
            lc.tenant("t")
            assert (await lc.add("default", "other", 3))[0] == 200
            w = lc.nodes["node-0"].worker
            w.faults.rules = {"placement_correct": Rule(1.0, mode)}
            code, b = await lc.add("default", "t", 2)
            w.faults.rules = {}
            assert code == 200, b
            assert sorted(d["index"] for d in b["devices"]) == [3, 4]
            await asyncio.sleep(0.05)
            assert len(lc.nodes["node-0"].node.allocated) == 5
            await _consistent(lc, "t", only_tenant=False)
    asyncio.run(main())


def test_failed_rpcs_are_counted_by_grpc_status():
    """gm_requests_total counts failures too (deploy/monitoring alerts on INTERNAL): a rolled-back
    attach under its status name, next to the reference's result enum for answered ones."""
    async def main():
        async with LocalCluster() as lc:
            lc.tenant("f")
            w = lc.nodes["node-0"].worker
            w.faults.rules = {"devnodes": Rule(1.0, "raise")}
            code, _ = await lc.add("default", "f", 1)
            w.faults.rules = {}
            assert code == 500
            code, b = await lc.add("default", "f", 1)
            assert code == 200
            m = w.service.metrics.requests
            assert m.labels(op="add", result="INTERNAL")._value.get() == 1
            assert m.labels(op="add", result="Success")._value.get() == 1
    asyncio.run(main())
