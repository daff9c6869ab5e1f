"""Ownership bookkeeping edge cases.

The reference only ever revokes what its ledger selects for the pod it was asked about
(reference: pkg/util/util.go:73-147): a node the container already had is never removed, and a
GPU still used by any process of the container — privileged or not — makes it busy
(util.go:152-196). The journal (node/journal.py) must keep to that across crashes, partial
kernel calls, upgrades and foreign BPF programs."""
import asyncio
import os
import subprocess

import pytest

from gpumounter_amd import _native
from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.models import pod as podu
from gpumounter_amd.node.hotmount import HotMount
from gpumounter_amd.node.journal import InjectionJournal


def run(coro_fn, **kw):
    async def main():
        async with LocalCluster(**kw) as lc:
            return await coro_fn(lc)
    return asyncio.run(main())


def node_of(lc):
    return lc.nodes["node-0"].node


def _marker(path, ma, mi):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        fh.write(f"gm-chr {ma}:{mi}\n")


class _Crash(BaseException):
    """A SIGKILL stand-in: nothing after it runs (no except-Exception rollback)."""


# ------------------------------------------------------------------------------ write-ahead
def test_crash_between_intent_and_create_never_journals_a_preexisting_node(monkeypatch):
    """Worker killed after the write-ahead record and before the create, with the GPU's render
    node already in the tenant's rootfs: after a restart the pre-existing node is not
    gpumounter's, so neither the orphan sweep nor a detach unlinks it."""
    async def body(lc):
        lc.tenant("t")
        cid = lc.container_ids("default", "t")[0]
        root = node_of(lc).container(cid).root_dir
        w = lc.nodes["node-0"].worker
        g = lc.inventory.gpus()[0]
        pre = os.path.join(root, f"dev/dri/renderD{g.render_minor}")
        _marker(pre, 226, g.render_minor)
        pod = lc.cluster.get("default", "t")

        def crash(*a, **k):
            raise _Crash()
        monkeypatch.setattr(w.service.hm.writer, "create", crash)
        with pytest.raises(_Crash):
            w.service.hm.attach(pod, [g], [], [])
        monkeypatch.undo()
        # what a restarted worker reads from the node's state dir
        j = InjectionJournal(os.path.join(node_of(lc).state_dir, "journal"))
        nodes = j.nodes_of(cid)
        assert (226, g.render_minor) not in nodes, nodes
        assert (226, g.card_minor) in nodes and (lc.inventory.kfd_major, 0) in nodes
        await lc.stop_worker("node-0")
        w2 = await lc.start_worker("node-0")
        rep = await w2.reconciler.run_once()        # no placeholder backs it: orphan sweep
        assert rep.revoked == ["default/t"], rep
        assert os.path.exists(pre)                  # the container's own node stays
        assert (226, g.render_minor) not in w2.journal.nodes_of(cid)
    run(body, worker_overrides={"reconcile_on_events": False})


def test_attach_with_preexisting_node_then_detach_keeps_it():
    async def body(lc):
        lc.tenant("t")
        cid = lc.container_ids("default", "t")[0]
        root = node_of(lc).container(cid).root_dir
        g = lc.inventory.gpus()[0]
        pre = os.path.join(root, f"dev/dri/renderD{g.render_minor}")
        _marker(pre, 226, g.render_minor)
        code, b = await lc.add("default", "t", 1)
        assert code == 200 and b["devices"][0]["index"] == g.index
        assert (226, g.render_minor) not in lc.nodes["node-0"].worker.journal.nodes_of(cid)
        code, _ = await lc.remove("default", "t", [b["devices"][0]["uuid"]])
        assert code == 200 and os.path.exists(pre)
        assert not os.path.exists(os.path.join(root, f"dev/dri/card{g.card_minor}"))
    run(body)


# ------------------------------------------------------------------------------ partial apply
@pytest.mark.parametrize("cgroup_mode", ["v1", "v2"])
def test_apply_failing_after_its_grant_took_effect_is_rolled_back(cgroup_mode):
    """The backend grants, then fails (a later line of a v1 write, a set-mode program step
    after the map update): the failing container's grant is revoked and nothing stays
    journaled."""
    async def body(lc):
        lc.tenant("t")
        w = lc.nodes["node-0"].worker
        be = w.service.hm.backend
        real = be.apply
        calls = []

        def flaky(cgdir, grant, revoke, desired):
            real(cgdir, grant, revoke, desired)
            calls.append(len(grant))
            if grant and len(calls) == 1:
                raise OSError("EIO after the grant")
        be.apply = flaky
        code, _ = await lc.add("default", "t", 1)
        be.apply = real
        assert code == 500
        cid = lc.container_ids("default", "t")[0]
        ctr = node_of(lc).container(cid)
        assert be.allowed(ctr.cgroup_dir) == set(), "grant left behind after rollback"
        assert w.journal.get(cid) is None
        assert not await lc.audit("default", "t")
        code, _ = await lc.add("default", "t", 1)      # and the next attach works normally
        assert code == 200 and not await lc.audit("default", "t")
    run(body, cgroup_mode=cgroup_mode)


# ------------------------------------------------------------------------------ adoption
def test_grants_from_a_worker_without_journal_are_adopted_and_revocable():
    """Upgrade path: a pod hot-mounted by a worker that kept no journal (state dir wiped). The
    new worker adopts the hot GPUs' granted rules and present nodes at startup, so a placeholder
    deleted by someone else afterwards still gets the tenant's access revoked."""
    async def body(lc):
        lc.tenant("t")
        code, b = await lc.add("default", "t", 2)
        assert code == 200
        cid = lc.container_ids("default", "t")[0]
        jdir = os.path.join(node_of(lc).state_dir, "journal")
        await lc.stop_worker("node-0")
        for f in os.listdir(jdir):                    # the record is lost
            os.unlink(os.path.join(jdir, f))
        w = await lc.start_worker("node-0")
        assert w.service.adopted
        assert len(w.journal.nodes_of(cid)) == 5 and len(w.journal.rules_of(cid)) == 5
        # someone deletes one placeholder: its GPU goes back to the scheduler
        ph = lc.cluster.placeholders()[0]
        lc.cluster.delete(ph["metadata"]["namespace"], ph["metadata"]["name"], grace=0)
        await asyncio.sleep(0.05)
        rep = await w.reconciler.run_once()
        assert rep.orphans >= 2, rep                  # its render + card rule and nodes
        assert not await lc.audit("default", "t")
        devs = node_of(lc).container_devices(cid)
        assert sum("renderD" in d for d in devs) == 1 and "dev/kfd" in devs
    run(body, worker_overrides={"reconcile_on_events": False})


def test_adoption_leaves_containers_with_a_record_alone(mock_inventory):
    async def body(lc):
        lc.tenant("t")
        await lc.add("default", "t", 1)
        w = lc.nodes["node-0"].worker
        w.service.adopted = False
        assert await w.service.adopt_existing() == 0
    run(body)


# ------------------------------------------------------------------------------ foreign veto
def test_audit_keeps_journaled_rule_that_a_foreign_program_vetoes():
    """v2: a foreign program (systemd re-realising its unit) vetoes a pair gpumounter still
    grants in its own program. The effective verdict says "not allowed", but our grant is
    there: the journal must keep it (and report it stale once the ledger drops it), or it
    would never be revoked once the foreign program is gone."""
    class Backend:
        name = "test"

        def __init__(self):
            self.own = {(226, 128)}

        def allowed(self, cgdir):
            return set()                      # vetoed by someone else's program

        def installed(self, cgdir):
            return set(self.own)

        def apply(self, cgdir, grant, revoke, desired):
            self.own -= {(n.major, n.minor) for n in revoke}

    class Writer:
        def present_many(self, t, nodes):
            return [False] * len(nodes)

        def present(self, t, n):
            return False

        def remove(self, t, nodes):
            return [0] * len(nodes)

    class Cfg:
        drm_major, inject_card_nodes, device_file_mode, container_root_prefix = 226, True, \
            0o666, "/nonexistent"

    class Resolver:
        def container_dir(self, pod, ref):
            return "/cg"

        def pids(self, cgdir):
            return []

    from gpumounter_amd.hw.inventory import Inventory
    inv = Inventory("mock")
    j = InjectionJournal()
    hm = HotMount(Cfg(), inv, Resolver(), Backend(), Writer(), journal=j)
    pod = {"metadata": {"name": "p", "namespace": "d", "uid": "u"},
           "spec": {"containers": [{"name": "c"}]},
           "status": {"phase": "Running", "containerStatuses": [
               {"name": "c", "containerID": "containerd://abc", "state": {"running": {}}}]}}
    j.intend("abc", [((226, 128), "/dev/dri/renderD128")], [], namespace="d", pod="p",
             pod_uid="u", container="c", cgdir="/cg")
    issues = hm.audit(pod, [], [])
    assert [(i.kind, i.minor) for i in issues] == [("stale_rule", 128)]
    assert j.rules_of("abc")                      # still ours: kept until revoked
    hm.revoke_issues(pod, issues, [], [])
    assert not j.rules_of("abc") and hm.backend.own == set()


# ------------------------------------------------------------------------------ privileged busy
def test_privileged_pod_gpu_process_is_busy_and_force_killed(tmp_path, mock_inventory):
    """A privileged pod gets a ledger-only attach (no rules or nodes written), but its
    processes count: RemoveGPU reports busy, and force kills them."""
    sleeper = subprocess.Popen(["sleep", "60"])
    table = tmp_path / "procs"
    _native.mock_smi().gm_mock_set_procs_file(str(table).encode())
    try:
        async def body(lc):
            c = {"name": "main", "image": "x", "command": ["sleep", "infinity"],
                 "securityContext": {"privileged": True}}
            lc.cluster.create_running_pod("default", {"metadata": {"name": "priv"},
                                                      "spec": {"containers": [c]}},
                                          "node-0", {"main": [sleeper.pid]})
            code, b = await lc.add("default", "priv", 1)
            assert code == 200
            dev = b["devices"][0]
            table.write_text(f"{dev['index']} {sleeper.pid} 4096 python\n")
            code, _ = await lc.remove("default", "priv", [dev["uuid"]])
            assert code == 400                               # busy, not silently released
            assert len(lc.cluster.placeholders()) == 1
            code, b2 = await lc.remove("default", "priv", [dev["uuid"]], force=True)
            assert code == 200 and b2["killed_pids"] == [sleeper.pid]
            assert lc.cluster.placeholders() == []
        run(body, worker_overrides={"busy_detection": "both"})
        assert sleeper.wait(timeout=10) == -15
    finally:
        _native.mock_smi().gm_mock_set_procs_file(b"")
        if sleeper.poll() is None:
            sleeper.kill()


# ------------------------------------------------------------------------------ candidates
def test_candidates_left_by_a_dead_pick_are_never_mounted_and_are_released():
    """A trim or placement-correction pick holds 1-GPU *candidate* placeholders and confirms
    only the ones it keeps. A worker that dies mid-pick leaves candidates owned by the tenant:
    nothing may mount them (the tenant asked for fewer GPUs), and the reconciler gives them
    back."""
    async def body(lc):
        lc.tenant("t")
        code, b = await lc.add("default", "t", 1)
        assert code == 200
        w = lc.nodes["node-0"].worker
        pod = lc.cluster.get("default", "t")
        left = await w.service.ph.hold_singles(pod, 3, False, "", "dead-attach", "", "")
        assert len(left) == 3 and all(p.candidate for p in left)
        st = await w.service.pod_state(pod, fresh=True)
        assert [g.uuid for g in st.hot] == [b["devices"][0]["uuid"]]     # not the candidates
        assert not await lc.audit("default", "t")
        rep = await w.reconciler.run_once()
        assert len(rep.stuck) == 3 and not rep.repaired, rep
        assert len(lc.cluster.placeholders()) == 1 and len(node_of(lc).allocated) == 1
        assert not await lc.audit("default", "t")
    run(body, worker_overrides={"reconcile_on_events": False})


def test_a_sweep_does_not_release_a_pick_confirmed_after_its_snapshot():
    """A sweep lists the placeholders once, then takes each owner's lock in turn. A trim pick
    that held the lock when the list was taken has confirmed its kept placeholder by the time
    the sweep gets the lock. Judged from the list, that placeholder was still a candidate of a
    pick that is not running, so the sweep released it and revoked a GPU the tenant had been
    answered (chaos seed 110: a trim attach answered 200, and its GPU left the ledger 12 ms
    later). The sweep judges what the owner holds once it has the lock."""
    async def body(lc):
        lc.tenant("t")
        svc = lc.nodes["node-0"].worker.service
        snap = []
        confirm = svc.ph.confirm

        async def confirm_spy(phs):
            snap.append(svc.ph.live())            # the sweep's list, taken mid-pick
            await confirm(phs)
        svc.ph.confirm = confirm_spy
        code, b = await lc.add("default", "t", 1)
        assert code == 200 and snap
        svc.ph.confirm = confirm
        # the sweep lists before it takes the first owner's lock; everything after reads now
        live, pod_lock, listing = svc.ph.live, svc.pod_lock, [True]

        def listed():
            return snap[0] if listing[0] else live()

        def lock(ns, name):
            listing[0] = False
            return pod_lock(ns, name)
        svc.ph.live, svc.pod_lock = listed, lock
        try:
            rep = await lc.nodes["node-0"].worker.reconciler.run_once()
        finally:
            svc.ph.live, svc.pod_lock = live, pod_lock
        assert not listing[0] and not rep.stuck, rep
        st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
        assert [g.uuid for g in st.hot] == [b["devices"][0]["uuid"]]
        assert not await lc.audit("default", "t")
    run(body, worker_overrides={"reconcile_on_events": False, "placement_enforce": "trim"})


def test_a_sweep_audits_an_owner_it_skipped_as_busy_once_the_operation_is_done():
    """A relist can carry a tenant's container restart without any MODIFIED event: the sweep it
    wakes is then the only repair. An owner whose lock an operation holds is skipped by the
    sweep, and its new container stayed without its hot GPUs until the next periodic sweep,
    30 s later (chaos seed 148: a failed attach of the same Pod held the lock). The skipped
    owner is audited as soon as the operation ends."""
    async def body(lc):
        lc.tenant("t")
        code, _ = await lc.add("default", "t", 1)
        assert code == 200
        w = lc.nodes["node-0"].worker
        svc = w.service
        lc.cluster.restart_container("default", "t", "main")   # no event reaction: relisted
        for _ in range(100):
            await asyncio.sleep(0.01)
            cur = svc.node_pods.get("default", "t")
            if cur and podu.running_containers(cur)[0].id == lc.container_ids("default", "t")[0]:
                break
        assert await lc.audit("default", "t")                  # the new container lacks it
        async with svc.pod_lock("default", "t"):               # an operation in flight
            rep = await w.reconciler.run_once()
            assert not rep.repaired
        for _ in range(200):
            await asyncio.sleep(0.01)
            if not await lc.audit("default", "t"):
                break
        assert not await lc.audit("default", "t")
    run(body, worker_overrides={"reconcile_on_events": False})


# ------------------------------------------------------------------------------ long-lived worker
def test_per_pod_caches_do_not_grow_with_pods_that_left():
    """A worker lives for the node's lifetime and sees many short-lived tenants: the per-pod
    locks and own-GPU cache only hold pods that are still there."""
    import gc

    async def body(lc):
        svc = lc.nodes["node-0"].worker.service
        uids = set()
        for i in range(6):
            lc.tenant(f"t{i}")
            uids.add(lc.cluster.get("default", f"t{i}")["metadata"]["uid"])
            code, b = await lc.add("default", f"t{i}", 1)
            assert code == 200
            code, _ = await lc.remove("default", f"t{i}", [b["devices"][0]["uuid"]])
            assert code == 200
            assert any(k[0] in uids for k in svc.hm.resolver._cache)
            lc.cluster.delete("default", f"t{i}", grace=0)
        for _ in range(50):
            await asyncio.sleep(0.02)
            if not svc._own:
                break
        gc.collect()
        assert not svc._own, svc._own
        assert len(svc._locks) == 0, list(svc._locks)
        assert not [k for k in svc.hm.resolver._cache if k[0] in uids]
    run(body)


# ------------------------------------------------------------------------------ dead attaches
def test_unadmitted_placeholder_of_a_dead_worker_is_released_at_once():
    """A worker SIGKILLed mid-attach leaves a placeholder the scheduler has not admitted (here:
    the node is full). Nothing will ever wait for it, and if a GPU freed up later the reconciler
    would mount it into a Pod whose request failed long ago: the next worker releases it on its
    first sweep instead of after stuck_after_s. An admitted one from the dead worker may be a
    finished attach whose reply went out; it stays and is mounted."""
    async def body(lc):
        for t in ("t", "filler"):
            lc.tenant(t)
        w = lc.nodes["node-0"].worker
        svc = w.service
        code, b = await lc.add("default", "t", 1)
        assert code == 200
        code, fb = await lc.add("default", "filler", 7)          # node full
        assert code == 200
        tenant = lc.cluster.get("default", "t")
        ph = svc.ph

        async def dead_worker_placeholder():
            mine = ph.incarnation
            ph.incarnation = "dead-worker"
            body = ph.build(tenant, 1, "single", attach_id="rq-dead")
            ph.incarnation = mine
            await svc.kube.create_pod(body["metadata"]["namespace"], body)
            await asyncio.sleep(0.1)
            return body["metadata"]["namespace"], body["metadata"]["name"]

        ns, name = await dead_worker_placeholder()
        assert lc.cluster.get(ns, name)["status"]["phase"] == "Pending"
        rep = await w.reconciler.run_once()
        assert name in rep.stuck, rep
        assert not any(p["metadata"]["name"] == name for p in lc.cluster.placeholders())
        st = await svc.pod_state(tenant, fresh=True)
        assert [g.uuid for g in st.hot] == [b["devices"][0]["uuid"]]
        assert not await lc.audit("default", "t")
        # a GPU is free: the dead worker's placeholder is admitted — kept, and mounted
        code, _ = await lc.remove("default", "filler", [fb["devices"][0]["uuid"]])
        assert code == 200
        ns, name = await dead_worker_placeholder()
        rep = await w.reconciler.run_once()
        assert name not in rep.stuck and rep.repaired == ["default/t"], rep
        st = await svc.pod_state(tenant, fresh=True)
        assert len(st.hot) == 2 and not await lc.audit("default", "t")
    run(body, worker_overrides={"reconcile_on_events": False})


def test_caller_going_away_mid_attach_does_not_leave_half_an_attach():
    """The master dies, or its deadline passes, while the worker waits for the placeholder's
    admission: gRPC cancels the handler. The attach must still run to its end — here it
    completes — instead of stopping between two steps with a placeholder created but never
    mounted (found by bench/configs.py chaos --master-kill-every)."""
    import grpc

    from gpumounter_amd.api import gpu_mount as api
    from gpumounter_amd.fakes.apiserver import LatencyModel

    async def body(lc):
        lc.tenant("t")
        ch = lc.master.workers.channel(lc.master.workers.target("node-0"))
        stub = ch.unary_unary(api.ADD_GPU, request_serializer=api.AddGPURequest.SerializeToString,
                              response_deserializer=api.AddGPUResponse.FromString)
        with pytest.raises(grpc.aio.AioRpcError) as ei:
            await stub(api.AddGPURequest(pod_name="t", namespace="default", gpu_num=2,
                                         is_entire_mount=False), timeout=0.05)
        assert ei.value.code() == grpc.StatusCode.DEADLINE_EXCEEDED
        w = lc.nodes["node-0"].worker
        svc = w.service
        tenant = lc.cluster.get("default", "t")
        for _ in range(200):                 # admission takes ~0.2 s here, then the mount
            await asyncio.sleep(0.02)
            if not w._ops:                   # the shielded operation has ended
                break
        assert not w._ops
        assert len((await svc.pod_state(tenant, fresh=True)).hot) == 2
        assert all(p["spec"].get("nodeName") for p in lc.cluster.placeholders())
        assert not await lc.audit("default", "t")
    run(body, latency=LatencyModel(schedule_ms=100.0, admit_ms=100.0))


def test_device_nodes_go_through_a_process_of_the_container_not_one_moved_in_from_outside(
        tmp_path):
    """The cgroup of a container can hold a process that was moved in from outside it (a debug
    tool, nsenter without -m, a test probe writing its PID to cgroup.procs). Its /proc/<pid>/root
    is the worker's own root: nodes written through it landed in the worker's /dev. The writer
    takes the first process in another mount namespace, and none at all when there is none."""
    from gpumounter_amd.node.devnodes import DevNodeWriter
    proc = tmp_path / "proc"
    for pid, ns in (("self", "mnt:[4026531840]"), ("100", "mnt:[4026531840]"),
                    ("200", "mnt:[4026532999]"), ("300", "mnt:[4026532999]")):
        (proc / pid / "ns").mkdir(parents=True)
        os.symlink(ns, proc / pid / "ns" / "mnt")
    w = DevNodeWriter("procroot", proc_root=str(proc))
    assert w.root_pid([100, 200, 300]) == 200      # 100 shares the worker's mount namespace
    assert w.root_pid([300]) == 300
    assert w.root_pid([100]) == 0                  # only an outsider: no root to write through
    assert w.root_pid([999, 200]) == 200           # exited meanwhile: skipped
    assert DevNodeWriter("emulate", proc_root=str(proc)).root_pid([100, 200]) == 100


def test_a_sweep_that_skipped_a_busy_owner_sweeps_again_soon():
    """A restarted worker's first sweep skipped the owner its lease expiry held; that owner's
    placeholders from the dead worker's last attach (never admitted: nothing waits for them)
    stayed unbound until the next periodic sweep, 30 s later (chaos rpl211). A sweep that
    skipped an owner now sweeps again SKIPPED_RESWEEP_S later."""
    from gpumounter_amd.cluster.placeholder import ANN_INCARNATION

    async def body(lc):
        pod = lc.tenant("t")
        w = lc.nodes["node-0"].worker
        svc = w.service
        body_ = svc.ph.build(pod, 9, "single")        # more GPUs than the node has: Pending
        body_["metadata"]["annotations"][ANN_INCARNATION] = "a-dead-worker"
        ph = await svc.kube.create_pod(body_["metadata"]["namespace"], body_)
        name = ph["metadata"]["name"]
        for _ in range(200):
            if any(p["metadata"]["name"] == name for p in svc.ph.owned_by(pod)):
                break
            await asyncio.sleep(0.01)
        async with svc.pod_lock("default", "t"):       # an operation in flight
            w.reconciler.wake()
            for _ in range(300):
                if "default/t" in w.reconciler.last.skipped:
                    break
                await asyncio.sleep(0.01)
            assert "default/t" in w.reconciler.last.skipped
            assert lc.cluster.get("gpu-pool", name) is not None
        t0 = asyncio.get_running_loop().time()
        while lc.cluster.get("gpu-pool", name) is not None:
            assert asyncio.get_running_loop().time() - t0 < 6, "not released within a re-sweep"
            await asyncio.sleep(0.05)
    run(body, reconcile_period_s=30.0)
