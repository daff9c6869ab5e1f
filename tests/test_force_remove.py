"""Force removal keeps the GPU booked until the killed processes are gone.

Reference order: deny → rm → kill (SIGTERM), then the slave pods are deleted with default
delete options and polled until NotFound (reference: pkg/util/util.go:112-143,
pkg/util/gpu/allocator/allocator.go:128-156,284-317). A cgroup revoke only gates open(): a
process that ignores SIGTERM still holds its render/KFD fds, so the placeholder must outlive it
(worker/drain.py)."""
import asyncio
import subprocess
import sys
import time

import pytest

from gpumounter_amd import _native
from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.node import procs as procs_mod

IGNORES_TERM = ("import signal, time; signal.signal(signal.SIGTERM, signal.SIG_IGN); "
                "print('ready', flush=True); time.sleep(120)")


@pytest.fixture
def stubborn(tmp_path, mock_inventory):
    """A process that ignores SIGTERM, reported by the mock amdsmi as a user of GPU 0."""
    p = subprocess.Popen([sys.executable, "-c", IGNORES_TERM], stdout=subprocess.PIPE)
    assert p.stdout.readline().strip() == b"ready"
    table = tmp_path / "procs"
    _native.mock_smi().gm_mock_set_procs_file(str(table).encode())
    yield p, table
    _native.mock_smi().gm_mock_set_procs_file(b"")
    if p.poll() is None:
        p.kill()
        p.wait()


def one_gpu_cluster(mock_inventory, **worker):
    g0 = mock_inventory.gpus()[0]
    return LocalCluster(node_gpu_bdfs=[g0.bdf],
                        worker_overrides={"busy_detection": "both", **worker})


def test_placeholder_held_until_sigterm_ignoring_process_is_killed(stubborn, mock_inventory):
    p, table = stubborn

    async def main():
        async with one_gpu_cluster(mock_inventory, kill_grace_s=0.6) as lc:
            lc.tenant("busy", pids={"main": [p.pid]})
            lc.tenant("other")
            code, b = await lc.add("default", "busy", 1)
            assert code == 200, b
            dev = b["devices"][0]
            table.write_text(f"{dev['index']} {p.pid} 4096 python\n")
            rm = asyncio.ensure_future(lc.remove("default", "busy", [dev["uuid"]], force=True))
            await asyncio.sleep(0.25)            # inside the SIGTERM grace: p still runs
            assert p.poll() is None and not rm.done()
            assert len(lc.cluster.placeholders()) == 1          # GPU still booked
            code, b2 = await lc.add("default", "other", 1)      # ... so nobody else gets it
            assert code == 500 and "Insufficient" in b2["message"], b2
            code, b3 = await rm
            assert code == 200 and b3["killed_pids"] == [p.pid], b3
            assert p.wait(timeout=5) == -9       # SIGTERM ignored → SIGKILL after the grace
            assert lc.cluster.placeholders() == []
            code, b4 = await lc.add("default", "other", 1)
            assert code == 200 and b4["devices"][0]["uuid"] == dev["uuid"]
            assert not await lc.audit("default", "busy")
    asyncio.run(main())


def test_detach_without_busy_processes_does_not_wait(mock_inventory):
    async def main():
        async with one_gpu_cluster(mock_inventory, kill_grace_s=5.0) as lc:
            lc.tenant("idle")
            _, b = await lc.add("default", "idle", 1)
            t0 = time.monotonic()
            code, _ = await lc.remove("default", "idle", [b["devices"][0]["uuid"]], force=True)
            assert code == 200 and time.monotonic() - t0 < 1.0
    asyncio.run(main())


def test_process_surviving_sigkill_leaves_a_draining_placeholder(stubborn, mock_inventory,
                                                                 monkeypatch):
    """A process still there after SIGKILL (uninterruptible sleep in the driver, simulated by
    withholding the SIGKILL) keeps the GPU booked in a draining placeholder, detached from the
    tenant. RemoveGPU names the PIDs; the GPU is released the moment the process exits."""
    p, table = stubborn
    real = procs_mod.Pinned.signal

    def no_sigkill(self, pids, sig):
        if sig == 9:
            return [0 for _ in pids]
        return real(self, pids, sig)
    monkeypatch.setattr(procs_mod.Pinned, "signal", no_sigkill)

    async def main():
        async with one_gpu_cluster(mock_inventory, kill_grace_s=0.2, kill_reap_s=0.3) as lc:
            lc.tenant("busy", pids={"main": [p.pid]})
            lc.tenant("other")
            _, b = await lc.add("default", "busy", 1)
            dev = b["devices"][0]
            table.write_text(f"{dev['index']} {p.pid} 4096 python\n")
            code, b2 = await lc.remove("default", "busy", [dev["uuid"]], force=True)
            assert code == 400 and str(p.pid) in b2["detail"], b2
            assert "still running" in b2["detail"] and b2["killed_pids"] == [p.pid]
            phs = lc.cluster.placeholders()
            assert len(phs) == 1
            md = phs[0]["metadata"]
            assert md["annotations"]["gpumounter.amd.com/mount-mode"] == "draining"
            assert md["annotations"]["gpumounter.amd.com/drain-pids"].startswith(f"{p.pid}:")
            assert "gpumounter.amd.com/owner" not in md["labels"]
            svc = lc.nodes["node-0"].worker.service
            st = await svc.pod_state(lc.cluster.get("default", "busy"))
            assert st.hot == [] and not await lc.audit("default", "busy")   # access revoked
            rep = await lc.nodes["node-0"].worker.reconciler.run_once()
            assert not rep.repaired and not rep.errors and len(lc.cluster.placeholders()) == 1
            code, _ = await lc.add("default", "other", 1)
            assert code == 500                                  # still booked
            p.kill()                                            # the process finally exits
            p.wait()
            for _ in range(100):
                if not lc.cluster.placeholders():
                    break
                await asyncio.sleep(0.02)
            assert lc.cluster.placeholders() == []              # released on pidfd readiness
            assert svc.drain.released == 1
            code, b3 = await lc.add("default", "other", 1)
            assert code == 200 and b3["devices"][0]["uuid"] == dev["uuid"]
    asyncio.run(main())


def test_restarted_worker_releases_a_drain_only_once_its_processes_exit(stubborn,
                                                                         mock_inventory,
                                                                         monkeypatch):
    """After a worker restart no pidfd is held: the reconciler's sweep reads the recorded
    (pid, start time) pairs and releases the placeholder only once they are gone."""
    p, table = stubborn
    real = procs_mod.Pinned.signal
    monkeypatch.setattr(procs_mod.Pinned, "signal",
                        lambda self, pids, sig: [0] * len(pids) if sig == 9 else
                        real(self, pids, sig))

    async def main():
        async with one_gpu_cluster(mock_inventory, kill_grace_s=0.1, kill_reap_s=0.1) as lc:
            lc.tenant("busy", pids={"main": [p.pid]})
            _, b = await lc.add("default", "busy", 1)
            dev = b["devices"][0]
            table.write_text(f"{dev['index']} {p.pid} 4096 python\n")
            code, _ = await lc.remove("default", "busy", [dev["uuid"]], force=True)
            assert code == 400
            w = lc.nodes["node-0"].worker
            await w.service.drain.stop()        # the worker's memory of the drain is gone
            assert await w.service.drain.sweep() == []          # process alive: kept
            assert len(lc.cluster.placeholders()) == 1
            p.kill()
            p.wait()
            rep = await w.reconciler.run_once()
            assert len(rep.drained) == 1 and lc.cluster.placeholders() == []
    asyncio.run(main())


def test_drain_survives_a_real_worker_crash_in_the_process_deployment(tmp_path, mock_inventory):
    """Daemons as processes (production entry points). SIGKILL is withheld by fault injection
    (GM_FAULT=kill_escalation:1), so the killed process outlives the RemoveGPU call and its
    placeholder drains. The worker is then SIGKILLed and restarted: the new incarnation holds no
    pidfd, finds the drain's pid:starttime record, keeps the GPU booked while the process lives
    and releases it once it has exited."""
    from gpumounter_amd.fakes.deployment import ProcessCluster

    p = subprocess.Popen([sys.executable, "-c", IGNORES_TERM], stdout=subprocess.PIPE)
    table = tmp_path / "procs"
    table.write_text("")
    pc = ProcessCluster(worker_env={"GM_FAULT": "kill_escalation:1.0", "GM_KILL_GRACE_S": "0.2",
                                    "GM_KILL_REAP_S": "0.2", "GM_BUSY_DETECTION": "both",
                                    "GM_AMDSMI_MOCK_PROCS": str(table),
                                    "GM_RECONCILE_PERIOD_S": "0.3"})
    try:
        assert p.stdout.readline().strip() == b"ready"
        pc.start()
        pc.tenant("busy", pids={"main": [p.pid]})
        code, b = pc.add("default", "busy", 1)
        assert code == 200, b
        dev = b["devices"][0]
        table.write_text(f"{dev['index']} {p.pid} 4096 python\n")
        code, b2 = pc.remove("default", "busy", [dev["uuid"]], force=True)
        assert code == 400 and str(p.pid) in b2["detail"], b2
        assert p.poll() is None
        assert pc.kill_worker() == -9
        pc.restart_worker()
        time.sleep(1.0)                                     # a few reconciler sweeps
        phs = pc.placeholders()
        assert len(phs) == 1, phs
        assert phs[0]["metadata"]["annotations"]["gpumounter.amd.com/mount-mode"] == "draining"
        assert pc.audit("default", "busy") == []            # access stays revoked
        p.kill()
        p.wait()
        deadline = time.time() + 10
        while pc.placeholders() and time.time() < deadline:
            time.sleep(0.1)
        assert pc.placeholders() == []
        assert 'gm_reconcile_actions_total{action="drain_release"} 1.0' in pc.worker_metrics()
    finally:
        pc.stop()
        if p.poll() is None:
            p.kill()
            p.wait()


def test_a_failed_draining_mark_is_retried_and_never_regranted(stubborn, mock_inventory,
                                                                monkeypatch):
    """the PATCH that turns a force-removed GPU's placeholder into a draining one
    fails. Its access is already revoked and the placeholder still names the tenant: the
    reconciler must not grant the GPU back, the GPU must stay booked while the killed process
    runs, and the mark is retried until it lands — across a worker restart too."""
    p, table = stubborn
    real = procs_mod.Pinned.signal
    monkeypatch.setattr(procs_mod.Pinned, "signal",
                        lambda self, pids, sig: [0] * len(pids) if sig == 9 else
                        real(self, pids, sig))

    async def main():
        async with one_gpu_cluster(mock_inventory, kill_grace_s=0.1, kill_reap_s=0.1) as lc:
            lc.tenant("busy", pids={"main": [p.pid]})
            _, b = await lc.add("default", "busy", 1)
            dev = b["devices"][0]
            table.write_text(f"{dev['index']} {p.pid} 4096 python\n")
            lc.cluster.fail_next("PATCH", 503, count=1000)        # every mark fails for now
            code, b2 = await lc.remove("default", "busy", [dev["uuid"]], force=True)
            assert code == 400 and "revoked" in b2["detail"], b2
            w = lc.nodes["node-0"].worker
            (ph,) = lc.cluster.placeholders()
            assert ph["metadata"]["annotations"].get("gpumounter.amd.com/mount-mode") != \
                "draining"                                       # still labelled the tenant's
            rep = await w.reconciler.run_once()
            assert not rep.repaired, rep                         # not granted back
            st = await w.service.pod_state(lc.cluster.get("default", "busy"), fresh=True)
            assert st.hot == [] and not await lc.audit("default", "busy")
            assert len(lc.cluster.placeholders()) == 1           # still booked
            assert len(w.service.drain.unmarked) == 1            # ... and its mark retried
            # a restart: the new worker knows the pending mark from its state_dir
            await lc.stop_worker("node-0")
            await lc.start_worker("node-0")
            w = lc.nodes["node-0"].worker
            assert len(w.service.drain.unmarked) == 1
            rep = await w.reconciler.run_once()
            assert not rep.repaired and not await lc.audit("default", "busy")
            lc.cluster._faults.clear()                           # noqa: SLF001 - PATCH works again
            for _ in range(200):                                 # the retry lands (≤ 0.5 s)
                if not w.service.drain.unmarked:
                    break
                await asyncio.sleep(0.02)
            (ph,) = lc.cluster.placeholders()
            assert ph["metadata"]["annotations"]["gpumounter.amd.com/mount-mode"] == "draining"
            p.kill()
            p.wait()
            rep = await w.reconciler.run_once()
            assert len(rep.drained) == 1 and lc.cluster.placeholders() == []
    asyncio.run(main())
