"""Regression tests for the reference defects listed in SURVEY §2.6 that no other test pins
down by name. (Covered elsewhere: 3 substring owner match — test_e2e::
test_owner_match_is_exact_not_substring; 4 cross-namespace ownerRef — test_fakes_and_ledger;
5 mount-type heuristic — test_e2e::test_pod_with_own_gpus_keeps_them; 6 gpuNum 0 —
test_e2e::test_add_parameter_validation; 7 locking — test_concurrency; 8 multi-container /
runtimes — test_e2e::test_runtime_and_cgroup_variants_with_multi_container_pods; 12 partial
state — test_faults; 13 authn/authz, TLS — test_authz, test_tls_and_metrics.)"""
import asyncio
import logging
import socket

import pytest

from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.fakes.apiserver import LatencyModel


def run(coro_fn, **kw):
    async def main():
        async with LocalCluster(**kw) as lc:
            return await coro_fn(lc)
    return asyncio.run(main())


def test_defect1_no_apiserver_busy_polling_while_waiting_for_placeholders():
    """Reference allocator.go:246-281 spins Pods.Get with no sleep until the slave is Running.
    Here readiness comes from the watch: with a slow scheduler + kubelet (≈30 ms per attach) an
    attach issues a constant handful of API requests, not hundreds."""
    async def body(lc):
        lc.tenant("t")
        before = dict(lc.cluster.requests_by_verb)
        code, b = await lc.add("default", "t", 2)
        assert code == 200, b
        after = lc.cluster.requests_by_verb
        gets = after.get("GET", 0) - before.get("GET", 0)
        posts = after.get("POST", 0) - before.get("POST", 0)
        assert gets <= 2, (before, after)       # the master's pod lookup (cached afterwards)
        assert posts <= 2                        # the placeholder create(s)
    run(body, latency=LatencyModel.realistic())


def test_defect2_placeholder_deleted_while_waiting_is_a_failure_not_success():
    """Reference allocator.go:251-253 treats NotFound during the wait as success."""
    async def body(lc):
        lc.tenant("t")
        svc = lc.nodes["node-0"].worker.service
        real = svc.ph._create  # noqa: SLF001

        async def create_then_vanish(bodies):
            created = await real(bodies)
            for ph in created:
                lc.cluster.delete(ph.namespace, ph.name, grace=0)
            return created
        svc.ph._create = create_then_vanish  # noqa: SLF001
        code, b = await lc.add("default", "t", 1)
        assert code != 200, b
        svc.ph._create = real  # noqa: SLF001
        st = await svc.pod_state(lc.cluster.get("default", "t"), fresh=True)
        assert st.hot == [] and await lc.audit("default", "t") == []
    run(body, latency=LatencyModel(schedule_ms=50))


def test_defect13_worker_listen_error_is_fatal_not_logged():
    """Reference worker main.go:26-28 logs a listen error and carries on without a server."""
    from gpumounter_amd.worker.server import Worker

    busy = socket.socket()
    busy.bind(("127.0.0.1", 0))
    busy.listen(1)
    port = busy.getsockname()[1]

    async def body(lc):
        h = lc.nodes["node-0"]
        cfg = h.cfg.replace(worker_port=port)
        w = Worker(cfg, inventory=lc.inventory)
        with pytest.raises(OSError):
            await w.start(http_port=-1, reconcile=False)
        await w.stop()
    try:
        run(body)
    finally:
        busy.close()


def test_defect14_log_file_is_appended_and_rotated_not_truncated(tmp_path):
    """Reference log.go:28 os.Create()s the log file at every start."""
    from gpumounter_amd.utils import log

    path = str(tmp_path / "worker.log")
    log.setup("INFO", json_format=True, log_file=path)
    logging.getLogger("gpumounter.test").info("first start")
    log.setup("INFO", json_format=True, log_file=path)     # a restart
    logging.getLogger("gpumounter.test").info("second start")
    for h in logging.getLogger("gpumounter").handlers:
        h.flush()
    text = open(path).read()
    assert "first start" in text and "second start" in text
    log.setup("WARNING", json_format=False)


def test_transient_apiserver_errors_are_retried_and_lost_creates_recovered():
    """An apiserver shedding load (503) or a create whose reply was lost must not fail or
    duplicate an attach: reads/deletes/patches and named creates are retried; a retried create
    that meets its own first attempt (409) adopts it."""
    async def body(lc):
        lc.tenant("t")
        c = lc.cluster
        c.fail_next("POST", 503, count=2)                  # placeholder create shed twice
        code, b = await lc.add("default", "t", 1)
        assert code == 200, b
        c.fail_next("POST", 504, after=True)               # created, but the reply is lost
        code, b2 = await lc.add("default", "t", 1)
        assert code == 200, b2
        live = [p for p in c.placeholders() if not p["metadata"].get("deletionTimestamp")]
        assert len(live) == 2                              # no duplicate from the retry
        c.fail_next("DELETE", 503)
        code, _ = await lc.remove("default", "t", [b["devices"][0]["uuid"]])
        assert code == 200
        assert await lc.audit("default", "t") == []
    run(body)
