"""Control-plane call accounting (utils/calls.py): what an attach and a detach wait for."""
import asyncio
import time

from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.utils import calls


def test_serial_depth_counts_chains_not_parallel_calls():
    cs = [(0.0, 1.0, "a"), (0.1, 0.9, "b"), (0.2, 1.1, "c"),     # sent together: one trip
          (1.2, 2.0, "d"),                                        # then one more
          (2.5, 2.5, "checkpoint read"),                          # a file read: no trip
          (2.1, 3.0, "e" + calls.BACKGROUND)]
    assert calls.serial_depth([c for c in cs if not c[2].endswith(calls.BACKGROUND)]) == 2
    s = calls.summary(cs)
    assert s["serial_round_trips"] == 2
    assert s["calls"] == {"a": 1, "b": 1, "c": 1, "checkpoint read": 1, "d": 1}
    assert s["background"] == {"e": 1}


def test_attach_and_detach_make_one_serial_apiserver_round_trip():
    async def main():
        async with LocalCluster(cgroup_mode="v2") as lc:
            lc.tenant("t")
            code, b = await lc.add("default", "t", 1)      # warm: channels, caches
            assert code == 200
            code, _ = await lc.remove("default", "t", [b["devices"][0]["uuid"]])
            assert code == 200
            await asyncio.sleep(0.05)
            t0 = time.monotonic()
            code, b = await lc.add("default", "t", 2, entire=True)
            t1 = time.monotonic()
            assert code == 200
            code, _ = await lc.remove("default", "t", [d["uuid"] for d in b["devices"]])
            t2 = time.monotonic()
            assert code == 200
            att = calls.summary(calls.since(t0, t1))
            det = calls.summary(calls.since(t1, t2))
            # attach: the placeholder POST (its admission is read from the checkpoint, no
            # kubelet RPC); detach: the DELETE. The reference: GET pod, LIST workers, one POST
            # per slave pod in sequence, a GET poll per slave pod, a PodResources List
            assert att["calls"].get("apiserver POST pods") == 1, att
            assert att["serial_round_trips"] == 1, att
            assert not any(k.startswith("kubelet") for k in att["calls"]), att
            assert det["calls"].get("apiserver DELETE pods") == 1, det
            assert det["serial_round_trips"] == 1, det
    asyncio.run(main())
