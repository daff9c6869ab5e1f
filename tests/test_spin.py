"""utils/spin.py: the loop polls while a request holds the spinner, for the tail after, and
never longer than the cap; off by default."""
import asyncio

from gpumounter_amd.utils.config import Config
from gpumounter_amd.utils.spin import LoopSpinner


def test_off_by_default():
    sp = LoopSpinner(Config().loop_spin_us, Config().loop_spin_max_ms)
    assert not sp.enabled

    async def main():
        with sp.hold():
            await asyncio.sleep(0.005)
    asyncio.run(main())
    assert sp.ticks == 0


def test_polls_while_held_then_for_the_tail_only():
    sp = LoopSpinner(tail_us=2000, max_ms=1000)

    async def main():
        with sp.hold():
            await asyncio.sleep(0.01)
        held = sp.ticks
        assert held > 10                        # the loop kept iterating during the sleep
        await asyncio.sleep(0.05)               # the 2 ms tail, then blocking waits again
        after = sp.ticks
        await asyncio.sleep(0.05)
        assert sp.ticks == after                # stopped
    asyncio.run(main())


def test_capped_per_stretch_and_nested_holds():
    sp = LoopSpinner(tail_us=100, max_ms=5)

    async def main():
        with sp.hold():
            with sp.hold():
                pass                            # inner exit: still held, no tail yet
            assert sp._spinning                 # noqa: SLF001
            await asyncio.sleep(0.03)           # past the 5 ms cap: polling stopped
            n = sp.ticks
            await asyncio.sleep(0.02)
            assert sp.ticks == n
        with sp.hold():                         # a new request starts a new stretch
            await asyncio.sleep(0.002)
        assert sp.ticks > n
    asyncio.run(main())


def test_attach_and_detach_with_polling_loops():
    """loop_spin_us on the master and the worker: requests are served as without it, the loops
    polled during them, and polling stops once they are answered."""
    from gpumounter_amd.fakes.harness import LocalCluster

    async def main():
        async with LocalCluster(worker_overrides={"loop_spin_us": 300},
                                master_overrides={"loop_spin_us": 300}) as lc:
            lc.tenant("t")
            code, b = await lc.add("default", "t", 1)
            assert code == 200
            code, _ = await lc.remove("default", "t", [b["devices"][0]["uuid"]])
            assert code == 200 and not await lc.audit("default", "t")
            spinners = [lc.master.spin, lc.nodes["node-0"].worker.spin]
            assert all(s.enabled and s.ticks > 0 for s in spinners)
            await asyncio.sleep(0.05)
            before = [s.ticks for s in spinners]
            await asyncio.sleep(0.05)
            assert [s.ticks for s in spinners] == before
    asyncio.run(main())
