"""Busy detection's process tables: KFD's sysfs table, the host-PID-namespace gate, and the
order KFD table → amdsmi for PIDs the fd scan cannot read (node/procs.py)."""
import os

import pytest

from gpumounter_amd.models.device import AmdGpu
from gpumounter_amd.node import procs


def _gpu(kfd_gpu_id=49070, index=0):
    # render minor 250: no such device here, so the fd scan never hits and only tables can
    return AmdGpu(index=index, uuid="u", bdf="0000:05:00.0", render_minor=250, card_minor=1,
                  kfd_gpu_id=kfd_gpu_id)


def _table(root, entries):
    for pid, files in entries.items():
        d = root / str(pid)
        d.mkdir(parents=True)
        for name, val in files.items():
            if "/" in name:
                (d / name.split("/")[0]).mkdir(exist_ok=True)
            (d / name).write_text(val + "\n")
    return str(root)


class _Smi:
    def __init__(self, pids=()):
        self.pids, self.calls = list(pids), 0

    def processes(self, index):
        self.calls += 1
        return [type("P", (), {"pid": p})() for p in self.pids]


def test_kfd_table_parses_sysfs_layout(tmp_path):
    # the layout measured on an MI355X box (profiles/r6_kfd_probe/kfd_probe.json)
    root = _table(tmp_path / "proc", {
        2370128: {"pasid": "0", "vram_49070": "268435456", "sdma_49070": "0",
                  "stats_49070/cu_occupancy": "0", "counters_49070/faults": "0"},
        792591: {"pasid": "0", "vram_49070": "0", "vram_111": "4096"},
        555: {"pasid": "0"},                                    # bound to no GPU yet
    })
    (tmp_path / "proc" / "notapid").mkdir()
    assert procs.kfd_table(root) == {49070: {2370128: 268435456, 792591: 0}, 111: {792591: 4096}}


def test_kfd_table_unreadable_raises(tmp_path):
    with pytest.raises(OSError):
        procs.kfd_table(str(tmp_path / "missing"))


def test_busy_pids_uses_kfd_table_before_amdsmi(tmp_path):
    me = os.getpid()
    root = _table(tmp_path / "proc", {me: {"vram_49070": "1"}, 1: {"vram_49070": "1"}})
    smi = _Smi([me])
    assert procs.busy_pids(smi, [_gpu()], [me], mode="both", kfd_root=root) == {0: [me]}
    assert smi.calls == 0
    # another GPU's gpu_id: the table says no, and amdsmi is not asked either
    assert procs.busy_pids(smi, [_gpu(kfd_gpu_id=7)], [me], mode="both", kfd_root=root) == {}
    assert smi.calls == 0


def test_busy_pids_falls_back_to_amdsmi(tmp_path):
    me = os.getpid()
    smi = _Smi([me])
    missing = str(tmp_path / "missing")
    assert procs.busy_pids(smi, [_gpu()], [me], mode="both", kfd_root=missing) == {0: [me]}
    assert smi.calls == 1
    assert procs.busy_pids(smi, [_gpu()], [me], mode="both", kfd_root="") == {0: [me]}
    assert smi.calls == 2
    # a GPU amdsmi enumerated without a KFD node id: amdsmi answers even with a table
    root = _table(tmp_path / "proc", {me: {"vram_49070": "1"}})
    assert procs.busy_pids(smi, [_gpu(kfd_gpu_id=0)], [me], mode="both",
                           kfd_root=root) == {0: [me]}
    assert smi.calls == 3


def test_busy_pids_outside_host_namespace_skips_tables(tmp_path):
    me = os.getpid()
    root = _table(tmp_path / "proc", {me: {"vram_49070": "1"}})
    smi = _Smi([me])
    assert procs.busy_pids(smi, [_gpu()], [me], mode="both", kfd_root=root, tables=False) == {}
    assert smi.calls == 0


def test_host_pid_ns_reads_the_namespace_inode(tmp_path):
    for name, link, want in (("host", f"pid:[{procs.PROC_PID_INIT_INO}]", True),
                             ("ctr", "pid:[4026532999]", False)):
        ns = tmp_path / name / "self" / "ns"
        ns.mkdir(parents=True)
        os.symlink(link, ns / "pid")
        assert procs.host_pid_ns(str(tmp_path / name)) is want
    assert procs.host_pid_ns(str(tmp_path / "nothing")) is False
    assert procs.PROC_PID_INIT_INO == 4026531836


IDLE = "import time; print('ready', flush=True); time.sleep(120)"


def test_worker_detach_takes_the_table_the_namespace_allows(tmp_path, monkeypatch,
                                                             mock_inventory):
    """End to end through the worker's detach: with the real library (``is_mock`` patched off)
    the KFD table at ``kfd_proc_path`` decides, and outside the host PID namespace neither the
    KFD table nor amdsmi's can make the GPU busy."""
    import asyncio
    import subprocess
    import sys

    from gpumounter_amd import _native
    from gpumounter_amd.fakes.harness import LocalCluster
    from gpumounter_amd.hw.inventory import Inventory

    g0 = mock_inventory.gpus()[0]
    p = subprocess.Popen([sys.executable, "-c", IDLE], stdout=subprocess.PIPE)
    assert p.stdout.readline().strip() == b"ready"
    smi_table = tmp_path / "smi"
    _native.mock_smi().gm_mock_set_procs_file(str(smi_table).encode())
    kfd = tmp_path / "kfd"
    (kfd / str(p.pid)).mkdir(parents=True)
    (kfd / str(p.pid) / f"vram_{g0.kfd_gpu_id}").write_text("4096\n")
    monkeypatch.setattr(Inventory, "is_mock", property(lambda self: False))

    async def cycle(lc, name, smi):
        lc.tenant(name, pids={"main": [p.pid]})
        code, b = await lc.add("default", name, 1)
        assert code == 200, b
        dev = b["devices"][0]
        smi_table.write_text(f"{dev['index']} {p.pid} 4096 python\n" if smi else "")
        code, b2 = await lc.remove("default", name, [dev["uuid"]], force=False)
        smi_table.write_text("")
        if code != 200:
            code3, b3 = await lc.remove("default", name, [dev["uuid"]], force=True)
            assert code3 == 200, b3
        return code, b2

    async def main(host):
        monkeypatch.setattr(procs, "host_pid_ns", lambda proc_root="/proc": host)
        async with LocalCluster(node_gpu_bdfs=[g0.bdf],
                                worker_overrides={"busy_detection": "both",
                                                  "kfd_proc_path": str(kfd)}) as lc:
            # in the host namespace amdsmi's table stays empty: the KFD table alone decides
            return await cycle(lc, f"t{int(host)}", smi=not host)
    try:
        code, b = asyncio.run(main(True))
        assert code == 400 and "running processes" in b["message"], b
        # outside the host namespace: the same tables, and no table is asked
        code, b = asyncio.run(main(False))
        assert code == 200, b
    finally:
        _native.mock_smi().gm_mock_set_procs_file(b"")
        if p.poll() is None:
            p.kill()
        p.wait()


def test_node_status_says_whose_pids_the_process_tables_hold(mock_inventory):
    import asyncio

    from gpumounter_amd.fakes.harness import LocalCluster

    async def main():
        async with LocalCluster(node_gpu_bdfs=[mock_inventory.gpus()[0].bdf],
                                start_master=False) as lc:
            svc = lc.nodes["node-0"].worker.service
            return await svc.node_status(True), await svc.node_status(False)
    with_procs, without = asyncio.run(main())
    assert with_procs["host_pid_ns"] is procs.host_pid_ns() and "processes" in with_procs
    assert "host_pid_ns" not in without
