"""On-MI355X tests (``pytest -m gpu`` on the GPU box). Each loads the in-tree native libraries:
libgm_smi.so against the real libamd_smi, libgm_probe.so (gfx950 kernels), libgm_host.so.
Numerics tests compare HIP kernels against plain PyTorch fp32 references.
"""
import asyncio
import os
import subprocess
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def real_inventory():
    if not torch.cuda.is_available():
        pytest.fail("gpu test on a host without a GPU")
    from gpumounter_amd.hw.inventory import Inventory

    return Inventory("")


def test_amdsmi_real_inventory(real_inventory):
    from gpumounter_amd.ops import probe

    inv = real_inventory
    assert "mock" not in inv.lib_path
    gpus = inv.gpus()
    assert len(gpus) >= 1
    hip_bdfs = {probe.props(i)["pci_bus_id"] for i in range(probe.device_count())}
    seen = [g for g in gpus if g.bdf in hip_bdfs]
    assert seen, (hip_bdfs, [g.bdf for g in gpus])
    for g in seen:
        assert g.gfx_target == "gfx950", g.gfx_target
        assert g.render_minor >= 128
        assert g.vram_bytes > 200 * (1 << 30)     # 288 GB HBM3E
        assert g.num_cu >= 256 or g.num_cu == 0   # CPX partitions report fewer
    links = inv.links()
    assert links.n == len(gpus)
    assert all(links.types[i][i] == 0 for i in range(links.n))
    # health: liveness + ECC (counts may be unsupported on some firmware → None)
    assert all(inv.healthy().values())
    for g in seen:
        ecc = inv.ecc(g.index)
        print(f"{g.bdf}: ECC (correctable, uncorrectable, deferred) = {ecc}")
        assert ecc is None or all(v >= 0 for v in ecc)


def test_amd_smi_tool_sees_the_same_gpus(real_inventory):
    """BASELINE config "rocm-smi inside the Pod sees it": the stock ROCm tool and gpumounter's
    amdsmi shim must agree on BDF and UUID of every GPU (the ledger joins on them)."""
    import json
    import re

    try:
        res = subprocess.run(["amd-smi", "list", "--json"], capture_output=True, text=True,
                             timeout=90)
    except FileNotFoundError:
        pytest.skip("amd-smi not installed")
    assert res.returncode == 0, res.stderr[-2000:]
    blob = json.loads(res.stdout[res.stdout.index("["):] if "[" in res.stdout else res.stdout)
    found = set()

    def walk(x):
        if isinstance(x, dict):
            for v in x.values():
                walk(v)
        elif isinstance(x, list):
            for v in x:
                walk(v)
        elif isinstance(x, str):
            found.add(x.lower())
    walk(blob)
    bdf_re = re.compile(r"^[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.[0-7]$")
    tool_bdfs = {s for s in found if bdf_re.match(s)}
    ours = real_inventory.gpus()
    assert {g.bdf.lower() for g in ours} <= tool_bdfs, (tool_bdfs, [g.bdf for g in ours])
    assert all(g.uuid.lower() in found for g in ours), ([g.uuid for g in ours], sorted(found))


def test_probe_props_and_quick():
    from gpumounter_amd.ops import probe

    p = probe.props(0)
    assert p["gcn_arch"].startswith("gfx950"), p
    assert p["warp_size"] == 64
    us = probe.quick(0)
    assert us < 1e6


def test_probe_hbm_and_mfma_rates():
    from gpumounter_amd.ops import probe

    gbps = probe.hbm_gbps(0, 1 << 30, 10)
    tf = probe.mfma_tflops(0, 20000)
    print(f"HBM copy {gbps:.0f} GB/s, MFMA bf16 {tf:.0f} TF/s")
    assert gbps > 2000, gbps          # MI355X measured ≈5.6 TB/s on copy; 2 TB/s = sick GPU
    rd = probe.hbm_read_gbps(0, 1 << 30, 10)
    assert rd > 2000, rd
    assert tf > 500, tf               # dense bf16 peak ≈2.5 PF/s


@pytest.mark.parametrize("m,n,k", [(64, 64, 32), (128, 192, 96), (256, 256, 512)])
def test_mfma_gemm_bf16_matches_torch_fp32(m, n, k):
    from gpumounter_amd.ops import probe

    g = torch.Generator(device="cuda:0").manual_seed(m * 7 + n * 3 + k)
    a = torch.randn(m, k, device="cuda:0", generator=g).to(torch.bfloat16)
    b = torch.randn(k, n, device="cuda:0", generator=g).to(torch.bfloat16)
    c = probe.gemm_bf16(a, b)
    torch.cuda.synchronize()
    ref = a.float() @ b.float()
    err = (c - ref).abs().max().item()
    assert err <= 1e-3 * k ** 0.5 * 4, err


def test_mfma_gemm_asymmetric_identity():
    """A = I with an asymmetric B catches row/col swaps in the C write-back."""
    from gpumounter_amd.ops import probe

    a = torch.eye(64, 64, device="cuda:0").to(torch.bfloat16)
    b = (torch.arange(64, device="cuda:0").view(64, 1) * 100
         + torch.arange(64, device="cuda:0").view(1, 64)).float().to(torch.bfloat16)
    c = probe.gemm_bf16(a.contiguous(), b.contiguous())
    assert torch.equal(c, b.float())


@pytest.mark.parametrize("variant", [1, 5])
@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (512, 768, 192), (1280, 1024, 640)])
def test_gemm_nt256_matches_torch_fp32(m, n, k, variant):
    """The 256²-tile global_load_lds GEMM (odd tile counts exercise the XCD remap's remainder
    and the partial GROUP_M raster) against an fp32 reference of the same bf16 operands."""
    from gpumounter_amd.ops import probe

    g = torch.Generator(device="cuda:0").manual_seed(m + 5 * n + 11 * k)
    a = (torch.rand(m, k, device="cuda:0", generator=g) * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand(n, k, device="cuda:0", generator=g) * 2 - 1).to(torch.bfloat16)
    c = probe.gemm_nt(a, bt, variant=variant)
    torch.cuda.synchronize()
    ref = a.float() @ bt.float().t()
    err = (c.float() - ref).abs()
    # bf16 output rounding (2^-8 relative) + fp32 accumulation-order noise
    assert (err <= ref.abs() * 2 ** -8 + 1e-3 * k ** 0.5).all(), err.max().item()


@pytest.mark.parametrize("variant", [None, 1, 5])
def test_gemm_nt256_asymmetric_identity(variant):
    """A = I with an asymmetric Bt: C must equal Btᵀ exactly (catches row/col swaps, swizzle
    mismatches between the staged source and the LDS read)."""
    from gpumounter_amd.ops import probe

    n, k = 512, 512
    a = torch.eye(n, k, device="cuda:0").to(torch.bfloat16)
    g = torch.Generator(device="cuda:0").manual_seed(7)
    b = torch.randn(k, n, device="cuda:0", generator=g).to(torch.bfloat16)  # distinct values
    c = probe.gemm_nt(a, b.t().contiguous(), variant=variant)
    assert torch.equal(c, b)


def test_gemm_nt256_throughput():
    from gpumounter_amd.ops import probe

    tf = probe.gemm_tflops(0, 4096, 4096, 4096, 10)
    print(f"gemm_nt 4096^3 bf16 {tf:.0f} TF/s")
    assert tf > 300, tf


def test_burn_in_is_bit_exact_and_sustained():
    from gpumounter_amd.ops import probe

    r = probe.burn_in(0, seconds=2.0, n=4096)
    print(r)
    assert r["ok"] and r["mismatches"] == 0, r
    assert r["iterations"] >= 8 and r["tflops"] > 300, r


def test_probe_cli_burn_in():
    res = subprocess.run([sys.executable, "-m", "gpumounter_amd", "probe", "--burn-in", "1"],
                         capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr[-2000:]
    import json
    out = json.loads(res.stdout)
    assert out and all(r["burn_in"]["ok"] for r in out), out


def test_doctor_gpu_checks_pass():
    """``doctor --gpu --burn-in 1``: every HIP GPU of the box runs the liveness kernel and a
    short bit-checked GEMM load; the amdsmi inventory and HIP agree on the BDFs."""
    import json

    res = subprocess.run([sys.executable, "-m", "gpumounter_amd", "doctor", "--json",
                          "--skip-cluster", "--gpu", "--burn-in", "1"],
                         capture_output=True, text=True, timeout=180,
                         env={**os.environ, "GM_SYSTEMD_DEVICE_ALLOW": "off"})
    checks = json.loads(res.stdout)
    gpu = [c for c in checks if c["name"].startswith("gpu")]
    assert gpu and all(c["status"] == "ok" for c in gpu), gpu
    assert all("0 mismatching words" in c["detail"] for c in gpu if c["name"] != "gpu"), gpu
    # the box runs us in a container's PID namespace, with KFD's process table readable
    (pidns,) = [c for c in checks if c["name"] == "pidns"]
    assert "KFD process table readable" in pidns["detail"], pidns


def test_gemm_check_host_reference():
    from gpumounter_amd.ops import probe

    r = probe.gemm_check(0, 128, 128, 256)
    assert r["max_abs_err"] < 1e-3 * r["ref_scale"] + 1e-3, r


def test_roctx_library_loads():
    from gpumounter_amd import _native

    assert _native.host().gm_roctx_available() == 1


def test_p2p_if_multi_gpu():
    from gpumounter_amd.ops import probe
    from gpumounter_amd.parallel.collectives import xgmi_matrix

    if probe.device_count() < 2:
        pytest.skip("single-GPU box")
    m = xgmi_matrix([0, 1], 64 << 20, 3)
    assert m["peer"][0][1]
    assert m["gbps"][0][1] > 10


def test_rank_pool_rccl_child_on_the_attached_gpu():
    """bench.py's single-process N>1 path: a rank process spawned by a parent that has not touched
    the GPU binds to the attached GPU by PCI address and runs a checked RCCL all-reduce."""
    import subprocess as sp
    code = ("import json; from gpumounter_amd.parallel.rankpool import RankPool; "
            "from gpumounter_amd.hw.inventory import Inventory; "
            "bdf = Inventory('').gpus()[0].bdf; p = RankPool(1); "
            "r = [p.allreduce([bdf]) for _ in range(2)]; print(json.dumps(r[-1])); "
            "print(json.dumps(p.close()))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = sp.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True,
                 timeout=180)
    assert res.returncode == 0, res.stderr[-3000:]
    out = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    import json
    r = json.loads(out[0])
    assert r["ok"] and r["backend"] == "nccl" and r["ms"] > 0
    assert json.loads(out[1]) == {"0": 0}


def test_unknown_gemm_schedule_is_rejected():
    from gpumounter_amd import _native
    lib = _native.probe()
    assert lib.gm_probe_gemm_nt_variant(3, None, None, None, 256, 256, 64, None) != 0


def _hip_child_code() -> str:
    return ("import torch, time, sys; x = torch.ones(1 << 20, device='cuda:0'); "
            "torch.cuda.synchronize(); print('ready', flush=True); time.sleep(120)")


def test_e2e_attach_verify_detach_real_inventory(real_inventory):
    """Full hot-mount cycle with the real amdsmi inventory; tenant-side kernel on the GPU."""
    from gpumounter_amd.fakes.harness import LocalCluster
    from gpumounter_amd.ops import probe

    bdf0 = probe.props(0)["pci_bus_id"]

    async def run():
        async with LocalCluster(amdsmi_lib="", cgroup_mode="v2", node_gpu_bdfs=[bdf0]) as lc:
            lc.tenant("t")
            code, body = await lc.add("default", "t", 1)
            assert code == 200, body
            assert body["devices"][0]["bdf"] == bdf0
            assert not await lc.audit("default", "t")
            cid = lc.container_ids("default", "t")[0]
            rm = body["devices"][0]["render_minor"]
            assert f"dev/dri/renderD{rm}" in lc.nodes["node-0"].node.container_devices(cid)
            assert probe.verify([bdf0])[0].quick_us > 0
            code, body2 = await lc.remove("default", "t", [body["devices"][0]["uuid"]])
            assert code == 200, body2
            assert not await lc.audit("default", "t")
    asyncio.run(run())


def test_daemons_as_processes_with_real_inventory(real_inventory):
    """The production entry points as separate processes (worker on the real libamd_smi),
    configured by GM_* env only; the attached GPU runs the gfx950 liveness kernel here."""
    from gpumounter_amd.fakes.deployment import ProcessCluster
    from gpumounter_amd.ops import probe

    bdf0 = probe.props(0)["pci_bus_id"]
    pc = ProcessCluster(amdsmi_lib="", gpu_bdfs=[bdf0])
    try:
        pc.start()
        pc.tenant("t")
        code, body = pc.add("default", "t", 1)
        assert code == 200, body
        assert body["devices"][0]["bdf"] == bdf0
        assert pc.audit("default", "t") == []
        assert probe.verify([bdf0])[0].quick_us > 0
        code, body2 = pc.remove("default", "t", [body["devices"][0]["uuid"]])
        assert code == 200, body2
        assert pc.audit("default", "t") == []
    finally:
        codes = pc.stop()
    assert set(codes.values()) == {0}, codes


def test_busy_detection_with_real_hip_process(real_inventory):
    """A real HIP process inside the tenant cgroup makes the GPU busy (amdsmi process list or the
    /proc fd fallback); force=true removes it and terminates the process."""
    from gpumounter_amd.fakes.harness import LocalCluster
    from gpumounter_amd.ops import probe

    bdf0 = probe.props(0)["pci_bus_id"]
    child = subprocess.Popen([sys.executable, "-c", _hip_child_code()], stdout=subprocess.PIPE,
                             text=True)
    try:
        assert child.stdout.readline().strip() == "ready"

        async def run():
            async with LocalCluster(amdsmi_lib="", cgroup_mode="v2",
                                    node_gpu_bdfs=[bdf0]) as lc:
                lc.tenant("busy", pids={"main": [child.pid]})
                smi_pids = [p.pid for p in lc.inventory.processes(0)]
                print(f"amdsmi process list for gpu0: {smi_pids} (child {child.pid})")
                code, body = await lc.add("default", "busy", 1)
                assert code == 200, body
                uuid = body["devices"][0]["uuid"]
                code, b2 = await lc.remove("default", "busy", [uuid], force=False)
                assert code == 400 and "running processes" in b2["message"], b2
                code, b3 = await lc.remove("default", "busy", [uuid], force=True)
                assert code == 200, b3
                assert child.pid in b3["killed_pids"]
        asyncio.run(run())
        t0 = time.time()
        while child.poll() is None and time.time() - t0 < 15:
            time.sleep(0.1)
        assert child.poll() is not None, "force removal did not terminate the GPU process"
    finally:
        if child.poll() is None:
            child.kill()
        child.wait()


def test_kfd_table_names_tenant_by_host_pid(real_inventory):
    """KFD's sysfs process table and amdsmi's list agree, name a tenant by its host-namespace
    PID (the box runs us in a container: the child's own PID is another number), and carry its
    VRAM; outside the host PID namespace busy detection leaves both tables out and still finds
    the tenant through its render fd."""
    from gpumounter_amd.node import procs

    inv = real_inventory
    g = inv.gpus()[0]
    assert g.kfd_gpu_id
    before = procs.kfd_table().get(g.kfd_gpu_id, {})
    child = subprocess.Popen([sys.executable, "-c", _hip_child_code()], stdout=subprocess.PIPE,
                             text=True)
    try:
        assert child.stdout.readline().strip() == "ready"
        table = procs.kfd_table().get(g.kfd_gpu_id, {})
        smi = {p.pid: p.vram_bytes for p in inv.processes(g.index)}
        new = {p: v for p, v in table.items() if p not in before}
        print(f"kfd table gpu {g.kfd_gpu_id}: {table}; amdsmi: {smi}; child {child.pid}")
        assert len(new) == 1, new
        (hpid, vram), = new.items()
        assert vram >= 4 << 20                     # the child's 4 MiB tensor, at least
        assert smi.get(hpid) == vram               # amdsmi reads the same table
        host = procs.host_pid_ns()
        assert (hpid == child.pid) == host
        busy = procs.busy_pids(inv, [g], [child.pid], mode="both", tables=host)
        assert busy == {g.index: [child.pid]}
    finally:
        child.kill()
        child.wait()
    t0 = time.time()
    while hpid in procs.kfd_table().get(g.kfd_gpu_id, {}) and time.time() - t0 < 10:
        time.sleep(0.1)
    assert hpid not in procs.kfd_table().get(g.kfd_gpu_id, {})


def test_tenant_validate_tool_runs_kernel_p2p_and_rccl():
    """``python -m gpumounter_amd.parallel.validate``: liveness kernel on every visible GPU,
    pairwise peer copies, an RCCL all-reduce with one process per GPU, and the bf16 burn-in."""
    import json

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, "-m", "gpumounter_amd.parallel.validate",
                          "--numel", str(1 << 22), "--burn-in", "1"], cwd=root,
                         capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, (res.stdout[-2000:], res.stderr[-3000:])
    rep = json.loads(res.stdout.strip().splitlines()[-1])
    assert rep["ok"] and rep["gpus"] and all(g["arch"].startswith("gfx950") for g in rep["gpus"])
    assert rep["allreduce"]["world"] == len(rep["gpus"]) and rep["allreduce"]["ok"]
    # per GPU: the bf16 GEMM burn-in
    assert len(rep["burn_in"]) == len(rep["gpus"]) and all(b["ok"] for b in rep["burn_in"])
    print(json.dumps(rep["allreduce"]))


def test_tenant_side_hip_sees_the_gpu_only_while_attached(real_inventory):
    """BASELINE config "attach 1 MI355X to a running Pod; the Pod sees it", from the tenant's
    side: a fresh HIP process in the tenant's view of /dev and of its device cgroup (the
    emulated node operations, resolved by libgm_tenant_view.so — the box allows no namespaces)
    enumerates no GPU before the attach, exactly the attached one after it, none after the
    detach; and it runs the gfx950 liveness kernel on it."""
    from gpumounter_amd.fakes.harness import LocalCluster
    from gpumounter_amd.ops import probe, tenant

    bdf0 = probe.props(0)["pci_bus_id"].lower()

    async def run():
        async with LocalCluster(amdsmi_lib="", cgroup_mode="v2", node_gpu_bdfs=[bdf0]) as lc:
            lc.tenant("t")
            cid = lc.container_ids("default", "t")[0]
            ctr = lc.nodes["node-0"].node.container(cid)
            view = (ctr.root_dir, ctr.cgroup_dir)
            before = await asyncio.to_thread(tenant.hip_devices, *view)
            assert before["count"] == 0, before
            code, body = await lc.add("default", "t", 1)
            assert code == 200, body
            during = await asyncio.to_thread(tenant.hip_devices, *view)
            assert during["count"] == 1 and during["bdfs"] == [bdf0], during
            code, _ = await lc.remove("default", "t", [body["devices"][0]["uuid"]])
            assert code == 200
            after = await asyncio.to_thread(tenant.hip_devices, *view)
            assert after["count"] == 0, after
            print("tenant view:", before, during, after)
    asyncio.run(run())


def test_tenant_side_pytorch_uses_the_gpu_only_while_attached(real_inventory):
    """The BASELINE config names a rocm/pytorch Pod: a fresh PyTorch process in the tenant's
    view sees no GPU before the attach; after it, exactly the attached GPU (same BDF, gfx950),
    on which a bf16 GEMM matches an fp32 host reference; none after the detach."""
    from gpumounter_amd.fakes.harness import LocalCluster
    from gpumounter_amd.ops import probe, tenant

    bdf0 = probe.props(0)["pci_bus_id"].lower()

    async def run():
        async with LocalCluster(amdsmi_lib="", cgroup_mode="v2", node_gpu_bdfs=[bdf0]) as lc:
            lc.tenant("pt")
            cid = lc.container_ids("default", "pt")[0]
            ctr = lc.nodes["node-0"].node.container(cid)
            view = (ctr.root_dir, ctr.cgroup_dir)
            before = await asyncio.to_thread(tenant.torch_devices, *view)
            assert before["count"] == 0, before
            code, body = await lc.add("default", "pt", 1)
            assert code == 200, body
            during = await asyncio.to_thread(tenant.torch_devices, *view)
            assert during["count"] == 1 and during["bdfs"] == [bdf0], during
            assert during["arch"].startswith("gfx950"), during
            assert during["gemm_max_rel_err"] < 1e-2, during
            code, _ = await lc.remove("default", "pt", [body["devices"][0]["uuid"]])
            assert code == 200
            after = await asyncio.to_thread(tenant.torch_devices, *view)
            assert after["count"] == 0, after
            print("tenant-side PyTorch:", before, during, after)
    asyncio.run(run())


def test_force_remove_waits_for_a_sigterm_ignoring_hip_process(real_inventory):
    """A real HIP process that ignores SIGTERM and holds 16 GiB of HBM: force removal revokes
    access, escalates to SIGKILL after the grace, and releases the placeholder only after the
    process (and its KFD context) is gone — the GPU is never schedulable while the tenant can
    still reach it through an open fd."""
    from gpumounter_amd.fakes.harness import LocalCluster
    from gpumounter_amd.ops import probe

    bdf0 = probe.props(0)["pci_bus_id"]
    code = ("import signal, time, torch; signal.signal(signal.SIGTERM, signal.SIG_IGN); "
            "x = torch.empty(16 << 30, dtype=torch.uint8, device='cuda:0'); x.fill_(1); "
            "torch.cuda.synchronize(); print('ready', flush=True); time.sleep(120)")
    child = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
    try:
        assert child.stdout.readline().strip() == "ready"

        async def run():
            async with LocalCluster(amdsmi_lib="", cgroup_mode="v2", node_gpu_bdfs=[bdf0],
                                    worker_overrides={"kill_grace_s": 0.5}) as lc:
                lc.tenant("busy", pids={"main": [child.pid]})
                code, body = await lc.add("default", "busy", 1)
                assert code == 200, body
                t0 = time.perf_counter()
                code, b2 = await lc.remove("default", "busy", [body["devices"][0]["uuid"]],
                                           force=True)
                dt = time.perf_counter() - t0
                assert code == 200 and child.pid in b2["killed_pids"], b2
                assert child.poll() == -9, "the GPU was released before its process exited"
                assert lc.cluster.placeholders() == []
                print(f"force removal with SIGKILL escalation: {dt * 1e3:.1f} ms")
                assert dt >= 0.5
        asyncio.run(run())
    finally:
        if child.poll() is None:
            child.kill()
        child.wait()


def test_tenant_view_needs_the_render_node_and_its_grant(tmp_path, real_inventory):
    """What the tenant-side view rests on, checked against the real ROCm stack: /dev/kfd alone
    exposes no GPU (ROCm skips a GPU whose render node it cannot open); a render node without
    the device-cgroup grant exposes none either; node + grant expose exactly that GPU."""
    import json
    import os as _os

    from gpumounter_amd.ops import probe, tenant

    g = next(x for x in real_inventory.gpus()
             if x.bdf == probe.props(0)["pci_bus_id"].lower())
    kfd = real_inventory.kfd_major
    root, cg = tmp_path / "root", tmp_path / "cg"
    (root / "dev" / "dri").mkdir(parents=True)
    cg.mkdir()
    (root / "dev" / "kfd").write_text(f"gm-chr {kfd}:0\n")
    grants = [[2, kfd, 0, 6]]
    (cg / "gm.bpf.json").write_text(json.dumps({"set": grants}))
    only_kfd = tenant.hip_devices(str(root), str(cg))
    assert only_kfd["count"] == 0, only_kfd
    (root / "dev" / "dri" / f"renderD{g.render_minor}").write_text(
        f"gm-chr 226:{g.render_minor}\n")
    no_grant = tenant.hip_devices(str(root), str(cg))
    assert no_grant["count"] == 0, no_grant
    grants.append([2, 226, g.render_minor, 6])
    (cg / "gm.bpf.json").write_text(json.dumps({"set": grants}))
    both = tenant.hip_devices(str(root), str(cg))
    assert both["count"] == 1 and both["bdfs"] == [g.bdf], both
    print("kfd only:", only_kfd, "render without grant:", no_grant, "both:", both)
    assert _os.path.exists("/dev/kfd")
