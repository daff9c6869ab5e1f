"""Full-stack attach/detach against a real kernel (root with mount + bpf; GM_PRIVILEGED_TESTS=0/1 forces off/on, root).

Runs tests/priv_e2e_driver.py in its own process (the mock inventory is configured through
GM_AMDSMI_MOCK_CONFIG at amdsmi init). See the driver docstring for the setup.
"""
import json
import os
import subprocess
import sys

import pytest
from conftest import privileged_skip

pytestmark = [pytest.mark.privileged, privileged_skip()]

HERE = os.path.dirname(os.path.abspath(__file__))


def test_full_stack_attach_detach_enforced_by_the_kernel(tmp_path):
    cfg = tmp_path / "mock.json"
    # "GPUs" whose render/card nodes are memory devices: 1:5 /dev/zero, 1:7 /dev/full,
    # 1:8 /dev/random, 1:9 /dev/urandom (drm_major=1 in the driver); kfd → 1:0
    cfg.write_text(json.dumps({"gpus": [
        {"bdf": "0000:05:00.0", "render": 5, "card": 7, "numa": 0},
        {"bdf": "0000:15:00.0", "render": 8, "card": 9, "numa": 0}]}))
    r = subprocess.run([sys.executable, os.path.join(HERE, "priv_e2e_driver.py")],
                       env={**os.environ, "GM_AMDSMI_MOCK_CONFIG": str(cfg)},
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    o = json.loads(r.stdout.strip().splitlines()[-1])
    assert o["backend"] == "cgroup-v2-bpf" and o["tenant_in_cgroup"]
    # [null, zero, full, random] as seen by a process inside the tenant's cgroup
    assert o["before"] == "1000"                              # runc program: /dev/null only
    assert o["add1"][0] == 200 and o["after_add1"] == "1110"  # + render 1:5, card 1:7
    assert o["progs_after_add1"] == ["gm_devallow"]           # replaced, not stacked
    assert o["nodes_after_add1"] == {"/dev/kfd": [1, 0], "/dev/dri/renderD5": [1, 5],
                                     "/dev/dri/card7": [1, 7]}
    assert o["host_dev_untouched"] and o["audit_after_add1"] == []
    # the probes join the tenant's cgroup from the worker's mount namespace: the worker
    # writes nodes only through the tenant's own process, never into its own /dev
    assert o["host_dev_untouched_at_end"]
    assert o["add2"][0] == 200 and o["after_add2"] == "1111"
    assert o["remove1"] == 200 and o["after_remove1"] == "1001"
    assert o["nodes_after_remove1"] == {"/dev/kfd": [1, 0], "/dev/dri/renderD5": None,
                                        "/dev/dri/renderD8": [1, 8]}
    assert o["remove2"] == 200 and o["after_remove2"] == "1000"
    assert o["progs_final"] == ["runc_devices"]               # runtime program restored
    assert o["nodes_final"] == {"/dev/kfd": None, "/dev/dri/renderD8": None}
    assert o["audit_final"] == [] and o["pins_left"] == []
    # the runtime attaches a fresh program next to ours: the GPU is cut, and the device guard
    # (shipped 1 s period) re-wraps the stack within 1.5 s — not at the 30 s sweep
    assert o["guard_add"] == 200 and o["guard_before_swap"] == "1110"
    assert o["guard_right_after_swap"] == "1000"
    assert o["guard_after"] == "1110" and o["guard_restored_s"] <= 1.5, o
    assert o["guard_repairs"] >= 1
    assert o["guard_remove"] == 200 and o["guard_final"] == "1000"
    assert o["guard_audit_final"] == []
    # a tenant whose /dev is a bind of the host's keeps every node through attach + sweep
    assert o["shared_sees_host_dev"] and o["shared_add"] == 200 and o["shared_gpus"] == [5, 8]
    assert o["shared_after_add_unchanged"] and o["shared_after_sweep_unchanged"]
    assert o["shared_host_listing"] == ["dri/card7", "dri/renderD5", "kfd"]
    # a tenant in its own user namespace (nodev /dev): bind-mounted nodes it can open, allowed
    # by the device program; nothing left after the detach
    assert o["userns_before"] == "00"
    assert o["userns_add"] == [200, [5]] and o["userns_after_add"] == "11"
    assert o["userns_audit"] == [] and o["userns_remove"] == 200
    assert o["userns_after_remove"] == "00"
    assert o["userns_nodes_final"] == {"/dev/dri/renderD5": None, "/dev/dri/card7": None,
                                       "/dev/kfd": None}


def test_soak_and_contention_on_real_kernel_objects_leave_nothing_behind():
    """bench/configs.py --node-ops real: tenants are real processes in real cgroups with a
    runc-style program; after the soak every tenant is back to the runtime's own program with
    no grant, no GPU node and no pin left; under contention the kernel's grants and nodes match
    the ledger (0 invariant violations)."""
    root = os.path.dirname(HERE)
    for scenario, extra in (("soak", ["--cycles", "40"]), ("contention", ["--rounds", "10"])):
        r = subprocess.run([sys.executable, os.path.join(root, "bench", "configs.py"), scenario,
                            "--node-ops", "real", *extra], capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-4000:]
        o = json.loads(r.stdout.strip().splitlines()[-1])
        k = o["kernel"]
        if scenario == "soak":
            assert o["orphaned_cgroup_entries"] == 0 and o["orphaned_device_nodes"] == 0
            assert set(map(tuple, k["programs"].values())) == {("runc_devices",)}
            assert all(g == [] for g in k["grants"].values()) and k["pins_left"] == []
            assert all(n == [] for n in k["dev_nodes"].values())
        else:
            assert o["invariant_violations"] == 0
            for t, grants in k["grants"].items():
                # every GPU the kernel grants has its render and card node in the tenant
                renders = {f"dri/renderD{mi}" for ma, mi in grants if ma == 226 and mi >= 128}
                assert renders <= set(k["dev_nodes"][t]), (t, grants, k["dev_nodes"][t])
                assert (k["programs"][t] == ["runc_devices"]) == (grants == [])
