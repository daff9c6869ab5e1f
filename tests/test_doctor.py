"""``gpumounter_amd doctor``: node preflight against a hermetic node (gpumounter_amd/utils/doctor.py)."""
import asyncio
import os
import subprocess
import sys

from gpumounter_amd.fakes.harness import LocalCluster
from gpumounter_amd.utils import doctor
from gpumounter_amd.utils.config import Config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_doctor_reports_a_healthy_hermetic_node():
    async def main():
        async with LocalCluster(cgroup_mode="v2", start_master=False) as lc:
            h = lc.nodes["node-0"]
            cfg = Config.load(env={}, amdsmi_lib="mock", kube_api=lc.api_url,
                              kubelet_socket=h.kubelet.socket_path,
                              cgroup_root=h.node.cgroup_root, cgroup_mode="v2",
                              bpf_pin_dir="", systemd_device_allow="off")
            # doctor.run drives its own event loop for the cluster checks
            return await asyncio.get_running_loop().run_in_executor(None, doctor.run, cfg)
    checks = {c.name: c for c in asyncio.run(main())}
    for name in ("amdsmi", "xgmi", "cgroup", "kubelet", "apiserver", "systemd"):
        assert checks[name].status == "ok", (name, checks[name])
    assert "8 GPU(s)" in checks["amdsmi"].detail and "gfx950" in checks["amdsmi"].detail
    assert "PodResources v1" in checks["kubelet"].detail
    assert checks["bpf"].status in ("ok", "fail")       # root with CAP_BPF here, or not


def test_doctor_cli_exit_code_and_json():
    env = {**os.environ, "GM_AMDSMI_LIB": "mock", "GM_KUBELET_SOCKET": "/nonexistent.sock",
           "GM_CGROUP_ROOT": "/nonexistent-cgroup"}
    res = subprocess.run([sys.executable, "-m", "gpumounter_amd", "doctor", "--json"], cwd=ROOT,
                         capture_output=True, text=True, timeout=120, env=env)
    assert res.returncode == 1, res.stderr[-2000:]
    import json
    checks = {c["name"]: c for c in json.loads(res.stdout)}
    assert checks["amdsmi"]["status"] == "ok"
    assert checks["cgroup"]["status"] == "fail" and checks["kubelet"]["status"] == "fail"


def test_doctor_gpu_check_fails_cleanly_without_a_gpu():
    """``doctor --gpu`` on a host whose GPUs HIP cannot see reports a failed check (exit 1)
    instead of crashing; on the MI355X box tests/test_gpu.py runs the passing case."""
    import torch

    if torch.cuda.is_available():
        import pytest
        pytest.skip("GPU present: covered by test_gpu.py::test_doctor_gpu_checks_pass")
    cfg = Config.load(env={}, amdsmi_lib="mock")
    checks = doctor.check_gpus(cfg)
    assert checks and all(c.status == "fail" for c in checks), checks
    assert checks[0].name == "gpu"


def test_doctor_reports_bind_mode_for_user_namespaced_pods():
    import os

    from gpumounter_amd.utils import doctor
    from gpumounter_amd.utils.config import Config

    (c,) = doctor.check_devnodes(Config(devnode_userns="off"))
    assert c.status == "ok" and "not used" in c.detail
    (c,) = doctor.check_devnodes(Config())
    if os.geteuid() == 0:
        assert c.status == "ok", c.detail            # CAP_SYS_ADMIN: open_tree works
    else:
        assert c.status == "warn" and "hostUsers" in c.detail


def test_doctor_reports_the_pid_namespace(tmp_path, monkeypatch):
    from gpumounter_amd.node import procs

    (tmp_path / "4242").mkdir()
    (tmp_path / "4242" / "vram_49070").write_text("4096\n")
    cfg = Config(kfd_proc_path=str(tmp_path))
    monkeypatch.setattr(procs, "host_pid_ns", lambda proc_root="/proc": True)
    (c,) = doctor.check_pidns(cfg)
    assert c.status == "ok" and "1 process(es)" in c.detail, c
    monkeypatch.setattr(procs, "host_pid_ns", lambda proc_root="/proc": False)
    (c,) = doctor.check_pidns(Config(kfd_proc_path=str(tmp_path / "none")))
    assert c.status == "warn" and "hostPID: true" in c.detail and "amdsmi's is used" in c.detail
