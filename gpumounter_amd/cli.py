"""Command line: daemons and operator tools.

    python -m gpumounter_amd master   [--config f.yaml] [--port 8080]
    python -m gpumounter_amd worker   [--config f.yaml] [--node NAME]
    python -m gpumounter_amd inventory [--amdsmi mock]          # amdsmi view of this node
    python -m gpumounter_amd topology  [--amdsmi mock] [-n 4]   # xGMI/NUMA placement preview
    python -m gpumounter_amd probe     [--bdf 0000:05:00.0] [--full] [--burn-in 60]  # gfx950 kernels
    python -m gpumounter_amd add    --master URL --ns NS --pod P -n 2 [--entire] [--lease 3600]
    python -m gpumounter_amd remove --master URL --ns NS --pod P --uuid U [--uuid U2] [--force]
    python -m gpumounter_amd status --master URL --node NODE
    python -m gpumounter_amd bpf-dump --allow 226:128 --allow 511:0   # generated device program
    python -m gpumounter_amd doctor  [--json] [--skip-cluster] [--gpu [--burn-in 30]]  # preflight
    python -m gpumounter_amd config-doc > docs/CONFIG.md   # every GM_* setting, from the source

The reference ships only the two daemons and documents curl calls (QuickStart.md:41-92); the
``add``/``remove`` commands speak exactly those HTTP routes.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
from typing import List, Optional


def _cfg(args, **over):
    from gpumounter_amd.utils.config import Config

    return Config.load(getattr(args, "config", None), **over)


def _run_daemon(serve, cfg) -> int:
    """asyncio.run(serve(cfg)); with GM_PROFILE_OUT=<file> under cProfile, stats written at
    (SIGTERM-clean) shutdown — for finding the hot spots of a live daemon (``{pid}`` in the
    name is replaced, so several daemons can share the setting)."""
    if getattr(cfg, "cpu_affinity", ""):
        from gpumounter_amd.utils import runtime
        runtime.pin_cpus(cfg.cpu_affinity)
    out = os.environ.get("GM_PROFILE_OUT", "").replace("{pid}", str(os.getpid()))
    if not out:
        asyncio.run(serve(cfg))
        return 0
    if os.environ.get("GM_PROFILE_MODE", "cprofile") == "sample":
        # statistical: setitimer(ITIMER_PROF) stack samples (gpumounter_amd/utils/sampler.py)
        from gpumounter_amd.utils.sampler import Sampler

        smp = Sampler(1.0 / float(os.environ.get("GM_PROFILE_HZ", "2000")))
        smp.start()
        try:
            asyncio.run(serve(cfg))
        finally:
            smp.stop()
            smp.dump(out, {"argv": sys.argv[1:]})
        return 0
    import cProfile

    prof = cProfile.Profile()
    prof.enable()
    try:
        asyncio.run(serve(cfg))
    finally:
        prof.disable()
        prof.dump_stats(out)
    return 0


def cmd_master(args) -> int:
    from gpumounter_amd.master.app import serve
    from gpumounter_amd.utils import log

    cfg = _cfg(args, master_port=args.port)
    log.setup(cfg.log_level, cfg.log_json, cfg.log_file)
    return _run_daemon(serve, cfg)


def cmd_worker(args) -> int:
    from gpumounter_amd.utils import log
    from gpumounter_amd.worker.server import serve

    cfg = _cfg(args, node_name=args.node, worker_port=args.port)
    log.setup(cfg.log_level, cfg.log_json, cfg.log_file)
    return _run_daemon(serve, cfg)


def cmd_device_plugin(args) -> int:
    """Standalone amd.com/gpu device plugin (topology-packed allocation for ordinary pods, no
    hot-mount worker). Runs until SIGTERM/SIGINT."""
    import signal

    from gpumounter_amd.deviceplugin.plugin import AmdGpuDevicePlugin
    from gpumounter_amd.hw.inventory import Inventory
    from gpumounter_amd.utils import log

    cfg = _cfg(args)
    log.setup(cfg.log_level, cfg.log_json, cfg.log_file)
    inv = Inventory(args.amdsmi if args.amdsmi is not None else cfg.amdsmi_lib, cfg.kfd_major,
                    cfg.kfd_dev_path)

    async def run():
        plugin = AmdGpuDevicePlugin(inv, cfg.resource_name, args.dir or cfg.device_plugin_dir,
                                    inject_devices=cfg.device_plugin_inject,
                                    health_period_s=cfg.device_plugin_health_s,
                                    policy=cfg.topology_policy)
        await plugin.start(register=not args.no_register)
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGTERM, signal.SIGINT):
            loop.add_signal_handler(sig, stop.set)
        print(json.dumps({"socket": plugin.socket_path, "devices": len(plugin.health)}),
              flush=True)
        await stop.wait()
        await plugin.stop()

    asyncio.run(run())
    return 0


def cmd_inventory(args) -> int:
    from gpumounter_amd.hw.inventory import Inventory

    inv = Inventory(args.amdsmi)
    out = inv.summary()
    if args.processes:
        out["processes"] = {g.index: [p.__dict__ for p in inv.processes(g.index)]
                            for g in inv.gpus()}
    print(json.dumps(out, indent=2))
    return 0


def cmd_topology(args) -> int:
    from gpumounter_amd.hw import topology
    from gpumounter_amd.hw.inventory import Inventory

    inv = Inventory(args.amdsmi)
    gpus = inv.gpus()
    out = {"describe": topology.describe(gpus, inv.links()), "plans": {}}
    for n in ([args.n] if args.n else range(1, len(gpus) + 1)):
        p = topology.choose(gpus, n, inv.links(), policy=args.policy)
        out["plans"][n] = p.to_dict() if p else None
    print(json.dumps(out, indent=2))
    return 0


def cmd_probe(args) -> int:
    from gpumounter_amd.ops import probe

    if args.bdf:
        bdfs = args.bdf
    else:
        bdfs = [probe.props(i)["pci_bus_id"] for i in range(probe.device_count())]
    res = [r.to_dict() for r in probe.verify(bdfs, full=args.full)]
    bad = False
    if args.burn_in:
        for r in res:
            r["burn_in"] = probe.burn_in(r["device"], args.burn_in)
            bad |= not r["burn_in"]["ok"]
    print(json.dumps(res, indent=2))
    return 1 if bad else 0


SA_TOKEN = "/var/run/secrets/kubernetes.io/serviceaccount/token"


def client_token(args) -> str:
    """The bearer token the master authenticates (GM_AUTHZ_MODE=kube: the caller's own
    Kubernetes token; GM_API_TOKEN: the shared one). First of: --token, $GM_TOKEN,
    --token-file, the pod's service-account token, the current kubeconfig user's token."""
    if getattr(args, "token", ""):
        return args.token
    if os.environ.get("GM_TOKEN"):
        return os.environ["GM_TOKEN"]
    for path in (getattr(args, "token_file", ""), SA_TOKEN):
        if path and os.path.exists(path):
            with open(path, encoding="utf-8") as fh:
                return fh.read().strip()
    kc = os.environ.get("KUBECONFIG", "").split(os.pathsep)[0] or \
        os.path.expanduser("~/.kube/config")
    if os.path.exists(kc):
        import yaml
        try:
            with open(kc, encoding="utf-8") as fh:
                doc = yaml.safe_load(fh) or {}
            ctx = next(c["context"] for c in doc.get("contexts", [])
                       if c["name"] == doc.get("current-context"))
            user = next((u["user"] for u in doc.get("users", [])
                         if u["name"] == ctx.get("user")), {})
            return user.get("token", "")
        except (OSError, ValueError, KeyError, StopIteration, yaml.YAMLError):
            return ""
    return ""


def client_tls(args):
    """How an https master is verified: against --ca / $GM_MASTER_CA, the system roots
    otherwise; --insecure skips verification (labs only). None for http URLs."""
    import ssl

    if not getattr(args, "master", "").startswith("https://"):
        return None
    if getattr(args, "insecure", False):
        return False
    ca = getattr(args, "ca", "") or os.environ.get("GM_MASTER_CA", "")
    return ssl.create_default_context(cafile=ca or None)


async def _http(method: str, url: str, data=None, token: str = "", tls=None) -> int:
    import aiohttp

    headers = {"Accept": "application/json"}
    if token:
        headers["Authorization"] = f"Bearer {token}"
        if url.startswith("http://") and not url.startswith(("http://127.", "http://localhost")):
            print("warning: sending a bearer token over plain HTTP; use the master's https:// "
                  "URL", file=sys.stderr)
    async with aiohttp.ClientSession() as s:
        async with s.request(method, url, data=data, headers=headers,
                             ssl=tls if tls is not None else True) as r:
            body = await r.text()
            print(body)
            if r.status == 401 and not token:
                print("unauthorized: the master wants a bearer token (--token, $GM_TOKEN, "
                      "--token-file or a kubeconfig user token)", file=sys.stderr)
            return 0 if r.status == 200 else 1


def cmd_add(args) -> int:
    from urllib.parse import urlencode

    url = (f"{args.master.rstrip('/')}/addgpu/namespace/{args.ns}/pod/{args.pod}/gpu/{args.n}/"
           f"isEntireMount/{'true' if args.entire else 'false'}")
    q = {k: v for k, v in (("container", args.container), ("lease", args.lease)) if v}
    if q:
        url += "?" + urlencode(q)
    return asyncio.run(_http("GET", url, token=client_token(args), tls=client_tls(args)))


def cmd_remove(args) -> int:
    import aiohttp

    url = (f"{args.master.rstrip('/')}/removegpu/namespace/{args.ns}/pod/{args.pod}/force/"
           f"{'true' if args.force else 'false'}")
    data = aiohttp.FormData()
    for u in args.uuid:
        data.add_field("uuids", u)
    return asyncio.run(_http("POST", url, data, token=client_token(args), tls=client_tls(args)))


def cmd_status(args) -> int:
    if args.pod:
        url = f"{args.master.rstrip('/')}/api/v1/namespaces/{args.ns}/pods/{args.pod}/gpus"
    else:
        url = f"{args.master.rstrip('/')}/api/v1/nodes/{args.node}/gpus"
    return asyncio.run(_http("GET", url, token=client_token(args), tls=client_tls(args)))


def disassemble(insns: List[int]) -> List[str]:
    from gpumounter_amd.node import bpfvm

    names = {0x61: "ldxw", 0xbf: "mov64", 0xb7: "mov64", 0x57: "and64", 0x77: "rsh64",
             0x55: "jne", 0x85: "call", 0x95: "exit", 0x18: "lddw"}
    out = []
    skip = False
    for i, raw in enumerate(insns):
        if skip:
            skip = False
            continue
        code, dst, src, off, imm = bpfvm.decode(raw)
        op = names.get(code, f"op{code:#x}")
        if code == 0x61:
            out.append(f"{i:3d}: r{dst} = *(u32 *)(r{src} + {off})")
        elif code == 0xbf:
            out.append(f"{i:3d}: r{dst} = r{src}")
        elif code == 0xb7:
            out.append(f"{i:3d}: r{dst} = {imm}")
        elif code == 0x57:
            out.append(f"{i:3d}: r{dst} &= {imm & 0xffffffff:#x}")
        elif code == 0x77:
            out.append(f"{i:3d}: r{dst} >>= {imm}")
        elif code == 0x55:
            out.append(f"{i:3d}: if r{dst} != {imm} goto +{off}")
        elif code == 0x18:
            out.append(f"{i:3d}: r{dst} = map[prog_array fd={imm}]")
            skip = True
        elif code == 0x85:
            out.append(f"{i:3d}: call bpf_tail_call#{imm}")
        elif code == 0x95:
            out.append(f"{i:3d}: exit")
        else:
            out.append(f"{i:3d}: {op} dst=r{dst} src=r{src} off={off} imm={imm}")
    return out


def cmd_bpf_dump(args) -> int:
    from gpumounter_amd.models.device import DeviceNode
    from gpumounter_amd.node.cgroup import build_program

    nodes = []
    for a in args.allow:
        ma, mi = a.split(":")
        nodes.append(DeviceNode(f"/dev/x{ma}_{mi}", int(ma), int(mi)))
    prog = build_program(nodes, chained=not args.unchained)
    print("\n".join(disassemble(prog)))
    return 0


def cmd_doctor(args) -> int:
    from gpumounter_amd.utils import doctor

    cfg = _cfg(args)
    checks = doctor.run(cfg, skip_cluster=args.skip_cluster, gpu=args.gpu or bool(args.burn_in),
                        burn_in_s=args.burn_in)
    print(doctor.render(checks, args.json))
    return 1 if any(c.status == "fail" for c in checks) else 0


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="gpumounter_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("master")
    p.add_argument("--config")
    p.add_argument("--port", type=int)
    p.set_defaults(fn=cmd_master)
    p = sub.add_parser("worker")
    p.add_argument("--config")
    p.add_argument("--node")
    p.add_argument("--port", type=int)
    p.set_defaults(fn=cmd_worker)
    p = sub.add_parser("device-plugin")
    p.add_argument("--config")
    p.add_argument("--amdsmi", default=None)
    p.add_argument("--dir", default="", help="kubelet device-plugin directory")
    p.add_argument("--no-register", action="store_true", help="serve only (testing)")
    p.set_defaults(fn=cmd_device_plugin)
    p = sub.add_parser("inventory")
    p.add_argument("--amdsmi", default="")
    p.add_argument("--processes", action="store_true")
    p.set_defaults(fn=cmd_inventory)
    p = sub.add_parser("topology")
    p.add_argument("--amdsmi", default="")
    p.add_argument("-n", type=int, default=0)
    p.add_argument("--policy", default="xgmi", choices=("xgmi", "first-fit"))
    p.set_defaults(fn=cmd_topology)
    p = sub.add_parser("probe")
    p.add_argument("--bdf", action="append")
    p.add_argument("--full", action="store_true")
    p.add_argument("--burn-in", type=float, default=0.0, metavar="SECONDS",
                   help="sustained GEMM load with bit-exact result checks (exit 1 on mismatch)")
    p.set_defaults(fn=cmd_probe)
    for name, fn in (("add", cmd_add), ("remove", cmd_remove), ("status", cmd_status)):
        p = sub.add_parser(name)
        p.add_argument("--master", default="http://127.0.0.1:8080")
        p.add_argument("--ns", default="default")
        p.add_argument("--pod", default="")
        p.add_argument("--token", default="", help="bearer token for the master (default: "
                       "$GM_TOKEN, --token-file, the service-account token, the kubeconfig "
                       "user's token)")
        p.add_argument("--token-file", default="")
        p.add_argument("--ca", default="", help="CA bundle that signed the master's HTTPS "
                       "certificate (default: $GM_MASTER_CA, else the system roots)")
        p.add_argument("--insecure", action="store_true",
                       help="do not verify the master's HTTPS certificate (labs only)")
        if name == "add":
            p.add_argument("-n", type=int, required=True)
            p.add_argument("--entire", action="store_true")
            p.add_argument("--container", default="")
            p.add_argument("--lease", default="", help="seconds until automatic detach")
        if name == "remove":
            p.add_argument("--uuid", action="append", required=True)
            p.add_argument("--force", action="store_true")
        if name == "status":
            p.add_argument("--node", default="")
        p.set_defaults(fn=fn)
    p = sub.add_parser("doctor", help="node preflight: amdsmi, cgroup/bpf, systemd, kubelet, "
                                      "apiserver")
    p.add_argument("--config")
    p.add_argument("--json", action="store_true")
    p.add_argument("--skip-cluster", action="store_true",
                   help="skip the kubelet and apiserver checks")
    p.add_argument("--gpu", action="store_true",
                   help="also run the gfx950 liveness kernel on every GPU")
    p.add_argument("--burn-in", type=float, default=0.0, metavar="SECONDS",
                   help="with --gpu: sustained bit-checked GEMM load per GPU")
    p.set_defaults(fn=cmd_doctor)
    p = sub.add_parser("bpf-dump")
    p.add_argument("--allow", action="append", default=[])
    p.add_argument("--unchained", action="store_true")
    p.set_defaults(fn=cmd_bpf_dump)
    p = sub.add_parser("config-doc")
    p.add_argument("--metrics", action="store_true", help="the metrics reference instead")
    p.set_defaults(fn=cmd_config_doc)
    return ap


def cmd_config_doc(args) -> int:
    from gpumounter_amd.utils.configdoc import render, render_metrics
    sys.stdout.write(render_metrics() if args.metrics else render())
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    args = build_parser().parse_args(argv)
    return args.fn(args)


if __name__ == "__main__":
    sys.exit(main())
