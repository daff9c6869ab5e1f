#!/usr/bin/env python3
"""Headline benchmark: p50 GPU attach latency at N MI355X per Pod (BASELINE.json metric).

One "step" = the full hot-mount cycle a user drives through the master's HTTP API:
  1. ``GET /addgpu/.../gpu/N/isEntireMount/true``   → placeholder ledger + cgroup rule + /dev nodes
     (timed at the client: this is the attach latency reported as ``value``)
  2. consistency audit: ledger == cgroup rules == device nodes for the tenant pod
  3. every rank runs the gfx950 liveness kernel on "its" newly attached GPU (found by PCI address)
     and, for N>1, an RCCL all-reduce over the attached set (tenant-side proof the GPUs work)
  4. ``POST /removegpu/.../force/false``            → revoke + unlink + ledger release
The control plane (apiserver, scheduler, kubelet PodResources) is the hermetic fake; inventory,
topology and process tables come from the real libamd_smi through the C++ shim, the node
operations run the production C++ code against a temp-dir cgroupfs/rootfs (the GPU box is
unprivileged), and the probe kernels run on the real GPUs. By default (``--deploy processes``)
the fake control plane, the worker and the master are separate processes started through the
production entry points, as deployed; ``--deploy inprocess`` runs them on one event loop.
After the timed loop the reference's call sequence is re-enacted in the same deployment shape
(``reference_emulated_same_run``, gpumounter_amd/fakes/refproto.py).

Launch: ``python bench.py --gpus 1`` or, for N>1, under torch.distributed.run with one rank per GPU.
Rank 0 hosts the control plane; all ranks take part in verification. Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pct(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    k = (len(xs) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


def calls_summary(runs) -> dict:
    """Per process: calls by kind and serial round trips, from the cycle with the median
    number of serial round trips (all cycles' round trips listed too)."""
    from gpumounter_amd.utils import calls
    # Events are queued and sent once no operation is in flight (worker/notify.py): they can
    # land in the window but are never waited for
    per = [{who: calls.summary([c for c in cs if c[2] != "apiserver POST events"])
            for who, cs in run.items()} for run in runs]
    depth = [sum(p["serial_round_trips"] for p in r.values()) for r in per]
    mid = sorted(range(len(per)), key=lambda i: depth[i])[len(per) // 2]
    return {"by_process": per[mid], "serial_round_trips": depth[mid],
            "serial_round_trips_all_cycles": depth}


class _LocalCP:
    """Control-plane adapter: everything on one event loop thread (LocalCluster)."""

    def __init__(self, tc, lc) -> None:
        self.tc, self.lc = tc, lc

    def add(self, n: int, entire: bool):
        return self.tc.call(self.lc.add("default", "tenant", n, entire=entire))

    def remove(self, uuids):
        return self.tc.call(self.lc.remove("default", "tenant", uuids))

    def audit(self) -> list:
        return self.tc.call(self.lc.audit("default", "tenant"))

    def placeholders_left(self) -> int:
        return len(self.lc.cluster.placeholders())

    def kubelet_calls(self) -> dict:
        return dict(self.lc.nodes["node-0"].kubelet.calls)

    def corrections(self) -> int:
        return int(self.lc.nodes["node-0"].worker.metrics.placement_corrections._value.get())

    def admission_refusals(self) -> dict:
        m = self.lc.nodes["node-0"].worker.metrics.admission_refusals
        return {s.labels["outcome"]: int(s.value) for metric in m.collect()
                for s in metric.samples if s.name.endswith("_total")}

    def tenant_view(self):
        node = self.lc.nodes["node-0"].node
        (c,) = [c for c in node.containers.values() if c.pod_name == "tenant"]
        return c.root_dir, c.cgroup_dir

    def calls(self, t0: float, t1: float) -> dict:
        from gpumounter_amd.utils import calls   # one process: master and worker share the log
        return {"master+worker": calls.since(t0, t1)}

    def wait_pool(self, want: int) -> None:
        pool = self.lc.nodes["node-0"].worker.pool
        t_wait = time.time()
        while len(pool.standby()) < want:
            if time.time() - t_wait > 120:
                raise RuntimeError("warm pool did not fill")
            time.sleep(0.001)

    def stop(self) -> None:
        self.tc.stop()


class _ProcCP:
    """Control-plane adapter: apiserver, worker and master in separate processes."""

    def __init__(self, pc) -> None:
        self.pc = pc

    def add(self, n: int, entire: bool):
        return self.pc.add("default", "tenant", n, entire)

    def remove(self, uuids):
        return self.pc.remove("default", "tenant", uuids)

    def audit(self) -> list:
        return self.pc.audit("default", "tenant")

    def placeholders_left(self) -> int:
        return len(self.pc.placeholders())

    def kubelet_calls(self) -> dict:
        return self.pc.kubelet_calls()

    def corrections(self) -> int:
        for ln in self.pc.worker_metrics().splitlines():
            if ln.startswith("gm_placement_corrections_total "):
                return int(float(ln.split()[1]))
        return 0

    def admission_refusals(self) -> dict:
        out = {}
        for ln in self.pc.worker_metrics().splitlines():
            if ln.startswith("gm_admission_refusals_total{"):
                outcome = ln.split('outcome="', 1)[1].split('"', 1)[0]
                out[outcome] = int(float(ln.split()[-1]))
        return out

    def tenant_view(self):
        from gpumounter_amd.ops import tenant
        cs = self.pc.tenant_pod["status"]["containerStatuses"]
        cid = cs[0]["containerID"].split("://", 1)[1]
        n = self.pc.info["nodes"]["node-0"]
        return tenant.locate(n["rootfs_root"], n["cgroup_root"], cid)

    def calls(self, t0: float, t1: float) -> dict:
        return self.pc.calls(t0, t1)

    def expire_authz(self, age: bool = True) -> None:
        """Age the master's cached authz answers (as a long idle would), same process;
        ``age=False`` sends the same request and ages nothing (the control cycles)."""
        code, body = self.pc.http("POST", "/debug/authz-expire" + ("" if age else "?age=0"))
        if code != 200:
            raise RuntimeError(f"authz expire: {code} {body[:200]!r}")

    def wait_pool(self, want: int) -> None:
        """Until ``want`` standby placeholders are admitted (the kubelet has posted their
        container statuses), as the in-process adapter's ``pool.standby()`` counts them."""
        from gpumounter_amd.models.types import ANN_MOUNT_MODE, MODE_STANDBY
        t_wait = time.time()
        while sum(1 for p in self.pc.placeholders()
                  if (p["metadata"].get("annotations") or {}).get(ANN_MOUNT_MODE) == MODE_STANDBY
                  and not p["metadata"].get("deletionTimestamp")
                  and (p.get("status") or {}).get("containerStatuses")) < want:
            if time.time() - t_wait > 120:
                raise RuntimeError("warm pool did not fill")
            time.sleep(0.002)

    def stop(self) -> None:
        codes = self.pc.stop()
        if any(c != 0 for c in codes.values()):
            print(f"daemon exit codes: {codes}", file=sys.stderr)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--mode", choices=("entire", "single"), default="entire")
    ap.add_argument("--latency", choices=("zero", "realistic"), default="zero",
                    help="fake control-plane latency model (zero = controller overhead only)")
    ap.add_argument("--amdsmi", default="", help='"" = real libamd_smi, "mock" = bundled mock')
    ap.add_argument("--cgroup", choices=("v1", "v2"), default="v2")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--warm-pool", type=int, default=0,
                    help="standby placeholders per node (claim instead of create); 0 = off")
    ap.add_argument("--placement", choices=("auto", "hint", "trim"), default="auto",
                    help="placement_enforce: auto (default) = correct a worse-placed plugin "
                         "choice by holding the other free GPUs; trim = always hold every free "
                         "GPU and release the surplus; hint = annotation only")
    ap.add_argument("--device-plugin", action="store_true",
                    help="the worker serves amd.com/gpu itself; the fake kubelet's device manager "
                         "calls GetPreferredAllocation/Allocate on it at admission")
    ap.add_argument("--ref-steps", type=int, default=0,
                    help="after the timed loop, re-run this many attach/detach cycles with the "
                         "emulated reference protocol on the same cluster (only with --latency "
                         "zero and no warm pool). Off by default: it compares call sequences on "
                         "a zero-latency fake, not a published reference figure")
    ap.add_argument("--deploy", choices=("inprocess", "processes"), default="processes",
                    help="processes: fake control plane, worker and master each in their own "
                         "process via the production entry points (gpumounter_amd/fakes/"
                         "deployment.py); inprocess: all on one event loop (LocalCluster)")
    ap.add_argument("--protocol", choices=("gpumounter", "reference"), default="gpumounter",
                    help="'reference' re-enacts the reference's call sequence on the same "
                         "cluster (emulated baseline, see gpumounter_amd/fakes/refproto.py)")
    ap.add_argument("--node-ops", choices=("emulated", "real"), default="emulated",
                    help="real (root): a private cgroup2 mount with a runc-style device program, "
                         "real BPF_PROG_LOAD/verify/BPF_F_REPLACE attach and mknodat into a "
                         "tenant in its own mount namespace (gpumounter_amd/fakes/realnode.py); "
                         "emulated: the JSON-recording cgroup-v2 backend and marker files, for "
                         "unprivileged boxes")
    ap.add_argument("--kernel-fs", choices=("tmpfs", "disk"), default="tmpfs",
                    help="where the emulated node keeps its cgroupfs and container /dev trees: "
                         "tmpfs (/dev/shm; a real node's are kernfs/tmpfs, in memory) or the "
                         "working directory's disk. The worker's journal is on disk either way. "
                         "The reference column uses the same choice")
    ap.add_argument("--security", choices=("shipped", "off"), default="shipped",
                    help="shipped: master⇄worker mTLS and TokenReview/SubjectAccessReview authz "
                         "as the manifests deploy them (--deploy processes); off: insecure gRPC, "
                         "no authz (the reference's posture)")
    ap.add_argument("--dump-samples", default="",
                    help="write every timed attach (wall time, client ms, worker stage ms) as "
                         "JSON lines to this file, for tail-latency analysis")
    ap.add_argument("--log-dir", default="",
                    help="--deploy processes: keep the daemons' logs in this directory")
    ap.add_argument("--cold-steps", type=int, default=10,
                    help="after the timed loop (--deploy processes): restart the master with "
                         "authz TTLs of --idle-s/2 and time this many attaches, each after "
                         "--idle-s of idleness, so each one finds its TokenReview and "
                         "SubjectAccessReview answers expired (cold_attach_p50_ms); 0 = skip")
    ap.add_argument("--idle-s", type=float, default=0.3,
                    help="idle time before each cold attach (see --cold-steps)")
    ap.add_argument("--no-calib", action="store_true",
                    help="skip the box calibration (CPU loop, process pingpong, gRPC floor) "
                         "recorded as \"box\" in the JSON")
    ap.add_argument("--pin", default="",
                    help="--deploy processes: pin the worker and the master to CPUs "
                         "(\"WORKER_CPUS:MASTER_CPUS\", cpuset lists, e.g. \"8:9\"; config "
                         "cpu_affinity, as with a static CPU manager); \"\" = unpinned")
    ap.add_argument("--daemon-env", action="append", default=[], metavar="KEY=VALUE",
                    help="--deploy processes: an environment setting for both daemons (a GM_* "
                         "config override, e.g. GM_AUTHZ_SELF_REVIEW=false); repeatable")
    ap.add_argument("--call-cycles", type=int, default=5,
                    help="after the timed loop: this many attach/detach cycles whose outbound "
                         "apiserver/kubelet calls are read from the daemons' call logs "
                         "(serial_calls_per_attach / _detach); 0 = skip")
    ap.add_argument("--gpu-api", choices=("device-plugin", "dra"), default="device-plugin",
                    help="dra: the node's GPUs come from a DRA driver; placeholders hold "
                         "ResourceClaims (gpu_allocation=dra)")
    args = ap.parse_args()
    # the amdgpu driver's KFD topology, not a /dev/kfd node (which any test or tool can mknod)
    if args.amdsmi == "mock" and os.path.isdir("/sys/class/kfd/kfd/topology/nodes"):
        # on a GPU box the mock inventory's GPUs are not the box's: the control plane is
        # measured alone (without a GPU the rank check still runs, on gloo)
        args.no_verify = True
    if args.gpu_api == "dra":
        if args.protocol == "reference" or args.device_plugin:
            print("--gpu-api dra: the reference protocol and the device plugin are "
                  "extended-resource models", file=sys.stderr)
            return 2
        args.ref_steps = 0
    if args.node_ops == "real":
        if args.deploy == "processes" and "--deploy" in sys.argv:
            print("--node-ops real runs --deploy inprocess", file=sys.stderr)
        args.deploy = "inprocess"
        args.cgroup = "v2"

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n = args.gpus
    box = None
    if rank == 0 and not args.no_calib:
        # the box's speed next to the value (gpumounter_amd/utils/calib.py): before anything
        # initialises the GPU, since the calibration forks and spawns
        from gpumounter_amd.utils import calib
        box = calib.measure(grpc_floor=True,
                            idle_s=args.idle_s if args.cold_steps > 0 else 0.0)
    if world > 1 and world != n:
        print(f"WORLD_SIZE={world} must equal --gpus={n}", file=sys.stderr)
        return 2

    # Single-process N>1 (the driver may run `bench.py --gpus 8` without a launcher): the
    # collective check needs one process per GPU, so N rank processes are spawned here, before
    # this process touches the GPU (a GPU-initialised process must never exec anything).
    rank_pool = None
    if world == 1 and n > 1 and not args.no_verify:
        from gpumounter_amd.parallel.rankpool import RankPool
        rank_pool = RankPool(n)

    import torch
    import torch.distributed as dist

    from gpumounter_amd.utils import log
    log.setup("WARNING", json_format=False)
    has_gpu = torch.cuda.is_available()
    if has_gpu:
        torch.cuda.set_device(local_rank % max(torch.cuda.device_count(), 1))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from gpumounter_amd.ops import probe

    visible = []
    if has_gpu:
        visible = [probe.props(i)["pci_bus_id"] for i in range(probe.device_count())]

    tc = lc = cp = None
    sleeper = None
    sandbox = None
    info = {}
    if rank == 0:
        from gpumounter_amd.fakes.apiserver import LatencyModel
        from gpumounter_amd.fakes.harness import ThreadedCluster
        from gpumounter_amd.hw.inventory import Inventory
        amdsmi = args.amdsmi if (has_gpu or args.amdsmi) else "mock"
        inv = Inventory(amdsmi)
        bdfs = [g.bdf for g in inv.gpus()]
        node_bdfs = [b for b in bdfs if b in visible] if visible and args.amdsmi != "mock" \
            else bdfs
        if len(node_bdfs) < n:
            print(f"need {n} GPUs visible to HIP and amdsmi; have {node_bdfs} (amdsmi {bdfs}, "
                  f"HIP {visible})", file=sys.stderr)
            return 3
        if args.node_ops == "real":
            from gpumounter_amd.fakes.realnode import RealNodeSandbox
            sandbox = RealNodeSandbox().__enter__()
            tenant_pid = sandbox.tenant_pid
        else:
            # its own stdio: if this process dies, it must not hold the caller's pipe open
            sleeper = subprocess.Popen(["sleep", "infinity"], stdin=subprocess.DEVNULL,
                                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            tenant_pid = sleeper.pid
            import atexit
            atexit.register(sleeper.kill)      # also when the setup below fails
        if args.deploy == "processes":
            if args.device_plugin:
                print("--device-plugin needs --deploy inprocess (the fake kubelet drives the "
                      "plugin in-process)", file=sys.stderr)
                return 2
            from gpumounter_amd.fakes.deployment import ProcessCluster
            wpin, _, mpin = args.pin.partition(":")
            denv = dict(kv.split("=", 1) for kv in args.daemon_env)
            pc = ProcessCluster(amdsmi_lib=amdsmi, cgroup_mode=args.cgroup, latency=args.latency,
                                gpu_bdfs=node_bdfs, protocol=args.protocol,
                                secure=args.security == "shipped" and args.protocol == "gpumounter",
                                gpu_api=args.gpu_api, log_dir=args.log_dir,
                                kernel_fs=args.kernel_fs,
                                worker_env={"GM_WARM_POOL_SIZE": str(args.warm_pool),
                                            "GM_PLACEMENT_ENFORCE": args.placement,
                                            **({"GM_CPU_AFFINITY": wpin} if wpin else {}),
                                            **denv},
                                master_env={**({"GM_CPU_AFFINITY": mpin} if mpin else {}),
                                            **denv}).start()
            pc.tenant_pod = pc.tenant("tenant", pids={"main": [tenant_pid]})
            cp = _ProcCP(pc)
        else:
            lat = LatencyModel.realistic() if args.latency == "realistic" else LatencyModel()
            wov = {"warm_pool_size": args.warm_pool, "placement_enforce": args.placement,
                   "gc_tune": True}   # as the daemons run
            kw = {}
            if sandbox is not None:
                wov["bpf_pin_dir"] = sandbox.bpffs
                kw = {"cgroup_root": sandbox.cgroup_root, "devnode_mode": "procroot"}
            elif args.kernel_fs == "tmpfs" and os.access("/dev/shm", os.W_OK):
                import tempfile
                kw = {"kernel_fs_dir": tempfile.mkdtemp(prefix="gm-kfs-", dir="/dev/shm")}
            tc = ThreadedCluster(amdsmi_lib=amdsmi, cgroup_mode=args.cgroup, latency=lat,
                                 node_gpu_bdfs=node_bdfs, device_plugin=args.device_plugin,
                                 worker_overrides=wov, master_overrides={"gc_tune": True},
                                 gpu_api=args.gpu_api, **kw)
            lc = tc.start()
            if args.protocol == "reference":
                from gpumounter_amd.fakes import refproto
                refproto.install(lc)
            lc.tenant("tenant", pids={"main": [tenant_pid]})
            if sandbox is not None:
                from gpumounter_amd.fakes.realnode import attach_runtime_program
                (ctr,) = [c for c in lc.nodes["node-0"].node.containers.values()
                          if c.pod_name == "tenant"]
                attach_runtime_program(ctr.cgroup_dir)
            cp = _LocalCP(tc, lc)
        if args.warm_pool:
            cp.wait_pool(min(args.warm_pool, len(node_bdfs)))
        info = {"amdsmi_lib": inv.lib_path, "node_gpus": len(node_bdfs),
                "amdsmi_gpus": len(bdfs), "gfx": sorted({g.gfx_target for g in inv.gpus()}),
                "hives": sorted({hex(g.xgmi_hive_id) for g in inv.gpus()})}
        gpu_by_bdf = {g.bdf: g for g in inv.gpus()}
        link_matrix = inv.links()

    nccl_group = None
    bound_dev = [None]
    pool_cap = info.get("node_gpus", 0) if rank == 0 else 0
    attach_ms, detach_ms, audit_issues, probe_us, stage = [], [], 0, [], {}
    dstage = {}          # detach: worker stage name → ms per timed detach
    mstage = {}          # attach: master stage name → ms (gm:master_* spans)
    hop_ms = []          # (master handler ms, worker ms) per timed attach
    ar_ms = []
    probe_by_gpu = {}
    last_bdfs = []
    ar_backend = [None]
    samples = [] if args.dump_samples and rank == 0 else None
    first_attach = []    # the first attach after the daemons started (cold everything)
    first_stages = {}    # ... and where its time went

    def one_step(record: bool):
        nonlocal audit_issues, nccl_group
        obj = [None]
        if rank == 0:
            t0 = time.perf_counter()
            code, body = cp.add(n, args.mode == "entire")
            t1 = time.perf_counter()
            if code != 200:
                raise RuntimeError(f"attach failed: {code} {body}")
            if not first_attach:
                first_attach.append((t1 - t0) * 1e3)
                mc = body.get("master_clock") or {}
                if mc:   # perf_counter is CLOCK_MONOTONIC, the master's clock, on Linux
                    first_stages.update({
                        "http.request_leg": round((mc["in"] - t0) * 1e3, 4),
                        "http.master_in_to_out": round((mc["out"] - mc["in"]) * 1e3, 4),
                        "http.response_leg": round((t1 - mc["out"]) * 1e3, 4)})
                first_stages.update({"client": round((t1 - t0) * 1e3, 4),
                                     "master": body.get("master_ms"),
                                     "worker": body.get("total_ms"),
                                     **{f"master.{t['name']}": t["ms"]
                                        for t in body.get("master_timings", [])},
                                     **{f"worker.{t['name']}": t["ms"]
                                        for t in body.get("timings", [])
                                        if "." not in t["name"]}})
            issues = cp.audit() if args.protocol == "gpumounter" else []
            obj = [{"bdfs": [d["bdf"] for d in body["devices"]],
                    "uuids": [d["uuid"] for d in body["devices"]],
                    "ms": (t1 - t0) * 1e3, "issues": len(issues),
                    "master_ms": body.get("master_ms"), "worker_ms": body.get("total_ms"),
                    "timings": {t["name"]: t["ms"] for t in body.get("timings", [])},
                    "mtimings": {t["name"]: t["ms"] for t in body.get("master_timings", [])}}]
        if world > 1:
            dist.broadcast_object_list(obj, src=0)
        st = obj[0]
        last_bdfs[:] = st["bdfs"]
        if has_gpu and not args.no_verify:
            bdfs = sorted(st["bdfs"])           # stable rank → attached-GPU mapping
            # one process per GPU: each rank checks its own; a single process checks them all
            mine_all = bdfs if world == 1 else [bdfs[rank % len(bdfs)]]
            for mine in mine_all:
                dev = probe.find_device(mine)
                if dev < 0:
                    raise RuntimeError(f"rank {rank}: attached GPU {mine} not visible to HIP")
                us = probe.quick(dev)
                if record:
                    probe_us.append(us)
                    probe_by_gpu.setdefault(mine, []).append(us)
            if world > 1:
                if nccl_group is None:
                    torch.cuda.set_device(dev)
                    nccl_group = dist.new_group(backend="nccl")
                    bound_dev[0] = dev
                elif bound_dev[0] != dev:
                    raise RuntimeError(f"rank {rank}: attached set changed between steps "
                                       f"({bound_dev[0]} → {dev}); placement must be stable")
                x = torch.ones(1 << 20, dtype=torch.bfloat16, device=f"cuda:{dev}")
                ta = time.perf_counter()
                dist.all_reduce(x, group=nccl_group)
                torch.cuda.synchronize(dev)
                if record:
                    ar_ms.append((time.perf_counter() - ta) * 1e3)
                if float(x[0].item()) != float(world):
                    raise RuntimeError("RCCL all-reduce over the attached GPUs returned wrong sum")
                ar_backend[0] = "nccl"
        if rank_pool is not None:
            r = rank_pool.allreduce(st["bdfs"])
            if not r["ok"]:
                raise RuntimeError(f"all-reduce over the attached GPUs failed: {r}")
            ar_backend[0] = r["backend"]
            if record:
                ar_ms.append(r["ms"])
        if world > 1:
            dist.barrier()
        if rank == 0:
            t0 = time.perf_counter()
            code, body = cp.remove(st["uuids"])
            t1 = time.perf_counter()
            if code != 200:
                raise RuntimeError(f"detach failed: {code} {body}")
            if args.warm_pool:   # steady state: the next attach finds a full pool
                cp.wait_pool(min(args.warm_pool, pool_cap))
            if record:
                attach_ms.append(st["ms"])
                if st.get("master_ms") is not None and st.get("worker_ms") is not None:
                    hop_ms.append((st["master_ms"], st["worker_ms"]))
                detach_ms.append((t1 - t0) * 1e3)
                for t in (body.get("timings") or []) if isinstance(body, dict) else []:
                    dstage.setdefault(t["name"], []).append(t["ms"])
                if samples is not None:
                    samples.append({"t": round(time.time(), 4), "attach_ms": round(st["ms"], 4),
                                    "detach_ms": round((t1 - t0) * 1e3, 4),
                                    "stages": st["timings"], "master": st["mtimings"],
                                    "worker_ms": st.get("worker_ms")})
                audit_issues += st["issues"]
                for k, v in st["timings"].items():
                    stage.setdefault(k, []).append(v)
                for k, v in st["mtimings"].items():
                    mstage.setdefault(k, []).append(v)

    last_note = [time.time()]

    def progress(phase: str, i: int, total: int) -> None:
        """A line on stderr at most every 10 s, so long runs (realistic control plane: the
        reference's detach waits out a 30 s grace period) visibly make progress."""
        if rank == 0 and time.time() - last_note[0] > 10:
            last_note[0] = time.time()
            print(f"bench: {phase} step {i}/{total}", file=sys.stderr, flush=True)

    # The client side of the measurement is this process (torch imported, the fake control
    # plane's handles): a full collection of that heap during a timed request would be charged
    # to the attach. Freeze what exists now, as the daemons do (utils/runtime.py).
    from gpumounter_amd.utils import runtime
    runtime.tune_gc()
    runtime.watch_gc_pauses(5.0)
    try:
        for i in range(args.warmup):
            one_step(False)
            progress("warmup", i + 1, args.warmup)
        if world > 1:
            dist.barrier()
        if has_gpu:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            one_step(True)
            progress("timed", i + 1, args.steps)
        if world > 1:
            dist.barrier()
        if has_gpu:
            torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        ms_per_step = elapsed * 1e3 / args.steps
        if box is not None:
            calib_after = calib.py_loop_us()   # no fork now: this process holds the GPU
        if world > 1:
            t = torch.tensor([ms_per_step], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ms_per_step = float(t.item())
        if rank == 0:
            # the attached set, from amdsmi: one hive, every pair on a direct xGMI link
            from gpumounter_amd.hw import topology
            att = {gpu_by_bdf[b].index: gpu_by_bdf[b] for b in last_bdfs if b in gpu_by_bdf}
            _, att_hives, att_numa, att_nx = topology.score_set(att, link_matrix, sorted(att))
            p2p = None
            if has_gpu and not args.no_verify and len(last_bdfs) > 1:
                devs = [probe.find_device(b) for b in sorted(last_bdfs)]
                pairs = [probe.p2p(a, b, 64 << 20, 3) for a in devs for b in devs if a != b]
                p2p = {"pairs": len(pairs),
                       "all_peer_access": all(x["peer_access"] for x in pairs),
                       "min_gbps": round(min(x["gbps"] for x in pairs), 1),
                       "max_gbps": round(max(x["gbps"] for x in pairs), 1)}
            tenant_view = tenant_view_pt = None
            if has_gpu and not args.no_verify and args.node_ops == "emulated" and \
                    args.protocol == "gpumounter" and args.cgroup == "v2":
                # BASELINE config "the Pod sees it", from a fresh tenant-side HIP process
                from gpumounter_amd.ops import tenant
                root, cg = cp.tenant_view()
                held = {}

                def _attach():
                    code, body = cp.add(n, args.mode == "entire")
                    if code != 200:
                        raise RuntimeError(f"attach failed: {code} {body}")
                    held["uuids"] = [d["uuid"] for d in body["devices"]]
                    return [d["bdf"] for d in body["devices"]]

                def _detach():
                    code, body = cp.remove(held["uuids"])
                    if code != 200:
                        raise RuntimeError(f"detach failed: {code} {body}")
                try:
                    tenant_view = tenant.check_attach_cycle(_attach, _detach, root, cg)
                except Exception as e:  # noqa: BLE001 - reported, never fatal to the bench
                    tenant_view = {"ok": False, "error": str(e)[-500:]}
                if not tenant_view["ok"]:
                    print(f"bench: tenant-side view check failed: {tenant_view}",
                          file=sys.stderr)
                # "a running rocm/pytorch Pod": the same cycle seen by a fresh PyTorch process,
                # which runs a bf16 GEMM on what it got
                try:
                    tenant_view_pt = tenant.check_attach_cycle(_attach, _detach, root, cg,
                                                               runtime="pytorch")
                except Exception as e:  # noqa: BLE001 - reported, never fatal to the bench
                    tenant_view_pt = {"ok": False, "error": str(e)[-500:]}
                if not tenant_view_pt["ok"]:
                    print(f"bench: tenant-side PyTorch check failed: {tenant_view_pt}",
                          file=sys.stderr)
            # the control-plane calls one attach and one detach wait for, counted on the fake:
            # by kind, and how many of them are serial (a real cluster charges each serial round
            # trip a millisecond or more; gpumounter_amd/utils/calls.py)
            accounting = None
            if args.protocol == "gpumounter" and args.call_cycles > 0:
                acc = {"attach": [], "detach": []}
                waits = []
                for i in range(args.call_cycles):
                    time.sleep(0.02)               # quiet: nothing else in the window
                    ta = time.monotonic()
                    code, body = cp.add(n, args.mode == "entire")
                    tb = time.monotonic()
                    if code != 200:
                        raise RuntimeError(f"attach failed: {code} {body}")
                    code, body2 = cp.remove([d["uuid"] for d in body["devices"]])
                    tc = time.monotonic()
                    if code != 200:
                        raise RuntimeError(f"detach failed: {code} {body2}")
                    if args.warm_pool:
                        cp.wait_pool(min(args.warm_pool, pool_cap))
                    logs = cp.calls(ta, tc)
                    for op, (lo, hi) in (("attach", (ta, tb)), ("detach", (tb, tc))):
                        acc[op].append({who: [c for c in cs if lo <= c[0] <= hi]
                                        for who, cs in logs.items()})
                    # besides calls, an attach that creates placeholders waits for the scheduler
                    # to bind them and the kubelet to admit them (no call of ours: a watch / the
                    # checkpoint tells); a warm-pool claim does not
                    st = {t["name"]: t["ms"] for t in body.get("timings", [])}
                    waits.append(st.get("placeholder_wait"))
                accounting = {op: calls_summary(runs) for op, runs in acc.items()}
                w = [x for x in waits if x is not None]
                accounting["attach"]["admission_waits"] = 1 if len(w) * 2 > len(waits) else 0
                accounting["attach"]["admission_wait_p50_ms"] = round(pct(w, 0.5), 4) \
                    if w else None
            cold = None
            if args.cold_steps > 0 and args.protocol == "gpumounter":
                # the attach an operator makes minutes after the last one: every cached authz
                # answer expired (the pod index is a watch, so it stays current). Two kinds of
                # cold cycle, interleaved A B A B on the same master process (round 5 ran all A
                # before a master restart and all B after it, and B came out faster than A with
                # more work: the order and the fresh process, not the work, decided):
                #   A "idle": idle_s of idle, authz answers still cached
                #   B "cold": idle_s of idle, authz answers expired (TokenReview + SAR again)
                # Before each attach both send one request to the master's debug port (B's ages
                # the caches, A's does not): what remains between them is the review itself
                expire = cp.expire_authz if args.deploy == "processes" else None
                runs = {"idle": ([], {}), "cold": ([], {})}

                def cycle(kind):
                    cms, cst = runs[kind]
                    time.sleep(args.idle_s)
                    if expire is not None:
                        # both kinds send the same request to the master first (only "cold"
                        # ages the caches), so both wake the master the same way
                        expire(kind == "cold")
                    ta = time.perf_counter()
                    code, body = cp.add(n, args.mode == "entire")
                    tb = time.perf_counter()
                    if code != 200:
                        raise RuntimeError(f"{kind} attach failed: {code} {body}")
                    cms.append((tb - ta) * 1e3)
                    for t in body.get("master_timings", []) + [
                            {"name": "worker", "ms": body.get("total_ms", 0.0)}] + [
                            {"name": f"worker.{t['name']}", "ms": t["ms"]}
                            for t in body.get("timings", []) if "." not in t["name"]]:
                        cst.setdefault(t["name"], []).append(t["ms"])
                    mc = body.get("master_clock") or {}
                    if mc:
                        for k, v in (("http.request_leg", mc["in"] - ta),
                                     ("http.response_leg", tb - mc["out"])):
                            cst.setdefault(k, []).append(v * 1e3)
                    code, body = cp.remove([d["uuid"] for d in body["devices"]])
                    if code != 200:
                        raise RuntimeError(f"{kind} detach failed: {code} {body}")

                def summary(kind):
                    cms, cst = runs[kind]
                    return {"attach_p50_ms": round(pct(cms, 0.5), 4),
                            "attach_max_ms": round(max(cms), 4),
                            "attach_ms": [round(x, 4) for x in cms],
                            "stage_p50_ms": {k: round(pct(v, 0.5), 4)
                                             for k, v in sorted(cst.items())}}
                kinds = ("idle", "cold") if expire is not None else ("idle",)
                for i in range(args.cold_steps):
                    for kind in (kinds if i % 2 == 0 else kinds[::-1]):   # ABBA ABBA: no
                        cycle(kind)                                        # kind always first
                    progress("cold", i + 1, args.cold_steps)
                idle_only = summary("idle")
                if expire is not None:
                    cold = {"steps": args.cold_steps, "idle_s": args.idle_s,
                            "authz": "expired", "order": "ABBA, one master process",
                            **summary("cold"), "idle_only": idle_only}
                else:        # one process, no authz (LocalCluster): idling alone
                    cold = {"steps": args.cold_steps, "idle_s": args.idle_s,
                            "authz": None, **idle_only, "idle_only": idle_only}
            orphan_issues = len(cp.audit()) if args.protocol == "gpumounter" else None
            corrections = cp.corrections() if args.protocol == "gpumounter" else None
            refusals = cp.admission_refusals() if args.protocol == "gpumounter" else None
            placeholders_left = cp.placeholders_left()
            kcalls = cp.kubelet_calls()
            p50 = pct(attach_ms, 0.5)
            ref = None
            if args.ref_steps > 0 and args.node_ops == "real":
                # the reference writes cgroup-v1 devices.allow/deny through `sh -c echo`
                # (pkg/util/cgroup/cgroup.go:143-169); the real-node sandbox is cgroup2, which
                # has no such files, so there is nothing faithful to re-enact here
                ref = {"skipped": "the reference's node operations are cgroup-v1 only "
                                  "(devices.allow via sh); --node-ops real runs on cgroup2"}
            elif args.ref_steps > 0 and args.protocol == "gpumounter" and \
                    args.latency == "zero" and not args.warm_pool:
                # the reference's call sequence, emulated in the same deployment shape
                # The reference dials the kubelet and Lists on every query with no retry
                # (collector.go:90-138): against the kubelet's PodResources limiter (100 qps,
                # burst 10) it fails requests. Its cycles are therefore timed on a kubelet that
                # serves every call and only counts those a limited kubelet would reject.
                if lc is not None:
                    from gpumounter_amd.fakes import refproto
                    refproto.install(lc)
                    for h in lc.nodes.values():
                        h.kubelet.limit_mode = "count"
                    ref_cp = cp
                else:
                    cp.stop()
                    from gpumounter_amd.fakes.deployment import ProcessCluster
                    rpc = ProcessCluster(amdsmi_lib=amdsmi, cgroup_mode=args.cgroup,
                                         gpu_bdfs=node_bdfs, protocol="reference",
                                         kubelet_limit="count", kernel_fs=args.kernel_fs).start()
                    rpc.tenant("tenant", pids={"main": [sleeper.pid]})
                    cp = ref_cp = _ProcCP(rpc)
                ra, rd = [], []
                k0 = ref_cp.kubelet_calls()
                for i in range(args.ref_steps + 2):
                    ta = time.perf_counter()
                    code, body = ref_cp.add(n, args.mode == "entire")
                    tb = time.perf_counter()
                    if code != 200:
                        raise RuntimeError(f"reference attach failed: {code} {body}")
                    code, body = ref_cp.remove([d["uuid"] for d in body["devices"]])
                    if code != 200:
                        raise RuntimeError(f"reference detach failed: {code} {body}")
                    if i >= 2:
                        ra.append((tb - ta) * 1e3)
                        rd.append((time.perf_counter() - tb) * 1e3)
                    progress("reference", i + 1, args.ref_steps + 2)
                ref = {"steps": args.ref_steps, "attach_p50_ms": round(pct(ra, 0.5), 4),
                       "detach_p50_ms": round(pct(rd, 0.5), 4),
                       "kubelet_limit": "count (served, not enforced)"}
                k1 = ref_cp.kubelet_calls()
                served = sum(k1[c] - k0[c] for c in ("List", "Get", "GetAllocatableResources"))
                ref["kubelet_calls_per_cycle"] = round(served / (args.ref_steps + 2), 2)
                ref["kubelet_calls_over_limit"] = k1["over_limit"] - k0["over_limit"]
            out = {
                "metric": "p50_gpu_attach_latency_ms",
                "value": round(p50, 4),
                "unit": "ms",
                "n_gpus": n,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": round(ms_per_step, 4),
                "higher_is_better": False,
                "scaling": "weak",
                "vs_baseline": None,
                # a control-plane latency: no tensor compute is timed (the post-attach RCCL
                # check all-reduces bf16)
                "dtype": "none",
                "data": "synthetic",
                # which node operations ran: "emulated" = JSON-recording cgroup-v2 backend +
                # marker files (unprivileged box), "real" = bpf(2) + mknodat on this kernel
                "node_ops": args.node_ops,
                "node_fs": "real" if args.node_ops == "real" else args.kernel_fs,
                "config": {
                    "model": f"gpumounter-amd {args.mode}-mount, {n} MI355X per Pod",
                    "global_batch": 1, "seq_len": None, "gpus_per_pod": n,
                    "parallelism": f"node-local attach of {n} GPU(s); tenant RCCL check over dp{n}",
                    "control_plane": f"hermetic fake apiserver/kubelet, latency={args.latency}",
                    "cgroup": args.cgroup,
                    "protocol": args.protocol if args.protocol == "gpumounter"
                    else "reference (emulated)",
                    "warm_pool": args.warm_pool, "placement": args.placement,
                    "device_plugin": args.device_plugin, "deploy": args.deploy,
                    "gpu_allocation": args.gpu_api,
                    "daemon_cpus": args.pin or None,
                    "daemon_env": args.daemon_env or None,
                    "security": "HTTPS client-master + mTLS master-worker + "
                                "TokenReview/SAR authz (cached)"
                    if args.deploy == "processes" and args.security == "shipped" and
                    args.protocol == "gpumounter" else "off (insecure gRPC, no authz)",
                },
                "attach_p99_ms": round(pct(attach_ms, 0.99), 4),
                "attach_p999_ms": round(pct(attach_ms, 0.999), 4) if len(attach_ms) >= 1000
                else None,
                "attach_max_ms": round(max(attach_ms), 4) if attach_ms else None,
                # spread of the timed attaches: a wide one with a normal "box" points at
                # interference during the run (another job on the host), not at the code
                "attach_iqr_ms": round(pct(attach_ms, 0.75) - pct(attach_ms, 0.25), 4)
                if attach_ms else None,
                # where the client-side attach time goes, p50: the worker's whole attach, the
                # master's handler (incl. the gRPC call to the worker) and what is left
                # (client ⇄ master HTTP)
                "attach_split_p50_ms": {
                    "worker": round(pct([w for _, w in hop_ms], 0.5), 4),
                    "master_minus_worker": round(pct([m - w for m, w in hop_ms], 0.5), 4),
                    "client_minus_master": round(pct([a - m for a, (m, _) in
                                                      zip(attach_ms, hop_ms)], 0.5), 4)}
                if hop_ms and len(hop_ms) == len(attach_ms) else None,
                # the attach an operator makes after idling past the master's authz TTLs
                # (TokenReview + SubjectAccessReview asked again), and the very first attach
                # after the daemons started
                "cold_attach_p50_ms": cold["attach_p50_ms"] if cold else None,
                "cold_attach": cold,
                "first_attach_ms": round(first_attach[0], 4) if first_attach else None,
                "first_attach_stages_ms": first_stages or None,
                # control-plane calls per operation on the critical path, by process and kind,
                # with the serial round trips (the median cycle of --call-cycles)
                "serial_calls_per_attach": accounting["attach"] if accounting else None,
                "serial_calls_per_detach": accounting["detach"] if accounting else None,
                "detach_p50_ms": round(pct(detach_ms, 0.5), 4),
                "detach_p99_ms": round(pct(detach_ms, 0.99), 4),
                "stage_p50_ms": {k: round(statistics.median(v), 4) for k, v in sorted(stage.items())},
                "stage_p99_ms": {k: round(pct(v, 0.99), 4) for k, v in sorted(stage.items())},
                "detach_stage_p50_ms": {k: round(statistics.median(v), 4)
                                        for k, v in sorted(dstage.items())},
                "master_stage_p50_ms": {k: round(statistics.median(v), 4)
                                        for k, v in sorted(mstage.items())},
                "probe_quick_p50_us": round(statistics.median(probe_us), 2) if probe_us else None,
                "probe_gpus_verified": len(probe_by_gpu) if world == 1 else None,
                "probe_quick_p50_us_by_gpu": {b: round(statistics.median(v), 2)
                                              for b, v in sorted(probe_by_gpu.items())}
                if world == 1 and probe_by_gpu else None,
                "allreduce_backend": ar_backend[0],
                "allreduce_2MiB_p50_ms": round(statistics.median(ar_ms), 4) if ar_ms else None,
                "rccl_allreduce_2MiB_p50_ms": round(statistics.median(ar_ms), 4)
                if ar_ms and ar_backend[0] == "nccl" else None,
                "tenant_view": tenant_view, "tenant_view_pytorch": tenant_view_pt,
                # attaches whose plugin-chosen GPUs were swapped for a better-placed set
                "placement_corrections": corrections,
                # placeholders the kubelet refused at admission and what followed (a teardown
                # on the attach path: rebooked)
                "admission_refusals": refusals,
                "attached_hives": att_hives, "attached_numa_nodes": att_numa,
                "non_xgmi_pairs": att_nx, "p2p": p2p,
                "ledger_audit_issues": audit_issues,
                "final_orphans": orphan_issues,
                # PodResources traffic of this run against the limited kubelet (100 qps,
                # burst 10): rejected calls were retried by the ledger client
                "kubelet_calls": {k: kcalls.get(k, 0) for k in
                                  ("List", "Get", "GetAllocatableResources", "rejected")},
                "placeholders_left": placeholders_left,
                # collections in this (client) process that paused it ≥ 5 ms: [generation, ms]
                "client_gc_pauses": [list(x) for x in runtime.gc_pauses],
                "reference_emulated_same_run": ref,
                "inventory": info,
                "box": box,
                "box_after": {"py_loop_us": round(calib_after, 1),
                              "loadavg_1m": round(os.getloadavg()[0], 2)}
                if box is not None else None,
            }
            if args.node_ops == "real":
                out["attach_p50_real_node_ops_ms"] = out["value"]
                out["real_node_ops_stage_p50_ms"] = {
                    k.split(".")[-1]: v for k, v in out["stage_p50_ms"].items()
                    if k.startswith("mount.cgroup_rule.bpf_") or k in (
                        "mount.cgroup_rule", "mount.devnodes", "mount")}
            if samples is not None:
                with open(args.dump_samples, "w") as fh:
                    for smp in samples:
                        fh.write(json.dumps(smp) + "\n")
            print(json.dumps(out), flush=True)
    finally:
        if rank_pool is not None:
            rank_pool.close()
        if rank == 0:
            if cp is not None:
                cp.stop()
            if sleeper is not None:
                sleeper.kill()
                sleeper.wait()
            if sandbox is not None:
                sandbox.__exit__(None, None, None)
        if world > 1:
            dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
