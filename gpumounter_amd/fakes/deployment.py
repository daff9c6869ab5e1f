"""A deployment-shaped hermetic cluster: every component in its own process.

``LocalCluster`` runs the fake control plane, the workers and the master in one event loop, which
is ideal for white-box tests but is not how gpumounter-amd runs. ``ProcessCluster`` starts

* the fake control plane (``python -m gpumounter_amd.fakes.controlplane``),
* one worker per node with the production entry point (``python -m gpumounter_amd worker``),
  configured only through ``GM_*`` environment variables like the DaemonSet,
* the master (``python -m gpumounter_amd master``) the same way,

waits until each reports ready, and talks to the master over HTTP. ``stop()`` sends SIGTERM and
expects every daemon to exit cleanly. ``secure=True`` (the default for the gpumounter protocol)
runs them as the shipped manifests do: master⇄worker mTLS with certificates from a throw-away CA
(:mod:`gpumounter_amd.fakes.pki`) and the master authorizing every call with TokenReview +
SubjectAccessReview (``GM_AUTHZ_MODE=kube``); the client sends a bearer token the fake apiserver
knows. Used by tests/test_processes.py and ``bench.py --deploy
processes`` (no shared interpreter, event loop or GIL between master, worker and apiserver).
"""
from __future__ import annotations

import http.client
import json
import os
import shutil
import signal
import ssl
import subprocess
import sys
import tempfile
import threading
import time
import urllib.error
import urllib.parse
import urllib.request
from typing import Dict, List, Optional, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _http(method: str, url: str, body: Optional[bytes] = None, headers: Optional[dict] = None,
          timeout: float = 60.0, context: Optional[ssl.SSLContext] = None) -> Tuple[int, bytes]:
    req = urllib.request.Request(url, data=body, method=method, headers=headers or {})
    try:
        with urllib.request.urlopen(req, timeout=timeout, context=context) as r:
            return r.status, r.read()
    except urllib.error.HTTPError as e:
        return e.code, e.read()


class ProcessCluster:
    def __init__(self, n_nodes: int = 1, amdsmi_lib: str = "mock", cgroup_mode: str = "v2",
                 latency: str = "zero", gpu_bdfs: Optional[List[str]] = None,
                 worker_env: Optional[Dict[str, str]] = None,
                 master_env: Optional[Dict[str, str]] = None, log_dir: str = "",
                 protocol: str = "gpumounter", kubelet_limit: str = "enforce",
                 secure: Optional[bool] = None, gpu_api: str = "device-plugin",
                 kernel_fs: str = "disk", lazy_checkpoint: bool = False) -> None:
        """``protocol="reference"`` runs worker and master with the reference's call sequence
        (gpumounter_amd/fakes/refproto.py) in the same deployment shape, for comparison; it is
        insecure like the reference unless ``secure`` says otherwise.
        ``kubelet_limit="count"`` serves PodResources calls over the kubelet's rate budget and
        only counts them (see :class:`FakeKubelet`).
        ``kernel_fs="tmpfs"`` keeps the emulated cgroupfs and /dev trees on ``/dev/shm`` (see
        :class:`FakeNode`), when it is a writable tmpfs."""
        self.n_nodes = n_nodes
        self.secure = protocol == "gpumounter" if secure is None else secure
        self.token = "gm-hermetic-client-token" if self.secure else ""
        self._auth = {"Authorization": f"Bearer {self.token}"} if self.token else {}
        self.entry = ["-m", "gpumounter_amd"] if protocol == "gpumounter" else \
            ["-m", "gpumounter_amd.fakes.refproto"]
        self.amdsmi_lib = amdsmi_lib
        self.cgroup_mode = cgroup_mode
        self.latency = latency
        self.kubelet_limit = kubelet_limit
        self.gpu_bdfs = gpu_bdfs or []
        self.lazy_checkpoint = lazy_checkpoint
        self.gpu_api = gpu_api
        self.worker_env = worker_env or {}
        self.master_env = master_env or {}
        self.workdir = tempfile.mkdtemp(prefix="gm-deploy-")
        self.kernel_fs_dir = ""
        if kernel_fs == "tmpfs" and os.access("/dev/shm", os.W_OK):
            self.kernel_fs_dir = tempfile.mkdtemp(prefix="gm-kfs-", dir="/dev/shm")
        self.log_dir = log_dir or self.workdir
        os.makedirs(self.log_dir, exist_ok=True)
        self.procs: Dict[str, subprocess.Popen] = {}
        self.info: dict = {}
        self.worker_ports: Dict[str, Tuple[int, int]] = {}   # node → (grpc, metrics)
        self._worker_env: Dict[str, Dict[str, str]] = {}
        self.master_url = ""
        self.ca = ""            # secure: the CA that signed the master's HTTPS certificate
        self.tls: Optional[ssl.SSLContext] = None    # secure: verifies the master
        self._local = threading.local()   # one keep-alive connection to the master per thread
        self._conns: List[http.client.HTTPConnection] = []

    def _master(self, method: str, path: str, body: Optional[bytes] = None,
                headers: Optional[dict] = None) -> Tuple[int, bytes]:
        """One request on a persistent connection (as a real client library would hold)."""
        for attempt in (0, 1):
            conn = getattr(self._local, "conn", None)
            if conn is None:
                host, port = self.master_url.split("://", 1)[1].split(":")
                conn = self._local.conn = http.client.HTTPSConnection(
                    host, int(port), timeout=120, context=self.tls) if self.tls is not None \
                    else http.client.HTTPConnection(host, int(port), timeout=120)
                self._conns.append(conn)
            try:
                conn.request(method, path, body=body, headers={**self._auth, **(headers or {})})
                r = conn.getresponse()
                return r.status, r.read()
            except (http.client.HTTPException, OSError):
                conn.close()
                self._local.conn = None
                if attempt:
                    raise
        raise AssertionError("unreachable")

    # ------------------------------------------------------------------------ lifecycle
    def _spawn(self, key: str, argv: List[str], env: Dict[str, str]) -> subprocess.Popen:
        # appended: a restarted daemon's log follows its predecessor's (chaos post-mortems)
        log = open(os.path.join(self.log_dir, f"{key}.log"), "a")
        full = {**os.environ, "PYTHONPATH": ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
                **env}
        p = subprocess.Popen([sys.executable, *argv], cwd=ROOT, env=full, stdout=log,
                             stderr=subprocess.STDOUT, start_new_session=True)
        self.procs[key] = p
        return p

    def _wait(self, what: str, ok, timeout: float = 120.0) -> None:
        end = time.time() + timeout
        while time.time() < end:
            for key, p in self.procs.items():
                if p.poll() is not None:
                    raise RuntimeError(f"{key} exited with {p.returncode} while waiting for "
                                       f"{what}:\n{self.log(key)[-3000:]}")
            try:
                if ok():
                    return
            except (OSError, ValueError):
                pass
            time.sleep(0.05)
        raise TimeoutError(f"timed out waiting for {what}")

    def log(self, key: str) -> str:
        try:
            with open(os.path.join(self.log_dir, f"{key}.log")) as fh:
                return fh.read()
        except OSError:
            return ""

    def start(self) -> "ProcessCluster":
        try:
            return self._start()
        except BaseException:
            self.stop()          # no daemon outlives a failed start
            raise

    def _start(self) -> "ProcessCluster":
        info_path = os.path.join(self.workdir, "info.json")
        self._spawn("controlplane", ["-m", "gpumounter_amd.fakes.controlplane", "--workdir",
                                     os.path.join(self.workdir, "cluster"), "--info", info_path,
                                     "--nodes", str(self.n_nodes), "--amdsmi", self.amdsmi_lib,
                                     "--cgroup", self.cgroup_mode, "--latency", self.latency,
                                     "--kubelet-limit", self.kubelet_limit,
                                     "--gpu-bdfs", ",".join(self.gpu_bdfs),
                                     "--gpu-api", self.gpu_api,
                                     "--kernel-fs-dir", self.kernel_fs_dir]
                                    + (["--lazy-checkpoint"] if self.lazy_checkpoint else []), {})
        self._wait("control plane", lambda: os.path.exists(info_path))
        with open(info_path) as fh:
            self.info = json.load(fh)
        api = self.info["api_url"]
        tls_w, tls_m = {"GM_AUTHZ_MODE": "none"}, {"GM_AUTHZ_MODE": "none"}
        if self.secure:
            from gpumounter_amd.fakes.pki import make_pki
            pki = make_pki(os.path.join(self.workdir, "pki"))
            tls_w = {"GM_TLS_CERT": pki["worker.crt"], "GM_TLS_KEY": pki["worker.key"],
                     "GM_TLS_CA": pki["ca"], "GM_AUTHZ_MODE": "kube"}
            # the shipped master: HTTPS on its API port, callers' tokens reviewed
            tls_m = {"GM_TLS_CERT": pki["master.crt"], "GM_TLS_KEY": pki["master.key"],
                     "GM_TLS_CA": pki["ca"], "GM_AUTHZ_MODE": "kube",
                     "GM_MASTER_TLS_CERT": pki["master-https.crt"],
                     "GM_MASTER_TLS_KEY": pki["master-https.key"]}
            self.ca = pki["ca"]
            self.tls = ssl.create_default_context(cafile=self.ca)
            code, _ = _http("POST", f"{api}/_fake/user", json.dumps(
                {"token": self.token, "user": "gm-hermetic-client",
                 "verbs": ["create", "delete", "get"], "resource": "pods/gpumount"}).encode(),
                {"Content-Type": "application/json"})
            if code != 201:
                raise RuntimeError(f"client token registration failed: {code}")
            _http("POST", f"{api}/_fake/user", json.dumps(
                {"token": self.token, "user": "gm-hermetic-client", "verbs": ["get"],
                 "resource": "nodes/gpumount"}).encode(), {"Content-Type": "application/json"})
        for node, n in self.info["nodes"].items():
            # ephemeral ports, published by the daemon itself (GM_READY_FILE): a port picked
            # here and bound later can be taken by another process in between
            env = {"GM_KUBE_API": api, "GM_NODE_NAME": node,
                   "GM_KUBELET_SOCKET": n["kubelet_socket"], "GM_CGROUP_ROOT": n["cgroup_root"],
                   "GM_KUBELET_CHECKPOINT": n["kubelet_checkpoint"],
                   "GM_CGROUP_MODE": self.cgroup_mode, "GM_DEVNODE_MODE": "emulate",
                   "GM_CONTAINER_ROOT_PREFIX": n["rootfs_root"], "GM_AMDSMI_LIB": self.amdsmi_lib,
                   "GM_STATE_DIR": n["state_dir"], "GM_HOST_DEV_PATH": n["host_dev"],
                   **({} if self.secure else {"GM_WORKER_INSECURE": "1"}), **tls_w,
                   "GM_WORKER_HOST": "127.0.0.1", "GM_WORKER_PORT": "0", "GM_WIRE_PORT": "0",
                   "GM_METRICS_PORT": "0", "GM_READY_FILE": self._ready_path(f"worker-{node}"),
                   "GM_LOG_LEVEL": "WARNING",
                   "GM_LOG_JSON": "false", "GM_GPU_ALLOCATION": self.gpu_api,
                   "GM_DEBUG_ENDPOINTS": "1",     # /debug/tasks for chaos post-mortems
                   **self.worker_env}
            self._worker_env[node] = env
            self._spawn(f"worker-{node}", [*self.entry, "worker"], env)
        for node in self._worker_env:
            self._await_worker(node)
        self._master_env = {"GM_KUBE_API": api, "GM_MASTER_HOST": "127.0.0.1", **tls_m,
                            "GM_DEBUG_ENDPOINTS": "1",     # /debug/calls (bench accounting)
                            "GM_MASTER_PORT": "0", "GM_READY_FILE": self._ready_path("master"),
                            "GM_LOG_LEVEL": "WARNING", "GM_LOG_JSON": "false",
                            **self.master_env}
        self._start_master()
        return self

    def _start_master(self) -> None:
        self._spawn("master", [*self.entry, "master"], self._master_env)
        scheme = "https" if self._master_env.get("GM_MASTER_TLS_CERT") else "http"
        self.master_url = f"{scheme}://127.0.0.1:{self._ready('master')['port']}"
        for node in self.info["nodes"]:   # the master has discovered every worker
            self._wait(f"master → {node}", lambda n=node: self.http(
                "GET", f"/api/v1/nodes/{n}/gpus", headers=self._auth)[0] == 200)

    def http(self, method: str, path: str, body: Optional[bytes] = None,
             headers: Optional[dict] = None, timeout: float = 60.0) -> Tuple[int, bytes]:
        """One request to the master on a fresh connection (HTTPS verified against the
        deployment's CA when secure)."""
        return _http(method, self.master_url + path, body, headers, timeout, self.tls)

    def restart_master(self, sig: int = signal.SIGKILL,
                       env: Optional[Dict[str, str]] = None) -> None:
        """Kill the master (SIGKILL: requests in flight lose their client connection; the
        workers carry on) and start a new one, with ``env`` added to its environment; it
        serves on a new port (``master_url``)."""
        if env:
            self._master_env = {**self._master_env, **env}
        p = self.procs["master"]
        p.send_signal(sig)
        p.wait(20)
        try:
            os.unlink(self._ready_path("master"))
        except FileNotFoundError:
            pass
        self._start_master()

    def _ready_path(self, key: str) -> str:
        return os.path.join(self.workdir, f"{key}.ready")

    def _ready(self, key: str) -> dict:
        """The ports daemon ``key`` bound, once it has published them."""
        path = self._ready_path(key)
        self._wait(f"{key} ready file", lambda: os.path.exists(path))
        with open(path) as fh:
            return json.load(fh)

    def _await_worker(self, node: str) -> None:
        r = self._ready(f"worker-{node}")
        gport, mport = self.worker_ports[node] = (int(r["grpc_port"]), int(r["http_port"]))
        self._wait(f"worker {node}",
                   lambda: _http("GET", f"http://127.0.0.1:{mport}/readyz")[0] == 200)
        code, _ = _http("POST", f"{self.info['api_url']}/_fake/worker",
                        json.dumps({"node": node, "port": gport,
                                    "wire_port": int(r.get("wire_port") or 0)}).encode(),
                        {"Content-Type": "application/json"})
        if code != 201:
            raise RuntimeError(f"worker registration for {node} failed: {code}")

    def kill_worker(self, node: str = "node-0", sig: int = signal.SIGKILL) -> int:
        """Crash (SIGKILL) or stop a worker process; returns its exit status."""
        p = self.procs[f"worker-{node}"]
        p.send_signal(sig)
        return p.wait(20)

    def restart_worker(self, node: str = "node-0") -> None:
        """Start the node's worker again (same environment, fresh ports) and wait until it is
        ready and registered under its new port."""
        try:
            os.unlink(self._ready_path(f"worker-{node}"))
        except FileNotFoundError:
            pass
        self._spawn(f"worker-{node}", [*self.entry, "worker"], self._worker_env[node])
        self._await_worker(node)

    def stop(self, timeout: float = 20.0) -> Dict[str, Optional[int]]:
        """SIGTERM every daemon (master and workers first) → their exit codes."""
        for conn in self._conns:
            conn.close()
        self._conns.clear()
        codes: Dict[str, Optional[int]] = {}
        order = [k for k in self.procs if k == "master"] + \
            [k for k in self.procs if k.startswith("worker-")] + \
            [k for k in self.procs if k == "controlplane"]
        for key in order:
            p = self.procs[key]
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
                try:
                    p.wait(timeout)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, signal.SIGKILL)
                    p.wait(5)
            codes[key] = p.returncode
        shutil.rmtree(self.workdir, ignore_errors=True)
        if self.kernel_fs_dir:
            shutil.rmtree(self.kernel_fs_dir, ignore_errors=True)
        return codes

    def __enter__(self) -> "ProcessCluster":
        try:
            return self.start()
        except BaseException:
            self.stop()
            raise

    def __exit__(self, *exc) -> None:
        self.stop()

    # ------------------------------------------------------------------------ operations
    def tenant(self, name: str, ns: str = "default", node: str = "node-0", gpus: int = 0,
               pids: Optional[Dict[str, List[int]]] = None) -> dict:
        code, body = _http("POST", f"{self.info['api_url']}/_fake/tenant",
                           json.dumps({"name": name, "ns": ns, "node": node,
                                       "gpus": gpus, "pids": pids}).encode(),
                           {"Content-Type": "application/json"})
        if code != 201:
            raise RuntimeError(f"tenant create failed: {code} {body[:300]!r}")
        return json.loads(body)

    def add(self, ns: str, pod: str, n: int, entire: bool = False, lease_s: float = 0.0
            ) -> Tuple[int, dict]:
        q = f"?lease={lease_s:g}" if lease_s else ""
        code, body = self._master("GET", f"/addgpu/namespace/{ns}/pod/{pod}/gpu/{n}/"
                                         f"isEntireMount/{'true' if entire else 'false'}{q}",
                                  headers={"Accept": "application/json"})
        return code, json.loads(body)

    def remove(self, ns: str, pod: str, uuids: List[str], force: bool = False
               ) -> Tuple[int, dict]:
        data = urllib.parse.urlencode([("uuids", u) for u in uuids]).encode()
        code, body = self._master("POST", f"/removegpu/namespace/{ns}/pod/{pod}/force/"
                                          f"{'true' if force else 'false'}", data,
                                  {"Accept": "application/json",
                                   "Content-Type": "application/x-www-form-urlencoded"})
        return code, json.loads(body)

    def pod_gpus(self, ns: str, pod: str) -> Tuple[int, dict]:
        code, body = self.http("GET", f"/api/v1/namespaces/{ns}/pods/{pod}/gpus",
                               headers={"Accept": "application/json", **self._auth})
        return code, json.loads(body)

    def kubelet_calls(self, node: str = "node-0") -> Dict[str, int]:
        code, body = _http("GET", f"{self.info['api_url']}/_fake/kubelet")
        if code != 200:
            raise RuntimeError(f"kubelet counters: {code}")
        return json.loads(body)[node]

    def restart_container(self, ns: str, pod: str, container: str = "main") -> str:
        """The kubelet restarts one container of a tenant Pod (fakes/apiserver.py)."""
        code, body = _http("POST", f"{self.info['api_url']}/_fake/restart",
                           json.dumps({"ns": ns, "pod": pod, "container": container}).encode(),
                           {"Content-Type": "application/json"})
        if code != 201:
            raise RuntimeError(f"container restart: {code} {body[:200]!r}")
        return json.loads(body)["container_id"]

    def restart_kubelet(self, node: str = "node-0", down_s: float = 0.0) -> None:
        code, body = _http("POST", f"{self.info['api_url']}/_fake/kubelet/restart",
                           json.dumps({"node": node, "down_s": down_s}).encode(),
                           {"Content-Type": "application/json"})
        if code != 201:
            raise RuntimeError(f"kubelet restart: {code} {body[:200]!r}")

    def recreate_pod(self, ns: str, pod: str, gap_s: float = 0.0) -> str:
        """Delete the tenant Pod and create it again under the same name; its new UID."""
        code, body = _http("POST", f"{self.info['api_url']}/_fake/recreate",
                           json.dumps({"ns": ns, "pod": pod, "gap_s": gap_s}).encode(),
                           {"Content-Type": "application/json"})
        if code != 201:
            raise RuntimeError(f"recreate: {code} {body[:200]!r}")
        return json.loads(body)["uid"]

    def api_faults(self, rate: float, seed: int = 0) -> int:
        """Random apiserver failures for Pod/ResourceClaim requests (fakes/apiserver.py
        random_failures); returns how many were served before this call."""
        code, body = _http("POST", f"{self.info['api_url']}/_fake/faults",
                           json.dumps({"rate": rate, "seed": seed}).encode(),
                           {"Content-Type": "application/json"})
        if code != 201:
            raise RuntimeError(f"fault setup: {code}")
        return int(json.loads(body)["served"])

    def placeholders(self) -> List[dict]:
        code, body = _http("GET", f"{self.info['api_url']}/api/v1/pods?labelSelector=app%3Dgpu-pool")
        return json.loads(body).get("items", []) if code == 200 else []

    def audit(self, ns: str, pod: str, node: str = "node-0") -> list:
        for _ in range(5):
            code, body = _http("GET",
                               f"http://127.0.0.1:{self.worker_ports[node][1]}/audit/{ns}/{pod}",
                               headers=self._auth)
            if code != 409:                 # 409: a container restarting under the audit
                break
            time.sleep(0.1)
        if code != 200:
            raise RuntimeError(f"audit {ns}/{pod}: {code} {body[:300]!r}")
        return json.loads(body)["issues"]

    def calls(self, since: float, until: float, node: str = "node-0") -> dict:
        """Outbound control-plane calls of the master and the node's worker that started in
        [since, until] (CLOCK_MONOTONIC, shared by the host's processes)."""
        q = f"?since={since!r}&until={until!r}"
        out = {}
        for who, url in (("master", f"{self.master_url}/debug/calls{q}"),
                         ("worker", f"http://127.0.0.1:{self.worker_ports[node][1]}"
                                    f"/debug/calls{q}")):
            code, body = _http("GET", url, headers=self._auth,
                               context=self.tls if who == "master" else None)
            if code != 200:
                raise RuntimeError(f"{who} /debug/calls: {code} {body[:200]!r}")
            out[who] = [tuple(c) for c in json.loads(body)]
        return out

    def worker_tasks(self, node: str = "node-0") -> str:
        """The worker's asyncio tasks and their stacks (``/debug/tasks``)."""
        return _http("GET", f"http://127.0.0.1:{self.worker_ports[node][1]}/debug/tasks")[1] \
            .decode()

    def worker_metrics(self, node: str = "node-0") -> str:
        return _http("GET", f"http://127.0.0.1:{self.worker_ports[node][1]}/metrics")[1].decode()

    def rootfs(self, node: str = "node-0") -> str:
        return self.info["nodes"][node]["rootfs_root"]
