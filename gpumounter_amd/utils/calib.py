"""Box-speed calibration recorded next to every bench value.

The headline is a control-plane latency: a handful of Python request handlers in three processes
(client, master, worker) plus the fake apiserver, joined by loopback HTTP/gRPC. Its value therefore
moves with two properties of the machine it runs on, which this module measures in a fixed way:

* ``py_loop_us`` — one fixed pure-Python workload (dict/str/int churn, no allocation growth),
  median of several repeats: how fast the interpreter runs the handlers;
* ``pingpong_us`` / ``tcp_rtt_us`` — the round trip between two processes over a socketpair and
  over a loopback TCP connection, median of many: what one hop between the daemons costs before
  any gpumounter code runs (scheduler wake-up of an idle core, C-state exit, cross-CCX cache);
* ``grpc_rtt_us`` — a unary AddGPU call between two grpc.aio processes answering at once,
  plaintext and mTLS: the floor under a gRPC master → worker hop;
* ``wire_rtt_us`` — the same call over gm-wire (api/wire.py), plaintext and mTLS: the floor
  under the master → worker hop as shipped;
* ``pingpong_after_idle_us`` / ``py_loop_after_idle_us`` (with ``idle_s``) — the same round
  trip and the same Python loop right after ``idle_s`` asleep: what a quiet spell costs.

A value measured on a box whose ``pingpong_us`` is 3× another's is not a regression of the code;
``bench.py`` puts this dict into its JSON as ``box`` so every number carries its box.
"""
from __future__ import annotations

import json
import os
import socket
import statistics
import time


def _py_loop_once() -> float:
    t0 = time.perf_counter()
    d: dict = {}
    acc = 0
    for i in range(20000):
        k = "k%d" % (i & 255)
        d[k] = d.get(k, 0) + i
        acc += len(k) ^ (i * 7)
    return (time.perf_counter() - t0) * 1e6 + (acc & 0)


def py_loop_us(repeats: int = 7) -> float:
    return statistics.median(_py_loop_once() for _ in range(repeats))


def _echo_child(sock: socket.socket, n: int) -> None:
    for _ in range(n):
        b = sock.recv(64)
        if not b:
            break
        sock.sendall(b)


def pingpong_us(n: int = 2000, tcp: bool = False, idle_s: float = 0.0) -> float:
    """Median round trip between this process and a forked echo child (socketpair or TCP);
    ``idle_s`` > 0: each round trip after that long asleep (both processes idle), what a
    request arriving after a quiet spell pays per hop."""
    if tcp:
        lsock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        lsock.bind(("127.0.0.1", 0))
        lsock.listen(1)
        port = lsock.getsockname()[1]
    else:
        a, b = socket.socketpair()
    pid = os.fork()
    if pid == 0:   # child: no GPU state exists in this process (calibration runs first)
        try:
            if tcp:
                c = socket.create_connection(("127.0.0.1", port))
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                _echo_child(c, n)
            else:
                a.close()
                _echo_child(b, n)
        finally:
            os._exit(0)
    try:
        if tcp:
            s, _ = lsock.accept()
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            lsock.close()
        else:
            b.close()
            s = a
        rtts = []
        msg = b"x" * 32
        for _ in range(n):
            if idle_s:
                time.sleep(idle_s)
            t0 = time.perf_counter()
            s.sendall(msg)
            got = 0
            while got < len(msg):
                got += len(s.recv(64))
            rtts.append((time.perf_counter() - t0) * 1e6)
        s.close()
        return statistics.median(rtts if idle_s else rtts[n // 10:])
    finally:
        os.waitpid(pid, 0)


def _grpc_server() -> None:
    """``python -m gpumounter_amd.utils.calib --grpc-server``: an AddGPU service answering
    Success at once, plaintext and mTLS ports printed on stdout, until stdin closes."""
    import asyncio
    import shutil
    import sys
    import tempfile

    import grpc

    from gpumounter_amd.api import gpu_mount as api
    from gpumounter_amd.fakes.pki import make_pki

    async def run():
        pki = make_pki(tempfile.mkdtemp(prefix="gm-calib-"))

        async def add(req, ctx):
            return api.AddGPUResponse(add_gpu_result=api.ADD_SUCCESS)
        server = grpc.aio.server()
        server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(
            f"{api.PACKAGE}.AddGPUService", {"AddGPU": grpc.unary_unary_rpc_method_handler(
                add, api.AddGPURequest.FromString, lambda m: m.SerializeToString())}),))
        rd = lambda p: open(p, "rb").read()   # noqa: E731
        creds = grpc.ssl_server_credentials([(rd(pki["worker.key"]), rd(pki["worker.crt"]))],
                                            root_certificates=rd(pki["ca"]),
                                            require_client_auth=True)
        plain = server.add_insecure_port("127.0.0.1:0")
        tls = server.add_secure_port("127.0.0.1:0", creds)
        await server.start()
        from gpumounter_amd.api import wire
        handlers = {wire.METHOD_ADD: (api.AddGPURequest.FromString, lambda r: add(r, None))}
        wplain = wire.WireServer(handlers)
        wtls = wire.WireServer(handlers, wire.server_context(pki["worker.crt"],
                                                             pki["worker.key"], pki["ca"]),
                               ["gpu-mounter-master"])
        ports = {"wire_plain": await wplain.start("127.0.0.1", 0),
                 "wire_tls": await wtls.start("127.0.0.1", 0)}
        print(json.dumps({"plain": plain, "tls": tls, "pki": pki, **ports}), flush=True)
        await asyncio.get_running_loop().run_in_executor(None, sys.stdin.read)
        await wplain.stop()
        await wtls.stop()
        await server.stop(0)
        shutil.rmtree(os.path.dirname(pki["ca"]), ignore_errors=True)
    asyncio.run(run())


def grpc_rtt_us(n: int = 1500) -> dict:
    """Median unary AddGPU round trip, grpc.aio client → grpc.aio server in another process,
    plaintext and with mTLS, and the same over gm-wire (``wire_plain``, ``wire_mtls``): the
    floors under the master → worker hop."""
    import asyncio
    import subprocess
    import sys

    import grpc

    from gpumounter_amd.api import gpu_mount as api

    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = {**os.environ, "PYTHONPATH": root + os.pathsep + os.environ.get("PYTHONPATH", "")}
    p = subprocess.Popen([sys.executable, "-m", "gpumounter_amd.utils.calib", "--grpc-server"],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)
    try:
        info = json.loads(p.stdout.readline())
        rd = lambda f: open(f, "rb").read()   # noqa: E731

        async def one(secure: bool) -> float:
            if secure:
                pki = info["pki"]
                creds = grpc.ssl_channel_credentials(rd(pki["ca"]), rd(pki["master.key"]),
                                                     rd(pki["master.crt"]))
                ch = grpc.aio.secure_channel(
                    f"127.0.0.1:{info['tls']}", creds,
                    options=[("grpc.ssl_target_name_override", "gpu-mounter-worker")])
            else:
                ch = grpc.aio.insecure_channel(f"127.0.0.1:{info['plain']}")
            stub = ch.unary_unary(api.ADD_GPU,
                                  request_serializer=api.AddGPURequest.SerializeToString,
                                  response_deserializer=api.AddGPUResponse.FromString)
            ts = []
            for _ in range(n):
                t0 = time.perf_counter()
                await stub(api.AddGPURequest(pod_name="t", namespace="default", gpu_num=1),
                           timeout=10)
                ts.append((time.perf_counter() - t0) * 1e6)
            await ch.close()
            return round(statistics.median(ts[n // 10:]), 1)

        async def wire_one(secure: bool) -> float:
            from gpumounter_amd.api import wire
            pki = info["pki"]
            if secure:
                ch = wire.WireChannel("127.0.0.1", info["wire_tls"], wire.client_context(
                    pki["ca"], pki["master.crt"], pki["master.key"]), "gpu-mounter-worker")
            else:
                ch = wire.WireChannel("127.0.0.1", info["wire_plain"])
            payload = api.AddGPURequest(pod_name="t", namespace="default",
                                        gpu_num=1).SerializeToString()
            ts = []
            for _ in range(n):
                t0 = time.perf_counter()
                api.AddGPUResponse.FromString(await ch.call(wire.METHOD_ADD, payload, 10))
                ts.append((time.perf_counter() - t0) * 1e6)
            await ch.close()
            return round(statistics.median(ts[n // 10:]), 1)

        async def both():
            return {"plain": await one(False), "mtls": await one(True),
                    "wire_plain": await wire_one(False), "wire_mtls": await wire_one(True)}
        return asyncio.run(both())
    finally:
        p.stdin.close()
        p.wait(10)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def _governor() -> str | None:
    try:
        with open("/sys/devices/system/cpu/cpu0/cpufreq/scaling_governor") as fh:
            return fh.read().strip()
    except OSError:
        return None


def measure(grpc_floor: bool = False, idle_s: float = 0.0) -> dict:
    """Fixed calibration, about 0.3 s (about 2 s more with ``grpc_floor``). Run it before the
    process initialises the GPU: the pingpong child is a fork (pure-Python socket code, then
    ``_exit``) and the gRPC server a subprocess."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    out = {
        "py_loop_us": round(py_loop_us(), 1),
        "pingpong_us": round(pingpong_us(), 2),
        "tcp_rtt_us": round(pingpong_us(1000, tcp=True), 2),
        "cpu": _cpu_model(),
        "cpus_online": os.cpu_count(),
        "cpus_allowed": aff,
        "loadavg_1m": round(os.getloadavg()[0], 2),
        "governor": _governor(),
    }
    if grpc_floor:
        out["grpc_rtt_us"] = grpc_rtt_us()
    if idle_s:
        # the same hop and the same Python work after idle_s asleep: what a quiet spell (caches
        # and cores gone cold, or to other jobs) costs on this box before any gpumounter code
        out["idle_s"] = idle_s
        out["pingpong_after_idle_us"] = round(pingpong_us(8, idle_s=idle_s), 2)
        cold = []
        for _ in range(5):
            time.sleep(idle_s)
            cold.append(_py_loop_once())
        out["py_loop_after_idle_us"] = round(statistics.median(cold), 1)
    return out


if __name__ == "__main__":
    import sys
    if "--grpc-server" in sys.argv:
        _grpc_server()
    else:
        print(json.dumps(measure(grpc_floor="--grpc" in sys.argv)))
