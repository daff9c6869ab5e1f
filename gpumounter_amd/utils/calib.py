"""Box-speed calibration recorded next to every bench value.

The headline is a control-plane latency: a handful of Python request handlers in three processes
(client, master, worker) plus the fake apiserver, joined by loopback HTTP/gRPC. Its value therefore
moves with two properties of the machine it runs on, which this module measures in a fixed way:

* ``py_loop_us`` — one fixed pure-Python workload (dict/str/int churn, no allocation growth),
  median of several repeats: how fast the interpreter runs the handlers;
* ``pingpong_us`` / ``tcp_rtt_us`` — the round trip between two processes over a socketpair and
  over a loopback TCP connection, median of many: what one hop between the daemons costs before
  any gpumounter code runs (scheduler wake-up of an idle core, C-state exit, cross-CCX cache).

A value measured on a box whose ``pingpong_us`` is 3× another's is not a regression of the code;
``bench.py`` puts this dict into its JSON as ``box`` so every number carries its box.
"""
from __future__ import annotations

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


def pingpong_us(n: int = 2000, tcp: bool = False) -> float:
    """Median round trip between this process and a forked echo child (socketpair or TCP)."""
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
            t0 = time.perf_counter()
            s.sendall(msg)
            got = 0
            while got < len(msg):
                got += len(s.recv(64))
            rtts.append((time.perf_counter() - t0) * 1e6)
        s.close()
        return statistics.median(rtts[n // 10:])
    finally:
        os.waitpid(pid, 0)


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


def measure() -> dict:
    """Fixed calibration, about 0.3 s. Safe before or after GPU initialisation (fork only runs
    pure-Python socket code in the child and ``_exit``s; it never execs)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {
        "py_loop_us": round(py_loop_us(), 1),
        "pingpong_us": round(pingpong_us(), 2),
        "tcp_rtt_us": round(pingpong_us(1000, tcp=True), 2),
        "cpu": _cpu_model(),
        "cpus_online": os.cpu_count(),
        "cpus_allowed": aff,
        "loadavg_1m": round(os.getloadavg()[0], 2),
        "governor": _governor(),
    }


if __name__ == "__main__":
    import json
    print(json.dumps(measure()))
