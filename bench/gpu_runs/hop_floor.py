"""The gRPC master → worker hop in isolation, on this box: a grpc.aio AddGPU server in another
process and a grpc.aio client, one call at a time, median round trip minus the handler's own time
(= transport: both gRPC stacks, TLS, both event loops).

    python bench/gpu_runs/hop_floor.py [--http] [--tls] [--retry] [--big] [--shield]

--http    the handler makes 3 aiohttp POSTs to a local server before answering (the worker's
          attach awaits the apiserver); default: answers at once
--tls     mTLS on both ends, as shipped
--retry   the master's channel options (retries enabled, AddGPU retry policy, keepalive)
--big     a response the size of a real attach's (20 stage timings, one device)
--shield  the worker's handler shape: the operation as its own task, awaited through shield
--sync    the client: a synchronous grpc stub called from a thread (run_in_executor)
Prints one JSON line."""
import argparse
import asyncio
import json
import multiprocessing as mp
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import aiohttp  # noqa: E402
import grpc  # noqa: E402
from aiohttp import web  # noqa: E402

from gpumounter_amd.api import gpu_mount as api  # noqa: E402


class Spin:
    """Keeps the event loop from blocking in epoll while work is in flight (and ``tail_s``
    after), so a completion signalled by another thread needs no wake-up of this one."""
    def __init__(self, tail_s=0.0003):
        self.n, self.until, self.tail, self.loop = 0, 0.0, tail_s, None

    def _tick(self):
        if self.n or time.perf_counter() < self.until:
            self.loop.call_soon(self._tick)
        else:
            self.on = False

    def __enter__(self):
        self.loop = asyncio.get_running_loop()
        self.n += 1
        if not getattr(self, "on", False):
            self.on = True
            self.loop.call_soon(self._tick)

    def __exit__(self, *a):
        self.n -= 1
        self.until = time.perf_counter() + self.tail


def rd(p):
    with open(p, "rb") as fh:
        return fh.read()


def server_main(args, q):
    async def run():
        app = web.Application()

        async def h(req):
            return web.json_response({"ok": 1})
        app.router.add_post("/x", h)
        r = web.AppRunner(app)
        await r.setup()
        site = web.TCPSite(r, "127.0.0.1", 0)
        await site.start()
        hport = site._server.sockets[0].getsockname()[1]   # noqa: SLF001
        sess = aiohttp.ClientSession()

        async def op(req):
            t0 = time.perf_counter()
            if args.sleep:
                await asyncio.sleep(args.sleep)
            if args.http:
                for _ in range(3):
                    async with sess.post(f"http://127.0.0.1:{hport}/x", json={"a": 1}) as resp:
                        await resp.read()
            resp = api.AddGPUResponse(add_gpu_result=api.ADD_SUCCESS)
            if args.big:
                resp.devices.add(uuid="a5ff74a1-0000-1000-8003-000000355003", bdf="0000:75:00.0",
                                 index=3, render_minor=131, card_minor=3, numa_node=0,
                                 xgmi_hive_id=0x202623C52A2ED94D, placeholder="t-slave-pod-1a2b3c")
                for i in range(20):
                    resp.timings.add(name=f"stage_{i}.sub", ms=0.123 * i)
                resp.message = "Add GPU Success"
            resp.total_ms = (time.perf_counter() - t0) * 1e3
            return resp

        spin = Spin()

        async def add(req, ctx):
            if args.spin:
                with spin:
                    if args.shield:
                        return await asyncio.shield(asyncio.ensure_future(op(req)))
                    return await op(req)
            if args.shield:
                t = asyncio.ensure_future(op(req))
                return await asyncio.shield(t)
            return await op(req)
        server = grpc.aio.server()
        server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(
            f"{api.PACKAGE}.AddGPUService", {"AddGPU": grpc.unary_unary_rpc_method_handler(
                add, api.AddGPURequest.FromString, lambda m: m.SerializeToString())}),))
        if args.tls:
            from gpumounter_amd.fakes.pki import make_pki
            pki = make_pki(tempfile.mkdtemp(prefix="gm-hop-"))
            creds = grpc.ssl_server_credentials([(rd(pki["worker.key"]), rd(pki["worker.crt"]))],
                                                root_certificates=rd(pki["ca"]),
                                                require_client_auth=True)
            port = server.add_secure_port("127.0.0.1:0", creds)
        else:
            pki = None
            port = server.add_insecure_port("127.0.0.1:0")
        await server.start()
        q.put((port, pki))
        await asyncio.sleep(600)
    asyncio.run(run())


async def client(args, port, pki, n):
    opts = []
    if args.retry:
        from gpumounter_amd.master.app import _SERVICE_CONFIG
        opts = [("grpc.keepalive_time_ms", 30000), ("grpc.enable_retries", 1),
                ("grpc.service_config", _SERVICE_CONFIG)]
    mod = grpc if args.sync else grpc.aio
    if args.tls:
        creds = grpc.ssl_channel_credentials(rd(pki["ca"]), rd(pki["master.key"]),
                                             rd(pki["master.crt"]))
        opts.append(("grpc.ssl_target_name_override", "gpu-mounter-worker"))
        ch = mod.secure_channel(f"127.0.0.1:{port}", creds, options=opts)
    else:
        ch = mod.insecure_channel(f"127.0.0.1:{port}", options=opts)
    stub = ch.unary_unary(api.ADD_GPU, request_serializer=api.AddGPURequest.SerializeToString,
                          response_deserializer=api.AddGPUResponse.FromString)
    loop = asyncio.get_running_loop()
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(1)

    spin = Spin(0.0)

    async def call(req):
        if args.spin:
            with spin:
                return await stub(req, timeout=10)
        if args.sync:
            return await loop.run_in_executor(pool, lambda: stub(req, timeout=10))
        return await stub(req, timeout=10)
    ts, inner = [], []
    for _ in range(n):
        t = time.perf_counter()
        r = await call(api.AddGPURequest(pod_name="t", namespace="default", gpu_num=1,
                                         request_id="add-0123456789ab",
                                         idempotency_key="add-0123456789ab"))
        ts.append((time.perf_counter() - t) * 1e6)
        inner.append(r.total_ms * 1e3)
    if args.sync:
        ch.close()
    else:
        await ch.close()
    return statistics.median(ts[n // 10:]), statistics.median(inner[n // 10:])


def main():
    ap = argparse.ArgumentParser()
    for f in ("http", "tls", "retry", "big", "shield", "sync", "spin"):
        ap.add_argument(f"--{f}", action="store_true")
    ap.add_argument("-n", type=int, default=1500)
    ap.add_argument("--sleep", type=float, default=0.0,
                    help="the handler sleeps this long (s) instead of / before its I/O")
    args = ap.parse_args()
    q = mp.Queue()
    p = mp.Process(target=server_main, args=(args, q), daemon=True)
    p.start()
    port, pki = q.get()
    try:
        rtt, inner = asyncio.run(client(args, port, pki, args.n))
    finally:
        p.kill()
    print(json.dumps({"opts": [f for f in ("http", "tls", "retry", "big", "shield", "sync", "spin")
                               if getattr(args, f)],
                      "rtt_us": round(rtt), "handler_us": round(inner),
                      "transport_us": round(rtt - inner)}))


if __name__ == "__main__":
    main()
