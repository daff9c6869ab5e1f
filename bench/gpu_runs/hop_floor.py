"""gRPC transport floor on this box: a grpc.aio AddGPU server in another process whose handler
(idle) answers at once, (sleep) awaits 2 ms, or (http) makes 3 aiohttp POSTs to a local server
before answering, as the worker's attach does; optional channel/server arg
grpc.optimization_target=latency ("lat"). Prints round trip, handler time and their difference
(the transport). Usage: python bench/gpu_runs/hop_floor.py idle|sleep|http [lat]"""
import asyncio, time, statistics, sys, os, tempfile, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import grpc
from aiohttp import web
import aiohttp
from gpumounter_amd.api import gpu_mount as api
import multiprocessing as mp

MODE = sys.argv[1]
OPTS = [("grpc.optimization_target", "latency")] if "lat" in sys.argv else []
def srv(q):
    async def run():
        # local http server to call
        app = web.Application()
        async def h(req): return web.json_response({"ok": 1})
        app.router.add_post("/x", h)
        r = web.AppRunner(app); await r.setup(); site = web.TCPSite(r, "127.0.0.1", 0); await site.start()
        hport = site._server.sockets[0].getsockname()[1]
        sess = aiohttp.ClientSession()
        async def add(req, ctx):
            t0 = time.perf_counter()
            if MODE == "sleep":
                await asyncio.sleep(0.002)
            elif MODE == "http":
                for _ in range(3):
                    async with sess.post(f"http://127.0.0.1:{hport}/x", json={"a": 1}) as resp:
                        await resp.read()
            resp = api.AddGPUResponse(add_gpu_result=0)
            resp.total_ms = (time.perf_counter() - t0) * 1e3
            return resp
        server = grpc.aio.server(options=OPTS)
        server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler("gpu_mount.AddGPUService", {
            "AddGPU": grpc.unary_unary_rpc_method_handler(add, api.AddGPURequest.FromString, lambda m: m.SerializeToString())}),))
        port = server.add_insecure_port("127.0.0.1:0")
        await server.start()
        q.put(port)
        await asyncio.sleep(120)
    asyncio.run(run())

async def client(port, n=1500):
    ch = grpc.aio.insecure_channel(f"127.0.0.1:{port}", options=OPTS)
    stub = ch.unary_unary(api.ADD_GPU, request_serializer=api.AddGPURequest.SerializeToString, response_deserializer=api.AddGPUResponse.FromString)
    ts=[]; inner=[]
    for i in range(n):
        t=time.perf_counter()
        r = await stub(api.AddGPURequest(pod_name="t", namespace="default", gpu_num=1), timeout=10)
        ts.append((time.perf_counter()-t)*1e6); inner.append(r.total_ms*1e3)
    return statistics.median(ts[100:]), statistics.median(inner[100:])

q = mp.Queue()
p = mp.Process(target=srv, args=(q,), daemon=True); p.start()
port = q.get()
rtt, inner = asyncio.run(client(port))
print(MODE, "rtt", round(rtt), "inner", round(inner), "transport", round(rtt-inner))
p.kill()
