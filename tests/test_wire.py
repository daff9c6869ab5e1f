"""gm-wire (api/wire.py): the master → worker fast path next to the reference's gRPC API.

Framing, multiplexing, deadlines, error statuses, connection loss, mTLS peer identity, the
master's choice of transport and its fallback to gRPC."""
import asyncio
import subprocess

import grpc
import pytest

from gpumounter_amd.api import gpu_mount as api
from gpumounter_amd.api import wire
from gpumounter_amd.fakes.harness import LocalCluster


def _openssl(*args, cwd):
    subprocess.run(["openssl", *args], cwd=cwd, check=True, capture_output=True)


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    d = tmp_path_factory.mktemp("wirepki")
    ec = ("-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes")
    _openssl("req", "-x509", *ec, "-keyout", "ca.key", "-out", "ca.crt", "-days", "2",
             "-subj", "/CN=gm-wire-ca", cwd=d)
    for name, cn in (("server", "gpu-mounter-worker"), ("client", "gpu-mounter-master"),
                     ("intruder", "some-other-pod")):
        (d / f"{name}.ext").write_text(f"subjectAltName=DNS:{cn}\n")
        _openssl("req", *ec, "-keyout", f"{name}.key", "-out", f"{name}.csr",
                 "-subj", f"/CN={cn}", cwd=d)
        _openssl("x509", "-req", "-in", f"{name}.csr", "-CA", "ca.crt", "-CAkey", "ca.key",
                 "-CAcreateserial", "-out", f"{name}.crt", "-days", "2", "-extfile",
                 f"{name}.ext", cwd=d)
    return d


def _handlers(log=None):
    async def add(req):
        if log is not None:
            log.append(req.pod_name)
        if req.pod_name == "slow":
            await asyncio.sleep(0.2)
        if req.pod_name == "denied":
            raise wire.WireStatus(grpc.StatusCode.FAILED_PRECONDITION, "no: policy")
        if req.pod_name == "boom":
            raise RuntimeError("handler bug")
        return api.AddGPUResponse(add_gpu_result=api.ADD_SUCCESS, message=req.pod_name)
    return {wire.METHOD_ADD: (api.AddGPURequest.FromString, add)}


async def _call(ch, pod, timeout=5.0):
    out = await ch.call(wire.METHOD_ADD, api.AddGPURequest(pod_name=pod).SerializeToString(),
                        timeout)
    return api.AddGPUResponse.FromString(out)


def test_round_trip_statuses_and_multiplexing():
    async def main():
        srv = wire.WireServer(_handlers())
        port = await srv.start("127.0.0.1", 0)
        ch = wire.WireChannel("127.0.0.1", port)
        try:
            assert (await _call(ch, "a")).message == "a"
            # one connection, calls answered out of order: the slow one does not hold the rest
            slow = asyncio.ensure_future(_call(ch, "slow"))
            fast = await asyncio.gather(*[_call(ch, f"p{i}") for i in range(20)])
            assert [r.message for r in fast] == [f"p{i}" for i in range(20)]
            assert not slow.done()
            assert (await slow).message == "slow"
            assert len(srv.conns) == 1
            with pytest.raises(wire.WireError) as e:
                await _call(ch, "denied")
            assert e.value.code() == grpc.StatusCode.FAILED_PRECONDITION
            assert e.value.details() == "no: policy"
            with pytest.raises(wire.WireError) as e:
                await _call(ch, "boom")
            assert e.value.code() == grpc.StatusCode.INTERNAL
            with pytest.raises(wire.WireError) as e:
                await ch.call(wire.METHOD_STATUS, b"", 5.0)
            assert e.value.code() == grpc.StatusCode.UNIMPLEMENTED
            # a deadline: the caller gets DEADLINE_EXCEEDED; the late answer is dropped
            with pytest.raises(wire.WireError) as e:
                await _call(ch, "slow", timeout=0.05)
            assert e.value.code() == grpc.StatusCode.DEADLINE_EXCEEDED
            await asyncio.sleep(0.25)
            assert (await _call(ch, "after")).message == "after"
        finally:
            await ch.close()
            await srv.stop()
    asyncio.run(main())


def test_warm_opens_and_pings():
    """warm() connects in the background and pings: the server answers PING itself (no
    handler runs) and the channel is connected before the first real call."""
    async def main():
        log = []
        srv = wire.WireServer(_handlers(log))
        port = await srv.start("127.0.0.1", 0)
        ch = wire.WireChannel("127.0.0.1", port)
        try:
            ch.warm()
            for _ in range(100):
                if ch._conn is not None and ch._stream > 1:   # noqa: SLF001
                    break
                await asyncio.sleep(0.01)
            assert ch._stream == 3                            # noqa: SLF001 - one ping sent
            assert await ch.call(wire.METHOD_PING, b"", 2.0) == b""
            assert log == []
            assert (await _call(ch, "p")).message == "p"
        finally:
            await ch.close()
            await srv.stop()
    asyncio.run(main())


def test_connection_loss_and_unreachable():
    async def main():
        srv = wire.WireServer(_handlers())
        port = await srv.start("127.0.0.1", 0)
        ch = wire.WireChannel("127.0.0.1", port)
        assert (await _call(ch, "a")).message == "a"
        slow = asyncio.ensure_future(_call(ch, "slow"))
        await asyncio.sleep(0.02)
        await srv.stop()                   # the worker goes away with a call in flight
        with pytest.raises(wire.WireError) as e:
            await slow
        assert e.value.code() == grpc.StatusCode.UNAVAILABLE and e.value.sent
        # nothing listens now: the request never leaves
        with pytest.raises(wire.WireError) as e:
            await _call(ch, "b")
        assert e.value.code() == grpc.StatusCode.UNAVAILABLE and not e.value.sent
        # a worker back on the same port: the channel reconnects by itself
        srv2 = wire.WireServer(_handlers())
        await srv2.start("127.0.0.1", port)
        try:
            assert (await _call(ch, "c")).message == "c"
        finally:
            await ch.close()
            await srv2.stop()
    asyncio.run(main())


def test_garbage_closes_the_connection():
    async def main():
        srv = wire.WireServer(_handlers())
        port = await srv.start("127.0.0.1", 0)
        try:
            r, w = await asyncio.open_connection("127.0.0.1", port)
            w.write(b"\xff\xff\xff\xff" + b"x" * 16)      # a length over the 4 MiB limit
            assert await asyncio.wait_for(r.read(), 5) == b""
            r, w = await asyncio.open_connection("127.0.0.1", port)
            w.write(wire._frame(1, wire.KIND_RESP, 0, b""))   # noqa: SLF001 - not a request
            assert await asyncio.wait_for(r.read(), 5) == b""
            w.close()
        finally:
            await srv.stop()
    asyncio.run(main())


def test_mtls_identity(pki):
    async def main():
        sctx = wire.server_context(str(pki / "server.crt"), str(pki / "server.key"),
                                   str(pki / "ca.crt"))
        srv = wire.WireServer(_handlers(), sctx, ["gpu-mounter-master"])
        port = await srv.start("127.0.0.1", 0)
        try:
            ok = wire.WireChannel("127.0.0.1", port, wire.client_context(
                str(pki / "ca.crt"), str(pki / "client.crt"), str(pki / "client.key")),
                "gpu-mounter-worker")
            assert (await _call(ok, "a")).message == "a"
            await ok.close()
            # signed by the same CA, but not a master's identity: connection closed
            intruder = wire.WireChannel("127.0.0.1", port, wire.client_context(
                str(pki / "ca.crt"), str(pki / "intruder.crt"), str(pki / "intruder.key")),
                "gpu-mounter-worker")
            with pytest.raises(wire.WireError) as e:
                await _call(intruder, "a")
            assert e.value.code() == grpc.StatusCode.UNAVAILABLE
            await intruder.close()
            # no client certificate at all: the handshake fails
            anon = wire.WireChannel("127.0.0.1", port, wire.client_context(str(pki / "ca.crt")),
                                    "gpu-mounter-worker")
            with pytest.raises(wire.WireError) as e:
                await _call(anon, "a")
            assert e.value.code() == grpc.StatusCode.UNAVAILABLE
            await anon.close()
            # the worker's certificate must name tls_server_name
            wrong = wire.WireChannel("127.0.0.1", port, wire.client_context(
                str(pki / "ca.crt"), str(pki / "client.crt"), str(pki / "client.key")),
                "another-service")
            with pytest.raises(wire.WireError) as e:
                await _call(wrong, "a")
            assert not e.value.sent
            await wrong.close()
        finally:
            await srv.stop()
    asyncio.run(main())


@pytest.mark.parametrize("transport", ["auto", "grpc"])
def test_master_uses_wire_when_advertised(pki, transport):
    w = {"tls_cert": str(pki / "server.crt"), "tls_key": str(pki / "server.key"),
         "tls_ca": str(pki / "ca.crt")}
    m = {"tls_cert": str(pki / "client.crt"), "tls_key": str(pki / "client.key"),
         "tls_ca": str(pki / "ca.crt"), "master_transport": transport}

    async def main():
        async with LocalCluster(worker_overrides=w, master_overrides=m) as lc:
            lc.tenant("t")
            code, b = await lc.add("default", "t", 1)
            assert code == 200, b
            assert (await lc.remove("default", "t", [b["devices"][0]["uuid"]]))[0] == 200
            conns = lc.nodes["node-0"].worker.wire_server.conns
            assert len(conns) == (1 if transport == "auto" else 0)
            # the worker's refusals map to the same HTTP answers over either transport
            code, b = await lc.add("default", "nope", 1)
            assert code == 404
    asyncio.run(main())


def test_master_falls_back_to_grpc_when_wire_unreachable():
    async def main():
        async with LocalCluster() as lc:
            lc.tenant("t")
            h = lc.nodes["node-0"]
            await h.worker.wire_server.stop()           # advertised, but nothing listens
            code, b = await lc.add("default", "t", 1)
            assert code == 200, b
            assert (await lc.remove("default", "t", [b["devices"][0]["uuid"]]))[0] == 200
            assert any(until > 0 for until in lc.master.workers._wire_down.values())  # noqa
    asyncio.run(main())


def test_worker_restart_mid_session_over_wire():
    """A worker restart closes the master's gm-wire connection; the next attach reconnects."""
    async def main():
        async with LocalCluster() as lc:
            lc.tenant("t")
            code, b = await lc.add("default", "t", 1)
            assert code == 200
            assert (await lc.remove("default", "t", [b["devices"][0]["uuid"]]))[0] == 200
            await lc.stop_worker("node-0")
            w = await lc.start_worker("node-0")
            await lc.master.workers.informer.wait_for(
                lambda: lc.master.workers.target("node-0") == f"127.0.0.1:{w.grpc_port}", 10)
            code, b = await lc.add("default", "t", 1)
            assert code == 200, b
    asyncio.run(main())
