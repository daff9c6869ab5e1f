"""The lean HTTP/1.1 client under the Kubernetes client (gpumounter_amd/cluster/http1.py):
bodies by length / chunks / close, keep-alive reuse, the idle-close race, watch streams split
into lines as they arrive, timeouts, cancellation and malformed answers."""
import asyncio

import pytest

from gpumounter_amd.cluster import http1


async def _server(handler):
    """A raw HTTP server: ``handler(reader, writer)`` per connection. Returns (server, url)."""
    srv = await asyncio.start_server(handler, "127.0.0.1", 0)
    port = srv.sockets[0].getsockname()[1]
    return srv, f"http://127.0.0.1:{port}"


async def _read_request(r):
    head = await r.readuntil(b"\r\n\r\n")
    lines = head.decode().split("\r\n")
    hdrs = {ln.split(":", 1)[0].lower(): ln.split(":", 1)[1].strip()
            for ln in lines[1:] if ":" in ln}
    body = await r.readexactly(int(hdrs.get("content-length", "0")))
    return lines[0], hdrs, body


def test_length_chunked_and_close_bodies_and_keepalive_reuse():
    conns = []

    async def handler(r, w):
        conns.append(w)
        try:
            while True:
                line, hdrs, body = await _read_request(r)
                path = line.split(" ")[1]
                if path == "/len":
                    w.write(b"HTTP/1.1 200 OK\r\nContent-Length: 5\r\n\r\nhello")
                elif path == "/chunked":
                    w.write(b"HTTP/1.1 201 Created\r\nTransfer-Encoding: chunked\r\n\r\n"
                            b"3\r\nabc\r\n4;ext=1\r\ndefg\r\n0\r\nX-Trailer: 1\r\n\r\n")
                elif path == "/continue":
                    w.write(b"HTTP/1.1 100 Continue\r\n\r\nHTTP/1.1 200 OK\r\n"
                            b"Content-Length: 2\r\n\r\nok")
                elif path == "/echo":
                    w.write(b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n" % len(body) + body)
                elif path.startswith("/q"):
                    w.write(b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n" % len(path)
                            + path.encode())
                elif path == "/close":
                    w.write(b"HTTP/1.1 200 OK\r\n\r\nuntil-close")
                    await w.drain()
                    w.close()
                    return
                await w.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            pass

    async def main():
        srv, url = await _server(handler)
        pool = http1.Pool(url, headers={"Accept": "application/json"})
        try:
            assert await pool.request("GET", "/len") == (200, {"content-length": "5"}, b"hello")
            st, hdrs, body = await pool.request("GET", "/chunked")
            assert (st, body) == (201, b"abcdefg")
            assert (await pool.request("GET", "/continue"))[2] == b"ok"
            assert (await pool.request("POST", "/echo", {"Content-Type": "x"}, b"payload"))[2] \
                == b"payload"
            assert (await pool.request("GET", pool.target("/q", {"a": "b c", "w": "1"})))[2] \
                == b"/q?a=b+c&w=1"
            assert len(conns) == 1                    # one keep-alive connection so far
            assert (await pool.request("GET", "/close"))[2] == b"until-close"
            assert (await pool.request("GET", "/len"))[2] == b"hello"
            assert len(conns) == 2                    # the closed one was not reused
        finally:
            await pool.close()
            srv.close()
    asyncio.run(main())


def test_a_connection_closed_while_idle_is_replaced_without_an_error():
    served = []

    async def handler(r, w):
        line, _, _ = await _read_request(r)
        served.append(line)
        w.write(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\nok")
        await w.drain()
        w.close()                # keep-alive announced, but closed after one answer

    async def main():
        srv, url = await _server(handler)
        pool = http1.Pool(url)
        try:
            for _ in range(3):
                assert (await pool.request("DELETE", "/x"))[0] == 200
                await asyncio.sleep(0.05)             # the close reaches the idle connection
            assert len(served) == 3
        finally:
            await pool.close()
            srv.close()
    asyncio.run(main())


def test_timeouts_cancellation_and_malformed_answers():
    async def handler(r, w):
        try:
            while True:
                line, _, _ = await _read_request(r)
                path = line.split(" ")[1]
                if path == "/slow":
                    await asyncio.sleep(0.5)
                    w.write(b"HTTP/1.1 200 OK\r\nContent-Length: 4\r\n\r\nslow")
                elif path == "/garbage":
                    w.write(b"NOT-HTTP garbage\r\n\r\n")
                elif path == "/cut":
                    w.write(b"HTTP/1.1 200 OK\r\nContent-Length: 10\r\n\r\nabc")
                    await w.drain()
                    w.close()
                    return
                else:
                    w.write(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\nok")
                await w.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            pass

    async def main():
        srv, url = await _server(handler)
        pool = http1.Pool(url, timeout_s=0.1)
        try:
            with pytest.raises(asyncio.TimeoutError):
                await pool.request("GET", "/slow")
            with pytest.raises(http1.HttpError):
                await pool.request("GET", "/garbage")
            with pytest.raises(http1.HttpError):
                await pool.request("GET", "/cut")
            pool.timeout_s = 5.0
            task = asyncio.ensure_future(pool.request("GET", "/slow"))
            await asyncio.sleep(0.05)
            task.cancel()
            with pytest.raises(asyncio.CancelledError):
                await task
            # the cancelled request's late answer never reaches the next request
            assert (await pool.request("GET", "/ok"))[2] == b"ok"
            assert not any(c._keep and c._state != "idle" for c, _ in pool._idle)
        finally:
            await pool.close()
            srv.close()
    asyncio.run(main())


def test_watch_stream_lines_arrive_as_sent_and_a_stall_times_out():
    gate = asyncio.Event()

    async def handler(r, w):
        line, _, _ = await _read_request(r)
        path = line.split(" ")[1]
        if path == "/gone":
            body = b'{"kind":"Status","code":410}'
            w.write(b"HTTP/1.1 410 Gone\r\nContent-Length: %d\r\n\r\n" % len(body) + body)
            await w.drain()
            return
        w.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n")
        # one event split over two chunks, then two events in one chunk
        for piece in (b'{"type":"ADDED",', b'"n":1}\n', b'{"type":"MODIFIED"}\n{"type":"X"}\n'):
            w.write(b"%x\r\n%s\r\n" % (len(piece), piece))
            await w.drain()
            await asyncio.sleep(0.01)
        if path == "/stall":
            await gate.wait()
        w.write(b"0\r\n\r\n")
        await w.drain()

    async def main():
        srv, url = await _server(handler)
        pool = http1.Pool(url)
        try:
            st, _, lines = await pool.stream("GET", "/watch")
            assert st == 200
            got = [ln async for ln in lines]
            assert got == [b'{"type":"ADDED","n":1}', b'{"type":"MODIFIED"}', b'{"type":"X"}']
            st, _, lines = await pool.stream("GET", "/stall", read_timeout_s=0.2)
            got = []
            with pytest.raises(asyncio.TimeoutError):
                async for ln in lines:
                    got.append(ln)
            assert len(got) == 3
            gate.set()
            st, _, lines = await pool.stream("GET", "/gone")
            assert st == 410 and [ln async for ln in lines] == [b'{"kind":"Status","code":410}']
        finally:
            await pool.close()
            srv.close()
    asyncio.run(main())


def test_header_override_and_https_options():
    seen = []

    async def handler(r, w):
        try:
            while True:
                line, hdrs, _ = await _read_request(r)
                seen.append(hdrs)
                w.write(b"HTTP/1.1 204 No Content\r\n\r\n")
                await w.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            pass

    async def main():
        srv, url = await _server(handler)
        pool = http1.Pool(url + "/prefix/", headers={"Authorization": "Bearer mine"})
        try:
            assert (await pool.request("GET", "/a"))[0] == 204
            assert (await pool.request("POST", "/b", {"Authorization": "Bearer theirs"}))[0] \
                == 204
        finally:
            await pool.close()
            srv.close()
        assert seen[0]["authorization"] == "Bearer mine"
        assert seen[1]["authorization"] == "Bearer theirs"      # replaced, not doubled
        assert seen[1]["content-length"] == "0"
    asyncio.run(main())
    p = http1.Pool("https://apiserver.example:6443", ssl_ctx=False)
    assert p.https and p.port == 6443 and p.ssl.verify_mode.name == "CERT_NONE"
    assert http1.Pool("https://[::1]").port == 443
