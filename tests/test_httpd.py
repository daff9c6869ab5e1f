"""The HTTP/1.1 server of the master and the worker (utils/httpd.py): framing, persistence,
routing answers as httprouter gives them (reference: cmd/GPUMounter-master/main.go:227-246), Go ParseForm bodies."""
import asyncio

import pytest

from gpumounter_amd.utils import httpd


def _server():
    r = httpd.Router()

    async def echo(req):
        form = await req.post()
        return httpd.json_response({"path": req.path, "info": req.match_info,
                                    "query": list(req.query.items()),
                                    "form": list(form.items()), "body": req.body.decode(),
                                    "auth": req.headers.get("authorization", "")})

    async def boom(req):
        raise RuntimeError("handler bug")

    r.add_get("/pods/{ns}/{pod}", echo)
    r.add_post("/pods/{ns}/{pod}", echo)
    r.add_get("/boom", boom)
    return httpd.HttpServer(r)


async def _exchange(port: int, raw: bytes, expect: int = 1) -> bytes:
    """Send ``raw`` on one connection; read until ``expect`` responses or EOF."""
    rd, wr = await asyncio.open_connection("127.0.0.1", port)
    wr.write(raw)
    out = b""
    while out.count(b"HTTP/1.1 ") < expect or not _complete(out, expect):
        chunk = await asyncio.wait_for(rd.read(65536), 5)
        if not chunk:
            break
        out += chunk
    wr.close()
    return out


def _complete(buf: bytes, n: int) -> bool:
    """``n`` responses with their whole Content-Length bodies are in ``buf``."""
    pos = 0
    for _ in range(n):
        end = buf.find(b"\r\n\r\n", pos)
        if end < 0:
            return False
        head = buf[pos:end].decode()
        cl = next((int(ln.split(":", 1)[1]) for ln in head.split("\r\n")
                   if ln.lower().startswith("content-length:")), 0)
        if len(buf) < end + 4 + cl:
            return False
        pos = end + 4 + cl
    return True


def run(coro_fn):
    async def main():
        srv = _server()
        port = await srv.start("127.0.0.1", 0)
        try:
            await coro_fn(port)
        finally:
            await srv.stop()
    asyncio.run(main())


def test_routes_and_httprouter_answers():
    async def go(port):
        out = await _exchange(port, b"GET /pods/default/a%2Db?x=1&x=2&y= HTTP/1.1\r\n"
                                    b"Host: h\r\nAuthorization: Bearer t\r\n\r\n")
        assert out.startswith(b"HTTP/1.1 200 OK\r\n")
        assert b'"info": {"ns": "default", "pod": "a-b"}' in out
        assert b'"query": [["x", "1"], ["x", "2"], ["y", ""]]' in out
        assert b'"auth": "Bearer t"' in out
        out = await _exchange(port, b"GET /nowhere HTTP/1.1\r\nHost: h\r\n\r\n")
        assert out.startswith(b"HTTP/1.1 404 Not Found\r\n") and out.endswith(
            b"404 page not found\n")
        out = await _exchange(port, b"DELETE /pods/a/b HTTP/1.1\r\nHost: h\r\n\r\n")
        assert out.startswith(b"HTTP/1.1 405 ") and b"Allow: GET, OPTIONS, POST\r\n" in out
        out = await _exchange(port, b"GET /boom HTTP/1.1\r\nHost: h\r\n\r\n")
        assert out.startswith(b"HTTP/1.1 500 ")
    run(go)


def test_forms_as_go_parseform():
    async def go(port):
        body = b"uuids=GPU-1&uuids=GPU-2"
        out = await _exchange(port, b"POST /pods/n/p HTTP/1.1\r\nHost: h\r\nContent-Type: "
                                    b"application/x-www-form-urlencoded\r\nContent-Length: "
                                    + str(len(body)).encode() + b"\r\n\r\n" + body)
        assert b'"form": [["uuids", "GPU-1"], ["uuids", "GPU-2"]]' in out
        # another content type contributes no fields (net/http ParseForm)
        out = await _exchange(port, b"POST /pods/n/p HTTP/1.1\r\nHost: h\r\nContent-Type: "
                                    b"text/plain\r\nContent-Length: 7\r\n\r\nuuids=x")
        assert b'"form": []' in out and b'"body": "uuids=x"' in out
        # chunked, with Expect: 100-continue
        out = await _exchange(port, b"POST /pods/n/p HTTP/1.1\r\nHost: h\r\nContent-Type: "
                                    b"application/x-www-form-urlencoded\r\n"
                                    b"Transfer-Encoding: chunked\r\n\r\n"
                                    b"6\r\nuuids=\r\n5\r\nGPU-9\r\n0\r\n\r\n")
        assert b'"form": [["uuids", "GPU-9"]]' in out
    run(go)


def test_expect_continue_before_the_body():
    async def go(port):
        rd, wr = await asyncio.open_connection("127.0.0.1", port)
        wr.write(b"POST /pods/n/p HTTP/1.1\r\nHost: h\r\nExpect: 100-continue\r\n"
                 b"Content-Length: 3\r\n\r\n")
        assert await asyncio.wait_for(rd.readuntil(b"\r\n\r\n"), 5) == \
            b"HTTP/1.1 100 Continue\r\n\r\n"
        wr.write(b"abc")
        head = await asyncio.wait_for(rd.readuntil(b"\r\n\r\n"), 5)
        assert head.startswith(b"HTTP/1.1 200 ")
        wr.close()
    run(go)


def test_keep_alive_pipelining_and_close():
    async def go(port):
        req = b"GET /pods/a/%d HTTP/1.1\r\nHost: h\r\n\r\n"
        out = await _exchange(port, b"".join(req % i for i in range(3)), expect=3)
        assert out.count(b"HTTP/1.1 200 OK") == 3
        assert out.index(b'"pod": "0"') < out.index(b'"pod": "1"') < out.index(b'"pod": "2"')
        # Connection: close → answered, then closed by the server
        rd, wr = await asyncio.open_connection("127.0.0.1", port)
        wr.write(b"GET /pods/a/b HTTP/1.1\r\nHost: h\r\nConnection: close\r\n\r\n")
        data = await asyncio.wait_for(rd.read(), 5)
        assert b"Connection: close" in data
        # HTTP/1.0 without keep-alive: closed after the answer too
        rd, wr = await asyncio.open_connection("127.0.0.1", port)
        wr.write(b"GET /pods/a/b HTTP/1.0\r\n\r\n")
        assert (await asyncio.wait_for(rd.read(), 5)).startswith(b"HTTP/1.1 200 ")
    run(go)


@pytest.mark.parametrize("raw,status", [
    (b"GARBAGE\r\n\r\n", b"400"),
    (b"GET /pods/a/b HTTP/2.0\r\n\r\n", b"400"),
    (b"GET /pods/a/b HTTP/1.1\r\nbad header\r\n\r\n", b"400"),
    (b"GET /pods/a/b HTTP/1.1\r\nX: " + b"a" * (20 << 10) + b"\r\n\r\n", b"431"),
    (b"POST /pods/a/b HTTP/1.1\r\nHost: h\r\nContent-Length: 99999999999\r\n\r\n", b"413"),
    (b"POST /pods/a/b HTTP/1.1\r\nHost: h\r\nContent-Length: -1\r\n\r\n", b"400"),
    (b"POST /pods/a/b HTTP/1.1\r\nHost: h\r\nTransfer-Encoding: gzip\r\n\r\n", b"501"),
    # round-5 findings: conflicting duplicate Content-Length (request smuggling behind a
    # proxy), a non-ASCII digit (str.isdigit accepted "\xb2" and int() then raised inside
    # data_received), Content-Length together with Transfer-Encoding
    (b"POST /pods/a/b HTTP/1.1\r\nHost: h\r\nContent-Length: 2\r\nContent-Length: 5\r\n\r\n"
     b"abcde", b"400"),
    (b"POST /pods/a/b HTTP/1.1\r\nHost: h\r\nContent-Length: \xb2\r\n\r\nab", b"400"),
    (b"POST /pods/a/b HTTP/1.1\r\nHost: h\r\nContent-Length: 3\r\n"
     b"Transfer-Encoding: chunked\r\n\r\n3\r\nabc\r\n0\r\n\r\n", b"400"),
    (b"POST /pods/a/b HTTP/1.1\r\nHost: h\r\nContent-Length: +3\r\n\r\nabc", b"400"),
    (b"POST /pods/a/b HTTP/1.1\r\nHost: h\r\nTransfer-Encoding: chunked\r\n\r\n"
     b"0x3\r\nabc\r\n0\r\n\r\n", b"400"),
    (b"POST /pods/a/b HTTP/1.1\r\nHost: h\r\nTransfer-Encoding: chunked\r\n\r\n"
     + b"f" * 5000, b"400"),
    (b"GET /pods/a/b HTTP/1.1\r\n\r\n", b"400"),                        # no Host
    (b"GET /pods/a%zz HTTP/1.1\r\nHost: h\r\n\r\n", b"400"),              # bad escape
    (b"GET /pods/a/b HTTP/1.1\r\nHost: h\r\nX : y\r\n\r\n", b"400"),
    (b"GET /pods/a/b HTTP/1.1\r\nHost: h\r\nX: a\x00b\r\n\r\n", b"400"),
])
def test_malformed_requests(raw, status):
    async def go(port):
        out = await _exchange(port, raw)
        assert out.startswith(b"HTTP/1.1 " + status), out[:80]
        assert b"Connection: close" in out
    run(go)
