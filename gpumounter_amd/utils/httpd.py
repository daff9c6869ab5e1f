"""The master's HTTP/1.1 server: a small asyncio protocol for a small, fixed API.

The reference serves its routes with julienschmidt/httprouter on net/http (reference:
cmd/GPUMounter-master/main.go:227-246). An aiohttp application did the same here until round 4;
for the attach path it cost more than the rest of the master's own work together (request and
response objects, a handler task, header multidicts, the access-log hook: ≈0.07 ms of the
client ⇄ master hop on an MI355X host, ``profiles/r5_hop/``). This server keeps only what the
API needs:

* request line + headers (≤ 16 KiB, else 431), ``Content-Length`` or ``chunked`` bodies
  (≤ 10 MiB, net/http's ``ParseForm`` limit), ``Expect: 100-continue``;
* persistent connections (HTTP/1.1 default, ``Connection: close``, HTTP/1.0 keep-alive) with
  requests on one connection answered in order, an idle timeout of 75 s;
* httprouter's routing answers: a path no route has → ``404 page not found``, a route without
  the method → ``405 Method Not Allowed`` with ``Allow``;
* handlers get a :class:`Request` (``match_info``, ``headers``, ``query``, ``post()``,
  ``json()``, ``remote``) and return a :class:`Response` (:func:`text`, :func:`json_response`).

``POST`` forms are parsed as Go's ``r.ParseForm`` does: ``application/x-www-form-urlencoded``
bodies; any other content type contributes no fields (main.go:121).
"""
from __future__ import annotations

import asyncio
import email.utils
import json
import re
import time
import urllib.parse
from typing import Awaitable, Callable, Dict, List, Optional, Tuple

from multidict import CIMultiDict, MultiDict

from gpumounter_amd.utils import log

_log = log.get("httpd")

MAX_HEAD = 16 << 10
MAX_BODY = 10 << 20
IDLE_TIMEOUT_S = 75.0
_REASONS = {100: "Continue", 200: "OK", 201: "Created", 301: "Moved Permanently",
            400: "Bad Request", 401: "Unauthorized", 403: "Forbidden", 404: "Not Found",
            405: "Method Not Allowed", 411: "Length Required", 413: "Payload Too Large",
            431: "Request Header Fields Too Large", 500: "Internal Server Error",
            501: "Not Implemented", 502: "Bad Gateway", 503: "Service Unavailable"}


class Response:
    __slots__ = ("status", "body", "content_type", "headers")

    def __init__(self, body: bytes = b"", status: int = 200,
                 content_type: str = "text/plain; charset=utf-8",
                 headers: Optional[Dict[str, str]] = None) -> None:
        self.status = status
        self.body = body
        self.content_type = content_type
        self.headers = headers or {}

    @property
    def text(self) -> str:
        return self.body.decode()


def text(body: str, status: int = 200, content_type: str = "text/plain; charset=utf-8"
         ) -> Response:
    return Response(body.encode(), status, content_type)


def json_response(data, status: int = 200) -> Response:
    return Response(json.dumps(data).encode(), status, "application/json; charset=utf-8")


class Request:
    __slots__ = ("method", "path", "query_string", "version", "headers", "body", "match_info",
                 "remote", "_query", "_vals", "t_in")

    def __init__(self, method: str, path: str, query_string: str, version: str,
                 headers: CIMultiDict, body: bytes, remote: Optional[str]) -> None:
        self.method = method
        self.path = path
        self.query_string = query_string
        self.version = version
        self.headers = headers
        self.body = body
        self.remote = remote
        self.match_info: Dict[str, str] = {}
        self._query: Optional[MultiDict] = None
        self._vals: Dict[str, object] = {}
        self.t_in = 0.0          # time.monotonic() of the data_received that began it

    @property
    def query(self) -> MultiDict:
        if self._query is None:
            self._query = MultiDict(urllib.parse.parse_qsl(self.query_string,
                                                           keep_blank_values=True))
        return self._query

    @property
    def can_read_body(self) -> bool:
        return bool(self.body)

    async def post(self) -> MultiDict:
        """The body's form fields (Go ``ParseForm``: url-encoded bodies only)."""
        ctype = self.headers.get("Content-Type", "").split(";", 1)[0].strip().lower()
        if ctype != "application/x-www-form-urlencoded" or not self.body:
            return MultiDict()
        return MultiDict(urllib.parse.parse_qsl(self.body.decode("utf-8"),
                                                keep_blank_values=True, strict_parsing=False))

    async def json(self):
        return json.loads(self.body or b"null")

    # per-request values set by the handlers (the caller's identity)
    def __getitem__(self, key: str):
        return self._vals[key]

    def __setitem__(self, key: str, value) -> None:
        self._vals[key] = value

    def get(self, key: str, default=None):
        return self._vals.get(key, default)


Handler = Callable[[Request], Awaitable[Response]]


class Router:
    """httprouter-style: ``/a/{name}/b`` patterns, one segment per ``{name}``."""

    def __init__(self) -> None:
        self._routes: List[Tuple[re.Pattern, Dict[str, Handler]]] = []
        self._index: Dict[str, int] = {}

    def add(self, method: str, pattern: str, handler: Handler) -> None:
        if pattern not in self._index:
            rx = "^" + re.sub(r"\\\{(\w+)\\\}", r"(?P<\1>[^/]+)", re.escape(pattern)) + "$"
            self._index[pattern] = len(self._routes)
            self._routes.append((re.compile(rx), {}))
        self._routes[self._index[pattern]][1][method] = handler

    def add_get(self, pattern: str, handler: Handler) -> None:
        self.add("GET", pattern, handler)

    def add_post(self, pattern: str, handler: Handler) -> None:
        self.add("POST", pattern, handler)

    def resolve(self, method: str, path: str):
        """(handler, match_info) | (None, allowed methods) | (None, None) for no route."""
        for rx, methods in self._routes:
            m = rx.match(path)
            if m is None:
                continue
            h = methods.get(method)
            if h is None:
                return None, sorted(methods)
            return h, {k: urllib.parse.unquote(v) for k, v in m.groupdict().items()}
        return None, None


_date_cache = [0, b""]


def _date() -> bytes:
    now = int(time.time())
    if now != _date_cache[0]:
        _date_cache[0] = now
        _date_cache[1] = email.utils.formatdate(now, usegmt=True).encode()
    return _date_cache[1]


class _Conn(asyncio.Protocol):
    def __init__(self, srv: "HttpServer") -> None:
        self.srv = srv
        self.t: Optional[asyncio.Transport] = None
        self.buf = bytearray()
        self.busy = False              # a request is being handled (answered in order)
        self.remote: Optional[str] = None
        self.idle: Optional[asyncio.TimerHandle] = None
        self._continued = False        # "100 Continue" sent for the request being read
        self.t_first = 0.0             # when the request being read began to arrive

    # ------------------------------------------------------------------ transport callbacks
    def connection_made(self, transport) -> None:
        self.t = transport
        peer = transport.get_extra_info("peername")
        self.remote = peer[0] if isinstance(peer, tuple) else None
        self.srv.conns.add(self)
        self._arm_idle()

    def connection_lost(self, exc) -> None:
        self.t = None
        self.srv.conns.discard(self)
        if self.idle is not None:
            self.idle.cancel()

    def data_received(self, data: bytes) -> None:
        if not self.buf:
            self.t_first = time.monotonic()
        self.buf += data
        if not self.busy:
            self._next()

    # ------------------------------------------------------------------ parsing
    def _arm_idle(self) -> None:
        if self.idle is not None:
            self.idle.cancel()
        self.idle = self.srv.loop.call_later(IDLE_TIMEOUT_S, self._idle_close)

    def _idle_close(self) -> None:
        if self.t is not None and not self.busy:
            self.t.close()

    def _fail(self, status: int, body: str = "") -> None:
        self._write(Response((body or _REASONS.get(status, "")).encode() + b"\n", status),
                    close=True)

    def _next(self) -> None:
        """Parse and dispatch the next complete request in the buffer, if there is one."""
        if self.t is None:
            return
        buf = self.buf
        end = buf.find(b"\r\n\r\n")
        if end < 0:
            if len(buf) > MAX_HEAD:
                self._fail(431)
            return
        if end > MAX_HEAD:
            self._fail(431)
            return
        lines = bytes(buf[:end]).decode("latin-1").split("\r\n")
        try:
            method, target, version = lines[0].split(" ")
        except ValueError:
            self._fail(400)
            return
        if version not in ("HTTP/1.1", "HTTP/1.0") or not target.startswith("/"):
            self._fail(400)
            return
        headers = CIMultiDict()
        for ln in lines[1:]:
            name, sep, value = ln.partition(":")
            if not sep or not name or name != name.strip():
                self._fail(400)
                return
            headers.add(name, value.strip())
        start = end + 4
        te = headers.get("Transfer-Encoding", "").lower()
        if te:
            if te != "chunked":
                self._fail(501)
                return
            got = self._dechunk(start)
            if got is None:
                return                       # incomplete (or failed: already answered)
            body, consumed = got
        else:
            cl = headers.get("Content-Length", "0")
            if not cl.isdigit():
                self._fail(400)
                return
            n = int(cl)
            if n > MAX_BODY:
                self._fail(413)
                return
            if len(buf) < start + n:
                self._continue(headers, version)
                return
            body, consumed = bytes(buf[start:start + n]), start + n
        del buf[:consumed]
        path, _, qs = target.partition("?")
        conn_hdr = headers.get("Connection", "").lower()
        keep = conn_hdr == "keep-alive" if version == "HTTP/1.0" else conn_hdr != "close"
        req = Request(method, path, qs, version, headers, body, self.remote)
        req.t_in = self.t_first
        if buf:
            self.t_first = time.monotonic()  # a pipelined request: already (partly) here
        self.busy = True
        if self.idle is not None:
            self.idle.cancel()
            self.idle = None
        self.srv.loop.create_task(self._handle(req, keep))

    def _continue(self, headers: CIMultiDict, version: str) -> None:
        if version == "HTTP/1.1" and headers.get("Expect", "").lower() == "100-continue" and \
                not self._continued:
            self._continued = True
            self.t.write(b"HTTP/1.1 100 Continue\r\n\r\n")

    def _dechunk(self, start: int):
        buf, pos, out = self.buf, start, bytearray()
        while True:
            eol = buf.find(b"\r\n", pos)
            if eol < 0:
                return None
            size_s = bytes(buf[pos:eol]).split(b";", 1)[0].strip()
            try:
                size = int(size_s, 16)
            except ValueError:
                self._fail(400)
                return None
            if size == 0:
                end = buf.find(b"\r\n\r\n", eol)    # optional trailers, then the blank line
                if end < 0:
                    return None
                return bytes(out), end + 4
            if len(out) + size > MAX_BODY:
                self._fail(413)
                return None
            if len(buf) < eol + 2 + size + 2:
                return None
            out += buf[eol + 2:eol + 2 + size]
            pos = eol + 2 + size + 2

    # ------------------------------------------------------------------ dispatch
    async def _handle(self, req: Request, keep: bool) -> None:
        self._continued = False
        h, info = self.srv.router.resolve(req.method, req.path)
        try:
            if h is None:
                if info is None:
                    resp = Response(b"404 page not found\n", 404)
                else:
                    resp = Response(b"Method Not Allowed\n", 405,
                                    headers={"Allow": ", ".join(info)})
            else:
                req.match_info = info
                resp = await h(req)
        except Exception:  # noqa: BLE001 - net/http answers 500 and keeps serving
            _log.exception("%s %s failed", req.method, req.path)
            resp = Response(b"Internal Server Error\n", 500)
        self._write(resp, close=not keep)
        self.busy = False
        if self.t is not None:
            if self.buf:
                self._next()                 # a pipelined request already arrived
            else:
                self._arm_idle()

    def _write(self, resp: Response, close: bool) -> None:
        if self.t is None:
            return
        head = [b"HTTP/1.1 %d %s\r\n" % (resp.status, _REASONS.get(resp.status, "").encode()),
                b"Content-Type: ", resp.content_type.encode(), b"\r\n",
                b"Content-Length: %d\r\n" % len(resp.body), b"Date: ", _date(), b"\r\n"]
        for k, v in resp.headers.items():
            head += [k.encode(), b": ", v.encode(), b"\r\n"]
        if close:
            head.append(b"Connection: close\r\n")
        head.append(b"\r\n")
        self.t.write(b"".join(head) + resp.body)
        if close:
            self.t.close()


class HttpServer:
    def __init__(self, router: Router) -> None:
        self.router = router
        self.conns: set = set()
        self.server: Optional[asyncio.AbstractServer] = None
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.port = 0

    async def start(self, host: str, port: int) -> int:
        self.loop = asyncio.get_running_loop()
        self.server = await self.loop.create_server(lambda: _Conn(self), host, port,
                                                    reuse_address=True)
        self.port = self.server.sockets[0].getsockname()[1]
        return self.port

    async def stop(self) -> None:
        if self.server is None:
            return
        self.server.close()
        for c in list(self.conns):
            if c.t is not None and not c.busy:
                c.t.close()
        await self.server.wait_closed()
        self.server = None
        # requests still being answered finish; their connections close once written
        for _ in range(100):
            if not any(c.busy for c in self.conns):
                break
            await asyncio.sleep(0.05)
        for c in list(self.conns):
            if c.t is not None:
                c.t.close()
