"""The master's (and the worker's status port's) HTTP/1.1 server: a small asyncio protocol for a
small, fixed API.

The reference serves its routes with julienschmidt/httprouter v1.3.0 on net/http (reference:
cmd/GPUMounter-master/main.go:227-246, go.mod:7). An aiohttp application did the same here until
round 4; for the attach path it cost more than the rest of the master's own work together
(``profiles/r5_hop/``). This server keeps only what the API needs, with net/http's limits:

* request line + headers (≤ 16 KiB, else 431), ``Content-Length`` or ``chunked`` bodies
  (≤ 10 MiB, net/http's ``ParseForm`` limit, else 413), ``Expect: 100-continue``;
* strict framing, as net/http answers it: a Content-Length of ASCII digits only, duplicate
  Content-Length headers only when equal, never together with Transfer-Encoding, only the
  ``chunked`` coding, a Host header on HTTP/1.1, header names that are tokens — anything else
  is ``400`` and the connection closes (a framing disagreement with a proxy in front is how
  requests are smuggled);
* bounded memory per connection: reading pauses while a request is being handled (pipelined
  bytes wait in the kernel, not here), a buffer beyond head + body limits is refused, chunked
  bodies are parsed incrementally (state kept between packets, linear time), and the server
  accepts at most ``max_conns`` connections (``503`` beyond);
* persistent connections (HTTP/1.1 default, ``Connection: close``, HTTP/1.0 keep-alive) with
  requests on one connection answered in order, an idle timeout of 75 s;
* httprouter's routing, on the percent-decoded path as net/http hands it to the router
  (``%2F`` is a ``/`` there, so it can never end up inside a path parameter): a route without
  the method → ``405`` with ``Allow``; ``OPTIONS`` → ``200`` with ``Allow``; a path with or
  without a trailing slash that a route has → redirect (``301``, ``307`` for methods other than
  GET); a path that matches once cleaned (``//``, ``.``, ``..``) or case-folded → the same
  redirect; otherwise ``404 page not found``;
* optional TLS (``ssl`` on :meth:`HttpServer.start`);
* handlers get a :class:`Request` (``match_info``, ``headers``, ``query``, ``post()``,
  ``json()``, ``remote``) and return a :class:`Response` (:func:`text`, :func:`json_response`).

``POST`` forms are parsed as Go's ``r.ParseForm`` does: ``application/x-www-form-urlencoded``
bodies; any other content type contributes no fields (main.go:121).
"""
from __future__ import annotations

import asyncio
import email.utils
import json
import posixpath
import re
import time
import urllib.parse
from typing import Awaitable, Callable, Dict, List, Optional, Tuple

from multidict import CIMultiDict, MultiDict

from gpumounter_amd.utils import log

_log = log.get("httpd")

MAX_HEAD = 16 << 10
MAX_BODY = 10 << 20
MAX_CHUNK_LINE = 4096          # a chunk-size line with its extensions
MAX_CONNS = 1024
IDLE_TIMEOUT_S = 75.0
_REASONS = {100: "Continue", 200: "OK", 201: "Created", 301: "Moved Permanently",
            307: "Temporary Redirect", 400: "Bad Request", 401: "Unauthorized",
            403: "Forbidden", 404: "Not Found", 405: "Method Not Allowed",
            411: "Length Required", 413: "Payload Too Large",
            431: "Request Header Fields Too Large", 500: "Internal Server Error",
            501: "Not Implemented", 502: "Bad Gateway", 503: "Service Unavailable"}
# RFC 9110 token characters (method and header names)
_TOKEN = re.compile(rb"^[!#$%&'*+\-.^_`|~0-9A-Za-z]+$")
_DIGITS = re.compile(rb"^[0-9]{1,15}$")
_HEXSIZE = re.compile(rb"^[0-9A-Fa-f]{1,15}$")
_BAD_ESCAPE = re.compile(r"%(?![0-9A-Fa-f]{2})")
# header values: visible ASCII, obs-text, SP and HTAB (no CTLs: NUL, bare CR/LF, DEL)
_FIELD_VALUE = re.compile(rb"^[\t\x20-\x7e\x80-\xff]*$")


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
    __slots__ = ("method", "path", "raw_path", "query_string", "version", "headers", "body",
                 "match_info", "remote", "_query", "_vals", "t_in")

    def __init__(self, method: str, path: str, query_string: str, version: str,
                 headers: CIMultiDict, body: bytes, remote: Optional[str],
                 raw_path: str = "") -> None:
        self.method = method
        self.path = path                  # percent-decoded (Go's r.URL.Path)
        self.raw_path = raw_path or path  # as sent
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


def clean_path(p: str) -> str:
    """httprouter's ``CleanPath``: ``path.Clean`` that keeps a trailing slash and roots the
    path."""
    if not p:
        return "/"
    out = posixpath.normpath("/" + p)
    if out.startswith("//"):            # normpath keeps a leading "//" (POSIX); Go does not
        out = "/" + out.lstrip("/")
    if p.endswith("/") and out != "/":
        out += "/"
    return out


class Router:
    """httprouter v1.3.0 semantics over ``/a/{name}/b`` patterns (one non-empty segment per
    ``{name}``; ``{name}`` here is httprouter's ``:name``)."""

    def __init__(self) -> None:
        # pattern segments ("" for the root) → {method: handler}
        self._routes: List[Tuple[Tuple[str, ...], Dict[str, Handler]]] = []
        self._index: Dict[str, int] = {}

    def add(self, method: str, pattern: str, handler: Handler) -> None:
        if pattern not in self._index:
            self._index[pattern] = len(self._routes)
            self._routes.append((tuple(pattern.split("/")[1:]), {}))
        self._routes[self._index[pattern]][1][method] = handler

    def add_get(self, pattern: str, handler: Handler) -> None:
        self.add("GET", pattern, handler)

    def add_post(self, pattern: str, handler: Handler) -> None:
        self.add("POST", pattern, handler)

    @staticmethod
    def _match(segs: Tuple[str, ...], parts: List[str], fold: bool
               ) -> Optional[Tuple[Dict[str, str], List[str]]]:
        """(params, canonical parts) when ``parts`` fits the pattern ``segs``."""
        if len(segs) != len(parts):
            return None
        params: Dict[str, str] = {}
        canon = []
        for s, p in zip(segs, parts):
            if s.startswith("{") and s.endswith("}"):
                if not p:
                    return None
                params[s[1:-1]] = p
                canon.append(p)
            elif s == p or (fold and s.lower() == p.lower()):
                canon.append(s)
            else:
                return None
        return params, canon

    def _lookup(self, method: str, path: str, fold: bool = False):
        parts = path.split("/")[1:]
        for segs, methods in self._routes:
            if method is not None and method not in methods:
                continue
            m = self._match(segs, parts, fold)
            if m is not None:
                return methods, m[0], "/" + "/".join(m[1])
        return None

    def allowed(self, path: str) -> List[str]:
        """httprouter ``allowed``: the methods some route serves at ``path``, plus OPTIONS."""
        if path == "*":
            out = {m for _, methods in self._routes for m in methods}
        else:
            parts = path.split("/")[1:]
            out = {m for segs, methods in self._routes for m in methods
                   if self._match(segs, parts, False) is not None}
        out.discard("OPTIONS")
        return sorted(out | {"OPTIONS"}) if out else []

    def _redirect(self, method: str, path: str) -> Optional[str]:
        """httprouter's RedirectTrailingSlash + RedirectFixedPath target for ``path``."""
        if method == "CONNECT" or path == "/":
            return None
        alt = path[:-1] if len(path) > 1 and path.endswith("/") else path + "/"
        if self._lookup(method, alt) is not None:
            return alt
        cleaned = clean_path(path)
        for cand in (cleaned, cleaned[:-1] if len(cleaned) > 1 and cleaned.endswith("/")
                     else cleaned + "/"):
            hit = self._lookup(method, cand, fold=True)
            if hit is not None:
                return hit[2]
        return None

    def resolve(self, method: str, path: str):
        """(handler, match_info) | (None, allowed methods) | (None, None) for no route."""
        hit = self._lookup(method, path)
        if hit is not None:
            return hit[0][method], hit[1]
        allow = self.allowed(path)
        return None, (allow or None)

    def route(self, req: Request) -> Tuple[Optional[Handler], Optional[Response]]:
        """What httprouter's ServeHTTP does with ``req``: the handler (and ``match_info`` set),
        or the answer it gives itself (redirect, OPTIONS, 405, 404)."""
        method, path = req.method, req.path
        if path != "*":
            hit = self._lookup(method, path)
            if hit is not None:
                req.match_info = hit[1]
                return hit[0][method], None
            if any(method in methods for _, methods in self._routes):
                to = self._redirect(method, path)
                if to is not None:
                    code = 301 if method == "GET" else 307
                    loc = urllib.parse.quote(to, safe="/:@!$&'()*+,;=-._~") + \
                        (f"?{req.query_string}" if req.query_string else "")
                    body = f'<a href="{loc}">{_REASONS[code]}</a>.\n\n'.encode() \
                        if method in ("GET", "HEAD") else b""
                    return None, Response(body, code, "text/html; charset=utf-8",
                                          headers={"Location": loc})
        allow = self.allowed(path)
        if method == "OPTIONS":
            if allow:
                return None, Response(b"", 200, "", headers={"Allow": ", ".join(allow)})
        elif allow:
            return None, Response(b"Method Not Allowed\n", 405,
                                  headers={"Allow": ", ".join(allow),
                                           "X-Content-Type-Options": "nosniff"})
        return None, Response(b"404 page not found\n", 404,
                              headers={"X-Content-Type-Options": "nosniff"})


_date_cache = [0, b""]


def _date() -> bytes:
    now = int(time.time())
    if now != _date_cache[0]:
        _date_cache[0] = now
        _date_cache[1] = email.utils.formatdate(now, usegmt=True).encode()
    return _date_cache[1]


class BadRequest(Exception):
    def __init__(self, status: int, msg: str = "") -> None:
        super().__init__(msg or _REASONS.get(status, ""))
        self.status = status


def decode_path(raw: str) -> str:
    """``r.URL.Path`` from the request target's path: percent-decoded; an invalid escape is a
    400 (net/http: "invalid URL escape")."""
    if "%" not in raw:
        return raw
    if _BAD_ESCAPE.search(raw):
        raise BadRequest(400, "invalid URL escape")
    return urllib.parse.unquote_to_bytes(raw).decode("utf-8", "surrogateescape")


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
        self._paused = False
        self._scan = 0                 # head: bytes of buf already searched for its end
        # the request being read past its head: (method, target, version, headers, keep)
        self._req: Optional[tuple] = None
        self._body = bytearray()
        self._need = 0                 # Content-Length bytes still to come
        self._chunk = ""               # "" | "size" | "data" | "crlf" | "trailer"

    # ------------------------------------------------------------------ transport callbacks
    def connection_made(self, transport) -> None:
        self.t = transport
        peer = transport.get_extra_info("peername")
        self.remote = peer[0] if isinstance(peer, tuple) else None
        if len(self.srv.conns) >= self.srv.max_conns:
            self.srv.refused += 1
            self._write(Response(b"Service Unavailable: too many connections\n", 503),
                        close=True)
            return
        self.srv.conns.add(self)
        self._arm_idle()

    def connection_lost(self, exc) -> None:
        self.t = None
        self.srv.conns.discard(self)
        if self.idle is not None:
            self.idle.cancel()

    def data_received(self, data: bytes) -> None:
        if self.t is None or self.t.is_closing():
            return
        if not self.buf and self._req is None:
            self.t_first = time.monotonic()
        self.buf += data
        if len(self.buf) > MAX_HEAD + MAX_BODY + (64 << 10):
            # only a transport that ignored pause_reading while a request is in flight gets
            # here: an answer now would overtake that request's, so the connection just ends
            self.buf.clear()
            self._req = None
            if self.busy:
                self.t.close()
            else:
                self._fail(413)
            return
        if self.busy:
            # one request at a time: later bytes stay in the kernel until it is answered
            self._pause()
            return
        self._next()

    def _pause(self) -> None:
        if not self._paused and self.t is not None:
            self._paused = True
            self.t.pause_reading()

    def _resume(self) -> None:
        if self._paused and self.t is not None:
            self._paused = False
            self.t.resume_reading()

    # ------------------------------------------------------------------ parsing
    def _arm_idle(self) -> None:
        if self.idle is not None:
            self.idle.cancel()
        self.idle = self.srv.loop.call_later(IDLE_TIMEOUT_S, self._idle_close)

    def _idle_close(self) -> None:
        if self.t is not None and not self.busy:
            self.t.close()

    def _fail(self, status: int, body: str = "") -> None:
        self._req = None
        self.buf.clear()
        self._write(Response((body or _REASONS.get(status, "")).encode() + b"\n", status),
                    close=True)

    def _next(self) -> None:
        """Parse what the buffer holds; dispatch a request once it is complete."""
        if self.t is None or self.t.is_closing():
            return
        try:
            if self._req is None and not self._parse_head():
                return
            body = self._parse_body()
        except BadRequest as e:
            self._fail(e.status, str(e))
            return
        if body is None:
            return
        method, target, version, headers, keep = self._req
        self._req = None
        raw_path, _, qs = target.partition("?")
        try:
            path = "*" if raw_path == "*" else decode_path(raw_path)
        except BadRequest as e:
            self._fail(e.status, str(e))
            return
        req = Request(method, path, qs, version, headers, body, self.remote, raw_path)
        req.t_in = self.t_first
        if self.buf:
            self.t_first = time.monotonic()  # a pipelined request: already (partly) here
        self.busy = True
        if self.idle is not None:
            self.idle.cancel()
            self.idle = None
        self._dispatch(req, keep)

    def _dispatch(self, req: Request, keep: bool) -> None:
        self.srv.loop.create_task(self._handle(req, keep))

    def _parse_head(self) -> bool:
        buf = self.buf
        end = buf.find(b"\r\n\r\n", max(self._scan - 3, 0), MAX_HEAD + 4)
        if end < 0:
            if len(buf) > MAX_HEAD:
                raise BadRequest(431)
            self._scan = len(buf)
            return False
        self._scan = 0
        head = bytes(buf[:end])
        del buf[:end + 4]
        lines = head.split(b"\r\n")
        rl = lines[0].split(b" ")
        if len(rl) != 3 or not _TOKEN.match(rl[0]):
            raise BadRequest(400, "malformed request line")
        method, target, version = (x.decode("latin-1") for x in rl)
        if version not in ("HTTP/1.1", "HTTP/1.0"):
            raise BadRequest(400, "unsupported protocol version")
        if not (target.startswith("/") or (target == "*" and method == "OPTIONS")) or \
                any(c <= " " or c == "\x7f" for c in target):
            raise BadRequest(400, "invalid request target")
        headers = CIMultiDict()
        for ln in lines[1:]:
            name, sep, value = ln.partition(b":")
            if not sep or not _TOKEN.match(name):
                raise BadRequest(400, "malformed header line")
            value = value.strip(b" \t")
            if not _FIELD_VALUE.match(value):
                raise BadRequest(400, "invalid header value")
            headers.add(name.decode("latin-1"), value.decode("latin-1"))
        if version == "HTTP/1.1" and len(headers.getall("Host", [])) != 1:
            raise BadRequest(400, "missing required Host header" if "Host" not in headers
                             else "too many Host headers")
        tes = headers.getall("Transfer-Encoding", [])
        cls = headers.getall("Content-Length", [])
        if tes:
            if cls:
                raise BadRequest(400, "Transfer-Encoding and Content-Length both present")
            if len(tes) != 1 or tes[0].lower() != "chunked":
                raise BadRequest(501, f"unsupported transfer encoding: {','.join(tes)!r}")
            if version == "HTTP/1.0":
                raise BadRequest(400, "chunked encoding in HTTP/1.0")
            self._chunk, self._need = "size", 0
        else:
            if cls and (len(set(cls)) != 1 or not _DIGITS.match(cls[0].encode("latin-1"))):
                raise BadRequest(400, "invalid Content-Length")
            self._need = int(cls[0]) if cls else 0
            if self._need > MAX_BODY:
                raise BadRequest(413)
            self._chunk = ""
        conn_hdr = ",".join(headers.getall("Connection", [])).lower()
        keep = "keep-alive" in conn_hdr if version == "HTTP/1.0" else "close" not in conn_hdr
        self._req = (method, target, version, headers, keep)
        self._body = bytearray()
        self._continued = False
        return True

    def _parse_body(self) -> Optional[bytes]:
        """The body once complete (None: more bytes needed); keeps its state between
        packets so a slow body costs linear time."""
        buf = self.buf
        if not self._chunk:
            if len(buf) < self._need:
                self._expect_continue()
                return None
            body = bytes(buf[:self._need])
            del buf[:self._need]
            return body
        while True:
            if self._chunk == "size":
                eol = buf.find(b"\r\n", 0, MAX_CHUNK_LINE + 2)
                if eol < 0:
                    if len(buf) > MAX_CHUNK_LINE:
                        raise BadRequest(400, "chunk-size line too long")
                    self._expect_continue()
                    return None
                size = bytes(buf[:eol]).split(b";", 1)[0].rstrip(b" \t")
                if not _HEXSIZE.match(size):
                    raise BadRequest(400, "invalid chunk size")
                del buf[:eol + 2]
                self._need = int(size, 16)
                if len(self._body) + self._need > MAX_BODY:
                    raise BadRequest(413)
                self._chunk = "data" if self._need else "trailer"
            elif self._chunk == "data":
                if not buf:
                    return None
                take = min(self._need, len(buf))
                self._body += buf[:take]
                del buf[:take]
                self._need -= take
                if self._need:
                    return None
                self._chunk = "crlf"
            elif self._chunk == "crlf":
                if len(buf) < 2:
                    return None
                if buf[:2] != b"\r\n":
                    raise BadRequest(400, "malformed chunk")
                del buf[:2]
                self._chunk = "size"
            else:                           # trailer fields, then the blank line
                eol = buf.find(b"\r\n", 0, MAX_HEAD + 2)
                if eol < 0:
                    if len(buf) > MAX_HEAD:
                        raise BadRequest(431)
                    return None
                line = bytes(buf[:eol])
                del buf[:eol + 2]
                if not line:
                    self._chunk = ""
                    return bytes(self._body)
                name, sep, _ = line.partition(b":")
                if not sep or not _TOKEN.match(name):
                    raise BadRequest(400, "malformed trailer")

    def _expect_continue(self) -> None:
        _, _, version, headers, _ = self._req
        if version == "HTTP/1.1" and headers.get("Expect", "").lower() == "100-continue" and \
                not self._continued:
            self._continued = True
            self.t.write(b"HTTP/1.1 100 Continue\r\n\r\n")

    # ------------------------------------------------------------------ dispatch
    async def _handle(self, req: Request, keep: bool) -> None:
        h, resp = self.srv.router.route(req)
        try:
            if h is not None:
                resp = await h(req)
        except Exception:  # noqa: BLE001 - net/http answers 500 and keeps serving
            _log.exception("%s %s failed", req.method, req.path)
            resp = Response(b"Internal Server Error\n", 500)
        self._write(resp, close=not keep)
        self.busy = False
        if self.t is not None and not self.t.is_closing():
            self._resume()
            if self.buf:
                self._next()                 # a pipelined request already arrived
            else:
                self._arm_idle()

    def _write(self, resp: Response, close: bool) -> None:
        if self.t is None or self.t.is_closing():
            return
        head = [b"HTTP/1.1 %d %s\r\n" % (resp.status, _REASONS.get(resp.status, "").encode())]
        if resp.content_type:
            head += [b"Content-Type: ", resp.content_type.encode(), b"\r\n"]
        head += [b"Content-Length: %d\r\n" % len(resp.body), b"Date: ", _date(), b"\r\n"]
        for k, v in resp.headers.items():
            head += [k.encode(), b": ", v.encode(), b"\r\n"]
        if close:
            head.append(b"Connection: close\r\n")
        head.append(b"\r\n")
        self.t.write(b"".join(head) + resp.body)
        if close:
            self.t.close()


class HttpServer:
    def __init__(self, router: Router, max_conns: int = MAX_CONNS) -> None:
        self.router = router
        self.max_conns = max_conns
        self.refused = 0                 # connections answered 503 (max_conns reached)
        self.conns: set = set()
        self.server: Optional[asyncio.AbstractServer] = None
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.port = 0
        self.tls = False

    async def start(self, host: str, port: int, ssl=None) -> int:
        """Listen on ``host:port`` (``ssl``: an ``ssl.SSLContext`` for HTTPS)."""
        self.loop = asyncio.get_running_loop()
        self.tls = ssl is not None
        self.server = await self.loop.create_server(lambda: _Conn(self), host, port,
                                                    reuse_address=True, ssl=ssl)
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
