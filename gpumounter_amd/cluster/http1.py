"""A lean HTTP/1.1 client for the Kubernetes API: keep-alive connections, one request at a
time per connection, Content-Length / chunked / read-to-close bodies, and watch streams parsed
into events as the bytes arrive.

The worker's apiserver calls are on the attach path (the placeholder POST, the watch events
that carry its binding and admission) and the detach path (the DELETE). aiohttp's client spent
about a fifth of the worker's CPU per attach/detach cycle (`profiles/r5_hop/after/`): request
and response objects, header multidicts, a timer context and a stream reader per request. The
reference's client-go is a compiled client with a connection pool; this is the same shape for
an asyncio process.

* ``Pool.request`` sends one request and returns ``(status, headers, body)``. Connections are
  kept for ``keepalive_s`` when idle. A *replayable* request (GET/HEAD, or one the caller marks
  so) that finds its reused connection closed by the server before any byte of an answer (the
  idle-close race) is sent once more on a new one; any other request surfaces the error, since
  the server may have processed it (Go's transport draws the same line).
* ``Pool.stream`` opens a connection of its own for a watch and yields the decoded JSON lines;
  ``read_timeout_s`` without a byte ends it with ``asyncio.TimeoutError``. A line longer than
  ``MAX_LINE`` ends it with ``HttpError``; while ``MAX_QUEUED`` bytes of lines wait for the
  consumer the connection stops reading (TCP backpressure on the apiserver).
* The parser accepts ASCII digits only (status, Content-Length, chunk sizes) and bounds every
  line it waits for, so a malformed or hostile answer is an ``HttpError``, never an unbounded
  buffer or an exception of another type.
* Transport failures are ``ConnectionError``/``OSError`` (``HttpError`` for a malformed or cut
  answer), timeouts ``asyncio.TimeoutError``, as the callers expect from any client.
"""
from __future__ import annotations

import asyncio
import collections
import ssl
import time
import urllib.parse
from typing import Callable, Deque, Dict, Optional, Tuple

MAX_HEAD = 64 * 1024
# one response body: every LIST is paged (cluster/kube.py list_pages, 500 objects a page), so
# an answer this large is a broken or hostile server
MAX_BODY = 32 * 1024 * 1024
MAX_LINE = 16 * 1024 * 1024     # one watch event (etcd objects are at most ~1.5 MiB)
MAX_QUEUED = 8 * 1024 * 1024    # watch bytes parsed but not consumed before reading pauses
MAX_CHUNK_LINE = 1024           # a chunk-size or trailer line
_DIGITS = frozenset(b"0123456789")
_HEX = frozenset(b"0123456789abcdefABCDEF")


def _ascii_int(b: bytes, base: int = 10) -> int:
    """A non-negative integer of ASCII digits only (``int()`` also takes signs, spaces,
    underscores and non-ASCII digits such as "²")."""
    if not b or len(b) > 18 or not set(b) <= (_DIGITS if base == 10 else _HEX):
        raise HttpError(f"bad number {bytes(b[:20])!r}")
    return int(b, base)


class HttpError(ConnectionError):
    """A malformed answer, or the connection closed before the answer was complete."""


class _Conn(asyncio.Protocol):
    """One connection; parses one response at a time (``expect``), or a streamed body."""

    def __init__(self, loop: asyncio.AbstractEventLoop) -> None:
        self.loop = loop
        self.t: Optional[asyncio.Transport] = None
        self.buf = bytearray()
        self.closed = False
        self.got_bytes = False        # any byte of the current answer arrived
        self.fut: Optional[asyncio.Future] = None
        self.sink: Optional[Callable[[Optional[bytes], Optional[BaseException]], None]] = None
        self._state = "idle"           # idle | head | length | chunk_size | chunk | close
        self._status = 0
        self._headers: Dict[str, str] = {}
        self._left = 0
        self._body = bytearray()
        self._keep = True
        self._stream = False

    # ------------------------------------------------------------------ transport callbacks
    def connection_made(self, transport) -> None:
        self.t = transport

    def connection_lost(self, exc) -> None:
        self.closed = True
        self.t = None
        if self._state == "close":                       # read-to-close body ends here
            self._finish()
            return
        if self._state != "idle":
            self._fail(exc or HttpError("connection closed by the server"))

    def eof_received(self):
        return False                                     # close our side too

    def data_received(self, data: bytes) -> None:
        if self._state == "idle":                        # unsolicited: never reused
            self._keep = False
            if self.t is not None:
                self.t.close()
            return
        self.got_bytes = True
        self.buf += data
        try:
            self._parse()
        except HttpError as e:
            self._fail(e)
            if self.t is not None:
                self.t.close()

    # ------------------------------------------------------------------ one exchange
    def expect(self, stream: bool = False) -> asyncio.Future:
        self.fut = self.loop.create_future()
        self._state, self._stream = "head", stream
        self._body = bytearray()
        self.got_bytes = False
        return self.fut

    def _fail(self, exc: BaseException) -> None:
        self._state = "idle"
        self._keep = False
        if self.fut is not None and not self.fut.done():
            self.fut.set_exception(exc)
        if self.sink is not None:
            sink, self.sink = self.sink, None
            sink(None, exc)

    def _finish(self) -> None:
        self._state = "idle"
        if self.sink is not None:
            sink, self.sink = self.sink, None
            sink(None, None)
            return
        if self.fut is not None and not self.fut.done():
            self.fut.set_result((self._status, self._headers, bytes(self._body)))

    def _deliver(self, piece: bytes) -> None:
        if self.sink is not None:
            self.sink(piece, None)
        else:
            self._body += piece
            if len(self._body) > MAX_BODY:
                raise HttpError("response body too large")

    def _parse(self) -> None:
        buf = self.buf
        while True:
            st = self._state
            if st == "head":
                end = buf.find(b"\r\n\r\n")
                if end < 0:
                    if len(buf) > MAX_HEAD:
                        raise HttpError("response head too large")
                    return
                if end > MAX_HEAD:
                    raise HttpError("response head too large")
                lines = bytes(buf[:end]).decode("latin-1").split("\r\n")
                del buf[:end + 4]
                parts = lines[0].split(" ", 2)
                if len(parts) < 2 or not parts[0].startswith("HTTP/1.") or \
                        len(parts[1]) != 3 or not set(parts[1].encode()) <= _DIGITS:
                    raise HttpError(f"malformed status line {lines[0][:80]!r}")
                status = int(parts[1])
                headers: Dict[str, str] = {}
                for ln in lines[1:]:
                    k, sep, v = ln.partition(":")
                    if sep:
                        k = k.strip().lower()
                        if k == "content-length" and k in headers and \
                                headers[k] != v.strip():
                            raise HttpError("conflicting Content-Length headers")
                        headers[k] = v.strip()
                if 100 <= status < 200:
                    continue                             # 100 Continue and friends
                self._status, self._headers = status, headers
                self._keep = parts[0] == "HTTP/1.1" and \
                    headers.get("connection", "").lower() != "close"
                te = headers.get("transfer-encoding", "").lower()
                if status in (204, 304):
                    self._state = "done"
                elif te == "chunked":
                    self._state = "chunk_size"
                elif "content-length" in headers:
                    self._left = _ascii_int(headers["content-length"].encode("latin-1"))
                    if self._left > MAX_BODY and self.sink is None:
                        raise HttpError("response body too large")
                    self._state = "length" if self._left else "done"
                else:
                    self._state, self._keep = "close", False
                if self._stream and self.fut is not None and not self.fut.done():
                    # the caller decides (status) before the body streams to its sink
                    self.fut.set_result((status, headers, b""))
            elif st == "length":
                if not buf:
                    return
                piece = bytes(buf[:self._left])
                del buf[:len(piece)]
                self._left -= len(piece)
                self._deliver(piece)
                if self._left == 0:
                    self._state = "done"
            elif st == "chunk_size":
                eol = buf.find(b"\r\n", 0, MAX_CHUNK_LINE + 2)
                if eol < 0:
                    if len(buf) > MAX_CHUNK_LINE:
                        raise HttpError("chunk-size line too long")
                    return
                size_s = bytes(buf[:eol]).split(b";", 1)[0].strip(b" \t")
                del buf[:eol + 2]
                self._left = _ascii_int(size_s, 16)
                self._state = "chunk" if self._left else "trailer"
            elif st == "chunk":
                if len(buf) < self._left + 2:
                    if self._left and buf and self.sink is not None:
                        # stream what there is of a long chunk already
                        n = min(len(buf), self._left)
                        piece = bytes(buf[:n])
                        del buf[:n]
                        self._left -= n
                        self._deliver(piece)
                    return
                piece = bytes(buf[:self._left])
                del buf[:self._left + 2]
                self._deliver(piece)
                self._state = "chunk_size"
            elif st == "trailer":
                end = buf.find(b"\r\n", 0, MAX_CHUNK_LINE + 2)
                if end < 0:
                    if len(buf) > MAX_CHUNK_LINE:
                        raise HttpError("trailer line too long")
                    return
                line = bytes(buf[:end])
                del buf[:end + 2]
                if not line:
                    self._state = "done"
            elif st == "close":
                if buf:
                    piece = bytes(buf)
                    del buf[:]
                    self._deliver(piece)
                return
            elif st == "done":
                self._finish()
                return
            else:
                return


class Pool:
    """Keep-alive connections to one ``base_url`` (``http[s]://host[:port][/prefix]``)."""

    def __init__(self, base_url: str, ssl_ctx=None, headers: Optional[Dict[str, str]] = None,
                 keepalive_s: float = 60.0, timeout_s: float = 30.0) -> None:
        u = urllib.parse.urlsplit(base_url)
        self.https = u.scheme == "https"
        self.host = u.hostname or "localhost"
        self.port = u.port or (443 if self.https else 80)
        self.prefix = u.path.rstrip("/")
        self.ssl = (ssl_ctx if ssl_ctx is not None else ssl.create_default_context()) \
            if self.https else None
        if self.https and ssl_ctx is False:              # insecure-skip-tls-verify
            ctx = ssl.create_default_context()
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
            self.ssl = ctx
        hostport = self.host if u.port is None else f"{self.host}:{u.port}"
        self.headers = {"Host": hostport, "User-Agent": "gpumounter-amd", **(headers or {})}
        self.base_head = "".join(f"{k}: {v}\r\n" for k, v in self.headers.items())
        self.keepalive_s = keepalive_s
        self.timeout_s = timeout_s
        self._idle: Deque[Tuple[_Conn, float]] = collections.deque()
        self._busy: set = set()
        self._closed = False

    # ------------------------------------------------------------------ connections
    async def _connect(self, timeout: float) -> _Conn:
        """A new connection within ``timeout``. Not ``asyncio.wait_for``: on Python 3.10 it
        returns the result instead of raising when the caller is cancelled just as the connect
        completes, and a cancelled informer then watched on (found by the ledger model: a
        worker stop that waited for a watch without end)."""
        loop = asyncio.get_running_loop()
        task = loop.create_task(loop.create_connection(
            lambda: _Conn(loop), self.host, self.port, ssl=self.ssl,
            server_hostname=self.host if self.ssl is not None else None))
        expired = []

        def expire() -> None:
            expired.append(True)
            task.cancel()
        timer = loop.call_later(max(timeout, 0.0), expire)
        try:
            _, conn = await task
        except asyncio.CancelledError:
            if expired:
                raise asyncio.TimeoutError(f"connect to {self.host}:{self.port}: no answer "
                                           f"within {timeout:g}s") from None
            raise
        finally:
            timer.cancel()
        self._busy.add(conn)               # close() reaches it from here on
        return conn

    def _take_idle(self) -> Optional[_Conn]:
        now = time.monotonic()
        while self._idle:
            conn, since = self._idle.pop()
            if conn.closed or conn.t is None or conn.t.is_closing():
                continue
            if now - since > self.keepalive_s:
                conn.t.close()
                continue
            return conn
        return None

    def _release(self, conn: _Conn) -> None:
        self._busy.discard(conn)
        if self._closed or conn.closed or not conn._keep or conn.t is None:  # noqa: SLF001
            if conn.t is not None:
                conn.t.close()
            return
        self._idle.append((conn, time.monotonic()))

    def _head(self, method: str, target: str, headers: Optional[Dict[str, str]],
              body: Optional[bytes]) -> bytes:
        head = self.base_head if not headers else "".join(
            f"{k}: {v}\r\n" for k, v in {**self.headers, **headers}.items())
        length = f"Content-Length: {len(body)}\r\n" if body is not None else \
            ("Content-Length: 0\r\n" if method in ("POST", "PUT", "PATCH") else "")
        return (f"{method} {self.prefix}{target} HTTP/1.1\r\n{head}{length}"
                "\r\n").encode("latin-1")

    @staticmethod
    def target(path: str, params: Optional[dict]) -> str:
        if not params:
            return path
        return f"{path}?{urllib.parse.urlencode(params)}"

    # ------------------------------------------------------------------ requests
    async def request(self, method: str, target: str, headers: Optional[Dict[str, str]] = None,
                      body: Optional[bytes] = None, timeout_s: Optional[float] = None,
                      replayable: Optional[bool] = None) -> Tuple[int, Dict[str, str], bytes]:
        """``replayable``: the request may be sent a second time when a reused connection
        turns out closed (default: GET and HEAD only)."""
        if replayable is None:
            replayable = method in ("GET", "HEAD")
        if self._closed:
            raise HttpError("client closed")
        msg = self._head(method, target, headers, body)
        if body:
            msg += body
        timeout = self.timeout_s if timeout_s is None else timeout_s
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout
        for attempt in (0, 1):
            conn = self._take_idle()
            reused = conn is not None
            if conn is None:
                conn = await self._connect(deadline - loop.time())
            self._busy.add(conn)
            fut = conn.expect()
            conn.t.write(msg)
            timer = loop.call_at(deadline, _expire, fut, conn, timeout)
            try:
                out = await fut
            except HttpError:
                if replayable and reused and attempt == 0 and not conn.got_bytes:
                    # the server closed the idle connection as we sent: a new one
                    self._busy.discard(conn)
                    continue
                raise
            finally:
                timer.cancel()
                if conn._state != "idle":                # noqa: SLF001 - cancelled mid-answer
                    conn._keep = False                   # noqa: SLF001
                self._release(conn)
            return out
        raise AssertionError("unreachable")

    async def stream(self, method: str, target: str, headers: Optional[Dict[str, str]] = None,
                     read_timeout_s: float = 330.0
                     ) -> Tuple[int, Dict[str, str], "_Lines"]:
        """A streamed response on a connection of its own: ``(status, headers, lines)``;
        iterate ``lines`` for the body's non-empty lines. Close it with ``lines.close()``."""
        conn = await self._connect(self.timeout_s)
        lines = _Lines(conn, read_timeout_s)
        conn.sink = lines.feed
        fut = conn.expect(stream=True)
        conn.t.write(self._head(method, target, headers, None))
        loop = asyncio.get_running_loop()
        timer = loop.call_later(self.timeout_s, _expire, fut, conn, self.timeout_s)
        try:
            status, hdrs, _ = await fut
        except BaseException:
            lines.close()
            raise
        finally:
            timer.cancel()
        lines.on_close = lambda: self._busy.discard(conn)
        return status, hdrs, lines

    async def close(self) -> None:
        self._closed = True
        while self._idle:
            conn, _ = self._idle.pop()
            if conn.t is not None:
                conn.t.close()
        for conn in list(self._busy):
            if conn.t is not None:
                conn.t.close()
        self._busy.clear()


def _expire(fut: asyncio.Future, conn: _Conn, timeout: float) -> None:
    if not fut.done():
        fut.set_exception(asyncio.TimeoutError(f"no answer within {timeout:g}s"))
    conn._keep = False                                   # noqa: SLF001 - answer would be stale
    if conn.t is not None:
        conn.t.close()


class _Lines:
    """The lines of a streamed body, split as the bytes arrive."""

    def __init__(self, conn: _Conn, read_timeout_s: float) -> None:
        self.conn = conn
        self.read_timeout_s = read_timeout_s
        self.lines: Deque[bytes] = collections.deque()
        self.partial = bytearray()
        self.queued = 0               # bytes in ``lines``
        self.paused = False
        self.done = False
        self.error: Optional[BaseException] = None
        self.waiter: Optional[asyncio.Future] = None
        self.on_close: Optional[Callable[[], None]] = None
        self._timer: Optional[asyncio.TimerHandle] = None

    def feed(self, piece: Optional[bytes], exc: Optional[BaseException]) -> None:
        if piece is None:
            self.done, self.error = True, exc
            if bytes(self.partial).strip():
                self._push(bytes(self.partial))
            self.partial = bytearray()
        else:
            # only the new piece is scanned for line ends: a long line arriving in small pieces
            # costs linear time, not quadratic
            start = 0
            while True:
                nl = piece.find(b"\n", start)
                if nl < 0:
                    self.partial += piece[start:]
                    break
                if self.partial:
                    self.partial += piece[start:nl]
                    line, self.partial = bytes(self.partial), bytearray()
                else:
                    line = piece[start:nl]
                if line.strip():
                    self._push(line)
                start = nl + 1
            if len(self.partial) > MAX_LINE:
                raise HttpError(f"watch line longer than {MAX_LINE} bytes")
            if self.queued > MAX_QUEUED and not self.paused and self.conn.t is not None:
                self.paused = True
                self.conn.t.pause_reading()
        w = self.waiter
        if w is not None and not w.done() and (self.lines or self.done):
            w.set_result(None)

    def _push(self, line: bytes) -> None:
        self.lines.append(line)
        self.queued += len(line)

    def _stall(self) -> None:
        self.error = asyncio.TimeoutError(f"no data for {self.read_timeout_s:g}s")
        self.done = True
        if self.waiter is not None and not self.waiter.done():
            self.waiter.set_result(None)
        self.close()

    def __aiter__(self) -> "_Lines":
        return self

    async def __anext__(self) -> bytes:
        while not self.lines:
            if self.done:
                self.close()
                if self.error is not None:
                    raise self.error
                raise StopAsyncIteration
            loop = asyncio.get_running_loop()
            self.waiter = loop.create_future()
            self._timer = loop.call_later(self.read_timeout_s, self._stall)
            try:
                await self.waiter
            finally:
                self._timer.cancel()
                self.waiter = None
        line = self.lines.popleft()
        self.queued -= len(line)
        if self.paused and self.queued <= MAX_QUEUED // 2 and self.conn.t is not None:
            self.paused = False
            self.conn.t.resume_reading()
        return line

    def close(self) -> None:
        t = self.conn.t
        if t is not None:
            t.close()
        if self.on_close is not None:
            cb, self.on_close = self.on_close, None
            cb()

