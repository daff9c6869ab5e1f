"""gm-wire: the master → worker fast path for the ``gpu_mount`` RPCs.

The worker serves the reference's gRPC API (reference: pkg/api/gpu-mount/api.proto, called by
cmd/GPUMounter-master/main.go:82-96 over a fresh insecure connection per request) unchanged, so a
reference master, ``grpcurl`` or any gRPC client keeps working. Between gpumounter's own master
and worker the same protobuf messages can instead travel over gm-wire: one persistent (m)TLS TCP
connection per worker, length-prefixed frames, many calls in flight on it at once.

Why a second transport: in Python, grpc.aio hands every completion from grpc's C-core poller
thread to the event loop through a socket pair and wraps each call in several layers of call,
metadata and deadline objects. A unary call between two processes costs ≈0.15 ms on an idle
MI355X host before either handler runs (``box.grpc_rtt_us`` in the bench JSON); the same
request/response over an asyncio protocol with the same mTLS costs a third of that
(``profiles/r5_hop/``). The attach path makes exactly one such call.

Frame (big-endian): ``u32 length`` (of everything after it), ``u32 stream``, ``u8 kind``,
``u8 code``, then the body.

* ``kind 0`` request: ``code`` = method (1 AddGPU, 2 RemoveGPU, 3 GetNodeStatus), body = the
  serialized request message;
* ``kind 1`` response: body = the serialized response message;
* ``kind 2`` error: ``code`` = the gRPC status code number, body = UTF-8 details.

Streams are chosen by the client (odd, increasing) and answered in any order. Frames are at
most 4 MiB. A connection that sends anything else is closed. Security is the gRPC port's:
the worker requires a client certificate from ``tls_ca`` naming one of ``tls_client_names``
(checked once per connection), the master verifies the worker's ``tls_server_name``.
"""
from __future__ import annotations

import asyncio
import ssl
import struct
from typing import Any, Awaitable, Callable, Dict, Iterable, Optional, Set, Tuple

import grpc

from gpumounter_amd.utils import log

_log = log.get("wire")
HDR = struct.Struct(">IIBB")          # length, stream, kind, code
MAX_FRAME = 4 << 20
KIND_REQ, KIND_RESP, KIND_ERR = 0, 1, 2
METHOD_ADD, METHOD_REMOVE, METHOD_STATUS = 1, 2, 3
METHOD_PING = 0        # answered by the server itself with an empty response (warm-up)
_CODES = {c.value[0]: c for c in grpc.StatusCode}


class WireError(Exception):
    """A failed call, shaped like ``grpc.aio.AioRpcError`` (``code()``, ``details()``) so the
    master maps both transports' failures the same way."""

    def __init__(self, code: grpc.StatusCode, details: str, sent: bool = True) -> None:
        super().__init__(f"{code.name}: {details}")
        self._code = code
        self._details = details
        self.sent = sent          # False: the request never left (no connection)

    def code(self) -> grpc.StatusCode:
        return self._code

    def details(self) -> str:
        return self._details


def _frame(stream: int, kind: int, code: int, body: bytes) -> bytes:
    return HDR.pack(len(body) + 6, stream, kind, code) + body


def peer_names(cert: Optional[dict]) -> Set[str]:
    """DNS SANs and CN of a peer certificate as ``ssl`` decodes it."""
    if not cert:
        return set()
    out = {v for k, v in cert.get("subjectAltName", ()) if k == "DNS"}
    for rdn in cert.get("subject", ()):
        for k, v in rdn:
            if k == "commonName":
                out.add(v)
    return out


def server_context(cert: str, key: str, ca: str) -> ssl.SSLContext:
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH, cafile=ca or None)
    ctx.load_cert_chain(cert, key)
    if ca:
        ctx.verify_mode = ssl.CERT_REQUIRED
    return ctx


def client_context(ca: str, cert: str = "", key: str = "") -> ssl.SSLContext:
    ctx = ssl.create_default_context(cafile=ca or None)
    if cert and key:
        ctx.load_cert_chain(cert, key)
    return ctx


class _Framer:
    """Reassembles frames from a byte stream; ``None`` from :meth:`feed` = protocol error."""

    def __init__(self) -> None:
        self.buf = bytearray()

    def feed(self, data: bytes):
        buf = self.buf
        buf += data
        out = []
        while len(buf) >= 4:
            n = int.from_bytes(buf[:4], "big")
            if n < 6 or n > MAX_FRAME:
                return None
            if len(buf) < 4 + n:
                break
            _, stream, kind, code = HDR.unpack_from(buf, 0)
            out.append((stream, kind, code, bytes(buf[10:4 + n])))
            del buf[:4 + n]
        return out


# ---------------------------------------------------------------------------------- server
Handler = Tuple[Callable[[bytes], Any], Callable[[Any], Awaitable[Any]]]


class WireStatus(Exception):
    """Raised by a handler: answer with this status instead of a response."""

    def __init__(self, code: grpc.StatusCode, details: str) -> None:
        super().__init__(details)
        self.code = code
        self.details = details


class _ServerConn(asyncio.Protocol):
    MAX_STREAMS = 256

    def __init__(self, srv: "WireServer") -> None:
        self.srv = srv
        self.t: Optional[asyncio.Transport] = None
        self.framer = _Framer()
        self.tasks: Set[asyncio.Task] = set()

    def connection_made(self, transport) -> None:
        self.t = transport
        names = peer_names(transport.get_extra_info("peercert"))
        if self.srv.allowed and not names & self.srv.allowed:
            # a certificate of the CA, but not a master's
            _log.warning("gm-wire: refused %s (certificate names %s)",
                         transport.get_extra_info("peername"), sorted(names))
            transport.close()
            self.t = None
            return
        self.srv.conns.add(self)

    def connection_lost(self, exc) -> None:
        self.t = None
        self.srv.conns.discard(self)
        # operations already running finish (the worker shields them); their answers go nowhere

    def data_received(self, data: bytes) -> None:
        if self.t is None:
            return
        frames = self.framer.feed(data)
        if frames is None:
            self.t.close()
            return
        loop = self.srv.loop
        for stream, kind, code, body in frames:
            if kind != KIND_REQ or len(self.tasks) >= self.MAX_STREAMS:
                self.t.close()
                return
            task = loop.create_task(self._serve(stream, code, body))
            self.tasks.add(task)
            task.add_done_callback(self.tasks.discard)

    async def _serve(self, stream: int, method: int, body: bytes) -> None:
        h = self.srv.handlers.get(method)
        if h is None and method == METHOD_PING:
            if self.t is not None:
                self.t.write(_frame(stream, KIND_RESP, 0, b""))
            return
        try:
            if h is None:
                raise WireStatus(grpc.StatusCode.UNIMPLEMENTED, f"method {method}")
            try:
                req = h[0](body)
            except Exception as e:  # noqa: BLE001 - a malformed message
                raise WireStatus(grpc.StatusCode.INTERNAL, f"bad request: {e}") from e
            out = _frame(stream, KIND_RESP, 0, (await h[1](req)).SerializeToString())
        except WireStatus as e:
            out = _frame(stream, KIND_ERR, e.code.value[0], e.details.encode()[:MAX_FRAME - 16])
        except Exception as e:  # noqa: BLE001 - the caller gets an answer, never a hang
            out = _frame(stream, KIND_ERR, grpc.StatusCode.INTERNAL.value[0],
                         f"{type(e).__name__}: {e}".encode()[:MAX_FRAME - 16])
        if self.t is not None:
            self.t.write(out)


class WireServer:
    """``handlers``: method id → (request parser, ``async (request) → response``); a handler
    raises :class:`WireStatus` to answer with an error status."""

    def __init__(self, handlers: Dict[int, Handler], ssl_ctx: Optional[ssl.SSLContext] = None,
                 allowed_names: Iterable[str] = ()) -> None:
        self.handlers = handlers
        self.ssl = ssl_ctx
        self.allowed = {n for n in allowed_names if n} if ssl_ctx is not None else set()
        self.server: Optional[asyncio.AbstractServer] = None
        self.conns: Set[_ServerConn] = set()
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.port = 0

    async def start(self, host: str, port: int) -> int:
        self.loop = asyncio.get_running_loop()
        self.server = await self.loop.create_server(lambda: _ServerConn(self), host, port,
                                                    ssl=self.ssl, reuse_address=True)
        self.port = self.server.sockets[0].getsockname()[1]
        return self.port

    async def stop(self) -> None:
        if self.server is None:
            return
        self.server.close()
        for c in list(self.conns):
            if c.t is not None:
                c.t.close()
        await self.server.wait_closed()
        self.server = None


# ---------------------------------------------------------------------------------- client
class _ClientConn(asyncio.Protocol):
    def __init__(self, ch: "WireChannel") -> None:
        self.ch = ch
        self.t: Optional[asyncio.Transport] = None
        self.framer = _Framer()
        self.pending: Dict[int, asyncio.Future] = {}

    def connection_made(self, transport) -> None:
        self.t = transport

    def connection_lost(self, exc) -> None:
        self.t = None
        if self.ch._conn is self:  # noqa: SLF001
            self.ch._conn = None   # noqa: SLF001
        err = WireError(grpc.StatusCode.UNAVAILABLE,
                        f"connection to {self.ch.target} lost: {exc or 'closed'}")
        for f in self.pending.values():
            if not f.done():
                f.set_exception(err)
        self.pending.clear()

    def data_received(self, data: bytes) -> None:
        frames = self.framer.feed(data)
        if frames is None:
            if self.t is not None:
                self.t.close()
            return
        for stream, kind, code, body in frames:
            f = self.pending.pop(stream, None)
            if f is None or f.done():
                continue                  # its caller gave up (deadline)
            if kind == KIND_RESP:
                f.set_result(body)
            else:
                f.set_exception(WireError(_CODES.get(code, grpc.StatusCode.UNKNOWN),
                                          body.decode(errors="replace")))


class WireChannel:
    """One persistent connection to a worker's gm-wire port, (re)opened on demand."""

    CONNECT_TIMEOUT_S = 5.0

    def __init__(self, host: str, port: int, ssl_ctx: Optional[ssl.SSLContext] = None,
                 server_hostname: str = "") -> None:
        self.host, self.port = host, port
        self.target = f"{host}:{port}"
        self.ssl = ssl_ctx
        self.server_hostname = server_hostname or None
        self._conn: Optional[_ClientConn] = None
        self._connecting: Optional[asyncio.Future] = None
        self._stream = 1
        self._closed = False

    async def _connected(self) -> _ClientConn:
        c = self._conn
        if c is not None and c.t is not None:
            return c
        if self._closed:
            raise WireError(grpc.StatusCode.UNAVAILABLE, "channel closed", sent=False)
        if self._connecting is None or self._connecting.done():
            self._connecting = asyncio.ensure_future(self._open())
        return await asyncio.shield(self._connecting)

    async def _open(self) -> _ClientConn:
        loop = asyncio.get_running_loop()
        try:
            _, proto = await asyncio.wait_for(loop.create_connection(
                lambda: _ClientConn(self), self.host, self.port, ssl=self.ssl,
                server_hostname=self.server_hostname if self.ssl is not None else None),
                self.CONNECT_TIMEOUT_S)
        except (OSError, asyncio.TimeoutError, ssl.SSLError) as e:
            raise WireError(grpc.StatusCode.UNAVAILABLE,
                            f"connect to {self.target}: {e!r}", sent=False) from e
        if proto.t is not None:
            self._conn = proto
        return proto

    def warm(self) -> None:
        """Open the connection in the background (TCP and TLS handshakes off the request) and
        send one ping over it, so the first request's frame path is not a cold one on either
        side."""
        if (self._conn is None or self._conn.t is None) and \
                (self._connecting is None or self._connecting.done()) and not self._closed:
            self._connecting = asyncio.ensure_future(self._open())
            # an unreachable worker is reported by the call that needs it
            self._connecting.add_done_callback(self._opened)

    def _opened(self, f: asyncio.Future) -> None:
        if f.cancelled() or f.exception() is not None or self._closed:
            return
        ping = asyncio.ensure_future(self.call(METHOD_PING, b"", self.CONNECT_TIMEOUT_S))
        ping.add_done_callback(lambda p: p.cancelled() or p.exception())

    async def call(self, method: int, payload: bytes, timeout: float) -> bytes:
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout
        conn = await self._connected()
        if conn.t is None:               # closed between the handshake and now
            raise WireError(grpc.StatusCode.UNAVAILABLE,
                            f"connection to {self.target} closed by the peer", sent=False)
        stream = self._stream
        self._stream += 2
        fut = loop.create_future()
        conn.pending[stream] = fut
        conn.t.write(_frame(stream, KIND_REQ, method, payload))
        # a timer handle, not asyncio.wait_for (which wraps the future in two more)
        expiry = loop.call_at(deadline, self._expire, fut, timeout)
        try:
            return await fut
        finally:
            expiry.cancel()
            conn.pending.pop(stream, None)

    def _expire(self, fut: asyncio.Future, timeout: float) -> None:
        if not fut.done():
            fut.set_exception(WireError(grpc.StatusCode.DEADLINE_EXCEEDED,
                                        f"no answer from {self.target} within {timeout:g}s"))

    async def close(self) -> None:
        self._closed = True
        if self._connecting is not None and not self._connecting.done():
            self._connecting.cancel()
        c = self._conn
        self._conn = None
        if c is not None and c.t is not None:
            c.t.close()
