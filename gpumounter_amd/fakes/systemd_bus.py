"""A fake systemd on a unix socket, speaking enough D-Bus for gpumounter's DeviceAllow= calls.

It answers ``org.freedesktop.DBus.Properties.Get(<unit iface>, "DeviceAllow")`` on unit object
paths and ``org.freedesktop.systemd1.Manager.SetUnitProperties(s, b, a(sv))`` with DeviceAllow
values, with systemd's semantics (entries append; an empty array resets the list). In ``bus``
mode it also wants the message bus ``Hello`` first and pushes a ``NameAcquired`` signal, as
dbus-daemon does. ``on_change(unit, entries)`` is called whenever a unit's list changes —
tests use it to "re-realise" the unit the way systemd would.

The wire codec here is independent of the C++ client (native/src/gm_sdbus.cpp) it tests.
"""
from __future__ import annotations

import os
import socket
import struct
import threading
from typing import Callable, Dict, List, Optional, Tuple

METHOD_CALL, METHOD_RETURN, ERROR, SIGNAL = 1, 2, 3, 4
F_PATH, F_IFACE, F_MEMBER, F_ERROR, F_REPLY, F_DEST, F_SENDER, F_SIG = 1, 2, 3, 4, 5, 6, 7, 8


# ------------------------------------------------------------------------------ codec
class _W:
    def __init__(self) -> None:
        self.b = bytearray()

    def align(self, n: int) -> None:
        self.b.extend(b"\0" * (-len(self.b) % n))

    def y(self, v: int) -> None:
        self.b.append(v)

    def u(self, v: int) -> None:
        self.align(4)
        self.b += struct.pack("<I", v)

    def s(self, v: str) -> None:
        raw = v.encode()
        self.u(len(raw))
        self.b += raw + b"\0"

    def g(self, v: str) -> None:
        self.y(len(v))
        self.b += v.encode() + b"\0"

    def array(self, elem_align: int, items, put) -> None:
        self.u(0)
        at = len(self.b) - 4
        self.align(elem_align)
        start = len(self.b)
        for it in items:
            put(it)
        struct.pack_into("<I", self.b, at, len(self.b) - start)


class _R:
    def __init__(self, b: bytes, p: int = 0) -> None:
        self.b, self.p = b, p

    def align(self, n: int) -> None:
        self.p += -self.p % n

    def y(self) -> int:
        v = self.b[self.p]
        self.p += 1
        return v

    def u(self) -> int:
        self.align(4)
        (v,) = struct.unpack_from("<I", self.b, self.p)
        self.p += 4
        return v

    def s(self) -> str:
        n = self.u()
        v = self.b[self.p:self.p + n].decode()
        self.p += n + 1
        return v

    def g(self) -> str:
        n = self.y()
        v = self.b[self.p:self.p + n].decode()
        self.p += n + 1
        return v


def encode(mtype: int, serial: int, fields: Dict[int, Tuple[str, object]], body: bytes) -> bytes:
    w = _W()
    w.b += b"l" + bytes([mtype, 0, 1])
    w.u(len(body))
    w.u(serial)

    def put(item):
        code, (sig, val) = item
        w.align(8)
        w.y(code)
        w.g(sig)
        if sig == "u":
            w.u(int(val))
        elif sig == "g":
            w.g(str(val))
        else:
            w.s(str(val))
    w.array(8, sorted(fields.items()), put)
    w.align(8)
    return bytes(w.b) + body


def decode_header(buf: bytes):
    """-> (type, serial, fields{code: value}, body_offset, total_length) or None if incomplete."""
    if len(buf) < 16:
        return None
    if buf[0:1] != b"l":
        raise ValueError("big-endian D-Bus messages are not supported by the fake")
    body_len, serial, flen = struct.unpack_from("<III", buf, 4)
    body_at = 16 + flen + (-(16 + flen) % 8)
    total = body_at + body_len
    if len(buf) < total:
        return None
    r = _R(buf, 16)
    fields = {}
    while r.p < 16 + flen:
        r.align(8)
        code = r.y()
        sig = r.g()
        fields[code] = r.u() if sig == "u" else (r.g() if sig == "g" else r.s())
    return buf[1], serial, fields, body_at, total


def unit_path(unit: str) -> str:
    out = []
    for i, ch in enumerate(unit.encode()):
        c = chr(ch)
        if c.isascii() and (c.isalpha() or (c.isdigit() and i > 0)):
            out.append(c)
        else:
            out.append(f"_{ch:02x}")
    return "/org/freedesktop/systemd1/unit/" + ("".join(out) or "_")


def unit_from_path(path: str) -> str:
    enc = path.rsplit("/", 1)[1]
    out, i = bytearray(), 0
    while i < len(enc):
        if enc[i] == "_" and i + 2 < len(enc) + 1 and len(enc[i + 1:i + 3]) == 2:
            out.append(int(enc[i + 1:i + 3], 16))
            i += 3
        else:
            out += enc[i].encode()
            i += 1
    return out.decode()


# ------------------------------------------------------------------------------ server
def _readline(conn: socket.socket, buf: bytes) -> Tuple[bytes, bytes]:
    while b"\r\n" not in buf:
        chunk = conn.recv(4096)
        if not chunk:
            raise OSError("peer closed during authentication")
        buf += chunk
    line, rest = buf.split(b"\r\n", 1)
    return line, rest


class FakeSystemd:
    # what runc asks systemd for on a container scope (its default device list)
    RUNTIME_DEFAULT = [("char-pts", "rwm"), ("/dev/null", "rwm"), ("/dev/zero", "rwm"),
                       ("/dev/full", "rwm"), ("/dev/random", "rwm"), ("/dev/urandom", "rwm"),
                       ("/dev/tty", "rwm"), ("/dev/net/tun", "rwm")]

    def __init__(self, path: str, mode: str = "private",
                 on_change: Optional[Callable[[str, List[Tuple[str, str]]], None]] = None,
                 auto_units: bool = False) -> None:
        assert mode in ("private", "bus")
        self.path = path
        self.mode = mode
        self.on_change = on_change
        self.auto_units = auto_units    # unknown *.scope units exist with RUNTIME_DEFAULT
        self.units: Dict[str, List[Tuple[str, str]]] = {}
        self.calls: List[Tuple[str, str]] = []          # (member, unit)
        self.fail_next: Optional[str] = None            # D-Bus error name for the next call
        self._lock = threading.Lock()
        self._sock: Optional[socket.socket] = None
        self._thread: Optional[threading.Thread] = None
        self._stop = False

    # -------------------------------------------------------------------- lifecycle
    def start(self) -> "FakeSystemd":
        if os.path.exists(self.path):
            os.unlink(self.path)
        self._sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self._sock.bind(self.path)
        self._sock.listen(16)
        self._sock.settimeout(0.2)
        self._thread = threading.Thread(target=self._accept, daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop = True
        if self._thread:
            self._thread.join(timeout=2)
        if self._sock:
            self._sock.close()
        if os.path.exists(self.path):
            os.unlink(self.path)

    def add_unit(self, unit: str, entries: List[Tuple[str, str]]) -> None:
        with self._lock:
            self.units[unit] = list(entries)

    # -------------------------------------------------------------------- protocol
    def _accept(self) -> None:
        while not self._stop:
            try:
                conn, _ = self._sock.accept()
            except socket.timeout:
                continue
            except OSError:
                return
            threading.Thread(target=self._serve, args=(conn,), daemon=True).start()

    def _serve(self, conn: socket.socket) -> None:
        conn.settimeout(5)
        try:
            line, buf = _readline(conn, b"")            # SASL: \0AUTH EXTERNAL <hex uid>
            parts = line.lstrip(b"\0").split()
            if parts[:2] != [b"AUTH", b"EXTERNAL"] or len(parts) != 3 or \
                    int(bytes.fromhex(parts[2].decode()).decode()) != os.getuid():
                conn.sendall(b"REJECTED EXTERNAL\r\n")
                return
            conn.sendall(b"OK 0123456789abcdef0123456789abcdef\r\n")
            line, buf = _readline(conn, buf)
            if line != b"BEGIN":
                return
            serial = 0
            hello_done = self.mode == "private"
            while True:
                hdr = decode_header(buf)
                while hdr is None:
                    chunk = conn.recv(65536)
                    if not chunk:
                        return
                    buf += chunk
                    hdr = decode_header(buf)
                mtype, mserial, fields, body_at, total = hdr
                body = buf[body_at:total]
                buf = buf[total:]
                if mtype != METHOD_CALL:
                    continue
                member = fields.get(F_MEMBER, "")
                if not hello_done:
                    if member != "Hello":
                        out = self._error(serial := serial + 1, mserial,
                                          "org.freedesktop.DBus.Error.AccessDenied",
                                          "Client tried to send a message other than Hello")
                        conn.sendall(out)
                        return
                    hello_done = True
                    w = _W()
                    w.s(":1.42")
                    conn.sendall(encode(METHOD_RETURN, serial := serial + 1,
                                        {F_REPLY: ("u", mserial), F_SIG: ("g", "s")},
                                        bytes(w.b)))
                    sig = _W()
                    sig.s(":1.42")
                    conn.sendall(encode(SIGNAL, serial := serial + 1,
                                        {F_PATH: ("o", "/org/freedesktop/DBus"),
                                         F_IFACE: ("s", "org.freedesktop.DBus"),
                                         F_MEMBER: ("s", "NameAcquired"), F_SIG: ("g", "s")},
                                        bytes(sig.b)))
                    continue
                serial += 1
                conn.sendall(self._dispatch(serial, mserial, fields, body))
        except (OSError, ValueError, struct.error):
            return
        finally:
            conn.close()

    def _error(self, serial: int, reply_to: int, name: str, text: str) -> bytes:
        w = _W()
        w.s(text)
        return encode(ERROR, serial, {F_REPLY: ("u", reply_to), F_ERROR: ("s", name),
                                      F_SIG: ("g", "s")}, bytes(w.b))

    def _dispatch(self, serial: int, reply_to: int, fields, body: bytes) -> bytes:
        member, iface, path = fields.get(F_MEMBER), fields.get(F_IFACE), fields.get(F_PATH)
        if self.mode == "bus" and fields.get(F_DEST) != "org.freedesktop.systemd1":
            return self._error(serial, reply_to, "org.freedesktop.DBus.Error.ServiceUnknown",
                               f"no destination {fields.get(F_DEST)!r}")
        if self.fail_next:
            name, self.fail_next = self.fail_next, None
            return self._error(serial, reply_to, name, "injected failure")
        r = _R(body)
        if iface == "org.freedesktop.DBus.Properties" and member == "Get":
            if fields.get(F_SIG) != "ss":
                return self._error(serial, reply_to, "org.freedesktop.DBus.Error.InvalidArgs",
                                   "bad signature")
            want_iface, prop = r.s(), r.s()
            unit = next((u for u in self.units if unit_path(u) == path), None)
            if unit is None and self.auto_units and path.endswith("_2escope"):
                unit = unit_from_path(path)
                self.add_unit(unit, self.RUNTIME_DEFAULT)
            self.calls.append(("Get", unit or path))
            if unit is None:
                return self._error(serial, reply_to, "org.freedesktop.systemd1.NoSuchUnit",
                                   f"unit for {path} not loaded")
            expect = "org.freedesktop.systemd1." + ("Scope" if unit.endswith(".scope")
                                                    else "Service")
            if want_iface != expect or prop != "DeviceAllow":
                return self._error(serial, reply_to, "org.freedesktop.DBus.Error.UnknownProperty",
                                   f"{want_iface}.{prop}")
            w = _W()
            w.g("a(ss)")
            with self._lock:
                entries = list(self.units[unit])

            def put(e):
                w.align(8)
                w.s(e[0])
                w.s(e[1])
            w.array(8, entries, put)
            return encode(METHOD_RETURN, serial, {F_REPLY: ("u", reply_to), F_SIG: ("g", "v")},
                          bytes(w.b))
        if iface == "org.freedesktop.systemd1.Manager" and member == "SetUnitProperties":
            if fields.get(F_SIG) != "sba(sv)" or path != "/org/freedesktop/systemd1":
                return self._error(serial, reply_to, "org.freedesktop.DBus.Error.InvalidArgs",
                                   "bad call")
            unit = r.s()
            runtime = r.u()
            self.calls.append(("SetUnitProperties", unit))
            if unit not in self.units and self.auto_units and unit.endswith(".scope"):
                self.add_unit(unit, self.RUNTIME_DEFAULT)
            if unit not in self.units:
                return self._error(serial, reply_to, "org.freedesktop.systemd1.NoSuchUnit",
                                   f"Unit {unit} not loaded.")
            if runtime != 1:
                return self._error(serial, reply_to, "org.freedesktop.DBus.Error.InvalidArgs",
                                   "gpumounter must only make runtime changes")
            n = r.u()
            r.align(8)
            end = r.p + n
            with self._lock:
                lst = list(self.units[unit])
                while r.p < end:
                    r.align(8)
                    name, sig = r.s(), r.g()
                    if name != "DeviceAllow" or sig != "a(ss)":
                        return self._error(serial, reply_to,
                                           "org.freedesktop.DBus.Error.PropertyReadOnly", name)
                    m = r.u()
                    r.align(8)
                    e_end = r.p + m
                    items = []
                    while r.p < e_end:
                        r.align(8)
                        items.append((r.s(), r.s()))
                    if not items:
                        lst = []                       # empty array = reset (systemd semantics)
                    for p, perm in items:              # same path: entry updated in place
                        lst = [(q, pm) for q, pm in lst if q != p] + [(p, perm)]
                changed = lst != self.units[unit]
                self.units[unit] = lst
            if changed and self.on_change:
                self.on_change(unit, list(lst))
            return encode(METHOD_RETURN, serial, {F_REPLY: ("u", reply_to)}, b"")
        return self._error(serial, reply_to, "org.freedesktop.DBus.Error.UnknownMethod",
                           f"{iface}.{member}")
