"""Structured logging with a per-request id.

The reference logs through a global zap SugaredLogger at Debug level, tee'd to stdout and a file
that is truncated at every start (reference: pkg/util/log/log.go:11-30, ``os.Create`` at 28). Here:
stdlib ``logging`` with a JSON formatter, a ``request_id`` carried in a ContextVar so every line of
one attach/detach (across awaits and threads spawned with ``contextvars.copy_context``) can be
correlated, and an append-mode rotating file.
"""
from __future__ import annotations

import contextvars
import json
import logging
import logging.handlers
import os
import sys
import time
import uuid
from typing import Optional

request_id: contextvars.ContextVar[str] = contextvars.ContextVar("gm_request_id", default="-")

_LOGGER_NAME = "gpumounter"


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        out = {
            "ts": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(record.created))
            + f".{int(record.msecs):03d}Z",
            "level": record.levelname,
            "logger": record.name,
            "rid": request_id.get(),
            "msg": record.getMessage(),
            "caller": f"{record.module}:{record.lineno}",
        }
        fields = getattr(record, "fields", None)
        if fields:
            out.update(fields)
        if record.exc_info:
            out["exc"] = self.formatException(record.exc_info)
        return json.dumps(out, default=str)


class TextFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        base = (f"{time.strftime('%H:%M:%S', time.localtime(record.created))}"
                f".{int(record.msecs):03d} {record.levelname[0]} [{request_id.get()}] "
                f"{record.name}: {record.getMessage()}")
        fields = getattr(record, "fields", None)
        if fields:
            base += " " + " ".join(f"{k}={v}" for k, v in fields.items())
        if record.exc_info:
            base += "\n" + self.formatException(record.exc_info)
        return base


def setup(level: str = "INFO", json_format: bool = True, log_file: str = "") -> logging.Logger:
    root = logging.getLogger(_LOGGER_NAME)
    root.setLevel(getattr(logging, level.upper(), logging.INFO))
    for h in list(root.handlers):
        root.removeHandler(h)
    fmt: logging.Formatter = JsonFormatter() if json_format else TextFormatter()
    sh = logging.StreamHandler(sys.stderr)
    sh.setFormatter(fmt)
    root.addHandler(sh)
    if log_file:
        os.makedirs(os.path.dirname(os.path.abspath(log_file)), exist_ok=True)
        # append + rotate instead of truncating on restart (reference log.go:28)
        fh = logging.handlers.RotatingFileHandler(log_file, maxBytes=64 << 20, backupCount=5)
        fh.setFormatter(fmt)
        root.addHandler(fh)
    root.propagate = False
    return root


def get(name: str) -> logging.Logger:
    return logging.getLogger(f"{_LOGGER_NAME}.{name}")


def new_request_id(prefix: str = "") -> str:
    rid = (prefix + "-" if prefix else "") + uuid.uuid4().hex[:12]
    request_id.set(rid)
    return rid


def kv(logger: logging.Logger, level: int, msg: str, **fields) -> None:
    """Log ``msg`` with structured key/values (rendered as JSON fields)."""
    if logger.isEnabledFor(level):
        logger.log(level, msg, extra={"fields": fields}, stacklevel=2)


def with_rid(rid: Optional[str]):
    """Context manager that sets the request id for the enclosed block."""
    class _Ctx:
        def __enter__(self):
            self._tok = request_id.set(rid or "-")
            return rid

        def __exit__(self, *exc):
            request_id.reset(self._tok)
            return False

    return _Ctx()
