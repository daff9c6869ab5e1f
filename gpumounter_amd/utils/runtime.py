"""Process-level latency tuning for the daemons.

After startup almost every Python object (modules, protobuf descriptors, gRPC/aiohttp machinery,
informer caches) lives for the whole process, yet a full (generation-2) collection walks all of
them: measured 30+ ms pauses on the attach path on a busy host. ``gc.freeze()`` moves what exists
after startup into the permanent generation, so later full collections only walk what requests
allocate. The young-generation threshold stays small: raising it (tried 50 000) trades many
sub-ms pauses for rare 25-40 ms ones, which is worse for the p99.
"""
from __future__ import annotations

import gc
import json
import os


def tune_gc(freeze: bool = True) -> None:
    if freeze:
        gc.collect()
        gc.freeze()


def write_ready_file(path: str, info: dict) -> None:
    """Atomically publish what a daemon bound (config ``ready_file``)."""
    if not path:
        return
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as fh:
        json.dump(info, fh)
    os.replace(tmp, path)
