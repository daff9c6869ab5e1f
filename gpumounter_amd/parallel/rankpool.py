"""A pool of collective ranks for a single-process caller: ``bench.py --gpus N`` without a launcher.

The driver may run ``bench.py --gpus 8`` as one process. That process can probe every attached GPU
itself (the liveness kernel, ``hipMemcpyPeer`` between every pair), but RCCL needs one process per
GPU. So the bench spawns N rank processes *before it touches the GPU* (a GPU-initialised process
must never exec; these are fresh children of a process that has only imported modules), each
speaking a line protocol on stdin/stdout:

* ``{"op": "allreduce", "bdfs": [...], "numel": K}`` → rank r binds to ``sorted(bdfs)[r]`` (the GPU
  it was attached; found by PCI address, so the mapping does not depend on HIP enumeration order),
  creates the ``nccl`` (RCCL over xGMI) process group on first use, all-reduces K bf16 elements
  holding ``r+1`` and checks the sum; replies ``{"ok", "ms", "bdf", "device", "backend"}``;
* ``{"op": "quit"}`` → destroys the group and exits 0.

Without a GPU the ranks use ``gloo`` on the CPU (hermetic tests). The reference has no
collective or post-attach validation at all.
"""
from __future__ import annotations

import argparse
import json
import os
import select
import subprocess
import sys
import tempfile
import time
from typing import Dict, List, Optional


_TAG = "@@gm-rank "


class RankPool:
    def __init__(self, world: int, timeout_s: float = 180.0) -> None:
        self.world = world
        self.timeout_s = timeout_s
        # file:// rendezvous: no TCP port to pick ahead of time (one picked with bind(0) and
        # bound later by rank 0 can be taken meanwhile, e.g. as a connection's local port)
        self._rdv_dir = tempfile.mkdtemp(prefix="gm-rankpool-")
        env = {**os.environ, "GM_RANKPOOL_RDV": "file://" + os.path.join(self._rdv_dir, "store"),
               "WORLD_SIZE": str(world)}
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"]
                                    if env.get("PYTHONPATH") else "")
        self.procs: List[subprocess.Popen] = []
        for r in range(world):
            self.procs.append(subprocess.Popen(
                [sys.executable, "-u", "-m", "gpumounter_amd.parallel.rankpool", "--rank", str(r),
                 "--world", str(world)],
                stdin=subprocess.PIPE, stdout=subprocess.PIPE, env={**env, "RANK": str(r)},
                text=True, bufsize=1))

    def _ask(self, msg: Dict) -> List[Dict]:
        line = json.dumps(msg) + "\n"
        for p in self.procs:
            p.stdin.write(line)
            p.stdin.flush()
        out: List[Optional[Dict]] = [None] * self.world
        deadline = time.monotonic() + self.timeout_s
        fds = {p.stdout.fileno(): i for i, p in enumerate(self.procs)}
        while any(o is None for o in out):
            left = deadline - time.monotonic()
            if left <= 0:
                raise TimeoutError(f"rank pool: no reply from ranks "
                                   f"{[i for i, o in enumerate(out) if o is None]}")
            ready, _, _ = select.select([p.stdout for i, p in enumerate(self.procs)
                                         if out[i] is None], [], [], min(left, 5.0))
            for f in ready:
                i = fds[f.fileno()]
                reply = f.readline()
                if not reply:
                    raise RuntimeError(f"rank pool: rank {i} exited "
                                       f"(code {self.procs[i].poll()})")
                if reply.startswith(_TAG):
                    out[i] = json.loads(reply[len(_TAG):])
                    if out[i].get("error"):
                        raise RuntimeError(f"rank pool: rank {i}: {out[i]['error']}")
        return out  # type: ignore[return-value]

    def allreduce(self, bdfs: List[str], numel: int = 1 << 20) -> Dict:
        """One checked all-reduce over the attached set; time = slowest rank."""
        res = self._ask({"op": "allreduce", "bdfs": list(bdfs), "numel": numel})
        return {"ok": all(r["ok"] for r in res), "ms": max(r["ms"] for r in res),
                "backend": res[0]["backend"], "bdfs": [r.get("bdf") for r in res],
                "bytes": numel * 2}

    def close(self) -> Dict[int, Optional[int]]:
        codes: Dict[int, Optional[int]] = {}
        for p in self.procs:
            try:
                p.stdin.write(json.dumps({"op": "quit"}) + "\n")
                p.stdin.flush()
            except (BrokenPipeError, OSError):
                pass
        for i, p in enumerate(self.procs):
            try:
                codes[i] = p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                codes[i] = p.wait()
        import shutil
        shutil.rmtree(self._rdv_dir, ignore_errors=True)
        return codes


# ------------------------------------------------------------------------------ rank process
def _rank_main(rank: int, world: int) -> int:
    # replies go over a private copy of the stdout pipe; fd 1 itself is pointed at stderr so
    # whatever the libraries print cannot corrupt the protocol
    reply_fd = os.dup(1)
    os.dup2(2, 1)
    chan = os.fdopen(reply_fd, "w", buffering=1)

    import torch
    import torch.distributed as dist

    rdv = os.environ.get("GM_RANKPOOL_RDV") or "env://"
    # GM_RANKPOOL_CPU=1: gloo on the CPU even where a GPU is visible (the hermetic test on a
    # GPU box, where an empty CUDA_VISIBLE_DEVICES does not hide the ROCm devices)
    on_gpu = os.environ.get("GM_RANKPOOL_CPU") != "1" and torch.cuda.is_available()
    backend = "nccl" if on_gpu else "gloo"
    dev = None
    bound = ""
    for line in sys.stdin:
        msg = json.loads(line)
        if msg["op"] == "quit":
            break
        bdfs = sorted(msg["bdfs"])
        mine = bdfs[rank % len(bdfs)] if bdfs else ""
        reply = {"rank": rank, "backend": backend, "bdf": mine, "ok": False, "ms": 0.0}
        try:
            if dev is None:
                if on_gpu:
                    from gpumounter_amd.ops import probe
                    d = probe.find_device(mine)
                    if d < 0:
                        raise RuntimeError(f"attached GPU {mine} not visible to HIP")
                    torch.cuda.set_device(d)
                    dev = torch.device("cuda", d)
                    dist.init_process_group("nccl", init_method=rdv, rank=rank,
                                            world_size=world, device_id=dev)
                else:
                    dev = torch.device("cpu")
                    dist.init_process_group("gloo", init_method=rdv, rank=rank,
                                            world_size=world)
                bound = mine
            elif mine != bound:
                raise RuntimeError(f"attached set changed between steps ({bound} → {mine})")
            dtype = torch.bfloat16 if on_gpu else torch.float32
            x = torch.full((int(msg["numel"]),), float(rank + 1), dtype=dtype, device=dev)
            if on_gpu:
                torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            dist.all_reduce(x)
            if on_gpu:
                torch.cuda.synchronize(dev)
            reply["ms"] = (time.perf_counter() - t0) * 1e3
            expect = world * (world + 1) / 2
            reply["ok"] = bool(torch.all(x == expect).item())
            reply["device"] = dev.index if dev.index is not None else -1
        except Exception as e:  # noqa: BLE001 - reported to the parent, which fails the run
            reply["error"] = f"{type(e).__name__}: {e}"
        chan.write(_TAG + json.dumps(reply) + "\n")
        chan.flush()
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="gpumounter_amd.parallel.rankpool")
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    a = ap.parse_args(argv)
    return _rank_main(a.rank, a.world)


if __name__ == "__main__":
    sys.exit(main())
