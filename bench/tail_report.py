"""Where the slowest attaches spent their time.

Reads ``bench.py --dump-samples`` files. Every sample holds the client's attach time, the
master's stage split (``gm:master_*``: authz, locate, the gRPC call, the reply payload) and the
worker's (its attach stages plus ``rpc_queue``/``rpc_tail``, the handler around the operation).
Each attach is cut into components that add up to the client's time:

* ``client_http``  — client ⇄ master HTTP (what the master's handler does not see);
* ``master_own``   — the master's handler outside the gRPC call (authz, lookup, reply);
* ``grpc``         — the gRPC call minus the worker's handler (transport, TLS, both loops);
  with a same-host clock also split into ``grpc:request`` and ``grpc:response`` (not added);
* ``worker_rpc``   — the worker's handler around the operation (peer check, task start, reply
  hand-off);
* ``worker:<stage>`` — the worker's attach stages (ledger_reserve, placeholder_wait, mount, ...),
  and ``worker:other`` for its time outside them.

Per file: percentiles, the 10 slowest cycles with their largest component, and for the slowest
1 % of the cycles how much each component exceeds its own median there (the tail's attribution).
"""
import json
import statistics
import sys


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))] if xs else None


def top_level(stages):
    return {k: v for k, v in stages.items() if "." not in k}


def components(r):
    st = top_level(r.get("stages") or {})
    ms = top_level(r.get("master") or {})
    worker_ops = {k: v for k, v in st.items() if not k.startswith("rpc_")}
    handler = sum(v for k, v in st.items() if k.startswith("rpc_"))
    out = {f"worker:{k}": v for k, v in worker_ops.items()}
    worker = r.get("worker_ms")
    if worker is not None:
        # the worker's attach outside its named stages (locks, policy, replies, metrics)
        out["worker:other"] = worker - sum(worker_ops.values())
    else:
        worker = sum(worker_ops.values())
    if ms:
        master = sum(ms.values())
        rpc = ms.get("master_rpc", 0.0)
        out["client_http"] = r["attach_ms"] - master
        out["master_own"] = master - rpc
        out["grpc"] = rpc - worker - handler
        out["worker_rpc"] = handler
        legs = r.get("master") or {}
        if "master_rpc.grpc_request" in legs:    # same-host clock: the two legs of the hop
            out["grpc:request"] = legs["master_rpc.grpc_request"]
            out["grpc:response"] = legs["master_rpc.grpc_response"]
    else:                       # samples from before the master stages were recorded
        out["outside_worker"] = r["attach_ms"] - sum(worker_ops.values())
    return out


def report(path):
    rows = [json.loads(line) for line in open(path) if line.strip()]
    att = [r["attach_ms"] for r in rows]
    comps = [components(r) for r in rows]
    keys = sorted({k for c in comps for k in c})
    med = {k: statistics.median([c.get(k, 0.0) for c in comps]) for k in keys}
    # the slowest 1 % of the cycles (at least one)
    by_time = sorted(zip(att, comps), key=lambda ac: -ac[0])
    tail = [c for _, c in by_time[:max(1, len(att) // 100)]]
    excess = {k: round(statistics.mean([c.get(k, 0.0) for c in tail]) - med[k], 3)
              for k in keys} if tail else {}
    slow = sorted(zip(rows, comps), key=lambda rc: -rc[0]["attach_ms"])[:10]
    t0 = rows[0]["t"] if rows else 0.0
    out = {"file": path, "cycles": len(rows),
           "attach_ms": {q: round(pct(att, p), 3) for q, p in
                         (("p50", .5), ("p90", .9), ("p99", .99), ("p999", .999),
                          ("max", 1.0))},
           "component_p50_ms": {k: round(v, 3) for k, v in med.items()},
           "tail_cycles": len(tail),
           # mean over the slowest 1 % of the cycles, minus the component's median
           "tail_excess_over_p50_ms": dict(sorted(excess.items(), key=lambda kv: -kv[1])),
           "slowest": []}
    for r, c in slow:
        big = max(c.items(), key=lambda kv: kv[1]) if c else ("", 0.0)
        out["slowest"].append({"at_s": round(r["t"] - t0, 2), "attach_ms": r["attach_ms"],
                               "largest": [big[0], round(big[1], 3)],
                               "over_median": {k: round(v - med.get(k, 0.0), 3)
                                               for k, v in c.items()
                                               if v - med.get(k, 0.0) > 0.1}})
    return out


if __name__ == "__main__":
    print(json.dumps([report(p) for p in sys.argv[1:]], indent=1))
