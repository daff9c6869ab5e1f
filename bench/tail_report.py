"""Where the slowest attaches spent their time: reads ``bench.py --dump-samples`` files and, per
file, prints the percentiles, the 10 slowest cycles with their worker stage split, and how much of
each slow cycle the worker accounts for (the rest is the client → master → worker hops)."""
import json
import sys


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))] if xs else None


def top_level(stages):
    return {k: v for k, v in stages.items() if "." not in k}


def report(path):
    rows = [json.loads(line) for line in open(path) if line.strip()]
    att = [r["attach_ms"] for r in rows]
    worker = [sum(top_level(r["stages"]).values()) for r in rows]
    slow = sorted(rows, key=lambda r: -r["attach_ms"])[:10]
    t0 = rows[0]["t"] if rows else 0.0
    out = {"file": path, "cycles": len(rows),
           "attach_ms": {q: round(pct(att, p), 3) for q, p in
                         (("p50", .5), ("p99", .99), ("p999", .999), ("max", 1.0))},
           "worker_ms": {q: round(pct(worker, p), 3) for q, p in
                         (("p50", .5), ("p99", .99), ("max", 1.0))},
           "slowest": []}
    for r in slow:
        st = top_level(r["stages"])
        w = sum(st.values())
        big = max(st.items(), key=lambda kv: kv[1]) if st else ("", 0.0)
        out["slowest"].append({"at_s": round(r["t"] - t0, 2), "attach_ms": r["attach_ms"],
                               "worker_ms": round(w, 3),
                               "outside_worker_ms": round(r["attach_ms"] - w, 3),
                               "largest_stage": [big[0], round(big[1], 3)]})
    return out


if __name__ == "__main__":
    print(json.dumps([report(p) for p in sys.argv[1:]], indent=1))
