"""Prometheus metrics (the reference exports none — SURVEY §5.5).

All collectors live in a private registry so several workers/masters can coexist in one test
process without clashing on the global default registry.
"""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

_BUCKETS = (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30,
            60, 120)


class Metrics:
    def __init__(self) -> None:
        self.registry = CollectorRegistry(auto_describe=True)
        r = self.registry
        self.attach_latency = Histogram("gm_attach_latency_seconds", "GPU attach latency",
                                        ["n_gpus", "mode"], buckets=_BUCKETS, registry=r)
        self.detach_latency = Histogram("gm_detach_latency_seconds", "GPU detach latency",
                                        ["n_gpus"], buckets=_BUCKETS, registry=r)
        self.stage_latency = Histogram("gm_stage_latency_seconds", "per-stage latency",
                                       ["op", "stage"], buckets=_BUCKETS, registry=r)
        self.requests = Counter("gm_requests_total", "RPCs by result", ["op", "result"],
                                registry=r)
        self.ledger_gpus = Gauge("gm_ledger_gpus", "GPUs on this node by state", ["state"],
                                 registry=r)
        self.orphans = Counter("gm_orphans_total", "orphans found by the reconciler", ["kind"],
                               registry=r)
        self.reconcile_actions = Counter("gm_reconcile_actions_total", "reconciler repairs",
                                         ["action"], registry=r)
        self.placement_mismatch = Counter("gm_placement_mismatch_total",
                                          "device plugin chose a set other than the preferred one",
                                          registry=r)
        self.placement_corrections = Counter(
            "gm_placement_corrections_total",
            "attaches whose plugin-chosen GPUs were swapped for a better-placed set", registry=r)
        self.verify_failures = Counter("gm_attach_verify_failures_total",
                                       "attaches rolled back because the read-back "
                                       "(attach_verify) found rules or nodes missing",
                                       registry=r)
        self.admission_refusals = Counter(
            "gm_admission_refusals_total",
            "placeholders the kubelet refused at admission (UnexpectedAdmissionError / "
            "OutOf<resource>), by what followed: rebooked (a teardown was in flight), full (no "
            "room in gpumounter's view either: answered as too few GPUs), exhausted (the GPUs "
            "looked free throughout and the re-bookings ran out)", ["outcome"], registry=r)
        self.gpu_busy = Gauge("gm_gpu_processes", "processes on a GPU (amdsmi)", ["gpu"],
                              registry=r)
        self.plugin_rpcs = Counter("gm_device_plugin_rpcs_total",
                                   "device-plugin RPCs served (steered = intent consumed)",
                                   ["rpc"], registry=r)
        self.plugin_healthy = Gauge("gm_device_plugin_healthy_gpus",
                                    "GPUs advertised Healthy", registry=r)
        self.gpu_healthy = Gauge("gm_gpu_healthy", "1 = usable for placement (liveness + ECC "
                                 "policy), 0 = excluded", ["gpu"], registry=r)
        self.hot_gpus = Gauge("gm_hot_mounted_gpus", "GPUs hot-mounted into pods, by the pods' "
                              "namespace (sum over time = GPU-seconds for chargeback)",
                              ["namespace"], registry=r)
        self.draining = Gauge("gm_draining_placeholders", "force-removed GPUs held until their "
                              "killed processes exit (worker/drain.py)", registry=r)
        self.http_requests = Counter("gm_http_requests_total", "master HTTP requests",
                                     ["route", "code"], registry=r)

    def observe_trace(self, op: str, root) -> None:
        for stage, ms in root.flat().items():
            if "." in stage:
                continue
            self.stage_latency.labels(op=op, stage=stage).observe(ms / 1e3)

    def render(self) -> bytes:
        return generate_latest(self.registry)
