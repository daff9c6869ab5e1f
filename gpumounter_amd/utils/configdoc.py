"""docs/CONFIG.md and docs/METRICS.md: every :class:`~gpumounter_amd.utils.config.Config` field with its environment
variable, default and the comment that documents it in ``config.py``.

The reference reads one setting from the environment (``CGROUP_DRIVER``, reference:
pkg/util/cgroup/cgroup.go:78-84) and hard-codes the rest; here every knob is a field, so the
table is generated from the source and a test keeps the checked-in copy in step
(``python -m gpumounter_amd config-doc > docs/CONFIG.md``). The reference exports no metrics;
:func:`render_metrics` lists ours from the registry itself (``config-doc --metrics``).
"""
from __future__ import annotations

import ast
import dataclasses
import inspect
import io
import tokenize
from typing import Dict, List, Tuple

from gpumounter_amd.utils import config as _config


def _comments() -> Tuple[Dict[str, str], Dict[str, str]]:
    """(field → its comment text, field → section) from config.py's source: the ``#`` block
    right above a field plus the comment at the end of its line."""
    src = inspect.getsource(_config)
    lines = src.splitlines()
    trailing: Dict[int, str] = {}
    for tok in tokenize.generate_tokens(io.StringIO(src).readline):
        if tok.type == tokenize.COMMENT:
            row, col = tok.start
            if lines[row - 1][:col].strip():
                trailing[row] = tok.string.lstrip("#").strip()
    cls = next(n for n in ast.parse(src).body
               if isinstance(n, ast.ClassDef) and n.name == "Config")
    docs: Dict[str, str] = {}
    sections: Dict[str, str] = {}
    section = ""
    prev_end = cls.lineno          # the `class Config:` line
    for node in cls.body:
        if not isinstance(node, ast.AnnAssign) or not isinstance(node.target, ast.Name):
            prev_end = getattr(node, "end_lineno", prev_end)
            continue
        block: List[str] = []
        for raw in lines[prev_end:node.lineno - 1]:
            s = raw.strip()
            if s.startswith("# ---"):
                section = s.strip("#- ").strip()
                block = []
            elif s.startswith("#"):
                block.append(s.lstrip("#").strip())
        tail = trailing.get(node.lineno, "")
        text = " ".join(block + ([tail] if tail else []))
        docs[node.target.id] = text
        sections[node.target.id] = section
        prev_end = node.end_lineno or node.lineno
    return docs, sections


def _default(f: dataclasses.Field) -> str:
    if f.default is not dataclasses.MISSING:
        v = f.default
    elif f.default_factory is not dataclasses.MISSING:  # type: ignore[misc]
        v = f.default_factory()  # type: ignore[misc]
    else:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    if f.name == "device_file_mode":
        return oct(v).replace("0o", "0")
    if v == "" or v == {}:
        return '""' if v == "" else "{}"
    return str(v)


def _cell(s: str) -> str:
    return s.replace("|", "\\|")


def render() -> str:
    docs, sections = _comments()
    out = ["# Configuration reference",
           "",
           "Generated from `gpumounter_amd/utils/config.py` by `python -m gpumounter_amd config-doc`;",
           "`tests/test_deploy_and_cli.py` checks that this file is current.",
           "",
           "Every setting resolves in this order: the default, then a YAML file named by",
           "`GM_CONFIG`, then the environment variable `GM_<FIELD>`, then explicit overrides.",
           "Booleans take `1 t true yes on` or `0 f false no off` (empty = false); integers take",
           "`0o`/`0x` prefixes. `NODE_NAME`, `POD_NAME`, `POD_NAMESPACE` (downward API) and the",
           "reference's only knob, `CGROUP_DRIVER` (reference: pkg/util/cgroup/cgroup.go:78-84), fill",
           "the matching fields when their `GM_` variable is unset.",
           ""]
    current = None
    for f in dataclasses.fields(_config.Config):
        if f.name == "extra":
            continue
        sec = sections.get(f.name, "") or "general"
        if sec != current:
            current = sec
            out += ["", f"## {sec}", "", "| variable | default | meaning |", "|---|---|---|"]
        out.append(f"| `GM_{f.name.upper()}` | `{_cell(_default(f))}` | "
                   f"{_cell(docs.get(f.name, ''))} |")
    return "\n".join(out) + "\n"


def render_metrics() -> str:
    from gpumounter_amd.utils.metrics import Metrics

    out = ["# Metrics reference",
           "",
           "Generated from `gpumounter_amd/utils/metrics.py` by",
           "`python -m gpumounter_amd config-doc --metrics`; `tests/test_deploy_and_cli.py` checks",
           "that this file is current.",
           "",
           "Workers serve these on `:9400/metrics` (`GM_METRICS_PORT`), the master on",
           "`/metrics` of its HTTP port. Histograms are in seconds, with buckets from 0.5 ms to",
           "120 s. Counters carry the `_total` suffix on the wire.",
           "",
           "`gm_requests_total{result}` holds the reference's result names for answered RPCs",
           "(`Success`, `InsufficientGPU`, `PodNotFound`, `GPUBusy`, `GPUNotFound`) and the gRPC",
           "status for failed ones: `INTERNAL` (rolled back), `RESOURCE_EXHAUSTED` (quota),",
           "`FAILED_PRECONDITION` (mount-type refusal). Alert rules on these metrics:",
           "`deploy/monitoring/prometheus-rules.yaml` (Prometheus Operator).",
           "",
           "| metric | type | labels | meaning |",
           "|---|---|---|---|"]
    for c in vars(Metrics()).values():
        if not hasattr(c, "_documentation"):
            continue
        name = c._name + ("_total" if c._type == "counter" else "")
        labels = ", ".join(f"`{x}`" for x in c._labelnames) or "—"
        out.append(f"| `{name}` | {c._type} | {labels} | {_cell(c._documentation)} |")
    return "\n".join(out) + "\n"
