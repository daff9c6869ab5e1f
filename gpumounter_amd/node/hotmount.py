"""Hot-mount transactions: grant + inject on attach, revoke + unlink on detach, with rollback.

Reference: ``MountGPU`` = container ID (docker only) → cgroup path → ``devices.allow`` → first PID
→ nsenter mknod (reference: pkg/util/util.go:17-71); ``UnmountGPU`` = busy check → ``devices.deny``
→ ``rm`` → ``kill`` (util.go:73-147). Partial failures are not rolled back (server.go:86-91 only
deletes slave pods — SURVEY §2.6 defect 12) and only ``ContainerStatuses[0]`` is handled
(defect 8).

Here one transaction covers every running container of the pod (or a named one), computes the
exact node set from the ledger (the pod's own device-plugin GPUs are never touched, ``/dev/kfd``
is granted with the first hot-mounted GPU and revoked with the last), and undoes completed steps
in reverse order if any step fails.

Ownership (what may ever be revoked) is scoped to what gpumounter itself injected, recorded per
container in the :class:`~gpumounter_amd.node.journal.InjectionJournal`: the audit only reports a
GPU rule/node as *stale* when the journal says gpumounter put it there, so pods it never touched —
privileged pods, pods mounting the host's ``/dev``, the worker itself — are never swept. Privileged
containers already hold every host device and are skipped entirely (ledger-only attach), and the
native layer refuses to mknod/unlink in a directory that is the host's ``/dev`` or ``/dev/dri``
(gm_devnodes_guard).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from gpumounter_amd.hw.inventory import Inventory
from gpumounter_amd.models.device import AmdGpu, DeviceNode, kfd_node
from gpumounter_amd.models.pod import ContainerRef, running_containers
from gpumounter_amd.node.cgroup import CgroupError, CgroupResolver, DeviceRuleBackend
from gpumounter_amd.node.devnodes import CREATED, DevNodeError, DevNodeWriter, Target
from gpumounter_amd.node.journal import InjectionJournal
from gpumounter_amd.utils import log, trace

_log = log.get("node.hotmount")


class MountError(RuntimeError):
    pass


@dataclass
class ContainerTarget:
    ref: ContainerRef
    cgdir: str
    target: Target
    pids: List[int] = field(default_factory=list)


@dataclass
class AuditIssue:
    container: str
    kind: str        # missing_rule | missing_node | stale_rule | stale_node
    path: str
    major: int
    minor: int


class HotMount:
    def __init__(self, cfg, inv: Inventory, resolver: CgroupResolver, backend: DeviceRuleBackend,
                 writer: DevNodeWriter, faults=None,
                 journal: Optional[InjectionJournal] = None) -> None:
        from gpumounter_amd.utils.faults import NONE

        self.cfg = cfg
        self.inv = inv
        self.resolver = resolver
        self.backend = backend
        self.writer = writer
        self.faults = faults if faults is not None else NONE
        self.journal = journal if journal is not None else InjectionJournal()
        # cgroup → the backend's fingerprint right after our last change: anything else that
        # changes the cgroup's device control shows as a different one (the device guard)
        self.expected: Dict[str, object] = {}

    def _apply(self, cgdir: str, grant, revoke, desired) -> None:
        try:
            self.backend.apply(cgdir, grant, revoke, desired)
        finally:
            fp = getattr(self.backend, "fingerprint", None)
            self.expected[cgdir] = fp(cgdir) if fp is not None else None

    # ------------------------------------------------------------------------ node sets
    def kfd(self) -> DeviceNode:
        return kfd_node(self.inv.kfd_major)

    def gpu_nodes(self, gpus: Sequence[AmdGpu]) -> List[DeviceNode]:
        out: List[DeviceNode] = []
        for g in sorted(gpus, key=lambda g: g.index):
            out.extend(g.device_nodes(self.cfg.drm_major, self.cfg.inject_card_nodes,
                                      self.cfg.device_file_mode))
        return out

    def managed_nodes(self, hot: Sequence[AmdGpu], base: Sequence[AmdGpu]) -> List[DeviceNode]:
        """Nodes gpumounter owns for a pod holding ``hot`` hot-mounted GPUs and ``base`` own GPUs."""
        base_keys = {(n.major, n.minor) for n in self.gpu_nodes(base)}
        nodes = [n for n in self.gpu_nodes(hot) if (n.major, n.minor) not in base_keys]
        if hot and not base:
            nodes.insert(0, self.kfd())
        return nodes

    # ------------------------------------------------------------------------ targets
    def targets(self, pod: dict, container: str = "",
                include_privileged: bool = False) -> List[ContainerTarget]:
        """Running containers to act on. Privileged ones are left out of rule and node writes:
        the runtime already gave them every host device (and often the host's own ``/dev``), so
        there is nothing to grant and nothing gpumounter may take away — an attach to them is
        ledger-only. Their processes still use the GPUs they are given, so the busy check and
        the force-kill take them in (``include_privileged``; the reference takes PIDs from the
        container's cgroup whatever its privileges, pkg/util/util.go:152-196)."""
        refs = [r for r in running_containers(pod, container) if r.running]
        if not refs:
            raise MountError(f"pod {pod['metadata'].get('name')} has no running container"
                             + (f" named {container}" if container else ""))
        out = []
        for r in refs:
            if r.privileged and not include_privileged:
                continue
            cgdir = self.resolver.container_dir(pod, r)
            pids = self.resolver.pids(cgdir)
            if self.cfg.container_root_prefix:
                t = Target(root=os.path.join(self.cfg.container_root_prefix, r.id))
            else:
                t = Target(pid=self.writer.root_pid(pids))
            out.append(ContainerTarget(r, cgdir, t, pids))
        return out

    def _owner(self, pod: dict, t: ContainerTarget) -> dict:
        md = pod.get("metadata", {})
        return {"namespace": md.get("namespace", ""), "pod": md.get("name", ""),
                "pod_uid": md.get("uid", ""), "container": t.ref.name, "cgdir": t.cgdir}

    def resolve(self, pod: dict, container: str = "",
                include_privileged: bool = False) -> List[ContainerTarget]:
        """:meth:`targets` for a transaction: a container that vanished meanwhile (pod deleted
        or restarted mid-attach) is a MountError, so the caller's rollback runs."""
        try:
            return self.targets(pod, container, include_privileged)
        except (CgroupError, OSError) as e:
            raise MountError(f"cannot resolve the pod's containers: {e}") from e

    # ------------------------------------------------------------------------ attach
    def attach(self, pod: dict, new: Sequence[AmdGpu], have: Sequence[AmdGpu],
               base: Sequence[AmdGpu] = (), container: str = "") -> List[ContainerTarget]:
        before = self.managed_nodes(have, base)
        after = self.managed_nodes(list(have) + list(new), base)
        before_keys = {(n.major, n.minor) for n in before}
        grant = [n for n in after if (n.major, n.minor) not in before_keys]
        with trace.span("resolve"):
            targets = self.resolve(pod, container)
        done: List[tuple] = []  # (target, granted, created_nodes)
        j = self.journal
        try:
            for t in targets:
                cid = t.ref.id
                known = j.nodes_of(cid)
                # nodes the container holds already and gpumounter did not create are never
                # recorded, not even for the moment between the write-ahead and the create: a
                # worker killed in that window must not leave them journaled as its own
                with trace.span("devnodes_probe", nodes=len(after)):
                    states = self.writer.present_states(t.target, after)
                theirs = {(n.major, n.minor) for n, st in zip(after, states)
                          if st and (n.major, n.minor) not in known}
                # write-ahead: the journal names the state before the kernel holds it
                j.intend(cid, [((n.major, n.minor), n.path) for n in grant],
                         [((n.major, n.minor), n.path) for n in after
                          if (n.major, n.minor) not in theirs], **self._owner(pod, t))
                # in `done` before the kernel call: an apply that fails part-way (a v1 write of
                # several lines, a set-mode map updated before a later step fails) is revoked
                # by the rollback like a completed one
                done.append((t, grant, []))
                with trace.span("cgroup_rule", backend=self.backend.name, rules=len(grant)):
                    self.faults.check("cgroup_rule")
                    self._apply(t.cgdir, grant, [], after)
                self.faults.check("cgroup_rule", "after")
                with trace.span("devnodes", nodes=len(after)):
                    self.faults.check("devnodes")
                    res = self.writer.create(t.target, after)
                done[-1] = (t, grant, [n for n, r in zip(after, res) if r == CREATED])
                # a node another party created between the probe and the create stays theirs
                j.settle(cid, [(n.major, n.minor) for n, r in zip(after, res)
                               if r != CREATED and (n.major, n.minor) not in known
                               and (n.major, n.minor) not in theirs])
                self.faults.check("devnodes", "after")
        except Exception as e:
            self._rollback_attach(done, before)
            # intents for containers whose kernel calls never ran are withdrawn as well
            for t in targets[len(done):]:
                self._forget_new(t.ref.id, grant, after, before)
            raise MountError(f"attach failed, rolled back: {e}") from e
        return targets

    def _forget_new(self, cid: str, granted, after, before) -> None:
        keep = {(n.major, n.minor) for n in before}
        self.journal.forget(cid, [(n.major, n.minor) for n in granted],
                            [(n.major, n.minor) for n in after if (n.major, n.minor) not in keep])

    def _rollback_attach(self, done, before: List[DeviceNode]) -> None:
        before_keys = {(n.major, n.minor) for n in before}
        for t, granted, created in reversed(done):
            try:
                self.writer.remove(t.target, created)
            except Exception as e:  # noqa: BLE001
                _log.error("rollback unlink in %s failed: %s", t.ref.name, e)
            else:
                self.journal.forget(t.ref.id, (), [(n.major, n.minor) for n in created
                                                   if (n.major, n.minor) not in before_keys])
            try:
                # revoke what the kernel holds of it: an apply that failed part-way granted
                # some of the set or none (a v1 deny of a rule never allowed would unbalance
                # the allow/deny bookkeeping of a later grant)
                try:
                    have = self.backend.installed(t.cgdir)
                    revoke = [n for n in granted if (n.major, n.minor) in have]
                except Exception:  # noqa: BLE001 - cannot read back: revoke all of it
                    revoke = list(granted)
                if revoke:
                    self._apply(t.cgdir, [], revoke, before)
            except Exception as e:  # noqa: BLE001
                _log.error("rollback revoke in %s failed: %s", t.cgdir, e)
            else:
                self.journal.forget(t.ref.id, [(n.major, n.minor) for n in granted])
            # intended nodes that were never created (the failing step) are not ours either
            ent = self.journal.nodes_of(t.ref.id)
            self.journal.forget(t.ref.id, (), [k for k in ent if k not in before_keys])

    # ------------------------------------------------------------------------ detach
    def detach(self, pod: dict, remove: Sequence[AmdGpu], keep: Sequence[AmdGpu],
               base: Sequence[AmdGpu] = (), container: str = "",
               targets: Optional[List[ContainerTarget]] = None) -> List[ContainerTarget]:
        before = self.managed_nodes(list(keep) + list(remove), base)
        after = self.managed_nodes(keep, base)
        after_keys = {(n.major, n.minor) for n in after}
        revoke = [n for n in before if (n.major, n.minor) not in after_keys]
        if targets is None:
            with trace.span("resolve"):
                targets = self.resolve(pod, container)
        try:
            self._detach(targets, revoke, after)
        except (CgroupError, DevNodeError, OSError) as e:
            # a container that went away meanwhile (restart, deletion): the caller rolls the pod
            # back to its ledger state, which covers the container running now
            raise MountError(f"detach failed: {e}") from e
        return targets

    def _detach(self, targets: List[ContainerTarget], revoke: List[DeviceNode],
                after: List[DeviceNode]) -> None:
        keys = [(n.major, n.minor) for n in revoke]
        for t in targets:
            # reference order: deny → rm → kill (util.go:112,131,139)
            with trace.span("cgroup_rule", backend=self.backend.name, rules=len(revoke)):
                self.faults.check("unmount")
                self._apply(t.cgdir, [], revoke, after)
            self.faults.check("unmount", "after")
            # only nodes gpumounter created: one the container already had stays (its rule is
            # revoked all the same, so it is as dead as it was before the attach)
            ours = self.journal.nodes_of(t.ref.id)
            unlink = [n for n in revoke if (n.major, n.minor) in ours]
            with trace.span("devnodes", nodes=len(unlink)):
                self.writer.remove(t.target, unlink)
            # one journal update for both steps: a worker that dies in between leaves revoked
            # rules journaled, which the audit forgets on sight (not in the kernel any more),
            # and its nodes, which the orphan sweep unlinks
            self.journal.forget(t.ref.id, keys, keys)

    def adopt(self, pod: dict, hot: Sequence[AmdGpu], base: Sequence[AmdGpu] = ()) -> int:
        """Seed the journal for containers of a pod that holds hot-mounted GPUs but has no
        journal record at all: grants made by a worker without a journal (before an upgrade,
        ``state_dir`` unset or wiped). The hot GPUs' managed rules that are granted and nodes
        that are present are recorded as gpumounter's, so a later detach, a foreign placeholder
        delete or the orphan sweep can revoke them. Containers with a record are left alone
        (their record is exact); returns the number of rules + nodes adopted."""
        want = self.managed_nodes(hot, base)
        if not want:
            return 0
        n = 0
        for t in self.targets(pod):
            if self.journal.get(t.ref.id) is not None:
                continue
            granted = self.backend.installed(t.cgdir)
            states = self.writer.present_states(t.target, want)
            rules = [((d.major, d.minor), d.path) for d in want if (d.major, d.minor) in granted]
            nodes = [((d.major, d.minor), d.path) for d, st in zip(want, states) if st == 1]
            if rules or nodes:
                self.journal.intend(t.ref.id, rules, nodes, **self._owner(pod, t))
                n += len(rules) + len(nodes)
        return n

    def repair(self, pod: dict, missing: Sequence[AuditIssue], hot: Sequence[AmdGpu],
               base: Sequence[AmdGpu] = ()) -> None:
        """Grant exactly the rules and create exactly the nodes :meth:`audit` reported missing
        (never re-granting a present rule, which would unbalance v1 allow/deny bookkeeping)."""
        desired = self.managed_nodes(hot, base)
        for t in self.targets(pod):
            mine = [i for i in missing if i.container == t.ref.name]
            rules = list({(i.major, i.minor): DeviceNode(i.path, i.major, i.minor)
                          for i in mine if i.kind == "missing_rule"}.values())
            nodes = [n for n in desired
                     if any(i.kind == "missing_node" and (i.major, i.minor) == (n.major, n.minor)
                            for i in mine)]
            if not rules and not nodes:
                continue
            known = self.journal.nodes_of(t.ref.id)
            self.journal.intend(t.ref.id, [((n.major, n.minor), n.path) for n in rules],
                                [((n.major, n.minor), n.path) for n in nodes],
                                **self._owner(pod, t))
            if rules:
                self._apply(t.cgdir, rules, [], desired)
            if nodes:
                res = self.writer.create(t.target, nodes)
                self.journal.settle(t.ref.id, [(n.major, n.minor) for n, r in zip(nodes, res)
                                               if r != CREATED and (n.major, n.minor) not in known])

    def revoke_issues(self, pod: dict, stale: Sequence[AuditIssue], hot: Sequence[AmdGpu],
                      base: Sequence[AmdGpu] = ()) -> None:
        """Revoke rules and unlink nodes reported as stale by :meth:`audit` (which only reports
        journaled state), per container."""
        keep = self.managed_nodes(hot, base)
        for t in self.targets(pod):
            mine = [i for i in stale if i.container == t.ref.name]
            rules = list({(i.major, i.minor): DeviceNode(i.path, i.major, i.minor)
                          for i in mine if i.kind == "stale_rule"}.values())
            unlink = list({(i.major, i.minor): DeviceNode(i.path, i.major, i.minor)
                           for i in mine if i.kind == "stale_node"}.values())
            if rules:
                self._apply(t.cgdir, [], rules, keep)
                self.journal.forget(t.ref.id, [(n.major, n.minor) for n in rules])
            if unlink:
                self.writer.remove(t.target, unlink)
                self.journal.forget(t.ref.id, (), [(n.major, n.minor) for n in unlink])

    def revoke_journaled(self, pod: dict, container_id: str) -> List[AuditIssue]:
        """Take back everything the journal says gpumounter injected into one container of a pod
        that no placeholder backs any more (the reconciler's orphan path). Returns what was
        revoked; state gpumounter did not record is never touched."""
        ent = self.journal.get(container_id)
        if ent is None:
            return []
        t = next((x for x in self.targets(pod) if x.ref.id == container_id), None)
        if t is None:
            return []
        rules = [DeviceNode(p, ma, mi) for (ma, mi), p in sorted(ent.rules.items())]
        nodes = [DeviceNode(p, ma, mi) for (ma, mi), p in sorted(ent.nodes.items())]
        out = [AuditIssue(t.ref.name, "stale_rule", n.path, n.major, n.minor) for n in rules]
        out += [AuditIssue(t.ref.name, "stale_node", n.path, n.major, n.minor) for n in nodes]
        if rules:
            self._apply(t.cgdir, [], rules, [])
            self.journal.forget(container_id, [(n.major, n.minor) for n in rules])
        if nodes:
            self.writer.remove(t.target, nodes)
            self.journal.forget(container_id, (), [(n.major, n.minor) for n in nodes])
        return out

    # ------------------------------------------------------------------------ audit
    def verify(self, pod: dict, hot: Sequence[AmdGpu], base: Sequence[AmdGpu] = (),
               container: str = "",
               targets: Optional[List[ContainerTarget]] = None) -> List[AuditIssue]:
        """Read back what an attach must have produced in every target container — the rules
        (as the kernel evaluates them) and nodes of every hot-mounted GPU (``hot``, the new ones
        included) and /dev/kfd when gpumounter manages it. A narrower, cheaper :meth:`audit`
        for the attach path: no journal walk, the attach's resolved ``targets`` are reused and
        every node is read back in one native call."""
        want = self.managed_nodes(hot, base)
        issues: List[AuditIssue] = []
        try:
            return self._verify(want, targets if targets is not None
                                else self.targets(pod, container), issues)
        except (CgroupError, DevNodeError, OSError) as e:
            # a container that restarted or went away after the mount: the attach rolls back
            raise MountError(f"read-back failed: {e}") from e

    def _verify(self, want: List[DeviceNode], targets: List[ContainerTarget],
                issues: List[AuditIssue]) -> List[AuditIssue]:
        for t in targets:
            allowed = self.backend.allowed(t.cgdir)
            present = self.writer.present_many(t.target, want)
            for n, ok in zip(want, present):
                if (n.major, n.minor) not in allowed:
                    issues.append(AuditIssue(t.ref.name, "missing_rule", n.path, n.major, n.minor))
                if not ok:
                    issues.append(AuditIssue(t.ref.name, "missing_node", n.path, n.major, n.minor))
        return issues

    def audit(self, pod: dict, hot: Sequence[AmdGpu], base: Sequence[AmdGpu] = (),
              container: str = "") -> List[AuditIssue]:
        """Compare the expected state (from the ledger) with cgroup rules and /dev contents."""
        want = self.managed_nodes(hot, base)
        want_keys = {(n.major, n.minor) for n in want}
        issues: List[AuditIssue] = []
        base_keys = {(n.major, n.minor) for n in self.gpu_nodes(base)}
        for t in self.targets(pod, container):
            allowed = self.backend.allowed(t.cgdir)
            for n, ok in zip(want, self.writer.present_many(t.target, want)):
                if (n.major, n.minor) not in allowed:
                    issues.append(AuditIssue(t.ref.name, "missing_rule", n.path, n.major, n.minor))
                if not ok:
                    issues.append(AuditIssue(t.ref.name, "missing_node", n.path, n.major, n.minor))
            # stale = recorded as injected by gpumounter and no longer backed by the ledger;
            # whatever else the container holds is not gpumounter's to judge
            ent = self.journal.get(t.ref.id)
            if ent is None:
                continue
            own = None
            for (ma, mi), path in sorted(ent.rules.items()):
                k = (ma, mi)
                if k in want_keys or k in base_keys:
                    continue
                if own is None:
                    # our own installed grants, not the effective verdict: a foreign program
                    # vetoing the pair today does not make our grant go away
                    own = self.backend.installed(t.cgdir)
                if k in own:
                    issues.append(AuditIssue(t.ref.name, "stale_rule", path, ma, mi))
                else:
                    self.journal.forget(t.ref.id, [k])        # already gone from the kernel
            for (ma, mi), path in sorted(ent.nodes.items()):
                k = (ma, mi)
                if k in want_keys or k in base_keys:
                    continue
                if self.writer.present(t.target, DeviceNode(path, ma, mi)):
                    issues.append(AuditIssue(t.ref.name, "stale_node", path, ma, mi))
                else:
                    self.journal.forget(t.ref.id, (), [k])
        return issues
