"""Deployment manifests agree with the code's defaults; CLI subcommands work on the mock."""
import json
import os
import subprocess
import sys

import yaml

from gpumounter_amd.utils.config import Config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(name):
    with open(os.path.join(ROOT, "deploy", name)) as fh:
        return [d for d in yaml.safe_load_all(fh) if d]


def test_worker_daemonset_shape():
    (ds,) = load("gpu-mounter-workers.yaml")
    spec = ds["spec"]["template"]["spec"]
    cfg = Config.load(env={})
    assert ds["metadata"]["namespace"] == cfg.worker_namespace
    k, v = cfg.worker_label.split("=")
    assert ds["spec"]["template"]["metadata"]["labels"][k] == v
    assert spec["hostPID"] is True
    c = spec["containers"][0]
    assert c["securityContext"]["privileged"] is True
    assert {p["containerPort"] for p in c["ports"]} == {cfg.worker_port, cfg.wire_port,
                                                        cfg.metrics_port}
    mounts = {m["mountPath"] for m in c["volumeMounts"]}
    assert {"/sys/fs/cgroup", "/sys/fs/bpf", "/var/lib/kubelet/pod-resources", "/dev",
            "/sys/class/kfd"} <= mounts
    env = {e["name"]: e for e in c["env"]}
    assert env["NODE_NAME"]["valueFrom"]["fieldRef"]["fieldPath"] == "spec.nodeName"
    assert env["GM_BPF_PIN_DIR"]["value"].startswith("/sys/fs/bpf")
    assert "NVIDIA_VISIBLE_DEVICES" not in env
    # secure by default: mTLS on :1200 with the master as the only accepted identity
    assert env["GM_TLS_CA"]["value"] and env["GM_TLS_CERT"]["value"] and env["GM_TLS_KEY"]["value"]
    assert env["GM_TLS_CLIENT_NAMES"]["value"] == "gpu-mounter-master"
    assert "GM_WORKER_INSECURE" not in env
    assert env["POD_NAME"]["valueFrom"]["fieldRef"]["fieldPath"] == "metadata.name"
    assert env["GM_STATE_DIR"]["value"] == "/var/lib/gpumounter"


def test_kind_overlay_env_is_valid_config():
    """Every GM_* variable in the kind patch parses into the Config the worker would run with."""
    (patch,) = load("kind/workers-mock-patch.yaml")
    c = patch["spec"]["template"]["spec"]["containers"][0]
    env = {e["name"]: e["value"] for e in c["env"]}
    cfg = Config.load(env=env)
    assert cfg.amdsmi_lib == "mock" and cfg.device_plugin and not cfg.device_plugin_inject
    assert cfg.devnode_mode == "emulate" and cfg.kfd_major == 511
    (ds,) = load("gpu-mounter-workers.yaml")
    names = {v["name"] for v in ds["spec"]["template"]["spec"]["volumes"]}
    assert {v["name"] for v in patch["spec"]["template"]["spec"]["volumes"]} <= names
    assert "/var/lib/kubelet/device-plugins" in {
        m["mountPath"] for m in ds["spec"]["template"]["spec"]["containers"][0]["volumeMounts"]}


def test_tenant_rbac_example_targets_the_gpumount_subresource():
    docs = load("rbac-tenant-example.yaml")
    roles = {d["metadata"]["name"]: d for d in docs if d["kind"] == "ClusterRole"}
    from gpumounter_amd.master.authz import RESOURCE_SUB
    assert roles["gpumount-user"]["rules"][0]["resources"] == [f"pods/{RESOURCE_SUB}"]
    assert set(roles["gpumount-user"]["rules"][0]["verbs"]) == {"create", "delete", "get"}
    (ctl,) = [d for d in load("rbac.yaml") if d["kind"] == "ClusterRole"]
    groups = {g for r in ctl["rules"] for g in r["apiGroups"]}
    assert {"authentication.k8s.io", "authorization.k8s.io"} <= groups


def test_rbac_is_least_privilege():
    docs = load("rbac.yaml")
    roles = [d for d in docs if d["kind"] == "ClusterRole"]
    binding = next(d for d in docs if d["kind"] == "ClusterRoleBinding")
    assert binding["roleRef"]["name"] != "cluster-admin"
    resources = {r for role in roles for rule in role["rules"] for r in rule["resources"]}
    assert resources <= {"pods", "pods/finalizers", "nodes", "events", "tokenreviews",
                         "subjectaccessreviews", "resourcequotas", "resourceclaims",
                         "resourceslices", "priorityclasses"}
    assert {v for role in roles for rule in role["rules"] if "pods/finalizers" in
            rule["resources"] for v in rule["verbs"]} == {"update"}
    dra = [rule for role in roles for rule in role["rules"]
           if rule["apiGroups"] == ["resource.k8s.io"]]
    assert {v for rule in dra if rule["resources"] == ["resourceslices"]
            for v in rule["verbs"]} == {"list"}           # slices are read-only
    assert all("*" not in rule["verbs"] for role in roles for rule in role["rules"])
    reviews = [rule for role in roles for rule in role["rules"]
               if set(rule["resources"]) & {"tokenreviews", "subjectaccessreviews"}]
    assert all(rule["verbs"] == ["create"] for rule in reviews)


def test_service_and_master_ports():
    (svc,) = load("gpu-mounter-svc.yaml")
    (dep,) = load("gpu-mounter-master.yaml")
    cfg = Config.load(env={})
    assert svc["spec"]["ports"][0]["port"] == 443 and svc["spec"]["ports"][0]["name"] == "https"
    assert svc["spec"]["ports"][0]["targetPort"] == cfg.master_port
    assert svc["spec"]["selector"] == dep["spec"]["template"]["metadata"]["labels"]
    assert load("namespace.yaml")[0]["metadata"]["name"] == cfg.pool_namespace


def _cli(*args):
    res = subprocess.run([sys.executable, "-m", "gpumounter_amd", *args], cwd=ROOT,
                         capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    return res.stdout


def test_cli_inventory_topology_bpf_dump():
    inv = json.loads(_cli("inventory", "--amdsmi", "mock"))
    assert inv["count"] == 8 and inv["gpus"][0]["gfx_target"] == "gfx950"
    topo = json.loads(_cli("topology", "--amdsmi", "mock", "-n", "4"))
    assert topo["plans"]["4"]["numa_nodes"] == 1 and topo["describe"]["all_pairs_xgmi"]
    dump = _cli("bpf-dump", "--allow", "226:128", "--allow", "511:0")
    assert "if r4 != 226" in dump and "call bpf_tail_call#12" in dump


def test_master_and_network_policy_are_secure_by_default():
    (dep,) = load("gpu-mounter-master.yaml")
    c = dep["spec"]["template"]["spec"]["containers"][0]
    env = {e["name"]: e.get("value") for e in c["env"]}
    cfg = Config.load(env={k: v for k, v in env.items() if v is not None})
    assert cfg.authz_mode == "kube" and cfg.tls_ca and cfg.tls_cert and cfg.tls_key
    # no cleartext token path: callers' bearer tokens reach the master over HTTPS only, its
    # certificate is in the Secret deploy.sh creates, and the probes speak HTTPS
    assert cfg.master_tls_cert and cfg.master_tls_key
    items = {i["key"] for v in dep["spec"]["template"]["spec"]["volumes"]
             for i in (v.get("secret") or {}).get("items", [])}
    assert {"master-https.crt", "master-https.key"} <= items
    for probe in ("readinessProbe", "livenessProbe"):
        assert c[probe]["httpGet"]["scheme"] == "HTTPS"
    with open(os.path.join(ROOT, "deploy.sh")) as fh:
        assert "master-https.crt" in fh.read()
    # the workers' status routes are authorized as the master's read routes are
    (ds,) = load("gpu-mounter-workers.yaml")
    wenv = {e["name"]: e.get("value") for e in
            ds["spec"]["template"]["spec"]["containers"][0]["env"]}
    wcfg = Config.load(env={k: v for k, v in wenv.items() if v is not None and
                            k.startswith("GM_")})
    assert wcfg.status_authz in ("auto", "kube") and wcfg.authz_mode == "kube"
    (np,) = load("networkpolicy.yaml")
    assert np["spec"]["podSelector"]["matchLabels"] == {"app": "gpu-mounter-worker"}
    rules = np["spec"]["ingress"]
    for port in (1200, 1201):        # gRPC and gm-wire: the master only
        grpc_rule = [r for r in rules if any(p["port"] == port for p in r["ports"])]
        assert len(grpc_rule) == 1
        assert grpc_rule[0]["from"] == [{"podSelector": {"matchLabels":
                                                         {"app": "gpu-mounter-master"}}}]
    # the DaemonSet advertises the gm-wire port the worker binds by default
    (ds,) = load("gpu-mounter-workers.yaml")
    tmpl = ds["spec"]["template"]
    assert tmpl["metadata"]["annotations"]["gpumounter.amd.com/wire-port"] == \
        str(Config.load(env={}).wire_port)
    ports = {p["containerPort"] for p in tmpl["spec"]["containers"][0]["ports"]}
    assert {1200, 1201} <= ports
    with open(os.path.join(ROOT, "deploy", "kustomization.yaml")) as fh:
        assert "networkpolicy.yaml" in yaml.safe_load(fh)["resources"]
    with open(os.path.join(ROOT, "deploy.sh")) as fh:
        text = fh.read()
    assert "deploy/networkpolicy.yaml" in text and "gpu-mounter-tls" in text


def test_cli_add_and_remove_authenticate_against_the_shipped_master(tmp_path):
    """The shipped master authorizes callers (GM_AUTHZ_MODE=kube): the CLI sends a bearer
    token (--token, $GM_TOKEN, --token-file, SA token, kubeconfig user) and is refused
    without one."""
    from gpumounter_amd.fakes.deployment import ProcessCluster

    with ProcessCluster() as pc:
        pc.tenant("cli")
        assert pc.master_url.startswith("https://")
        env = {**os.environ, "KUBECONFIG": str(tmp_path / "none"), "GM_TOKEN": "",
               "GM_MASTER_CA": pc.ca}
        base = [sys.executable, "-m", "gpumounter_amd"]
        r = subprocess.run(base + ["add", "--master", pc.master_url, "--pod", "cli", "-n", "1"],
                           capture_output=True, text=True, cwd=ROOT, env=env, timeout=120)
        assert r.returncode == 1 and "bearer token" in r.stderr
        (tmp_path / "tok").write_text(pc.token + "\n")
        r = subprocess.run(base + ["add", "--master", pc.master_url, "--pod", "cli", "-n", "1",
                                   "--token-file", str(tmp_path / "tok")],
                           capture_output=True, text=True, cwd=ROOT, env=env, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        uuid = json.loads(r.stdout)["devices"][0]["uuid"]
        # the master's certificate is verified: without the CA the CLI refuses to talk to it
        r2 = subprocess.run(base + ["status", "--master", pc.master_url, "--node", "node-0",
                                    "--token-file", str(tmp_path / "tok")],
                            capture_output=True, text=True, cwd=ROOT,
                            env={**env, "GM_MASTER_CA": ""}, timeout=120)
        assert r2.returncode != 0 and "CERTIFICATE_VERIFY_FAILED" in r2.stderr
        r = subprocess.run(base + ["remove", "--master", pc.master_url, "--pod", "cli",
                                   "--uuid", uuid],
                           capture_output=True, text=True, cwd=ROOT,
                           env={**env, "GM_TOKEN": pc.token}, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr


def test_cluster_role_grants_every_api_call_the_daemons_make():
    """Each KubeClient call needs one (verb, resource) in deploy/rbac.yaml's ClusterRole; a new
    call without a grant would fail only on a real cluster (the hermetic apiserver does not
    enforce RBAC), so the mapping is checked here."""
    import inspect

    import yaml

    from gpumounter_amd.cluster.kube import KubeClient

    needs = {
        "get_pod": ("", "pods", "get"), "list_pods": ("", "pods", "list"),
        "watch_pods": ("", "pods", "watch"), "create_pod": ("", "pods", "create"),
        "delete_pod": ("", "pods", "delete"), "patch_pod": ("", "pods", "patch"),
        "create_claim": ("resource.k8s.io", "resourceclaims", "create"),
        "get_claim": ("resource.k8s.io", "resourceclaims", "get"),
        "delete_claim": ("resource.k8s.io", "resourceclaims", "delete"),
        "list_claims": ("resource.k8s.io", "resourceclaims", "list"),
        "list_claims_rv": ("resource.k8s.io", "resourceclaims", "list"),
        "watch_claims": ("resource.k8s.io", "resourceclaims", "watch"),
        "list_slices": ("resource.k8s.io", "resourceslices", "list"),
        "token_review": ("authentication.k8s.io", "tokenreviews", "create"),
        "subject_access_review": ("authorization.k8s.io", "subjectaccessreviews", "create"),
        # sent with the caller's token: the caller's own rights (system:basic-user), not ours
        "self_subject_access_review": None,
        "list_resource_quotas": ("", "resourcequotas", "list"),
        "list_quotas_rv": ("", "resourcequotas", "list"),
        "get_quota": ("", "resourcequotas", "get"),
        "watch_quotas": ("", "resourcequotas", "watch"),
        "create_event": ("", "events", "create"),
        "get_priority_class": ("scheduling.k8s.io", "priorityclasses", "get"),
    }
    calls = {n for n, f in inspect.getmembers(KubeClient)
             if (inspect.iscoroutinefunction(f) or inspect.isasyncgenfunction(f))
             and not n.startswith("_") and n not in ("close", "watch", "list_pages")}
    assert calls == set(needs), ("map new KubeClient calls to their RBAC verb",
                                 calls ^ set(needs))
    docs = list(yaml.safe_load_all(open(os.path.join(ROOT, "deploy", "rbac.yaml"))))
    role = next(d for d in docs if d and d.get("kind") == "ClusterRole")
    granted = {(g, r, v) for rule in role["rules"] for g in rule.get("apiGroups", [])
               for r in rule.get("resources", []) for v in rule.get("verbs", [])}
    missing = {n: need for n, need in needs.items() if need is not None and need not in granted}
    assert not missing, missing


def test_config_reference_is_current_and_documents_every_setting():
    """docs/CONFIG.md is generated from config.py (every field, its GM_ variable, default and
    comment); a field added without a comment, or a stale copy, fails here."""
    from gpumounter_amd.utils.configdoc import render

    text = render()
    with open(os.path.join(ROOT, "docs", "CONFIG.md")) as fh:
        assert fh.read() == text, "regenerate: python -m gpumounter_amd config-doc > docs/CONFIG.md"
    rows = [ln for ln in text.splitlines() if ln.startswith("| `GM_")]
    assert len(rows) == len(Config.__dataclass_fields__) - 1          # all but `extra`
    assert not [r for r in rows if r.endswith("|  |")], "fields without a comment"
    assert "| `GM_PLACEMENT_ENFORCE` | `auto` |" in text
    assert "| `GM_DEVICE_FILE_MODE` | `0666` |" in text


def test_metrics_reference_is_current():
    from gpumounter_amd.utils.configdoc import render_metrics

    text = render_metrics()
    with open(os.path.join(ROOT, "docs", "METRICS.md")) as fh:
        assert fh.read() == text, \
            "regenerate: python -m gpumounter_amd config-doc --metrics > docs/METRICS.md"
    assert "| `gm_attach_latency_seconds` | histogram | `n_gpus`, `mode` |" in text
    assert "`gm_draining_placeholders`" in text and "`gm_requests_total`" in text


def test_alert_rules_use_existing_metrics():
    import re

    from gpumounter_amd.utils.metrics import Metrics

    (rule,) = load("monitoring/prometheus-rules.yaml")
    names = set()
    for c in vars(Metrics()).values():
        if hasattr(c, "_documentation"):
            base = c._name
            names |= {base, base + "_total", base + "_bucket", base + "_sum", base + "_count"}
    used = {m for g in rule["spec"]["groups"] for r in g["rules"]
            for m in re.findall(r"\bgm_[a-z_]+", r["expr"])}
    assert used and used <= names, used - names
    with open(os.path.join(ROOT, "deploy", "kustomization.yaml")) as fh:
        assert "monitoring" not in fh.read()          # needs the operator's CRDs: opt-in
