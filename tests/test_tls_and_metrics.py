"""mTLS between master and worker (reference: insecure gRPC, main.go:82) and the worker's
periodic per-GPU metrics."""
import asyncio
import subprocess

import grpc
import pytest

from gpumounter_amd.fakes.harness import LocalCluster


def _openssl(*args, cwd):
    subprocess.run(["openssl", *args], cwd=cwd, check=True, capture_output=True)


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    d = tmp_path_factory.mktemp("pki")
    _openssl("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "ca.key", "-out",
             "ca.crt", "-days", "2", "-subj", "/CN=gm-test-ca", cwd=d)
    for name, cn in (("server", "gpu-mounter-worker"), ("client", "gpu-mounter-master"),
                     ("intruder", "some-other-pod")):
        (d / f"{name}.ext").write_text(f"subjectAltName=DNS:{cn}\n")
        _openssl("req", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{name}.key", "-out",
                 f"{name}.csr", "-subj", f"/CN={cn}", cwd=d)
        _openssl("x509", "-req", "-in", f"{name}.csr", "-CA", "ca.crt", "-CAkey", "ca.key",
                 "-CAcreateserial", "-out", f"{name}.crt", "-days", "2", "-extfile",
                 f"{name}.ext", cwd=d)
    return d


def test_mtls_master_worker(pki):
    w = {"tls_cert": str(pki / "server.crt"), "tls_key": str(pki / "server.key"),
         "tls_ca": str(pki / "ca.crt")}
    m = {"tls_cert": str(pki / "client.crt"), "tls_key": str(pki / "client.key"),
         "tls_ca": str(pki / "ca.crt")}

    async def main():
        async with LocalCluster(worker_overrides=w, master_overrides=m) as lc:
            lc.tenant("t")
            code, b = await lc.add("default", "t", 1)
            assert code == 200
            # a client without a certificate is rejected by the worker
            port = lc.nodes["node-0"].worker.grpc_port
            creds = grpc.ssl_channel_credentials(root_certificates=(pki / "ca.crt").read_bytes())
            ch = grpc.aio.secure_channel(f"127.0.0.1:{port}", creds, options=[
                ("grpc.ssl_target_name_override", "gpu-mounter-worker")])
            from gpumounter_amd.api import gpu_mount as api
            stub = ch.unary_unary(api.NODE_STATUS,
                                  request_serializer=api.NodeStatusRequest.SerializeToString,
                                  response_deserializer=api.NodeStatusResponse.FromString)
            with pytest.raises(grpc.aio.AioRpcError):
                await stub(api.NodeStatusRequest(), timeout=5)
            await ch.close()
            assert (await lc.remove("default", "t", [b["devices"][0]["uuid"]]))[0] == 200
    asyncio.run(main())


def test_worker_metrics_collector():
    async def main():
        async with LocalCluster() as lc:
            lc.tenant("m")
            await lc.add("default", "m", 3)
            w = lc.nodes["node-0"].worker
            await w.collect_metrics()
            text = w.metrics.render().decode()
            assert 'gm_ledger_gpus{state="GPU_ALLOCATED_STATE"} 3.0' in text
            assert 'gm_gpu_processes{gpu="0000:05:00.0"}' in text
    asyncio.run(main())


def test_hot_mounted_gpus_gauge_per_namespace():
    import asyncio

    from gpumounter_amd.fakes.harness import LocalCluster

    async def main():
        async with LocalCluster() as lc:
            lc.tenant("a", ns="team-a")
            lc.tenant("b", ns="team-b")
            assert (await lc.add("team-a", "a", 3))[0] == 200
            code, b = await lc.add("team-b", "b", 2)
            assert code == 200
            w = lc.nodes["node-0"].worker
            await w.collect_metrics()
            text = w.metrics.render().decode()
            assert 'gm_hot_mounted_gpus{namespace="team-a"} 3.0' in text
            assert 'gm_hot_mounted_gpus{namespace="team-b"} 2.0' in text
            assert (await lc.remove("team-b", "b", [d["uuid"] for d in b["devices"]]))[0] == 200
            await w.collect_metrics()
            assert 'gm_hot_mounted_gpus{namespace="team-b"} 0.0' in w.metrics.render().decode()
    asyncio.run(main())


def test_worker_with_a_ca_signed_but_foreign_identity_is_denied(pki):
    """Same CA, wrong identity (another component's certificate): PERMISSION_DENIED."""
    w = {"tls_cert": str(pki / "server.crt"), "tls_key": str(pki / "server.key"),
         "tls_ca": str(pki / "ca.crt")}
    m = {"tls_cert": str(pki / "client.crt"), "tls_key": str(pki / "client.key"),
         "tls_ca": str(pki / "ca.crt")}

    async def main():
        async with LocalCluster(worker_overrides=w, master_overrides=m) as lc:
            port = lc.nodes["node-0"].worker.grpc_port
            creds = grpc.ssl_channel_credentials(
                root_certificates=(pki / "ca.crt").read_bytes(),
                private_key=(pki / "intruder.key").read_bytes(),
                certificate_chain=(pki / "intruder.crt").read_bytes())
            ch = grpc.aio.secure_channel(f"127.0.0.1:{port}", creds, options=[
                ("grpc.ssl_target_name_override", "gpu-mounter-worker")])
            from gpumounter_amd.api import gpu_mount as api
            stub = ch.unary_unary(api.REMOVE_GPU,
                                  request_serializer=api.RemoveGPURequest.SerializeToString,
                                  response_deserializer=api.RemoveGPUResponse.FromString)
            with pytest.raises(grpc.aio.AioRpcError) as ei:
                await stub(api.RemoveGPURequest(pod_name="x", namespace="default", force=True),
                           timeout=5)
            assert ei.value.code() == grpc.StatusCode.PERMISSION_DENIED
            await ch.close()
            lc.tenant("t")                      # the master's own identity still works
            assert (await lc.add("default", "t", 1))[0] == 200
    asyncio.run(main())


def test_secure_defaults():
    """Out of the box: the master authorizes callers against Kubernetes RBAC and the worker
    will not serve its gRPC API without mTLS (reference: neither — main.go:82,185)."""
    from gpumounter_amd.utils.config import Config
    cfg = Config.load(env={})
    assert cfg.authz_mode == "kube" and cfg.worker_insecure is False

    async def main():
        async with LocalCluster(start_workers=False, start_master=False) as lc:
            from gpumounter_amd.worker.server import Worker
            h = lc.nodes["node-0"]
            c = Config.load(env={}, kube_api=lc.api_url, node_name="node-0",
                            kubelet_socket=h.kubelet.socket_path, amdsmi_lib="mock",
                            cgroup_root=h.node.cgroup_root, devnode_mode="emulate",
                            container_root_prefix=h.node.rootfs_root, state_dir=h.node.state_dir,
                            host_dev_path=h.node.host_dev, worker_host="127.0.0.1")
            w = Worker(c, inventory=lc.inventory)
            with pytest.raises(ValueError, match="mTLS"):
                await w.start(grpc_port=0, http_port=-1, reconcile=False)
            await w.stop()
        async with LocalCluster(master_overrides={"authz_mode": "kube"}) as lc:
            lc.tenant("t")
            # no bearer token → 401 at the master
            async with lc.session.get(lc.master_url + "/addgpu/namespace/default/pod/t/gpu/1/"
                                      "isEntireMount/false") as r:
                assert r.status == 401
            assert lc.cluster.placeholders() == []
    asyncio.run(main())


def test_deploy_sh_pki_works_end_to_end(tmp_path):
    """The certificates deploy.sh creates (stub kubectl captures the Secret) carry the identities
    the worker and master check: the master's certificate is accepted by the worker."""
    import os
    import stat
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "secret"
    out.mkdir()
    bindir = tmp_path / "bin"
    bindir.mkdir()
    kubectl = bindir / "kubectl"
    kubectl.write_text(f"""#!/bin/bash
if [[ "$*" == *"get secret"* ]]; then exit 1; fi
for a in "$@"; do
  case "$a" in --from-file=*) kv="${{a#--from-file=}}"; cp "${{kv#*=}}" "{out}/${{kv%%=*}}";; esac
done
""")
    kubectl.chmod(kubectl.stat().st_mode | stat.S_IEXEC)
    script = (f'set -euo pipefail; source <(sed -n "/^pki()/,/^}}/p" {root}/deploy.sh); '
              f'NS=kube-system; SECRET=gpu-mounter-tls; pki')
    subprocess.run(["bash", "-c", script], check=True, timeout=120,
                   env={**os.environ, "PATH": f"{bindir}:{os.environ['PATH']}"})
    assert sorted(p.name for p in out.iterdir()) == [
        "ca.crt", "master-https.crt", "master-https.key", "master.crt", "master.key",
        "worker.crt", "worker.key"]
    w = {"tls_cert": str(out / "worker.crt"), "tls_key": str(out / "worker.key"),
         "tls_ca": str(out / "ca.crt")}
    m = {"tls_cert": str(out / "master.crt"), "tls_key": str(out / "master.key"),
         "tls_ca": str(out / "ca.crt"), "master_tls_cert": str(out / "master-https.crt"),
         "master_tls_key": str(out / "master-https.key")}

    async def main():
        import ssl

        async with LocalCluster(worker_overrides=w, master_overrides=m) as lc:
            lc.tenant("t")
            # the master's API is HTTPS, verifiable against the deploy's CA by the Service's
            # in-cluster name and by localhost (kubectl port-forward)
            assert lc.master.http.tls
            ctx = ssl.create_default_context(cafile=str(out / "ca.crt"))
            for host in ("localhost", "gpu-mounter-service.kube-system.svc", "127.0.0.1"):
                r, wr = await asyncio.open_connection(
                    "127.0.0.1", lc.master.port, ssl=ctx, server_hostname=host)
                wr.write(b"GET /healthz HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
                assert (await r.read()).startswith(b"HTTP/1.1 200 ")
                wr.close()
            url = f"https://127.0.0.1:{lc.master.port}/addgpu/namespace/default/pod/t/gpu/1/" \
                  "isEntireMount/false"
            async with lc.session.get(url, ssl=ctx,
                                      headers={"Accept": "application/json"}) as resp:
                assert resp.status == 200, await resp.text()
            # plain HTTP on the same port is not served
            with pytest.raises(Exception):
                async with lc.session.get(url.replace("https", "http")) as resp:
                    await resp.read()
    asyncio.run(main())


def test_worker_status_routes_need_rbac_like_the_masters_read_routes():
    """/status lists every Pod's GPUs on the node and /audit one Pod's rules: a caller without
    a token gets 401, one RBAC does not allow gets 403 (the shipped networkpolicy leaves the
    port open for Prometheus and probes, which keep /metrics, /healthz, /readyz)."""
    async def main():
        async with LocalCluster(worker_overrides={"status_authz": "kube"}) as lc:
            lc.tenant("t")
            c = lc.cluster
            c.add_user("tok-nobody", "nobody")
            c.add_user("tok-tenant", "tenant")
            c.grant("tenant", ["get"], "pods/gpumount", ["default"])
            c.add_user("tok-admin", "admin")
            c.grant("admin", ["get"], "nodes/gpumount")
            port = lc.nodes["node-0"].worker.http_port
            base = f"http://127.0.0.1:{port}"

            async def get(path, token=""):
                h = {"Authorization": f"Bearer {token}"} if token else {}
                async with lc.session.get(base + path, headers=h) as r:
                    return r.status
            assert await get("/audit/default/t") == 401
            assert await get("/status") == 401
            assert await get("/audit/default/t", "tok-nobody") == 403
            assert await get("/status", "tok-nobody") == 403
            assert await get("/audit/default/t", "tok-tenant") == 200
            assert await get("/audit/other/t", "tok-tenant") == 403
            assert await get("/status", "tok-tenant") == 403
            assert await get("/status", "tok-admin") == 200
            assert await get("/audit/default/a%2Fb", "tok-tenant") == 404     # not a route
            assert await get("/audit/default/Not_A_Name", "tok-tenant") == 400  # not a name
            for open_path in ("/healthz", "/readyz", "/metrics"):
                assert await get(open_path) == 200
    asyncio.run(main())
