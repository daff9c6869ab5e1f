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
    for name, cn in (("server", "gpu-mounter-worker"), ("client", "gpu-mounter-master")):
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
