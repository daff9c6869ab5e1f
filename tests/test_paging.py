"""Paged LISTs (cluster/kube.py ``list_pages``) and the master's pod index.

client-go's reflector reads a collection in pages of 500 (``limit`` + ``continue``); a single
unpaged LIST of every Pod in a large cluster is hundreds of MB, over any sane response bound.
The reference only LISTs the worker DaemonSet's pods (reference:
cmd/GPUMounter-master/main.go:255-257); the master here indexes every Pod (pod → node without a
GET per request), so it pages, keeps only slim projections page by page, and restarts a list
whose continue token expired (410)."""
import asyncio
import time

from gpumounter_amd.cluster import http1
from gpumounter_amd.cluster.kube import ApiError, KubeClient
from gpumounter_amd.fakes.harness import LocalCluster

N_PODS = 50_000


def _bulk(cluster, n: int) -> None:
    """n Pods across 50 namespaces, created without scheduling (as if bound elsewhere)."""
    for i in range(n):
        pod = cluster.create_pod(f"ns-{i % 50}", {
            "metadata": {"name": f"p-{i}", "labels": {"app": "bulk"},
                         "annotations": {"note": "x" * 200}},
            "spec": {"nodeName": f"other-{i % 97}",
                     "containers": [{"name": "c", "image": "registry.example/app:1.0",
                                     "resources": {"requests": {"cpu": "100m"}}}]}},
            schedule=False)
        pod["status"]["phase"] = "Running"


def test_master_index_syncs_50k_pods_in_pages_of_bounded_size():
    async def main():
        async with LocalCluster() as lc:
            c = lc.cluster
            _bulk(c, N_PODS)
            c.list_pages, c.max_list_bytes = 0, 0
            relists = lc.master.pods.relists
            c.expire_watches()                   # 410 Gone: the master's index relists
            t0 = time.monotonic()
            while lc.master.pods.relists == relists or len(lc.master.pods.cache) < N_PODS:
                assert time.monotonic() - t0 < 120, len(lc.master.pods.cache)
                await asyncio.sleep(0.05)
            assert len(lc.master.pods.cache) >= N_PODS
            # every page ≤ 500 Pods: a few hundred KB here, a few MB at most with real Pods
            assert c.list_pages >= N_PODS // KubeClient.PAGE
            assert c.max_list_bytes < 2 << 20, c.max_list_bytes
            # slim projections only (not whole Pods) are kept
            p = lc.master.pods.get("ns-7", "p-7")
            assert p["spec"] == {"nodeName": "other-7"} and "annotations" not in p["metadata"]
            # a lookup goes through the index, with no GET
            gets = c.requests_by_verb.get("GET", 0)
            pod, target, err, cached = await lc.master._locate("ns-7", "p-7")   # noqa: SLF001
            assert cached == "index" and c.requests_by_verb.get("GET", 0) == gets
    asyncio.run(main())


def test_expired_continue_token_restarts_the_list():
    async def main():
        async with LocalCluster(start_master=False) as lc:
            c = lc.cluster
            _bulk(c, 1200)
            kube = KubeClient(lc.api_url)
            pages, restarts = [], 0
            async for page, rv in kube.list_pages("/api/v1/pods", "app=bulk", limit=500):
                if page is None:
                    restarts += 1
                    c.expire_continue = False       # the retry's tokens are fresh
                    pages = []
                    continue
                pages.append(len(page))
                if len(pages) == 1 and restarts == 0:
                    c.expire_continue = True        # compaction between page 1 and page 2
            assert restarts == 1 and pages == [500, 500, 200]
            items, _ = await kube.list_pods(None, "app=bulk", limit=500)
            assert len(items) == 1200 and len({p["metadata"]["name"] for p in items}) == 1200
            # a token that keeps expiring: the error reaches the caller after a few restarts
            c.expire_continue = True
            try:
                await kube.list_pods(None, "app=bulk", limit=500)
                raise AssertionError("expected 410")
            except ApiError as e:
                assert e.status == 410
            await kube.close()
    asyncio.run(main())


def test_no_code_path_accepts_a_whole_cluster_in_one_response():
    """The client's response bound is far below an unpaged cluster LIST (256 MiB in round 5)."""
    assert http1.MAX_BODY <= 32 << 20
    assert KubeClient.PAGE == 500
