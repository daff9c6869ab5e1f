"""Per-tenant authorization on the master (authz_mode=kube): TokenReview + SubjectAccessReview
on the virtual subresource pods/gpumount. The reference authorizes nobody (SURVEY defect 13)."""
import asyncio

from gpumounter_amd.fakes.harness import LocalCluster


def run(body, self_review=True):
    async def main():
        async with LocalCluster(master_overrides={"authz_mode": "kube",
                                                  "authz_self_review": self_review}) as lc:
            c = lc.cluster
            c.add_user("tok-alice", "alice", groups=["team-a"])
            c.add_user("tok-bob", "bob")
            c.add_user("tok-ops", "ops", groups=["gpu-admins"])
            c.grant("group:team-a", ["create", "delete", "get"], namespaces=["team-a"])
            c.grant("group:gpu-admins", ["create", "delete", "get"])            # all namespaces
            c.grant("group:gpu-admins", ["get"], resource="nodes/gpumount")
            return await body(lc)
    return asyncio.run(main())


def test_kube_mode_authorizes_per_namespace_and_verb():
    async def body(lc):
        lc.tenant("a1", ns="team-a")
        lc.tenant("d1", ns="default")
        assert (await lc.add("team-a", "a1", 1))[0] == 401                      # no token
        assert (await lc.add("team-a", "a1", 1, token="nope"))[0] == 401          # unknown token
        code, b = await lc.add("default", "d1", 1, token="tok-alice")
        assert code == 403 and "alice cannot create pods/gpumount in namespace default" \
            in b["message"]
        assert (await lc.add("team-a", "a1", 1, token="tok-bob"))[0] == 403       # no rights
        code, b = await lc.add("team-a", "a1", 2, token="tok-alice")
        assert code == 200 and len(b["devices"]) == 2
        u = [d["uuid"] for d in b["devices"]]
        assert (await lc.remove("team-a", "a1", u, token="tok-bob"))[0] == 403
        assert (await lc.remove("team-a", "a1", u, token="tok-alice"))[0] == 200
        assert (await lc.add("default", "d1", 1, token="tok-ops"))[0] == 200      # cluster-wide
        # read routes are authorized too
        async with lc.session.get(f"{lc.master_url}/api/v1/nodes/node-0/gpus",
                                  headers={"Authorization": "Bearer tok-alice"}) as r:
            assert r.status == 403
        async with lc.session.get(f"{lc.master_url}/api/v1/nodes/node-0/gpus",
                                  headers={"Authorization": "Bearer tok-ops"}) as r:
            assert r.status == 200
    run(body)


def test_reviews_are_cached():
    async def body(lc):
        lc.tenant("a1", ns="team-a")
        authz = lc.master.authz
        for _ in range(3):
            code, b = await lc.add("team-a", "a1", 1, token="tok-alice")
            assert code == 200
            assert (await lc.remove("team-a", "a1", [b["devices"][0]["uuid"]],
                                    token="tok-alice"))[0] == 200
        # per (user, verb, ns, pod): the first (create) answered by the self-review that went
        # out with the TokenReview, the delete by a SubjectAccessReview
        assert (authz.reviews["token"], authz.reviews["self"], authz.reviews["sar"]) == (1, 1, 1)
    run(body)


def test_a_new_token_is_reviewed_as_itself_in_one_round_trip():
    """First sight of a token: TokenReview ∥ SelfSubjectAccessReview sent with that token (the
    apiserver answers for whoever it authenticates as); where the self-review is not served the
    SubjectAccessReview follows the TokenReview, with the same decisions."""
    async def body(lc):
        lc.tenant("a1", ns="team-a")
        lc.tenant("d1", ns="default")
        authz, c = lc.master.authz, lc.cluster
        kube = authz.kube
        spans = []
        real_tr, real_ssar = kube.token_review, kube.self_subject_access_review

        async def tr(token):
            t0 = asyncio.get_running_loop().time()
            out = await real_tr(token)
            spans.append(("tr", t0, asyncio.get_running_loop().time()))
            return out

        async def ssar(token, attrs):
            t0 = asyncio.get_running_loop().time()
            out = await real_ssar(token, attrs)
            spans.append(("ssar", t0, asyncio.get_running_loop().time()))
            return out
        kube.token_review, kube.self_subject_access_review = tr, ssar
        code, b = await lc.add("team-a", "a1", 1, token="tok-alice")
        assert code == 200 and c.ssar_count == 1 and c.sar_count == 0
        (t_tr,), (t_own,) = [x for x in spans if x[0] == "tr"], [x for x in spans if x[0] == "ssar"]
        assert t_own[1] < t_tr[2]                          # sent before the TokenReview answered
        code, b2 = await lc.add("default", "d1", 1, token="tok-bob")
        assert code == 403 and "bob cannot create" in b2["message"] and c.ssar_count == 2
        assert (await lc.add("team-a", "a1", 1, token="nope"))[0] == 401
        # an apiserver without the self-review API: TokenReview, then SubjectAccessReview
        c.serve_self_review = False
        assert (await lc.add("default", "d1", 1, token="tok-ops"))[0] == 200
        c.add_user("tok-carol", "carol")
        code, b3 = await lc.add("team-a", "a1", 1, token="tok-carol")
        assert code == 403 and "carol cannot create" in b3["message"]
        assert c.sar_count == 2 and authz.reviews["self"] == 5
    run(body)


def test_no_self_review_when_the_master_authenticates_by_certificate():
    """With a TLS client certificate the apiserver would review the master itself, not the
    caller: the master then asks SubjectAccessReviews only."""
    from gpumounter_amd.master.authz import Authorizer

    class Cfg:
        authz_mode, api_token, authz_self_review = "kube", "", True

    class Kube:
        bearer_only = False
    assert not Authorizer(Cfg(), Kube()).self_review
    Kube.bearer_only = True
    assert Authorizer(Cfg(), Kube()).self_review
    Cfg.authz_self_review = False
    assert not Authorizer(Cfg(), Kube()).self_review


def test_batch_checks_every_operation():
    async def body(lc):
        lc.tenant("a1", ns="team-a")
        lc.tenant("d1", ns="default")
        async with lc.session.post(f"{lc.master_url}/api/v1/batch", json={"operations": [
                {"op": "add", "namespace": "team-a", "pod": "a1", "gpus": 1},
                {"op": "add", "namespace": "default", "pod": "d1", "gpus": 1}]},
                headers={"Authorization": "Bearer tok-alice"}) as r:
            res = (await r.json())["results"]
        assert [x["code"] for x in res] == [200, 403]
    run(body)


def test_events_record_who_asked():
    """The caller's identity travels master → worker (requested_by) into the tenant's Events."""
    async def body(lc):
        lc.tenant("a1", ns="team-a")
        code, b = await lc.add("team-a", "a1", 1, token="tok-alice")
        assert code == 200
        code, _ = await lc.remove("team-a", "a1", [b["devices"][0]["uuid"]], token="tok-ops")
        assert code == 200
        await lc.nodes["node-0"].worker.service.notify.drain()
        msgs = {e["reason"]: e["message"] for e in lc.cluster.events_for("team-a", "a1")}
        assert msgs["GPUAttached"].endswith("(requested by alice)")
        assert msgs["GPUDetached"].endswith("(requested by ops)")
    run(body)


def test_anonymous_callers_are_recorded_by_address():
    async def main():
        async with LocalCluster() as lc:
            lc.tenant("t")
            assert (await lc.add("default", "t", 1))[0] == 200
            await lc.nodes["node-0"].worker.service.notify.drain()
            (ev,) = lc.cluster.events_for("default", "t")
            assert "(requested by anonymous@127.0.0.1)" in ev["message"]
    asyncio.run(main())


def test_an_expired_token_is_reviewed_together_with_its_sar():
    """Past the TTLs, a known token's TokenReview and SubjectAccessReview go out together (one
    apiserver round trip, not two); the SAR answer counts only for the identity the TokenReview
    confirms — a token that now maps to another user is authorized afresh."""
    async def body(lc):
        lc.tenant("a1", ns="team-a")
        authz = lc.master.authz
        authz.token_ttl_s = authz.sar_ttl_s = 0.05
        kube = authz.kube
        spans = []
        real_tr, real_sar = kube.token_review, kube.subject_access_review

        async def tr(token):
            t0 = asyncio.get_running_loop().time()
            out = await real_tr(token)
            spans.append(("tr", t0, asyncio.get_running_loop().time()))
            return out

        async def sar(user, attrs):
            t0 = asyncio.get_running_loop().time()
            out = await real_sar(user, attrs)
            spans.append(("sar", t0, asyncio.get_running_loop().time()))
            return out
        kube.token_review, kube.subject_access_review = tr, sar
        authz.self_review = False        # first sight as on an apiserver without the API
        code, b = await lc.add("team-a", "a1", 1, token="tok-alice")
        assert code == 200
        first = list(spans)
        assert [k for k, *_ in first] == ["tr", "sar"] and first[1][1] >= first[0][2]  # serial
        spans.clear()
        await asyncio.sleep(0.1)                          # both answers expired
        code, _ = await lc.remove("team-a", "a1", [b["devices"][0]["uuid"]], token="tok-alice")
        assert code == 200 and authz.reviews["speculative"] == 1
        (t_tr,) = [x for x in spans if x[0] == "tr"]
        (t_sar,) = [x for x in spans if x[0] == "sar"]
        assert t_sar[1] < t_tr[2]                         # the SAR left before the TR answered
        # the token now belongs to bob, who may not attach in team-a: the guessed SAR (alice)
        # must not decide
        lc.cluster.add_user("tok-alice", "bob")
        await asyncio.sleep(0.1)
        code, b2 = await lc.add("team-a", "a1", 1, token="tok-alice")
        assert code == 403 and "bob cannot create" in b2["message"], b2
    run(body)


def test_a_decision_used_late_in_its_life_is_refreshed_in_the_background():
    async def body(lc):
        lc.tenant("a1", ns="team-a")
        authz = lc.master.authz
        authz.token_ttl_s = authz.sar_ttl_s = 0.4
        code, b = await lc.add("team-a", "a1", 1, token="tok-alice")
        assert code == 200
        await asyncio.sleep(0.25)                         # past half the lifetime
        code, _ = await lc.remove("team-a", "a1", [b["devices"][0]["uuid"]], token="tok-alice")
        assert code == 200
        await asyncio.sleep(0.05)
        assert authz.reviews["refresh"] >= 1
        await asyncio.sleep(0.2)                          # the original answer has expired ...
        code, _ = await lc.add("team-a", "a1", 1, token="tok-alice")
        assert code == 200 and authz.reviews["speculative"] == 0   # ... but was renewed
    run(body)
