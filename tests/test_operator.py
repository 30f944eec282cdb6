"""Operator: reconcile state machine, object contract, events, scaling, rollout,
GC, shared store, work queue, leader election -- against the in-memory fake apiserver."""
import time

import pytest

from ollama_operator_amd.operator import api, resources as R
from ollama_operator_amd.operator.controller import Manager, WorkQueue
from ollama_operator_amd.operator.fake import FakeKube
from ollama_operator_amd.operator.kube import ApiError
from ollama_operator_amd.operator.reconciler import ModelReconciler

NS = "default"


def model(name="phi", image="phi", **spec):
    return {"apiVersion": api.API_VERSION, "kind": "Model", "metadata": {"name": name, "namespace": NS},
            "spec": {"image": image, **spec}}


def drive(k, rec, name="phi", max_steps=30, tick=True):
    stages = []
    for _ in range(max_steps):
        r = rec.reconcile(NS, name)
        stages.append(r.stage)
        if r.requeue_after is None:
            return stages
        if tick:
            k.tick()
    raise AssertionError(f"did not converge: {stages}")


def test_full_flow_objects_and_events():
    k = FakeKube()
    k.create("Model", NS, model())
    rec = ModelReconciler(k)
    stages = drive(k, rec)
    assert stages[0] == "progressing" and stages[-1] == "available"
    m = k.get("Model", NS, "phi")
    assert api.conditions(m)[0]["type"] == "Available" and len(api.conditions(m)) == 1
    assert m["status"]["readyReplicas"] == 1 and m["status"]["replicas"] == 1
    # --- store objects (reference image_store.go)
    pvc = k.get("PersistentVolumeClaim", NS, "ollama-models-store-pvc")
    assert pvc["spec"]["accessModes"] == ["ReadWriteMany"]
    assert pvc["spec"]["resources"]["requests"]["storage"] == "100Gi"
    assert "ownerReferences" not in pvc["metadata"]
    sts = k.get("StatefulSet", NS, "ollama-models-store")
    assert sts["spec"]["replicas"] == 1 and sts["metadata"]["labels"] == {"app": "ollama-models-store"}
    c = sts["spec"]["template"]["spec"]["containers"][0]
    assert c["name"] == "server" and c["args"] == ["serve"]
    assert c["env"][0] == {"name": "OLLAMA_HOST", "value": "0.0.0.0"}
    assert c["volumeMounts"][0] == {"name": "image-storage", "mountPath": "/root/.ollama", "readOnly": False}
    assert c["readinessProbe"]["httpGet"] == {"path": "/api/tags", "port": "ollama"}
    assert c["livenessProbe"]["failureThreshold"] == 2500
    ssvc = k.get("Service", NS, "ollama-models-store")
    assert ssvc["spec"]["ports"][0]["port"] == 11434 and ssvc["spec"]["ports"][0]["name"] == "ollama"
    assert ssvc["metadata"]["ownerReferences"][0]["kind"] == "StatefulSet"
    # --- model objects (reference model.go / pod.go)
    dep = k.get("Deployment", NS, "ollama-model-phi")
    assert dep["metadata"]["labels"] == {"app": "ollama-model-phi"}
    ref = dep["metadata"]["ownerReferences"][0]
    assert ref["kind"] == "Model" and ref["name"] == "phi" and ref["blockOwnerDeletion"] is True
    ps = dep["spec"]["template"]["spec"]
    init = ps["initContainers"][0]
    assert init["name"] == "ollama-image-pull" and init["args"] == ["pull", "phi"]
    assert init["env"] == [{"name": "OLLAMA_HOST", "value": "ollama-models-store.default"}]
    srv = ps["containers"][0]
    assert srv["volumeMounts"][0]["readOnly"] is True
    assert srv["resources"]["limits"]["amd.com/gpu"] == "1"
    assert ps["volumes"][0]["persistentVolumeClaim"] == {"claimName": "ollama-models-store-pvc", "readOnly": True}
    msvc = k.get("Service", NS, "ollama-model-phi")
    assert msvc["spec"]["selector"] == {"app": "ollama-model-phi"}
    assert msvc["metadata"]["ownerReferences"][0]["kind"] == "Deployment"
    ev = k.event_reasons("phi")
    order = ["ModelProgressing", "ProvisionedImageStoragePVC", "ProvisionedImageStoreStatefulSet",
             "ProvisionedImageStoreService", "DeploymentCreated", "ServiceCreated", "ModelAvailable"]
    idx = [ev.index(r) for r in order]
    assert idx == sorted(idx), ev


def test_scale_rollout_and_readiness_loss():
    k = FakeKube()
    k.create("Model", NS, model())
    rec = ModelReconciler(k)
    drive(k, rec)
    m = k.get("Model", NS, "phi")
    m["spec"]["replicas"] = 3
    k.update("Model", NS, m)
    stages = drive(k, rec)
    assert "updated" in stages
    assert k.get("Deployment", NS, "ollama-model-phi")["spec"]["replicas"] == 3
    assert k.get("Model", NS, "phi")["status"]["readyReplicas"] == 3
    assert "ModelScaled" in k.event_reasons("phi")
    # image change rolls out (the reference never updates the pod template)
    m = k.get("Model", NS, "phi")
    m["spec"]["image"] = "llama2:7b"
    k.update("Model", NS, m)
    drive(k, rec)
    dep = k.get("Deployment", NS, "ollama-model-phi")
    assert dep["spec"]["template"]["spec"]["initContainers"][0]["args"] == ["pull", "llama2:7b"]
    assert "ModelUpdated" in k.event_reasons("phi")
    # pods die: the Model goes back to Progressing until ready again
    d = k.get("Deployment", NS, "ollama-model-phi")
    d["status"]["readyReplicas"] = 1
    k.objs[("Deployment", NS, "ollama-model-phi")]["status"] = d["status"]
    r = rec.reconcile(NS, "phi")
    assert r.stage == "wait-deployment"
    assert api.conditions(k.get("Model", NS, "phi"))[0]["type"] == "Progressing"
    drive(k, rec)
    assert api.conditions(k.get("Model", NS, "phi"))[0]["type"] == "Available"


def test_shared_store_and_gc():
    k = FakeKube()
    k.create("Model", NS, model("a", "phi"))
    k.create("Model", NS, model("b", "llama2"))
    rec = ModelReconciler(k)
    drive(k, rec, "a")
    drive(k, rec, "b")
    assert sum(1 for v, kind, n in k.log if v == "create" and kind == "StatefulSet") == 1
    k.delete("Model", NS, "a")
    assert k.get("Deployment", NS, "ollama-model-a") is None
    assert k.get("Service", NS, "ollama-model-a") is None
    assert k.get("StatefulSet", NS, "ollama-models-store") is not None  # cache persists
    assert k.get("Deployment", NS, "ollama-model-b") is not None
    assert rec.reconcile(NS, "a").stage == "deleted"


def test_existing_pvc_tp_and_placement():
    k = FakeKube()
    k.create("Model", NS, model(persistentVolumeClaim={"claimName": "my-models"}, tensorParallelSize=8,
                                nodeSelector={"amd.com/gpu.product": "MI355X"}, numCtx=8192,
                                persistentVolume={"accessMode": "ReadWriteOnce"}))
    rec = ModelReconciler(k)
    drive(k, rec)
    assert k.get("PersistentVolumeClaim", NS, "ollama-models-store-pvc") is None
    sts = k.get("StatefulSet", NS, "ollama-models-store")
    assert sts["spec"]["template"]["spec"]["volumes"][0]["persistentVolumeClaim"]["claimName"] == "my-models"
    ps = k.get("Deployment", NS, "ollama-model-phi")["spec"]["template"]["spec"]
    assert ps["containers"][0]["resources"]["limits"]["amd.com/gpu"] == "8"
    env = {e["name"]: e["value"] for e in ps["containers"][0]["env"]}
    assert env["OMX_TP"] == "8" and env["OLLAMA_CONTEXT_LENGTH"] == "8192"
    assert ps["nodeSelector"] == {"amd.com/gpu.product": "MI355X"}


def test_validation():
    k = FakeKube()
    with pytest.raises(ApiError):
        k.create("Model", NS, model(image=""))
    with pytest.raises(ApiError):
        k.create("Model", NS, model(tensorParallelSize=16))


def test_workqueue_dedupe_delay_backoff():
    q = WorkQueue()
    q.add("a")
    q.add("a")
    q.add("b", delay=0.2)
    assert q.get(0.05) == "a"
    assert q.get(0.05) is None  # 'a' deduplicated, 'b' not due yet
    q.done("a")
    assert q.get(0.5) == "b"
    q.done("b")
    q.add_rate_limited("c")
    q.add_rate_limited("c")
    assert q.get(1.0) == "c"


def test_workqueue_requeue_after_during_processing_is_a_timer():
    """RequeueAfter issued while the key is being processed must wait its delay (regression: it
    used to mark the key dirty, so done() re-queued it at once -- a hot reconcile loop that the
    process-level apply->ready e2e exposed as thousands of Waiting* events)."""
    q = WorkQueue()
    q.add("m")
    assert q.get(0.05) == "m"
    q.add("m", delay=0.3)  # what process_one does with Result.requeue_after
    q.done("m")
    assert q.get(0.1) is None
    assert q.get(0.5) == "m"
    q.done("m")
    # an event during processing still triggers an immediate re-run
    q.add("m")
    assert q.get(0.05) == "m"
    q.add("m")
    q.done("m")
    assert q.get(0.05) == "m"


def test_manager_event_driven():
    k = FakeKube()
    mgr = Manager(k, poll_s=600)
    mgr.start(watch=True)
    try:
        k.create("Model", NS, model())
        deadline = time.time() + 20
        while time.time() < deadline:
            k.tick()
            m = k.get("Model", NS, "phi")
            if api.has_condition(m, api.COND_AVAILABLE):
                break
            time.sleep(0.05)
        assert api.has_condition(k.get("Model", NS, "phi"), api.COND_AVAILABLE)
    finally:
        mgr.shutdown()


def test_leader_election_single_leader():
    k = FakeKube()
    a = Manager(k, leader_elect=True, lease_namespace="ollama-operator-system", identity="a")
    b = Manager(k, leader_elect=True, lease_namespace="ollama-operator-system", identity="b")
    a.start(watch=False)
    time.sleep(0.3)
    b.start(watch=False)
    time.sleep(0.5)
    try:
        assert a.is_leader and not b.is_leader
        lease = k.get("Lease", "ollama-operator-system", "300b498d.ayaka.io")
        assert lease["spec"]["holderIdentity"] == "a"
    finally:
        a.shutdown()
        b.shutdown()


def test_crd_schema_contract():
    c = api.crd()
    v = c["spec"]["versions"][0]
    assert c["metadata"]["name"] == "models.ollama.ayaka.io"
    assert [p["jsonPath"] for p in v["additionalPrinterColumns"]] == [".spec.image", ".status.conditions[0].type"]
    assert v["subresources"] == {"status": {}}
    props = v["schema"]["openAPIV3Schema"]["properties"]["spec"]
    assert props["required"] == ["image"]
    for f in ("replicas", "image", "imagePullPolicy", "imagePullSecrets", "storageClassName",
              "persistentVolumeClaim", "persistentVolume"):
        assert f in props["properties"]
    assert props["properties"]["persistentVolumeClaim"]["required"] == ["claimName"]
    assert R.model_app_name("x") == "ollama-model-x"


def test_secure_metrics_tokenreview_and_sar():
    """--metrics-secure: TLS + TokenReview + SubjectAccessReview (kube-rbac-proxy semantics)."""
    import shutil
    import ssl
    import urllib.error
    import urllib.request

    import pytest
    if shutil.which("openssl") is None:
        pytest.skip("openssl not available")
    from ollama_operator_amd.operator.controller import Manager, serve_probes
    from ollama_operator_amd.operator.e2e import free_port
    k = FakeKube()
    k.tokens = {"good": "system:serviceaccount:monitoring:prometheus", "nobody": "alice"}
    k.metrics_readers = {"system:serviceaccount:monitoring:prometheus"}
    mgr = Manager(k)
    port = free_port()
    servers = serve_probes(mgr, "0", f"127.0.0.1:{port}", secure=True)
    ctx = ssl.create_default_context()
    ctx.check_hostname = False
    ctx.verify_mode = ssl.CERT_NONE

    def get(token):
        req = urllib.request.Request(f"https://127.0.0.1:{port}/metrics")
        if token:
            req.add_header("Authorization", f"Bearer {token}")
        try:
            with urllib.request.urlopen(req, context=ctx, timeout=10) as r:
                return r.status, r.read()
        except urllib.error.HTTPError as e:
            return e.code, b""
    import socket
    try:
        # a client that connects and never sends a ClientHello must not block the endpoint (the TLS
        # handshake runs in the per-connection thread)
        idle = socket.create_connection(("127.0.0.1", port))
        assert get(None)[0] == 401
        assert get("forged")[0] == 401
        assert get("nobody")[0] == 403
        code, body = get("good")
        assert code == 200 and b"controller_runtime_reconcile_total" in body
        idle.close()
    finally:
        for s in servers:
            s.shutdown()


def test_metrics_auth_cache_bounded_and_hashed():
    from ollama_operator_amd.operator.controller import MetricsAuth
    k = FakeKube()
    k.tokens = {"good": "system:serviceaccount:monitoring:prometheus"}
    k.metrics_readers = {"system:serviceaccount:monitoring:prometheus"}
    a = MetricsAuth(k)
    a.MAX_ENTRIES = 8
    a.REVIEWS_PER_S = 1e9  # no rate limit for the size check
    a._bucket = 1e9
    for i in range(50):
        assert a.check(f"Bearer random{i}") == 401
    assert len(a._cache) <= 8
    assert all("random" not in key for key in a._cache)  # digests, not raw tokens
    assert a.check("Bearer good") == 200
    b = MetricsAuth(k)
    b.REVIEWS_PER_S = 2.0
    b._bucket = 2.0
    calls = [b.check(f"Bearer flood{i}") for i in range(10)]
    assert calls.count(401) == 10
    assert len(b._cache) <= 3  # at most the bucket's reviews were made (and cached)


def test_sigterm_drains_and_releases_lease():
    """SIGTERM (reference ctrl.SetupSignalHandler, cmd/main.go:146): the leader stops, finishes its
    work and releases the Lease so a standby takes over without waiting out the lease duration."""
    import os
    import signal
    import threading

    from ollama_operator_amd.operator.controller import Manager, run_until_signal
    k = FakeKube()
    a = Manager(k, leader_elect=True, lease_namespace="ollama-operator-system", identity="a")
    a.start(watch=False)
    for _ in range(100):
        if a.is_leader:
            break
        time.sleep(0.05)
    assert a.is_leader
    threading.Timer(0.3, os.kill, (os.getpid(), signal.SIGTERM)).start()
    run_until_signal(a)  # returns after the graceful shutdown
    lease = k.get("Lease", "ollama-operator-system", "300b498d.ayaka.io")
    assert lease["spec"]["holderIdentity"] == "" and not a.is_leader
    assert all(not t.is_alive() for t in a.threads)
    b = Manager(k, leader_elect=True, lease_namespace="ollama-operator-system", identity="b")
    b.start(watch=False)
    for _ in range(100):
        if b.is_leader:
            break
        time.sleep(0.05)
    assert b.is_leader  # immediate takeover, no 15 s lease wait
    b.shutdown()
