"""Process-level CRD-apply -> Available end-to-end on CPU (ollama_operator_amd/operator/e2e.py):
the production controller against the fake apiserver, with a process kubelet that runs the pods'
real programs -- `ollama serve` for the store StatefulSet, the `ollama pull` init container through
the store Service from a local OCI registry mirror, then `ollama serve` for the model Deployment,
readiness by the pod templates' own probes. Asserts the reference's event sequence and that the
ready model server answers /api/generate (the SURVEY.md §4 e2e gap: the reference's e2e never
creates a Model)."""
import json
import os
import threading
import time
import urllib.request

import uvicorn

from ollama_operator_amd.operator.e2e import apply_to_ready, free_port, http_ok
from ollama_operator_amd.server.registry_server import create_registry_app
from ollama_operator_amd.server.store import ModelStore


def test_apply_to_available_with_real_processes(tmp_path, tiny_models):
    reg = ModelStore(str(tmp_path / "registry"))
    reg.create("library/tiny:latest", gguf_path=tiny_models["tiny-llama"], template="{{ .Prompt }}",
               params={"temperature": 0.0})
    port = free_port()
    srv = uvicorn.Server(uvicorn.Config(create_registry_app(reg.root), host="127.0.0.1", port=port,
                                        log_level="error"))
    threading.Thread(target=srv.run, daemon=True).start()
    while not http_ok(f"http://127.0.0.1:{port}/v2/"):
        time.sleep(0.05)
    model = {"apiVersion": "ollama.ayaka.io/v1", "kind": "Model",
             "metadata": {"name": "tiny", "namespace": "default"}, "spec": {"image": "tiny"}}
    env = {"OMX_REGISTRY_MIRROR": f"http://127.0.0.1:{port}", "CUDA_VISIBLE_DEVICES": "",
           "HIP_VISIBLE_DEVICES": ""}
    captured = {}

    import ollama_operator_amd.operator.e2e as e2e
    orig = e2e.ProcessKubelet.shutdown

    def check_then_shutdown(self):  # query the model server before the kubelet stops it
        url = self.svc_port.get("ollama-model-tiny.default")
        body = json.dumps({"model": "tiny", "prompt": "hello", "stream": False,
                           "options": {"num_predict": 4}}).encode()
        req = urllib.request.Request(f"http://127.0.0.1:{url}/api/generate", data=body,
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=120) as r:
            captured["gen"] = json.loads(r.read())
        orig(self)

    e2e.ProcessKubelet.shutdown = check_then_shutdown
    try:
        res = apply_to_ready(model, str(tmp_path / "pv"), env, timeout=300)
    finally:
        e2e.ProcessKubelet.shutdown = orig
        srv.should_exit = True
    assert res["apply_to_ready_s"] < 120
    ev = res["events"]
    for reason in ("ModelProgressing", "ProvisionedImageStoragePVC", "ProvisionedImageStoreStatefulSet",
                   "ProvisionedImageStoreService", "DeploymentCreated", "ServiceCreated", "ModelAvailable"):
        assert reason in ev, (reason, ev)
    assert ev.count("WaitingForImageStoreStatefulSet") < 20  # no hot reconcile loop
    ph = res["phases_s"]
    assert ph["store_ready"] <= ph["model_scheduled"] <= ph["model_init_done"] <= ph["model_ready"]
    assert os.path.exists(tmp_path / "pv" / "default" / "ollama-models-store-pvc" / "models" / "manifests")
    assert captured["gen"]["done"] and captured["gen"]["eval_count"] >= 1
