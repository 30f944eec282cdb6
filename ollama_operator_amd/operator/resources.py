"""Object builders: the per-namespace model image store (PVC + StatefulSet + Service) and the
per-model Deployment + Service. Names, labels, ports, volumes, probes and owner references match
the reference (pkg/model/image_store.go:20-297, pkg/model/model.go:20-256, pkg/model/pod.go:10-83;
SURVEY.md §2.3). MI355X additions: `amd.com/gpu` requests (tensorParallelSize GPUs per replica),
a startupProbe so readiness is not floored at 15 s, and the new server image in place of
`ollama/ollama`.
"""
from __future__ import annotations

import os

from . import api

STORE_NAME = "ollama-models-store"
STORE_PVC = "ollama-models-store-pvc"
STORE_LABEL = {"app": STORE_NAME}
PORT = 11434
PORT_NAME = "ollama"
VOLUME = "image-storage"
MOUNT = "/root/.ollama"
STORE_SIZE = "100Gi"


def model_app_name(name: str) -> str:
    """reference pkg/model/model.go:20-22"""
    return f"ollama-model-{name}"


def server_image(model: dict | None = None) -> str:
    if model is not None and api.spec(model).get("serverImage"):
        return api.spec(model)["serverImage"]
    return os.environ.get("OMX_SERVER_IMAGE", api.DEFAULT_SERVER_IMAGE)


def owner_ref(obj: dict, controller: bool = True) -> dict:
    md = obj["metadata"]
    ref = {"apiVersion": obj["apiVersion"], "kind": obj["kind"], "name": md["name"], "uid": md.get("uid", ""),
           "blockOwnerDeletion": True}
    if controller:
        ref["controller"] = True
    return ref


def _probe(timeout: int, initial_delay: int, period: int | None = None) -> dict:
    p = {"httpGet": {"path": "/api/tags", "port": PORT_NAME}, "initialDelaySeconds": initial_delay,
         "successThreshold": 1, "failureThreshold": 2500, "timeoutSeconds": timeout}
    if period:
        p["periodSeconds"] = period
    return p


def server_container(read_only: bool, model: dict | None = None, gpus: int = 0) -> dict:
    """reference NewOllamaServerContainer (pkg/model/pod.go:14-66) + GPU resources + startupProbe."""
    env = [{"name": "OLLAMA_HOST", "value": "0.0.0.0"}]
    c: dict = {
        "name": "server",
        "image": server_image(model),
        "args": ["serve"],
        "env": env,
        "ports": [{"name": PORT_NAME, "protocol": "TCP", "containerPort": PORT}],
        "volumeMounts": [{"name": VOLUME, "mountPath": MOUNT, "readOnly": read_only}],
        # the server answers /api/tags as soon as it listens (models load lazily), so the startup
        # probe can poll every second instead of waiting a fixed 15 s twice
        "startupProbe": {"httpGet": {"path": "/api/tags", "port": PORT_NAME}, "periodSeconds": 1,
                         "failureThreshold": 600, "timeoutSeconds": 1},
        "readinessProbe": _probe(5, 0, 2),
        "livenessProbe": _probe(1, 0),
    }
    if model is not None:
        s = api.spec(model)
        if s.get("imagePullPolicy"):
            c["imagePullPolicy"] = s["imagePullPolicy"]
        if s.get("numCtx"):
            env.append({"name": "OLLAMA_CONTEXT_LENGTH", "value": str(s["numCtx"])})
        env.append({"name": "OLLAMA_KEEP_ALIVE", "value": str(s.get("keepAlive", "-1"))})
        env.append({"name": "OMX_PRELOAD", "value": s.get("image", "")})
        tp = api.tensor_parallel(model)
        if tp > 1:
            env.append({"name": "OMX_TP", "value": str(tp)})
        env.extend(s.get("env") or [])
        res = s.get("resources")
        if res:
            c["resources"] = res
        elif gpus:
            c["resources"] = {"limits": {api.GPU_RESOURCE: str(gpus)}, "requests": {api.GPU_RESOURCE: str(gpus)}}
    return c


def puller_container(image: str, namespace: str, model: dict | None = None) -> dict:
    """reference NewOllamaPullerContainer (pkg/model/pod.go:68-83)."""
    c = {"name": "ollama-image-pull", "image": server_image(model), "args": ["pull", image],
         "env": [{"name": "OLLAMA_HOST", "value": f"{STORE_NAME}.{namespace}"}]}
    if model is not None and api.spec(model).get("imagePullPolicy"):
        c["imagePullPolicy"] = api.spec(model)["imagePullPolicy"]
    return c


def store_pvc(namespace: str, model: dict) -> dict:
    """reference EnsureImageStorePVCCreated (image_store.go:41-94): 100Gi, RWX by default."""
    s = api.spec(model)
    access = (s.get("persistentVolume") or {}).get("accessMode") or "ReadWriteMany"
    pvc = {"apiVersion": "v1", "kind": "PersistentVolumeClaim",
           "metadata": {"name": STORE_PVC, "namespace": namespace, "labels": dict(STORE_LABEL)},
           "spec": {"accessModes": [access], "resources": {"requests": {"storage": STORE_SIZE}}}}
    if s.get("storageClassName"):
        pvc["spec"]["storageClassName"] = s["storageClassName"]
    return pvc


def store_claim_name(model: dict) -> str:
    """The reference accepts spec.persistentVolumeClaim but ignores it (image_store.go:46); here an
    existing claim, when given, backs the store."""
    pvc = api.spec(model).get("persistentVolumeClaim")
    return pvc["claimName"] if pvc and pvc.get("claimName") else STORE_PVC


def store_statefulset(namespace: str, model: dict) -> dict:
    """reference EnsureImageStoreStatefulSetCreated (image_store.go:126-197)."""
    return {
        "apiVersion": "apps/v1", "kind": "StatefulSet",
        "metadata": {"name": STORE_NAME, "namespace": namespace, "labels": dict(STORE_LABEL)},
        "spec": {
            "replicas": 1,
            "serviceName": STORE_NAME,
            "selector": {"matchLabels": dict(STORE_LABEL)},
            "template": {
                "metadata": {"labels": dict(STORE_LABEL)},
                "spec": {
                    "restartPolicy": "Always",
                    "containers": [server_container(False)],
                    "volumes": [{"name": VOLUME, "persistentVolumeClaim": {"claimName": store_claim_name(model)}}],
                },
            },
        },
    }


def store_service(namespace: str, sts: dict) -> dict:
    """reference EnsureImageStoreServiceCreated (image_store.go:239-297); owner -> StatefulSet."""
    return {"apiVersion": "v1", "kind": "Service",
            "metadata": {"name": STORE_NAME, "namespace": namespace, "labels": dict(STORE_LABEL),
                         "ownerReferences": [owner_ref(sts, controller=False)]},
            "spec": {"type": "ClusterIP", "selector": dict(STORE_LABEL),
                     "ports": [{"name": PORT_NAME, "protocol": "TCP", "port": PORT,
                                "targetPort": PORT_NAME}]}}


def model_deployment(namespace: str, model: dict) -> dict:
    """reference EnsureDeploymentCreated (model.go:39-115) + GPU resources; owner -> Model."""
    name = model["metadata"]["name"]
    app = model_app_name(name)
    labels = {"app": app}
    s = api.spec(model)
    pod_spec: dict = {
        "initContainers": [puller_container(s["image"], namespace, model)],
        "containers": [server_container(True, model, gpus=api.tensor_parallel(model))],
        "volumes": [{"name": VOLUME, "persistentVolumeClaim": {"claimName": store_claim_name(model),
                                                               "readOnly": True}}],
    }
    if s.get("imagePullSecrets"):
        pod_spec["imagePullSecrets"] = s["imagePullSecrets"]
    if s.get("nodeSelector"):
        pod_spec["nodeSelector"] = s["nodeSelector"]
    if s.get("tolerations"):
        pod_spec["tolerations"] = s["tolerations"]
    return {
        "apiVersion": "apps/v1", "kind": "Deployment",
        "metadata": {"name": app, "namespace": namespace, "labels": dict(labels),
                     "ownerReferences": [owner_ref(model)]},
        "spec": {"replicas": api.replicas(model), "selector": {"matchLabels": dict(labels)},
                 "template": {"metadata": {"labels": dict(labels)}, "spec": pod_spec}},
    }


def model_service(namespace: str, name: str, deployment: dict) -> dict:
    """reference EnsureServiceCreated (model.go:203-256); owner -> Deployment."""
    app = model_app_name(name)
    return {"apiVersion": "v1", "kind": "Service",
            "metadata": {"name": app, "namespace": namespace, "labels": {"app": app},
                         "ownerReferences": [owner_ref(deployment, controller=False)]},
            "spec": {"type": "ClusterIP", "selector": {"app": app},
                     "ports": [{"name": PORT_NAME, "protocol": "TCP", "port": PORT, "targetPort": PORT_NAME}]}}


def template_fingerprint(dep: dict) -> tuple:
    """What a spec change must roll out (the reference only reconciles replicas, model.go:149-186)."""
    ps = dep["spec"]["template"]["spec"]
    c = ps["containers"][0]
    init = ps["initContainers"][0]
    return (c.get("image"), tuple(init.get("args", [])), repr(c.get("resources")), repr(c.get("env")),
            repr(ps.get("imagePullSecrets")), repr(ps.get("nodeSelector")), repr(ps.get("tolerations")),
            c.get("imagePullPolicy"))
