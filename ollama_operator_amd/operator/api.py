"""`ollama.ayaka.io/v1` `Model` API: group/version/kind, spec defaults, conditions and the CRD
OpenAPI schema. Field names and semantics match the reference (api/v1/model_types.go:24-166,
config/crd/bases/ollama.ayaka.io_models.yaml); fields marked ADDITIVE are new, optional and
backward compatible: clusters running the reference can apply the same YAML.
"""
from __future__ import annotations

import copy
from typing import Any

GROUP = "ollama.ayaka.io"
VERSION = "v1"
API_VERSION = f"{GROUP}/{VERSION}"
KIND = "Model"
PLURAL = "models"

# condition types (reference api/v1/model_types.go:84-97)
COND_UNKNOWN = "ModelUnknown"
COND_AVAILABLE = "Available"
COND_PROGRESSING = "Progressing"
COND_REPLICA_FAILURE = "ReplicaFailure"

DEFAULT_SERVER_IMAGE = "ollama-operator-amd/server:latest"
GPU_RESOURCE = "amd.com/gpu"


def spec(model: dict) -> dict:
    return model.get("spec") or {}


def replicas(model: dict) -> int:
    r = spec(model).get("replicas")
    return 1 if r is None else int(r)


def tensor_parallel(model: dict) -> int:
    return int(spec(model).get("tensorParallelSize") or 1)


def conditions(model: dict) -> list[dict]:
    return list((model.get("status") or {}).get("conditions") or [])


def has_condition(model: dict, ctype: str) -> bool:
    return any(c.get("type") == ctype for c in conditions(model))


_STR = {"type": "string"}
_INT32 = {"type": "integer", "format": "int32"}


def _resources_schema() -> dict:
    q = {"anyOf": [{"type": "integer"}, {"type": "string"}], "x-kubernetes-int-or-string": True,
         "pattern": r"^(\+|-)?(([0-9]+(\.[0-9]*)?)|(\.[0-9]+))(([KMGTPE]i)|[numkMGTPE]|([eE](\+|-)?(([0-9]+(\.[0-9]*)?)|(\.[0-9]+))))?$"}
    return {"type": "object", "description": "ADDITIVE. Compute resources of each model pod (default: "
            f"{GPU_RESOURCE}: tensorParallelSize).",
            "properties": {"limits": {"type": "object", "additionalProperties": q},
                           "requests": {"type": "object", "additionalProperties": q}}}


def crd() -> dict:
    spec_props: dict[str, Any] = {
        "replicas": {**_INT32, "description": "Number of desired pods (data-parallel serving replicas). Defaults to 1."},
        "image": {**_STR, "description": "Model image to pull from the registry, e.g. `phi` or `llama2:7b`."},
        "imagePullPolicy": {**_STR, "description": "Image pull policy of the server containers."},
        "imagePullSecrets": {"type": "array", "items": {"type": "object", "properties": {"name": _STR},
                                                        "x-kubernetes-map-type": "atomic"},
                             "description": "Secrets for pulling the server image."},
        "storageClassName": {**_STR, "description": "StorageClass of the shared model-store PVC."},
        "persistentVolumeClaim": {"type": "object", "required": ["claimName"],
                                  "properties": {"claimName": _STR, "readOnly": {"type": "boolean"}},
                                  "description": "Use an existing PVC as the model store."},
        "persistentVolume": {"type": "object", "properties": {"accessMode": _STR},
                             "description": "Access mode of the model-store PVC (default ReadWriteMany)."},
        # ---- ADDITIVE fields
        "serverImage": {**_STR, "description": "ADDITIVE. Server container image (default: the operator's "
                                                "OMX_SERVER_IMAGE)."},
        "tensorParallelSize": {**_INT32, "minimum": 1, "maximum": 8,
                               "description": "ADDITIVE. GPUs per replica for tensor parallelism over xGMI."},
        "resources": _resources_schema(),
        "numCtx": {**_INT32, "description": "ADDITIVE. Context length (OLLAMA_CONTEXT_LENGTH)."},
        "keepAlive": {**_STR, "description": "ADDITIVE. Keep-alive of the loaded model (default: forever)."},
        "env": {"type": "array", "items": {"type": "object", "x-kubernetes-preserve-unknown-fields": True},
                "description": "ADDITIVE. Extra environment for the server container."},
        "nodeSelector": {"type": "object", "additionalProperties": _STR, "description": "ADDITIVE."},
        "tolerations": {"type": "array", "items": {"type": "object", "x-kubernetes-preserve-unknown-fields": True},
                        "description": "ADDITIVE."},
    }
    cond = {"type": "object", "required": ["status", "type"], "properties": {
        "lastTransitionTime": {"type": "string", "format": "date-time"},
        "lastUpdateTime": {"type": "string", "format": "date-time"},
        "message": _STR, "reason": _STR, "status": _STR, "type": _STR}}
    status_props = {"replicas": _INT32, "readyReplicas": _INT32, "availableReplicas": _INT32,
                    "unavailableReplicas": _INT32, "conditions": {"type": "array", "items": cond}}
    return {
        "apiVersion": "apiextensions.k8s.io/v1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{PLURAL}.{GROUP}"},
        "spec": {
            "group": GROUP,
            "names": {"kind": KIND, "listKind": "ModelList", "plural": PLURAL, "singular": "model"},
            "scope": "Namespaced",
            "versions": [{
                "name": VERSION, "served": True, "storage": True,
                "additionalPrinterColumns": [
                    {"jsonPath": ".spec.image", "name": "Model", "type": "string"},
                    {"jsonPath": ".status.conditions[0].type", "name": "Status", "type": "string"}],
                "schema": {"openAPIV3Schema": {
                    "description": "Model is the Schema for the models API", "type": "object",
                    "properties": {"apiVersion": _STR, "kind": _STR, "metadata": {"type": "object"},
                                   "spec": {"type": "object", "required": ["image"], "properties": spec_props},
                                   "status": {"type": "object", "properties": status_props}}}},
                "subresources": {"status": {}},
            }],
        },
    }


def validate(model: dict) -> list[str]:
    """Server-side-like validation for the fake apiserver and the admission path."""
    errs = []
    s = spec(model)
    if not s.get("image"):
        errs.append("spec.image: Required value")
    r = s.get("replicas")
    if r is not None and (not isinstance(r, int) or r < 0):
        errs.append("spec.replicas: must be a non-negative integer")
    pvc = s.get("persistentVolumeClaim")
    if pvc is not None and not pvc.get("claimName"):
        errs.append("spec.persistentVolumeClaim.claimName: Required value")
    tp = s.get("tensorParallelSize")
    if tp is not None and not (1 <= int(tp) <= 8):
        errs.append("spec.tensorParallelSize: must be in [1, 8]")
    return errs


def deepcopy(o):
    return copy.deepcopy(o)
