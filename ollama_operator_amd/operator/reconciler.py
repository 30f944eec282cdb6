"""Model reconciler: drives a `Model` to its serving state (reference
internal/controller/model_controller.go:61-169; call stack in SURVEY.md §3.2).

Linear, idempotent state machine, identical in order, object names and Event reasons:
  Progressing -> store PVC -> store StatefulSet (wait ready) -> store Service (wait ClusterIP) ->
  model Deployment (create / scale / roll out) (wait ready) -> model Service (wait ClusterIP) ->
  mirror replica counts into status -> Available.
Requeue cadence 1 s after setting Progressing and 5 s per wait (reference :78-157), but the
controller also re-enqueues on watch events of owned StatefulSets/Deployments, so progress is
event-driven rather than polled (fix for SURVEY.md §2.5 item 1).
Further fixes over the reference: spec changes (image, serverImage, resources,
pull policy/secrets, env, placement) roll out; a Model that loses ready replicas returns to
Progressing (item 4); spec.persistentVolumeClaim is honoured (item 2).
"""
from __future__ import annotations

import time
from dataclasses import dataclass

from . import api, resources as R
from .kube import Conflict

REQUEUE_FAST = 1.0
REQUEUE_WAIT = 5.0


@dataclass
class Result:
    requeue_after: float | None = None
    stage: str = ""


def _now() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


class Recorder:
    """reference pkg/model/recorder.go (WrappedRecorder bound to one object)."""

    def __init__(self, kube, obj: dict, component: str = "ollama-model-controller"):
        self.kube, self.obj, self.component = kube, obj, component

    def event(self, etype: str, reason: str, message: str):
        md = self.obj["metadata"]
        ts = _now()
        self.kube.create_event(md.get("namespace", "default"), {
            "apiVersion": "v1", "kind": "Event",
            "metadata": {"generateName": f"{md['name']}.", "namespace": md.get("namespace", "default")},
            "involvedObject": {"apiVersion": self.obj.get("apiVersion"), "kind": self.obj.get("kind"),
                               "name": md["name"], "namespace": md.get("namespace"), "uid": md.get("uid")},
            "reason": reason, "message": message, "type": etype, "source": {"component": self.component},
            "firstTimestamp": ts, "lastTimestamp": ts, "count": 1})


class ModelReconciler:
    def __init__(self, kube):
        self.kube = kube

    # ------------------------------------------------------------------ conditions (reference :178-273)
    def _set_condition(self, m: dict, ctype: str, reason: str, message: str) -> tuple[dict, bool]:
        cur = api.conditions(m)
        if cur and cur[0].get("type") == ctype and len(cur) == 1:
            return m, False
        ts = _now()
        m.setdefault("status", {})["conditions"] = [{
            "type": ctype, "status": "True", "lastUpdateTime": ts, "lastTransitionTime": ts,
            "reason": reason, "message": message}]
        return self.kube.update_status("Model", m["metadata"]["namespace"], m), True

    def set_progressing(self, m: dict) -> tuple[dict, bool]:
        return self._set_condition(m, api.COND_PROGRESSING, "ModelProgressing", "Model is progressing")

    def set_available(self, m: dict) -> tuple[dict, bool]:
        return self._set_condition(m, api.COND_AVAILABLE, "ModelAvailable", "Model is available")

    @staticmethod
    def _counts(dep: dict) -> dict:
        st = dep.get("status") or {}
        return {k: int(st.get(k) or 0) for k in ("replicas", "readyReplicas", "availableReplicas",
                                                  "unavailableReplicas")}

    def set_replicas(self, m: dict, dep: dict) -> tuple[dict, bool]:
        want = self._counts(dep)
        st = m.setdefault("status", {})
        if all(int(st.get(k) or 0) == v for k, v in want.items()):
            return m, False
        st.update(want)
        return self.kube.update_status("Model", m["metadata"]["namespace"], m), True

    # ------------------------------------------------------------------ ensure helpers
    def _ensure(self, kind: str, ns: str, desired: dict, rec: Recorder, reason: str, msg: str) -> dict:
        cur = self.kube.get(kind, ns, desired["metadata"]["name"])
        if cur is not None:
            return cur
        try:
            obj = self.kube.create(kind, ns, desired)
        except Conflict:
            return self.kube.get(kind, ns, desired["metadata"]["name"])
        rec.event("Normal", reason, msg)
        return obj

    # ------------------------------------------------------------------ reconcile
    def reconcile(self, ns: str, name: str) -> Result:
        m = self.kube.get("Model", ns, name)
        if m is None:
            return Result(stage="deleted")  # children are garbage-collected via ownerReferences
        rec = Recorder(self.kube, m)
        available = api.has_condition(m, api.COND_AVAILABLE)
        if not available:
            m, changed = self.set_progressing(m)
            if changed:
                rec.event("Normal", "ModelProgressing", "Model is progressing")
                return Result(REQUEUE_FAST, "progressing")

        # ---- per-namespace model image store (reference image_store.go)
        if not api.spec(m).get("persistentVolumeClaim"):
            self._ensure("PersistentVolumeClaim", ns, R.store_pvc(ns, m), rec, "ProvisionedImageStoragePVC",
                         f"Provisioned image storage PVC {R.STORE_PVC}")
        sts = self._ensure("StatefulSet", ns, R.store_statefulset(ns, m), rec, "ProvisionedImageStoreStatefulSet",
                           f"Provisioned image store StatefulSet {R.STORE_NAME}")
        if int((sts.get("status") or {}).get("readyReplicas") or 0) != 1:
            rec.event("Normal", "WaitingForImageStoreStatefulSet", "Waiting for image store StatefulSet to be ready")
            return Result(REQUEUE_WAIT, "wait-store")
        svc = self._ensure("Service", ns, R.store_service(ns, sts), rec, "ProvisionedImageStoreService",
                           f"Provisioned image store Service {R.STORE_NAME}")
        if not (svc.get("spec") or {}).get("clusterIP"):
            rec.event("Normal", "WaitingForImageStoreService", "Waiting for image store Service to be ready")
            return Result(REQUEUE_WAIT, "wait-store-svc")

        # ---- the model's serving Deployment (reference model.go)
        desired = R.model_deployment(ns, m)
        dep = self._ensure("Deployment", ns, desired, rec, "DeploymentCreated",
                           f"Created deployment {desired['metadata']['name']}")
        updated = False
        if int(dep["spec"].get("replicas") or 0) != api.replicas(m):
            dep["spec"]["replicas"] = api.replicas(m)
            dep = self.kube.update("Deployment", ns, dep)
            rec.event("Normal", "ModelScaled", f"Model scaled to {api.replicas(m)} replicas")
            updated = True
        if R.template_fingerprint(dep) != R.template_fingerprint(desired):
            dep["spec"]["template"] = desired["spec"]["template"]
            dep = self.kube.update("Deployment", ns, dep)
            rec.event("Normal", "ModelUpdated", "Model deployment rolled out with the new spec")
            updated = True
        if updated:
            return Result(REQUEUE_WAIT, "updated")
        st = dep.get("status") or {}
        ready = (int(st.get("readyReplicas") or 0) == api.replicas(m) and
                 int(st.get("observedGeneration") or dep["metadata"].get("generation", 1)) >=
                 int(dep["metadata"].get("generation", 1)))
        if not ready:
            m, _ = self.set_replicas(m, dep)
            if available:  # lost ready replicas: back to Progressing (reference never reverts)
                m, _ = self.set_progressing(m)
            rec.event("Normal", "WaitingForDeployment", "Waiting for deployment to be ready")
            return Result(REQUEUE_WAIT, "wait-deployment")
        msvc = self._ensure("Service", ns, R.model_service(ns, name, dep), rec, "ServiceCreated",
                            f"Created service {R.model_app_name(name)}")
        if not (msvc.get("spec") or {}).get("clusterIP"):
            rec.event("Normal", "WaitingForService", "Waiting for service to be ready")
            return Result(REQUEUE_WAIT, "wait-service")
        m, changed = self.set_replicas(m, dep)
        if changed:
            return Result(REQUEUE_WAIT, "replicas")
        m, changed = self.set_available(m)
        if changed:
            rec.event("Normal", "ModelAvailable", "Model is available")
        return Result(None, "available")
