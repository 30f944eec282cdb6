"""In-memory fake apiserver (+ a simulated kubelet/controllers) for operator tests and for the
CRD-apply -> ready timeline simulation. There is no kind/kubectl/Go in the build sandbox
(SURVEY.md §7.4 hard part 5), so this plays the role the reference's envtest suite plays
(internal/controller/suite_test.go:46-90), extended with workload readiness so the whole state
machine is exercised (envtest has no kubelet, so the reference's test never gets past waiting).
"""
from __future__ import annotations

import copy
import itertools
import threading
import uuid

from . import api
from .kube import ApiError, Conflict


class FakeKube:
    def __init__(self):
        self.objs: dict[tuple[str, str, str], dict] = {}
        self.events: list[dict] = []
        self.mu = threading.RLock()
        self._rv = itertools.count(1)
        self._ip = itertools.count(10)
        self.watchers: list = []
        self.log: list[tuple[str, str, str]] = []  # (verb, kind, name)
        # authn / authz for TokenReview / SubjectAccessReview: bearer token -> user, users allowed
        # `get` on the /metrics non-resource URL (the metrics-reader ClusterRole)
        self.tokens: dict[str, str] = {}
        self.metrics_readers: set[str] = set()

    # ------------------------------------------------------------------ storage
    def _key(self, kind, ns, name):
        return (kind, ns or "", name)

    def _bump(self, obj):
        obj["metadata"]["resourceVersion"] = str(next(self._rv))

    def _notify(self, typ, kind, obj):
        for w in list(self.watchers):
            w(typ, kind, copy.deepcopy(obj))

    def get(self, kind, ns, name):
        with self.mu:
            o = self.objs.get(self._key(kind, ns, name))
            return copy.deepcopy(o) if o else None

    def _review(self, kind, obj):
        obj = copy.deepcopy(obj)
        spec = obj.get("spec") or {}
        if kind == "TokenReview":
            user = self.tokens.get(spec.get("token", ""))
            obj["status"] = {"authenticated": user is not None, "user": {"username": user or ""}}
        else:
            nra = spec.get("nonResourceAttributes") or {}
            ok = (spec.get("user") in self.metrics_readers and nra.get("path") == "/metrics"
                  and nra.get("verb") == "get")
            obj["status"] = {"allowed": ok}
        return obj

    def create(self, kind, ns, obj):
        if kind in ("TokenReview", "SubjectAccessReview"):
            return self._review(kind, obj)
        with self.mu:
            obj = copy.deepcopy(obj)
            md = obj.setdefault("metadata", {})
            if ns:
                md["namespace"] = ns
            k = self._key(kind, ns, md["name"])
            if k in self.objs:
                raise Conflict(409, f"{kind} {md['name']} already exists")
            if kind == "Model":
                errs = api.validate(obj)
                if errs:
                    raise ApiError(422, "; ".join(errs))
            md.setdefault("uid", str(uuid.uuid4()))
            md.setdefault("generation", 1)
            obj.setdefault("status", {})
            if kind == "Service" and obj.get("spec", {}).get("type", "ClusterIP") == "ClusterIP":
                obj["spec"]["clusterIP"] = f"10.96.0.{next(self._ip)}"
            self._bump(obj)
            self.objs[k] = obj
            self.log.append(("create", kind, md["name"]))
            self._notify("ADDED", kind, obj)
            return copy.deepcopy(obj)

    def _write(self, kind, ns, obj, status_only):
        with self.mu:
            k = self._key(kind, ns, obj["metadata"]["name"])
            cur = self.objs.get(k)
            if cur is None:
                raise ApiError(404, "not found")
            rv = obj["metadata"].get("resourceVersion")
            if rv and rv != cur["metadata"]["resourceVersion"]:
                raise Conflict(409, "the object has been modified")
            new = copy.deepcopy(cur)
            if status_only:
                new["status"] = copy.deepcopy(obj.get("status", {}))
            else:
                if new.get("spec") != obj.get("spec"):
                    new["metadata"]["generation"] = new["metadata"].get("generation", 1) + 1
                for f in ("spec", "data"):
                    if f in obj:
                        new[f] = copy.deepcopy(obj[f])
                new["metadata"]["labels"] = copy.deepcopy(obj["metadata"].get("labels", {}))
                if kind == "Service":
                    new["spec"]["clusterIP"] = cur["spec"].get("clusterIP")
            self._bump(new)
            self.objs[k] = new
            self.log.append(("update_status" if status_only else "update", kind, obj["metadata"]["name"]))
            self._notify("MODIFIED", kind, new)
            return copy.deepcopy(new)

    def update(self, kind, ns, obj):
        return self._write(kind, ns, obj, False)

    def update_status(self, kind, ns, obj):
        return self._write(kind, ns, obj, True)

    def delete(self, kind, ns, name):
        with self.mu:
            o = self.objs.pop(self._key(kind, ns, name), None)
            if o is None:
                return
            self.log.append(("delete", kind, name))
            self._notify("DELETED", kind, o)
            uid = o["metadata"].get("uid")
            # garbage collection through ownerReferences (the reference relies on it, model.go:63-69)
            for k2, o2 in list(self.objs.items()):
                refs = o2["metadata"].get("ownerReferences") or []
                if any(r.get("uid") == uid for r in refs):
                    self.delete(k2[0], k2[1], k2[2])

    def list(self, kind, ns=None, label_selector=None):
        with self.mu:
            out = []
            sel = dict(p.split("=", 1) for p in label_selector.split(",")) if label_selector else {}
            for (k, n, _), o in self.objs.items():
                if k != kind or (ns and n != ns):
                    continue
                labels = o["metadata"].get("labels") or {}
                if all(labels.get(a) == b for a, b in sel.items()):
                    out.append(copy.deepcopy(o))
            return out

    def create_event(self, ns, ev):
        with self.mu:
            self.events.append(copy.deepcopy(ev))

    def event_reasons(self, name: str | None = None) -> list[str]:
        return [e["reason"] for e in self.events
                if name is None or e.get("involvedObject", {}).get("name") == name]

    # ------------------------------------------------------------------ simulated kubelet
    def tick(self, ready_sts: bool = True, ready_deploy: bool = True):
        """Advance workload controllers one step: mark StatefulSets / Deployments ready."""
        with self.mu:
            for (kind, ns, name), o in list(self.objs.items()):
                if kind == "StatefulSet" and ready_sts:
                    want = o["spec"].get("replicas", 1)
                    st = {"replicas": want, "readyReplicas": want, "availableReplicas": want,
                          "currentReplicas": want}
                    if o.get("status") != st:
                        o["status"] = st
                        self._bump(o)
                        self._notify("MODIFIED", kind, o)
                elif kind == "Deployment" and ready_deploy:
                    want = o["spec"].get("replicas", 1)
                    st = {"replicas": want, "readyReplicas": want, "availableReplicas": want,
                          "unavailableReplicas": 0, "updatedReplicas": want,
                          "observedGeneration": o["metadata"].get("generation", 1)}
                    if o.get("status") != st:
                        o["status"] = st
                        self._bump(o)
                        self._notify("MODIFIED", kind, o)
