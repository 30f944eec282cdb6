"""Minimal Kubernetes REST client for the operator (the reference uses controller-runtime's
client, cmd/main.go:98). In-cluster service-account config or a kubeconfig; JSON objects as
dicts; get/create/update/update_status/delete/list/watch; Events; Leases for leader election."""
from __future__ import annotations

import base64
import json
import os
import ssl
import tempfile
from typing import Iterator

import httpx
import yaml

from . import api


class ApiError(Exception):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{status}: {msg}")
        self.status = status


class NotFound(ApiError):
    pass


class Conflict(ApiError):
    pass


# kind -> (api prefix, plural, namespaced)
KINDS = {
    "Model": (f"/apis/{api.GROUP}/{api.VERSION}", api.PLURAL, True),
    "Deployment": ("/apis/apps/v1", "deployments", True),
    "StatefulSet": ("/apis/apps/v1", "statefulsets", True),
    "Service": ("/api/v1", "services", True),
    "PersistentVolumeClaim": ("/api/v1", "persistentvolumeclaims", True),
    "Pod": ("/api/v1", "pods", True),
    "Event": ("/api/v1", "events", True),
    "Lease": ("/apis/coordination.k8s.io/v1", "leases", True),
    "CustomResourceDefinition": ("/apis/apiextensions.k8s.io/v1", "customresourcedefinitions", False),
    # authn / authz reviews for the secure metrics endpoint (create-only, cluster scoped)
    "TokenReview": ("/apis/authentication.k8s.io/v1", "tokenreviews", False),
    "SubjectAccessReview": ("/apis/authorization.k8s.io/v1", "subjectaccessreviews", False),
}


def path_for(kind: str, ns: str | None, name: str | None = None, sub: str | None = None) -> str:
    prefix, plural, namespaced = KINDS[kind]
    p = prefix
    if namespaced and ns:
        p += f"/namespaces/{ns}"
    p += f"/{plural}"
    if name:
        p += f"/{name}"
    if sub:
        p += f"/{sub}"
    return p


class KubeClient:
    """Interface also implemented by `fake.FakeKube`."""

    def __init__(self, server: str, token: str | None = None, verify: bool | str | ssl.SSLContext = True,
                 cert: tuple[str, str] | None = None):
        self.c = httpx.Client(base_url=server, verify=verify, cert=cert, timeout=httpx.Timeout(30.0, read=None))
        self.token = token

    # ------------------------------------------------------------------ config
    @classmethod
    def from_env(cls) -> "KubeClient":
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        sa = "/var/run/secrets/kubernetes.io/serviceaccount"
        if host and os.path.exists(os.path.join(sa, "token")):
            token = open(os.path.join(sa, "token")).read().strip()
            return cls(f"https://{host}:{port}", token, verify=os.path.join(sa, "ca.crt"))
        return cls.from_kubeconfig(os.environ.get("KUBECONFIG", os.path.expanduser("~/.kube/config")))

    @classmethod
    def from_kubeconfig(cls, path: str) -> "KubeClient":
        cfg = yaml.safe_load(open(path))
        ctx_name = cfg.get("current-context")
        ctx = next(c["context"] for c in cfg["contexts"] if c["name"] == ctx_name)
        cl = next(c["cluster"] for c in cfg["clusters"] if c["name"] == ctx["cluster"])
        user = next(u["user"] for u in cfg["users"] if u["name"] == ctx["user"])

        def materialise(data_key, file_key, src):
            if src.get(file_key):
                return src[file_key]
            if src.get(data_key):
                f = tempfile.NamedTemporaryFile(delete=False)
                f.write(base64.b64decode(src[data_key]))
                f.close()
                return f.name
            return None

        verify: bool | str = not cl.get("insecure-skip-tls-verify", False)
        ca = materialise("certificate-authority-data", "certificate-authority", cl)
        if ca and verify:
            verify = ca
        cert = None
        crt = materialise("client-certificate-data", "client-certificate", user)
        key = materialise("client-key-data", "client-key", user)
        if crt and key:
            cert = (crt, key)
        return cls(cl["server"], user.get("token"), verify=verify, cert=cert)

    # ------------------------------------------------------------------ REST
    def _req(self, method: str, path: str, body: dict | None = None, params: dict | None = None,
             content_type: str = "application/json") -> dict:
        hdr = {"Content-Type": content_type}
        if self.token:
            hdr["Authorization"] = f"Bearer {self.token}"
        r = self.c.request(method, path, content=json.dumps(body) if body is not None else None, headers=hdr,
                           params=params)
        if r.status_code == 404:
            raise NotFound(404, r.text[:300])
        if r.status_code == 409:
            raise Conflict(409, r.text[:300])
        if r.status_code >= 400:
            raise ApiError(r.status_code, r.text[:300])
        return r.json() if r.content else {}

    def get(self, kind: str, ns: str | None, name: str) -> dict | None:
        try:
            return self._req("GET", path_for(kind, ns, name))
        except NotFound:
            return None

    def create(self, kind: str, ns: str | None, obj: dict) -> dict:
        return self._req("POST", path_for(kind, ns), obj)

    def update(self, kind: str, ns: str | None, obj: dict) -> dict:
        return self._req("PUT", path_for(kind, ns, obj["metadata"]["name"]), obj)

    def update_status(self, kind: str, ns: str | None, obj: dict) -> dict:
        return self._req("PUT", path_for(kind, ns, obj["metadata"]["name"], "status"), obj)

    def delete(self, kind: str, ns: str | None, name: str) -> None:
        try:
            self._req("DELETE", path_for(kind, ns, name))
        except NotFound:
            pass

    def list(self, kind: str, ns: str | None = None, label_selector: str | None = None) -> list[dict]:
        params = {"labelSelector": label_selector} if label_selector else None
        return self._req("GET", path_for(kind, ns), params=params).get("items", [])

    def watch(self, kind: str, ns: str | None = None, resource_version: str | None = None,
              timeout_s: int = 300) -> Iterator[tuple[str, dict]]:
        params = {"watch": "1", "timeoutSeconds": str(timeout_s), "allowWatchBookmarks": "true"}
        if resource_version:
            params["resourceVersion"] = resource_version
        hdr = {"Authorization": f"Bearer {self.token}"} if self.token else {}
        with self.c.stream("GET", path_for(kind, ns), params=params, headers=hdr) as r:
            if r.status_code >= 400:
                raise ApiError(r.status_code, "watch failed")
            for line in r.iter_lines():
                if line:
                    ev = json.loads(line)
                    yield ev["type"], ev["object"]

    def create_event(self, ns: str, ev: dict) -> None:
        try:
            self.create("Event", ns, ev)
        except ApiError:
            pass  # events are best effort (the reference's recorder drops failures too)
