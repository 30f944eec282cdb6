"""Render the deployable manifests (reference config/** and dist/install.yaml):
CRD, RBAC, manager Deployment, samples, kustomize overlays and the single-file installer.
`python -m ollama_operator_amd.operator.manifests [outdir]` regenerates deploy/; a test checks
the committed files are current.

Differences from the reference, on purpose: Events RBAC is cluster-wide (reference only grants it
in the operator namespace); model pods request `amd.com/gpu`; and the
metrics endpoint is protected by the manager itself (`--metrics-secure`: TLS + TokenReview +
SubjectAccessReview, operator/controller.py `MetricsAuth`) instead of a kube-rbac-proxy sidecar
image (reference config/default/manager_auth_proxy_patch.yaml:11-39) -- same :8443 https port, same
`metrics-reader` ClusterRole for scrapers (config/rbac/auth_proxy_client_clusterrole.yaml), same
tokenreview/subjectaccessreview grant (config/rbac/auth_proxy_role.yaml), and the same optional,
off-by-default Prometheus ServiceMonitor (config/prometheus/monitor.yaml:1-25).
"""
from __future__ import annotations

import os
import sys

import yaml

from . import api

NAMESPACE = "ollama-operator-system"
PREFIX = "ollama-operator-"
OPERATOR_IMAGE = "ollama-operator-amd/operator:latest"
SERVER_IMAGE = api.DEFAULT_SERVER_IMAGE


def _dump(objs: list[dict]) -> str:
    return "---\n" + "---\n".join(yaml.safe_dump(o, sort_keys=False) for o in objs)


def rbac() -> dict[str, list[dict]]:
    rules = [
        {"apiGroups": ["apps"], "resources": ["deployments", "statefulsets"],
         "verbs": ["create", "delete", "get", "list", "patch", "update", "watch"]},
        {"apiGroups": [""], "resources": ["services", "persistentvolumeclaims"],
         "verbs": ["create", "delete", "get", "list", "patch", "update", "watch"]},
        {"apiGroups": [""], "resources": ["persistentvolumes", "namespaces", "pods"], "verbs": ["get", "list", "watch"]},
        {"apiGroups": ["storage.k8s.io"], "resources": ["storageclasses"], "verbs": ["get", "list", "watch"]},
        {"apiGroups": [""], "resources": ["events"], "verbs": ["create", "patch"]},
        {"apiGroups": [api.GROUP], "resources": ["models"],
         "verbs": ["create", "delete", "get", "list", "patch", "update", "watch"]},
        {"apiGroups": [api.GROUP], "resources": ["models/finalizers"], "verbs": ["update"]},
        {"apiGroups": [api.GROUP], "resources": ["models/status"], "verbs": ["get", "patch", "update"]},
    ]
    le = [{"apiGroups": [""], "resources": ["configmaps"],
           "verbs": ["get", "list", "watch", "create", "update", "patch", "delete"]},
          {"apiGroups": ["coordination.k8s.io"], "resources": ["leases"],
           "verbs": ["get", "list", "watch", "create", "update", "patch", "delete"]},
          {"apiGroups": [""], "resources": ["events"], "verbs": ["create", "patch"]}]
    sa = {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "controller-manager", "namespace": "system"}}
    return {
        "service_account.yaml": [sa],
        "role.yaml": [{"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                       "metadata": {"name": "manager-role"}, "rules": rules}],
        "role_binding.yaml": [{"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
                               "metadata": {"name": "manager-rolebinding"},
                               "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                                           "name": "manager-role"},
                               "subjects": [{"kind": "ServiceAccount", "name": "controller-manager",
                                             "namespace": "system"}]}],
        "leader_election_role.yaml": [{"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
                                       "metadata": {"name": "leader-election-role", "namespace": "system"},
                                       "rules": le}],
        "leader_election_role_binding.yaml": [{
            "apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
            "metadata": {"name": "leader-election-rolebinding", "namespace": "system"},
            "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": "leader-election-role"},
            "subjects": [{"kind": "ServiceAccount", "name": "controller-manager", "namespace": "system"}]}],
        "model_editor_role.yaml": [{"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                                    "metadata": {"name": "model-editor-role"},
                                    "rules": [{"apiGroups": [api.GROUP], "resources": ["models"],
                                               "verbs": ["create", "delete", "get", "list", "patch", "update",
                                                         "watch"]},
                                              {"apiGroups": [api.GROUP], "resources": ["models/status"],
                                               "verbs": ["get"]}]}],
        "model_viewer_role.yaml": [{"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                                    "metadata": {"name": "model-viewer-role"},
                                    "rules": [{"apiGroups": [api.GROUP], "resources": ["models"],
                                               "verbs": ["get", "list", "watch"]},
                                              {"apiGroups": [api.GROUP], "resources": ["models/status"],
                                               "verbs": ["get"]}]}],
        "metrics_service.yaml": [{"apiVersion": "v1", "kind": "Service",
                                  "metadata": {"name": "controller-manager-metrics-service", "namespace": "system",
                                               "labels": {"control-plane": "controller-manager"}},
                                  "spec": {"selector": {"control-plane": "controller-manager"},
                                           "ports": [{"name": "https", "port": 8443, "targetPort": "https",
                                                      "protocol": "TCP"}]}}],
        # the manager authorises scrapes itself: it may create token / access reviews
        "metrics_auth_role.yaml": [{"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                                    "metadata": {"name": "metrics-auth-role"},
                                    "rules": [{"apiGroups": ["authentication.k8s.io"], "resources": ["tokenreviews"],
                                               "verbs": ["create"]},
                                              {"apiGroups": ["authorization.k8s.io"],
                                               "resources": ["subjectaccessreviews"], "verbs": ["create"]}]}],
        "metrics_auth_role_binding.yaml": [{
            "apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
            "metadata": {"name": "metrics-auth-rolebinding"},
            "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "metrics-auth-role"},
            "subjects": [{"kind": "ServiceAccount", "name": "controller-manager", "namespace": "system"}]}],
        # bind this to a Prometheus service account to let it scrape
        "metrics_reader_role.yaml": [{"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                                      "metadata": {"name": "metrics-reader"},
                                      "rules": [{"nonResourceURLs": ["/metrics"], "verbs": ["get"]}]}],
    }


def prometheus() -> list[dict]:
    """ServiceMonitor for the prometheus-operator (reference config/prometheus/monitor.yaml:1-25);
    not part of the default overlay or the installer, as in the reference."""
    return [{"apiVersion": "monitoring.coreos.com/v1", "kind": "ServiceMonitor",
             "metadata": {"name": "controller-manager-metrics-monitor", "namespace": "system",
                          "labels": {"control-plane": "controller-manager"}},
             "spec": {"endpoints": [{"path": "/metrics", "port": "https", "scheme": "https",
                                     "bearerTokenFile": "/var/run/secrets/kubernetes.io/serviceaccount/token",
                                     "tlsConfig": {"insecureSkipVerify": True}}],
                      "selector": {"matchLabels": {"control-plane": "controller-manager"}}}}]


def manager() -> list[dict]:
    ns = {"apiVersion": "v1", "kind": "Namespace",
          "metadata": {"name": "system", "labels": {"control-plane": "controller-manager"}}}
    dep = {
        "apiVersion": "apps/v1", "kind": "Deployment",
        "metadata": {"name": "controller-manager", "namespace": "system",
                     "labels": {"control-plane": "controller-manager"}},
        "spec": {
            "replicas": 1,
            "selector": {"matchLabels": {"control-plane": "controller-manager"}},
            "template": {
                "metadata": {"labels": {"control-plane": "controller-manager"},
                             "annotations": {"kubectl.kubernetes.io/default-container": "manager"}},
                "spec": {
                    "securityContext": {"runAsNonRoot": True},
                    "serviceAccountName": "controller-manager",
                    "terminationGracePeriodSeconds": 10,
                    "containers": [{
                        "name": "manager", "image": OPERATOR_IMAGE,
                        "command": ["python3", "-m", "ollama_operator_amd.operator"],
                        "args": ["--leader-elect", "--health-probe-bind-address=:8081",
                                 "--metrics-bind-address=:8443", "--metrics-secure"],
                        "env": [{"name": "OMX_SERVER_IMAGE", "value": SERVER_IMAGE},
                                {"name": "POD_NAMESPACE", "valueFrom": {"fieldRef": {"fieldPath": "metadata.namespace"}}}],
                        "ports": [{"containerPort": 8443, "name": "https", "protocol": "TCP"}],
                        "securityContext": {"allowPrivilegeEscalation": False, "capabilities": {"drop": ["ALL"]}},
                        "livenessProbe": {"httpGet": {"path": "/healthz", "port": 8081},
                                          "initialDelaySeconds": 15, "periodSeconds": 20},
                        "readinessProbe": {"httpGet": {"path": "/readyz", "port": 8081},
                                           "initialDelaySeconds": 5, "periodSeconds": 10},
                        "resources": {"limits": {"cpu": "500m", "memory": "256Mi"},
                                      "requests": {"cpu": "10m", "memory": "64Mi"}},
                    }],
                },
            },
        },
    }
    return [ns, dep]


def samples() -> dict[str, list[dict]]:
    def m(name, image, **spec):
        return {"apiVersion": api.API_VERSION, "kind": "Model",
                "metadata": {"name": name, "labels": {"app.kubernetes.io/name": "model"}},
                "spec": {"image": image, **spec}}
    return {
        "ollama_v1_model.yaml": [m("model-sample", "phi")],
        "llama2_7b_mi355x.yaml": [m("llama2-7b", "llama2:7b-chat-q4_K_M", numCtx=4096)],
        "mistral_7b_dp8.yaml": [m("mistral", "mistral", replicas=8)],
        "llama2_70b_tp8.yaml": [m("llama2-70b", "llama2:70b", tensorParallelSize=8)],
        "mixtral_8x7b.yaml": [m("mixtral", "mixtral:8x7b", tensorParallelSize=2)],
        "synthetic_demo.yaml": [m("synthetic-llama", "synthetic/tiny-llama:q4_k_m",
                                  resources={"limits": {"cpu": "2", "memory": "4Gi"}})],
    }


def kustomizations() -> dict[str, dict]:
    return {
        "config/default/kustomization.yaml": {
            "namespace": NAMESPACE, "namePrefix": PREFIX,
            # add "../prometheus" to scrape with the prometheus-operator (off by default, as in the
            # reference config/default/kustomization.yaml:26-27)
            "resources": ["../crd", "../rbac", "../manager"]},
        "config/prometheus/kustomization.yaml": {"resources": ["monitor.yaml"]},
        "config/crd/kustomization.yaml": {"resources": ["bases/ollama.ayaka.io_models.yaml"]},
        "config/rbac/kustomization.yaml": {"resources": sorted(rbac())},
        "config/manager/kustomization.yaml": {
            "resources": ["manager.yaml"],
            "images": [{"name": OPERATOR_IMAGE.split(":")[0], "newName": OPERATOR_IMAGE.split(":")[0],
                        "newTag": "latest"}]},
        "config/samples/kustomization.yaml": {"resources": sorted(samples())},
    }


def _prefixed(objs: list[dict]) -> list[dict]:
    """Apply the default overlay (namespace + namePrefix) for the single-file installer."""
    out = []
    for o in objs:
        o = yaml.safe_load(yaml.safe_dump(o))
        kind = o["kind"]
        md = o["metadata"]
        if kind == "Namespace":
            md["name"] = NAMESPACE
        elif kind != "CustomResourceDefinition":
            md["name"] = PREFIX + md["name"]
            if kind not in ("ClusterRole", "ClusterRoleBinding"):
                md["namespace"] = NAMESPACE
        if "roleRef" in o:
            o["roleRef"]["name"] = PREFIX + o["roleRef"]["name"]
        for s in o.get("subjects", []):
            s["name"] = PREFIX + s["name"]
            s["namespace"] = NAMESPACE
        if kind == "Deployment":
            o["spec"]["template"]["spec"]["serviceAccountName"] = PREFIX + "controller-manager"
        out.append(o)
    return out


def render_all() -> dict[str, str]:
    files: dict[str, str] = {"config/crd/bases/ollama.ayaka.io_models.yaml": _dump([api.crd()])}
    for n, objs in rbac().items():
        files[f"config/rbac/{n}"] = _dump(objs)
    files["config/manager/manager.yaml"] = _dump(manager())
    for n, objs in samples().items():
        files[f"config/samples/{n}"] = _dump(objs)
    files["config/prometheus/monitor.yaml"] = _dump(prometheus())
    for n, k in kustomizations().items():
        files[n] = yaml.safe_dump({"apiVersion": "kustomize.config.k8s.io/v1beta1", "kind": "Kustomization", **k},
                                  sort_keys=False)
    allobjs = [manager()[0], api.crd()] + [o for objs in rbac().values() for o in objs] + [manager()[1]]
    files["dist/install.yaml"] = _dump(_prefixed(allobjs))
    return files


def write(outdir: str) -> list[str]:
    written = []
    for rel, text in render_all().items():
        p = os.path.join(outdir, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(text)
        written.append(p)
    return written


def main(argv: list[str] | None = None) -> None:
    """python -m ollama_operator_amd.operator.manifests [outdir] [--image IMG] [--server-image IMG]
    (reference Makefile:117-121 build-installer: kustomize edit set image + kustomize build)."""
    import argparse
    global OPERATOR_IMAGE, SERVER_IMAGE
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir", nargs="?", default=os.path.join(os.path.dirname(__file__), "..", "..", "deploy"))
    ap.add_argument("--image", default=None, help="operator image for the manager Deployment")
    ap.add_argument("--server-image", default=None, help="default model-server image (OMX_SERVER_IMAGE)")
    a = ap.parse_args(argv)
    if a.image:
        OPERATOR_IMAGE = a.image
    if a.server_image:
        SERVER_IMAGE = a.server_image
    for p in write(a.outdir):
        print(p)


if __name__ == "__main__":
    main()
