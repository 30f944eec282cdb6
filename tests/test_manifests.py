"""deploy/ must be exactly what the generator renders (golden files), and parse as YAML."""
import os

import yaml

from ollama_operator_amd.operator import manifests

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "deploy")


def test_deploy_tree_is_current():
    for rel, text in manifests.render_all().items():
        p = os.path.join(ROOT, rel)
        assert os.path.exists(p), f"{rel} missing: run `make manifests`"
        assert open(p).read() == text, f"{rel} is stale: run `make manifests`"


def test_install_bundle_contents():
    docs = [d for d in yaml.safe_load_all(open(os.path.join(ROOT, "dist", "install.yaml"))) if d]
    kinds = {(d["kind"], d["metadata"]["name"]) for d in docs}
    assert ("Namespace", "ollama-operator-system") in kinds
    assert ("CustomResourceDefinition", "models.ollama.ayaka.io") in kinds
    assert ("Deployment", "ollama-operator-controller-manager") in kinds
    role = next(d for d in docs if d["kind"] == "ClusterRole" and d["metadata"]["name"] == "ollama-operator-manager-role")
    assert any("events" in r["resources"] for r in role["rules"])  # cluster-wide events (reference gap)
    dep = next(d for d in docs if d["kind"] == "Deployment")
    assert "--leader-elect" in dep["spec"]["template"]["spec"]["containers"][0]["args"]
    sample = yaml.safe_load(open(os.path.join(ROOT, "config", "samples", "ollama_v1_model.yaml")))
    assert sample["spec"]["image"] == "phi"


def test_metrics_auth_objects_and_servicemonitor():
    """Secure metrics (reference config/default/manager_auth_proxy_patch.yaml, config/rbac/auth_proxy_*,
    config/prometheus/monitor.yaml): https :8443 Service, token/access review grant for the manager,
    the metrics-reader role for scrapers, and an off-by-default ServiceMonitor."""
    docs = [d for d in yaml.safe_load_all(open(os.path.join(ROOT, "dist", "install.yaml"))) if d]
    by = {(d["kind"], d["metadata"]["name"]): d for d in docs}
    svc = by[("Service", "ollama-operator-controller-manager-metrics-service")]
    assert svc["spec"]["ports"][0]["port"] == 8443 and svc["spec"]["ports"][0]["name"] == "https"
    auth = by[("ClusterRole", "ollama-operator-metrics-auth-role")]
    res = {r for rule in auth["rules"] for r in rule["resources"]}
    assert res == {"tokenreviews", "subjectaccessreviews"}
    b = by[("ClusterRoleBinding", "ollama-operator-metrics-auth-rolebinding")]
    assert b["roleRef"]["name"] == "ollama-operator-metrics-auth-role"
    assert b["subjects"][0]["name"] == "ollama-operator-controller-manager"
    reader = by[("ClusterRole", "ollama-operator-metrics-reader")]
    assert reader["rules"] == [{"nonResourceURLs": ["/metrics"], "verbs": ["get"]}]
    dep = by[("Deployment", "ollama-operator-controller-manager")]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert "--metrics-secure" in c["args"] and "--metrics-bind-address=:8443" in c["args"]
    assert c["ports"][0]["containerPort"] == 8443
    assert not any(d["kind"] == "ServiceMonitor" for d in docs)  # opt-in, as in the reference
    mon = yaml.safe_load(open(os.path.join(ROOT, "config", "prometheus", "monitor.yaml")))
    ep = mon["spec"]["endpoints"][0]
    assert mon["kind"] == "ServiceMonitor" and ep["scheme"] == "https" and ep["port"] == "https"
    assert "bearerTokenFile" in ep
    kz = yaml.safe_load(open(os.path.join(ROOT, "config", "default", "kustomization.yaml")))
    assert "../prometheus" not in kz["resources"]
