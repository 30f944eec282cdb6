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
