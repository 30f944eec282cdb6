"""Repository lint policy (scripts/lint.py; reference .golangci.yml) and the CI /
kind dev-cluster files (R28, R34) stay valid."""
import os
import subprocess
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lint_clean():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "lint.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-4000:]


def test_lint_catches_forbidden_native(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import lint
    bad = tmp_path / "k.hip"
    bad.write_text('#include <cuda_runtime.h>\n__global__ void k() {}\n'
                   "#ifdef __HIP_PLATFORM_AMD__\n#endif\n")
    msgs = lint.lint_file(str(bad))
    assert any("CUDA header" in m for m in msgs) and any("dual path" in m for m in msgs)
    py = tmp_path / "m.py"
    py.write_text("import os\nimport sys\nprint(sys.argv)\n")
    assert any("unused import 'os'" in m for m in lint.lint_file(str(py)))


def test_workflows_and_kind_configs_parse():
    for rel in (".github/workflows/ci.yml", ".github/workflows/release.yml"):
        wf = yaml.safe_load(open(os.path.join(ROOT, rel)))
        assert wf["jobs"], rel
    ci = yaml.safe_load(open(os.path.join(ROOT, ".github/workflows/ci.yml")))
    steps = " ".join(s.get("run", "") for s in ci["jobs"]["cpu"]["steps"])
    assert "pytest" in steps and "build_native.py" in steps and "lint.py" in steps
    kind = yaml.safe_load(open(os.path.join(ROOT, "deploy/kind/kind-config.yaml")))
    roles = [n["role"] for n in kind["nodes"]]
    assert roles == ["control-plane", "worker", "worker", "worker"]
    ports = [n["extraPortMappings"][0]["hostPort"] for n in kind["nodes"][1:]]
    assert ports == [30101, 30102, 30103]  # reference hack/kind-config.yaml:5-19
    gpu = yaml.safe_load(open(os.path.join(ROOT, "deploy/kind/kind-gpu-config.yaml")))
    mounts = {m["hostPath"] for n in gpu["nodes"] for m in n.get("extraMounts", [])}
    assert {"/dev/kfd", "/dev/dri"} <= mounts


def test_manifests_image_override(tmp_path):
    from ollama_operator_amd.operator import manifests
    old = manifests.OPERATOR_IMAGE
    try:
        manifests.main([str(tmp_path), "--image", "ghcr.io/x/op:1.2.3"])
        text = open(tmp_path / "dist" / "install.yaml").read()
        assert "ghcr.io/x/op:1.2.3" in text
    finally:
        manifests.OPERATOR_IMAGE = old
