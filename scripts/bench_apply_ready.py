"""CRD-apply -> Model Available, end to end with real processes (second north-star metric).

    python scripts/bench_apply_ready.py [--preset phi2 --ftype q4_0] [--replicas 1]

Builds a local OCI registry mirror holding `library/<name>:latest` (a random-init GGUF of the
preset's real size: Phi-2 Q4_0 ~1.6 GB like the reference demo's `phi` image), then applies a
`Model{image: <name>}` to the operator running against the fake apiserver with a process kubelet
(ollama_operator_amd/operator/e2e.py): store StatefulSet -> `ollama serve`; model Deployment ->
init `ollama pull` through the store -> `ollama serve` -> probes -> Available. Prints one JSON line.
Reference: ≈51.6 s on kind/OrbStack, CPU, Phi-2 (docs/public/demo-full.cast).
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import uvicorn  # noqa: E402

from ollama_operator_amd.gguf.constants import FileType  # noqa: E402
from ollama_operator_amd.models.config import preset  # noqa: E402
from ollama_operator_amd.models.random_init import write_random_gguf  # noqa: E402
from ollama_operator_amd.operator.e2e import apply_to_ready, free_port, http_ok  # noqa: E402
from ollama_operator_amd.server.registry_server import create_registry_app  # noqa: E402
from ollama_operator_amd.server.store import ModelStore  # noqa: E402

def _gpu() -> bool:
    import torch
    return torch.cuda.is_available()


FTYPES = {"q4_0": FileType.MOSTLY_Q4_0, "q4_k_m": FileType.MOSTLY_Q4_K_M, "q8_0": FileType.MOSTLY_Q8_0}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="phi2")
    ap.add_argument("--ftype", default="q4_0")
    ap.add_argument("--name", default="phi")
    ap.add_argument("--replicas", type=int, default=1)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--timeout", type=float, default=600.0)
    a = ap.parse_args(argv)
    work = a.workdir or tempfile.mkdtemp(prefix="omx_apply_")
    try:
        reg_root = os.path.join(work, "registry")
        gguf = os.path.join(work, f"{a.preset}.gguf")
        t = time.perf_counter()
        write_random_gguf(gguf, preset(a.preset), FTYPES[a.ftype], seed=1)
        ModelStore(reg_root).create(f"library/{a.name}:latest", gguf_path=gguf,
                                    template="{{ .Prompt }}", params={"temperature": 0.0})
        os.remove(gguf)
        setup_s = time.perf_counter() - t
        port = free_port()
        srv = uvicorn.Server(uvicorn.Config(create_registry_app(reg_root), host="127.0.0.1", port=port,
                                            log_level="error"))
        threading.Thread(target=srv.run, daemon=True).start()
        while not http_ok(f"http://127.0.0.1:{port}/v2/"):
            time.sleep(0.05)
        model = {"apiVersion": "ollama.ayaka.io/v1", "kind": "Model",
                 "metadata": {"name": a.name, "namespace": "default"},
                 "spec": {"image": a.name, "replicas": a.replicas}}
        env = {"OMX_REGISTRY_MIRROR": f"http://127.0.0.1:{port}"}
        res = apply_to_ready(model, os.path.join(work, "pv"), env, timeout=a.timeout)
        srv.should_exit = True
        size = os.path.getsize(ModelStore(os.path.join(work, "pv", "default", "ollama-models-store-pvc",
                                                       "models")).model_blob(a.name))
        print(json.dumps({"metric": "CRD apply -> Model Available", "value": res["apply_to_ready_s"], "unit": "s",
                          "higher_is_better": False, "model": f"{a.preset} {a.ftype}", "blob_bytes": size,
                          "replicas": a.replicas, "device": "cuda" if _gpu() else "cpu", "phases_s": res["phases_s"],
                          "events": res["events"], "registry_setup_s": round(setup_s, 2),
                          "reference_s": 51.6,
                          "note": "fake apiserver + process kubelet; container image pull / pod sandbox excluded"}))
    finally:
        if not a.workdir:
            shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
