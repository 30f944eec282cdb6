"""Process-level "kind-less" end-to-end: CRD apply -> Model Available, with every data-plane step
really executed (the second north-star metric, SURVEY.md §6: the reference's ≈51.6 s on kind/
OrbStack for a Phi-2 Model, `docs/public/demo-full.cast` lines 217-218 -> 416-417).

There is no kube-apiserver / kubelet / container runtime in the build sandbox, so the cluster is
`FakeKube` (in-memory apiserver with watches) plus `ProcessKubelet`, which plays kubelet for the
two workloads the operator creates and runs the SAME programs their pod specs name:
  * StatefulSet `ollama-models-store`: starts `ollama serve` (our server) on the shared PV dir;
  * Deployment `ollama-model-<name>`: runs the init container `ollama pull <image>` against the
    store Service (which pulls from the registry -- here a local OCI registry mirror serving a
    synthetic GGUF of the requested size), then starts `ollama serve` with the PV mounted;
  * readiness follows each container's own startupProbe / readinessProbe timings from the
    rendered pod template (initialDelaySeconds, periodSeconds on GET /api/tags).
The operator is the production controller (`Manager`: watch-driven work queue, owner-reference
watches, requeues) reconciling against the fake apiserver. What is NOT included: image pulls of
the server container itself and pod scheduling/sandbox creation (sub-second to seconds on a warm
node) -- reported as such.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import threading
import time
import urllib.request

from . import api
from . import resources as R
from .controller import Manager
from .fake import FakeKube
from .kube import Conflict


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def http_ok(url: str, timeout: float = 1.0) -> bool:
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.status == 200
    except Exception:  # noqa: BLE001 - any failure is "not ready yet"
        return False


class ProcessKubelet:
    """Runs the pod specs of StatefulSets / Deployments as local processes and reports readiness."""

    def __init__(self, kube: FakeKube, pv_root: str, env: dict | None = None, log_dir: str | None = None):
        self.kube = kube
        self.pv_root = pv_root
        self.env = dict(env or {})
        self.log_dir = log_dir or pv_root
        self.procs: list[subprocess.Popen] = []
        self.svc_port: dict[str, int] = {}  # "<service>.<ns>" -> local port of the backing server
        self.timeline: dict[str, float] = {}
        self.errors: list[str] = []
        self.mu = threading.Lock()
        self._seen: set[tuple[str, str]] = set()
        kube.watchers.append(self.on_event)

    # ------------------------------------------------------------------ helpers
    def mark(self, what: str):
        with self.mu:
            self.timeline.setdefault(what, time.perf_counter())

    def _pv_dir(self, ns: str, claim: str) -> str:
        d = os.path.join(self.pv_root, ns, claim)
        os.makedirs(d, exist_ok=True)
        return d

    def _container_env(self, c: dict, ns: str, models_dir: str, port: int | None) -> dict:
        env = dict(os.environ)
        env.update(self.env)
        for e in c.get("env") or []:
            v = str(e.get("value", ""))
            if e["name"] == "OLLAMA_HOST":
                if port is not None:  # the container's own bind address -> a local port
                    v = f"127.0.0.1:{port}"
                else:  # a Service name -> its backing server's local port
                    key = v if "." in v else f"{v}.{ns}"
                    v = f"127.0.0.1:{self.svc_port[key]}"
            env[e["name"]] = v
        env["OLLAMA_MODELS"] = models_dir
        return env

    def _cmd(self, c: dict) -> list[str]:
        return [sys.executable, "-m", "ollama_operator_amd", *c.get("args", [])]

    def _probe_wait(self, c: dict, port: int, deadline: float) -> bool:
        """startupProbe then readinessProbe, each with its own initialDelaySeconds / periodSeconds."""
        url = f"http://127.0.0.1:{port}/api/tags"
        for key in ("startupProbe", "readinessProbe"):
            p = c.get(key)
            if not p:
                continue
            time.sleep(float(p.get("initialDelaySeconds", 0)))
            period = float(p.get("periodSeconds", 10))
            while not http_ok(url, float(p.get("timeoutSeconds", 1))):
                if time.perf_counter() > deadline:
                    return False
                time.sleep(period)
        return True

    def _set_ready(self, kind: str, ns: str, name: str, n: int):
        for _ in range(20):  # optimistic concurrency, like a real status writer
            o = self.kube.get(kind, ns, name)
            if o is None:
                return
            st = {"replicas": n, "readyReplicas": n, "availableReplicas": n}
            if kind == "Deployment":
                st.update(unavailableReplicas=0, updatedReplicas=n,
                          observedGeneration=o["metadata"].get("generation", 1))
            else:
                st["currentReplicas"] = n
            o["status"] = st
            try:
                self.kube.update_status(kind, ns, o)
                return
            except Conflict:
                time.sleep(0.01)

    # ------------------------------------------------------------------ workloads
    def on_event(self, typ: str, kind: str, obj: dict):
        if kind not in ("StatefulSet", "Deployment") or typ not in ("ADDED", "MODIFIED"):
            return
        md = obj["metadata"]
        key = (kind, f"{md.get('namespace', '')}/{md['name']}")
        with self.mu:
            if key in self._seen:
                return
            self._seen.add(key)
        threading.Thread(target=self._run, args=(kind, obj), daemon=True).start()

    def _run(self, kind: str, obj: dict, timeout: float = 600.0):
        md = obj["metadata"]
        ns, name = md.get("namespace", ""), md["name"]
        try:
            spec = obj["spec"]["template"]["spec"]
            vols = {v["name"]: v for v in spec.get("volumes") or []}
            claim = R.STORE_PVC
            for v in vols.values():
                if "persistentVolumeClaim" in v:
                    claim = v["persistentVolumeClaim"]["claimName"]
            models_dir = os.path.join(self._pv_dir(ns, claim), "models")
            deadline = time.perf_counter() + timeout
            tag = "store" if kind == "StatefulSet" else "model"
            self.mark(f"{tag}_scheduled")
            for c in spec.get("initContainers") or []:
                env = self._container_env(c, ns, models_dir, None)
                log = open(os.path.join(self.log_dir, f"{name}-{c['name']}.log"), "wb")
                rc = subprocess.run(self._cmd(c), env=env, stdout=log, stderr=subprocess.STDOUT,
                                    timeout=timeout).returncode
                if rc != 0:
                    raise RuntimeError(f"init container {c['name']} of {name} exited {rc}")
                self.mark(f"{tag}_init_done")
            c = next(c for c in spec["containers"] if c["name"] == "server")
            n = int(obj["spec"].get("replicas", 1))
            ports = []
            for i in range(n):
                port = free_port()
                env = self._container_env(c, ns, models_dir, port)
                log = open(os.path.join(self.log_dir, f"{name}-{i}.log"), "wb")
                self.procs.append(subprocess.Popen(self._cmd(c), env=env, stdout=log, stderr=subprocess.STDOUT))
                ports.append(port)
            self.mark(f"{tag}_started")
            for port in ports:
                if not self._probe_wait(c, port, deadline):
                    raise RuntimeError(f"{name} never became ready")
            if kind == "StatefulSet":  # the store Service resolves to the store pod
                self.svc_port[f"{R.STORE_NAME}.{ns}"] = ports[0]
            else:
                self.svc_port[f"{name}.{ns}"] = ports[0]
            self.mark(f"{tag}_ready")
            self._set_ready(kind, ns, name, n)
        except Exception as e:  # noqa: BLE001 - surfaced through .errors and the timeout
            self.errors.append(f"{kind} {name}: {e}")

    def shutdown(self):
        for p in self.procs:
            if p.poll() is None:
                p.terminate()
        for p in self.procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()


def is_available(m: dict | None) -> bool:
    conds = ((m or {}).get("status") or {}).get("conditions") or []
    return bool(conds) and conds[0].get("type") == api.COND_AVAILABLE and conds[0].get("status") == "True"


def apply_to_ready(model: dict, pv_root: str, env: dict, timeout: float = 600.0) -> dict:
    """Create `model` on a fresh fake cluster and time it to `Available` (readyReplicas met)."""
    kube = FakeKube()
    kubelet = ProcessKubelet(kube, pv_root, env)
    mgr = Manager(kube, workers=1)
    mgr.start(watch=True)
    ns = model["metadata"].get("namespace", "default")
    try:
        t0 = time.perf_counter()
        kube.create("Model", ns, model)
        name = model["metadata"]["name"]
        while time.perf_counter() - t0 < timeout:
            if is_available(kube.get("Model", ns, name)):
                break
            if kubelet.errors:
                raise RuntimeError("; ".join(kubelet.errors))
            time.sleep(0.02)
        else:
            raise TimeoutError(f"Model {name} not Available after {timeout}s")
        t1 = time.perf_counter()
        phases = {k: round(v - t0, 3) for k, v in sorted(kubelet.timeline.items(), key=lambda kv: kv[1])}
        return {"apply_to_ready_s": round(t1 - t0, 3), "phases_s": phases,
                "events": kube.event_reasons(name), "model_url": f"127.0.0.1:{kubelet.svc_port.get(f'{R.model_app_name(name)}.{ns}')}"}
    finally:
        mgr.shutdown()
        kubelet.shutdown()
