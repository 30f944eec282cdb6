"""Controller manager (reference cmd/main.go:54-150 + controller-runtime semantics):
work queue with per-key de-duplication, delayed requeues and exponential error backoff; watches on
Models AND the owned StatefulSets / Deployments (the reference watches only Models,
model_controller.go:172-176); Lease-based leader election with ID `300b498d.ayaka.io`
(cmd/main.go:108); /healthz + /readyz (:8081) and Prometheus /metrics (:8080) endpoints.

`--metrics-secure` (reference cmd/main.go:66-67,100-104) serves /metrics over TLS and authorises
every scrape the way the reference's kube-rbac-proxy sidecar does
(config/default/manager_auth_proxy_patch.yaml:11-39): the bearer token goes through a TokenReview,
the user through a SubjectAccessReview for `get` on the `/metrics` non-resource URL (granted by the
`metrics-reader` ClusterRole). HTTP/2 is never offered (`--enable-http2` is accepted for flag
compatibility; the reference disables it by default for the same CVEs, cmd/main.go:78-92).
SIGTERM/SIGINT stop the manager gracefully (reference `ctrl.SetupSignalHandler()`, cmd/main.go:146):
the queue closes, in-flight reconciles finish, and a leader releases its Lease so a standby replica
takes over at once instead of after the lease duration.
"""
from __future__ import annotations

import argparse
import collections
import hashlib
import heapq
import json
import logging
import os
import signal
import socket
import ssl
import subprocess
import tempfile
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from . import api, resources as R
from .kube import ApiError, Conflict
from .reconciler import ModelReconciler

log = logging.getLogger("ollama-operator")
LEADER_ELECTION_ID = "300b498d.ayaka.io"


class WorkQueue:
    def __init__(self):
        self.cv = threading.Condition()
        self.heap: list[tuple[float, str]] = []
        self.due: dict[str, float] = {}
        self.processing: set[str] = set()
        self.dirty: set[str] = set()
        self.failures: dict[str, int] = {}
        self.closed = False

    def add(self, key: str, delay: float = 0.0):
        with self.cv:
            t = time.monotonic() + delay
            if key in self.processing and delay == 0.0:
                # an event during processing: reprocess right after done(); a delayed requeue
                # (RequeueAfter) is a timer and must NOT mark the key dirty, or every "wait 5 s"
                # turns into an immediate hot loop
                self.dirty.add(key)
                return
            if key in self.due and self.due[key] <= t:
                return
            self.due[key] = t
            heapq.heappush(self.heap, (t, key))
            self.cv.notify()

    def add_rate_limited(self, key: str):
        n = self.failures.get(key, 0)
        self.failures[key] = n + 1
        self.add(key, min(0.005 * (2 ** n), 1000.0))

    def forget(self, key: str):
        self.failures.pop(key, None)

    def get(self, timeout: float | None = None) -> str | None:
        with self.cv:
            end = None if timeout is None else time.monotonic() + timeout
            while not self.closed:
                now = time.monotonic()
                while self.heap and (self.due.get(self.heap[0][1]) != self.heap[0][0]):
                    heapq.heappop(self.heap)  # stale entry
                if self.heap and self.heap[0][0] <= now:
                    _, key = heapq.heappop(self.heap)
                    self.due.pop(key, None)
                    if key in self.processing:
                        self.dirty.add(key)
                        continue
                    self.processing.add(key)
                    return key
                wait = (self.heap[0][0] - now) if self.heap else None
                if end is not None:
                    rem = end - now
                    if rem <= 0:
                        return None
                    wait = rem if wait is None else min(wait, rem)
                self.cv.wait(wait)
            return None

    def done(self, key: str):
        with self.cv:
            self.processing.discard(key)
            if key in self.dirty:
                self.dirty.discard(key)
                self.due[key] = time.monotonic()
                heapq.heappush(self.heap, (self.due[key], key))
                self.cv.notify()

    def depth(self) -> int:
        with self.cv:
            return len(self.due)

    def close(self):
        with self.cv:
            self.closed = True
            self.cv.notify_all()


class Metrics:
    def __init__(self):
        from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram
        self.reg = CollectorRegistry()
        self.total = Counter("controller_runtime_reconcile_total", "reconciles", ["controller", "result"],
                             registry=self.reg)
        self.time = Histogram("controller_runtime_reconcile_time_seconds", "reconcile latency", ["controller"],
                              registry=self.reg)
        self.depth = Gauge("workqueue_depth", "queue depth", ["name"], registry=self.reg)
        self.leader = Gauge("leader_election_master_status", "leader", ["name"], registry=self.reg)


class Manager:
    def __init__(self, kube, namespace: str | None = None, workers: int = 1, leader_elect: bool = False,
                 lease_namespace: str | None = None, identity: str | None = None, poll_s: float | None = None):
        self.kube = kube
        self.namespace = namespace
        self.q = WorkQueue()
        self.rec = ModelReconciler(kube)
        self.workers = workers
        self.leader_elect = leader_elect
        self.lease_ns = lease_namespace or os.environ.get("POD_NAMESPACE", "ollama-operator-system")
        self.identity = identity or f"{socket.gethostname()}_{os.getpid()}"
        self.is_leader = not leader_elect
        self.stop = threading.Event()
        self.metrics = Metrics()
        self.threads: list[threading.Thread] = []
        self.poll_s = poll_s

    # ------------------------------------------------------------------ event mapping
    def on_event(self, typ: str, kind: str, obj: dict):
        md = obj.get("metadata", {})
        ns = md.get("namespace", "")
        if self.namespace and ns != self.namespace:
            return
        if kind == "Model":
            self.q.add(f"{ns}/{md['name']}")
        elif kind == "Deployment":
            for ref in md.get("ownerReferences") or []:
                if ref.get("kind") == api.KIND:
                    self.q.add(f"{ns}/{ref['name']}")
        elif kind in ("StatefulSet", "Service", "PersistentVolumeClaim") and \
                (md.get("labels") or {}).get("app") == R.STORE_NAME:
            for m in self.kube.list("Model", ns):
                self.q.add(f"{ns}/{m['metadata']['name']}")

    # ------------------------------------------------------------------ workers
    def process_one(self, timeout: float | None = None) -> bool:
        key = self.q.get(timeout)
        if key is None:
            return False
        ns, name = key.split("/", 1)
        t0 = time.perf_counter()
        try:
            res = self.rec.reconcile(ns, name)
            self.q.forget(key)
            if res.requeue_after is not None:
                self.q.add(key, res.requeue_after)
                self.metrics.total.labels("model", "requeue_after").inc()
            else:
                self.metrics.total.labels("model", "success").inc()
        except Conflict:
            self.q.add(key)  # optimistic-concurrency retry
            self.metrics.total.labels("model", "requeue").inc()
        except Exception as e:  # noqa: BLE001 - any reconcile failure is retried with backoff
            log.warning("reconcile %s failed: %s", key, e)
            self.q.add_rate_limited(key)
            self.metrics.total.labels("model", "error").inc()
        finally:
            self.metrics.time.labels("model").observe(time.perf_counter() - t0)
            self.q.done(key)
        return True

    def _worker(self):
        while not self.stop.is_set():
            if not self.is_leader:
                time.sleep(0.2)
                continue
            self.process_one(timeout=0.5)

    def _watch_loop(self, kind: str):
        rv = None
        while not self.stop.is_set():
            try:
                if rv is None:
                    for o in self.kube.list(kind, self.namespace):
                        self.on_event("ADDED", kind, o)
                for typ, obj in self.kube.watch(kind, self.namespace, rv):
                    if self.stop.is_set():
                        return
                    if typ == "BOOKMARK":
                        rv = obj.get("metadata", {}).get("resourceVersion", rv)
                        continue
                    if typ == "ERROR":
                        rv = None
                        break
                    rv = obj.get("metadata", {}).get("resourceVersion", rv)
                    self.on_event(typ, kind, obj)
            except Exception as e:  # noqa: BLE001
                log.info("watch %s restarting: %s", kind, e)
                rv = None
                time.sleep(1.0)

    def _resync_loop(self):
        while not self.stop.wait(self.poll_s or 600):
            for m in self.kube.list("Model", self.namespace):
                self.q.add(f"{m['metadata']['namespace']}/{m['metadata']['name']}")

    # ------------------------------------------------------------------ leader election (Lease)
    def _lease_loop(self, duration: float = 15.0, renew: float = 10.0, retry: float = 2.0):
        name = LEADER_ELECTION_ID
        while not self.stop.is_set():
            now = time.time()
            try:
                lease = self.kube.get("Lease", self.lease_ns, name)
                ts = time.strftime("%Y-%m-%dT%H:%M:%S.000000Z", time.gmtime(now))
                if lease is None:
                    self.kube.create("Lease", self.lease_ns, {
                        "apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                        "metadata": {"name": name, "namespace": self.lease_ns},
                        "spec": {"holderIdentity": self.identity, "leaseDurationSeconds": int(duration),
                                 "acquireTime": ts, "renewTime": ts, "leaseTransitions": 0}})
                    self.is_leader = True
                else:
                    spec = lease.get("spec") or {}
                    holder = spec.get("holderIdentity")
                    renew_t = spec.get("renewTime")
                    expired = True
                    if renew_t:
                        t = time.mktime(time.strptime(renew_t[:19], "%Y-%m-%dT%H:%M:%S")) - time.timezone
                        expired = now - t > float(spec.get("leaseDurationSeconds", duration))
                    if holder == self.identity or expired or not holder:
                        if holder != self.identity:
                            spec["leaseTransitions"] = int(spec.get("leaseTransitions", 0)) + 1
                            spec["acquireTime"] = ts
                        spec.update({"holderIdentity": self.identity, "renewTime": ts,
                                     "leaseDurationSeconds": int(duration)})
                        lease["spec"] = spec
                        self.kube.update("Lease", self.lease_ns, lease)
                        self.is_leader = True
                    else:
                        self.is_leader = False
            except (ApiError, OSError) as e:
                log.info("leader election: %s", e)
                self.is_leader = False
            self.metrics.leader.labels("ollama-operator").set(1 if self.is_leader else 0)
            self.stop.wait(renew if self.is_leader else retry)

    # ------------------------------------------------------------------ run
    def start(self, watch: bool = True):
        if self.leader_elect:
            self._spawn(self._lease_loop)
        if watch:
            if hasattr(self.kube, "watchers"):  # fake apiserver: direct callbacks
                self.kube.watchers.append(self.on_event)
                for m in self.kube.list("Model", self.namespace):
                    self.on_event("ADDED", "Model", m)
            else:
                for kind in ("Model", "Deployment", "StatefulSet"):
                    self._spawn(self._watch_loop, kind)
        self._spawn(self._resync_loop)
        for _ in range(self.workers):
            self._spawn(self._worker)

    def _spawn(self, fn, *args):
        t = threading.Thread(target=fn, args=args, daemon=True)
        t.start()
        self.threads.append(t)

    def shutdown(self, drain_timeout: float = 10.0):
        """Stop watching and dequeuing, let in-flight reconciles finish, release the Lease if held."""
        self.stop.set()
        self.q.close()
        deadline = time.monotonic() + drain_timeout
        for t in self.threads:
            if t is not threading.current_thread():
                t.join(max(0.0, deadline - time.monotonic()))
        if self.leader_elect and self.is_leader:
            self.release_lease()

    def release_lease(self) -> bool:
        """controller-runtime LeaderElectionReleaseOnCancel: clear the holder so another replica
        acquires immediately."""
        try:
            lease = self.kube.get("Lease", self.lease_ns, LEADER_ELECTION_ID)
            if not lease or (lease.get("spec") or {}).get("holderIdentity") != self.identity:
                return False
            lease["spec"].update({"holderIdentity": "", "leaseDurationSeconds": 1})
            self.kube.update("Lease", self.lease_ns, lease)
            self.is_leader = False
            self.metrics.leader.labels("ollama-operator").set(0)
            log.info("released leader lease %s", LEADER_ELECTION_ID)
            return True
        except (ApiError, OSError) as e:
            log.info("lease release failed: %s", e)
            return False


class MetricsAuth:
    """kube-rbac-proxy semantics in process: TokenReview (authn) + SubjectAccessReview (authz on the
    /metrics non-resource URL). Decisions are cached briefly, as the proxy does."""

    MAX_ENTRIES = 1024       # bounded: random bearer tokens cannot grow memory
    REVIEWS_PER_S = 20.0     # TokenReview calls for unseen tokens (token bucket, burst = 1 s)

    def __init__(self, kube, ttl: float = 30.0):
        self.kube = kube
        self.ttl = ttl
        self._cache: "collections.OrderedDict[str, tuple[float, int]]" = collections.OrderedDict()
        self._lock = threading.Lock()
        self._bucket = self.REVIEWS_PER_S
        self._bucket_t = time.monotonic()

    def _allow_review(self) -> bool:
        now = time.monotonic()
        self._bucket = min(self.REVIEWS_PER_S, self._bucket + (now - self._bucket_t) * self.REVIEWS_PER_S)
        self._bucket_t = now
        if self._bucket < 1.0:
            return False
        self._bucket -= 1.0
        return True

    def check(self, header: str | None) -> int:
        """HTTP status for a request carrying this Authorization header: 200, 401 or 403."""
        if not header or not header.startswith("Bearer "):
            return 401
        # keyed by a digest: raw bearer tokens are never kept in memory
        key = hashlib.sha256(header[7:].strip().encode()).hexdigest()
        token = header[7:].strip()
        now = time.monotonic()
        with self._lock:
            hit = self._cache.get(key)
            if hit and hit[0] > now:
                self._cache.move_to_end(key)
                return hit[1]
            if not self._allow_review():  # a flood of unseen tokens: no apiserver call
                return 401
        try:
            tr = self.kube.create("TokenReview", None, {
                "apiVersion": "authentication.k8s.io/v1", "kind": "TokenReview", "spec": {"token": token}})
            st = tr.get("status") or {}
            if not st.get("authenticated"):
                code = 401
            else:
                user = st.get("user") or {}
                sar = self.kube.create("SubjectAccessReview", None, {
                    "apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview",
                    "spec": {"user": user.get("username", ""), "groups": user.get("groups") or [],
                             "nonResourceAttributes": {"path": "/metrics", "verb": "get"}}})
                code = 200 if (sar.get("status") or {}).get("allowed") else 403
        except (ApiError, OSError) as e:
            log.info("metrics authn/authz failed: %s", e)
            return 401
        with self._lock:
            now = time.monotonic()
            for k in [k for k, (exp, _) in self._cache.items() if exp <= now]:
                del self._cache[k]  # expired entries go on insert
            self._cache[key] = (now + self.ttl, code)
            while len(self._cache) > self.MAX_ENTRIES:
                self._cache.popitem(last=False)
        return code


def self_signed_cert(cert_dir: str | None = None) -> tuple[str, str]:
    """(cert, key) for TLS metrics: `tls.crt`/`tls.key` from cert_dir, else a self-signed pair (as
    controller-runtime generates when no certificate is mounted)."""
    if cert_dir and os.path.exists(os.path.join(cert_dir, "tls.crt")):
        return os.path.join(cert_dir, "tls.crt"), os.path.join(cert_dir, "tls.key")
    d = tempfile.mkdtemp(prefix="omx-metrics-tls-")
    crt, key = os.path.join(d, "tls.crt"), os.path.join(d, "tls.key")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "365", "-keyout", key,
                    "-out", crt, "-subj", "/CN=ollama-operator-metrics"], check=True, capture_output=True)
    return crt, key


def serve_probes(manager: Manager, health_addr: str, metrics_addr: str, secure: bool = False,
                 cert_dir: str | None = None):
    from prometheus_client import generate_latest
    auth = MetricsAuth(manager.kube) if secure else None

    def make(handler_map, authz=None):
        class H(BaseHTTPRequestHandler):
            timeout = 10  # per-connection socket timeout (StreamRequestHandler.setup)

            def setup(self):
                # TLS handshake in this per-connection thread, bounded by the timeout: a client that
                # connects and never sends a ClientHello cannot block accept() for everyone
                if isinstance(self.request, ssl.SSLSocket):
                    self.request.settimeout(self.timeout)
                    self.request.do_handshake()
                super().setup()

            def do_GET(self):
                fn = handler_map.get(self.path.split("?")[0])
                if fn is None:
                    self.send_response(404)
                    self.end_headers()
                    return
                if authz is not None:
                    code = authz.check(self.headers.get("Authorization"))
                    if code != 200:
                        self.send_response(code)
                        self.end_headers()
                        self.wfile.write(b"Unauthorized" if code == 401 else b"Forbidden")
                        return
                code, body, ctype = fn()
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):
                pass
        return H

    def addr(a):
        host, _, port = a.rpartition(":")
        return (host or "0.0.0.0", int(port))

    servers = []
    ok = lambda: (200, b"ok", "text/plain")  # noqa: E731
    if health_addr and health_addr != "0":
        s = ThreadingHTTPServer(addr(health_addr), make({"/healthz": ok, "/readyz": ok}))
        threading.Thread(target=s.serve_forever, daemon=True).start()
        servers.append(s)
    if metrics_addr and metrics_addr != "0":
        def met():
            manager.metrics.depth.labels("model").set(manager.q.depth())
            return 200, generate_latest(manager.metrics.reg), "text/plain; version=0.0.4"
        s = ThreadingHTTPServer(addr(metrics_addr), make({"/metrics": met}, auth))
        if secure:
            crt, key = self_signed_cert(cert_dir)
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.minimum_version = ssl.TLSVersion.TLSv1_2
            ctx.set_alpn_protocols(["http/1.1"])  # never h2 (reference cmd/main.go:78-92)
            ctx.load_cert_chain(crt, key)
            s.socket = ctx.wrap_socket(s.socket, server_side=True, do_handshake_on_connect=False)
        threading.Thread(target=s.serve_forever, daemon=True).start()
        servers.append(s)
    return servers


def run_until_signal(mgr: Manager, servers: list | None = None, stop: threading.Event | None = None) -> None:
    """Block until SIGTERM / SIGINT (or `stop`), then shut down gracefully (reference
    ctrl.SetupSignalHandler, cmd/main.go:146). Must run on the main thread (signal handlers)."""
    stop = stop or threading.Event()
    prev = {}

    def handler(signum, _frame):
        log.info("received signal %d: shutting down", signum)
        stop.set()
    for sig in (signal.SIGTERM, signal.SIGINT):
        prev[sig] = signal.signal(sig, handler)
    try:
        while not stop.wait(0.2):
            pass
    finally:
        for sig, h in prev.items():
            signal.signal(sig, h)
        mgr.shutdown()
        for s in servers or []:
            s.shutdown()


def main(argv=None):
    """Flags of the reference manager (cmd/main.go:61-74); zap flags are accepted and mapped to
    Python logging."""
    p = argparse.ArgumentParser(prog="ollama-operator")
    p.add_argument("--metrics-bind-address", default=":8080")
    p.add_argument("--health-probe-bind-address", default=":8081")
    p.add_argument("--leader-elect", action="store_true")
    p.add_argument("--metrics-secure", action="store_true",
                   help="serve /metrics over TLS with TokenReview + SubjectAccessReview authorisation")
    p.add_argument("--metrics-cert-dir", default=os.environ.get("METRICS_CERT_DIR"),
                   help="directory with tls.crt / tls.key (default: self-signed)")
    p.add_argument("--enable-http2", action="store_true", help="accepted for compatibility; HTTP/2 is never served")
    p.add_argument("--namespace", default=os.environ.get("WATCH_NAMESPACE") or None)
    p.add_argument("--zap-devel", action="store_true")
    p.add_argument("--zap-log-level", default="info")
    p.add_argument("--zap-encoder", default="console")
    p.add_argument("--zap-stacktrace-level", default="error")
    a, _ = p.parse_known_args(argv)
    lvl = {"debug": logging.DEBUG, "info": logging.INFO, "error": logging.ERROR}.get(a.zap_log_level, logging.INFO)
    logging.basicConfig(level=logging.DEBUG if a.zap_devel else lvl,
                        format='{"ts":"%(asctime)s","level":"%(levelname)s","logger":"%(name)s","msg":%(message)r}'
                        if a.zap_encoder == "json" else "%(asctime)s %(levelname)s %(name)s %(message)s")
    from .kube import KubeClient
    if a.enable_http2:
        log.info("--enable-http2: HTTP/2 is not served by this manager; metrics stay on HTTP/1.1")
    kube = KubeClient.from_env()
    mgr = Manager(kube, namespace=a.namespace, leader_elect=a.leader_elect)
    servers = serve_probes(mgr, a.health_probe_bind_address, a.metrics_bind_address, secure=a.metrics_secure,
                           cert_dir=a.metrics_cert_dir)
    mgr.start()
    log.info("starting manager %s", json.dumps({"leaderElection": a.leader_elect, "namespace": a.namespace,
                                                  "metricsSecure": a.metrics_secure}))
    run_until_signal(mgr, servers)


if __name__ == "__main__":
    main()
