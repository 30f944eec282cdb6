"""Registry client for `pull` / `push` (Docker/OCI distribution v2, as registry.ollama.ai speaks)
plus offline synthetic models.

The reference's init container runs `ollama pull <image>` against the namespace's store pod
(reference pkg/model/pod.go:68-83), which downloads from the registry into the shared PV. Here:
  * resumable blob downloads (`blobs/sha256-<hex>-partial` + HTTP Range), sha256 verification,
    atomic rename, manifest written last -- a crashed pull never leaves a half model visible;
  * anonymous bearer-token challenge handling (`WWW-Authenticate: Bearer realm=...`);
  * `OMX_REGISTRY_MIRROR` redirects the default registry (air-gapped clusters / tests);
  * `synthetic/<preset>:<ftype>` names are materialised locally as random-init GGUF models of the
    real architecture (no network needed: kind demos, CI, benchmarks).
Progress events use Ollama's NDJSON shape: {"status", "digest", "total", "completed"}.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import tempfile
from typing import Callable, Iterator

import httpx

from .store import (DEFAULT_REGISTRY, MT_CONFIG, MT_MANIFEST, MT_MODEL, MT_PARAMS, MT_TEMPLATE, Manifest,
                    ModelName, ModelStore, StoreError)

CHUNK = 1 << 20

# default chat templates for synthetic models (Go text/template, as Ollama Modelfiles use)
TEMPLATES = {
    "llama": "[INST] {{ if .System }}<<SYS>>{{ .System }}<</SYS>>\n\n{{ end }}{{ .Prompt }} [/INST]",
    "mistral": "[INST] {{ if .System }}{{ .System }} {{ end }}{{ .Prompt }} [/INST]",
    "phi2": "{{ if .System }}{{ .System }}\n{{ end }}Instruct: {{ .Prompt }}\nOutput:",
}
STOPS = {"llama": ["[INST]", "[/INST]", "<<SYS>>", "<</SYS>>"], "mistral": ["[INST]", "[/INST]"],
         "phi2": ["User:", "Assistant:", "System:", "Instruct:"]}


class PullError(Exception):
    pass


def registry_base(name: ModelName, insecure: bool = False) -> str:
    mirror = os.environ.get("OMX_REGISTRY_MIRROR")
    if mirror and name.registry == DEFAULT_REGISTRY:
        return mirror.rstrip("/")
    scheme = "http" if insecure or _is_local(name.registry) else "https"
    return f"{scheme}://{name.registry}"


def _is_local(host: str) -> bool:
    h = host.split(":")[0]
    return h in ("localhost", "127.0.0.1", "::1") or h.endswith(".local") or h.endswith(".svc") or \
        h.endswith(".cluster.local")


class _Session:
    def __init__(self, timeout: float = 60.0):
        self.c = httpx.Client(follow_redirects=True, timeout=httpx.Timeout(timeout, read=300.0))
        self.token: str | None = None

    def _auth(self, resp: httpx.Response) -> bool:
        h = resp.headers.get("www-authenticate", "")
        if not h.lower().startswith("bearer"):
            return False
        kv = dict(re.findall(r'(\w+)="([^"]*)"', h))
        realm = kv.pop("realm", None)
        if not realm:
            return False
        r = self.c.get(realm, params=kv)
        if r.status_code != 200:
            return False
        self.token = r.json().get("token") or r.json().get("access_token")
        return bool(self.token)

    def request(self, method: str, url: str, **kw) -> httpx.Response:
        for _ in range(2):
            hdr = dict(kw.pop("headers", {}) or {})
            if self.token:
                hdr["Authorization"] = f"Bearer {self.token}"
            r = self.c.request(method, url, headers=hdr, **kw)
            if r.status_code == 401 and self._auth(r):
                kw["headers"] = hdr
                continue
            return r
        return r

    def stream(self, method: str, url: str, **kw):
        hdr = dict(kw.pop("headers", {}) or {})
        if self.token:
            hdr["Authorization"] = f"Bearer {self.token}"
        return self.c.stream(method, url, headers=hdr, **kw)

    def close(self):
        self.c.close()


def pull(store: ModelStore, model: str, insecure: bool = False,
         cancelled: Callable[[], bool] | None = None) -> Iterator[dict]:
    name = ModelName.parse(model)
    if name.namespace == "synthetic":
        yield from pull_synthetic(store, name)
        return
    base = registry_base(name, insecure)
    s = _Session()
    try:
        yield {"status": "pulling manifest"}
        r = s.request("GET", f"{base}/v2/{name.repository}/manifests/{name.tag}",
                      headers={"Accept": MT_MANIFEST})
        if r.status_code == 404:
            raise PullError(f"pull model manifest: file does not exist")
        if r.status_code != 200:
            raise PullError(f"pull model manifest: {r.status_code} {r.text[:200]}")
        body = r.content
        man = json.loads(body)
        blobs = [man["config"]] + list(man.get("layers", []))
        for layer in blobs:
            digest, size = layer["digest"], int(layer.get("size", 0))
            short = digest.split(":")[-1][:12]
            if store.has_blob(digest, size):
                yield {"status": f"pulling {short}", "digest": digest, "total": size, "completed": size}
                continue
            yield from _download(store, s, base, name, digest, size, short, cancelled)
        yield {"status": "verifying sha256 digest"}
        yield {"status": "writing manifest"}
        store.write_manifest_raw(name, body)
        yield {"status": "success"}
    except httpx.HTTPError as e:
        raise PullError(f"pull model manifest: {e}") from e
    finally:
        s.close()


def _download(store: ModelStore, s: _Session, base: str, name: ModelName, digest: str, size: int, short: str,
              cancelled) -> Iterator[dict]:
    os.makedirs(store.blobs_dir, exist_ok=True)
    final = store.blob_path(digest)
    part = final + "-partial"
    have = os.path.getsize(part) if os.path.exists(part) else 0
    if size and have > size:
        os.remove(part)
        have = 0
    h = hashlib.sha256()
    if have:
        with open(part, "rb") as f:
            while True:
                b = f.read(CHUNK)
                if not b:
                    break
                h.update(b)
    yield {"status": f"pulling {short}", "digest": digest, "total": size, "completed": have}
    if not size or have < size:
        hdr = {"Range": f"bytes={have}-"} if have else {}
        with s.stream("GET", f"{base}/v2/{name.repository}/blobs/{digest}", headers=hdr) as r:
            if r.status_code == 200 and have:  # server ignored the range: restart
                have = 0
                h = hashlib.sha256()
                mode = "wb"
            elif r.status_code in (200, 206):
                mode = "ab" if have else "wb"
            else:
                raise PullError(f"blob {short}: HTTP {r.status_code}")
            done = have
            last = 0
            with open(part, mode) as f:
                for chunk in r.iter_bytes(CHUNK):
                    if cancelled is not None and cancelled():
                        raise PullError("pull cancelled")
                    f.write(chunk)
                    h.update(chunk)
                    done += len(chunk)
                    if done - last >= 8 * CHUNK or (size and done >= size):
                        last = done
                        yield {"status": f"pulling {short}", "digest": digest, "total": size, "completed": done}
    got = "sha256:" + h.hexdigest()
    if got != digest:
        os.remove(part)
        raise PullError(f"digest mismatch for {short}: got {got[7:19]}, want {digest[7:19]}")
    os.replace(part, final)


def push(store: ModelStore, model: str, insecure: bool = False) -> Iterator[dict]:
    name = ModelName.parse(model)
    m = store.read_manifest(name)
    base = registry_base(name, insecure)
    s = _Session()
    try:
        yield {"status": "retrieving manifest"}
        for layer in [m.config] + m.layers:
            digest, size = layer["digest"], int(layer.get("size", 0))
            short = digest.split(":")[-1][:12]
            r = s.request("HEAD", f"{base}/v2/{name.repository}/blobs/{digest}")
            if r.status_code == 200:
                yield {"status": f"pushing {short}", "digest": digest, "total": size, "completed": size}
                continue
            r = s.request("POST", f"{base}/v2/{name.repository}/blobs/uploads/")
            if r.status_code not in (200, 201, 202):
                raise PullError(f"upload init: HTTP {r.status_code}")
            loc = r.headers.get("location", "")
            if loc.startswith("/"):
                loc = base + loc
            with open(store.blob_path(digest), "rb") as f:
                sep = "&" if "?" in loc else "?"
                r = s.request("PUT", f"{loc}{sep}digest={digest}", content=f.read(),
                              headers={"Content-Type": "application/octet-stream"})
            if r.status_code not in (200, 201, 204):
                raise PullError(f"upload {short}: HTTP {r.status_code}")
            yield {"status": f"pushing {short}", "digest": digest, "total": size, "completed": size}
        yield {"status": "pushing manifest"}
        r = s.request("PUT", f"{base}/v2/{name.repository}/manifests/{name.tag}",
                      content=json.dumps(m.raw).encode(), headers={"Content-Type": MT_MANIFEST})
        if r.status_code not in (200, 201, 204):
            raise PullError(f"push manifest: HTTP {r.status_code}")
        yield {"status": "success"}
    finally:
        s.close()


# ------------------------------------------------------------------------------------------------
# synthetic/<preset>:<ftype>  ->  random-init GGUF of the real architecture, created in place
SYNTH_FTYPES = {"q4_k_m": "MOSTLY_Q4_K_M", "q4_k_s": "MOSTLY_Q4_K_S", "q4_0": "MOSTLY_Q4_0",
                "q8_0": "MOSTLY_Q8_0", "q6_k": "MOSTLY_Q6_K", "f16": "MOSTLY_F16", "latest": None}


def pull_synthetic(store: ModelStore, name: ModelName) -> Iterator[dict]:
    from ..gguf.constants import FileType
    from ..models.config import PRESETS
    from ..models.random_init import write_random_gguf
    preset = name.model
    if preset not in PRESETS:
        raise PullError(f"unknown synthetic model {preset!r}; have {sorted(PRESETS)}")
    cfg = PRESETS[preset]
    ft = SYNTH_FTYPES.get(name.tag.lower(), "unknown")
    if ft == "unknown":
        raise PullError(f"unknown synthetic quantization {name.tag!r}; have {sorted(SYNTH_FTYPES)}")
    if ft is None:
        ft = "MOSTLY_Q4_0" if cfg.arch == "phi2" else "MOSTLY_Q4_K_M"
    try:
        store.read_manifest(name)
        yield {"status": "success"}
        return
    except StoreError:
        pass
    yield {"status": "pulling manifest"}
    os.makedirs(store.blobs_dir, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=store.blobs_dir, prefix="synthetic-", suffix=".tmp")
    os.close(fd)
    try:
        yield {"status": f"generating {preset} ({ft[7:]}) random-init weights"}
        write_random_gguf(tmp, cfg, FileType[ft], seed=0)
        yield {"status": "verifying sha256 digest"}
        family = "phi2" if cfg.arch == "phi2" else ("mistral" if "mistral" in preset or "mixtral" in preset else "llama")
        store.create(str(name), gguf_path=tmp, template=TEMPLATES[family], params={"stop": STOPS[family]})
        yield {"status": "writing manifest"}
        yield {"status": "success"}
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)
