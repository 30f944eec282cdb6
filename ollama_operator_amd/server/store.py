"""Ollama on-disk model store: `$OLLAMA_MODELS` (default ~/.ollama/models) holding
`manifests/<registry>/<namespace>/<model>/<tag>` (Docker v2 manifest JSON) and
`blobs/sha256-<hex>` (the model layer is the GGUF file). The operator mounts this tree from the
shared PVC at /root/.ollama (reference pkg/model/pod.go:34-40) read-write in the store pod and
read-only in model pods, so every read path here works on a read-only filesystem.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import shutil
import time
from dataclasses import dataclass, field
from typing import Any, Iterator

DEFAULT_REGISTRY = "registry.ollama.ai"
DEFAULT_NAMESPACE = "library"
DEFAULT_TAG = "latest"

MT_MANIFEST = "application/vnd.docker.distribution.manifest.v2+json"
MT_CONFIG = "application/vnd.docker.container.image.v1+json"
MT_MODEL = "application/vnd.ollama.image.model"
MT_TEMPLATE = "application/vnd.ollama.image.template"
MT_SYSTEM = "application/vnd.ollama.image.system"
MT_PARAMS = "application/vnd.ollama.image.params"
MT_LICENSE = "application/vnd.ollama.image.license"
MT_ADAPTER = "application/vnd.ollama.image.adapter"
MT_PROJECTOR = "application/vnd.ollama.image.projector"
MT_MESSAGES = "application/vnd.ollama.image.messages"


class StoreError(Exception):
    pass


_NAME_RE = re.compile(r"^[A-Za-z0-9][A-Za-z0-9._-]*$")


@dataclass(frozen=True)
class ModelName:
    registry: str
    namespace: str
    model: str
    tag: str

    @classmethod
    def parse(cls, name: str) -> "ModelName":
        """`phi` -> registry.ollama.ai/library/phi:latest (reference README.md:45-59)."""
        s = name.strip()
        if not s:
            raise StoreError("empty model name")
        if "://" in s:
            s = s.split("://", 1)[1]
        tag = DEFAULT_TAG
        last = s.rsplit("/", 1)[-1]
        if ":" in last:
            base, tag = s.rsplit(":", 1)
            s = base
        parts = s.split("/")
        if len(parts) == 1:
            reg, ns, model = DEFAULT_REGISTRY, DEFAULT_NAMESPACE, parts[0]
        elif len(parts) == 2:
            reg, ns, model = DEFAULT_REGISTRY, parts[0], parts[1]
        else:
            reg, ns, model = parts[0], "/".join(parts[1:-1]), parts[-1]
        for piece in (model, tag):
            if not _NAME_RE.match(piece):
                raise StoreError(f"invalid model name {name!r}")
        return cls(reg.lower(), ns.lower(), model.lower(), tag)

    def __str__(self) -> str:
        return f"{self.registry}/{self.namespace}/{self.model}:{self.tag}"

    @property
    def short(self) -> str:
        """Display name the way `ollama list` prints it."""
        if self.registry == DEFAULT_REGISTRY and self.namespace == DEFAULT_NAMESPACE:
            return f"{self.model}:{self.tag}"
        if self.registry == DEFAULT_REGISTRY:
            return f"{self.namespace}/{self.model}:{self.tag}"
        return str(self)

    @property
    def repository(self) -> str:
        return f"{self.namespace}/{self.model}"


@dataclass
class Manifest:
    config: dict
    layers: list[dict]
    raw: dict = field(default_factory=dict)
    digest: str = ""
    mtime: float = 0.0

    def layer(self, media_type: str) -> dict | None:
        for l in self.layers:
            if l.get("mediaType") == media_type:
                return l
        return None

    @property
    def size(self) -> int:
        return sum(int(l.get("size", 0)) for l in self.layers) + int(self.config.get("size", 0))

    def to_json(self) -> dict:
        return {"schemaVersion": 2, "mediaType": MT_MANIFEST, "config": self.config, "layers": self.layers}


def default_root() -> str:
    return os.environ.get("OLLAMA_MODELS") or os.path.join(os.path.expanduser("~"), ".ollama", "models")


def sha256_file(path: str, bufsize: int = 1 << 22) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        while True:
            b = f.read(bufsize)
            if not b:
                break
            h.update(b)
    return "sha256:" + h.hexdigest()


class ModelStore:
    def __init__(self, root: str | None = None):
        self.root = root or default_root()

    # ------------------------------------------------------------------ paths
    @property
    def blobs_dir(self) -> str:
        return os.path.join(self.root, "blobs")

    @property
    def manifests_dir(self) -> str:
        return os.path.join(self.root, "manifests")

    def blob_path(self, digest: str) -> str:
        if not re.fullmatch(r"sha256[:-][0-9a-f]{64}", digest):
            raise StoreError(f"invalid digest {digest!r}")
        return os.path.join(self.blobs_dir, digest.replace(":", "-"))

    def manifest_path(self, name: ModelName) -> str:
        return os.path.join(self.manifests_dir, name.registry, *name.namespace.split("/"), name.model, name.tag)

    # ------------------------------------------------------------------ read
    def has_blob(self, digest: str, size: int | None = None) -> bool:
        p = self.blob_path(digest)
        return os.path.exists(p) and (size is None or os.path.getsize(p) == size)

    def read_manifest(self, name: ModelName | str) -> Manifest:
        n = ModelName.parse(name) if isinstance(name, str) else name
        p = self.manifest_path(n)
        if not os.path.exists(p):
            raise StoreError(f"model '{n.short}' not found")
        raw_b = open(p, "rb").read()
        raw = json.loads(raw_b)
        return Manifest(raw.get("config", {}), list(raw.get("layers", [])), raw,
                        "sha256:" + hashlib.sha256(raw_b).hexdigest(), os.path.getmtime(p))

    def list(self) -> Iterator[tuple[ModelName, Manifest]]:
        md = self.manifests_dir
        if not os.path.isdir(md):
            return
        for dirpath, _, files in os.walk(md):
            for tag in files:
                rel = os.path.relpath(os.path.join(dirpath, tag), md).split(os.sep)
                if len(rel) < 4:
                    continue
                n = ModelName(rel[0], "/".join(rel[1:-2]), rel[-2], rel[-1])
                try:
                    yield n, self.read_manifest(n)
                except (StoreError, json.JSONDecodeError):
                    continue

    def model_blob(self, name: ModelName | str) -> str:
        m = self.read_manifest(name)
        l = m.layer(MT_MODEL)
        if l is None:
            raise StoreError(f"model '{name}' has no model layer")
        return self.blob_path(l["digest"])

    def text_layer(self, m: Manifest, mt: str) -> str | None:
        l = m.layer(mt)
        if l is None:
            return None
        p = self.blob_path(l["digest"])
        return open(p, encoding="utf-8").read() if os.path.exists(p) else None

    def params(self, m: Manifest) -> dict[str, Any]:
        t = self.text_layer(m, MT_PARAMS)
        return json.loads(t) if t else {}

    def config(self, m: Manifest) -> dict:
        d = m.config.get("digest")
        if d and self.has_blob(d):
            try:
                return json.load(open(self.blob_path(d)))
            except json.JSONDecodeError:
                return {}
        return {}

    # ------------------------------------------------------------------ write
    def _ensure(self):
        os.makedirs(self.blobs_dir, exist_ok=True)
        os.makedirs(self.manifests_dir, exist_ok=True)

    def put_blob_bytes(self, data: bytes) -> dict:
        self._ensure()
        digest = "sha256:" + hashlib.sha256(data).hexdigest()
        p = self.blob_path(digest)
        if not os.path.exists(p):
            tmp = p + f".tmp{os.getpid()}"
            with open(tmp, "wb") as f:
                f.write(data)
            os.replace(tmp, p)
        return {"digest": digest, "size": len(data)}

    def put_blob_file(self, path: str, move: bool = False) -> dict:
        self._ensure()
        digest = sha256_file(path)
        dst = self.blob_path(digest)
        if not os.path.exists(dst):
            if move:
                shutil.move(path, dst)
            else:
                tmp = dst + f".tmp{os.getpid()}"
                shutil.copyfile(path, tmp)
                os.replace(tmp, dst)
        return {"digest": digest, "size": os.path.getsize(dst)}

    def write_manifest(self, name: ModelName | str, config: dict, layers: list[dict]) -> Manifest:
        n = ModelName.parse(name) if isinstance(name, str) else name
        self._ensure()
        p = self.manifest_path(n)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        body = json.dumps({"schemaVersion": 2, "mediaType": MT_MANIFEST, "config": config, "layers": layers},
                          indent=None).encode()
        tmp = p + f".tmp{os.getpid()}"
        with open(tmp, "wb") as f:
            f.write(body)
        os.replace(tmp, p)
        return self.read_manifest(n)

    def write_manifest_raw(self, name: ModelName, body: bytes) -> Manifest:
        self._ensure()
        p = self.manifest_path(name)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        tmp = p + f".tmp{os.getpid()}"
        with open(tmp, "wb") as f:
            f.write(body)
        os.replace(tmp, p)
        return self.read_manifest(name)

    def delete(self, name: ModelName | str) -> None:
        n = ModelName.parse(name) if isinstance(name, str) else name
        p = self.manifest_path(n)
        if not os.path.exists(p):
            raise StoreError(f"model '{n.short}' not found")
        os.remove(p)
        d = os.path.dirname(p)
        while d != self.manifests_dir and os.path.isdir(d) and not os.listdir(d):
            os.rmdir(d)
            d = os.path.dirname(d)
        self.prune()

    def copy(self, src: str, dst: str) -> None:
        m = self.read_manifest(src)
        self.write_manifest_raw(ModelName.parse(dst), json.dumps(m.raw).encode())

    def prune(self) -> int:
        """Delete blobs no manifest references (Ollama prunes on delete)."""
        used = set()
        for _, m in self.list():
            used.add(m.config.get("digest", ""))
            used.update(l.get("digest", "") for l in m.layers)
        n = 0
        if os.path.isdir(self.blobs_dir):
            for f in os.listdir(self.blobs_dir):
                if f.endswith("-partial") or ".tmp" in f:
                    continue
                if f.replace("-", ":", 1) not in used:
                    os.remove(os.path.join(self.blobs_dir, f))
                    n += 1
        return n

    # ------------------------------------------------------------------ create
    def create(self, name: str, gguf_path: str | None = None, from_model: str | None = None,
               template: str | None = None, system: str | None = None, params: dict | None = None,
               license_text: str | None = None, messages: list | None = None,
               projector_path: str | None = None) -> Manifest:
        """`ollama create` from a local GGUF (FROM ./x.gguf) or an existing model (FROM name).
        projector_path: a CLIP projector GGUF (LLaVA mmproj; a second FROM line in a Modelfile)."""
        layers: list[dict] = []
        cfg_extra: dict = {}
        if from_model:
            base = self.read_manifest(from_model)
            layers = [dict(l) for l in base.layers]
            cfg_extra = self.config(base)
        elif gguf_path:
            l = self.put_blob_file(gguf_path)
            layers = [{"mediaType": MT_MODEL, **l}]
            cfg_extra = gguf_config(gguf_path)
        else:
            raise StoreError("create needs FROM")

        def replace(mt: str, text: str | None):
            nonlocal layers
            if text is None:
                return
            layers = [l for l in layers if l.get("mediaType") != mt]
            layers.append({"mediaType": mt, **self.put_blob_bytes(text.encode())})

        if projector_path:
            layers = [l for l in layers if l.get("mediaType") != MT_PROJECTOR]
            layers.append({"mediaType": MT_PROJECTOR, **self.put_blob_file(projector_path)})
            fam = list(cfg_extra.get("model_families") or [cfg_extra.get("model_family", "")])
            if "clip" not in fam:
                cfg_extra = dict(cfg_extra, model_families=[f for f in fam if f] + ["clip"])
        replace(MT_TEMPLATE, template)
        replace(MT_SYSTEM, system)
        replace(MT_LICENSE, license_text)
        if params:
            merged = dict(self.params(Manifest({}, layers))) if from_model else {}
            merged.update(params)
            replace(MT_PARAMS, json.dumps(merged))
        if messages:
            replace(MT_MESSAGES, json.dumps(messages))
        cfg = {"model_format": "gguf", "model_family": cfg_extra.get("model_family", ""),
               "model_families": cfg_extra.get("model_families", []), "model_type": cfg_extra.get("model_type", ""),
               "file_type": cfg_extra.get("file_type", ""), "architecture": "amd64", "os": "linux",
               "rootfs": {"type": "layers", "diff_ids": [l["digest"] for l in layers]}}
        c = self.put_blob_bytes(json.dumps(cfg).encode())
        return self.write_manifest(name, {"mediaType": MT_CONFIG, **c}, layers)


def gguf_config(path: str) -> dict:
    """Model family / size / quant level from GGUF metadata (for /api/tags `details`)."""
    from ..gguf import read_gguf
    from ..gguf.constants import FILE_TYPE_NAMES, FileType
    try:
        g = read_gguf(path)
    except Exception:
        return {}
    md = g.metadata
    arch = str(md.get("general.architecture", ""))
    n_params = 0
    for t in g.tensors.values():
        n_params += t.n_elements
    g.close()
    ft = md.get("general.file_type")
    try:
        ftn = FILE_TYPE_NAMES.get(FileType(int(ft)), str(ft)) if ft is not None else ""
    except ValueError:
        ftn = str(ft)
    return {"model_family": arch, "model_families": [arch], "model_type": human_params(n_params),
            "file_type": ftn, "n_params": n_params}


def human_params(n: int) -> str:
    if n >= 1e9:
        return f"{n / 1e9:.1f}B"
    if n >= 1e6:
        return f"{n / 1e6:.0f}M"
    return str(n)


def parse_modelfile(text: str) -> dict[str, Any]:
    """Modelfile: FROM, TEMPLATE, SYSTEM, PARAMETER k v, LICENSE, MESSAGE role text, ADAPTER."""
    out: dict[str, Any] = {"parameters": {}, "messages": []}
    lines = text.splitlines()
    i = 0

    def read_value(rest: str) -> str:
        nonlocal i
        rest = rest.strip()
        for q in ('"""', "'''"):
            if rest.startswith(q):
                body = rest[3:]
                if q in body:
                    return body[:body.index(q)]
                acc = [body]
                while True:
                    i += 1
                    if i >= len(lines):
                        raise StoreError("unterminated triple-quoted string in Modelfile")
                    ln = lines[i]
                    if q in ln:
                        acc.append(ln[:ln.index(q)])
                        return "\n".join(acc)
                    acc.append(ln)
        if len(rest) >= 2 and rest[0] == rest[-1] == '"':
            return rest[1:-1]
        return rest

    while i < len(lines):
        ln = lines[i].strip()
        i0 = i
        if not ln or ln.startswith("#"):
            i += 1
            continue
        kw, _, rest = ln.partition(" ")
        kw = kw.upper()
        if kw == "FROM":  # a second FROM (a CLIP projector GGUF for LLaVA) is kept in "froms"
            out.setdefault("froms", []).append(read_value(rest))
            out.setdefault("from", out["froms"][0])
        elif kw in ("TEMPLATE", "SYSTEM", "LICENSE", "ADAPTER"):
            out[kw.lower()] = read_value(lines[i0].strip()[len(kw):])
        elif kw == "PARAMETER":
            k, _, v = rest.strip().partition(" ")
            v = read_value(v)
            out["parameters"].setdefault(k, []).append(v)
        elif kw == "MESSAGE":
            role, _, v = rest.strip().partition(" ")
            out["messages"].append({"role": role, "content": read_value(v)})
        else:
            raise StoreError(f"unknown Modelfile command {kw}")
        i += 1
    params: dict[str, Any] = {}
    for k, vs in out["parameters"].items():
        conv = [_param_value(k, v) for v in vs]
        params[k] = conv if k == "stop" else conv[-1]
    out["parameters"] = params
    return out


_INT_PARAMS = {"num_ctx", "num_predict", "top_k", "repeat_last_n", "seed", "num_keep", "num_batch", "num_gpu",
               "num_thread", "mirostat"}


def _param_value(k: str, v: str):
    if k == "stop":
        return v
    if k in _INT_PARAMS:
        return int(float(v))
    if v.lower() in ("true", "false"):
        return v.lower() == "true"
    try:
        return float(v)
    except ValueError:
        return v


def render_modelfile(name: str, m: Manifest, store: ModelStore) -> str:
    out = [f"# Modelfile generated by \"ollama show\"", f"FROM {name}"]
    t = store.text_layer(m, MT_TEMPLATE)
    if t is not None:
        out.append(f'TEMPLATE """{t}"""')
    s = store.text_layer(m, MT_SYSTEM)
    if s is not None:
        out.append(f'SYSTEM """{s}"""')
    for k, v in store.params(m).items():
        for vv in (v if isinstance(v, list) else [v]):
            out.append(f"PARAMETER {k} {json.dumps(vv) if isinstance(vv, str) else vv}")
    return "\n".join(out) + "\n"


def now_rfc3339(ts: float | None = None) -> str:
    t = time.time() if ts is None else ts
    return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(t)) + f".{int((t % 1) * 1e6):06d}Z"


def gguf_arch(path: str) -> str | None:
    """general.architecture of a GGUF file, None when it is not one."""
    from ..gguf import read_gguf
    try:
        g = read_gguf(path)
    except Exception:  # noqa: BLE001
        return None
    try:
        return g.architecture
    finally:
        g.close()
