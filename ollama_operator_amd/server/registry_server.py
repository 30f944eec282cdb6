"""A minimal OCI distribution v2 registry backed by a ModelStore directory.

Lets any node's model store act as a pull mirror for others (air-gapped clusters: point
`OMX_REGISTRY_MIRROR` at it) and is the fake registry the tests pull from. Supports manifests,
ranged blob GETs (resume), HEAD, and monolithic uploads for `push`.
"""
from __future__ import annotations

import hashlib
import os
import uuid

from fastapi import FastAPI, Request, Response
from fastapi.responses import JSONResponse, StreamingResponse

from .store import MT_MANIFEST, ModelName, ModelStore, StoreError


def create_registry_app(root: str, fault: dict | None = None) -> FastAPI:
    """`fault`: test hooks, e.g. {"truncate": digest_prefix} (serve a short blob) or
    {"corrupt": digest_prefix} (flip bytes) -- exercises resume and digest verification."""
    store = ModelStore(root)
    app = FastAPI()
    uploads: dict[str, str] = {}
    fault = fault if fault is not None else {}

    def mname(path: str, ref: str) -> ModelName:
        parts = path.strip("/").split("/")
        return ModelName("registry", "/".join(parts[:-1]) or "library", parts[-1], ref)

    def find_manifest(path: str, tag: str) -> bytes | None:
        parts = path.strip("/").split("/")
        ns, model = "/".join(parts[:-1]) or "library", parts[-1]
        for n, m in store.list():
            if n.namespace == ns and n.model == model and n.tag == tag:
                return open(store.manifest_path(n), "rb").read()
        return None

    @app.get("/v2/")
    def root_v2():
        return JSONResponse({})

    @app.get("/v2/{path:path}/manifests/{tag}")
    def get_manifest(path: str, tag: str):
        body = find_manifest(path, tag)
        if body is None:
            return JSONResponse({"errors": [{"code": "MANIFEST_UNKNOWN"}]}, status_code=404)
        return Response(body, media_type=MT_MANIFEST)

    @app.put("/v2/{path:path}/manifests/{tag}")
    async def put_manifest(path: str, tag: str, request: Request):
        body = await request.body()
        parts = path.strip("/").split("/")
        store.write_manifest_raw(ModelName("registry.local", "/".join(parts[:-1]) or "library", parts[-1], tag), body)
        return Response(status_code=201)

    @app.head("/v2/{path:path}/blobs/{digest}")
    def head_blob(path: str, digest: str):
        try:
            p = store.blob_path(digest)
        except StoreError:
            return Response(status_code=400)
        if not os.path.exists(p):
            return Response(status_code=404)
        return Response(status_code=200, headers={"Content-Length": str(os.path.getsize(p))})

    @app.get("/v2/{path:path}/blobs/{digest}")
    def get_blob(path: str, digest: str, request: Request):
        try:
            p = store.blob_path(digest)
        except StoreError:
            return Response(status_code=400)
        if not os.path.exists(p):
            return JSONResponse({"errors": [{"code": "BLOB_UNKNOWN"}]}, status_code=404)
        size = os.path.getsize(p)
        start = 0
        rng = request.headers.get("range")
        if rng and rng.startswith("bytes="):
            start = int(rng[6:].split("-")[0] or 0)
        end = size
        if fault.get("truncate") and digest[7:].startswith(fault["truncate"]):
            end = max(start, size // 2)
            fault.pop("truncate")  # only the first attempt is cut short
        corrupt = bool(fault.get("corrupt") and digest[7:].startswith(fault["corrupt"]))

        def gen():
            with open(p, "rb") as f:
                f.seek(start)
                left = end - start
                while left > 0:
                    b = f.read(min(1 << 20, left))
                    if not b:
                        break
                    left -= len(b)
                    yield bytes(x ^ 0xFF for x in b[:16]) + b[16:] if corrupt else b

        status = 206 if start else 200
        hdr = {"Content-Length": str(end - start)}
        if start:
            hdr["Content-Range"] = f"bytes {start}-{size - 1}/{size}"
        return StreamingResponse(gen(), status_code=status, headers=hdr, media_type="application/octet-stream")

    @app.post("/v2/{path:path}/blobs/uploads/")
    def start_upload(path: str):
        uid = uuid.uuid4().hex
        uploads[uid] = path
        return Response(status_code=202, headers={"Location": f"/v2/{path}/blobs/uploads/{uid}"})

    @app.put("/v2/{path:path}/blobs/uploads/{uid}")
    async def finish_upload(path: str, uid: str, digest: str, request: Request):
        body = await request.body()
        if "sha256:" + hashlib.sha256(body).hexdigest() != digest:
            return Response(status_code=400)
        os.makedirs(store.blobs_dir, exist_ok=True)
        with open(store.blob_path(digest), "wb") as f:
            f.write(body)
        uploads.pop(uid, None)
        return Response(status_code=201)

    return app
