"""Ollama-REST-compatible server (replaces the `ollama/ollama` image the reference launches,
reference pkg/model/pod.go:10-66; contract in SURVEY.md §2.4).

Endpoints: HEAD/GET /, GET /api/version, GET /api/tags (the operator's readiness/liveness probe,
reference pkg/model/pod.go:41-64), POST /api/pull, /api/push, /api/create, /api/copy,
DELETE /api/delete, POST /api/show, POST /api/generate, /api/chat, /api/embed, /api/embeddings,
GET /api/ps, HEAD/POST /api/blobs/{digest}, OpenAI /v1/chat/completions, /v1/completions,
/v1/models, /v1/embeddings, and Prometheus /metrics.
Streaming responses are NDJSON (Ollama) or SSE (OpenAI), exactly one JSON object per chunk.
"""
from __future__ import annotations

import hashlib
import json
import os
import threading
import time
import uuid
from typing import Any, Iterator

from fastapi import FastAPI, Request
from starlette.concurrency import run_in_threadpool
from fastapi.responses import JSONResponse, PlainTextResponse, Response, StreamingResponse

from .. import __version__
from .manager import GenResult, ModelManager
from .registry import PullError, pull, push
from .store import (MT_TEMPLATE, ModelName, ModelStore, StoreError, gguf_arch, gguf_config, now_rfc3339,
                    parse_modelfile,
                    render_modelfile)
from ..models.clip import VisionError
from .template import TemplateError, render_chat, render_generate

OLLAMA_COMPAT_VERSION = "0.5.4"


def is_device_fault(exc: BaseException) -> bool:
    """A HIP runtime error (sticky: the context is lost) or a tensor-parallel group that fell out of
    step (parallel/custom_ar.py TPCollectiveError), as opposed to an engine-level failure."""
    name = type(exc).__name__
    msg = str(exc)
    return (name in ("AcceleratorError", "TPCollectiveError") or "HIP error" in msg or "hipError" in msg)


def _err(msg: str, code: int = 400) -> JSONResponse:
    return JSONResponse({"error": msg}, status_code=code)


def _ndjson(it: Iterator[dict], on_fault=None) -> StreamingResponse:
    def gen():
        try:
            for ev in it:
                yield json.dumps(ev) + "\n"
        except (PullError, StoreError, TemplateError) as e:
            yield json.dumps({"error": str(e)}) + "\n"
        except Exception as e:  # engine failure mid-stream: Ollama ends the stream with an error line
            if on_fault is not None and is_device_fault(e):
                on_fault()
            yield json.dumps({"error": f"{type(e).__name__}: {e}"}) + "\n"
    return StreamingResponse(gen(), media_type="application/x-ndjson")


def _images(raw) -> list[bytes]:
    """Ollama `images`: base64 strings (a data: URL prefix is tolerated)."""
    import base64
    import binascii
    out = []
    for v in raw or []:
        v = str(v)
        if v.startswith("data:") and "," in v:
            v = v.split(",", 1)[1]
        try:
            out.append(base64.b64decode(v, validate=False))
        except (binascii.Error, ValueError):
            raise VisionError("images must be base64-encoded") from None
    return out


def _with_image_marks(text: str, n: int, first: int) -> str:
    """Images [first, first + n) of the request go where their [img-N] markers are, else in front."""
    missing = [i for i in range(first, first + n) if f"[img-{i}]" not in text]
    return "".join(f"[img-{i}] " for i in missing) + text


def _chat_images(msgs: list[dict]) -> tuple[list[dict], list[bytes]]:
    out, images = [], []
    for m in msgs:
        imgs = _images(m.get("images"))
        m = dict(m)
        if imgs:
            m["content"] = _with_image_marks(m.get("content") or "", len(imgs), len(images))
            images += imgs
        m.pop("images", None)
        out.append(m)
    return out, images


def _model_of(body: dict) -> str:
    m = body.get("model") or body.get("name")
    if not m:
        raise StoreError("model is required")
    return m


def _details(store: ModelStore, m) -> dict:
    cfg = store.config(m)
    return {"parent_model": "", "format": cfg.get("model_format", "gguf"), "family": cfg.get("model_family", ""),
            "families": cfg.get("model_families") or None, "parameter_size": cfg.get("model_type", ""),
            "quantization_level": cfg.get("file_type", "")}


def create_app(store: ModelStore | None = None, manager: ModelManager | None = None) -> FastAPI:
    store = store or ModelStore()
    manager = manager or ModelManager(store)
    app = FastAPI(title="ollama-operator-amd server", version=__version__)
    app.state.store = store
    app.state.manager = manager
    metrics = _Metrics()

    # GPU health: a HIP runtime fault leaves the device context unusable, so after
    # answering the request the process exits non-zero and Kubernetes restarts the pod
    # (liveness / restartPolicy); tests replace the hook
    app.state.on_device_fault = lambda: threading.Timer(0.2, os._exit, args=(70,)).start()

    @app.exception_handler(Exception)
    async def _engine_error(request: Request, exc: Exception):
        # an engine failure answers as Ollama does -- {"error"} with 500. Recoverable ones (out of KV
        # blocks, a bad request that got this far) keep the server serving: the failed request's rows
        # are released by the runner / scheduler (tests/test_server.py::test_engine_fault_injection)
        if is_device_fault(exc):
            app.state.on_device_fault()
        return JSONResponse({"error": f"{type(exc).__name__}: {exc}"}, status_code=500)

    preload = os.environ.get("OMX_PRELOAD")
    if preload:  # operator-managed model pods load weights at start-up (the probe stays /api/tags)
        import threading

        def _preload():
            try:
                manager.get(preload, os.environ.get("OLLAMA_KEEP_ALIVE", "-1"))
            except Exception as e:  # noqa: BLE001 - a failed preload retries lazily on first request
                print(f"preload of {preload} failed: {e}", flush=True)
        threading.Thread(target=_preload, daemon=True).start()

    @app.get("/")
    @app.head("/")
    def root():
        return PlainTextResponse("Ollama is running")

    @app.get("/api/version")
    def version():
        return {"version": OLLAMA_COMPAT_VERSION, "omx_version": __version__}

    @app.get("/api/tags")
    def tags():
        out = []
        for n, m in store.list():
            out.append({"name": n.short, "model": n.short, "modified_at": now_rfc3339(m.mtime), "size": m.size,
                        "digest": m.digest.split(":")[-1], "details": _details(store, m)})
        out.sort(key=lambda x: x["modified_at"], reverse=True)
        return {"models": out}

    @app.post("/api/pull")
    async def api_pull(request: Request):
        body = await _json(request)
        try:
            model = _model_of(body)
        except StoreError as e:
            return _err(str(e))
        it = pull(store, model, insecure=bool(body.get("insecure")))
        if body.get("stream", True):
            return _ndjson(it)
        try:
            last = {}
            for last in it:
                pass
            return last
        except PullError as e:
            return _err(str(e), 500)

    @app.post("/api/push")
    async def api_push(request: Request):
        body = await _json(request)
        try:
            it = push(store, _model_of(body), insecure=bool(body.get("insecure")))
        except StoreError as e:
            return _err(str(e), 404)
        return _ndjson(it)

    @app.post("/api/create")
    async def api_create(request: Request):
        body = await _json(request)
        try:
            name = _model_of(body)
            if body.get("modelfile") or body.get("path"):
                text = body.get("modelfile") or open(body["path"]).read()
                mf = parse_modelfile(text)
                frm = mf.get("from")
                extra = list(mf.get("froms") or [])[1:]
                tmpl, system, params = mf.get("template"), mf.get("system"), mf.get("parameters") or None
                messages = mf.get("messages") or None
                license_text = mf.get("license")
            else:
                frm = body.get("from")
                tmpl, system, params = body.get("template"), body.get("system"), body.get("parameters")
                messages, license_text = body.get("messages"), body.get("license")
                extra = []
                if body.get("files"):  # {"name.gguf": "sha256:..."} uploaded via /api/blobs
                    paths = [store.blob_path(d) for d in body["files"].values()]
                    frm, extra = paths[0], paths[1:]
            if not frm:
                raise StoreError("no FROM line")
            # LLaVA: the CLIP GGUF (mmproj) among the FROM files becomes the projector layer
            files = [os.path.expanduser(f) for f in [frm] + extra]
            proj = [f for f in files if os.path.isfile(f) and gguf_arch(f) == "clip"]
            rest = [f for f in files if f not in proj]
            if len(proj) > 1 or len(rest) != 1:
                raise StoreError("create takes one model and at most one projector")
            src = rest[0]
            is_file = os.path.isfile(src) or src.startswith(store.blobs_dir)
            store.create(name, gguf_path=src if is_file else None, from_model=None if is_file else src,
                         template=tmpl, system=system, params=params, license_text=license_text, messages=messages,
                         projector_path=proj[0] if proj else None)
        except (StoreError, OSError, ValueError) as e:
            return _err(str(e))
        evs = [{"status": "reading model metadata"}, {"status": "writing manifest"}, {"status": "success"}]
        return _ndjson(iter(evs)) if body.get("stream", True) else evs[-1]

    @app.post("/api/copy")
    async def api_copy(request: Request):
        body = await _json(request)
        try:
            store.copy(body["source"], body["destination"])
        except (StoreError, KeyError) as e:
            return _err(str(e), 404)
        return Response(status_code=200)

    @app.delete("/api/delete")
    async def api_delete(request: Request):
        body = await _json(request)
        try:
            name = _model_of(body)
            manager.unload(name)
            store.delete(name)
        except StoreError as e:
            return _err(str(e), 404)
        return Response(status_code=200)

    @app.head("/api/blobs/{digest}")
    def blob_head(digest: str):
        try:
            return Response(status_code=200 if store.has_blob(digest) else 404)
        except StoreError:
            return Response(status_code=400)

    @app.post("/api/blobs/{digest}")
    async def blob_post(digest: str, request: Request):
        data = await request.body()
        if "sha256:" + hashlib.sha256(data).hexdigest() != digest.replace("-", ":", 1):
            return _err("digest mismatch")
        store.put_blob_bytes(data)
        return Response(status_code=201)

    @app.post("/api/show")
    async def api_show(request: Request):
        body = await _json(request)
        try:
            name = ModelName.parse(_model_of(body))
            m = store.read_manifest(name)
        except StoreError as e:
            return _err(str(e), 404)
        params = store.params(m)
        ptxt = "\n".join(f"{k:<30} {json.dumps(x) if isinstance(x, str) else x}"
                         for k, v in params.items() for x in (v if isinstance(v, list) else [v]))
        info: dict[str, Any] = {}
        try:
            from ..gguf import read_gguf
            g = read_gguf(store.model_blob(name))
            for k, v in g.metadata.items():
                if k.startswith("tokenizer.ggml.") and isinstance(v, list) and not body.get("verbose"):
                    info[k] = None
                else:
                    info[k] = v
            info["general.parameter_count"] = sum(t.n_elements for t in g.tensors.values())
            g.close()
        except Exception:
            pass
        return {"modelfile": render_modelfile(name.short, m, store), "parameters": ptxt,
                "template": store.text_layer(m, MT_TEMPLATE) or "", "details": _details(store, m),
                "model_info": info, "modified_at": now_rfc3339(m.mtime), "capabilities": ["completion"]}

    @app.get("/api/ps")
    def api_ps():
        out = []
        for lm in manager.ps():
            m = store.read_manifest(lm.name)
            out.append({"name": lm.name.short, "model": lm.name.short, "size": lm.size,
                        "digest": lm.digest.split(":")[-1], "details": _details(store, m),
                        "expires_at": now_rfc3339(min(lm.expires_at, time.time() + 10 * 365 * 86400)),
                        "size_vram": lm.size})
        return {"models": out}

    # -------------------------------------------------------------------------- generation
    def _load(body: dict):
        t0 = time.perf_counter()
        opts = body.get("options") or {}
        lm = manager.get(_model_of(body), body.get("keep_alive"), opts.get("num_ctx"))
        return lm, int((time.perf_counter() - t0) * 1e9)

    def _final(base: dict, r: GenResult, with_context: bool) -> dict:
        d = dict(base)
        d.update({"done": True, "done_reason": r.done_reason, "total_duration": r.total_duration,
                  "load_duration": r.load_duration, "prompt_eval_count": r.prompt_eval_count,
                  "prompt_eval_duration": r.prompt_eval_duration, "eval_count": r.eval_count,
                  "eval_duration": r.eval_duration})
        if with_context:
            d["context"] = r.context
        return d

    @app.post("/api/generate")
    async def api_generate(request: Request):
        body = await _json(request)
        t_start = time.perf_counter()
        try:
            model = _model_of(body)
            if not body.get("prompt") and not body.get("suffix"):
                if body.get("keep_alive") in (0, "0", "0s"):
                    manager.unload(model)
                    return {"model": model, "created_at": now_rfc3339(), "response": "", "done": True,
                            "done_reason": "unload"}
                await run_in_threadpool(_load, body)
                return {"model": model, "created_at": now_rfc3339(), "response": "", "done": True,
                        "done_reason": "load"}
            lm, load_ns = await run_in_threadpool(_load, body)
            images = _images(body.get("images"))
            prompt = _with_image_marks(body.get("prompt", ""), len(images), 0)
            if body.get("raw"):
                text = prompt
            else:
                text = render_generate(body.get("template") or lm.template, prompt,
                                       body.get("system") or lm.system, body.get("suffix"))
            ids = manager.check_context(lm, list(body.get("context") or [])) + await run_in_threadpool(
                manager.encode_prompt, lm, text, images, not body.get("context"))
        except (StoreError, TemplateError, VisionError) as e:
            return _err(str(e), 404 if "not found" in str(e) else 400)
        gen = manager.generate(lm, ids, body.get("options"), load_ns, t_start)
        base = {"model": model, "created_at": ""}
        metrics.requests.labels("generate").inc()

        def events():
            for piece, res in gen:
                if res is None:
                    yield {"model": model, "created_at": now_rfc3339(), "response": piece, "done": False}
                else:
                    metrics.observe(res)
                    base["created_at"] = now_rfc3339()
                    d = _final(base, res, True)
                    d["response"] = ""
                    yield d

        if body.get("stream", True):
            return _ndjson(events(), lambda: app.state.on_device_fault())
        def collect():  # off the event loop: concurrent requests share batched decode steps
            text_parts, final = [], None
            for ev in events():
                if ev["done"]:
                    final = ev
                else:
                    text_parts.append(ev["response"])
            final["response"] = "".join(text_parts)
            return final
        return await run_in_threadpool(collect)

    @app.post("/api/chat")
    async def api_chat(request: Request):
        body = await _json(request)
        t_start = time.perf_counter()
        try:
            model = _model_of(body)
            msgs = body.get("messages") or []
            if not msgs:
                if body.get("keep_alive") in (0, "0", "0s"):
                    manager.unload(model)
                    return {"model": model, "created_at": now_rfc3339(), "message": {"role": "assistant", "content": ""},
                            "done": True, "done_reason": "unload"}
                await run_in_threadpool(_load, body)
                return {"model": model, "created_at": now_rfc3339(), "message": {"role": "assistant", "content": ""},
                        "done": True, "done_reason": "load"}
            lm, load_ns = await run_in_threadpool(_load, body)
            msgs, images = _chat_images(msgs)
            text = render_chat(lm.template, msgs, lm.system, body.get("tools"))
            ids = await run_in_threadpool(manager.encode_prompt, lm, text, images)
        except (StoreError, TemplateError, VisionError) as e:
            return _err(str(e), 404 if "not found" in str(e) else 400)
        gen = manager.generate(lm, ids, body.get("options"), load_ns, t_start)
        metrics.requests.labels("chat").inc()

        def events():
            for piece, res in gen:
                if res is None:
                    yield {"model": model, "created_at": now_rfc3339(),
                           "message": {"role": "assistant", "content": piece}, "done": False}
                else:
                    metrics.observe(res)
                    d = _final({"model": model, "created_at": now_rfc3339(),
                                "message": {"role": "assistant", "content": ""}}, res, False)
                    yield d

        if body.get("stream", True):
            return _ndjson(events(), lambda: app.state.on_device_fault())
        def collect():
            parts, final = [], None
            for ev in events():
                if ev["done"]:
                    final = ev
                else:
                    parts.append(ev["message"]["content"])
            final["message"]["content"] = "".join(parts)
            return final
        return await run_in_threadpool(collect)

    @app.post("/api/embed")
    async def api_embed(request: Request):
        body = await _json(request)
        t0 = time.perf_counter()
        try:
            lm, load_ns = await run_in_threadpool(_load, body)
            inp = body.get("input", "")
            texts = [inp] if isinstance(inp, str) else list(inp)
            embs, n = await run_in_threadpool(manager.embed, lm, texts, body.get("truncate", True))
        except StoreError as e:
            return _err(str(e), 404 if "not found" in str(e) else 400)
        return {"model": _model_of(body), "embeddings": embs, "total_duration": int((time.perf_counter() - t0) * 1e9),
                "load_duration": load_ns, "prompt_eval_count": n}

    @app.post("/api/embeddings")
    async def api_embeddings(request: Request):
        body = await _json(request)
        try:
            lm, _ = await run_in_threadpool(_load, body)
            embs, _ = await run_in_threadpool(manager.embed, lm, [body.get("prompt", "")])
        except StoreError as e:
            return _err(str(e), 404 if "not found" in str(e) else 400)
        return {"embedding": embs[0]}

    # -------------------------------------------------------------------------- OpenAI compatibility
    def _oa_options(body: dict) -> dict:
        o: dict[str, Any] = {}
        for k_src, k_dst in (("temperature", "temperature"), ("top_p", "top_p"), ("seed", "seed"),
                             ("frequency_penalty", "frequency_penalty"), ("presence_penalty", "presence_penalty")):
            if body.get(k_src) is not None:
                o[k_dst] = body[k_src]
        if body.get("max_tokens") is not None:
            o["num_predict"] = body["max_tokens"]
        if body.get("max_completion_tokens") is not None:
            o["num_predict"] = body["max_completion_tokens"]
        if body.get("stop") is not None:
            o["stop"] = body["stop"] if isinstance(body["stop"], list) else [body["stop"]]
        return o

    def _oa_stream(chunks: Iterator[dict]) -> StreamingResponse:
        def gen():
            try:
                for c in chunks:
                    yield "data: " + json.dumps(c) + "\n\n"
            except (StoreError, TemplateError) as e:
                yield "data: " + json.dumps({"error": {"message": str(e)}}) + "\n\n"
            yield "data: [DONE]\n\n"
        return StreamingResponse(gen(), media_type="text/event-stream")

    @app.post("/v1/chat/completions")
    async def oa_chat(request: Request):
        body = await _json(request)
        t_start = time.perf_counter()
        try:
            model = _model_of(body)
            lm, load_ns = await run_in_threadpool(_load, {"model": model, "keep_alive": body.get("keep_alive")})
            msgs = []
            for m in body.get("messages") or []:
                c = m.get("content", "")
                imgs = []
                if isinstance(c, list):  # content parts; images as base64 data URLs
                    for p in c:
                        if p.get("type") == "image_url":
                            url = (p.get("image_url") or {}).get("url", "") if isinstance(p.get("image_url"), dict) \
                                else str(p.get("image_url") or "")
                            if not url.startswith("data:") or "," not in url:
                                raise VisionError("only base64 data: URLs are supported for image_url")
                            imgs.append(url.split(",", 1)[1])
                    c = "".join(p.get("text", "") for p in c if p.get("type") == "text")
                msgs.append({"role": m.get("role"), "content": c, "images": imgs})
            msgs, images = _chat_images(msgs)
            ids = await run_in_threadpool(manager.encode_prompt, lm, render_chat(lm.template, msgs, lm.system), images)
        except (StoreError, TemplateError, VisionError) as e:
            return JSONResponse({"error": {"message": str(e), "type": "invalid_request_error"}},
                                status_code=404 if "not found" in str(e) else 400)
        cid = "chatcmpl-" + uuid.uuid4().hex[:12]
        created = int(time.time())
        gen = manager.generate(lm, ids, _oa_options(body), load_ns, t_start)
        metrics.requests.labels("v1_chat").inc()
        fin = {"stop": "stop", "length": "length"}
        if body.get("stream"):
            def chunks():
                first = True
                for piece, res in gen:
                    if res is None:
                        delta = {"role": "assistant", "content": piece} if first else {"content": piece}
                        first = False
                        yield {"id": cid, "object": "chat.completion.chunk", "created": created, "model": model,
                               "system_fingerprint": "fp_omx", "choices": [{"index": 0, "delta": delta,
                                                                            "finish_reason": None}]}
                    else:
                        metrics.observe(res)
                        last = {"id": cid, "object": "chat.completion.chunk", "created": created, "model": model,
                                "system_fingerprint": "fp_omx",
                                "choices": [{"index": 0, "delta": {"role": "assistant", "content": ""} if first else {},
                                             "finish_reason": fin.get(res.done_reason, "stop")}]}
                        yield last
                        if (body.get("stream_options") or {}).get("include_usage"):
                            yield {"id": cid, "object": "chat.completion.chunk", "created": created, "model": model,
                                   "choices": [], "usage": {"prompt_tokens": res.prompt_eval_count,
                                                            "completion_tokens": res.eval_count,
                                                            "total_tokens": res.prompt_eval_count + res.eval_count}}
            return _oa_stream(chunks())
        def collect():
            parts, res = [], None
            for piece, r in gen:
                if r is None:
                    parts.append(piece)
                else:
                    res = r
            return parts, res
        parts, res = await run_in_threadpool(collect)
        metrics.observe(res)
        return {"id": cid, "object": "chat.completion", "created": created, "model": model,
                "system_fingerprint": "fp_omx",
                "choices": [{"index": 0, "message": {"role": "assistant", "content": "".join(parts)},
                             "finish_reason": fin.get(res.done_reason, "stop")}],
                "usage": {"prompt_tokens": res.prompt_eval_count, "completion_tokens": res.eval_count,
                          "total_tokens": res.prompt_eval_count + res.eval_count}}

    @app.post("/v1/completions")
    async def oa_completions(request: Request):
        body = await _json(request)
        t_start = time.perf_counter()
        try:
            model = _model_of(body)
            lm, load_ns = await run_in_threadpool(_load, {"model": model})
            prompt = body.get("prompt", "")
            if isinstance(prompt, list):
                prompt = prompt[0] if prompt else ""
            ids = lm.tokenizer.encode(prompt)
        except StoreError as e:
            return JSONResponse({"error": {"message": str(e)}}, status_code=404)
        cid = "cmpl-" + uuid.uuid4().hex[:12]
        created = int(time.time())
        gen = manager.generate(lm, ids, _oa_options(body), load_ns, t_start)
        if body.get("stream"):
            def chunks():
                for piece, res in gen:
                    yield {"id": cid, "object": "text_completion", "created": created, "model": model,
                           "choices": [{"text": piece, "index": 0,
                                        "finish_reason": None if res is None else res.done_reason}]}
            return _oa_stream(chunks())
        def collect():
            parts, res = [], None
            for piece, r in gen:
                if r is None:
                    parts.append(piece)
                else:
                    res = r
            return parts, res
        parts, res = await run_in_threadpool(collect)
        return {"id": cid, "object": "text_completion", "created": created, "model": model,
                "choices": [{"text": "".join(parts), "index": 0, "finish_reason": res.done_reason}],
                "usage": {"prompt_tokens": res.prompt_eval_count, "completion_tokens": res.eval_count,
                          "total_tokens": res.prompt_eval_count + res.eval_count}}

    @app.get("/v1/models")
    def oa_models():
        return {"object": "list", "data": [{"id": n.short, "object": "model", "created": int(m.mtime),
                                            "owned_by": n.namespace} for n, m in store.list()]}

    @app.get("/v1/models/{model:path}")
    def oa_model(model: str):
        try:
            m = store.read_manifest(model)
        except StoreError as e:
            return JSONResponse({"error": {"message": str(e)}}, status_code=404)
        return {"id": model, "object": "model", "created": int(m.mtime), "owned_by": ModelName.parse(model).namespace}

    @app.post("/v1/embeddings")
    async def oa_embeddings(request: Request):
        body = await _json(request)
        try:
            lm, _ = await run_in_threadpool(_load, {"model": _model_of(body)})
            inp = body.get("input", "")
            texts = [inp] if isinstance(inp, str) else list(inp)
            embs, n = await run_in_threadpool(manager.embed, lm, texts)
        except StoreError as e:
            return JSONResponse({"error": {"message": str(e)}}, status_code=404)
        return {"object": "list", "data": [{"object": "embedding", "embedding": e, "index": i}
                                           for i, e in enumerate(embs)],
                "model": body.get("model"), "usage": {"prompt_tokens": n, "total_tokens": n}}

    @app.get("/metrics")
    def prom():
        metrics.loaded.set(len(manager.loaded))
        return Response(metrics.render(), media_type="text/plain; version=0.0.4")

    return app


async def _json(request: Request) -> dict:
    try:
        b = await request.body()
        return json.loads(b) if b else {}
    except json.JSONDecodeError:
        return {}


class _Metrics:
    def __init__(self):
        from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest
        self.reg = CollectorRegistry()
        self._gen = generate_latest
        self.requests = Counter("omx_requests_total", "generation requests", ["endpoint"], registry=self.reg)
        self.tokens = Counter("omx_generated_tokens_total", "generated tokens", registry=self.reg)
        self.prompt_tokens = Counter("omx_prompt_tokens_total", "prompt tokens evaluated", registry=self.reg)
        self.tps = Histogram("omx_decode_tokens_per_second", "decode tokens/s per request", registry=self.reg,
                             buckets=(10, 50, 100, 200, 400, 800, 1600, 3200))
        self.ttft = Histogram("omx_prompt_eval_seconds", "prompt evaluation time", registry=self.reg)
        self.loaded = Gauge("omx_loaded_models", "models resident on the GPU", registry=self.reg)

    def observe(self, r: GenResult | None):
        if r is None:
            return
        self.tokens.inc(r.eval_count)
        self.prompt_tokens.inc(r.prompt_eval_count)
        if r.eval_duration > 0:
            self.tps.observe(r.eval_count / (r.eval_duration / 1e9))
        self.ttft.observe(r.prompt_eval_duration / 1e9)

    def render(self) -> bytes:
        return self._gen(self.reg)
