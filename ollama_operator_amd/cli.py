"""`ollama`-compatible CLI. The operator's pods invoke exactly `serve` and `pull <image>`
(reference pkg/model/pod.go:18-20, 72-75) with OLLAMA_HOST set (`0.0.0.0` for the server,
`ollama-models-store.<ns>` for the puller, pod.go:21-26, 76-81); users run `run`, `list`, `show`,
`ps`, `rm`, `cp`, `create`, `push`, `stop` against a Service (getting-started.md:129-149).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

DEFAULT_PORT = 11434


def parse_host(value: str | None, for_server: bool = False) -> tuple[str, str, int]:
    """OLLAMA_HOST -> (scheme, host, port); a bare host means port 11434 (reference pod.go:76-81)."""
    v = (value or "").strip() or "127.0.0.1"
    scheme = "http"
    if "://" in v:
        scheme, v = v.split("://", 1)
    v = v.rstrip("/")
    host, port = v, DEFAULT_PORT
    if v.startswith("["):
        host, _, rest = v[1:].partition("]")
        if rest.startswith(":"):
            port = int(rest[1:])
    elif v.count(":") == 1:
        host, p = v.split(":")
        port = int(p) if p else DEFAULT_PORT
    if not host:
        host = "0.0.0.0" if for_server else "127.0.0.1"
    return scheme, host, port


def base_url() -> str:
    scheme, host, port = parse_host(os.environ.get("OLLAMA_HOST"))
    if host in ("0.0.0.0", "::"):
        host = "127.0.0.1"
    if ":" in host:
        host = f"[{host}]"
    return f"{scheme}://{host}:{port}"


def _client():
    import httpx
    return httpx.Client(base_url=base_url(), timeout=httpx.Timeout(30.0, read=None))


def _stream(c, method: str, path: str, body: dict):
    with c.stream(method, path, json=body) as r:
        if r.status_code >= 400:
            r.read()
            try:
                msg = r.json().get("error", r.text)
            except Exception:
                msg = r.text
            raise SystemExit(f"Error: {msg}")
        for line in r.iter_lines():
            if line.strip():
                ev = json.loads(line)
                if "error" in ev:
                    raise SystemExit(f"Error: {ev['error']}")
                yield ev


def _progress(events):
    last = None
    for ev in events:
        st = ev.get("status", "")
        if "total" in ev and ev.get("total"):
            pct = 100.0 * ev.get("completed", 0) / ev["total"]
            sys.stderr.write(f"\r{st} {pct:5.1f}% ({ev.get('completed', 0)}/{ev['total']})")
            last = st
        else:
            if last:
                sys.stderr.write("\n")
                last = None
            sys.stderr.write(st + "\n")
    if last:
        sys.stderr.write("\n")


def cmd_serve(a):
    import uvicorn
    from .parallel.tp import tp_size_from_env
    from .server.app import create_app
    _, host, port = parse_host(os.environ.get("OLLAMA_HOST"), for_server=True)
    manager = None
    world = None
    tp = tp_size_from_env()
    if tp > 1:  # OMX_TP: spawn the worker ranks before this process touches the GPU
        from .parallel.tp import shutdown_leader, start_leader
        from .server.manager import ModelManager
        from .server.store import ModelStore
        world = start_leader(tp)
        manager = ModelManager(ModelStore(), tp_world=world)
    try:
        uvicorn.run(create_app(store=manager.store if manager else None, manager=manager), host=host, port=port,
                    log_level=os.environ.get("OMX_LOG_LEVEL", "info"), timeout_keep_alive=300)
    finally:
        if world is not None:
            shutdown_leader(world)


def cmd_pull(a):
    with _client() as c:
        _progress(_stream(c, "POST", "/api/pull", {"model": a.model, "insecure": a.insecure}))


def cmd_push(a):
    with _client() as c:
        _progress(_stream(c, "POST", "/api/push", {"model": a.model, "insecure": a.insecure}))


def cmd_list(a):
    with _client() as c:
        r = c.get("/api/tags").json()
    print(f"{'NAME':40s} {'ID':14s} {'SIZE':>10s}  MODIFIED")
    for m in r.get("models", []):
        print(f"{m['name']:40s} {m['digest'][:12]:14s} {m['size'] / 1e9:8.1f} GB  {m['modified_at']}")


def cmd_ps(a):
    with _client() as c:
        r = c.get("/api/ps").json()
    print(f"{'NAME':40s} {'ID':14s} {'SIZE':>10s}  UNTIL")
    for m in r.get("models", []):
        print(f"{m['name']:40s} {m['digest'][:12]:14s} {m['size'] / 1e9:8.1f} GB  {m['expires_at']}")


def cmd_show(a):
    with _client() as c:
        r = c.post("/api/show", json={"model": a.model})
    if r.status_code >= 400:
        raise SystemExit(f"Error: {r.json().get('error')}")
    d = r.json()
    if a.modelfile:
        print(d["modelfile"])
    elif a.template:
        print(d["template"])
    elif a.parameters:
        print(d["parameters"])
    else:
        det = d["details"]
        print(f"  Model\n    architecture    {det.get('family')}\n    parameters      {det.get('parameter_size')}\n"
              f"    quantization    {det.get('quantization_level')}")


def cmd_rm(a):
    with _client() as c:
        for m in a.models:
            r = c.request("DELETE", "/api/delete", json={"model": m})
            if r.status_code >= 400:
                raise SystemExit(f"Error: {r.json().get('error')}")
            print(f"deleted '{m}'")


def cmd_cp(a):
    with _client() as c:
        r = c.post("/api/copy", json={"source": a.source, "destination": a.destination})
        if r.status_code >= 400:
            raise SystemExit(f"Error: {r.json().get('error')}")
    print(f"copied '{a.source}' to '{a.destination}'")


def cmd_create(a):
    text = open(a.file).read()
    base = os.path.dirname(os.path.abspath(a.file))
    lines = []
    for ln in text.splitlines():  # resolve relative FROM paths against the Modelfile's directory
        if ln.strip().upper().startswith("FROM "):
            p = ln.strip()[5:].strip()
            cand = os.path.join(base, p)
            if os.path.exists(cand):
                ln = f"FROM {cand}"
        lines.append(ln)
    with _client() as c:
        _progress(_stream(c, "POST", "/api/create", {"model": a.model, "modelfile": "\n".join(lines)}))


def cmd_stop(a):
    with _client() as c:
        c.post("/api/generate", json={"model": a.model, "keep_alive": 0})


_IMAGE_EXT = (".png", ".jpg", ".jpeg", ".webp", ".bmp", ".gif")


def _extract_images(prompt: str) -> tuple[str, list[str]]:
    """As `ollama run`: words naming existing image files are attached as base64 images (multimodal
    models) and dropped from the prompt text."""
    import base64
    words, images = [], []
    for w in prompt.split(" "):
        p = os.path.expanduser(w.strip("'\""))
        if p.lower().endswith(_IMAGE_EXT) and os.path.isfile(p):
            with open(p, "rb") as f:
                images.append(base64.b64encode(f.read()).decode())
        else:
            words.append(w)
    return " ".join(words), images


def cmd_run(a):
    with _client() as c:
        r = c.post("/api/show", json={"model": a.model})
        if r.status_code == 404:
            _progress(_stream(c, "POST", "/api/pull", {"model": a.model}))
        if a.prompt:
            prompt, images = _extract_images(" ".join(a.prompt))
            req = {"model": a.model, "prompt": prompt}
            if images:
                req["images"] = images
            for ev in _stream(c, "POST", "/api/generate", req):
                sys.stdout.write(ev.get("response", ""))
                sys.stdout.flush()
                if ev.get("done") and a.verbose:
                    _stats(ev)
            print()
            return
        msgs = []
        while True:
            try:
                line = input(">>> ")
            except EOFError:
                print()
                return
            if line.strip() in ("/bye", "/exit"):
                return
            if not line.strip():
                continue
            msgs.append({"role": "user", "content": line})
            out = []
            for ev in _stream(c, "POST", "/api/chat", {"model": a.model, "messages": msgs}):
                piece = ev.get("message", {}).get("content", "")
                out.append(piece)
                sys.stdout.write(piece)
                sys.stdout.flush()
                if ev.get("done") and a.verbose:
                    _stats(ev)
            print("\n")
            msgs.append({"role": "assistant", "content": "".join(out)})


def _stats(ev):
    ec, ed = ev.get("eval_count", 0), ev.get("eval_duration", 1)
    pc, pd = ev.get("prompt_eval_count", 0), ev.get("prompt_eval_duration", 1)
    sys.stderr.write(f"\ntotal duration:       {ev.get('total_duration', 0) / 1e9:.3f}s\n"
                     f"load duration:        {ev.get('load_duration', 0) / 1e9:.3f}s\n"
                     f"prompt eval count:    {pc} token(s)\n"
                     f"prompt eval rate:     {pc / max(pd, 1) * 1e9:.2f} tokens/s\n"
                     f"eval count:           {ec} token(s)\n"
                     f"eval rate:            {ec / max(ed, 1) * 1e9:.2f} tokens/s\n")


def main(argv=None):
    p = argparse.ArgumentParser(prog="ollama", description="Ollama-compatible CLI (MI355X-native server)")
    sub = p.add_subparsers(dest="cmd", required=True)
    sub.add_parser("serve").set_defaults(f=cmd_serve)
    for name, f in (("pull", cmd_pull), ("push", cmd_push)):
        s = sub.add_parser(name)
        s.add_argument("model")
        s.add_argument("--insecure", action="store_true")
        s.set_defaults(f=f)
    s = sub.add_parser("run")
    s.add_argument("model")
    s.add_argument("prompt", nargs="*")
    s.add_argument("--verbose", action="store_true")
    s.set_defaults(f=cmd_run)
    sub.add_parser("list", aliases=["ls"]).set_defaults(f=cmd_list)
    sub.add_parser("ps").set_defaults(f=cmd_ps)
    s = sub.add_parser("show")
    s.add_argument("model")
    s.add_argument("--modelfile", action="store_true")
    s.add_argument("--template", action="store_true")
    s.add_argument("--parameters", action="store_true")
    s.set_defaults(f=cmd_show)
    s = sub.add_parser("rm")
    s.add_argument("models", nargs="+")
    s.set_defaults(f=cmd_rm)
    s = sub.add_parser("cp")
    s.add_argument("source")
    s.add_argument("destination")
    s.set_defaults(f=cmd_cp)
    s = sub.add_parser("create")
    s.add_argument("model")
    s.add_argument("-f", "--file", default="Modelfile")
    s.set_defaults(f=cmd_create)
    s = sub.add_parser("stop")
    s.add_argument("model")
    s.set_defaults(f=cmd_stop)
    a = p.parse_args(argv)
    a.f(a)


if __name__ == "__main__":
    main()
