"""Server layer on CPU: store layout, Modelfile, Go templates, registry pull/push (fake registry),
and the Ollama / OpenAI REST surface backed by a synthetic random-init model."""
import json
import os
import socket
import threading
import time

import pytest
import uvicorn
from fastapi.testclient import TestClient

from ollama_operator_amd.cli import parse_host
from ollama_operator_amd.server.app import create_app
from ollama_operator_amd.server.manager import ModelManager, parse_keep_alive
from ollama_operator_amd.server.registry import PullError, pull, push
from ollama_operator_amd.server.registry_server import create_registry_app
from ollama_operator_amd.server.store import ModelName, ModelStore, StoreError, parse_modelfile
from ollama_operator_amd.server.template import Template, render_chat, render_generate


# ------------------------------------------------------------------------------------------ names
@pytest.mark.parametrize("name,want", [
    ("phi", "registry.ollama.ai/library/phi:latest"),
    ("llama2:7b", "registry.ollama.ai/library/llama2:7b"),
    ("user/model:q4", "registry.ollama.ai/user/model:q4"),
    ("localhost:5000/ns/m:t", "localhost:5000/ns/m:t"),
    ("synthetic/tiny-llama:q8_0", "registry.ollama.ai/synthetic/tiny-llama:q8_0"),
])
def test_model_name_parse(name, want):
    assert str(ModelName.parse(name)) == want


def test_model_name_short():
    assert ModelName.parse("phi").short == "phi:latest"
    with pytest.raises(StoreError):
        ModelName.parse("bad name!")


@pytest.mark.parametrize("v,want", [("0.0.0.0", ("http", "0.0.0.0", 11434)),
                                    ("ollama-models-store.default", ("http", "ollama-models-store.default", 11434)),
                                    ("localhost:30101", ("http", "localhost", 30101)),
                                    ("https://h:1", ("https", "h", 1)), (None, ("http", "127.0.0.1", 11434))])
def test_ollama_host(v, want):
    assert parse_host(v) == want


def test_keep_alive():
    assert parse_keep_alive("5m") == 300
    assert parse_keep_alive("1h30m") == 5400
    assert parse_keep_alive(-1) == float("inf")
    assert parse_keep_alive(10) == 10


def test_modelfile_parse():
    mf = parse_modelfile('FROM ./m.gguf\nTEMPLATE """[INST] {{ .Prompt }} [/INST]"""\nSYSTEM be brief\n'
                         'PARAMETER temperature 0.5\nPARAMETER stop "[INST]"\nPARAMETER stop "[/INST]"\n'
                         'PARAMETER num_ctx 4096\nMESSAGE user hi\n')
    assert mf["from"] == "./m.gguf"
    assert mf["template"] == "[INST] {{ .Prompt }} [/INST]"
    assert mf["system"] == "be brief"
    assert mf["parameters"] == {"temperature": 0.5, "stop": ["[INST]", "[/INST]"], "num_ctx": 4096}
    assert mf["messages"] == [{"role": "user", "content": "hi"}]


# ------------------------------------------------------------------------------------------ templates
def test_template_basic_and_trim():
    t = Template("{{- if .System }}<<{{ .System }}>>\n{{ end -}}\n[INST] {{ .Prompt }} [/INST]")
    assert t.render({"System": "S", "Prompt": "P"}) == "<<S>>\n[INST] P [/INST]"
    assert t.render({"System": "", "Prompt": "P"}) == "[INST] P [/INST]"


def test_template_messages_range():
    src = ("{{- range $i, $m := .Messages }}{{- $last := eq (len (slice $.Messages $i)) 1 }}"
           "{{- if eq .Role \"user\" }}[U]{{ .Content }}{{ else if eq .Role \"assistant\" }}[A]{{ .Content }}"
           "{{ end }}{{ if and $last (eq .Role \"user\") }}[A]{{ end }}{{ end }}")
    msgs = [{"role": "user", "content": "hi"}, {"role": "assistant", "content": "yo"}, {"role": "user", "content": "q"}]
    assert render_chat(src, msgs, None) == "[U]hi[A]yo[U]q[A]"


def test_legacy_chat_template_turns():
    tmpl = "{{ if .System }}<s>{{ .System }}</s>{{ end }}U:{{ .Prompt }}\nA:{{ .Response }}\n"
    msgs = [{"role": "system", "content": "sys"}, {"role": "user", "content": "a"},
            {"role": "assistant", "content": "b"}, {"role": "user", "content": "c"}]
    assert render_chat(tmpl, msgs, None) == "<s>sys</s>U:a\nA:b\nU:c\nA:"
    assert render_generate(tmpl, "p", None) == "U:p\nA:"


# ------------------------------------------------------------------------------------------ registry
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def source_store(tmp_path_factory, tiny_models):
    root = str(tmp_path_factory.mktemp("src_store"))
    st = ModelStore(root)
    st.create("library/tiny:latest", gguf_path=tiny_models["tiny-llama"],
              template="[INST] {{ .Prompt }} [/INST]", params={"stop": ["[INST]"], "temperature": 0.0})
    return st


@pytest.fixture(scope="module")
def registry(source_store):
    fault: dict = {}
    app = create_registry_app(source_store.root, fault)
    port = _free_port()
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    for _ in range(100):
        if server.started:
            break
        time.sleep(0.05)
    yield f"localhost:{port}", fault
    server.should_exit = True
    th.join(timeout=5)


def test_pull_resume_and_verify(tmp_path, registry, source_store):
    host, fault = registry
    dst = ModelStore(str(tmp_path / "dst"))
    m = source_store.read_manifest("library/tiny:latest")
    model_digest = m.layer("application/vnd.ollama.image.model")["digest"]
    fault["truncate"] = model_digest[7:19]
    with pytest.raises(PullError):  # first attempt is cut short -> digest mismatch, partial removed
        list(pull(dst, f"{host}/library/tiny:latest"))
    evs = list(pull(dst, f"{host}/library/tiny:latest"))
    assert evs[0]["status"] == "pulling manifest" and evs[-1]["status"] == "success"
    assert any(e.get("digest") == model_digest and e.get("completed") == e.get("total") for e in evs)
    assert os.path.getsize(dst.model_blob(f"{host}/library/tiny:latest")) == os.path.getsize(
        source_store.model_blob("library/tiny:latest"))
    # second pull is a no-op on blobs
    evs2 = list(pull(dst, f"{host}/library/tiny:latest"))
    assert evs2[-1]["status"] == "success"


def test_pull_corrupt_blob_rejected(tmp_path, registry, source_store):
    host, fault = registry
    m = source_store.read_manifest("library/tiny:latest")
    d = m.layer("application/vnd.ollama.image.model")["digest"]
    fault["corrupt"] = d[7:19]
    dst = ModelStore(str(tmp_path / "dst2"))
    try:
        with pytest.raises(PullError, match="digest mismatch"):
            list(pull(dst, f"{host}/library/tiny:latest"))
        with pytest.raises(StoreError):
            dst.read_manifest(f"{host}/library/tiny:latest")  # no half-written model is visible
    finally:
        fault.pop("corrupt", None)


def test_pull_missing_model(tmp_path, registry):
    host, _ = registry
    with pytest.raises(PullError, match="does not exist"):
        list(pull(ModelStore(str(tmp_path / "x")), f"{host}/library/nope:latest"))


def test_push_roundtrip(tmp_path, registry, source_store):
    host, _ = registry
    src = ModelStore(str(tmp_path / "p"))
    list(pull(src, f"{host}/library/tiny:latest"))
    src.copy(f"{host}/library/tiny:latest", f"{host}/team/tiny2:v1")
    evs = list(push(src, f"{host}/team/tiny2:v1"))
    assert evs[-1]["status"] == "success"
    back = ModelStore(str(tmp_path / "q"))
    assert list(pull(back, f"{host}/team/tiny2:v1"))[-1]["status"] == "success"


def test_synthetic_pull(tmp_path):
    st = ModelStore(str(tmp_path / "s"))
    evs = list(pull(st, "synthetic/tiny-phi2:q4_0"))
    assert evs[-1]["status"] == "success"
    m = st.read_manifest("synthetic/tiny-phi2:q4_0")
    assert st.config(m)["model_family"] == "phi2"
    with pytest.raises(PullError):
        list(pull(st, "synthetic/nonexistent:q4_0"))


# ------------------------------------------------------------------------------------------ REST API
@pytest.fixture(scope="module")
def client(tmp_path_factory, tiny_models):
    root = str(tmp_path_factory.mktemp("api_store"))
    st = ModelStore(root)
    st.create("tiny", gguf_path=tiny_models["tiny-llama"], template="[INST] {{ .Prompt }} [/INST]",
              params={"temperature": 0.0, "stop": ["[INST]"], "num_ctx": 128})
    import os
    os.environ.setdefault("OLLAMA_NUM_PARALLEL", "4")  # exercise continuous batching on the CPU twin
    app = create_app(st, ModelManager(st, device="cpu"))
    return TestClient(app)


def test_root_version_tags(client):
    assert client.get("/").text == "Ollama is running"
    assert client.head("/").status_code == 200
    assert "version" in client.get("/api/version").json()
    tags = client.get("/api/tags").json()["models"]
    assert tags[0]["name"] == "tiny:latest"
    assert tags[0]["details"]["family"] == "llama"
    assert tags[0]["details"]["quantization_level"] == "Q4_K_M"


def test_show(client):
    d = client.post("/api/show", json={"model": "tiny"}).json()
    assert "FROM tiny:latest" in d["modelfile"]
    assert d["template"] == "[INST] {{ .Prompt }} [/INST]"
    assert d["model_info"]["general.architecture"] == "llama"
    assert client.post("/api/show", json={"model": "nope"}).status_code == 404


def test_generate_stream_and_stats(client):
    with client.stream("POST", "/api/generate", json={"model": "tiny", "prompt": "hello",
                                                      "options": {"num_predict": 8, "seed": 1}}) as r:
        lines = [json.loads(l) for l in r.iter_lines() if l]
    assert all(not l["done"] for l in lines[:-1])
    fin = lines[-1]
    assert fin["done"] and fin["done_reason"] in ("stop", "length")
    for k in ("total_duration", "load_duration", "prompt_eval_count", "prompt_eval_duration", "eval_count",
              "eval_duration", "context"):
        assert k in fin
    assert fin["eval_count"] >= 1 and fin["eval_duration"] > 0
    assert "".join(l["response"] for l in lines[:-1]) is not None


def test_generate_non_stream_deterministic(client):
    body = {"model": "tiny", "prompt": "why is the sky blue?", "stream": False,
            "options": {"num_predict": 6, "temperature": 0}}
    a = client.post("/api/generate", json=body).json()
    b = client.post("/api/generate", json=body).json()
    assert a["response"] == b["response"] and a["eval_count"] == b["eval_count"]
    # continuing with the returned context reuses the KV prefix
    c = client.post("/api/generate", json={**body, "prompt": "more", "context": a["context"]}).json()
    assert c["done"]


def test_generate_load_and_unload(client):
    assert client.post("/api/generate", json={"model": "tiny"}).json()["done_reason"] == "load"
    assert client.get("/api/ps").json()["models"][0]["name"] == "tiny:latest"
    assert client.post("/api/generate", json={"model": "tiny", "keep_alive": 0}).json()["done_reason"] == "unload"
    assert client.get("/api/ps").json()["models"] == []


def test_chat(client):
    with client.stream("POST", "/api/chat", json={"model": "tiny", "messages": [{"role": "user", "content": "hi"}],
                                                  "options": {"num_predict": 5}}) as r:
        lines = [json.loads(l) for l in r.iter_lines() if l]
    assert lines[-1]["done"] and lines[-1]["message"]["role"] == "assistant"
    assert "eval_count" in lines[-1]
    d = client.post("/api/chat", json={"model": "tiny", "stream": False,
                                       "messages": [{"role": "user", "content": "hi"}],
                                       "options": {"num_predict": 3}}).json()
    assert d["message"]["role"] == "assistant" and d["done"]


def test_openai_chat(client):
    r = client.post("/v1/chat/completions", json={"model": "tiny", "max_tokens": 4,
                                                  "messages": [{"role": "user", "content": "hi"}]}).json()
    assert r["object"] == "chat.completion"
    assert r["choices"][0]["message"]["role"] == "assistant"
    assert r["usage"]["completion_tokens"] >= 1
    with client.stream("POST", "/v1/chat/completions", json={"model": "tiny", "max_tokens": 4, "stream": True,
                                                             "messages": [{"role": "user", "content": "hi"}]}) as s:
        evs = [l for l in s.iter_lines() if l]
    assert evs[-1] == "data: [DONE]"
    first = json.loads(evs[0][6:])
    assert first["object"] == "chat.completion.chunk"
    assert json.loads(evs[-2][6:])["choices"][0]["finish_reason"] in ("stop", "length")
    assert client.get("/v1/models").json()["data"][0]["id"] == "tiny:latest"
    comp = client.post("/v1/completions", json={"model": "tiny", "prompt": "x", "max_tokens": 2}).json()
    assert comp["object"] == "text_completion"


def test_embeddings(client):
    e = client.post("/api/embed", json={"model": "tiny", "input": ["a b", "c"]}).json()
    assert len(e["embeddings"]) == 2 and len(e["embeddings"][0]) == 256
    n = sum(x * x for x in e["embeddings"][0])
    assert abs(n - 1) < 1e-3
    assert len(client.post("/api/embeddings", json={"model": "tiny", "prompt": "a"}).json()["embedding"]) == 256
    oa = client.post("/v1/embeddings", json={"model": "tiny", "input": "a"}).json()
    assert oa["data"][0]["object"] == "embedding"


def test_copy_delete_metrics(client):
    assert client.post("/api/copy", json={"source": "tiny", "destination": "tiny2"}).status_code == 200
    assert {m["name"] for m in client.get("/api/tags").json()["models"]} == {"tiny:latest", "tiny2:latest"}
    assert client.request("DELETE", "/api/delete", json={"model": "tiny2"}).status_code == 200
    assert client.request("DELETE", "/api/delete", json={"model": "tiny2"}).status_code == 404
    m = client.get("/metrics").text
    assert "omx_generated_tokens_total" in m


def test_create_from_modelfile(client, tiny_models):
    mf = f"FROM {tiny_models['tiny-phi2']}\nSYSTEM you are terse\nPARAMETER temperature 0.3\n"
    r = client.post("/api/create", json={"model": "phi-custom", "modelfile": mf, "stream": False})
    assert r.status_code == 200, r.text
    d = client.post("/api/show", json={"model": "phi-custom"}).json()
    assert "you are terse" in d["modelfile"] and "temperature" in d["parameters"]
    assert d["details"]["family"] == "phi2"
    # derive from an existing model
    r = client.post("/api/create", json={"model": "phi-custom2", "from": "phi-custom", "system": "other"})
    assert r.status_code == 200
    assert "other" in client.post("/api/show", json={"model": "phi-custom2"}).json()["modelfile"]


def test_concurrent_generate_batched(client):
    """OLLAMA_NUM_PARALLEL (default 4): concurrent requests share batched decode steps and return what
    each returns alone (greedy)."""
    import threading
    prompts = ["alpha beta", "the quick brown fox", "one two three four five", "zz"]
    body = lambda p: {"model": "tiny", "prompt": p, "stream": False,  # noqa: E731
                      "options": {"num_predict": 10, "temperature": 0}}
    alone = [client.post("/api/generate", json=body(p)).json()["response"] for p in prompts]
    got = [None] * len(prompts)

    def work(i):
        got[i] = client.post("/api/generate", json=body(prompts[i])).json()["response"]

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(prompts))]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert got == alone


@pytest.mark.parametrize("parallel", ["1", "4"])
def test_engine_fault_injection(tmp_path, tiny_models, monkeypatch, parallel):
    """A decode step that fails mid-generation (injected, as a HIP error would) answers that request
    with Ollama's {"error"} / 500; the model stays loaded and the next request matches a clean run."""
    monkeypatch.setenv("OLLAMA_NUM_PARALLEL", parallel)
    st = ModelStore(str(tmp_path / "store"))
    st.create("tiny", gguf_path=tiny_models["tiny-llama"], params={"temperature": 0.0, "num_ctx": 128})
    mgr = ModelManager(st, device="cpu")
    c = TestClient(create_app(st, mgr), raise_server_exceptions=False)
    body = {"model": "tiny", "prompt": "alpha beta gamma", "stream": False, "options": {"num_predict": 8}}
    clean = c.post("/api/generate", json=body).json()["response"]
    runner = mgr.get("tiny").runner
    real = runner.decode_batch
    calls = {"n": 0}

    def flaky(*a, **k):
        calls["n"] += 1
        if calls["n"] == 3:
            raise RuntimeError("injected: no free KV blocks")
        return real(*a, **k)

    monkeypatch.setattr(runner, "decode_batch", flaky)
    r = c.post("/api/generate", json=body)
    assert r.status_code == 500 and "injected" in r.json()["error"]
    again = c.post("/api/generate", json=body)
    assert again.status_code == 200 and again.json()["response"] == clean
    assert mgr.get("tiny").runner is runner  # not reloaded: the failure stayed with its request


def test_device_fault_exits_process(tmp_path, tiny_models, monkeypatch):
    """A HIP runtime fault is not recoverable in-process: the request gets {"error"} / 500 and the
    server's device-fault hook (default: exit 70 -> Kubernetes restarts the pod) fires."""
    monkeypatch.setenv("OLLAMA_NUM_PARALLEL", "1")
    st = ModelStore(str(tmp_path / "store"))
    st.create("tiny", gguf_path=tiny_models["tiny-llama"], params={"temperature": 0.0, "num_ctx": 128})
    mgr = ModelManager(st, device="cpu")
    app = create_app(st, mgr)
    fired = []
    app.state.on_device_fault = lambda: fired.append(1)
    c = TestClient(app, raise_server_exceptions=False)
    runner = mgr.get("tiny").runner

    def broken(*a, **k):
        raise RuntimeError("HIP error: an illegal memory access was encountered")

    monkeypatch.setattr(runner, "decode_batch", broken)
    r = c.post("/api/generate", json={"model": "tiny", "prompt": "x", "stream": False, "options": {"num_predict": 4}})
    assert r.status_code == 500 and "HIP error" in r.json()["error"]
    assert fired == [1]


def test_engine_fault_mid_stream(tmp_path, tiny_models, monkeypatch):
    """Streaming: an engine failure ends the NDJSON stream with an {"error"} line, as Ollama does."""
    monkeypatch.setenv("OLLAMA_NUM_PARALLEL", "1")
    st = ModelStore(str(tmp_path / "store"))
    st.create("tiny", gguf_path=tiny_models["tiny-llama"], params={"temperature": 0.0, "num_ctx": 128})
    mgr = ModelManager(st, device="cpu")
    c = TestClient(create_app(st, mgr), raise_server_exceptions=False)
    runner = mgr.get("tiny").runner
    real, calls = runner.decode_batch, {"n": 0}

    def flaky(*a, **k):
        calls["n"] += 1
        if calls["n"] == 4:
            raise RuntimeError("injected fault")
        return real(*a, **k)

    monkeypatch.setattr(runner, "decode_batch", flaky)
    lines = [json.loads(x) for x in c.post("/api/generate", json={"model": "tiny", "prompt": "a b c",
                                                                  "options": {"num_predict": 12}}).iter_lines() if x]
    assert "injected fault" in lines[-1]["error"]
    assert not any(x.get("done") for x in lines)
