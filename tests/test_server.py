"""The llama-server-compatible HTTP front end (llmi/server.py) against the wire
contract the reference's gateway relies on: /health 503 -> 200,
Bearer auth on /v1/*, OpenAI-shaped non-stream bodies with usage, SSE `data:` events
ending in `data: [DONE]`, Connection: close, --version exit 0.  The engine is a
deterministic stand-in here (no GPU); tests/test_gpu_server.py drives the real one."""
from __future__ import annotations

import http.client
import json
import os
import subprocess
import sys
import threading

import pytest

from llmi.server import Vocab, chat_prompt, make_server

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEY = "gateway-test-key"


class FakeEngine:
    def __init__(self):
        pieces = ["<unk>", "<s>", "</s>"] + [f" w{i}" for i in range(3, 100)]
        self.vocab = Vocab(pieces, 1, 2)
        self.ready = False
        self.error = None
        self.model_id = "fake.gguf"
        self.n_ctx = 256
        self.calls = []

    def generate(self, prompt, max_tokens, ignore_eos, on_tokens, chunk=8, sampling=None, stop=None):
        self.calls.append((list(prompt), max_tokens, ignore_eos))
        self.last_sampling, self.last_stop = sampling, stop
        out = []
        t = prompt[-1]
        while len(out) < max_tokens:
            t = 3 + (t * 7 + 1) % 97
            if t == 50 and not ignore_eos:
                return out, "stop"
            out.append(t)
            on_tokens([t])
        return out, "length"


@pytest.fixture()
def server():
    eng = FakeEngine()
    srv = make_server(eng, "127.0.0.1", 0, KEY)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    yield eng, srv.server_address[1]
    srv.shutdown()
    srv.server_close()


def req(port, method, path, body=None, auth=True, headers=None):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    h = {"Connection": "close", "content-type": "application/json"}
    if auth:
        h["Authorization"] = f"Bearer {KEY}"
    h.update(headers or {})
    data = json.dumps(body).encode() if body is not None else None
    c.request(method, path, body=data, headers=h)
    r = c.getresponse()
    raw = r.read()
    c.close()
    return r, raw


def test_health_loading_then_ok(server):
    eng, port = server
    r, raw = req(port, "GET", "/health", auth=False)
    assert r.status == 503
    eng.ready = True
    for auth in (False, True):
        r, raw = req(port, "GET", "/health", auth=auth)
        assert r.status == 200 and json.loads(raw) == {"status": "ok"}
        assert r.getheader("Connection") == "close"


def test_auth_required_on_v1(server):
    eng, port = server
    eng.ready = True
    r, raw = req(port, "POST", "/v1/completions", {"prompt": [1, 5]}, auth=False)
    assert r.status == 401 and json.loads(raw)["error"]["code"] == 401
    r, raw = req(port, "GET", "/v1/models", auth=False)
    assert r.status == 401
    r, raw = req(port, "POST", "/v1/completions", {"prompt": [1, 5]},
                 headers={"Authorization": "Bearer wrong"})
    assert r.status == 401
    # llama-server's non-/v1 completion route is not public either (only /health is)
    r, raw = req(port, "POST", "/completion", {"prompt": [1, 5]}, auth=False)
    assert r.status == 401
    r, raw = req(port, "POST", "/completion", {"prompt": [1, 5], "max_tokens": 2})
    assert r.status == 200
    r, raw = req(port, "GET", "/v1/health", auth=False)
    assert r.status == 200


def test_decode_failure_is_json_500(server):
    """A failing llama_decode inside generate() answers an OpenAI-shaped 500 (non-stream)
    or an error event before the close (SSE), never a dropped connection."""
    eng, port = server
    eng.ready = True

    def boom(*a, **k):
        raise RuntimeError("llama_decode returned -4")

    eng.generate = boom
    r, raw = req(port, "POST", "/v1/completions", {"prompt": [1, 5], "max_tokens": 3})
    d = json.loads(raw)
    assert r.status == 500 and d["error"]["type"] == "server_error" and "-4" in d["error"]["message"]
    r, raw = req(port, "POST", "/v1/completions", {"prompt": [1, 5], "max_tokens": 3, "stream": True})
    events = [e for e in raw.decode().split("\n\n") if e]
    assert r.status == 200 and json.loads(events[-1][6:])["error"]["code"] == 500


def test_embeddings_not_supported(server):
    """/v1/embeddings (docs/API_REFERENCE.md:537-590) exists only when llama-server runs
    with embedding support, which the reference's start.sh does not pass: the answer is
    upstream's 501 not_supported_error, behind the same auth as every /v1 route."""
    eng, port = server
    eng.ready = True
    r, raw = req(port, "POST", "/v1/embeddings", {"model": "any", "input": "Hello world"}, auth=False)
    assert r.status == 401
    for path in ("/v1/embeddings", "/embeddings"):
        r, raw = req(port, "POST", path, {"model": "any", "input": ["a", "b"]})
        err = json.loads(raw)["error"]
        assert r.status == 501 and err["code"] == 501 and err["type"] == "not_supported_error"
        assert "--embeddings" in err["message"]


def test_models(server):
    eng, port = server
    eng.ready = True
    r, raw = req(port, "GET", "/v1/models")
    d = json.loads(raw)
    assert r.status == 200 and d["object"] == "list" and d["data"][0]["id"] == "fake.gguf"


def test_completion_token_ids_non_stream(server):
    eng, port = server
    eng.ready = True
    r, raw = req(port, "POST", "/v1/completions", {"prompt": [1, 5, 9], "max_tokens": 6, "ignore_eos": True})
    d = json.loads(raw)
    assert r.status == 200 and d["object"] == "text_completion"
    assert eng.calls[-1] == ([1, 5, 9], 6, True)
    ids = d["llmi"]["tokens"]
    assert len(ids) == 6 and d["choices"][0]["text"] == "".join(f" w{i}" for i in ids)
    assert d["usage"] == {"prompt_tokens": 3, "completion_tokens": 6, "total_tokens": 9}
    assert d["choices"][0]["finish_reason"] == "length"


def test_text_prompt_tokenized(server):
    eng, port = server
    eng.ready = True
    r, raw = req(port, "POST", "/v1/completions", {"prompt": " w7 w12 w3", "max_tokens": 2})
    assert r.status == 200
    assert eng.calls[-1][0] == [1, 7, 12, 3]


def test_chat_stream_sse(server):
    eng, port = server
    eng.ready = True
    r, raw = req(port, "POST", "/v1/chat/completions",
                 {"messages": [{"role": "user", "content": " w5 w6"}], "max_tokens": 5, "stream": True,
                  "ignore_eos": True})
    assert r.status == 200 and r.getheader("Content-Type") == "text/event-stream"
    assert r.getheader("Connection") == "close"
    events = [ln for ln in raw.decode().split("\n\n") if ln]
    assert all(e.startswith("data: ") for e in events) and events[-1] == "data: [DONE]"
    chunks = [json.loads(e[6:]) for e in events[:-1]]
    assert chunks[0]["choices"][0]["delta"] == {"role": "assistant"}
    content = [c["choices"][0]["delta"].get("content") for c in chunks[1:-1]]
    assert len(content) == 5 and all(content)
    assert chunks[-1]["choices"][0]["finish_reason"] == "length"
    assert chunks[-1]["usage"]["completion_tokens"] == 5


def test_chat_non_stream_shape(server):
    eng, port = server
    eng.ready = True
    r, raw = req(port, "POST", "/v1/chat/completions", {"messages": [{"role": "user", "content": "hi"}],
                                                        "max_tokens": 3})
    d = json.loads(raw)
    assert d["object"] == "chat.completion" and d["choices"][0]["message"]["role"] == "assistant"
    assert set(d["usage"]) == {"prompt_tokens", "completion_tokens", "total_tokens"}


def test_bad_requests(server):
    eng, port = server
    eng.ready = True
    r, raw = req(port, "POST", "/v1/chat/completions", {"messages": []})
    assert r.status == 400 and json.loads(raw)["error"]["type"] == "invalid_request_error"
    r, raw = req(port, "POST", "/v1/completions", {"prompt": [1, 10 ** 6]})
    assert r.status == 400
    r, raw = req(port, "GET", "/v1/nothing")
    assert r.status == 404


def test_eos_stops(server):
    eng, port = server
    eng.ready = True
    # the fake engine emits token 50 as EOS for some prompt; find one that reaches it
    for p in range(3, 100):
        r, raw = req(port, "POST", "/v1/completions", {"prompt": [1, p], "max_tokens": 40})
        d = json.loads(raw)
        if d["choices"][0]["finish_reason"] == "stop":
            assert 50 not in d["llmi"]["tokens"]
            return
    pytest.fail("no prompt reached the stand-in EOS")


def test_vocab_and_template():
    v = Vocab(["<unk>", "<s>", "</s>", "▁hello", "▁world", "<0x0A>", "!"], 1, 2)
    assert v.tokenize(" hello world!", add_bos=False) == [3, 4, 6]
    assert v.detokenize([1, 3, 4, 5, 2]) == " hello world\n"
    assert chat_prompt([{"role": "user", "content": "x"}], v).endswith("assistant:")


def test_version_and_argv():
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "llama-gguf-inference_amd"))
    out = subprocess.run([os.path.join(ROOT, "llama-gguf-inference_amd", "bin", "llama-server"), "--version"],
                         capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0 and "llmi" in out.stdout
    from llmi.server import parse_args

    a, extra = parse_args(["-m", "/m.gguf", "--host", "127.0.0.1", "--port", "18080", "-c", "16384", "-ngl", "99",
                           "--api-key-file", "/k", "-t", "8", "--flash-attn"])
    assert (a.model, a.port, a.ctx_size, a.ngl, a.api_key_file, a.threads) == ("/m.gguf", 18080, 16384, 99, "/k", 8)
    assert extra == ["--flash-attn"]


def test_numerics_env_validated(monkeypatch):
    """LLMI_NUMERICS is checked like --numerics' choices (argparse does not check a
    default): case-folded, and an unknown value is an error, never a silent generic."""
    from llmi.server import parse_args

    monkeypatch.setenv("LLMI_NUMERICS", "X86")
    assert parse_args(["-m", "/m.gguf"])[0].numerics == "x86"
    monkeypatch.setenv("LLMI_NUMERICS", "1")
    with pytest.raises(SystemExit):
        parse_args(["-m", "/m.gguf"])
    assert parse_args(["-m", "/m.gguf", "--numerics", "generic"])[0].numerics == "generic"
    monkeypatch.delenv("LLMI_NUMERICS")
    assert parse_args(["-m", "/m.gguf"])[0].numerics == "generic"
    from llmi.server import numerics_value

    assert [numerics_value(n) for n in ("generic", "x86", "generic-fa", "x86-fa")] == [0, 1, 2, 3]
    assert parse_args(["-m", "/m.gguf", "--numerics", "x86-fa"])[0].numerics == "x86-fa"


def test_gateway_forwarded_bytes(server):
    """The exact request shape the reference gateway forwards (SURVEY.md §8b capture of
    scripts/gateway.py:721-745: lowercase client headers, backend Bearer key, Connection:
    close) sent as raw bytes; the response is status line + headers + body and the
    server closes the socket (the gateway copies until EOF, gateway.py:776-783)."""
    import socket

    eng, port = server
    eng.ready = True
    body = json.dumps({"messages": [{"role": "user", "content": "Write a short poem about the sea"}],
                       "max_tokens": 4, "stream": True}).encode()
    head = (f"POST /v1/chat/completions HTTP/1.1\r\nHost: 127.0.0.1:{port}\r\n"
            f"content-type: application/json\r\ncontent-length: {len(body)}\r\n"
            f"Authorization: Bearer {KEY}\r\nConnection: close\r\n\r\n").encode()
    s = socket.create_connection(("127.0.0.1", port), timeout=10)
    s.sendall(head + body)
    chunks = []
    while True:
        b = s.recv(65536)
        if not b:
            break  # server closed: EOF delimits the response
        chunks.append(b)
    s.close()
    raw = b"".join(chunks).decode()
    status, rest = raw.split("\r\n", 1)
    assert status == "HTTP/1.1 200 OK"
    hdr, payload = rest.split("\r\n\r\n", 1)
    assert len(hdr) < 64 * 1024  # gateway header-block limit (gateway.py:123)
    assert "Content-Type: text/event-stream" in hdr and "Connection: close" in hdr
    events = [e for e in payload.split("\n\n") if e]
    assert events[-1] == "data: [DONE]" and all(e.startswith("data: ") for e in events)
