"""The HTTP front end driving the real HIP path: token ids through /v1/completions
(non-stream and SSE) equal a direct greedy decode through the C ABI."""
from __future__ import annotations

import http.client
import json
import threading

import pytest

import llmi
from llmi.server import Engine, make_server

pytestmark = pytest.mark.gpu


def test_server_matches_direct_decode(gpu, tiny_models):
    path = tiny_models["tiny-mixed"]
    prompt, n = [1, 17, 300, 42], 20
    m = llmi.Model(path)
    c = llmi.Context(m, n_ctx=128)
    assert c.decode(prompt) == 0
    first = c.greedy(-1)
    want = [first] + c.generate_greedy(first, len(prompt), n - 1)

    eng = Engine(path, 128, 99, [0])
    eng.load()
    assert eng.ready, eng.error
    srv = make_server(eng, "127.0.0.1", 0, None)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    port = srv.server_address[1]
    try:
        for stream in (False, True):
            conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
            conn.request("POST", "/v1/completions", body=json.dumps(
                {"prompt": prompt, "max_tokens": n, "ignore_eos": True, "stream": stream, "temperature": 0}),
                headers={"content-type": "application/json", "Connection": "close"})
            r = conn.getresponse()
            raw = r.read().decode()
            conn.close()
            assert r.status == 200
            if not stream:
                got = json.loads(raw)["llmi"]["tokens"]
                assert got == want
            else:
                events = [e for e in raw.split("\n\n") if e]
                text = "".join(json.loads(e[6:])["choices"][0]["text"] for e in events[:-1])
                assert text == "".join(m.token_text(t) for t in want)
        # sampled (llama-server's chain on the host logits): a fixed seed reproduces, and
        # top_p -> 0 (only the most likely token kept) equals greedy through the sampled
        # path's per-token batched steps
        outs = []
        for body in ({"temperature": 1.0, "seed": 11}, {"temperature": 1.0, "seed": 11},
                     {"temperature": 1.0, "top_k": 0, "top_p": 1e-6, "min_p": 0.0}):
            conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
            conn.request("POST", "/v1/completions", body=json.dumps(
                {"prompt": prompt, "max_tokens": n, "ignore_eos": True, **body}),
                headers={"content-type": "application/json", "Connection": "close"})
            r = conn.getresponse()
            outs.append(json.loads(r.read())["llmi"]["tokens"])
            conn.close()
        assert outs[0] == outs[1] and len(outs[0]) == n
        assert outs[2] == want
    finally:
        srv.shutdown()
        srv.server_close()
