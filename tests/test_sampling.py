"""The HTTP front end's sampling and stop strings (llmi/sampling.py, llmi/server.py),
against llama-server's sampler chain as documented for the reference's API
(docs/API_REFERENCE.md:363-379: temperature, top_p, frequency/presence penalty, stop).
CPU only: the sampler works on host logits; tests/test_gpu_server.py drives it on a GPU."""
from __future__ import annotations

import json

import numpy as np
import pytest

from llmi.sampling import Sampler, SamplingParams, StopFilter, find_stop, parse_stop


def _draws(params, logits, n=400, history=()):
    s = Sampler(params)
    return [s.sample(logits, list(history)) for _ in range(n)]


def test_defaults_are_llama_servers():
    p = SamplingParams()
    assert (p.temperature, p.top_k, p.top_p, p.min_p, p.repeat_penalty, p.repeat_last_n) == (0.8, 40, 0.95, 0.05, 1.0, 64)
    assert not p.greedy
    assert SamplingParams(temperature=0.0).greedy and SamplingParams(top_k=1).greedy
    assert not SamplingParams(temperature=0.0, repeat_penalty=1.1).greedy  # penalties need the host logits


def test_temperature_zero_is_argmax_first_max_wins():
    lg = np.array([0.5, 2.0, 2.0, -1.0], np.float32)
    assert set(_draws(SamplingParams(temperature=0.0), lg, 20)) == {1}


def test_top_k_limits_support():
    rng = np.random.default_rng(0)
    lg = rng.standard_normal(1000).astype(np.float32)
    top3 = set(np.argsort(-lg)[:3].tolist())
    got = set(_draws(SamplingParams(temperature=5.0, top_k=3, top_p=1.0, min_p=0.0, seed=1), lg))
    assert got <= top3 and len(got) == 3


def test_top_p_keeps_smallest_prefix_reaching_p():
    lg = np.log(np.array([0.5, 0.3, 0.15, 0.05], np.float32))
    # p = 0.75: 0.5 + 0.3 reaches it -> tokens {0, 1}
    got = set(_draws(SamplingParams(temperature=1.0, top_k=0, top_p=0.75, min_p=0.0, seed=2), lg))
    assert got == {0, 1}
    got = set(_draws(SamplingParams(temperature=1.0, top_k=0, top_p=0.5, min_p=0.0, seed=2), lg))
    assert got == {0}


def test_min_p_relative_to_max():
    lg = np.log(np.array([0.6, 0.3, 0.07, 0.03], np.float32))
    # min_p 0.1: keep p >= 0.06 -> {0, 1, 2}
    got = set(_draws(SamplingParams(temperature=1.0, top_k=0, top_p=1.0, min_p=0.1, seed=3), lg, 2000))
    assert got == {0, 1, 2}


def test_penalties_follow_llama_cpp():
    lg = np.array([3.0, 2.9, -1.0, 0.5], np.float32)
    # repeat penalty divides a positive logit, multiplies a negative one: token 0 repeated
    p = SamplingParams(temperature=0.0, repeat_penalty=1.5)
    assert Sampler(p).sample(lg, [0]) == 1
    # frequency penalty scales with the count, presence is flat
    p = SamplingParams(temperature=0.0, frequency_penalty=0.06)
    assert Sampler(p).sample(lg, [0]) == 0 and Sampler(p).sample(lg, [0, 0]) == 1
    p = SamplingParams(temperature=0.0, presence_penalty=0.2)
    assert Sampler(p).sample(lg, [0, 0, 0]) == 1
    # only the last repeat_last_n tokens count
    p = SamplingParams(temperature=0.0, repeat_penalty=1.5, repeat_last_n=1)
    assert Sampler(p).sample(lg, [0, 3]) == 0


def test_seed_reproducible_and_distribution_sane():
    lg = np.log(np.array([0.5, 0.25, 0.25], np.float32))
    p = SamplingParams(temperature=1.0, top_k=0, top_p=1.0, min_p=0.0, seed=1234)
    a, b = _draws(p, lg, 2000), _draws(p, lg, 2000)
    assert a == b
    freq = np.bincount(a, minlength=3) / len(a)
    assert abs(freq[0] - 0.5) < 0.05 and abs(freq[1] - 0.25) < 0.05


def test_request_overrides_and_validation():
    d = SamplingParams()
    p = d.with_request({"temperature": 0.2, "top_p": 0.5, "seed": 7, "frequency_penalty": 1.0})
    assert (p.temperature, p.top_p, p.seed, p.frequency_penalty, p.top_k) == (0.2, 0.5, 7, 1.0, 40)
    for bad in ({"temperature": -1}, {"top_p": 1.5}, {"presence_penalty": 3.0}, {"temperature": "hot"},
                {"top_k": True}):
        with pytest.raises(ValueError):
            d.with_request(bad)


def test_stop_helpers():
    assert parse_stop(None) == [] and parse_stop("x") == ["x"] and parse_stop(["a", "b"]) == ["a", "b"]
    with pytest.raises(ValueError):
        parse_stop([1])
    assert find_stop("hello world", ["wor", "lo"]) == 3
    f = StopFilter(["END"])
    out = f.push("abc E") + f.push("N") + f.push("D tail")
    assert out == "abc " and f.stopped and f.flush() == ""
    f = StopFilter(["END"])  # no stop: everything comes out, a possible stop prefix only later
    assert f.push("abc EN") == "abc "
    assert f.push("x") + f.flush() == "ENx" and not f.stopped


# ---- through the HTTP front end (stand-in engine with logits) --------------------------
class _LogitCtx:
    """llmi.Context stand-in: logits = a fixed function of the last token."""

    V = 64

    def __init__(self):
        self.last = {}
        self.batch = []

    def seq_rm(self, seq, p0=0, p1=-1):
        return True

    def _lg(self, t):
        lg = np.full(self.V, -5.0, np.float32)
        lg[(t * 5 + 3) % self.V] = 2.0
        lg[(t * 7 + 1) % self.V] = 1.5
        lg[(t * 11 + 2) % self.V] = 1.0
        return lg

    def decode(self, tokens, pos=None, logits_all=False, seq=None):
        self.batch = list(tokens) if logits_all else [tokens[-1]]
        return 0

    def logits(self, i=-1):
        return self._lg(self.batch[i])

    def greedy(self, i=-1):
        return int(np.argmax(self.logits(i)))

    def generate_greedy_batch(self, seqs, first, pos0, n):
        outs = []
        for f in first:
            t, o = f, []
            for _ in range(n):
                t = int(np.argmax(self._lg(t)))
                o.append(t)
            outs.append(o)
        return outs

    def stats(self):
        return 1.0, 1.0


@pytest.fixture()
def server():
    import http.client
    import threading

    from llmi.server import Engine, Vocab, make_server

    vocab = Vocab(["<unk>", "<s>", "</s>"] + [f" w{i}" for i in range(3, _LogitCtx.V)], 1, 2)
    eng = Engine("fake.gguf", 256, 99, [0], slots=4, chunk=4, contexts=([_LogitCtx()], vocab))
    eng.load()
    srv = make_server(eng, "127.0.0.1", 0, None)
    threading.Thread(target=srv.serve_forever, daemon=True).start()

    def post(body):
        c = http.client.HTTPConnection("127.0.0.1", srv.server_address[1], timeout=30)
        c.request("POST", "/v1/completions", body=json.dumps(body).encode(),
                  headers={"content-type": "application/json", "Connection": "close"})
        r = c.getresponse()
        raw = r.read()
        c.close()
        return r.status, raw

    yield eng, post
    srv.shutdown()
    srv.server_close()


def test_http_greedy_vs_sampled(server):
    eng, post = server
    st, raw = post({"prompt": [1, 9], "max_tokens": 12, "temperature": 0, "ignore_eos": True})
    greedy = json.loads(raw)["llmi"]["tokens"]
    assert st == 200 and len(greedy) == 12
    seeded = [json.loads(post({"prompt": [1, 9], "max_tokens": 12, "temperature": 1.5, "top_k": 0, "top_p": 1.0,
                               "min_p": 0.0, "seed": 5, "ignore_eos": True})[1])["llmi"]["tokens"] for _ in range(2)]
    assert seeded[0] == seeded[1] and seeded[0] != greedy
    # no temperature field: llama-server's default chain (temperature 0.8), still valid tokens
    st, raw = post({"prompt": [1, 9], "max_tokens": 8, "ignore_eos": True})
    assert st == 200 and all(0 <= t < _LogitCtx.V for t in json.loads(raw)["llmi"]["tokens"])


def test_http_stop_string_and_bad_fields(server):
    eng, post = server
    st, raw = post({"prompt": [1, 9], "max_tokens": 12, "temperature": 0, "ignore_eos": True})
    full = json.loads(raw)["choices"][0]["text"]
    words = full.split(" ")
    stop = " " + words[3]
    st, raw = post({"prompt": [1, 9], "max_tokens": 12, "temperature": 0, "ignore_eos": True, "stop": stop})
    d = json.loads(raw)
    assert st == 200 and d["choices"][0]["finish_reason"] == "stop"
    assert d["choices"][0]["text"] == full[:full.find(stop)]
    # streamed: the same text, the stop string never sent
    st, raw = post({"prompt": [1, 9], "max_tokens": 12, "temperature": 0, "ignore_eos": True, "stop": [stop],
                    "stream": True})
    events = [json.loads(e[6:]) for e in raw.decode().split("\n\n") if e.startswith("data: {")]
    assert "".join(e["choices"][0]["text"] for e in events) == full[:full.find(stop)]
    assert events[-1]["choices"][0]["finish_reason"] == "stop"
    for bad in ({"temperature": -0.5}, {"top_p": 2}, {"n": 2}, {"logprobs": 5}, {"stop": [3]}):
        st, raw = post({"prompt": [1, 9], "max_tokens": 4, **bad})
        assert st == 400 and "error" in json.loads(raw), bad
