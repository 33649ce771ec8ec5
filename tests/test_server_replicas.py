"""Replica serving without GPUs: the server's least-loaded router
and per-replica continuous-batching scheduler (llmi/server.py Engine / Replica) over
stand-in contexts with the llmi.Context decode surface, and the `--replicas N` wiring
of llmi_model_load_replicated checked with a stand-in llmi module.

Each stand-in context computes a deterministic per-sequence recurrence, so every
request's tokens can be checked against a reference no matter how requests were
batched together or interleaved."""
from __future__ import annotations

import http.client
import json
import threading
import time

import pytest

from llmi.sampling import SamplingParams
from llmi.server import Engine, Vocab, make_server

V = 100


def nxt(t: int, pos: int) -> int:
    return 3 + (t * 7 + pos * 3 + 1) % (V - 3)


def reference(prompt, n):
    """What one sequence alone produces: first token from the prompt, then the recurrence."""
    t = nxt(prompt[-1], len(prompt) - 1)
    out, pos = [t], len(prompt)
    while len(out) < n:
        t = nxt(t, pos)
        out.append(t)
        pos += 1
    return out


class FakeCtx:
    """llmi.Context stand-in: per-sequence state, batched and single decode calls."""

    def __init__(self, n_ctx=512, delay=0.002):
        self.n_ctx, self.delay = n_ctx, delay
        self.last_tok = {}
        self.batch_sizes = []
        self.prefills = 0
        self.lock = threading.Lock()

    def seq_rm(self, seq, p0=0, p1=-1):
        return True

    def decode(self, tokens, pos=None, logits_all=False, seq=None):
        with self.lock:
            self.prefills += 1
        time.sleep(self.delay)
        self._g = nxt(tokens[-1], len(tokens) - 1)
        return 0

    def greedy(self, i=-1):
        return self._g

    def generate_greedy_batch(self, seqs, first, pos0, n):
        assert len(seqs) == len(set(seqs)) and len(seqs) <= 8
        self.batch_sizes.append(len(seqs))
        time.sleep(self.delay)
        outs = []
        for f, p in zip(first, pos0):
            t, o = f, []
            for k in range(n):
                t = nxt(t, p + k)
                o.append(t)
            outs.append(o)
        return outs

    def stats(self):
        return 4.9e9, 1700.0


def _engine(n_rep, slots, delay=0.002):
    vocab = Vocab(["<unk>", "<s>", "</s>"] + [f" w{i}" for i in range(3, V)], 1, 2)
    ctxs = [FakeCtx(delay=delay) for _ in range(n_rep)]
    # the server started with --temp 0 (greedy by default; per-request fields still override)
    eng = Engine("fake.gguf", 512, 99, list(range(n_rep)), slots=slots, chunk=4, contexts=(ctxs, vocab),
                 sampling=SamplingParams(temperature=0.0))
    eng.load()
    assert eng.ready, eng.error
    return eng, ctxs


def _post(port, body):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    c.request("POST", "/v1/completions", body=json.dumps(body).encode(),
              headers={"Connection": "close", "content-type": "application/json"})
    r = c.getresponse()
    raw = r.read()
    c.close()
    return r.status, json.loads(raw)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("n_rep,slots", [(3, 4), (1, 4), (2, 1)])
def test_concurrent_requests_least_loaded(n_rep, slots):
    eng, ctxs = _engine(n_rep, slots)
    srv = make_server(eng, "127.0.0.1", 0, None)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    port = srv.server_address[1]
    prompts = [[1, 3 + i, 10 + 2 * i] for i in range(8)]
    n_tok = [20 + 3 * i for i in range(8)]
    res = [None] * 8

    def one(i):
        res[i] = _post(port, {"prompt": prompts[i], "max_tokens": n_tok[i], "ignore_eos": True})

    ths = [threading.Thread(target=one, args=(i,)) for i in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    try:
        for i in range(8):
            st, d = res[i]
            assert st == 200, d
            assert d["llmi"]["tokens"] == reference(prompts[i], n_tok[i]), f"request {i}"
            assert d["choices"][0]["finish_reason"] == "length"
        reps = [r.requests for r in eng.replicas]
        assert sum(reps) == 8
        # least loaded: with 8 requests in flight every replica got a share
        assert min(reps) >= 8 // n_rep - 1, reps
        if slots > 1:  # requests shared batched decode steps
            assert max(max(c.batch_sizes or [0]) for c in ctxs) >= 2
        else:
            assert all(b == 1 for c in ctxs for b in c.batch_sizes)
        h = eng.health()
        assert h["slots_processing"] == 0 and h["slots_idle"] == slots * n_rep
        assert sum(r["tokens"] for r in h["replicas"]) == sum(n_tok)
        assert all(r["hbm_gbps"] > 0 for r in h["replicas"] if r["tokens"])
    finally:
        srv.shutdown()
        srv.server_close()


@pytest.mark.timeout(120)
def test_no_starvation_more_requests_than_slots():
    """12 requests through one replica with 2 slots: admission waits for a free slot,
    every request completes with its own tokens (none starves behind long ones)."""
    eng, ctxs = _engine(1, 2)
    reqs = [eng.submit([1, 5 + i], 6 if i % 3 else 40, True) for i in range(12)]
    t0 = time.time()
    for r in reqs:
        while r.finish is None and r.error is None:
            assert time.time() - t0 < 60
            time.sleep(0.005)
    for i, r in enumerate(reqs):
        assert r.error is None and r.out == reference([1, 5 + i], 6 if i % 3 else 40)
    assert max(ctxs[0].batch_sizes) == 2


def test_eos_and_health_json_size():
    vocab = Vocab(["<unk>", "<s>", "</s>"] + [f" w{i}" for i in range(3, V)], 1, 50)  # token 50 ends generation
    eng = Engine("fake.gguf", 512, 99, list(range(16)), slots=8,
                 contexts=([FakeCtx() for _ in range(16)], vocab))
    eng.load()
    # the gateway reads 4096 bytes of /health (scripts/gateway.py:350)
    assert len(json.dumps({"status": "ok", **eng.health()})) < 3500
    # EOS: a prompt whose recurrence reaches token 50 stops there, without emitting it
    for p in range(3, V):
        ref = reference([1, p], 60)
        if 50 in ref:
            r = eng.submit([1, p], 60, False)
            t0 = time.time()
            while r.finish is None:
                assert time.time() - t0 < 30
                time.sleep(0.01)
            assert r.finish == "stop" and r.out == ref[:ref.index(50)]
            return
    pytest.skip("no prompt reaches the stand-in EOS")


def test_replicas_flag_wires_llmi_replicate(tmp_path, monkeypatch):
    """`--replicas 3` -> Model.load_replicated(path, 0, [1, 2]) (llmi_model_load_replicated:
    the in-process RCCL broadcast pipelined behind the upload), one Context per replica
    with the slot count as n_seq."""
    import llmi as real

    path = str(tmp_path / "t.gguf")
    real.write_synthetic_gguf(path, "tiny-mixed", seed=1)
    log = []

    class M:
        def __init__(self, p, n_gpu_layers=999, main_gpu=0, **k):
            log.append(("model", p, main_gpu))
            self.n_vocab, self.bos, self.eos = 1000, 1, 2

        @classmethod
        def load_replicated(cls, p, main_gpu, devices, **k):
            log.append(("load_replicated", p, main_gpu, list(devices)))
            m = cls.__new__(cls)
            m.n_vocab, m.bos, m.eos = 1000, 1, 2
            return m, [cls.__new__(cls) for _ in devices]

        def token_text(self, i):
            return f" w{i}"

    class C:
        def __init__(self, m, n_ctx=0, n_seq=1, **k):
            log.append(("context", n_ctx, n_seq))
            self.n_ctx = n_ctx

    monkeypatch.setattr(real, "Model", M)
    monkeypatch.setattr(real, "Context", C)

    eng = Engine(path, 256, 99, [0, 1, 2], slots=3)
    eng.load()
    assert eng.ready, eng.error
    assert log[0] == ("load_replicated", path, 0, [1, 2])
    assert log[1:] == [("context", 256, 3)] * 3
    assert [r.device for r in eng.replicas] == [0, 1, 2]
    assert eng.vocab.tok.kind == "greedy" and eng.vocab.tokenize(" w5") == [1, 5]
    for r in eng.replicas:
        r.stop = True
