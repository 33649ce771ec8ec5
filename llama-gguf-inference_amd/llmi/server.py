"""llama-server-compatible HTTP front end over libllmi.so.

The reference launches `/app/llama-server -m PATH --host 127.0.0.1 --port N -c CTX
-ngl NGL --api-key-file FILE [-t THREADS] [EXTRA...]` (scripts/start.sh:473-494),
probes `GET /health` (scripts/start.sh:600-635, scripts/gateway.py:326-376) and
proxies `/v1/*` to it (scripts/gateway.py:699-804).  The gateway sends one request per
TCP connection with `Connection: close` and copies the response until EOF.  This
module answers that contract:

  GET  /health                 200 {"status":"ok"} when ready, 503 while loading (no auth)
  GET  /v1/models              OpenAI model list
  POST /v1/completions         prompt: str | [token ids]; non-stream or SSE
  POST /v1/chat/completions    messages -> chat template -> tokens; non-stream or SSE
  POST /v1/embeddings          501 not_supported_error (the reference starts llama-server
                               without embedding support)
  Authorization: Bearer <key> required on every route but /health when a key is
  configured (401 otherwise; llama-server's public endpoints are /health and /v1/health)

  GET /health adds per-replica serving metrics: active/queued requests, generated
  tokens, tok/s over decode time, HBM GB/s of the last decode call (the gateway passes
  the body through, scripts/gateway.py:360-363)

Sampling follows llama-server (llmi/sampling.py): temperature / top_k / top_p / min_p /
repeat, presence and frequency penalties / seed per request, llama-server's defaults
(temperature 0.8, top_k 40, top_p 0.95, min_p 0.05) or the --temp / --top-k / ... flags;
`stop` strings end the generation (the text stops before them); `ignore_eos` and
`n_predict` follow llama-server; `n` > 1 and `logprobs` are rejected with a 400.
Greedy requests (temperature 0 or top_k 1, no penalties) decode on the device with
on-device argmax feedback; sampled ones copy each step's logits to the host.  Every GPU
replica is one llmi Context with `--parallel` sequences (llama-server's slots) driven by
one scheduler thread: requests go to the least-loaded replica and are decoded there
together, one batched step per token for up to 8 sequences (continuous batching,
SURVEY.md §8f row 3).

Text: the GGUF's own tokenizer (SPM or byte-level BPE from tokenizer.ggml.*) and chat
template (tokenizer.chat_template, sandboxed Jinja2), llmi/tokenizer.py; streamed text
holds incomplete UTF-8 sequences back until their last byte.
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import sys
import threading
import time
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Iterable, Optional

from .sampling import Sampler, SamplingParams, StopFilter, find_stop, parse_stop

VERSION = "llmi-server 0.1 (libllmi, gfx950)"


# --------------------------------------------------------------------------------------
# text codecs: the GGUF's tokenizer + chat template (llmi/tokenizer.py), or the legacy
# greedy Vocab (kept for stand-in engines)
# --------------------------------------------------------------------------------------
class _SimpleStream:
    def __init__(self, v):
        self.v = v

    def push(self, t: int) -> str:
        return self.v.detokenize([t])

    def flush(self) -> str:
        return ""


class Vocab:
    """Greedy longest match over token texts (stand-in engines and synthetic vocabularies)."""

    def __init__(self, pieces: list[str], bos: int, eos: int):
        self.bos, self.eos = bos, eos
        self.text = [self._surface(p) for p in pieces]
        self.by_text: dict[str, int] = {}
        for i, t in enumerate(self.text):
            if t and not (pieces[i].startswith("<") and pieces[i].endswith(">")):
                self.by_text.setdefault(t, i)
        self.max_len = max((len(t) for t in self.by_text), default=1)
        self.eog = {eos}

    @property
    def n_vocab(self) -> int:
        return len(self.text)

    @staticmethod
    def _surface(p: str) -> str:
        if len(p) == 6 and p.startswith("<0x") and p.endswith(">"):
            try:
                return chr(int(p[3:5], 16))
            except ValueError:
                return p
        return p.replace("▁", " ").replace("Ġ", " ").replace("Ċ", "\n")

    def detokenize(self, ids: Iterable[int]) -> str:
        return "".join(self.text[i] for i in ids if 0 <= i < len(self.text) and i not in (self.bos, self.eos))

    def tokenize(self, s: str, add_bos: bool = True) -> list[int]:
        out = [self.bos] if add_bos and self.bos >= 0 else []
        i = 0
        while i < len(s):
            for n in range(min(self.max_len, len(s) - i), 0, -1):
                t = self.by_text.get(s[i:i + n])
                if t is not None:
                    out.append(t)
                    i += n
                    break
            else:
                i += 1  # no piece covers this character: skipped
        return out

    def chat_ids(self, messages: list[dict]) -> list[int]:
        return self.tokenize(chat_prompt(messages, self), add_bos=True)

    def stream(self):
        return _SimpleStream(self)


def chat_prompt(messages: list[dict], vocab: Vocab) -> str:
    """Llama-3 header template when the vocabulary has its special tokens, else a
    plain role-prefixed transcript ending with the assistant turn (legacy Vocab only)."""
    if "<|start_header_id|>" in vocab.by_text or any(t == "<|start_header_id|>" for t in vocab.text):
        s = ""
        for m in messages:
            s += f"<|start_header_id|>{m.get('role', 'user')}<|end_header_id|>\n\n{m.get('content', '')}<|eot_id|>"
        return s + "<|start_header_id|>assistant<|end_header_id|>\n\n"
    return "".join(f"{m.get('role', 'user')}: {m.get('content', '')}\n" for m in messages) + "assistant:"


class TextCodec:
    """The GGUF's own tokenizer (SPM / byte-level BPE / greedy for synthetic vocabularies)
    and chat template (tokenizer.chat_template; llama.cpp's chatml default), as
    llama-server applies them: prompts tokenized with parse_special, BOS added unless the
    rendered chat already starts with it, generation stops at any end-of-generation token."""

    EOG_TEXTS = ("<|eot_id|>", "<|eom_id|>", "<|end_of_text|>", "<|im_end|>", "<|endoftext|>", "</s>", "<|end|>")

    def __init__(self, tok, template: Optional[str]):
        from . import tokenizer as T

        self.T = T
        self.tok = tok
        self.template = template
        self.bos, self.eos = tok.bos, tok.eos
        self.bos_text = tok.tokens[tok.bos] if 0 <= tok.bos < tok.n_vocab else ""
        self.eos_text = tok.tokens[tok.eos] if 0 <= tok.eos < tok.n_vocab else ""
        self.eog = {tok.eos} | {tok.by_text[t] for t in self.EOG_TEXTS
                                if t in tok.by_text and tok.types[tok.by_text[t]] == T.CONTROL}
        self.eog.discard(-1)

    @property
    def n_vocab(self) -> int:
        return self.tok.n_vocab

    def tokenize(self, s: str, add_bos: bool = True) -> list[int]:
        return self.tok.tokenize(s, add_special=add_bos, parse_special=True)

    def detokenize(self, ids: Iterable[int]) -> str:
        return self.tok.detokenize(ids)

    def chat_ids(self, messages: list[dict]) -> list[int]:
        for m in messages:
            if not isinstance(m, dict) or not isinstance(m.get("content", ""), str):
                raise ValueError("each message must be an object with string 'content'")
        try:
            text = self.T.render_chat(self.template, messages, self.bos_text, self.eos_text)
        except self.T.TemplateError as e:
            raise ValueError(str(e)) from e
        add_bos = not (self.bos_text and text.startswith(self.bos_text))
        return self.tokenize(text, add_bos=add_bos)

    def stream(self):
        return self.tok.stream()


# --------------------------------------------------------------------------------------
# engine: replicas of one GGUF; each replica = one llmi Context with `slots` sequences,
# driven by one scheduler thread (continuous batching)
# --------------------------------------------------------------------------------------
class Request:
    """One generation: prompt ids in, token lists out through `q` (None terminates).
    `sampling` None or greedy: device argmax; else a host Sampler over each step's logits.
    `stop`: strings that end the generation (checked on the detokenized output)."""

    def __init__(self, prompt: list[int], max_tokens: int, ignore_eos: bool,
                 sampling: Optional[SamplingParams] = None, stop: Optional[list[str]] = None):
        self.prompt, self.max_tokens, self.ignore_eos = list(prompt), max_tokens, ignore_eos
        self.sampler = Sampler(sampling) if sampling is not None and not sampling.greedy else None
        self.stop = list(stop or [])
        self.out: list[int] = []
        self.q: "queue.Queue" = queue.Queue()
        self.finish: Optional[str] = None
        self.error: Optional[str] = None
        self.t_submit = time.perf_counter()
        self.t_first: Optional[float] = None
        self.replica = -1
        # scheduler state
        self.seq = -1
        self.last = -1
        self.pos = 0

    def emit(self, toks: list[int]) -> None:
        if toks:
            if self.t_first is None:
                self.t_first = time.perf_counter()
            self.out += toks
            self.q.put(list(toks))

    def done(self, finish: str) -> None:
        self.finish = finish
        self.q.put(None)

    def fail(self, err: str) -> None:
        self.error = err
        self.q.put(None)


class Replica:
    """One context (device) serving up to `slots` requests at once.  Its thread admits
    queued requests into free sequences (prefill through llama_decode with their seq id)
    and advances all active ones together with llmi_generate_greedy_batch (one weight
    stream per step for up to 8 sequences), `chunk` tokens per call."""

    def __init__(self, idx: int, ctx, slots: int, eog: set, chunk: int, n_ctx: int, device: int = 0,
                 detok: Optional[Callable[[list[int]], str]] = None):
        self.idx, self.ctx, self.slots, self.eog, self.chunk, self.n_ctx = idx, ctx, slots, eog, chunk, n_ctx
        self.device = device
        self.detok = detok
        self.pending: "queue.Queue[Request]" = queue.Queue()
        self.active: list[Request] = []
        self.free = list(range(slots))
        self.lock = threading.Lock()
        self.n_queued = 0
        self.tokens = 0          # generated tokens served
        self.busy_s = 0.0        # time inside decode calls
        self.last_gbps = 0.0     # HBM GB/s of the last decode call (algorithmic bytes / device time)
        self.requests = 0
        self.stop = False
        self.th = threading.Thread(target=self._run, name=f"llmi-replica-{idx}", daemon=True)
        self.th.start()

    def load(self) -> int:
        with self.lock:
            return self.n_queued + len(self.active)

    def submit(self, r: Request) -> None:
        with self.lock:
            self.n_queued += 1
            self.requests += 1
        r.replica = self.idx
        self.pending.put(r)

    def _stats(self) -> None:
        try:
            b, us = self.ctx.stats()
            if us > 0:
                self.last_gbps = b / (us * 1e-6) / 1e9
        except Exception:
            pass

    # -- admission: prefill into a free sequence, emit the first token
    def _admit(self, r: Request) -> None:
        with self.lock:
            self.n_queued -= 1
        seq = self.free.pop()
        try:
            c = self.ctx
            c.seq_rm(seq)
            max_tokens = r.max_tokens
            if len(r.prompt) + max_tokens > self.n_ctx:
                max_tokens = max(0, self.n_ctx - len(r.prompt))
            r.max_tokens = max_tokens
            if not r.prompt or max_tokens <= 0:
                self.free.append(seq)
                r.done("length")
                return
            t0 = time.perf_counter()
            rc = c.decode(r.prompt, seq=[seq] * len(r.prompt))
            self.busy_s += time.perf_counter() - t0
            if rc != 0:
                raise RuntimeError(f"llama_decode returned {rc}")
            first = c.greedy(-1) if r.sampler is None else r.sampler.sample(c.logits(-1), r.prompt)
            r.seq, r.pos = seq, len(r.prompt)
            if self._take(r, [first]):
                self.free.append(seq)
            else:
                r.last = first
                self.active.append(r)
        except Exception as e:  # this request fails; the replica keeps serving
            self.free.append(seq)
            r.fail(str(e))

    def _take(self, r: Request, toks: list[int]) -> bool:
        """Emit generated tokens up to EOS / max_tokens; True when the request is done."""
        emit = []
        for t in toks:
            if t in self.eog and not r.ignore_eos:
                r.emit(emit)
                self.tokens += len(emit)
                r.done("stop")
                return True
            emit.append(t)
            if len(r.out) + len(emit) >= r.max_tokens:
                break
        r.emit(emit)
        self.tokens += len(emit)
        if r.stop and self.detok is not None and emit and self._stop_seen(r, len(emit)):
            r.done("stop")
            return True
        if len(r.out) >= r.max_tokens:
            r.done("length")
            return True
        return False

    def _stop_seen(self, r: Request, n_new: int) -> bool:
        """Did the n_new tokens just emitted complete a stop string?  Earlier text was
        checked when it was new, so only a window is detokenized: the new tokens plus
        enough older ones to hold a stop string that starts before them (every token is at
        least one byte, so max(len(stop)) + 4 tokens cover any stop string plus a split
        UTF-8 sequence) -- O(1) per call instead of the whole output."""
        tail = max(len(x.encode("utf-8")) for x in r.stop) + 4
        return find_stop(self.detok(r.out[-(n_new + tail):]), r.stop) is not None

    def _step(self) -> None:
        batch = self.active[:8]
        k = max(1, min(self.chunk, min(r.max_tokens - len(r.out) for r in batch)))
        if any(r.stop for r in batch):
            k = min(k, 4)  # stop strings are checked between decode calls
        c = self.ctx
        t0 = time.perf_counter()
        greedy = [r for r in batch if r.sampler is None]
        sampled = [r for r in batch if r.sampler is not None]
        outs: dict[int, list[int]] = {}
        if greedy:
            # greedy slots decode k tokens per call with the argmax fed back on the device,
            # whether or not sampled requests share the replica
            try:
                got = c.generate_greedy_batch([r.seq for r in greedy], [r.last for r in greedy],
                                              [r.pos for r in greedy], k)
            except Exception:
                # not batchable here (e.g. a context past the batched attention's bound):
                # one sequence at a time, same results
                got = [c.generate_greedy_batch([r.seq], [r.last], [r.pos], k)[0] for r in greedy]
            for r, toks in zip(greedy, got):
                outs[id(r)] = toks
        if sampled:
            # one token per call: every sampled slot's logits (llama_decode with one token
            # per sequence = one batched step), sampled on the host
            rc = c.decode([r.last for r in sampled], pos=[r.pos for r in sampled], seq=[r.seq for r in sampled],
                          logits_all=True)
            if rc != 0:
                raise RuntimeError(f"llama_decode returned {rc}")
            for i, r in enumerate(sampled):
                outs[id(r)] = [r.sampler.sample(c.logits(i), r.prompt + r.out)]
        self.busy_s += time.perf_counter() - t0
        self._stats()
        done = []
        for r in batch:
            toks = outs[id(r)]
            r.pos += len(toks)
            r.last = toks[-1]
            if self._take(r, toks):
                done.append(r)
        for r in done:
            self.active.remove(r)
            self.free.append(r.seq)
        # rotate so more than 8 active requests share the steps fairly
        if len(self.active) > 8:
            self.active = self.active[len(batch):] + self.active[:len(batch)]

    def _run(self) -> None:
        while not self.stop:
            try:
                while self.free and (not self.pending.empty() or not self.active):
                    r = self.pending.get(timeout=0.5 if not self.active else None) if not self.active else \
                        self.pending.get_nowait()
                    self._admit(r)
            except queue.Empty:
                pass
            if not self.active:
                continue
            try:
                self._step()
            except Exception as e:  # the context failed: every active request fails
                for r in self.active:
                    r.fail(str(e))
                    self.free.append(r.seq)
                self.active = []


class Engine:
    """Owns the GPU replicas.  Requests go to the least-loaded replica (active + queued;
    ties to the lowest index) and are served there with continuous batching."""

    def __init__(self, path: str, n_ctx: int, n_gpu_layers: int, devices: list[int], slots: int = 4,
                 chunk: int = 8, contexts=None, sampling: Optional[SamplingParams] = None, numerics: int = 0):
        self.path, self.n_ctx, self.ngl, self.devices = path, n_ctx, n_gpu_layers, devices
        self.numerics = numerics  # llmi.NUMERICS_GENERIC / NUMERICS_X86
        self.sampling = sampling or SamplingParams()  # server defaults (llama-server's)
        self.slots, self.chunk = max(1, slots), max(1, chunk)
        self.ready = False
        self.error: Optional[str] = None
        self.vocab = None
        self.model_id = os.path.basename(path)
        self.replicas: list[Replica] = []
        self._models = []
        self._contexts = contexts  # test hook: (list of context-like objects, codec)
        self.t_ready: Optional[float] = None
        self.load_s = 0.0

    def load(self) -> None:
        t0 = time.perf_counter()
        try:
            if self._contexts is not None:
                ctxs, self.vocab = self._contexts
            else:
                import llmi
                from . import tokenizer as T

                if len(self.devices) > 1:  # replicas: RCCL pieces pipelined behind the upload
                    m0, reps = llmi.Model.load_replicated(self.path, self.devices[0], self.devices[1:],
                                                          n_gpu_layers=self.ngl, numerics=self.numerics)
                else:
                    m0, reps = llmi.Model(self.path, n_gpu_layers=self.ngl, main_gpu=self.devices[0],
                                          numerics=self.numerics), []
                models = [m0] + reps
                self._models = models
                ctxs = [llmi.Context(m, n_ctx=self.n_ctx, n_seq=self.slots) for m in models]
                self.n_ctx = ctxs[0].n_ctx
                meta = T.read_gguf_meta(self.path)
                tok = T.make_tokenizer(meta, tokens=[m0.token_text(i) for i in range(m0.n_vocab)],
                                       bos=m0.bos, eos=m0.eos) if not meta.get("tokenizer.ggml.tokens") \
                    else T.make_tokenizer(meta)
                self.vocab = TextCodec(tok, meta.get("tokenizer.chat_template"))
            eog = getattr(self.vocab, "eog", {self.vocab.eos})
            detok = getattr(self.vocab, "detokenize", None)
            self.replicas = [Replica(i, c, self.slots, eog, self.chunk, self.n_ctx,
                                     self.devices[i] if i < len(self.devices) else i, detok)
                             for i, c in enumerate(ctxs)]
            self.load_s = time.perf_counter() - t0
            self.t_ready = time.perf_counter()
            self.ready = True
        except Exception as e:  # reported by /health
            self.error = str(e)

    def submit(self, prompt: list[int], max_tokens: int, ignore_eos: bool,
               sampling: Optional[SamplingParams] = None, stop: Optional[list[str]] = None) -> Request:
        r = Request(prompt, max_tokens, ignore_eos, sampling, stop)
        rep = min(self.replicas, key=lambda x: (x.load(), x.idx))
        rep.submit(r)
        return r

    def generate(self, prompt: list[int], max_tokens: int, ignore_eos: bool, on_tokens: Callable[[list[int]], None],
                 chunk: int = 8, sampling: Optional[SamplingParams] = None,
                 stop: Optional[list[str]] = None) -> tuple[list[int], str]:
        r = self.submit(prompt, max_tokens, ignore_eos, sampling, stop)
        while True:
            toks = r.q.get()
            if toks is None:
                break
            on_tokens(toks)
        if r.error:
            raise RuntimeError(r.error)
        return r.out, r.finish or "length"

    def health(self) -> dict:
        """Per-replica serving metrics for /health (kept well under the gateway's 4 KB read,
        scripts/gateway.py:350)."""
        up = max(1e-9, time.perf_counter() - (self.t_ready or time.perf_counter()))
        reps = []
        for r in self.replicas:
            reps.append({"id": r.idx, "device": r.device, "active": len(r.active), "queued": r.n_queued,
                         "tokens": r.tokens, "tok_s": round(r.tokens / max(r.busy_s, 1e-9), 1) if r.tokens else 0.0,
                         "hbm_gbps": round(r.last_gbps, 1), "busy": round(r.busy_s / up, 3)})
        busy = sum(len(r.active) for r in self.replicas)
        return {"slots_idle": self.slots * len(self.replicas) - busy, "slots_processing": busy,
                "load_s": round(self.load_s, 2), "replicas": reps[:16]}


# --------------------------------------------------------------------------------------
# HTTP
# --------------------------------------------------------------------------------------
def _error(code: int, msg: str, typ: str) -> dict:
    return {"error": {"message": msg, "type": typ, "code": code}}


class Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "llmi-server"
    engine: Engine = None  # set by make_server
    api_key: Optional[str] = None

    def log_message(self, fmt, *args):  # quiet; the gateway logs requests
        if os.environ.get("LLMI_SERVER_LOG"):
            sys.stderr.write("[llmi-server] " + fmt % args + "\n")

    # ---- plumbing
    def _send_json(self, code: int, obj: dict) -> None:
        body = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.send_header("Connection", "close")
        self.end_headers()
        self.wfile.write(body)
        self.close_connection = True

    PUBLIC = ("/health", "/v1/health")

    def _authorized(self, route: str) -> bool:
        if not self.api_key or route in self.PUBLIC:
            return True
        return self.headers.get("Authorization", "") == f"Bearer {self.api_key}"

    def _body(self) -> Optional[dict]:
        n = int(self.headers.get("Content-Length") or 0)
        raw = self.rfile.read(n) if n > 0 else b""
        try:
            return json.loads(raw or b"{}")
        except json.JSONDecodeError:
            return None

    # ---- routes
    def do_GET(self):
        eng = self.engine
        route = self.path.split("?")[0]
        if route in self.PUBLIC:
            if eng.error:
                return self._send_json(500, {"status": "error", "error": eng.error})
            if not eng.ready:
                return self._send_json(503, _error(503, "Loading model", "unavailable_error"))
            h = {"status": "ok"}
            if hasattr(eng, "health"):
                h.update(eng.health())
            return self._send_json(200, h)
        if not self._authorized(route):
            return self._send_json(401, _error(401, "Invalid API Key", "authentication_error"))
        if route == "/v1/models":
            return self._send_json(200, {"object": "list", "data": [
                {"id": eng.model_id, "object": "model", "created": int(time.time()), "owned_by": "llmi"}]})
        return self._send_json(404, _error(404, "File Not Found", "not_found_error"))

    def do_POST(self):
        eng = self.engine
        route = self.path.split("?")[0]
        if not self._authorized(route):
            return self._send_json(401, _error(401, "Invalid API Key", "authentication_error"))
        if route in ("/v1/embeddings", "/embeddings", "/embedding"):
            # the reference launches llama-server without embedding support (start.sh
            # passes no --embeddings; docs/API_REFERENCE.md:537-540 "only available if ...
            # started with embedding support"): upstream then answers 501 not_supported_error
            return self._send_json(501, _error(
                501, "This server does not support embeddings. Start it with `--embeddings`", "not_supported_error"))
        if route not in ("/v1/completions", "/v1/chat/completions", "/completion"):
            return self._send_json(404, _error(404, "File Not Found", "not_found_error"))
        if not eng.ready:
            return self._send_json(503, _error(503, "Loading model", "unavailable_error"))
        req = self._body()
        if req is None:
            return self._send_json(400, _error(400, "invalid JSON body", "invalid_request_error"))
        chat = route == "/v1/chat/completions"
        v = eng.vocab
        try:
            if chat:
                msgs = req.get("messages")
                if not isinstance(msgs, list) or not msgs:
                    raise ValueError("'messages' must be a non-empty list")
                prompt = v.chat_ids(msgs)
            else:
                p = req.get("prompt", "")
                if isinstance(p, list) and all(isinstance(t, int) for t in p):
                    prompt = list(p)
                    if not prompt or not (0 <= min(prompt) and max(prompt) < v.n_vocab):
                        raise ValueError("token ids out of range")
                elif isinstance(p, str):
                    prompt = v.tokenize(p, add_bos=True)
                else:
                    raise ValueError("'prompt' must be a string or a list of token ids")
            max_tokens = int(req.get("max_tokens", req.get("n_predict", 16 if not chat else 256)))
            if max_tokens < 0:
                max_tokens = eng.n_ctx
            if int(req.get("n", 1)) != 1:
                raise ValueError("only n = 1 is supported")
            if req.get("logprobs") not in (None, False, 0) or req.get("top_logprobs") not in (None, 0):
                raise ValueError("logprobs are not supported")
            sampling = getattr(eng, "sampling", SamplingParams()).with_request(req)
            stop = parse_stop(req.get("stop"))
        except (ValueError, TypeError) as e:
            return self._send_json(400, _error(400, str(e), "invalid_request_error"))
        ignore_eos = bool(req.get("ignore_eos", False))
        stream = bool(req.get("stream", False))
        rid = ("chatcmpl-" if chat else "cmpl-") + uuid.uuid4().hex[:24]
        created = int(time.time())
        obj = "chat.completion" if chat else "text_completion"
        if not stream:
            try:
                ids, finish = eng.generate(prompt, max_tokens, ignore_eos, lambda _t: None, chunk=32,
                                           sampling=sampling, stop=stop)
            except Exception as e:  # a failed llama_decode: OpenAI-shaped 500, not a dropped socket
                return self._send_json(500, _error(500, str(e), "server_error"))
            text = v.detokenize(ids)
            cut = find_stop(text, stop)
            if cut is not None:
                text, finish = text[:cut], "stop"
            choice = ({"index": 0, "message": {"role": "assistant", "content": text}, "finish_reason": finish}
                      if chat else {"index": 0, "text": text, "logprobs": None, "finish_reason": finish})
            return self._send_json(200, {
                "id": rid, "object": obj, "created": created, "model": eng.model_id, "choices": [choice],
                "usage": {"prompt_tokens": len(prompt), "completion_tokens": len(ids),
                          "total_tokens": len(prompt) + len(ids)},
                "llmi": {"tokens": ids}})
        # SSE: headers, one data: line per token batch, final chunk, [DONE], close
        self.send_response(200)
        self.send_header("Content-Type", "text/event-stream")
        self.send_header("Cache-Control", "no-cache")
        self.send_header("Connection", "close")
        self.end_headers()
        self.close_connection = True
        cobj = "chat.completion.chunk" if chat else "text_completion"

        def event(payload: dict) -> None:
            self.wfile.write(b"data: " + json.dumps(payload).encode() + b"\n\n")
            self.wfile.flush()

        if chat:
            event({"id": rid, "object": cobj, "created": created, "model": eng.model_id,
                   "choices": [{"index": 0, "delta": {"role": "assistant"}, "finish_reason": None}]})

        sd = v.stream()
        sf = StopFilter(stop)

        def on_tokens(ts: list[int]) -> None:
            for t in ts:
                piece = sf.push(sd.push(t))
                if not piece:
                    continue  # an incomplete UTF-8 sequence, or a possible stop-string prefix: held back
                ch = ({"index": 0, "delta": {"content": piece}, "finish_reason": None} if chat
                      else {"index": 0, "text": piece, "logprobs": None, "finish_reason": None})
                event({"id": rid, "object": cobj, "created": created, "model": eng.model_id, "choices": [ch]})

        try:
            ids, finish = eng.generate(prompt, max_tokens, ignore_eos, on_tokens, chunk=4, sampling=sampling, stop=stop)
            tail = sf.push(sd.flush()) + sf.flush()
            if sf.stopped:
                finish = "stop"
            if tail:
                ch = ({"index": 0, "delta": {"content": tail}, "finish_reason": None} if chat
                      else {"index": 0, "text": tail, "logprobs": None, "finish_reason": None})
                event({"id": rid, "object": cobj, "created": created, "model": eng.model_id, "choices": [ch]})
            last = ({"index": 0, "delta": {}, "finish_reason": finish} if chat
                    else {"index": 0, "text": "", "logprobs": None, "finish_reason": finish})
            event({"id": rid, "object": cobj, "created": created, "model": eng.model_id, "choices": [last],
                   "usage": {"prompt_tokens": len(prompt), "completion_tokens": len(ids),
                             "total_tokens": len(prompt) + len(ids)}})
            self.wfile.write(b"data: [DONE]\n\n")
            self.wfile.flush()
        except (BrokenPipeError, ConnectionResetError):
            pass
        except Exception as e:  # decode failed mid-stream: an error event, then close
            try:
                event(_error(500, str(e), "server_error"))
            except (BrokenPipeError, ConnectionResetError):
                pass


def make_server(engine: Engine, host: str, port: int, api_key: Optional[str]) -> ThreadingHTTPServer:
    handler = type("LlmiHandler", (Handler,), {"engine": engine, "api_key": api_key})
    srv = ThreadingHTTPServer((host, port), handler)
    srv.daemon_threads = True
    return srv


def parse_args(argv=None):
    ap = argparse.ArgumentParser(prog="llama-server", add_help=True)
    ap.add_argument("--version", action="store_true")
    ap.add_argument("-m", "--model")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("-c", "--ctx-size", type=int, default=4096)
    ap.add_argument("-ngl", "--n-gpu-layers", "--gpu-layers", dest="ngl", type=int, default=999)
    ap.add_argument("--api-key-file")
    ap.add_argument("--api-key")
    ap.add_argument("-t", "--threads", type=int, default=0)
    ap.add_argument("--replicas", type=int, default=int(os.environ.get("LLMI_REPLICAS", "1")),
                    help="GPU replicas (devices 0..N-1), one context each")
    ap.add_argument("-np", "--parallel", type=int, default=int(os.environ.get("LLMI_SLOTS", "4")),
                    help="sequences (slots) per replica decoded together (continuous batching)")
    ap.add_argument("--decode-chunk", type=int, default=8, help="tokens per batched decode call")
    ap.add_argument("--numerics", choices=NUMERICS_CHOICES, default=None,
                    help="fp32 association of every kernel: ggml's generic order, or the oracle's model of "
                         "upstream's x86 AVX2 association (non-repack); '-fa': decode attention in ggml's CPU "
                         "flash-attention numerics (match with the reference's CPU image unpinned)")
    # llama-server's sampling flags and defaults (per-request fields override them)
    d = SamplingParams()
    ap.add_argument("--temp", type=float, default=d.temperature)
    ap.add_argument("--top-k", type=int, default=d.top_k)
    ap.add_argument("--top-p", type=float, default=d.top_p)
    ap.add_argument("--min-p", type=float, default=d.min_p)
    ap.add_argument("--repeat-penalty", type=float, default=d.repeat_penalty)
    ap.add_argument("--repeat-last-n", type=int, default=d.repeat_last_n)
    ap.add_argument("--presence-penalty", type=float, default=d.presence_penalty)
    ap.add_argument("--frequency-penalty", type=float, default=d.frequency_penalty)
    ap.add_argument("-s", "--seed", type=int, default=d.seed)
    args, extra = ap.parse_known_args(argv)
    if args.numerics is None:
        # argparse does not check a default against `choices`: validate the env value here
        env = os.environ.get("LLMI_NUMERICS", "generic").strip().lower()
        if env not in NUMERICS_CHOICES:
            ap.error(f"LLMI_NUMERICS={os.environ.get('LLMI_NUMERICS')!r}: expected one of {', '.join(NUMERICS_CHOICES)}")
        args.numerics = env
    return args, extra


# --numerics values -> llama_model_params.numerics (llmi.h LLMI_NUMERICS_*)
NUMERICS_CHOICES = ("generic", "x86", "generic-fa", "x86-fa")


def numerics_value(name: str) -> int:
    return (1 if name.startswith("x86") else 0) | (2 if name.endswith("-fa") else 0)


def main(argv=None) -> int:
    args, extra = parse_args(argv)
    if args.version:
        print(VERSION)
        return 0
    if extra:
        print(f"[llmi-server] ignoring unsupported arguments: {' '.join(extra)}", file=sys.stderr)
    if not args.model:
        print("error: -m/--model is required", file=sys.stderr)
        return 2
    key = args.api_key
    if args.api_key_file:
        key = open(args.api_key_file).read().strip()
    sp = SamplingParams(temperature=args.temp, top_k=args.top_k, top_p=args.top_p, min_p=args.min_p,
                        repeat_penalty=args.repeat_penalty, repeat_last_n=args.repeat_last_n,
                        presence_penalty=args.presence_penalty, frequency_penalty=args.frequency_penalty, seed=args.seed)
    eng = Engine(args.model, args.ctx_size, args.ngl, list(range(max(1, args.replicas))), slots=args.parallel,
                 chunk=args.decode_chunk, sampling=sp, numerics=numerics_value(args.numerics))
    srv = make_server(eng, args.host, args.port, key)
    threading.Thread(target=eng.load, daemon=True).start()
    print(f"[llmi-server] listening on {args.host}:{args.port}", file=sys.stderr, flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
