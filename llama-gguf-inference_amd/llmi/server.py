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
  Authorization: Bearer <key> required on every route but /health when a key is
  configured (401 otherwise; llama-server's public endpoints are /health and /v1/health)

Decoding is greedy (temperature is accepted and ignored: the north star's workload is
greedy); `ignore_eos` and `n_predict` follow llama-server.  Every GPU replica is one
llmi Context driven by one thread; requests take the least-loaded free replica.

Text handling is the §8f "next" item: token-id prompts are exact; text is tokenized
by greedy longest match over the GGUF vocabulary (exact for the synthetic vocab, an
approximation of BPE/SPM for real vocabularies) and detokenized by piece concatenation.
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

VERSION = "llmi-server 0.1 (libllmi, gfx950)"


# --------------------------------------------------------------------------------------
# vocabulary: detokenize + greedy longest-match tokenizer
# --------------------------------------------------------------------------------------
class Vocab:
    def __init__(self, pieces: list[str], bos: int, eos: int):
        self.bos, self.eos = bos, eos
        self.text = [self._surface(p) for p in pieces]
        self.by_text: dict[str, int] = {}
        for i, t in enumerate(self.text):
            if t and not (pieces[i].startswith("<") and pieces[i].endswith(">")):
                self.by_text.setdefault(t, i)
        self.max_len = max((len(t) for t in self.by_text), default=1)

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


def chat_prompt(messages: list[dict], vocab: Vocab) -> str:
    """Llama-3 header template when the vocabulary has its special tokens, else a
    plain role-prefixed transcript ending with the assistant turn."""
    if "<|start_header_id|>" in vocab.by_text or any(t == "<|start_header_id|>" for t in vocab.text):
        s = ""
        for m in messages:
            s += f"<|start_header_id|>{m.get('role', 'user')}<|end_header_id|>\n\n{m.get('content', '')}<|eot_id|>"
        return s + "<|start_header_id|>assistant<|end_header_id|>\n\n"
    return "".join(f"{m.get('role', 'user')}: {m.get('content', '')}\n" for m in messages) + "assistant:"


# --------------------------------------------------------------------------------------
# engine: replicas of one GGUF, one llmi Context each
# --------------------------------------------------------------------------------------
class Engine:
    """Owns the GPU replicas.  generate() runs on a free replica (least loaded first)."""

    def __init__(self, path: str, n_ctx: int, n_gpu_layers: int, devices: list[int]):
        self.path, self.n_ctx, self.ngl, self.devices = path, n_ctx, n_gpu_layers, devices
        self.ready = False
        self.error: Optional[str] = None
        self.vocab: Optional[Vocab] = None
        self.model_id = os.path.basename(path)
        self._free: "queue.Queue[int]" = queue.Queue()
        self._ctxs = []
        self._models = []

    def load(self) -> None:
        try:
            import llmi

            m0 = llmi.Model(self.path, n_gpu_layers=self.ngl, main_gpu=self.devices[0])
            models = [m0] + (m0.replicate(self.devices[1:]) if len(self.devices) > 1 else [])
            self._models = models
            self._ctxs = [llmi.Context(m, n_ctx=self.n_ctx) for m in models]
            self.n_ctx = self._ctxs[0].n_ctx
            self.vocab = Vocab([m0.token_text(i) for i in range(m0.n_vocab)], m0.bos, m0.eos)
            for i in range(len(self._ctxs)):
                self._free.put(i)
            self.ready = True
        except Exception as e:  # reported by /health
            self.error = str(e)

    def generate(self, prompt: list[int], max_tokens: int, ignore_eos: bool, on_tokens: Callable[[list[int]], None],
                 chunk: int = 8) -> tuple[list[int], str]:
        i = self._free.get()
        try:
            c = self._ctxs[i]
            c.kv_clear()
            if len(prompt) + max_tokens > self.n_ctx:
                max_tokens = max(0, self.n_ctx - len(prompt))
            if not prompt or max_tokens <= 0:
                return [], "length"
            rc = c.decode(prompt)
            if rc != 0:
                raise RuntimeError(f"llama_decode returned {rc}")
            # generate_greedy(t, pos, k) decodes t at pos and returns the k tokens after it
            out: list[int] = []
            pending, pos = [c.greedy(-1)], len(prompt)
            while True:
                emit = []
                for t in pending:
                    if t == self.vocab.eos and not ignore_eos:
                        if emit:
                            on_tokens(emit)
                        return out + emit, "stop"
                    emit.append(t)
                    if len(out) + len(emit) >= max_tokens:
                        break
                out += emit
                on_tokens(emit)
                if len(out) >= max_tokens:
                    return out, "length"
                k = min(chunk, max_tokens - len(out))
                pending = c.generate_greedy(out[-1], pos, k)
                pos += k
        finally:
            self._free.put(i)


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
            return self._send_json(200, {"status": "ok"})
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
                prompt = v.tokenize(chat_prompt(msgs, v), add_bos=True)
            else:
                p = req.get("prompt", "")
                if isinstance(p, list) and all(isinstance(t, int) for t in p):
                    prompt = list(p)
                    if not prompt or not (0 <= min(prompt) and max(prompt) < len(v.text)):
                        raise ValueError("token ids out of range")
                elif isinstance(p, str):
                    prompt = v.tokenize(p, add_bos=True)
                else:
                    raise ValueError("'prompt' must be a string or a list of token ids")
            max_tokens = int(req.get("max_tokens", req.get("n_predict", 16 if not chat else 256)))
            if max_tokens < 0:
                max_tokens = eng.n_ctx
        except (ValueError, TypeError) as e:
            return self._send_json(400, _error(400, str(e), "invalid_request_error"))
        ignore_eos = bool(req.get("ignore_eos", False))
        stream = bool(req.get("stream", False))
        rid = ("chatcmpl-" if chat else "cmpl-") + uuid.uuid4().hex[:24]
        created = int(time.time())
        obj = "chat.completion" if chat else "text_completion"
        if not stream:
            try:
                ids, finish = eng.generate(prompt, max_tokens, ignore_eos, lambda _t: None, chunk=32)
            except Exception as e:  # a failed llama_decode: OpenAI-shaped 500, not a dropped socket
                return self._send_json(500, _error(500, str(e), "server_error"))
            text = v.detokenize(ids)
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

        def on_tokens(ts: list[int]) -> None:
            for t in ts:
                piece = v.detokenize([t])
                ch = ({"index": 0, "delta": {"content": piece}, "finish_reason": None} if chat
                      else {"index": 0, "text": piece, "logprobs": None, "finish_reason": None})
                event({"id": rid, "object": cobj, "created": created, "model": eng.model_id, "choices": [ch]})

        try:
            ids, finish = eng.generate(prompt, max_tokens, ignore_eos, on_tokens, chunk=4)
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
    args, extra = ap.parse_known_args(argv)
    return args, extra


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
    eng = Engine(args.model, args.ctx_size, args.ngl, list(range(max(1, args.replicas))))
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
