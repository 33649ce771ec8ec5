#!/usr/bin/env python3
"""benchmark.py-compatible serving measurement.

The reference measures inference through the gateway with scripts/benchmark.py:
streaming /v1/chat/completions requests at a concurrency level (:279-447), TTFT = time
to the first `delta.content` chunk, tokens_per_sec = whitespace-split word count of the
streamed text / total request latency (:120-125, :443-447), nearest-rank percentiles
(:43-60) and the JSON shape of format_json_output (:542-577).  This tool restates that
measurement so the numbers line up with the reference's own reports, and adds what the
word count hides: the exact generated-token count from the final chunk's usage and the
aggregate token rate over the wall time.

  tools/http_bench.py --url http://127.0.0.1:8080 [--api-key K] [--concurrency 1,4,8]
  tools/http_bench.py --serve PRESET [--slots 8]   # start llmi's server in-process on a
                                                   # synthetic GGUF of PRESET (GPU)
Prints one JSON object: {"inference": {...reference keys...}, "llmi": {...}} per level.
"""
from __future__ import annotations

import argparse
import http.client
import json
import os
import statistics
import sys
import threading
import time
from typing import Any, Optional
from urllib.parse import urlparse

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def percentile(data: list[float], pct: float) -> float:
    """Nearest-rank percentile (scripts/benchmark.py:43-60)."""
    if not data:
        return 0.0
    s = sorted(data)
    k = max(0, min(int(len(s) * pct / 100.0 + 0.5) - 1, len(s) - 1))
    return s[k]


def compute_stats(values: list[float]) -> dict[str, float]:
    """min/max/mean/p50/p95/p99/count (scripts/benchmark.py:63-79)."""
    if not values:
        return {"min": 0.0, "max": 0.0, "mean": 0.0, "p50": 0.0, "p95": 0.0, "p99": 0.0, "count": 0}
    return {"min": min(values), "max": max(values), "mean": statistics.mean(values), "p50": percentile(values, 50),
            "p95": percentile(values, 95), "p99": percentile(values, 99), "count": len(values)}


def count_words(text: str) -> int:
    """The reference's token count: whitespace split (scripts/benchmark.py:120-125)."""
    return len(text.split())


def one_request(url: str, prompt: str, max_tokens: int, api_key: Optional[str], timeout: float = 120.0) -> dict:
    """One streaming chat completion: TTFT, latency, streamed text, usage tokens."""
    u = urlparse(url)
    body = json.dumps({"model": "default", "messages": [{"role": "user", "content": prompt}],
                       "max_tokens": max_tokens, "stream": True}).encode()
    headers = {"Content-Type": "application/json", "Connection": "close"}
    if api_key:
        headers["Authorization"] = f"Bearer {api_key}"
    res: dict[str, Any] = {"ttft": None, "total_latency": None, "text": "", "usage_tokens": None, "error": None}
    t0 = time.monotonic()
    try:
        c = http.client.HTTPConnection(u.hostname, u.port or 80, timeout=timeout)
        c.request("POST", "/v1/chat/completions", body=body, headers=headers)
        r = c.getresponse()
        if r.status != 200:
            res["error"] = f"HTTP {r.status}: {r.read()[:200].decode('utf-8', 'replace')}"
            res["total_latency"] = time.monotonic() - t0
            return res
        buf, parts = b"", []
        while True:
            chunk = r.read1(4096) if hasattr(r, "read1") else r.read(4096)
            if not chunk:
                break
            buf += chunk
            while b"\n" in buf:
                line, buf = buf.split(b"\n", 1)
                line = line.strip()
                if not line.startswith(b"data:"):
                    continue
                data = line[5:].strip()
                if data == b"[DONE]":
                    continue
                try:
                    obj = json.loads(data)
                except json.JSONDecodeError:
                    continue
                if "usage" in obj:
                    res["usage_tokens"] = obj["usage"].get("completion_tokens")
                ch = obj.get("choices") or []
                if ch:
                    content = (ch[0].get("delta") or {}).get("content")
                    if content:
                        if res["ttft"] is None:
                            res["ttft"] = time.monotonic() - t0
                        parts.append(content)
        c.close()
        res["text"] = "".join(parts)
    except Exception as e:  # counted as a failed request, as the reference does
        res["error"] = str(e)
    res["total_latency"] = time.monotonic() - t0
    return res


def run_level(url: str, prompt: str, max_tokens: int, api_key: Optional[str], concurrency: int, n_requests: int,
              warmup: int = 1) -> dict:
    for _ in range(warmup):
        one_request(url, prompt, max_tokens, api_key)
    sem = threading.Semaphore(concurrency)
    out: list[dict] = [None] * n_requests

    def run(i):
        with sem:
            out[i] = one_request(url, prompt, max_tokens, api_key)

    t0 = time.monotonic()
    ths = [threading.Thread(target=run, args=(i,)) for i in range(n_requests)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    wall = time.monotonic() - t0
    ttft, tps, lat, exact = [], [], [], []
    ok = fail = 0
    gen = 0
    for r in out:
        if r["error"]:
            fail += 1
            continue
        ok += 1
        lat.append(r["total_latency"])
        if r["ttft"] is not None:
            ttft.append(r["ttft"])
        w = count_words(r["text"])
        if w > 0 and r["total_latency"] > 0:
            tps.append(w / r["total_latency"])
        if r["usage_tokens"]:
            gen += r["usage_tokens"]
            exact.append(r["usage_tokens"] / r["total_latency"])
    return {
        "inference": {"ttft": compute_stats(ttft), "tokens_per_sec": compute_stats(tps),
                      "total_latency": compute_stats(lat), "requests_total": n_requests, "requests_success": ok,
                      "requests_failed": fail, "wall_time": wall, "concurrency": concurrency},
        "llmi": {"generated_tokens": gen, "aggregate_tok_s": gen / wall if wall > 0 else 0.0,
                 "per_request_tok_s": compute_stats(exact),
                 "note": "tokens_per_sec is the reference's whitespace word count / latency; "
                         "aggregate_tok_s counts generated tokens (usage) over the wall time"},
    }


def serve_inprocess(preset: str, slots: int, n_ctx: int, n_layer: int = 0) -> tuple[str, Any]:
    sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
    import torch  # noqa: F401  (one HIP runtime per process, llmi/_lib.py)

    import llmi
    from llmi.server import Engine, make_server

    path = f"/tmp/llmi_bench/{preset}-s3{'-L%d' % n_layer if n_layer else ''}.gguf"
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        llmi.write_synthetic_gguf(path, preset, seed=3, n_layer=n_layer)
    eng = Engine(path, n_ctx, 999, [0], slots=slots, chunk=8)
    eng.load()
    if not eng.ready:
        raise SystemExit(f"engine failed: {eng.error}")
    srv = make_server(eng, "127.0.0.1", 0, None)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return f"http://127.0.0.1:{srv.server_address[1]}", eng


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--url")
    ap.add_argument("--serve", help="synthetic preset to serve in-process (needs a GPU)")
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--n-layer", type=int, default=0)
    ap.add_argument("--api-key")
    ap.add_argument("--prompt", default="Write a short poem about the sea")
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--concurrency", default="1,4,8")
    ap.add_argument("--requests", type=int, default=16)
    a = ap.parse_args(argv)
    eng = None
    url = a.url
    if a.serve:
        url, eng = serve_inprocess(a.serve, a.slots, a.ctx, a.n_layer)
    if not url:
        ap.error("--url or --serve")
    levels = {}
    for c in [int(x) for x in a.concurrency.split(",")]:
        levels[str(c)] = run_level(url, a.prompt, a.max_tokens, a.api_key, c, max(a.requests, c))
        print(f"[http_bench] concurrency {c}: {json.dumps(levels[str(c)]['llmi'])}", file=sys.stderr, flush=True)
    res = {"url": url, "preset": a.serve, "levels": levels}
    if eng is not None:
        res["health"] = eng.health()
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
