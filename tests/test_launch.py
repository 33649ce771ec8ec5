"""llmi/launch.py: the GPU probe and configurable readiness wait of scripts/start.sh
(:371-377, :600-635) around llmi's llama-server, checked with stand-in servers."""
from __future__ import annotations

import json
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, HTTPServer
from types import SimpleNamespace

from llmi import launch


def test_gpu_probe_amd_smi_json(monkeypatch):
    out = json.dumps([{"gpu": 0, "asic": {"market_name": "AMD Instinct MI355X"},
                       "vram": {"size": {"value": 294896, "unit": "MB"}}}] * 2)
    monkeypatch.setattr(launch.shutil, "which", lambda n: "/usr/bin/" + n if n == "amd-smi" else None)
    line = launch.gpu_probe(run=lambda *a, **k: SimpleNamespace(returncode=0, stdout=out))
    assert line == "GPU: 2 x [AMD Instinct MI355X, 294896 MB; AMD Instinct MI355X, 294896 MB] (amd-smi)"
    monkeypatch.setattr(launch.shutil, "which", lambda n: None)
    assert "not available" in launch.gpu_probe()


def _stub(ready_after: float, key: str):
    t0 = time.monotonic()
    seen = []

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):
            seen.append(self.headers.get("Authorization"))
            ok = time.monotonic() - t0 >= ready_after
            body = b'{"status":"ok"}' if ok else b'{"error":"Loading model"}'
            self.send_response(200 if ok else 503)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

    srv = HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv, seen


def test_wait_ready_503_then_200():
    srv, seen = _stub(0.5, "k")
    try:
        assert launch.wait_ready(srv.server_address[1], "k", max_wait=10, alive=lambda: True, interval=0.1)
        assert seen and all(h == "Bearer k" for h in seen) and len(seen) >= 2
    finally:
        srv.shutdown()


def test_wait_ready_timeout_and_dead_process():
    srv, _ = _stub(1e9, None)
    try:
        t0 = time.monotonic()
        assert not launch.wait_ready(srv.server_address[1], None, max_wait=0.5, alive=lambda: True, interval=0.1)
        assert time.monotonic() - t0 < 5
        assert not launch.wait_ready(srv.server_address[1], None, max_wait=30, alive=lambda: False, interval=0.1)
    finally:
        srv.shutdown()


def test_main_fails_when_server_dies(monkeypatch):
    monkeypatch.setenv("LLMI_SERVER", f"{sys.executable} -c import sys;sys.exit(3)")
    monkeypatch.setattr(launch, "gpu_probe", lambda: "GPU: stub")
    assert launch.main(["--max-wait", "20", "--interval", "0.1", "--", "--port", "1"]) == 1


def test_main_times_out_and_stops_server(monkeypatch):
    monkeypatch.setenv("LLMI_SERVER", f"{sys.executable} -c import time;time.sleep(60)")
    monkeypatch.setattr(launch, "gpu_probe", lambda: "GPU: stub")
    t0 = time.monotonic()
    assert launch.main(["--max-wait", "1", "--interval", "0.2", "--", "--port", "1"]) == 1
    assert time.monotonic() - t0 < 20
