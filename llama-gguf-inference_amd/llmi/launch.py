"""GPU-path launcher: the GPU probe and readiness wait of the reference's
scripts/start.sh around llmi's llama-server (ops parity).

start.sh logs `nvidia-smi --query-gpu=name,memory.total` (:371-377), starts
`/app/llama-server ...` (:473-521) and then polls `GET /health` with the backend key once
a second for MAX_WAIT=30 s (:600-635), failing when the server process dies or never
answers.  This restates those steps for MI355X: the probe is `amd-smi` (rocm-smi as the
fallback), the wait is configurable (a cold 42.5 GB 70B load needs more than 30 s), and
the launcher then forwards signals and exits with the server's status.

  python -m llmi.launch [--max-wait S] [--port P] [--api-key-file F] -- <llama-server args>
  env: LLMI_READY_WAIT (default 30, start.sh's MAX_WAIT), LLMI_SERVER (server command)
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import signal
import subprocess
import sys
import time
import urllib.error
import urllib.request
from typing import Callable, Optional

HERE = os.path.dirname(os.path.abspath(__file__))
SERVER = os.path.join(os.path.dirname(HERE), "bin", "llama-server")


def log(msg: str) -> None:
    print(f"[llmi-launch] {msg}", file=sys.stderr, flush=True)


def gpu_probe(run: Callable = subprocess.run) -> str:
    """One log line naming the GPUs and their memory (start.sh:371-377's counterpart)."""
    if shutil.which("amd-smi"):
        try:
            r = run(["amd-smi", "static", "--asic", "--vram", "--json"], capture_output=True, text=True, timeout=20)
            if r.returncode == 0:
                data = json.loads(r.stdout)
                gpus = data if isinstance(data, list) else data.get("gpu_data", data.get("gpus", []))
                parts = []
                for g in gpus:
                    name = (g.get("asic") or {}).get("market_name", "?")
                    vram = (g.get("vram") or {}).get("size", {})
                    size = f"{vram.get('value')} {vram.get('unit', '')}".strip() if isinstance(vram, dict) else str(vram)
                    parts.append(f"{name}, {size}")
                if parts:
                    return f"GPU: {len(parts)} x [{'; '.join(parts)}] (amd-smi)"
        except (OSError, ValueError, subprocess.SubprocessError):
            pass
    if shutil.which("rocm-smi"):
        try:
            r = run(["rocm-smi", "--showproductname", "--showmeminfo", "vram", "--csv"], capture_output=True,
                    text=True, timeout=20)
            if r.returncode == 0 and r.stdout.strip():
                return "GPU: " + " | ".join(ln for ln in r.stdout.strip().splitlines()[1:] if ln) + " (rocm-smi)"
        except (OSError, subprocess.SubprocessError):
            pass
    return "amd-smi / rocm-smi not available (no GPU visible to the launcher)"


def wait_ready(port: int, key: Optional[str], max_wait: float, alive: Callable[[], bool], interval: float = 1.0,
               host: str = "127.0.0.1") -> bool:
    """Poll /health (start.sh:600-635): True once it answers 200; False when the process
    died or max_wait seconds passed.  Progress is logged every 5 attempts."""
    t0 = time.monotonic()
    attempt = 0
    while True:
        attempt += 1
        req = urllib.request.Request(f"http://{host}:{port}/health")
        if key:
            req.add_header("Authorization", f"Bearer {key}")
        try:
            with urllib.request.urlopen(req, timeout=2) as r:
                if r.status == 200:
                    log(f"backend ready (attempt {attempt}, {time.monotonic() - t0:.1f}s): {r.read()[:200].decode()}")
                    return True
        except (urllib.error.URLError, OSError):
            pass
        if not alive():
            log("ERROR: llama-server process died during the readiness wait")
            return False
        if time.monotonic() - t0 >= max_wait:
            log(f"ERROR: backend not ready after {max_wait:.0f} seconds")
            return False
        if attempt % 5 == 0:
            log(f"waiting for backend to be ready ({time.monotonic() - t0:.0f}/{max_wait:.0f}s)...")
        time.sleep(interval)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="llmi-launch")
    ap.add_argument("--max-wait", type=float, default=float(os.environ.get("LLMI_READY_WAIT", "30")))
    ap.add_argument("--interval", type=float, default=1.0)
    ap.add_argument("server_args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    args = [x for x in a.server_args if x != "--"]
    port, key = 8080, None
    for i, x in enumerate(args):
        if x == "--port" and i + 1 < len(args):
            port = int(args[i + 1])
        if x == "--api-key-file" and i + 1 < len(args):
            key = open(args[i + 1]).read().strip()
        if x == "--api-key" and i + 1 < len(args):
            key = args[i + 1]
    log("--- GPU Check ---")
    log(gpu_probe())
    cmd = os.environ.get("LLMI_SERVER", SERVER).split() + args
    log(f"starting: {' '.join(cmd)}")
    child = subprocess.Popen(cmd)
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda s, f: child.send_signal(s))
    if not wait_ready(port, key, a.max_wait, lambda: child.poll() is None, a.interval):
        if child.poll() is None:
            child.terminate()
            try:
                child.wait(10)
            except subprocess.TimeoutExpired:
                child.kill()
        return 1
    return child.wait()


if __name__ == "__main__":
    sys.exit(main())
