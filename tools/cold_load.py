"""Cold-start readiness of the llama-server drop-in: the time from
exec of `llama-server -m <model> -c <ctx> -ngl 99` to the first `GET /health` 200, with
the model file's pages dropped from the page cache first (fsync + posix_fadvise
DONTNEED: the state of a freshly booted pod), then once more warm.  Compared against
scripts/start.sh's readiness loop (MAX_WAIT=30 attempts, one a second, :600-620).

  python tools/cold_load.py [--preset llama3-70b-q4km] [--ctx 16384] [--port 18089]

Prints one JSON line.  The parent never touches the GPU; the server is a child process
group, ended by its own pgid."""
import argparse
import json
import os
import signal
import subprocess
import sys
import time
import urllib.error
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERVER = os.path.join(ROOT, "llama-gguf-inference_amd", "bin", "llama-server")


def drop_cache(path: str) -> None:
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
    finally:
        os.close(fd)


def resident_frac(path: str) -> float:
    """Fraction of the file's pages in the page cache (mincore over a read-only mapping)."""
    import ctypes

    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    libc.mincore.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    size = os.path.getsize(path)
    page = os.sysconf("SC_PAGE_SIZE")
    fd = os.open(path, os.O_RDONLY)
    try:
        addr = libc.mmap(None, size, 1, 1, fd, 0)  # PROT_READ, MAP_SHARED
        if addr in (None, ctypes.c_void_p(-1).value):
            return -1.0
        n = (size + page - 1) // page
        vec = (ctypes.c_ubyte * n)()
        rc = libc.mincore(ctypes.c_void_p(addr), size, vec)
        libc.munmap(ctypes.c_void_p(addr), size)
        if rc != 0:
            return -1.0
        return sum(bytes(vec).count(b) for b in (b"\x01", b"\x03")) / n
    finally:
        os.close(fd)


def health(port: int) -> int:
    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/health", timeout=2) as r:
            return r.status
    except urllib.error.HTTPError as e:
        return e.code
    except OSError:
        return 0


def ready_time(path: str, ctx: int, port: int, limit: float, log: str) -> dict:
    t0 = time.perf_counter()
    with open(log, "w") as lf:
        p = subprocess.Popen([SERVER, "-m", path, "-c", str(ctx), "-ngl", "99", "--host", "127.0.0.1", "--port", str(port)],
                             stdout=lf, stderr=subprocess.STDOUT, start_new_session=True)
    first_503 = None
    try:
        while True:
            el = time.perf_counter() - t0
            code = health(port)
            if code == 503 and first_503 is None:
                first_503 = el
            if code == 200:
                return {"ready_s": round(el, 2), "http_up_s": round(first_503 if first_503 is not None else el, 2)}
            if p.poll() is not None:
                return {"error": f"server exited rc={p.returncode}", "after_s": round(el, 2)}
            if el > limit:
                return {"error": f"not ready after {limit:.0f}s"}
            time.sleep(0.1)
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGTERM)
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama3-70b-q4km")
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--ctx", type=int, default=16384)
    ap.add_argument("--port", type=int, default=18089)
    ap.add_argument("--model-dir", default=os.environ.get("LLMI_BENCH_DIR", "/tmp/llmi_bench"))
    ap.add_argument("--limit", type=float, default=240.0)
    ap.add_argument("--out", default="gpurun_out/cold_load")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    path = os.path.join(a.model_dir, f"{a.preset}-s{a.seed}.gguf")
    res = {"preset": a.preset, "ctx": a.ctx, "model": path}
    if not os.path.exists(path):  # the synthetic writer in a child (this process loads no HIP library)
        os.makedirs(a.model_dir, exist_ok=True)
        t = time.perf_counter()
        tmp = path + f".tmp{os.getpid()}"
        subprocess.run([sys.executable, "-c", "import sys, llmi; llmi.write_synthetic_gguf(sys.argv[1], sys.argv[2], seed=int(sys.argv[3]))",
                        tmp, a.preset, str(a.seed)], check=True, env=dict(os.environ, PYTHONPATH=os.path.join(ROOT, "llama-gguf-inference_amd")))
        os.replace(tmp, path)
        res["write_s"] = round(time.perf_counter() - t, 1)
    res["file_GB"] = round(os.path.getsize(path) / 1e9, 2)
    res["resident_before_drop"] = round(resident_frac(path), 4)
    drop_cache(path)
    res["resident_after_drop"] = round(resident_frac(path), 4)
    res["cold"] = ready_time(path, a.ctx, a.port, a.limit, os.path.join(a.out, "cold.log"))
    res["warm"] = ready_time(path, a.ctx, a.port, a.limit, os.path.join(a.out, "warm.log"))
    res["start_sh_window_s"] = 30
    print(json.dumps(res), flush=True)
    return 0 if "ready_s" in res["cold"] else 1


if __name__ == "__main__":
    sys.exit(main())
