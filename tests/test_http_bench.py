"""tools/http_bench.py: the reference benchmark.py's statistics restated (nearest-rank
percentiles, compute_stats keys; the cases of the reference's own tests/test_benchmark.py)
and an end-to-end run against the stand-in server producing the reference JSON shape."""
from __future__ import annotations

import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import http_bench as hb  # noqa: E402


def test_percentile_nearest_rank():
    assert hb.percentile([], 50) == 0.0
    assert hb.percentile([5.0], 50) == 5.0 and hb.percentile([5.0], 99) == 5.0
    assert hb.percentile([1.0, 2.0, 3.0, 4.0], 50) in (2.0, 3.0)
    assert hb.percentile([1.0, 2.0, 3.0, 4.0, 5.0], 50) == 3.0
    assert hb.percentile([float(x) for x in range(1, 101)], 95) >= 95.0
    assert hb.percentile([float(x) for x in range(1, 101)], 99) >= 99.0
    assert hb.percentile([10.0, 20.0, 30.0], 0) == 10.0 and hb.percentile([10.0, 20.0, 30.0], 100) == 30.0
    d = [50.0, 10.0, 30.0, 20.0, 40.0]
    assert hb.percentile(d, 50) == 30.0 and d == [50.0, 10.0, 30.0, 20.0, 40.0]


def test_compute_stats_keys():
    assert hb.compute_stats([]) == {"min": 0.0, "max": 0.0, "mean": 0.0, "p50": 0.0, "p95": 0.0, "p99": 0.0,
                                    "count": 0}
    s = hb.compute_stats([1.0, 2.0, 3.0])
    assert set(s) == {"min", "max", "mean", "p50", "p95", "p99", "count"} and s["mean"] == 2.0


def test_end_to_end_against_stand_in_server():
    from test_server import FakeEngine

    from llmi.server import make_server

    eng = FakeEngine()
    eng.ready = True
    srv = make_server(eng, "127.0.0.1", 0, "k")
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        url = f"http://127.0.0.1:{srv.server_address[1]}"
        res = hb.run_level(url, "w5 w6", 12, "k", concurrency=4, n_requests=8)
        inf = res["inference"]
        assert inf["requests_success"] == 8 and inf["requests_failed"] == 0 and inf["concurrency"] == 4
        assert inf["ttft"]["count"] == 8 and inf["tokens_per_sec"]["count"] == 8
        assert res["llmi"]["generated_tokens"] > 0
        bad = hb.run_level(url, "x", 4, "wrong-key", concurrency=1, n_requests=2, warmup=0)
        assert bad["inference"]["requests_failed"] == 2
    finally:
        srv.shutdown()
        srv.server_close()
