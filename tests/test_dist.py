"""Multi-process (world_size 2, gloo on CPU) coverage of bench.py's N>1 harness: the
barrier-bracketed timed region, the max-over-ranks time, whole-job aggregation and
the rank-0 broadcast used for the RCCL unique id.  Replicas only: no data-path
collective exists to test."""
from __future__ import annotations

import os
import socket
import sys
import time

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FakeEngine:
    """Stands in for LlmiEngine: rank r takes (r+1)*10 ms per run()."""

    def __init__(self, rank):
        self.rank = rank
        self.runs = []
        self.pos = 128  # after the C2 prompt


    def warmup(self, n):
        self.runs.append(("warmup", n))

    def run(self, n):
        self.runs.append(("run", n))
        time.sleep(0.01 * (self.rank + 1))

    def sync(self):
        pass


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench

    d = bench.Dist("gloo")
    eng = FakeEngine(rank)
    dt, dt_max = bench.timed_decode(eng, d, steps=7, warmup=3)
    uid = d.bcast_bytes(b"unique-id-from-rank0" if rank == 0 else None)
    q.put((rank, dt, dt_max, eng.runs, uid))
    d.close()


@pytest.mark.timeout(120)
def test_two_rank_timed_region_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    (r0, dt0, max0, runs0, uid0), (r1, dt1, max1, runs1, uid1) = res
    assert max0 == max1 == pytest.approx(max(dt0, dt1))
    assert max0 >= 0.02  # the slower rank's 20 ms dominates the job time
    # untimed steps up to the C2 trajectory's mid window (bench.window_start), then K
    sys.path.insert(0, ROOT)
    import bench

    pre = bench.window_start(128, 7, 3) - 128
    assert pre >= 3
    assert runs0 == runs1 == [("warmup", pre), ("run", 7)]
    assert uid0 == uid1 == b"unique-id-from-rank0"


class StubLoader:
    """Records how bench.load_replica loads this rank's replica (no GPU, no RCCL)."""

    def __init__(self):
        self.calls = []

    def fanout(self, path, gpu, uid, nranks, rank):
        self.calls.append(("fanout", path, gpu, uid, nranks, rank))
        return "model"

    def plain(self, path, gpu):
        self.calls.append(("plain", path, gpu))
        return "model"


def _fanout_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench

    d = bench.Dist("gloo")
    made = []

    def uid_fn():
        made.append(rank)
        return b"rccl-uid-" + bytes([7] * 8)

    ld = StubLoader()
    m, s = bench.load_replica("/x.gguf", d, uid_fn, ld.fanout, ld.plain)
    q.put((rank, made, ld.calls, m == "model" and s >= 0))
    d.close()


@pytest.mark.timeout(120)
def test_replica_fanout_call_sequence_gloo():
    """bench.py's weight fan-out at world size 2: only rank 0 creates the RCCL unique id,
    both ranks receive the same bytes over the process group and load through
    llmi_model_load_fanout once with (path, their GPU, uid, nranks=2, their rank)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fanout_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    (r0, made0, calls0, ok0), (r1, made1, calls1, ok1) = res
    assert made0 == [0] and made1 == []
    uid = b"rccl-uid-" + bytes([7] * 8)
    assert calls0 == [("fanout", "/x.gguf", 0, uid, 2, 0)] and calls1 == [("fanout", "/x.gguf", 1, uid, 2, 1)]
    assert ok0 and ok1


def test_single_rank_loads_plain():
    """One rank: no RCCL id, no fan-out, a plain load on LOCAL_RANK's GPU."""
    sys.path.insert(0, ROOT)
    import bench

    class D:
        world, rank, local_rank = 1, 0, 0

    ld = StubLoader()
    m, s = bench.load_replica("/x.gguf", D(), lambda: pytest.fail("no uid on one rank"), ld.fanout, ld.plain)
    assert m == "model" and s == 0.0 and ld.calls == [("plain", "/x.gguf", 0)]


def _check_worker(rank, world, port, q, mode):
    """mode 'fail1': rank 1's load raises; 'hash': the replicas' hashes differ; 'ok'."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench

    d = bench.Dist("gloo")

    def fanout(path, gpu, uid, nranks, r):
        if mode == "fail1" and r == 1:
            raise RuntimeError("llmi_model_load_fanout: the root rank's upload failed")
        return f"model{r}"

    def arena_hash(m):
        return 1234 + (int(m[-1]) if mode == "hash" else 0)

    try:
        bench.load_replica("/x.gguf", d, lambda: b"uid", fanout, lambda p, g: "plain", arena_hash=arena_hash)
        q.put((rank, "ok"))
    except RuntimeError as e:
        q.put((rank, str(e)))
        d.close()
        sys.exit(3)
    d.close()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("mode", ["fail1", "hash", "ok"])
def test_replica_check_every_rank_fails_together_gloo(mode):
    """after the fan-out every rank's load status and arena hash are
    gathered; a failure on ANY rank (or a replica whose hash differs from rank 0's) makes
    BOTH ranks exit non-zero, with no hang; equal hashes let both go on."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_check_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(30)
    codes = [p.exitcode for p in procs]
    if mode == "ok":
        assert codes == [0, 0] and res == {0: "ok", 1: "ok"}
    else:
        assert codes == [3, 3], (codes, res)
        want = "failed on rank(s) [(1," if mode == "fail1" else "hashes differ"
        assert all(want in res[r] for r in range(world)), res
