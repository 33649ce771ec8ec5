"""The replica fan-out schedule (engine.cpp fanout_plan), host only:
the arena goes out in 256 MB pieces, each issued after the first upload prefix that
covers it -- so the broadcast of piece k overlaps the upload of what follows it.
(llmi_model_load_fanout / llmi_model_load_replicated run this schedule on RCCL;
unmeasured on more than one GPU until the driver's 8-GPU run.)"""
from __future__ import annotations

import numpy as np

import llmi

MB = 1 << 20


def _check(arena, chunk, prefix):
    ready = llmi.fanout_plan(arena, chunk, prefix)
    n = (arena + chunk - 1) // chunk
    assert len(ready) == n
    # pieces tile [0, arena) exactly, none longer than chunk
    ends = [min((k + 1) * chunk, arena) for k in range(n)]
    assert ends[-1] == arena and all(e - k * chunk <= chunk for k, e in enumerate(ends))
    for k, r in enumerate(ready):
        assert 0 <= r < len(prefix)
        assert prefix[r] >= ends[k], "a piece goes out before the upload finished it"
        assert r == 0 or prefix[r - 1] < ends[k], "a piece waits longer than it must"
    assert ready == sorted(ready)
    return ready


def test_pieces_follow_the_upload_prefix():
    # 8B-like arena: embedding 295 MB, norm, output 431 MB, then 32 layers of ~131 MB
    sizes = [295 * MB, 16 * 1024, 431 * MB] + [131 * MB] * 32
    prefix = list(np.cumsum(sizes))
    arena = prefix[-1] + 4096
    prefix[-1] = arena  # the last hook reports the padded arena end
    ready = _check(arena, 256 * MB, prefix)
    assert ready[0] == 0 and ready[1] == 2  # 256 MB after the embedding; 512 MB needs the output head


def test_small_arena_single_piece_and_exact_multiples():
    assert _check(1000, 256 * MB, [400, 1000]) == [1]
    assert _check(512 * MB, 256 * MB, [256 * MB, 512 * MB]) == [0, 1]


def test_huge_tensor_releases_many_pieces_at_once():
    ready = _check(4096 * MB, 256 * MB, [100 * MB, 4000 * MB, 4096 * MB])
    assert ready.count(1) == 15 and ready[-1] == 2


def test_empty_arena():
    assert llmi.fanout_plan(0, 256 * MB, []) == []
