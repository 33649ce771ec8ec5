"""The replica check of the fan-out: an order-independent
64-bit arena hash computed on the device (llmi_model_arena_hash / llmi_device_hash,
kernels.hip k_arena_hash) and compared across ranks after the pieces.

hash(bytes) = sum over 8-byte little-endian words i (mod 2^64) of
mix64(word_i ^ (i * 0x9E3779B97F4A7C15)), mix64 = splitmix64's finalizer, the last word
zero-padded.  restated below in numpy; the GPU tests compare the device with it."""
from __future__ import annotations

import numpy as np
import pytest

PHI = np.uint64(0x9E3779B97F4A7C15)


def mix64(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def arena_hash_np(b: bytes | np.ndarray) -> int:
    a = np.frombuffer(bytes(b), dtype=np.uint8)
    pad = (-len(a)) % 8
    w = np.concatenate([a, np.zeros(pad, np.uint8)]).view("<u8")
    i = np.arange(len(w), dtype=np.uint64)
    with np.errstate(over="ignore"):
        return int(mix64(w ^ (i * PHI)).sum(dtype=np.uint64))


def test_hash_restatement_properties():
    rng = np.random.default_rng(1)
    b = rng.integers(0, 256, 4099, dtype=np.uint8).tobytes()
    h = arena_hash_np(b)
    assert h == arena_hash_np(b)
    flipped = bytearray(b)
    flipped[4000] ^= 1
    assert arena_hash_np(bytes(flipped)) != h
    # swapping two words changes it too (the index enters every term)
    sw = bytearray(b)
    sw[0:8], sw[8:16] = b[8:16], b[0:8]
    assert arena_hash_np(bytes(sw)) != h
    assert arena_hash_np(b"") == 0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [8, 16, 4099, 1 << 20, (1 << 20) + 24])
def test_device_hash_equals_restatement(gpu, n):
    import torch

    import llmi

    g = torch.Generator().manual_seed(n)
    host = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g)
    dev = host.to("cuda:0")
    assert llmi.device_hash(dev.data_ptr(), n) == arena_hash_np(host.numpy().tobytes())
    dev[n // 2] ^= 0x10
    torch.cuda.synchronize()
    assert llmi.device_hash(dev.data_ptr(), n) != arena_hash_np(host.numpy().tobytes())


@pytest.mark.gpu
def test_arena_hash_plain_equals_fanout_one_rank(gpu, synth_dir):
    """The hash of a plain load equals the hash of llmi_model_load_fanout(nranks=1) of the
    same file, and matches the numpy restatement of the arena bytes."""
    import torch

    import llmi

    path = str(synth_dir / "tinyllama-q8_0-L2h.gguf")
    llmi.write_synthetic_gguf(path, "tinyllama-q8_0", seed=11, n_layer=2)
    a = llmi.Model(path)
    b = llmi.Model.load_fanout(path, 0, llmi.rccl_unique_id(), 1, 0)
    ha, hb = a.arena_hash(), b.arena_hash()
    assert ha == hb
    ptr, nbytes = a.arena()
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemcpy(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 3) == 0
    assert ha == arena_hash_np(buf.cpu().numpy().tobytes())
    b.close()
    a.close()
