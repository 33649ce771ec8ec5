"""Independent pure-Python GGUF v3 reader (test infrastructure).

Restates the container format (upstream gguf.c / ggml docs: magic "GGUF", version,
tensor count, KV count, KV pairs, tensor infos, alignment padding, data section) from
scratch, so the C++ writer (csrc/synth_writer.cpp) and the C loaders (csrc/gguf.cpp,
oracle/ggml_oracle.c) are checked against a third implementation."""
from __future__ import annotations

import struct

GGUF_MAGIC = b"GGUF"
# value types
U8, I8, U16, I16, U32, I32, F32, BOOL, STR, ARR, U64, I64, F64 = range(13)
_SCALAR = {U8: "<B", I8: "<b", U16: "<H", I16: "<h", U32: "<I", I32: "<i", F32: "<f", BOOL: "<?",
           U64: "<Q", I64: "<q", F64: "<d"}
# ggml types: (block elements, block bytes)
GGML_TYPES = {0: ("F32", 1, 4), 1: ("F16", 1, 2), 8: ("Q8_0", 32, 34), 12: ("Q4_K", 256, 144),
              13: ("Q5_K", 256, 176), 14: ("Q6_K", 256, 210)}


class Reader:
    def __init__(self, data: bytes):
        self.d = data
        self.o = 0

    def take(self, fmt):
        v = struct.unpack_from(fmt, self.d, self.o)[0]
        self.o += struct.calcsize(fmt)
        return v

    def string(self):
        n = self.take("<Q")
        s = self.d[self.o:self.o + n].decode("utf-8")
        self.o += n
        return s

    def value(self, t):
        if t in _SCALAR:
            return self.take(_SCALAR[t])
        if t == STR:
            return self.string()
        if t == ARR:
            et = self.take("<I")
            n = self.take("<Q")
            return [self.value(et) for _ in range(n)]
        raise ValueError(f"bad GGUF value type {t}")


def read_gguf(path: str) -> dict:
    data = open(path, "rb").read()
    r = Reader(data)
    if data[:4] != GGUF_MAGIC:
        raise ValueError("not a GGUF file")
    r.o = 4
    version = r.take("<I")
    n_tensors = r.take("<Q")
    n_kv = r.take("<Q")
    kv = {}
    for _ in range(n_kv):
        k = r.string()
        t = r.take("<I")
        kv[k] = r.value(t)
    tensors = []
    for _ in range(n_tensors):
        name = r.string()
        nd = r.take("<I")
        ne = [r.take("<Q") for _ in range(nd)]
        typ = r.take("<I")
        off = r.take("<Q")
        tensors.append({"name": name, "ne": ne, "type": typ, "offset": off})
    align = kv.get("general.alignment", 32)
    data_start = (r.o + align - 1) // align * align
    for t in tensors:
        _, be, bb = GGML_TYPES[t["type"]]
        n = 1
        for e in t["ne"]:
            n *= e
        t["nbytes"] = n // be * bb
        t["data"] = data[data_start + t["offset"]: data_start + t["offset"] + t["nbytes"]]
    return {"version": version, "kv": kv, "tensors": tensors, "alignment": align, "data_start": data_start,
            "file_size": len(data)}
