"""Diagnostic: which llmi call leaves a sticky HIP error behind (peek after each call)."""
import ctypes as C, os, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
import llmi
hip = C.CDLL("libamdhip64.so")
hip.hipPeekAtLastError.restype = C.c_int
hip.hipGetErrorString.restype = C.c_char_p
def peek(tag):
    e = hip.hipPeekAtLastError()
    print(f"{tag:40s} lastError={e} {hip.hipGetErrorString(e).decode()}", flush=True)
peek("start")
print("devices", llmi.device_count()); peek("device_count")
td = tempfile.mkdtemp(); path = os.path.join(td, "t.gguf")
llmi.write_synthetic_gguf(path, "tiny-mixed", seed=1); peek("write")
m = llmi.Model(path); peek("model")
c = llmi.Context(m, n_ctx=32); peek("context")
print(c.decode([1], pos=[32])); peek("decode no-slot")
print(c.decode([m.n_vocab])); peek("decode bad token")
print(c.decode([1, 2, 3])); peek("decode ok")
c.logits(-1); peek("logits")
try:
    llmi.Model(path, n_gpu_layers=0)
except llmi.LlmiError as e:
    print("expected:", e)
peek("ngl0")
c.kv_clear(); peek("kv_clear")
print(c.generate_greedy(1, 0, 5)); peek("generate")
del c; peek("del ctx")
del m; peek("del model")
import torch
x = torch.zeros(10, device="cuda"); peek("torch alloc")
print("ok")
