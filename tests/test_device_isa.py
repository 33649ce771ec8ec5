"""Device-code guard (CPU): libllmi.so's gfx950 code object holds no mixed-precision
fused ops (v_fma_mix* / v_mad_mix*).

hipcc folds `(_Float16)(a * b)` into v_fma_mixlo_f16 even under -ffp-contract=off: one
rounding of the exact product straight to f16, where ggml rounds to f32 and then to f16.
On an exact f16 tie the two differ by one ulp, which moved softmax probabilities off
the oracle ("Resolved: the attention divergence").  f2h() in
csrc/kernels.hip hides its operand from that fold; this test keeps it that way."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "llama-gguf-inference_amd", "lib", "libllmi.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else shutil.which(name)


@pytest.mark.skipif(not os.path.exists(SO), reason="libllmi.so not built")
def test_no_mixed_precision_fma_in_device_code(tmp_path):
    objcopy, bundler, objdump = _tool("llvm-objcopy"), _tool("clang-offload-bundler"), _tool("llvm-objdump")
    if not (objcopy and bundler and objdump):
        pytest.skip("ROCm LLVM tools not found")
    fat, dev = tmp_path / "fat.bin", tmp_path / "dev.o"
    subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fat}", SO], check=True)
    subprocess.run([bundler, "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}",
                    f"--output={dev}", "--unbundle"], check=True)
    asm = subprocess.run([objdump, "-d", str(dev)], check=True, capture_output=True, text=True).stdout
    assert "v_cvt_f16_f32" in asm, "device code not found in the bundle"
    bad = [ln.strip() for ln in asm.splitlines() if "_mix" in ln and ("v_fma_mix" in ln or "v_mad_mix" in ln)]
    assert not bad, f"{len(bad)} mixed-precision fused ops, e.g. {bad[:3]}"
