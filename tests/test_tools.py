"""Host-side checks of the measurement tools (no GPU): the per-class counter summary of
tools/kernel_classes.py, bench.py's host-CPU probe, and the numerics field of the C ABI's
model params."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)


def _write_counters(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Process_Id", "Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value",
                                          "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_kernel_classes_by_name_and_place(tmp_path):
    import kernel_classes as kc

    names = ["llmi::k_embed(llmi::EmbArgs)",
             "void llmi::k_matvec<0, true, 2, 12, 1, 12, 256, 0>(llmi::MVArgs)",
             "void llmi::k_attn_d<128, 4, 8>(llmi::AttnArgs, int, int, int, int)",
             "void llmi::k_matvec<0, false, 1, 12, 1, 12, 256, 0>(llmi::MVArgs)",   # attn_output
             "void llmi::k_matvec<0, true, 3, 12, 1, 12, 256, 0>(llmi::MVArgs)",
             "void llmi::k_matvec<0, false, 1, 12, 2, 12, 512, 0>(llmi::MVArgs)",   # ffn_down
             "void llmi::k_matvec<0, true, 4, 14, 1, 14, 256, 0>(llmi::MVArgs)"]
    rows = []
    for i, n in enumerate(names):
        rows.append({"Process_Id": 1, "Dispatch_Id": i + 1, "Kernel_Name": n, "Counter_Name": "FETCH_SIZE",
                     "Counter_Value": 1000.0 * (i + 1), "Start_Timestamp": 0, "End_Timestamp": 2000 * (i + 1)})
    _write_counters(str(tmp_path / "p1" / "run_counter_collection.csv"), rows)
    res = kc.step_classes(str(tmp_path), "t")["classes"]
    assert set(res) == {"embed", "qkv", "attention", "attn_output", "gate_up", "ffn_down", "output"}
    assert res["attn_output"]["fetch_MB_per_launch"] == round(4000.0 * 2048 / 1e6, 3)
    assert res["ffn_down"]["fetch_MB_per_launch"] == round(6000.0 * 2048 / 1e6, 3)
    assert res["gate_up"]["us_profiled"] == 10.0


def test_bench_host_cpu_probe():
    import bench

    c = bench.host_cpu()
    assert c["logical_cpus_granted"] >= 1 and c["logical_cpus"] >= c["logical_cpus_granted"]
    assert c["cgroup_cpu_quota"] is None or c["cgroup_cpu_quota"] >= 1


def test_model_params_numerics_default():
    sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))
    from llmi._lib import lib

    p = lib().llama_model_default_params()
    assert p.numerics == 0 and p.n_gpu_layers != 0
