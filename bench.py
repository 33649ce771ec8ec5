#!/usr/bin/env python3
"""bench.py — decode tokens/sec + achieved HBM GB/s, Llama-3-8B Q4_K_M, 1->8 MI355X.

BASELINE.json `metric` on `configs[1]`: Llama-3-8B-Instruct Q4_K_M, 128-token prompt ->
512-token greedy decode (context 128 -> 640), one model replica per GPU.  A STEP is one
decoded token (one pass of the hot path: 162 kernel launches replayed from a HIP graph;
the next token is fed back on the device).  Workload per rank: prefill the 128-token
prompt (untimed), then untimed decode steps up to the timed window, W warmup tokens
among them, then K timed tokens.  The window is placed on the C2 trajectory so that its
mean context is the trajectory's (383.5): the defaults (W=32, K=480) time positions
160..639; a short window (e.g. the driver's K=20) is centred at position 374..393.
Beside `value`, `c2_full` times the whole trajectory: all 512 decode tokens after a
fresh 128-token prompt.

Multi-GPU (`torch.distributed.run --nproc-per-node N`): replicas only — each rank
decodes its own stream (prompt seed 4+rank) with no data-path collective; rank 0's
weights are fanned out to the other ranks by RCCL broadcasts over xGMI
(llmi_model_load_fanout: 256 MB pieces pipelined behind rank 0's upload), outside the
timed region.  value = N*K / max-over-ranks time.

Synthetic data: a GGUF with the exact Llama-3-8B Q4_K_M shapes and type table,
random-init blocks (llmi_synth.h); there is no network for real checkpoints.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "llama-gguf-inference_amd"))

import torch  # noqa: E402  (before libllmi: one HIP runtime per process, see llmi/_lib.py)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak per GPU (MI355X_MICROARCH.md)
DOMINANT = "ffn_gate_up"  # k_matvec<..., EPI_SWIGLU>: fused ffn_gate+ffn_up matvec + SwiGLU
# ffn_gate / ffn_up weight type of each synthetic preset (llmi_synth.h type tables)
GATE_TYPE = {"llama3-8b-q4km": "Q4_K", "llama3-70b-q4km": "Q4_K", "mistral7b-q6k": "Q6_K",
             "mistral7b-q5km": "Q5_K", "tinyllama-q8_0": "Q8_0"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=480)
    ap.add_argument("--warmup", type=int, default=32)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--preset", default="llama3-8b-q4km")
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--model-dir", default=os.environ.get("LLMI_BENCH_DIR", "/tmp/llmi_bench"))
    ap.add_argument("--profile-steps", type=int, default=20)
    ap.add_argument("--cpu-sample-tokens", type=int, default=20, help="timed CPU-baseline tokens (at the GPU window)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--batch-seqs", default="2,4,8",
                    help="continuous-batching leg: sequence counts to time (comma list, '' to skip)")
    ap.add_argument("--batch-steps", type=int, default=64)
    ap.add_argument("--eager", action="store_true",
                    help="launch the step kernels one by one instead of replaying HIP graphs (PMC passes)")
    ap.add_argument("--no-c2-full", action="store_true", help="skip the full-trajectory (128 -> 640) timing")
    ap.add_argument("--profile-dir", default=os.path.join(ROOT, "profiles", "r06"),
                    help="committed rocprof evidence: traffic_<preset>.json (FETCH_SIZE pass, rocprof us)")
    ap.add_argument("--experiment", action="store_true", help="allow LLMI_EXP_* knobs (line marked as an experiment)")
    ap.add_argument("--numerics", choices=("generic", "x86"), default="generic",
                    help="fp32 association of every kernel (DESIGN.md §5): ggml's generic order, or the oracle's "
                         "model of upstream's x86 AVX2 association (match with the reference's CPU image unpinned)")
    ap.add_argument("--no-other-numerics", action="store_true",
                    help="skip the leg that times the same window in the other numerics mode")
    return ap.parse_args(argv)


class Dist:
    """Barrier / max-reduce / broadcast over torch.distributed when WORLD_SIZE > 1."""

    def __init__(self, backend: str):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if backend == "nccl":
                torch.cuda.set_device(self.local_rank)
            dist.init_process_group(backend=backend)
            self.dist = dist
            self.backend = backend

    def barrier(self):
        if self.dist:
            if self.backend == "nccl":
                import torch

                self.dist.barrier(device_ids=[self.local_rank])
                torch.cuda.synchronize()
            else:
                self.dist.barrier()

    def max(self, v: float) -> float:
        if not self.dist:
            return v
        import torch

        dev = f"cuda:{self.local_rank}" if self.backend == "nccl" else "cpu"
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, obj) -> list:
        """Every rank's `obj`, in rank order (all_gather_object; [obj] on one rank)."""
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def bcast_bytes(self, b: bytes | None) -> bytes:
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


C2_PROMPT, C2_DECODE = 128, 512  # BASELINE.json configs[1]: 128-token prompt -> 512-token decode


def window_start(prompt: int, steps: int, warmup: int) -> int:
    """First position of the timed window: its mean context is the C2 trajectory's
    (positions prompt .. prompt+511), and at least W warmup steps precede it."""
    mid = prompt + (C2_DECODE - 1) / 2.0
    return max(prompt + warmup, int(round(mid - (steps - 1) / 2.0)))


def timed_decode(engine, dist: Dist, steps: int, warmup: int) -> tuple[float, float]:
    """The contract's timed region: untimed steps up to the window (the last W of them the
    warmup), then exactly K steps bracketed by barrier + device sync on both sides;
    returns (this rank's seconds, max over ranks)."""
    pre = window_start(engine.pos, steps, warmup) - engine.pos
    engine.warmup(pre)
    dist.barrier()
    engine.sync()
    t0 = time.perf_counter()
    engine.run(steps)
    engine.sync()
    dist.barrier()
    dt = time.perf_counter() - t0
    return dt, dist.max(dt)


def load_replica(path: str, dist: Dist, rccl_unique_id, load_fanout, load_plain, arena_hash=None):
    """This rank's replica of the model.  One rank: load_plain(path, gpu).
    Several: rank 0 makes the RCCL unique id, the torch.distributed group broadcasts it,
    and every rank calls load_fanout(path, gpu, uid, nranks, rank) (llmi_model_load_fanout):
    rank 0 uploads the GGUF and the arena reaches the other ranks over xGMI in 256 MB
    pieces pipelined behind that upload.  Then every rank's (load error, arena_hash(model))
    is gathered over the process group: if any rank failed or any replica's hash differs
    from rank 0's, EVERY rank raises (and exits non-zero) instead of timing garbage or
    hanging in the next barrier.  Returns (model, fan-out seconds of this rank, 0.0 on one
    rank)."""
    if dist.world <= 1:
        return load_plain(path, dist.local_rank), 0.0
    uid = dist.bcast_bytes(rccl_unique_id() if dist.rank == 0 else None)
    t = time.perf_counter()
    m, err, h = None, None, None
    try:
        m = load_fanout(path, dist.local_rank, uid, dist.world, dist.rank)
        if arena_hash is not None:
            h = arena_hash(m)
    except Exception as e:  # reported to every rank below
        err = f"{type(e).__name__}: {e}"
    dt = time.perf_counter() - t
    views = dist.gather((err, h))
    failed = [(r, e) for r, (e, _) in enumerate(views) if e]
    if failed:
        raise RuntimeError(f"replica load failed on rank(s) {failed}")
    if len({hv for _, hv in views}) > 1:
        raise RuntimeError(f"replica arena hashes differ: {[hv for _, hv in views]}")
    return m, dt


class LlmiEngine:
    """One replica on this rank's GPU driven through the C ABI (libllmi.so)."""

    def __init__(self, args, dist: Dist):
        import numpy as np

        import llmi

        self.llmi = llmi
        self.args = args
        self.dist = dist
        path = os.path.join(args.model_dir, f"{args.preset}-s{args.seed}.gguf")
        if dist.local_rank == 0 and not os.path.exists(path):
            os.makedirs(args.model_dir, exist_ok=True)
            tmp = path + f".tmp{os.getpid()}"
            t = time.perf_counter()
            llmi.write_synthetic_gguf(tmp, args.preset, seed=args.seed)
            os.replace(tmp, path)
            log(f"wrote {path} in {time.perf_counter() - t:.1f}s")
        dist.barrier()
        self.path = path
        self.gate_type = GATE_TYPE.get(args.preset, "?")
        t = time.perf_counter()
        self.numerics = llmi.NUMERICS_X86 if args.numerics == "x86" else llmi.NUMERICS_GENERIC
        num = self.numerics
        self.model, self.fanout_s = load_replica(
            path, dist, llmi.rccl_unique_id,
            lambda p, g, uid, nr, r: llmi.Model.load_fanout(p, g, uid, nr, r, numerics=num),
            lambda p, g: llmi.Model(p, main_gpu=g, numerics=num),
            arena_hash=lambda m: m.arena_hash())
        self.load_s = time.perf_counter() - t
        last = window_start(args.prompt, args.steps, args.warmup) + args.steps
        n_ctx = ((max(last, args.prompt + C2_DECODE) + args.profile_steps + 2 + 255) // 256) * 256
        self.ctx = llmi.Context(self.model, n_ctx=n_ctx, use_graphs=not args.eager)
        rng = np.random.default_rng(4 + dist.rank)
        bos = self.model.bos if self.model.bos >= 0 else 1
        self.prompt = [bos] + [int(t) for t in rng.integers(0, min(128000, self.model.n_vocab), args.prompt - 1)]
        t = time.perf_counter()
        assert self.ctx.decode(self.prompt) == 0
        self.prefill_s = time.perf_counter() - t
        # warm prefill (TTFT) of the same prompt: the KV cache is rebuilt identically
        self.ctx.kv_clear()
        t = time.perf_counter()
        assert self.ctx.decode(self.prompt) == 0
        self.prefill_warm_s = time.perf_counter() - t
        self.next = self.ctx.greedy(-1)
        self.pos = len(self.prompt)
        self.generated: list[int] = []

    def warmup(self, n):
        if n > 0:
            self.run(n)

    def run(self, n):
        toks = self.ctx.generate_greedy(self.next, self.pos, n)
        self.generated += toks
        self.pos += n
        self.next = toks[-1]
        self.bytes, self.us = self.ctx.stats()

    def sync(self):
        import torch

        torch.cuda.synchronize()

    def c2_full(self) -> dict:
        """The whole C2 trajectory: the 128-token prompt again (KV cache rebuilt), then all
        512 greedy decode tokens timed (context 128 -> 640), device-resident feedback."""
        self.ctx.kv_clear()
        assert self.ctx.decode(self.prompt) == 0
        first = self.ctx.greedy(-1)
        self.sync()
        t0 = time.perf_counter()
        self.ctx.generate_greedy(first, len(self.prompt), C2_DECODE)
        self.sync()
        dt = time.perf_counter() - t0
        return {"tokens": C2_DECODE, "ctx": f"{len(self.prompt)}->{len(self.prompt) + C2_DECODE}",
                "tok_s": round(C2_DECODE / dt, 2), "ms_per_token": round(dt / C2_DECODE * 1e3, 4)}

    def profile(self, n):
        """Per-class kernel time at the current position (consumes no tokens)."""
        return self.ctx.profile_kernels(self.next, self.pos, n)

    def other_numerics(self, window: tuple[int, int]) -> dict:
        """The same timed window and the C2 trajectory in the OTHER numerics mode (a second
        replica of the weights in that mode's byte order on this GPU): reported beside
        `value`, never as it."""
        llmi = self.llmi
        num = llmi.NUMERICS_GENERIC if self.numerics == llmi.NUMERICS_X86 else llmi.NUMERICS_X86
        m = llmi.Model(self.path, main_gpu=self.dist.local_rank, numerics=num)
        ctx = llmi.Context(m, n_ctx=self.ctx.n_ctx)
        assert ctx.decode(self.prompt) == 0
        first = ctx.greedy(-1)
        pre = window[0] - len(self.prompt)
        toks = ctx.generate_greedy(first, len(self.prompt), pre) if pre > 0 else []
        nxt = toks[-1] if toks else first
        self.sync()
        t0 = time.perf_counter()
        gen = ctx.generate_greedy(nxt, window[0], window[1] - window[0])
        self.sync()
        dt = time.perf_counter() - t0
        k = window[1] - window[0]
        out = {"numerics": "x86" if num == llmi.NUMERICS_X86 else "generic", "tok_s": round(k / dt, 2),
               "ms_per_step": round(dt / k * 1e3, 4), "timed_window": list(window),
               "prefill_path": "mfma" if m.prefill_supported else "decode-steps"}
        if self.args.profile_steps > 0 and len(gen):
            prof = ctx.profile_kernels(int(gen[-1]), window[1], self.args.profile_steps)
            out["kernels"] = {k2: {"us": round(v["us"], 3), "per_step": v["launches_per_step"]} for k2, v in prof.items()}
        if self.args.prompt == C2_PROMPT and not self.args.no_c2_full:
            ctx.kv_clear()
            assert ctx.decode(self.prompt) == 0
            first = ctx.greedy(-1)
            self.sync()
            t0 = time.perf_counter()
            ctx.generate_greedy(first, len(self.prompt), C2_DECODE)
            self.sync()
            out["c2_full_tok_s"] = round(C2_DECODE / (time.perf_counter() - t0), 2)
        ctx.close()
        m.close()
        return out

    def batched(self, counts: list[int], steps: int) -> dict:
        """Continuous-batching leg (reported beside `value`, never as it): k sequences of one
        context (the same 128-token prompt length, different prompts) advance together
        through batched steps (llmi_generate_greedy_batch); aggregate tokens/s = k *
        steps / time of `steps` steps after 8 warmup steps."""
        import numpy as np

        llmi = self.llmi
        kmax = max(counts)
        n_ctx = ((self.args.prompt + steps + 8 + 2 + 255) // 256) * 256
        ctx = llmi.Context(self.model, n_ctx=n_ctx, n_seq=kmax, use_graphs=not self.args.eager)
        rng = np.random.default_rng(40)
        bos = self.model.bos if self.model.bos >= 0 else 1
        prompts = [[bos] + [int(t) for t in rng.integers(0, min(128000, self.model.n_vocab), self.args.prompt - 1)]
                   for _ in range(kmax)]
        firsts = []
        for s, p in enumerate(prompts):
            assert ctx.decode(p, seq=[s] * len(p)) == 0
            firsts.append(ctx.greedy(-1))
        out = {}
        for k in counts:
            seqs = list(range(k))
            for s in seqs:
                ctx.seq_rm(s, len(prompts[s]), -1)
            pos = [len(prompts[s]) for s in seqs]
            g = ctx.generate_greedy_batch(seqs, firsts[:k], pos, 8)
            nxt = [t[-1] for t in g]
            pos = [q + 8 for q in pos]
            self.sync()
            t0 = time.perf_counter()
            ctx.generate_greedy_batch(seqs, nxt, pos, steps)
            self.sync()
            dt = time.perf_counter() - t0
            out[str(k)] = {"tok_s": round(k * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 4)}
        ctx.close()
        return out


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def host_cpu() -> dict:
    """The host's CPU model, the logical CPUs this process may run on and its physical cores."""
    model = "?"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None  # the cgroup's CPU bandwidth limit (cpu.max "quota period"), in CPUs
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        try:  # cgroup v1
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f, open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as g:
                q, per = int(f.read()), int(g.read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return {"model": model, "logical_cpus_granted": len(os.sched_getaffinity(0)), "logical_cpus": os.cpu_count(),
            "cgroup_cpu_quota": quota, "omp_num_threads": int(omp) if omp.isdigit() else None}


def cpu_baseline(path: str, prompt: list[int], generated: list[int], window: tuple[int, int], n_tokens: int) -> dict:
    """The reference's CPU path (NGL=0: llama.cpp built for the host, Dockerfile.cpu:84-89)
    restated — oracle/, test infrastructure — timed on this host, on the GPU run's own
    workload: the same prompt and the GPU's generated tokens fill the KV cache up to the
    GPU's timed window (untimed, decode steps without logits), then n_tokens greedy decode
    steps at the window's first positions are timed.  The -O3 -march=x86-64-v3 build with
    its AVX2 dot products (the x86 kernels' maddubs/madd structure and 8-lane fp32 block
    accumulation; or_set_fast_dots), OpenMP threads = every physical core of the CPUs this
    process may run on (the reference's THREADS=0, scripts/start.sh:484-486: llama.cpp's
    own default), and again at 8 threads (its documented CPU config,
    docs/CONFIGURATION.md:579-587).  Beside it the host DRAM streaming-read rate, the
    fraction of it the decode reaches, and the decode roofline it implies."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import pyoracle as po

    po.prefer_simd()
    cpu = host_cpu()
    phys = po.physical_cores()
    # every physical core the process may use: the affinity mask, capped by the cgroup's CPU
    # quota (a GPU box grants a share of a larger host: its mask lists every CPU)
    # quota (a GPU box grants a share of a larger host: its mask lists every CPU) and by the
    # OMP_NUM_THREADS the box sets to that share
    threads = max(1, min(phys, cpu["logical_cpus_granted"], cpu["cgroup_cpu_quota"] or 1 << 30,
                         cpu["omp_num_threads"] or 1 << 30))
    fast = po.set_fast_dots(True)
    ctx_toks = (prompt + list(generated))[: window[0]]
    om = po.OracleModel(path, n_ctx=window[0] + n_tokens + 8, threads=threads)
    # the weights out of the file's page cache (on the node that wrote the file) into
    # memory whose rows are first-touched by the threads that read them (NUMA placement)
    local_bytes = om.localize()
    res = {}
    try:
        t = time.perf_counter()
        for i, tk in enumerate(ctx_toks[:-1]):  # KV rows up to the window (untimed)
            om.decode(tk, i, logits=False)
        fill_s = time.perf_counter() - t
        lg = om.decode(ctx_toks[-1], len(ctx_toks) - 1)  # -> the window's first token (untimed)
        tok0 = int(np.argmax(lg))

        def timed(nth: int) -> float:
            om.threads = nth
            tok = tok0
            t0 = time.perf_counter()
            for k in range(n_tokens):
                out = om.decode(tok, window[0] + k)
                tok = int(np.argmax(out))
            return n_tokens / (time.perf_counter() - t0)

        res["all"] = timed(threads)
        res["t8"] = timed(8)
    finally:
        po.set_fast_dots(False)
    bpt = om.bytes_per_token(window[0] + n_tokens // 2)
    om.close()
    host_gbps = po.host_stream_gbps(1 << 30, 3, threads)
    tok_s = res["all"]
    gbps = tok_s * bpt / 1e9
    return {"value": round(tok_s, 3), "unit": "tokens/s", "cores": threads, "kind": "port", "threads": threads,
            "physical_cores": phys, "host_cpu": cpu,
            "ctx_window": [window[0], window[0] + n_tokens - 1],
            "achieved_GBps": round(gbps, 2),
            "stream_frac": round(gbps / host_gbps, 4) if host_gbps > 0 else None,
            "threads_8": {"value": round(res["t8"], 3), "unit": "tokens/s",
                          "achieved_GBps": round(res["t8"] * bpt / 1e9, 2)},
            "dots": {2: "avx512bw (the AVX2 kernels at twice the width, 16-lane fp32 block accumulators)",
                     1: "avx2 (x86 kernel association)"}.get(fast, "generic scalar (no AVX2 in this build)"),
            "placement": f"decode matrices ({local_bytes / 1e9:.2f} GB) copied into rows first-touched by their "
                         f"reading thread of {threads} (oracle or_model_localize)",
            "host_dram_roofline": {"stream_read_GBps": round(host_gbps, 1),
                                   "decode_tok_s_at_roofline": round(host_gbps * 1e9 / bpt, 2)},
            "sample": f"{n_tokens} greedy decode steps at ctx {window[0]}..{window[0] + n_tokens - 1}, the GPU's timed "
                      f"window, after the same {len(prompt)}-token prompt and the GPU's generated tokens (KV rows "
                      f"filled by {len(ctx_toks) - 1} decode steps in {fill_s:.1f}s, untimed) on {os.path.basename(path)}; "
                      f"oracle/ggml_oracle.c -O3 -march=x86-64-v3 with AVX2 dots, OpenMP {threads} threads "
                      f"(every core granted: {cpu['logical_cpus_granted']} logical CPUs in the mask, cgroup quota "
                      f"{cpu['cgroup_cpu_quota']} CPUs, OMP_NUM_THREADS {cpu['omp_num_threads']}, {phys} physical "
                      f"cores; {cpu['model']}) "
                      f"and 8 threads (the reference's documented CPU config)"}


def env_knobs(allow_exp: bool = False) -> dict:
    """Every LLMI_* variable in the environment (recorded in the line); experiment-build
    knobs are refused (they remove or reorder work inside the timed region) unless
    --experiment marks the line as an experiment's, never a result."""
    knobs = {k: v for k, v in os.environ.items() if k.startswith("LLMI_")}
    bad = [k for k in knobs if k.startswith("LLMI_EXP_")]
    if bad and not allow_exp:
        raise SystemExit(f"bench.py: refusing to run with experiment knobs set: {bad}")
    return knobs


def committed_profile(profile_dir: str, preset: str) -> dict:
    """rocprof evidence committed for THIS preset (profiles/<round>/traffic_<preset>.json:
    FETCH_SIZE bytes per launch of the dominant kernel, rocprof average us); {} if none."""
    f = os.path.join(profile_dir, f"traffic_{preset}.json")
    if not os.path.exists(f):
        return {}
    try:
        d = json.load(open(f))
    except (OSError, ValueError):
        return {}
    return d if d.get("preset") == preset else {}


def dump_maps(tag: str) -> None:
    """LLMI_DUMP_MAPS=<dir>: this process's address map at a named point (profiler-crash
    forensics: resolving unsymbolised frames and fault addresses against the mapped
    objects)."""
    d = os.environ.get("LLMI_DUMP_MAPS")
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    with open("/proc/self/maps") as f, open(os.path.join(d, f"maps_{os.getpid()}_{tag}.txt"), "w") as g:
        g.write(f.read())


def main(argv=None):
    if os.environ.get("LLMI_DUMP_MAPS"):
        import faulthandler
        faulthandler.enable(all_threads=True)
    args = parse(argv)
    knobs = env_knobs(args.experiment)
    dist = Dist(os.environ.get("LLMI_DIST_BACKEND", "nccl"))
    if dist.world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={dist.world}; using WORLD_SIZE")
    n = dist.world
    eng = LlmiEngine(args, dist)
    log(f"rank {dist.rank}: {eng.model.desc} load {eng.load_s:.1f}s fanout {eng.fanout_s:.2f}s prefill "
        f"{args.prompt} tok {eng.prefill_s:.2f}s")
    dump_maps("before_timed")
    dt, dt_max = timed_decode(eng, dist, args.steps, args.warmup)
    dump_maps("after_timed")
    tok_s = n * args.steps / dt_max
    # end-to-end roofline: algorithmic bytes of the timed tokens / time (this rank)
    e2e_gbps = eng.bytes / (eng.us * 1e-6) / 1e9 if eng.us > 0 else 0.0
    window = (eng.pos - args.steps, eng.pos)
    prof = eng.profile(args.profile_steps) if args.profile_steps > 0 else {}
    c2 = eng.c2_full() if not args.no_c2_full and args.prompt == C2_PROMPT else None
    other = None
    if not args.no_other_numerics:
        try:
            other = eng.other_numerics(window)
        except Exception as e:  # reported beside the metric, never required
            log(f"other-numerics leg failed: {e}")
    counts = [int(x) for x in args.batch_seqs.split(",") if x.strip()]
    batched = None
    if counts:
        try:
            batched = eng.batched(counts, args.batch_steps)
        except Exception as e:  # reported beside the metric, never required
            log(f"batched leg failed: {e}")
    result = None
    if dist.rank == 0:
        k = prof.get(DOMINANT, {"us": 0.0, "bytes": 0.0})
        achieved = k["bytes"] / (k["us"] * 1e-6) / 1e9 if k["us"] > 0 else 0.0
        prof_c = committed_profile(args.profile_dir, args.preset)
        traffic = prof_c.get("hbm_bytes_per_launch")
        cpu = None
        if n == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(eng.path, eng.prompt, eng.generated, window,
                                   min(args.cpu_sample_tokens, window[1] - window[0]))
            except Exception as e:  # the baseline is reported, never required
                log(f"cpu baseline failed: {e}")
        result = {
            "metric": "decode tokens/sec + achieved HBM GB/s, Llama-3-8B Q4_K_M, 1->8 MI355X",
            "value": round(tok_s, 2),
            "unit": "tokens/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int8",
            "data": f"synthetic: random-init GGUF blocks with the exact {args.preset} shapes/type table "
                    f"(llmi_synth.h); random {args.prompt}-token prompts",
            "config": {"workload": f"{args.preset}: {args.prompt}-token prompt -> greedy decode on the "
                                   f"{args.prompt}->{args.prompt + C2_DECODE} trajectory, {args.steps} timed tokens at "
                                   f"positions {window[0]}..{window[1] - 1} (mean context of the trajectory), "
                                   "1 replica per GPU",
                       "model": args.preset, "prompt_tokens": args.prompt, "timed_window": list(window),
                       "parallelism": f"replicas x{n} (RCCL weight fan-out)", "global_batch": n},
            "c2_full": c2,
            "numerics": args.numerics,
            "other_numerics": other,
            "roofline": {"bound": "hbm", "kernel": f"k_matvec (ffn_gate+ffn_up {eng.gate_type} + SwiGLU)",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "traffic_source": (prof_c.get("source") if traffic else
                                            f"null: no FETCH_SIZE pass committed for preset {args.preset}"),
                         "bytes_per_launch": k["bytes"], "us_per_launch": round(k["us"], 3),
                         "us_source": "kernel start/stop events on every launch of 20 whole decode steps "
                                      "in this run, each kernel in its place in the step (llmi_profile_kernels)",
                         "rocprof_us_per_launch": prof_c.get("rocprof_us"),
                         "rocprof_frac": (round(k["bytes"] / (prof_c["rocprof_us"] * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)
                                          if prof_c.get("rocprof_us") else None)},
            "hbm_end_to_end": {"achieved_GBps": round(e2e_gbps, 1),
                               "frac_of_peak": round(e2e_gbps / HBM_PEAK_GBPS, 4),
                               "bytes_per_token": eng.bytes / max(1, args.steps)},
            "kernels": {k2: {"us": round(v["us"], 3), "GBps": round(v["GBps"], 1),
                             "per_step": v["launches_per_step"]} for k2, v in prof.items()},
            "load_s": round(eng.load_s, 2),
            "upload_s": round(eng.model.upload_s, 3),
            "prefill": {"tokens": args.prompt, "path": "mfma" if eng.model.prefill_supported else "decode-steps",
                        "ttft_ms": round(eng.prefill_warm_s * 1e3, 2),
                        "tok_per_s": round(args.prompt / max(eng.prefill_warm_s, 1e-9), 1)},
            "fanout_s": round(eng.fanout_s, 3),
            "continuous_batching": {"sequences": batched,
                                    "note": "k sequences per replica in batched steps (one weight stream per step), "
                                            f"{args.prompt}-token prompts, {args.batch_steps} timed steps; "
                                            "aggregate tokens/s of this rank; not the metric's value",
                                    "matvec": ("k_bmd's x86 fold (f16 MFMA integer sums, x86 fma lane chains) from "
                                               f"{os.environ.get('LLMI_BMM_MIN', '3')} sequences on K-quant "
                                               "segments, else k_mvn's x86 form (VALU); attention per slot"
                                               if eng.numerics == eng.llmi.NUMERICS_X86 else
                                               "k_bmd (f16 MFMA, weights staged by LDS-DMA, batch.hip; k_bmm "
                                               "with LLMI_BMM_DMA=0) from "
                                               f"{os.environ.get('LLMI_BMM_MIN', '3')} sequences on K-quant "
                                               "segments, else k_mvn (VALU)")}
            if batched else None,
            "cpu_baseline": cpu,
            "env": knobs,
            "eager": bool(args.eager),
            **({"experiment": "LLMI_EXP_* knobs set: timing of an experiment build, not a result"}
               if args.experiment else {}),
        }
        print(json.dumps(result), flush=True)
    dist.close()
    return result


if __name__ == "__main__":
    main()
