/*
 * llmi.h — the drop-in C ABI of the MI355X-native GGUF decode path (libllmi.so).
 *
 * The reference (zepfu/llama-gguf-inference) has no FFI of its own: it launches the
 * external llama.cpp `llama-server` (scripts/start.sh:235, argv at :473-494) and
 * proxies HTTP to it (scripts/gateway.py:699-804).  Inside that binary the decode
 * loop is driven through llama.cpp's C API (llama.h, upstream, not vendored).  This
 * header restates that llama.h surface — same names, argument meaning, return codes
 * and ownership rules — for the functions on the decode path, so the
 * ctypes binding (llmi/), a llama-server-compatible HTTP front end or any cgo caller
 * can bind it the way it would bind libllama.  Structs are llmi's own (llama.h's
 * carry many more fields), so this is API-shape compatible, not ABI compatible.
 *
 * Each entry point names the upstream function it replaces and the reference call
 * site that reaches it.  llmi_* entries are build extras.
 *
 * Threading: a context is NOT thread-safe (one host thread per context).  A model is
 * read-only and shared by contexts on its device.  No C++ exception crosses the ABI;
 * failures return NULL / a non-zero code and set the thread-local llmi_last_error().
 */
#ifndef LLMI_H
#define LLMI_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#pragma GCC visibility push(default)

typedef int32_t llama_token;
typedef int32_t llama_pos;
typedef int32_t llama_seq_id;

struct llama_model;
struct llama_context;
struct llama_vocab;

/* upstream llama_model_params (subset).  n_gpu_layers: llmi is GPU-only; 0 means the
 * reference's CPU llama-server path (Dockerfile.cpu:84-89, NGL=0) and is rejected —
 * there is no CPU fallback in the product.  Any value > 0 offloads every layer. */
struct llama_model_params {
    int32_t n_gpu_layers;
    int32_t main_gpu;      /* HIP device index */
    bool vocab_only;       /* parse metadata + vocab, upload no weights */
    bool use_mmap;         /* always true in llmi; kept for signature parity */
    bool no_upload;        /* llmi: build the device arena layout but leave it unfilled
                              (a replica that will receive the arena by RCCL broadcast) */
    int32_t numerics;      /* llmi: the fp32 association every kernel reproduces bit for bit,
                              fixed at load (the weights' device byte order depends on it):
                              LLMI_NUMERICS_GENERIC (default) ggml's generic scalar order;
                              LLMI_NUMERICS_X86 the oracle's model of upstream's x86 AVX2
                              association (non-repacked Q4_K, non-flash attention).  Whether
                              the reference's CPU image (Dockerfile.cpu:11: AVX-512 variant,
                              CPU_REPACK, -fa auto) computes these bits is unpinned — DESIGN.md §5 */
};
#define LLMI_NUMERICS_GENERIC 0
#define LLMI_NUMERICS_X86 1
/* OR-ed into either: decode attention in ggml's CPU flash-attention numerics (online
 * softmax, f16 V accumulation, glibc expf; what a llama-server without --flash-attn runs
 * when -fa auto resolves to on), oracle flag OR_X86_FA.  Such a model runs prompts as
 * decode steps (batched steps advance its sequences together, the flash attention of
 * every slot in one launch); up to 8192 positions. */
#define LLMI_NUMERICS_FA 2

/* upstream llama_context_params (subset) */
struct llama_context_params {
    uint32_t n_ctx;        /* 0 = model's context_length capped at 4096 */
    uint32_t n_batch;      /* max tokens per llama_decode call (logical batch) */
    uint32_t n_ubatch;
    uint32_t n_seq_max;    /* sequences (KV caches) per context; >= 2 enables batched
                              decode steps (continuous batching, up to 8 per step) */
    int32_t n_threads;     /* ignored (GPU) */
    bool use_graphs;       /* llmi: replay the decode step as a HIP graph (default true) */
};

/* upstream llama_batch, field for field */
struct llama_batch {
    int32_t n_tokens;
    llama_token* token;
    float* embd;           /* unsupported in llmi: must be NULL */
    llama_pos* pos;        /* NULL: consecutive positions after the context's last token */
    int32_t* n_seq_id;
    llama_seq_id** seq_id;
    int8_t* logits;        /* NULL: logits for the last token only */
};

/* ---------- lifecycle (upstream llama.h; reached via llama-server startup,
 *            scripts/start.sh:473-521) ---------- */
void llama_backend_init(void);
void llama_backend_free(void);
struct llama_model_params llama_model_default_params(void);
struct llama_context_params llama_context_default_params(void);
/* upstream llama_model_load_from_file (`-m $MODEL`, scripts/start.sh:474). NULL on error. */
struct llama_model* llama_model_load_from_file(const char* path_model, struct llama_model_params params);
void llama_model_free(struct llama_model* model);
/* upstream llama_init_from_model (`-c $CTX`, scripts/start.sh:477). NULL on error. */
struct llama_context* llama_init_from_model(struct llama_model* model, struct llama_context_params params);
void llama_free(struct llama_context* ctx);

/* ---------- batches ---------- */
struct llama_batch llama_batch_get_one(llama_token* tokens, int32_t n_tokens);
struct llama_batch llama_batch_init(int32_t n_tokens, int32_t embd, int32_t n_seq_max);
void llama_batch_free(struct llama_batch batch);

/* ---------- decode: THE HOT PATH ----------
 * upstream llama_decode, called by llama-server's slot loop for every prompt batch
 * and every generated token of /v1/chat/completions (docs/API_REFERENCE.md:341-605,
 * proxied by scripts/gateway.py:699-804).
 * Returns 0 ok; 1 no KV slot (pos >= n_ctx; recoverable); 2 aborted;
 * -1 invalid batch; < -1 fatal (-6: an in-kernel bounded wait gave up, the outputs of
 * the call are invalid).  Synchronises the device before returning. */
int32_t llama_decode(struct llama_context* ctx, struct llama_batch batch);
/* legacy upstream llama_eval: tokens at positions n_past..n_past+n_tokens-1; 0 = ok */
int llama_eval(struct llama_context* ctx, llama_token* tokens, int32_t n_tokens, int32_t n_past);

/* logits: context-owned host memory, valid until the next decode/free; never freed by
 * the caller.  i = index in the last batch of a token whose logits were requested,
 * or -1 for the last one.  NULL (and llmi_last_error) if i had no logits. */
float* llama_get_logits(struct llama_context* ctx);
float* llama_get_logits_ith(struct llama_context* ctx, int32_t i);

/* ---------- model / context introspection ---------- */
const struct llama_vocab* llama_model_get_vocab(const struct llama_model* model);
int32_t llama_vocab_n_tokens(const struct llama_vocab* vocab);
llama_token llama_vocab_bos(const struct llama_vocab* vocab);
llama_token llama_vocab_eos(const struct llama_vocab* vocab);
/* raw GGUF token text of `token` */
const char* llama_vocab_get_text(const struct llama_vocab* vocab, llama_token token);
bool llama_vocab_get_add_bos(const struct llama_vocab* vocab);
/* ---------- tokenizer (upstream llama-vocab.cpp, reached through llama-server's prompt
 * tokenization and streamed detokenization, scripts/gateway.py:699-804 -> upstream).
 * The GGUF's own tokenizer: tokenizer.ggml.model "llama" + scores -> SPM, "gpt2" +
 * merges -> byte-level BPE (llama3 / gpt-2 pre-tokenizer), otherwise greedy longest
 * match; special tokens partitioned first when parse_special (csrc/tokenizer.h). ---------- */
/* upstream llama_tokenize: writes the ids and returns their count, or -(count) when
 * n_tokens_max is too small (nothing written); INT32_MIN on bad arguments */
int32_t llama_tokenize(const struct llama_vocab* vocab, const char* text, int32_t text_len, llama_token* tokens,
                       int32_t n_tokens_max, bool add_special, bool parse_special);
/* upstream llama_token_to_piece: the token's bytes (no NUL) and their count, or -(count)
 * when length is too small; up to lstrip leading spaces skipped; special: CONTROL
 * tokens render their text (else nothing) */
int32_t llama_token_to_piece(const struct llama_vocab* vocab, llama_token token, char* buf, int32_t length,
                             int32_t lstrip, bool special);
/* upstream llama_detokenize: the pieces concatenated (remove_special: without a leading
 * BOS / trailing EOS; unparse_special: CONTROL text kept); count or -(count needed) */
int32_t llama_detokenize(const struct llama_vocab* vocab, const llama_token* tokens, int32_t n_tokens, char* text,
                         int32_t text_len_max, bool remove_special, bool unparse_special);
int32_t llama_model_n_embd(const struct llama_model* model);
int32_t llama_model_n_layer(const struct llama_model* model);
int32_t llama_model_n_head(const struct llama_model* model);
int32_t llama_model_n_head_kv(const struct llama_model* model);
int32_t llama_model_n_ctx_train(const struct llama_model* model);
uint64_t llama_model_size(const struct llama_model* model);  /* tensor bytes */
int32_t llama_model_desc(const struct llama_model* model, char* buf, size_t buf_size);
uint32_t llama_n_ctx(const struct llama_context* ctx);
/* upstream llama_memory_clear / llama_kv_self_clear: reset the KV cache of ctx */
void llama_kv_self_clear(struct llama_context* ctx);
/* upstream llama_kv_self_seq_rm / llama_memory_seq_rm (the server's slot release and
 * prompt-cache truncation): remove positions [p0, p1) of seq_id (-1: every sequence).
 * Only tail removal (p1 < 0) is supported; p0 <= 0 clears the sequence. */
bool llama_kv_self_seq_rm(struct llama_context* ctx, llama_seq_id seq_id, llama_pos p0, llama_pos p1);
/* upstream llama_memory_seq_pos_max: last position held by seq_id, -1 if empty */
int32_t llmi_seq_pos_max(const struct llama_context* ctx, llama_seq_id seq_id);

/* ---------- llmi extras ---------- */
const char* llmi_last_error(void);
/* the model's numerics (llama_model_params.numerics), -1 for NULL */
int32_t llmi_model_numerics(const struct llama_model* model);
int32_t llmi_device_count(void);
/* device-side argmax of the logits of batch entry i (-1 = last); first max wins, as
 * upstream llama_sampler_greedy.  Avoids the n_vocab*4 B logits copy. */
llama_token llmi_greedy_ith(struct llama_context* ctx, int32_t i);
/* Greedy decode of n_gen tokens starting from `first` at position pos0, entirely on
 * the device (token feedback through the on-device argmax; no host round trip per
 * token).  out[k] = token sampled after step k.  Returns n_gen or < 0 on error. */
int32_t llmi_generate_greedy(struct llama_context* ctx, llama_token first, int32_t pos0, int32_t n_gen, llama_token* out);
/* Continuous-batching form: n (1..8) distinct sequences seqs[k] of a context created with
 * n_seq_max >= 2 advance together, one batched step per token (every weight byte read
 * once per step for all of them).  Sequence k starts from first[k] at pos0[k];
 * out[k * n_gen + j] = its token after step j, bit-identical to llmi_generate_greedy of
 * that sequence alone (n = 1 runs the single-sequence step).  Returns n_gen or < 0 on error. */
int32_t llmi_generate_greedy_batch(struct llama_context* ctx, int32_t n, const int32_t* seqs, const llama_token* first,
                                   const int32_t* pos0, int32_t n_gen, llama_token* out);
/* seconds the weight upload took in llama_model_load_from_file (chunked pinned H2D,
 * double-buffered against the on-device repack; file reads included) */
double llmi_model_upload_s(const struct llama_model* model);
/* Roofline accounting of the last llama_decode / llmi_generate_greedy call:
 * algorithmic HBM bytes it streamed and its device time in microseconds. */
void llmi_last_step_stats(struct llama_context* ctx, double* bytes, double* usec);
/* Per-kernel-class device timing (roofline evidence), in situ: n_steps whole decode
 * steps at position pos0 (token `first`; the decode graph's exact kernels, grids and
 * arguments in their order) are launched one by one, every kernel armed with an event
 * pair recorded at kernel start and end (hipExtLaunchKernelGGL), so each kernel runs
 * after its real predecessor: us[k] = mean device microseconds per launch of class k
 * (execution only, no launch gaps), bytes[k] = mean algorithmic HBM bytes per launch,
 * launches[k] = launches per step.  Consumes no tokens: the context is left ready to
 * decode `first` at pos0.  Classes (arrays of LLMI_KERNEL_CLASSES): 0 embed, 1 qkv(+RoPE,
 * KV write), 2 attention (1-4 kernels, timed as one), 3 attn_output(+residual), 4
 * ffn_gate_up(+SwiGLU), 5 ffn_down(+residual), 6 output(+argmax), 7 layer engine (one
 * persistent launch = attn_output + ffn_gate_up + ffn_down + the next layer's qkv; when it
 * runs, classes 3-5 and all but layer 0's qkv have no launches).  0 on success. */
#define LLMI_KERNEL_CLASSES 8
/* Microbenchmark of the layer engine's weight stream (tools/lestream.py): GB/s of `iters`
 * launches in which every CU streams its share of `bytes` at device pointer src (mode 0
 * one LDS-DMA loader wave, asm; 1 the same by the compiler builtin; 2 / 3 two / four
 * loader waves; 4 eight waves of plain 16-B loads).  < 0 on error. */
double llmi_le_stream_bench(const void* src, int64_t bytes, int32_t mode, int32_t iters, int32_t nt);
/* Timeline of one layer-engine launch (leng.hip): one eager step at (first, pos0) with
 * layer `layer`'s launch writing s_memrealtime stamps (100 MHz) to out[block][wave][32]
 * (n_out >= CUs * 512: [CU][16 waves][32]); the state is left ready to decode `first` at pos0.  Returns the
 * grid size (CUs), < 0 on error.  Stamp layout: tools/letrace.py. */
int32_t llmi_engine_trace(struct llama_context* ctx, llama_token first, int32_t pos0, int32_t layer, uint64_t* out,
                          int64_t n_out);
int32_t llmi_profile_kernels(struct llama_context* ctx, llama_token first, int32_t pos0, int32_t n_steps,
                             double* us, double* bytes, int32_t* launches);
/* Test options (tests only; no environment variable reaches these): sets `name` to
 * `value` (value < 0: query) and returns the previous value, -1 for an unknown name.
 *   "pf_attn_simple"  1: batched-prefill attention one head per workgroup (bit-identical)
 *   "pf_max_kv"       longest KV length the batched prefill takes (default 32768); a prompt
 *                     reaching past it continues as decode steps (bit-identical)
 *   "xspin_limit"     polls before k_attn_x's bounded wait gives up; a give-up makes the
 *                     decode call return -6 with llmi_last_error set (fault surfacing)
 *   "xtag_skew"       1: k_attn_x consumers wait for a tag no producer writes (with
 *                     xspin_limit 0: every such wait gives up at once; fault-path test)
 *   "numerics"        this thread's numerics for the kernel-level entry points below
 *                     (llmi_repack's byte order, llmi_matvec, llmi_quantize_act,
 *                     llmi_attention, llmi_pf_attention): LLMI_NUMERICS_* */
int32_t llmi_test_option(const char* name, int32_t value);
/* Algorithmic bytes of one decode step at KV length n_kv (weights + one embedding row
 * + norms + KV read/write), the numerator of achieved GB/s. */
double llmi_bytes_per_token(const struct llama_model* model, int32_t n_kv);
/* 1 when llama_decode runs a prompt (a leading run of >= 2 tokens at consecutive
 * positions that need no logits) through the batched MFMA prefill path (one launch per
 * op over all its tokens; bit-identical to decode steps), 0 when every token of such a
 * batch is a decode step (shapes the prefill kernels do not take).  LLMI_NO_PREFILL=1
 * in the environment forces decode steps. */
int32_t llmi_prefill_supported(const struct llama_model* model);
/* Device weight arena (for RCCL broadcast by a caller that owns the communicator). */
int32_t llmi_model_arena(const struct llama_model* model, void** dev_ptr, uint64_t* bytes);
/* Replica check: an order-independent 64-bit hash of the model's device arena (sum over
 * 8-byte words i mod 2^64 of splitmix64's finalizer of word_i ^ (i * 0x9E3779B97F4A7C15),
 * the last word zero-padded).  Equal arenas give equal hashes on any device.  0 ok. */
int32_t llmi_model_arena_hash(const struct llama_model* model, uint64_t* out);
/* The same hash of `bytes` of any device memory (test hook; synchronous). */
int32_t llmi_device_hash(const void* dev_ptr, uint64_t bytes, uint64_t* out);
/* In-process replica fan-out: copies model's arena to devices[0..n) with an RCCL
 * broadcast over xGMI and returns one model handle per device (out[i]). 0 on success;
 * -1 (nothing allocated) for bad arguments, an out-of-range device, or a device listed
 * twice or equal to the source model's device. */
int32_t llmi_replicate(struct llama_model* model, const int32_t* devices, int32_t n, struct llama_model** out);

/* Multi-process replica fan-out (one process per GPU): rank 0 holds the
 * uploaded weights, ranks 1..n-1 loaded the same GGUF with params.no_upload.  Every rank
 * calls llmi_model_fanout with the same 128-byte RCCL unique id (made by rank 0 with
 * llmi_rccl_unique_id and shared by any out-of-band channel); the arena is broadcast
 * from rank 0 over xGMI as 256 MB ncclBroadcast pieces on a dedicated stream.  After
 * the pieces, rank 0's status word and arena hash go to every rank (one more broadcast):
 * a rank whose root failed, or whose arena hash differs from the root's, fails too.
 * Returns 0 on success, -6 when the root failed or the hashes differ (llmi_last_error). */
int32_t llmi_rccl_unique_id(uint8_t* out, int32_t n);
int32_t llmi_model_fanout(struct llama_model* model, const uint8_t* uid, int32_t nranks, int32_t rank);

/* Load + fan-out in one call, the broadcast pipelined behind the upload:
 * the arena goes out in 256 MB pieces, piece k as soon as the upload has completed the
 * arena prefix covering it.  llmi_model_load_fanout: every rank calls it with the same
 * RCCL unique id; rank 0 reads and uploads the GGUF, the others only plan the layout and
 * receive.  llmi_model_load_replicated: one process, the model on params.main_gpu plus a
 * replica on each of `devices` (out[i]), as llmi_replicate.  Both end with the status +
 * hash check above (a rank whose root's upload failed returns NULL with llmi_last_error
 * set, instead of a partly written arena).  NULL on error. */
struct llama_model* llmi_model_load_fanout(const char* path, struct llama_model_params params, const uint8_t* uid,
                                           int32_t nranks, int32_t rank);
struct llama_model* llmi_model_load_replicated(const char* path, struct llama_model_params params,
                                               const int32_t* devices, int32_t n, struct llama_model** out);
/* The fan-out schedule (engine.cpp fanout_plan; host only, for tests): pieces of `chunk`
 * bytes over an arena of arena_bytes; ready[k] = the index of the first upload prefix
 * (prefix_ends, ascending) that covers piece k.  Returns the number of pieces. */
int32_t llmi_fanout_plan(uint64_t arena_bytes, uint64_t chunk, const uint64_t* prefix_ends, int32_t n_prefix,
                         int32_t* ready, int32_t max_pieces);

/* A tokenizer-only vocabulary handle from a GGUF's tokenizer.* metadata (no tensors
 * or device needed); free with llmi_vocab_free (handles from llama_model_get_vocab are
 * owned by their model).  NULL on error. */
struct llama_vocab* llmi_vocab_load_from_file(const char* path);
void llmi_vocab_free(struct llama_vocab* vocab);

/* Synthetic GGUF writer: preset = "llama3-8b-q4km", "tinyllama-q8_0",
 * "mistral7b-q6k", "mistral7b-q5km", "llama3-70b-q4km", or "tiny-mixed" (2 layers, E=256,
 * all four quant types).  Overrides (0 = preset value): n_layer, n_ctx_train, n_vocab.
 * Returns bytes written or < 0. */
int64_t llmi_synth_write_gguf(const char* path, const char* preset, uint64_t seed,
                              int32_t n_layer, int32_t n_vocab, int32_t n_threads);

/* Debug taps of the last decode step (host copy, synchronous): 0 the step's embedding
 * row (get_rows of its token, n_embd), 1 residual x after the
 * last layer (n_embd), 2 roped q (n_head*head_dim), 3 attention output, 4 SwiGLU output
 * (n_ff) — the last layer's.  Mirrors the oracle's or_tap.  7/8: the last layer's raw
 * f16 K/V cache.  11-15: the last batched step's buffers, 8 slot rows each: x, q,
 * attention output, SwiGLU output, logits.  0 on success. */
int32_t llmi_debug_tap(struct llama_context* ctx, int32_t which, float* out);

/* ---------- kernel-level entry points (tests and microbenchmarks) ----------
 * All pointers are DEVICE pointers on the current HIP device; the call is enqueued
 * on the NULL stream and synchronised.  Types are ggml type ids (Q4_K=12, Q5_K=13,
 * Q6_K=14, Q8_0=8).  `w_dev` holds the weight in llmi's device layout produced by
 * llmi_repack (identity for Q4_K/Q5_K/F32).  Return 0 on success. */
int64_t llmi_device_layout_bytes(int32_t type, int64_t rows, int64_t cols);
int32_t llmi_repack(int32_t type, const void* raw_dev, void* w_dev, int64_t rows, int64_t cols);
/* y = W . quantize(norm_w ? rmsnorm(x)*norm_w : x); mode 0 store, 1 accumulate (y += .) */
int32_t llmi_matvec(int32_t type, const void* w_dev, int64_t rows, int64_t cols, const float* x_dev,
                    const float* norm_w_dev, float eps, float* y_dev, int32_t mode);
/* batched prefill GEMM (prefill.hip.inc): Y[t] = W . quantize(norm_w ? rmsnorm(x[t])*norm_w
 * : x[t]) for n_tok rows x[t] of `cols` floats (row-major), Y [n_tok][rows]; must equal
 * n_tok llmi_matvec calls bit for bit.  usec (optional): device time of the GEMM launch. */
int32_t llmi_pf_gemm(int32_t type, const void* w_dev, int64_t rows, int64_t cols, const float* x_dev,
                     const float* norm_w_dev, float eps, int32_t n_tok, float* y_dev, double* usec);
/* the activation quantization the matvec prologue performs, written out in ggml block
 * form (block_q8_K for K-quant weight types, block_q8_0 for Q8_0) for bit-exact checks */
int32_t llmi_quantize_act(int32_t type, int64_t cols, const float* x_dev, const float* norm_w_dev,
                          float eps, void* out_dev);
/* timed microbenchmark: `reps` matvecs rotating over n_mats distinct weight copies
 * (to defeat the 256 MB Infinity Cache); returns average microseconds per matvec */
double llmi_bench_matvec(int32_t type, const void* w_dev, int32_t n_mats, int64_t rows, int64_t cols,
                         const float* x_dev, float* y_dev, int32_t reps);
/* the same with epilogue/prologue variants (mode bit 0: fused RMSNorm with unit weights,
 * bit 1: logits epilogue with device argmax); launches graph-replayed */
double llmi_bench_matvec_ex(int32_t type, const void* w_dev, int32_t n_mats, int64_t rows, int64_t cols,
                            const float* x_dev, float* y_dev, int32_t reps, int32_t mode);

/* streaming-read reference: average microseconds to read `bytes` from each of n_bufs
 * distinct buffers (stride `stride` bytes) with coalesced 16-B/lane loads */
double llmi_bench_stream(const void* dev, int32_t n_bufs, uint64_t stride, uint64_t bytes, int32_t reps, int32_t blocks);
/* One decode attention (the step's launch_attention, path `mode`: 0 auto as the step
 * chooses, else LLMI_ATTN_MODE's numbering) of the query q (f32 [n_head*head_dim], roped)
 * over the first n_kv positions of one layer's f16 caches in the step's layout: K
 * [n_head_kv][n_ctx][head_dim], V transposed [n_head_kv][head_dim][n_ctx]; out f32
 * [n_head*head_dim].  n_ctx a multiple of 256.  0 on success. */
int32_t llmi_attention(int32_t n_head, int32_t n_head_kv, int32_t head_dim, int32_t n_kv, int32_t n_ctx, const float* q,
                       const uint16_t* kc, const uint16_t* vc, float* out, int32_t mode);
/* One batched-prefill attention (prefill_enqueue's launch_pf_attn) of T query tokens at
 * positions pos0..pos0+T-1 (q f32 [T][n_head*head_dim], roped; token t attends to
 * positions 0..pos0+t) over one layer's caches in the step's layout (as llmi_attention);
 * out f32 [T][n_head*head_dim].  mode 0: the tiled FP64-MFMA kernel (k_pf_fa), 1: the
 * grouped LDS kernel, 2: one head per workgroup.  scratch_bytes > 0 bounds k_pf_fa's
 * score scratch (so the launch is chunked), <= 0 takes the engine's size.  Returns
 * elapsed device microseconds (>= 0) or < 0 on error. */
double llmi_pf_attention(int32_t n_head, int32_t n_head_kv, int32_t head_dim, int32_t T, int32_t pos0, int32_t n_ctx,
                         const float* q, const uint16_t* kc, const uint16_t* vc, float* out, int32_t mode,
                         int64_t scratch_bytes);
/* Attention microbenchmark: n_kv positions, one launch per layer over >= 512 MB of
 * distinct KV caches, graph-replayed `reps` times; microseconds per launch (< 0 error).
 * mode: 0 auto, 1 fused, 2 split, 3 two-kernel.  trace_dev != NULL (LLMI_EXP_TRACE
 * builds): one eager launch on a cold layer writing per-wave s_memrealtime stamps
 * [kernel][block][wave < 16][4] (zero-initialised, 2*4096*64 uint64); returns 0. */
double llmi_bench_attention(int32_t n_head, int32_t n_head_kv, int32_t head_dim, int32_t n_kv, int32_t mode, int32_t reps,
                            uint64_t* trace_dev);
/* Experiment hook: one STORE matvec launch; builds with -DLLMI_EXP_TRACE write per-wave
 * s_memrealtime stamps {entry, after prologue, first pair done, exit, HW_ID,
 * XCC_ID<<32 | pairs, activation arrived, quantized} to trace_dev (8 x uint64 per wave,
 * zero-initialised by the caller).
 * Returns the requested grid size, < 0 on error. */
int32_t llmi_trace_matvec(int32_t type, const void* w_dev, int64_t rows, int64_t cols, const float* x_dev, float* y_dev,
                          int32_t mode, uint64_t* trace_dev);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif
#endif /* LLMI_H */
