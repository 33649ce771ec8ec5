/*
 * ggml_oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's
 * NGL=0 decode numerics, used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the CHECKER.  The product (libllmi.so) never links or calls it.
 *
 * What it restates: the hot path of SURVEY.md §8(a) rows a4-a16.  That path lives in
 * llama.cpp/ggml, an un-vendored third-party dependency that the reference consumes
 * as the floating Docker tag ghcr.io/ggml-org/llama.cpp:server (Dockerfile.cpu:11;
 * GPU variant :server-cuda, Dockerfile:11) and launches from scripts/start.sh:235,473-521.
 * No source, version pin, binary or .gguf file of it exists in this container, so the
 * functions below restate ggml's published *generic scalar* C semantics
 * (ggml-quants.c / ggml-cpu quants.c / ops.cpp / vec.cpp, recalled — SURVEY.md
 * Appendix A) and are pinned only by the known-answer tests in tests/ and the golden
 * vectors this oracle generated under tests/golden/.
 *
 *   ==> PARITY UNPINNED by the reference: no reference test, fixture
 *       or runnable binary pins a logit, token id or dequantized value for this path.
 */
#ifndef GGML_ORACLE_H
#define GGML_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_F32 = 0, OR_F16 = 1, OR_Q8_0 = 8, OR_Q4_K = 12, OR_Q5_K = 13, OR_Q6_K = 14, OR_Q8_K = 15 };

size_t or_type_size(int type);  /* bytes per block (F32/F16: per element) */
int or_block_size(int type);    /* elements per block */
int or_vec_dot_type(int wtype); /* activation type the CPU quantizes to for this weight type */

float or_fp16_to_fp32(uint16_t h);
uint16_t or_fp32_to_fp16(float f);
float or_expf(float x);
int64_t or_expf_glibc_check(float lo, float hi, int fma, int stride, float* first);

/* ggml dequantize_row_<type> (upstream ggml-quants.c) */
int or_dequantize_row(int type, const void* src, float* dst, int64_t n);
/* ggml quantize_row_q8_K_ref / quantize_row_q8_0_ref */
void or_quantize_row_q8_K(const float* x, void* y, int64_t n);
void or_quantize_row_q8_0(const float* x, void* y, int64_t n);
/* ggml_vec_dot_<wtype>_<vec_dot_type>_generic: one weight row against one quantized activation */
float or_vec_dot(int wtype, int n, const void* wrow, const void* act);
/* CPU baseline timing only: AVX2 dots in the x86 kernels' association (not the
 * generic order; never used by a parity check).  Returns 0 if this build has no AVX2. */
int or_set_fast_dots(int on);
/* Switch the dots, q8_0 quantization, f16 attention dots and exp onto upstream's x86
 * association (flags in ggml_oracle.c: 1 dots, 2 q8_0, 4 f16 dots, 8 ggml_v_expf, 16 libm
 * expf, 32 no FMA contraction).  0 = generic (default).  X86_ALL = 1|2|4|8 is the checker
 * of the GPU's x86 numerics mode (LLMI_NUMERICS_X86).  Which upstream CPU build it models:
 *   - the AVX2+FMA+F16C ("haswell") variant of ggml-cpu's x86 kernels (arch/x86/quants.c,
 *     vec.h/vec.cpp, simd-mappings.h).  A GGML_CPU_ALL_VARIANTS image picks its variant per
 *     host at run time: on an AVX-512 host the avx512/icelake/sapphirerapids variant runs,
 *     whose K-quant dots associate in 16-lane registers -- not modelled (unpinned);
 *   - llm_build_llama's non-flash attention: KQ = mul_mat(K f16, Q -> f16) per head with
 *     ggml_vec_dot_f16, soft_max_ext, KQV = mul_mat(V^T f16, softmax -> f16).  The
 *     reference's start.sh passes no --flash-attn flag, so a 2026 llama-server runs its
 *     default "-fa auto", which on CPU selects ggml_compute_forward_flash_attn_ext (online
 *     softmax, f16 V accumulation) -- a different association, not modelled (unpinned);
 *   - plain row-major weight dots: the CPU_REPACK buffer type (q4_K interleaved 8x8 GEMV,
 *     default on AVX2 builds) associates per 8 rows differently -- not modelled (unpinned). */
int or_set_x86_mode(int flags);
/* the activation conversion or_matvec applies to x for weight type wtype (current mode) */
int or_quantize_act(int wtype, const float* x, void* out, int64_t cols);
int or_get_x86_mode(void);
/* y[r] = vec_dot(W[r], quantize(x)) for r < rows (x is f32[cols]); OpenMP over rows */
int or_matvec(int wtype, const void* W, int64_t rows, int64_t cols, const float* x, float* y, int nthreads);

/* ggml_compute_forward_rms_norm (double accumulation) followed by ggml_mul by w */
void or_rms_norm_mul(const float* x, const float* w, float* y, int n, float eps);

/* ---- whole-model decode (llm_build_llama graph order, f16 KV cache) ---- */
typedef struct or_model or_model;

/* Opens a GGUF v3 file with its own reader (independent of the product's loader). */
or_model* or_model_load(const char* path, int n_ctx);
void or_model_free(or_model* m);
/* copy the decode matrices into anonymous memory, each row first-touched by the OpenMP
 * thread (of nth) that reads it in or_decode (NUMA placement for the CPU baseline);
 * returns the bytes copied, < 0 on allocation failure */
int64_t or_model_localize(or_model* m, int nth);
const char* or_last_error(void);
/* out[0..9] = n_embd, n_layer, n_head, n_head_kv, n_ff, n_vocab, n_rot, n_ctx, head_dim, file_type */
void or_model_info(const or_model* m, int64_t* out);
/* Processes one token at position pos (KV cache holds 0..pos-1); writes f32[n_vocab] logits. */
int or_decode(or_model* m, int32_t token, int32_t pos, float* logits, int nthreads);
void or_kv_clear(or_model* m);
/* Debug taps of the last or_decode: which = 0 embedding row, 1 final hidden (pre-norm) */
int or_tap(const or_model* m, int which, float* out);
/* Algorithmic bytes streamed per decoded token (weights + one embd row + KV at ctx). */
double or_bytes_per_token(const or_model* m, int ctx);

#ifdef __cplusplus
}
#endif
#endif
