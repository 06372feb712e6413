/* zonos_hip.h -- C ABI of libzonos_hip.so, the MI355X (gfx950) engine for the Zonos
 * decode hot path: generate() autoregressive DAC-token decode and the DAC decoder.
 *
 * Conventions
 *   - Plain C types only: device pointers are passed as `void*`/typed pointers obtained
 *     from the caller's allocator (torch.Tensor.data_ptr() in zonos_amd), sizes as int.
 *   - Every call is asynchronous on the `stream` argument (a hipStream_t passed as void*;
 *     NULL = default stream) and returns 0 on success, <0 on error; the message is
 *     available from zk_last_error() (thread-local). No C++ exception crosses the ABI.
 *   - bf16 tensors are raw uint16 bit patterns (torch.bfloat16 storage).
 *   - The reference interface each entry point replaces is cited as file:line relative
 *     to the coezbek/Zonos checkout (modeling_dac.py = transformers' DAC).
 */
#ifndef ZONOS_HIP_H
#define ZONOS_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ library */
int zk_version(void);                 /* ABI version (monotonic) */
const char* zk_last_error(void);      /* thread-local message of the last failing call */
int zk_device_sync(void);             /* hipDeviceSynchronize + error check */
long zk_abi_size(int which);          /* sizeof / offsetof of the ABI structs (binding self-check) */

/* ------------------------------------------------------------------ sampling
 * Mirrors sample_from_logits (zonos/sampling.py:232-328) incl.
 * modify_logit_for_repetition_penalty (131-169), apply_unified (54-75),
 * apply_top_p (96-111), apply_top_k (77-93), apply_min_p (114-128) and the
 * exponential-race multinomial (11-33). The Exp(1) noise is the engine's
 * Philox4x32-10 stream keyed by (seed, step, draw, row_base+b, codebook, token);
 * see oracle/philox.py for the exact definition. */
typedef struct zk_sampling_params {
    float temperature;        /* 0 => argmax (sampling.py:325-326) */
    float top_p;              /* 0 disables */
    float min_p;              /* 0 disables */
    float linear, conf, quad; /* unified sampler; linear<=0 disables */
    int32_t top_k;            /* 0 disables */
    int32_t rp_window;        /* repetition_penalty_window */
    float cfg_scale;          /* classifier-free guidance scale (model.py:112-114) */
    int32_t force_full_length;/* benchmark mode: cb0 EOS logit forced to -inf every step */
} zk_sampling_params;

/* Standalone sampler over fp32 logits [B][K][V] (already CFG-combined).
 * generated: int64 [B][K][gen_stride] token history (the reference passes
 *            delayed_codes[..., :offset]); the last rp_window of the first `gen_len`
 *            columns are penalised; NULL => no repetition penalty (prefill call).
 * rp:        float [B] per-row repetition penalty (model.py:342,356).
 * out:       int64 [B][K] sampled tokens. */
int zk_sample_logits(const float* logits, int B, int K, int V,
                     const int64_t* generated, int gen_stride, int gen_len, const float* rp,
                     const zk_sampling_params* sp, uint64_t seed, int step, int draw, int row_base,
                     int64_t* out, void* stream);

/* zk_sample_logits with torch's GPU noise instead of the keyed stream: the [B][K][V] race noise is
 * what `torch.empty_like(logits).exponential_(1)` returns when torch's CUDA generator holds
 * (seed, offset) (sampling.py:26-28); stride from zk_torch_noise_policy(B*K*V, ...). The caller
 * advances the generator by the policy's incr, as torch's own call would. */
int zk_sample_logits_torch(const float* logits, int B, int K, int V,
                           const int64_t* generated, int gen_stride, int gen_len, const float* rp,
                           const zk_sampling_params* sp, uint64_t seed, uint64_t offset, int stride,
                           int64_t* out, void* stream);
/* out[e] = element e of torch's GPU `Tensor.exponential_(1)` over n elements whose call took the
 * generator's Philox (seed, offset) (torch 2.10 ATen/native/hip/DistributionTemplates.h:52-91 with
 * hiprand Philox4x32-10 and TransformationHelper.h:129-146; oracle/torch_philox.py). */
int zk_torch_exponential(float* out, long n, uint64_t seed, uint64_t offset, int stride, void* stream);
/* Host-only: torch's calc_execution_policy for an n-element distribution call on a device with
 * mp_count CUs of max_threads_per_mp threads: the kernel's grid-stride (256 x grid) and the Philox
 * offset the call consumes (DistributionTemplates.h:52-63). */
int zk_torch_noise_policy(long n, int mp_count, int max_threads_per_mp, int* stride, long* incr);

/* Delay pattern (zonos/codebook_pattern.py:5-12). codes int64 [B][K][T] ->
 * delayed int64 [B][K][T+K]; revert: delayed [B][K][L] -> codes [B][K][L-K]. */
int zk_delay_apply(const int64_t* codes, int B, int K, int T, int64_t mask_token,
                   int64_t* delayed, void* stream);
int zk_delay_revert(const int64_t* delayed, int B, int K, int L, int64_t* codes, void* stream);

/* ------------------------------------------------------------------ backbone building blocks
 * (zonos/backbone/_torch.py). All activations bf16 row-major. */

/* embed_codes (model.py:97-98) + the CFG row duplication (model.py:141) + the first
 * LayerNorm of layer 0 (_torch.py:100). ids: int64 codes read at ids[b*ids_bstride +
 * k*ids_kstride + col] with col = t + (col_dev ? *col_dev + col_add : 0), t in [0,S).
 * Output row r*out_S + out_t0 + t for r in [0, rows_dup*B) uses utterance r % B.
 * x_out = embedding sum; if ln_w != NULL also xn_out = LayerNorm(x_out).
 * skip (nullable, device int32): when *skip != 0 the kernel does nothing (generation done). */
int zk_embed_codes(const int64_t* ids, int B, int S, int K, long ids_bstride, long ids_kstride,
                   const int32_t* col_dev, int col_add, const void* emb, int V, int D, int rows_dup,
                   void* x_out, int out_S, int out_t0, const void* ln_w, const void* ln_b, float eps,
                   void* xn_out, const int32_t* skip, void* stream);

/* y = LayerNorm(x) (nn.LayerNorm with bias, _torch.py:88,90,62), rows x D. */
int zk_layernorm(const void* x, const void* w, const void* b, float eps, int rows, int D,
                 void* y, void* stream);

/* x_out = bf16(x_in + bf16(sum_s part[s])) ; xn = LayerNorm(x_out) (_torch.py:100-101).
 * ln_on_sum is a flags word. Bit 0: xn = LayerNorm(x_in + bf16(sum)) of the fp32 sum before rounding
 * (mamba_ssm layer_norm_fn with prenorm, the hybrid backbone's fused add + norm). With bit 0 set, the
 * hybrid config variants (mamba_ssm Block, _mamba_ssm.py:18-31,49-57): bit 1 RMS norm
 * (is_rms_norm: y = x * rsqrt(mean(x^2) + eps) * w (+ b); b may be NULL), bit 2 x_in is fp32, bit 3
 * x_out is fp32 (residual_in_fp32), and nsplit = 0 adds no projection (part unused: the first
 * block's norm of the embedding, layer_norm_fn with residual = None).
 * part: fp32 [nsplit][rows][D] split-K slabs of the preceding projection. */
int zk_resid_ln(const float* part, int nsplit, const void* x_in, const void* w, const void* b,
                float eps, int rows, int D, void* x_out, void* xn_out, int ln_on_sum,
                const int32_t* skip, void* stream);

/* C = A[M][K] . W[N][K]^T (nn.Linear, bias-free). bf16 in, fp32 accumulation (MFMA).
 * mode 0: fp32 split-K slabs Cpart[split][M][N] (nsplit = K-split count);
 * mode 1: SwiGLU epilogue for FeedForward fc1 (_torch.py:147,151-152): W rows must be
 *         in the engine's interleaved order (zk_permute_fc1) and Cout is bf16 [M][N/2].
 * lda = row stride of A in elements (lets the heads GEMM read only the last token).
 * W is in the engine's fragment-packed layout (zk_pack_weights; rows padded to 64). */
int zk_gemm_bf16(const void* A, long lda, const void* W, int M, int N, int K, int nsplit, int mode,
                 float* Cpart, void* Cout, const int32_t* skip, void* stream);
/* Host-only (no GPU): the number of 16-column tiles of W's packed image that the L2 warm-up of
 * this decode GEMM (warm.h: issued by the kernel before it) reads; 0 when the GEMM is not warmed.
 * Never more than ceil(N / 16), the tiles of the packed image that hold a column < N. */
int zk_gemm_warm_tiles(int M, int N, int K, int nsplit, int mode, int chunks);
/* Small-batch (M <= 16) GEMV without split-K, for the B <= 8 decode layer (five launches per
 * transformer block instead of seven; replaces the k_resid_ln launches of _torch.py:100-101):
 *   ln_w/ln_b non-NULL: A holds the residual rows x (bf16, K = D = 2048) and every workgroup
 *     applies nn.LayerNorm(eps) to them in its prologue (TransformerBlock.norm / norm2 /
 *     backbone norm_f, _torch.py:78,100-101) before the product;
 *   mode 0: Cf fp32 [M][N] = LN?(A) . W^T            (in_proj, heads: one "slab", nsplit 1)
 *   mode 1: Cb bf16 [M][N/2] = SwiGLU(LN?(A) . W^T)  (fc1, interleaved rows as zk_gemm_bf16)
 *   mode 2: Cb bf16 [M][N] += bf16(A . W^T), i.e. x = bf16(x + bf16(proj))   (out_proj, fc2)
 * W fragment-packed (zk_pack_weights). K in {2048, 4096, 8192}; results depend on (N, K) only. */
int zk_gemv_fused(const void* A, long lda, const void* W, int M, int N, int K, int mode,
                  const void* ln_w, const void* ln_b, float eps, float* Cf, void* Cb,
                  const int32_t* skip, void* stream);
/* Attention out_proj of a small decode batch (M = 2B <= 2 rows) straight from the split
 * partials of zk_attn_decode_qkv_part: x[M][N] = bf16(x + bf16(merge(work) . W^T))
 * (_torch.py:66 + the residual add of :100), the merge being k_attn_combine's arithmetic
 * (bit-identical to zk_attn_decode_qkv + zk_gemv_fused mode 2 with the same nsplit).
 * K = 2048 (16 heads x 128), nsplit in {2, 4, 8, 16}. Also the consumer of zk_attn_decode_q_part. */
int zk_gemv_attn_out(const float* work, int nsplit, int Hkv, const void* W, int M, int N, int K,
                     void* x, const int32_t* skip, void* stream);
/* in_proj of the B = 1 decode layer (M = 2 rows) with the RoPE / KV-write epilogue
 * (_torch.py:61-65 + apply_rotary_emb :18-30 + _update_kv_cache :33-49): LayerNorm(x) (ln_w, ln_b,
 * the norm prologue of zk_gemv_fused) . Wqkv^T, each column rounded to bf16, q and k rotated by the
 * interleaved RoPE pairs at position p = min(*pos_dev, Smax - 1) (freqs as zk_qkv_rope), q stored to
 * q_out bf16 [M][H*hd], k and v written into the layer's cache at key p (layout of zk_qkv_rope).
 * Bit-identical to zk_gemv_fused mode 0 + the fused prologue of zk_attn_decode_qkv. d_model = H*hd =
 * 2048, hd = 128. */
int zk_gemv_qkv_rope(const void* x, const void* W, int M, int H, int Hkv, int hd, const void* ln_w,
                     const void* ln_b, float eps, void* q_out, void* k_cache, void* vt_cache, int Smax,
                     const int32_t* pos_dev, const float* freqs, const int32_t* skip, void* stream);
/* fc1 weight [2F][D] (rows: F "y" then F "gate") -> interleaved groups of 8 y + 8 gate rows. */
int zk_permute_fc1(const void* w_fc1, int F, int D, void* w_out, void* stream);
/* nn.Linear weight [N][K] bf16 -> fragment-packed [ceil64(N)/16][K/32][64][8] (rows >= N zero):
 * each 16x32 MFMA B fragment is one contiguous 1 KB block in lane order, a 16-row tile's
 * K-slices consecutive, so every wave streams its weights as one sequential run.
 * out holds ceil64(N)*K elements. K % 64 == 0. */
int zk_pack_weights(const void* w, int N, int K, void* out, void* stream);

/* Sum split-K slabs of in_proj, round to bf16, apply interleaved RoPE to q and k
 * (apply_rotary_emb _torch.py:18-30; positions pos0 + t (+ *pos_dev if non-NULL);
 * freqs = precompute_freqs_cis table [16384][hd/2][2], _torch.py:9-15), store q
 * [rows][H*hd] and write k, v into the layer cache (_update_kv_cache _torch.py:33-49).
 * Cache layout (engine-owned; hd = 128): per (row, kv head) Smax keys in 32-key slices of
 * 8 KB stored in MFMA-fragment order (backbone.hip k_off / v_off; zonos_amd.kvlayout):
 *   K: [R][Hkv][Smax/32][h 2][ks 4][lane 64][8],  V: [R][Hkv][Smax/32][dt 8][lane 64][8].
 * v_rows (nullable): also write V as [R][Hkv][S][hd] (prefill scratch).
 * rope_neox = 0: interleaved pairs (2j, 2j+1) (the transformer); 1: GPT-NeoX pairs (j, j+hd/2)
 * (mamba_ssm MHA via flash_attn RotaryEmbedding, interleaved=False; hybrid backbone). freqs is
 * then the bf16-rounded cos/sin cache (oracle/hybrid_ref.py rotary_table).
 * rows = R*S tokens ordered r*S + t. */
int zk_qkv_rope(const float* part, int nsplit, int R, int S, int H, int Hkv, int hd,
                const float* freqs, int pos0, const int32_t* pos_dev,
                void* q_out, void* k_cache, void* vt_cache, int Smax, void* v_rows,
                int rope_neox, const int32_t* skip, void* stream);

/* Scaled-dot-product attention over the cache (F.scaled_dot_product_attention,
 * _torch.py:136; GQA, scale 1/sqrt(hd)).
 * decode: one query per row, keys [0, ctx) with ctx = ctx0 + *ctx_dev; flash-decoding
 *         over 128-key blocks split across `nsplit` workgroups per (row, kv head)
 *         (nsplit <= Smax/128; work: fp32 [R][Hkv][nsplit][8 + 4*hd] when nsplit > 1).
 * prefill: S queries per row at positions 0..S-1, causal (is_causal=S>1), K and V from the cache.
 * Output bf16 [rows][H*hd]. */
int zk_attn_decode(const void* q, const void* k_cache, const void* vt_cache, int R, int H, int Hkv,
                   int hd, int Smax, int ctx0, const int32_t* ctx_dev, float* work, int nsplit,
                   void* out, const int32_t* skip, void* stream);
int zk_attn_prefill(const void* q, const void* k_cache, const void* vt_cache, int R, int S, int H,
                    int Hkv, int hd, int Smax, void* out, void* stream);
/* Decode with the in_proj epilogue fused in (= zk_qkv_rope at pos = ctx-1, S = 1, followed by
 * zk_attn_decode): reduces the in_proj slabs (gemm_nsplit x [R][(H+2Hkv)*hd] fp32), applies
 * RoPE, writes the new K / V^T cache entries and attends over keys [0, ctx). q is not stored. */
int zk_attn_decode_qkv(const float* part, int gemm_nsplit, const float* freqs, void* k_cache,
                       void* vt_cache, int R, int H, int Hkv, int hd, int Smax, int ctx0,
                       const int32_t* ctx_dev, float* work, int nsplit, void* out, int rope_neox,
                       const int32_t* skip, void* stream);

/* zk_attn_decode_qkv with the split-KV partials merged inside the launch (no k_attn_combine):
 * counters = uint32 [R][Hkv], zeroed once before the first launch (each launch adds nsplit per
 * (row, kv head); the workgroup drawing the last ticket merges). nsplit == 1 or counters == NULL
 * is zk_attn_decode_qkv. Same results as the two-launch form, bit for bit. */
int zk_attn_decode_qkv_sc(const float* part, int gemm_nsplit, const float* freqs, void* k_cache,
                          void* vt_cache, int R, int H, int Hkv, int hd, int Smax, int ctx0,
                          const int32_t* ctx_dev, float* work, int nsplit, uint32_t* counters, void* out,
                          int rope_neox, const int32_t* skip, void* stream);

/* zk_attn_decode_qkv for nsplit >= 2 key ranges WITHOUT the merge: leaves the split partials
 * (m, l, unnormalised O per query head) in work [R][Hkv][nsplit][8 + 4*128] fp32 for the
 * consumer, zk_gemv_attn_out, which merges them in its prologue (replaces the
 * F.scaled_dot_product_attention output of _torch.py:64-65 feeding out_proj, :66). */
int zk_attn_decode_qkv_part(const float* part, int gemm_nsplit, const float* freqs, void* k_cache,
                            void* vt_cache, int R, int H, int Hkv, int hd, int Smax, int ctx0,
                            const int32_t* ctx_dev, float* work, int nsplit, int rope_neox,
                            const int32_t* skip, void* stream);

/* Decode attention of the B = 1 step when q and the new key / value come from zk_gemv_qkv_rope:
 * F.scaled_dot_product_attention of one query per row over keys [0, ctx), ctx = min(ctx0 + *ctx_dev,
 * Smax) (_torch.py:64-65), with the keys split in 32-key slices over nsplit workgroups per (row, kv
 * head) (workgroup s, wave w: slices 4s + w + 4 nsplit j). Leaves the partials (m, l, unnormalised O)
 * in work [R][Hkv][nsplit][8 + 4*128] fp32 for zk_gemv_attn_out. nsplit <= 64. */
int zk_attn_decode_q_part(const void* q, const void* k_cache, const void* vt_cache, int R, int H, int Hkv,
                          int hd, int Smax, int ctx0, const int32_t* ctx_dev, float* work, int nsplit,
                          const int32_t* skip, void* stream);

/* ------------------------------------------------------------------ graphs and timing
 * The decode step is captured once into a hipGraph and replayed (the reference runs the
 * transformer step eagerly: model.py:138-142, 220-222). */
int zk_graph_begin(void* stream);
int zk_graph_end(void* stream, void** graph_exec);
int zk_graph_launch(void* graph_exec, int repeat, void* stream);
int zk_graph_destroy(void* graph_exec);
int zk_event_create(void** ev);
int zk_event_record(void* ev, void* stream);
int zk_event_elapsed_ms(void* start, void* end, float* ms);
int zk_event_destroy(void* ev);

/* ------------------------------------------------------------------ generation state machine
 * One step of the generate() loop body after the backbone (model.py:353-424). */
typedef struct zk_gen_state {
    int32_t* scal;        /* device int32[16]: 0 offset, 1 pos, 2 step, 3 done, 4 any_new_eos,
                             5 max_steps, 6 error flags */
    int32_t* eos_mode;    /* [B] */
    int32_t* steps_after; /* [B] */
    int32_t* remaining;   /* [B] */
    int32_t* stopping;    /* [B] */
    int32_t* act;         /* [B] eos_active for the current step */
    float* rp;            /* [B] repetition penalty in effect */
    int32_t* tok0;        /* [B*K] draw-0 tokens */
    int32_t* tok1;        /* [B*K] draw-1 (EOS resample) tokens */
    int64_t* delayed;     /* [B][K][Ld] delayed codes (model.py:295) */
    int32_t B, K, Ld, V;
    uint64_t seed;
    int32_t row_base;     /* global index of utterance 0 (batch sharding) */
    /* Noise mode. 0: the engine's keyed stream (seed, step, draw, row_base + b, codebook, token).
     * 1: torch's own GPU stream -- the values `torch.empty_like(probs).exponential_(1)` gives the
     * reference's sampler (sampling.py:26-28) when torch's CUDA generator holds (seed, noise_offset):
     * sampler call c (0 = the prefill sample, model.py:304; then one per decode step, model.py:365,
     * and one per EOS resample, model.py:388) reads the stream at Philox offset noise_offset +
     * c * noise_incr over the [B][K][V] tensor with grid-stride noise_stride (zk_torch_noise_policy). */
    int32_t noise_mode;
    uint64_t noise_offset;
    int32_t noise_stride;
    int32_t noise_incr;
} zk_gen_state;

/* Engine sampler: logits from the heads GEMM split-K slabs part [nsplit][2B][K*V] (rows
 * [0,B) cond, [B,2B) uncond), bf16-rounded per head (model.py:111), CFG-combined
 * (model.py:112-115), biased (model.py:322-324,353,360-362) and sampled. prefill=1 is the
 * first sample (model.py:304: no bias, no penalty). draw 1 = EOS resample (model.py:386-393):
 * a no-op unless some row has a new EOS. dbg_logits (nullable) receives the fp32 CFG logits
 * before bias [B][K][V]. */
int zk_sample_heads(const float* part, int nsplit, const zk_gen_state* st, const zk_sampling_params* sp,
                    int prefill, int draw, float* dbg_logits, void* stream);
/* EOS protocol + frame write + counters (model.py:376-424); prefill=1 only writes the
 * first frame (model.py:310-319). */
int zk_eos_step(const zk_gen_state* st, int prefill, int prefix_len, void* stream);

/* ------------------------------------------------------------------ one decode step
 * The whole autoregressive step of Zonos.generate (model.py:322-424: _decode_one_token's
 * embed -> 26 blocks -> norm_f -> 9 heads -> CFG, then the sampler, the EOS protocol and the
 * delayed-frame write) enqueued on `stream` with no host synchronisation, exactly the launch
 * sequence of zonos_amd.engine.HipDecoder._decode_step (the Python engine calls this entry):
 * small = 1 (B <= 8): five launches per block (zk_gemv_fused LayerNorm prologues / residual
 * epilogues; attn_merge > 0: zk_gemv_qkv_rope + zk_attn_decode_q_part + zk_gemv_attn_out, or with
 * rope_neox zk_gemv_fused + zk_attn_decode_qkv_part + zk_gemv_attn_out); small = 0: seven
 * (split-K zk_gemm_bf16 + zk_attn_decode_qkv_sc + zk_resid_ln). Every position/offset is read
 * from st.scal on the device, so one call is captured once into a hipGraph and replayed.
 * Replaces the per-token Python loop body of model.py:322-424 for a C/C++ host. */
typedef struct zk_step_layer {
    const void* ln1_w;    /* norm.weight / bias (bf16 [D]) */
    const void* ln1_b;
    const void* wqkv;     /* mixer.in_proj, packed (zk_pack_weights) */
    const void* wo;       /* mixer.out_proj, packed */
    const void* ln2_w;    /* norm2 */
    const void* ln2_b;
    const void* fc1;      /* mlp.fc1 in zk_permute_fc1 order, packed */
    const void* fc2;      /* mlp.fc2, packed */
    void* k_cache;        /* this layer's K / V^T cache (fragment order, Smax keys per (row, kv head)) */
    void* vt_cache;
} zk_step_layer;

typedef struct zk_step_desc {
    int32_t B, n_layer, d_model, n_heads, n_kv, head_dim, d_ff, smax;
    int32_t split_qkv, split_o, split_fc2, split_heads;   /* split-K counts (small = 0) */
    int32_t attn_splits, attn_merge, rope_neox, small;
    float eps;
    const zk_step_layer* layers;   /* [n_layer] */
    const void* emb;               /* codebook embeddings bf16 [9][1026][D] */
    const void* heads;             /* 9 heads stacked, packed */
    const void* lnf_w;             /* norm_f */
    const void* lnf_b;
    const float* freqs;            /* RoPE table (engine.rope_table) */
    void* x;                       /* residual rows bf16 [2B][D] */
    void* xn;                      /* LayerNorm'd rows bf16 [2B][D] */
    void* y;                       /* attention output bf16 [2B][H*hd] */
    void* h;                       /* SwiGLU output bf16 [2B][d_ff] */
    float* part;                   /* split-K slabs / logits */
    float* attn_work;              /* split-KV partials */
    uint32_t* attn_cnt;            /* in-launch combine tickets [2B][Hkv] */
    float* dbg;                    /* nullable: fp32 CFG logits of draw 0 */
    zk_gen_state st;
    zk_sampling_params sp;
} zk_step_desc;

int zk_decode_step(const zk_step_desc* d, void* stream);

/* The prefill of Zonos.generate (model.py:297-319, _prefill 181-202) on the same descriptor:
 * x rows [2B][S][D] = [prefix conditioning (cond, bf16 [2B][Lc][D]) | codebook embeddings of the
 * P audio-prefix frames + the first delayed frame], layer 0's LayerNorm, the 26 blocks over all
 * 2B*S positions (split-K 1, causal prefill attention filling the KV cache), the heads on the
 * last position, the first sample (model.py:304: no bias, no penalty) and the first frame write.
 * S = Lc + P + 1; q: bf16 [2B*S][H*hd] scratch; x / xn / y / h / part sized for 2B*S rows.
 * The loop state (st.scal, eos_mode, ...) is initialised by the host afterwards (model.py:316-342).
 * Fails (-1, before any launch) unless smax >= Lc + st.Ld, the context of the last decode step. */
int zk_prefill(const zk_step_desc* d, const void* cond, int Lc, int P, void* q, void* stream);

/* ------------------------------------------------------------------ hybrid decode step
 * The same two entries for the Zonos-v0.1-hybrid backbone (zonos/backbone/_mamba_ssm.py:9-57 ->
 * mamba_ssm create_block: Mamba2 mixers, MHA + GatedMLP at attn_layer_idx, fused add + LayerNorm
 * of the fp32 sum), the launch sequence of zonos_amd.hybrid.HybridDecoder:
 *   Mamba2 layer : in_proj GEMM -> zk_mamba_step (conv + SSM state update, y * silu(z)) ->
 *                  zk_gated_rmsnorm -> out_proj GEMM -> zk_resid_ln(ln_on_sum = 1, next norm)
 *   attention    : Wqkv GEMM -> zk_attn_decode_qkv (GPT-NeoX RoPE) -> out_proj -> zk_resid_ln(norm2)
 *                  -> fc1 (SwiGLU) -> fc2 -> zk_resid_ln(next norm)
 * (a Mamba2 block with d_mlp > 0 continues like the attention block from zk_resid_ln(norm2); with
 * norm_flags != 0 the first block's norm is its own zk_resid_ln(nsplit = 0) after the embedding)
 * then norm_f, the 9 heads, the sampler and the EOS protocol exactly as zk_decode_step. Conv and
 * SSM states are double-buffered by step parity ({a, b}, zk_mamba_step). Replaces the
 * `_decode_one_token` / `_prefill` bodies of model.py:118-202 for the mamba_ssm backbone (the one
 * the reference CUDA-graph-captures, model.py:220-222). */
typedef struct zk_hybrid_layer {
    int32_t type;           /* 0 attention block, 1 Mamba2 block */
    int32_t d_mlp;          /* Mamba2 block: GatedMLP width (d_intermediate; 0 = no norm2 / MLP, the
                               Zonos-v0.1-hybrid case); attention block: 0 = d_ff of the descriptor */
    const void* ln1_w;      /* norm.weight / bias (bf16 [D]; ln1_b NULL under rms_norm) */
    const void* ln1_b;
    /* attention block (norm2 / mlp also of a Mamba2 block with d_mlp > 0) */
    const void* wqkv;       /* mixer.in_proj, packed */
    const void* wo;         /* mixer.out_proj, packed */
    const void* ln2_w;      /* norm2 (ln2_b NULL under rms_norm: bias-free RMSNorm) */
    const void* ln2_b;
    const void* fc1;        /* mlp.fc1 (zk_permute_fc1 order), packed */
    const void* fc2;        /* mlp.fc2, packed */
    void* k_cache;          /* fragment-order K / V^T caches */
    void* vt_cache;
    /* Mamba2 block */
    const void* w_in;       /* mixer.in_proj, packed [2 d_inner + 2 d_state + nheads][D] */
    const float* conv_w;    /* conv1d weight fp32 [conv_dim][4] */
    const float* conv_b;    /* conv1d bias fp32 [conv_dim] */
    const float* A;         /* -exp(A_log) fp32 [nheads] */
    const float* dt_bias;   /* fp32 [nheads] */
    const float* Dskip;     /* D fp32 [nheads] */
    const float* norm_w;    /* RMSNormGated weight fp32 [d_inner] */
    const void* w_out;      /* mixer.out_proj, packed [D][d_inner] */
    void* conv_state[2];    /* bf16 [R][conv_dim][4], parity buffers */
    void* ssm_state[2];     /* bf16 [R][nheads][headdim][d_state], parity buffers */
} zk_hybrid_layer;

typedef struct zk_hybrid_desc {
    int32_t B, n_layer, d_model, n_heads, n_kv, head_dim, d_ff, smax;
    int32_t d_inner, nheads_ssm, headdim_ssm, d_state;
    int32_t split_qkv, split_o, split_fc2, split_heads, split_inp, split_out, attn_splits;
    int32_t norm_flags;            /* BackboneConfig variants: bit 1 rms_norm (block norms are bias-free
                                      RMSNorms, norm_f an RMS norm with its bias), bit 2 residual_in_fp32
                                      (residual stream in xf, fp32); 0 = Zonos-v0.1-hybrid */
    float eps;                     /* LayerNorm eps (norm_epsilon) */
    float gate_eps;                /* RMSNormGated eps (1e-5 in mamba_ssm Mamba2) */
    const zk_hybrid_layer* layers; /* [n_layer] */
    const void* emb;               /* codebook embeddings bf16 [9][1026][D] */
    const void* heads;             /* 9 heads stacked, packed */
    const void* lnf_w;             /* norm_f */
    const void* lnf_b;
    const float* freqs;            /* bf16-rounded cos/sin cache [pos][hd/2][2] (rope_neox) */
    void* x;                       /* residual rows bf16 [rows][D] */
    void* xn;                      /* LayerNorm'd rows bf16 */
    void* y;                       /* attention output bf16 [rows][H*hd] */
    void* h;                       /* SwiGLU output bf16 [rows][d_ff] */
    float* part;                   /* split-K slabs / logits */
    float* attn_work;              /* split-KV partials */
    float* yz;                     /* Mamba y * silu(z) fp32 [rows][d_inner] */
    void* ym;                      /* RMSNormGated output bf16 [rows][d_inner] */
    void* xc;                      /* prefill conv scratch bf16 [rows][conv_dim] */
    float* dbg;                    /* nullable: fp32 CFG logits of draw 0 */
    zk_gen_state st;
    zk_sampling_params sp;
    void* xf;                      /* residual rows fp32 [rows][D] (norm_flags bit 2; else unused) */
} zk_hybrid_desc;

int zk_hybrid_decode_step(const zk_hybrid_desc* d, void* stream);
int zk_hybrid_prefill(const zk_hybrid_desc* d, const void* cond, int Lc, int P, void* q, void* stream);

/* ------------------------------------------------------------------ DAC decoder
 * (zonos/autoencoder.py:44-47 -> modeling_dac.py:610-640). fp32 activations, layout
 * [B][C][T] (channels-first, like torch). Per-row valid lengths (in frames) make a
 * padded batch decode identical to per-utterance decode (autoencoder.py:219-226). */

/* E_k[c][ch] = out_proj_k(codebook_k[c]) + bias_k  (modeling_dac.py:364-370), k < ncb. */
int zk_dac_rvq_tables(const float* codebooks, const float* out_w, const float* out_b, int ncb,
                      int ncode, int cdim, int hidden, float* tables, void* stream);
/* z[b][ch][t] = sum_k E_k[codes[b][k][t]][ch] (sequential fp32, k ascending). */
int zk_dac_rvq_decode(const int64_t* codes, int B, int ncb, int T, long code_bstride,
                      const float* tables, int ncode, int hidden, float* z, int Tz,
                      const int32_t* lens, void* stream);
/* Generic conv over time with fused Snake input activation and epilogue:
 *   out[b][co][t_out(q)] = bias[co] + sum_{ci,k} W[co][ci][k] * act(in[b][ci][q + k*dil - pad])
 *                          (+ resid[b][co][t_out]) (tanh if do_tanh)
 * t_out(q) = q*out_stride + out_off. act = Snake(alpha) if alpha != NULL (modeling_dac.py:95-100).
 * in positions outside [0, len_in_b) read as 0; len_in_b = lens[b]*in_scale (lens NULL => Tin).
 * Outputs outside [0, len_out_b) are written as 0. */
int zk_dac_conv(const float* in, int B, int Cin, int Tin, const float* alpha,
                const float* w, const float* bias, int Cout, int ks, int dil, int pad,
                int Qn, int out_stride, int out_off, float* out, int Tout, const float* resid,
                int do_tanh, const int32_t* lens, int in_scale, int out_scale, void* stream);
/* ConvTranspose1d weight [Cin][Cout][2s] -> s polyphase 2-tap conv weights
 * [s][Cout][Cin][2] so that zk_dac_conv(ks=2, pad=1, out_stride=s, out_off=r-ceil(s/2)). */
int zk_dac_prep_convt(const float* w, int Cin, int Cout, int s, float* w_out, void* stream);

/* fp16-MFMA variant of zk_dac_conv (same semantics). npass = 3: split precision
 * (hi/lo fp16 operands, hi*hi + lo*hi + hi*lo, ~fp32 accuracy); npass = 1: plain fp16
 * operands (the reference's own GPU numerics: autocast fp16, autoencoder.py:46).
 * Weights prepacked by zk_dac_prep_w16: mode 0 conv [Cout][Cin][ks] -> [ks][Cout][Cin];
 * mode 1 ConvTranspose1d [Cin][Cout][2s] -> [s][2][Cout][Cin] (phase r at offset 2*r*Cout*Cin,
 * run with ks=2, dil=1, pad=1, out_stride=s, out_off=r-ceil(s/2)). Cin % 32 == 0. w_lo may be
 * NULL (plain fp16 packing). */
int zk_dac_prep_w16(const float* w, int Cout, int Cin, int ks, int s, int mode, uint16_t* w_hi,
                    uint16_t* w_lo, void* stream);
int zk_dac_conv16(const float* in, int B, int Cin, int Tin, const float* alpha, const uint16_t* w_hi,
                  const uint16_t* w_lo, const float* bias, int Cout, int ks, int dil, int pad,
                  int Qn, int out_stride, int out_off, float* out, int Tout, const float* resid,
                  int do_tanh, const int32_t* lens, int in_scale, int out_scale, int npass, void* stream);
/* Final Snake -> Conv1d(C -> 1, k7, pad 3) -> tanh (modeling_dac.py:437-439); out [B][T]. */
int zk_dac_tail(const float* in, int B, int C, int T, const float* alpha, const float* w,
                const float* bias, float* out, const int32_t* lens, int scale, void* stream);

/* ---- channels-last fp16 pipeline (default "fp16" precision; dac_cl.hip). Activations are
 * s = fp16(Snake(x)) [B][T][C] with C padded to a multiple of 32 (zero channels), the
 * residual stream x fp32 [B][T][C]. Each conv applies the NEXT Snake in its epilogue. */
/* z[b][t][ch] = fp16(sum_k E_k[codes[b][k][t]][ch]) (k ascending), channels [hidden, cpad) = 0. */
int zk_dac_rvq_decode_cl(const int64_t* codes, int B, int ncb, int T, long code_bstride,
                         const float* tables, int ncode, int hidden, int cpad, uint16_t* z,
                         const int32_t* lens, void* stream);
/* For q < Qn, phase r < nphase, t = q*out_stride + out_off0 + r in [0, Tout):
 *   v = bias[co] + sum_{ci,k} W_r[k][co][ci] * in[b][q + k*dil - pad][ci]  (+ resid[b][t][co])
 *   x_out[b][t][co] = v (if x_out);  s_out[b][t][co] = fp16(Snake_{alpha_next}(v))
 *   (s_f32 = 1: s_out is fp32 and the Snake uses the exact sinf -- the input of zk_dac_tail_cl)
 * W_r = w + r*w_phase_stride (zk_dac_prep_w16 hi layout). Inputs outside [0, lens[b]*in_scale)
 * read 0; outputs at t >= lens[b]*out_scale are written 0. Cin, Cout % 32 == 0; ks <= 7,
 * (ks-1)*dil <= 64. Conv1d: nphase=1, out_stride=1, out_off0=0. ConvTranspose1d(stride s):
 * ks=2, dil=1, pad=1, Qn=Tin+1, nphase=s, out_stride=s, out_off0=-ceil(s/2). */
int zk_dac_conv_cl(const uint16_t* in, int B, int Cin, int Tin, const uint16_t* w, long w_phase_stride,
                   const float* bias, int Cout, int ks, int dil, int pad, int Qn, int nphase,
                   int out_stride, int out_off0, int Tout, const float* resid, float* x_out,
                   const float* alpha_next, void* s_out, int s_f32, const int32_t* lens, int in_scale,
                   int out_scale, void* stream);
/* One whole DAC residual unit (modeling_dac.py:222-233, ResidualUnit.forward) in one launch:
 *   y  = b7 + conv7_dil(s_in)                      (s_in = fp16 Snake_a1(x), [B][T][C])
 *   s2 = fp16(Snake_a2(y));  v = x + b1 + W1 s2     (1x1 conv; the fp16 s2 never leaves the chip)
 *   x[b][t][c] = v;  s_out[b][t][c] = fp16(Snake_{alpha_next}(v))  (s_f32 = 1: fp32, exact sinf)
 * Replaces the pair zk_dac_conv_cl(k7 -> s2) + zk_dac_conv_cl(1x1, resid = x); the same masking
 * (inputs at t >= lens[b]*scale read 0, outputs there written 0). w7 fp16 [7][C][C], w1 fp16
 * [C][C] (zk_dac_prep_w16 layouts). s_out must not alias s_in. Built for C = 96, 192; the 1x1 sums
 * run on 16x16x16 MFMAs (a different fp32 summation grouping than the 32-deep unfused conv:
 * results equal to rounding, not bit for bit). zk_dac_resunit_supported(C): 0 = not fused at this
 * C, 1 = fused except the decode's last unit (the fp32-Snake one), 2 = every unit; zk_dac_decode
 * and the Python-issued sequence both follow it. */
int zk_dac_resunit_supported(int C);
int zk_dac_resunit_cl(const uint16_t* s_in, int B, int C, int T, const uint16_t* w7, const float* b7, int dil,
                      const float* a2, const uint16_t* w1, const float* b1, float* x, const float* alpha_next,
                      void* s_out, int s_f32, const int32_t* lens, int scale, void* stream);
/* out[b][t] = tanh(bias + sum_{c,k} w[c*7+k] * s[b][t+k-3][c]), 0 at t >= lens[b]*scale
 * (s = fp32 output of the final Snake, zk_dac_conv_cl with s_f32 = 1; modeling_dac.py:437-439). */
int zk_dac_tail_cl(const float* s, int B, int C, int T, const float* w, const float* bias,
                   float* out, const int32_t* lens, int scale, void* stream);

/* The whole channels-last DAC decode (DACAutoencoder.decode, autoencoder.py:44-47 ->
 * DacModel.decode, modeling_dac.py:610-640) as one call: RVQ lookup -> conv1 -> per block
 * ConvTranspose1d + 3 residual units (k7 dilated + 1x1 with the residual add) -> Snake -> conv2
 * -> tanh, the launch sequence of zonos_amd.autoencoder.HipDacDecoder._decode_cl. Weights in the
 * zk_dac_conv_cl layouts (channels padded to 32; zk_dac_prep_w16). codes int64 [B][ncb][T];
 * lens int32 [B] frames (nullable = all T); out fp32 [B][1][T * prod(strides)]; workspace of
 * zk_dac_decode_workspace(d, B, T) bytes (device memory). */
#define ZK_DAC_MAXB 6
#define ZK_DAC_MAXR 3
typedef struct zk_dac_resunit {
    int32_t dil;
    const float* a1;       /* Snake alpha before the k7 conv */
    const uint16_t* w1;    /* k7 conv, fp16 [7][C][C] */
    const float* b1;
    const float* a2;       /* Snake alpha before the 1x1 conv */
    const uint16_t* w2;    /* 1x1 conv, fp16 [1][C][C] */
    const float* b2;
} zk_dac_resunit;
typedef struct zk_dac_block {
    int32_t stride, cin, cout, nres;
    const float* alpha;    /* Snake alpha before the ConvTranspose1d */
    const uint16_t* wt;    /* ConvTranspose1d, fp16 [stride][2][cout][cin] */
    const float* bt;
    zk_dac_resunit res[ZK_DAC_MAXR];
} zk_dac_block;
typedef struct zk_dac_desc {
    int32_t nblocks, ncb, codebook_size, hidden, cin0, c0;
    const float* tables;   /* RVQ codebooks projected to the latent (zk_dac_rvq_decode_cl) */
    const uint16_t* conv1_w;
    const float* conv1_b;
    const float* final_alpha;
    const float* conv2_w;  /* [C][7] fp32 */
    const float* conv2_b;
    zk_dac_block blocks[ZK_DAC_MAXB];
} zk_dac_desc;
size_t zk_dac_decode_workspace(const zk_dac_desc* d, int B, int T);
int zk_dac_decode(const zk_dac_desc* d, const int64_t* codes, int B, int T, const int32_t* lens, void* workspace,
                  size_t workspace_bytes, float* out, void* stream);

/* ---- DAC encoder (prefix audio -> codes; DACAutoencoder.encode, autoencoder.py:27-28 ->
 * DacModel.encode). Convolutions run on zk_dac_conv_cl (channels-last fp16 operands); a strided
 * Conv1d(k = 2s, stride s, pad ceil(s/2)) runs as a stride-1 3-tap conv over the input folded to
 * [T/s][s*C] (weights repacked on the host). zk_dac_conv_cl accepts s_out = NULL (x_out only). */
/* conv1 (1 -> C, k7, pad 3) of wav fp32 [B][T]: x_out fp32 [B][T][Cp], s_out = fp16(Snake(x)). */
int zk_dac_enc_conv1(const float* wav, int B, int T, const float* w, const float* bias,
                     const float* alpha_next, int C, int Cp, float* x_out, uint16_t* s_out, void* stream);
/* Residual VQ encode of z fp32 [B][T][hidden] -> codes int64 [B][ncb][T]: per codebook
 * e = normalize(in_w z + in_b); code = argmax_n -(|e|^2 - 2 e.cn_n) + |cn_n|^2 (first on ties,
 * cn = normalised codebook); z -= out_w cb[code] + out_b (modeling_dac DacVectorQuantize). */
int zk_dac_rvq_encode(const float* z, int B, int T, int hidden, int ncb, int ncode, int cdim,
                      const float* in_w, const float* in_b, const float* cb_norm, const float* cb_norm_sq,
                      const float* cb, const float* out_w, const float* out_b, int64_t* codes, void* stream);

/* Resampler of DACAutoencoder.preprocess (autoencoder.py:21-25 -> torchaudio.functional.resample,
 * sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99): x fp32 [B][T] -> out fp32 [B][Tout],
 * out[n] = sum_k kern[n % up][k] * x[(n / up) * down + k - width] (zero outside [0, T)), where
 * up/down = new/orig rate over their gcd and kern [up][K = 2 width + down] the windowed-sinc table. */
int zk_resample(const float* x, int B, long T, const float* kern, int up, int down, int width, int K,
                float* out, long Tout, void* stream);

/* ---- PrefixConditioner.forward (zonos/conditioning.py:373-389; Zonos.prepare_conditioning,
 * model.py:210-218): conditioner rows -> concat over the sequence -> prefix projection ->
 * LayerNorm, one launch, out bf16 [B][L][D]. A plan lists the segments in the conditioners'
 * order; a segment's input batch `bin` is 1 (broadcast, the reference's expand) or B. */
#define ZK_COND_MAXSEG 16
#define ZK_COND_MAXIN 64
enum { ZK_SEG_VECTOR = 0,   /* learned uncond vector: table bf16 [D], len 1 */
       ZK_SEG_EMBED = 1,    /* embedding: input int64 ids [bin][in_bstride], row = table[id - id_min] */
       ZK_SEG_FOURIER = 2,  /* Fourier: input fp32 [bin][len][in_dim], table = W bf16 [cin/2][in_dim] */
       ZK_SEG_PASS = 3 };   /* passthrough: input bf16 [bin][len][cin] */
typedef struct {
    int type, len, cin, in_dim, bin, proj;   /* proj: 0 none, 1 linear, 2 mlp (conditioning.py:27-34) */
    long in_bstride, id_min;
    float vmin, vden;                        /* Fourier: (x - vmin) / vden */
    const void* table;
    const void* input;
    const void* pw0; const void* pb0; const void* pw1; const void* pb1;   /* bf16 projection [D][cin], [D][D] */
} ZkCondSeg;
typedef struct {
    int nseg, D, L, proj;
    float eps;
    const void* pw0; const void* pb0; const void* pw1; const void* pb1;   /* prefix projection */
    const void* norm_w; const void* norm_b;                                /* LayerNorm (NULL: none) */
    ZkCondSeg seg[ZK_COND_MAXSEG];
} ZkCondPlan;
int zk_prefix_cond(const ZkCondPlan* plan, int B, void* out, void* stream);

/* ------------------------------------------------------------------ hybrid backbone: Mamba2 mixer
 * (zonos/backbone/_mamba_ssm.py -> mamba_ssm Mamba2; restated in oracle/hybrid_ref.py).
 * in_proj output columns [z (d_inner) | xBC (conv_dim = d_inner + 2 d_state) | dt (nheads)].
 * Conv state bf16 [R][conv_dim][4] (last 4 inputs), double-buffered by step parity: the step at
 * position *pos_dev reads buffer (pos & 1) of {a, b} and writes the other. SSM state bf16
 * [R][nheads][headdim][d_state]: updated in place when ssm_state_b is NULL, otherwise
 * double-buffered like the conv state ({ssm_state, ssm_state_b}: read (pos & 1), write the other;
 * the in-place read-modify-write of the same lines streams ~5 % slower). A = -exp(A_log), dt_bias, D fp32 [nheads]; conv_w fp32
 * [conv_dim][4], conv_b fp32 [conv_dim]. yz (fp32 [rows][d_inner]) = bf16(C.h + D x) * silu(z),
 * normalised by zk_gated_rmsnorm (RMSNormGated, norm_before_gate=False) into the out_proj input.
 * (headdim, d_state) in {(64,128), (64,64), (32,64)}. */
int zk_mamba_step(const float* part, int gemm_nsplit, int R, int d_inner, int nheads, int headdim,
                  int d_state, const float* conv_w, const float* conv_b, void* conv_state_a,
                  void* conv_state_b, const int32_t* pos_dev, void* ssm_state, void* ssm_state_b,
                  const float* A, const float* dt_bias, const float* D, float* yz, const int32_t* skip,
                  void* stream);
/* zk_mamba_step computed by the per-(head, row) kernel instead of the grouped one: same arguments,
 * same results (bit for bit, or within 1 bf16 ulp of y where the C.h row sum is reduced in another
 * order). The verification twin of zk_mamba_step; not on the decode path. */
int zk_mamba_step_per_head(const float* part, int gemm_nsplit, int R, int d_inner, int nheads, int headdim,
                           int d_state, const float* conv_w, const float* conv_b, void* conv_state_a,
                           void* conv_state_b, const int32_t* pos_dev, void* ssm_state, void* ssm_state_b,
                           const float* A, const float* dt_bias, const float* D, float* yz, const int32_t* skip,
                           void* stream);
/* prefill over S positions per row: zx = in_proj output fp32 [R*S][cols] (split 1); xc_scratch
 * bf16 [R*S][conv_dim]; conv_state receives the last 4 inputs (the buffer the first decode step
 * reads); ssm_state receives the final state (bf16; with double-buffered decode states, the
 * buffer the first decode step reads). */
int zk_mamba_prefill(const float* zx, int R, int S, int d_inner, int nheads, int headdim, int d_state,
                     const float* conv_w, const float* conv_b, void* xc_scratch, void* conv_state,
                     void* ssm_state, const float* A, const float* dt_bias, const float* D, float* yz,
                     void* stream);
int zk_gated_rmsnorm(const float* g, int rows, int d_inner, const float* w, float eps, void* out,
                     const int32_t* skip, void* stream);

/* ------------------------------------------------------------------ codes_to_wavs post-processing
 * Loudness of each decoded utterance as normalize_loudness measures it (autoencoder.py:172-186
 * -> pyloudnorm 0.1.1 Meter(rate, block).integrated_loudness, BS.1770-4 K-weighting + gating;
 * block 0.4 s if the utterance is longer than 2 s else 0.1 s). wav fp32 [B][T] (row b valid for
 * lens[b] samples, NULL = T). gains[b] = 10^((target - L_b)/20), loudness[b] = L_b; utterances
 * shorter than one block get gain 1 and loudness NaN (the reference's except path).
 * scratch: fp64, B*T + B*zk_loudness_max_blocks(T, rate) elements. */
int zk_loudness_max_blocks(long T, int rate);
int zk_loudness_gains(const float* wav, int B, long T, const int32_t* lens, int rate, double target_lufs,
                      double* scratch, double* gains, double* loudness, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ZONOS_HIP_H */
