// C ABI glue for libzonos_hip.so: error reporting, device sync and hipGraph capture of the
// decode step (the reference runs the transformer step eagerly, model.py:138-142,220-222).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stddef.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "../../include/zonos_hip.h"
#include "warm.h"

static thread_local char g_err[1024] = "";

extern "C" void zk_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

extern "C" const char* zk_last_error(void) { return g_err; }

extern "C" int zk_version(void) { return 1; }

// sizeof / offsetof of the by-value ABI structs, so a binding (ctypes here) can verify its
// layout without a GPU: which = 0 zk_sampling_params, 1 zk_gen_state, 4 ZkCondSeg, 5 ZkCondPlan,
// 6 zk_step_layer, 7 zk_step_desc, 8 zk_dac_desc; 12-21 sizes / field offsets (see the cases).
extern "C" long zk_abi_size(int which) {
    switch (which) {
        case 0: return (long)sizeof(zk_sampling_params);
        case 1: return (long)sizeof(zk_gen_state);
        case 4: return (long)sizeof(ZkCondSeg);
        case 5: return (long)sizeof(ZkCondPlan);
        case 12: return (long)offsetof(zk_gen_state, seed);
        case 6: return (long)sizeof(zk_step_layer);
        case 7: return (long)sizeof(zk_step_desc);
        case 13: return (long)offsetof(zk_step_desc, eps);
        case 14: return (long)offsetof(zk_step_desc, st);
        case 15: return (long)offsetof(zk_step_desc, sp);
        case 8: return (long)sizeof(zk_dac_desc);
        case 16: return (long)offsetof(zk_dac_desc, blocks);
        case 17: return (long)sizeof(zk_dac_block);
        case 18: return (long)sizeof(zk_hybrid_layer);
        case 19: return (long)sizeof(zk_hybrid_desc);
        case 20: return (long)offsetof(zk_hybrid_desc, st);
        case 21: return (long)offsetof(zk_hybrid_desc, eps);
        case 22: return (long)offsetof(zk_gen_state, noise_offset);
        default: return -1;
    }
}

extern "C" int zk_device_sync(void) {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        zk_set_error("hipDeviceSynchronize: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

#define HIPCHK(expr, what)                                                 \
    do {                                                                   \
        hipError_t _e = (expr);                                            \
        if (_e != hipSuccess) {                                            \
            zk_set_error("%s: %s", what, hipGetErrorString(_e));           \
            return -1;                                                     \
        }                                                                  \
    } while (0)

extern "C" int zk_graph_begin(void* stream) {
    HIPCHK(hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeThreadLocal), "zk_graph_begin");
    return 0;
}

extern "C" int zk_graph_end(void* stream, void** graph_exec) {
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamEndCapture((hipStream_t)stream, &g), "zk_graph_end(capture)");
    hipGraphExec_t ex = nullptr;
    hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIPCHK(e, "zk_graph_end(instantiate)");
    *graph_exec = (void*)ex;
    return 0;
}

extern "C" int zk_graph_launch(void* graph_exec, int repeat, void* stream) {
    for (int i = 0; i < repeat; ++i)
        HIPCHK(hipGraphLaunch((hipGraphExec_t)graph_exec, (hipStream_t)stream), "zk_graph_launch");
    return 0;
}

extern "C" int zk_graph_destroy(void* graph_exec) {
    if (graph_exec) HIPCHK(hipGraphExecDestroy((hipGraphExec_t)graph_exec), "zk_graph_destroy");
    return 0;
}

// ---------------------------------------------------------------- event timing (bench roofline)
extern "C" int zk_event_create(void** ev) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e), "zk_event_create");
    *ev = (void*)e;
    return 0;
}
extern "C" int zk_event_record(void* ev, void* stream) {
    HIPCHK(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream), "zk_event_record");
    return 0;
}
extern "C" int zk_event_elapsed_ms(void* a, void* b, float* ms) {
    HIPCHK(hipEventSynchronize((hipEvent_t)b), "zk_event_elapsed(sync)");
    HIPCHK(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b), "zk_event_elapsed");
    return 0;
}
extern "C" int zk_event_destroy(void* ev) {
    if (ev) HIPCHK(hipEventDestroy((hipEvent_t)ev), "zk_event_destroy");
    return 0;
}

// ------------------------------------------------------------------ one decode step
// The launch sequence of zonos_amd.engine.HipDecoder._decode_step (see zonos_hip.h). Each
// entry below checks its own arguments; the first failing one aborts the step with its message.
#define ZK_STEP(call)                  \
    do {                               \
        if ((call) != 0) return -1;    \
    } while (0)

// L2 warm-up descriptor of the decode GEMM zk_gemm_bf16(M, N, K, nsplit) (2 chunks per wave:
// profiles/r3_l2_warm_micro.txt); ZK_L2_WARM=0 builds the step without it (A/B)
#ifndef ZK_L2_WARM
#define ZK_L2_WARM 1
#endif
static ZkWarm warm_desc(const void* W, int M, int N, int K, int nsplit, int mode = 0) {
    return ZK_L2_WARM ? zk_gemm_warm_desc(W, M, N, K, nsplit, mode, 2) : ZkWarm{nullptr, 0, 0, 0, 0};
}

// B = 1: RoPE + KV write in the in_proj epilogue and the prologue-free attention (round 6);
// ZK_B1_QKV_EPI=0 builds the round-5 sequence (in_proj slab -> fused-prologue attention) for A/Bs
#ifndef ZK_B1_QKV_EPI
#define ZK_B1_QKV_EPI 1
#endif

extern "C" int zk_decode_step(const zk_step_desc* d, void* stream) {
    if (d == nullptr || d->layers == nullptr || d->n_layer <= 0 || d->B <= 0) {
        zk_set_error("zk_decode_step: bad descriptor");
        return -1;
    }
    const int K = d->st.K, V = d->st.V, B = d->B, R = 2 * B;
    const int D = d->d_model, H = d->n_heads, Hk = d->n_kv, hd = d->head_dim, Fd = d->d_ff;
    const int Nqkv = (H + 2 * Hk) * hd;
    int32_t* scal = d->st.scal;
    const int32_t* skip = scal + 3;
    const int32_t* pos = scal + 1;
    const zk_step_layer& L0 = d->layers[0];
    // embed_codes (model.py:97-98) + CFG row duplication; layer 0's LayerNorm here unless the
    // small path runs it in the in_proj prologue
    ZK_STEP(zk_embed_codes(d->st.delayed, B, 1, K, (long)d->st.Ld * K, d->st.Ld, scal, -1, d->emb, V, D, 2, d->x, 1,
                           0, d->small ? nullptr : L0.ln1_w, d->small ? nullptr : L0.ln1_b, d->eps,
                           d->small ? nullptr : d->xn, skip, stream));
    for (int i = 0; i < d->n_layer; ++i) {
        const zk_step_layer& L = d->layers[i];
        if (ZK_B1_QKV_EPI && d->small && d->attn_merge > 0 && !d->rope_neox) {
            // B = 1: RoPE + KV write in the in_proj epilogue, a prologue-free attention over 32-key
            // slices, its partials merged by the out_proj GEMV
            ZK_STEP(zk_gemv_qkv_rope(d->x, L.wqkv, R, H, Hk, hd, L.ln1_w, L.ln1_b, d->eps, d->y, L.k_cache,
                                     L.vt_cache, d->smax, pos, d->freqs, skip, stream));
            ZK_STEP(zk_attn_decode_q_part(d->y, L.k_cache, L.vt_cache, R, H, Hk, hd, d->smax, 1, pos, d->attn_work,
                                          d->attn_merge, skip, stream));
            ZK_STEP(zk_gemv_attn_out(d->attn_work, d->attn_merge, Hk, L.wo, R, D, H * hd, d->x, skip, stream));
            ZK_STEP(zk_gemv_fused(d->x, D, L.fc1, R, 2 * Fd, D, 1, L.ln2_w, L.ln2_b, d->eps, nullptr, d->h, skip,
                                  stream));
            ZK_STEP(zk_gemv_fused(d->h, Fd, L.fc2, R, D, Fd, 2, nullptr, nullptr, d->eps, nullptr, d->x, skip,
                                  stream));
        } else if (d->small) {
            ZK_STEP(zk_gemv_fused(d->x, D, L.wqkv, R, Nqkv, D, 0, L.ln1_w, L.ln1_b, d->eps, d->part, nullptr, skip,
                                  stream));
            if (d->attn_merge > 0) {
                ZK_STEP(zk_attn_decode_qkv_part(d->part, 1, d->freqs, L.k_cache, L.vt_cache, R, H, Hk, hd, d->smax, 1,
                                                pos, d->attn_work, d->attn_merge, d->rope_neox, skip, stream));
                ZK_STEP(zk_gemv_attn_out(d->attn_work, d->attn_merge, Hk, L.wo, R, D, H * hd, d->x, skip, stream));
            } else {
                ZK_STEP(zk_attn_decode_qkv_sc(d->part, 1, d->freqs, L.k_cache, L.vt_cache, R, H, Hk, hd, d->smax, 1,
                                              pos, d->attn_work, d->attn_splits, d->attn_cnt, d->y, d->rope_neox,
                                              skip, stream));
                ZK_STEP(zk_gemv_fused(d->y, H * hd, L.wo, R, D, H * hd, 2, nullptr, nullptr, d->eps, nullptr, d->x,
                                      skip, stream));
            }
            ZK_STEP(zk_gemv_fused(d->x, D, L.fc1, R, 2 * Fd, D, 1, L.ln2_w, L.ln2_b, d->eps, nullptr, d->h, skip,
                                  stream));
            ZK_STEP(zk_gemv_fused(d->h, Fd, L.fc2, R, D, Fd, 2, nullptr, nullptr, d->eps, nullptr, d->x, skip,
                                  stream));
        } else {
            ZK_STEP(zk_gemm_bf16(d->xn, D, L.wqkv, R, Nqkv, D, d->split_qkv, 0, d->part, nullptr, skip, stream));
            ZK_STEP(zk_attn_decode_qkv_sc(d->part, d->split_qkv, d->freqs, L.k_cache, L.vt_cache, R, H, Hk, hd,
                                          d->smax, 1, pos, d->attn_work, d->attn_splits, d->attn_cnt, d->y,
                                          d->rope_neox, skip, stream));
            ZK_STEP(zk_gemm_bf16(d->y, H * hd, L.wo, R, D, H * hd, d->split_o, 0, d->part, nullptr, skip, stream));
            // each k_resid_ln and the fc1 GEMM warm the next GEMM's first weight chunks into L2 (warm.h)
            ZK_STEP(zk_resid_ln_warm(d->part, d->split_o, d->x, L.ln2_w, L.ln2_b, d->eps, R, D, d->x, d->xn, 0, skip,
                                     warm_desc(L.fc1, R, 2 * Fd, D, 1, 1), stream));
            ZK_STEP(zk_gemm_bf16_warm(d->xn, D, L.fc1, R, 2 * Fd, D, 1, 1, nullptr, d->h, skip,
                                      warm_desc(L.fc2, R, D, Fd, d->split_fc2), stream));
            ZK_STEP(zk_gemm_bf16(d->h, Fd, L.fc2, R, D, Fd, d->split_fc2, 0, d->part, nullptr, skip, stream));
            const bool last = i + 1 == d->n_layer;
            const ZkWarm next = last ? warm_desc(d->heads, R, K * V, D, d->split_heads)
                                     : warm_desc(d->layers[i + 1].wqkv, R, Nqkv, D, d->split_qkv);
            ZK_STEP(zk_resid_ln_warm(d->part, d->split_fc2, d->x, last ? d->lnf_w : d->layers[i + 1].ln1_w,
                                     last ? d->lnf_b : d->layers[i + 1].ln1_b, d->eps, R, D, d->x, d->xn, 0, skip,
                                     next, stream));
        }
    }
    // 9 heads (model.py:104-111): small path with norm_f as the GEMV prologue, one slab
    if (d->small)
        ZK_STEP(zk_gemv_fused(d->x, D, d->heads, R, K * V, D, 0, d->lnf_w, d->lnf_b, d->eps, d->part, nullptr, skip,
                              stream));
    else
        ZK_STEP(zk_gemm_bf16(d->xn, D, d->heads, R, K * V, D, d->split_heads, 0, d->part, nullptr, skip, stream));
    const int nsp = d->small ? 1 : d->split_heads;
    ZK_STEP(zk_sample_heads(d->part, nsp, &d->st, &d->sp, 0, 0, d->dbg, stream));
    ZK_STEP(zk_sample_heads(d->part, nsp, &d->st, &d->sp, 0, 1, nullptr, stream));
    ZK_STEP(zk_eos_step(&d->st, 0, 0, stream));
    return 0;
}

extern "C" int zk_prefill(const zk_step_desc* d, const void* cond, int Lc, int P, void* q, void* stream) {
    if (d == nullptr || d->layers == nullptr || d->n_layer <= 0 || d->B <= 0 || cond == nullptr || q == nullptr ||
        Lc < 0 || P < 0) {
        zk_set_error("zk_prefill: bad arguments");
        return -1;
    }
    // The last decode step attends over Lc + Ld keys (S = Lc + P + 1 after the prefill, plus
    // Ld - (P + 1) steps, model.py:335-345). The decode attention clamps its context to smax so a
    // no-op launch after the last step stays in bounds; a real step must never need that clamp.
    if (Lc + d->st.Ld > d->smax) {
        zk_set_error("zk_prefill: KV cache of %d keys is shorter than Lc + Ld = %d", d->smax, Lc + d->st.Ld);
        return -1;
    }
    const int K = d->st.K, V = d->st.V, B = d->B, R = 2 * B, S = Lc + P + 1, M = R * S;
    const int D = d->d_model, H = d->n_heads, Hk = d->n_kv, hd = d->head_dim, Fd = d->d_ff;
    const int Nqkv = (H + 2 * Hk) * hd;
    const size_t row = (size_t)D * 2;
    // prefix conditioning into the first Lc positions of every row (model.py:184-186)
    if (Lc > 0) {
        hipError_t e = hipMemcpy2DAsync(d->x, S * row, cond, Lc * row, Lc * row, R, hipMemcpyDeviceToDevice,
                                        (hipStream_t)stream);
        if (e != hipSuccess) {
            zk_set_error("zk_prefill: conditioning copy: %s", hipGetErrorString(e));
            return -1;
        }
    }
    ZK_STEP(zk_embed_codes(d->st.delayed, B, P + 1, K, (long)d->st.Ld * K, d->st.Ld, nullptr, 0, d->emb, V, D, 2,
                           d->x, S, Lc, nullptr, nullptr, d->eps, nullptr, nullptr, stream));
    ZK_STEP(zk_layernorm(d->x, d->layers[0].ln1_w, d->layers[0].ln1_b, d->eps, M, D, d->xn, stream));
    for (int i = 0; i < d->n_layer; ++i) {
        const zk_step_layer& L = d->layers[i];
        ZK_STEP(zk_gemm_bf16(d->xn, D, L.wqkv, M, Nqkv, D, 1, 0, d->part, nullptr, nullptr, stream));
        ZK_STEP(zk_qkv_rope(d->part, 1, R, S, H, Hk, hd, d->freqs, 0, nullptr, q, L.k_cache, L.vt_cache, d->smax,
                            nullptr, d->rope_neox, nullptr, stream));
        ZK_STEP(zk_attn_prefill(q, L.k_cache, L.vt_cache, R, S, H, Hk, hd, d->smax, d->y, stream));
        ZK_STEP(zk_gemm_bf16(d->y, H * hd, L.wo, M, D, H * hd, 1, 0, d->part, nullptr, nullptr, stream));
        ZK_STEP(zk_resid_ln(d->part, 1, d->x, L.ln2_w, L.ln2_b, d->eps, M, D, d->x, d->xn, 0, nullptr, stream));
        ZK_STEP(zk_gemm_bf16(d->xn, D, L.fc1, M, 2 * Fd, D, 1, 1, nullptr, d->h, nullptr, stream));
        ZK_STEP(zk_gemm_bf16(d->h, Fd, L.fc2, M, D, Fd, 1, 0, d->part, nullptr, nullptr, stream));
        const bool last = i + 1 == d->n_layer;
        ZK_STEP(zk_resid_ln(d->part, 1, d->x, last ? d->lnf_w : d->layers[i + 1].ln1_w,
                            last ? d->lnf_b : d->layers[i + 1].ln1_b, d->eps, M, D, d->x, d->xn, 0, nullptr, stream));
    }
    // heads on the last position of every row (rows r*S + S-1 via lda = S*D)
    ZK_STEP(zk_gemm_bf16(static_cast<const char*>(d->xn) + (size_t)(S - 1) * row, (long)S * D, d->heads, R, K * V, D,
                         d->split_heads, 0, d->part, nullptr, nullptr, stream));
    ZK_STEP(zk_sample_heads(d->part, d->split_heads, &d->st, &d->sp, 1, 0, d->dbg, stream));
    ZK_STEP(zk_eos_step(&d->st, 1, P + 1, stream));
    return 0;
}

// ------------------------------------------------------------------ hybrid step (zonos_amd.hybrid)
namespace {
bool hybrid_ok(const zk_hybrid_desc* d) {
    return d != nullptr && d->layers != nullptr && d->n_layer > 0 && d->B > 0 && d->d_inner > 0 &&
           d->nheads_ssm * d->headdim_ssm == d->d_inner && (d->norm_flags & ~6) == 0;
}

// the block sequence of HybridDecoder._layers over M = R*S rows; prefill: S positions per row
// norm_flags (zk_hybrid_desc): bit 1 rms_norm, bit 2 residual_in_fp32 -> zk_resid_ln flag words
int hybrid_resid_flags(const zk_hybrid_desc* d) {
    return 1 | (d->norm_flags & 2) | ((d->norm_flags & 4) ? (4 | 8) : 0);
}
void* hybrid_resid(const zk_hybrid_desc* d) { return (d->norm_flags & 4) ? d->xf : d->x; }

// split-K of a GEMM with reduction length K: the requested split, lowered until it divides K into
// 64-deep chunks (the Mamba-block MLP may be narrower than the attention MLP split_fc2 was chosen for)
int fit_split(int K, int s) {
    while (s > 1 && K % (s * 64) != 0) --s;
    return s;
}

// the first block's norm of the embedding when the config variants are on (layer_norm_fn with
// residual = None: residual = hidden, in fp32 under residual_in_fp32); x holds the embedding rows
int hybrid_prenorm(const zk_hybrid_desc* d, int M, const int32_t* skip, void* stream) {
    const int rf = 1 | (d->norm_flags & 2) | ((d->norm_flags & 4) ? 8 : 0);
    return zk_resid_ln(nullptr, 0, d->x, d->layers[0].ln1_w, d->layers[0].ln1_b, d->eps, M, d->d_model,
                       hybrid_resid(d), d->xn, rf, skip, stream);
}

int hybrid_layers(const zk_hybrid_desc* d, int R, int S, bool prefill, void* q, void* stream) {
    const int M = R * S;
    const int D = d->d_model, H = d->n_heads, Hk = d->n_kv, hd = d->head_dim;
    const int Nqkv = (H + 2 * Hk) * hd, di = d->d_inner, nh = d->nheads_ssm;
    const int nin = 2 * di + 2 * d->d_state + nh;
    const int32_t* scal = d->st.scal;
    const int32_t* skip = prefill ? nullptr : scal + 3;
    const int32_t* pos = prefill ? nullptr : scal + 1;
    const int sq = prefill ? 1 : d->split_qkv, so = prefill ? 1 : d->split_o, sf = prefill ? 1 : d->split_fc2;
    const int si = prefill ? 1 : d->split_inp, su = prefill ? 1 : d->split_out;
    const int K = d->st.K, V = d->st.V;
    const int rf = hybrid_resid_flags(d);
    void* xr = hybrid_resid(d);
    if ((d->norm_flags & 4) && d->xf == nullptr) {
        zk_set_error("zk_hybrid: residual_in_fp32 needs the fp32 residual buffer xf");
        return -1;
    }
    const ZkWarm none{nullptr, 0, 0, 0, 0};
    // L2 warm-up (warm.h) of the GEMM that follows layer i's last k_resid_ln: the next layer's first
    // GEMM, or the heads
    auto next_warm = [&](int i) {
        if (prefill) return none;
        if (i + 1 == d->n_layer) return warm_desc(d->heads, M, K * V, D, d->split_heads);
        const zk_hybrid_layer& N1 = d->layers[i + 1];
        return N1.type == 0 ? warm_desc(N1.wqkv, M, Nqkv, D, sq) : warm_desc(N1.w_in, M, nin, D, si);
    };
    for (int i = 0; i < d->n_layer; ++i) {
        const zk_hybrid_layer& L = d->layers[i];
        const bool last = i + 1 == d->n_layer;
        const void* nw = last ? d->lnf_w : d->layers[i + 1].ln1_w;
        const void* nb = last ? d->lnf_b : d->layers[i + 1].ln1_b;
        int smix;                               // split-K of the mixer's output projection
        if (L.type == 0) {
            ZK_STEP(zk_gemm_bf16(d->xn, D, L.wqkv, M, Nqkv, D, sq, 0, d->part, nullptr, skip, stream));
            if (prefill) {
                ZK_STEP(zk_qkv_rope(d->part, 1, R, S, H, Hk, hd, d->freqs, 0, nullptr, q, L.k_cache, L.vt_cache,
                                    d->smax, nullptr, 1, nullptr, stream));
                ZK_STEP(zk_attn_prefill(q, L.k_cache, L.vt_cache, R, S, H, Hk, hd, d->smax, d->y, stream));
            } else {
                ZK_STEP(zk_attn_decode_qkv(d->part, sq, d->freqs, L.k_cache, L.vt_cache, R, H, Hk, hd, d->smax, 1,
                                           pos, d->attn_work, d->attn_splits, d->y, 1, skip, stream));
            }
            ZK_STEP(zk_gemm_bf16(d->y, H * hd, L.wo, M, D, H * hd, so, 0, d->part, nullptr, skip, stream));
            smix = so;
        } else if (L.type == 1) {
            ZK_STEP(zk_gemm_bf16(d->xn, D, L.w_in, M, nin, D, si, 0, d->part, nullptr, skip, stream));
            if (prefill) {
                // the first decode step (position S) reads the parity-(S & 1) buffers
                ZK_STEP(zk_mamba_prefill(d->part, R, S, di, nh, d->headdim_ssm, d->d_state, L.conv_w, L.conv_b, d->xc,
                                         L.conv_state[S & 1], L.ssm_state[S & 1], L.A, L.dt_bias, L.Dskip, d->yz,
                                         stream));
            } else {
                ZK_STEP(zk_mamba_step(d->part, si, R, di, nh, d->headdim_ssm, d->d_state, L.conv_w, L.conv_b,
                                      L.conv_state[0], L.conv_state[1], pos, L.ssm_state[0], L.ssm_state[1], L.A,
                                      L.dt_bias, L.Dskip, d->yz, skip, stream));
            }
            ZK_STEP(zk_gated_rmsnorm(d->yz, M, di, L.norm_w, d->gate_eps, d->ym, skip, stream));
            ZK_STEP(zk_gemm_bf16(d->ym, di, L.w_out, M, D, di, su, 0, d->part, nullptr, skip, stream));
            smix = su;
        } else {
            zk_set_error("zk_hybrid: layer %d has unknown type %d", i, L.type);
            return -1;
        }
        // Block.mlp (_mamba_ssm.py:18-22: GatedMLP of d_intermediate on Mamba2 blocks when it is
        // nonzero, of attn_mlp_d_intermediate on attention blocks): norm2 -> fc1 (SwiGLU) -> fc2
        const int Fl = L.type == 0 ? (L.d_mlp > 0 ? L.d_mlp : d->d_ff) : L.d_mlp;
        if (Fl > 0) {
            const int sfl = prefill ? 1 : fit_split(Fl, sf);
            ZK_STEP(zk_resid_ln_warm(d->part, smix, xr, L.ln2_w, L.ln2_b, d->eps, M, D, xr, d->xn, rf, skip,
                                     prefill ? none : warm_desc(L.fc1, M, 2 * Fl, D, 1, 1), stream));
            ZK_STEP(zk_gemm_bf16_warm(d->xn, D, L.fc1, M, 2 * Fl, D, 1, 1, nullptr, d->h, skip,
                                      prefill ? none : warm_desc(L.fc2, M, D, Fl, sfl), stream));
            ZK_STEP(zk_gemm_bf16(d->h, Fl, L.fc2, M, D, Fl, sfl, 0, d->part, nullptr, skip, stream));
            smix = sfl;
        }
        ZK_STEP(zk_resid_ln_warm(d->part, smix, xr, nw, nb, d->eps, M, D, xr, d->xn, rf, skip, next_warm(i), stream));
    }
    return 0;
}
}  // namespace

extern "C" int zk_hybrid_decode_step(const zk_hybrid_desc* d, void* stream) {
    if (!hybrid_ok(d)) {
        zk_set_error("zk_hybrid_decode_step: bad descriptor");
        return -1;
    }
    const int K = d->st.K, V = d->st.V, B = d->B, R = 2 * B, D = d->d_model;
    int32_t* scal = d->st.scal;
    const int32_t* skip = scal + 3;
    const bool var = (d->norm_flags & 6) != 0;       // config variants: the first norm is its own launch
    ZK_STEP(zk_embed_codes(d->st.delayed, B, 1, K, (long)d->st.Ld * K, d->st.Ld, scal, -1, d->emb, V, D, 2, d->x, 1, 0,
                           var ? nullptr : d->layers[0].ln1_w, var ? nullptr : d->layers[0].ln1_b, d->eps,
                           var ? nullptr : d->xn, skip, stream));
    if (var) ZK_STEP(hybrid_prenorm(d, R, skip, stream));
    ZK_STEP(hybrid_layers(d, R, 1, false, nullptr, stream));
    ZK_STEP(zk_gemm_bf16(d->xn, D, d->heads, R, K * V, D, d->split_heads, 0, d->part, nullptr, skip, stream));
    ZK_STEP(zk_sample_heads(d->part, d->split_heads, &d->st, &d->sp, 0, 0, d->dbg, stream));
    ZK_STEP(zk_sample_heads(d->part, d->split_heads, &d->st, &d->sp, 0, 1, nullptr, stream));
    ZK_STEP(zk_eos_step(&d->st, 0, 0, stream));
    return 0;
}

extern "C" int zk_hybrid_prefill(const zk_hybrid_desc* d, const void* cond, int Lc, int P, void* q, void* stream) {
    if (!hybrid_ok(d) || cond == nullptr || q == nullptr || Lc < 0 || P < 0) {
        zk_set_error("zk_hybrid_prefill: bad arguments");
        return -1;
    }
    if (Lc + d->st.Ld > d->smax) {     // as zk_prefill: no real step may need the attention's clamp
        zk_set_error("zk_hybrid_prefill: KV cache of %d keys is shorter than Lc + Ld = %d", d->smax, Lc + d->st.Ld);
        return -1;
    }
    const int K = d->st.K, V = d->st.V, B = d->B, R = 2 * B, S = Lc + P + 1, D = d->d_model;
    const size_t row = (size_t)D * 2;
    if (Lc > 0) {
        hipError_t e = hipMemcpy2DAsync(d->x, S * row, cond, Lc * row, Lc * row, R, hipMemcpyDeviceToDevice,
                                        (hipStream_t)stream);
        if (e != hipSuccess) {
            zk_set_error("zk_hybrid_prefill: conditioning copy: %s", hipGetErrorString(e));
            return -1;
        }
    }
    ZK_STEP(zk_embed_codes(d->st.delayed, B, P + 1, K, (long)d->st.Ld * K, d->st.Ld, nullptr, 0, d->emb, V, D, 2,
                           d->x, S, Lc, nullptr, nullptr, d->eps, nullptr, nullptr, stream));
    if (d->norm_flags & 6) ZK_STEP(hybrid_prenorm(d, R * S, nullptr, stream));
    else ZK_STEP(zk_layernorm(d->x, d->layers[0].ln1_w, d->layers[0].ln1_b, d->eps, R * S, D, d->xn, stream));
    ZK_STEP(hybrid_layers(d, R, S, true, q, stream));
    ZK_STEP(zk_gemm_bf16(static_cast<const char*>(d->xn) + (size_t)(S - 1) * row, (long)S * D, d->heads, R, K * V, D,
                         d->split_heads, 0, d->part, nullptr, nullptr, stream));
    ZK_STEP(zk_sample_heads(d->part, d->split_heads, &d->st, &d->sp, 1, 0, d->dbg, stream));
    ZK_STEP(zk_eos_step(&d->st, 1, P + 1, stream));
    return 0;
}
#undef ZK_STEP

// ------------------------------------------------------------------ DAC decode (whole)
namespace {
struct DacPlan {
    size_t z, a, b, x, tmp, last, total;
};
size_t zk_align(size_t v) { return (v + 255) & ~(size_t)255; }
bool dac_plan(const zk_dac_desc* d, int B, int T, DacPlan& p) {
    if (d == nullptr || d->nblocks < 0 || d->nblocks > ZK_DAC_MAXB || B <= 0 || T <= 0) return false;
    size_t L = (size_t)T, act = (size_t)B * T * d->c0, big = 0, lastc = d->c0;
    for (int i = 0; i < d->nblocks; ++i) {
        const zk_dac_block& k = d->blocks[i];
        if (k.nres < 1 || k.nres > ZK_DAC_MAXR) return false;
        L *= (size_t)k.stride;
        const size_t n = (size_t)B * L * k.cout;
        act = std::max(act, n);
        big = std::max(big, n);
        lastc = k.cout;
    }
    p.z = 0;
    p.a = zk_align(p.z + (size_t)B * T * d->cin0 * 2);
    p.b = zk_align(p.a + act * 2);
    p.x = zk_align(p.b + act * 2);
    p.tmp = zk_align(p.x + big * 4);
    p.last = zk_align(p.tmp + act * 2);
    p.total = zk_align(p.last + (size_t)B * L * lastc * 4);
    return true;
}
}  // namespace

extern "C" size_t zk_dac_decode_workspace(const zk_dac_desc* d, int B, int T) {
    DacPlan p;
    return dac_plan(d, B, T, p) ? p.total : 0;
}

#define ZK_DSTEP(call)                 \
    do {                               \
        if ((call) != 0) return -1;    \
    } while (0)

extern "C" int zk_dac_decode(const zk_dac_desc* d, const int64_t* codes, int B, int T, const int32_t* lens,
                             void* workspace, size_t workspace_bytes, float* out, void* stream) {
    DacPlan p;
    if (!dac_plan(d, B, T, p) || codes == nullptr || out == nullptr || workspace == nullptr) {
        zk_set_error("zk_dac_decode: bad arguments");
        return -1;
    }
    if (workspace_bytes < p.total) {
        zk_set_error("zk_dac_decode: workspace %zu bytes < %zu needed", workspace_bytes, p.total);
        return -1;
    }
    char* ws = static_cast<char*>(workspace);
    uint16_t* z = reinterpret_cast<uint16_t*>(ws + p.z);
    // three fp16 activation buffers; each conv writes one its input is not in (a fused residual unit
    // reads its input's neighbours as the k7 halo, so it never writes in place)
    uint16_t* bufs[3] = {reinterpret_cast<uint16_t*>(ws + p.a), reinterpret_cast<uint16_t*>(ws + p.b),
                         reinterpret_cast<uint16_t*>(ws + p.tmp)};
    auto other = [&](const void* u, const void* v) -> uint16_t* {
        for (uint16_t* c : bufs)
            if (c != u && c != v) return c;
        return nullptr;
    };
    float* x = reinterpret_cast<float*>(ws + p.x);
    float* last_act = reinterpret_cast<float*>(ws + p.last);
    ZK_DSTEP(zk_dac_rvq_decode_cl(codes, B, d->ncb, T, (long)d->ncb * T, d->tables, d->codebook_size, d->hidden,
                                  d->cin0, z, lens, stream));
    const float* a_next = d->nblocks ? d->blocks[0].alpha : d->final_alpha;
    ZK_DSTEP(zk_dac_conv_cl(z, B, d->cin0, T, d->conv1_w, 0, d->conv1_b, d->c0, 7, 1, 3, T, 1, 1, 0, T, nullptr,
                            nullptr, a_next, bufs[0], 0, lens, 1, 1, stream));
    int L = T, scale = 1, cch = d->c0;
    const void* act = bufs[0];
    bool act_f32 = false;
    for (int bi = 0; bi < d->nblocks; ++bi) {
        const zk_dac_block& k = d->blocks[bi];
        const int st = k.stride, Lo = L * st;
        uint16_t* s_new = other(act, nullptr);
        ZK_DSTEP(zk_dac_conv_cl(static_cast<const uint16_t*>(act), B, k.cin, L, k.wt, 2L * k.cout * k.cin, k.bt,
                                k.cout, 2, 1, 1, L + 1, st, st, -((st + 1) / 2), Lo, nullptr, x, k.res[0].a1, s_new, 0,
                                lens, scale, scale * st, stream));
        act = s_new;
        scale *= st;
        L = Lo;
        for (int j = 0; j < k.nres; ++j) {
            const zk_dac_resunit& ru = k.res[j];
            const float* an = j + 1 < k.nres ? k.res[j + 1].a1 : (bi + 1 < d->nblocks ? d->blocks[bi + 1].alpha
                                                                                           : d->final_alpha);
            const bool last = j + 1 == k.nres && bi + 1 == d->nblocks;
            uint16_t* tmp = other(act, nullptr);
            const int fm = zk_dac_resunit_supported(k.cout);
            if (fm == 2 || (fm == 1 && !last)) {
                // the whole unit in one launch (k7 -> Snake -> 1x1 -> + x -> next Snake)
                void* s_out = last ? static_cast<void*>(last_act) : static_cast<void*>(tmp);
                ZK_DSTEP(zk_dac_resunit_cl(static_cast<const uint16_t*>(act), B, k.cout, L, ru.w1, ru.b1, ru.dil,
                                           ru.a2, ru.w2, ru.b2, x, an, s_out, last ? 1 : 0, lens, scale, stream));
                act = s_out;
            } else {
                ZK_DSTEP(zk_dac_conv_cl(static_cast<const uint16_t*>(act), B, k.cout, L, ru.w1, 0, ru.b1, k.cout, 7,
                                        ru.dil, 3 * ru.dil, L, 1, 1, 0, L, nullptr, nullptr, ru.a2, tmp, 0, lens,
                                        scale, scale, stream));
                void* s_out = last ? static_cast<void*>(last_act) : const_cast<void*>(act);
                ZK_DSTEP(zk_dac_conv_cl(tmp, B, k.cout, L, ru.w2, 0, ru.b2, k.cout, 1, 1, 0, L, 1, 1, 0, L, x, x, an,
                                        s_out, last ? 1 : 0, lens, scale, scale, stream));
                act = s_out;
            }
            if (last) act_f32 = true;
        }
        cch = k.cout;
    }
    if (!act_f32) {
        zk_set_error("zk_dac_decode: the tail needs at least one block (fp32 Snake input)");
        return -1;
    }
    ZK_DSTEP(zk_dac_tail_cl(static_cast<const float*>(act), B, cch, L, d->conv2_w, d->conv2_b, out, lens, scale,
                            stream));
    return 0;
}
#undef ZK_DSTEP
