// CPU AddressSanitizer build of the host-side C ABI code (zonos_amd/csrc/capi.cpp): descriptor
// validation, DAC workspace planning and the step / prefill / DAC launch sequences, with every
// device entry point replaced by a recording stub (no GPU, no HIP kernels). Built and run by
// tests/test_capi_asan_cpu.py:
//   g++ -fsanitize=address,undefined -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include capi.cpp capi_asan.cpp -lamdhip64
// Exit 0 = every check passed and ASAN saw no invalid access.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/zonos_hip.h"

static std::vector<std::string> g_calls;
static int g_fail_at = -1;          // make the n-th stubbed call fail (error propagation)
static int stub(const char* name) {
    g_calls.push_back(name);
    return (int)g_calls.size() - 1 == g_fail_at ? -1 : 0;
}
#define STUB(ret_name, ...) extern "C" int ret_name(__VA_ARGS__) { return stub(#ret_name); }

// ---- the device entry points capi.cpp enqueues (signatures of include/zonos_hip.h)
STUB(zk_embed_codes, const int64_t*, int, int, int, long, long, const int32_t*, int, const void*, int, int, int, void*,
     int, int, const void*, const void*, float, void*, const int32_t*, void*)
STUB(zk_layernorm, const void*, const void*, const void*, float, int, int, void*, void*)
STUB(zk_resid_ln, const float*, int, const void*, const void*, const void*, float, int, int, void*, void*, int,
     const int32_t*, void*)
STUB(zk_gemm_bf16, const void*, long, const void*, int, int, int, int, int, float*, void*, const int32_t*, void*)
STUB(zk_gemv_fused, const void*, long, const void*, int, int, int, int, const void*, const void*, float, float*, void*,
     const int32_t*, void*)
STUB(zk_gemv_attn_out, const float*, int, int, const void*, int, int, int, void*, const int32_t*, void*)
STUB(zk_qkv_rope, const float*, int, int, int, int, int, int, const float*, int, const int32_t*, void*, void*, void*,
     int, void*, int, const int32_t*, void*)
STUB(zk_attn_prefill, const void*, const void*, const void*, int, int, int, int, int, int, void*, void*)
STUB(zk_attn_decode_qkv, const float*, int, const float*, void*, void*, int, int, int, int, int, int, const int32_t*,
     float*, int, void*, int, const int32_t*, void*)
STUB(zk_attn_decode_qkv_sc, const float*, int, const float*, void*, void*, int, int, int, int, int, int,
     const int32_t*, float*, int, uint32_t*, void*, int, const int32_t*, void*)
STUB(zk_attn_decode_qkv_part, const float*, int, const float*, void*, void*, int, int, int, int, int, int,
     const int32_t*, float*, int, int, const int32_t*, void*)
STUB(zk_gemv_qkv_rope, const void*, const void*, int, int, int, int, const void*, const void*, float, void*, void*,
     void*, int, const int32_t*, const float*, const int32_t*, void*)
STUB(zk_attn_decode_q_part, const void*, const void*, const void*, int, int, int, int, int, int, const int32_t*, float*,
     int, const int32_t*, void*)
STUB(zk_sample_heads, const float*, int, const zk_gen_state*, const zk_sampling_params*, int, int, float*, void*)
STUB(zk_eos_step, const zk_gen_state*, int, int, void*)
STUB(zk_mamba_step, const float*, int, int, int, int, int, int, const float*, const float*, void*, void*,
     const int32_t*, void*, void*, const float*, const float*, const float*, float*, const int32_t*, void*)
STUB(zk_mamba_prefill, const float*, int, int, int, int, int, int, const float*, const float*, void*, void*, void*,
     const float*, const float*, const float*, float*, void*)
STUB(zk_gated_rmsnorm, const float*, int, int, const float*, float, void*, const int32_t*, void*)
STUB(zk_dac_rvq_decode_cl, const int64_t*, int, int, int, long, const float*, int, int, int, uint16_t*,
     const int32_t*, void*)
STUB(zk_dac_conv_cl, const uint16_t*, int, int, int, const uint16_t*, long, const float*, int, int, int, int, int, int,
     int, int, int, const float*, float*, const float*, void*, int, const int32_t*, int, int, void*)
STUB(zk_dac_tail_cl, const float*, int, int, int, const float*, const float*, float*, const int32_t*, int, void*)
static int g_alias = 0;             // fused residual units whose output buffer aliased their input
extern "C" int zk_dac_resunit_supported(int C) { return C == 96 ? 1 : 0; }
extern "C" int zk_dac_resunit_cl(const uint16_t* s_in, int, int, int, const uint16_t*, const float*, int, const float*,
                                 const uint16_t*, const float*, float*, const float*, void* s_out, int,
                                 const int32_t*, int, void*) {
    g_alias += s_out == static_cast<const void*>(s_in);
    return stub("zk_dac_resunit_cl");
}

// ---- internal entries of zonos_amd/csrc/warm.h (C++ linkage): a warm-up variant records as the launch it
// replaces, so the per-layer launch counts below are the same with and without the L2 warm-up
#include "../../zonos_amd/csrc/warm.h"
static int g_warm = 0;              // launches that carried a warm-up descriptor
ZkWarm zk_gemm_warm_desc(const void* W, int, int N, int K, int nsplit, int, int chunks) {
    return ZkWarm{W, K, N / 64, nsplit, chunks};
}
int zk_resid_ln_warm(const float*, int, const void*, const void*, const void*, float, int, int, void*, void*, int,
                     const int32_t*, ZkWarm warm, void*) {
    g_warm += warm.W != nullptr;
    return stub("zk_resid_ln");
}
int zk_gemm_bf16_warm(const void*, long, const void*, int, int, int, int, int, float*, void*, const int32_t*,
                      ZkWarm warm, void*) {
    g_warm += warm.W != nullptr;
    return stub("zk_gemm_bf16");
}

static int g_bad = 0;
#define CHECK(cond, ...)                                     \
    do {                                                     \
        if (!(cond)) {                                       \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                    \
            fprintf(stderr, "\n");                           \
            ++g_bad;                                         \
        }                                                    \
    } while (0)

static size_t count(const char* name) {
    size_t n = 0;
    for (auto& c : g_calls) n += c == name;
    return n;
}

// host buffers stand in for device memory: the host code only forms addresses from them
static std::vector<char> g_mem(1 << 20);
static void* P(size_t off) { return g_mem.data() + off; }

static void transformer(int n_layer, int small, int merge) {
    std::vector<zk_step_layer> layers(n_layer);
    for (int i = 0; i < n_layer; ++i) layers[i] = zk_step_layer{P(64 * i), P(64 * i + 8), P(1024), P(2048), P(3072),
                                                                 P(4096), P(5120), P(6144), P(7168), P(8192)};
    static int32_t scal[16];
    zk_step_desc d;
    memset(&d, 0, sizeof d);
    d.B = small ? 1 : 64; d.n_layer = n_layer; d.d_model = 2048; d.n_heads = 16; d.n_kv = 4; d.head_dim = 128;
    d.d_ff = 8192; d.smax = 3072; d.split_qkv = 4; d.split_o = 4; d.split_fc2 = 8; d.split_heads = 1;
    d.attn_splits = 1; d.attn_merge = merge; d.small = small; d.eps = 1e-5f; d.layers = layers.data();
    d.emb = d.heads = d.lnf_w = d.lnf_b = P(0);
    d.freqs = (const float*)P(0);
    d.x = d.xn = d.y = d.h = P(0);
    d.part = d.attn_work = (float*)P(0);
    d.st.scal = scal; d.st.K = 9; d.st.V = 1026; d.st.Ld = 2599; d.st.B = d.B;
    g_calls.clear();
    g_warm = 0;
    CHECK(zk_decode_step(&d, nullptr) == 0, "zk_decode_step: %s", zk_last_error());
    // full step: both k_resid_ln and the fc1 GEMM of every layer warm the next GEMM's weights
    if (!small) CHECK(g_warm == 3 * n_layer, "L2 warm-up descriptors: %d", g_warm);
    // embed + per layer (small: 5 with merge, 5 without; else 7) + heads + 2 samples + eos
    const size_t per = small ? 5 : 7;
    CHECK(g_calls.size() == 1 + per * n_layer + 4, "decode step: %zu calls", g_calls.size());
    CHECK(count("zk_sample_heads") == 2 && count("zk_eos_step") == 1, "decode tail");
    if (!small) CHECK(count("zk_resid_ln") == (size_t)2 * n_layer, "resid_ln x2 per layer");
    if (small && merge) CHECK(count("zk_gemv_attn_out") == (size_t)n_layer, "merged out_proj per layer");
    // B = 1 with merged splits: the in_proj RoPE epilogue + the prologue-free attention
    if (small && merge)
        CHECK(count("zk_gemv_qkv_rope") == (size_t)n_layer && count("zk_attn_decode_q_part") == (size_t)n_layer &&
                  count("zk_attn_decode_qkv_part") == 0,
              "B = 1 layer sequence");
    // prefill
    g_calls.clear();
    g_warm = 0;
    CHECK(zk_prefill(&d, P(0), 0, 10, P(0), nullptr) == 0, "zk_prefill: %s", zk_last_error());
    CHECK(g_warm == 0, "prefill must not warm (%d)", g_warm);
    CHECK(g_calls.size() == 2 + 8 * (size_t)n_layer + 3, "prefill: %zu calls", g_calls.size());
    // error propagation: the 5th enqueue fails -> the step stops there and reports it
    g_calls.clear();
    g_fail_at = 4;
    CHECK(zk_decode_step(&d, nullptr) != 0 && g_calls.size() == 5, "failure must stop the step (%zu)", g_calls.size());
    g_fail_at = -1;
    // descriptor validation
    CHECK(zk_decode_step(nullptr, nullptr) != 0 && strstr(zk_last_error(), "bad descriptor"), "null desc");
    zk_step_desc e = d;
    e.layers = nullptr;
    CHECK(zk_decode_step(&e, nullptr) != 0, "null layers");
    e = d;
    e.n_layer = 0;
    CHECK(zk_decode_step(&e, nullptr) != 0, "zero layers");
    e = d;
    e.B = 0;
    CHECK(zk_prefill(&e, P(0), 4, 0, P(0), nullptr) != 0, "zero batch");
    CHECK(zk_prefill(&d, nullptr, 4, 0, P(0), nullptr) != 0, "null cond");
    CHECK(zk_prefill(&d, P(0), -1, 0, P(0), nullptr) != 0, "negative Lc");
}

static void hybrid() {
    std::vector<zk_hybrid_layer> layers(5);
    for (int i = 0; i < 5; ++i) {
        memset(&layers[i], 0, sizeof(zk_hybrid_layer));
        layers[i].type = i == 2 ? 0 : 1;
    }
    static int32_t scal[16];
    zk_hybrid_desc d;
    memset(&d, 0, sizeof d);
    d.B = 64; d.n_layer = 5; d.d_model = 2048; d.n_heads = 16; d.n_kv = 4; d.head_dim = 128; d.d_ff = 8192;
    d.smax = 3072; d.d_inner = 4096; d.nheads_ssm = 64; d.headdim_ssm = 64; d.d_state = 128; d.split_qkv = 4;
    d.split_o = 4; d.split_fc2 = 8; d.split_heads = 1; d.split_inp = 1; d.split_out = 2; d.attn_splits = 1;
    d.eps = 1e-5f; d.gate_eps = 1e-5f; d.layers = layers.data(); d.st.scal = scal; d.st.K = 9; d.st.V = 1026;
    d.st.Ld = 2599; d.x = d.xn = P(0);
    g_calls.clear();
    CHECK(zk_hybrid_decode_step(&d, nullptr) == 0, "zk_hybrid_decode_step: %s", zk_last_error());
    CHECK(count("zk_mamba_step") == 4 && count("zk_attn_decode_qkv") == 1 && count("zk_gated_rmsnorm") == 4,
          "hybrid layer sequence");
    CHECK(g_calls.size() == 1 + 4 * 5 + 1 * 7 + 4, "hybrid step: %zu calls", g_calls.size());
    g_calls.clear();
    CHECK(zk_hybrid_prefill(&d, P(0), 0, 4, P(0), nullptr) == 0, "zk_hybrid_prefill: %s", zk_last_error());
    CHECK(count("zk_mamba_prefill") == 4 && count("zk_attn_prefill") == 1, "hybrid prefill sequence");
    layers[3].type = 7;
    CHECK(zk_hybrid_decode_step(&d, nullptr) != 0 && strstr(zk_last_error(), "unknown type"), "bad layer type");
    layers[3].type = 1;
    d.nheads_ssm = 63;
    CHECK(zk_hybrid_decode_step(&d, nullptr) != 0, "nheads * headdim != d_inner");
    CHECK(zk_hybrid_decode_step(nullptr, nullptr) != 0, "null hybrid desc");
}

static zk_dac_desc dac_desc(int nblocks) {
    zk_dac_desc d;
    memset(&d, 0, sizeof d);
    d.nblocks = nblocks; d.ncb = 9; d.codebook_size = 1024; d.hidden = 1024; d.cin0 = 1024; d.c0 = 1536;
    const int strides[4] = {8, 8, 4, 2};
    int c = 1536;
    for (int i = 0; i < nblocks && i < ZK_DAC_MAXB; ++i) {
        d.blocks[i].stride = strides[i % 4];
        d.blocks[i].cin = c;
        d.blocks[i].cout = c / 2 < 32 ? 32 : c / 2;
        d.blocks[i].nres = 3;
        c = d.blocks[i].cout;
    }
    return d;
}

static void dac() {
    zk_dac_desc d = dac_desc(4);
    const size_t w1 = zk_dac_decode_workspace(&d, 1, 43), w64 = zk_dac_decode_workspace(&d, 64, 2590);
    CHECK(w1 > 0 && w64 > w1 && w64 % 256 == 0, "workspace sizes %zu %zu", w1, w64);
    // activation at the last block: B * T * 512 * 96 channels, fp32 -> the plan holds at least that
    CHECK(w64 >= (size_t)64 * 2590 * 512 * 96 * 4, "plan too small for the last activation");
    CHECK(zk_dac_decode_workspace(&d, 0, 43) == 0 && zk_dac_decode_workspace(&d, 1, 0) == 0, "empty shapes");
    zk_dac_desc bad = dac_desc(4);
    bad.nblocks = ZK_DAC_MAXB + 1;
    CHECK(zk_dac_decode_workspace(&bad, 1, 43) == 0, "too many blocks");
    bad = dac_desc(4);
    bad.blocks[1].nres = ZK_DAC_MAXR + 1;
    CHECK(zk_dac_decode_workspace(&bad, 1, 43) == 0, "too many residual units");
    std::vector<char> ws(w1);
    static int64_t codes[9 * 43];
    static float out[43 * 512];
    g_calls.clear();
    CHECK(zk_dac_decode(&d, codes, 1, 43, nullptr, ws.data(), ws.size(), out, nullptr) == 0, "dac: %s",
          zk_last_error());
    // rvq + conv1 + per block (ConvT + 3 x (k7 + 1x1)) + tail; the 96-channel block's first two units
    // fused (one launch each), never writing their input buffer
    CHECK(g_calls.size() == 1 + 1 + 4 * 7 + 1 - 2, "dac decode: %zu calls", g_calls.size());
    int nfused = 0;
    for (const std::string& c : g_calls) nfused += c == "zk_dac_resunit_cl";
    CHECK(nfused == 2 && g_alias == 0, "fused units %d, aliased %d", nfused, g_alias);
    CHECK(zk_dac_decode(&d, codes, 1, 43, nullptr, ws.data(), ws.size() - 1, out, nullptr) != 0 &&
              strstr(zk_last_error(), "workspace"), "small workspace must fail");
    zk_dac_desc nob = dac_desc(0);
    std::vector<char> ws0(zk_dac_decode_workspace(&nob, 1, 43));
    CHECK(zk_dac_decode(&nob, codes, 1, 43, nullptr, ws0.data(), ws0.size(), out, nullptr) != 0, "no blocks");
    CHECK(zk_dac_decode(&d, nullptr, 1, 43, nullptr, ws.data(), ws.size(), out, nullptr) != 0, "null codes");
}

int main() {
    transformer(26, 0, 0);
    transformer(26, 1, 4);
    transformer(3, 1, 0);
    hybrid();
    dac();
    CHECK(zk_abi_size(99) == -1, "unknown abi id");
    if (g_bad) {
        fprintf(stderr, "%d check(s) failed\n", g_bad);
        return 1;
    }
    printf("capi_asan: all checks passed\n");
    return 0;
}
