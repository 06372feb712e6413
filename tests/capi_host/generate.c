/* A C host for libzonos_hip.so: Zonos.generate (zonos/model.py:224-457) driven entirely through the
 * C ABI of include/zonos_hip.h -- no Python, no torch. It shows what a non-Python host needs:
 * upload the checkpoint tensors, bring them into the engine layouts with the library's own
 * entries (zk_permute_fc1, zk_pack_weights), size the workspace, then
 *   zk_delay_apply -> zk_prefill -> [host: loop state, model.py:316-342] ->
 *   hipGraph capture of zk_decode_step (zk_graph_begin / zk_graph_end) -> replay until the `done`
 *   word is set -> zk_delay_revert -> trim (model.py:437-457).
 *
 * Test helper of tests/test_gpu_capi_host.py (which writes the input file and checks the codes).
 *   usage: generate <input.bin> <output.bin>
 * Input (little endian): int32 header[16] = {magic 0x5a4b4831, D, n_layer, H, Hkv, d_ff, B, Lc, P,
 * max_new, head_rows, poll_every, rp_window, top_k, noise_mode, noise_stride}, float32 fparams[8] = {eps,
 * cfg_scale, temperature, top_p, min_p, linear, conf, quad}, float32 rep_penalty, uint64 seed (noise_mode 1:
 * + uint64 noise_offset, uint64 noise_incr -- torch's GPU exponential_ stream, zk_gen_state), then bf16
 * tensors per layer (norm.w, norm.b, in_proj [3D'][D], out_proj [D][D], norm2.w, norm2.b,
 * fc1 [2F][D], fc2 [D][F]), norm_f.w, norm_f.b, 9 embeddings [1026][D], 9 heads [head_rows][D],
 * fp32 RoPE table [16384][hd/2][2], bf16 conditioning [2B][Lc][D], int64 prefix codes [B][9][P].
 * Output: int32 B, then per utterance int32 length T_i and int64 codes [9][T_i]; stdout reports the
 * sampler calls made (scal[2] + scal[4]: the Philox offset a torch-noise run consumed is calls * incr). */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zonos_hip.h"

#define NCB 9
#define VOCAB 1026
#define EOS_ID 1024
#define MASK_ID 1025
#define ROPE_LEN 16384

static void die(const char* what) {
    fprintf(stderr, "generate: %s: %s\n", what, zk_last_error());
    exit(2);
}
#define ZK(call) do { if ((call) != 0) die(#call); } while (0)
#define HIP(call)                                                                   \
    do {                                                                            \
        hipError_t e_ = (call);                                                     \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "generate: %s: %s\n", #call, hipGetErrorString(e_));    \
            exit(2);                                                                \
        }                                                                           \
    } while (0)

static FILE* g_in;
static void rd(void* p, size_t n) {
    if (fread(p, 1, n, g_in) != n) { fprintf(stderr, "generate: short input\n"); exit(2); }
}
static void* dalloc(size_t n) {
    void* p = NULL;
    HIP(hipMalloc(&p, n ? n : 16));
    return p;
}
static void* dzero(size_t n) {
    void* p = dalloc(n);
    HIP(hipMemset(p, 0, n ? n : 16));
    return p;
}
/* read n bytes of the input straight into a fresh device buffer */
static void* dread(size_t n) {
    void* h = malloc(n ? n : 16);
    rd(h, n);
    void* d = dalloc(n);
    HIP(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
    free(h);
    return d;
}
/* nn.Linear bf16 [N][K] -> the GEMM's fragment-packed layout (rows padded to 64) */
static void* packed(const void* w, int N, int K, hipStream_t s) {
    void* out = dzero((size_t)(N + 63) / 64 * 64 * K * 2);
    ZK(zk_pack_weights(w, N, K, out, s));
    return out;
}
/* zonos_amd.engine._split_for: K-split count that covers the CUs, a function of (N, K) only */
static int split_for(int N, int K, int M, int target) {
    if (M > 128) return 1;
    const int tiles = (N + 63) / 64, want = (target + tiles - 1) / tiles > 1 ? (target + tiles - 1) / tiles : 1;
    int s = 1;
    for (int c = 1; c <= want; ++c)
        if (K % (c * 64) == 0) s = c;
    return s;
}

int main(int argc, char** argv) {
    if (argc != 3) { fprintf(stderr, "usage: generate <input.bin> <output.bin>\n"); return 2; }
    g_in = fopen(argv[1], "rb");
    if (!g_in) { perror(argv[1]); return 2; }
    int32_t hdr[16];
    float fp[8], rp;
    uint64_t seed;
    rd(hdr, sizeof hdr);
    rd(fp, sizeof fp);
    rd(&rp, sizeof rp);
    rd(&seed, sizeof seed);
    if (hdr[0] != 0x5a4b4831) { fprintf(stderr, "generate: bad magic\n"); return 2; }
    uint64_t noise_off = 0, noise_incr = 0;
    if (hdr[14]) {
        rd(&noise_off, sizeof noise_off);
        rd(&noise_incr, sizeof noise_incr);
    }
    const int D = hdr[1], NL = hdr[2], H = hdr[3], Hk = hdr[4], Fd = hdr[5], B = hdr[6], Lc = hdr[7], P = hdr[8];
    const int max_new = hdr[9], head_rows = hdr[10], poll_every = hdr[11];
    const int hd = D / H, Nqkv = (H + 2 * Hk) * hd, R = 2 * B;
    hipStream_t s;
    HIP(hipStreamCreate(&s));

    /* ---- weights into the engine layouts (zonos_amd.engine.HipBackbone.__init__) */
    zk_step_layer* layers = (zk_step_layer*)calloc(NL, sizeof(zk_step_layer));
    for (int i = 0; i < NL; ++i) {
        zk_step_layer* L = &layers[i];
        L->ln1_w = dread((size_t)D * 2);
        L->ln1_b = dread((size_t)D * 2);
        void* wqkv = dread((size_t)Nqkv * D * 2);
        void* wo = dread((size_t)D * D * 2);
        L->ln2_w = dread((size_t)D * 2);
        L->ln2_b = dread((size_t)D * 2);
        void* fc1 = dread((size_t)2 * Fd * D * 2);
        void* fc2 = dread((size_t)D * Fd * 2);
        void* fc1p = dalloc((size_t)2 * Fd * D * 2);
        ZK(zk_permute_fc1(fc1, Fd, D, fc1p, s));   /* y / gate rows interleaved for the SwiGLU epilogue */
        L->wqkv = packed(wqkv, Nqkv, D, s);
        L->wo = packed(wo, D, D, s);
        L->fc1 = packed(fc1p, 2 * Fd, D, s);
        L->fc2 = packed(fc2, D, Fd, s);
        HIP(hipStreamSynchronize(s));
        HIP(hipFree(wqkv)); HIP(hipFree(wo)); HIP(hipFree(fc1)); HIP(hipFree(fc2)); HIP(hipFree(fc1p));
    }
    void* lnf_w = dread((size_t)D * 2);
    void* lnf_b = dread((size_t)D * 2);
    void* emb = dread((size_t)NCB * VOCAB * D * 2);
    /* 9 heads stacked [9][1026][D]; pad_weight_ (zonos/utils.py:30-35): 1025 -> 1026 rows */
    char* heads_h = (char*)calloc((size_t)NCB * VOCAB * D, 2);
    for (int k = 0; k < NCB; ++k) rd(heads_h + (size_t)k * VOCAB * D * 2, (size_t)head_rows * D * 2);
    void* heads_raw = dalloc((size_t)NCB * VOCAB * D * 2);
    HIP(hipMemcpy(heads_raw, heads_h, (size_t)NCB * VOCAB * D * 2, hipMemcpyHostToDevice));
    free(heads_h);
    void* heads = packed(heads_raw, NCB * VOCAB, D, s);
    float* freqs = (float*)dread((size_t)ROPE_LEN * (hd / 2) * 2 * 4);
    void* cond = dread((size_t)R * Lc * D * 2);
    int64_t* prefix_h = (int64_t*)malloc((size_t)B * NCB * (P ? P : 1) * 8);
    rd(prefix_h, (size_t)B * NCB * P * 8);
    fclose(g_in);

    /* ---- workspace (HipDecoder._alloc) */
    const int T = P + max_new, Ld = T + NCB, seq_len = Lc + T + NCB;
    const int smax = (seq_len + 255) / 256 * 256, S = Lc + P + 1, Mp = R * S;
    const int small = R <= 16 && D == 2048;
    const int sq = split_for(Nqkv, D, R, 256), so = split_for(D, H * hd, R, 128), sf = split_for(D, Fd, R, 256);
    int want = (512 + R * Hk - 1) / (R * Hk), cap = (smax + 2047) / 2048, asplit = smax / 128;
    asplit = want < asplit ? want : asplit;
    asplit = cap < asplit ? cap : asplit;
    if (asplit < 1) asplit = 1;
    int merge = 0;
    if (R <= 2) {
        const int n = 4 < smax / 128 ? 4 : smax / 128;
        merge = n >= 8 ? 8 : n >= 4 ? 4 : n >= 2 ? 2 : 0;
    }
    size_t part_n = (size_t)Mp * Nqkv;
    const size_t cand[5] = {(size_t)Mp * D, (size_t)sq * R * Nqkv, (size_t)so * R * D, (size_t)sf * R * D,
                            (size_t)R * NCB * VOCAB};
    for (int i = 0; i < 5; ++i) part_n = cand[i] > part_n ? cand[i] : part_n;
    const size_t kv_layer = (size_t)R * Hk * smax * hd * 2;
    for (int i = 0; i < NL; ++i) {
        layers[i].k_cache = dzero(kv_layer);
        layers[i].vt_cache = dzero(kv_layer);
    }
    const int wsplit = asplit > merge ? asplit : merge;
    zk_step_desc d;
    memset(&d, 0, sizeof d);
    d.B = B; d.n_layer = NL; d.d_model = D; d.n_heads = H; d.n_kv = Hk; d.head_dim = hd; d.d_ff = Fd; d.smax = smax;
    d.split_qkv = sq; d.split_o = so; d.split_fc2 = sf; d.split_heads = 1;
    d.attn_splits = asplit; d.attn_merge = merge; d.rope_neox = 0; d.small = small; d.eps = fp[0];
    d.layers = layers;   /* host array: zk_decode_step walks it on the host while enqueueing */
    d.emb = emb; d.heads = heads; d.lnf_w = lnf_w; d.lnf_b = lnf_b; d.freqs = freqs;
    d.x = dalloc((size_t)Mp * D * 2);
    d.xn = dalloc((size_t)Mp * D * 2);
    d.y = dalloc((size_t)Mp * H * hd * 2);
    d.h = dalloc((size_t)Mp * Fd * 2);
    d.part = (float*)dalloc(part_n * 4);
    d.attn_work = (float*)dalloc((size_t)R * Hk * wsplit * (8 + 4 * hd) * 4);
    d.attn_cnt = (uint32_t*)dzero((size_t)R * Hk * 4);
    d.dbg = NULL;
    void* q = dalloc((size_t)Mp * H * hd * 2);
    /* generation state (zk_gen_state) */
    int32_t* scal = (int32_t*)dzero(16 * 4);
    d.st.scal = scal;
    d.st.eos_mode = (int32_t*)dzero((size_t)B * 4);
    d.st.steps_after = (int32_t*)dzero((size_t)B * 4);
    d.st.remaining = (int32_t*)dzero((size_t)B * 4);
    d.st.stopping = (int32_t*)dzero((size_t)B * 4);
    d.st.act = (int32_t*)dzero((size_t)B * 4);
    d.st.rp = (float*)dzero((size_t)B * 4);
    d.st.tok0 = (int32_t*)dzero((size_t)B * NCB * 4);
    d.st.tok1 = (int32_t*)dzero((size_t)B * NCB * 4);
    d.st.delayed = (int64_t*)dalloc((size_t)B * NCB * Ld * 8);
    d.st.B = B; d.st.K = NCB; d.st.Ld = Ld; d.st.V = VOCAB; d.st.seed = seed; d.st.row_base = 0;
    d.st.noise_mode = hdr[14]; d.st.noise_offset = noise_off; d.st.noise_stride = hdr[15];
    d.st.noise_incr = (int32_t)noise_incr;
    d.sp.cfg_scale = fp[1]; d.sp.temperature = fp[2]; d.sp.top_p = fp[3]; d.sp.min_p = fp[4];
    d.sp.linear = fp[5]; d.sp.conf = fp[6]; d.sp.quad = fp[7]; d.sp.top_k = hdr[13]; d.sp.rp_window = hdr[12];
    d.sp.force_full_length = 0;

    /* ---- codes -> delayed codes (model.py:288-295) */
    int64_t* codes_h = (int64_t*)malloc((size_t)B * NCB * T * 8);
    for (int b = 0; b < B; ++b)
        for (int k = 0; k < NCB; ++k)
            for (int t = 0; t < T; ++t)
                codes_h[((size_t)b * NCB + k) * T + t] = t < P ? prefix_h[((size_t)b * NCB + k) * P + t] : -1;
    int64_t* codes_d = (int64_t*)dalloc((size_t)B * NCB * T * 8);
    HIP(hipMemcpy(codes_d, codes_h, (size_t)B * NCB * T * 8, hipMemcpyHostToDevice));
    ZK(zk_delay_apply(codes_d, B, NCB, T, MASK_ID, d.st.delayed, s));

    /* ---- prefill (model.py:297-319) */
    ZK(zk_prefill(&d, cond, Lc, P, q, s));
    /* ---- loop state (model.py:316-342) */
    const int max_steps = Ld - (P + 1);
    int32_t sc[16] = {P + 2, S, 1, 0, 0, max_steps, 0};
    HIP(hipMemcpyAsync(scal, sc, sizeof sc, hipMemcpyHostToDevice, s));
    int32_t* six = (int32_t*)malloc((size_t)B * 4);
    int32_t* rem = (int32_t*)malloc((size_t)B * 4);
    float* rps = (float*)malloc((size_t)B * 4);
    for (int b = 0; b < B; ++b) { six[b] = 6; rem[b] = max_steps; rps[b] = rp; }
    HIP(hipMemcpyAsync(d.st.steps_after, six, (size_t)B * 4, hipMemcpyHostToDevice, s));
    HIP(hipMemcpyAsync(d.st.remaining, rem, (size_t)B * 4, hipMemcpyHostToDevice, s));
    HIP(hipMemcpyAsync(d.st.rp, rps, (size_t)B * 4, hipMemcpyHostToDevice, s));
    HIP(hipStreamSynchronize(s));

    /* ---- decode loop (model.py:345-432): one step captured once, replayed in chunks */
    hipStream_t cs;
    HIP(hipStreamCreate(&cs));
    void* graph = NULL;
    ZK(zk_graph_begin(cs));
    if (zk_decode_step(&d, cs) != 0) die("zk_decode_step (capture)");
    ZK(zk_graph_end(cs, &graph));
    int done_steps = 0;
    for (;;) {
        int n = max_steps - done_steps < poll_every ? max_steps - done_steps : poll_every;
        if (n <= 0) break;
        ZK(zk_graph_launch(graph, n, cs));
        done_steps += n;
        HIP(hipMemcpyAsync(sc, scal, sizeof sc, hipMemcpyDeviceToHost, cs));
        HIP(hipStreamSynchronize(cs));
        if (sc[3]) break;
    }
    ZK(zk_graph_destroy(graph));
    const int offset = sc[0] - 1;

    /* ---- output trim (model.py:437-457) */
    const int Tr = Ld - NCB;
    int64_t* rev_d = (int64_t*)dalloc((size_t)B * NCB * Tr * 8);
    ZK(zk_delay_revert(d.st.delayed, B, NCB, Ld, rev_d, cs));
    int64_t* rev = (int64_t*)malloc((size_t)B * NCB * Tr * 8);
    HIP(hipMemcpyAsync(rev, rev_d, (size_t)B * NCB * Tr * 8, hipMemcpyDeviceToHost, cs));
    HIP(hipStreamSynchronize(cs));
    FILE* fo = fopen(argv[2], "wb");
    if (!fo) { perror(argv[2]); return 2; }
    int32_t nb = B;
    fwrite(&nb, 4, 1, fo);
    const int keep = offset - NCB;
    for (int b = 0; b < B; ++b) {
        int eos = Tr;                          /* first EOS in codebook 0 (argmax; 0 = none), else all */
        for (int t = 0; t < Tr; ++t)
            if (rev[(size_t)b * NCB * Tr + t] == EOS_ID) { eos = t ? t : Tr; break; }
        int end = eos < keep ? eos : keep;
        int32_t len = end > P ? end - P : 0;
        fwrite(&len, 4, 1, fo);
        for (int k = 0; k < NCB; ++k)
            for (int t = P; t < P + len; ++t) {
                int64_t v = rev[((size_t)b * NCB + k) * Tr + t];
                if (v >= 1024) v = 0;           /* out[out >= 1024] = 0 */
                fwrite(&v, 8, 1, fo);
            }
    }
    fclose(fo);
    printf("generate: B=%d, %d decode steps, offset %d, sampler calls %d\n", B, done_steps, offset, sc[2] + sc[4]);
    return 0;
}
