// Sampler, EOS protocol and delay-pattern kernels for gfx950.
//
// One 256-thread workgroup per (utterance, codebook) row of 1026 logits: every value
// lives in registers (5 per lane), reductions are wave64 shuffles + one LDS hop, the
// top-p/top-k sorts are a 2048-entry bitonic sort in LDS. The whole step -- CFG
// combine of the heads GEMM slabs, logit bias, EOS hold-off mask, repetition penalty,
// temperature softmax, unified/top-p/top-k/min-p shaping and the exponential race --
// is one launch, so the decode step has no host synchronisation (the reference syncs
// at model.py:345,380,410-414).
//
// Reference: zonos/sampling.py:11-33,54-128,131-169,232-328; zonos/model.py:103-116,
// 322-424; zonos/codebook_pattern.py:5-12.
#include "common.h"
#include "../../include/zonos_hip.h"

namespace {

constexpr int NT = 256;
constexpr int NPT = 5;          // values per lane: V <= 1280
constexpr int SORTN = 2048;
constexpr int MAXW = 512;       // repetition-penalty window held in LDS
constexpr int EOS = 1024, MASK = 1025;
constexpr int EOS_MAXK = 16;    // codebooks handled by k_eos_step's unrolled frame write
// float32(log(1024)) as torch computes it (model.py:324)
constexpr float LOG1024F = 6.931471824645996f;

// ------------------------------------------------------------------ Philox4x32-10
ZK_DEV uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

ZK_DEV uint32_t philox_w0(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return c0;
}

// Exp(1) sample; identical definition in oracle/philox.py.
ZK_DEV float exp_noise(uint64_t seed, int step, int draw, int row, int cb, int v) {
    const uint32_t x = philox_w0((uint32_t)v, (uint32_t)row * 16u + (uint32_t)cb, (uint32_t)step,
                                 (uint32_t)draw, (uint32_t)seed, (uint32_t)(seed >> 32));
    const double u = ((double)(x >> 8) + 0.5) * (1.0 / 16777216.0);
    return (float)(-log(u));
}

// All four Philox4x32-10 output words (the same rounds as philox_w0).
ZK_DEV uint4 philox4(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return uint4{c0, c1, c2, c3};
}

// Element e of torch's GPU `Tensor.exponential_(1)` over a tensor whose call took Philox
// (seed, offset) and ran with grid-stride `stride` (oracle/torch_philox.py; torch 2.10
// ATen/native/hip/DistributionTemplates.h:52-91, rocrand_philox4x32_10.h, rocrand_uniform.h:66-68,
// ATen/core/TransformationHelper.h:129-146): thread t = e % stride of iteration j = (e / stride) / 4
// draws Philox(counter (offset / 4 + j, t), key seed) and takes word (e / stride) % 4.
ZK_DEV float torch_exp_noise(uint64_t seed, uint64_t offset, long e, int stride) {
    const long t = e % stride, q = e / stride;
    const uint64_t ctr = offset / 4 + (uint64_t)(q >> 2);
    const uint4 r = philox4((uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)t, (uint32_t)(t >> 32), (uint32_t)seed,
                            (uint32_t)(seed >> 32));
    const int ii = (int)(q & 3);
    const uint32_t w = ii == 0 ? r.x : ii == 1 ? r.y : ii == 2 ? r.z : r.w;
    const float u = 2.3283064e-10f + (float)w * 2.3283064e-10f;       // hiprand_uniform4: (0, 1]
    // torch: log = u >= 1 - eps/2 ? -eps/2 : __logf(u) (ATen/NumericUtils.h:150-160); q = -1 / 1 * log.
    // torch's __logf is the hardware log2 (v_log_f32) times ln2 in extended precision (ln2 split
    // into float hi + lo, one fma): bit-identical to torch on 1.2 M probed values, where a plain
    // float multiply by ln2 differs in 3 % and this clang's __builtin_logf in 33 % of them
    // (tools/torch_noise_probe.py, profiles/r5_torch_noise_probe.txt)
    const float y = __builtin_amdgcn_logf(u);
    const float ln = __builtin_fmaf(y, __builtin_bit_cast(float, 0x3f317218u), y * __builtin_bit_cast(float, 0xb102e308u));
    const float lg = u >= 1.0f - 5.96046448e-08f ? -5.96046448e-08f : ln;
    return -1.0f * lg;
}

struct Smem {
    float key[SORTN];
    int idx[SORTN];
    float pv[SORTN];
    double dred[NT / 64];
    float red[NT / 64];
    int ired[NT / 64];
    int win[MAXW];
    int flag;
};

ZK_DEV bool before(float a, int ia, float b, int ib) { return a > b || (a == b && ia < ib); }

// Bitonic sort of smem.key/idx (SORTN entries) into descending key order, ties by index.
ZK_DEV void sort_desc(Smem& s) {
    for (int k = 2; k <= SORTN; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < SORTN; i += NT) {
                const int p = i ^ j;
                if (p > i) {
                    const float a = s.key[i], b = s.key[p];
                    const int ia = s.idx[i], ib = s.idx[p];
                    const bool up = (i & k) == 0;
                    if (up ? !before(a, ia, b, ib) : before(a, ia, b, ib)) {
                        s.key[i] = b; s.key[p] = a; s.idx[i] = ib; s.idx[p] = ia;
                    }
                }
            }
            __syncthreads();
        }
    }
}

ZK_DEV void fill_sort(Smem& s, const float* p, int V) {
#pragma unroll
    for (int i = 0; i < SORTN / NT; ++i) {
        const int v = threadIdx.x + NT * i;
        float val = -1.f;
        if (i < NPT && v < V) val = p[i];
        s.key[v] = val;
        s.idx[v] = v;
    }
    __syncthreads();
}

ZK_DEV void renorm(float* p, int V, Smem& s) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NPT; ++i) if (threadIdx.x + NT * i < V) t += p[i];
    const float sum = block_sum<NT>(t, s.red);
#pragma unroll
    for (int i = 0; i < NPT; ++i) p[i] = __fdiv_rn(p[i], sum);
}

// In-block softmax over the V values held in x (sampling.py:298, 75).
ZK_DEV void softmax(float* x, int V, Smem& s) {
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < NPT; ++i) if (threadIdx.x + NT * i < V) m = fmaxf(m, x[i]);
    m = block_max<NT>(m, s.red);
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        const bool ok = threadIdx.x + NT * i < V;
        x[i] = ok ? expf(__fsub_rn(x[i], m)) : 0.f;
        t += x[i];
    }
    const float sum = block_sum<NT>(t, s.red);
#pragma unroll
    for (int i = 0; i < NPT; ++i) x[i] = __fdiv_rn(x[i], sum);
}

// Block argmax, first index on ties (torch.argmax semantics).
ZK_DEV int block_argmax(const float* x, int V, Smem& s) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        const int v = threadIdx.x + NT * i;
        if (v < V && before(x[i], v, bv, bi)) { bv = x[i]; bi = v; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (before(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) { s.red[w] = bv; s.ired[w] = bi; }
    __syncthreads();
    bv = s.red[0]; bi = s.ired[0];
#pragma unroll
    for (int i = 1; i < NT / 64; ++i)
        if (before(s.red[i], s.ired[i], bv, bi)) { bv = s.red[i]; bi = s.ired[i]; }
    return bi;
}

// apply_top_p (sampling.py:96-111): sort desc, cumsum (torch CPU accumulates float cumsum
// in double), zero where cumsum - p > top_p, scatter back, renormalise.
ZK_DEV void top_p_filter(float* p, int V, float top_p, Smem& s) {
    fill_sort(s, p, V);
    sort_desc(s);
    constexpr int SEG = (SORTN + NT - 1) / NT;   // 8 sorted entries per lane (contiguous)
    const int base = threadIdx.x * SEG;
    double loc = 0.0;
#pragma unroll
    for (int j = 0; j < SEG; ++j) if (base + j < V) loc += (double)s.key[base + j];
    // exclusive scan of `loc` over the block
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double inc = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) s.dred[w] = inc;
    __syncthreads();
    double pre = 0.0;
    for (int i = 0; i < w; ++i) pre += s.dred[i];
    double run = pre + inc - loc;
#pragma unroll
    for (int j = 0; j < SEG; ++j) {
        const int i = base + j;
        if (i < V) {
            run += (double)s.key[i];
            const float cs = (float)run;
            const float ps = s.key[i];
            s.pv[s.idx[i]] = (__fsub_rn(cs, ps) > top_p) ? 0.f : ps;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        const int v = threadIdx.x + NT * i;
        p[i] = v < V ? s.pv[v] : 0.f;
    }
    __syncthreads();
    renorm(p, V, s);
}

// apply_top_k (sampling.py:77-93): pivot = k-th largest, zero everything below, renormalise.
ZK_DEV void top_k_filter(float* p, int V, int k, Smem& s) {
    fill_sort(s, p, V);
    sort_desc(s);
    const float pivot = s.key[min(k, V) - 1];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NPT; ++i) if (p[i] < pivot) p[i] = 0.f;
    renorm(p, V, s);
}

struct RowCtx {
    int b, k, V;
    const int64_t* gen;   // token history row (delayed codes) or nullptr
    int gen_len;          // columns [0, gen_len) are history
    float rp;
    int step, draw, row;
    uint64_t seed;
    // torch noise mode (nstride > 0): torch's exponential_ stream of the call at Philox offset
    // `noff`, this row's elements starting at `ebase` of the [B][K][V] noise tensor
    uint64_t noff;
    int nstride;
    long ebase;
};

// Everything after the logits are in registers: rep-penalty, shaping, race / argmax.
// TN: the noise is torch's stream (c.noff, c.nstride, c.ebase), else the keyed one -- a template
// argument, so neither sampler carries the other's branch (a runtime test cost 2-3 us per B = 1 step,
// profiles/r5_torch_noise_branch_ab.txt)
template <bool TN>
ZK_DEV int sample_row(float* x, const RowCtx& c, const zk_sampling_params& sp, Smem& s) {
    const int V = c.V;
    // ---- repetition penalty (sampling.py:142-169); rp == 1 is an exact identity
    if (c.gen != nullptr && sp.rp_window > 0) {
        const int W = min(min(sp.rp_window, c.gen_len), MAXW);
        const int j0 = c.gen_len - W;
        for (int j = threadIdx.x; j < W; j += NT) {
            const int64_t t = c.gen[j0 + j];
            s.win[j] = (int)(t > V - 1 ? V - 1 : t);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NPT; ++i) {
            const int v = threadIdx.x + NT * i;
            float f = 1.f;
            for (int j = 0; j < W; ++j) if (s.win[j] == v) f = __fmul_rn(f, c.rp);
            x[i] = (x[i] <= 0.f) ? __fmul_rn(x[i], f) : __fdiv_rn(x[i], f);
        }
        __syncthreads();
    }
    if (!(sp.temperature > 0.f)) return block_argmax(x, V, s);   // sampling.py:325-326

#pragma unroll
    for (int i = 0; i < NPT; ++i) x[i] = __fdiv_rn(x[i], sp.temperature);
    softmax(x, V, s);
    if (sp.linear > 0.f) {   // apply_unified (sampling.py:54-75)
        float lp[NPT];
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < NPT; ++i) {
            const bool ok = threadIdx.x + NT * i < V;
            lp[i] = logf(fmaxf(x[i], 1e-20f));
            if (ok) t += __fmul_rn(x[i], lp[i]);
        }
        const float ent = -block_sum<NT>(t, s.red);
        const float scale = __fadd_rn(sp.linear, __fmul_rn(ent, sp.conf));
#pragma unroll
        for (int i = 0; i < NPT; ++i)
            x[i] = __fsub_rn(__fmul_rn(lp[i], scale), __fmul_rn(__fmul_rn(lp[i], lp[i]), sp.quad));
        softmax(x, V, s);
    }
    if (sp.top_p > 0.f) top_p_filter(x, V, sp.top_p, s);
    if (sp.top_k > 0) top_k_filter(x, V, sp.top_k, s);
    if (sp.min_p > 0.f) {    // apply_min_p (sampling.py:114-128)
        float m = 0.f;
#pragma unroll
        for (int i = 0; i < NPT; ++i) if (threadIdx.x + NT * i < V) m = fmaxf(m, x[i]);
        m = block_max<NT>(m, s.red);
        const float thr = __fmul_rn(sp.min_p, m);
#pragma unroll
        for (int i = 0; i < NPT; ++i) if (x[i] < thr) x[i] = 0.f;
        renorm(x, V, s);
    }
    // exponential race (sampling.py:26-28)
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        const int v = threadIdx.x + NT * i;
        if (v < V)
            x[i] = __fdiv_rn(x[i], TN ? torch_exp_noise(c.seed, c.noff, c.ebase + v, c.nstride)
                                      : exp_noise(c.seed, c.step, c.draw, c.row, c.k, v));
    }
    return block_argmax(x, V, s);
}

template <bool TN>
__global__ __launch_bounds__(NT) void k_sample_logits(const float* logits, int B, int K, int V,
                                                      const int64_t* gen, int gen_stride, int gen_len,
                                                      const float* rp, zk_sampling_params sp, uint64_t seed,
                                                      int step, int draw, int row_base, uint64_t noff, int nstride,
                                                      int64_t* out) {
    __shared__ Smem s;
    const int b = blockIdx.x / K, k = blockIdx.x % K;
    float x[NPT];
    const float* row = logits + ((size_t)b * K + k) * V;
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        const int v = threadIdx.x + NT * i;
        x[i] = v < V ? row[v] : -INFINITY;
    }
    RowCtx c{b, k, V, gen ? gen + ((size_t)b * K + k) * gen_stride : nullptr, gen_len,
             rp ? rp[b] : 1.f, step, draw, row_base + b, seed, noff, nstride, ((long)b * K + k) * V};
    const int t = sample_row<TN>(x, c, sp, s);
    if (threadIdx.x == 0) out[(size_t)b * K + k] = t;
}

// Engine sampler: CFG-combine the heads GEMM slabs, bias, EOS masks, sample.
template <bool TN>
__global__ __launch_bounds__(NT) void k_sample_heads(const float* part, int nsplit, zk_gen_state st,
                                                     zk_sampling_params sp, int prefill, int draw,
                                                     float* dbg) {
    __shared__ Smem s;
    const int B = st.B, K = st.K, V = st.V;
    const int b = blockIdx.x / K, k = blockIdx.x % K;
    const int32_t* scal = st.scal;
    // Every load that does not depend on another one is issued up front (one memory round trip):
    // the done word, the step scalars, this row's state and the logits; the finished check comes
    // after them (the loads are in bounds either way).
    const int done = scal[3];
    const int offset = scal[0], step = scal[2], nres = scal[4];
    const float rpb = st.rp[b];
    const int actb = st.act[b];
    int new_eos_b = 0;
    if (draw == 1) {   // EOS resample happens only if some row has a new EOS (model.py:380)
        int any = 0;   // one row per thread
        for (int r = threadIdx.x; r < B; r += NT) any |= (st.tok0[r * K] == EOS) && !st.eos_mode[r];
        if (!__syncthreads_or(any && !done)) return;
        new_eos_b = (st.tok0[b * K] == EOS) && !st.eos_mode[b];
    }
    const size_t N = (size_t)K * V;
    const size_t slab = (size_t)2 * B * N;
    const float* pc = part + (size_t)b * N + (size_t)k * V;
    const float* pu = part + (size_t)(b + B) * N + (size_t)k * V;
    float x[NPT];
    if (nsplit == 1) {     // the unsplit heads GEMM (c3, B <= 8): all 2 x NPT loads before the first use
        float c1[NPT], u1[NPT];
#pragma unroll
        for (int i = 0; i < NPT; ++i) {
            const int v = min(threadIdx.x + NT * i, V - 1);
            c1[i] = pc[v];
            u1[i] = pu[v];
        }
#pragma unroll
        for (int i = 0; i < NPT; ++i) {
            const int v = threadIdx.x + NT * i;
            float val = -INFINITY;
            if (v < V) {
                const float c = round_bf(0.f + c1[i]), u = round_bf(0.f + u1[i]);   // head output bf16 (model.py:111)
                val = __fadd_rn(u, __fmul_rn(__fsub_rn(c, u), sp.cfg_scale));       // model.py:114
                if (v >= 1025) val = -INFINITY;                                    // model.py:115
            }
            x[i] = val;
        }
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        if (nsplit == 1) break;
        const int v = threadIdx.x + NT * i;
        float val = -INFINITY;
        if (v < V) {
            float c = 0.f, u = 0.f;
            for (int sp_ = 0; sp_ < nsplit; ++sp_) { c += pc[sp_ * slab + v]; u += pu[sp_ * slab + v]; }
            c = round_bf(c); u = round_bf(u);                              // head output bf16 (model.py:111)
            val = __fadd_rn(u, __fmul_rn(__fsub_rn(c, u), sp.cfg_scale)); // model.py:114
            if (v >= 1025) val = -INFINITY;                                // model.py:115
        }
        x[i] = val;
    }
    if (done) return;                                       // generation finished
    if (dbg != nullptr && draw == 0) {
        float* d = dbg + ((size_t)b * K + k) * V;
#pragma unroll
        for (int i = 0; i < NPT; ++i) { const int v = threadIdx.x + NT * i; if (v < V) d[v] = x[i]; }
    }
    // bias + EOS masks for the EOS column only (threads owning v == EOS)
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        const int v = threadIdx.x + NT * i;
        if (v == EOS) {
            if (!prefill) {
                if (k >= 1) x[i] = -INFINITY;                                  // model.py:323
                else x[i] = __fadd_rn(x[i], 0.0f - LOG1024F);                  // model.py:324,353
                if (k == 0 && actb) x[i] = -INFINITY;                          // model.py:360-361
                if (k == 0 && new_eos_b) x[i] = -INFINITY;                     // model.py:387
            }
            if (k == 0 && sp.force_full_length) x[i] = -INFINITY;              // benchmark mode
        }
    }
    // torch noise mode: the reference's sampler calls so far -- the prefill sample, one per earlier
    // decode step (scal[2] starts at 1) and one per earlier EOS resample (scal[4]) -- each took
    // noise_incr of the generator's Philox offset (model.py:304,365,388)
    const long call = prefill ? 0 : (long)step + nres + draw;
    RowCtx c{b, k, V, prefill ? nullptr : st.delayed + ((size_t)b * K + k) * st.Ld, offset,
             prefill ? 1.f : rpb, prefill ? 0 : step, draw, st.row_base + b, st.seed,
             st.noise_offset + (uint64_t)call * (uint64_t)st.noise_incr, st.noise_mode ? st.noise_stride : 0,
             ((long)(st.row_base + b) * K + k) * V};
    const int t = sample_row<TN>(x, c, sp, s);
    if (threadIdx.x == 0) (draw ? st.tok1 : st.tok0)[b * K + k] = t;
}

// EOS protocol, frame write and step counters (model.py:376-424), one workgroup.
__global__ __launch_bounds__(NT) void k_eos_step(zk_gen_state st, int prefill, int prefix_len) {
    __shared__ int s_any, s_max;
    const int B = st.B, K = st.K, Ld = st.Ld;
    int32_t* scal = st.scal;
    if (prefill) {   // model.py:310-314: first frame, no EOS logic
        for (int i = threadIdx.x; i < B * K; i += NT) {
            int64_t* d = st.delayed + (size_t)i * Ld + prefix_len;
            if (*d == -1) *d = st.tok0[i];
        }
        return;
    }
    if (scal[3]) return;
    if (threadIdx.x == 0) { s_any = 0; s_max = -0x7fffffff; }
    __syncthreads();
    for (int b = threadIdx.x; b < B; b += NT)
        if (st.tok0[b * K] == EOS && !st.eos_mode[b]) atomicOr(&s_any, 1);
    __syncthreads();
    const int any = s_any;
    const int offset = scal[0];
    for (int b = threadIdx.x; b < B; b += NT) {
        const int newe = (st.tok0[b * K] == EOS) && !st.eos_mode[b];
        const int32_t* tok = (any ? st.tok1 : st.tok0) + b * K;
        if (newe) { st.eos_mode[b] = 1; st.steps_after[b] = 6; }          // model.py:383-384
        int rem = st.remaining[b];
        if (tok[0] == EOS) { rem = min(rem, 9); st.stopping[b] = 1; }      // model.py:399-402
        const int stop = st.stopping[b];
        const int idx = min(9 - rem, K - 1);                               // model.py:405-406
        if (offset < Ld) {       // the reference's last iteration writes an empty slice
            // all K frame cells and tokens loaded before the first store (one round trip)
            int64_t cur[EOS_MAXK];
            int tv[EOS_MAXK];
#pragma unroll
            for (int k = 0; k < EOS_MAXK; ++k)
                if (k < K) {
                    cur[k] = st.delayed[((size_t)b * K + k) * Ld + offset];
                    tv[k] = tok[k];
                }
#pragma unroll
            for (int k = 0; k < EOS_MAXK; ++k) {
                if (k >= K) break;
                int v = tv[k];
                if (stop) v = k < idx ? MASK : (k == idx ? EOS : v);       // model.py:410-414
                if (cur[k] == -1) st.delayed[((size_t)b * K + k) * Ld + offset] = v;   // model.py:417-418
            }
        }
        rem -= 1;                                                          // model.py:424
        st.remaining[b] = rem;
        atomicMax(&s_max, rem);
        // prepare the next step (model.py:356,360-362 run at the top of the next iteration)
        const int em = st.eos_mode[b];
        if (em) st.rp[b] = 1.0f;
        const int a = em && st.steps_after[b] > 0;
        st.act[b] = a;
        if (a) st.steps_after[b] -= 1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        scal[0] = offset + 1;
        scal[1] += 1;
        scal[2] += 1;
        if (s_max <= 0 || offset >= Ld) scal[3] = 1;
        if (any) scal[4] += 1;
    }
}

__global__ void k_delay_apply(const int64_t* codes, int B, int K, int T, int64_t mask, int64_t* out) {
    const int L = T + K;
    const size_t n = (size_t)B * K * L;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int t = (int)(i % L);
        const size_t bk = i / L;
        const int k = (int)(bk % K);
        const int src = t - k - 1;
        out[i] = (src >= 0 && src < T) ? codes[bk * T + src] : mask;
    }
}

__global__ void k_delay_revert(const int64_t* d, int B, int K, int L, int64_t* out) {
    const int T = L - K;
    const size_t n = (size_t)B * K * T;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int t = (int)(i % T);
        const size_t bk = i / T;
        const int k = (int)(bk % K);
        out[i] = d[bk * L + t + k + 1];
    }
}

}  // namespace

extern "C" int zk_sample_logits(const float* logits, int B, int K, int V, const int64_t* generated,
                                int gen_stride, int gen_len, const float* rp, const zk_sampling_params* sp,
                                uint64_t seed, int step, int draw, int row_base, int64_t* out, void* stream) {
    ZK_REQUIRE(V > 0 && V <= NT * NPT, "zk_sample_logits: V=%d must be in (0, %d]", V, NT * NPT);
    ZK_REQUIRE(B > 0 && K > 0, "zk_sample_logits: empty batch");
    ZK_REQUIRE(sp != nullptr, "zk_sample_logits: null params");
    ZK_REQUIRE(sp->top_k >= 0 && sp->rp_window >= 0, "zk_sample_logits: negative top_k/window");
    hipLaunchKernelGGL(k_sample_logits<false>, dim3(B * K), dim3(NT), 0, (hipStream_t)stream, logits, B, K, V,
                       generated, gen_stride, gen_len, rp, *sp, seed, step, draw, row_base, (uint64_t)0, 0, out);
    ZK_CHECK_LAUNCH("zk_sample_logits");
    return 0;
}

extern "C" int zk_sample_logits_torch(const float* logits, int B, int K, int V, const int64_t* generated,
                                      int gen_stride, int gen_len, const float* rp, const zk_sampling_params* sp,
                                      uint64_t seed, uint64_t offset, int stride, int64_t* out, void* stream) {
    ZK_REQUIRE(V > 0 && V <= NT * NPT, "zk_sample_logits_torch: V=%d must be in (0, %d]", V, NT * NPT);
    ZK_REQUIRE(B > 0 && K > 0, "zk_sample_logits_torch: empty batch");
    ZK_REQUIRE(sp != nullptr, "zk_sample_logits_torch: null params");
    ZK_REQUIRE(sp->top_k >= 0 && sp->rp_window >= 0, "zk_sample_logits_torch: negative top_k/window");
    ZK_REQUIRE(stride > 0 && stride % 256 == 0, "zk_sample_logits_torch: stride %d (256 x grid)", stride);
    hipLaunchKernelGGL(k_sample_logits<true>, dim3(B * K), dim3(NT), 0, (hipStream_t)stream, logits, B, K, V,
                       generated, gen_stride, gen_len, rp, *sp, seed, 0, 0, 0, offset, stride, out);
    ZK_CHECK_LAUNCH("zk_sample_logits_torch");
    return 0;
}

namespace {
__global__ void k_torch_exponential(float* out, long n, uint64_t seed, uint64_t offset, int stride) {
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x)
        out[e] = torch_exp_noise(seed, offset, e, stride);
}
}  // namespace

extern "C" int zk_torch_exponential(float* out, long n, uint64_t seed, uint64_t offset, int stride, void* stream) {
    ZK_REQUIRE(n >= 0 && out != nullptr, "zk_torch_exponential: bad output");
    ZK_REQUIRE(stride > 0 && stride % 256 == 0, "zk_torch_exponential: stride %d (256 x grid)", stride);
    if (n == 0) return 0;
    const int grid = (int)std::min<long>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_torch_exponential, dim3(grid), dim3(256), 0, (hipStream_t)stream, out, n, seed, offset,
                       stride);
    ZK_CHECK_LAUNCH("zk_torch_exponential");
    return 0;
}

extern "C" int zk_torch_noise_policy(long n, int mp_count, int max_threads_per_mp, int* stride, long* incr) {
    ZK_REQUIRE(n > 0 && mp_count > 0 && max_threads_per_mp >= 256 && stride && incr,
               "zk_torch_noise_policy: n=%ld mp=%d max_threads=%d", n, mp_count, max_threads_per_mp);
    const long grid = std::min<long>((long)mp_count * (max_threads_per_mp / 256), (n + 255) / 256);
    *stride = (int)(256 * grid);
    *incr = ((n - 1) / (256 * grid * 4) + 1) * 4;
    return 0;
}

extern "C" int zk_sample_heads(const float* part, int nsplit, const zk_gen_state* st,
                               const zk_sampling_params* sp, int prefill, int draw, float* dbg_logits,
                               void* stream) {
    ZK_REQUIRE(st && sp && part, "zk_sample_heads: null argument");
    ZK_REQUIRE(st->V > 0 && st->V <= NT * NPT, "zk_sample_heads: V=%d unsupported", st->V);
    ZK_REQUIRE(!st->noise_mode || (st->noise_stride > 0 && st->noise_stride % 256 == 0 && st->noise_incr > 0),
               "zk_sample_heads: torch noise needs a stride (256 x grid) and an increment (zk_torch_noise_policy)");
    auto kern = st->noise_mode ? k_sample_heads<true> : k_sample_heads<false>;
    hipLaunchKernelGGL(kern, dim3(st->B * st->K), dim3(NT), 0, (hipStream_t)stream, part, nsplit, *st, *sp, prefill,
                       draw, dbg_logits);
    ZK_CHECK_LAUNCH("zk_sample_heads");
    return 0;
}

extern "C" int zk_eos_step(const zk_gen_state* st, int prefill, int prefix_len, void* stream) {
    ZK_REQUIRE(st != nullptr, "zk_eos_step: null state");
    ZK_REQUIRE(st->K <= EOS_MAXK, "zk_eos_step: K=%d codebooks > %d", st->K, EOS_MAXK);
    hipLaunchKernelGGL(k_eos_step, dim3(1), dim3(NT), 0, (hipStream_t)stream, *st, prefill, prefix_len);
    ZK_CHECK_LAUNCH("zk_eos_step");
    return 0;
}

extern "C" int zk_delay_apply(const int64_t* codes, int B, int K, int T, int64_t mask_token, int64_t* delayed,
                              void* stream) {
    ZK_REQUIRE(B >= 0 && K > 0 && T >= 0, "zk_delay_apply: bad shape");
    const size_t n = (size_t)B * K * (T + K);
    if (n == 0) return 0;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_delay_apply, dim3(grid), dim3(256), 0, (hipStream_t)stream, codes, B, K, T, mask_token,
                       delayed);
    ZK_CHECK_LAUNCH("zk_delay_apply");
    return 0;
}

extern "C" int zk_delay_revert(const int64_t* delayed, int B, int K, int L, int64_t* codes, void* stream) {
    ZK_REQUIRE(B >= 0 && K > 0 && L >= K, "zk_delay_revert: bad shape");
    const size_t n = (size_t)B * K * (L - K);
    if (n == 0) return 0;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_delay_revert, dim3(grid), dim3(256), 0, (hipStream_t)stream, delayed, B, K, L, codes);
    ZK_CHECK_LAUNCH("zk_delay_revert");
    return 0;
}
