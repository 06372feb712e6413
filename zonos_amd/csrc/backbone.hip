// Transformer backbone step kernels for gfx950 (zonos/backbone/_torch.py restated).
//
//   k_embed_ln   : sum of 9 codebook embeddings (bf16 left-to-right adds, model.py:97-98),
//                  duplicated for the CFG rows (model.py:141) + layer-0 LayerNorm.
//   k_resid_ln   : split-K slab reduction of the preceding projection + residual add
//                  (bf16, _torch.py:100-101) + the next LayerNorm, one pass over the row.
//   k_qkv_rope   : in_proj slab reduction -> bf16 -> interleaved RoPE (_torch.py:18-30)
//                  -> q buffer + KV cache store (_torch.py:33-49).
//   k_attn_decode: split-KV GQA decode attention on MFMA 16x16x32 bf16 (K on the A side,
//                  the 4 query heads of a KV head on the B side), k_attn_combine merges splits.
//   k_attn_prefill: causal prefill attention on MFMA (16 queries per wave, two passes).
//
// KV cache layout: see "KV cache layout" below (32-key slices in MFMA-fragment order).
#include "common.h"
#include "../../include/zonos_hip.h"
#include <algorithm>
#include <stdlib.h>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

ZK_DEV bf16x8 as_frag(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

// ------------------------------------------------------------------ KV cache layout
// Per (row, kv head) the cache holds Smax keys in 32-key slices of 8 KB. Inside a slice the
// data is stored in exactly the order the decode wave's MFMA fragments consume it, so every
// fragment load is one contiguous 1 KB read:
//   K: [slice][h 2][ks 4][lane 64][8]  lane = 16*lg + ln holds key 8*(ln>>2) + 4h + (ln&3)
//      of the slice, dims 32ks + 8lg .. +8          (A operand of S^T = K.Q^T)
//   V: [slice][dt 8][lane 64][8]       lane holds channel 16dt + ln, keys 8lg .. 8lg+7
//                                                  (A operand of O^T = V^T.P^T)
// Element offsets within one (row, kv head) block of Smax*128 elements:
ZK_DEV size_t k_off(int key, int c8) {      // dims 8*c8 .. 8*c8+7 of key
    const int o = key & 31, grp = o >> 3, h = (o >> 2) & 1, i = o & 3;
    const int ln = 4 * grp + i, ks = c8 >> 2, lg = c8 & 3;
    return (size_t)(key >> 5) * 4096 + ((h * 4 + ks) * 64 + lg * 16 + ln) * 8;
}
ZK_DEV size_t v_off(int key, int ch) {      // channel ch of key
    const int o = key & 31, lg = o >> 3, e = o & 7;
    return (size_t)(key >> 5) * 4096 + ((ch >> 4) * 64 + lg * 16 + (ch & 15)) * 8 + e;
}

// ------------------------------------------------------------------ LayerNorm helper
// Row of D elements, 8 per thread (D = 8 * NT * n8). Two-pass mean/var in fp32,
// y = (x - mean) * rstd * w + b rounded to bf16 (nn.LayerNorm, eps from config).
// wv / bv: this thread's 8-element chunks of w and b, loaded by the caller before its own
// loads complete (so they share the row's memory round trip); red: 2 * NT / 64 floats (one
// partial-sum slot per wave for the mean and one for the variance: one barrier per reduction).
template <int NT, int n8>
ZK_DEV void ln_row_pre(const float* x, const uint4* wv, const uint4* bv, float eps, int D, bf16_t* y, float* red) {
    const int w = threadIdx.x >> 6;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < n8; ++j)
        if ((threadIdx.x + NT * j) * 8 < D)
            for (int e = 0; e < 8; ++e) s += x[j * 8 + e];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[w] = s;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    const float mean = t / (float)D;
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < n8; ++j)
        if ((threadIdx.x + NT * j) * 8 < D)
            for (int e = 0; e < 8; ++e) { const float d = x[j * 8 + e] - mean; v += d * d; }
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[NT / 64 + w] = v;
    __syncthreads();
    t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[NT / 64 + i];
    const float var = t / (float)D;
    const float rstd = 1.0f / sqrtf(var + eps);
    const float nb = -rstd * mean;
#pragma unroll
    for (int j = 0; j < n8; ++j) {
        const int c = (threadIdx.x + NT * j) * 8;
        if (c >= D) continue;
        float wf[8], bf[8], o[8];
        unpack8(wv[j], wf);
        unpack8(bv[j], bf);
#pragma unroll
        for (int e = 0; e < 8; ++e)
            o[e] = __fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(x[j * 8 + e], rstd), nb), wf[e]), bf[e]);
        *reinterpret_cast<uint4*>(y + c) = pack8(o);
    }
}
// the caller's w / b chunks (clamped index: unconditional loads stay in registers)
template <int NT, int n8>
ZK_DEV void ln_load_wb(const bf16_t* w, const bf16_t* b, int D, uint4* wv, uint4* bv) {
#pragma unroll
    for (int j = 0; j < n8; ++j) {
        const int c = min((int)(threadIdx.x + NT * j) * 8, D - 8);
        wv[j] = *reinterpret_cast<const uint4*>(w + c);
        bv[j] = *reinterpret_cast<const uint4*>(b + c);
    }
}
template <int NT, int n8>
ZK_DEV void ln_row(const float* x, const bf16_t* w, const bf16_t* b, float eps, int D, bf16_t* y, float* red) {
    uint4 wv[n8], bv[n8];
    ln_load_wb<NT, n8>(w, b, D, wv, bv);
    ln_row_pre<NT, n8>(x, wv, bv, eps, D, y, red);
}

constexpr int LN_NT = 256;
constexpr int RL_MAXS = 8;    // split-K slabs k_resid_ln reduces with all loads in flight
constexpr int MAX_N8 = 4;     // D <= 8192
constexpr int EMB_MAXK = 9;   // codebooks summed by k_embed_ln (Zonos: 9)

template <int N8>
__global__ __launch_bounds__(LN_NT) void k_embed_ln(const int64_t* ids, int B, int S, int K, long bstr, long kstr,
                                                    const int32_t* col_dev, int col_add, const bf16_t* emb, int V,
                                                    int D, bf16_t* x_out, int out_S, int out_t0, const bf16_t* lw,
                                                    const bf16_t* lb, float eps, bf16_t* xn_out, const int32_t* skip) {
    __shared__ float red[2 * LN_NT / 64];
    if (skip && *skip) return;
    const int r = blockIdx.x / S, t = blockIdx.x % S, b = r % B;
    const int row = r * out_S + out_t0 + t;   // output row
    const int col = t + (col_dev ? *col_dev + col_add : 0);
    constexpr int n8 = N8;
    float x[N8 * 8];
    // all code ids, then all embedding rows, issued before the first add (two memory round
    // trips per step instead of 2K dependent ones); K <= EMB_MAXK (host-checked)
    // (loads unconditional with a clamped codebook index, so the arrays stay in registers)
    int64_t idv[EMB_MAXK];
#pragma unroll
    for (int k = 0; k < EMB_MAXK; ++k) {
        const int64_t id = ids[b * bstr + min(k, K - 1) * kstr + col];
        idv[k] = id < 0 ? 0 : (id >= V ? V - 1 : id);
    }
#pragma unroll
    for (int j = 0; j < n8; ++j) {
        const int c = (threadIdx.x + LN_NT * j) * 8;
        if (c >= D) continue;
        float acc[8];
        uint4 ev[EMB_MAXK];
#pragma unroll
        for (int k = 0; k < EMB_MAXK; ++k)
            ev[k] = *reinterpret_cast<const uint4*>(emb + ((size_t)min(k, K - 1) * V + idv[k]) * D + c);
#pragma unroll
        for (int k = 0; k < EMB_MAXK; ++k) {
            float e[8];
            unpack8(ev[k], e);
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (k < K) acc[q] = (k == 0) ? e[q] : round_bf(acc[q] + e[q]);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) x[j * 8 + q] = acc[q];
        *reinterpret_cast<uint4*>(x_out + (size_t)row * D + c) = pack8(acc);
    }
    if (lw != nullptr) ln_row<LN_NT, N8>(x, lw, lb, eps, D, xn_out + (size_t)row * D, red);
}

template <int N8>
__global__ __launch_bounds__(LN_NT) void k_layernorm(const bf16_t* x, const bf16_t* w, const bf16_t* b, float eps,
                                                     int D, bf16_t* y) {
    __shared__ float red[2 * LN_NT / 64];
    const int row = blockIdx.x;
    constexpr int n8 = N8;
    float xv[N8 * 8];
#pragma unroll
    for (int j = 0; j < n8; ++j) {
        const int c = (threadIdx.x + LN_NT * j) * 8;
        if (c >= D) continue;
        unpack8(*reinterpret_cast<const uint4*>(x + (size_t)row * D + c), xv + 8 * j);
    }
    ln_row<LN_NT, N8>(xv, w, b, eps, D, y + (size_t)row * D, red);
}

template <int N8>
__global__ __launch_bounds__(LN_NT) void k_resid_ln(const float* part, int nsplit, const bf16_t* x_in,
                                                    const bf16_t* w, const bf16_t* b, float eps, int rows, int D,
                                                    bf16_t* x_out, bf16_t* xn_out, int ln_on_sum,
                                                    const int32_t* skip) {
    __shared__ float red[2 * LN_NT / 64];
    if (skip && *skip) return;
    const int row = blockIdx.x;
    constexpr int n8 = N8;
    const size_t slab = (size_t)rows * D;
    // LayerNorm weights and the residual row issued with the slab loads: one memory round trip
    uint4 wv[N8], bv[N8], xiv[N8];
    ln_load_wb<LN_NT, N8>(w, b, D, wv, bv);
#pragma unroll
    for (int j = 0; j < n8; ++j)
        xiv[j] = *reinterpret_cast<const uint4*>(x_in + (size_t)row * D + min((int)(threadIdx.x + LN_NT * j) * 8, D - 8));
    float xv[N8 * 8];
#pragma unroll
    for (int j = 0; j < n8; ++j) {
        const int c = (threadIdx.x + LN_NT * j) * 8;
        if (c >= D) continue;
        const float* p = part + (size_t)row * D + c;
        float acc[8];
        if (nsplit <= RL_MAXS) {
            // every slab load issued before the first add (clamped index, sum masked), so the
            // row costs one memory round trip instead of nsplit; same left-to-right fp32 sum
            float4 a0[RL_MAXS], a1[RL_MAXS];
#pragma unroll
            for (int s = 0; s < RL_MAXS; ++s) {
                const float* ps = p + (size_t)min(s, nsplit - 1) * slab;
                a0[s] = *reinterpret_cast<const float4*>(ps);
                a1[s] = *reinterpret_cast<const float4*>(ps + 4);
            }
            acc[0] = a0[0].x; acc[1] = a0[0].y; acc[2] = a0[0].z; acc[3] = a0[0].w;
            acc[4] = a1[0].x; acc[5] = a1[0].y; acc[6] = a1[0].z; acc[7] = a1[0].w;
#pragma unroll
            for (int s = 1; s < RL_MAXS; ++s)
                if (s < nsplit) {
                    acc[0] += a0[s].x; acc[1] += a0[s].y; acc[2] += a0[s].z; acc[3] += a0[s].w;
                    acc[4] += a1[s].x; acc[5] += a1[s].y; acc[6] += a1[s].z; acc[7] += a1[s].w;
                }
        } else {
            const float4 a0 = *reinterpret_cast<const float4*>(p);
            const float4 a1 = *reinterpret_cast<const float4*>(p + 4);
            acc[0] = a0.x; acc[1] = a0.y; acc[2] = a0.z; acc[3] = a0.w;
            acc[4] = a1.x; acc[5] = a1.y; acc[6] = a1.z; acc[7] = a1.w;
            for (int s = 1; s < nsplit; ++s) {
                const float4 b0 = *reinterpret_cast<const float4*>(p + s * slab);
                const float4 b1 = *reinterpret_cast<const float4*>(p + s * slab + 4);
                acc[0] += b0.x; acc[1] += b0.y; acc[2] += b0.z; acc[3] += b0.w;
                acc[4] += b1.x; acc[5] += b1.y; acc[6] += b1.z; acc[7] += b1.w;
            }
        }
        float xi[8];
        unpack8(xiv[j], xi);
        // transformer (_torch.py:100-101): x = bf16(x + bf16(proj)), LN of the rounded x;
        // ln_on_sum (mamba_ssm layer_norm_fn prenorm): LN of the fp32 sum, residual stored bf16
#pragma unroll
        for (int e = 0; e < 8; ++e) xv[j * 8 + e] = xi[e] + round_bf(acc[e]);
        *reinterpret_cast<uint4*>(x_out + (size_t)row * D + c) = pack8(xv + 8 * j);
        if (!ln_on_sum) {
#pragma unroll
            for (int e = 0; e < 8; ++e) xv[j * 8 + e] = round_bf(xv[j * 8 + e]);
        }
    }
    ln_row_pre<LN_NT, N8>(xv, wv, bv, eps, D, xn_out + (size_t)row * D, red);
}

// k_resid_ln for D = 2048 with whole-line slab reads: thread t owns the float4 pieces t and
// t + 256 of the row, so every fp32 slab load instruction of a wave reads 1 KB contiguous (the
// 8-element-per-thread layout of k_resid_ln reads 16 B of every 32 B per instruction, each
// line twice). Same arithmetic per element; the LayerNorm sums group the elements differently.
__global__ __launch_bounds__(LN_NT) void k_resid_ln_d2k(const float* part, int nsplit, const bf16_t* x_in,
                                                        const bf16_t* w, const bf16_t* b, float eps, int rows,
                                                        bf16_t* x_out, bf16_t* xn_out, int ln_on_sum,
                                                        const int32_t* skip) {
    constexpr int D = 2048;
    __shared__ float red[2 * LN_NT / 64];
    if (skip && *skip) return;
    const int row = blockIdx.x, t = threadIdx.x;
    const size_t slab = (size_t)rows * D;
    const int c0 = 4 * t, c1 = 1024 + 4 * t;
    // one memory round trip: LN weights, residual and every slab issued before the first add
    const uint2 w0 = *reinterpret_cast<const uint2*>(w + c0), w1 = *reinterpret_cast<const uint2*>(w + c1);
    const uint2 b0 = *reinterpret_cast<const uint2*>(b + c0), b1 = *reinterpret_cast<const uint2*>(b + c1);
    const uint2 x0 = *reinterpret_cast<const uint2*>(x_in + (size_t)row * D + c0);
    const uint2 x1 = *reinterpret_cast<const uint2*>(x_in + (size_t)row * D + c1);
    const float* p = part + (size_t)row * D;
    float4 a0[RL_MAXS], a1[RL_MAXS];
#pragma unroll
    for (int sp = 0; sp < RL_MAXS; ++sp) {
        const float* ps = p + (size_t)min(sp, nsplit - 1) * slab;
        a0[sp] = *reinterpret_cast<const float4*>(ps + c0);
        a1[sp] = *reinterpret_cast<const float4*>(ps + c1);
    }
    float acc[8] = {a0[0].x, a0[0].y, a0[0].z, a0[0].w, a1[0].x, a1[0].y, a1[0].z, a1[0].w};
#pragma unroll
    for (int sp = 1; sp < RL_MAXS; ++sp)
        if (sp < nsplit) {
            acc[0] += a0[sp].x; acc[1] += a0[sp].y; acc[2] += a0[sp].z; acc[3] += a0[sp].w;
            acc[4] += a1[sp].x; acc[5] += a1[sp].y; acc[6] += a1[sp].z; acc[7] += a1[sp].w;
        }
    auto un4 = [](uint2 v, float* f) {
        f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
        f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
    };
    float xi[8], wf[8], bf[8], xv[8];
    un4(x0, xi); un4(x1, xi + 4);
    un4(w0, wf); un4(w1, wf + 4);
    un4(b0, bf); un4(b1, bf + 4);
#pragma unroll
    for (int e = 0; e < 8; ++e) xv[e] = xi[e] + round_bf(acc[e]);      // x = bf16(x + bf16(proj))
    *reinterpret_cast<uint2*>(x_out + (size_t)row * D + c0) = make_uint2(pack2(xv[0], xv[1]), pack2(xv[2], xv[3]));
    *reinterpret_cast<uint2*>(x_out + (size_t)row * D + c1) = make_uint2(pack2(xv[4], xv[5]), pack2(xv[6], xv[7]));
    if (!ln_on_sum) {
#pragma unroll
        for (int e = 0; e < 8; ++e) xv[e] = round_bf(xv[e]);
    }
    const int wv = t >> 6;
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) sum += xv[e];
    sum = wave_sum(sum);
    if ((t & 63) == 0) red[wv] = sum;
    __syncthreads();
    const float mean = (red[0] + red[1] + red[2] + red[3]) / (float)D;
    float var = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = xv[e] - mean; var += d * d; }
    var = wave_sum(var);
    if ((t & 63) == 0) red[4 + wv] = var;
    __syncthreads();
    const float rstd = 1.0f / sqrtf((red[4] + red[5] + red[6] + red[7]) / (float)D + eps);
    const float nb = -rstd * mean;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = __fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(xv[e], rstd), nb), wf[e]), bf[e]);
    *reinterpret_cast<uint2*>(xn_out + (size_t)row * D + c0) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
    *reinterpret_cast<uint2*>(xn_out + (size_t)row * D + c1) = make_uint2(pack2(o[4], o[5]), pack2(o[6], o[7]));
}

// ------------------------------------------------------------------ in_proj epilogue
// RoPE pair j (0..hd/2-1) of a head: interleaved (_torch.py:18-30: dims 2j, 2j+1) or, NEOX,
// GPT-NeoX "rotate half" (flash_attn apply_rotary, interleaved=False: dims j, j + hd/2).
// Both use (cos, sin) entry j of the position's [hd/2][2] table.
template <bool NEOX>
ZK_DEV void rope_dims(int j, int hd, int& d0, int& d1) {
    d0 = NEOX ? j : 2 * j;
    d1 = NEOX ? j + hd / 2 : 2 * j + 1;
}

template <bool NEOX>
__global__ __launch_bounds__(256) void k_qkv_rope(const float* part, int nsplit, int R, int S, int H, int Hkv,
                                                  int hd, const float* freqs, int pos0, const int32_t* pos_dev,
                                                  bf16_t* q_out, bf16_t* kc, bf16_t* vt, int Smax, bf16_t* v_rows,
                                                  const int32_t* skip) {
    if (skip && *skip) return;
    const int row = blockIdx.x;   // r*S + t
    const int r = row / S, t = row % S;
    const int pos = pos0 + t + (pos_dev ? *pos_dev : 0);
    const int N = (H + 2 * Hkv) * hd;
    const size_t slab = (size_t)R * S * N;
    const float* p = part + (size_t)row * N;
    const float* fc = freqs + (size_t)pos * hd;     // [hd/2][2]
    for (int pi = threadIdx.x; pi < N / 2; pi += blockDim.x) {
        const int head = pi / (hd / 2), j = pi % (hd / 2);     // head over q | k | v heads
        int d0, d1;
        rope_dims<NEOX>(j, hd, d0, d1);
        const int c0 = head * hd + d0, c1 = head * hd + d1;
        float a = p[c0], bb = p[c1];
        for (int s = 1; s < nsplit; ++s) { a += p[s * slab + c0]; bb += p[s * slab + c1]; }
        a = round_bf(a); bb = round_bf(bb);
        if (head < H + Hkv) {
            const float c = fc[2 * j], sn = fc[2 * j + 1];
            const float o0 = __fsub_rn(__fmul_rn(a, c), __fmul_rn(bb, sn));
            const float o1 = __fadd_rn(__fmul_rn(bb, c), __fmul_rn(a, sn));
            const bf16_t b0 = f2bf(o0), b1 = f2bf(o1);
            if (head < H) {
                bf16_t* qr = q_out + (size_t)row * H * hd + head * hd;
                qr[d0] = b0;
                qr[d1] = b1;
            } else {
                bf16_t* kb = kc + ((size_t)r * Hkv + (head - H)) * Smax * hd;
                kb[k_off(pos, d0 >> 3) + (d0 & 7)] = b0;
                kb[k_off(pos, d1 >> 3) + (d1 & 7)] = b1;
            }
        } else {
            const int g = head - H - Hkv;
            bf16_t* base = vt + ((size_t)r * Hkv + g) * Smax * hd;
            const bf16_t va = f2bf(a), vb = f2bf(bb);
            base[v_off(pos, d0)] = va;
            base[v_off(pos, d1)] = vb;
            if (v_rows) {
                bf16_t* vr = v_rows + (((size_t)r * Hkv + g) * S + t) * hd;
                vr[d0] = va;
                vr[d1] = vb;
            }
        }
    }
}

// ------------------------------------------------------------------ decode attention
constexpr int AT_KB = 128;      // keys per workgroup iteration (4 waves x 32)
constexpr int AT_G = 4;         // query heads per KV head handled by the B operand (<= 16)
constexpr int AT_STR = 2 * AT_G + AT_G * 128;   // work floats per (r, g, split)
constexpr int AT_MAXGS = 8;     // max in_proj split-K slabs the fused prologue reduces

// One 32-key step of one wave: registers for K (A operand of S^T = K.Q^T) and V^T
// (A operand of O^T = V^T.P^T). Key mapping inside the 32: MFMA row r = 4*grp + i of tile h
// holds key 8*grp + 4*h + i, so a lane's 8 score values are the 8 CONTIGUOUS keys
// 8*grp .. 8*grp+7 and its V^T fragment is one 16-byte load.
struct KVFrag {
    uint4 k[2][4];   // [tile h][d-step]
    uint4 v[8];      // [d-tile]
};

// KV cache slices. NT: loaded non-temporally -- chosen by the host when one launch streams
// >= KV_NT_BYTES of cache (B=64: 0.8 GB, read once per step, far beyond L2 and the MALL: nt 3.815
// vs 3.954 ms per decode step); small caches (B=1: 4 MB per layer) stay MALL-resident across
// steps and plain loads keep them there (1.32 vs 1.35 ms per step).
constexpr double KV_NT_BYTES = 64e6;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
template <bool NT>
ZK_DEV uint4 ld_kv(const bf16_t* p) {
    if constexpr (NT) return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p)));
    else return *reinterpret_cast<const uint4*>(p);
}

template <bool NT>
ZK_DEV void load_kv(KVFrag& f, const bf16_t* kb, const bf16_t* vb, int Smax, int key_base, int ln, int lg) {
    (void)Smax;
    const int lane = lg * 16 + ln;
    const bf16_t* k0 = kb + (size_t)(key_base >> 5) * 4096 + lane * 8;
    const bf16_t* v0 = vb + (size_t)(key_base >> 5) * 4096 + lane * 8;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) f.k[h][ks] = ld_kv<NT>(k0 + (h * 4 + ks) * 512);
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) f.v[dt] = ld_kv<NT>(v0 + dt * 512);
}

struct AttnState {
    float m, l;
    f32x4 o[8];      // o[dt][i] = O^T[d = dt*16 + 4lg + i][head = ln]
};

ZK_DEV void attn_step(AttnState& st, const KVFrag& f, const bf16x8* qf, int key_base, int ctx, float scale,
                      int lg) {
    f32x4 sacc[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        sacc[h] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            sacc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(f.k[h][ks]), qf[ks], sacc[h], 0, 0, 0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int key = key_base + 8 * lg + 4 * h + i;
            const float sv = key < ctx ? sacc[h][i] * scale : -INFINITY;
            sacc[h][i] = sv;
            mx = fmaxf(mx, sv);
        }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(st.m, mx);
    if (mn == -INFINITY) return;                       // nothing visible yet (all keys masked)
    const float corr = (st.m == -INFINITY) ? 0.f : __expf(st.m - mn);
    float ps = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float pv = __expf(sacc[h][i] - mn);
            sacc[h][i] = pv;
            ps += pv;
        }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    st.l = st.l * corr + ps;
    st.m = mn;
    const uint4 pa = make_uint4(pack2(sacc[0][0], sacc[0][1]), pack2(sacc[0][2], sacc[0][3]),
                                pack2(sacc[1][0], sacc[1][1]), pack2(sacc[1][2], sacc[1][3]));
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
#pragma unroll
        for (int i = 0; i < 4; ++i) st.o[dt][i] *= corr;
        st.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(f.v[dt]), as_frag(pa), st.o[dt], 0, 0, 0);
    }
}

// Flash-decoding over the KV cache: grid (nsplit, Hkv, R); each workgroup streams its share
// of 128-key blocks, each wave a 32-key slice of every block, with the next slice's K/V
// loads in flight (two register sets) while the current one is multiplied; the 4 waves merge
// (m, l, O) through LDS at the end. nsplit == 1 writes the normalised bf16 output directly.
// Replace the newest key's K row / V^T entries in a loaded 32-key slice by the values kept in
// LDS (their cache lines are written at the end of the fused kernel). Wave-uniform early out.
ZK_DEV void patch_kv(KVFrag& f, const uint32_t* s_kn, const uint16_t* s_vn, int key_base, int pos, int ln, int lg) {
    if (pos < key_base || pos >= key_base + 32) return;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int key = key_base + 8 * (ln >> 2) + 4 * h + (ln & 3);
        if (key == pos) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) f.k[h][ks] = *reinterpret_cast<const uint4*>(s_kn + ks * 16 + lg * 4);
        }
    }
    const int e = pos - key_base - 8 * lg;      // element of this lane's 8-key V^T group
    if (e >= 0 && e < 8) {
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            uint16_t tmp[8];
            *reinterpret_cast<uint4*>(tmp) = f.v[dt];
            tmp[e] = s_vn[dt * 16 + ln];
            f.v[dt] = *reinterpret_cast<const uint4*>(tmp);
        }
    }
}

// FUSED: the in_proj epilogue (k_qkv_rope) runs as this kernel's prologue -- each workgroup
// reduces the split-K slabs of its own 4 query heads + 1 KV head (768 columns), applies RoPE,
// keeps q in LDS and (the split that owns the newest key) stores the new K / V^T entries
// before the key loop reads them. One launch per layer instead of two.
// COMB (nsplit > 1): the splits of one (row, kv head) combine in this launch instead of in
// k_attn_combine -- each workgroup publishes its partial (m, l, O) (stores drained, agent-scope
// release) and takes a ticket on cnt[row][kv head]; the workgroup drawing the last ticket of the
// launch (tickets are monotonic: the count is a multiple of nsplit before every launch) acquires
// and merges all nsplit partials exactly as k_attn_combine does. Saves the combine launch.
template <bool FUSED, bool NEOX, bool KVNT, bool COMB = false>
__global__ __launch_bounds__(256, 2) void k_attn_decode(const bf16_t* q, bf16_t* kc, bf16_t* vt, int R, int H,
                                                        int Hkv, int Smax, int ctx0, const int32_t* ctx_dev,
                                                        float* work, float scale, bf16_t* out, const int32_t* skip,
                                                        const float* part, int gsplit, const float* freqs,
                                                        uint32_t* cnt = nullptr) {
    constexpr int HD = 128;
    __shared__ float s_m[4][16];
    __shared__ float s_l[4][16];
    __shared__ float s_o[4][AT_G][HD];
    __shared__ __attribute__((aligned(16))) uint32_t s_q[AT_G][HD / 2];
    __shared__ __attribute__((aligned(16))) uint32_t s_kn[HD / 2];   // new key (post-RoPE), bf16 pairs
    __shared__ uint16_t s_vn[HD];                                    // new value
    __shared__ int s_last;                                           // COMB: this workgroup merges
    if (skip && *skip) return;
    const int split = blockIdx.x, nsplit = gridDim.x, g = blockIdx.y, r = blockIdx.z;
    const int ctx = ctx0 + (ctx_dev ? *ctx_dev : 0);
    const int nkb = (ctx + AT_KB - 1) / AT_KB;
    const int kb0 = (int)((long)split * nkb / nsplit), kb1 = (int)((long)(split + 1) * nkb / nsplit);
    const int G = H / Hkv;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ln = lane & 15, lg = lane >> 4;
    bf16_t* kb = kc + ((size_t)r * Hkv + g) * Smax * HD;
    bf16_t* vb = vt + ((size_t)r * Hkv + g) * HD * (size_t)Smax;

    bf16x8 qf[4];
    KVFrag fa, fb;
    const int last = kb1 - 1;
    // the first key block can be fetched before the prologue unless it holds the new key
    // FUSED: the new key's cache lines are written only at the end of the kernel (a store
    // followed by loads of the same partially written lines stalls the key loop); the key loop
    // patches the new K/V into its registers from LDS instead, so the arithmetic is exactly
    // that of reading the cache. The first key block can therefore be fetched before the prologue.
    const int pos = ctx - 1;
    const bool early = FUSED && kb1 > kb0;
    if (early) {      // the first TWO key blocks are in flight during the prologue
        load_kv<KVNT>(fa, kb, vb, Smax, kb0 * AT_KB + 32 * w, ln, lg);
        load_kv<KVNT>(fb, kb, vb, Smax, min(kb0 + 1, last) * AT_KB + 32 * w, ln, lg);
    }
    if constexpr (FUSED) {
        // pairs: [0, G*64) q of heads g*G.., then 64 k pairs, then 64 v pairs
        const int N = (H + 2 * Hkv) * HD;
        const size_t slab = (size_t)R * N;
        const float* prow = part + (size_t)r * N;
        const float* fc = freqs + (size_t)pos * HD;
        uint16_t* q16 = reinterpret_cast<uint16_t*>(&s_q[0][0]);
        uint16_t* k16 = reinterpret_cast<uint16_t*>(s_kn);
        for (int pi = threadIdx.x; pi < (G + 2) * (HD / 2); pi += 256) {
            const int hp = pi / (HD / 2), j = pi % (HD / 2);      // hp < G: q head g*G+hp; G: k; G+1: v
            int d0, d1;
            rope_dims<NEOX>(j, HD, d0, d1);
            const int cb = hp < G ? (g * G + hp) * HD : (hp == G ? H * HD + g * HD : (H + Hkv) * HD + g * HD);
            // all slab loads issued together (clamped slab index, select after) -- same
            // left-to-right fp32 sum as k_qkv_rope
            float v0[AT_MAXGS], v1[AT_MAXGS];
#pragma unroll
            for (int sl = 0; sl < AT_MAXGS; ++sl) {
                const float* ps = prow + (size_t)min(sl, gsplit - 1) * slab + cb;
                v0[sl] = ps[d0];
                v1[sl] = ps[d1];
            }
            const float2 cs = *reinterpret_cast<const float2*>(fc + 2 * j);
            float a = v0[0], bb = v1[0];
#pragma unroll
            for (int sl = 1; sl < AT_MAXGS; ++sl)
                if (sl < gsplit) { a += v0[sl]; bb += v1[sl]; }
            a = round_bf(a);
            bb = round_bf(bb);
            if (hp <= G) {
                const float o0 = __fsub_rn(__fmul_rn(a, cs.x), __fmul_rn(bb, cs.y));
                const float o1 = __fadd_rn(__fmul_rn(bb, cs.x), __fmul_rn(a, cs.y));
                uint16_t* dst = hp < G ? q16 + hp * HD : k16;
                dst[d0] = f2bf(o0);
                dst[d1] = f2bf(o1);
            } else {
                s_vn[d0] = f2bf(a);
                s_vn[d1] = f2bf(bb);
            }
        }
        __syncthreads();      // q, new k, new v in LDS
#ifdef ZK_ATT_DBGQ
        if (q != nullptr && split == 0)
            for (int i = threadIdx.x; i < G * HD / 2; i += 256)
                reinterpret_cast<uint32_t*>(const_cast<bf16_t*>(q))[((size_t)r * H + g * G) * (HD / 2) + i] =
                    s_q[i / (HD / 2)][i % (HD / 2)];
#endif
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (ln < G) v = *reinterpret_cast<const uint4*>(&s_q[ln][ks * 16 + lg * 4]);
            qf[ks] = as_frag(v);
        }
    } else {
        const bf16_t* qr = q + (size_t)r * H * HD + (size_t)(g * G + ln) * HD;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (ln < G) v = *reinterpret_cast<const uint4*>(qr + ks * 32 + lg * 8);
            qf[ks] = as_frag(v);
        }
    }
    AttnState st;
    st.m = -INFINITY;
    st.l = 0.f;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) st.o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (kb1 > kb0) {
        if (!early) load_kv<KVNT>(fa, kb, vb, Smax, kb0 * AT_KB + 32 * w, ln, lg);
        for (int it = kb0; it < kb1; it += 2) {
            if (!(early && it == kb0)) load_kv<KVNT>(fb, kb, vb, Smax, min(it + 1, last) * AT_KB + 32 * w, ln, lg);
            if (FUSED) patch_kv(fa, s_kn, s_vn, it * AT_KB + 32 * w, pos, ln, lg);
            attn_step(st, fa, qf, it * AT_KB + 32 * w, ctx, scale, lg);
            load_kv<KVNT>(fa, kb, vb, Smax, min(it + 2, last) * AT_KB + 32 * w, ln, lg);
            if (it + 1 < kb1) {
                if (FUSED) patch_kv(fb, s_kn, s_vn, (it + 1) * AT_KB + 32 * w, pos, ln, lg);
                attn_step(st, fb, qf, (it + 1) * AT_KB + 32 * w, ctx, scale, lg);
            }
        }
    }
    if (FUSED && split == nsplit - 1) {      // the split owning the newest key stores it (cache for later steps)
        const int t = threadIdx.x;
        if (t < HD / 2) *reinterpret_cast<uint32_t*>(kb + k_off(pos, t >> 2) + ((2 * t) & 7)) = s_kn[t];
        else if (t < HD / 2 + HD) reinterpret_cast<uint16_t*>(vb)[v_off(pos, t - HD / 2)] = s_vn[t - HD / 2];
    }
    // merge the 4 waves
    if (lg == 0) { s_m[w][ln] = st.m; s_l[w][ln] = st.l; }
    __syncthreads();
    const float M = fmaxf(fmaxf(s_m[0][ln], s_m[1][ln]), fmaxf(s_m[2][ln], s_m[3][ln]));
    const float cw = (st.m == -INFINITY) ? 0.f : __expf(st.m - M);
    if (ln < AT_G) {
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) s_o[w][ln][dt * 16 + lg * 4 + i] = st.o[dt][i] * cw;
    }
    __syncthreads();
    if (nsplit == 1) {
        // normalised output for the G heads: thread -> (head, 2 channels)
        for (int i = threadIdx.x; i < G * HD / 2; i += 256) {
            const int h = i / (HD / 2), d = (i % (HD / 2)) * 2;
            float Mh = -INFINITY;
            for (int k = 0; k < 4; ++k) Mh = fmaxf(Mh, s_m[k][h]);
            float L = 0.f;
            for (int k = 0; k < 4; ++k) L += (s_m[k][h] == -INFINITY) ? 0.f : s_l[k][h] * __expf(s_m[k][h] - Mh);
            const float o0 = s_o[0][h][d] + s_o[1][h][d] + s_o[2][h][d] + s_o[3][h][d];
            const float o1 = s_o[0][h][d + 1] + s_o[1][h][d + 1] + s_o[2][h][d + 1] + s_o[3][h][d + 1];
            const float inv = 1.0f / L;
            *reinterpret_cast<uint32_t*>(out + (size_t)r * H * HD + (size_t)(g * G + h) * HD + d) =
                pack2(o0 * inv, o1 * inv);
        }
        return;
    }
    float* wp = work + (((size_t)r * Hkv + g) * nsplit + split) * AT_STR;
    for (int i = threadIdx.x; i < AT_G * HD; i += 256) {
        const int h = i / HD, d = i % HD;
        wp[2 * AT_G + i] = s_o[0][h][d] + s_o[1][h][d] + s_o[2][h][d] + s_o[3][h][d];
    }
    if (threadIdx.x < AT_G) {
        const int h = threadIdx.x;
        float Mh = -INFINITY;
        for (int k = 0; k < 4; ++k) Mh = fmaxf(Mh, s_m[k][h]);
        float L = 0.f;
        for (int k = 0; k < 4; ++k) L += (s_m[k][h] == -INFINITY) ? 0.f : s_l[k][h] * __expf(s_m[k][h] - Mh);
        wp[h] = Mh;
        wp[AT_G + h] = L;
    }
    if constexpr (COMB) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");           // every storing wave drains
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // keep the fence's wait (ROCm 7.2)
            const uint32_t old = __hip_atomic_fetch_add(cnt + (size_t)r * Hkv + g, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            s_last = ((old + 1) % (uint32_t)nsplit) == 0;
        }
        __syncthreads();
        if (!s_last) return;
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        const float* base = work + ((size_t)r * Hkv + g) * nsplit * AT_STR;
        for (int i = threadIdx.x; i < G * HD / 2; i += 256) {       // k_attn_combine's arithmetic
            const int j = i / (HD / 2), d = (i % (HD / 2)) * 2;
            float M = -INFINITY;
            for (int sp = 0; sp < nsplit; ++sp) M = fmaxf(M, base[sp * AT_STR + j]);
            float L = 0.f, o0 = 0.f, o1 = 0.f;
            for (int sp = 0; sp < nsplit; ++sp) {
                const float* p = base + sp * AT_STR;
                const float c = (p[j] == -INFINITY) ? 0.f : __expf(p[j] - M);
                L += p[AT_G + j] * c;
                o0 += p[2 * AT_G + j * HD + d] * c;
                o1 += p[2 * AT_G + j * HD + d + 1] * c;
            }
            const float inv = 1.0f / L;
            *reinterpret_cast<uint32_t*>(out + (size_t)r * H * HD + (size_t)(g * G + j) * HD + d) =
                pack2(o0 * inv, o1 * inv);
        }
    }
}

__global__ __launch_bounds__(64) void k_attn_combine(const float* work, int H, int Hkv, int nsplit, bf16_t* out,
                                                     const int32_t* skip) {
    constexpr int HD = 128;
    if (skip && *skip) return;
    const int h = blockIdx.x, r = blockIdx.y;
    const int G = H / Hkv, g = h / G, j = h % G;
    const float* base = work + ((size_t)r * Hkv + g) * nsplit * AT_STR;
    float M = -INFINITY;
    for (int s = 0; s < nsplit; ++s) M = fmaxf(M, base[s * AT_STR + j]);
    float L = 0.f, o0 = 0.f, o1 = 0.f;
    const int d = threadIdx.x * 2;
    for (int s = 0; s < nsplit; ++s) {
        const float* p = base + s * AT_STR;
        const float c = (p[j] == -INFINITY) ? 0.f : __expf(p[j] - M);
        L += p[AT_G + j] * c;
        o0 += p[2 * AT_G + j * HD + d] * c;
        o1 += p[2 * AT_G + j * HD + d + 1] * c;
    }
    const float inv = 1.0f / L;
    *reinterpret_cast<uint32_t*>(out + (size_t)r * H * HD + (size_t)h * HD + d) = pack2(o0 * inv, o1 * inv);
}

// ------------------------------------------------------------------ prefill attention (causal)
// MFMA form of the decode kernel's slice step with 16 QUERIES as the B operand: workgroup =
// (64-query tile, head, row), each wave owns 16 queries and walks the 32-key slices of the
// packed cache up to its last query (causal). Two passes like the reference's CPU flash kernel
// on a single KV block: the exact row max first (S^T = K.Q^T), then p = exp(s - max) summed in
// fp32 and rounded to bf16 for O^T = V^T.P^T. Each wave's queries are independent (no merge).
__global__ __launch_bounds__(256) void k_attn_prefill(const bf16_t* q, const bf16_t* kc, const bf16_t* vt, int R,
                                                      int S, int H, int Hkv, int Smax, float scale, bf16_t* out) {
    constexpr int HD = 128;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ln = lane & 15, lg = lane >> 4;
    const int h = blockIdx.y, r = blockIdx.z;
    const int q0 = blockIdx.x * 64 + w * 16;               // this wave's first query
    if (q0 >= S) return;
    const int G = H / Hkv, g = h / G;
    const int qt = min(q0 + ln, S - 1);                     // query of this lane's B column
    bf16x8 qf[4];
    {
        const bf16_t* qr = q + ((size_t)(r * S + qt) * H + h) * HD;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) qf[ks] = as_frag(*reinterpret_cast<const uint4*>(qr + ks * 32 + lg * 8));
    }
    const bf16_t* kb = kc + ((size_t)r * Hkv + g) * Smax * HD;
    const bf16_t* vb = vt + ((size_t)r * Hkv + g) * Smax * HD;
    const int last = min(q0 + 15, S - 1);                   // keys 0..last can be visible
    const int nsl = last / 32 + 1;
    // lane's 8 score values: keys 8lg .. 8lg+7 of the slice (tile h: 8lg + 4h + i), query qt
    auto scores = [&](int sl, f32x4* sacc) {
        const int lanei = lg * 16 + ln;
        const bf16_t* k0 = kb + (size_t)sl * 4096 + lanei * 8;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            sacc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
                sacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    as_frag(*reinterpret_cast<const uint4*>(k0 + (t * 4 + ks) * 512)), qf[ks], sacc[t], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int key = sl * 32 + 8 * lg + 4 * t + i;
                sacc[t][i] = key <= qt ? sacc[t][i] * scale : -INFINITY;
            }
    };
    float m = -INFINITY;
    for (int sl = 0; sl < nsl; ++sl) {
        f32x4 sacc[2];
        scores(sl, sacc);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) m = fmaxf(m, sacc[t][i]);
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
    f32x4 o[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int sl = 0; sl < nsl; ++sl) {
        f32x4 sacc[2];
        scores(sl, sacc);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float pv = __expf(sacc[t][i] - m);       // masked keys: exp(-inf) = 0
                sacc[t][i] = pv;
                l += pv;
            }
        const uint4 pa = make_uint4(pack2(sacc[0][0], sacc[0][1]), pack2(sacc[0][2], sacc[0][3]),
                                    pack2(sacc[1][0], sacc[1][1]), pack2(sacc[1][2], sacc[1][3]));
        const bf16_t* v0 = vb + (size_t)sl * 4096 + (lg * 16 + ln) * 8;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(*reinterpret_cast<const uint4*>(v0 + dt * 512)),
                                                            as_frag(pa), o[dt], 0, 0, 0);
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    // o[dt][i] = O^T[dim = 16dt + 4lg + i][query q0 + ln]
    if (q0 + ln < S) {
        const float inv = 1.0f / l;
        bf16_t* orow = out + ((size_t)(r * S + q0 + ln) * H + h) * HD;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            const int d = dt * 16 + lg * 4;
            *reinterpret_cast<uint2*>(orow + d) =
                make_uint2(pack2(o[dt][0] * inv, o[dt][1] * inv), pack2(o[dt][2] * inv, o[dt][3] * inv));
        }
    }
}

}  // namespace

#define ZK_LN_DISPATCH(D, kern, ...)                                              \
    do {                                                                           \
        const int _n8 = ((D) / 8 + LN_NT - 1) / LN_NT;                             \
        if (_n8 == 1) hipLaunchKernelGGL(kern<1>, __VA_ARGS__);                    \
        else if (_n8 == 2) hipLaunchKernelGGL(kern<2>, __VA_ARGS__);               \
        else if (_n8 == 3) hipLaunchKernelGGL(kern<3>, __VA_ARGS__);               \
        else hipLaunchKernelGGL(kern<4>, __VA_ARGS__);                             \
    } while (0)

extern "C" int zk_embed_codes(const int64_t* ids, int B, int S, int K, long ids_bstride, long ids_kstride,
                              const int32_t* col_dev, int col_add, const void* emb, int V, int D, int rows_dup,
                              void* x_out, int out_S, int out_t0, const void* ln_w, const void* ln_b, float eps,
                              void* xn_out, const int32_t* skip, void* stream) {
    ZK_REQUIRE(D % 8 == 0 && D <= 8 * LN_NT * MAX_N8, "zk_embed_codes: D=%d must be a multiple of 8 (<= %d)", D,
               8 * LN_NT * MAX_N8);
    ZK_REQUIRE(B > 0 && S > 0 && K > 0 && rows_dup > 0, "zk_embed_codes: empty shape");
    ZK_REQUIRE(K <= EMB_MAXK, "zk_embed_codes: K=%d codebooks > %d", K, EMB_MAXK);
    const int rows = rows_dup * B * S;
    ZK_REQUIRE(out_S >= out_t0 + S, "zk_embed_codes: out_S=%d < out_t0+S", out_S);
    ZK_LN_DISPATCH(D, k_embed_ln, dim3(rows), dim3(LN_NT), 0, (hipStream_t)stream, ids, B, S, K, ids_bstride,
                   ids_kstride, col_dev, col_add, (const bf16_t*)emb, V, D, (bf16_t*)x_out, out_S, out_t0,
                   (const bf16_t*)ln_w, (const bf16_t*)ln_b, eps, (bf16_t*)xn_out, skip);
    ZK_CHECK_LAUNCH("zk_embed_codes");
    return 0;
}

extern "C" int zk_layernorm(const void* x, const void* w, const void* b, float eps, int rows, int D, void* y,
                            void* stream) {
    ZK_REQUIRE(D % 8 == 0 && D <= 8 * LN_NT * MAX_N8, "zk_layernorm: unsupported D=%d", D);
    if (rows == 0) return 0;
    ZK_LN_DISPATCH(D, k_layernorm, dim3(rows), dim3(LN_NT), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (const bf16_t*)w, (const bf16_t*)b, eps, D, (bf16_t*)y);
    ZK_CHECK_LAUNCH("zk_layernorm");
    return 0;
}

extern "C" int zk_resid_ln(const float* part, int nsplit, const void* x_in, const void* w, const void* b, float eps,
                           int rows, int D, void* x_out, void* xn_out, int ln_on_sum, const int32_t* skip,
                           void* stream) {
    ZK_REQUIRE(D % 8 == 0 && D <= 8 * LN_NT * MAX_N8, "zk_resid_ln: unsupported D=%d", D);
    ZK_REQUIRE(nsplit >= 1, "zk_resid_ln: nsplit must be >= 1");
    if (rows == 0) return 0;
    static const bool d2k = [] {               // ZK_RESID_D2K=0: generic layout (A/B knob, read once)
        const char* e = getenv("ZK_RESID_D2K");
        return !(e && e[0] == '0');
    }();
    if (D == 2048 && nsplit <= RL_MAXS && d2k) {
        hipLaunchKernelGGL(k_resid_ln_d2k, dim3(rows), dim3(LN_NT), 0, (hipStream_t)stream, part, nsplit,
                           (const bf16_t*)x_in, (const bf16_t*)w, (const bf16_t*)b, eps, rows, (bf16_t*)x_out,
                           (bf16_t*)xn_out, ln_on_sum, skip);
        ZK_CHECK_LAUNCH("zk_resid_ln");
        return 0;
    }
    ZK_LN_DISPATCH(D, k_resid_ln, dim3(rows), dim3(LN_NT), 0, (hipStream_t)stream, part, nsplit,
                       (const bf16_t*)x_in, (const bf16_t*)w, (const bf16_t*)b, eps, rows, D, (bf16_t*)x_out,
                       (bf16_t*)xn_out, ln_on_sum, skip);
    ZK_CHECK_LAUNCH("zk_resid_ln");
    return 0;
}

extern "C" int zk_qkv_rope(const float* part, int nsplit, int R, int S, int H, int Hkv, int hd, const float* freqs,
                           int pos0, const int32_t* pos_dev, void* q_out, void* k_cache, void* vt_cache, int Smax,
                           void* v_rows, int rope_neox, const int32_t* skip, void* stream) {
    ZK_REQUIRE(hd % 2 == 0 && nsplit >= 1, "zk_qkv_rope: bad args");
    if (R * S == 0) return 0;
    if (rope_neox)
        hipLaunchKernelGGL(k_qkv_rope<true>, dim3(R * S), dim3(256), 0, (hipStream_t)stream, part, nsplit, R, S, H,
                           Hkv, hd, freqs, pos0, pos_dev, (bf16_t*)q_out, (bf16_t*)k_cache, (bf16_t*)vt_cache, Smax,
                           (bf16_t*)v_rows, skip);
    else
        hipLaunchKernelGGL(k_qkv_rope<false>, dim3(R * S), dim3(256), 0, (hipStream_t)stream, part, nsplit, R, S, H,
                           Hkv, hd, freqs, pos0, pos_dev, (bf16_t*)q_out, (bf16_t*)k_cache, (bf16_t*)vt_cache, Smax,
                           (bf16_t*)v_rows, skip);
    ZK_CHECK_LAUNCH("zk_qkv_rope");
    return 0;
}

extern "C" int zk_attn_decode(const void* q, const void* k_cache, const void* vt_cache, int R, int H, int Hkv,
                              int hd, int Smax, int ctx0, const int32_t* ctx_dev, float* work, int nsplit,
                              void* out, const int32_t* skip, void* stream) {
    ZK_REQUIRE(hd == 128, "zk_attn_decode: head_dim %d unsupported (128 only)", hd);
    ZK_REQUIRE(H % Hkv == 0 && H / Hkv <= AT_G, "zk_attn_decode: GQA group %d > %d", H / Hkv, AT_G);
    ZK_REQUIRE(Smax % AT_KB == 0, "zk_attn_decode: Smax=%d must be a multiple of %d", Smax, AT_KB);
    ZK_REQUIRE(nsplit >= 1 && nsplit <= Smax / AT_KB, "zk_attn_decode: nsplit=%d out of [1, %d]", nsplit,
               Smax / AT_KB);
    ZK_REQUIRE(nsplit == 1 || work != nullptr, "zk_attn_decode: nsplit > 1 needs the work buffer");
    const float scale = 1.0f / sqrtf((float)hd);
    const bool kvnt = (double)R * Hkv * Smax * hd * 4 >= KV_NT_BYTES;
    auto kern = kvnt ? k_attn_decode<false, false, true> : k_attn_decode<false, false, false>;
    hipLaunchKernelGGL(kern, dim3(nsplit, Hkv, R), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)q, (bf16_t*)k_cache, (bf16_t*)vt_cache, R, H, Hkv, Smax, ctx0, ctx_dev, work,
                       scale, (bf16_t*)out, skip, nullptr, 0, nullptr, nullptr);
    ZK_CHECK_LAUNCH("zk_attn_decode");
    if (nsplit > 1) {
        hipLaunchKernelGGL(k_attn_combine, dim3(H, R), dim3(64), 0, (hipStream_t)stream, work, H, Hkv, nsplit,
                           (bf16_t*)out, skip);
        ZK_CHECK_LAUNCH("zk_attn_combine");
    }
    return 0;
}

extern "C" int zk_attn_decode_qkv(const float* part, int gemm_nsplit, const float* freqs, void* k_cache,
                                  void* vt_cache, int R, int H, int Hkv, int hd, int Smax, int ctx0,
                                  const int32_t* ctx_dev, float* work, int nsplit, void* out, int rope_neox,
                                  const int32_t* skip, void* stream) {
    ZK_REQUIRE(hd == 128, "zk_attn_decode_qkv: head_dim %d unsupported (128 only)", hd);
    ZK_REQUIRE(H % Hkv == 0 && H / Hkv <= AT_G, "zk_attn_decode_qkv: GQA group %d > %d", H / Hkv, AT_G);
    ZK_REQUIRE(Smax % AT_KB == 0, "zk_attn_decode_qkv: Smax=%d must be a multiple of %d", Smax, AT_KB);
    ZK_REQUIRE(nsplit >= 1 && nsplit <= Smax / AT_KB, "zk_attn_decode_qkv: nsplit=%d out of [1, %d]", nsplit,
               Smax / AT_KB);
    ZK_REQUIRE(nsplit == 1 || work != nullptr, "zk_attn_decode_qkv: nsplit > 1 needs the work buffer");
    ZK_REQUIRE(part != nullptr && freqs != nullptr && gemm_nsplit >= 1 && gemm_nsplit <= AT_MAXGS,
               "zk_attn_decode_qkv: bad arguments (gemm_nsplit=%d, max %d)", gemm_nsplit, AT_MAXGS);
    const float scale = 1.0f / sqrtf((float)hd);
#ifdef ZK_ATT_DBGQ
    const bf16_t* dbgq = (const bf16_t*)work;
#else
    const bf16_t* dbgq = nullptr;
#endif
    const bool kvnt = (double)R * Hkv * Smax * hd * 4 >= KV_NT_BYTES;
    auto kern = rope_neox ? (kvnt ? k_attn_decode<true, true, true> : k_attn_decode<true, true, false>)
                          : (kvnt ? k_attn_decode<true, false, true> : k_attn_decode<true, false, false>);
    hipLaunchKernelGGL(kern, dim3(nsplit, Hkv, R), dim3(256), 0, (hipStream_t)stream, dbgq, (bf16_t*)k_cache,
                       (bf16_t*)vt_cache, R, H, Hkv, Smax, ctx0, ctx_dev, work, scale, (bf16_t*)out, skip, part,
                       gemm_nsplit, freqs, nullptr);
    ZK_CHECK_LAUNCH("zk_attn_decode_qkv");
    if (nsplit > 1) {
        hipLaunchKernelGGL(k_attn_combine, dim3(H, R), dim3(64), 0, (hipStream_t)stream, work, H, Hkv, nsplit,
                           (bf16_t*)out, skip);
        ZK_CHECK_LAUNCH("zk_attn_combine");
    }
    return 0;
}

extern "C" int zk_attn_decode_qkv_sc(const float* part, int gemm_nsplit, const float* freqs, void* k_cache,
                                     void* vt_cache, int R, int H, int Hkv, int hd, int Smax, int ctx0,
                                     const int32_t* ctx_dev, float* work, int nsplit, uint32_t* counters, void* out,
                                     int rope_neox, const int32_t* skip, void* stream) {
    if (nsplit == 1 || counters == nullptr)
        return zk_attn_decode_qkv(part, gemm_nsplit, freqs, k_cache, vt_cache, R, H, Hkv, hd, Smax, ctx0, ctx_dev,
                                  work, nsplit, out, rope_neox, skip, stream);
    ZK_REQUIRE(hd == 128, "zk_attn_decode_qkv_sc: head_dim %d unsupported (128 only)", hd);
    ZK_REQUIRE(H % Hkv == 0 && H / Hkv <= AT_G, "zk_attn_decode_qkv_sc: GQA group %d > %d", H / Hkv, AT_G);
    ZK_REQUIRE(Smax % AT_KB == 0, "zk_attn_decode_qkv_sc: Smax=%d must be a multiple of %d", Smax, AT_KB);
    ZK_REQUIRE(nsplit >= 1 && nsplit <= Smax / AT_KB, "zk_attn_decode_qkv_sc: nsplit=%d out of [1, %d]", nsplit,
               Smax / AT_KB);
    ZK_REQUIRE(work != nullptr, "zk_attn_decode_qkv_sc: nsplit > 1 needs the work buffer");
    ZK_REQUIRE(part != nullptr && freqs != nullptr && gemm_nsplit >= 1 && gemm_nsplit <= AT_MAXGS,
               "zk_attn_decode_qkv_sc: bad arguments (gemm_nsplit=%d, max %d)", gemm_nsplit, AT_MAXGS);
    const float scale = 1.0f / sqrtf((float)hd);
    const bool kvnt = (double)R * Hkv * Smax * hd * 4 >= KV_NT_BYTES;
    auto kern = rope_neox ? (kvnt ? k_attn_decode<true, true, true, true> : k_attn_decode<true, true, false, true>)
                          : (kvnt ? k_attn_decode<true, false, true, true> : k_attn_decode<true, false, false, true>);
    hipLaunchKernelGGL(kern, dim3(nsplit, Hkv, R), dim3(256), 0, (hipStream_t)stream, nullptr, (bf16_t*)k_cache,
                       (bf16_t*)vt_cache, R, H, Hkv, Smax, ctx0, ctx_dev, work, scale, (bf16_t*)out, skip, part,
                       gemm_nsplit, freqs, counters);
    ZK_CHECK_LAUNCH("zk_attn_decode_qkv_sc");
    return 0;
}

extern "C" int zk_attn_prefill(const void* q, const void* k_cache, const void* vt_cache, int R, int S, int H,
                               int Hkv, int hd, int Smax, void* out, void* stream) {
    ZK_REQUIRE(hd == 128, "zk_attn_prefill: head_dim %d unsupported (128 only)", hd);
    ZK_REQUIRE(H % Hkv == 0, "zk_attn_prefill: H %% Hkv != 0");
    if (R * S == 0) return 0;
    const float scale = 1.0f / sqrtf((float)hd);
    ZK_REQUIRE(S <= Smax && Smax % 32 == 0, "zk_attn_prefill: S=%d Smax=%d", S, Smax);
    hipLaunchKernelGGL(k_attn_prefill, dim3((S + 63) / 64, H, R), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)q, (const bf16_t*)k_cache, (const bf16_t*)vt_cache, R, S, H, Hkv, Smax, scale,
                       (bf16_t*)out);
    ZK_CHECK_LAUNCH("zk_attn_prefill");
    return 0;
}
