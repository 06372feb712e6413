// Mamba2 mixer of the hybrid backbone (zonos/backbone/_mamba_ssm.py -> mamba_ssm Mamba2,
// restated in oracle/hybrid_ref.py) for gfx950.
//
//   k_mamba_step   : decode. One workgroup per (head, row): split-K slab reduction of the
//                    in_proj columns it needs (z, x of its head, B, C, dt) -> bf16; causal
//                    depthwise conv update (4 taps, fp32 math, SiLU, bf16 out) for its x channels
//                    and for B/C; the SSM state update h = exp(dt A) h + (B dt) x with the bf16
//                    state [headdim][d_state] streamed once (read + write, 16 KB per head);
//                    y = C.h + D x -> bf16 -> y * silu(z) (fp32) for the gated RMSNorm.
//                    The conv state is double-buffered by step parity (B/C channels are read by
//                    every head's workgroup and rewritten by head 0's).
//   k_mamba_conv_seq / k_mamba_scan : prefill. Causal conv over the whole prefix (parallel),
//                    then the exact recurrence per (head, row), LDS-staged 16 steps at a time,
//                    the fp32 state in registers; final state stored bf16.
//   k_gated_norm   : RMSNormGated(norm_before_gate=False): out = bf16(g * rsqrt(mean(g^2)+eps) * w)
//                    over the d_inner channels of a row (g = y * silu(z) from the kernels above).
// The state update is HBM-bound: per decode step and Mamba layer 2 * R * d_inner * d_state * 2 B.
#include "common.h"
#include "../../include/zonos_hip.h"
#include <algorithm>
#include <stdlib.h>

namespace {

constexpr int MB_THREADS = 256;
constexpr int MB_MAXGS = 8;
constexpr int GN_MAXJ = 16;      // k_gated_norm: row elements per thread held in registers (d_inner <= 4096)

ZK_DEV float silu_f(float v) { return v / (1.0f + expf(-v)); }
ZK_DEV float softplus_thr(float v) { return v <= 20.0f ? log1pf(expf(v)) : v; }

// sum of the split-K slabs of one in_proj column, rounded to bf16 (the GEMM output dtype)
ZK_DEV float slab_col(const float* p, size_t slab, int gs, int col) {
    float v[MB_MAXGS];
#pragma unroll
    for (int s = 0; s < MB_MAXGS; ++s) v[s] = p[(size_t)min(s, gs - 1) * slab + col];
    float a = v[0];
#pragma unroll
    for (int s = 1; s < MB_MAXGS; ++s)
        if (s < gs) a += v[s];
    return round_bf(a);
}

template <int HP, int DS>
__global__ __launch_bounds__(MB_THREADS) void k_mamba_step(
    const float* __restrict__ part, int gs, int R, int di, int nh, const float* __restrict__ conv_w,
    const float* __restrict__ conv_b, const bf16_t* __restrict__ cs_a, bf16_t* __restrict__ cs_b,
    const int32_t* __restrict__ pos_dev, bf16_t* __restrict__ ssm, bf16_t* __restrict__ ssm_b,
    const float* __restrict__ A,
    const float* __restrict__ dt_bias, const float* __restrict__ Dv, float* __restrict__ yz,
    const int32_t* __restrict__ skip) {
    constexpr int TPP = MB_THREADS / HP;     // threads per headdim row
    constexpr int EPT = DS / TPP;            // state elements per thread
    static_assert(TPP * HP == MB_THREADS && EPT * TPP == DS && EPT % 8 == 0, "tile");
    __shared__ float s_x[HP], s_z[HP], s_B[DS], s_C[DS], s_dt;
    if (skip && *skip) return;
    const int h = blockIdx.x, r = blockIdx.y;
    const int conv_dim = di + 2 * DS;
    const int ncol = 2 * di + 2 * DS + nh;
    const size_t slab = (size_t)R * ncol;
    const float* prow = part + (size_t)r * ncol;
    // conv state parity: step at position pos reads buffer (pos & 1), writes the other
    const int par = pos_dev ? (*pos_dev & 1) : 0;
    const bf16_t* csi = (par ? cs_b : cs_a) + (size_t)r * conv_dim * 4;
    bf16_t* cso = (par ? const_cast<bf16_t*>(cs_a) : cs_b) + (size_t)r * conv_dim * 4;
    // SSM state: in place (ssm_b == nullptr) or ping-pong like the conv state (read buffer pos & 1)
    const bf16_t* ssr = (ssm_b && par) ? ssm_b : ssm;
    bf16_t* ssw = ssm_b ? (par ? ssm : ssm_b) : ssm;
    // (loading the state slice before this prologue measured 1 % slower: occupancy 8 -> 7 waves)
    const int t = threadIdx.x, p = t / TPP, n0 = (t % TPP) * EPT;
    const size_t soff = (((size_t)r * nh + h) * HP + p) * DS + n0;
    const bf16_t* sp = ssr + soff;
    bf16_t* spw = ssw + soff;
    uint4 st8[EPT / 8];

    for (int i = threadIdx.x; i < HP + 2 * DS + HP + 1; i += MB_THREADS) {
        if (i < HP + 2 * DS) {
            // conv channel: x channel of this head, or B / C
            const int ch = i < HP ? h * HP + i : di + (i - HP);
            const float xnew = slab_col(prow, slab, gs, di + ch);
            const uint2 st = *reinterpret_cast<const uint2*>(csi + (size_t)ch * 4);
            const float s1 = __uint_as_float((st.x >> 16) << 16), s2 = __uint_as_float((st.y & 0xffffu) << 16);
            const float s3 = __uint_as_float((st.y >> 16) << 16);
            const float* w = conv_w + (size_t)ch * 4;
            float acc = conv_b[ch];
            acc += w[0] * s1;
            acc += w[1] * s2;
            acc += w[2] * s3;
            acc += w[3] * xnew;
            const float o = round_bf(silu_f(acc));
            if (i < HP) s_x[i] = o;
            else if (i < HP + DS) s_B[i - HP] = o;
            else s_C[i - HP - DS] = o;
            if (i < HP || h == 0) {
                const uint32_t lo = (st.x >> 16) | (st.y << 16);                       // s1, s2
                const uint32_t hi = (st.y >> 16) | ((uint32_t)f2bf(xnew) << 16);        // s3, xnew
                *reinterpret_cast<uint2*>(cso + (size_t)ch * 4) = make_uint2(lo, hi);
            }
        } else if (i < HP + 2 * DS + HP) {
            const int j = i - HP - 2 * DS;
            s_z[j] = slab_col(prow, slab, gs, h * HP + j);
        } else {
            s_dt = slab_col(prow, slab, gs, 2 * di + 2 * DS + h);
        }
    }
    __syncthreads();
    const float dt = softplus_thr(s_dt + dt_bias[h]);
    const float dA = expf(dt * A[h]);
    const float xp = s_x[p];
    float acc = 0.f;
#pragma unroll
    for (int e8 = 0; e8 < EPT; e8 += 8) st8[e8 / 8] = *reinterpret_cast<const uint4*>(sp + e8);
#pragma unroll
    for (int e8 = 0; e8 < EPT; e8 += 8) {
        float sv[8];
        unpack8(st8[e8 / 8], sv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int n = n0 + e8 + e;
            const float s = sv[e] * dA + (s_B[n] * dt) * xp;
            sv[e] = s;
            acc += s * s_C[n];
        }
        *reinterpret_cast<uint4*>(spw + e8) = pack8(sv);
    }
#pragma unroll
    for (int off = 1; off < TPP; off <<= 1) acc += __shfl_xor(acc, off, 64);
    if (t % TPP == 0) {
        const float y = round_bf(acc + xp * Dv[h]);
        const float zz = s_z[p];
        yz[(size_t)r * di + h * HP + p] = y * (zz * (1.0f / (1.0f + expf(-zz))));
    }
}

// Grouped form of k_mamba_step: one workgroup per (row, group of HG heads). The B / C conv
// channels (2 * d_state of them, shared by all heads of a row) are computed once per group
// instead of once per head, every prologue load is issued before the first one is waited for
// (the in_proj slab columns, conv states and taps of all the group's channels), the first two
// heads' SSM state slices are in flight during the prologue, and the heads are then streamed
// with the next head's state loads in flight while the current one is updated. The per-element
// arithmetic and the y reduction are those of k_mamba_step (bit-identical outputs and states).
#ifndef ZK_MB_HG
#define ZK_MB_HG 1                   // heads per workgroup (1: 54.4 us, 2: 60.2, 4: 61.9, 8: 68.6 at c5; tools/mamba_ab.sh)
#endif
#ifndef ZK_MB_PD
#define ZK_MB_PD 1                   // heads' state slices in flight
#endif
#ifndef ZK_MB_DEFER
#define ZK_MB_DEFER 1                // k_mamba_step_g / k_gated_norm test the step word after their first loads
#endif
#ifndef ZK_MB_NT
#define ZK_MB_NT 3                   // non-temporal SSM state loads (1) / stores (2): c5 decode 4.42 -> 4.34 ms (the stores; loads alone 4.47-4.49)
#endif
typedef __attribute__((ext_vector_type(4))) unsigned int mb_u32x4;
__device__ __forceinline__ uint4 mb_ld_state(const bf16_t* p) {
    if constexpr (ZK_MB_NT & 1)
        return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const mb_u32x4*>(p)));
    else return *reinterpret_cast<const uint4*>(p);
}
__device__ __forceinline__ void mb_st_state(bf16_t* p, uint4 v) {
    if constexpr (ZK_MB_NT & 2)
        __builtin_nontemporal_store(__builtin_bit_cast(mb_u32x4, v), reinterpret_cast<mb_u32x4*>(p));
    else *reinterpret_cast<uint4*>(p) = v;
}
template <int HP, int DS, int HG, int GS>
__global__ __launch_bounds__(MB_THREADS) void k_mamba_step_g(
    const float* __restrict__ part, int R, int di, int nh, const float* __restrict__ conv_w,
    const float* __restrict__ conv_b, const bf16_t* __restrict__ cs_a, bf16_t* __restrict__ cs_b,
    const int32_t* __restrict__ pos_dev, bf16_t* __restrict__ ssm, bf16_t* __restrict__ ssm_b,
    const float* __restrict__ A,
    const float* __restrict__ dt_bias, const float* __restrict__ Dv, float* __restrict__ yz,
    const int32_t* __restrict__ skip) {
    constexpr int TPP = MB_THREADS / HP;     // threads per headdim row
    constexpr int EPT = DS / TPP;            // state elements per thread
    constexpr int NV = EPT / 8;              // 16-B state loads per thread and head
    constexpr int NX = HG * HP;              // x (and z) channels of the group
    constexpr int NI = 2 * NX + 2 * DS + HG; // prologue items: x conv, B/C conv, z, dt
    constexpr int NIT = (NI + MB_THREADS - 1) / MB_THREADS;
    static_assert(TPP * HP == MB_THREADS && EPT * TPP == DS && EPT % 8 == 0, "tile");
    __shared__ float s_x[NX], s_z[NX], s_B[DS], s_C[DS], s_dt[HG];
    if (!ZK_MB_DEFER)
        if (skip && *skip) return;
    const int h0 = blockIdx.x * HG, r = blockIdx.y;
    const int conv_dim = di + 2 * DS;
    const int ncol = 2 * di + 2 * DS + nh;
    const size_t slab = (size_t)R * ncol;
    const float* prow = part + (size_t)r * ncol;
    const int par = pos_dev ? (*pos_dev & 1) : 0;
    const bf16_t* csi = (par ? cs_b : cs_a) + (size_t)r * conv_dim * 4;
    bf16_t* cso = (par ? const_cast<bf16_t*>(cs_a) : cs_b) + (size_t)r * conv_dim * 4;
    const bf16_t* ssr = (ssm_b && par) ? ssm_b : ssm;       // SSM state ping-pong (see k_mamba_step)
    bf16_t* ssw = ssm_b ? (par ? ssm : ssm_b) : ssm;
    const int t = threadIdx.x, p = t / TPP, n0 = (t % TPP) * EPT;

    // ---- prologue loads (all issued before any is used)
    int col[NIT], ch[NIT];
    float sv[NIT][GS];
    uint2 cst[NIT];
    float4 cw[NIT];
    float cb[NIT];
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
        const int i = min(t + MB_THREADS * k, NI - 1);
        int c, cc;
        if (i < NX) { cc = h0 * HP + i; c = di + cc; }                              // x conv channel
        else if (i < NX + 2 * DS) { cc = di + (i - NX); c = di + cc; }              // B / C conv channel
        else if (i < 2 * NX + 2 * DS) { cc = 0; c = h0 * HP + (i - NX - 2 * DS); }  // z column
        else { cc = 0; c = 2 * di + 2 * DS + h0 + (i - 2 * NX - 2 * DS); }         // dt column
        col[k] = c;
        ch[k] = cc;
#pragma unroll
        for (int g = 0; g < GS; ++g) sv[k][g] = prow[(size_t)g * slab + c];
        cst[k] = *reinterpret_cast<const uint2*>(csi + (size_t)cc * 4);
        cw[k] = *reinterpret_cast<const float4*>(conv_w + (size_t)cc * 4);
        cb[k] = conv_b[cc];
    }
    (void)col;
    // the first PD heads' state slices. COAL (d_state = 128): every state load / store
    // instruction of a wave covers 1 KB contiguous (8 whole 128-B lines) -- lane L of wave w holds,
    // for v = 0..NV-1, row pv = (w*NV + v)*4 + L/16, channels 8*(L%16) .. +7 -- instead of 16 B of
    // every 64 B (thread-contiguous 64-B runs: each instruction touching 32 lines partially).
    constexpr bool COAL = DS == 128 && HP * DS / 8 == MB_THREADS * NV;
    constexpr int PD = ZK_MB_PD < HG ? ZK_MB_PD : HG;
    const int lw = t >> 6, ll = t & 63;
    uint4 st[PD][NV];
    auto st_off = [&](int v) -> size_t {        // element offset of piece v in the (row, head) state
        if constexpr (COAL) return ((size_t)(lw * NV + v) * 64 + ll) * 8;
        else return (size_t)p * DS + n0 + 8 * v;
    };
    auto load_state = [&](int hh, int buf) {
        const bf16_t* sb = ssr + ((size_t)r * nh + h0 + hh) * HP * DS;
#pragma unroll
        for (int v = 0; v < NV; ++v) st[buf][v] = mb_ld_state(sb + st_off(v));
    };
#pragma unroll
    for (int hh = 0; hh < PD; ++hh) load_state(hh, hh);
    if constexpr (ZK_MB_DEFER) {
        // the step word once the prologue and the first state slices are in flight (every load above
        // is in bounds; nothing is written before this test)
        if (ld_word_here(skip)) {
#pragma unroll
            for (int k = 0; k < NIT; ++k) {
#pragma unroll
                for (int g = 0; g < GS; ++g) asm volatile("" ::"v"(sv[k][g]));
                asm volatile("" ::"v"(cst[k].x), "v"(cst[k].y), "v"(cb[k]));
                keep_live(cw[k]);
            }
#pragma unroll
            for (int hh = 0; hh < PD; ++hh)
#pragma unroll
                for (int v = 0; v < NV; ++v) keep_live(st[hh][v]);
            return;
        }
    }

    // ---- prologue arithmetic (the per-item arithmetic of k_mamba_step)
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
        const int i = t + MB_THREADS * k;
        if (i >= NI) break;
        float a = sv[k][0];
#pragma unroll
        for (int g = 1; g < GS; ++g) a += sv[k][g];
        a = round_bf(a);                                                              // slab_col
        if (i < NX + 2 * DS) {
            const uint2 s2 = cst[k];
            const float s1 = __uint_as_float((s2.x >> 16) << 16), sa = __uint_as_float((s2.y & 0xffffu) << 16);
            const float s3 = __uint_as_float((s2.y >> 16) << 16);
            float acc = cb[k];
            acc += cw[k].x * s1;
            acc += cw[k].y * sa;
            acc += cw[k].z * s3;
            acc += cw[k].w * a;
            const float o = round_bf(silu_f(acc));
            if (i < NX) s_x[i] = o;
            else if (i < NX + DS) s_B[i - NX] = o;
            else s_C[i - NX - DS] = o;
            if (i < NX || h0 == 0) {
                const uint32_t lo = (s2.x >> 16) | (s2.y << 16);
                const uint32_t hi = (s2.y >> 16) | ((uint32_t)f2bf(a) << 16);
                *reinterpret_cast<uint2*>(cso + (size_t)ch[k] * 4) = make_uint2(lo, hi);
            }
        } else if (i < 2 * NX + 2 * DS) {
            s_z[i - NX - 2 * DS] = a;
        } else {
            s_dt[i - 2 * NX - 2 * DS] = a;
        }
    }
    __syncthreads();

    // ---- the group's heads, one state slice in flight ahead
#pragma unroll
    for (int hh = 0; hh < HG; ++hh) {
        const int h = h0 + hh, buf = hh % PD;
        const float dt = softplus_thr(s_dt[hh] + dt_bias[h]);
        const float dA = expf(dt * A[h]);
        if constexpr (COAL) {
            const int nb = 8 * (ll & 15);
            float Bv[8], Cv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) { Bv[e] = s_B[nb + e] * dt; Cv[e] = s_C[nb + e]; }
            float accv[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const int pv = (lw * NV + v) * 4 + (ll >> 4);
                const float xpv = s_x[hh * HP + pv];
                float svv[8];
                unpack8(st[buf][v], svv);
                float a = 0.f;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float sn = svv[e] * dA + Bv[e] * xpv;
                    svv[e] = sn;
                    a += sn * Cv[e];
                }
                accv[v] = a;
                mb_st_state(ssw + ((size_t)r * nh + h) * HP * DS + st_off(v), pack8(svv));
            }
            if (hh + PD < HG) load_state(hh + PD, buf);
#pragma unroll
            for (int v = 0; v < NV; ++v) {         // sum over the row's 16 lanes (DPP rotations)
                float a = accv[v];
                a += row_ror<8>(a);
                a += row_ror<4>(a);
                a += row_ror<2>(a);
                a += row_ror<1>(a);
                const int pv = (lw * NV + v) * 4 + (ll >> 4);
                if ((ll & 15) == 0) {
                    const float y = round_bf(a + s_x[hh * HP + pv] * Dv[h]);
                    const float zz = s_z[hh * HP + pv];
                    yz[(size_t)r * di + h * HP + pv] = y * (zz * (1.0f / (1.0f + expf(-zz))));
                }
            }
            continue;
        }
        const float xp = s_x[hh * HP + p];
        bf16_t* sp = ssw + (((size_t)r * nh + h) * HP + p) * DS + n0;
        float acc = 0.f;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            float svv[8];
            unpack8(st[buf][v], svv);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int n = n0 + 8 * v + e;
                const float s = svv[e] * dA + (s_B[n] * dt) * xp;
                svv[e] = s;
                acc += s * s_C[n];
            }
            mb_st_state(sp + 8 * v, pack8(svv));
        }
        if (hh + PD < HG) load_state(hh + PD, buf);
#pragma unroll
        for (int off = 1; off < TPP; off <<= 1) acc += __shfl_xor(acc, off, 64);
        if (t % TPP == 0) {
            const float y = round_bf(acc + xp * Dv[h]);
            const float zz = s_z[hh * HP + p];
            yz[(size_t)r * di + h * HP + p] = y * (zz * (1.0f / (1.0f + expf(-zz))));
        }
    }
}

// prefill conv: xc[r][t][ch] = bf16(silu(b + sum_k w[k] in[t-3+k])), in = bf16(in_proj xBC column);
// final_state[r][ch] = last 4 inputs (zero-padded) -> the buffer the first decode step reads
__global__ __launch_bounds__(MB_THREADS) void k_mamba_conv_seq(const float* __restrict__ zx, int S, int di, int ds,
                                                               int nh, const float* __restrict__ conv_w,
                                                               const float* __restrict__ conv_b,
                                                               bf16_t* __restrict__ xc, bf16_t* __restrict__ cs) {
    const int conv_dim = di + 2 * ds, ncol = 2 * di + 2 * ds + nh;
    const int r = blockIdx.y;
    const long idx = (long)blockIdx.x * MB_THREADS + threadIdx.x;
    if (idx >= (long)(S + 1) * conv_dim) return;
    const int ch = (int)(idx % conv_dim);
    const int t = (int)(idx / conv_dim);
    const float* base = zx + (size_t)r * S * ncol + di + ch;
    auto in = [&](int u) -> float { return (u >= 0 && u < S) ? round_bf(base[(size_t)u * ncol]) : 0.f; };
    if (t < S) {
        const float* w = conv_w + (size_t)ch * 4;
        float acc = conv_b[ch];
        acc += w[0] * in(t - 3);
        acc += w[1] * in(t - 2);
        acc += w[2] * in(t - 1);
        acc += w[3] * in(t);
        xc[((size_t)r * S + t) * conv_dim + ch] = f2bf(silu_f(acc));
    } else {
        const uint32_t lo = (uint32_t)f2bf(in(S - 4)) | ((uint32_t)f2bf(in(S - 3)) << 16);
        const uint32_t hi = (uint32_t)f2bf(in(S - 2)) | ((uint32_t)f2bf(in(S - 1)) << 16);
        *reinterpret_cast<uint2*>(cs + ((size_t)r * conv_dim + ch) * 4) = make_uint2(lo, hi);
    }
}

template <int HP, int DS>
__global__ __launch_bounds__(MB_THREADS) void k_mamba_scan(const float* __restrict__ zx, const bf16_t* __restrict__ xc,
                                                           int S, int di, int nh, const float* __restrict__ A,
                                                           const float* __restrict__ dt_bias,
                                                           const float* __restrict__ Dv, bf16_t* __restrict__ ssm,
                                                           float* __restrict__ yz) {
    constexpr int TPP = MB_THREADS / HP, EPT = DS / TPP, TC = 16;
    __shared__ float s_x[TC][HP], s_z[TC][HP], s_B[TC][DS], s_C[TC][DS], s_dt[TC];
    const int h = blockIdx.x, r = blockIdx.y;
    const int conv_dim = di + 2 * DS, ncol = 2 * di + 2 * DS + nh;
    const int t = threadIdx.x, p = t / TPP, n0 = (t % TPP) * EPT;
    const float Ah = A[h], dtb = dt_bias[h], Dh = Dv[h];
    float st[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) st[e] = 0.f;
    for (int c0 = 0; c0 < S; c0 += TC) {
        const int nt = min(TC, S - c0);
        __syncthreads();
        for (int i = threadIdx.x; i < nt * (2 * HP + 2 * DS + 1); i += MB_THREADS) {
            const int tt = i / (2 * HP + 2 * DS + 1), k = i % (2 * HP + 2 * DS + 1);
            const size_t row = (size_t)r * S + c0 + tt;
            const bf16_t* xr = xc + row * conv_dim;
            if (k < HP) s_x[tt][k] = bf2f(xr[h * HP + k]);
            else if (k < HP + DS) s_B[tt][k - HP] = bf2f(xr[di + (k - HP)]);
            else if (k < HP + 2 * DS) s_C[tt][k - HP - DS] = bf2f(xr[di + DS + (k - HP - DS)]);
            else if (k < 2 * HP + 2 * DS) s_z[tt][k - HP - 2 * DS] = round_bf(zx[row * ncol + h * HP + (k - HP - 2 * DS)]);
            else s_dt[tt] = round_bf(zx[row * ncol + 2 * di + 2 * DS + h]);
        }
        __syncthreads();
        for (int tt = 0; tt < nt; ++tt) {
            const float dt = softplus_thr(s_dt[tt] + dtb);
            const float dA = expf(dt * Ah);
            const float xp = s_x[tt][p];
            float acc = 0.f;
#pragma unroll
            for (int e = 0; e < EPT; ++e) {
                const int n = n0 + e;
                st[e] = st[e] * dA + (s_B[tt][n] * dt) * xp;
                acc += st[e] * s_C[tt][n];
            }
#pragma unroll
            for (int off = 1; off < TPP; off <<= 1) acc += __shfl_xor(acc, off, 64);
            if (t % TPP == 0) {
                const float y = round_bf(acc + xp * Dh);
                const float zz = s_z[tt][p];
                yz[((size_t)r * S + c0 + tt) * di + h * HP + p] = y * (zz * (1.0f / (1.0f + expf(-zz))));
            }
        }
    }
    bf16_t* sp = ssm + (((size_t)r * nh + h) * HP + p) * DS + n0;
#pragma unroll
    for (int e8 = 0; e8 < EPT; e8 += 8) *reinterpret_cast<uint4*>(sp + e8) = pack8(st + e8);
}

__global__ __launch_bounds__(MB_THREADS) void k_gated_norm(const float* __restrict__ g, int di,
                                                           const float* __restrict__ w, float eps,
                                                           bf16_t* __restrict__ out, const int32_t* __restrict__ skip) {
    __shared__ float red[MB_THREADS / 64];
    if (!ZK_MB_DEFER || di > GN_MAXJ * MB_THREADS)
        if (skip && *skip) return;
    const int row = blockIdx.x;
    const float* gr = g + (size_t)row * di;
    if (di <= GN_MAXJ * MB_THREADS) {
        // the row's values and weights loaded together up front (one memory round trip), summed in
        // the same per-thread order as the strided loop below
        float gv[GN_MAXJ], wv[GN_MAXJ];
#pragma unroll
        for (int k = 0; k < GN_MAXJ; ++k) {
            const int j = threadIdx.x + k * MB_THREADS;
            gv[k] = j < di ? gr[j] : 0.f;
            wv[k] = j < di ? w[j] : 0.f;
        }
        if constexpr (ZK_MB_DEFER) {
            if (ld_word_here(skip)) {        // the step word after the row's loads (in bounds)
#pragma unroll
                for (int k = 0; k < GN_MAXJ; ++k) asm volatile("" ::"v"(gv[k]), "v"(wv[k]));
                return;
            }
        }
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < GN_MAXJ; ++k)
            if (threadIdx.x + k * MB_THREADS < di) s += gv[k] * gv[k];
        s = block_sum<MB_THREADS>(s, red);
        const float rstd = 1.0f / sqrtf(s / (float)di + eps);
#pragma unroll
        for (int k = 0; k < GN_MAXJ; ++k) {
            const int j = threadIdx.x + k * MB_THREADS;
            if (j < di) out[(size_t)row * di + j] = f2bf((gv[k] * rstd) * wv[k]);
        }
        return;
    }
    float s = 0.f;
    for (int j = threadIdx.x; j < di; j += MB_THREADS) s += gr[j] * gr[j];
    s = block_sum<MB_THREADS>(s, red);
    const float rstd = 1.0f / sqrtf(s / (float)di + eps);
    for (int j = threadIdx.x; j < di; j += MB_THREADS) out[(size_t)row * di + j] = f2bf((gr[j] * rstd) * w[j]);
}

}  // namespace

#define ZK_MB_DISPATCH(HP_, DS_, CALL)                                                     \
    if (hp == HP_ && ds == DS_) { CALL(HP_, DS_); handled = true; }

namespace {

// grouped = true: ZK_MB_HG heads per workgroup (default 1, the fastest measured; B/C conv once per
// group), in_proj splits 1 / 2 / 4. grouped = false: one workgroup per (head, row), any split.
int mamba_step(bool grouped, const float* part, int gemm_nsplit, int R, int d_inner, int nheads, int headdim,
               int d_state, const float* conv_w, const float* conv_b, void* conv_state_a, void* conv_state_b,
               const int32_t* pos_dev, void* ssm_state, void* ssm_state_b, const float* A, const float* dt_bias,
               const float* D, float* yz, const int32_t* skip, void* stream) {
    const int hp = headdim, ds = d_state;
    ZK_REQUIRE(gemm_nsplit >= 1 && gemm_nsplit <= MB_MAXGS, "zk_mamba_step: gemm_nsplit=%d", gemm_nsplit);
    ZK_REQUIRE(nheads * headdim == d_inner, "zk_mamba_step: nheads*headdim != d_inner");
    bool handled = false;
    if (grouped && nheads % ZK_MB_HG == 0 && (gemm_nsplit == 1 || gemm_nsplit == 2 || gemm_nsplit == 4)) {
#define ZK_MB_STEPG(HP_, DS_)                                                                                       \
    do {                                                                                                           \
        const dim3 g_(nheads / ZK_MB_HG, R);                                                                              \
        if (gemm_nsplit == 1)                                                                                      \
            hipLaunchKernelGGL((k_mamba_step_g<HP_, DS_, ZK_MB_HG, 1>), g_, dim3(MB_THREADS), 0, (hipStream_t)stream,     \
                               part, R, d_inner, nheads, conv_w, conv_b, (const bf16_t*)conv_state_a,             \
                               (bf16_t*)conv_state_b, pos_dev, (bf16_t*)ssm_state, (bf16_t*)ssm_state_b, A, dt_bias, D, yz, skip);      \
        else if (gemm_nsplit == 2)                                                                                 \
            hipLaunchKernelGGL((k_mamba_step_g<HP_, DS_, ZK_MB_HG, 2>), g_, dim3(MB_THREADS), 0, (hipStream_t)stream,     \
                               part, R, d_inner, nheads, conv_w, conv_b, (const bf16_t*)conv_state_a,             \
                               (bf16_t*)conv_state_b, pos_dev, (bf16_t*)ssm_state, (bf16_t*)ssm_state_b, A, dt_bias, D, yz, skip);      \
        else                                                                                                       \
            hipLaunchKernelGGL((k_mamba_step_g<HP_, DS_, ZK_MB_HG, 4>), g_, dim3(MB_THREADS), 0, (hipStream_t)stream,     \
                               part, R, d_inner, nheads, conv_w, conv_b, (const bf16_t*)conv_state_a,             \
                               (bf16_t*)conv_state_b, pos_dev, (bf16_t*)ssm_state, (bf16_t*)ssm_state_b, A, dt_bias, D, yz, skip);      \
    } while (0)
        ZK_MB_DISPATCH(64, 128, ZK_MB_STEPG)
        ZK_MB_DISPATCH(32, 64, ZK_MB_STEPG)
        ZK_MB_DISPATCH(64, 64, ZK_MB_STEPG)
#undef ZK_MB_STEPG
        if (handled) {
            ZK_CHECK_LAUNCH("zk_mamba_step");
            return 0;
        }
    }
#define ZK_MB_STEP(HP_, DS_)                                                                                       \
    hipLaunchKernelGGL((k_mamba_step<HP_, DS_>), dim3(nheads, R), dim3(MB_THREADS), 0, (hipStream_t)stream, part,  \
                       gemm_nsplit, R, d_inner, nheads, conv_w, conv_b, (const bf16_t*)conv_state_a,                \
                       (bf16_t*)conv_state_b, pos_dev, (bf16_t*)ssm_state, (bf16_t*)ssm_state_b, A, dt_bias, D, yz, skip)
    ZK_MB_DISPATCH(64, 128, ZK_MB_STEP)
    ZK_MB_DISPATCH(32, 64, ZK_MB_STEP)
    ZK_MB_DISPATCH(64, 64, ZK_MB_STEP)
#undef ZK_MB_STEP
    ZK_REQUIRE(handled, "zk_mamba_step: (headdim %d, d_state %d) not instantiated", hp, ds);
    ZK_CHECK_LAUNCH("zk_mamba_step");
    return 0;
}

}  // namespace

extern "C" int zk_mamba_step(const float* part, int gemm_nsplit, int R, int d_inner, int nheads, int headdim,
                             int d_state, const float* conv_w, const float* conv_b, void* conv_state_a,
                             void* conv_state_b, const int32_t* pos_dev, void* ssm_state, void* ssm_state_b,
                             const float* A, const float* dt_bias, const float* D, float* yz, const int32_t* skip,
                             void* stream) {
    return mamba_step(true, part, gemm_nsplit, R, d_inner, nheads, headdim, d_state, conv_w, conv_b, conv_state_a,
                      conv_state_b, pos_dev, ssm_state, ssm_state_b, A, dt_bias, D, yz, skip, stream);
}

extern "C" int zk_mamba_step_per_head(const float* part, int gemm_nsplit, int R, int d_inner, int nheads,
                                      int headdim, int d_state, const float* conv_w, const float* conv_b,
                                      void* conv_state_a, void* conv_state_b, const int32_t* pos_dev, void* ssm_state,
                                      void* ssm_state_b, const float* A, const float* dt_bias, const float* D,
                                      float* yz, const int32_t* skip, void* stream) {
    return mamba_step(false, part, gemm_nsplit, R, d_inner, nheads, headdim, d_state, conv_w, conv_b, conv_state_a,
                      conv_state_b, pos_dev, ssm_state, ssm_state_b, A, dt_bias, D, yz, skip, stream);
}

extern "C" int zk_mamba_prefill(const float* zx, int R, int S, int d_inner, int nheads, int headdim, int d_state,
                                const float* conv_w, const float* conv_b, void* xc_scratch, void* conv_state,
                                void* ssm_state, const float* A, const float* dt_bias, const float* D, float* yz,
                                void* stream) {
    const int hp = headdim, ds = d_state;
    ZK_REQUIRE(nheads * headdim == d_inner && S >= 1, "zk_mamba_prefill: bad shape");
    const int conv_dim = d_inner + 2 * d_state;
    const long n = (long)(S + 1) * conv_dim;
    hipLaunchKernelGGL(k_mamba_conv_seq, dim3((unsigned)((n + MB_THREADS - 1) / MB_THREADS), R), dim3(MB_THREADS), 0,
                       (hipStream_t)stream, zx, S, d_inner, d_state, nheads, conv_w, conv_b, (bf16_t*)xc_scratch,
                       (bf16_t*)conv_state);
    ZK_CHECK_LAUNCH("zk_mamba_prefill/conv");
    bool handled = false;
#define ZK_MB_SCAN(HP_, DS_)                                                                                      \
    hipLaunchKernelGGL((k_mamba_scan<HP_, DS_>), dim3(nheads, R), dim3(MB_THREADS), 0, (hipStream_t)stream, zx,   \
                       (const bf16_t*)xc_scratch, S, d_inner, nheads, A, dt_bias, D, (bf16_t*)ssm_state, yz)
    ZK_MB_DISPATCH(64, 128, ZK_MB_SCAN)
    ZK_MB_DISPATCH(32, 64, ZK_MB_SCAN)
    ZK_MB_DISPATCH(64, 64, ZK_MB_SCAN)
#undef ZK_MB_SCAN
    ZK_REQUIRE(handled, "zk_mamba_prefill: (headdim %d, d_state %d) not instantiated", hp, ds);
    ZK_CHECK_LAUNCH("zk_mamba_prefill/scan");
    return 0;
}

extern "C" int zk_gated_rmsnorm(const float* g, int rows, int d_inner, const float* w, float eps, void* out,
                                const int32_t* skip, void* stream) {
    ZK_REQUIRE(rows >= 0 && d_inner > 0, "zk_gated_rmsnorm: bad shape");
    if (rows == 0) return 0;
    hipLaunchKernelGGL(k_gated_norm, dim3(rows), dim3(MB_THREADS), 0, (hipStream_t)stream, g, d_inner, w, eps,
                       (bf16_t*)out, skip);
    ZK_CHECK_LAUNCH("zk_gated_rmsnorm");
    return 0;
}
