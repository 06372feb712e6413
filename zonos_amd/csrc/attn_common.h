// Decode-attention building blocks shared by k_attn_decode (backbone.hip) and the persistent
// small-batch decode step (step_small.hip): KV cache layout, RoPE pair mapping, the 32-key MFMA
// step and the whole-workgroup flash-decoding body (attn_decode_wg).
#pragma once
#include "common.h"

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

// ------------------------------------------------------------------ in_proj epilogue
// RoPE pair j (0..hd/2-1) of a head: interleaved (_torch.py:18-30: dims 2j, 2j+1) or, NEOX,
// GPT-NeoX "rotate half" (flash_attn apply_rotary, interleaved=False: dims j, j + hd/2).
// Both use (cos, sin) entry j of the position's [hd/2][2] table.
template <bool NEOX>
ZK_DEV void rope_dims(int j, int hd, int& d0, int& d1) {
    d0 = NEOX ? j : 2 * j;
    d1 = NEOX ? j + hd / 2 : 2 * j + 1;
}

// ------------------------------------------------------------------ decode attention
#ifndef ZK_ATT_TRIM
#define ZK_ATT_TRIM 1      // per-wave key-slice trimming (0: whole 128-key blocks, clamped tail load)
#endif
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
// sum of the in_proj split-K slabs of one RoPE pair (d0, d1) of a column block, left to right
// in fp32 like k_qkv_rope: every slab load issued before the first add
template <int NS, bool NEOX>
ZK_DEV void slab_pair(const float* p, size_t slab, int d0, int d1, float& a, float& b) {
    float v0[NS], v1[NS];
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
        if constexpr (NEOX) {
            v0[sl] = p[sl * slab + d0];
            v1[sl] = p[sl * slab + d1];
        } else {                                      // interleaved pair: d1 = d0 + 1, d0 even
            const float2 t = *reinterpret_cast<const float2*>(p + sl * slab + d0);
            v0[sl] = t.x;
            v1[sl] = t.y;
        }
    }
    a = v0[0];
    b = v1[0];
#pragma unroll
    for (int sl = 1; sl < NS; ++sl) { a += v0[sl]; b += v1[sl]; }
}
ZK_DEV void slab_pair_n(const float* p, size_t slab, int ns, int d0, int d1, float& a, float& b) {
    float v0[AT_MAXGS], v1[AT_MAXGS];
#pragma unroll
    for (int sl = 0; sl < AT_MAXGS; ++sl) {
        const float* ps = p + (size_t)min(sl, ns - 1) * slab;
        v0[sl] = ps[d0];
        v1[sl] = ps[d1];
    }
    a = v0[0];
    b = v1[0];
#pragma unroll
    for (int sl = 1; sl < AT_MAXGS; ++sl)
        if (sl < ns) { a += v0[sl]; b += v1[sl]; }
}

// ZK_ATT_PROF (profiling builds only): thread 0 of each workgroup writes s_memrealtime stamps
// [entry, loads issued, prologue done, key loop done, merged, end] to prof[wg * 8 + k].
// The pointer is read once, at the top of the kernel (ZK_ATT_PROF_PTR, by a scalar load before any data
// load), so a stamp is a register-sourced store: re-reading the global at each stamp put a vector load
// behind the key blocks in flight, and the wait for it drained them (the stamps moved the kernel).
#ifdef ZK_ATT_PROF
__device__ uint64_t* g_att_prof;
#define ZK_ATT_PROF_PTR                                                                                     \
    uint64_t* const zk_pp = reinterpret_cast<uint64_t*>(                                                    \
        (uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)reinterpret_cast<uintptr_t>(g_att_prof)) | \
        ((uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(reinterpret_cast<uintptr_t>(g_att_prof) >> 32)) << 32))
#define ZK_ATT_STAMP(k)                                                                                     \
    do {                                                                                                    \
        if (threadIdx.x == 0 && zk_pp)                                                                      \
            zk_pp[((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 8 + (k)] =               \
                __builtin_amdgcn_s_memrealtime();                                                           \
    } while (0)
// slots 6 / 7: HW_ID and XCC_ID of the workgroup's wave 0 (where it ran)
#define ZK_ATT_HWID()                                                                                       \
    do {                                                                                                    \
        if (threadIdx.x == 0 && zk_pp) {                                                                    \
            const size_t b_ = ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 8;          \
            zk_pp[b_ + 6] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);                              \
            zk_pp[b_ + 7] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);                             \
        }                                                                                                   \
    } while (0)
#else
#define ZK_ATT_PROF_PTR do {} while (0)
#define ZK_ATT_STAMP(k) do {} while (0)
#define ZK_ATT_HWID() do {} while (0)
#endif

// LDS of one attention workgroup (4 waves)
struct __attribute__((aligned(16))) AttnSmem {
    float s_o[4][AT_G][128];
    uint32_t s_q[AT_G][64];
    uint32_t s_kn[64];       // new key (post-RoPE), bf16 pairs
    float s_m[4][16];
    float s_l[4][16];
    uint16_t s_vn[128];      // new value
    int s_last;              // COMB: this workgroup merges
};

// One workgroup of 4 waves (threads 0..255) = one (split, kv head g, row r). `bar` is the barrier
// among those 4 waves (__syncthreads in k_attn_decode); `issued` runs right after the first key
// blocks' loads are in flight and before anything reads the in_proj output or writes anything:
// it returns true when the launch is to be skipped (generation finished).
// PGS > 0 (FUSED, exactly PGS in_proj slabs): the prologue's slab loads are issued FIRST, then the context
// word is waited for, then the RoPE row and the first key blocks are requested: the prologue then waits only
// for its own (older) loads while the key blocks stream, instead of for everything (vmcnt retires in issue
// order), and the key loop starts while the early key blocks are still arriving.
template <bool FUSED, bool NEOX, bool KVNT, bool COMB, int PGS, class Bar, class Issued>
ZK_DEV void attn_decode_wg(AttnSmem& sm, const Bar& bar, const Issued& issued, int split, int nsplit, int g, int r,
                           const bf16_t* q, bf16_t* kc, bf16_t* vt, int R, int H, int Hkv, int Smax, int ctx0,
                           int cwr, float* work, float scale, bf16_t* out, const float* part, int gsplit,
                           const float* freqs, uint32_t* cnt) {
    constexpr int HD = 128;
    ZK_ATT_PROF_PTR;
    ZK_ATT_STAMP(0);
    static_assert(PGS == 0 || FUSED, "slab pre-loads: the fused prologue");
    constexpr int NPI = 2;                       // prologue pairs per thread: (G + 2) * 64 <= 384 <= 2 * 256
    static_assert((AT_G + 2) * (HD / 2) <= NPI * 256, "prologue pairs per thread");
    float2 psl[PGS > 0 ? NPI : 1][PGS > 0 ? PGS : 1];
    float2 pcs[PGS > 0 ? NPI : 1];
    if constexpr (PGS > 0) {
        const int N = (H + 2 * Hkv) * HD;
        const size_t slab = (size_t)R * N;
        const float* prow = part + (size_t)r * N;
        const int Gq = H / Hkv;
#pragma unroll
        for (int it = 0; it < NPI; ++it) {
            const int pi = min((int)threadIdx.x + 256 * it, (Gq + 2) * (HD / 2) - 1);
            const int hp = pi / (HD / 2), j = pi % (HD / 2);
            int d0, d1;
            rope_dims<NEOX>(j, HD, d0, d1);
            const int cb = hp < Gq ? (g * Gq + hp) * HD : (hp == Gq ? H * HD + g * HD : (H + Hkv) * HD + g * HD);
#pragma unroll
            for (int sl = 0; sl < PGS; ++sl) {
                if constexpr (NEOX) psl[it][sl] = make_float2(prow[cb + sl * slab + d0], prow[cb + sl * slab + d1]);
                else psl[it][sl] = *reinterpret_cast<const float2*>(prow + cb + sl * slab + d0);
            }
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    }
    const int ctx = min(ctx0 + uni(cwr), Smax);
    if constexpr (PGS > 0) {
        const float* fc = freqs + (size_t)(ctx - 1) * HD;
#pragma unroll
        for (int it = 0; it < NPI; ++it) {
            const int pi = min((int)threadIdx.x + 256 * it, (H / Hkv + 2) * (HD / 2) - 1);
            pcs[it] = *reinterpret_cast<const float2*>(fc + 2 * (pi % (HD / 2)));
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    }
    auto& s_m = sm.s_m;
    auto& s_l = sm.s_l;
    auto& s_o = sm.s_o;
    auto& s_q = sm.s_q;
    auto& s_kn = sm.s_kn;
    auto& s_vn = sm.s_vn;
    auto& s_last = sm.s_last;
    const int nkb = (ctx + AT_KB - 1) / AT_KB;
    const int kb0 = (int)((long)split * nkb / nsplit), kb1 = (int)((long)(split + 1) * nkb / nsplit);
    const int G = H / Hkv;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ln = lane & 15, lg = lane >> 4;
    bf16_t* kb = kc + ((size_t)r * Hkv + g) * Smax * HD;
    bf16_t* vb = vt + ((size_t)r * Hkv + g) * HD * (size_t)Smax;

    bf16x8 qf[4];
    KVFrag fa, fb;
#if ZK_ATT_TRIM
    // This wave's 32-key slice of block b holds keys b*128 + 32w ..: it loads and multiplies only
    // the blocks whose slice holds a visible key (b*128 + 32w < ctx) and never re-loads the last
    // one. (Reading whole 128-key blocks plus a clamped tail prefetch fetched 11 % more than the
    // algorithmic bytes at ctx 1705; a fully masked slice adds exactly nothing to (m, l, O).)
    const int vis = ctx - 32 * w;
    const int kbw = vis <= 0 ? kb0 : max(kb0, min(kb1, (vis + AT_KB - 1) / AT_KB));
#else
    const int kbw = kb1;
#endif
    const int last = kbw - 1;
    // the first key block can be fetched before the prologue unless it holds the new key
    // FUSED: the new key's cache lines are written only at the end of the kernel (a store
    // followed by loads of the same partially written lines stalls the key loop); the key loop
    // patches the new K/V into its registers from LDS instead, so the arithmetic is exactly
    // that of reading the cache. The first key block can therefore be fetched before the prologue.
    const int pos = ctx - 1;
    // (PGS > 0: both blocks unconditionally, clamped into the cache -- straight-line loads, so the prologue's
    // wait for its older slab loads is exact and leaves these in flight; an unused block costs 32 KB)
    const bool early = FUSED && (PGS > 0 || kbw > kb0);
    if (early) {      // the first TWO key blocks are in flight during the prologue
        load_kv<KVNT>(fa, kb, vb, Smax, kb0 * AT_KB + 32 * w, ln, lg);
        if (PGS > 0 || !ZK_ATT_TRIM || kb0 + 1 < kbw)
            load_kv<KVNT>(fb, kb, vb, Smax, min(kb0 + 1, max(last, kb0)) * AT_KB + 32 * w, ln, lg);
    }
    if (issued()) {          // skip: nothing is written (the loads above are in bounds)
        if constexpr (PGS > 0) {
#pragma unroll
            for (int it = 0; it < NPI; ++it) {
                asm volatile("" ::"v"(pcs[it].x), "v"(pcs[it].y));
#pragma unroll
                for (int sl = 0; sl < PGS; ++sl) asm volatile("" ::"v"(psl[it][sl].x), "v"(psl[it][sl].y));
            }
        }
        if (early) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) { keep_live(fa.k[h][ks]); keep_live(fb.k[h][ks]); }
#pragma unroll
            for (int dt = 0; dt < 8; ++dt) { keep_live(fa.v[dt]); keep_live(fb.v[dt]); }
        }
        return;
    }
    ZK_ATT_STAMP(1);
    if constexpr (FUSED) {
        // pairs: [0, G*64) q of heads g*G.., then 64 k pairs, then 64 v pairs
        const int N = (H + 2 * Hkv) * HD;
        const size_t slab = (size_t)R * N;
        const float* prow = part + (size_t)r * N;
        const float* fc = freqs + (size_t)pos * HD;
        uint16_t* q16 = reinterpret_cast<uint16_t*>(&s_q[0][0]);
        uint16_t* k16 = reinterpret_cast<uint16_t*>(s_kn);
        if constexpr (PGS > 0) {
#pragma unroll
            for (int it = 0; it < NPI; ++it) {
                const int pi = threadIdx.x + 256 * it;
                if (pi >= (G + 2) * (HD / 2)) break;
                const int hp = pi / (HD / 2), j = pi % (HD / 2);
                int d0, d1;
                rope_dims<NEOX>(j, HD, d0, d1);
                float a = psl[it][0].x, bb = psl[it][0].y;          // slab_pair's left-to-right sum
#pragma unroll
                for (int sl = 1; sl < PGS; ++sl) { a += psl[it][sl].x; bb += psl[it][sl].y; }
                const float2 cs = pcs[it];
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
        }
        for (int pi = PGS > 0 ? (G + 2) * (HD / 2) : threadIdx.x; pi < (G + 2) * (HD / 2); pi += 256) {
            const int hp = pi / (HD / 2), j = pi % (HD / 2);      // hp < G: q head g*G+hp; G: k; G+1: v
            int d0, d1;
            rope_dims<NEOX>(j, HD, d0, d1);
            const int cb = hp < G ? (g * G + hp) * HD : (hp == G ? H * HD + g * HD : (H + Hkv) * HD + g * HD);
            // all slab loads issued together (clamped slab index, select after) -- same
            // left-to-right fp32 sum as k_qkv_rope
            // the slab count is dispatched to an exact-size instantiation (B <= 8: 1 slab, c3: 4),
            // so only real slabs are loaded (one 8-byte load per slab for the interleaved pair)
            float a, bb;
            switch (gsplit) {
                case 1: slab_pair<1, NEOX>(prow + cb, slab, d0, d1, a, bb); break;
                case 2: slab_pair<2, NEOX>(prow + cb, slab, d0, d1, a, bb); break;
                case 4: slab_pair<4, NEOX>(prow + cb, slab, d0, d1, a, bb); break;
                default: slab_pair_n(prow + cb, slab, gsplit, d0, d1, a, bb); break;
            }
            const float2 cs = *reinterpret_cast<const float2*>(fc + 2 * j);
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
        bar();      // q, new k, new v in LDS
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
    ZK_ATT_STAMP(2);
    AttnState st;
    st.m = -INFINITY;
    st.l = 0.f;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) st.o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (kbw > kb0) {
        if (!early) load_kv<KVNT>(fa, kb, vb, Smax, kb0 * AT_KB + 32 * w, ln, lg);
        for (int it = kb0; it < kbw; it += 2) {
            if (!(early && it == kb0) && (!ZK_ATT_TRIM || it + 1 < kbw))
                load_kv<KVNT>(fb, kb, vb, Smax, min(it + 1, last) * AT_KB + 32 * w, ln, lg);
            if (FUSED) patch_kv(fa, s_kn, s_vn, it * AT_KB + 32 * w, pos, ln, lg);
            attn_step(st, fa, qf, it * AT_KB + 32 * w, ctx, scale, lg);
            if (!ZK_ATT_TRIM || it + 2 < kbw) load_kv<KVNT>(fa, kb, vb, Smax, min(it + 2, last) * AT_KB + 32 * w, ln, lg);
            if (it + 1 < kbw) {
                if (FUSED) patch_kv(fb, s_kn, s_vn, (it + 1) * AT_KB + 32 * w, pos, ln, lg);
                attn_step(st, fb, qf, (it + 1) * AT_KB + 32 * w, ctx, scale, lg);
            }
        }
    }
    ZK_ATT_STAMP(3);
    if (FUSED && split == nsplit - 1) {      // the split owning the newest key stores it (cache for later steps)
        const int t = threadIdx.x;
        if (t < HD / 2) *reinterpret_cast<uint32_t*>(kb + k_off(pos, t >> 2) + ((2 * t) & 7)) = s_kn[t];
        else if (t < HD / 2 + HD) reinterpret_cast<uint16_t*>(vb)[v_off(pos, t - HD / 2)] = s_vn[t - HD / 2];
    }
    // merge the 4 waves
    if (lg == 0) { s_m[w][ln] = st.m; s_l[w][ln] = st.l; }
    bar();
    const float M = fmaxf(fmaxf(s_m[0][ln], s_m[1][ln]), fmaxf(s_m[2][ln], s_m[3][ln]));
    const float cw = (st.m == -INFINITY) ? 0.f : __expf(st.m - M);
    if (ln < AT_G) {
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) s_o[w][ln][dt * 16 + lg * 4 + i] = st.o[dt][i] * cw;
    }
    bar();
    ZK_ATT_STAMP(4);
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
        ZK_ATT_STAMP(5);
        ZK_ATT_HWID();
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
        bar();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // keep the fence's wait (ROCm 7.2)
            const uint32_t old = __hip_atomic_fetch_add(cnt + (size_t)r * Hkv + g, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            s_last = ((old + 1) % (uint32_t)nsplit) == 0;
        }
        bar();
        ZK_ATT_STAMP(5);
        if (!s_last) return;
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        ZK_ATT_STAMP(6);
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
        ZK_ATT_STAMP(7);
    }
}

// B = 1 decode attention over 32-key slices (zk_attn_decode_q_part): q comes from the in_proj GEMV's
// RoPE epilogue (zk_gemv_qkv_rope), which also wrote the new key / value into the cache, so there is no
// prologue: the q fragments and the step words are loaded at entry, the first slice as soon as the
// context is known. Workgroup (split, kv head g, row r), wave w takes the slices split * 4 + w + j * 4 *
// nsplit (interleaved, so every split gets an equal share at any context and all 4 * nsplit waves of a
// (row, kv head) start with one slice), two slices in flight; the 4 waves merge through LDS and the
// workgroup writes its (m, l, O) partial, which the out_proj GEMV merges (zk_gemv_attn_out).
template <bool KVNT>
__global__ __launch_bounds__(256, 2) void k_attn_decode_qs(const bf16_t* q, const bf16_t* kc, const bf16_t* vt,
                                                           int H, int Hkv, int Smax, int ctx0, const int32_t* ctx_dev,
                                                           float* work, float scale, const int32_t* skip) {
    constexpr int HD = 128;
    ZK_ATT_PROF_PTR;
    __shared__ AttnSmem sm;
    const int split = blockIdx.x, nsplit = gridDim.x, g = blockIdx.y, r = blockIdx.z;
    const int G = H / Hkv;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ln = lane & 15, lg = lane >> 4;
    ZK_ATT_STAMP(0);
    const int sk = ld_word(skip);
    const int cw = ld_word(ctx_dev);
    // q fragments (B operand of S^T = K.Q^T: lane ln < G holds head g*G + ln), independent of the context
    const bf16_t* qr = q + (size_t)r * H * HD + (size_t)(g * G + min(ln, G - 1)) * HD;
    uint4 qv[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qv[ks] = *reinterpret_cast<const uint4*>(qr + ks * 32 + lg * 8);
    const bf16_t* kb = kc + ((size_t)r * Hkv + g) * Smax * HD;
    const bf16_t* vb = vt + ((size_t)r * Hkv + g) * HD * (size_t)Smax;
    const int step = 4 * nsplit;
    const int s0 = split * 4 + w;
    // the wave's first slice is loaded before the context is known (in bounds: clamped to the cache;
    // unused when the context ends before it), so the context word's round trip overlaps it
    // (loading its second slice speculatively as well measured slower: the CU's load issue, 64 KB per
    // workgroup and slice, then holds back the context word's test, profiles/r6_c2_attn_stamps.txt)
    KVFrag fa, fb;
    load_kv<KVNT>(fa, kb, vb, Smax, min(s0, Smax / 32 - 1) * 32, ln, lg);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);       // (the wait for the context word below, not above these loads)
    const int ctx = min(ctx0 + uni(cw), Smax);
    ZK_ATT_STAMP(1);
    const int nsl = (ctx + 31) >> 5;
    if (s0 + step < nsl) load_kv<KVNT>(fb, kb, vb, Smax, (s0 + step) * 32, ln, lg);
    if (uni(sk) != 0) {        // skip: nothing is written (the loads above are in bounds)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) { keep_live(fa.k[h][ks]); keep_live(fb.k[h][ks]); }
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) { keep_live(fa.v[dt]); keep_live(fb.v[dt]); }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) keep_live(qv[ks]);
        return;
    }
    bf16x8 qf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[ks] = as_frag(ln < G ? qv[ks] : make_uint4(0, 0, 0, 0));
    AttnState st;
    st.m = -INFINITY;
    st.l = 0.f;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) st.o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = s0; s < nsl; s += 2 * step) {
        attn_step(st, fa, qf, s * 32, ctx, scale, lg);
        if (s == s0) ZK_ATT_STAMP(2);
        if (s + 2 * step < nsl) load_kv<KVNT>(fa, kb, vb, Smax, (s + 2 * step) * 32, ln, lg);
        if (s + step < nsl) {
            attn_step(st, fb, qf, (s + step) * 32, ctx, scale, lg);
            if (s + 3 * step < nsl) load_kv<KVNT>(fb, kb, vb, Smax, (s + 3 * step) * 32, ln, lg);
        }
    }
    ZK_ATT_STAMP(3);
    // merge the 4 waves with one barrier: each wave leaves its unscaled (m, l, O) in LDS and every thread
    // combines its (head, dim) items -- the products and the wave order of attn_decode_wg's two-barrier
    // merge (O_w * exp(m_w - M), summed w = 0..3), so the same numbers
    if (lg == 0) { sm.s_m[w][ln] = st.m; sm.s_l[w][ln] = st.l; }
    if (ln < AT_G) {
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) sm.s_o[w][ln][dt * 16 + lg * 4 + i] = st.o[dt][i];
    }
    __syncthreads();
    ZK_ATT_STAMP(4);
    float* wp = work + (((size_t)r * Hkv + g) * nsplit + split) * AT_STR;
    for (int i = threadIdx.x; i < AT_G * HD; i += 256) {
        const int h = i / HD, d = i % HD;
        const float Mh = fmaxf(fmaxf(sm.s_m[0][h], sm.s_m[1][h]), fmaxf(sm.s_m[2][h], sm.s_m[3][h]));
        float o = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float c = (sm.s_m[k][h] == -INFINITY) ? 0.f : __expf(sm.s_m[k][h] - Mh);
            o = k == 0 ? sm.s_o[0][h][d] * c : o + sm.s_o[k][h][d] * c;
        }
        wp[2 * AT_G + i] = o;
    }
    if (threadIdx.x < AT_G) {
        const int h = threadIdx.x;
        float Mh = -INFINITY;
        for (int k = 0; k < 4; ++k) Mh = fmaxf(Mh, sm.s_m[k][h]);
        float L = 0.f;
        for (int k = 0; k < 4; ++k) L += (sm.s_m[k][h] == -INFINITY) ? 0.f : sm.s_l[k][h] * __expf(sm.s_m[k][h] - Mh);
        wp[h] = Mh;
        wp[AT_G + h] = L;
    }
    ZK_ATT_STAMP(5);
}

template <bool FUSED, bool NEOX, bool KVNT, bool COMB = false, int PGS = 0>
__global__ __launch_bounds__(256, 2) void k_attn_decode(const bf16_t* q, bf16_t* kc, bf16_t* vt, int R, int H,
                                                        int Hkv, int Smax, int ctx0, const int32_t* ctx_dev,
                                                        float* work, float scale, bf16_t* out, const int32_t* skip,
                                                        const float* part, int gsplit, const float* freqs,
                                                        uint32_t* cnt = nullptr) {
    __shared__ AttnSmem sm;
    // both step scalars in one round trip; the skip word is tested once the first key blocks'
    // loads are in flight (issued -> return), so its latency overlaps theirs
    const int sk = ld_word(skip);
    // (the context is clamped to the cache: a skipped launch after the last step may see ctx = Smax + 1,
    // and its first key blocks are loaded before the skip test; every real step has ctx <= Smax)
    const int cwr = ld_word(ctx_dev);
    attn_decode_wg<FUSED, NEOX, KVNT, COMB, PGS>(sm, [] { __syncthreads(); }, [sk] { return uni(sk) != 0; },
                                                blockIdx.x, gridDim.x, blockIdx.y, blockIdx.z, q, kc, vt, R, H, Hkv,
                                                Smax, ctx0, cwr, work, scale, out, part, gsplit, freqs, cnt);
}

}  // namespace
