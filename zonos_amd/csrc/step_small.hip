// Persistent small-batch decode step (B <= 2: R = 2B <= 4 rows with CFG) for gfx950.
//
// At batch 1 a decode step is a chain of ~130 dependent weight-streaming launches (3.2 GB of
// weights, 5 per layer); each launch pays a ramp-up and a drain during which HBM idles, and the
// attention launch streams almost nothing. Here the whole backbone + heads of one step is ONE
// launch of one workgroup per CU:
//
//   * wave 4 (the loader) streams this CU's share of every layer's weights, in the order the
//     step consumes them, through an 8-slot LDS ring (16 KB per slot = 16 k-steps of one
//     16-column fragment-packed tile) by LDS-DMA. The weights do not depend on the activations,
//     so the loader runs ahead across every data dependency, limited only by free slots;
//   * waves 0-3 (consumers) walk the same schedule: for each layer phase they wait until every
//     CU has finished the previous phase (agent-scope counters, one per XCD shard, release /
//     acquire), stage the phase's activation rows in LDS (with the residual add and LayerNorm
//     recomputed redundantly per CU from the K-quarter partials -- no extra hand-off), and
//     multiply the landed slots on MFMA 16x16x32 (rows = batch, columns = the tile).
//
// Phases per layer (zonos/backbone/_torch.py:99-102,117-152):
//   IN : x_new = x + bf16(fc2 of the previous layer), LN1 -> in_proj K-quarter partials
//   ATT: the fused decode attention of k_attn_decode (attn_decode_wg: in_proj quarters reduced,
//        RoPE, KV write, flash-decoding over the cache), one unit per (row, kv head)
//   OUT: out_proj K-quarter partials
//   FC1: x_mid = x + bf16(out_proj), LN2 -> fc1 -> SwiGLU -> h
//   FC2: fc2 K-quarter partials
// then norm_f + the stacked heads as K-quarter partials for the sampler.
//
// Work units are the packed weights' own 16 KB blocks (tile, 16 k-steps): in_proj 768, out_proj
// 512, fc1 4096, fc2 2048, heads 2312 -> 3 + 2 + 16 + 8 units per CU and layer at 256 CUs.
// A unit is multiplied by ONE wave as a 16-step MFMA chain, and each K quarter is one wave's
// chain, summed in quarter order by the consumer: exactly the arithmetic of zk_gemv_fused with
// 4 K-quarter waves (layout 1), so the step is bit-identical to that launch sequence.
//
// Every wait is bounded: a wait that gives up sets sync[ERR] and all later waits fall through,
// so a broken run ends (with garbage) instead of hanging the GPU.
#include "common.h"
#include "attn_common.h"
#include "../../include/zonos_hip.h"
#include <algorithm>

namespace {

constexpr int SD = 2048, SF = 8192, SH = 16, SHKV = 4, SHD = 128;
constexpr int SNQKV = (SH + 2 * SHKV) * SHD;     // 3072
constexpr int NCW = 4;                           // consumer waves
constexpr int NLD = 2;                           // loader waves (each fills half of every slot)
constexpr int NTHR = 64 * (NCW + NLD);
constexpr int NS = 8;                            // ring slots
constexpr int SLOT = 16384;                      // bytes per slot (one unit)
constexpr int DFLY = 5;                          // slots in flight per loader wave (8 loads each, vmcnt <= 63)
constexpr int LPW = 16 / NLD;                    // 1 KB loads per slot and loader wave
constexpr int MAXR = 4;
constexpr int ACT_STR = SD + 8;                  // bf16 per staged activation row
constexpr uint32_t SPIN_G = 1u << 19;            // global polls before giving up (~1 s)
constexpr uint32_t SPIN_L = 1u << 22;            // LDS polls (~0.5 s)
#ifndef ZK_SS_SLEEP_C
#define ZK_SS_SLEEP_C 1      // s_sleep argument of the consumer waves' LDS polls
#endif
#ifndef ZK_SS_SLEEP_L
#define ZK_SS_SLEEP_L 4      // ... of the loader waves' free-slot polls (they share SIMDs with consumers)
#endif
enum { PH_IN = 0, PH_ATT = 1, PH_OUT = 2, PH_FC1 = 3, PH_FC2 = 4, NPH = 5 };
// sync words (each counter on its own 64-B line)
constexpr int SY_EPOCH = 0, SY_EXIT = 16, SY_ERR = 32, SY_CNT = 48;

typedef __attribute__((address_space(1))) uint32_t gu32;

// LDS map (dynamic): ring | act rows | fc1 reduction | attention | flags
constexpr int L_RING = 0;
constexpr int L_ACT = L_RING + NS * SLOT;
constexpr int L_RED = L_ACT + MAXR * ACT_STR * 2;
constexpr int L_ATT = L_RED + 2 * NCW * 16 * 16;
constexpr int L_FLG = L_ATT + (int)((sizeof(AttnSmem) + 15) / 16 * 16);
constexpr int L_TOTAL = L_FLG + 128;
static_assert(L_TOTAL <= 160 * 1024, "LDS budget");

struct Flags {
    uint32_t full[NS];      // loaders: halves landed in the slot so far (NLD per use)
    uint32_t freed[NS];     // consumers: uses of the slot finished
    uint32_t bar;           // consumer-wave barrier counter
    uint32_t pad[3];
};

ZK_DEV uint32_t lds_ld(const uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
ZK_DEV void lds_add(uint32_t* p) { __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
ZK_DEV uint32_t g_ld(uint32_t* p) {
    return __hip_atomic_load((gu32*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS-DMA of one 1 KB piece (64 lanes x 16 B) to the wave-uniform LDS byte address `lds`, non-temporal.
// Inline asm so that hipcc neither counts it (the loader waits with explicit vmcnt) nor drains it
// before the loader's own LDS polls.
ZK_DEV void glds16(const void* gsrc, uint32_t lds) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds)
        : "memory");
}
template <int N_>
ZK_DEV void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory"); }

// ---------------------------------------------------------------- the step's work schedule
// Per phase: G groups, a CU owns groups [G*c/ncu, G*(c+1)/ncu); units per group; unit u of group g
// = 16 k-steps starting at kstep(g, u) of packed tile tile(g).
struct Ph {
    const bf16_t* W;
    int kt;       // k-steps per packed tile (K / 32)
    int G;        // groups
    int upg;      // units per group
    int kind;     // PH_IN, PH_OUT, PH_FC1, PH_FC2 or 5 = heads
};
constexpr int PH_HEADS = 5;
ZK_DEV int ph_tile(const Ph& p, int g) {
    if (p.kind == PH_FC1) return g;
    if (p.kind == PH_FC2) return g % (SD / 16);
    return g >> 2;
}
ZK_DEV int ph_kstep(const Ph& p, int g, int u) {
    if (p.kind == PH_FC1) return u * 16;
    if (p.kind == PH_FC2) return (g / (SD / 16)) * 64 + u * 16;
    return (g & 3) * 16;
}
ZK_DEV Ph layer_phase(const zk_small_layer& L, int kind) {
    switch (kind) {
        case PH_IN: return Ph{(const bf16_t*)L.wqkv, SD / 32, SNQKV / 16 * 4, 1, PH_IN};
        case PH_OUT: return Ph{(const bf16_t*)L.wo, SD / 32, SD / 16 * 4, 1, PH_OUT};
        case PH_FC1: return Ph{(const bf16_t*)L.fc1, SD / 32, 2 * SF / 16, 4, PH_FC1};
        default: return Ph{(const bf16_t*)L.fc2, SF / 32, SD / 16 * 4, 4, PH_FC2};
    }
}

// ---------------------------------------------------------------- consumer-side helpers
// barrier of the 4 consumer waves (the loader wave never joins: it runs ahead). Stateless: the
// value returned by this wave's arrival tells which generation it waits for.
ZK_DEV void cbar(Flags* fl, uint32_t* sync, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(&fl->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t target = (__builtin_amdgcn_readfirstlane(old) / NCW + 1) * NCW;
    for (uint32_t it = 0; lds_ld(&fl->bar) < target; ++it) {
        if (it > SPIN_L) {
            __hip_atomic_store((gu32*)(sync + SY_ERR), 0x100u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(ZK_SS_SLEEP_C);
    }
    asm volatile("" ::: "memory");
}
// every CU has signalled phase (l, p): wave 0 polls the 8 XCD shards (lanes 0-7), then the
// agent-scope acquire; the other waves are released by the barrier after it.
ZK_DEV void seam_wait(Flags* fl, uint32_t* sync, uint32_t epoch, int ncu, int l, int p, int w, int lane) {
    if (w == 0) {
        const int x = lane & 7;
        const uint32_t nx = (uint32_t)((ncu - x + 7) / 8);
        const uint32_t target = (epoch + 1) * nx;
        uint32_t* ctr = sync + SY_CNT + ((l * NPH + p) * 8 + x) * 16;
        for (uint32_t it = 0;; ++it) {
            const bool ok = g_ld(ctr) >= target;
            if (__all(ok)) break;
            if ((it & 255) == 255 && (it > SPIN_G || g_ld(sync + SY_ERR) != 0)) {
                if (lane == 0)
                    __hip_atomic_store((gu32*)(sync + SY_ERR), 0x200u + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    cbar(fl, sync, lane);
}

// One attention unit (row r, kv head g, key split) of layer l: k_attn_decode's fused body (the 4
// in_proj K-quarter slabs), waiting for the in_proj seam once its first key blocks are in flight;
// with nsplit > 1 the splits merge in the launch (the last one to arrive combines, tickets per
// layer). Not inlined: its ~210 VGPRs get their own allocation instead of adding to the step loop's.
__attribute__((noinline)) __device__ void att_unit(Flags* fl, uint32_t* sync, uint32_t epoch, int ncu, int l, bool wait,
                                                   AttnSmem* sm, int split, int nsplit, int g, int r, bf16_t* kc,
                                                   bf16_t* vt, int R, int Smax, int ctx, bf16_t* Y, const float* pq,
                                                   const float* freqs, float* work, uint32_t* cnt) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    auto bar = [&] { cbar(fl, sync, lane); };
    auto issued = [&] { if (wait) seam_wait(fl, sync, epoch, ncu, l, PH_IN, w, lane); };
    const float scale = 1.0f / sqrtf((float)SHD);
    if (nsplit > 1)
        attn_decode_wg<true, false, false, true>(*sm, bar, issued, split, nsplit, g, r, nullptr, kc, vt, R, SH, SHKV,
                                                 Smax, ctx, work, scale, Y, pq, 4, freqs, cnt);
    else
        attn_decode_wg<true, false, false, false>(*sm, bar, issued, 0, 1, g, r, nullptr, kc, vt, R, SH, SHKV, Smax,
                                                  ctx, nullptr, scale, Y, pq, 4, freqs, nullptr);
    cbar(fl, sync, lane);       // LDS reuse by the next unit
}

struct Cons {
    char* smem;
    Flags* fl;
    uint32_t* sync;
    int w, lane, ln, lg, c, ncu, R;
    uint32_t epoch;
    int j;              // stream index of the next slot

    ZK_DEV bool failed() { return g_ld(sync + SY_ERR) != 0; }
    ZK_DEV void fail(uint32_t code) {
        __hip_atomic_store((gu32*)(sync + SY_ERR), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    ZK_DEV void bar() { cbar(fl, sync, lane); }
    ZK_DEV void seam(int l, int p) { seam_wait(fl, sync, epoch, ncu, l, p, w, lane); }
    // this CU finished phase (l, p): every wave's stores drained, then one agent-scope release + add
    ZK_DEV void signal(int l, int p) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
        if (w == 0 && lane == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add((gu32*)(sync + SY_CNT + ((l * NPH + p) * 8 + (c & 7)) * 16), 1u,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    ZK_DEV bf16_t* act() { return reinterpret_cast<bf16_t*>(smem + L_ACT); }

    // one unit (slot j) multiplied into acc: 16 k-steps, activation k offset k0 (elements)
    ZK_DEV void unit(f32x4& acc, int k0) {
        const int slot = j % NS;
        for (uint32_t it = 0; lds_ld(&fl->full[slot]) < (uint32_t)(NLD * (j / NS + 1)); ++it) {
            if (it > SPIN_L) { fail(0x300); break; }
            __builtin_amdgcn_s_sleep(ZK_SS_SLEEP_C);
        }
        asm volatile("" ::: "memory");
        const char* sb = smem + L_RING + slot * SLOT + lane * 16;
        const bf16_t* ar = act() + min(ln, R - 1) * ACT_STR + k0 + lg * 8;
        // two halves of 8 k-steps (64 VGPRs of operands at a time); the slot is released once the
        // second half's fragments are in registers
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            uint4 wf[8], af[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) wf[s] = *reinterpret_cast<const uint4*>(sb + (hf * 8 + s) * 1024);
#pragma unroll
            for (int s = 0; s < 8; ++s) af[s] = *reinterpret_cast<const uint4*>(ar + (hf * 8 + s) * 32);
            if (hf == 1) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (lane == 0) lds_add(&fl->freed[slot]);
            }
#pragma unroll
            for (int s = 0; s < 8; ++s)
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(af[s]), as_frag(wf[s]), acc, 0, 0, 0);
        }
        ++j;
    }
};

// Residual update + LayerNorm of one row by one wave (lane: columns lane*8 + 512*jj), the
// arithmetic of zk_gemv_fused's LN prologue and mode-2 epilogue:
//   x = nsl ? bf16(xsrc + bf16(p0 + p1 + p2 + p3)) : xsrc;  columns [s0, s1) of x -> xdst
//   arow = LayerNorm(x) (two-pass fp32 statistics, bf16 output)
ZK_DEV void stage_ln_row(const bf16_t* xsrc, const float* slabs, size_t sstr, int nsl, bf16_t* xdst, int s0, int s1,
                         const bf16_t* lnw, const bf16_t* lnb, float eps, bf16_t* arow, int lane) {
    uint4 xv[4], wv[4], bv[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
        xv[jj] = *reinterpret_cast<const uint4*>(xsrc + lane * 8 + jj * 512);
        wv[jj] = *reinterpret_cast<const uint4*>(lnw + lane * 8 + jj * 512);
        bv[jj] = *reinterpret_cast<const uint4*>(lnb + lane * 8 + jj * 512);
    }
    float xf[32];
    if (nsl) {
        // the 4 K-quarter partials of two 8-column chunks at a time (64 VGPRs of loads in flight)
#pragma unroll
        for (int jp = 0; jp < 4; jp += 2) {
            f32x4 sv[4][2][2];
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int jq = 0; jq < 2; ++jq) {
                    const float* p = slabs + s * sstr + lane * 8 + (jp + jq) * 512;
                    sv[s][jq][0] = *reinterpret_cast<const f32x4*>(p);
                    sv[s][jq][1] = *reinterpret_cast<const f32x4*>(p + 4);
                }
#pragma unroll
            for (int jq = 0; jq < 2; ++jq) {
                const int jj = jp + jq;
                float xo[8];
                unpack8(xv[jj], xo);
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float sum = sv[0][jq][e >> 2][e & 3];
#pragma unroll
                    for (int s = 1; s < 4; ++s) sum = sum + sv[s][jq][e >> 2][e & 3];
                    xf[8 * jj + e] = round_bf(xo[e] + round_bf(sum));
                }
            }
        }
        if (xdst) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int c0 = lane * 8 + jj * 512;
                if (c0 >= s0 && c0 + 8 <= s1) {
                    *reinterpret_cast<uint4*>(xdst + c0) = pack8(xf + 8 * jj);
                } else if (c0 + 8 > s0 && c0 < s1) {
                    for (int e = 0; e < 8; ++e)
                        if (c0 + e >= s0 && c0 + e < s1) xdst[c0 + e] = f2bf(xf[8 * jj + e]);
                }
            }
        }
    } else {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) unpack8(xv[jj], xf + 8 * jj);
    }
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 32; ++e) s += xf[e];
    const float mean = wave_sum_dpp(s) / (float)SD;
    float v = 0.f;
#pragma unroll
    for (int e = 0; e < 32; ++e) { const float d = xf[e] - mean; v += d * d; }
    const float var = wave_sum_dpp(v) / (float)SD;
    const float rstd = 1.0f / sqrtf(var + eps);
    const float nb = -rstd * mean;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
        float wf[8], bf[8], o[8];
        unpack8(wv[jj], wf);
        unpack8(bv[jj], bf);
#pragma unroll
        for (int e = 0; e < 8; ++e)
            o[e] = __fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(xf[8 * jj + e], rstd), nb), wf[e]), bf[e]);
        *reinterpret_cast<uint4*>(arow + lane * 8 + jj * 512) = pack8(o);
    }
}

__global__ __launch_bounds__(NTHR, 1) void k_decode_small(zk_small_args a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (a.skip && *a.skip) return;
    Flags* fl = reinterpret_cast<Flags*>(smem + L_FLG);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = blockIdx.x, ncu = gridDim.x;
    if (threadIdx.x < 32) reinterpret_cast<uint32_t*>(fl)[threadIdx.x] = 0;
    __syncthreads();      // the only full-workgroup barrier: flags zeroed

    const int NL = a.n_layer;
    const int ntiles_h = (a.n_heads_out + 15) / 16;
    const Ph heads_ph{(const bf16_t*)a.heads, SD / 32, ntiles_h * 4, 1, PH_HEADS};

    if (w >= NCW) {
        // ================= loaders: this CU's units of every phase, in consumption order; loader
        // wave h moves pieces h*LPW .. h*LPW+LPW-1 of every slot and announces its half once landed
        const int h = w - NCW;
        const uint32_t ring = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(smem + L_RING));
        int j = 0;
        bool dead = false;
        const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
        uint64_t t_wait = 0;
        auto fill = [&](const bf16_t* src) {
            if (j >= DFLY) {       // announce the half issued DFLY slots ago (its loads have landed)
                vmwait<LPW * (DFLY - 1)>();
                if (lane == 0) lds_add(&fl->full[(j - DFLY) % NS]);
            }
            const int slot = j % NS;
            if (j >= NS && !dead && lds_ld(&fl->freed[slot]) < (uint32_t)(j / NS)) {
                const uint64_t t0 = a.prof ? __builtin_amdgcn_s_memrealtime() : 0;
                for (uint32_t it = 0; lds_ld(&fl->freed[slot]) < (uint32_t)(j / NS); ++it) {
                    if (it > SPIN_L) { dead = true; break; }
                    __builtin_amdgcn_s_sleep(ZK_SS_SLEEP_L);
                }
                if (a.prof) t_wait += __builtin_amdgcn_s_memrealtime() - t0;
            }
            const bf16_t* s = src + h * LPW * 512 + lane * 8;
            const uint32_t d = ring + slot * SLOT + h * LPW * 1024;
#pragma unroll
            for (int i = 0; i < LPW; ++i) glds16(s + i * 512, __builtin_amdgcn_readfirstlane(d + i * 1024));
            ++j;
        };
        auto stream_phase = [&](const Ph& p) {
            const int g0 = (int)((long)p.G * c / ncu), g1 = (int)((long)p.G * (c + 1) / ncu);
            for (int g = g0; g < g1; ++g)
                for (int u = 0; u < p.upg; ++u)
                    fill(p.W + ((size_t)ph_tile(p, g) * p.kt + ph_kstep(p, g, u)) * 512);
        };
        for (int ph = 0; ph <= NL * 4; ++ph) {
            if (ph == NL * 4) { stream_phase(heads_ph); break; }
            const int kind = ph & 3;
            stream_phase(layer_phase(a.layers[ph >> 2], kind == 0 ? PH_IN : (kind == 1 ? PH_OUT : (kind == 2 ? PH_FC1 : PH_FC2))));
        }
        vmwait<0>();
        if (lane == 0)
            for (int k = std::max(0, j - DFLY); k < j; ++k) lds_add(&fl->full[k % NS]);
        if (a.prof && lane == 0 && h == 0) {
            uint64_t* pr = a.prof + ((size_t)c * (NL * NPH + 2) + NL * NPH + 1) * 4;
            pr[0] = t_start;
            pr[1] = __builtin_amdgcn_s_memrealtime();
            pr[2] = t_wait;
            pr[3] = (uint64_t)j;
        }
        return;
    }

    // ================= consumers
    Cons cs;
    cs.smem = smem;
    cs.fl = fl;
    cs.sync = a.sync;
    cs.w = w;
    cs.lane = lane;
    cs.ln = lane & 15;
    cs.lg = lane >> 4;
    cs.c = c;
    cs.ncu = ncu;
    cs.R = a.R;
    cs.j = 0;
    cs.epoch = g_ld(a.sync + SY_EPOCH);
    const int R = a.R;
    const int pos = *a.pos_dev;
    const int ctx = pos + 1;
    const int s0 = (int)((long)SD * c / ncu), s1 = (int)((long)SD * (c + 1) / ncu);   // residual columns stored here
    const size_t sl_d = (size_t)R * SD;
    bf16_t* X = (bf16_t*)a.x;
    bf16_t* XM = (bf16_t*)a.xm;
    bf16_t* Y = (bf16_t*)a.y;
    bf16_t* Hb = (bf16_t*)a.h;
    f32x4* red = reinterpret_cast<f32x4*>(smem + L_RED);      // [2][NCW][16]
    AttnSmem& asm_ = *reinterpret_cast<AttnSmem*>(smem + L_ATT);
    int rb = 0;

    // a GEMM phase of this CU: items (one wave's MFMA chain) go to waves round-robin
    auto gemm_phase = [&](const Ph& p, int l) {
        const int g0 = (int)((long)p.G * c / ncu), g1 = (int)((long)p.G * (c + 1) / ncu);
        int item = 0;
        int staged_q = -1;
        for (int g = g0; g < g1; ++g) {
            const int tile = ph_tile(p, g);
            if (p.kind == PH_FC2) {       // activation = the K quarter q of h
                const int q = g / (SD / 16);
                if (q != staged_q) {
                    if (staged_q >= 0) cs.bar();
                    if (w < R) {
                        const uint4* src = reinterpret_cast<const uint4*>(Hb + (size_t)w * SF + q * SD);
                        uint4* dst = reinterpret_cast<uint4*>(cs.act() + w * ACT_STR);
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) dst[lane + 64 * jj] = src[lane + 64 * jj];
                    }
                    cs.bar();
                    staged_q = q;
                }
            }
            if (p.kind == PH_FC1) {
                // 4 items (K quarters of the tile), one per wave, reduced in quarter order -> SwiGLU
                f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
                for (int u = 0; u < 4; ++u) {
                    if (((item + u) & 3) == w) cs.unit(acc, u * 512);
                    else ++cs.j;
                }
                item += 4;
                if (cs.ln == cs.lane) red[(rb * NCW + w) * 16 + cs.ln] = acc;
                cs.bar();
                if (w == 0) {
                    const int ll = lane & 15;
                    f32x4 sum = red[(rb * NCW + 0) * 16 + ll];
#pragma unroll
                    for (int q = 1; q < NCW; ++q) {
                        const f32x4 o = red[(rb * NCW + q) * 16 + ll];
#pragma unroll
                        for (int i = 0; i < 4; ++i) sum[i] = sum[i] + o[i];
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float mine = round_bf(sum[i]);
                        const float other = __shfl_xor(mine, 8, 64);
                        if (lane < 8 && i < R) {
                            const float sl = round_bf(other / (1.0f + expf(-other)));
                            Hb[(size_t)i * SF + tile * 8 + lane] = f2bf(mine * sl);
                        }
                    }
                }
                rb ^= 1;
                continue;
            }
            // one item: the group's units as one chain
            if ((item & 3) == w) {
                f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
                for (int u = 0; u < p.upg; ++u) {
                    const int ks = ph_kstep(p, g, u);
                    cs.unit(acc, p.kind == PH_FC2 ? u * 512 : ks * 32);
                }
                if (lane < 16) {
                    const int col = tile * 16 + lane;
                    const int q = p.kind == PH_FC2 ? g / (SD / 16) : (g & 3);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if (i >= R) break;
                        if (p.kind == PH_IN) a.p_qkv[((size_t)q * R + i) * SNQKV + col] = acc[i];
                        else if (p.kind == PH_OUT) a.p_o[((size_t)q * R + i) * SD + col] = acc[i];
                        else if (p.kind == PH_FC2) a.p_f[((size_t)q * R + i) * SD + col] = acc[i];
                        else if (col < a.n_heads_out) a.p_heads[((size_t)q * R + i) * a.n_heads_out + col] = acc[i];
                    }
                }
            } else {
                cs.j += p.upg;
            }
            ++item;
        }
        (void)l;
    };

    // optional phase timestamps (profiling): [seam start, seam done, staged, phase done]
    uint64_t* prof = a.prof ? a.prof + (size_t)c * (NL * NPH + 2) * 4 : nullptr;
    auto stamp = [&](int ph, int k) {
        if (prof && w == 0 && lane == 0) prof[ph * 4 + k] = __builtin_amdgcn_s_memrealtime();
    };
    // phases in step order; heads = phase NL * NPH
    for (int ph = 0; ph <= NL * NPH; ++ph) {
        stamp(ph, 0);
        const int l = ph / NPH, kind = ph % NPH;
        const bool heads = ph == NL * NPH;
        const zk_small_layer* L = heads ? nullptr : a.layers + l;
        // wait for the previous phase everywhere, then stage this phase's activation rows
        if (ph > 0 && !(kind == PH_ATT && !heads)) cs.seam(heads ? NL - 1 : (kind == PH_IN ? l - 1 : l),
                                                      (heads || kind == PH_IN) ? PH_FC2 : kind - 1);
        stamp(ph, 1);
        if (heads || kind == PH_IN || kind == PH_FC1) {
            // IN: x_new = xm + bf16(fc2 quarters) (layer 0: the embedding), stored to x, LN1;
            // FC1: x_mid = x + bf16(out_proj quarters), stored to xm, LN2; heads: norm_f(x_final)
            const bool first = ph == 0;
            const bf16_t* xs = (kind == PH_FC1) ? X : (first ? X : XM);
            const float* sl = (kind == PH_FC1) ? a.p_o : a.p_f;
            bf16_t* xd = heads ? nullptr : (kind == PH_FC1 ? XM : X);
            const bf16_t* lw = heads ? (const bf16_t*)a.lnf_w : (kind == PH_FC1 ? (const bf16_t*)L->ln2_w : (const bf16_t*)L->ln1_w);
            const bf16_t* lb = heads ? (const bf16_t*)a.lnf_b : (kind == PH_FC1 ? (const bf16_t*)L->ln2_b : (const bf16_t*)L->ln1_b);
            if (w < R)
                stage_ln_row(xs + (size_t)w * SD, sl + (size_t)w * SD, sl_d, first ? 0 : 4,
                             first ? nullptr : (xd ? xd + (size_t)w * SD : nullptr), s0, s1, lw, lb, a.eps,
                             cs.act() + w * ACT_STR, lane);
            cs.bar();
        } else if (kind == PH_OUT) {
            if (w < R) {
                const uint4* src = reinterpret_cast<const uint4*>(Y + (size_t)w * SD);
                uint4* dst = reinterpret_cast<uint4*>(cs.act() + w * ACT_STR);
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) dst[lane + 64 * jj] = src[lane + 64 * jj];
            }
            cs.bar();
        }
        stamp(ph, 2);
        if (heads) {
            gemm_phase(heads_ph, l);
            stamp(ph, 3);
            break;
        }
        if (kind == PH_ATT) {
            // one unit per (row, kv head), fused in_proj epilogue (k_attn_decode, nsplit 1); the
            // in_proj seam is waited for after the first key blocks' loads are issued
            const int nsp = a.attn_splits;
            for (int u = c; u < R * SHKV * nsp; u += ncu)
                att_unit(fl, a.sync, cs.epoch, ncu, l, u == c, &asm_, u % nsp, nsp, (u / nsp) % SHKV, u / nsp / SHKV,
                         (bf16_t*)L->k_cache, (bf16_t*)L->vt_cache, R, a.Smax, ctx, Y, a.p_qkv, a.freqs, a.attn_work,
                         a.sync + SY_CNT + NL * NPH * 8 * 16 + l * MAXR * SHKV);
        } else {
            gemm_phase(layer_phase(*L, kind), l);
        }
        cs.signal(l, kind);
        stamp(ph, 3);
    }
    // exit ticket: the last workgroup out advances the epoch for the next launch
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    cs.bar();
    if (w == 0 && lane == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t old = __hip_atomic_fetch_add((gu32*)(a.sync + SY_EXIT), 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        if (old == (uint32_t)ncu - 1) {
            __hip_atomic_store((gu32*)(a.sync + SY_EXIT), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store((gu32*)(a.sync + SY_EPOCH), cs.epoch + 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

int g_ncu = 0;

}  // namespace

extern "C" int zk_small_sync_words(int n_layer) { return SY_CNT + n_layer * NPH * 8 * 16 + n_layer * MAXR * SHKV; }

extern "C" int zk_decode_small(const zk_small_args* a, void* stream) {
    ZK_REQUIRE(a != nullptr && a->layers != nullptr && a->n_layer >= 1, "zk_decode_small: no layers");
    ZK_REQUIRE(a->R >= 1 && a->R <= MAXR, "zk_decode_small: R=%d (1..%d)", a->R, MAXR);
    ZK_REQUIRE(a->Smax > 0 && a->Smax % AT_KB == 0, "zk_decode_small: Smax=%d", a->Smax);
    ZK_REQUIRE(a->attn_splits >= 1 && a->attn_splits <= a->Smax / AT_KB && (a->attn_splits == 1 || a->attn_work),
               "zk_decode_small: attn_splits=%d (1..%d, > 1 needs attn_work)", a->attn_splits, a->Smax / AT_KB);
    ZK_REQUIRE(a->n_heads_out > 0 && a->heads && a->lnf_w && a->lnf_b, "zk_decode_small: heads");
    ZK_REQUIRE(a->freqs && a->pos_dev && a->x && a->xm && a->p_qkv && a->y && a->p_o && a->h && a->p_f &&
                   a->p_heads && a->sync,
               "zk_decode_small: missing buffer");
    if (g_ncu == 0) {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) {
            zk_set_error("zk_decode_small: device query failed");
            return -1;
        }
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_decode_small),
                                hipFuncAttributeMaxDynamicSharedMemorySize, L_TOTAL) != hipSuccess) {
            zk_set_error("zk_decode_small: %d B of LDS refused", L_TOTAL);
            return -1;
        }
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&k_decode_small),
                                                         NTHR, L_TOTAL) != hipSuccess || per_cu < 1) {
            zk_set_error("zk_decode_small: kernel not resident (%d per CU)", per_cu);
            return -1;
        }
        g_ncu = prop.multiProcessorCount;     // one workgroup per CU: every workgroup resident
    }
    hipLaunchKernelGGL(k_decode_small, dim3(g_ncu), dim3(NTHR), L_TOTAL, (hipStream_t)stream, *a);
    ZK_CHECK_LAUNCH("zk_decode_small");
    return 0;
}
