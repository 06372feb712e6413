// bf16 "nn.Linear" GEMM for gfx950: C[M][N] = A[M][K] . W[N][K]^T, fp32 accumulation on
// MFMA 16x16x32 bf16.
//
// Shape of the work: the decode step multiplies 2B = 128 activation rows by weight
// matrices streamed once from HBM (3.2 GB of weights per step), so the
// tile is 128 rows x 64 columns: every row of the batch lives in one workgroup and each
// weight element is read exactly once per step. Three kernels:
//   k_gemm     (M > 128: prefill) 4 waves, activation tile staged in LDS by the waves themselves;
//   k_gemm_ws  (16 < M <= 128: decode) 4 compute waves stream the weights into registers, 4
//              loader waves move the activation chunks into LDS by LDS-DMA;
//   k_gemv_rk  (M <= 16: small-batch decode) pure register weight stream, K quarters per wave.
// Wave w of a 64-column tile owns 16 weight rows (output columns), so its B fragments come
// straight from HBM into registers (no LDS round trip for the once-read stream) while the
// activation tile -- re-read by every column tile, L2-resident -- comes from LDS. Split-K over
// gridDim.z fills the 256 CUs when N is small; the partial slabs are reduced by the consumer
// kernel (k_resid_ln / the attention prologue / the sampler) in a fixed order, so the results
// depend on (N, K, nsplit) and the kernel regime, not on M within a regime.
//
// mode 0: fp32 partial slabs; mode 1: fused SwiGLU for FeedForward.fc1 (_torch.py:150-152).
#include "common.h"
#include "attn_common.h"
#include "../../include/zonos_hip.h"
#include "warm.h"
#include <algorithm>
#include <stdlib.h>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 128, BN = 64, BK = 64, NT = 256;


typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
// streamed-once weights: non-temporal 16-byte load (global_load_dwordx4 ... nt)
template <bool NT_>
ZK_DEV uint4 ldg_w(const bf16_t* p) {
    if constexpr (NT_) return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)));
    else return *reinterpret_cast<const uint4*>(p);
}

// Weight layout. ZK_W_PACKED: "fragment-packed" [N/16][K/32][64 lanes][8] -- the 16x32 B
// fragment of n-tile nt and k-slice kc is one contiguous 1 KB block in lane order, and a
// tile's K-slices follow each other, so a wave streams its 16 weight rows as ONE sequential
// run (each wave-instruction reads 1 KB contiguous instead of 16 rows x 64 B).
// Otherwise nn.Linear row-major [N][K].
#ifndef ZK_W_PACKED
#define ZK_W_PACKED 1
#endif
#if ZK_W_PACKED
constexpr int WCH = 1024;     // elements per 64-wide K chunk of one wave (2 fragments)
constexpr int WHALF = 512;
ZK_DEV const bf16_t* w_base(const bf16_t* W, int ntile_row0, int, int K, int kbeg, int lane) {
    return W + ((size_t)(ntile_row0 >> 4) * (K >> 5) + (kbeg >> 5)) * 512 + lane * 8;
}
#else
constexpr int WCH = BK;
constexpr int WHALF = 32;
ZK_DEV const bf16_t* w_base(const bf16_t* W, int, int row, int K, int kbeg, int lane) {
    return W + (size_t)row * K + kbeg + (lane >> 4) * 8;
}
#endif

// LDS byte offset of 16-byte chunk c (0..7) of tile row `row` (128-byte rows, XOR swizzle)
ZK_DEV int lds_off(int row, int c) { return row * 128 + ((c ^ (row & 7)) << 4); }

// NTW 16-column tiles per wave (tile 128 x 64*NTW): every activation fragment read from LDS
// feeds NTW MFMAs -- with NTW = 1 the four waves' fragment reads (1 KB per MFMA each) exceed the
// LDS array's 256 B/clk, with NTW = 2 the prefill GEMMs become MFMA-bound.
template <int MODE, int U, bool WNT = false, int NTW = 1>
__global__ __launch_bounds__(NT) void k_gemm(const bf16_t* __restrict__ A, long lda, const bf16_t* __restrict__ W,
                                             int M, int N, int K, int kslice, float* __restrict__ Cpart,
                                             bf16_t* __restrict__ Cout, const int32_t* skip) {
    __shared__ __attribute__((aligned(16))) char smem[2 * BM * BK * 2];
    if (skip && *skip) return;
    const int n0 = blockIdx.x * BN * NTW, m0 = blockIdx.y * BM, split = blockIdx.z;
    const int kbeg = split * kslice;
    const int nchunks = kslice / BK;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ln = lane & 15, lg = lane >> 4;

    // this lane's weight rows (one per 16-column tile of the wave)
    int wn[NTW];
    bool wvalid[NTW];
    const bf16_t* wrow[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
        const int c0 = n0 + (w * NTW + t) * 16;
        wn[t] = c0 + ln;
        wvalid[t] = wn[t] < N;
        wrow[t] = w_base(W, c0, wvalid[t] ? wn[t] : 0, K, kbeg, lane);
    }

    // activation staging: 4 x 16 B per thread per K chunk (row = q>>3, 16-B chunk = q&7)
    const bf16_t* arow[4];
    int aoff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int q = tid + NT * i;
        const int m = min(m0 + (q >> 3), M - 1);     // rows >= M compute garbage that is never stored
        arow[i] = A + (size_t)m * lda + kbeg + (q & 7) * 8;
        aoff[i] = lds_off(q >> 3, q & 7);
    }
    uint4 a0, a1, a2, a3;
#define ZK_LOAD_A(ch)                                                         \
    do {                                                                      \
        const int _k = (ch) * BK;                                             \
        a0 = *reinterpret_cast<const uint4*>(arow[0] + _k);                   \
        a1 = *reinterpret_cast<const uint4*>(arow[1] + _k);                   \
        a2 = *reinterpret_cast<const uint4*>(arow[2] + _k);                   \
        a3 = *reinterpret_cast<const uint4*>(arow[3] + _k);                   \
    } while (0)
#define ZK_STORE_A(buf)                                                       \
    do {                                                                      \
        char* _b = smem + (buf) * (BM * BK * 2);                              \
        *reinterpret_cast<uint4*>(_b + aoff[0]) = a0;                         \
        *reinterpret_cast<uint4*>(_b + aoff[1]) = a1;                         \
        *reinterpret_cast<uint4*>(_b + aoff[2]) = a2;                         \
        *reinterpret_cast<uint4*>(_b + aoff[3]) = a3;                         \
    } while (0)

    f32x4 acc[8][NTW];
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
        for (int t = 0; t < NTW; ++t) acc[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Weight stream: a register ring of U chunk slots keeps U-1 chunks (2 KB per wave and tile
    // each) of the weights in flight while the current chunk is multiplied. Every load is
    // unconditional (indices clamped; invalid columns stream row 0 and are never stored) so
    // hipcc emits counted vmcnt waits, and the activation loads of the next chunk are issued
    // BEFORE the weight prefetch so the wait that retires them (vmcnt counts in issue order)
    // leaves the weight loads in flight. nchunks % U == 0 (host-checked).
    constexpr int PF = U - 1;
    uint4 wr0[U][NTW], wr1[U][NTW];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const int pc = min(p, nchunks - 1);
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
            wr0[p][t] = ldg_w<WNT>(wrow[t] + pc * WCH);
            wr1[p][t] = ldg_w<WNT>(wrow[t] + pc * WCH + WHALF);
        }
    }
    ZK_LOAD_A(0);
    ZK_STORE_A(0);
    __syncthreads();
    for (int ch0 = 0; ch0 < nchunks; ch0 += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int ch = ch0 + u;
            ZK_LOAD_A(min(ch + 1, nchunks - 1));
            {
                const int pc = min(ch + PF, nchunks - 1);
#pragma unroll
                for (int t = 0; t < NTW; ++t) {
                    wr0[(u + PF) % U][t] = ldg_w<WNT>(wrow[t] + pc * WCH);
                    wr1[(u + PF) % U][t] = ldg_w<WNT>(wrow[t] + pc * WCH + WHALF);
                }
            }
            const char* base = smem + (ch & 1) * (BM * BK * 2);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    const uint4 a = *reinterpret_cast<const uint4*>(base + lds_off(mt * 16 + ln, ks * 4 + lg));
#pragma unroll
                    for (int t = 0; t < NTW; ++t)
                        acc[mt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            as_frag(a), as_frag(ks == 0 ? wr0[u][t] : wr1[u][t]), acc[mt][t], 0, 0, 0);
                }
            }
            ZK_STORE_A((ch + 1) & 1);
            __syncthreads();
        }
    }
#undef ZK_LOAD_A
#undef ZK_STORE_A

    // epilogue: acc[mt][t][i] = C[m0 + 16mt + 4lg + i][wn[t]]
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
        if (MODE == 0) {
            float* C = Cpart + (size_t)split * M * N;
            if (wvalid[t]) {
#pragma unroll
                for (int mt = 0; mt < 8; ++mt)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int m = m0 + mt * 16 + lg * 4 + i;
                        if (m < M) C[(size_t)m * N + wn[t]] = acc[mt][t][i];
                    }
            }
        } else {
            // interleaved fc1 rows: within each group of 16 columns, 0..7 = y[f0..f0+7], 8..15 = gate[f0..]
            const int F = N / 2;
            const int f = (n0 + (w * NTW + t) * 16) / 2 + (ln & 7);
#pragma unroll
            for (int mt = 0; mt < 8; ++mt)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float mine = round_bf(acc[mt][t][i]);
                    const float other = __shfl_xor(mine, 8, 64);
                    const int m = m0 + mt * 16 + lg * 4 + i;
                    if (ln < 8 && m < M && f < F) {
                        const float y = mine, g = other;
                        const float sl = round_bf(g / (1.0f + expf(-g)));     // F.silu in bf16
                        Cout[(size_t)m * F + f] = f2bf(y * sl);
                    }
                }
        }
    }
}

// ------------------------------------------------------------------ decode GEMM, loader-wave form
// M <= 128. Problem with a single load queue: vmcnt retires loads in issue order, so a wave
// that stages activations AND streams weights drains its weight prefetch every time it waits
// for an activation chunk. Here the roles are split across waves, each with its own vmcnt
// queue: wave 4 (the loader) moves activation chunks into an LDS ring by LDS-DMA
// (global_load_lds_dwordx4, DA chunks ahead, XOR swizzle applied on the source address), and
// waves 0-3 only stream weights into a PF-chunk register ring; one raw s_barrier per chunk
// publishes the next activation chunk (it does not drain VMEM).
#ifndef ZK_WS_NB
#define ZK_WS_NB 6
#define ZK_WS_DA 4
#define ZK_WS_OCC 1
#endif
constexpr int WS_NB = ZK_WS_NB;  // LDS ring slots (16 KB each)
constexpr int WS_DA = ZK_WS_DA;  // activation chunks in flight (loader); WS_NB >= WS_DA + 2
#ifndef ZK_WS_NLD
#define ZK_WS_NLD 4
#endif
constexpr int WS_NLD = ZK_WS_NLD;            // loader waves (each moves 1/WS_NLD of every chunk)
#ifndef ZK_WS_PF
#define ZK_WS_PF 4
#endif
#ifndef ZK_WS_NT
#define ZK_WS_NT 1
#endif
constexpr int WS_LDSPF = 1;      // chunks published ahead of the one being multiplied
constexpr int WS_PF = ZK_WS_PF;  // weight chunks in flight per compute wave: the SwiGLU fc1 (mode 1)
#ifndef ZK_WS_PF0
#define ZK_WS_PF0 3
#endif
constexpr int WS_PF0 = ZK_WS_PF0; // ... and the split-K slab GEMMs (mode 0): 3 measured faster for the
                                  // in_proj / out_proj / fc2 shapes, 4 for fc1 (profiles/r3s2_gemm_pf_ab.txt)
constexpr bool WS_NT = ZK_WS_NT; // non-temporal weight loads
#ifndef ZK_WS_DEFER
#define ZK_WS_DEFER 0              // k_gemm_ws: step word tested after the first loads (A/B only)
#endif


// k_gemm_ws split-K slab stores (read once by the consumer kernel): non-temporal with ZK_SLAB_NT
// (B=64: decode step 3.928 vs 3.959 ms; the B <= 8 GEMV keeps plain stores: its slabs are small
// and nt cost 2.5 % per step at B=1)
#ifndef ZK_SLAB_NT
#define ZK_SLAB_NT 1
#endif
#ifndef ZK_SLAB_SC1
#define ZK_SLAB_SC1 0              // write-through (sc1) slab stores: nothing left dirty in L2 at the boundary
#endif
#ifndef ZK_WS_EPI
#define ZK_WS_EPI 1                // k_gemm_ws epilogue staged through LDS (whole-row stores)
#endif
ZK_DEV void st_slab(float* p, float v) {
    if constexpr (ZK_SLAB_NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int N_>
ZK_DEV void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory"); }

// MT = 16-row M tiles actually present (1, 2, 4, 8): small batches stage and multiply only
// the rows they have (B = 1 decode: 2 rows -> one 16-row tile instead of 8).
// NG = 16-column groups per compute wave: every activation fragment read from LDS feeds NG MFMAs,
// and a workgroup covers 16 * NCW * NG columns, so a wider tile stages the same activation once
// for NG times the weights (LDS reads and per-CU activation intake per weight byte / NG).
// NB = activation fragment buffers (2: the next chunk's fragments are read while this one is
// multiplied).
// Loader waves: WS_NLD, fewer when that would put a ninth wave (a third per SIMD: 168 VGPRs) in the
// workgroup, and fewer again until every loader that issues pieces issues the same number of them
// (2*MT pieces per chunk): each loader's counted vmcnt waits assume NP pieces per younger chunk, so
// a loader with fewer would pass the publishing barrier with pieces of that chunk still in flight
// (NCW = 5 at MT = 8: 3 loaders would split 16 pieces 6 / 5 / 5 -- 2 loaders split them 8 / 8).
template <int NCW, int MT>
constexpr int ws_nld() {
    int n = NCW + WS_NLD > 8 ? 8 - NCW : WS_NLD;
    while (n > 1 && n < 2 * MT && (2 * MT) % n != 0) --n;
    return n;
}
template <int MODE, int NCH, int PF, int MT, int NCW = 4, int NG = 1, int NB = (NCW > 5 ? 1 : 2)>
__global__ __launch_bounds__(64 * (NCW + ws_nld<NCW, MT>()), ZK_WS_OCC) void k_gemm_ws(const bf16_t* __restrict__ A, long lda,
                                                           const bf16_t* __restrict__ W, int M, int N, int K,
                                                           int kslice, float* __restrict__ Cpart,
                                                           bf16_t* __restrict__ Cout, const int32_t* skip,
                                                           const bf16_t* __restrict__ wW, int wK, int wgx, int wgz,
                                                           int wch) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // (the skip word is tested first here: deferring the test behind the first loads, as k_gemv_f
    // does, measured 0.3-1.2 % slower per c3 step with a vector or a scalar load of the word,
    // profiles/r3s2_skip_defer_ab.txt; again in round 6, 3.500-3.510 vs 3.473-3.489 ms, while k_resid_ln gained:
    // profiles/r6_c3_gemm_ws_defer_ab.txt; ZK_WS_DEFER=1 builds that form)
    if (!ZK_WS_DEFER)
        if (skip && *skip) return;
    int bx, bz;
    ws_tile(blockIdx.x + gridDim.x * blockIdx.z, gridDim.x, gridDim.z, bx, bz);     // gridDim.y == 1
    constexpr int BNW = 16 * NCW * NG;            // columns per workgroup
    const int n0 = bx * BNW, split = bz;
    const int kbeg = split * kslice;
    const int nchunks = kslice / BK;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ln = lane & 15, lg = lane >> 4;

    constexpr int NLD = ws_nld<NCW, MT>();
    static_assert(NLD >= 1 && (NLD >= 2 * MT || (2 * MT) % NLD == 0),
                  "every loader wave must issue the same number of pieces per chunk (its vmcnt waits count NP)");
    if (w >= NCW) {
        // ---------------- loader wave(s): 2*MT x 1 KB LDS-DMA pieces per chunk (16*MT rows x 64 k),
        // loader l moving pieces l, l + NLD, ...
        // piece i covers tile rows 8i..8i+7; lane L lands at byte 16L of the piece:
        // row = 8i + (L>>3), slot = L&7  ->  source 16-B chunk = slot ^ (row&7)
        constexpr int NP = (2 * MT + NLD - 1) / NLD;      // pieces per loader per chunk
        const int ld = __builtin_amdgcn_readfirstlane(w - NCW);   // wave-uniform: scalar piece loop
        const int rl = lane >> 3, sl = lane & 7;
        auto issue = [&](int ch) {
            char* dst = smem + (ch % WS_NB) * (MT * 16 * BK * 2);
            const int k0 = kbeg + ch * BK;
#pragma unroll
            for (int j = 0; j < NP; ++j) {
                const int i = j * NLD + ld;
                if (NLD > 1 && i >= 2 * MT) break;          // (MT = 1, 2 loaders: 1 piece each)
                const int row = 8 * i + rl;
                const int m = min(row, M - 1);
                const bf16_t* src = A + (size_t)m * lda + k0 + ((sl ^ (row & 7)) << 3);
#ifndef ZK_DBG_NOALOAD
                __builtin_amdgcn_global_load_lds((const void*)src, (void*)(dst + i * 1024), 16, 0, 0);
#else
                (void)src; (void)dst;
#endif
            }
        };
        const int pre = min(WS_DA, nchunks);
        for (int c = 0; c < pre; ++c) issue(c);
        if constexpr (ZK_WS_DEFER) {
            if (ld_word_here(skip)) {           // the LDS-DMA writes land before the workgroup may leave
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                return;
            }
        }
        for (int c = 0; c < nchunks; ++c) {
            // barrier c publishes chunk `need` (one chunk ahead, so the compute
            // waves can read chunk c+1's fragments while they multiply chunk c)
            const int need = min(c + WS_LDSPF, nchunks - 1);
            const int younger = min(c - 1 + WS_DA, nchunks - 1) - need;   // chunks issued after `need`
            if (younger >= 5) vm_wait<5 * NP>();
            else if (younger == 4) vm_wait<4 * NP>();
            else if (younger == 3) vm_wait<3 * NP>();
            else if (younger == 2) vm_wait<2 * NP>();
            else if (younger == 1) vm_wait<NP>();
            else vm_wait<0>();
            __builtin_amdgcn_s_barrier();                           // publish chunk `need`
            asm volatile("" ::: "memory");
            if (c + WS_DA < nchunks) issue(c + WS_DA);              // its slot was read >= 2 chunks ago
        }
        if (wW != nullptr) {
            // L2 warm-up of the NEXT GEMM (warm.h): its workgroups L, L + nwg, ... run on this XCD;
            // the loaders, idle from here on, stream their compute waves' first chunks into L2 (LDS-DMA
            // into the 1 KB sink past the ring), then keep the workgroup's barrier count: the epilogue's
            // two __syncthreads must not wait for these loads
            warm_units(wW, wK, wgx, wgz, wch, blockIdx.x + gridDim.x * blockIdx.z, gridDim.x * gridDim.z, ld, NLD,
                       lane, smem + WS_NB * (MT * 16 * BK * 2));
            if (ZK_WS_EPI && (MODE == 1 || N % 4 == 0)) {
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_s_barrier();
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        return;
    }

    // ---------------- compute waves: wave w owns the 16-column groups w * NG + g
    const bf16_t* wrow[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int c0 = n0 + (w * NG + g) * 16;
        // a 16-row tile wholly past N streams tile 0 (never stored): the packed image ends at ceil64(N)
        const int trow = c0 < N ? c0 : 0;
        wrow[g] = w_base(W, trow, c0 + ln < N ? c0 + ln : 0, K, kbeg, lane);
    }
    f32x4 acc[NG][MT];
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[g][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // Fully unrolled K loop (NCH chunks known at compile time): no loop back edge, so hipcc's
    // waitcnt pass counts exactly and keeps PF chunks (2 loads per group each) of weights in flight
    // (its loop-header merge otherwise drains the ring). Ring slots are compile-time indices.
    constexpr int U = PF + 1;
    uint4 wr0[NG][U], wr1[NG][U];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const int pc = p < NCH ? p : NCH - 1;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            wr0[g][p] = ldg_w<WS_NT>(wrow[g] + pc * WCH);
            wr1[g][p] = ldg_w<WS_NT>(wrow[g] + pc * WCH + WHALF);
        }
    }
    if constexpr (ZK_WS_DEFER) {
        if (ld_word_here(skip)) {
#pragma unroll
            for (int p = 0; p < PF; ++p)
#pragma unroll
                for (int g = 0; g < NG; ++g) {
                    keep_live(wr0[g][p]);
                    keep_live(wr1[g][p]);
                }
            return;
        }
    }
    // activation fragments of the next chunk are read from LDS (register double buffer) while
    // the current chunk is multiplied: the LDS latency after each barrier is off the MFMA path
    // (NB = 1: one fragment set, read after the MFMAs)
    uint4 af[NB][2][MT];
    auto read_frags = [&](int ch, int buf) {
        const char* base = smem + (ch % WS_NB) * (MT * 16 * BK * 2);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
                af[buf][ks][mt] = *reinterpret_cast<const uint4*>(base + lds_off(mt * 16 + ln, ks * 4 + lg));
    };
    __builtin_amdgcn_s_barrier();                                   // chunk 0 (and 1) in LDS
    asm volatile("" ::: "memory");
    read_frags(0, 0);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
        if (ch + PF < NCH) {
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                wr0[g][(ch + PF) % U] = ldg_w<WS_NT>(wrow[g] + (ch + PF) * WCH);
                wr1[g][(ch + PF) % U] = ldg_w<WS_NT>(wrow[g] + (ch + PF) * WCH + WHALF);
            }
        }
        if (NB == 2 && ch + 1 < NCH) {
            __builtin_amdgcn_s_barrier();                           // chunk ch+1 (and ch+2) in LDS
            asm volatile("" ::: "memory");
            read_frags(ch + 1, (ch + 1) & 1);
        }
        __builtin_amdgcn_sched_barrier(0);     // keep the fragment reads ahead of this chunk's MFMAs
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const bf16x8 a = as_frag(af[NB == 2 ? (ch & 1) : 0][ks][mt]);
#pragma unroll
                for (int g = 0; g < NG; ++g)
                    acc[g][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        a, as_frag(ks == 0 ? wr0[g][ch % U] : wr1[g][ch % U]), acc[g][mt], 0, 0, 0);
            }
        }
        if (NB == 1 && ch + 1 < NCH) {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();                           // chunk ch+1 (and ch+2) in LDS
            asm volatile("" ::: "memory");
            read_frags(ch + 1, 0);
        }
    }
    if (ZK_WS_EPI && (MODE == 1 || N % 4 == 0)) {
        // Epilogue staged through the (now idle) LDS ring so that every store instruction writes
        // whole rows: slabs of BNW floats per row (full 128-B lines) instead of 64-B pieces, SwiGLU
        // rows of BNW / 2 bf16 instead of 16-B pieces. (The loader waves have exited; a workgroup
        // barrier no longer counts them.)
        constexpr int TS = BNW + 4;                              // fp32 tile row stride (+ pad)
        float* tile = reinterpret_cast<float*>(smem);
        __syncthreads();                                         // every wave's last LDS fragment read
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    // MODE 1: the bf16-rounded y / gate columns as they are (8 + 8 interleaved per
                    // 16-column group); SwiGLU runs in the store pass below, on every lane (here it
                    // would run on half the lanes behind a branch per value: fc1 23.4 -> 18.x us)
                    tile[(mt * 16 + lg * 4 + i) * TS + (w * NG + g) * 16 + ln] =
                        MODE == 0 ? acc[g][mt][i] : round_bf(acc[g][mt][i]);
        __syncthreads();
        if (MODE == 0) {
            float* C = Cpart + (size_t)split * M * N;
            constexpr int LPR = BNW / 4;                         // lanes per row (4 floats each)
            constexpr int RPI = 64 / LPR;                        // whole rows per instruction
            constexpr int NQI = (MT * 16 + RPI - 1) / RPI;       // (BNW = 48: 5 rows per instruction, 4 lanes idle)
            const int c4 = (lane % LPR) * 4;
#pragma unroll
            for (int q = w; q < NQI; q += NCW) {
                const int m = q * RPI + lane / LPR;
                if (lane < RPI * LPR && m < M && n0 + c4 < N) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(tile + m * TS + c4);
                    float* dst = C + (size_t)m * N + n0 + c4;
                    if (n0 + c4 + 3 < N) {
                        if constexpr (ZK_SLAB_SC1)
                            asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
                        else if constexpr (ZK_SLAB_NT) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst));
                        else *reinterpret_cast<f32x4*>(dst) = v;
                    } else {
                        for (int e = 0; e < 4 && n0 + c4 + e < N; ++e) dst[e] = v[e];
                    }
                }
            }
        } else {
            const int F = N / 2;
            constexpr int GPR = BNW / 16;                        // 16-column groups per row
            constexpr int RPI = 64 / GPR;                        // rows per instruction
            constexpr int NQI = (MT * 16 + RPI - 1) / RPI;
            const int f0 = n0 / 2, gi = lane % GPR;              // group gi -> outputs f0 + 8 gi ..
#pragma unroll
            for (int q = w; q < NQI; q += NCW) {
                const int m = q * RPI + lane / GPR;
                if (lane < RPI * GPR && m < M && f0 + gi * 8 < F) {
                    const float* yv = tile + m * TS + gi * 16;
                    float o[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float g = yv[8 + j];
                        const float sl = round_bf(g / (1.0f + expf(-g)));     // F.silu in bf16
                        o[j] = yv[j] * sl;
                    }
                    *reinterpret_cast<uint4*>(Cout + (size_t)m * F + f0 + gi * 8) = pack8(o);
                }
            }
        }
        return;
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int wn = n0 + (w * NG + g) * 16 + ln;
        if (MODE == 0) {
            float* C = Cpart + (size_t)split * M * N;
            if (wn < N) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int m = mt * 16 + lg * 4 + i;
                        if (m < M) st_slab(C + (size_t)m * N + wn, acc[g][mt][i]);
                    }
            }
        } else {
            const int F = N / 2;
            const int f = (n0 + (w * NG + g) * 16) / 2 + (ln & 7);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float mine = round_bf(acc[g][mt][i]);
                    const float other = __shfl_xor(mine, 8, 64);
                    const int m = mt * 16 + lg * 4 + i;
                    if (ln < 8 && m < M && f < F) {
                        const float sl = round_bf(other / (1.0f + expf(-other)));
                        Cout[(size_t)m * F + f] = f2bf(mine * sl);
                    }
                }
        }
    }
}

// ------------------------------------------------------------------ decode GEMV, M <= 16
// Small batches (B = 1 decode: 2 rows) are a pure weight stream: one 16-row activation tile
// per K step feeds NTW MFMAs, so nothing is staged through LDS and there are no barriers in
// the main loop. The workgroup's 4 waves split the K range (wave w owns quarter w) and each
// streams all NTW*16 columns of the tile for its quarter -- weights fragment-packed, nt, PF
// k-steps in flight (sched_barrier-pinned), the activation fragment from L2. The quarters are
// summed through LDS in a fixed order (q0 + q1 + q2 + q3): results depend on (N, K, nsplit).
// (At M = 128 this form is slower than k_gemm_ws: its 8 activation fragments per k-step are
// 16-row gathers -- DESIGN.md "rejected designs".)
template <int MODE, int NTW, int KS, int PF>
__global__ __launch_bounds__(256, 1) void k_gemv_rk(const bf16_t* __restrict__ A, long lda,
                                                    const bf16_t* __restrict__ W, int M, int N, int K, int kslice,
                                                    float* __restrict__ Cpart, bf16_t* __restrict__ Cout,
                                                    const int32_t* skip) {
    __shared__ __attribute__((aligned(16))) f32x4 red[4][NTW][64];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ln = lane & 15, lg = lane >> 4;
    const int split = blockIdx.z;
    const int nt0 = blockIdx.x * NTW;                          // first 16-column tile
    const int ntiles = (N + 63) / 64 * 4;                      // packed rows are padded to 64
    const int kbeg = split * kslice + w * (kslice >> 2);
    const bf16_t* wp[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t)
        wp[t] = W + ((size_t)min(nt0 + t, ntiles - 1) * (K >> 5) + (kbeg >> 5)) * 512 + lane * 8;
    const bf16_t* ap = A + (size_t)min(ln, M - 1) * lda + kbeg + lg * 8;
    f32x4 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int U = PF + 1;
    uint4 wr[U][NTW], ar[U];
    auto issue = [&](int st, int slot) {
#pragma unroll
        for (int t = 0; t < NTW; ++t) wr[slot][t] = ldg_w<true>(wp[t] + st * 512);
        ar[slot] = *reinterpret_cast<const uint4*>(ap + st * 32);
    };
#pragma unroll
    for (int p = 0; p < PF; ++p)
        if (p < KS) issue(p, p);
    __builtin_amdgcn_sched_barrier(0);
    if (ld_word_here(skip)) {                                  // tested once the prefetch is in flight
#pragma unroll
        for (int p = 0; p < PF; ++p)
            if (p < KS) {
                keep_live(ar[p]);
#pragma unroll
                for (int t = 0; t < NTW; ++t) keep_live(wr[p][t]);
            }
        return;
    }
#pragma unroll
    for (int st = 0; st < KS; ++st) {
        if (st + PF < KS) issue(st + PF, (st + PF) % U);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < NTW; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(ar[st % U]), as_frag(wr[st % U][t]), acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int t = 0; t < NTW; ++t) red[w][t][lane] = acc[t];
    __syncthreads();
    // wave w finishes tiles t with t % 4 == w (NTW <= 4: one tile per wave at most)
    const int t = w;
    if (t >= NTW) return;
    f32x4 sum = red[0][t][lane];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
        const f32x4 o = red[q][t][lane];
#pragma unroll
        for (int i = 0; i < 4; ++i) sum[i] = sum[i] + o[i];
    }
    const int n = (nt0 + t) * 16 + ln;
    if (MODE == 0) {
        if (n < N) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = lg * 4 + i;
                if (m < M) Cpart[(size_t)split * M * N + (size_t)m * N + n] = sum[i];   // (B <= 8: plain, measured)
            }
        }
    } else {
        const int F = N / 2;
        const int f = (nt0 + t) * 8 + (ln & 7);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float mine = round_bf(sum[i]);
            const float other = __shfl_xor(mine, 8, 64);
            const int m = lg * 4 + i;
            if (ln < 8 && m < M && f < F) {
                const float sl = round_bf(other / (1.0f + expf(-other)));
                Cout[(size_t)m * F + f] = f2bf(mine * sl);
            }
        }
    }
}

// ------------------------------------------------------------------ small-batch fused GEMV
// M <= 16 (B <= 8 decode) without split-K, so a transformer layer is five launches:
//   [LN1 prologue + in_proj] -> attention -> [out_proj + residual] -> [LN2 prologue + fc1 +
//   SwiGLU] -> [fc2 + residual]   (and [norm_f prologue + heads]).
// The M <= 16 activation is tiny, so instead of a separate k_resid_ln launch per residual
// every workgroup of the consuming GEMV recomputes the LayerNorm of the (<= 16) input rows
// into LDS; its weight prefetch is issued right behind the row loads, so the prologue runs
// under the weight stream's first round trip. The producing GEMV adds its bf16 output to the
// residual row in its epilogue (x = bf16(x + bf16(A.W^T)), _torch.py:100-101) -- no fp32
// split-K slabs leave the workgroup: the 4 waves split K and are summed through LDS in a
// fixed order (q0 + q1 + q2 + q3), so results depend on (N, K) only, not on M <= 16.
// Layouts: NTW 16-column tiles per workgroup; HALF: 8 columns (half a packed tile: the lanes
// of the other half load nothing, the tile's other 8 columns belong to the neighbouring
// workgroup -- 4 of the 8 128-B lines of every 1 KB fragment each) so N = 2048 still gives
// 256 workgroups.
// mode 0: fp32 Cf[M][N]; mode 1: SwiGLU -> bf16 Cb[M][N/2]; mode 2: residual, Cb = x bf16 [M][N].
// ZK_GF_PROF (profiling builds only): lane 0 of wave 0 of each k_gemv_f workgroup writes s_memrealtime
// stamps [entry, first MFMA issued, last MFMA issued, end] to g_gf_prof[slot][blockIdx.x][k], slot =
// 2 * MODE + (MRG > 0) (so the launches of one kind in a step overwrite each other: the last one stays).
#ifdef ZK_GF_PROF
__device__ uint64_t* g_gf_prof;
#define ZK_GF_STAMP(k)                                                                                      \
    do {                                                                                                    \
        if (threadIdx.x == 0 && g_gf_prof)                                                                  \
            g_gf_prof[((size_t)(2 * MODE + (MRG > 0)) * 2048 + blockIdx.x) * 4 + (k)] =                     \
                __builtin_amdgcn_s_memrealtime();                                                           \
    } while (0)
#else
#define ZK_GF_STAMP(k) do {} while (0)
#endif
ZK_DEV void opaque(uint4& v) {
    u32x4 t = __builtin_bit_cast(u32x4, v);
    asm volatile("" : "+v"(t));
    v = __builtin_bit_cast(uint4, t);
}

constexpr int GF_XS = 2048 + 8;    // LDS row stride (bf16) of the LayerNorm'd rows (K = 2048)

// NW waves split K (wave w: K range w/NW); KS k-steps of 32 per wave; PF loads in flight.
// HALF: every weight load instruction fetches 1 KB of this workgroup's 8 columns by pairing
// k-steps -- the owning lanes read k-step 2j of the packed fragment, the other half's lanes
// read k-step 2j+1 at their neighbour's position (lane ^ 8); a DPP row rotation by 8 then moves
// the k-step 2j+1 values to the owning lanes for the second MFMA. The other half's output
// columns are garbage and never stored.
// MRG (0, 2, 4, 8): the activation is the decode attention's output, still split over MRG key
// ranges -- the [row][kv head][split] (m, l, O) partials of zk_attn_decode_qkv_part in `mw` --
// and the prologue merges them exactly as k_attn_combine does (backbone.hip) into LDS; each
// wave merges the 2 heads of its own K range (K = 2048, NW = 8), rows < M <= 2.
constexpr int GF_AT_G = AT_G, GF_AT_STR = AT_STR;    // the partials layout of attn_common.h (one definition)
static_assert(GF_AT_STR == 2 * GF_AT_G + GF_AT_G * 128, "attention partials layout");
// XR: rows the LDS activation image holds (2 for B = 1, 16 otherwise): a 16-row image is 66 KB and
// caps the LayerNorm-prologue GEMVs at 2 workgroups per CU; the 2-row image (8 KB) does not.
// XC (ZK_GF_XC, B = 1 GEMVs without a LayerNorm or merge prologue: fc2): the activation rows are copied
// into the LDS image once per wave -- each wave its own K range, 4 x 16 B per lane at K = 8192 -- instead
// of being re-loaded from L2 beside every weight load (two 16-B-per-lane loads per weight piece, 16 lanes
// per row for the 2 real rows: 2/3 of the wave's load instructions). Same operands, same MFMA order:
// bit-identical. A pure-stream probe of the fc2 shape: 6.45 -> 7.01 us per launch with those loads
// (profiles/r6_stream_order_probe.txt).
#ifndef ZK_GF_XC
#define ZK_GF_XC 1
#endif
#ifndef ZK_GF_LNW
#define ZK_GF_LNW 1
#endif
#ifndef ZK_GF_OCC2
#define ZK_GF_OCC2 1               // min waves per SIMD the B = 1 (XR = 2) instantiations are sized for
#endif
// mode 3 (in_proj of the B = 1 step): the epilogue of the decode attention's old prologue. The GEMV
// output is final (no split-K), so each column pair (2j, 2j+1) of a q / k head -- two neighbouring lanes
// of one 16-column tile -- is rounded to bf16 and rotated here (interleaved RoPE, _torch.py:18-30, the
// arithmetic of k_qkv_rope / attn_decode_wg's prologue), q is stored to Cb [M][H*hd] and the new key /
// value straight into the fragment-ordered KV cache at position *pos, so the attention kernel reads q
// and the whole cache and has no prologue.
struct GfQkv {
    bf16_t* kc;            // K cache of the layer ([row][kv head] blocks of Smax * 128)
    bf16_t* vt;            // V^T cache
    const int32_t* pos;    // device position word (= context - 1 of this step)
    const float* freqs;    // [pos][64][2] (cos, sin)
    int H, Hkv, Smax;
};

template <int MODE, bool LN, int NTW, bool HALF, int NW, int KS, int PF, int MRG = 0, int XR = 16>
__global__ __launch_bounds__(64 * NW, XR == 2 ? ZK_GF_OCC2 : 1) void k_gemv_f(const bf16_t* __restrict__ A, long lda,
                                                       const bf16_t* __restrict__ W, int M, int N, int K,
                                                       const bf16_t* __restrict__ lnw, const bf16_t* __restrict__ lnb,
                                                       float eps, float* __restrict__ Cf, bf16_t* __restrict__ Cb,
                                                       const int32_t* skip, const float* __restrict__ mw = nullptr,
                                                       int mhkv = 1, GfQkv qk = GfQkv{}) {
    static_assert(MODE != 3 || (LN && NTW == 1 && !HALF && XR == 2), "qkv RoPE epilogue: the B = 1 in_proj");
    ZK_GF_STAMP(0);
    static_assert(!HALF || NTW == 1, "HALF is one half tile");
    static_assert(!LN || KS * NW * 32 == 2048, "LN prologue: K = 2048");
    static_assert(!MRG || (!LN && NW == 8 && KS * NW * 32 == 2048), "merge prologue: K = 2048, 8 waves");
    static_assert(NTW <= NW, "one finishing wave per tile");
    constexpr bool XC = ZK_GF_XC && XR == 2 && !LN && !MRG;          // activation copied to LDS (see above)
    constexpr bool XS = LN || MRG || XC;                             // activation from LDS
    constexpr int XSTR = XC ? NW * KS * 32 + 8 : GF_XS;              // LDS image row stride (bf16)
    constexpr int XCN = XC ? KS * 32 * 2 / 512 : 1;                  // XC: 16-B loads per lane (2 rows)
    static_assert(!XC || (KS * 32 * 2) % 512 == 0, "XC: whole 512-element load rounds per wave");
    constexpr int KPL = HALF ? 2 : 1;                                // k-steps per weight load
    constexpr int NL = KS / KPL;                                     // weight loads per wave and tile
    static_assert(NL * KPL == KS, "HALF pairs k-steps");
    constexpr int MR = (XR + NW - 1) / NW;                           // LN rows per wave
    static_assert(!MRG || XR == 2, "merge prologue: M <= 2");
    __shared__ __attribute__((aligned(16))) uint4 xs[XS ? XR * XSTR / 8 : 1];
    __shared__ __attribute__((aligned(16))) f32x4 red[NW][NTW][64];

    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ln = lane & 15, lg = lane >> 4;
    const int nt0 = HALF ? (blockIdx.x >> 1) : blockIdx.x * NTW;    // first 16-column tile
    const int half = HALF ? (blockIdx.x & 1) : 0;
    const bool wl = !HALF || ((ln >> 3) == half);                   // this lane's column is ours
    const int ntiles = (N + 63) / 64 * 4;                           // packed rows padded to 64
    const int kbeg = w * (K / NW);
    const int mrow = min(ln, M - 1);

    // Loads that do not depend on the weight stream go FIRST: vmcnt retires in issue order, so
    // the prologue (LN rows) / epilogue (residual) data must be older than the weight prefetch
    // to be waited for without draining it. The empty asm with a memory clobber + sched_barrier
    // keep the compiler from moving these loads behind the prefetch.
    constexpr int NJ = LN ? 4 : 1;                                   // 16-B chunks per lane per row
    uint4 xv[LN ? MR : 1][NJ] = {}, wv[NJ] = {}, bv[NJ] = {};
    // ZK_GF_LNW (B = 1): only the waves that normalise a row (w < M) load the row and the LayerNorm
    // weights; the others issue nothing before their weight prefetch (wave-uniform branch)
    if constexpr (LN) if (!(ZK_GF_LNW && XR == 2 && MR == 1) || w < M) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            wv[j] = *reinterpret_cast<const uint4*>(lnw + lane * 8 + j * 512);
            bv[j] = *reinterpret_cast<const uint4*>(lnb + lane * 8 + j * 512);
        }
#pragma unroll
        for (int rr = 0; rr < MR; ++rr)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                xv[rr][j] = *reinterpret_cast<const uint4*>(A + (size_t)min(w + NW * rr, M - 1) * lda + lane * 8 + j * 512);
    }
    // XC: element e = 512 j + 8 lane of the wave's 2-row image (row e / (K / NW), column kbeg + e % (K / NW))
    uint4 xc[XCN];
    if constexpr (XC) {
#pragma unroll
        for (int j = 0; j < XCN; ++j) {
            const int e = j * 512 + lane * 8, row = e / (KS * 32), col = e % (KS * 32);
            xc[j] = *reinterpret_cast<const uint4*>(A + (size_t)min(row, M - 1) * lda + kbeg + col);
        }
    }
    // MRG: lane = 4 consecutive dims (kbeg + 4 lane: lanes 0-31 the wave's first head, 32-63 its
    // second) of each row m < 2: every split's (m, l, O quad) loaded here (3 loads per split and row),
    // merged after the weight prefetch
    constexpr int NS = MRG ? MRG : 1;
    float mm[MRG ? 2 : 1][NS], ml[MRG ? 2 : 1][NS];
    float4 mo[MRG ? 2 : 1][NS];
    if constexpr (MRG) {
        const int G = (K >> 7) / mhkv;
        const int k = kbeg + 4 * lane;
        const int h = k >> 7, d = k & 127, g = h / G, j = h - g * G;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int m = min(i, M - 1);
            const float* base = mw + ((size_t)m * mhkv + g) * MRG * GF_AT_STR;
#pragma unroll
            for (int sp = 0; sp < NS; ++sp) {
                mm[i][sp] = base[sp * GF_AT_STR + j];
                ml[i][sp] = base[sp * GF_AT_STR + GF_AT_G + j];
                mo[i][sp] = *reinterpret_cast<const float4*>(base + sp * GF_AT_STR + 2 * GF_AT_G + j * 128 + d);
            }
        }
    }
    // mode 3: the position word (scalar, waited below with the skip word) and the lane's RoPE pair
    int posv = 0;
    float2 rcs = make_float2(0.f, 0.f);
    bf16_t rv[4] = {0, 0, 0, 0};                                     // residual x of the epilogue
    const int t = w;                                                 // wave w finishes tile w
    const int n_out = (nt0 + t) * 16 + ln;
    if constexpr (MODE == 2) {
        if (t < NTW && wl && n_out < N) {
#pragma unroll
            for (int i = 0; i < 4; ++i) rv[i] = Cb[(size_t)min(lg * 4 + i, M - 1) * N + n_out];
        }
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    const int lsrc = wl ? lane * 8 : 512 + (lane ^ 8) * 8;          // HALF: k-step 2j+1 for the other half
    const bf16_t* wp[NTW];
#pragma unroll
    for (int tt = 0; tt < NTW; ++tt)
        wp[tt] = W + ((size_t)min(nt0 + tt, ntiles - 1) * (K >> 5) + (kbeg >> 5)) * 512 + lsrc;
    const bf16_t* ap = A + (size_t)mrow * lda + kbeg + lg * 8;
    constexpr int U = PF + 1;
    uint4 wr[U][NTW], ar[U][KPL];
    auto issue = [&](int ls, int slot) {
#pragma unroll
        for (int tt = 0; tt < NTW; ++tt) wr[slot][tt] = ldg_w<true>(wp[tt] + ls * 512 * KPL);
        if constexpr (!XS) {
#pragma unroll
            for (int q = 0; q < KPL; ++q) ar[slot][q] = *reinterpret_cast<const uint4*>(ap + (ls * KPL + q) * 32);
        }
    };
#pragma unroll
    for (int p = 0; p < PF; ++p)
        if (p < NL) issue(p, p);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // the skip word: a scalar load issued here, after the prologue loads and the weight prefetch
    // (every load above is in bounds; nothing is written yet); mode 3 reads the position word in the
    // same round trip and issues its (cos, sin) load, which lands during the weight stream
    int skv;
    if constexpr (MODE == 3) {
        ld_words_here(skip, qk.pos, skv, posv);
        posv = min(max(posv, 0), qk.Smax - 1);
        const int nq = (qk.H + 2 * qk.Hkv) * 128;      // (N) columns [0, H*128) q, then k, then v
        const int ncol = min((nt0 + w) * 16 + ln, nq - 1);
        rcs = *reinterpret_cast<const float2*>(qk.freqs + (size_t)posv * 128 + 2 * ((ncol & 127) >> 1));
    } else {
        skv = ld_word_here(skip);
    }
    if (skv) {
        // (the prologue / epilogue loads too: sunk below this test they would queue behind the
        // weight prefetch and drain it when waited for)
#pragma unroll
        for (int p = 0; p < PF; ++p)
            if (p < NL) {
#pragma unroll
                for (int tt = 0; tt < NTW; ++tt) keep_live(wr[p][tt]);
            }
        if constexpr (LN) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                keep_live(wv[j]);
                keep_live(bv[j]);
#pragma unroll
                for (int rr = 0; rr < MR; ++rr) keep_live(xv[rr][j]);
            }
        }
        if constexpr (MRG) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int sp = 0; sp < NS; ++sp) {
                    asm volatile("" ::"v"(mm[i][sp]), "v"(ml[i][sp]));
                    keep_live(mo[i][sp]);
                }
        }
        if constexpr (XC) {
#pragma unroll
            for (int j = 0; j < XCN; ++j) keep_live(xc[j]);
        }
        if constexpr (MODE == 3) asm volatile("" ::"v"(rcs.x), "v"(rcs.y));
        if constexpr (MODE == 2) asm volatile("" ::"v"((int)rv[0]), "v"((int)rv[1]), "v"((int)rv[2]), "v"((int)rv[3]));
        return;
    }

    if constexpr (LN) {
        // the row values pass through an empty asm here, so no arithmetic on them (and therefore
        // no wait for them) can be hoisted above the weight prefetch
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            opaque(wv[j]);
            opaque(bv[j]);
#pragma unroll
            for (int rr = 0; rr < MR; ++rr) opaque(xv[rr][j]);
        }
        // LayerNorm of each row by one wave (nn.LayerNorm: two-pass fp32 mean / var,
        // y = (x - mean) * rstd * w + b rounded to bf16 -- the arithmetic of ln_row_pre)
        bf16_t* xsb = reinterpret_cast<bf16_t*>(xs);
#pragma unroll
        for (int rr = 0; rr < MR; ++rr) {       // the (clamped) loads above were issued for every
            const int m = w + NW * rr;            // row; only rows < M are normalised (wave-uniform)
            if (m >= M) break;
            float xf[NJ * 8];
#pragma unroll
            for (int j = 0; j < NJ; ++j) unpack8(xv[rr][j], xf + 8 * j);
            float s = 0.f;
#pragma unroll
            for (int e = 0; e < NJ * 8; ++e) s += xf[e];
            const float mean = wave_sum_dpp(s) / (float)K;
            float v = 0.f;
#pragma unroll
            for (int e = 0; e < NJ * 8; ++e) { const float d = xf[e] - mean; v += d * d; }
            const float var = wave_sum_dpp(v) / (float)K;
            const float rstd = 1.0f / sqrtf(var + eps);
            const float nb = -rstd * mean;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                float wf[8], bf[8], o[8];
                unpack8(wv[j], wf);
                unpack8(bv[j], bf);
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    o[e] = __fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(xf[8 * j + e], rstd), nb), wf[e]), bf[e]);
                *reinterpret_cast<uint4*>(xsb + m * XSTR + lane * 8 + j * 512) = pack8(o);
            }
        }
        __syncthreads();
    }
    if constexpr (XC) {
        // each wave writes (and later reads) only its own K range: no workgroup barrier
        bf16_t* xsb = reinterpret_cast<bf16_t*>(xs);
#pragma unroll
        for (int j = 0; j < XCN; ++j) {
            opaque(xc[j]);
            const int e = j * 512 + lane * 8, row = e / (KS * 32), col = e % (KS * 32);
            *reinterpret_cast<uint4*>(xsb + row * XSTR + kbeg + col) = xc[j];
        }
    }
    if constexpr (MRG) {
        // k_attn_combine's arithmetic, split by split in order (fp32, no contraction)
        uint2* xsw = reinterpret_cast<uint2*>(xs);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int sp = 0; sp < NS; ++sp) {
                float2 t2 = make_float2(mm[i][sp], ml[i][sp]);
                asm volatile("" : "+v"(t2.x), "+v"(t2.y), "+v"(mo[i][sp].x), "+v"(mo[i][sp].y), "+v"(mo[i][sp].z),
                             "+v"(mo[i][sp].w));      // no merge arithmetic above the weight prefetch
                mm[i][sp] = t2.x;
                ml[i][sp] = t2.y;
            }
            float Mx = -INFINITY;
#pragma unroll
            for (int sp = 0; sp < NS; ++sp) Mx = fmaxf(Mx, mm[i][sp]);
            float L = 0.f, o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f;
#pragma unroll
            for (int sp = 0; sp < NS; ++sp) {
                const float c = (mm[i][sp] == -INFINITY) ? 0.f : __expf(mm[i][sp] - Mx);
                L += ml[i][sp] * c;
                o0 += mo[i][sp].x * c;
                o1 += mo[i][sp].y * c;
                o2 += mo[i][sp].z * c;
                o3 += mo[i][sp].w * c;
            }
            const float inv = 1.0f / L;
            const int k = kbeg + 4 * lane;
            if (i < M) xsw[(i * XSTR + k) >> 2] = make_uint2(pack2(o0 * inv, o1 * inv), pack2(o2 * inv, o3 * inv));
        }
        // each wave reads back only the dims it wrote (its own K range): no workgroup barrier
    }

    f32x4 acc[NTW];
#pragma unroll
    for (int tt = 0; tt < NTW; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16_t* xrow = reinterpret_cast<const bf16_t*>(xs) + mrow * XSTR + kbeg + lg * 8;
#pragma unroll
    for (int ls = 0; ls < NL; ++ls) {
        if (ls + PF < NL) issue(ls + PF, (ls + PF) % U);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < KPL; ++q) {
            uint4 a;
            if constexpr (XS) a = *reinterpret_cast<const uint4*>(xrow + (ls * KPL + q) * 32);
            else a = ar[ls % U][q];
#pragma unroll
            for (int tt = 0; tt < NTW; ++tt) {
                const uint4 b = q == 0 ? wr[ls % U][tt] : row_ror4<8>(wr[ls % U][tt]);
                acc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a), as_frag(b), acc[tt], 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (ls == 0) ZK_GF_STAMP(1);
    }
    ZK_GF_STAMP(2);
#pragma unroll
    for (int tt = 0; tt < NTW; ++tt) red[w][tt][lane] = acc[tt];
    __syncthreads();
    if (t >= NTW) return;
    f32x4 sum = red[0][t][lane];
#pragma unroll
    for (int q = 1; q < NW; ++q) {
        const f32x4 o = red[q][t][lane];
#pragma unroll
        for (int i = 0; i < 4; ++i) sum[i] = sum[i] + o[i];
    }
    ZK_GF_STAMP(3);
    if (MODE == 1) {
        const int F = N / 2;
        const int f = (nt0 + t) * 8 + (ln & 7);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float mine = round_bf(sum[i]);
            const float other = __shfl_xor(mine, 8, 64);
            const int m = lg * 4 + i;
            if (ln < 8 && m < M && f < F) {
                const float sl = round_bf(other / (1.0f + expf(-other)));
                Cb[(size_t)m * F + f] = f2bf(mine * sl);
            }
        }
        return;
    }
    if constexpr (MODE == 3) {
        const int Hq = qk.H * 128, Hk = qk.Hkv * 128;
        const int d = n_out & 127;
        const bool even = (d & 1) == 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float mine = round_bf(sum[i]);
            const float other = __shfl_xor(mine, 1, 64);      // the pair's other dim (lane ln ^ 1)
            const int m = lg * 4 + i;
            if (m >= M || n_out >= N) continue;
            // (a, b) = dims (2j, 2j+1): o0 = a c - b s, o1 = b c + a s (attn_decode_wg's prologue)
            const float a = even ? mine : other, b = even ? other : mine;
            const float rot = even ? __fsub_rn(__fmul_rn(a, rcs.x), __fmul_rn(b, rcs.y))
                                   : __fadd_rn(__fmul_rn(b, rcs.x), __fmul_rn(a, rcs.y));
            if (n_out < Hq) {
                Cb[(size_t)m * Hq + n_out] = f2bf(rot);
            } else if (n_out < Hq + Hk) {
                const int g = (n_out - Hq) >> 7;
                qk.kc[((size_t)m * qk.Hkv + g) * qk.Smax * 128 + k_off(posv, d >> 3) + (d & 7)] = f2bf(rot);
            } else {
                const int g = (n_out - Hq - Hk) >> 7;
                qk.vt[((size_t)m * qk.Hkv + g) * qk.Smax * 128 + v_off(posv, d)] = f2bf(mine);
            }
        }
        return;
    }
    if (!wl || n_out >= N) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = lg * 4 + i;
        if (m >= M) continue;
        if (MODE == 0) Cf[(size_t)m * N + n_out] = sum[i];
        else Cb[(size_t)m * N + n_out] = f2bf(bf2f(rv[i]) + round_bf(sum[i]));
    }
}

// nn.Linear [N][K] -> fragment-packed [Npad/16][K/32][64][8] (rows >= N zero)
__global__ void k_pack_w(const bf16_t* __restrict__ w, int N, int K, int Npad, bf16_t* __restrict__ out) {
    const size_t total = (size_t)Npad / 16 * (K / 32) * 64;      // 16-byte pieces
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int lane = (int)(i & 63);
        const size_t frag = i >> 6;
        const int kc = (int)(frag % (K / 32));
        const int nt = (int)(frag / (K / 32));
        const int n = nt * 16 + (lane & 15), k = kc * 32 + (lane >> 4) * 8;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (n < N) v = *reinterpret_cast<const uint4*>(w + (size_t)n * K + k);
        *reinterpret_cast<uint4*>(out + i * 8) = v;
    }
}

__global__ void k_permute_fc1(const bf16_t* w, int F, int D, bf16_t* out) {
    const int nr = blockIdx.x;         // new row
    const int q = nr / 16, j = nr % 16;
    const int src = (j < 8) ? (q * 8 + j) : (F + q * 8 + (j - 8));
    const uint4* s = reinterpret_cast<const uint4*>(w + (size_t)src * D);
    uint4* d = reinterpret_cast<uint4*>(out + (size_t)nr * D);
    for (int i = threadIdx.x; i < D / 8; i += blockDim.x) d[i] = s[i];
}

}  // namespace

extern "C" int zk_pack_weights(const void* w, int N, int K, void* out, void* stream) {
    ZK_REQUIRE(N > 0 && K > 0 && K % 64 == 0, "zk_pack_weights: N=%d K=%d (K %% 64 != 0)", N, K);
    const int Npad = (N + 63) / 64 * 64;
    const size_t total = (size_t)Npad / 16 * (K / 32) * 64;
    const int grid = (int)std::min<size_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(k_pack_w, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)w, N, K, Npad,
                       (bf16_t*)out);
    ZK_CHECK_LAUNCH("zk_pack_weights");
    return 0;
}

#ifndef ZK_WS_NCW
#define ZK_WS_NCW 4                // k_gemm_ws compute waves (16-column tiles) per workgroup
#endif
#ifndef ZK_WS_NARROW
#define ZK_WS_NARROW 2             // fewest compute waves of the narrow workgroups (2 or 3; 0: off)
#endif
#ifndef ZK_WS_WIDE
#define ZK_WS_WIDE 5               // compute waves of the wide workgroups for slab GEMMs with > 256 64-column tiles (0: off)
#endif
#define ZK_WS_WIDE_W (ZK_WS_WIDE > 0 ? ZK_WS_WIDE : 1)
#ifndef ZK_WS_NARROW_BELOW
#define ZK_WS_NARROW_BELOW 192     // ... when the 64-column grid has fewer workgroups than this
#endif

// k_gemm_ws regime of zk_gemm_bf16_warm below (16 < M <= 128 or M <= 16 with K/nsplit % 128 != 0)
static bool ws_regime(int M, int K, int nsplit) {
    if (M <= 16 && (K / nsplit) % 128 == 0) return false;
    return M <= BM && K / nsplit / BK <= 32;
}

// k_gemm_ws column groups per compute wave (NG): 16 * 4 * NG columns per workgroup. The slab
// epilogue needs N % 4 == 0 for its whole-row stores (the heads GEMM, N = 9234, keeps NG = 1).
#ifndef ZK_WS_NG0
#define ZK_WS_NG0 1                // split-K slab GEMMs (mode 0)
#endif
#ifndef ZK_WS_NG1
#define ZK_WS_NG1 1                // SwiGLU fc1 (mode 1)
#endif
#ifndef ZK_WS_NGNB
#define ZK_WS_NGNB 1               // activation fragment buffers at NG = 2 (2 exceeds 256 VGPRs at PF 3)
#endif
static int ws_ng(int N, int mode) {
    if (mode == 1) return ZK_WS_NG1;
    return N % 4 == 0 ? ZK_WS_NG0 : 1;
}

#ifndef ZK_GEMM_PF
#define ZK_GEMM_PF 1               // 256 x 256-tile prefill GEMM (gemm_pf.hip) where it fills the chip
#endif
bool zk_gemm_pf_applies(int M, int N, int K, int nsplit);
int zk_gemm_pf(const void* A, long lda, const void* W, int M, int N, int K, int mode, float* C, void* Cb,
               const int32_t* skip, void* stream);

// k_gemm_ws compute waves per workgroup for this GEMM: 4 (64 columns), or for the slab GEMMs whose
// 64-column grid fits the 256 CUs badly ZK_WS_NARROW (fewer than ZK_WS_NARROW_BELOW workgroups: more,
// narrower ones) or ZK_WS_WIDE (more than 256: fewer, wider ones, so no CU runs two)
static int ws_ncw(int M, int N, int nsplit, int mode, int ng) {
    if (ZK_WS_NCW != 4 || mode != 0 || M <= 64 || ng != 1) return ZK_WS_NCW;
    auto tiles = [&](int nw) { return (long)((N + 16 * nw - 1) / (16 * nw)) * nsplit; };
    if (ZK_WS_NARROW > 0 && tiles(4) < ZK_WS_NARROW_BELOW)
        for (int nw = ZK_WS_NARROW; nw <= 3; ++nw)          // the largest grid that still fits the CUs
            if (tiles(nw) <= 256) return nw;
    if (ZK_WS_WIDE > 0 && tiles(4) > 256 && tiles(ZK_WS_WIDE) <= 256) return ZK_WS_WIDE;
    return 4;
}

ZkWarm zk_gemm_warm_desc(const void* W, int M, int N, int K, int nsplit, int mode, int chunks) {
    if (W == nullptr || M <= 16 || ZK_WS_NCW != 4 || !ws_regime(M, K, nsplit) || K % (nsplit * BK) != 0)
        return ZkWarm{nullptr, 0, 0, 0, 0};
    const int ng = ws_ng(N, mode);
    const int nw = ws_ncw(M, N, nsplit, mode, ng);
    const int gx = (N + 16 * nw * ng - 1) / (16 * nw * ng);
    const int excess = gx * nw * ng - (N + 15) / 16;            // grid tiles wholly past N (< nw * ng)
    return ZkWarm{W, K, gx, nsplit,
                  std::min(chunks, K / nsplit / BK) | (ng > 1 ? ng << 8 : 0) | (nw != 4 ? nw << 16 : 0) |
                      (excess << 24)};
}

// Host mirror of warm_unit's tile bound for the descriptor zk_gemm_warm_desc builds: the number of
// 16-column tiles of the packed image the warm-up of this GEMM reads (0 when it is off). Tests check
// it against ceil(N / 16), the tiles the packed image holds a column of (the 48-column
// grid of the c5 Mamba in_proj once warmed 2 tiles past the image).
extern "C" int zk_gemm_warm_tiles(int M, int N, int K, int nsplit, int mode, int chunks) {
    static const char dummy = 0;
    const ZkWarm d = zk_gemm_warm_desc(&dummy, M, N, K, nsplit, mode, chunks);
    if (d.W == nullptr) return 0;
    const int ng = std::max(1, (d.chunks >> 8) & 255), nw = ((d.chunks >> 16) & 255) ? ((d.chunks >> 16) & 255) : 4;
    int hi = 0;
    for (int bx = 0; bx < d.gx; ++bx)
        for (int w = 0; w < nw; ++w)
            for (int g = 0; g < ng; ++g) {
                const int tile = (bx * nw + w) * ng + g;
                if (tile < d.gx * nw * ng - ((d.chunks >> 24) & 255)) hi = std::max(hi, tile + 1);
            }
    return hi;
}

extern "C" int zk_gemm_bf16(const void* A, long lda, const void* W, int M, int N, int K, int nsplit, int mode,
                            float* Cpart, void* Cout, const int32_t* skip_flag, void* stream) {
    return zk_gemm_bf16_warm(A, lda, W, M, N, K, nsplit, mode, Cpart, Cout, skip_flag, ZkWarm{nullptr, 0, 0, 0, 0},
                             stream);
}

int zk_gemm_bf16_warm(const void* A, long lda, const void* W, int M, int N, int K, int nsplit, int mode,
                      float* Cpart, void* Cout, const int32_t* skip_flag, ZkWarm warm, void* stream) {
    ZK_REQUIRE(M > 0 && N > 0 && K > 0, "zk_gemm_bf16: empty shape M=%d N=%d K=%d", M, N, K);
    ZK_REQUIRE(nsplit >= 1 && K % (nsplit * BK) == 0, "zk_gemm_bf16: K=%d must be a multiple of nsplit*%d", K, BK);
    ZK_REQUIRE(lda >= K && lda % 8 == 0, "zk_gemm_bf16: lda=%ld", lda);
    ZK_REQUIRE(mode == 0 || (mode == 1 && nsplit == 1 && N % 16 == 0), "zk_gemm_bf16: bad mode/nsplit");
    const int nchunks = K / nsplit / BK;
    if (M <= 16 && (K / nsplit) % 128 == 0) {
        // weight-stream GEMV (B <= 8 decode): 2 column tiles per workgroup, K quarters per wave
        const int ks = K / nsplit / 128;
        dim3 g((N + 31) / 32, 1, nsplit);
        bool handled = false;
#define ZK_GV(MODE_, KS_)                                                                                         \
    do {                                                                                                          \
        constexpr int PF_ = KS_ < 8 ? KS_ : 8;                                                                    \
        hipLaunchKernelGGL((k_gemv_rk<MODE_, 2, KS_, PF_>), g, dim3(256), 0, (hipStream_t)stream,                 \
                           (const bf16_t*)A, lda, (const bf16_t*)W, M, N, K, K / nsplit, Cpart, (bf16_t*)Cout,     \
                           skip_flag);                                                                             \
        handled = true;                                                                                           \
    } while (0)
        if (mode == 0) {
            switch (ks) {
                case 1: ZK_GV(0, 1); break;
                case 2: ZK_GV(0, 2); break;
                case 4: ZK_GV(0, 4); break;
                case 8: ZK_GV(0, 8); break;
                case 16: ZK_GV(0, 16); break;
                default: break;
            }
        } else {
            switch (ks) {
                case 4: ZK_GV(1, 4); break;
                case 8: ZK_GV(1, 8); break;
                case 16: ZK_GV(1, 16); break;
                default: break;
            }
        }
#undef ZK_GV
        if (handled) {
            ZK_CHECK_LAUNCH("zk_gemm_bf16");
            return 0;
        }
    }
    if (M <= BM && nchunks <= 32) {
        constexpr int NCW = ZK_WS_NCW;            // compute waves per workgroup
        const int ng = M > 16 && NCW == 4 ? ws_ng(N, mode) : 1;
        // a slab GEMM whose 64-column tiles x splits leave a quarter of the CUs idle (the c5 Mamba
        // in_proj: N = 8512 unsplit, 133 tiles; the c3 out_proj, split 4: 128) runs narrower
        // workgroups of 2 or 3 compute waves (16 columns each), the most that still fit one
        // workgroup per CU (the Mamba in_proj at 2 waves would be 266 workgroups for 256 CUs:
        // c5 decode 4.34 -> 4.64 ms); the same per-column K order (bit-identical results).
        const int ncw = M > 16 ? ws_ncw(M, N, nsplit, mode, ng) : NCW;
        dim3 g((N + 16 * ncw * ng - 1) / (16 * ncw * ng), 1, nsplit);
        const int MT = M <= 16 ? 1 : (M <= 32 ? 2 : (M <= 64 ? 4 : 8));
        const size_t lds = (size_t)WS_NB * MT * 16 * BK * 2 + (warm.W ? 1024 : 0);     // + warm-up sink
#define ZK_WS_LAUNCH5(MODE_, NCH_, MT_, NG_, NCW_)                                                                 \
    do {                                                                                                          \
        constexpr int NB_ = NG_ > 1 ? ZK_WS_NGNB : (NCW_ > 5 ? 1 : 2);                                            \
        auto kern_ = &k_gemm_ws<MODE_, NCH_, (MODE_ ? WS_PF : WS_PF0), MT_, NCW_, NG_, NB_>;                       \
        if (lds > 65536)                                                                                          \
            hipFuncSetAttribute(reinterpret_cast<const void*>(kern_), hipFuncAttributeMaxDynamicSharedMemorySize, \
                                (int)lds);                                                                        \
        hipLaunchKernelGGL(kern_, g, dim3(64 * (NCW_ + ws_nld<NCW_, MT_>())), lds, (hipStream_t)stream,                \
                           (const bf16_t*)A, lda, (const bf16_t*)W, M, N, K, K / nsplit, Cpart, (bf16_t*)Cout,      \
                           skip_flag, (const bf16_t*)warm.W, warm.K, warm.gx, warm.gz, warm.chunks);              \
        handled = true;                                                                                           \
    } while (0)
#define ZK_WS_LAUNCH4(MODE_, NCH_, MT_, NG_) ZK_WS_LAUNCH5(MODE_, NCH_, MT_, NG_, NCW)
#define ZK_WS_LAUNCH3(MODE_, NCH_, MT_)                                                                            \
    do {                                                                                                          \
        if ((MT_) == 8 && ng == 2) ZK_WS_LAUNCH4(MODE_, NCH_, MT_, 2);                                            \
        else if ((MODE_) == 0 && (MT_) == 8 && ncw == 2 && NCW == 4)                                              \
            ZK_WS_LAUNCH5(MODE_, NCH_, MT_, 1, 2);                                                                 \
        else if ((MODE_) == 0 && (MT_) == 8 && ncw == 3 && NCW == 4)                                              \
            ZK_WS_LAUNCH5(MODE_, NCH_, MT_, 1, 3);                                                                 \
        else if ((MODE_) == 0 && (MT_) == 8 && ncw == ZK_WS_WIDE_W && ncw != NCW)                                   \
            ZK_WS_LAUNCH5(MODE_, NCH_, MT_, 1, ZK_WS_WIDE_W);                                                      \
        else ZK_WS_LAUNCH4(MODE_, NCH_, MT_, 1);                                                                  \
    } while (0)
#define ZK_WS_LAUNCH(MODE_, NCH_)                                                                                  \
    do {                                                                                                          \
        switch (MT) {                                                                                             \
            case 1: ZK_WS_LAUNCH3(MODE_, NCH_, 1); break;                                                         \
            case 2: ZK_WS_LAUNCH3(MODE_, NCH_, 2); break;                                                         \
            case 4: ZK_WS_LAUNCH3(MODE_, NCH_, 4); break;                                                         \
            default: ZK_WS_LAUNCH3(MODE_, NCH_, 8); break;                                                        \
        }                                                                                                         \
    } while (0)
        bool handled = false;
        if (mode == 0) {
            switch (nchunks) {
                case 2: ZK_WS_LAUNCH(0, 2); break;
                case 4: ZK_WS_LAUNCH(0, 4); break;
                case 8: ZK_WS_LAUNCH(0, 8); break;
                case 16: ZK_WS_LAUNCH(0, 16); break;
                case 32: ZK_WS_LAUNCH(0, 32); break;
                default: break;
            }
        } else {
            switch (nchunks) {
                case 4: ZK_WS_LAUNCH(1, 4); break;
                case 8: ZK_WS_LAUNCH(1, 8); break;
                case 16: ZK_WS_LAUNCH(1, 16); break;
                case 32: ZK_WS_LAUNCH(1, 32); break;
                default: break;
            }
        }
        if (handled) {
            ZK_CHECK_LAUNCH("zk_gemm_bf16");
            return 0;
        }
#undef ZK_WS_LAUNCH5
#undef ZK_WS_LAUNCH4
#undef ZK_WS_LAUNCH3
#undef ZK_WS_LAUNCH
    }
    // large M (prefill) with at least one 256 x 256 tile per CU: gemm_pf.hip
    if (ZK_GEMM_PF && zk_gemm_pf_applies(M, N, K, nsplit))
        return zk_gemm_pf(A, lda, W, M, N, K, mode, Cpart, Cout, skip_flag, stream);
    // large M (prefill): two 16-column tiles per wave for the slab GEMMs (c3 prefill: in_proj
    // 1.01 vs 1.09 ms, fc2 1.98 vs 2.29 ms; the SwiGLU fc1 is faster with one: 4.87 vs 5.24 ms)
    const int ntw = (mode == 0 && M > BM && N >= 8 * BN) ? 2 : 1;
    dim3 grid((N + BN * ntw - 1) / (BN * ntw), (M + BM - 1) / BM, nsplit);
    const int U = (nchunks % 4 == 0) ? 4 : (nchunks % 2 == 0 ? 2 : 1);
#define ZK_GEMM_LAUNCH(MODE_, U_)                                                                         \
    do {                                                                                                  \
        if (ntw == 2)                                                                                     \
            hipLaunchKernelGGL((k_gemm<MODE_, U_, false, 2>), grid, dim3(NT), 0, (hipStream_t)stream,     \
                               (const bf16_t*)A, lda, (const bf16_t*)W, M, N, K, K / nsplit, Cpart,       \
                               (bf16_t*)Cout, skip_flag);                                                 \
        else                                                                                              \
            hipLaunchKernelGGL((k_gemm<MODE_, U_>), grid, dim3(NT), 0, (hipStream_t)stream,               \
                               (const bf16_t*)A, lda, (const bf16_t*)W, M, N, K, K / nsplit, Cpart,       \
                               (bf16_t*)Cout, skip_flag);                                                 \
    } while (0)
    if (mode == 0) {
        if (U == 4) ZK_GEMM_LAUNCH(0, 4); else if (U == 2) ZK_GEMM_LAUNCH(0, 2); else ZK_GEMM_LAUNCH(0, 1);
    } else {
        if (U == 4) ZK_GEMM_LAUNCH(1, 4); else if (U == 2) ZK_GEMM_LAUNCH(1, 2); else ZK_GEMM_LAUNCH(1, 1);
    }
#undef ZK_GEMM_LAUNCH
    ZK_CHECK_LAUNCH("zk_gemm_bf16");
    return 0;
}

extern "C" int zk_gemv_fused(const void* A, long lda, const void* W, int M, int N, int K, int mode,
                             const void* ln_w, const void* ln_b, float eps, float* Cf, void* Cb,
                             const int32_t* skip_flag, void* stream) {
    ZK_REQUIRE(M >= 1 && M <= 16 && N > 0, "zk_gemv_fused: M=%d (1..16) N=%d", M, N);
    ZK_REQUIRE(K == 2048 || K == 4096 || K == 8192, "zk_gemv_fused: K=%d (2048, 4096 or 8192)", K);
    ZK_REQUIRE(lda >= K && lda % 8 == 0, "zk_gemv_fused: lda=%ld", lda);
    ZK_REQUIRE(mode >= 0 && mode <= 2, "zk_gemv_fused: mode %d", mode);
    ZK_REQUIRE(mode != 1 || N % 16 == 0, "zk_gemv_fused: SwiGLU needs N %% 16 == 0");
    ZK_REQUIRE((ln_w == nullptr) == (ln_b == nullptr), "zk_gemv_fused: LN needs both w and b");
    ZK_REQUIRE(ln_w == nullptr || K == 2048, "zk_gemv_fused: LN prologue needs K = 2048 (K=%d)", K);
    ZK_REQUIRE(mode == 0 ? Cf != nullptr : Cb != nullptr, "zk_gemv_fused: missing output");
    const int tiles = (N + 15) / 16;
    // >= 256 workgroups: half tiles below 256 tiles (out_proj / fc2: N = 2048), pairs of tiles
    // from 512 (fc1, heads). With the LayerNorm prologue one tile per workgroup even below 256
    // tiles (in_proj, N = 3072: 192 workgroups, 6.5 vs 7.5 us with half tiles at B = 1 --
    // the prologue's latency, not the weight stream, sets its time; tools/gemv_probe.sh)
    int lay = (mode != 1 && tiles < 256 && !ln_w) ? 0 : (tiles >= 512 ? 2 : 1);
    const int grid = lay == 0 ? 2 * tiles : (lay == 2 ? (tiles + 1) / 2 : tiles);
    const bool ln = ln_w != nullptr;
    (void)ln;
    bool handled = false;
    // tuning knobs (compile-time, build_variant): waves per workgroup, k-steps in flight per wave
#ifndef ZK_GF_NW
#define ZK_GF_NW 4
#endif
#ifndef ZK_GF_NWH
#define ZK_GF_NWH 8
#endif
#ifndef ZK_GF_PF
#define ZK_GF_PF 8
#endif
#ifndef ZK_GF_PF2
#define ZK_GF_PF2 ZK_GF_PF         // k-steps in flight of the B = 1 (XR = 2) instantiations
#endif
#ifndef ZK_GF_PFLN
#define ZK_GF_PFLN 12              // k-steps in flight of the B = 1 LayerNorm-prologue one-tile GEMV (in_proj):
#endif                             // c2 step 1.045-1.048 vs 1.051-1.053 ms at 8, 1.054-1.055 at 16 (r3_b1_gemv_pf_ab)
#define ZK_GF(MODE_, LN_, NTW_, HALF_, NW_, KSW_)                                                            \
    do {                                                                                                      \
        constexpr int KS_ = (KSW_) / (NW_);                                                                   \
        constexpr int NL_ = HALF_ ? KS_ / 2 : KS_;                                                            \
        constexpr int PB_ = (LN_ && NTW_ == 1 && !HALF_) ? ZK_GF_PFLN : ZK_GF_PF2;                            \
        if (M <= 2)                                                                               \
            hipLaunchKernelGGL((k_gemv_f<MODE_, LN_, NTW_, HALF_, NW_, KS_, (NL_ < PB_ ? NL_ : PB_),              \
                                          0, 2>),                                                             \
                               dim3(grid), dim3(64 * (NW_)), 0, (hipStream_t)stream, (const bf16_t*)A, lda,    \
                               (const bf16_t*)W, M, N, K, (const bf16_t*)ln_w, (const bf16_t*)ln_b, eps, Cf,    \
                               (bf16_t*)Cb, skip_flag, nullptr, 1);                                            \
        else                                                                                                  \
            hipLaunchKernelGGL((k_gemv_f<MODE_, LN_, NTW_, HALF_, NW_, KS_, (NL_ < ZK_GF_PF ? NL_ : ZK_GF_PF)>),  \
                               dim3(grid), dim3(64 * (NW_)), 0, (hipStream_t)stream, (const bf16_t*)A, lda,    \
                               (const bf16_t*)W, M, N, K, (const bf16_t*)ln_w, (const bf16_t*)ln_b, eps, Cf,    \
                               (bf16_t*)Cb, skip_flag, nullptr, 1);                                            \
        handled = true;                                                                                       \
    } while (0)
#define ZK_GF_LAY(MODE_, LN_, KSW_)                                     \
    do {                                                                \
        if (lay == 0) ZK_GF(MODE_, LN_, 1, true, ZK_GF_NWH, KSW_);      \
        else if (lay == 1) ZK_GF(MODE_, LN_, 1, false, ZK_GF_NW, KSW_); \
        else ZK_GF(MODE_, LN_, 2, false, ZK_GF_NW, KSW_);               \
    } while (0)
#define ZK_GF_MODE(LN_, KSW_)                       \
    do {                                            \
        if (mode == 0) ZK_GF_LAY(0, LN_, KSW_);     \
        else if (mode == 1) ZK_GF_LAY(1, LN_, KSW_); \
        else ZK_GF_LAY(2, LN_, KSW_);               \
    } while (0)
    // KSW = K / 32: k-steps of the whole workgroup
    if (ln) ZK_GF_MODE(true, 64);
    else if (K == 2048) ZK_GF_MODE(false, 64);
    else if (K == 4096) ZK_GF_MODE(false, 128);
    else ZK_GF_MODE(false, 256);
#undef ZK_GF_MODE
#undef ZK_GF_LAY
#undef ZK_GF
    ZK_REQUIRE(handled, "zk_gemv_fused: no kernel for K=%d", K);
    ZK_CHECK_LAUNCH("zk_gemv_fused");
    return 0;
}

// Experiment (tools/microbench.py gemv_warm): a launch that pre-reads into each XCD's L2 the first
// `steps` weight loads of every wave of a k_gemv_f launch of the given layout (same grid, same
// workgroup -> tile / K-range map and per-lane addresses), by LDS-DMA into a sink.
template <int NTW, bool HALF, int NW>
__global__ __launch_bounds__(64 * NW) void k_gemv_warm(const bf16_t* __restrict__ W, int N, int K, int steps) {
    __shared__ __attribute__((aligned(16))) char sink[1024];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ln = lane & 15;
    const int nt0 = HALF ? (blockIdx.x >> 1) : blockIdx.x * NTW;
    const int half = HALF ? (blockIdx.x & 1) : 0;
    const bool wl = !HALF || ((ln >> 3) == half);
    constexpr int KPL = HALF ? 2 : 1;
    const int ntiles = (N + 63) / 64 * 4;
    const int kbeg = w * (K / NW);
    const int lsrc = wl ? lane * 8 : 512 + (lane ^ 8) * 8;
    void* snk = sink;
    for (int tt = 0; tt < NTW; ++tt) {
        const bf16_t* p = W + ((size_t)min(nt0 + tt, ntiles - 1) * (K >> 5) + (kbeg >> 5)) * 512 + lsrc;
        for (int ls = 0; ls < steps; ++ls)
            __builtin_amdgcn_global_load_lds((const void*)(p + (size_t)ls * 512 * KPL), snk, 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

extern "C" int zk_gemv_warm(const void* W, int N, int K, int lay, int steps, void* stream) {
    ZK_REQUIRE(lay >= 0 && lay <= 2 && steps >= 1 && K % 2048 == 0, "zk_gemv_warm: lay %d steps %d K %d", lay, steps,
               K);
    const int tiles = (N + 15) / 16;
    if (lay == 0)
        hipLaunchKernelGGL((k_gemv_warm<1, true, 8>), dim3(2 * tiles), dim3(512), 0, (hipStream_t)stream,
                           (const bf16_t*)W, N, K, steps);
    else if (lay == 1)
        hipLaunchKernelGGL((k_gemv_warm<1, false, 4>), dim3(tiles), dim3(256), 0, (hipStream_t)stream,
                           (const bf16_t*)W, N, K, steps);
    else
        hipLaunchKernelGGL((k_gemv_warm<2, false, 4>), dim3((tiles + 1) / 2), dim3(256), 0, (hipStream_t)stream,
                           (const bf16_t*)W, N, K, steps);
    ZK_CHECK_LAUNCH("zk_gemv_warm");
    return 0;
}

#ifdef ZK_GF_PROF
extern "C" int zk_gf_prof_set(uint64_t* p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_gf_prof), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int zk_gemv_qkv_rope(const void* x, const void* W, int M, int H, int Hkv, int hd, const void* ln_w,
                                const void* ln_b, float eps, void* q_out, void* k_cache, void* vt_cache, int Smax,
                                const int32_t* pos_dev, const float* freqs, const int32_t* skip_flag, void* stream) {
    ZK_REQUIRE(M >= 1 && M <= 2, "zk_gemv_qkv_rope: M=%d (1..2)", M);
    ZK_REQUIRE(hd == 128 && H % Hkv == 0 && H / Hkv <= AT_G, "zk_gemv_qkv_rope: H=%d Hkv=%d hd=%d", H, Hkv, hd);
    const int K = H * hd, N = (H + 2 * Hkv) * hd;
    ZK_REQUIRE(K == 2048, "zk_gemv_qkv_rope: d_model %d (2048 only: the LayerNorm prologue)", K);
    ZK_REQUIRE(x && W && ln_w && ln_b && q_out && k_cache && vt_cache && pos_dev && freqs,
               "zk_gemv_qkv_rope: null argument");
    ZK_REQUIRE(Smax > 0 && Smax % 32 == 0, "zk_gemv_qkv_rope: Smax=%d", Smax);
    const GfQkv qk{(bf16_t*)k_cache, (bf16_t*)vt_cache, pos_dev, freqs, H, Hkv, Smax};
    constexpr int KS = 64 / ZK_GF_NW, NL = KS, PB = ZK_GF_PFLN;
    hipLaunchKernelGGL((k_gemv_f<3, true, 1, false, ZK_GF_NW, KS, (NL < PB ? NL : PB), 0, 2>), dim3(N / 16),
                       dim3(64 * ZK_GF_NW), 0, (hipStream_t)stream, (const bf16_t*)x, (long)K, (const bf16_t*)W, M, N,
                       K, (const bf16_t*)ln_w, (const bf16_t*)ln_b, eps, nullptr, (bf16_t*)q_out, skip_flag, nullptr, 1,
                       qk);
    ZK_CHECK_LAUNCH("zk_gemv_qkv_rope");
    return 0;
}

extern "C" int zk_gemv_attn_out(const float* work, int nsplit, int Hkv, const void* W, int M, int N, int K,
                                void* x, const int32_t* skip_flag, void* stream) {
    ZK_REQUIRE(M >= 1 && M <= 2, "zk_gemv_attn_out: M=%d (1..2)", M);
    ZK_REQUIRE(K == 2048 && N > 0 && N % 16 == 0, "zk_gemv_attn_out: K=%d (2048) N=%d", K, N);
    ZK_REQUIRE(Hkv >= 1 && (K / 128) % Hkv == 0 && (K / 128) / Hkv <= GF_AT_G, "zk_gemv_attn_out: Hkv=%d", Hkv);
    ZK_REQUIRE(work != nullptr && x != nullptr, "zk_gemv_attn_out: null buffer");
    const int grid = 2 * ((N + 15) / 16);                   // half tiles, 8 K-range waves
#define ZK_GAO(NS_)                                                                                              \
    hipLaunchKernelGGL((k_gemv_f<2, false, 1, true, 8, 8, 4, NS_, 2>), dim3(grid), dim3(512), 0,               \
                       (hipStream_t)stream, reinterpret_cast<const bf16_t*>(work), (long)K, (const bf16_t*)W, M,  \
                       N, K, nullptr, nullptr, 0.f, nullptr, (bf16_t*)x, skip_flag, work, Hkv)
    switch (nsplit) {
        case 2: ZK_GAO(2); break;
        case 4: ZK_GAO(4); break;
        case 8: ZK_GAO(8); break;
        case 16: ZK_GAO(16); break;
        default: ZK_REQUIRE(false, "zk_gemv_attn_out: nsplit=%d (2, 4, 8 or 16)", nsplit);
    }
#undef ZK_GAO
    ZK_CHECK_LAUNCH("zk_gemv_attn_out");
    return 0;
}

// L2 warm-up of a k_gemm_ws launch's first weight chunks (experiment): workgroup r of a 1-D grid
// (same XCD as r % 8) reads, for every GEMM workgroup L = r, r + nwg, ... (same XCD), the first
// `chunks` 2 KB weight chunks of each of its 4 compute waves, so they are L2 hits when it starts.
__global__ __launch_bounds__(256) void k_l2_warm_ws(const bf16_t* __restrict__ W, int K, int gx, int gz, int chunks,
                                                    uint32_t* sink) {
    __shared__ __attribute__((aligned(16))) char lsink[1024];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    warm_units(W, K, gx, gz, chunks, blockIdx.x, gridDim.x, w, 4, lane, lsink);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    (void)sink;
}

extern "C" int zk_l2_warm_gemm(const void* W, int N, int K, int nsplit, int chunks, int nwg, void* sink, void* stream) {
    ZK_REQUIRE(N > 0 && K % (nsplit * BK) == 0 && chunks >= 1 && chunks <= K / nsplit / BK && nwg > 0,
               "zk_l2_warm_gemm: N=%d K=%d nsplit=%d chunks=%d", N, K, nsplit, chunks);
    hipLaunchKernelGGL(k_l2_warm_ws, dim3(nwg), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)W, K,
                       (N + BN - 1) / BN, nsplit, chunks, (uint32_t*)sink);
    ZK_CHECK_LAUNCH("zk_l2_warm_gemm");
    return 0;
}

extern "C" int zk_permute_fc1(const void* w_fc1, int F, int D, void* w_out, void* stream) {
    ZK_REQUIRE(F % 8 == 0 && D % 8 == 0, "zk_permute_fc1: F=%d D=%d", F, D);
    hipLaunchKernelGGL(k_permute_fc1, dim3(2 * F), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)w_fc1, F, D,
                       (bf16_t*)w_out);
    ZK_CHECK_LAUNCH("zk_permute_fc1");
    return 0;
}
