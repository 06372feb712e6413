// Prefill GEMM for gfx950: C[M][N] = A[M][K] . W[N][K]^T at large M (the prefill of
// Zonos.generate runs every projection over R * (Lc + P + 1) rows: 52,608 at c3).
//
// The decode GEMMs (gemm.hip) stream each weight byte once for 128 rows; here the same weights
// meet hundreds of row blocks, so the work is MFMA-bound and the tile is sized for reuse: a
// 256 x 256 output tile per workgroup of 8 waves (2 row halves x 4 column quarters, 128 x 64 per
// wave: 32 accumulator tiles, every LDS fragment feeds 4 or 8 MFMAs), K in 64-deep steps through
// two 64 KB LDS stages filled by LDS-DMA (global_load_lds_dwordx4): the activation rows in the
// XOR-swizzled 128-B row layout of the decode GEMM (lds_off: conflict-free ds_read_b128), the
// weights as the fragment-packed image itself ([N/16][K/32][64 lanes][8]: every 16 x 32 B
// fragment is a lane-linear 1 KB block, so the copy needs no address math and the read no swizzle).
// The next step's stage is issued after the barrier that retires the stage it overwrites, one
// piece per 4 MFMAs over the step's first k-slice (ZK_PF_SPREAD), so the rest of the step covers its
// latency and the issues do not stall the MFMAs. Tiles are handed to the 8 XCDs in
// contiguous runs and walked in 4 x 8 (row x column) blocks, so each XCD's L2 re-serves both
// operands to the 32 workgroups it runs at once.
//
// mode 0: fp32 C (the split-1 "slab" the prefill consumers read); mode 1: fused SwiGLU of the
// interleaved fc1 rows (8 y + 8 gate per 16-column group) -> bf16 Cb[M][N/2] (_torch.py:150-152).
// Results depend on K only (fixed k order per output element), not on M, N or the tile position.
#include "common.h"
#include "attn_common.h"
#include "../../include/zonos_hip.h"

namespace {

constexpr int PF_BM = 256, PF_NT = 512;
#ifndef ZK_PF_EPI
#define ZK_PF_EPI 1                        // LDS-staged whole-row epilogues (0: direct register stores, A/B)
#endif
// diagnostic builds only (timing of the main loop's parts; results are wrong): NOWAIT skips the copy
// waits (the barrier stays), NOMFMA the MFMAs (the LDS reads stay), NOLDS the LDS fragment reads
#ifndef ZK_PF_DIAG_NOWAIT
#define ZK_PF_DIAG_NOWAIT 0
#endif
#ifndef ZK_PF_DIAG_NOFILL          // (no LDS-DMA at all: MFMAs + LDS reads + barriers only)
#define ZK_PF_DIAG_NOFILL 0
#endif
#ifndef ZK_PF_DIAG_NOEPI           // (no epilogue stores)
#define ZK_PF_DIAG_NOEPI 0
#endif
#ifndef ZK_PF_DIAG_NOMFMA
#define ZK_PF_DIAG_NOMFMA 0
#endif
// the refill of the next stage: piece j of a wave issued right after MFMA j * ZK_PF_SPREAD of the step
// (0: all pieces at the top of the step). A burst of 8 LDS-DMA issues holds the wave's MFMAs back;
// one piece per 4 MFMAs (over the step's first k-slice) measured fastest: fc1 3.31-3.38 -> 3.18 ms,
// qkv 0.77 -> 0.73, o 0.47-0.48 -> 0.45, fc2 1.50 -> 1.42 (1, 2 or 8 MFMAs per piece, 32-deep stages
// and 256 x 384 tiles slower; profiles/r5_prefill_spread_ab.txt)
#ifndef ZK_PF_SPREAD
#define ZK_PF_SPREAD 4
#endif
#ifndef ZK_PF_DIAG_NOLDS
#define ZK_PF_DIAG_NOLDS 0
#endif

// Activation rows in LDS: BKS-deep steps give rows of 2 * BKS bytes. The 16-B chunk c of row r is
// stored at chunk c ^ swz(r), which makes every ds_read_b128 of an A fragment (16 rows x one chunk
// per lane quarter) conflict-free: rows of 128 B (BKS = 64) XOR with r % 8, rows of 64 B
// (BKS = 32) with 2 * ((r / 8) % 2) (searched exhaustively over the four lane groups).
template <int BKS>
ZK_DEV int pf_swz(int r) { return BKS == 64 ? (r & 7) : (((r >> 3) & 1) << 1); }
template <int BKS>
ZK_DEV int pf_a_off(int r, int c) { return r * (2 * BKS) + ((c ^ pf_swz<BKS>(r)) << 4); }

template <int N_>
ZK_DEV void pf_vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory"); }
// wait until at most `after` stages of LPS pieces are outstanding (after <= MAXA)
template <int LPS, int MAXA>
ZK_DEV void pf_wait_after(int after) {
    static_assert(MAXA <= 3 && MAXA * LPS <= 63, "vmcnt field");
    if constexpr (MAXA >= 3) {
        if (after >= 3) { pf_vm_wait<3 * LPS>(); return; }
    }
    if constexpr (MAXA >= 2) {
        if (after == 2) { pf_vm_wait<2 * LPS>(); return; }
    }
    if constexpr (MAXA >= 1) {
        if (after == 1) { pf_vm_wait<LPS>(); return; }
    }
    pf_vm_wait<0>();
}

// LDS-DMA of one 1 KB piece (64 lanes x 16 B) to the wave-uniform LDS byte address `lds`. Inline asm:
// hipcc's waitcnt pass would otherwise treat the pending LDS write as aliasing every ds_read of
// the step and wait vmcnt(0) -- for the NEXT stage's copies -- before the first one. The kernel
// waits for its copies itself (pf_vm_wait + barrier).
ZK_DEV void pf_glds(const void* gsrc, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds)
                 : "memory");
}
// The same with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane byte offset: one VGPR per
// piece instead of a 64-bit address pair.
ZK_DEV void pf_glds_s(const void* sbase, uint32_t voff, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds)
                 : "memory");
}

// Tile order: workgroup id -> (row block, column block). Ids are dispatched round-robin over the
// XCDs (id % 8); each XCD gets a contiguous run of the tile sequence (bijective for any count),
// and the sequence walks 4 x 8 blocks of tiles, column-minor, so concurrently running tiles of an
// XCD share 4 activation row blocks and 8 weight column blocks. Placement only.
ZK_DEV void pf_tile(int L, int nwg, int tm, int tn, int& bm, int& bn) {
    const int xcd = L & 7, q = nwg >> 3, r = nwg & 7;
    const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
    constexpr int GM = 4, GN = 8;
    const int gcols = (tn + GN - 1) / GN;              // column groups of GN
    const int per = GM * tn;                           // tiles per band of GM row blocks
    const int band = t / per, in = t - band * per;
    const int rows = min(GM, tm - band * GM);          // row blocks in this band
    const int cg = in / (rows * GN), rem = in - cg * rows * GN;
    const int cols = min(GN, tn - cg * GN);            // column blocks in this group
    bm = band * GM + rem / cols;
    bn = cg * GN + rem % cols;
    (void)gcols;
}

// acc[mt][nt][i] = C[m0 + wr*128 + mt*16 + lg*4 + i][n0 + wc*16*NTN + nt*16 + ln]
template <int MODE, int NTN>
ZK_DEV void pf_epilogue(const f32x4 (&acc)[8][NTN], int m0, int n0, int wr, int wc, int ln, int lg, int M, int N,
                        float* __restrict__ C, bf16_t* __restrict__ Cb) {
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) {
        const int c0 = n0 + wc * 16 * NTN + nt * 16;
        if (MODE == 0) {
            const int n = c0 + ln;
            if (n < N) {
#pragma unroll
                for (int mt = 0; mt < 8; ++mt)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int m = m0 + wr * 128 + mt * 16 + lg * 4 + i;
                        if (m < M) C[(size_t)m * N + n] = acc[mt][nt][i];
                    }
            }
        } else {
            const int F = N / 2;
            const int f = c0 / 2 + (ln & 7);
#pragma unroll
            for (int mt = 0; mt < 8; ++mt)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float mine = round_bf(acc[mt][nt][i]);
                    const float other = __shfl_xor(mine, 8, 64);
                    const int m = m0 + wr * 128 + mt * 16 + lg * 4 + i;
                    if (ln < 8 && m < M && f < F) {
                        const float sl = round_bf(other / (1.0f + expf(-other)));     // F.silu in bf16
                        Cb[(size_t)m * F + f] = f2bf(mine * sl);
                    }
                }
        }
    }
}

// Epilogues staged through the (then idle) LDS stages, so every global store writes whole rows:
// the register layout above writes 16 columns of 4 rows per instruction (64-B fp32 pieces, or 16-B
// bf16 pieces from half the lanes in the SwiGLU form).
//   mode 1: the bf16-rounded y / gate columns of the tile (row stride pf_es halves, padded against
//           bank conflicts; the 256 x 384 tile in two passes of 128 rows, one per wave row half),
//           then every lane computes y * silu(gate) for 8 outputs and stores them as one 16-B piece:
//           a row's 16-column groups write one contiguous row segment (the arithmetic and rounding
//           points of pf_epilogue<1>, bit-identical);
//   mode 0: the fp32 tile in two halves of 128 rows (row stride pf_ef floats), each stored as whole
//           1 KB rows (one wave instruction per row; 256-column tiles only).
template <int NTN> constexpr int pf_bn = 64 * NTN;                 // tile columns: 4 waves x NTN x 16
template <int NTN> constexpr int pf_es = pf_bn<NTN> + 8;          // mode 1 staging row stride (halves)
template <int NTN> constexpr int pf_rh = NTN > 4 ? 128 : 256;     // mode 1 rows per staging pass
template <int NTN> constexpr int pf_ef = pf_bn<NTN> + 4;          // mode 0 staging row stride (floats)
template <int NTN> constexpr int pf_epi_lds1 = pf_rh<NTN> * pf_es<NTN> * 2;   // 135,168 B (4) / 100,352 B (6)
template <int NTN> constexpr int pf_epi_lds0 = NTN == 4 ? (PF_BM / 2) * pf_ef<NTN> * 4 : 0;   // 133,120 B
template <int MODE, int NTN>
ZK_DEV void pf_epilogue_lds(const f32x4 (&acc)[8][NTN], char* smem, int m0, int n0, int wr, int wc, int ln, int lg,
                            int M, int N, float* __restrict__ C, bf16_t* __restrict__ Cb) {
    static_assert(MODE == 1 || NTN == 4, "fp32 staged epilogue: 256-column tiles");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();                                   // every wave's last stage read
    if constexpr (MODE == 1) {
        constexpr int ES = pf_es<NTN>, RH = pf_rh<NTN>, G = pf_bn<NTN> / 16;   // G 16-column groups per row
        bf16_t* t = reinterpret_cast<bf16_t*>(smem);
        const int F = N / 2, f0 = n0 / 2;
#pragma unroll
        for (int pass = 0; pass < PF_BM / RH; ++pass) {
            if (RH == PF_BM || wr == pass) {
                const int rb = RH == PF_BM ? wr * 128 : 0;
#pragma unroll
                for (int mt = 0; mt < 8; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            t[(rb + mt * 16 + lg * 4 + i) * ES + wc * 16 * NTN + nt * 16 + ln] = f2bf(acc[mt][nt][i]);
            }
            __syncthreads();
            // item q = (row q / G, group q % G): outputs f0 + 8 (q % G) .. + 7 of that row
            auto item = [&](int q) {
                const int r = q / G, gi = q - r * G, m = m0 + pass * RH + r;
                if (m >= M || f0 + gi * 8 >= F) return;
                const bf16_t* src = t + r * ES + gi * 16;
                const uint4 yv = *reinterpret_cast<const uint4*>(src), gv = *reinterpret_cast<const uint4*>(src + 8);
                float y[8], g[8], o[8];
                unpack8(yv, y);
                unpack8(gv, g);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float sl = round_bf(g[j] / (1.0f + expf(-g[j])));     // F.silu in bf16
                    o[j] = y[j] * sl;
                }
                *reinterpret_cast<uint4*>(Cb + (size_t)m * F + f0 + gi * 8) = pack8(o);
            };
            if constexpr (NTN > 4) {                   // (the other row half's 192 accumulators are live)
#pragma unroll 1
                for (int q = tid; q < RH * G; q += PF_NT) item(q);
            } else {
#pragma unroll 2
                for (int q = tid; q < RH * G; q += PF_NT) item(q);
            }
            if (pass + 1 < PF_BM / RH) __syncthreads();   // the next pass overwrites the staging rows
        }
    } else {
        constexpr int EF = pf_ef<NTN>;
        float* t = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            if (wr == half) {
#pragma unroll
                for (int mt = 0; mt < 8; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            t[(mt * 16 + lg * 4 + i) * EF + wc * 64 + nt * 16 + ln] = acc[mt][nt][i];
            }
            __syncthreads();
            // 128 rows x 1 KB: wave w stores rows w, w + 8, ...; lane L the floats 4L .. 4L + 3
#pragma unroll 4
            for (int r = w; r < 128; r += 8) {
                const int m = m0 + half * 128 + r;
                if (m < M && n0 + 4 * lane < N) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(t + r * EF + 4 * lane);
                    *reinterpret_cast<f32x4*>(C + (size_t)m * N + n0 + 4 * lane) = v;
                }
            }
            if (half == 0) __syncthreads();            // the second half overwrites the staging rows
        }
    }
}

// BKS: K depth of one LDS stage (32 or 64); NSTG: stages in the ring (NSTG - 1 in flight);
// NTN: 16-column tiles per wave (4: 256 x 256 workgroup tiles; 6: 256 x 384, 1.2x fewer fill bytes
// per FLOP -- two 80 KB stages fill the 160 KB LDS).
template <int MODE, int BKS, int NSTG, int NTN>
__global__ __launch_bounds__(PF_NT, 1) void k_gemm_pf(const bf16_t* __restrict__ A, long lda,
                                                      const bf16_t* __restrict__ W, int M, int N, int K,
                                                      float* __restrict__ C, bf16_t* __restrict__ Cb,
                                                      const int32_t* skip) {
    constexpr int KSS = BKS / 32;                        // 32-deep MFMA k-slices per stage
    constexpr int BN = pf_bn<NTN>;
    constexpr int AST = PF_BM * BKS * 2, BST = BN * BKS * 2, ST = AST + BST;
    constexpr int RPP = 1024 / (2 * BKS);                // activation rows per 1 KB LDS-DMA piece
    constexpr int CPR = 2 * BKS / 16;                    // 16-B chunks per activation row
    constexpr int NA = AST / 1024 / 8, NB = BST / 1024 / 8;     // pieces per wave and stage
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (skip && *skip) return;
    const int tm = (M + PF_BM - 1) / PF_BM, tn = (N + BN - 1) / BN;
    int bm, bn;
    pf_tile(blockIdx.x, gridDim.x, tm, tn, bm, bn);
    const int m0 = bm * PF_BM, n0 = bn * BN;
    const int nk = K / BKS;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ln = lane & 15, lg = lane >> 4;
    const int wr = w >> 2, wc = w & 3;

    // ---- loader addresses. Activation piece p = i * 8 + w covers tile rows RPP p .. RPP p + RPP - 1:
    // lane L lands at row RPP p + L / CPR, chunk slot L % CPR, which holds source chunk slot ^ swz(row)
    // (32-bit byte offsets from wave-uniform bases: the tile's first activation row and the packed
    // weights; the packed image of one projection is < 4 GB, the activation offsets < 256 rows)
    uint32_t aoff[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int p = i * 8 + w, row = RPP * p + lane / CPR;
        const int m = min(m0 + row, M - 1);            // rows >= M compute garbage that is never stored
        aoff[i] = (uint32_t)(((long)(m - m0) * lda + (((lane % CPR) ^ pf_swz<BKS>(row)) << 3)) * 2);
    }
    const bf16_t* const abase = A + (size_t)m0 * lda;
    // weight block b = i * 8 + w: 16-column group b / KSS, k-slice b % KSS of the stage
    uint32_t boff[NB];
    const int ntl = (N + 15) / 16;                      // packed 16-row tiles present (padded to 64 rows)
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int b = i * 8 + w, g = n0 / 16 + b / KSS;
        const int gg = g < ntl ? g : 0;                 // groups past N stream group 0 (never stored)
        boff[i] = (uint32_t)((((long)gg * (K >> 5) + (b % KSS)) * 512 + lane * 8) * 2);
    }
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem + w * 1024);
    auto issue = [&](int kt, int st) {
        if (ZK_PF_DIAG_NOFILL) return;
        const uint32_t sa = lds0 + st * ST, sb = sa + AST;
#pragma unroll
        for (int i = 0; i < NA; ++i) pf_glds_s(abase + kt * BKS, aoff[i], sa + i * 8192);
#pragma unroll
        for (int i = 0; i < NB; ++i) pf_glds_s(W + (size_t)kt * KSS * 512, boff[i], sb + i * 8192);
    };
    constexpr int LPS = NA + NB;                         // LDS-DMA loads per wave and stage
    // one piece j of the stage: activation pieces first, then weight pieces
    auto issue_piece = [&](int kt, int st, int j) {
        if (ZK_PF_DIAG_NOFILL) return;
        const uint32_t sa = lds0 + st * ST, sb = sa + AST;
        if (j < NA) pf_glds_s(abase + kt * BKS, aoff[j], sa + j * 8192);
        else pf_glds_s(W + (size_t)kt * KSS * 512, boff[j - NA], sb + (j - NA) * 8192);
    };
    // ZK_PF_SPREAD = P > 0: the refill's pieces are issued between the step's MFMAs, piece j right after
    // MFMA j * P of the step, instead of all at the top of the step (0)
    constexpr int QS = KSS * 8;                          // MFMA groups (ks, mt) per step
    constexpr int SP = ZK_PF_SPREAD;
    static_assert(SP == 0 || (LPS - 1) * SP < QS * NTN, "spread: every piece inside the step");

    f32x4 acc[8][NTN];
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int s0 = 0; s0 < NSTG - 1; ++s0)
        if (s0 < nk) issue(s0, s0);
    for (int kt = 0; kt < nk; ++kt) {
        // step kt's copies: everything issued after them may stay in flight (with the spread refill every
        // step issues one stage, clamped past the end, so that is NSTG - 2 stages once the ring is full)
        const int after = ZK_PF_SPREAD ? min(NSTG - 2, min(NSTG - 1, nk) - 1) : min(NSTG - 2, nk - 1 - kt);
        if constexpr (ZK_PF_DIAG_NOWAIT) {
        } else {
            pf_wait_after<LPS, NSTG - 2>(after);
        }
        // the barrier publishes every wave's copies of step kt and ends every read of the stage the
        // refill below overwrites (read in step kt - 1; this wave's reads retired here)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (!ZK_PF_SPREAD && kt + NSTG - 1 < nk) issue(kt + NSTG - 1, (kt + NSTG - 1) % NSTG);
        const char* sa = smem + (kt % NSTG) * ST;
        const char* sb = sa + AST;
        auto rd_a = [&](int q) -> uint4 {
            const int ks = q >> 3, mt = q & 7;
            return ZK_PF_DIAG_NOLDS ? make_uint4(mt, lane, ks, kt)
                                    : *reinterpret_cast<const uint4*>(sa + pf_a_off<BKS>(wr * 128 + mt * 16 + ln, ks * 4 + lg));
        };
        auto rd_b = [&](int ks, int nt) -> uint4 {
            return ZK_PF_DIAG_NOLDS ? make_uint4(lane, nt, ks, kt)
                                    : *reinterpret_cast<const uint4*>(sb + (((wc * NTN + nt) * KSS + ks) << 10) + lane * 16);
        };
        uint4 bf[2][NTN];
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt) bf[0][nt] = rd_b(0, nt);
        uint4 a = rd_a(0);
#pragma unroll
        for (int q = 0; q < QS; ++q) {
            const int ks = q >> 3, mt = q & 7;
            if (mt == 0 && ks > 0) {
#pragma unroll
                for (int nt = 0; nt < NTN; ++nt) bf[ks & 1][nt] = rd_b(ks, nt);
            }
#pragma unroll
            for (int nt = 0; nt < NTN; ++nt) {
                if constexpr (ZK_PF_DIAG_NOMFMA) {
                    acc[mt][nt][0] += __uint_as_float(a.x ^ bf[ks & 1][nt].y);
                } else {
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a), as_frag(bf[ks & 1][nt]), acc[mt][nt],
                                                                          0, 0, 0);
                }
                if constexpr (SP != 0) {
                    // no branch around the pieces (one basic block per step, so the LDS reads can be
                    // scheduled ahead of the MFMAs): past the last step the refill re-reads step nk - 1
                    // into the stage nothing reads any more (the epilogue drains vmcnt first)
                    const int f = q * NTN + nt;
                    if (f % SP == 0 && f / SP < LPS)
                        issue_piece(min(kt + NSTG - 1, nk - 1), (kt + NSTG - 1) % NSTG, f / SP);
                }
            }
            if (q + 1 < QS) a = rd_a(q + 1);
        }
    }

    if constexpr (ZK_PF_DIAG_NOEPI) {          // (diagnostic: no stores; one lane keeps the sums live)
        float t = 0.f;
#pragma unroll
        for (int mt = 0; mt < 8; ++mt)
#pragma unroll
            for (int nt = 0; nt < NTN; ++nt) t += acc[mt][nt][0] + acc[mt][nt][3];
        if (t == 1.2345f && C) C[0] = t;
        return;
    }
    if constexpr (ZK_PF_EPI && (MODE == 1 || NTN == 4)) {
        if (MODE == 1 || N % 4 == 0) {
            pf_epilogue_lds<MODE, NTN>(acc, smem, m0, n0, wr, wc, ln, lg, M, N, C, Cb);
            return;
        }
    }
    pf_epilogue<MODE, NTN>(acc, m0, n0, wr, wc, ln, lg, M, N, C, Cb);
}

}  // namespace

// The prefill regime of zk_gemm_bf16 (split 1, large M): true when the 256-row-tile kernel takes the call.
bool zk_gemm_pf_applies(int M, int N, int K, int nsplit) {
    if (nsplit != 1 || K % 64 != 0 || N % 64 != 0) return false;
    const long tiles = (long)((M + PF_BM - 1) / PF_BM) * ((N + 255) / 256);
    return tiles >= 256;                              // at least one tile per CU
}

// stage depth and ring length: 64-deep stages x 2 (default), or 32-deep x 4 (3 in flight; 128 KB either
// way): 32 x 4 measured 2-4 % slower at the c3 prefill shapes (profiles/r4_prefill_gemm_bks_ab.txt), so the
// kernel is not waiting on copy latency
#ifndef ZK_PF_BKS
#define ZK_PF_BKS 64
#endif
// 256 x 384 tiles for the SwiGLU (fc1) form when N >= 8192 (the partial last column tile wastes <= 1.6 %
// of its MFMAs there); 0: 256 x 256 everywhere
#ifndef ZK_PF_WIDE
#define ZK_PF_WIDE 0
#endif
#ifndef ZK_PF_NSTG
#define ZK_PF_NSTG (ZK_PF_BKS == 64 ? 2 : 4)
#endif
constexpr int PF_BKS = ZK_PF_BKS, PF_NSTG = ZK_PF_NSTG;
constexpr int pf_max(int a, int b) { return a > b ? a : b; }
template <int MODE, int NTN>
constexpr int pf_lds() {
    return pf_max(PF_NSTG * (PF_BM + pf_bn<NTN>) * PF_BKS * 2,
                  ZK_PF_EPI ? (MODE == 1 ? pf_epi_lds1<NTN> : pf_epi_lds0<NTN>) : 0);
}
static_assert((!ZK_PF_WIDE || pf_lds<1, 6>() <= 163840) && pf_lds<0, 4>() <= 163840 && pf_lds<1, 4>() <= 163840, "LDS");

template <int MODE, int NTN>
static int pf_launch(const void* A, long lda, const void* W, int M, int N, int K, float* C, void* Cb,
                      const int32_t* skip, hipStream_t stream) {
    const long tiles = (long)((M + PF_BM - 1) / PF_BM) * ((N + pf_bn<NTN> - 1) / pf_bn<NTN>);
    ZK_REQUIRE(tiles < (1L << 31), "zk_gemm_bf16 (prefill): too many tiles");
    // the LDS-DMA sources are 32-bit byte offsets: from the packed weights and from a tile's first row
    ZK_REQUIRE((long)((N + 63) / 64 * 64) * K * 2 < (1L << 32) && (long)PF_BM * lda * 2 < (1L << 31),
               "zk_gemm_bf16 (prefill): N=%d K=%d lda=%ld exceed the 32-bit source offsets", N, K, lda);
    auto kern = &k_gemm_pf<MODE, PF_BKS, PF_NSTG, NTN>;
    constexpr int lds = pf_lds<MODE, NTN>();
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(PF_NT), lds, stream, (const bf16_t*)A, lda, (const bf16_t*)W,
                       M, N, K, C, (bf16_t*)Cb, skip);
    return 0;
}

int zk_gemm_pf(const void* A, long lda, const void* W, int M, int N, int K, int mode, float* C, void* Cb,
               const int32_t* skip, void* stream) {
    // (a staggered four-phase form of the step -- two wave groups offset by one barrier, reads of one
    // overlapping the other's MFMAs -- measured 1-3 % slower: DESIGN.md §6 round 4)
    const hipStream_t st = (hipStream_t)stream;
    int rc;
#if ZK_PF_WIDE
    if (mode == 1 && N >= 8192) rc = pf_launch<1, 6>(A, lda, W, M, N, K, C, Cb, skip, st);
    else
#endif
    if (mode == 0) rc = pf_launch<0, 4>(A, lda, W, M, N, K, C, Cb, skip, st);
    else rc = pf_launch<1, 4>(A, lda, W, M, N, K, C, Cb, skip, st);
    if (rc) return rc;
    ZK_CHECK_LAUNCH("zk_gemm_bf16 (prefill)");
    return 0;
}
