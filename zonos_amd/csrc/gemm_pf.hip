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
// The next step's stage is issued right after the barrier that retires the stage it overwrites,
// so a whole step of MFMAs (64 per wave) covers its latency. Tiles are handed to the 8 XCDs in
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

constexpr int PF_BM = 256, PF_BN = 256, PF_BK = 64, PF_NT = 512;
constexpr int PF_AST = PF_BM * PF_BK * 2;          // activation stage bytes (32 KB)
constexpr int PF_BST = PF_BN * PF_BK * 2;          // weight stage bytes (32 KB)
constexpr int PF_ST = PF_AST + PF_BST;             // one stage
constexpr int PF_LDS = 2 * PF_ST;                  // two stages: 128 KB

ZK_DEV int pf_lds_off(int row, int c) { return row * 128 + ((c ^ (row & 7)) << 4); }

template <int N_>
ZK_DEV void pf_vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory"); }

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

template <int MODE>
__global__ __launch_bounds__(PF_NT, 1) void k_gemm_pf(const bf16_t* __restrict__ A, long lda,
                                                      const bf16_t* __restrict__ W, int M, int N, int K,
                                                      float* __restrict__ C, bf16_t* __restrict__ Cb,
                                                      const int32_t* skip) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (skip && *skip) return;
    const int tm = (M + PF_BM - 1) / PF_BM, tn = (N + PF_BN - 1) / PF_BN;
    int bm, bn;
    pf_tile(blockIdx.x, gridDim.x, tm, tn, bm, bn);
    const int m0 = bm * PF_BM, n0 = bn * PF_BN;
    const int nk = K / PF_BK;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ln = lane & 15, lg = lane >> 4;
    const int wr = w >> 2, wc = w & 3;

    // ---- loader addresses: 4 activation pieces + 4 weight blocks of 1 KB per thread and step
    // activation piece p = i * 8 + w covers tile rows 8p..8p+7: lane L -> row 8p + L/8, LDS slot L%8
    // holding source chunk (L%8) ^ (row%8) (pf_lds_off's swizzle applied on the source address)
    const bf16_t* asrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int p = i * 8 + w, row = 8 * p + (lane >> 3);
        const int m = min(m0 + row, M - 1);            // rows >= M compute garbage that is never stored
        asrc[i] = A + (size_t)m * lda + (((lane & 7) ^ (row & 7)) << 3);
    }
    // weight block b = i * 8 + w: 16-column group g = b / 2, k-slice b % 2 of the step
    const bf16_t* bsrc[4];
    const int ntl = (N + 15) / 16;                      // packed 16-row tiles present (padded to 64 rows)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int b = i * 8 + w, g = n0 / 16 + (b >> 1);
        const int gg = g < ntl ? g : 0;                 // groups past N stream group 0 (never stored)
        bsrc[i] = W + ((size_t)gg * (K >> 5) + (b & 1)) * 512 + lane * 8;
    }
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem + w * 1024);
    auto issue = [&](int kt, int st) {
        const uint32_t sa = lds0 + st * PF_ST, sb = sa + PF_AST;
#pragma unroll
        for (int i = 0; i < 4; ++i) pf_glds(asrc[i] + kt * PF_BK, sa + i * 8192);
#pragma unroll
        for (int i = 0; i < 4; ++i) pf_glds(bsrc[i] + (size_t)kt * 1024, sb + i * 8192);
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

    issue(0, 0);
    pf_vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int kt = 0; kt < nk; ++kt) {
        // the other stage was last read in step kt - 1, which every wave finished before the
        // barrier that ended it
        if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);
        const char* sa = smem + (kt & 1) * PF_ST;
        const char* sb = sa + PF_AST;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            uint4 bf[4];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
                bf[nt] = *reinterpret_cast<const uint4*>(sb + (((wc * 4 + nt) * 2 + ks) << 10) + lane * 16);
#pragma unroll
            for (int mt = 0; mt < 8; ++mt) {
                const uint4 a = *reinterpret_cast<const uint4*>(sa + pf_lds_off(wr * 128 + mt * 16 + ln, ks * 4 + lg));
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a), as_frag(bf[nt]), acc[mt][nt], 0,
                                                                          0, 0);
            }
        }
        // this wave's copies of step kt + 1 have landed and its reads of stage kt & 1 retired; the
        // barrier publishes everyone's copies and ends every read of the stage the next step refills
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pf_vm_wait<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }

    // ---- epilogue: acc[mt][nt][i] = C[m0 + wr*128 + mt*16 + lg*4 + i][n0 + wc*64 + nt*16 + ln]
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int c0 = n0 + wc * 64 + nt * 16;
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

}  // namespace

// The prefill regime of zk_gemm_bf16 (split 1, large M): true when the 256 x 256 kernel takes the call.
bool zk_gemm_pf_applies(int M, int N, int K, int nsplit) {
    if (nsplit != 1 || K % PF_BK != 0 || N % 64 != 0) return false;
    const long tiles = (long)((M + PF_BM - 1) / PF_BM) * ((N + PF_BN - 1) / PF_BN);
    return tiles >= 256;                              // at least one tile per CU
}

int zk_gemm_pf(const void* A, long lda, const void* W, int M, int N, int K, int mode, float* C, void* Cb,
               const int32_t* skip, void* stream) {
    const long tiles = (long)((M + PF_BM - 1) / PF_BM) * ((N + PF_BN - 1) / PF_BN);
    ZK_REQUIRE(tiles < (1L << 31), "zk_gemm_bf16 (prefill): too many tiles");
    auto kern = mode == 0 ? &k_gemm_pf<0> : &k_gemm_pf<1>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, PF_LDS);
    hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(PF_NT), PF_LDS, (hipStream_t)stream, (const bf16_t*)A, lda,
                       (const bf16_t*)W, M, N, K, C, (bf16_t*)Cb, skip);
    ZK_CHECK_LAUNCH("zk_gemm_bf16 (prefill)");
    return 0;
}
