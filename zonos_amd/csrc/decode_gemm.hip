// Decode-step GEMM for 16 < M <= 128 rows (B = 9..64 utterances x 2 CFG rows) on gfx950:
// C[M][N] = A[M][K] . W[N][K]^T, bf16 operands, fp32 accumulation on MFMA 16x16x32.
//
// Why a second decode GEMM (gemm.hip's k_gemm_ws is the LDS form): at M = 128 every weight byte
// meets 128 activation rows, so a column tile of BN columns takes in M/BN activation bytes per
// weight byte from L2 -- more than the weights themselves. k_gemm_ws stages those activation
// chunks in LDS and publishes them with one workgroup barrier per 64-deep K chunk, which locks the
// 4 compute waves together: the slowest wave's weight load sets every chunk's pace, and the MFMA
// phase is not hidden under the weight stream.
//
// Here the activation is handed over in the MFMA A-operand order ("apack", below: the producer
// kernels -- k_resid_ln, the decode attention, the fc1 epilogue -- write it that way), so each
// 16 x 32 A fragment is ONE contiguous 1 KB block that a wave loads straight into registers with
// a fully coalesced 16-B-per-lane load. The workgroup's NW waves split the K range (wave w owns
// k-steps [w*KS, (w+1)*KS) of the workgroup's slice) and each streams ALL NC*16 columns of the
// tile: every activation byte is loaded by exactly one wave, every weight byte by exactly one
// wave, and no wave ever waits for another until the end -- no LDS and no barrier in the main
// loop. Per k-step a wave has NC weight fragments (HBM, non-temporal) and MT activation fragments
// (L2) in flight for PF k-steps ahead, fully unrolled so hipcc's waitcnt counts are exact.
// The NW partial tiles are summed through LDS in a fixed order (w = 0, 1, ..., NW-1), so results
// depend on (N, K, nsplit, NW) only, not on M: batch-invariant within this kernel.
//
// apack layout of an M x K activation (MT = ceil(M/16) row tiles, K % 32 == 0): element (m, k) at
//   ((k/32 * MT + m/16) * 64 + (m%16) + 16 * ((k%32)/8)) * 8 + k%8
// i.e. [k-step][row tile][lane][8] -- lane l of the 16x16x32 A fragment holds row (l%16) and
// k-offsets 8*(l/16) .. +7 (cdna_hip_programming.md §3 fragment layout).
//
// mode 0: fp32 split-K slabs Cpart[split][M][N] (consumer reduces them in a fixed order);
// mode 1: FeedForward fc1 + SwiGLU (_torch.py:147,151-152; W rows in zk_permute_fc1 order): the
//         bf16 h = y * silu(gate) written in apack order for fc2 (K = N/2).
#include "common.h"
#include "../../include/zonos_hip.h"
#include <algorithm>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

ZK_DEV bf16x8 frag(uint4 v) { return __builtin_bit_cast(bf16x8, v); }
ZK_DEV uint4 ldg_nt(const bf16_t* p) {
    return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)));
}
ZK_DEV uint4 ldg(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }

// offset (elements) of element (m, k) in the apack layout
ZK_DEV size_t apack_off(int m, int k, int MT) {
    return ((size_t)((k >> 5) * MT + (m >> 4)) * 64 + (m & 15) + 16 * ((k & 31) >> 3)) * 8 + (k & 7);
}

// DBG (diagnostic instantiations of the sweep tool only): 1 = no activation loads, 2 = no weight loads
template <int MODE, int MT, int NC, int NW, int KS, int PF, int DBG = 0>
__global__ __launch_bounds__(64 * NW, 1) void k_gemm_ks(const bf16_t* __restrict__ Ap, const bf16_t* __restrict__ W,
                                                        int M, int N, int K, int kslice, float* __restrict__ Cpart,
                                                        bf16_t* __restrict__ Cout, const int32_t* skip, int rot) {
    constexpr int ROWS = MT * 16, COLS = NC * 16;
    constexpr int RS = COLS + 4;                       // LDS row stride (floats) of a partial tile
    extern __shared__ __attribute__((aligned(16))) float red[];   // [min(NW, 4)][ROWS][RS]
    if (skip && *skip) return;
    int bx = blockIdx.x, bz = blockIdx.z;
    // XCD-aware order (as k_gemm_ws): the workgroups of one K split on one XCD, so its L2 holds
    // only that split's activation slice. Placement only.
    if (gridDim.z > 1 && ((gridDim.x * gridDim.z) & 7) == 0) {
        const int L = blockIdx.x + gridDim.x * blockIdx.z;
        const int I = (L & 7) * ((gridDim.x * gridDim.z) >> 3) + (L >> 3);
        bz = I / gridDim.x;
        bx = I - bz * gridDim.x;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ln = lane & 15, lg = lane >> 4;
    const int n0 = bx * COLS, split = bz;
    // rot 1: the waves' K ranges rotate with the tile (wave w takes range (w + bx) % NW; the partial
    // tiles are summed in range order, so the result is the same); rot 2: also each wave starts its
    // range at k-step bx % KS (changes the accumulation order per tile). Both spread the 256
    // workgroups' reads of the shared activation over the L2 instead of marching in lockstep.
    const int wr_ = rot ? (w + bx) % NW : w;
    const int r0 = rot == 2 ? bx % KS : 0;
    const int ks0 = (split * kslice >> 5) + wr_ * KS;  // first k-step of this wave's range
    const int KT = K >> 5;
    const bf16_t* wp[NC];
#pragma unroll
    for (int t = 0; t < NC; ++t) wp[t] = W + ((size_t)(n0 / 16 + t) * KT + ks0) * 512 + lane * 8;
    const bf16_t* ap = Ap + (size_t)ks0 * MT * 512 + lane * 8;

    f32x4 acc[MT][NC];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int t = 0; t < NC; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int U = PF + 1;
    uint4 wr[U][NC], ar[U][MT];
    auto issue = [&](int s, int slot) {
        const int sa = (s + r0) & (KS - 1);
#pragma unroll
        for (int t = 0; t < NC; ++t) wr[slot][t] = (DBG & 2) ? make_uint4(sa, t, lane, 0) : ldg_nt(wp[t] + sa * 512);
#pragma unroll
        for (int m = 0; m < MT; ++m) ar[slot][m] = (DBG & 1) ? make_uint4(sa, m, lane, 1) : ldg(ap + ((size_t)sa * MT + m) * 512);
    };
#pragma unroll
    for (int p = 0; p < PF; ++p)
        if (p < KS) issue(p, p);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        if (s + PF < KS) issue(s + PF, (s + PF) % U);
        __builtin_amdgcn_sched_barrier(0);             // loads of step s+PF ahead of step s's MFMAs
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int t = 0; t < NC; ++t)
                acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag(ar[s % U][m]), frag(wr[s % U][t]), acc[m][t],
                                                                    0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    // ---- partial tiles -> LDS: acc[m][t][i] = C[16m + 4lg + i][16t + ln]. At most 4 tiles are
    // held at once: with NW = 8 waves w >= 4 hand theirs to wave w - 4 first, so the fixed summation
    // order is (w0 + w4) + (w1 + w5) + (w2 + w6) + (w3 + w7).
    constexpr int NWL = NW > 4 ? 4 : NW;
    float* mine = red + (size_t)(wr_ % NWL) * ROWS * RS;
    auto tile_io = [&](bool store) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int t = 0; t < NC; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float* p = mine + (m * 16 + lg * 4 + i) * RS + t * 16 + ln;
                    if (store) *p = acc[m][t][i];
                    else acc[m][t][i] = acc[m][t][i] + *p;
                }
    };
    if constexpr (NW > 4) {
        if (wr_ >= 4) tile_io(true);
        __syncthreads();
        if (wr_ < 4) tile_io(false);
        __syncthreads();
    }
    if (wr_ < NWL) tile_io(true);
    __syncthreads();
    constexpr int NTH = 64 * NW;
    if constexpr (MODE == 0) {
        // fixed-order sum over the waves; whole-row float4 stores (COLS/4 per row)
        constexpr int C4 = COLS / 4;
        float* C = Cpart + (size_t)split * M * N;
        for (int q = threadIdx.x; q < ROWS * C4; q += NTH) {
            const int r = q / C4, c = (q % C4) * 4;
            if (r >= M) break;
            f32x4 s = *reinterpret_cast<const f32x4*>(red + r * RS + c);
#pragma unroll
            for (int v = 1; v < NWL; ++v) {
                const f32x4 o = *reinterpret_cast<const f32x4*>(red + ((size_t)v * ROWS + r) * RS + c);
#pragma unroll
                for (int e = 0; e < 4; ++e) s[e] = s[e] + o[e];
            }
            const int n = n0 + c;
            if (n + 3 < N) {
                __builtin_nontemporal_store(s, reinterpret_cast<f32x4*>(C + (size_t)r * N + n));
            } else {
                for (int e = 0; e < 4 && n + e < N; ++e) C[(size_t)r * N + n + e] = s[e];
            }
        }
    } else {
        // SwiGLU: tile column 16t + j (j < 8) = y[f0 + 8t + j], 16t + 8 + j = gate[...]; the 8*NC h
        // columns of this tile go to apack positions of the (N/2)-deep fc2 activation: lane l of
        // row tile mt holds row 16mt + l%16, h columns 8*(l/16) .. +7 of k-step (f0 + 8t) / 32.
        const int F = N / 2, f0 = n0 / 2;
        for (int q = threadIdx.x; q < MT * 16 * NC; q += NTH) {
            const int t = q / ROWS, r = q % ROWS;          // one 8-column h group of one row
            if (r >= M) continue;
            float y[8], g[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) { y[j] = 0.f; g[j] = 0.f; }
#pragma unroll
            for (int v = 0; v < NWL; ++v) {
                const float* row = red + ((size_t)v * ROWS + r) * RS + t * 16;
#pragma unroll
                for (int j = 0; j < 8; ++j) { y[j] = y[j] + row[j]; g[j] = g[j] + row[8 + j]; }
            }
            float h[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float yb = round_bf(y[j]), gb = round_bf(g[j]);      // fc1 output in bf16
                const float sl = round_bf(gb / (1.0f + expf(-gb)));        // F.silu in bf16
                h[j] = yb * sl;
            }
            const int f = f0 + 8 * t;                                      // first h column (multiple of 8)
            if (f < F) *reinterpret_cast<uint4*>(Cout + apack_off(r, f, MT)) = pack8(h);
        }
    }
}

__global__ void k_pack_act(const bf16_t* __restrict__ A, long lda, int M, int K, int MT, bf16_t* __restrict__ Ap) {
    // one thread per 8-element group (m, k8); rows >= M are written as zeros
    const long n = (long)MT * 16 * (K / 8);
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int m = (int)(i / (K / 8)), k = (int)(i % (K / 8)) * 8;
        const uint4 v = m < M ? *reinterpret_cast<const uint4*>(A + (size_t)m * lda + k) : make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(Ap + apack_off(m, k, MT)) = v;
    }
}

__global__ void k_unpack_act(const bf16_t* __restrict__ Ap, int M, int K, int MT, bf16_t* __restrict__ A, long lda) {
    const long n = (long)M * (K / 8);
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int m = (int)(i / (K / 8)), k = (int)(i % (K / 8)) * 8;
        *reinterpret_cast<uint4*>(A + (size_t)m * lda + k) = *reinterpret_cast<const uint4*>(Ap + apack_off(m, k, MT));
    }
}

template <int MODE, int MT, int NC, int NW, int KS, int PF, int DBG = 0>
int launch_ks(const bf16_t* Ap, const bf16_t* W, int M, int N, int K, int nsplit, float* Cpart, bf16_t* Cout,
              const int32_t* skip, int rot, hipStream_t st) {
    const int tiles = (N + NC * 16 - 1) / (NC * 16);
    const size_t lds = (size_t)(NW > 4 ? 4 : NW) * MT * 16 * (NC * 16 + 4) * sizeof(float);
    auto kern = &k_gemm_ks<MODE, MT, NC, NW, KS, PF, DBG>;
    if (lds > 65536) hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)lds);
    hipLaunchKernelGGL(kern, dim3(tiles, 1, nsplit), dim3(64 * NW), lds, st, Ap, W, M, N, K, K / nsplit, Cpart, Cout,
                       skip, rot);
    return 0;
}

}  // namespace

// Tile configuration of the c3 decode shapes (K per wave = KS k-steps of 32):
//   in_proj  N 3072, K 2048: 64 columns, split 4, 4 waves x 4 k-steps  -> 192 workgroups
//   out_proj N 2048, K 2048: 64 columns, split 8, 4 waves x 2 k-steps  -> 256 workgroups
//   fc1      N 16384, K 2048: 64 columns, split 1, 4 waves x 16 k-steps -> 256 workgroups
//   fc2      N 2048, K 8192: 64 columns, split 8, 4 waves x 8 k-steps  -> 256 workgroups
//   heads    N 9234, K 2048: 64 columns, split 1, 4 waves x 16 k-steps -> 145 workgroups
// `cfg` selects (NC, NW, PF) for the sweep tool: 0 = default (NC 4, NW 4, PF 3), 1 = (4, 8, 1),
// 2 = (2, 4, 4), 3 = (4, 4, 2), 7 = (4, 4, 4); 4 / 5 / 6 = 3 without activation / weight / any
// loads (diagnostics, wrong results); + 16 * rot (k_gemm_ks `rot`).
extern "C" int zk_gemm_apack(const void* Ap, const void* W, int M, int N, int K, int nsplit, int mode, float* Cpart,
                             void* Cout, const int32_t* skip, int cfg, void* stream) {
    ZK_REQUIRE(M > 0 && M <= 128 && N > 0 && K > 0 && nsplit >= 1 && K % (32 * nsplit) == 0,
               "zk_gemm_apack: M=%d N=%d K=%d nsplit=%d", M, N, K, nsplit);
    ZK_REQUIRE(mode == 0 || mode == 1, "zk_gemm_apack: mode %d", mode);
    ZK_REQUIRE(mode == 0 ? Cpart != nullptr : (Cout != nullptr && nsplit == 1 && N % 64 == 0),
               "zk_gemm_apack: mode %d needs %s", mode, mode == 0 ? "Cpart" : "Cout, nsplit 1, N % 64 == 0");
    const int MT = (M + 15) / 16;
    const int steps = K / nsplit / 32;      // k-steps per workgroup
    const int rot = cfg >> 4;               // cfg bits 4-5: K-order rotation (k_gemm_ks `rot`)
    cfg &= 15;
    hipStream_t st = (hipStream_t)stream;
    const auto* A = (const bf16_t*)Ap;
    const auto* Wp = (const bf16_t*)W;
    auto* Cb = (bf16_t*)Cout;
    int rc = -1;
#define ZK_KS_MT(MODE_, NC_, NW_, KS_, PF_)                                                                         \
    switch (MT) {                                                                                                   \
        case 8: rc = cfg == 4 ? launch_ks<MODE_, 8, NC_, NW_, KS_, PF_, 1>(A, Wp, M, N, K, nsplit, Cpart, Cb, skip, rot, st) \
                   : cfg == 5 ? launch_ks<MODE_, 8, NC_, NW_, KS_, PF_, 2>(A, Wp, M, N, K, nsplit, Cpart, Cb, skip, rot, st) \
                   : cfg == 6 ? launch_ks<MODE_, 8, NC_, NW_, KS_, PF_, 3>(A, Wp, M, N, K, nsplit, Cpart, Cb, skip, rot, st) \
                   : launch_ks<MODE_, 8, NC_, NW_, KS_, PF_>(A, Wp, M, N, K, nsplit, Cpart, Cb, skip, rot, st); break;    \
        case 4: rc = launch_ks<MODE_, 4, NC_, NW_, KS_, PF_>(A, Wp, M, N, K, nsplit, Cpart, Cb, skip, rot, st); break;    \
        case 2: rc = launch_ks<MODE_, 2, NC_, NW_, KS_, PF_>(A, Wp, M, N, K, nsplit, Cpart, Cb, skip, rot, st); break;    \
        default: break;                                                                                             \
    }
#define ZK_KS_STEPS(MODE_, NC_, NW_, PF_)                                                                           \
    switch (steps / NW_) {                                                                                          \
        case 1: if (steps == NW_) { ZK_KS_MT(MODE_, NC_, NW_, 1, PF_) } break;                                      \
        case 2: if (steps == 2 * NW_) { ZK_KS_MT(MODE_, NC_, NW_, 2, PF_) } break;                                  \
        case 4: if (steps == 4 * NW_) { ZK_KS_MT(MODE_, NC_, NW_, 4, PF_) } break;                                  \
        case 8: if (steps == 8 * NW_) { ZK_KS_MT(MODE_, NC_, NW_, 8, PF_) } break;                                  \
        case 16: if (steps == 16 * NW_) { ZK_KS_MT(MODE_, NC_, NW_, 16, PF_) } break;                               \
        default: break;                                                                                             \
    }
#define ZK_KS_CFG(MODE_)                                                \
    switch (cfg) {                                                      \
        case 1: ZK_KS_STEPS(MODE_, 4, 8, 1) break;                      \
        case 2: ZK_KS_STEPS(MODE_, 2, 4, 4) break;                      \
        case 3: ZK_KS_STEPS(MODE_, 4, 4, 2) break;                      \
        case 4: case 5: case 6: ZK_KS_STEPS(MODE_, 4, 4, 2) break;      \
        case 7: ZK_KS_STEPS(MODE_, 4, 4, 4) break;                      \
        default: ZK_KS_STEPS(MODE_, 4, 4, 3) break;                     \
    }
    if (mode == 0) { ZK_KS_CFG(0) } else { ZK_KS_CFG(1) }
#undef ZK_KS_CFG
#undef ZK_KS_STEPS
#undef ZK_KS_MT
    ZK_REQUIRE(rc == 0, "zk_gemm_apack: no instantiation for M=%d (MT %d) K/nsplit=%d cfg %d", M, MT, K / nsplit, cfg);
    ZK_CHECK_LAUNCH("zk_gemm_apack");
    return 0;
}

extern "C" int zk_pack_act(const void* A, long lda, int M, int K, void* Ap, void* stream) {
    ZK_REQUIRE(M > 0 && M <= 128 && K % 32 == 0 && lda >= K && lda % 8 == 0, "zk_pack_act: M=%d K=%d", M, K);
    const int MT = (M + 15) / 16;
    const long n = (long)MT * 16 * (K / 8);
    hipLaunchKernelGGL(k_pack_act, dim3((unsigned)std::min<long>((n + 255) / 256, 4096)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)A, lda, M, K, MT, (bf16_t*)Ap);
    ZK_CHECK_LAUNCH("zk_pack_act");
    return 0;
}

extern "C" int zk_unpack_act(const void* Ap, int M, int K, void* A, long lda, void* stream) {
    ZK_REQUIRE(M > 0 && M <= 128 && K % 32 == 0 && lda >= K && lda % 8 == 0, "zk_unpack_act: M=%d K=%d", M, K);
    const int MT = (M + 15) / 16;
    const long n = (long)M * (K / 8);
    hipLaunchKernelGGL(k_unpack_act, dim3((unsigned)std::min<long>((n + 255) / 256, 4096)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)Ap, M, K, MT, (bf16_t*)A, lda);
    ZK_CHECK_LAUNCH("zk_unpack_act");
    return 0;
}
