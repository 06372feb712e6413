// DAC decoder convolutions on fp16 MFMA (16x16x32) for gfx950, with optional split
// precision ("fp16x3"): every fp32 operand x is carried as hi = fp16(x), lo = fp16(x - hi)
// and the product is hi*hi + lo*hi + hi*lo accumulated in fp32 -- ~22 mantissa bits, i.e.
// within a few ulp of the reference's fp32 CPU convs, at 3/16 of the fp32-MFMA cost.
// NPASS = 1 is plain fp16 operands with fp32 accumulation, the numerics of the reference's
// own GPU path (torch.autocast fp16, zonos/autoencoder.py:46).
//
// Implicit GEMM: M = output channels (co), N = output positions (q), K = (input channel,
// tap). A workgroup owns CO_T = 32*MT output channels x 128 positions; 4 waves split the
// positions (32 each), each wave holds MT x 2 accumulator tiles. Per 32-channel K chunk
// the input window (128 + (ks-1)*dil positions) is staged time-major in LDS with the Snake
// activation and the hi/lo split applied once per element; the chunk's weights for all
// taps are staged [tap][co][ci]. Both images use a 4-row XOR swizzle of the 16-byte
// channel groups so that a 16-lane ds_read_b128 group touches 16 distinct bank slots.
//
// Weights are prepacked once (k_prep_w16): conv [Cout][Cin][ks] -> [ks][Cout][Cin] hi/lo,
// ConvTranspose1d [Cin][Cout][2s] -> s phases x [2 taps][Cout][Cin] (polyphase, see dac.hip).
#include "common.h"
#include "../../include/zonos_hip.h"
#include <algorithm>

namespace {

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int QT = 128;        // output positions per workgroup
constexpr int CIC = 32;        // input channels per K chunk (one MFMA k-step)
constexpr int KSM = 7;         // max taps
constexpr int WINM = QT + 6 * 9;   // max input window (k7, dilation 9)

ZK_DEV f16x8 as_h8(uint4 v) { return __builtin_bit_cast(f16x8, v); }

ZK_DEV float snake_f(float x, float a) {
    const float s = sinf(__fmul_rn(a, x));
    const float r = __fdiv_rn(1.0f, __fadd_rn(a, 1e-9f));
    return __fadd_rn(x, __fmul_rn(r, __fmul_rn(s, s)));
}

// 16-byte group g (0..3) of row `row` of a [rows][32 fp16] image: XOR swizzle table {0,2,3,1}
ZK_DEV int swz(int row, int g) {
    const int t = (row >> 2) & 3;
    const int f = (t == 0) ? 0 : (t == 1 ? 2 : (t == 2 ? 3 : 1));
    return row * 64 + ((g ^ f) << 4);
}

ZK_DEV void split8(const float* v, uint4& hi, uint4& lo) {
    _Float16 h[8], l[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        h[i] = (_Float16)v[i];
        l[i] = (_Float16)(v[i] - (float)h[i]);
    }
    hi = __builtin_bit_cast(uint4, *reinterpret_cast<f16x8*>(h));
    lo = __builtin_bit_cast(uint4, *reinterpret_cast<f16x8*>(l));
}

template <int NPASS, int MT>
__global__ __launch_bounds__(256, 2) void k_conv16(const float* __restrict__ in, int Cin, int Tin,
                                                   const float* __restrict__ alpha, const uint16_t* __restrict__ whi,
                                                   const uint16_t* __restrict__ wlo, const float* __restrict__ bias,
                                                   int Cout, int ks, int dil, int pad, int Qn, int out_stride,
                                                   int out_off, float* __restrict__ out, int Tout,
                                                   const float* __restrict__ resid, int do_tanh,
                                                   const int32_t* __restrict__ lens, int in_scale, int out_scale) {
    constexpr int CO_T = 32 * MT;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* xs_hi = smem;
    char* xs_lo = smem + WINM * 64;
    char* ws_hi = smem + (NPASS == 3 ? 2 : 1) * WINM * 64;
    char* ws_lo = ws_hi + KSM * CO_T * 64;

    const int q0 = blockIdx.x * QT, co0 = blockIdx.y * CO_T, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ln = lane & 15, lg = lane >> 4;
    const int len_in = lens ? lens[b] * in_scale : Tin;
    const int len_out = lens ? lens[b] * out_scale : Tout;
    const int win = QT + (ks - 1) * dil;
    const int u0 = q0 - pad;
    const float* inb = in + (size_t)b * Cin * Tin;
    const size_t wstride = (size_t)Cout * Cin;    // per tap

    f32x4 acc[MT * 2][2];
#pragma unroll
    for (int m = 0; m < 2 * MT; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int ci0 = 0; ci0 < Cin; ci0 += CIC) {
        __syncthreads();
        // ---- input window: (position j, 8-channel group g) items
        for (int it = tid; it < win * 4; it += 256) {
            const int j = it % win, g = it / win;
            const int u = u0 + j;
            float v[8];
            const bool ok = (u >= 0) && (u < len_in) && (u < Tin);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int c = ci0 + g * 8 + e;
                float x = ok ? inb[(size_t)c * Tin + u] : 0.f;
                if (alpha != nullptr && ok) x = snake_f(x, alpha[c]);
                v[e] = x;
            }
            uint4 hi, lo;
            split8(v, hi, lo);
            *reinterpret_cast<uint4*>(xs_hi + swz(j, g)) = hi;
            if (NPASS == 3) *reinterpret_cast<uint4*>(xs_lo + swz(j, g)) = lo;
        }
        // ---- weights: rows (tap, co) x 4 groups of 8 channels
        for (int it = tid; it < ks * CO_T * 4; it += 256) {
            const int g = it & 3, row = it >> 2;        // row = tap*CO_T + r
            const int tap = row / CO_T, r = row % CO_T;
            const int co = min(co0 + r, Cout - 1);
            const size_t off = tap * wstride + (size_t)co * Cin + ci0 + g * 8;
            *reinterpret_cast<uint4*>(ws_hi + swz(row, g)) = *reinterpret_cast<const uint4*>(whi + off);
            if (NPASS == 3) *reinterpret_cast<uint4*>(ws_lo + swz(row, g)) = *reinterpret_cast<const uint4*>(wlo + off);
        }
        __syncthreads();
        for (int tap = 0; tap < ks; ++tap) {
            uint4 ah[2 * MT], al[2 * MT], bh[2], bl[2];
#pragma unroll
            for (int m = 0; m < 2 * MT; ++m) {
                const int row = tap * CO_T + m * 16 + ln;
                ah[m] = *reinterpret_cast<const uint4*>(ws_hi + swz(row, lg));
                if (NPASS == 3) al[m] = *reinterpret_cast<const uint4*>(ws_lo + swz(row, lg));
            }
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                const int j = wv * 32 + n * 16 + ln + tap * dil;
                bh[n] = *reinterpret_cast<const uint4*>(xs_hi + swz(j, lg));
                if (NPASS == 3) bl[n] = *reinterpret_cast<const uint4*>(xs_lo + swz(j, lg));
            }
#pragma unroll
            for (int m = 0; m < 2 * MT; ++m)
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                    acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(ah[m]), as_h8(bh[n]), acc[m][n], 0, 0, 0);
                    if (NPASS == 3) {
                        acc[m][n] =
                            __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(al[m]), as_h8(bh[n]), acc[m][n], 0, 0, 0);
                        acc[m][n] =
                            __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(ah[m]), as_h8(bl[n]), acc[m][n], 0, 0, 0);
                    }
                }
        }
    }
    // acc[m][n][i] = C[co = co0 + 16m + 4lg + i][q = q0 + 32wv + 16n + ln]
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int q = q0 + wv * 32 + n * 16 + ln;
        if (q >= Qn) continue;
        const int t = q * out_stride + out_off;
        if (t < 0 || t >= Tout) continue;
#pragma unroll
        for (int m = 0; m < 2 * MT; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int co = co0 + m * 16 + lg * 4 + i;
                if (co >= Cout) continue;
                const size_t o = ((size_t)b * Cout + co) * Tout + t;
                float v = 0.f;
                if (t < len_out) {
                    v = __fadd_rn(acc[m][n][i], bias[co]);
                    if (resid) v = __fadd_rn(resid[o], v);
                    if (do_tanh) v = tanhf(v);
                }
                out[o] = v;
            }
    }
}

// conv weight [Cout][Cin][ks] (mode 0) or ConvTranspose1d [Cin][Cout][2s] (mode 1, s phases)
// -> fp16 hi/lo in [phase][tap][Cout][Cin]
__global__ void k_prep_w16(const float* w, int Cout, int Cin, int ks, int s, int mode, uint16_t* hi,
                           uint16_t* lo) {
    const int taps = mode == 0 ? ks : 2;
    const int phases = mode == 0 ? 1 : s;
    const size_t n = (size_t)phases * taps * Cout * Cin;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int ci = (int)(i % Cin);
        const int co = (int)((i / Cin) % Cout);
        const int tap = (int)((i / ((size_t)Cin * Cout)) % taps);
        const int r = (int)(i / ((size_t)Cin * Cout * taps));
        float v;
        if (mode == 0) v = w[((size_t)co * Cin + ci) * ks + tap];
        else v = w[((size_t)ci * Cout + co) * (2 * s) + (tap == 0 ? r + s : r)];   // tap0 reads in[q-1]
        const _Float16 h = (_Float16)v;
        const _Float16 l = (_Float16)(v - (float)h);
        hi[i] = __builtin_bit_cast(uint16_t, h);
        if (lo) lo[i] = __builtin_bit_cast(uint16_t, l);
    }
}

// Final Snake -> Conv1d(C -> 1, k7, p3) -> tanh (modeling_dac.py:437-439), VALU: the output has
// one channel, so an MFMA tile would be 1/16 used. Window staged in LDS with Snake applied.
constexpr int TAIL_T = 256;
__global__ __launch_bounds__(256) void k_dac_tail(const float* __restrict__ in, int C, int T,
                                                  const float* __restrict__ alpha, const float* __restrict__ w,
                                                  const float* __restrict__ bias, float* __restrict__ out,
                                                  const int32_t* __restrict__ lens, int scale) {
    extern __shared__ float xs[];     // [C][TAIL_T + 6]
    const int t0 = blockIdx.x * TAIL_T, b = blockIdx.y;
    const int len = lens ? lens[b] * scale : T;
    const int W = TAIL_T + 6;
    for (int i = threadIdx.x; i < C * W; i += 256) {
        const int c = i / W, j = i % W;
        const int u = t0 - 3 + j;
        float x = 0.f;
        if (u >= 0 && u < len && u < T) x = snake_f(in[((size_t)b * C + c) * T + u], alpha[c]);
        xs[c * W + j] = x;
    }
    __syncthreads();
    const int t = t0 + threadIdx.x;
    if (t >= T) return;
    float acc = 0.f;
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int k = 0; k < 7; ++k) acc = fmaf(w[c * 7 + k], xs[c * W + threadIdx.x + k], acc);
    out[(size_t)b * T + t] = (t < len) ? tanhf(__fadd_rn(acc, bias[0])) : 0.f;
}

// Raise the dynamic-LDS cap of a kernel (needed above 64 KiB); cheap, idempotent.
void ensure_lds(const void* fn, size_t bytes) {
    if (bytes > 65536) hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace

extern "C" int zk_dac_prep_w16(const float* w, int Cout, int Cin, int ks, int s, int mode, uint16_t* hi, uint16_t* lo,
                               void* stream) {
    ZK_REQUIRE(Cout > 0 && Cin > 0 && (mode == 0 ? (ks >= 1 && ks <= KSM) : s >= 1), "zk_dac_prep_w16: bad shape");
    const size_t n = (size_t)(mode == 0 ? ks : 2 * s) * Cout * Cin;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 16384);
    hipLaunchKernelGGL(k_prep_w16, dim3(grid), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, ks, s, mode, hi, lo);
    ZK_CHECK_LAUNCH("zk_dac_prep_w16");
    return 0;
}

extern "C" int zk_dac_conv16(const float* in, int B, int Cin, int Tin, const float* alpha, const uint16_t* whi,
                             const uint16_t* wlo, const float* bias, int Cout, int ks, int dil, int pad, int Qn,
                             int out_stride, int out_off, float* out, int Tout, const float* resid, int do_tanh,
                             const int32_t* lens, int in_scale, int out_scale, int npass, void* stream) {
    ZK_REQUIRE(Cin % CIC == 0, "zk_dac_conv16: Cin=%d must be a multiple of %d", Cin, CIC);
    ZK_REQUIRE(ks >= 1 && ks <= KSM && (ks - 1) * dil <= WINM - QT, "zk_dac_conv16: ks=%d dil=%d unsupported", ks, dil);
    ZK_REQUIRE(npass == 1 || npass == 3, "zk_dac_conv16: npass must be 1 or 3");
    ZK_REQUIRE(npass == 1 || wlo != nullptr, "zk_dac_conv16: npass=3 needs the lo weights");
    if (B == 0 || Qn <= 0) return 0;
    const int MT = (Cout % 64 == 0) ? 2 : 1;
    const int co_t = 32 * MT;
    const size_t lds = (size_t)(npass == 3 ? 2 : 1) * (WINM * 64 + KSM * co_t * 64);
    dim3 grid((Qn + QT - 1) / QT, (Cout + co_t - 1) / co_t, B);
#define ZK_C16(NP, M_)                                                                                          \
    ensure_lds(reinterpret_cast<const void*>(&k_conv16<NP, M_>), lds);                                                           \
    hipLaunchKernelGGL((k_conv16<NP, M_>), grid, dim3(256), lds, (hipStream_t)stream, in, Cin, Tin, alpha, whi, \
                       wlo, bias, Cout, ks, dil, pad, Qn, out_stride, out_off, out, Tout, resid, do_tanh, lens,   \
                       in_scale, out_scale)
    if (npass == 3) {
        if (MT == 2) { ZK_C16(3, 2); } else { ZK_C16(3, 1); }
    } else {
        if (MT == 2) { ZK_C16(1, 2); } else { ZK_C16(1, 1); }
    }
#undef ZK_C16
    ZK_CHECK_LAUNCH("zk_dac_conv16");
    return 0;
}

extern "C" int zk_dac_tail(const float* in, int B, int C, int T, const float* alpha, const float* w, const float* bias,
                           float* out, const int32_t* lens, int scale, void* stream) {
    ZK_REQUIRE(C > 0 && T >= 0, "zk_dac_tail: bad shape");
    if (B == 0 || T == 0) return 0;
    const size_t lds = (size_t)C * (TAIL_T + 6) * sizeof(float);
    ZK_REQUIRE(lds <= 160 * 1024, "zk_dac_tail: C=%d too large", C);
    ensure_lds(reinterpret_cast<const void*>(&k_dac_tail), lds);
    hipLaunchKernelGGL(k_dac_tail, dim3((T + TAIL_T - 1) / TAIL_T, B), dim3(256), lds, (hipStream_t)stream, in, C, T,
                       alpha, w, bias, out, lens, scale);
    ZK_CHECK_LAUNCH("zk_dac_tail");
    return 0;
}
