// DAC decoder kernels for gfx950 (transformers' DacModel.decode restated,
// modeling_dac.py:86-100, 175-264, 347-371, 407-441).
//
// Every Conv1d / ConvTranspose1d of the decoder is one implicit-GEMM kernel, k_conv:
//   out[b][co][t(q)] = bias[co] + sum_{ci,k} W[co][ci][k] * act(in[b][ci][q + k*dil - pad])
// with the Snake activation fused into the input staging (each input element is
// activated once per workgroup, not once per tap), the residual add / tanh fused into the
// epilogue, and ConvTranspose1d(stride s, kernel 2s) run as s polyphase 2-tap convolutions
// (t(q) = q*s + r - ceil(s/2)). The GEMM is M = Cout, N = time, K = Cin x taps on
// MFMA 16x16x4 f32 (exact fp32 products, the precision of the reference's CPU path).
//
// Per-row valid lengths make a zero-padded batch decode equal to decoding each utterance
// alone (codes_to_wavs decodes one utterance at a time, autoencoder.py:219-226): inputs
// beyond a row's length read as zero at every layer, exactly like the conv padding of a
// shorter standalone sequence.
#include "common.h"
#include "../../include/zonos_hip.h"
#include <algorithm>

namespace {

typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int CBM = 64;      // output channels per workgroup
constexpr int CBN = 64;      // output positions per workgroup
constexpr int CI = 16;       // input channels per K chunk
constexpr int KS_MAX = 7;
constexpr int WIN_MAX = CBN + (KS_MAX - 1) * 9;   // 118

ZK_DEV float snake(float x, float a) {
    // x + (a + 1e-9)^-1 * sin(a x)^2   (Snake1d.forward, modeling_dac.py:98)
    const float s = sinf(__fmul_rn(a, x));
    const float r = __fdiv_rn(1.0f, __fadd_rn(a, 1e-9f));
    return __fadd_rn(x, __fmul_rn(r, __fmul_rn(s, s)));
}

__global__ __launch_bounds__(256) void k_conv(const float* __restrict__ in, int Cin, int Tin,
                                              const float* __restrict__ alpha, const float* __restrict__ w,
                                              const float* __restrict__ bias, int Cout, int ks, int dil, int pad,
                                              int Qn, int out_stride, int out_off, float* __restrict__ out, int Tout,
                                              const float* __restrict__ resid, int do_tanh,
                                              const int32_t* __restrict__ lens, int in_scale, int out_scale) {
    __shared__ float xs[CI][WIN_MAX + 2];
    __shared__ float ws[CBM][CI * KS_MAX + 1];
    const int q0 = blockIdx.x * CBN, co0 = blockIdx.y * CBM, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ln = lane & 15, lg = lane >> 4;
    const int len_in = lens ? lens[b] * in_scale : Tin;
    const int len_out = lens ? lens[b] * out_scale : Tout;
    const int win = CBN + (ks - 1) * dil;
    const int u0 = q0 - pad;
    const float* inb = in + (size_t)b * Cin * Tin;

    f32x4 acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int ci0 = 0; ci0 < Cin; ci0 += CI) {
        __syncthreads();
        for (int i = tid; i < CI * win; i += 256) {
            const int c = i / win, j = i % win;
            const int u = u0 + j;
            float v = 0.f;
            if (u >= 0 && u < len_in && u < Tin) {
                v = inb[(size_t)(ci0 + c) * Tin + u];
                if (alpha) v = snake(v, alpha[ci0 + c]);
            }
            xs[c][j] = v;
        }
        for (int i = tid; i < CBM * CI * ks; i += 256) {
            const int r = i / (CI * ks), e = i % (CI * ks);
            const int co = co0 + r;
            ws[r][e] = co < Cout ? w[((size_t)co * Cin + ci0) * ks + e] : 0.f;
        }
        __syncthreads();
        for (int tap = 0; tap < ks; ++tap) {
#pragma unroll
            for (int c4 = 0; c4 < CI / 4; ++c4) {
                const int ci = c4 * 4 + lg;
                const float a = ws[wv * 16 + ln][ci * ks + tap];
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
                    const float bv = xs[ci][nt * 16 + ln + tap * dil];
                    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc[nt], 0, 0, 0);
                }
            }
        }
    }
    // acc[nt][i] = C[co = co0 + 16wv + 4lg + i][q = q0 + 16nt + ln]
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int q = q0 + nt * 16 + ln;
        if (q >= Qn) continue;
        const int t = q * out_stride + out_off;
        if (t < 0 || t >= Tout) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int co = co0 + wv * 16 + lg * 4 + i;
            if (co >= Cout) continue;
            const size_t o = ((size_t)b * Cout + co) * Tout + t;
            float v = 0.f;
            if (t < len_out) {
                v = __fadd_rn(acc[nt][i], bias[co]);
                if (resid) v = __fadd_rn(resid[o], v);
                if (do_tanh) v = tanhf(v);
            }
            out[o] = v;
        }
    }
}

__global__ void k_rvq_tables(const float* cb, const float* ow, const float* ob, int ncode, int cdim, int hidden,
                             float* tables) {
    const int c = blockIdx.x, k = blockIdx.y;
    const float* e = cb + ((size_t)k * ncode + c) * cdim;
    for (int ch = threadIdx.x; ch < hidden; ch += blockDim.x) {
        const float* wr = ow + ((size_t)k * hidden + ch) * cdim;
        float s = 0.f;
        for (int d = 0; d < cdim; ++d) s = fmaf(wr[d], e[d], s);
        tables[((size_t)k * ncode + c) * hidden + ch] = s + ob[(size_t)k * hidden + ch];
    }
}

__global__ void k_rvq_decode(const int64_t* codes, int ncb, int T, long bstr, const float* tables, int ncode,
                             int hidden, float* z, int Tz, const int32_t* lens) {
    const int t = blockIdx.x, b = blockIdx.y;
    const int len = lens ? lens[b] : T;
    for (int ch = threadIdx.x; ch < hidden; ch += blockDim.x) {
        float s = 0.f;
        if (t < len && t < T) {
            for (int k = 0; k < ncb; ++k) {
                int64_t c = codes[b * bstr + (size_t)k * T + t];
                c = c < 0 ? 0 : (c >= ncode ? ncode - 1 : c);
                const float e = tables[((size_t)k * ncode + c) * hidden + ch];
                s = (k == 0) ? e : __fadd_rn(s, e);
            }
        }
        z[((size_t)b * hidden + ch) * Tz + t] = s;
    }
}

__global__ void k_prep_convt(const float* w, int Cin, int Cout, int s, float* out) {
    // out[r][co][ci][0] = w[ci][co][r+s] (tap reads in[q-1]); out[r][co][ci][1] = w[ci][co][r] (in[q])
    const size_t n = (size_t)s * Cout * Cin;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int ci = (int)(i % Cin);
        const int co = (int)((i / Cin) % Cout);
        const int r = (int)(i / ((size_t)Cin * Cout));
        const float* src = w + ((size_t)ci * Cout + co) * (2 * s);
        out[i * 2 + 0] = src[r + s];
        out[i * 2 + 1] = src[r];
    }
}

}  // namespace

extern "C" int zk_dac_rvq_tables(const float* codebooks, const float* out_w, const float* out_b, int ncb, int ncode,
                                 int cdim, int hidden, float* tables, void* stream) {
    ZK_REQUIRE(ncb > 0 && ncode > 0 && cdim > 0 && hidden > 0, "zk_dac_rvq_tables: bad shape");
    hipLaunchKernelGGL(k_rvq_tables, dim3(ncode, ncb), dim3(256), 0, (hipStream_t)stream, codebooks, out_w, out_b,
                       ncode, cdim, hidden, tables);
    ZK_CHECK_LAUNCH("zk_dac_rvq_tables");
    return 0;
}

extern "C" int zk_dac_rvq_decode(const int64_t* codes, int B, int ncb, int T, long code_bstride,
                                 const float* tables, int ncode, int hidden, float* z, int Tz, const int32_t* lens,
                                 void* stream) {
    ZK_REQUIRE(Tz >= T, "zk_dac_rvq_decode: Tz < T");
    if (B == 0 || T == 0) return 0;
    hipLaunchKernelGGL(k_rvq_decode, dim3(T, B), dim3(256), 0, (hipStream_t)stream, codes, ncb, T, code_bstride,
                       tables, ncode, hidden, z, Tz, lens);
    ZK_CHECK_LAUNCH("zk_dac_rvq_decode");
    return 0;
}

extern "C" int zk_dac_conv(const float* in, int B, int Cin, int Tin, const float* alpha, const float* w,
                           const float* bias, int Cout, int ks, int dil, int pad, int Qn, int out_stride, int out_off,
                           float* out, int Tout, const float* resid, int do_tanh, const int32_t* lens, int in_scale,
                           int out_scale, void* stream) {
    ZK_REQUIRE(Cin % CI == 0, "zk_dac_conv: Cin=%d must be a multiple of %d", Cin, CI);
    ZK_REQUIRE(ks >= 1 && ks <= KS_MAX && (ks - 1) * dil <= WIN_MAX - CBN, "zk_dac_conv: ks=%d dil=%d unsupported", ks,
               dil);
    if (B == 0 || Qn <= 0) return 0;
    dim3 grid((Qn + CBN - 1) / CBN, (Cout + CBM - 1) / CBM, B);
    hipLaunchKernelGGL(k_conv, grid, dim3(256), 0, (hipStream_t)stream, in, Cin, Tin, alpha, w, bias, Cout, ks, dil,
                       pad, Qn, out_stride, out_off, out, Tout, resid, do_tanh, lens, in_scale, out_scale);
    ZK_CHECK_LAUNCH("zk_dac_conv");
    return 0;
}

extern "C" int zk_dac_prep_convt(const float* w, int Cin, int Cout, int s, float* w_out, void* stream) {
    ZK_REQUIRE(Cin > 0 && Cout > 0 && s > 0, "zk_dac_prep_convt: bad shape");
    const size_t n = (size_t)s * Cout * Cin;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_prep_convt, dim3(grid), dim3(256), 0, (hipStream_t)stream, w, Cin, Cout, s, w_out);
    ZK_CHECK_LAUNCH("zk_dac_prep_convt");
    return 0;
}
