// codes_to_wavs post-processing on the GPU: the loudness measurement of normalize_loudness
// (zonos/autoencoder.py:172-186 -> pyloudnorm 0.1.1 Meter.integrated_loudness, ITU-R
// BS.1770-4) for a whole batch of decoded utterances at once (the reference runs it on the
// CPU, one utterance at a time, autoencoder.py:219-243).
//
//   k_kweight : K-weighting = high shelf then high pass biquad (RBJ cookbook coefficients as
//               pyloudnorm computes them), direct form II transposed like scipy.signal.lfilter,
//               float64; the recurrence is sequential, so one lane per utterance (B lanes).
//   k_blocks  : gating-block energies z_j = sum(y[l_j:u_j]^2) / (T_g * rate), one workgroup
//               per (block, utterance), fp64 reduction; l_j, u_j with pyloudnorm's own float64
//               expressions int(T_g * (j * 0.25) * rate), int(T_g * (j * 0.25 + 1) * rate).
//   k_gate    : absolute (-70 LUFS) and relative (-10 LU) gates -> integrated loudness ->
//               gain = 10^((target - L) / 20); utterances shorter than one block keep gain 1
//               (the reference's except path).
#include "common.h"
#include "../../include/zonos_hip.h"
#include <cmath>

namespace {

struct Biquad { double b0, b1, b2, a1, a2; };

ZK_DEV Biquad rbj(double G, double Q, double fc, double rate, bool shelf) {
    const double A = pow(10.0, G / 40.0);
    const double w0 = 2.0 * M_PI * (fc / rate);
    const double alpha = sin(w0) / (2.0 * Q);
    const double cw = cos(w0);
    double b0, b1, b2, a0, a1, a2;
    if (shelf) {
        b0 = A * ((A + 1) + (A - 1) * cw + 2 * sqrt(A) * alpha);
        b1 = -2 * A * ((A - 1) + (A + 1) * cw);
        b2 = A * ((A + 1) + (A - 1) * cw - 2 * sqrt(A) * alpha);
        a0 = (A + 1) - (A - 1) * cw + 2 * sqrt(A) * alpha;
        a1 = 2 * ((A - 1) - (A + 1) * cw);
        a2 = (A + 1) - (A - 1) * cw - 2 * sqrt(A) * alpha;
    } else {
        b0 = (1 + cw) / 2;
        b1 = -(1 + cw);
        b2 = (1 + cw) / 2;
        a0 = 1 + alpha;
        a1 = -2 * cw;
        a2 = 1 - alpha;
    }
    // pyloudnorm divides both vectors by a0; lfilter normalises by a[0] (= 1 then)
    return Biquad{b0 / a0, b1 / a0, b2 / a0, a1 / a0, a2 / a0};
}

ZK_DEV double block_size_of(int n, int rate) { return n > 2.0 * rate ? 0.400 : 0.100; }

__global__ __launch_bounds__(64) void k_kweight(const float* __restrict__ wav, int B, long T,
                                                const int32_t* __restrict__ lens, int rate, double* __restrict__ y) {
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= B) return;
    const long n = lens ? lens[b] : T;
    const Biquad f1 = rbj(4.0, 1.0 / sqrt(2.0), 1500.0, (double)rate, true);
    const Biquad f2 = rbj(0.0, 0.5, 38.0, (double)rate, false);
    const float* x = wav + (size_t)b * T;
    double* o = y + (size_t)b * T;
    double s1 = 0, s2 = 0, t1 = 0, t2 = 0;     // DF2T states of the two stages
    // scipy's lfilter (_linear_filter, double): y = Z0 + b0 x; Z0 = (Z1 + x b1) - y a1;
    // Z1 = x b2 - y a2 -- same operation order (built with -ffp-contract=off)
#define ZK_KW_STEP(XI, OUT)                                          \
    {                                                                \
        const double xi_ = (XI);                                     \
        const double u_ = s1 + f1.b0 * xi_;                          \
        s1 = (s2 + xi_ * f1.b1) - u_ * f1.a1;                        \
        s2 = xi_ * f1.b2 - u_ * f1.a2;                               \
        const double v_ = t1 + f2.b0 * u_;                           \
        t1 = (t2 + u_ * f2.b1) - v_ * f2.a1;                         \
        t2 = u_ * f2.b2 - v_ * f2.a2;                                \
        (OUT) = v_;                                                  \
    }
    long i = 0;
    if ((T & 3) == 0) {        // rows 16-B aligned: 8 samples per pair of vector loads, loads ahead of the chain
        for (; i + 8 <= n; i += 8) {
            const float4 xa = *reinterpret_cast<const float4*>(x + i);
            const float4 xb = *reinterpret_cast<const float4*>(x + i + 4);
            ZK_KW_STEP(xa.x, o[i + 0]) ZK_KW_STEP(xa.y, o[i + 1]) ZK_KW_STEP(xa.z, o[i + 2]) ZK_KW_STEP(xa.w, o[i + 3])
            ZK_KW_STEP(xb.x, o[i + 4]) ZK_KW_STEP(xb.y, o[i + 5]) ZK_KW_STEP(xb.z, o[i + 6]) ZK_KW_STEP(xb.w, o[i + 7])
        }
    }
    for (; i < n; ++i) ZK_KW_STEP((double)x[i], o[i])
#undef ZK_KW_STEP
}

__global__ __launch_bounds__(256) void k_blocks(const double* __restrict__ y, long T, const int32_t* __restrict__ lens,
                                                int rate, int max_blocks, double* __restrict__ z) {
    __shared__ double red[4];
    const int j = blockIdx.x, b = blockIdx.y;
    const long n = lens ? lens[b] : T;
    const double Tg = block_size_of((int)n, rate);
    const double Tsec = (double)n / rate;
    const long nb = (long)rint((Tsec - Tg) / (Tg * 0.25)) + 1;
    if (j >= nb || n < Tg * rate) {
        if (threadIdx.x == 0) z[(size_t)b * max_blocks + j] = -1.0;   // not a block
        return;
    }
    const long lo = (long)(Tg * (j * 0.25) * rate);
    const long hi = min((long)(Tg * (j * 0.25 + 1) * rate), n);
    const double* p = y + (size_t)b * T;
    double acc = 0;
    for (long i = lo + threadIdx.x; i < hi; i += 256) acc += p[i] * p[i];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) z[(size_t)b * max_blocks + j] = (1.0 / (Tg * rate)) * (red[0] + red[1] + red[2] + red[3]);
}

__global__ __launch_bounds__(64) void k_gate(const double* __restrict__ z, int B, long T, const int32_t* __restrict__ lens,
                                             int rate, int max_blocks, double target, double* __restrict__ gain,
                                             double* __restrict__ loud) {
    const int b = blockIdx.x;
    const long n = lens ? lens[b] : T;
    const double Tg = block_size_of((int)n, rate);
    if (n < Tg * rate) {
        if (threadIdx.x == 0) { gain[b] = 1.0; loud[b] = NAN; }
        return;
    }
    const double* zb = z + (size_t)b * max_blocks;
    // pass 1: absolute gate
    double s = 0;
    int c = 0;
    for (int j = threadIdx.x; j < max_blocks; j += 64) {
        const double zj = zb[j];
        if (zj < 0) continue;
        const double lj = -0.691 + 10.0 * log10(zj);
        if (lj >= -70.0) { s += zj; ++c; }
    }
    for (int off = 32; off > 0; off >>= 1) { s += __shfl_xor(s, off, 64); c += __shfl_xor(c, off, 64); }
    const double gamma_r = -0.691 + 10.0 * log10(c ? s / c : NAN) - 10.0;
    double s2 = 0;
    int c2 = 0;
    for (int j = threadIdx.x; j < max_blocks; j += 64) {
        const double zj = zb[j];
        if (zj < 0) continue;
        const double lj = -0.691 + 10.0 * log10(zj);
        if (lj > gamma_r && lj > -70.0) { s2 += zj; ++c2; }
    }
    for (int off = 32; off > 0; off >>= 1) { s2 += __shfl_xor(s2, off, 64); c2 += __shfl_xor(c2, off, 64); }
    if (threadIdx.x == 0) {
        const double zavg = c2 ? s2 / c2 : 0.0;            // np.nan_to_num(mean of nothing) = 0
        const double L = -0.691 + 10.0 * log10(zavg);
        loud[b] = L;
        gain[b] = pow(10.0, (target - L) / 20.0);
    }
}

// Polyphase windowed-sinc resampler (DACAutoencoder.preprocess -> torchaudio.functional.resample,
// autoencoder.py:21-25): out[n] = sum_k kern[n % up][k] * x[(n / up) * down + k - width], zero
// outside [0, T); fp32 taps in order k = 0..K-1. One thread per output sample.
__global__ __launch_bounds__(256) void k_resample(const float* __restrict__ x, long T, const float* __restrict__ kern,
                                                  int up, int down, int width, int K, float* __restrict__ out,
                                                  long Tout) {
    const long n = (long)blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (n >= Tout) return;
    const float* xb = x + (size_t)b * T;
    const float* kp = kern + (size_t)(n % up) * K;
    const long base = (n / up) * down - width;
    float acc = 0.f;
    for (int k = 0; k < K; ++k) {
        const long u = base + k;
        if (u >= 0 && u < T) acc = __fadd_rn(acc, __fmul_rn(kp[k], xb[u]));
    }
    out[(size_t)b * Tout + n] = acc;
}

}  // namespace

extern "C" int zk_resample(const float* x, int B, long T, const float* kern, int up, int down, int width, int K,
                           float* out, long Tout, void* stream) {
    ZK_REQUIRE(up > 0 && down > 0 && K > 0 && width >= 0 && T >= 0 && Tout >= 0, "zk_resample: bad arguments");
    if (B == 0 || Tout == 0) return 0;
    hipLaunchKernelGGL(k_resample, dim3((unsigned)((Tout + 255) / 256), B), dim3(256), 0, (hipStream_t)stream, x, T,
                       kern, up, down, width, K, out, Tout);
    ZK_CHECK_LAUNCH("zk_resample");
    return 0;
}

extern "C" int zk_loudness_gains(const float* wav, int B, long T, const int32_t* lens, int rate, double target_lufs,
                                 double* scratch, double* gains, double* loudness, void* stream) {
    ZK_REQUIRE(B >= 0 && T >= 0 && rate > 0 && scratch && gains && loudness, "zk_loudness_gains: bad arguments");
    if (B == 0) return 0;
    const int max_blocks = zk_loudness_max_blocks(T, rate);
    hipStream_t st = (hipStream_t)stream;
    double* y = scratch;
    double* z = scratch + (size_t)B * T;
    hipLaunchKernelGGL(k_kweight, dim3((B + 63) / 64), dim3(64), 0, st, wav, B, T, lens, rate, y);
    ZK_CHECK_LAUNCH("zk_loudness_gains/kweight");
    if (max_blocks > 0) {
        hipLaunchKernelGGL(k_blocks, dim3(max_blocks, B), dim3(256), 0, st, y, T, lens, rate, max_blocks, z);
        ZK_CHECK_LAUNCH("zk_loudness_gains/blocks");
    }
    hipLaunchKernelGGL(k_gate, dim3(B), dim3(64), 0, st, z, B, T, lens, rate, max_blocks, target_lufs, gains,
                       loudness);
    ZK_CHECK_LAUNCH("zk_loudness_gains/gate");
    return 0;
}

extern "C" int zk_loudness_max_blocks(long T, int rate) {
    // the most gating blocks any utterance of <= T samples can have (100 ms blocks, 25 ms hop)
    const double Tsec = (double)T / rate;
    const long nb = (long)std::rint((Tsec - 0.1) / (0.1 * 0.25)) + 1;
    return nb > 0 ? (int)nb : 0;
}
