// PrefixConditioner.forward on the GPU (zonos/conditioning.py:373-389): every conditioner's rows,
// their concatenation along the sequence, the optional prefix projection and the final LayerNorm
// in ONE launch -- one workgroup per output row (position l of utterance b), the row built in LDS
// at the bf16 rounding points of the bf16 module:
//   phoneme / integer embedding  : table row                            (nn.Embedding, bf16)
//   learned unconditional vector : uncond_vector                        (Conditioner.forward 46-48)
//   Fourier features             : x' = bf16((x - min) / (max - min)); s = bf16(2pi * x');
//                                  f = bf16(s @ W^T); row = [bf16(cos f), bf16(sin f)]  (318-337)
//   passthrough                  : the bf16 input row                   (352-358)
//   projection linear / mlp      : bf16(W x + b) / bf16(W2 bf16(silu(bf16(W1 x + b1))) + b2)  (27-34)
//   LayerNorm (eps 1e-5)         : fp32 statistics, bf16(((v - mean) * rstd) * w + b)
#include "common.h"
#include "../../include/zonos_hip.h"
#include <cmath>

namespace {

constexpr int CN_THREADS = 256;
constexpr int CN_MAXD = 4096;

ZK_DEV float silu_f(float x) { return x / (1.0f + expf(-x)); }

// out[d] = bf16(sum_c in[c] * W[d][c] + b[d]) for d < dout (fp32 accumulation, c ascending)
ZK_DEV void row_linear(const float* in, int cin, const bf16_t* __restrict__ W, const bf16_t* __restrict__ b,
                       int dout, float* out) {
    for (int d = threadIdx.x; d < dout; d += CN_THREADS) {
        const bf16_t* w = W + (size_t)d * cin;
        float acc = 0.f;
        for (int c = 0; c < cin; ++c) acc += in[c] * bf2f(w[c]);
        out[d] = round_bf(acc + (b ? bf2f(b[d]) : 0.f));
    }
}

// projection 1 = linear, 2 = mlp; the row lives in `a` (length cin) and ends in `a` (length D)
ZK_DEV void project(int kind, float* a, float* t, int cin, int D, const bf16_t* w0, const bf16_t* b0,
                    const bf16_t* w1, const bf16_t* b1) {
    if (kind == 0) return;
    __syncthreads();
    row_linear(a, cin, w0, b0, D, t);
    __syncthreads();
    if (kind == 1) {
        for (int d = threadIdx.x; d < D; d += CN_THREADS) a[d] = t[d];
    } else {
        for (int d = threadIdx.x; d < D; d += CN_THREADS) t[d] = round_bf(silu_f(t[d]));
        __syncthreads();
        row_linear(t, D, w1, b1, D, a);
    }
    __syncthreads();
}

__global__ __launch_bounds__(CN_THREADS) void k_prefix_cond(ZkCondPlan plan, bf16_t* __restrict__ out) {
    __shared__ float a[CN_MAXD];
    __shared__ float t[CN_MAXD];
    __shared__ float red[CN_THREADS / 64];
    __shared__ float xs[ZK_COND_MAXIN];
    const int l = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const int D = plan.D;
    int s = 0, r = l;
    while (s + 1 < plan.nseg && r >= plan.seg[s].len) r -= plan.seg[s++].len;
    const ZkCondSeg& g = plan.seg[s];
    const int bb = g.bin > 1 ? b : 0;
    const int cin = g.cin;
    switch (g.type) {
        case ZK_SEG_VECTOR:
            for (int d = tid; d < D; d += CN_THREADS) a[d] = bf2f(((const bf16_t*)g.table)[d]);
            break;
        case ZK_SEG_EMBED: {
            const long id = ((const int64_t*)g.input)[(size_t)bb * g.in_bstride + r] - g.id_min;
            const bf16_t* row = (const bf16_t*)g.table + (size_t)id * cin;
            for (int d = tid; d < cin; d += CN_THREADS) a[d] = bf2f(row[d]);
            break;
        }
        case ZK_SEG_FOURIER: {
            const float* x = (const float*)g.input + (size_t)bb * g.in_bstride + (size_t)r * g.in_dim;
            if (tid < g.in_dim) {
                const float xn = round_bf(__fdiv_rn(__fsub_rn(x[tid], g.vmin), g.vden));
                xs[tid] = round_bf(__fmul_rn(6.28318530717958647692f, xn));
            }
            __syncthreads();
            const int half = cin / 2;
            const bf16_t* W = (const bf16_t*)g.table;
            for (int d = tid; d < half; d += CN_THREADS) {
                float f = 0.f;
                for (int j = 0; j < g.in_dim; ++j) f += xs[j] * bf2f(W[(size_t)d * g.in_dim + j]);
                f = round_bf(f);
                a[d] = round_bf(cosf(f));
                a[d + half] = round_bf(sinf(f));
            }
            break;
        }
        case ZK_SEG_PASS: {
            const bf16_t* x = (const bf16_t*)g.input + (size_t)bb * g.in_bstride + (size_t)r * cin;
            for (int d = tid; d < cin; d += CN_THREADS) a[d] = bf2f(x[d]);
            break;
        }
        default:
            break;
    }
    if (g.type != ZK_SEG_VECTOR)
        project(g.proj, a, t, cin, D, (const bf16_t*)g.pw0, (const bf16_t*)g.pb0, (const bf16_t*)g.pw1,
                (const bf16_t*)g.pb1);
    project(plan.proj, a, t, D, D, (const bf16_t*)plan.pw0, (const bf16_t*)plan.pb0, (const bf16_t*)plan.pw1,
            (const bf16_t*)plan.pb1);
    __syncthreads();
    bf16_t* o = out + ((size_t)b * plan.L + l) * D;
    if (!plan.norm_w) {
        for (int d = tid; d < D; d += CN_THREADS) o[d] = f2bf(a[d]);
        return;
    }
    // LayerNorm: two-pass fp32 statistics over the row
    float sum = 0.f;
    for (int d = tid; d < D; d += CN_THREADS) sum += a[d];
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
    if ((tid & 63) == 0) red[tid >> 6] = sum;
    __syncthreads();
    const float mean = (red[0] + red[1] + red[2] + red[3]) / (float)D;
    __syncthreads();
    float sq = 0.f;
    for (int d = tid; d < D; d += CN_THREADS) {
        const float c = a[d] - mean;
        sq += c * c;
    }
    for (int off = 32; off > 0; off >>= 1) sq += __shfl_xor(sq, off, 64);
    if ((tid & 63) == 0) red[tid >> 6] = sq;
    __syncthreads();
    const float rstd = 1.0f / sqrtf((red[0] + red[1] + red[2] + red[3]) / (float)D + plan.eps);
    const bf16_t* nw = (const bf16_t*)plan.norm_w;
    const bf16_t* nb = (const bf16_t*)plan.norm_b;
    for (int d = tid; d < D; d += CN_THREADS) o[d] = f2bf((a[d] - mean) * rstd * bf2f(nw[d]) + bf2f(nb[d]));
}

}  // namespace

extern "C" int zk_prefix_cond(const ZkCondPlan* plan, int B, void* out, void* stream) {
    ZK_REQUIRE(plan && plan->nseg > 0 && plan->nseg <= ZK_COND_MAXSEG, "zk_prefix_cond: nseg");
    ZK_REQUIRE(plan->D > 0 && plan->D <= CN_MAXD && plan->D % 2 == 0, "zk_prefix_cond: D=%d", plan->D);
    int L = 0;
    for (int i = 0; i < plan->nseg; ++i) {
        const ZkCondSeg& g = plan->seg[i];
        ZK_REQUIRE(g.len >= 0 && g.cin > 0 && g.cin <= CN_MAXD && (g.table != nullptr || g.type == ZK_SEG_PASS),
                   "zk_prefix_cond: segment %d", i);
        ZK_REQUIRE(g.type != ZK_SEG_FOURIER || (g.in_dim > 0 && g.in_dim <= ZK_COND_MAXIN && g.cin % 2 == 0),
                   "zk_prefix_cond: Fourier segment %d input_dim %d", i, g.in_dim);
        ZK_REQUIRE(g.type == ZK_SEG_VECTOR || g.input != nullptr, "zk_prefix_cond: segment %d has no input", i);
        ZK_REQUIRE(g.proj != 0 || g.type == ZK_SEG_VECTOR || g.cin == plan->D,
                   "zk_prefix_cond: segment %d width %d != D without projection", i, g.cin);
        L += g.len;
    }
    ZK_REQUIRE(L == plan->L, "zk_prefix_cond: segment lengths sum to %d, plan L=%d", L, plan->L);
    if (B == 0 || L == 0) return 0;
    hipLaunchKernelGGL(k_prefix_cond, dim3(L, B), dim3(CN_THREADS), 0, (hipStream_t)stream, *plan, (bf16_t*)out);
    ZK_CHECK_LAUNCH("zk_prefix_cond");
    return 0;
}
