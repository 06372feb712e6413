// Probe: which float32 log reproduces torch's CUDA/ROCm `Tensor.exponential_(1)` bit for bit?
// (ATen/native/hip/DistributionTemplates.h: distribution_elementwise_grid_stride_kernel +
// hiprand_uniform4 + transformation::exponential, whose device `at::log` is `__logf`.)
// Element e of an n-element tensor: t = e % stride, q = e / stride, word (q & 3) of
// Philox4x32-10(counter = (offset / 4 + (q >> 2), t), key = seed); u = 2^-32 + word * 2^-32;
// q = -log(u) unless u >= 1 - 2^-24 (then 2^-24).
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/torch_noise_probe.hip -o tools/torch_noise_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" __device__ float __ocml_native_log_f32(float);
extern "C" __device__ float __ocml_log_f32(float);
extern "C" __device__ float __ocml_native_log2_f32(float);

namespace {
__device__ uint32_t mulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

__device__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = mulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = mulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = uint4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

__global__ void k_probe(float* out, long n, uint64_t seed, uint64_t off, int stride, int variant) {
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
        const long t = e % stride, q = e / stride;
        const uint64_t ctr = off / 4 + (uint64_t)(q >> 2);
        const uint4 r = philox(uint4{(uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)t, (uint32_t)(t >> 32)},
                               (uint32_t)seed, (uint32_t)(seed >> 32));
        const uint32_t w = (q & 3) == 0 ? r.x : (q & 3) == 1 ? r.y : (q & 3) == 2 ? r.z : r.w;
        const float u = 2.3283064e-10f + (float)w * 2.3283064e-10f;
        float lg;
        const float y = __builtin_amdgcn_logf(u);
        if (variant == 0) lg = __builtin_logf(u);
        else if (variant == 1) lg = y * 0.693147182f;
        else if (variant == 2) lg = (float)log((double)u);
        else if (variant == 3) lg = __logf(u);
        else if (variant == 4) lg = y * __builtin_bit_cast(float, 0x3f317217u);
        else if (variant == 5) lg = (float)((double)y * 0.6931471805599453);
        else if (variant == 6) lg = __ocml_native_log_f32(u);
        else if (variant == 7) lg = __ocml_log_f32(u);
        else if (variant == 8) lg = __ocml_native_log2_f32(u) * 0.693147182f;
        else {                                     // y * ln2 with ln2 split hi + lo (fma)
            const float ch = __builtin_bit_cast(float, 0x3f317218u), cl = __builtin_bit_cast(float, 0xb102e308u);
            lg = __builtin_fmaf(y, ch, y * cl);
        }
        const float l = u >= 1.0f - 5.96046448e-08f ? -5.96046448e-08f : lg;
        out[e] = -1.0f * l;
    }
}
}  // namespace

extern "C" int probe_noise(float* out, long n, uint64_t seed, uint64_t off, int stride, int variant) {
    hipLaunchKernelGGL(k_probe, dim3(1024), dim3(256), 0, 0, out, n, seed, off, stride, variant);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
