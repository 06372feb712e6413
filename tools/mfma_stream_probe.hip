// Probe: does MFMA work in the SAME wave slow a once-read HBM weight stream (the decode GEMMs'
// structure), and do dedicated LDS-DMA loader waves fix it? fc1-sized stream (67 MB), 256
// workgroups (one per CU), back-to-back launches rotating over > 256 MB of buffers.
//   A: 4 waves, each streams its 64 KB share into registers (PF loads in flight) and issues NM
//      MFMA 16x16x32 per 1 KB loaded (the data as the B operand, a constant A), 8 accumulators.
//   B: 4 loader waves move the same bytes into per-wave LDS rings by LDS-DMA (nt) and publish each
//      1 KB slot with an LDS flag; 4 compute waves wait for the flag, read the slot (ds_read_b128),
//      free it and issue the NM MFMAs.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_stream_probe.hip -o /tmp/mfma_stream_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int NCH = 64;          // 1 KB chunks per wave (64 KB per wave, 256 KB per workgroup)

template <int NM, int PF>
__global__ __launch_bounds__(256, 1) void k_reg(const u32x4* __restrict__ W, float* out) {
    const int lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const u32x4* p = W + wave * NCH * 64 + lane;
    u32x4 r[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) r[i] = __builtin_nontemporal_load(p + i * 64);
    const bf16x8 a = __builtin_bit_cast(bf16x8, u32x4{lane * 0x00010001u, 0x3f803f80u, 7u, 9u});
    f32x4 acc[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const u32x4 v = r[c % PF];
        if (c + PF < NCH) r[c % PF] = __builtin_nontemporal_load(p + (c + PF) * 64);
        const bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
        for (int m = 0; m < NM; ++m) acc[m % 8] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m % 8], 0, 0, 0);
        if (NM == 0) acc[0][0] += __builtin_bit_cast(float, v.x ^ v.w);
    }
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) s += acc[m][0] + acc[m][3];
    if (s == 1.2345f) out[0] = s;
}

// B: loader wave l (waves 4..7) fills ring l (RS slots of 1 KB) for compute wave l (waves 0..3)
template <int NM, int RS, int DA>
__global__ __launch_bounds__(512, 1) void k_split(const u32x4* __restrict__ W, float* out) {
    __shared__ __attribute__((aligned(16))) char ring[4][RS][1024];
    __shared__ int full[4][RS], freed[4][RS];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, pair = wv & 3;
    if (threadIdx.x < 4 * RS) { (&full[0][0])[threadIdx.x] = -1; (&freed[0][0])[threadIdx.x] = -1; }
    __syncthreads();
    const size_t wave = (size_t)blockIdx.x * 4 + pair;
    const char* src = reinterpret_cast<const char*>(W) + wave * NCH * 1024 + lane * 16;
    if (wv >= 4) {
        // loader: DA slots in flight; publish slot c once its DMA landed (counted vmcnt)
        for (int c = 0; c < NCH + DA; ++c) {
            if (c < NCH) {
                const int slot = c % RS;
                if (c >= RS) {           // wait until the consumer freed this slot's previous use (bounded)
                    for (int spin = 0; spin < (1 << 22) && __atomic_load_n(&freed[pair][slot], __ATOMIC_RELAXED) < c - RS;
                         ++spin) __builtin_amdgcn_s_sleep(1);
                }
                __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)c * 1024), (void*)ring[pair][slot], 16, 0, 2);
            }
            const int pub = c - DA;
            if (pub >= 0) {
                if (c < NCH) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DA) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) __atomic_store_n(&full[pair][pub % RS], pub, __ATOMIC_RELAXED);
            }
        }
        return;
    }
    const bf16x8 a = __builtin_bit_cast(bf16x8, u32x4{lane * 0x00010001u, 0x3f803f80u, 7u, 9u});
    f32x4 acc[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < NCH; ++c) {
        const int slot = c % RS;
        for (int spin = 0; spin < (1 << 22) && __atomic_load_n(&full[pair][slot], __ATOMIC_RELAXED) < c; ++spin)
            __builtin_amdgcn_s_sleep(1);
        const u32x4 v = *reinterpret_cast<const u32x4*>(ring[pair][slot] + lane * 16);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __atomic_store_n(&freed[pair][slot], c, __ATOMIC_RELAXED);
        const bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
        for (int m = 0; m < NM; ++m) acc[m % 8] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m % 8], 0, 0, 0);
        if (NM == 0) acc[0][0] += __builtin_bit_cast(float, v.x ^ v.w);
    }
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) s += acc[m][0] + acc[m][3];
    if (s == 1.2345f) out[0] = s;
}

// C: the stream of A (NM = 0) in waves 0-3 and NM MFMA per KB-equivalent in waves 4-7 on
// register-constant operands, no dependency between them: does MFMA work elsewhere on the CU
// (or the chip) slow the stream?
template <int NM>
__global__ __launch_bounds__(512, 1) void k_side(const u32x4* __restrict__ W, float* out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const bf16x8 a = __builtin_bit_cast(bf16x8, u32x4{lane * 0x00010001u, 0x3f803f80u, 7u, 9u});
    f32x4 acc[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (wv < 4) {
        const size_t wave = (size_t)blockIdx.x * 4 + wv;
        const u32x4* p = W + wave * NCH * 64 + lane;
        constexpr int PF = 8;
        u32x4 r[PF];
#pragma unroll
        for (int i = 0; i < PF; ++i) r[i] = __builtin_nontemporal_load(p + i * 64);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const u32x4 v = r[c % PF];
            if (c + PF < NCH) r[c % PF] = __builtin_nontemporal_load(p + (c + PF) * 64);
            acc[0][0] += __builtin_bit_cast(float, v.x ^ v.w);
        }
    } else {
        const bf16x8 b = __builtin_bit_cast(bf16x8, u32x4{lane * 3u, 0x3f803f80u, 5u, 11u});
        for (int c = 0; c < NCH; ++c) {
#pragma unroll
            for (int m = 0; m < NM; ++m) acc[m % 8] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m % 8], 0, 0, 0);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) s += acc[m][0] + acc[m][3];
    if (s == 1.2345f) out[0] = s;
}

// D: split with SLOT-KB slots: loader wave publishes SLOT x 1 KB per handshake
template <int NM, int RS, int DA, int SLOT>
__global__ __launch_bounds__(512, 1) void k_split2(const u32x4* __restrict__ W, float* out) {
    __shared__ __attribute__((aligned(16))) char ring[4][RS][SLOT * 1024];
    __shared__ int full[4][RS], freed[4][RS];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, pair = wv & 3;
    if (threadIdx.x < 4 * RS) { (&full[0][0])[threadIdx.x] = -1; (&freed[0][0])[threadIdx.x] = -1; }
    __syncthreads();
    const size_t wave = (size_t)blockIdx.x * 4 + pair;
    const char* src = reinterpret_cast<const char*>(W) + wave * NCH * 1024 + lane * 16;
    constexpr int NS = NCH / SLOT;
    if (wv >= 4) {
        for (int c = 0; c < NS + DA; ++c) {
            if (c < NS) {
                const int slot = c % RS;
                if (c >= RS)
                    for (int spin = 0; spin < (1 << 22) && __atomic_load_n(&freed[pair][slot], __ATOMIC_RELAXED) < c - RS;
                         ++spin) __builtin_amdgcn_s_sleep(1);
#pragma unroll
                for (int j = 0; j < SLOT; ++j)
                    __builtin_amdgcn_global_load_lds((const void*)(src + ((size_t)c * SLOT + j) * 1024),
                                                     (void*)(ring[pair][slot] + j * 1024), 16, 0, 2);
            }
            const int pub = c - DA;
            if (pub >= 0) {
                if (c < NS) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DA * SLOT) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) __atomic_store_n(&full[pair][pub % RS], pub, __ATOMIC_RELAXED);
            }
        }
        return;
    }
    const bf16x8 a = __builtin_bit_cast(bf16x8, u32x4{lane * 0x00010001u, 0x3f803f80u, 7u, 9u});
    f32x4 acc[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < NS; ++c) {
        const int slot = c % RS;
        for (int spin = 0; spin < (1 << 22) && __atomic_load_n(&full[pair][slot], __ATOMIC_RELAXED) < c; ++spin)
            __builtin_amdgcn_s_sleep(1);
        u32x4 v[SLOT];
#pragma unroll
        for (int j = 0; j < SLOT; ++j) v[j] = *reinterpret_cast<const u32x4*>(ring[pair][slot] + j * 1024 + lane * 16);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __atomic_store_n(&freed[pair][slot], c, __ATOMIC_RELAXED);
#pragma unroll
        for (int j = 0; j < SLOT; ++j) {
            const bf16x8 b = __builtin_bit_cast(bf16x8, v[j]);
#pragma unroll
            for (int m = 0; m < NM; ++m) acc[m % 8] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m % 8], 0, 0, 0);
            if (NM == 0) acc[0][0] += __builtin_bit_cast(float, v[j].x ^ v[j].w);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) s += acc[m][0] + acc[m][3];
    if (s == 1.2345f) out[0] = s;
}

template <class F>
float timeit(F launch, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 4; ++i) launch(i);
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) launch(i);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f / reps;
}

int main() {
    const size_t bytes = (size_t)256 * 4 * NCH * 1024;   // 67 MB
    const int ncopy = 6;                                 // > 256 MB rotating
    std::vector<u32x4*> bufs(ncopy);
    for (auto& b : bufs) {
        CK(hipMalloc(&b, bytes));
        CK(hipMemset(b, 0x3c, bytes));
    }
    float* out;
    CK(hipMalloc(&out, 64));
#define RUN_REG(NM, PF)                                                                                  \
    {                                                                                                    \
        float us = timeit([&](int i) { hipLaunchKernelGGL((k_reg<NM, PF>), dim3(256), dim3(256), 0, 0,   \
                                                           bufs[i % ncopy], out); }, 30);                \
        printf("A reg    MFMA/KB=%2d PF=%2d         : %7.2f us  %6.0f GB/s\n", NM, PF, us, bytes / us / 1e3); \
    }
#define RUN_SPLIT(NM, RS, DA)                                                                            \
    {                                                                                                    \
        float us = timeit([&](int i) { hipLaunchKernelGGL((k_split<NM, RS, DA>), dim3(256), dim3(512), 0, 0, \
                                                           bufs[i % ncopy], out); }, 30);                \
        printf("B split  MFMA/KB=%2d ring=%2d DA=%2d : %7.2f us  %6.0f GB/s\n", NM, RS, DA, us, bytes / us / 1e3); \
    }
#define RUN_SIDE(NM)                                                                                     \
    {                                                                                                    \
        float us = timeit([&](int i) { hipLaunchKernelGGL((k_side<NM>), dim3(256), dim3(512), 0, 0,       \
                                                           bufs[i % ncopy], out); }, 30);                \
        printf("C side   MFMA/KB=%2d (other waves)  : %7.2f us  %6.0f GB/s\n", NM, us, bytes / us / 1e3); \
    }
#define RUN_SPLIT2(NM, RS, DA, SLOT)                                                                     \
    {                                                                                                    \
        float us = timeit([&](int i) { hipLaunchKernelGGL((k_split2<NM, RS, DA, SLOT>), dim3(256), dim3(512), 0, 0, \
                                                           bufs[i % ncopy], out); }, 30);                \
        printf("D split  MFMA/KB=%2d ring=%2d DA=%2d slot=%2d KB : %7.2f us  %6.0f GB/s\n", NM, RS, DA, SLOT, us,   \
               bytes / us / 1e3);                                                                        \
    }
    for (int rep = 0; rep < 2; ++rep) {
        RUN_REG(0, 8) RUN_REG(1, 8) RUN_REG(2, 8) RUN_REG(8, 8)
        RUN_SIDE(0) RUN_SIDE(1) RUN_SIDE(8) RUN_SIDE(16)
        RUN_SPLIT2(0, 4, 2, 8) RUN_SPLIT2(8, 4, 2, 8) RUN_SPLIT2(8, 4, 3, 8) RUN_SPLIT2(8, 8, 4, 4) RUN_SPLIT2(8, 2, 1, 16)
    }
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
