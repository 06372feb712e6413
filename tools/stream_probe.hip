// Weight-stream probe: how fast can one launch read a once-read bf16 weight matrix of the
// decode GEMM sizes (8.4 / 12.6 / 33.5 / 67 MB) from HBM, as a function of bytes in flight
// per wave (register ring depth PF) and waves per CU? No MFMA, no activations: the ceiling a
// decode GEMM launch can reach. Launches run back to back (boundaries included, as in the
// hipGraph replay), rotating over >400 MB of buffers so the Infinity Cache does not serve them.
//   hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o tools/stream_probe && ./tools/stream_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// each wave streams NCH x 1 KB (64 lanes x 16 B) contiguous; PF loads in flight
template <int NCH, int PF>
__global__ void k_reg(const uint4* __restrict__ W, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const u32x4* p = reinterpret_cast<const u32x4*>(W) + wave * NCH * 64 + lane;
    u32x4 r[PF];
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < PF; ++i) r[i] = __builtin_nontemporal_load(p + i * 64);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const u32x4 v = r[c % PF];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
        if (c + PF < NCH) r[c % PF] = __builtin_nontemporal_load(p + (c + PF) * 64);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// LDS-DMA: each wave moves its NCH x 1 KB by global_load_lds into a DEPTH-slot ring (no consumer)
template <int NCH, int DEPTH>
__global__ void k_dma(const uint4* __restrict__ W, uint32_t* out) {
    extern __shared__ char smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t wave = (size_t)blockIdx.x * (blockDim.x >> 6) + wv;
    const char* p = reinterpret_cast<const char*>(W) + wave * NCH * 1024 + lane * 16;
    char* ring = smem + wv * DEPTH * 1024;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        __builtin_amdgcn_global_load_lds((const void*)(p + c * 1024), (void*)(ring + (c % DEPTH) * 1024), 16, 0, 2);
        if (c >= DEPTH - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH - 1) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (reinterpret_cast<uint32_t*>(ring)[lane] == 0x12345678u) out[0] = 1;
}

// Attention-shaped stream (k_attn_decode at B=64: 512 workgroups = (row, kv head), 2 per CU,
// each streaming its row's K and V^T caches in 32-key slices of 8 KB + 8 KB, wave w taking slice
// 4*blk + w, two register sets in flight). ROT: each workgroup starts at a different key block
// (address stagger); ADJ: K and V slices adjacent in one array (16 KB contiguous per slice).
struct Frag { uint4 k[8]; uint4 v[8]; };
template <bool ADJ, bool NTL = false>
__device__ __forceinline__ void ld(Frag& f, const char* kb, const char* vb, int slice, int lane) {
    const char* k0 = ADJ ? kb + (size_t)slice * 16384 + lane * 16 : kb + (size_t)slice * 8192 + lane * 16;
    const char* v0 = ADJ ? k0 + 8192 : vb + (size_t)slice * 8192 + lane * 16;
    auto g = [](const char* a) -> uint4 {
        if constexpr (NTL) return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a)));
        else return *reinterpret_cast<const uint4*>(a);
    };
#pragma unroll
    for (int i = 0; i < 8; ++i) f.k[i] = g(k0 + i * 1024);
#pragma unroll
    for (int i = 0; i < 8; ++i) f.v[i] = g(v0 + i * 1024);
}
__device__ __forceinline__ uint32_t eat(const Frag& f) {
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) a ^= f.k[i].x ^ f.k[i].w ^ f.v[i].y ^ f.v[i].z;
    return a;
}
// same access shape moved by LDS-DMA (no consumer): every wave streams its slices 1 KB at a time into its own
// RING-slot LDS ring, RING-1 KB in flight; AUX 2 = nt, 0 = default policy
template <int RING, int AUX>
__global__ __launch_bounds__(256, 2) void k_att_dma(const char* K, const char* V, int ctx, size_t region, uint32_t* out) {
    extern __shared__ char smem[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int unit = blockIdx.x;
    const int nblk = (ctx + 127) / 128;
    const char* kb = K + unit * region;
    const char* vb = V + unit * region;
    char* ring = smem + w * RING * 1024;
    int n = 0;
    for (int b = 0; b < nblk; ++b) {
        const int slice = 4 * b + w;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const char* src = (i < 8 ? kb + (size_t)slice * 8192 + i * 1024 : vb + (size_t)slice * 8192 + (i - 8) * 1024) + lane * 16;
            __builtin_amdgcn_global_load_lds((const void*)src, (void*)(ring + (n % RING) * 1024), 16, 0, AUX);
            ++n;
            if (n >= RING - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RING - 2) : "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (reinterpret_cast<uint32_t*>(ring)[lane] == 0x12345678u) out[0] = 1;
}

template <bool ROT, bool ADJ, int SPLIT = 1, bool NTL = false>
__global__ __launch_bounds__(256, 2) void k_att(const char* K, const char* V, int ctx, size_t region, uint32_t* out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int unit = blockIdx.x / SPLIT, part = blockIdx.x % SPLIT;
    const int nblk_all = (ctx + 127) / 128;
    const int b0 = part * nblk_all / SPLIT, nblk = (part + 1) * nblk_all / SPLIT - b0;
    const char* kb = K + unit * region * (ADJ ? 2 : 1) + (size_t)b0 * (ADJ ? 65536 : 32768);
    const char* vb = V + unit * region + (size_t)b0 * 32768;
    if (nblk <= 0) return;
    const int rot = ROT ? (int)((blockIdx.x * 5u) % nblk) : 0;
    auto sl = [&](int b) { b = b < nblk ? b : nblk - 1; b += rot; b -= b >= nblk ? nblk : 0; return 4 * b + w; };
    Frag fa, fb;
    uint32_t acc = 0;
    ld<ADJ, NTL>(fa, kb, vb, sl(0), lane);
    for (int it = 0; it < nblk; it += 2) {
        ld<ADJ, NTL>(fb, kb, vb, sl(it + 1), lane);
        acc ^= eat(fa);
        ld<ADJ, NTL>(fa, kb, vb, sl(it + 2), lane);
        if (it + 1 < nblk) acc ^= eat(fb);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int att_probe(char* big, size_t total, uint32_t* out, hipEvent_t e0, hipEvent_t e1) {
    const size_t region = 3072 * 256;      // Smax 3072 keys x 256 B (K or V of one (row, kv head))
    const char* K = big;
    const char* V = big + 512 * region;
    for (int ctx : {512, 1705, 2999}) {
        const double bytes = 512.0 * ctx * 512;
        int grid_mult = 1;
        size_t lds = 0;
        auto go = [&](const char* name, auto kern) -> int {
            const int grid = 512 * (int)grid_mult;
            for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, K, V, ctx, region, out);
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, K, V, ctx, region, out);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / 50;
            printf("att %-8s ctx %5d : %7.2f us %6.0f GB/s\n", name, ctx, us, bytes / us / 1e3);
            return 0;
        };
        go("base", k_att<false, false>);
        go("base-nt", k_att<false, false, 1, true>);
        if (getenv("ATT_ALL")) {
            go("adj+rot", k_att<true, true>);
            grid_mult = 2; go("split2", k_att<false, false, 2>);
            grid_mult = 4; go("split4", k_att<false, false, 4>);
            grid_mult = 8; go("split8", k_att<false, false, 8>);
            grid_mult = 1;
        }
        lds = 4 * 8 * 1024; go("dma8-nt", k_att_dma<8, 2>);
        lds = 4 * 16 * 1024; go("dma16-nt", k_att_dma<16, 2>);
        go("dma16", k_att_dma<16, 0>);
        lds = 4 * 20 * 1024; go("dma20-nt", k_att_dma<20, 2>);
        lds = 0;
    }
    (void)total;
    return 0;
}

template <typename K>
int run(const char* name, K kern, int waves, int nch, size_t lds, std::vector<uint4*>& bufs, size_t bytes,
        uint32_t* out, hipEvent_t e0, hipEvent_t e1) {
    const int grid = (int)(bytes / ((size_t)waves * nch * 1024));
    if ((size_t)grid * waves * nch * 1024 != bytes) return 0;
    // consecutive launches read disjoint slices of a 768 MiB region (3x the Infinity Cache)
    const size_t nslots = ((size_t)bufs.size() << 26) / bytes;
    int reps = 120, warm = 10;
    auto launch = [&](int i) {
        const uint4* W = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(bufs[0]) + (i % nslots) * bytes);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), lds, 0, W, out);
    };
    for (int i = 0; i < warm; ++i) launch(i);
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) launch(i + warm);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    printf("%-5s %6.1f MB grid %4d waves/WG %2d chunks/wave %3d : %7.2f us %6.0f GB/s\n", name, bytes / 1e6, grid, waves,
           nch, us, bytes / us / 1e3);
    return 0;
}

int main() {
    // 64 MiB buffers, contiguous allocation so a launch spanning several reads one region
    const int NB = 14;    // 896 MiB (the attention probe reads 768 MiB of K/V)
    uint4* big;
    CK(hipMalloc(&big, (size_t)NB * (64ull << 20)));
    CK(hipMemset(big, 1, (size_t)NB * (64ull << 20)));
    std::vector<uint4*> bufs;
    for (int i = 0; i < NB; ++i) bufs.push_back(reinterpret_cast<uint4*>(reinterpret_cast<char*>(big) + ((size_t)i << 26)));
    uint32_t* out;
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    if (getenv("ATT")) return att_probe(reinterpret_cast<char*>(big), (size_t)NB << 26, out, e0, e1);
    const size_t sizes[] = {8ull << 20, 16ull << 20, 32ull << 20, 64ull << 20};
    for (size_t bytes : sizes) {
        printf("---- %zu MiB\n", bytes >> 20);
#define R(NCH, PF, WV) run("reg" #PF, k_reg<NCH, PF>, WV, NCH, 0, bufs, bytes, out, e0, e1)
        R(8, 4, 4); R(8, 8, 4); R(4, 4, 8); R(16, 4, 4); R(16, 8, 4); R(16, 16, 4); R(8, 8, 8); R(4, 4, 16);
        R(32, 4, 4); R(32, 8, 4); R(32, 16, 4); R(32, 32, 4); R(16, 16, 8); R(8, 8, 16);
        R(64, 4, 4); R(64, 8, 4); R(64, 16, 4); R(64, 32, 4); R(32, 16, 8); R(32, 32, 8); R(16, 16, 16);
        R(128, 16, 4); R(128, 32, 4); R(64, 32, 8); R(32, 32, 16); R(64, 16, 8);
#undef R
#define D(NCH, DEP, WV) run("dma" #DEP, k_dma<NCH, DEP>, WV, NCH, (size_t)WV * DEP * 1024, bufs, bytes, out, e0, e1)
        D(8, 8, 4); D(16, 16, 4); D(32, 16, 4); D(32, 32, 4); D(64, 32, 4); D(16, 16, 8); D(32, 16, 8); D(64, 16, 8);
        D(32, 8, 16); D(16, 8, 16); D(128, 32, 4);
#undef D
    }
    return 0;
}
