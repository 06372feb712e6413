// Weight-stream order probe (diagnostic, not part of the product). A B = 1 decode GEMV is a pure weight
// stream: 256 workgroups x 8 waves, each wave reading its own contiguous K range of the fragment-packed
// image (16 x 1 KB here, 8 loads in flight), so at entry every wave's first load sits at a multiple of
// 16 KB. Does the order in which the waves walk their ranges change how long the stream takes?
//   mode 0: every wave walks its range from the start (the product's order)
//   mode 1: wave (b, w) starts at piece (b * 8 + w) % 16 and wraps (same bytes, rotated start)
//   mode 2: pieces interleaved across waves (piece l of wave g at (l * nwaves + g) KB): at any time
//           all waves read neighbouring KBs
//   mode 4: interleaved across the waves of a workgroup only (piece l of wave w of workgroup b at
//           b * 128 KB + (l * 8 + w) KB): the k-step assignment a GEMV could change without a new layout
//   mode 5: mode 0 + the decode kernels' step word: a scalar load of a device word issued after the
//           prefetch and waited for (s_waitcnt lgkmcnt(0)) before the loop, as ld_word_here does
//   mode 3: mode 0 + the B = 1 fc2 GEMV's activation loads: per weight piece two 16-B-per-lane loads
//           of a 2 x 8192 bf16 activation (L2-resident; 16 lanes per row, so 2 distinct rows)
// Each launch reads a different copy of the image (LAYERS copies, far beyond L2 + MALL), as a decode
// step does; time per launch from hipEvents around LAYERS launches.
// Build: hipcc --offload-arch=gfx950 -O3 tools/stream_order_probe.hip -o tools/stream_order_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
constexpr int NWG = 256, NW = 8, NL = 16, PF = 8;

template <int MODE>
__global__ __launch_bounds__(64 * NW) void k_stream(const u32x4* __restrict__ img, u32x4* __restrict__ out,
                                                     unsigned long long* __restrict__ st, const uint16_t* __restrict__ act,
                                                     const int* skip) {
    const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, b = blockIdx.x;
    const int g = b * NW + w;                               // global wave
        auto piece = [&](int l) -> const u32x4* {               // 1 KB piece l (0..NL-1) of wave g
        long kb;
        if constexpr (MODE == 0 || MODE == 3 || MODE == 5) kb = (long)g * NL + l;
        else if constexpr (MODE == 1) kb = (long)g * NL + (l + g) % NL;
        else if constexpr (MODE == 4) kb = (long)b * NW * NL + l * NW + w;
        else kb = (long)l * (NWG * NW) + g;
        return img + kb * 64 + lane;
    };
    u32x4 r[PF], ra[PF][2];
    u32x4 acc = {0, 0, 0, 0};
    const int ln = lane & 15, lg = lane >> 4;
    const uint16_t* ap = act + (size_t)min(ln, 1) * 8192 + w * 1024 + lg * 8;
    auto aload = [&](int l, int q) { return *reinterpret_cast<const u32x4*>(ap + (l * 2 + q) * 32); };
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        r[p] = __builtin_nontemporal_load(piece(p));
        if constexpr (MODE == 3) { ra[p][0] = aload(p, 0); ra[p][1] = aload(p, 1); }
    }
    unsigned long long t_first = 0, t_skip = 0;
    if constexpr (MODE == 5) {
        int skv;
        asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(skv) : "s"(skip) : "memory");
        t_skip = __builtin_amdgcn_s_memrealtime();
        if (skv) {
#pragma unroll
            for (int p = 0; p < PF; ++p) asm volatile("" ::"v"(r[p].x), "v"(r[p].y), "v"(r[p].z), "v"(r[p].w));
            return;
        }
    }
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        const u32x4 v = r[l % PF];
        if (l == 0) {
            asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PF - 1) : "memory");
            t_first = __builtin_amdgcn_s_memrealtime();
        }
        if constexpr (MODE == 3) acc ^= ra[l % PF][0] ^ ra[l % PF][1];
        if (l + PF < NL) {
            r[l % PF] = __builtin_nontemporal_load(piece(l + PF));
            if constexpr (MODE == 3) { ra[l % PF][0] = aload(l + PF, 0); ra[l % PF][1] = aload(l + PF, 1); }
        }
        acc ^= v;
    }
    if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) out[threadIdx.x] = acc;   // never true
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    if (st && lane == 0) {
        st[(size_t)g * 4 + 0] = t_entry;
        st[(size_t)g * 4 + 1] = t_first;
        st[(size_t)g * 4 + 2] = t_end;
        st[(size_t)g * 4 + 3] = t_skip;
    }
}

int main(int argc, char** argv) {
    const int layers = 26, reps = 20;
    const size_t img_bytes = (size_t)NWG * NW * NL * 1024;             // 33.5 MB: the c2 fc2 image
    char* buf;
    u32x4* out;
    uint16_t* act;
    int* skipw;
    CK(hipMalloc(&skipw, 256));
    CK(hipMemset(skipw, 0, 256));
    CK(hipMalloc(&act, 2 * 8192 * 2));
    CK(hipMemset(act, 3, 2 * 8192 * 2));
    CK(hipMalloc(&buf, img_bytes * layers));
    CK(hipMalloc(&out, 64 * NW * 16));
    CK(hipMemset(buf, 1, img_bytes * layers));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](int mode) -> float {
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r)
            for (int L = 0; L < layers; ++L) {
                const u32x4* img = reinterpret_cast<const u32x4*>(buf + (size_t)L * img_bytes);
                if (mode == 0) hipLaunchKernelGGL(k_stream<0>, dim3(NWG), dim3(64 * NW), 0, 0, img, out, (unsigned long long*)nullptr, act, skipw);
                else if (mode == 1) hipLaunchKernelGGL(k_stream<1>, dim3(NWG), dim3(64 * NW), 0, 0, img, out, (unsigned long long*)nullptr, act, skipw);
                else if (mode == 2) hipLaunchKernelGGL(k_stream<2>, dim3(NWG), dim3(64 * NW), 0, 0, img, out, (unsigned long long*)nullptr, act, skipw);
                else if (mode == 3) hipLaunchKernelGGL(k_stream<3>, dim3(NWG), dim3(64 * NW), 0, 0, img, out, (unsigned long long*)nullptr, act, skipw);
                else if (mode == 4) hipLaunchKernelGGL(k_stream<4>, dim3(NWG), dim3(64 * NW), 0, 0, img, out, (unsigned long long*)nullptr, act, skipw);
                else hipLaunchKernelGGL(k_stream<5>, dim3(NWG), dim3(64 * NW), 0, 0, img, out, (unsigned long long*)nullptr, act, skipw);
            }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms * 1000.f / (reps * layers);
    };
    for (int m = 0; m < 6; ++m) run(m);                                  // warm-up
    const char* names[6] = {"0 contiguous (product order)", "1 rotated start", "2 interleaved across waves", "3 mode 0 + activation loads", "4 interleaved within a workgroup", "5 mode 0 + step word"};
    printf("# %d workgroups x %d waves x %d KB, %d loads in flight per wave, %d image copies of %.1f MB (us per launch, back to back)\n",
           NWG, NW, NL, PF, layers, img_bytes / 1e6);
    for (int round = 0; round < 3; ++round)
        for (int m = 0; m < 6; ++m) {
            const float us = run(m);
            printf("mode %-30s %7.2f us  %6.2f TB/s\n", names[m], us, img_bytes / us / 1e6);
        }
    // stamps: one launch of mode 0 / 3 / 5 after 25 launches on the other copies (the last of a "step")
    unsigned long long* st;
    CK(hipMalloc(&st, sizeof(unsigned long long) * NWG * NW * 4));
    for (int trial = 0; trial < 6; ++trial) {
        const int mm = trial % 3 == 0 ? 0 : (trial % 3 == 1 ? 3 : 5);
        for (int L = 0; L < layers - 1; ++L)
            hipLaunchKernelGGL(k_stream<0>, dim3(NWG), dim3(64 * NW), 0, 0,
                               reinterpret_cast<const u32x4*>(buf + (size_t)L * img_bytes), out, (unsigned long long*)nullptr, act, skipw);
        const u32x4* lastimg = reinterpret_cast<const u32x4*>(buf + (size_t)(layers - 1) * img_bytes);
        if (mm == 3) hipLaunchKernelGGL(k_stream<3>, dim3(NWG), dim3(64 * NW), 0, 0, lastimg, out, st, act, skipw);
        else if (mm == 5) hipLaunchKernelGGL(k_stream<5>, dim3(NWG), dim3(64 * NW), 0, 0, lastimg, out, st, act, skipw);
        else hipLaunchKernelGGL(k_stream<0>, dim3(NWG), dim3(64 * NW), 0, 0, lastimg, out, st, act, skipw);
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> h((size_t)NWG * NW * 4);
        CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull;
        for (int g = 0; g < NWG * NW; ++g) t0 = std::min(t0, h[(size_t)g * 4]);
        std::vector<double> ent, fst, end, skp;
        for (int g = 0; g < NWG * NW; ++g) {
            ent.push_back((h[(size_t)g * 4] - t0) * 0.01);
            fst.push_back((h[(size_t)g * 4 + 1] - t0) * 0.01);
            end.push_back((h[(size_t)g * 4 + 2] - t0) * 0.01);
            skp.push_back(mm == 5 ? (h[(size_t)g * 4 + 3] - t0) * 0.01 : 0.0);
        }
        auto q = [](std::vector<double> v, double f) { std::sort(v.begin(), v.end()); return v[(size_t)(f * (v.size() - 1))]; };
        printf("mode %d stamps (us from the first wave's entry): entry p50 %.2f max %.2f | step word back p50 %.2f max %.2f | first load back p10 %.2f p50 %.2f p90 %.2f max %.2f | end p10 %.2f p50 %.2f max %.2f\n",
               mm, q(ent, 0.5), q(ent, 1.0), q(skp, 0.5), q(skp, 1.0), q(fst, 0.1), q(fst, 0.5), q(fst, 0.9), q(fst, 1.0), q(end, 0.1), q(end, 0.5), q(end, 1.0));
    }
    return 0;
}
