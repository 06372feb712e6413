// Address-translation probe (diagnostic, not part of the product): how much of a decode kernel's
// first-load latency is the translation of a page the chip has not touched since a multi-GB weight
// stream went through? One lane issues dependent single-dword loads and times each with s_memtime
// (core clock) after a vmcnt(0) wait:
//   cold page + cold line, then lines at +4 KB / +64 KB / +1 MB / +2 MB / +8 MB of it (translation
//   possibly warm, lines cold), then the first address again (L2 hit).
// Between rounds a streaming kernel reads STREAM_GB of another buffer (evicts L2, MALL and TLBs).
// Build: hipcc --offload-arch=gfx950 -O3 tools/tlb_probe.hip -o tools/tlb_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int NPROBE = 9;

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
__global__ void k_stream(const u32x4* __restrict__ p, size_t n, u32x4* sink) {
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) sink[threadIdx.x] = acc;   // never true: keeps the loads
}

// offsets in bytes from base, probed in order by lane 0 of one wave
__global__ void k_probe(const char* base, const long* offs, long long* out) {
    if (threadIdx.x != 0) return;
    int dep = 0;
    for (int i = 0; i < NPROBE; ++i) {
        const int* p = reinterpret_cast<const int*>(base + offs[i] + (dep & 0));
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        const long long t0 = __builtin_amdgcn_s_memtime();
        const long long r0 = __builtin_amdgcn_s_memrealtime();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int v = __builtin_nontemporal_load(p);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        dep += v;
        const long long t1 = __builtin_amdgcn_s_memtime();
        const long long r1 = __builtin_amdgcn_s_memrealtime();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        out[i] = t1 - t0;
        out[NPROBE + 1 + i] = (r1 - r0) * 10;      // ns (100 MHz constant clock)
    }
    out[2 * NPROBE + 1] = dep;
}

int main(int argc, char** argv) {
    const size_t stream_gb = argc > 1 ? atoi(argv[1]) : 4;
    const size_t probe_bytes = (size_t)1 << 30;          // 1 GB probe region, a fresh 64 MB window per round
    const size_t sbytes = stream_gb << 30;
    char *probe, *stream;
    long* d_offs;
    long long* d_out;
    u32x4* sink;
    CK(hipMalloc(&probe, probe_bytes));
    CK(hipMalloc(&stream, sbytes));
    CK(hipMalloc(&d_offs, sizeof(long) * NPROBE));
    CK(hipMalloc(&d_out, sizeof(long long) * (2 * NPROBE + 2)));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(probe, 1, probe_bytes));
    CK(hipMemset(stream, 2, sbytes));
    CK(hipDeviceSynchronize());
    const char* names[NPROBE] = {"cold page", "+4 KB", "+64 KB", "+1 MB", "+2 MB", "+8 MB", "+32 MB", "+2 MB again(+256B)", "first again"};
    const long rel[NPROBE] = {0, 4096, 65536, 1 << 20, 2 << 20, 8 << 20, 32 << 20, (2 << 20) + 256, 0};
    std::vector<std::vector<long long>> res(NPROBE), resn(NPROBE);
    const int rounds = 12;
    for (int r = 0; r < rounds; ++r) {
        hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, (const u32x4*)stream, sbytes / 16, sink);
        long offs[NPROBE];
        const long base = ((long)(r % 15) * (64L << 20)) + 128 * 1024 + 64;   // a window untouched since the memset
        for (int i = 0; i < NPROBE; ++i) offs[i] = base + rel[i];
        CK(hipMemcpy(d_offs, offs, sizeof(offs), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, (const u32x4*)stream, sbytes / 16, sink);
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, probe, d_offs, d_out);
        long long h[2 * NPROBE + 2];
        CK(hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost));
        if (r >= 2)
            for (int i = 0; i < NPROBE; ++i) { res[i].push_back(h[i]); resn[i].push_back(h[NPROBE + 1 + i]); }
    }
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    printf("# s_memtime cycles per dependent single-dword load (median / min / max over %zu rounds), after a %zu GB stream; clock attr %d kHz\n",
           res[0].size(), stream_gb, clk);
    for (int i = 0; i < NPROBE; ++i) {
        std::vector<long long> v = res[i];
        std::vector<long long> w = resn[i];
        std::sort(v.begin(), v.end());
        std::sort(w.begin(), w.end());
        printf("%-22s cycles median %6lld  min %6lld  max %6lld   |  ns median %6lld  min %6lld  max %6lld\n", names[i],
               v[v.size() / 2], v.front(), v.back(), w[w.size() / 2], w.front(), w.back());
    }
    return 0;
}
