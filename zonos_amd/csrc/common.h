// Shared device helpers for the Zonos MI355X (gfx950) kernels.
// Wave = 64 lanes everywhere; all reductions are written for wave64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ZK_DEV __device__ __forceinline__

typedef uint16_t bf16_t;   // raw bf16 bits (torch.bfloat16 storage)
typedef uint16_t f16_t;

// ---------------------------------------------------------------- device step words
// A nullable device int32 (skip / context / offset words) read without a branch and as a VECTOR
// load (relaxed atomic: never scalarised), issued before the kernel's data loads: vmcnt retires in
// issue order, so the test of the word waits for it alone, where a scalar load's wait (lgkmcnt(0),
// scalar loads return out of order) would also hold every later kernel-argument load. Each lane
// holds the same value; callers take it with readfirstlane where they branch or index on it.
static __device__ int32_t zk_zero_word = 0;    // never written; not const, so the load is not folded
ZK_DEV int32_t ld_word(const int32_t* p) {
    return __hip_atomic_load(p != nullptr ? p : &zk_zero_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
ZK_DEV int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// The same word by a scalar load issued exactly here (inline asm: hipcc can neither hoist it above
// the loads before it nor turn it into a vector load) and waited for at once.
ZK_DEV int32_t ld_word_here(const int32_t* p) {
    const int32_t* q = p != nullptr ? p : &zk_zero_word;
    int32_t v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(q) : "memory");
    return v;
}
// Two step words by scalar loads issued here and waited for together (one round trip).
ZK_DEV void ld_words_here(const int32_t* p0, const int32_t* p1, int32_t& v0, int32_t& v1) {
    const int32_t* q0 = p0 != nullptr ? p0 : &zk_zero_word;
    const int32_t* q1 = p1 != nullptr ? p1 : &zk_zero_word;
    asm volatile("s_load_dword %0, %2, 0x0\n\ts_load_dword %1, %3, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(v0), "=&s"(v1)
                 : "s"(q0), "s"(q1)
                 : "memory");
}
// Use of loaded registers on a kernel's early-exit path: without a use there, hipcc sinks the
// loads into the path that consumes them, i.e. below the exit test, which then waits for the
// step word before the first data load is issued.
ZK_DEV void keep_live(const uint4& v) { asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w)); }
ZK_DEV void keep_live(const uint2& v) { asm volatile("" ::"v"(v.x), "v"(v.y)); }
ZK_DEV void keep_live(const float4& v) { asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w)); }

// ---------------------------------------------------------------- bf16 <-> f32
// Round-to-nearest-even exactly like torch's float->bfloat16 conversion (c10/util/BFloat16.h),
// NaN kept as a quiet NaN.
ZK_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
ZK_DEV bf16_t f2bf(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (bf16_t)0x7fc0;
    u += 0x7fffu + ((u >> 16) & 1u);
    return (bf16_t)(u >> 16);
}
ZK_DEV float round_bf(float f) { return bf2f(f2bf(f)); }

// Unpack 8 bf16 held in a uint4 (16 B) to floats.
ZK_DEV void unpack8(const uint4 v, float* f) {
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
    f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
    f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
ZK_DEV uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }
ZK_DEV uint4 pack8(const float* f) {
    return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// ---------------------------------------------------------------- decode GEMM tile order
#ifndef ZK_WS_XCD
#define ZK_WS_XCD 1                // k_gemm_ws: XCD-aware split-major tile order
#endif
// Tile (bx, bz) of linear workgroup id L (= blockIdx.x + gx * blockIdx.z) of a k_gemm_ws grid
// gx x 1 x gz. XCD-aware order: workgroups are dispatched round-robin over the 8 XCDs (L % 8),
// and every workgroup of one K split reads the same activation slice. Numbering the work
// split-major and handing each XCD a contiguous run of it puts one split (fc2: 8 splits) or half a
// split (in_proj / out_proj: 4) on each XCD, so its L2 fetches only that K slice of the activation
// instead of all of it. Placement only: every tile computes the same numbers.
ZK_DEV void ws_tile(int L, int gx, int gz, int& bx, int& bz) {
    if (ZK_WS_XCD && gz > 1 && ((gx * gz) & 7) == 0) {
        const int I = (L & 7) * ((gx * gz) >> 3) + (L >> 3);
        bz = I / gx;
        bx = I - bz * gx;
    } else {
        bz = L / gx;
        bx = L - bz * gx;
    }
}

// L2 warm-up (warm.h): compute wave w of k_gemm_ws workgroup L starts by streaming its first
// `chunks` 2 KB chunks of fragment-packed weights ([N/16][K/32][64 lanes][8]: 16 rows x 64 k =
// 2 KB). Issue them as LDS-DMA (default cache policy, so the lines stay in this XCD's L2) into a
// 1 KB LDS sink the issuing wave never reads: no registers, nothing for the other waves to wait on.
// Returns the number of loads issued (2 per chunk).
// `chunks` packs the GEMM's column groups per compute wave (k_gemm_ws NG) in bits 8+: wave w of
// workgroup (bx, bz) streams the 16-row tiles (bx * 4 + w) * NG + g, g < NG.
// chunks: bits 0-7 chunks per wave, 8-15 column groups per wave (NG, 0 = 1), 16-23 compute waves per
// workgroup of the warmed GEMM (0 = 4), 24-31 trailing 16-column tiles of its grid wholly past N
// (the packed image holds ceil(N / 16) tiles, padded to 64 columns; a 48-column grid can overshoot
// even that -- c5 Mamba in_proj: 178 x 3 = 534 tiles for a 532-tile image -- so those are skipped)
ZK_DEV int warm_nw(int chunks) { return ((chunks >> 16) & 255) ? ((chunks >> 16) & 255) : 4; }
ZK_DEV int warm_unit(const bf16_t* W, int K, int gx, int gz, int chunks, int L, int w, int lane, void* sink) {
    int bx, bz;
    ws_tile(L, gx, gz, bx, bz);
    const int ng = max(1, (chunks >> 8) & 255), nch = chunks & 255, nw = warm_nw(chunks);
    const int ntiles = gx * nw * ng - ((chunks >> 24) & 255);      // 16-column tiles holding a column < N
    const int kbeg = bz * (K / gz);
    for (int g = 0; g < ng; ++g) {
        const int tile = (bx * nw + w) * ng + g;
        if (tile >= ntiles) break;
        const bf16_t* p = W + ((size_t)tile * (K >> 5) + (kbeg >> 5)) * 512 + lane * 8;
        for (int c = 0; c < nch; ++c) {
            __builtin_amdgcn_global_load_lds((const void*)(p + c * 1024), sink, 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void*)(p + c * 1024 + 512), sink, 16, 0, 0);
        }
    }
    return 0;
}

// All warm-up units of workgroup r of an nwg-workgroup launch (nwg % 8 == 0 keeps the GEMM
// workgroups L = r, r + nwg, ... on r's XCD), unit u = (GEMM workgroup, compute wave), this wave
// taking units first, first + step, ...
ZK_DEV void warm_units(const bf16_t* W, int K, int gx, int gz, int chunks, int r, int nwg, int first, int step,
                       int lane, void* sink) {
    const int nw = warm_nw(chunks);
    for (int u = first;; u += step) {
        const int L = r + (u / nw) * nwg;
        if (L >= gx * gz) break;
        warm_unit(W, K, gx, gz, chunks, L, u % nw, lane, sink);
    }
}

// ---------------------------------------------------------------- wave64 reductions
ZK_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
ZK_DEV double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
ZK_DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Block-wide reductions for blocks of NT threads (NT multiple of 64, <= 1024).
// `red` is NT/64 floats of LDS scratch. All threads receive the result.
template <int NT>
ZK_DEV float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    return t;
}
template <int NT>
ZK_DEV float block_max(float v, float* red) {
    v = wave_max(v);
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float t = red[0];
#pragma unroll
    for (int i = 1; i < NT / 64; ++i) t = fmaxf(t, red[i]);
    return t;
}

// ---------------------------------------------------------------- DPP reductions
// DPP row rotation (within each 16-lane row) of a 32-bit value
template <int R>
ZK_DEV float row_ror(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xF, 0xF, false));
}
template <int R>
ZK_DEV uint4 row_ror4(uint4 v) {
    uint4 o;
    o.x = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.x, 0x120 + R, 0xF, 0xF, false);
    o.y = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.y, 0x120 + R, 0xF, 0xF, false);
    o.z = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.z, 0x120 + R, 0xF, 0xF, false);
    o.w = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.w, 0x120 + R, 0xF, 0xF, false);
    return o;
}
// wave64 sum without LDS permutes: rotations inside each 16-lane row, then the 4 row sums
// (read lanes 0, 16, 32, 48) added in row order. Every lane gets the same value.
ZK_DEV float wave_sum_dpp(float v) {
    v += row_ror<8>(v);
    v += row_ror<4>(v);
    v += row_ror<2>(v);
    v += row_ror<1>(v);
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return ((r0 + r1) + r2) + r3;
}

// ---------------------------------------------------------------- host-side error plumbing
#ifdef __cplusplus
extern "C" void zk_set_error(const char* fmt, ...);
#endif
#define ZK_CHECK_LAUNCH(name)                                                  \
    do {                                                                       \
        hipError_t _e = hipGetLastError();                                     \
        if (_e != hipSuccess) {                                                \
            zk_set_error("%s: launch failed: %s", name, hipGetErrorString(_e)); \
            return -1;                                                         \
        }                                                                      \
    } while (0)
#define ZK_REQUIRE(cond, ...)           \
    do {                                \
        if (!(cond)) {                  \
            zk_set_error(__VA_ARGS__);  \
            return -2;                  \
        }                               \
    } while (0)
// a HIP runtime call that must succeed (host code returning int status)
#define ZK_HIP(call)                                                                   \
    do {                                                                               \
        hipError_t _e = (call);                                                        \
        if (_e != hipSuccess) {                                                        \
            zk_set_error("%s failed: %s", #call, hipGetErrorString(_e));               \
            return -1;                                                                 \
        }                                                                              \
    } while (0)
// propagate a nonzero status of an internal host helper
#define ZK_TRY(expr)                \
    do {                            \
        const int _rc = (expr);     \
        if (_rc != 0) return _rc;   \
    } while (0)
