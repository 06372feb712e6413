// L2 warm-up of the next decode GEMM's first weight chunks (internal to the library).
//
// A k_gemm_ws launch is short (5-18 us at c3) and starts cold: every compute wave's first
// weight chunks come from HBM before its first MFMA. The kernel that runs just before it
// (k_resid_ln before in_proj / fc1, the fc1 GEMM before fc2) reads those chunks into the
// L2 of the XCD the GEMM workgroup will run on, from a wave that has nothing else to do, so
// the GEMM starts on L2 hits (tools/microbench.py warm). Results are
// unchanged: the warm-up only loads.
#pragma once
#include <stdint.h>

struct ZkWarm {
    const void* W;     // packed weights of the GEMM to warm (nullptr: off)
    int K;             // GEMM K
    int gx, gz;        // its k_gemm_ws grid (column tiles, K splits)
    int chunks;        // 64-deep chunks per compute wave to warm | column groups per wave (NG) << 8
};

// k_gemm_ws grid of zk_gemm_bf16(M, N, K, nsplit, mode) in the decode regime, or W = nullptr
ZkWarm zk_gemm_warm_desc(const void* W, int M, int N, int K, int nsplit, int mode, int chunks);

int zk_resid_ln_warm(const float* part, int nsplit, const void* x_in, const void* w, const void* b, float eps,
                     int rows, int D, void* x_out, void* xn_out, int ln_on_sum, const int32_t* skip, ZkWarm warm,
                     void* stream);
int zk_gemm_bf16_warm(const void* A, long lda, const void* W, int M, int N, int K, int nsplit, int mode, float* Cpart,
                      void* Cout, const int32_t* skip_flag, ZkWarm warm, void* stream);
