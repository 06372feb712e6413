// DAC decoder, channels-last fp16 pipeline (the default "fp16" precision: the numerics of the
// reference's own GPU path, torch.autocast fp16 around DacModel.decode, autoencoder.py:46 --
// fp16 conv operands, fp32 accumulation; here the residual stream additionally stays fp32).
//
// Layout: every conv reads s = fp16(Snake(x)) as [B][T][C] (channels-last, C padded to a
// multiple of 32 with zero channels) and its epilogue applies the NEXT Snake, so the conv
// main loop is pure data movement + MFMA:
//   conv7(res unit)   : s' = Snake_a2(conv + b)                      (fp16 out only)
//   conv1(res unit)   : x  = x + conv + b ; s = Snake_next(x)         (fp32 x + fp16 s)
//   ConvTranspose1d   : x  = conv + b     ; s = Snake_res1(x)         (s polyphase 2-tap convs)
//   first conv        : s = Snake_block0(conv + b)
// (modeling_dac.py:95-100 Snake, :222-233 residual unit, :266-278 decoder block, :420-439).
//
// Implicit GEMM on v_mfma_f32_16x16x32_f16: M = output channels, N = positions, K = (tap,
// input channel). Workgroup tile CO_T = 32*FM channels x QT = 32*NQ positions (128, or 256 for
// the convs without a residual: twice the positions per prologue / barrier / epilogue), 4 waves
// as 2x2, each wave (16*FM) x (16*NQ). K is walked as steps (channel chunk c of CI, tap t): per chunk the
// input window (QT + (ks-1)*dil positions x CI channels) is staged once and reused by all
// taps (tap t reads rows shifted by t*dil); the (tap, chunk) weight slice is staged per step.
// Both images land in LDS by LDS-DMA (global_load_lds_dwordx4, lane-linear destination, XOR
// swizzle of the 16-B channel groups applied on the source address); out-of-range positions
// read a zero page, which is the conv's zero padding AND the per-row length masking of a
// ragged batch. A dedicated loader wave keeps several weight slices and windows in flight
// (LDS rings, counted vmcnt, one raw s_barrier per step); the 4 compute waves never load.
#include "common.h"
#include "../../include/zonos_hip.h"
#include <algorithm>
#include <stdlib.h>

namespace {

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int QT = 128;          // positions per workgroup (NQ = 4)
constexpr int MAXSPAN = 64;      // max (ks-1)*dil

__device__ __attribute__((aligned(256))) uint4 g_zero_page[16];   // 256 zero bytes (LDS-DMA source for padding)

template <int CI>
struct Img {                      // [rows][CI fp16] image, 16-B groups XOR-swizzled per 256-B bank row
    static constexpr int G = CI / 8;
    static constexpr int RB = CI * 2;
    static constexpr int RPB = 256 / RB;
    static constexpr int RPR = 4096 / RB;        // rows per load round (256 lanes x 16 B)
    ZK_DEV static int swz(int row) { return (int)(((unsigned)row / RPB) % G); }
    ZK_DEV static int off(int row, int g) { return row * RB + ((g ^ swz(row)) << 4); }
};

ZK_DEV f16x8 as_h8(uint4 v) { return __builtin_bit_cast(f16x8, v); }
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
ZK_DEV f16x4 as_h4(uint2 v) { return __builtin_bit_cast(f16x4, v); }

ZK_DEV float snake(float x, float a) {     // x + 1/(a + 1e-9) * sin(a x)^2   (modeling_dac.py:95-100)
    const float s = sinf(__fmul_rn(a, x));
    return __fadd_rn(x, __fmul_rn(__fdiv_rn(1.0f, __fadd_rn(a, 1e-9f)), __fmul_rn(s, s)));
}

// fp16-output Snake: hardware sine (abs. error ~1e-6 at these arguments, far below the fp16
// rounding of the result) and a per-channel reciprocal.
ZK_DEV float snake_fast(float x, float a, float ra) {
    const float s = __sinf(a * x);
    return fmaf(ra, s * s, x);
}

ZK_DEV uint2 pack_h4(float a, float b, float c, float d) {
    _Float16 h[4] = {(_Float16)a, (_Float16)b, (_Float16)c, (_Float16)d};
    return *reinterpret_cast<const uint2*>(h);
}

// s_waitcnt vmcnt(n) for a runtime n (clamped to the 6-bit field): a jump table of immediates.
ZK_DEV void wait_vm(int n) {
#define ZK_W1(N_) case N_: asm volatile("s_waitcnt vmcnt(" #N_ ")" ::: "memory"); break;
#define ZK_W8(B_) ZK_W1(B_ + 0) ZK_W1(B_ + 1) ZK_W1(B_ + 2) ZK_W1(B_ + 3) ZK_W1(B_ + 4) ZK_W1(B_ + 5) ZK_W1(B_ + 6) ZK_W1(B_ + 7)
    switch (n < 0 ? 0 : (n > 63 ? 63 : n)) {
        ZK_W8(0) ZK_W8(8) ZK_W8(16) ZK_W8(24) ZK_W8(32) ZK_W8(40) ZK_W8(48) ZK_W8(56)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef ZK_W8
#undef ZK_W1
}

#ifndef ZK_CL_DA
#define ZK_CL_DA 3
#endif
#ifdef ZK_CL_PROF                  // diagnostic builds only: per-step s_memtime stamps of 64 workgroups
__device__ uint64_t g_clprof[64][3][64];   // [wg][0: loader before wait, 1: loader after barrier, 2: compute after barrier][step]
__device__ uint64_t g_clprof_end[64][2];   // compute wave: after the MFMAs of the last step, at the end
__device__ uint64_t g_clprof_rt[64][6];    // wave 0: realtime at start, first barrier, loop end, epilogue end; memtime at start, end
__device__ uint64_t g_clwg[4096][2];       // every workgroup < 4096: realtime at start / end of wave 0
__device__ uint32_t g_clhw[4096][8];       // every workgroup < 4096: HW_ID of waves 0-5, XCC_ID
#define ZK_CL_STAMP(role, st)                                                                          \
    do {                                                                                               \
        if (blockIdx.x < 64 && (st) < 64 && lane == 0) g_clprof[blockIdx.x][role][st] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define ZK_CL_STAMP(role, st) do { } while (0)
#endif
#ifndef ZK_CL_DIAG_NOW             // diagnostic builds only: weight slices loaded once (stale data)
#define ZK_CL_DIAG_NOW 0
#endif
#ifndef ZK_CL_DIAG_NOMFMA          // diagnostic builds only: no MFMAs (wrong results)
#define ZK_CL_DIAG_NOMFMA 0
#endif
constexpr int CL_DA = ZK_CL_DA;          // weight slices in flight ahead of the step being computed
constexpr int CL_NW = CL_DA + 2;         // weight ring slots
#ifndef ZK_CL_NLD
#define ZK_CL_NLD 2
#endif
constexpr int CL_NLD = ZK_CL_NLD;        // loader waves (LDS-DMA issue is the per-step limit with one)
constexpr int CL_THREADS = 256 + 64 * CL_NLD;   // 4 compute waves + the loaders

// Loader-wave implicit GEMM, persistent. Waves 4.. only move bytes (LDS-DMA) and count their own
// vmcnt; waves 0-3 only read LDS + MFMA, so the vmcnt(0) that hipcc places before their ds_reads
// (it cannot tell the DMA's LDS range) costs nothing -- they have no loads in flight.
// Step i = (chunk c, tap t); the loader runs CL_DA steps ahead for weights and DX steps
// ahead for windows (DX >= CL_DA, window ring of NX slots), one raw s_barrier per step.
// Persistent: the grid holds as many workgroups as are resident at once (2 per CU), and each walks
// its share of the (row, position tile, channel tile) tiles as ONE step stream: the loaders run
// into the next tile while the compute waves store this one, and no workgroup waits to be
// dispatched (a one-tile-per-workgroup grid kept 58 % of the slots busy: the dispatcher waits for
// a free slot on the XCD the next workgroup id is bound to).
// DA: weight slices the loader keeps in flight (ring of DA + 2 slots); OCC: workgroups per CU the
// registers are sized for
// NWY: position waves (2 compute waves per position range: the two channel halves), NLDK loader
// waves: 2 x NWY + NLDK waves per workgroup.
// SPB: steps published per barrier -- the compute waves multiply SPB (tap, chunk) steps between two
// barriers (a step is only FM x NQ MFMAs per wave, so a barrier per step holds the waves at the
// barrier and the LDS read restart for a large share of the step); the rings hold 2 (SPB - 1) more
// weight slots and the window ring ceil((DX + 2 SPB - 1) / ks) + 1 slots.
#ifndef ZK_CL_SPB
#define ZK_CL_SPB 1
#endif
constexpr int CL_SPB = ZK_CL_SPB;
#ifndef ZK_RU_XPD
#define ZK_RU_XPD 4                  // fused unit: residual output blocks in flight in the epilogue
#endif
// NWM: channel waves (2: the two channel halves; 1: every wave holds all CO_T channels of its
// positions). FUSE (NWM = 1, one channel tile = all C channels): a whole residual unit in one
// launch -- the k7 conv's accumulators, Snake'd to fp16, are already the B operands of
// v_mfma_f32_16x16x16_f16 (lane (p, g) holds channels 4g..4g+3 of position p), so the 1x1 conv
// multiplies them in registers against the C x C weights staged once in LDS, adds the residual
// and writes x and the next Snake: the fp16 intermediate never goes to HBM (4 of the unit's 16 B
// per element) and the 1x1 conv's launch, rings and barriers are gone.
template <int FM, bool SF32, bool RES, int NQ, int DA = CL_DA, int OCC = 2, int NWY = 2, int NLDK = CL_NLD,
          int SPB = CL_SPB, int NWM = 2, bool FUSE = false>
#ifndef ZK_CL_LBW
#define ZK_CL_LBW(OCC_, NT_) ((OCC_ * (NT_) + 255) / 256)
#endif
__global__ __launch_bounds__(64 * (NWM * NWY + NLDK), ZK_CL_LBW(OCC, 64 * (NWM * NWY + NLDK))) void k_conv_cl(
    const uint16_t* __restrict__ in, int Cin, int Tin, const uint16_t* __restrict__ w, long wphase,
    const float* __restrict__ bias, int Cout, int ks, int dil, int pad, int Qn, int nphase, int out_stride,
    int out_off0, int Tout, const float* resid, float* xout, const float* __restrict__ alpha,
    void* __restrict__ sout, int s_f32, const int32_t* __restrict__ lens, int in_scale, int out_scale, int nq,
    int nx_slots, int dx, int B, const uint16_t* __restrict__ w1x1, const float* __restrict__ b1x1,
    const float* __restrict__ alpha_out) {
    constexpr int CI = 32;
    using I = Img<CI>;
    constexpr int CO_T = 16 * FM * NWM;
    constexpr int WS = CO_T * I::RB;             // weight slot bytes
    constexpr int NWP = CO_T / 16;               // weight pieces (1 KiB = 16 rows) per step
    constexpr int NCW = NWM * NWY;               // compute waves
    static_assert(!FUSE || (NWM == 1 && !RES), "fused residual unit: one channel wave, residual in the epilogue");
    constexpr int W1S = CO_T + 8;                // fused: 1x1 weight image row stride (halves)
    // fused: the 1x1 weights as an LDS image when one workgroup per CU has room for it (C = 96), else
    // read per output block from L1 / L2, one block ahead
    constexpr bool W1LDS = FUSE && OCC == 1 && CO_T * W1S * 2 <= 24 * 1024;
    constexpr int QTT = 16 * NQ * NWY;           // positions per tile
    extern __shared__ __attribute__((aligned(16))) char smem[];   // [W ring][X ring][epilogue tables x 2]

    // Tiles: XCD x (= blockIdx.x % 8 under round-robin dispatch) owns the contiguous range [lo, hi)
    // of the tile order (channel tile fastest, then position tile, then row), and its
    // gridDim.x / 8 workgroups stride through it, so the co-tiles of one window run side by side
    // on one XCD and re-read the window from its L2 rather than from HBM.
    const int nco = (Cout / CO_T) * nphase;
    const int ntiles = B * nq * nco;
    const int kx = blockIdx.x >> 3, nper = gridDim.x >> 3;
    const int lo = (int)((long)(blockIdx.x & 7) * ntiles / 8), hi = (int)((long)((blockIdx.x & 7) + 1) * ntiles / 8);
    const int nt = hi - lo > kx ? (hi - lo - kx + nper - 1) / nper : 0;
    auto tile_of = [&](int i, int& b, int& phase, int& co0, int& q0) {
        const int L = lo + kx + i * nper;
        const int cot = L % nco;
        b = L / (nco * nq);
        q0 = ((L / nco) % nq) * QTT;
        phase = cot % nphase;
        co0 = (cot / nphase) * CO_T;
    };

    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int win = QTT + (ks - 1) * dil;
    const int nxp = (win + 15) >> 4;             // window pieces (16 rows each)
    const int XS = nxp * 1024;
    // weight ring slots: the loader refills a slot at most 2 SPB steps after the barrier that let it
    // run (it can be SPB steps ahead of the barrier it passed, the compute waves SPB behind it)
    constexpr int NWS = DA + 2 * SPB;
    char* const wring = smem;
    char* const xring = smem + NWS * WS;
    const int nchunk = Cin / CI, nstep = nchunk * ks;

#ifdef ZK_CL_PROF
    if (blockIdx.x < 4096 && lane == 0 && wv < 6) {
        g_clhw[blockIdx.x][wv] = __builtin_amdgcn_s_getreg((31 << 11) | 4);           // HW_REG_HW_ID
        if (wv == 0) g_clhw[blockIdx.x][6] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
    }
    if (wv == 0 && blockIdx.x < 4096 && lane == 0) g_clwg[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
    if (wv == 0 && blockIdx.x < 64 && lane == 0) {
        g_clprof_rt[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
        g_clprof_rt[blockIdx.x][4] = __builtin_amdgcn_s_memtime();
    }
#endif
    if (wv >= NCW) {
        // ---------------- loader waves: loader lw moves the pieces p with p % NLDK == lw
        // wave-uniform (readfirstlane): the piece counts and the vmcnt switch below stay scalar;
        // derived from threadIdx they would be per-lane values and the 64-way wait_vm switch a
        // chain of exec-masked branches (the loader then paced every step: convs +20 %)
        const int lw = __builtin_amdgcn_readfirstlane(wv - NCW);
        const size_t wtap = (size_t)Cout * Cin;
        // A 1 KiB piece = 16 rows x 4 16-B slots; lane -> (row prow, slot pslot). With CI = 32 the
        // image swizzle of row p*16 + prow does not depend on the piece p, so this lane's source
        // offset inside any piece is one constant: no per-piece index math on the loader's path
        // (the per-step divisions and 64-bit address arithmetic of the plain form made the loader,
        // not the MFMAs, pace every step).
        static_assert((16 / I::RPB) % I::G == 0, "piece-invariant swizzle needs 16-row pieces to span whole swizzle periods");
        const int prow = lane >> 2, pslot = lane & 3;
        const int g = pslot ^ I::swz(prow);
        const int loff = prow * Cin + g * 8;
        const long prs = 16L * Cin;                                  // elements per 16-row piece
        const int nxl = (nxp - lw + NLDK - 1) / NLDK, nwl = (NWP - lw + NLDK - 1) / NLDK;
        // window stream (global step sx = j + dx): tile ix, tap tx, chunk cx; the tile's source row u0
        int ix = 0, tx = 0, cx = 0, u0 = 0, len_in = Tin;
        bool xfast = false;
        const uint16_t* xsrc0 = in;
        auto set_xtile = [&](int i) {
            int b_, ph_, co_, q_;
            tile_of(i, b_, ph_, co_, q_);
            len_in = lens ? min(lens[b_] * in_scale, Tin) : Tin;
            u0 = q_ - pad;
            xsrc0 = in + (size_t)b_ * Tin * Cin + loff + (long)u0 * Cin;     // row u0 of the window
            // every window row inside [0, len_in): no per-lane range checks (rows past `win` are read but unused)
            xfast = u0 >= 0 && u0 + nxp * 16 <= len_in;
        };
        // weight stream (global step sw = j + DA): tile iw, tap tw, chunk cw
        int iw = 0, tw = 0, cw = 0;
        const uint16_t* wsrc0 = w;
        auto set_wtile = [&](int i) {
            int b_, ph_, co_, q_;
            tile_of(i, b_, ph_, co_, q_);
            wsrc0 = w + (size_t)ph_ * wphase + (size_t)co_ * Cin + loff;
        };
        if (nt > 0) {
            set_xtile(0);
            set_wtile(0);
        }
        int xslot = 0, wslot = 0;                    // ring slots: one stream across the tiles
        int hist[DA + 1] = {};                       // loads issued by iterations j-DA .. j
        const int total = nt * nstep;
        for (int j = -dx; j < total; ++j) {
            int nl = 0;
            // window first: a window issued in the same iteration as W(j+DA) is then older
            // than it, so waiting for W(j) below also covers every window step j can need
            if (ix < nt) {
                if (tx == 0) {
                    char* dst = xring + xslot * XS;
                    const uint16_t* src = xsrc0 + cx * CI;
                    if (xfast) {
                        for (int p = lw; p < nxp; p += NLDK)
                            __builtin_amdgcn_global_load_lds((const void*)(src + p * prs), (void*)(dst + p * 1024), 16,
                                                             0, 0);
                    } else {
                        for (int p = lw; p < nxp; p += NLDK) {
                            const int row = p * 16 + prow, u = u0 + row;
                            const void* sp = (row < win && u >= 0 && u < len_in) ? (const void*)(src + p * prs)
                                                                                 : (const void*)g_zero_page;
                            __builtin_amdgcn_global_load_lds(sp, (void*)(dst + p * 1024), 16, 0, 0);
                        }
                    }
                    nl += nxl;
                    if (++xslot == nx_slots) xslot = 0;
                }
                if (++tx == ks) {
                    tx = 0;
                    if (++cx == nchunk) {
                        cx = 0;
                        if (++ix < nt) set_xtile(ix);
                    }
                }
            }
            if (j + DA >= 0 && iw < nt) {
                if (!ZK_CL_DIAG_NOW || j + DA < DA + 2) {     // (diag: each weight slot filled once)
                    char* dst = wring + wslot * WS;
                    const uint16_t* src = wsrc0 + tw * wtap + cw * CI;
#pragma unroll
                    for (int pp = 0; pp < (NWP + NLDK - 1) / NLDK; ++pp) {
                        const int p = pp * NLDK + lw;
                        if (p >= NWP) break;
                        __builtin_amdgcn_global_load_lds((const void*)(src + p * prs), (void*)(dst + p * 1024), 16, 0,
                                                         0);
                    }
                    nl += nwl;
                }
                if (++wslot == NWS) wslot = 0;
                if (++tw == ks) {
                    tw = 0;
                    if (++cw == nchunk) {
                        cw = 0;
                        if (++iw < nt) set_wtile(iw);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < DA; ++k) hist[k] = hist[k + 1];
            hist[DA] = nl;
            if (j >= 0 && (j % SPB == SPB - 1 || j == total - 1)) {
                // steps up to j need W(j), issued by iteration j - DA; everything issued later may stay in flight
                int pend = 0;
#pragma unroll
                for (int k = 1; k <= DA; ++k) pend += hist[k];
                if (lw == 0) ZK_CL_STAMP(0, j);
                wait_vm(pend);
                __builtin_amdgcn_s_barrier();           // publish step j
                if (lw == 0) ZK_CL_STAMP(1, j);
            }
        }
        return;
    }

    // ---------------- compute waves 0 .. NCW-1: NWM (co) x NWY (positions)
    const int ln = lane & 15, lg = lane >> 4, wm = wv / NWY, wn = wv % NWY;
    int t = 0, xslot = 0, wslot = 0;             // tap, window ring slot, weight ring slot of the step
    constexpr int NE = FUSE ? 6 : 3;             // epilogue constant tables per tile
    // fused: the 1x1 weights [co][ci] as an LDS image (row stride W1S halves), staged once per
    // workgroup; visible to every compute wave after the first step barrier
    uint16_t* const w1img = reinterpret_cast<uint16_t*>(xring + nx_slots * XS + 2 * NE * CO_T * sizeof(float));
    if constexpr (W1LDS) {
        for (int i = tid; i < CO_T * CO_T / 8; i += 64 * NCW) {
            const int row = i / (CO_T / 8), c8 = i % (CO_T / 8);
            *reinterpret_cast<uint4*>(w1img + row * W1S + c8 * 8) =
                *reinterpret_cast<const uint4*>(w1x1 + (size_t)row * CO_T + c8 * 8);
        }
    }
    for (int it = 0; it < nt; ++it) {
        int b, phase, co0, q0;
        tile_of(it, b, phase, co0, q0);
        f32x4 acc[FM][NQ];
#pragma unroll
        for (int m = 0; m < FM; ++m)
#pragma unroll
            for (int n = 0; n < NQ; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

        // Epilogue constants of this tile's CO_T channels -- bias, Snake alpha, 1/(alpha + 1e-9) --
        // staged into an LDS table (two, by tile parity: a wave may still read the previous tile's)
        // while the steps run (the epilogue used to start with their global loads and four IEEE
        // divisions per channel quartet)
        float* const ept = reinterpret_cast<float*>(xring + nx_slots * XS) + (it & 1) * NE * CO_T;
        for (int i = tid; i < CO_T; i += 64 * NCW) {
            const float a_ = (FUSE || sout) ? alpha[co0 + i] : 1.f;
            ept[i] = bias[co0 + i];
            ept[CO_T + i] = a_;
            ept[2 * CO_T + i] = __fdiv_rn(1.0f, __fadd_rn(a_, 1e-9f));
            if constexpr (FUSE) {
                const float an = alpha_out[i];
                ept[3 * CO_T + i] = b1x1[i];
                ept[4 * CO_T + i] = an;
                ept[5 * CO_T + i] = __fdiv_rn(1.0f, __fadd_rn(an, 1e-9f));
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");            // visible after the next barrier
        const int len_out = lens ? lens[b] * out_scale : Tout;

        // RES (resid != nullptr: the 1x1 convs of the residual units): the residual tile is loaded
        // before the main loop, so its latency overlaps the steps instead of following the last
        // MFMA (clamped, unconditional loads; out-of-range positions are never stored). A separate
        // instantiation: the 64 extra registers would cost the k7 convs occupancy.
        float4 rv[RES ? FM : 1][NQ];
        if constexpr (RES) {
#pragma unroll
            for (int m = 0; m < FM; ++m)
#pragma unroll
                for (int n = 0; n < NQ; ++n) {
                    const int q = q0 + wn * 16 * NQ + n * 16 + ln;
                    const int tt = min(max(q * out_stride + out_off0 + phase, 0), Tout - 1);
                    rv[m][n] = *reinterpret_cast<const float4*>(
                        resid + ((size_t)b * Tout + tt) * Cout + co0 + wm * 16 * FM + m * 16 + lg * 4);
                }
        }

        for (int s = 0; s < nstep; ++s) {
            if (SPB == 1 || (it * nstep + s) % SPB == 0) {
                __builtin_amdgcn_s_barrier();        // steps s .. s + SPB - 1 are in LDS
                asm volatile("" ::: "memory");
            }
            if (wv == 0 && it == 0) ZK_CL_STAMP(2, s);
#ifdef ZK_CL_PROF
            if (it == 0 && s == 0 && wv == 0 && blockIdx.x < 64 && lane == 0)
                g_clprof_rt[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
#endif
            const char* xb = xring + xslot * XS;
            const char* wb = wring + wslot * WS;
            if (++wslot == NWS) wslot = 0;
            uint4 a[FM], bq[NQ];
#pragma unroll
            for (int m = 0; m < FM; ++m)
                a[m] = *reinterpret_cast<const uint4*>(wb + I::off(wm * 16 * FM + m * 16 + ln, lg));
#pragma unroll
            for (int n = 0; n < NQ; ++n)
                bq[n] = *reinterpret_cast<const uint4*>(xb + I::off(wn * 16 * NQ + n * 16 + ln + t * dil, lg));
            if (ZK_CL_DIAG_NOMFMA) {          // diag: keep the operand reads, drop the MFMAs
#pragma unroll
                for (int m = 0; m < FM; ++m)
#pragma unroll
                    for (int n = 0; n < NQ; ++n) acc[m][n][0] += __uint_as_float(a[m].x ^ bq[n].y);
            } else {
#pragma unroll
                for (int m = 0; m < FM; ++m)
#pragma unroll
                    for (int n = 0; n < NQ; ++n)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(a[m]), as_h8(bq[n]), acc[m][n], 0, 0,
                                                                           0);
            }
            if (++t == ks) {
                t = 0;
                if (++xslot == nx_slots) xslot = 0;
            }
        }

#ifdef ZK_CL_PROF
        if (it == 0 && wv == 0 && blockIdx.x < 64 && lane == 0) {
            float keep = 0.f;
#pragma unroll
            for (int m = 0; m < FM; ++m)
#pragma unroll
                for (int n = 0; n < NQ; ++n) keep += acc[m][n][0];
            g_clprof_end[blockIdx.x][0] = __builtin_amdgcn_s_memtime() + (keep == 1.2345f);
            g_clprof_rt[blockIdx.x][2] = __builtin_amdgcn_s_memrealtime();
        }
#endif
        // acc[m][n][i] = C[co = co0 + wm*16FM + 16m + 4lg + i][q = q0 + 16NQ wn + 16n + ln]
        const int out_off = out_off0 + phase;
        if constexpr (FUSE) {
            // s2 = fp16(Snake_a2(conv7 + b7)) in the accumulator layout = the 16x16x16 B fragments
            uint2 h[FM][NQ];
#pragma unroll
            for (int m = 0; m < FM; ++m) {
                const int cl = m * 16 + lg * 4;
                const float4 bb = *reinterpret_cast<const float4*>(ept + cl);
                const float4 aa = *reinterpret_cast<const float4*>(ept + CO_T + cl);
                const float4 rr = *reinterpret_cast<const float4*>(ept + 2 * CO_T + cl);
#pragma unroll
                for (int n = 0; n < NQ; ++n)
                    h[m][n] = pack_h4(snake_fast(__fadd_rn(acc[m][n][0], bb.x), aa.x, rr.x),
                                      snake_fast(__fadd_rn(acc[m][n][1], bb.y), aa.y, rr.y),
                                      snake_fast(__fadd_rn(acc[m][n][2], bb.z), aa.z, rr.z),
                                      snake_fast(__fadd_rn(acc[m][n][3], bb.w), aa.w, rr.w));
            }
            // residual rows of output block mo (clamped loads; out-of-range positions are not stored),
            // one block ahead of the block being multiplied
            // (XPD output blocks of residual rows in flight: the accumulators are packed into h by now,
            // so their registers hold the prefetch)
            constexpr int XPD = ZK_RU_XPD < FM ? ZK_RU_XPD : FM;
            float4 xr[XPD][NQ];
            auto load_x = [&](int mo, int buf) {
#pragma unroll
                for (int n = 0; n < NQ; ++n) {
                    const int q = q0 + wn * 16 * NQ + n * 16 + ln;
                    const int tt = min(max(q * out_stride + out_off, 0), Tout - 1);
                    xr[buf][n] = *reinterpret_cast<const float4*>(resid + ((size_t)b * Tout + tt) * Cout + mo * 16 + lg * 4);
                }
            };
#pragma unroll
            for (int p = 0; p < XPD; ++p) load_x(p, p);
            // (!W1LDS) the 1x1 weight fragments of output block mo + 1 are loaded while block mo is
            // multiplied; the opaque pointer keeps hipcc from hoisting all of them out of the tile
            // loop into registers held across the main loop
            const uint16_t* w1p = w1x1;
            asm volatile("" : "+s"(w1p));
            uint2 wf[2][W1LDS ? 1 : FM];
            auto load_w = [&](int mo, int buf) {
                if constexpr (!W1LDS) {
#pragma unroll
                    for (int m = 0; m < FM; ++m)
                        wf[buf][m] = *reinterpret_cast<const uint2*>(w1p + (mo * 16 + ln) * CO_T + m * 16 + lg * 4);
                }
            };
            load_w(0, 0);
#pragma unroll
            for (int mo = 0; mo < FM; ++mo) {
                if (mo + 1 < FM) load_w(mo + 1, (mo + 1) & 1);
                f32x4 z[NQ];
#pragma unroll
                for (int n = 0; n < NQ; ++n) z[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int m = 0; m < FM; ++m) {
                    const uint2 wa = W1LDS ? *reinterpret_cast<const uint2*>(w1img + (mo * 16 + ln) * W1S + m * 16 + lg * 4)
                                           : wf[mo & 1][W1LDS ? 0 : m];
#pragma unroll
                    for (int n = 0; n < NQ; ++n)
                        z[n] = __builtin_amdgcn_mfma_f32_16x16x16f16(as_h4(wa), as_h4(h[m][n]), z[n], 0, 0, 0);
                }
                const int co = mo * 16 + lg * 4;
                const float4 bb = *reinterpret_cast<const float4*>(ept + 3 * CO_T + co);
                const float4 aa = *reinterpret_cast<const float4*>(ept + 4 * CO_T + co);
                const float4 rr = *reinterpret_cast<const float4*>(ept + 5 * CO_T + co);
#pragma unroll
                for (int n = 0; n < NQ; ++n) {
                    const int q = q0 + wn * 16 * NQ + n * 16 + ln;
                    const int tt = q * out_stride + out_off;
                    if (q >= Qn || tt < 0 || tt >= Tout) continue;
                    const size_t o = ((size_t)b * Tout + tt) * Cout + co;
                    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
                    if (tt < len_out) {
                        const float4 r = xr[mo % XPD][n];
                        v0 = __fadd_rn(r.x, __fadd_rn(z[n][0], bb.x));
                        v1 = __fadd_rn(r.y, __fadd_rn(z[n][1], bb.y));
                        v2 = __fadd_rn(r.z, __fadd_rn(z[n][2], bb.z));
                        v3 = __fadd_rn(r.w, __fadd_rn(z[n][3], bb.w));
                    }
                    *reinterpret_cast<float4*>(xout + o) = make_float4(v0, v1, v2, v3);
                    if (SF32)
                        reinterpret_cast<float4*>(sout)[o >> 2] =
                            make_float4(snake(v0, aa.x), snake(v1, aa.y), snake(v2, aa.z), snake(v3, aa.w));
                    else
                        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(sout) + o) =
                            pack_h4(snake_fast(v0, aa.x, rr.x), snake_fast(v1, aa.y, rr.y),
                                    snake_fast(v2, aa.z, rr.z), snake_fast(v3, aa.w, rr.w));
                }
                if (mo + XPD < FM) load_x(mo + XPD, mo % XPD);       // into the slot just consumed
            }
            continue;
        }
#pragma unroll
        for (int m = 0; m < FM; ++m) {
            const int cl = wm * 16 * FM + m * 16 + lg * 4, co = co0 + cl;
            const float4 bb = *reinterpret_cast<const float4*>(ept + cl);
            const float4 aa = *reinterpret_cast<const float4*>(ept + CO_T + cl);
            const float4 rr = *reinterpret_cast<const float4*>(ept + 2 * CO_T + cl);
            const float r0 = rr.x, r1 = rr.y, r2 = rr.z, r3 = rr.w;
#pragma unroll
            for (int n = 0; n < NQ; ++n) {
                const int q = q0 + wn * 16 * NQ + n * 16 + ln;
                const int tt = q * out_stride + out_off;
                if (q >= Qn || tt < 0 || tt >= Tout) continue;
                const size_t o = ((size_t)b * Tout + tt) * Cout + co;
                float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
                if (tt < len_out) {
                    v0 = __fadd_rn(acc[m][n][0], bb.x);
                    v1 = __fadd_rn(acc[m][n][1], bb.y);
                    v2 = __fadd_rn(acc[m][n][2], bb.z);
                    v3 = __fadd_rn(acc[m][n][3], bb.w);
                    if constexpr (RES) {
                        const float4 r = rv[m][n];
                        v0 = __fadd_rn(r.x, v0);
                        v1 = __fadd_rn(r.y, v1);
                        v2 = __fadd_rn(r.z, v2);
                        v3 = __fadd_rn(r.w, v3);
                    }
                }
                if (xout) *reinterpret_cast<float4*>(xout + o) = make_float4(v0, v1, v2, v3);
                if (!sout) continue;
                // fp32 Snake output for the fp32 tail (exact sinf, reference formula); a separate
                // instantiation so the common epilogue stays small enough to unroll fully (the
                // accumulators then never leave registers)
                if (SF32)
                    reinterpret_cast<float4*>(sout)[o >> 2] =
                        make_float4(snake(v0, aa.x), snake(v1, aa.y), snake(v2, aa.z), snake(v3, aa.w));
                else
                    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(sout) + o) =
                        pack_h4(snake_fast(v0, aa.x, r0), snake_fast(v1, aa.y, r1), snake_fast(v2, aa.z, r2),
                                snake_fast(v3, aa.w, r3));
            }
        }
#ifdef ZK_CL_PROF
        if (it == 0 && wv == 0 && blockIdx.x < 64 && lane == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            g_clprof_rt[blockIdx.x][3] = __builtin_amdgcn_s_memrealtime();
            g_clprof_rt[blockIdx.x][5] = __builtin_amdgcn_s_memtime();
        }
#endif
    }
#ifdef ZK_CL_PROF
    if (wv == 0 && blockIdx.x < 4096 && lane == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        g_clwg[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// z[b][t][ch] = fp16(sum_k E_k[code_k][ch]) channels-last, zero beyond the row's length
// (quantizer.from_codes, modeling_dac.py:520-538; summation order k = 0..ncb-1 as there).
__global__ __launch_bounds__(256) void k_rvq_cl(const int64_t* __restrict__ codes, int ncb, int T, long bstr,
                                                const float* __restrict__ tables, int ncode, int hidden, int cpad,
                                                uint16_t* __restrict__ z, const int32_t* __restrict__ lens) {
    const int t = blockIdx.x, b = blockIdx.y;
    const int len = lens ? lens[b] : T;
    for (int ch = threadIdx.x * 4; ch < cpad; ch += 1024) {
        float s[4] = {0.f, 0.f, 0.f, 0.f};
        if (t < len && ch < hidden) {
            for (int k = 0; k < ncb; ++k) {
                int64_t cd = codes[b * bstr + (size_t)k * T + t];
                cd = cd < 0 ? 0 : (cd >= ncode ? ncode - 1 : cd);
                const float4 e = *reinterpret_cast<const float4*>(tables + ((size_t)k * ncode + cd) * hidden + ch);
                if (k == 0) {
                    s[0] = e.x; s[1] = e.y; s[2] = e.z; s[3] = e.w;
                } else {
                    s[0] = __fadd_rn(s[0], e.x); s[1] = __fadd_rn(s[1], e.y);
                    s[2] = __fadd_rn(s[2], e.z); s[3] = __fadd_rn(s[3], e.w);
                }
            }
        }
        *reinterpret_cast<uint2*>(z + ((size_t)b * T + t) * cpad + ch) = pack_h4(s[0], s[1], s[2], s[3]);
    }
}

// out[b][t] = tanh(b + sum_{c,k} w[c][k] s[t+k-3][c]) from the channels-last fp32 Snake output
// of the last residual unit (modeling_dac.py:437-439; one output channel, so VALU: an MFMA
// tile would be 1/16 used). fp32 here keeps the waveform within the fp32 reference's 1e-4.
// The TAIL_T + 6 input rows of a workgroup are one contiguous [rows][C] block: staged into LDS
// by whole float4 loads (row stride C + 4 floats: the 16 lanes of a ds_read_b128 hit distinct
// banks), then each thread sums its position's 7 x C products in the order k, c, in four chains
// (c mod 4) added at the end.
#ifndef ZK_TAIL_T
#define ZK_TAIL_T 128
#endif
#ifndef ZK_TAIL_NB
#define ZK_TAIL_NB 16
#endif
constexpr int TAIL_T = ZK_TAIL_T;    // positions (threads) per workgroup
__global__ __launch_bounds__(TAIL_T) void k_tail_cl(const float* __restrict__ s, int C, int T,
                                                    const float* __restrict__ w, const float* __restrict__ bias,
                                                    float* __restrict__ out, const int32_t* __restrict__ lens,
                                                    int scale) {
    extern __shared__ __attribute__((aligned(16))) float tl[];     // [7][C] weights, then [TAIL_T + 6][C + 4] rows
    const int CS = C + 4, C4 = C / 4;
    float* wl = tl;
    float* rows = tl + ((C * 7 + 3) & ~3);
    const int b = blockIdx.y, t0 = blockIdx.x * TAIL_T;
    const int len = lens ? min(lens[b] * scale, T) : T;
    for (int i = threadIdx.x; i < C * 7; i += TAIL_T) {            // w [C][7] -> [7][C]
        const int c = i / 7, k = i - c * 7;
        wl[k * C + c] = w[i];
    }
    const float4* src = reinterpret_cast<const float4*>(s + (size_t)b * T * C);
    const int nrow = TAIL_T + 6, total = nrow * C4;
    // staging in batches of TAIL_NB loads per thread, all issued before the first LDS store: one
    // load in flight per thread (load -> store -> next load) made the kernel a chain of ~25 memory
    // round trips per workgroup (1.3 TB/s)
    constexpr int TAIL_NB = ZK_TAIL_NB;
    for (int i0 = threadIdx.x; i0 < total; i0 += TAIL_T * TAIL_NB) {
        float4 v[TAIL_NB];
#pragma unroll
        for (int j = 0; j < TAIL_NB; ++j) {
            const int i = i0 + j * TAIL_T;
            const int r = i / C4, c4 = i - r * C4;
            const int u = t0 - 3 + r;
            v[j] = (i < total && u >= 0 && u < len) ? src[(size_t)u * C4 + c4] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < TAIL_NB; ++j) {
            const int i = i0 + j * TAIL_T;
            const int r = i / C4, c4 = i - r * C4;
            if (i < total) *reinterpret_cast<float4*>(rows + r * CS + 4 * c4) = v[j];
        }
    }
    __syncthreads();
    const int t = t0 + threadIdx.x;
    if (t >= T) return;
    // four independent accumulation chains (channel c mod 4), each weight quad one broadcast
    // ds_read_b128: the single dependent chain with a scalar LDS weight read per FMA left one
    // wave per SIMD waiting on LDS latency (1.3 TB/s on a streaming kernel)
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int k = 0; k < 7; ++k) {
        const int u = t + k - 3;
        if (u < 0 || u >= len) continue;
        const float* row = rows + (threadIdx.x + k) * CS;
        const float* wk = wl + k * C;
#pragma unroll 4
        for (int c = 0; c < C; c += 4) {
            const float4 v = *reinterpret_cast<const float4*>(row + c);
            const float4 q = *reinterpret_cast<const float4*>(wk + c);
            a0 = fmaf(q.x, v.x, a0);
            a1 = fmaf(q.y, v.y, a1);
            a2 = fmaf(q.z, v.z, a2);
            a3 = fmaf(q.w, v.w, a3);
        }
    }
    const float acc = (a0 + a1) + (a2 + a3);
    out[(size_t)b * T + t] = (t < len) ? tanhf(__fadd_rn(acc, bias[0])) : 0.f;
}

// ---------------------------------------------------------------- encoder (prefix audio)
// DacEncoder.conv1 (1 -> C channels, k7, pad 3) from the waveform, channels-last outputs: fp32
// x (residual stream of the first residual unit) and fp16 Snake_a(x) (its conv input).
__global__ __launch_bounds__(256) void k_enc_conv1(const float* __restrict__ wav, int T, const float* __restrict__ w,
                                                   const float* __restrict__ bias, const float* __restrict__ alpha,
                                                   int C, int Cp, float* __restrict__ x, uint16_t* __restrict__ s) {
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (idx >= (long)T * Cp) return;
    const int c = (int)(idx % Cp);
    const int t = (int)(idx / Cp);
    float v = 0.f, sv = 0.f;
    if (c < C) {
        const float* wb = wav + (size_t)b * T;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const int u = t + k - 3;
            acc += w[c * 7 + k] * ((u >= 0 && u < T) ? wb[u] : 0.f);
        }
        v = acc + bias[c];
        sv = snake_fast(v, alpha[c], __fdiv_rn(1.0f, __fadd_rn(alpha[c], 1e-9f)));
    }
    const size_t o = ((size_t)b * T + t) * Cp + c;
    x[o] = v;
    s[o] = __builtin_bit_cast(uint16_t, (_Float16)sv);
}

// DacResidualVectorQuantizer (eval) for one latent frame per workgroup: per codebook in_proj
// (hidden -> cd), L2 normalisation, nearest normalised code by the reference's distance
// -(|e|^2 - 2 e.c) + |c|^2 (first index of the max), codebook row -> out_proj -> residual update.
constexpr int RVQ_CD = 8;
__global__ __launch_bounds__(256) void k_rvq_encode(const float* __restrict__ z, int T, int hidden, int ncb, int ncode,
                                                    const float* __restrict__ in_w, const float* __restrict__ in_b,
                                                    const float* __restrict__ cbn, const float* __restrict__ cbn2,
                                                    const float* __restrict__ cb, const float* __restrict__ out_w,
                                                    const float* __restrict__ out_b, int64_t* __restrict__ codes) {
    extern __shared__ float sm[];                       // residual [hidden]
    __shared__ float red[4][RVQ_CD];
    __shared__ float bestv[4];
    __shared__ int besti[4];
    __shared__ float qv[RVQ_CD];
    const int t = blockIdx.x, b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const float* zr = z + ((size_t)b * T + t) * hidden;
    for (int c = tid; c < hidden; c += 256) sm[c] = zr[c];
    __syncthreads();
    for (int k = 0; k < ncb; ++k) {
        // in_proj
        float part[RVQ_CD];
#pragma unroll
        for (int j = 0; j < RVQ_CD; ++j) part[j] = 0.f;
        const float* wk = in_w + (size_t)k * RVQ_CD * hidden;
        for (int c = tid; c < hidden; c += 256) {
            const float r = sm[c];
#pragma unroll
            for (int j = 0; j < RVQ_CD; ++j) part[j] += wk[(size_t)j * hidden + c] * r;
        }
#pragma unroll
        for (int j = 0; j < RVQ_CD; ++j) {
            float v = part[j];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
            if (lane == 0) red[wv][j] = v;
        }
        __syncthreads();
        float e[RVQ_CD];
        float nrm = 0.f;
#pragma unroll
        for (int j = 0; j < RVQ_CD; ++j) {
            e[j] = red[0][j] + red[1][j] + red[2][j] + red[3][j] + in_b[k * RVQ_CD + j];
            nrm += e[j] * e[j];
        }
        const float inv = 1.0f / fmaxf(sqrtf(nrm), 1e-12f);
        float l2 = 0.f;
#pragma unroll
        for (int j = 0; j < RVQ_CD; ++j) {
            e[j] *= inv;
            l2 += e[j] * e[j];
        }
        // nearest code
        float bv = -INFINITY;
        int bi = 0x7fffffff;
        const float* cbk = cbn + (size_t)k * ncode * RVQ_CD;
        for (int n = tid; n < ncode; n += 256) {
            float dot = 0.f;
#pragma unroll
            for (int j = 0; j < RVQ_CD; ++j) dot += e[j] * cbk[n * RVQ_CD + j];
            const float d = -(l2 - 2.0f * dot) + cbn2[k * ncode + n];
            if (d > bv || (d == bv && n < bi)) { bv = d; bi = n; }
        }
        for (int off = 32; off > 0; off >>= 1) {
            const float ov = __shfl_xor(bv, off, 64);
            const int oi = __shfl_xor(bi, off, 64);
            if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
        if (lane == 0) { bestv[wv] = bv; besti[wv] = bi; }
        __syncthreads();
        if (tid == 0) {
            float v = bestv[0];
            int i = besti[0];
            for (int w2 = 1; w2 < 4; ++w2)
                if (bestv[w2] > v || (bestv[w2] == v && besti[w2] < i)) { v = bestv[w2]; i = besti[w2]; }
            codes[((size_t)b * ncb + k) * T + t] = i;
#pragma unroll
            for (int j = 0; j < RVQ_CD; ++j) qv[j] = cb[((size_t)k * ncode + i) * RVQ_CD + j];
        }
        __syncthreads();
        const float* ow = out_w + (size_t)k * hidden * RVQ_CD;
        for (int c = tid; c < hidden; c += 256) {
            float acc = 0.f;
#pragma unroll
            for (int j = 0; j < RVQ_CD; ++j) acc += ow[(size_t)c * RVQ_CD + j] * qv[j];
            sm[c] -= acc + out_b[(size_t)k * hidden + c];
        }
        __syncthreads();
    }
}

// Persistent grid: as many workgroups as are resident at once (occupancy query for this kernel and
// LDS size x CUs), a multiple of 8 (the kernel's XCD split), at most one per tile.
template <int FM, int NQ, int NWY = 2, int NLDK = CL_NLD, int DA = CL_DA, int OCC = 2>
int launch_conv(long ntiles, size_t lds, hipStream_t st, const uint16_t* in, int B, int Cin, int Tin,
                const uint16_t* w, long wphase, const float* bias, int Cout, int ks, int dil, int pad, int Qn,
                int nphase, int out_stride, int out_off0, int Tout, const float* resid, float* xout,
                const float* alpha, void* sout, int s_f32, const int32_t* lens, int in_scale, int out_scale, int nq,
                int nx, int dx) {
    constexpr int NT = 64 * (2 * NWY + NLDK);
    auto kern = &k_conv_cl<FM, false, false, NQ, DA, OCC, NWY, NLDK>;     // NQ = 8: fp16 output, no residual only
    if constexpr (NQ == 4 && DA == CL_DA && NWY == 2)
        kern = resid ? (s_f32 ? &k_conv_cl<FM, true, true, NQ> : &k_conv_cl<FM, false, true, NQ>)
                     : (s_f32 ? &k_conv_cl<FM, true, false, NQ> : kern);
    if (lds > 65536)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
    // the current device's CU count (queried per call: a process may drive several devices)
    int dev = 0, ncu = 0;
    ZK_HIP(hipGetDevice(&dev));
    ZK_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    int occ = 0;
    ZK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(kern), NT, lds));
    ZK_REQUIRE(occ >= 1, "zk_dac_conv_cl: kernel does not fit a CU (LDS %zu)", lds);
    const long resident = (long)ncu * occ / 8 * 8;
    const long grid = std::min<long>((ntiles + 7) / 8 * 8, std::max<long>(resident, 8));
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), lds, st, in, Cin, Tin, w, wphase, bias, Cout, ks,
                       dil, pad, Qn, nphase, out_stride, out_off0, Tout, resid, xout, alpha, sout, s_f32, lens,
                       in_scale, out_scale, nq, nx, dx, B, nullptr, nullptr, nullptr);
    return 0;
}

// The fused residual unit: position waves each holding all C channels (C = 96: 64 positions,
// FM = 6, NQ = 4; C = 192: 32 positions, FM = 12, NQ = 2), persistent like launch_conv. ZK_RU_OCC
// (C = 96) 1: one workgroup per CU of 8 position waves + 4 loaders, the 1x1 weights in LDS; 2: two
// workgroups per CU of 4 position waves + 2 loaders, the 1x1 weights read through L1. C = 192: one
// workgroup per CU of 8 position waves (256-position tiles) + 4 loaders, the 1x1 weights (72 KB)
// read from L2 one output block ahead.
#ifndef ZK_RU_OCC
#define ZK_RU_OCC 1
#endif
#ifndef ZK_DAC_FUSE192
#define ZK_DAC_FUSE192 0             // C = 192 fused: 11.6 ms per unit vs 10.9 for the pair
#endif
template <int C_, bool SF32>
int launch_resunit(const uint16_t* s_in, int B, int T, const uint16_t* w7, const float* b7, int dil, const float* a2,
                   const uint16_t* w1, const float* b1, float* x, const float* alpha_next, void* s_out,
                   const int32_t* lens, int scale, hipStream_t st) {
    constexpr int FM = C_ / 16, NQ = C_ == 96 ? 4 : 2, OCC = C_ == 96 ? ZK_RU_OCC : 1;
    constexpr int NWY = OCC == 1 ? 8 : 4, NLD = OCC == 1 ? 4 : 2;
    constexpr int NT = 64 * (NWY + NLD);
    constexpr int qt = 16 * NQ * NWY;
    constexpr bool w1lds = OCC == 1 && C_ * (C_ + 8) * 2 <= 24 * 1024;     // = the kernel's W1LDS
    auto kern = &k_conv_cl<FM, SF32, false, NQ, CL_DA, OCC, NWY, NLD, CL_SPB, 1, true>;
    const int ks = 7, win = qt + (ks - 1) * dil;
    const size_t xs = (size_t)((win + 15) / 16) * 1024, ws = (size_t)C_ * 64;
    const size_t fixed = (size_t)2 * 6 * C_ * sizeof(float) + (w1lds ? (size_t)C_ * (C_ + 8) * 2 : 0);
    const size_t cap = OCC == 1 ? 160 * 1024 : 80 * 1024;
    const int spb = CL_SPB, nws = CL_DA + 2 * spb;
    int dx = std::max(CL_DA, ks), nx = 1 + (dx + 2 * spb - 1 + ks - 1) / ks;
    while (dx > CL_DA && nws * ws + nx * xs + fixed > cap) {
        --dx;
        nx = 1 + (dx + 2 * spb - 1 + ks - 1) / ks;
    }
    const size_t lds = nws * ws + nx * xs + fixed;
    ZK_REQUIRE(lds <= cap, "zk_dac_resunit_cl: LDS %zu too large (C %d dil %d)", lds, C_, dil);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    int dev = 0, ncu = 0, occ = 0;
    ZK_HIP(hipGetDevice(&dev));
    ZK_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    ZK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(kern), NT, lds));
    ZK_REQUIRE(occ >= 1, "zk_dac_resunit_cl: kernel does not fit a CU (LDS %zu)", lds);
    const int nq = (T + qt - 1) / qt;
    const long ntiles = (long)B * nq;
    ZK_REQUIRE(ntiles < (1L << 31), "zk_dac_resunit_cl: too many tiles");
    const long resident = (long)ncu * occ / 8 * 8;
    const long grid = std::min<long>((ntiles + 7) / 8 * 8, std::max<long>(resident, 8));
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), lds, st, s_in, C_, T, w7, 0L, b7, C_, ks, dil,
                       3 * dil, T, 1, 1, 0, T, x, x, a2, s_out, (int)SF32, lens, scale, scale, nq, nx, dx, B, w1, b1,
                       alpha_next);
    return 0;
}

}  // namespace

extern "C" int zk_dac_enc_conv1(const float* wav, int B, int T, const float* w, const float* bias,
                                const float* alpha_next, int C, int Cp, float* x_out, uint16_t* s_out, void* stream) {
    ZK_REQUIRE(C > 0 && Cp >= C && Cp % 32 == 0, "zk_dac_enc_conv1: C=%d Cp=%d", C, Cp);
    if (B == 0 || T == 0) return 0;
    const long n = (long)T * Cp;
    hipLaunchKernelGGL(k_enc_conv1, dim3((unsigned)((n + 255) / 256), B), dim3(256), 0, (hipStream_t)stream, wav, T, w,
                       bias, alpha_next, C, Cp, x_out, s_out);
    ZK_CHECK_LAUNCH("zk_dac_enc_conv1");
    return 0;
}

extern "C" int zk_dac_rvq_encode(const float* z, int B, int T, int hidden, int ncb, int ncode, int cdim,
                                 const float* in_w, const float* in_b, const float* cb_norm, const float* cb_norm_sq,
                                 const float* cb, const float* out_w, const float* out_b, int64_t* codes,
                                 void* stream) {
    ZK_REQUIRE(cdim == RVQ_CD && hidden > 0 && ncb > 0 && ncode > 0, "zk_dac_rvq_encode: cdim=%d (8 only)", cdim);
    ZK_REQUIRE((size_t)hidden * 4 <= 64 * 1024, "zk_dac_rvq_encode: hidden=%d too large", hidden);
    if (B == 0 || T == 0) return 0;
    hipLaunchKernelGGL(k_rvq_encode, dim3(T, B), dim3(256), (size_t)hidden * 4, (hipStream_t)stream, z, T, hidden, ncb,
                       ncode, in_w, in_b, cb_norm, cb_norm_sq, cb, out_w, out_b, codes);
    ZK_CHECK_LAUNCH("zk_dac_rvq_encode");
    return 0;
}

extern "C" int zk_dac_rvq_decode_cl(const int64_t* codes, int B, int ncb, int T, long code_bstride,
                                    const float* tables, int ncode, int hidden, int cpad, uint16_t* z,
                                    const int32_t* lens, void* stream) {
    ZK_REQUIRE(hidden % 4 == 0 && cpad >= hidden && cpad % 32 == 0, "zk_dac_rvq_decode_cl: hidden=%d cpad=%d", hidden,
               cpad);
    if (B == 0 || T == 0) return 0;
    hipLaunchKernelGGL(k_rvq_cl, dim3(T, B), dim3(256), 0, (hipStream_t)stream, codes, ncb, T, code_bstride, tables,
                       ncode, hidden, cpad, z, lens);
    ZK_CHECK_LAUNCH("zk_dac_rvq_decode_cl");
    return 0;
}

extern "C" int zk_dac_conv_cl(const uint16_t* in, int B, int Cin, int Tin, const uint16_t* w, long w_phase_stride,
                              const float* bias, int Cout, int ks, int dil, int pad, int Qn, int nphase,
                              int out_stride, int out_off0, int Tout, const float* resid, float* x_out,
                              const float* alpha_next, void* s_out, int s_f32, const int32_t* lens, int in_scale,
                              int out_scale, void* stream) {
    ZK_REQUIRE(Cin > 0 && Cin % 32 == 0, "zk_dac_conv_cl: Cin=%d must be a multiple of 32", Cin);
    ZK_REQUIRE(Cout > 0 && Cout % 32 == 0, "zk_dac_conv_cl: Cout=%d must be a multiple of 32", Cout);
    ZK_REQUIRE(ks >= 1 && ks <= 7 && dil >= 1 && (ks - 1) * dil <= MAXSPAN, "zk_dac_conv_cl: ks=%d dil=%d", ks, dil);
    ZK_REQUIRE(nphase >= 1 && bias != nullptr && (s_out == nullptr || alpha_next != nullptr) &&
                   (s_out != nullptr || x_out != nullptr),
               "zk_dac_conv_cl: bad arguments");
    if (B == 0 || Qn <= 0) return 0;
    const int nco = Cout / 32;
    const int FM = nco % 4 == 0 ? 4 : (nco % 3 == 0 ? 3 : (nco % 2 == 0 ? 2 : 1));
    // 256-position tiles for the plain convs without a residual at FM <= 3 (the 96-192-channel k7
    // convs, overhead-bound at 128: -6 % / -15 %); the residual convs keep 128 (their prefetched
    // residual tile would not fit the registers beside twice the accumulators), and so do the
    // polyphase ConvTranspose convs (+12-22 % with 256, profiles/r1_dac_wide_tiles_ab.txt)
    // (one workgroup per CU with a deeper weight ring measured slower: DESIGN.md §6)
#ifndef ZK_CL_WIDE
#define ZK_CL_WIDE 1
#endif
    const bool wide = ZK_CL_WIDE && resid == nullptr && !s_f32 && nphase == 1 && FM <= 3;
    // fat: the wide convs as ONE workgroup per CU of 8 compute waves (2 channel halves x 4 position
    // quarters, 512-position tiles) + 4 loaders = 12 waves, exactly 3 per SIMD. Two 6-wave
    // workgroups per CU (the same compute per step) were co-resident only where the wave placement
    // happened to balance the SIMDs (3 waves per SIMD is the register limit at 150 VGPRs): 1.3 per CU
    // on average (tools/dac_conv_stamps.py HW_ID census); one workgroup also shares each weight slice
    // among twice the waves.
#ifndef ZK_CL_FAT
#define ZK_CL_FAT 1
#endif
    const bool fat = ZK_CL_FAT && wide;
    const int qt = fat ? 4 * QT : (wide ? 2 * QT : QT);
    const int win = qt + (ks - 1) * dil;
    const size_t xs = (size_t)((win + 15) / 16) * 1024;
    const size_t ws = (size_t)32 * FM * 64;
    const int da = CL_DA;
    const size_t lds_cap = fat ? 160 * 1024 : 80 * 1024;
    // window lead DX >= da steps, ring NX = 1 + ceil((DX + 2 SPB - 1)/ks) slots, weight ring da + 2 SPB;
    // keep LDS <= 80 KiB (2 per CU)
    const size_t ept = (size_t)2 * 3 * 32 * FM * sizeof(float);      // epilogue constants tables (x 2)
    const int spb = CL_SPB, nws = da + 2 * spb;
    int dx = std::max(da, ks), nx = 1 + (dx + 2 * spb - 1 + ks - 1) / ks;
    while (dx > da && nws * ws + nx * xs + ept > lds_cap) {
        --dx;
        nx = 1 + (dx + 2 * spb - 1 + ks - 1) / ks;
    }
    const size_t lds = nws * ws + nx * xs + ept;
    ZK_REQUIRE(lds <= 160 * 1024, "zk_dac_conv_cl: LDS %zu too large", lds);
    const int nq = (Qn + qt - 1) / qt;
    const long ntiles = (long)B * nq * (Cout / (32 * FM)) * nphase;
    ZK_REQUIRE(ntiles < (1L << 31), "zk_dac_conv_cl: too many tiles");
    hipStream_t st = (hipStream_t)stream;
#define ZK_CL(F_, NQ_)                                                                                           \
    ZK_TRY((launch_conv<F_, NQ_>(ntiles, lds, st, in, B, Cin, Tin, w, w_phase_stride, bias, Cout, ks, dil, pad, Qn,  \
                                 nphase, out_stride, out_off0, Tout, resid, x_out, alpha_next, s_out, s_f32, lens,   \
                                 in_scale, out_scale, nq, nx, dx)))
#define ZK_CLF(F_)                                                                                                \
    ZK_TRY((launch_conv<F_, 8, 4, 4, CL_DA, 1>(ntiles, lds, st, in, B, Cin, Tin, w, w_phase_stride, bias, Cout, ks, dil, \
                                     pad, Qn, nphase, out_stride, out_off0, Tout, resid, x_out, alpha_next, s_out,    \
                                     s_f32, lens, in_scale, out_scale, nq, nx, dx)))
    switch (FM) {
        case 4: ZK_CL(4, 4); break;
        case 3: if (fat) ZK_CLF(3); else if (wide) ZK_CL(3, 8); else ZK_CL(3, 4); break;
        case 2: if (fat) ZK_CLF(2); else if (wide) ZK_CL(2, 8); else ZK_CL(2, 4); break;
        default: if (fat) ZK_CLF(1); else if (wide) ZK_CL(1, 8); else ZK_CL(1, 4); break;
    }
#undef ZK_CLF
#undef ZK_CL
    ZK_CHECK_LAUNCH("zk_dac_conv_cl");
    return 0;
}

// ZK_DAC_FUSE: 0 = every residual unit as two convs; 1 = the units of C = 96 fused except the last
// (its fp32 Snake output makes the fused epilogue spill); 2 = the last one too
#ifndef ZK_DAC_FUSE
#define ZK_DAC_FUSE 1
#endif
extern "C" int zk_dac_resunit_supported(int C) {
    return C == 96 ? ZK_DAC_FUSE : (C == 192 && ZK_DAC_FUSE192 ? ZK_DAC_FUSE : 0);
}

extern "C" int zk_dac_resunit_cl(const uint16_t* s_in, int B, int C, int T, const uint16_t* w7, const float* b7,
                                 int dil, const float* a2, const uint16_t* w1, const float* b1, float* x,
                                 const float* alpha_next, void* s_out, int s_f32, const int32_t* lens, int scale,
                                 void* stream) {
    ZK_REQUIRE(C == 96 || C == 192, "zk_dac_resunit_cl: C=%d (the fused unit is built for C = 96 and 192)", C);
    ZK_REQUIRE(dil >= 1 && 6 * dil <= MAXSPAN, "zk_dac_resunit_cl: dil=%d", dil);
    ZK_REQUIRE(s_in != nullptr && w7 && b7 && a2 && w1 && b1 && x && alpha_next && s_out,
               "zk_dac_resunit_cl: null argument");
    ZK_REQUIRE(s_out != static_cast<const void*>(s_in),
               "zk_dac_resunit_cl: s_out must not alias s_in (neighbouring tiles read it as their halo)");
    if (B == 0 || T <= 0) return 0;
    hipStream_t st = (hipStream_t)stream;
#define ZK_RU(C_, F_) ZK_TRY((launch_resunit<C_, F_>(s_in, B, T, w7, b7, dil, a2, w1, b1, x, alpha_next, s_out, lens, scale, st)))
    if (C == 96) { if (s_f32) ZK_RU(96, true); else ZK_RU(96, false); }
    else { if (s_f32) ZK_RU(192, true); else ZK_RU(192, false); }
#undef ZK_RU
    ZK_CHECK_LAUNCH("zk_dac_resunit_cl");
    return 0;
}

#ifdef ZK_CL_PROF
extern "C" int zk_cl_prof_read(void* dst, void* dst_end) {
    if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_clprof), sizeof(g_clprof)) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(dst_end, HIP_SYMBOL(g_clprof_rt), sizeof(g_clprof_rt)) != hipSuccess) return -1;
    return 0;
}
extern "C" int zk_cl_prof_read_wg(void* dst) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_clwg), sizeof(g_clwg)) == hipSuccess ? 0 : -1;
}
extern "C" int zk_cl_prof_read_hw(void* dst) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_clhw), sizeof(g_clhw)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int zk_dac_tail_cl(const float* s, int B, int C, int T, const float* w, const float* bias, float* out,
                              const int32_t* lens, int scale, void* stream) {
    ZK_REQUIRE(C > 0 && C % 4 == 0 && T >= 0, "zk_dac_tail_cl: bad shape C=%d", C);
    if (B == 0 || T == 0) return 0;
    const size_t lds = ((size_t)((C * 7 + 3) & ~3) + (size_t)(TAIL_T + 6) * (C + 4)) * sizeof(float);
    ZK_REQUIRE(lds <= 160 * 1024, "zk_dac_tail_cl: C=%d too large", C);
    if (lds > 65536)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tail_cl), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
    hipLaunchKernelGGL(k_tail_cl, dim3((T + TAIL_T - 1) / TAIL_T, B), dim3(TAIL_T), lds, (hipStream_t)stream, s, C, T, w,
                       bias, out, lens, scale);
    ZK_CHECK_LAUNCH("zk_dac_tail_cl");
    return 0;
}
