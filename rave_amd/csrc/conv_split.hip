// Split-f16 implicit-GEMM Conv1d / ConvTranspose1d on gfx950
// (RAVE_PREC_SPLIT16, include/rave_amd.h): the same operator as conv1d.hip --
// cached_conv's Conv1d / ConvTranspose1d forward at every call site of
// rave/blocks.py (DilatedUnit :96-106, EncoderV2 :533-584, GeneratorV2
// :631-677, NoiseGeneratorV2 :257-266) fused with the preceding activation and
// the Residual add (rave/blocks.py:44-46) -- computed on the f16 matrix cores.
//
// Arithmetic.  Every fp32 operand v becomes an f16 pair hi = f16(v),
// lo = f16((v - hi) * 2^11); weights are first scaled per GEMM row by 2^e_m
// (max |w'| in [8, 16)).  One fp32 accumulator takes
//     (hi_w * 2^11) * hi_x  +  hi_w * lo_x  +  lo_w * hi_x
// (three v_mfma_f32_32x32x16_f16, 32 cycles each per 16-deep K-step, against
// eight 64-cycle v_mfma_f32_32x32x2_f32 for the same K in fp32: 5.3x the
// rate).  f16 x f16 products are exact in fp32; the dropped lo*lo term and the
// two roundings are ~2^-22 relative; the epilogue multiplies by 2^-(e_m+11)
// exactly.  Result error is on par with the fp32 MFMA path (tests).
//
// GEMM view: Y[m, n] = sum_kk W[m, kk] X[kk, n], kk = (tap q, virtual channel).
// Strided convs (k = 2s, stride s) run polyphase: virtual channel (ci, p) at
// window row u is x[ci][u*s + p - pad], tap q reads row n + q, so every family
// is a stride-1 conv over rows of the staged window:
//     k1: 1 tap       k3: 3 taps at row shift d      k7: 7 taps
//     k4 s2 / k8 s4: 2 taps over (ci, phase)         ConvT: 2 taps (u-1|u, u|u+1)
// Per K-chunk (VC virtual channels x all taps) a workgroup stages in LDS:
//   * the weight image of its BM rows: (hi, lo) A-fragments in lane order,
//     host-packed, copied by LDS-DMA (global_load_lds_dwordx4), no VGPRs;
//   * the activation window [rows][VC] channels-last as two f16 planes (hi, lo),
//     activation applied and split once per element on the way in, so each
//     B-fragment (8 channels of one column) is one ds_read_b128.
// Double-buffered planes (one barrier per chunk); window DMAs three chunks
// ahead in a 4-deep ring.  Each wave owns 2 or 4 blocks of 32x32
// (32x64, 64x64 or 32x128 outputs); optionally two waves ("K-groups") share a
// tile's K-steps.  Split-K over workgroups for short-N layers (fp32 slabs,
// fixed-order combine: deterministic).  The autotuner picks the tile.
#include "conv_shared.h"

#include <cmath>
#include <cstring>
#include <vector>

namespace rave {

typedef _Float16 s_h8 __attribute__((ext_vector_type(8)));
typedef float s_f32x8 __attribute__((ext_vector_type(8)));
typedef float s_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 s_b8 __attribute__((ext_vector_type(8)));
// fp32 x 8 -> three bf16 parts with v == hi + mid + lo exactly (each remainder exact in fp32)
__device__ __forceinline__ void s_bf3_split(const s_f32x8& v, s_b8& hi, s_b8& mid, s_b8& lo) {
    bf3_split_pk(v, hi, mid, lo);
}

// (taps after polyphase Q, phases S, virtual channels per chunk VC, max row shift)
template <int KT> struct SFam;
template <> struct SFam<1> { static constexpr int Q = 1, S = 1, VC = 32, DMAX = 0; };
template <> struct SFam<2> { static constexpr int Q = 2, S = 1, VC = 16, DMAX = 1; };   // ConvT
template <> struct SFam<3> { static constexpr int Q = 3, S = 1, VC = 16, DMAX = kMaxDil; };
template <> struct SFam<4> { static constexpr int Q = 2, S = 2, VC = 16, DMAX = 1; };
template <> struct SFam<7> { static constexpr int Q = 7, S = 1, VC = 16, DMAX = 1; };
template <> struct SFam<8> { static constexpr int Q = 2, S = 4, VC = 16, DMAX = 1; };

template <int KT> struct SInfo {
    static constexpr int Q = SFam<KT>::Q, S = SFam<KT>::S, VC = SFam<KT>::VC;
    static constexpr int KSC = Q * VC / 16;        // 16-deep K-steps per chunk
    static constexpr int CPC = VC / S;             // real input channels per chunk
};

[[maybe_unused]] static inline int split_cpc(int taps) {
    switch (taps) {
        case 1: return SInfo<1>::CPC;
        case 2: return SInfo<2>::CPC;
        case 3: return SInfo<3>::CPC;
        case 4: return SInfo<4>::CPC;
        case 7: return SInfo<7>::CPC;
        case 8: return SInfo<8>::CPC;
        default: return 0;
    }
}
[[maybe_unused]] static inline int split_ksc(int taps) {
    switch (taps) {
        case 1: return SInfo<1>::KSC;
        case 2: return SInfo<2>::KSC;
        case 3: return SInfo<3>::KSC;
        case 4: return SInfo<4>::KSC;
        case 7: return SInfo<7>::KSC;
        case 8: return SInfo<8>::KSC;
        default: return 0;
    }
}

// LDS-DMA issue (inline asm: invisible to hipcc's vmcnt bookkeeping, so no
// compiler drain of the ring; completion is counted by hand).  M0 = the
// wave-uniform LDS destination, written and restored inside the statement.
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
// 4 bytes per lane through a buffer descriptor: out-of-range offsets land zeros
__device__ __forceinline__ void dma4(u32x4_t rsrc, unsigned voff, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds_dst) : "memory");
}
// 16 bytes per lane through a buffer descriptor (aligned window rows)
__device__ __forceinline__ void dma16b(u32x4_t rsrc, unsigned voff, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds_dst) : "memory");
}
// 16-byte register load through a buffer descriptor, hidden from hipcc's vmcnt
// bookkeeping (form (ii) of the guide: the consumer waits with the registers
// named "+v"); out-of-range offsets read zeros
__device__ __forceinline__ u32x4_t bload16(u32x4_t rsrc, unsigned voff) {
    u32x4_t r;
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(r) : "v"(voff), "s"(rsrc) : "memory");
    return r;
}
template <int N>
__device__ __forceinline__ void wait_vm_regs(u32x4_t& a0, u32x4_t& a1) {
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a0), "+v"(a1) : "n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm_regs3(u32x4_t& a0, u32x4_t& a1, u32x4_t& a2) {
    asm volatile("s_waitcnt vmcnt(%3)" : "+v"(a0), "+v"(a1), "+v"(a2) : "n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Keeps a bload16 destination live (and in its register) up to this point:
// placed after the wait that covers the load, it forbids hipcc to reuse the
// register for anything else while the load may still write it (volatile asm
// statements keep their order).  tools/ring_hazard_check.py checks the built
// code object for any read, copy or write of a ring register before its wait.
__device__ __forceinline__ void ring_keep(u32x4_t& a) { asm volatile("" : "+v"(a)); }
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)p);
}
__device__ __forceinline__ u32x4_t raw_rsrc(const void* p, int bytes) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    u32x4_t r;
    r[0] = __builtin_amdgcn_readfirstlane((uint32_t)v);
    r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) & 0xFFFFu;
    r[2] = __builtin_amdgcn_readfirstlane((uint32_t)bytes);
    r[3] = 0x00020000u;
    return r;
}

// Workgroup tile: BN time columns x BM GEMM rows.  A wave owns WM rows x WN
// columns (WM = 32: 128 columns; WM = 64: 64 columns), four 32x32 blocks.
// KG = 2 or 4: KG waves per output tile ("K-groups"), each taking a contiguous
// share of every chunk's K-steps (group g: ks_of(g) steps from st_of(g));
// summed through LDS at the end in group order.
// VCX: one staged chunk is VCX packed weight chunks ("sub-chunks") of the
// family's VC virtual channels -- more K-steps per barrier and per window DMA
// round, and enough of them for four K-groups on the short-N layers (C >= 512
// at 64-128 frames), which would otherwise need split-K slabs in HBM.
// NP: operand planes per staged buffer (2: the split16 (hi, lo) pair or one
// fp32 plane in its bytes; 3: bf16x3 hi, lo, mid); NPW: 16-byte weight
// fragment loads per K-step and 32-row block (NP, or 2 for the bf16x3 kernel on
// the fp32 weight image, RAVE_BF3_W4)
template <int KT, int BM, int BN, int WM, bool XV = true, int KG = 1, int WN_ = 4096 / WM, int VCX = 1, int NS_ = 3,
          int NP = 2, int NPW = (NP == 3 && RAVE_BF3_W4) ? 2 : NP>
struct SGeo {
    using F = SFam<KT>;
    static constexpr int Q = F::Q, S = F::S, VC0 = F::VC, VC = VC0 * VCX;
    static constexpr int KSC0 = Q * VC0 / 16;                // K-steps per packed weight chunk
    static constexpr int HPS0 = VC0 / 16;                    // K-steps per tap within a packed chunk
    static constexpr int KSC = KSC0 * VCX, CPC = VC / S;     // per staged chunk
    static constexpr int WN = WN_, NJ = WM / 32, NI = WN / 32;
    static constexpr int WGM = BM / WM, WGN = BN / WN, NWT = WGM * WGN, NW = NWT * KG, NT = 64 * NW;
    static constexpr int ks_of(int g) { return KSC / KG + (g < KSC % KG ? 1 : 0); }
    static constexpr int st_of(int g) { return g * (KSC / KG) + (g < KSC % KG ? g : KSC % KG); }
    static constexpr int KS0 = ks_of(0);                     // most K-steps of any group
    // window rows: columns + tap reach (+1: ConvT phase group 1 reads one row later)
    static constexpr int XW_MAX = BN + (Q - 1) * F::DMAX + (KT == 2 ? 1 : 0);
    static constexpr int PH = VC + 8;                        // halves per plane row (conflict-free b128)
    static constexpr int XPLANE = XW_MAX * PH * 2;           // bytes per f16 plane
    static constexpr int WR = KS0 * NJ * NPW;                // weight fragment loads per wave per chunk (max)
    // raw window rows: XV = 16-byte pieces from a 4-sample-aligned start (row
    // stride rounded up to 4 samples), else 4-byte pieces
    static constexpr int RS_MAX = XV ? ((XW_MAX * S + 3 + 3) / 4) * 4 : XW_MAX * S;
    static constexpr int RAW_F = CPC * RS_MAX;               // raw window floats of one chunk
    static constexpr int PF = XV ? 4 : 1;                    // floats per lane per DMA
    static constexpr int PB = 256 * PF;                      // bytes per wave DMA piece
    static constexpr int NPIECE = (RAW_F * 4 + PB - 1) / PB; // pieces one chunk's window needs
    static constexpr int XI = (NPIECE + NW - 1) / NW;        // window DMA pieces per wave
    // ring slot: the pieces the window needs; every wave still issues XI DMAs
    // (uniform hand counts), the surplus ones land in one dump piece
    static constexpr int STAGE = NPIECE * PB;
    // window DMA ring of NS slots: chunk c's window is issued at the top of
    // chunk c - NS (into the slot chunk c - NS's window left: split during
    // chunk c - NS - 1) and split during chunk c - 1, so it has NS - 1 chunks
    // of K-steps to land (NS = 2 trades that for room for wider chunks)
    static constexpr int NS = NS_;
    // hand-counted vmcnt waits (kernel body): prologue, end of chunk, weights
    static constexpr int WAIT_PRO = (NS - 1) * XI + NPW * KS0 * NJ;
    static constexpr int WAIT_END = (NS - 1) * NPW * KS0 * NJ + (NS - 2) * XI;
    static constexpr int WAIT_MAX = WAIT_PRO > WAIT_END ? WAIT_PRO : WAIT_END;
    static constexpr int ALPHA = 4096;                       // Snake alphas (<= 1024 channels)
    static constexpr int EROW = WN + 4;                      // epilogue transpose row stride (floats)
    static constexpr int EPI = NW * WM * EROW * 4;           // epilogue transpose area (reuses the ring)
    // ring + two plane buffers (NP planes each) + Snake alphas + the surplus DMAs' dump piece
    static constexpr int MAIN = NS * STAGE + 2 * NP * XPLANE + ALPHA + PB;
    static constexpr int LDS = MAIN > EPI ? MAIN : EPI;
    // + the split-K "last arriver" word, the range guard's per-wave overflow votes
    // (two plane buffers + the tile vote, x 16 waves, bytes) and wave maxima (16 floats)
    static constexpr int VOTE = LDS + 16, VRED = LDS + 64;
    static constexpr int LDS_ALL = LDS + 128;
    static constexpr int G8 = VC / 8;                        // 8-channel groups per row
    static constexpr int XT = (XW_MAX * G8 + NT - 1) / NT;   // convert tasks per thread
    static_assert(XPLANE % 16 == 0 && STAGE % 16 == 0, "16-byte LDS alignment");
    static_assert((NI * NJ == 4 || NI * NJ == 2) && NW >= 1 && NW <= 16, "tile");
    static_assert(KG == 1 || KG == 2 || KG == 4, "K-groups");
    // a configuration is built only if its hand-counted waits fit the vmcnt
    // field, its LDS fits the CU and every K-group has a K-step
    static constexpr int NPW_ = NPW;
    static constexpr bool VALID = WAIT_MAX <= 63 && WR + XI <= 63 && LDS_ALL <= 160 * 1024 && ks_of(KG - 1) >= 1 &&
                                  (NS == 2 || NS == 3);
};

template <int V> struct IC {
    static constexpr int value = V;
};

// AR: 0 split16; 1 F32: the same machinery with exact fp32 operands
// (RAVE_PREC_F32_RING): one fp32 plane per staged buffer (row pitch PH floats,
// the bytes of the hi / lo pair), weight fragments of 8 floats per lane in the
// split image's slots, and eight v_mfma_f32_32x32x2_f32 per 16-deep K-step
// (K-slot (s, half h) = channel 8h + s of the step's 16); no range guard, row
// scales 1.  2 BF (RAVE_PREC_BF16X3): every operand split exactly into bf16
// (hi, lo, mid) -- three planes per staged buffer, three weight fragments per
// K-step, six v_mfma_f32_32x32x16_bf16 (every cross product but mid*lo, lo*mid,
// lo*lo: each < 2^-25 |a b|), smallest first; no range guard, row scales 1.
template <int KT, int BM, int BN, int WM, bool SNAKE, bool XV, int KG, int WN_, int VCX, int NS, int AR>
__device__ __forceinline__ void conv1d_split_body(const ConvKArgs& a) {
    constexpr bool F32 = AR == 1, BF = AR == 2;
    constexpr int NP = BF ? 3 : 2;
    using G = SGeo<KT, BM, BN, WM, XV, KG, WN_, VCX, NS, NP>;
    constexpr int NPW = G::NPW_;                     // weight fragment loads per K-step and row block
    constexpr bool W4 = BF && NPW == 2;              // bf16x3 on the fp32 weight image
    constexpr int S = G::S, CPC = G::CPC, PH = G::PH;
    constexpr int NT = G::NT, NW = G::NW, NWT = G::NWT, WGM = G::WGM, G8 = G::G8, XT = G::XT;
    constexpr int NI = G::NI, NJ = G::NJ, WN = G::WN;
    constexpr int KSC0 = G::KSC0, HPS0 = G::HPS0, VC0 = G::VC0;
    constexpr unsigned kOOB = 0xFFFFFFF0u;

    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x;
#ifdef RAVE_STAMPS
    const int wg_lin = blockIdx.x;
    auto stamp = [&](int k) {
        if (tid == 0 && a.stamps) {
            a.stamps[wg_lin * 8 + k] = __builtin_amdgcn_s_memtime();
            if (k == 0) a.stamps[wg_lin * 8 + 7] = __builtin_amdgcn_s_memrealtime();
        }
    };
    // cycle accumulators of wave 0 in the K loop: the weight waits (slot 5) and
    // the chunk-end window wait + barrier (slot 6)
    unsigned long long acc_ww = 0, acc_we = 0;
    auto now = []() { return __builtin_amdgcn_s_memtime(); };
    auto stamp_sum = [&](int k, unsigned long long v) {
        if (tid == 0 && a.stamps) a.stamps[wg_lin * 8 + k] = v;
    };
#else
    auto stamp = [](int) {};
#endif
    stamp(0);
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kg = wave / NWT;                   // K-group
    const int twave = wave - kg * NWT;           // wave within the output tile
    const int wm = twave % WGM, wn = twave / WGM;
    const int h = lane >> 5, l32 = lane & 31;

    // 1-D grid, logical id remapped so that consecutive ids -- a tile's K-splits,
    // then neighbouring tiles -- land on one XCD (blocks are dealt round-robin
    // over the 8 XCDs): split-K slabs are summed out of the XCD's own L2.
    int lg = blockIdx.x;
    if ((gridDim.x & 7) == 0) lg = (lg & 7) * (gridDim.x >> 3) + (lg >> 3);
    lg = __builtin_amdgcn_readfirstlane(lg);
    const int tix = __builtin_amdgcn_readfirstlane(lg / a.S);          // tile (ticket) index
    const int split = __builtin_amdgcn_readfirstlane(lg - tix * a.S);
    const int bxy = __builtin_amdgcn_readfirstlane(tix % (a.gx * a.gy));
    const int b = __builtin_amdgcn_readfirstlane(tix / (a.gx * a.gy));
    const int by = __builtin_amdgcn_readfirstlane(bxy / a.gx);
    const int n0 = (bxy - by * a.gx) * BN;
    const int m0 = by * BM;
    const int mw = m0 + wm * WM;                 // this wave's first GEMM row
    const int c_begin = split * a.cps;
    const int c_end = min(a.nchunks, c_begin + a.cps);
    // input time of window row 0 (ConvT: group 0's window; group 1 reads one row later)
    const int tb = n0 * S - a.pad_l;
    const int gshift = (mw >= a.split_row) ? (a.pad_l - a.pad_g1) : 0;
    const int XW = a.XW;
    const int RL = XW * S;                        // raw row length (input samples)
    const int ta = XV ? (tb & ~3) : tb;           // DMA start (XV: 4-sample aligned)
    const int off0 = tb - ta;
    const int RS = XV ? ((RL + off0 + 3) & ~3) : RL;  // raw row stride (floats)
    const int P4 = XV ? RS / 4 : RS;              // DMA pieces per raw row
    const unsigned rl_magic = XV ? (unsigned)((0x100000000ull + P4 - 1) / P4) : a.rl_magic;
    const int ntask = XW * G8;
    const int ci_lim = min(a.c_in, c_end * CPC);  // window DMA past c_end lands zeros
    const u32x4_t xrs = raw_rsrc(a.x + (int64_t)b * a.x_sb, a.x_bytes);
    const float slope = a.act == RAVE_ACT_LEAKY ? a.slope : 1.0f;
    const u32x4_t wrs = raw_rsrc(a.w, a.w_bytes);
    // packed weights: [packed chunk][32-row block][KSC0 K-steps][hi|lo][64 lanes][8 halves]
    const unsigned wcstride = (unsigned)(a.MB * KSC0 * NPW) * 1024u;
    const unsigned wbase = (unsigned)((mw / 32) * KSC0 * NPW) * 1024u + (unsigned)lane * 16u;
    const uint32_t lds0 = lds_addr(smem);
    char* planes = smem + G::NS * G::STAGE;
    float* alpha_s = reinterpret_cast<float*>(smem + G::NS * G::STAGE + 2 * NP * G::XPLANE);
    if constexpr (SNAKE) {
        for (int i = tid; i < a.c_in; i += NT) alpha_s[i] = a.alpha[i];
    }
    // range guard: per-wave overflow votes of the chunk converted into plane
    // buffer pb at vote[pb * 16 + wave] (unused waves' bytes stay 0), wave maxima
    unsigned char* vote = reinterpret_cast<unsigned char*>(smem + G::VOTE);
    float* vred = reinterpret_cast<float*>(smem + G::VRED);
    if (tid < 12) reinterpret_cast<uint32_t*>(vote)[tid] = 0u;  // ordered by the prologue's first barrier

    floatx16 acc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // epilogue per-row constants, fetched now so their latency hides under the K loop
    float e_rs[NJ], e_bias[NJ];
    int e_co[NJ], e_q[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int m = mw + j * 32 + l32;
        e_rs[j] = m < a.Mpad ? a.rscale[m] : 0.f;   // tiles taller than the padded rows
        int co = m, q = 0;
        if (a.transposed) convt_row(a, m, co, q);
        e_co[j] = co;
        e_q[j] = q;
        const bool rowok = a.transposed ? co < a.bias_rows : m < a.M;
        e_bias[j] = (a.bias && rowok && a.S == 1) ? a.bias[co] : 0.f;
    }

    // window of chunk c -> ring slot (per-lane offsets, out-of-range -> zeros)
    const uint32_t dump = lds0 + G::NS * G::STAGE + 2 * NP * G::XPLANE + G::ALPHA;
    auto issue = [&](int c, int stage) __attribute__((always_inline)) {
        const uint32_t sbase = lds0 + stage * G::STAGE;
        const int ci0 = c * CPC;
#pragma unroll
        for (int i = 0; i < G::XI; ++i) {
            const int piece = i * NW + wave;
            const unsigned f = (unsigned)(piece * 64 + lane);
            const int cl = (int)__umulhi(f, rl_magic);
            const int tt = (int)f - cl * P4;
            const int ci = ci0 + cl;
            const int t = ta + tt * G::PF;
            const bool ok = (cl < CPC) && (ci < ci_lim) && (t >= 0) && (t < a.t_in);
            const unsigned voff = ok ? (unsigned)(ci * a.x_sc + t) * 4u : kOOB;
            const uint32_t dst = piece < G::NPIECE ? sbase + piece * G::PB : dump;
            if constexpr (XV) dma16b(xrs, voff, dst);
            else dma4(xrs, voff, dst);
        }
    };
    // this wave's weight fragments: register ring, one chunk ahead (chunks past
    // the packed image read zeros)
    // (slot = this group's local K-step; st = the chunk's K-step)
    u32x4_t wr[G::KS0][NJ][NPW];
    // (staged chunk c, K-step st = sub-chunk u, packed K-step s0)
    auto load_w = [&](int c, int slot, int st) __attribute__((always_inline)) {
        const int u = st / KSC0, s0 = st - u * KSC0;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int pl = 0; pl < NPW; ++pl)
                wr[slot][j][pl] = bload16(wrs, wbase + (unsigned)(c * VCX + u) * wcstride +
                                                   (unsigned)(((j * KSC0 + s0) * NPW + pl) * 1024));
    };
    // raw window of a stage -> activation (* xs) -> (hi, lo) f16 planes; returns
    // max |act| of the task's values (the range guard's vote input)
    auto convert_task = [&](int c, int stage, int pb, int i, float xs) __attribute__((always_inline)) {
        const float* raw = reinterpret_cast<const float*>(smem + stage * G::STAGE);
        _Float16* xh = reinterpret_cast<_Float16*>(planes + pb * NP * G::XPLANE);
        _Float16* xl = reinterpret_cast<_Float16*>(planes + pb * NP * G::XPLANE + G::XPLANE);
        _Float16* xm = reinterpret_cast<_Float16*>(planes + pb * NP * G::XPLANE + 2 * G::XPLANE);   // BF
        const int ci0 = c * CPC;
        float m = 0.f;
        {
            const int e = tid + i * NT;
            const int g = (int)(((unsigned)e * a.xw_magic) >> 24);
            const int w = e - g * XW;
            if (e < ntask) {
#ifdef RAVE_EXP_NOCVT
                // timing-only A/B variant (wrong results, never shipped): the planes
                // arrive ready-made, as a producer-side split would deliver them --
                // one 16-byte copy per plane row piece instead of act + split
                if constexpr (AR == 0 || AR == 2) {
                    const s_h8 r8 = *reinterpret_cast<const s_h8*>(raw + (g * 8 / S) * RS + off0 + w * S);
                    *reinterpret_cast<s_h8*>(xh + w * PH + g * 8) = r8;
                    *reinterpret_cast<s_h8*>(xl + w * PH + g * 8) = r8;
                    if constexpr (AR == 2) *reinterpret_cast<s_h8*>(xm + w * PH + g * 8) = r8;
                    return m;
                }
#endif
                s_f32x8 v8;
#pragma unroll
                for (int v = 0; v < 8; ++v) {
                    const int vc = g * 8 + v;
                    float val = raw[(vc / S) * RS + off0 + w * S + (vc % S)];
                    if constexpr (SNAKE) {
                        const float al = alpha_s[min(ci0 + vc / S, a.c_in - 1)];
                        val = val + (1.0f / (al + 1e-9f)) * sin_squared(al * val);
                    } else {
                        val = fmaxf(val, val * slope);     // leaky ReLU, slope <= 1 (host check)
                    }
                    v8[v] = val * xs;
                }
                if constexpr (F32) {
                    float* xf = reinterpret_cast<float*>(planes + pb * NP * G::XPLANE);
                    *reinterpret_cast<s_f32x4*>(xf + w * PH + g * 8) = s_f32x4{v8[0], v8[1], v8[2], v8[3]};
                    *reinterpret_cast<s_f32x4*>(xf + w * PH + g * 8 + 4) = s_f32x4{v8[4], v8[5], v8[6], v8[7]};
                } else if constexpr (BF) {
                    s_b8 hi, mid, lo;
                    s_bf3_split(v8, hi, mid, lo);
                    *reinterpret_cast<s_b8*>(xh + w * PH + g * 8) = hi;
                    *reinterpret_cast<s_b8*>(xl + w * PH + g * 8) = lo;
                    *reinterpret_cast<s_b8*>(xm + w * PH + g * 8) = mid;
                } else {
                    m = absmax8(v8);
                    const s_h8 hi = __builtin_convertvector(v8, s_h8);
                    const s_h8 lo = __builtin_convertvector((v8 - __builtin_convertvector(hi, s_f32x8)) * 2048.0f, s_h8);
                    *reinterpret_cast<s_h8*>(xh + w * PH + g * 8) = hi;
                    *reinterpret_cast<s_h8*>(xl + w * PH + g * 8) = lo;
                }
            }
        }
        return m;
    };
    auto convert = [&](int c, int stage, int pb) __attribute__((always_inline)) {
        float m = 0.f;
#pragma unroll
        for (int i = 0; i < XT; ++i) m = fmaxf(m, convert_task(c, stage, pb, i, 1.0f));
        return m;
    };
    // range guard.  vote: after a chunk's conversion into plane buffer pb, each
    // wave records whether any of its values reached kSplitLimit.  After the
    // barrier every wave reads the votes (one 16-byte LDS read); only when one
    // is set does the workgroup take the rare path: the wave maxima of the
    // conversion meet in LDS, the chunk is re-converted as act * 2^-s and the
    // chunk's K-steps run on acc * 2^-s, scaled back by 2^s after them (exact).
    auto cast_vote = [&](int pb, float m) __attribute__((always_inline)) {
        if (!RAVE_SPLIT_GUARD) return;
        const bool over = __builtin_amdgcn_ballot_w64(m >= kSplitLimit) != 0;
        if (lane == 0) vote[pb * 16 + wave] = over ? 1 : 0;
    };
    auto read_vote = [&](int pb) __attribute__((always_inline)) {
        if (!RAVE_SPLIT_GUARD) return false;
        const uint32_t* v = reinterpret_cast<const uint32_t*>(vote + pb * 16);
        return __builtin_amdgcn_readfirstlane((v[0] | v[1] | v[2] | v[3]) != 0u ? 1 : 0) != 0;
    };
    auto rescue = [&](int c, int stage, int pb, float m) __attribute__((always_inline)) {
        m = wave_max(m);
        if (lane == 0) vred[wave] = m;
        __syncthreads();
        float mx = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) mx = fmaxf(mx, vred[w]);
        const int sh = __builtin_amdgcn_readfirstlane(split_shift(mx));
        const float xs = ldexpf(1.0f, -sh);
#pragma nounroll
        for (int i = 0; i < XT; ++i) (void)convert_task(c, stage, pb, i, xs);
        __syncthreads();
        return sh;
    };
    auto scale_acc = [&](float f) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] *= f;
    };

    // per-lane A-fragment offsets (halves): window row wn*WN + l32 + q*d (+ group shift)
    int xoff[G::Q];
#pragma unroll
    for (int q = 0; q < G::Q; ++q) xoff[q] = (wn * WN + l32 + q * a.d + gshift) * PH + 8 * h;

    struct AFrag {
        s_h8 h[NI], l[NI], m[NI];
    };
    auto read_a = [&](int pb, int st, AFrag& f) __attribute__((always_inline)) {
        const int u = st / KSC0, s0 = st - u * KSC0;
        const int q = s0 / HPS0, hv = u * (VC0 / 16) + (s0 - q * HPS0);   // 16-channel column group
        const _Float16* xh = reinterpret_cast<const _Float16*>(planes + pb * NP * G::XPLANE);
        const _Float16* xl = reinterpret_cast<const _Float16*>(planes + pb * NP * G::XPLANE + G::XPLANE);
        const _Float16* xm = reinterpret_cast<const _Float16*>(planes + pb * NP * G::XPLANE + 2 * G::XPLANE);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if constexpr (F32) {   // 8 floats: channels 8h..8h+7 of the step's 16 (xoff counts floats)
                const float* xf = reinterpret_cast<const float*>(planes + pb * NP * G::XPLANE) + xoff[q] + i * 32 * PH +
                                  hv * 16;
                f.h[i] = *reinterpret_cast<const s_h8*>(xf);
                f.l[i] = *reinterpret_cast<const s_h8*>(xf + 4);
            } else {
                f.h[i] = *reinterpret_cast<const s_h8*>(xh + xoff[q] + i * 32 * PH + hv * 16);
                f.l[i] = *reinterpret_cast<const s_h8*>(xl + xoff[q] + i * 32 * PH + hv * 16);
                if constexpr (BF) f.m[i] = *reinterpret_cast<const s_h8*>(xm + xoff[q] + i * 32 * PH + hv * 16);
            }
        }
    };

    // ------------------------------------------------------------ prologue + K loop
    // vmcnt bookkeeping (every load below is hand-counted asm): per chunk a
    // wave issues XI window DMAs, then per own K-step 2*NJ weight loads.  The
    // body is instantiated per K-group (its K-step range fixes the counts);
    // both groups pass the same barriers.
    // GUARDED (compile time): the per-chunk range guard of the rare second
    // attempt; the first attempt's loop carries no guard code at all
    auto body = [&](auto gtag, auto guardtag) __attribute__((always_inline)) {
        constexpr int GG = decltype(gtag)::value;
        constexpr bool guarded = decltype(guardtag)::value != 0;
        constexpr int KS = G::ks_of(GG);                // own K-steps per chunk
        constexpr int ST0 = G::st_of(GG);               // first own K-step
        constexpr int WR = KS * NJ * NPW, XI = G::XI;
#pragma unroll
        for (int i = 0; i < NS; ++i) issue(c_begin + i, i);
#pragma unroll
        for (int k = 0; k < KS; ++k) load_w(c_begin, k, ST0 + k);
        wait_vm<(NS - 1) * XI + WR>();          // window c_begin landed
        __syncthreads();
        float cmax = convert(c_begin, 0, 0);
        if constexpr (guarded) cast_vote(0, cmax);
        wait_vm<(NS - 2) * XI + WR>();          // window c_begin+1 landed
        __syncthreads();
        stamp(1);

        // per chunk c: DMA window c+NS into window c's slot (split during chunk
        // c-1) | own K-steps (weights of c from the ring, refill with c+1) | split
        // window c+1 into the other plane pair | wait + barrier
        // (a do-while: every split owns >= 1 chunk, S = ceil(nchunks / cps) on the
        // host, so no zero-trip path leaves the ring's loads outstanding)
        int stage = 0;
        int c = c_begin;
        do {
            const int pb = (c - c_begin) & 1;
            const int s1 = stage + 1 == NS ? 0 : stage + 1;
            AFrag f[2];
            read_a(pb, ST0, f[0]);
            // range guard of chunk c (converted during chunk c-1 or the prologue;
            // its raw window is still in `stage` until the DMA below): the vote
            // read rides with the first fragment reads
            int sh_cur = 0;
            if (guarded && __builtin_expect(read_vote(pb), 0)) {
                sh_cur = rescue(c, stage, pb, cmax);
                read_a(pb, ST0, f[0]);
            }
            issue(c + NS, stage);
            if (__builtin_expect(sh_cur != 0, 0)) scale_acc(ldexpf(1.0f, -sh_cur));
            cmax = 0.f;
#pragma unroll
            for (int k = 0; k < KS; ++k) {
                if (k + 1 < KS) read_a(pb, ST0 + k + 1, f[(k + 1) & 1]);   // next reads in flight
                // weights of (c, k): issued one chunk ago; younger: the rest of that
                // chunk's weights, this chunk's window DMA and this chunk's earlier refills
#ifdef RAVE_STAMPS
                const unsigned long long tw0 = now();
#endif
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    if constexpr (BF && !W4) wait_vm_regs3<WR - NPW * NJ + XI>(wr[k][j][0], wr[k][j][1], wr[k][j][2]);
                    else wait_vm_regs<WR - NPW * NJ + XI>(wr[k][j][0], wr[k][j][1]);
                }
#ifdef RAVE_STAMPS
                acc_ww += now() - tw0;
#endif
                __builtin_amdgcn_sched_barrier(0);
                const AFrag& g = f[k & 1];
                if constexpr (BF) {
                    // the weight parts: from the image, or (W4) split from its 8 fp32 values
                    s_b8 wh[NJ], wl[NJ], wmd[NJ];
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        if constexpr (W4) {
                            const s_f32x4 u0 = __builtin_bit_cast(s_f32x4, wr[k][j][0]);
                            const s_f32x4 u1 = __builtin_bit_cast(s_f32x4, wr[k][j][1]);
                            s_bf3_split(s_f32x8{u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]}, wh[j], wmd[j],
                                        wl[j]);
                        } else {
                            wh[j] = __builtin_bit_cast(s_b8, wr[k][j][0]);
                            wl[j] = __builtin_bit_cast(s_b8, wr[k][j][1]);
                            wmd[j] = __builtin_bit_cast(s_b8, wr[k][j][NPW - 1]);
                        }
                    }
                    // smallest products first: (x, w) = hi*lo, lo*hi, mid*mid, hi*mid, mid*hi, hi*hi
#pragma unroll
                    for (int i = 0; i < NI; ++i)
#pragma unroll
                        for (int j = 0; j < NJ; ++j) {
                            const s_b8 xh8 = __builtin_bit_cast(s_b8, g.h[i]), xl8 = __builtin_bit_cast(s_b8, g.l[i]),
                                       xm8 = __builtin_bit_cast(s_b8, g.m[i]);
                            const s_b8 wh8 = wh[j], wl8 = wl[j], wm8 = wmd[j];
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh8, wl8, acc[i][j], 0, 0, 0);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl8, wh8, acc[i][j], 0, 0, 0);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xm8, wm8, acc[i][j], 0, 0, 0);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh8, wm8, acc[i][j], 0, 0, 0);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xm8, wh8, acc[i][j], 0, 0, 0);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh8, wh8, acc[i][j], 0, 0, 0);
                        }
                } else if constexpr (F32) {
#pragma unroll
                    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                        for (int e = 0; e < 4; ++e)
#pragma unroll
                            for (int i = 0; i < NI; ++i)
#pragma unroll
                                for (int j = 0; j < NJ; ++j) {
                                    const s_f32x4 av = __builtin_bit_cast(s_f32x4, hf ? g.l[i] : g.h[i]);
                                    const s_f32x4 bv = __builtin_bit_cast(s_f32x4, wr[k][j][hf]);
                                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], bv[e], acc[i][j], 0, 0, 0);
                                }
                } else {
                    s_h8 bh[NJ], bl[NJ], b2[NJ];
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        bh[j] = __builtin_bit_cast(s_h8, wr[k][j][0]);
                        bl[j] = __builtin_bit_cast(s_h8, wr[k][j][1]);
                        b2[j] = bh[j] * (_Float16)2048.0f;
                    }
#pragma unroll
                    for (int i = 0; i < NI; ++i)
#pragma unroll
                        for (int j = 0; j < NJ; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(g.h[i], b2[j], acc[i][j], 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < NI; ++i)
#pragma unroll
                        for (int j = 0; j < NJ; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(g.l[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < NI; ++i)
#pragma unroll
                        for (int j = 0; j < NJ; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(g.h[i], bl[j], acc[i][j], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
                load_w(c + 1, k, ST0 + k);      // refill the slot one chunk ahead
                // split part of window c+1 into the other plane pair (VALU beside the MFMAs)
                if (c + 1 < c_end) {
#pragma unroll
                    for (int i = k; i < XT; i += KS) cmax = fmaxf(cmax, convert_task(c + 1, s1, pb ^ 1, i, 1.0f));
                }
            }
            if (__builtin_expect(sh_cur != 0, 0)) scale_acc(ldexpf(1.0f, sh_cur));
            if constexpr (guarded) {
                if (c + 1 < c_end) cast_vote(pb ^ 1, cmax);
            }
            // window c+2 landed: younger are, per chunk since its issue, the
            // weight refills and the next windows
#ifdef RAVE_STAMPS
            const unsigned long long te0 = now();
#endif
            wait_vm<(NS - 1) * WR + (NS - 2) * XI>();
            __syncthreads();
#ifdef RAVE_STAMPS
            acc_we += now() - te0;
#endif
            stage = s1;
            if (c == c_begin) stamp(2);
        } while (++c < c_end);
        // drain the ring (its last refills read past the image): the registers
        // stay tied up to the wait, so nothing reuses them while a refill lands
        wait_vm<0>();
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int pl = 0; pl < NPW; ++pl) ring_keep(wr[k][j][pl]);
    };
    // Range guard, two attempts: the first runs the plain K loop (no guard
    // code); an operand past the f16 range became inf in its hi half, so it
    // shows as a non-finite partial sum.  Only when some wave of the tile holds
    // one (one vote per tile) does the loop run again from its prologue with
    // the per-chunk rescue (rare: activations past 2^15; a genuine inf / NaN
    // input takes the second attempt too and passes through, as in fp32).
    auto run_k = [&](auto guardtag) __attribute__((always_inline)) {
        if (kg == 0) body(IC<0>{}, guardtag);
        else if constexpr (KG >= 2) {
            if (kg == 1) body(IC<1>{}, guardtag);
            else if constexpr (KG == 4) {
                if (kg == 2) body(IC<2>{}, guardtag);
                else body(IC<3>{}, guardtag);
            }
        }
    };
    run_k(IC<0>{});
    if (RAVE_SPLIT_GUARD && AR == 0) {
        bool bad = false;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) bad |= !__builtin_isfinite(acc[i][j][r]);
        const bool wover = __builtin_amdgcn_ballot_w64(bad) != 0;
        if (lane == 0) vote[32 + wave] = wover ? 1 : 0;
        __syncthreads();
        if (__builtin_expect(vote_any<NW>(vote + 32), 0)) {
            __syncthreads();                // every wave read the tile vote
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
            run_k(IC<1>{});
        }
    }
    stamp(3);
#ifdef RAVE_STAMPS
    stamp_sum(5, acc_ww);
    stamp_sum(6, acc_we);
#endif
#ifndef RAVE_CONV_KGPAR
#define RAVE_CONV_KGPAR 1
#endif
    if constexpr (KG >= 2 && RAVE_CONV_KGPAR != 0) {
        // Plain output (no ConvT interleave, no split-K slab, aligned rows), round 6:
        // every K-group parks its partial tile in LDS in the row-major layout the
        // stores read, and every wave -- not only group 0 -- finishes 1/KG of its
        // tile's rows: the partials summed in group order (((p0 + p1) + p2) + p3,
        // bitwise the group-0 reduction), row scale + bias, residual, 16-byte
        // stores.  The reduction reads, residual loads and stores are spread over
        // KG times as many waves.
        if (!a.transposed && a.S == 1 && a.vec_y) {
            constexpr int LPR = WN / 4;                  // lanes per row
            constexpr int RPI = 64 / LPR;                // rows per instruction
            constexpr int RW = WM / KG;                  // rows this wave finishes
            static_assert(RW % RPI == 0, "K-group row shares");
            const int rr = lane / LPR, cc = (lane % LPR) * 4;
            const int n = n0 + wn * WN + cc;
            const int rbase = kg * RW;
            // row constants and residual of the wave's rows, in flight across the barriers
            float rs_r[RW / RPI], bias_r[RW / RPI];
            s_f32x4 rv[RW / RPI];
            const __amdgpu_buffer_rsrc_t rrs = make_rsrc(a.res ? a.res + (int64_t)b * a.r_sb : a.y, a.res ? a.r_bytes : 0);
#pragma unroll
            for (int it = 0; it < RW / RPI; ++it) {
                const int m = mw + rbase + it * RPI + rr;
                rs_r[it] = m < a.Mpad ? a.rscale[m] : 0.f;
                bias_r[it] = (a.bias && m < a.M) ? a.bias[m] : 0.f;
                const bool ok = a.res && m < a.M && n + 3 < a.U;
                rv[it] = __builtin_bit_cast(s_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                    rrs, ok ? (unsigned)(m * a.r_sc + n) * 4u : kOOB, 0, 0));
            }
            __syncthreads();                             // ring and planes dead
            float* et = reinterpret_cast<float*>(smem) + wave * WM * G::EROW;
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int i = 0; i < NI; ++i)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const s_f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2],
                                           acc[i][j][4 * g + 3]};
                        *reinterpret_cast<s_f32x4*>(et + (j * 32 + l32) * G::EROW + i * 32 + 8 * g + 4 * h) = v;
                    }
            __syncthreads();                             // every group's partial tile parked
            const __amdgpu_buffer_rsrc_t yrs = make_rsrc(a.y + (int64_t)b * a.y_sb, a.y_bytes);
#pragma unroll
            for (int it = 0; it < RW / RPI; ++it) {
                const int r = rbase + it * RPI + rr;
                const int m = mw + r;
                s_f32x4 v = *reinterpret_cast<const s_f32x4*>(reinterpret_cast<const float*>(smem) +
                                                               (size_t)twave * WM * G::EROW + r * G::EROW + cc);
#pragma unroll
                for (int g = 1; g < KG; ++g)
                    v += *reinterpret_cast<const s_f32x4*>(reinterpret_cast<const float*>(smem) +
                                                           (size_t)(twave + g * NWT) * WM * G::EROW + r * G::EROW + cc);
                v = v * rs_r[it] + bias_r[it];
                if (m < a.M && n + 3 < a.U) {
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v + rv[it]), yrs,
                                                           (unsigned)(m * a.y_sc + n) * 4u, 0, RAVE_YAUX);
                } else {
                    float vv[4];
                    *reinterpret_cast<s_f32x4*>(vv) = v;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const bool ok = m < a.M && n + e < a.U;
                        const float rsd = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                            rrs, ok ? (unsigned)(m * a.r_sc + n + e) * 4u : kOOB, 0, 0));
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, vv[e] + rsd), yrs,
                                                              ok ? (unsigned)(m * a.y_sc + n + e) * 4u : kOOB, 0, RAVE_YAUX);
                    }
                }
            }
            stamp(4);
            return;
        }
    }
    if constexpr (KG >= 2) {
        // groups 1.. hand their partial tiles to group 0 through LDS (ring and
        // planes are dead); group 0 adds them in group order (fixed: bitwise
        // reproducible).  The others then run the epilogue's barriers with their
        // stores muted ("live" below).
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem) + (size_t)wave * WM * G::EROW;
        if (kg != 0) {
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) red[((i * NJ + j) * 16 + r) * 64 + lane] = acc[i][j][r];
        }
        __syncthreads();
        if (kg == 0) {
#pragma unroll
            for (int g = 1; g < KG; ++g) {
                const float* o = reinterpret_cast<const float*>(smem) + (size_t)(wave + g * NWT) * WM * G::EROW;
#pragma unroll
                for (int i = 0; i < NI; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) acc[i][j][r] += o[((i * NJ + j) * 16 + r) * 64 + lane];
            }
        }
        __syncthreads();                    // partner areas read before the epilogue reuses LDS
    }

    // ---------------------------------------------------------------- epilogue
    // lane = one GEMM row per m-block; registers 4g..4g+3 of a block = 4 consecutive columns
    const bool partial = a.S > 1;
    const bool live = KG == 1 || kg == 0;   // the wave that stores its tile
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = acc[i][j][r] * e_rs[j] + e_bias[j];
    }
    if (!a.transposed || partial) {     // (split-K slabs are GEMM rows even for ConvT)
        // Row-contiguous stores: each wave parks its WM x WN tile in LDS (the
        // ring is dead) and re-reads it so that a store instruction writes whole
        // rows (the accumulator layout gives 16-byte pieces of 32 rows).
        __syncthreads();
        float* et = reinterpret_cast<float*>(smem) + wave * WM * G::EROW;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const s_f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2],
                                       acc[i][j][4 * g + 3]};
                    *reinterpret_cast<s_f32x4*>(et + (j * 32 + l32) * G::EROW + i * 32 + 8 * g + 4 * h) = v;
                }
        __builtin_amdgcn_s_waitcnt(0xc07f);          // lgkmcnt(0): own writes landed (wave-private area)
        constexpr int LPR = WN / 4;                  // lanes per row
        constexpr int RPI = 64 / LPR;                // rows per instruction
        const int rr = lane / LPR, cc = (lane % LPR) * 4;
        const int n = n0 + wn * WN + cc;
        if (partial) {
            const __amdgpu_buffer_rsrc_t prs = make_rsrc(
                a.partial + ((int64_t)split * a.B + b) * (int64_t)a.M * a.U, a.M * a.U * 4);
#pragma unroll
            for (int it = 0; it < WM / RPI; ++it) {
                if (!live) break;
                const int r = it * RPI + rr;
                const int m = mw + r;
                const float* vp = et + r * G::EROW + cc;
                if (a.vec_p && m < a.M && n + 3 < a.U) {
                    __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4_t*>(vp), prs,
                                                           (unsigned)(m * a.U + n) * 4u, 0, 0);
                } else {
                    // element-wise tail (no ext-vector lane indexing here: hipcc
                    // miscompiled v[e] of an LDS-loaded vector in this branch)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const unsigned off = (m < a.M && n + e < a.U) ? (unsigned)(m * a.U + n + e) * 4u : kOOB;
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, vp[e]), prs, off, 0, 0);
                    }
                }
            }
            if (!a.inlaunch) {
                stamp(4);
                return;
            }
            // In-launch combine (guide §5 "In-launch split-K reduction"): publish the
            // slab with an agent-scope release, draw a ticket; the split that draws
            // S-1 acquires and sums every slab of the tile in split order.
            wait_vm<0>();
            __syncthreads();
            volatile int* last_s = reinterpret_cast<volatile int*>(smem + G::LDS);
            if (tid == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                wait_vm<0>();
                const int prev = __hip_atomic_fetch_add(a.tickets + tix, 1, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
                const int last = prev == a.S - 1;
                if (last) {
                    __hip_atomic_store(a.tickets + tix, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    wait_vm<0>();
                }
                *last_s = last;
            }
            __syncthreads();
            if (!*last_s) {
                stamp(4);
                return;
            }
            if (!live) {
                stamp(4);
                return;                             // (no barrier follows)
            }
            constexpr int IT = WM / RPI;
            s_f32x4 sum[IT];
#pragma unroll
            for (int it = 0; it < IT; ++it) sum[it] = s_f32x4{0.f, 0.f, 0.f, 0.f};
            for (int s = 0; s < a.S; ++s) {        // slabs outer: IT independent loads per round trip
                const __amdgpu_buffer_rsrc_t srs = make_rsrc(
                    a.partial + ((int64_t)s * a.B + b) * (int64_t)a.M * a.U, a.M * a.U * 4);
                s_f32x4 pv[IT];
#pragma unroll
                for (int it = 0; it < IT; ++it) {
                    const int m = mw + it * RPI + rr;
                    const bool ok = m < a.M && n < a.U;          // U % 4 == 0 here (vec_p)
                    pv[it] = __builtin_bit_cast(s_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                        srs, ok ? (unsigned)(m * a.U + n) * 4u : kOOB, 0, 0));
                }
#pragma unroll
                for (int it = 0; it < IT; ++it) sum[it] += pv[it];
            }
            // then the separate reduce's store_out: + bias, + residual, ConvT interleave
            if (!a.transposed && a.vec_y) {
                const __amdgpu_buffer_rsrc_t yrs = make_rsrc(a.y + (int64_t)b * a.y_sb, a.y_bytes);
                const __amdgpu_buffer_rsrc_t rrs =
                    make_rsrc(a.res ? a.res + (int64_t)b * a.r_sb : a.y, a.res ? a.r_bytes : 0);
                s_f32x4 rv[IT];
#pragma unroll
                for (int it = 0; it < IT; ++it) {
                    const int m = mw + it * RPI + rr;
                    const bool ok = a.res && m < a.M && n < a.U;
                    rv[it] = __builtin_bit_cast(s_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                        rrs, ok ? (unsigned)(m * a.r_sc + n) * 4u : kOOB, 0, 0));
                }
#pragma unroll
                for (int it = 0; it < IT; ++it) {
                    const int m = mw + it * RPI + rr;
                    if (m < a.M && n < a.U) {
                        s_f32x4 v = sum[it];
                        if (a.bias) v += a.bias[m];
                        if (a.res) v += rv[it];
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), yrs,
                                                               (unsigned)(m * a.y_sc + n) * 4u, 0, RAVE_YAUX);
                    }
                }
            } else {
#pragma unroll
                for (int it = 0; it < IT; ++it) {
                    const int m = mw + it * RPI + rr;
                    float vv[4];
                    *reinterpret_cast<s_f32x4*>(vv) = sum[it];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (m < a.M && n + e < a.U) store_out(a, b, m, n + e, vv[e]);
                }
            }
            stamp(4);
            return;
        }
        if (!live) return;                          // (no barrier follows)
        const __amdgpu_buffer_rsrc_t yrs = make_rsrc(a.y + (int64_t)b * a.y_sb, a.y_bytes);
        const __amdgpu_buffer_rsrc_t rrs = make_rsrc(a.res ? a.res + (int64_t)b * a.r_sb : a.y, a.res ? a.r_bytes : 0);
        if (a.vec_y) {
            s_f32x4 rv[WM / RPI];
#pragma unroll
            for (int it = 0; it < WM / RPI; ++it) {  // every residual load before the first store
                const int m = mw + it * RPI + rr;
                const bool ok = a.res && m < a.M && n + 3 < a.U;
                rv[it] = __builtin_bit_cast(s_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                    rrs, ok ? (unsigned)(m * a.r_sc + n) * 4u : kOOB, 0, 0));
            }
#pragma unroll
            for (int it = 0; it < WM / RPI; ++it) {
                const int r = it * RPI + rr;
                const int m = mw + r;
                const s_f32x4 v = *reinterpret_cast<const s_f32x4*>(et + r * G::EROW + cc) + rv[it];
                if (m < a.M && n + 3 < a.U) {
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), yrs,
                                                           (unsigned)(m * a.y_sc + n) * 4u, 0, RAVE_YAUX);
                } else {
                    float vv[4];
                    *reinterpret_cast<s_f32x4*>(vv) = *reinterpret_cast<const s_f32x4*>(et + r * G::EROW + cc);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const bool ok = m < a.M && n + e < a.U;
                        const float rs = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                            rrs, ok ? (unsigned)(m * a.r_sc + n + e) * 4u : kOOB, 0, 0));
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, vv[e] + rs), yrs,
                                                              ok ? (unsigned)(m * a.y_sc + n + e) * 4u : kOOB, 0, RAVE_YAUX);
                    }
                }
            }
        } else {                                    // unaligned rows: element-wise
#pragma unroll
            for (int it = 0; it < WM / RPI; ++it) {
                const int r = it * RPI + rr;
                const int m = mw + r;
                const float* vp = et + r * G::EROW + cc;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const bool ok = m < a.M && n + e < a.U;
                    const float rs = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                        rrs, ok ? (unsigned)(m * a.r_sc + n + e) * 4u : kOOB, 0, 0));
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, vp[e] + rs), yrs,
                                                          ok ? (unsigned)(m * a.y_sc + n + e) * 4u : kOOB, 0, RAVE_YAUX);
                }
            }
        }
        stamp(4);
        return;
    }
    if (!live) return;
    const __amdgpu_buffer_rsrc_t yrs = make_rsrc(a.y + (int64_t)b * a.y_sb, a.y_bytes);
    {   // ConvTranspose: phase-interleaved columns t = n*R + q, one store per element
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int co = e_co[j], q = e_q[j];
            const bool rowok = co < a.bias_rows;
            const float bv = 0.f;   // added above
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int n = n0 + wn * WN + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const int t = n * a.R + q;
                    const unsigned off = (rowok && n < a.U && t < a.t_y) ? (unsigned)(co * a.y_sc + t) * 4u : kOOB;
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, acc[i][j][r] + bv), yrs, off, 0, RAVE_YAUX);
                }
        }
        stamp(4);
    }
}

template <int KT, int BM, int BN, int WM, bool SNAKE, bool XV, int KG, int WN_, int VCX, int NS>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN_) * KG) void conv1d_split_kernel(ConvKArgs a) {
    conv1d_split_body<KT, BM, BN, WM, SNAKE, XV, KG, WN_, VCX, NS, 0>(a);
}
template <int KT, int BM, int BN, int WM, bool SNAKE, bool XV, int KG, int WN_, int VCX, int NS>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN_) * KG) void conv1d_ring_f32_kernel(ConvKArgs a) {
    conv1d_split_body<KT, BM, BN, WM, SNAKE, XV, KG, WN_, VCX, NS, 1>(a);
}
template <int KT, int BM, int BN, int WM, bool SNAKE, bool XV, int KG, int WN_, int VCX, int NS>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN_) * KG) void conv1d_bf3_kernel(ConvKArgs a) {
    conv1d_split_body<KT, BM, BN, WM, SNAKE, XV, KG, WN_, VCX, NS, 2>(a);
}

// --------------------------------------------------------------------- tiles
struct SplitCfg {
    int tile, S, sep;     // kSplitTiles index, K-splits, separate reduce launch
};

// Tiles (BM rows x BN columns, wave WM x WN, KG waves per output tile, VCX
// packed chunks per staged chunk).  The table index is part of the
// launch-configuration code.  Slots 10-15 are round 1's 32 x 64 wave tiles
// (what the autotuner picks on every RAVE layer, profiles/r01_final/
// tuning.json); slots 0-7 (round 1's retired 64-row / 128-column wave tiles,
// which never won) now hold the wide-chunk tiles for the short-N layers:
// two or four K-groups on 2- or 4-chunk windows; slot 4 stages 4 packed chunks
// in a two-slot ring (NS = 2: the LDS of a third slot buys the wider chunk;
// picked for the ConvT / strided layers and some C = 512 k3).  Slot 6 (32 x 64,
// four K-groups, 4-chunk windows) measured no better than these on any v2 layer
// and is not built; neither are 64-row wave tiles with K-groups or eight
// K-groups on 4/8-chunk windows, tried in round 2.  Slots
// 8-9 (round 2, last session): 256-column tiles of 32x64 waves for the layers
// with few rows and a long time axis (the edge convs, the C = 64 ConvT), so
// that one round of workgroups covers the layer.  Only
// the rows marked built are instantiated.  Split-K counts of wide-chunk tiles
// are in staged chunks.  Round 5 (build time): slots 3, 5, 7 and 13, which no
// committed tuning (profiles/tuning/, every pinned and candidate file of rounds
// 3-4) ever picked, are no longer built, and the 4-byte window DMA form (XV =
// false: unaligned input rows, split16 only) is built for the KG = 1 tiles
// (8-12), the heuristic's set.
constexpr int kNumSplitTiles = 16;
[[maybe_unused]] constexpr int kSplitTiles[kNumSplitTiles][7] = {   // BM, BN, WM, KG, WN, VCX, NS
    {64, 64, 32, 4, 64, 2, 3},   {64, 64, 32, 4, 64, 4, 3},   {128, 64, 32, 2, 64, 2, 3},  {32, 64, 32, 4, 64, 2, 3},
    {64, 64, 32, 4, 64, 4, 2},   {64, 128, 32, 2, 64, 2, 3},  {32, 64, 32, 4, 64, 4, 3},   {64, 64, 32, 2, 64, 2, 3},
    {32, 256, 32, 1, 64, 1, 3},  {64, 256, 32, 1, 64, 1, 3},  {128, 64, 32, 1, 64, 1, 3},  {64, 128, 32, 1, 64, 1, 3},
    {256, 64, 32, 1, 64, 1, 3},  {256, 64, 32, 2, 64, 1, 3},  {128, 64, 32, 2, 64, 1, 3},  {64, 128, 32, 2, 64, 1, 3}};
[[maybe_unused]] constexpr bool kSplitTileBuilt[kNumSplitTiles] = {true,  true,  true,  false, true,  false, false, false,
                                                  true,  true,  true,  true,  true,  false, true,  true};
// the 4-byte window DMA form (unaligned rows) is built for the KG = 1 tiles only
[[maybe_unused]] static constexpr bool split_tile_xv0(int ti) { return kSplitTiles[ti][3] == 1; }
[[maybe_unused]] constexpr int kSplitDefaultTile = 10;

// Calls f(IC<BM>, IC<BN>, IC<WM>, IC<KG>, IC<WN>, IC<VCX>, IC<NS>) for a built tile
// index ti (compile-time dispatch; callers check kSplitTileBuilt first).
template <typename Fn>
static inline auto with_tile(int ti, Fn&& f) {
    switch (ti) {
        case 0: return f(IC<64>{}, IC<64>{}, IC<32>{}, IC<4>{}, IC<64>{}, IC<2>{}, IC<3>{});
        case 1: return f(IC<64>{}, IC<64>{}, IC<32>{}, IC<4>{}, IC<64>{}, IC<4>{}, IC<3>{});
        case 2: return f(IC<128>{}, IC<64>{}, IC<32>{}, IC<2>{}, IC<64>{}, IC<2>{}, IC<3>{});
        case 4: return f(IC<64>{}, IC<64>{}, IC<32>{}, IC<4>{}, IC<64>{}, IC<4>{}, IC<2>{});
        case 8: return f(IC<32>{}, IC<256>{}, IC<32>{}, IC<1>{}, IC<64>{}, IC<1>{}, IC<3>{});
        case 9: return f(IC<64>{}, IC<256>{}, IC<32>{}, IC<1>{}, IC<64>{}, IC<1>{}, IC<3>{});
        case 11: return f(IC<64>{}, IC<128>{}, IC<32>{}, IC<1>{}, IC<64>{}, IC<1>{}, IC<3>{});
        case 12: return f(IC<256>{}, IC<64>{}, IC<32>{}, IC<1>{}, IC<64>{}, IC<1>{}, IC<3>{});
        case 14: return f(IC<128>{}, IC<64>{}, IC<32>{}, IC<2>{}, IC<64>{}, IC<1>{}, IC<3>{});
        case 15: return f(IC<64>{}, IC<128>{}, IC<32>{}, IC<2>{}, IC<64>{}, IC<1>{}, IC<3>{});
        default: return f(IC<128>{}, IC<64>{}, IC<32>{}, IC<1>{}, IC<64>{}, IC<1>{}, IC<3>{});   // 10
    }
}

// Launch of one (family, activation) for a tile index.  The kernel
// instantiations are spread over separate translation units (the Makefile
// compiles this file once per (KT, SNAKE, XV) with -DRAVE_SPLIT_KT / _SNAKE / _XV,
// and once without them for the host side) so the build runs in parallel.
template <int KT, bool SNAKE, bool XV, int AR>
int split_launch_inst(ConvKArgs k, int tile, hipStream_t st);

#ifdef RAVE_SPLIT_KT
template <int KT, int BM, int BN, int WM, int KG, int WN, int VCX, int NS, bool SNAKE, bool XV, int AR>
static int split_launch_xv(ConvKArgs k, hipStream_t st) {
    using G = SGeo<KT, BM, BN, WM, XV, KG, WN, VCX, NS, AR == 2 ? 3 : 2>;
    if constexpr (!G::VALID) {
        set_error("conv1d(split16): tile exceeds LDS or the vmcnt range");
        return RAVE_ERR_UNSUPPORTED;
    } else if constexpr (!XV && KG != 1) {
        set_error("conv1d(split16): unaligned input rows run the KG = 1 tiles only");
        return RAVE_ERR_UNSUPPORTED;
    } else {
        if (k.XW > G::XW_MAX) {
            set_error("conv1d(split16): dilation too large for the staged window");
            return RAVE_ERR_UNSUPPORTED;
        }
        constexpr size_t lds = (size_t)G::LDS_ALL;
        static_assert(lds <= 160 * 1024, "LDS budget");
        dim3 grid(k.gx * k.gy * k.B * k.S);
        auto kern = [] {
            if constexpr (AR == 2) return conv1d_bf3_kernel<KT, BM, BN, WM, SNAKE, XV, KG, WN, VCX, NS>;
            else if constexpr (AR == 1) return conv1d_ring_f32_kernel<KT, BM, BN, WM, SNAKE, XV, KG, WN, VCX, NS>;
            else return conv1d_split_kernel<KT, BM, BN, WM, SNAKE, XV, KG, WN, VCX, NS>;
        }();
        if (lds > 64 * 1024) {
            static bool done = false;
            if (!done) {
                RAVE_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                done = true;
            }
        }
        launch(kern, grid, dim3(G::NT), (uint32_t)lds, st, k);
        return launch_status(AR == 2 ? "conv1d_bf3_kernel" : AR == 1 ? "conv1d_ring_f32_kernel" : "conv1d_split_kernel");
    }
}

template <int KT, bool SNAKE, bool XV, int AR>
int split_launch_inst(ConvKArgs k, int tile, hipStream_t st) {
    return with_tile(tile, [&](auto bm, auto bn, auto wm, auto kg, auto wn, auto vcx, auto ns) {
        constexpr int BM = decltype(bm)::value, BN = decltype(bn)::value, WM = decltype(wm)::value,
                      KG = decltype(kg)::value, WN = decltype(wn)::value, VCX = decltype(vcx)::value,
                      NS = decltype(ns)::value;
        return split_launch_xv<KT, BM, BN, WM, KG, WN, VCX, NS, SNAKE, XV, AR>(k, st);
    });
}
#ifndef RAVE_SPLIT_F32
#define RAVE_SPLIT_F32 0
#endif
template int split_launch_inst<RAVE_SPLIT_KT, (RAVE_SPLIT_SNAKE != 0), (RAVE_SPLIT_XV != 0), RAVE_SPLIT_F32>(
    ConvKArgs, int, hipStream_t);

}  // namespace rave
#else   // ------------------------------------------------------- host side

// Sum the split-K slabs in split order (fixed order: deterministic), then
// bias / residual / ConvT interleave.  One thread = 4 consecutive floats of
// the flat [B][M][U] slab image (U % 4 == 0 when vec_p), grid-stride: every
// lane busy whatever the row length (short-N layers have U = 64..128).
__global__ __launch_bounds__(256) void split_reduce_kernel(ConvKArgs a) {
    const int64_t total = (int64_t)a.B * a.M * a.U;
    const int64_t stride = (int64_t)gridDim.x * 256;
    if (a.vec_p) {
        for (int64_t q = blockIdx.x * 256ll + threadIdx.x; q < (total >> 2); q += stride) {
            const int64_t i = q << 2;
            s_f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
            for (int s = 0; s < a.S; ++s) v += *reinterpret_cast<const s_f32x4*>(a.partial + s * total + i);
            const int64_t row = i / a.U;
            const int n = (int)(i - row * a.U);
            const int b = (int)(row / a.M), m = (int)(row - (int64_t)b * a.M);
            if (!a.transposed && a.vec_y) {
                if (a.bias) v += a.bias[m];
                if (a.res) v += *reinterpret_cast<const s_f32x4*>(a.res + (int64_t)b * a.r_sb + (int64_t)m * a.r_sc + n);
                *reinterpret_cast<s_f32x4*>(a.y + (int64_t)b * a.y_sb + (int64_t)m * a.y_sc + n) = v;
            } else {
                float vv[4];
                *reinterpret_cast<s_f32x4*>(vv) = v;
#pragma unroll
                for (int e = 0; e < 4; ++e) store_out(a, b, m, n + e, vv[e]);
            }
        }
        return;
    }
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += stride) {
        float v = 0.f;
        for (int s = 0; s < a.S; ++s) v += a.partial[s * total + i];
        const int64_t row = i / a.U;
        const int n = (int)(i - row * a.U);
        const int b = (int)(row / a.M), m = (int)(row - (int64_t)b * a.M);
        store_out(a, b, m, n, v);
    }
}

// Tile + split-K choice: least padding with the most waves per workgroup
// that still fills the chip; K split over workgroups (fp32 slabs, fixed-order
// combine) when the output alone cannot give every SIMD a wave.
// operand planes / weight fragments per K-step of an arithmetic (bf16x3: three)
static int split_planes(int precision) { return precision == RAVE_PREC_BF16X3 ? 3 : 2; }
// 16-byte weight fragments per K-step and row block in the packed image
static int split_wplanes(int precision) { return precision == RAVE_PREC_BF16X3 && !RAVE_BF3_W4 ? 3 : 2; }
static inline int tile_waves(int ti) {   // waves per workgroup
    const int* t = kSplitTiles[ti];
    return (t[0] / t[2]) * (t[1] / t[4]) * t[3];
}

template <int KT>
static bool split_tile_fits(int idx, int np) {   // both DMA variants must fit (np: operand planes)
    return with_tile(idx, [np](auto bm, auto bn, auto wm, auto kg, auto wn, auto vcx, auto ns) {
        constexpr int BM = decltype(bm)::value, BN = decltype(bn)::value, WM = decltype(wm)::value,
                      KG = decltype(kg)::value, WN = decltype(wn)::value, VCX = decltype(vcx)::value,
                      NS = decltype(ns)::value;
        if (np == 3)
            return SGeo<KT, BM, BN, WM, true, KG, WN, VCX, NS, 3>::VALID &&
                   SGeo<KT, BM, BN, WM, false, KG, WN, VCX, NS, 3>::VALID;
        return SGeo<KT, BM, BN, WM, true, KG, WN, VCX, NS>::VALID &&
               SGeo<KT, BM, BN, WM, false, KG, WN, VCX, NS>::VALID;
    });
}
static bool split_fits(int taps, int idx, int np) {
    if (idx < 0 || idx >= kNumSplitTiles || !kSplitTileBuilt[idx]) return false;
    switch (taps) {
        case 1: return split_tile_fits<1>(idx, np);
        case 2: return split_tile_fits<2>(idx, np);
        case 3: return split_tile_fits<3>(idx, np);
        case 4: return split_tile_fits<4>(idx, np);
        case 7: return split_tile_fits<7>(idx, np);
        default: return split_tile_fits<8>(idx, np);
    }
}

static SplitCfg split_choose(int taps, int M, int U, int B, int nchunks, int split_row, int np) {
    const auto& all = kSplitTiles;
    auto waste = [&](int bm, int bn) {
        return double(ceil_div(M, bm) * bm) * double(ceil_div(U, bn) * bn) / (double(M) * double(U));
    };
    SplitCfg best{kSplitDefaultTile, 1, 0};
    double bscore = 1e30;
    for (int ti = 0; ti < kNumSplitTiles; ++ti) {   // the heuristic keeps to the KG = 1 tiles
        const int* c = all[ti];
        if (c[3] != 1) continue;
        if (!split_fits(taps, ti, np)) continue;
        if (split_row < M && split_row % c[2] != 0) continue;      // a wave never straddles ConvT groups
        const int nw = tile_waves(ti);
        const int64_t wgs = (int64_t)ceil_div(M, c[0]) * ceil_div(U, c[1]) * B;
        const int64_t waves = wgs * nw;
        double score = waste(c[0], c[1]);
        if (waves < 1024) score *= 1.0 + 0.5 * (1024.0 / waves - 1.0) / std::max(1, nchunks / 8);
        score *= 1.0 + 0.03 * (4 - nw);                                 // prefer fat workgroups
        if (score < bscore) { bscore = score; best = {ti, 1, 0}; }
    }
    const int* bt = all[best.tile];
    const int64_t waves = (int64_t)ceil_div(M, bt[0]) * ceil_div(U, bt[1]) * B * tile_waves(best.tile);
    if (waves < 1024 && nchunks >= 8) {
        int S = (int)std::min<int64_t>(16, ceil_div64(2048, waves));
        S = std::min(S, nchunks / 4);
        best.S = std::max(1, S);
    }
    return best;
}

template <int KT>
static int split_launch_family(ConvKArgs k, const SplitCfg& c, int ar, hipStream_t st) {
    const int* t = kSplitTiles[c.tile];
    k.XW = t[1] + (SFam<KT>::Q - 1) * k.d + (k.transposed ? 1 : 0);
    k.xw_magic = (unsigned)(((1u << 24) + k.XW - 1) / k.XW);
    const unsigned rl = (unsigned)(k.XW * SFam<KT>::S);
    k.rl_magic = (unsigned)((0x100000000ull + rl - 1) / rl);
    const bool snake = k.act == RAVE_ACT_SNAKE;
    if (ar != 0 && !k.x_vec) {
        // the fp32 ring and bf16x3 kernels are built for 16-byte window DMA only
        // (the register-staged RAVE_PREC_F32 kernel covers unaligned inputs)
        set_error(ar == 2 ? "conv1d(bf16x3): needs 16-byte aligned input rows and t_in % 4 == 0"
                          : "conv1d(f32_ring): needs 16-byte aligned input rows and t_in % 4 == 0");
        return RAVE_ERR_UNSUPPORTED;
    }
    auto fn = ar == 2 ? (snake ? split_launch_inst<KT, true, true, 2> : split_launch_inst<KT, false, true, 2>)
              : ar == 1 ? (snake ? split_launch_inst<KT, true, true, 1> : split_launch_inst<KT, false, true, 1>)
              : (snake ? (k.x_vec ? split_launch_inst<KT, true, true, 0> : split_launch_inst<KT, true, false, 0>)
                       : (k.x_vec ? split_launch_inst<KT, false, true, 0> : split_launch_inst<KT, false, false, 0>));
    return fn(k, c.tile, st);
}

static int split_prepare(const rave_conv1d_args& a, ConvKArgs& k, int& taps) {
    int rc = prepare_common(a, k, taps);
    if (rc != RAVE_OK) return rc;
    k.nchunks = ceil_div(a.c_in, split_cpc(taps));
    k.Mpad = ceil_div(k.M, 128) * 128;
    k.MB = k.Mpad / 32;
    const int64_t frag_floats = (int64_t)k.nchunks * k.MB * split_ksc(taps) * split_wplanes(a.precision) * 256;
    RAVE_CHECK_ARG(frag_floats * 4 < (1ll << 31), "conv1d(split16): packed weight beyond 2 GiB");
    k.w_bytes = (int)(frag_floats * 4);
    k.rscale = a.weight + frag_floats;                 // after the fragments
    auto aligned = [](const void* p, int64_t sb, int64_t sc) {
        return (reinterpret_cast<uintptr_t>(p) % 16 == 0) && sb % 4 == 0 && sc % 4 == 0;
    };
    k.vec_y = aligned(a.y, a.y_sb, a.y_sc) && (!a.residual || aligned(a.residual, a.r_sb, a.r_sc));
    k.vec_p = (k.U % 4 == 0) && (!a.partial || reinterpret_cast<uintptr_t>(a.partial) % 16 == 0);
    // 16-byte window DMA: rows 16-byte aligned and whole 4-sample pieces inside [0, t_in)
    k.x_vec = aligned(a.x, a.x_sb, a.x_sc) && a.t_in % 4 == 0;
    return RAVE_OK;
}

static bool split_tile_ok(int taps, int ti, int M, int split_row, int np, bool x_vec) {
    return ti >= 0 && ti < kNumSplitTiles && split_fits(taps, ti, np) && (x_vec || split_tile_xv0(ti)) &&
           (split_row >= M || split_row % kSplitTiles[ti][2] == 0);   // a wave never straddles ConvT groups
}

// The launch configuration: args.config when set (validated), else the heuristic.
static int split_resolve(const rave_conv1d_args& a, const ConvKArgs& k, int taps, SplitCfg& c) {
    if (a.config == 0) {
        c = split_choose(taps, k.M, k.U, k.B, k.nchunks, k.split_row, split_planes(a.precision));
        return RAVE_OK;
    }
    ConfigCode cc;
    RAVE_CHECK_ARG(decode_config(a.config, cc) && split_tile_ok(taps, cc.tile, k.M, k.split_row, split_planes(a.precision), k.x_vec) &&
                       split_count_distinct(cc.S, ceil_div(k.nchunks, kSplitTiles[cc.tile][5])),
                   "conv1d(split16): config not valid for these args (see rave_conv1d_configs)");
    c = {cc.tile, cc.S, cc.sep};
    return RAVE_OK;
}

int conv1d_split_configs(const rave_conv1d_args& a, int32_t* cfgs, int max_cfgs) {
    ConvKArgs k;
    int taps;
    int rc = split_prepare(a, k, taps);
    if (rc != RAVE_OK) return rc;
    int n = 0;
    auto put = [&](int v) {
        if (n < max_cfgs && cfgs) cfgs[n] = v;
        ++n;
    };
    for (int ti = 0; ti < kNumSplitTiles; ++ti) {
        if (!split_tile_ok(taps, ti, k.M, k.split_row, split_planes(a.precision), k.x_vec)) continue;
        const int* t = kSplitTiles[ti];
        const int nw = tile_waves(ti);
        const int64_t ntiles = (int64_t)ceil_div(k.M, t[0]) * ceil_div(k.U, t[1]) * k.B;
        const int nst = ceil_div(k.nchunks, t[5]);   // staged chunks
        for (int S : kSplitCands) {
            if (!split_count_distinct(S, nst)) continue;
            const int64_t waves = ntiles * nw * S;
            if (S > 1 && (waves > 16384 || ntiles * nw >= 4096)) continue;   // enough waves unsplit
            // in-launch combine: the last split reads S slabs serially -- only for few splits
            if (S == 1 || (S <= 4 && ntiles <= kSplitTicketsUsable)) put(encode_config(ti, S, 0));
            if (S > 1) put(encode_config(ti, S, 1));
        }
    }
    return n;
}

int64_t conv1d_split_workspace(const rave_conv1d_args& a) {
    ConvKArgs k;
    int taps;
    if (split_prepare(a, k, taps) != RAVE_OK) return -1;
    SplitCfg c;
    if (split_resolve(a, k, taps, c) != RAVE_OK) return -1;
    if (c.S <= 1) return 0;
    return kSplitTickets + (int64_t)c.S * k.B * (int64_t)k.M * k.U;
}

int conv1d_split(const rave_conv1d_args& a, void* stream) {
    ConvKArgs k;
    int taps;
    int rc = split_prepare(a, k, taps);
    if (rc != RAVE_OK) return rc;
    RAVE_CHECK_ARG(a.act != RAVE_ACT_SNAKE || a.c_in <= 1024, "conv1d(split16): Snake on more than 1024 channels");
    RAVE_CHECK_ARG(a.act != RAVE_ACT_LEAKY || a.leaky_slope <= 1.0f, "conv1d(split): leaky slope above 1");
    SplitCfg c;
    rc = split_resolve(a, k, taps, c);
    if (rc != RAVE_OK) return rc;
    if (c.S > 1 && a.partial == nullptr) c.S = 1;
    k.nchunks = ceil_div(k.nchunks, kSplitTiles[c.tile][5]);   // staged chunks (the kernel's unit)
    k.cps = ceil_div(k.nchunks, c.S);
    k.S = ceil_div(k.nchunks, k.cps);
    k.tickets = reinterpret_cast<int*>(a.partial);
    k.partial = a.partial ? a.partial + kSplitTickets : nullptr;   // slabs after the counters
    k.vec_p = (k.U % 4 == 0) && (!k.partial || reinterpret_cast<uintptr_t>(k.partial) % 16 == 0);
    k.gx = ceil_div(k.U, kSplitTiles[c.tile][1]);
    k.gy = ceil_div(k.M, kSplitTiles[c.tile][0]);
    const int64_t ntiles = (int64_t)k.gx * k.gy * k.B;
    RAVE_CHECK_ARG(ntiles * k.S < (1ll << 31), "conv1d(split16): grid too large");
    // the last-arriving split sums the tile's slabs (16-byte slab rows, counters for every tile)
    k.inlaunch = k.S > 1 && !c.sep && k.vec_p && ntiles <= kSplitTicketsUsable;
#ifdef RAVE_STAMPS
    k.stamps = a.stamps;
#endif
    hipStream_t st = as_stream(stream);
    const int ar = a.precision == RAVE_PREC_BF16X3 ? 2 : a.precision == RAVE_PREC_F32_RING ? 1 : 0;
    switch (taps) {
        case 1: rc = split_launch_family<1>(k, c, ar, st); break;
        case 2: rc = split_launch_family<2>(k, c, ar, st); break;
        case 3: rc = split_launch_family<3>(k, c, ar, st); break;
        case 4: rc = split_launch_family<4>(k, c, ar, st); break;
        case 7: rc = split_launch_family<7>(k, c, ar, st); break;
        case 8: rc = split_launch_family<8>(k, c, ar, st); break;
        default: set_error("conv1d: unsupported kernel size"); return RAVE_ERR_UNSUPPORTED;
    }
    if (rc != RAVE_OK || k.S <= 1 || k.inlaunch) return rc;
    const int64_t work = k.vec_p ? ((int64_t)k.B * k.M * k.U) >> 2 : (int64_t)k.B * k.M * k.U;
    launch(split_reduce_kernel, dim3((unsigned)std::min<int64_t>(ceil_div64(work, 256), 4096)), dim3(256), 0, st, k);
    return launch_status("split_reduce_kernel");
}

// ------------------------------------------------------------ weight packing
// Power-of-two row exponent: max |w * 2^e| in [8, 16) (e = 0 for an all-zero row).
static int row_exponent(double amax) {
    if (!(amax > 0.0)) return 0;
    int e = (int)std::floor(std::log2(16.0 / amax));
    while (std::ldexp(amax, e) >= 16.0) --e;
    while (std::ldexp(amax, e) < 8.0) ++e;
    return e;
}

}  // namespace rave

using namespace rave;

// GEMM-row geometry of a layer (shared by the size query and the packer)
static int split_geometry(int c_in, int c_out, int kernel, int stride, int dilation, int transposed,
                          int out_shift, int& taps, int& M, int& Mpad, int& nchunks, int& split_row,
                          int& q0) {
    (void)dilation;
    if (transposed) {
        if (kernel != 2 * stride || stride % 2) return -1;
        taps = 2;
        q0 = stride - out_shift;
        split_row = convt_group1_row(c_out, stride, q0);
        M = split_row + c_out * (stride - q0);
    } else {
        if (!family_supported(kernel) || family_stride(kernel) != stride) return -1;
        taps = kernel;
        q0 = 1;
        split_row = 1 << 30;
        M = c_out;
    }
    Mpad = ceil_div(M, 128) * 128;
    nchunks = ceil_div(c_in, split_cpc(taps));
    return 0;
}

static int64_t split_packed_floats(int c_in, int c_out, int kernel, int stride, int dilation, int transposed,
                                   int np) {
    if (c_in <= 0 || c_out <= 0) return -1;
    int taps, M, Mpad, nchunks, split_row, q0;
    // transposed: the larger of the two row layouts (out_shift 0 / stride/2)
    int64_t best = -1;
    for (int os = 0; os <= (transposed ? 1 : 0); ++os) {
        if (split_geometry(c_in, c_out, kernel, stride, dilation, transposed, os ? stride / 2 : 0, taps, M,
                           Mpad, nchunks, split_row, q0) != 0)
            return -1;
        const int64_t n = (int64_t)nchunks * (Mpad / 32) * split_ksc(taps) * np * 256 + Mpad;
        best = std::max(best, n);
    }
    return best;
}

extern "C" int64_t rave_conv1d_split_packed_size(int c_in, int c_out, int kernel, int stride, int dilation,
                                                 int transposed) {
    return split_packed_floats(c_in, c_out, kernel, stride, dilation, transposed, 2);
}

extern "C" int64_t rave_conv1d_bf3_packed_size(int c_in, int c_out, int kernel, int stride, int dilation,
                                               int transposed) {
    return split_packed_floats(c_in, c_out, kernel, stride, dilation, transposed, RAVE_BF3_W4 ? 2 : 3);
}

// host fp32 -> bf16, round to nearest even (finite weights)
static uint16_t bf16_bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
static float bf16_value(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

static int split_pack(const float* w, int c_in, int c_out, int kernel, int stride, int dilation, int transposed,
                      int out_shift, float* packed, int mode) {   // 0 split16, 1 fp32, 2 bf16x3
    RAVE_CHECK_ARG(w && packed, "split_pack_weight: null pointer");
    const bool f32 = mode != 0;                        // (row scales 1)
    const int NPW = mode == 2 ? 3 : 2;
    RAVE_CHECK_ARG(c_in > 0 && c_out > 0 && kernel > 0 && stride > 0 && dilation > 0,
                   "split_pack_weight: bad shape");
    RAVE_CHECK_ARG(!transposed || out_shift == 0 || out_shift == stride / 2,
                   "split_pack_weight: transposed out_shift must be 0 or stride/2");
    int taps, M, Mpad, nchunks, split_row, q0;
    if (split_geometry(c_in, c_out, kernel, stride, dilation, transposed, out_shift, taps, M, Mpad, nchunks,
                       split_row, q0) != 0) {
        set_error("split_pack_weight: unsupported layer shape");
        return RAVE_ERR_UNSUPPORTED;
    }
    const int R = transposed ? stride : 1;
    const int S = transposed ? 1 : family_stride(taps);
    const int VC = split_cpc(taps) * S;
    const int KSC = split_ksc(taps), HPS = VC / 16, CPC = VC / S;
    const int MB = Mpad / 32;
    // GEMM weight of (row m, input channel ci, original tap j); 0 outside
    auto wval = [&](int m, int ci, int j) -> float {
        if (m >= M || ci >= c_in) return 0.f;
        if (!transposed) return w[((int64_t)m * c_in + ci) * kernel + j];
        int co, q;
        if (m < split_row) { co = m / q0; q = m % q0; }
        else { const int p = R - q0; co = (m - split_row) / p; q = q0 + (m - split_row) % p; }
        if (co >= c_out) return 0.f;                    // group-0 padding rows
        int kidx;
        if (q < q0) kidx = (j == 0) ? q + out_shift + R : q + out_shift;
        else kidx = (j == 0) ? q + out_shift : q + out_shift - R;
        return w[((int64_t)ci * c_out + co) * kernel + kidx];
    };
    // (tap q after polyphase, virtual channel vc of chunk c) -> (ci, original tap)
    auto kmap = [&](int c, int q, int vc, int& ci, int& j) {
        ci = c * CPC + vc / S;
        j = (S > 1) ? q * S + vc % S : q;
    };
    const int KT_orig = transposed ? 2 : kernel;
    std::vector<int> ex(Mpad, 0);
    for (int m = 0; m < Mpad && !f32; ++m) {
        double amax = 0.0;
        for (int ci = 0; ci < c_in; ++ci)
            for (int j = 0; j < KT_orig; ++j) amax = std::max(amax, (double)std::fabs(wval(m, ci, j)));
        ex[m] = row_exponent(amax);
    }
    _Float16* out = reinterpret_cast<_Float16*>(packed);
    uint16_t* bout = reinterpret_cast<uint16_t*>(packed);
    for (int c = 0; c < nchunks; ++c)
        for (int mb = 0; mb < MB; ++mb)
            for (int st = 0; st < KSC; ++st) {
                const int q = st / HPS, hv = st % HPS;
                const int64_t blk = ((int64_t)(c * MB + mb) * KSC + st) * NPW;   // 1 KB slots
                uint16_t* bp = bout + blk * 512;       // bf16x3: hi, lo, mid
                _Float16* hi = out + blk * 512;
                _Float16* lo = hi + 512;
                float* f32s = packed + blk * 256;      // fp32: floats 0-3 of a lane in slot 0, 4-7 in slot 1
                for (int l = 0; l < 64; ++l)
                    for (int e = 0; e < 8; ++e) {
                        const int m = mb * 32 + (l & 31);
                        const int vc = hv * 16 + 8 * (l >> 5) + e;
                        int ci, j;
                        kmap(c, q, vc, ci, j);
                        if (mode == 2) {
                            const float v = wval(m, ci, j);
                            const uint16_t h = bf16_bits(v);
                            const float r = v - bf16_value(h);
                            const uint16_t md = bf16_bits(r);
                            bp[l * 8 + e] = h;
                            bp[1024 + l * 8 + e] = md;
                            bp[512 + l * 8 + e] = bf16_bits(r - bf16_value(md));
                            continue;
                        }
                        if (f32) {
                            f32s[(e >> 2) * 256 + l * 4 + (e & 3)] = wval(m, ci, j);
                            continue;
                        }
                        const float v = std::ldexp(wval(m, ci, j), ex[m]);
                        const _Float16 vh = (_Float16)v;
                        const _Float16 vl = (_Float16)((v - (float)vh) * 2048.0f);
                        hi[l * 8 + e] = vh;
                        lo[l * 8 + e] = vl;
                    }
            }
    float* rs = packed + (int64_t)nchunks * MB * KSC * NPW * 256;
    for (int m = 0; m < Mpad; ++m) rs[m] = f32 ? 1.0f : (float)std::ldexp(1.0, -(ex[m] + 11));
    return RAVE_OK;
}

extern "C" int rave_conv1d_split_pack_weight(const float* w, int c_in, int c_out, int kernel, int stride,
                                             int dilation, int transposed, int out_shift, float* packed) {
    return split_pack(w, c_in, c_out, kernel, stride, dilation, transposed, out_shift, packed, 0);
}

extern "C" int rave_conv1d_ring_pack_weight(const float* w, int c_in, int c_out, int kernel, int stride,
                                            int dilation, int transposed, int out_shift, float* packed) {
    return split_pack(w, c_in, c_out, kernel, stride, dilation, transposed, out_shift, packed, 1);
}

// (RAVE_BF3_W4: the bf16x3 kernels read the exact-fp32 image and split it in registers)
extern "C" int rave_conv1d_bf3_pack_weight(const float* w, int c_in, int c_out, int kernel, int stride,
                                           int dilation, int transposed, int out_shift, float* packed) {
    return split_pack(w, c_in, c_out, kernel, stride, dilation, transposed, out_shift, packed, RAVE_BF3_W4 ? 1 : 2);
}
#endif  // RAVE_SPLIT_KT
