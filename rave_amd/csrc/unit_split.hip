// Fused Residual(DilatedUnit) on the f16 matrix cores (RAVE_PREC_SPLIT16):
// rave/blocks.py:32-46 (Residual / AlignBranches sum) around rave/blocks.py:84-113
// (DilatedUnit):
//
//     y = x + conv1x1(act2(conv3_d(act0(x)) + b1)) + b2
//
// Arithmetic as conv_split.hip: fp32 operands split into f16 (hi, lo) pairs,
// three v_mfma_f32_32x32x16_f16 per 16-deep K-step into one fp32 accumulator,
// power-of-two row scales undone in the epilogues.
//
// A workgroup owns every channel of a BN-column slab of one batch item:
//   prologue  act0(x) window [rows][C] -> two f16 planes in LDS, staged in ONE
//             pass (every load of the window in flight at once; the dilated
//             halo is read once and shared by the three taps)
//   phase 1   h = W1 (C x 3C) . window: A = weight fragments streamed from L2
//             through a register ring (fully unrolled, static slots), B = window
//             fragments (ds_read_b128, next step's reads in flight)
//   seam      h = act2(h * rs1 + b1) -> (hi, lo) planes over the dead window
//   phase 2   y = W2 (C x C) . h, ring running on from W1 into W2
//   epilogue  y * rs2 + b2 + x (residual re-read, L2-hot) -> HBM
// Each wave owns 32 rows x 64 columns (1 x 2 blocks of 32x32).
//
// Cooperative form (RB > 1, C in {256, 512}; needs the rave_unit_workspace
// buffer): a GROUP of RB workgroups shares one column slab, workgroup rb owning
// output rows [rb C/RB, (rb+1) C/RB) of BOTH GEMMs, so a slab's weights stream
// through RB CUs instead of one (1 MB per CU at C = 512 instead of 4 MB).  Phase 2
// needs every row of h: at the seam each member publishes its act2(h) rows
// write-through (sc1 stores, drained, then an agent-scope counter add), waits for
// the group's other members (ONE wave polls, bounded, one agent acquire), and
// stages their rows into its planes.  Members are dealt so that a group's RB
// blocks are consecutive in one XCD's dispatch order (blocks b, b + 8, ...): a
// group is resident together whenever its first member is, and every other
// resident group completes without waiting on a non-resident one.  The range
// guard of h is group-wide (members publish their max |h|).  The arithmetic is
// that of the one-workgroup form, but not its fp32 summation order: each
// member's phase 2 starts at its own channel block (smap) and alternate K-steps
// accumulate into two chains (DA), so the two forms agree within tolerance, not
// bitwise.  The poll is bounded: a member that gives up writes NaN outputs AND
// sets the workspace's RAVE_SPLITK_STATUS_WORD (sticky), which the owner of the
// workspace reads back and reports (the engine returns RAVE_ERR_COOP).
#include "common.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace rave {

typedef _Float16 us_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 us_h4 __attribute__((ext_vector_type(4)));
typedef float us_f32x8 __attribute__((ext_vector_type(8)));
typedef float us_f32x4 __attribute__((ext_vector_type(4)));
typedef float us_f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned us_u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 us_b8 __attribute__((ext_vector_type(8)));
typedef __bf16 us_b4 __attribute__((ext_vector_type(4)));

// fp32 -> three bf16 parts with v == hi + mid + lo exactly (8 + 8 + 8 bits of
// the 24-bit significand; each remainder is exact in fp32)
template <typename FV, typename BV>
__device__ __forceinline__ void bf3_split(const FV& v, BV& hi, BV& mid, BV& lo) {
    bf3_split_pk(v, hi, mid, lo);
}

constexpr int kUSMaxDil = 16;
#ifndef RAVE_COOP_SC1
#define RAVE_COOP_SC1 1
#endif
#ifndef RAVE_US_R
#define RAVE_US_R 3
#endif
#ifndef RAVE_US_RC
#define RAVE_US_RC 6                // weight ring depth of the cooperative form (4 waves per CU)
#endif
constexpr unsigned kUSSpinLimit = 1u << 18;   // cooperative seam: bounded poll (give-up -> status word + NaN)
template <int V> struct IC {
    static constexpr int value = V;
};

#ifdef RAVE_STAMPS
// diagnostic build only: 8 clock stamps per workgroup (tools/layer_bench.py --stamps)
__device__ unsigned long long* g_us_stamps = nullptr;
#define US_STAMP(k)                                                                            \
    do {                                                                                       \
        if (threadIdx.x == 0 && g_us_stamps) {                                                 \
            g_us_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime();                  \
            if ((k) == 0) g_us_stamps[blockIdx.x * 8 + 7] = __builtin_amdgcn_s_memrealtime();  \
        }                                                                                      \
    } while (0)
#else
#define US_STAMP(k) \
    do {            \
    } while (0)
#endif
// US_AT(k, kc): stamp slot k in the diagnostic build, slot kc in the cooperative-detail
// one (-DRAVE_STAMPS_COOP: 0 start, 1 window staged, 2 phase 1, 3 published, 4 own
// phase-2 steps done, 5 poll done, 6 partner rows staged); -1 = no stamp there
#ifdef RAVE_STAMPS_COOP
#define US_AT(k, kc)                \
    do {                            \
        if ((kc) >= 0) US_STAMP(kc); \
    } while (0)
#else
#define US_AT(k, kc)               \
    do {                           \
        if ((k) >= 0) US_STAMP(k); \
    } while (0)
#endif
constexpr unsigned kUSOOB = 0xFFFFFFF0u;
constexpr int kXcds = 8;                      // gfx950: blocks dealt round-robin over 8 XCDs
constexpr int kCoopNoFit = 1;                 // us_launch: a group does not fit one XCD
constexpr int kCoopMaxRB = 4;                 // largest cooperative group (C = 512 / 128)

struct USArgs {
    const float* x; float* y; const float* w; const float* rs1; const float* rs2;
    const float* b1; const float* b2; const float* a0; const float* a2;
    int64_t x_sb, x_sc, y_sb, y_sc;
    int T, d, pad_l, ntiles, XW;
    int XL, rsh;             // valid input columns; residual column shift (cached form)
    int x_bytes, y_bytes, w_bytes, bias_bytes;
    int act;
    float slope;
    unsigned xw_magic;
    // cooperative form: per group {arrivals, departures} counters (zero at rest),
    // the give-up word, members' max |h|, the act2(h) exchange [group][BN][C]
    unsigned* flags; unsigned* tmo; float* xmax; float* xch;
    int ngroups, xch_bytes;
    int xv;                  // 16-byte window loads (XL % 4 == 0, 16-byte aligned rows)
    unsigned nb_magic;       // ceil(2^24 / window blocks per row)
    int flag_stride;         // counter words per group (cooperative form)
    unsigned* status;        // optional caller's give-up word (host-mapped: system scope)
    unsigned spin_limit;     // polls before a member gives up (rave_debug_coop)
    int force_giveup;        // debug: every group reports a give-up after a normal hand-off
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t us_rsrc(const void* p, int bytes) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint64_t u = ((uint64_t)hi << 32) | lo;
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0,
                                             __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

template <bool SNAKE>
__device__ __forceinline__ float us_act(float v, float slope, float alpha) {
    if constexpr (SNAKE) {
        const float r = 1.0f / (alpha + 1e-9f);
        return v + r * sin_squared(alpha * v);
    } else {
        return fmaxf(v, v * slope);         // leaky ReLU for slope <= 1 (host check); slope 1 == none
    }
}

// C channels; WGN waves along time (each 64 columns); C/(32 MI) waves along
// rows (each MI 32-row blocks).
// NP = 3 (bf16x3) at C = 512: the window is sized for dilations <= kUSBf512Dil so
// that three planes fit the CU's LDS (RAVE's C = 512 stages use dilations 1 and 3)
constexpr int kUSBf512Dil = 4;
template <int C, int WGN, int MI, int KG = 1, int CB = 2, int RB = 1, int NP = 2> struct USGeo {
    static constexpr int WGM = C / (32 * MI * RB), NWT = WGM * WGN, NW = NWT * KG, NT = 64 * NW;
    static constexpr int BN = 32 * CB * WGN;           // CB 32-column blocks per wave
    static constexpr int S1 = 3 * C / 16, S2 = C / 16, ST = S1 + S2;   // K-steps
    static constexpr int PH = C + 8;                  // halves per LDS row (conflict-free b128)
    static constexpr int XW_MAX = BN + 2 * ((NP == 3 && C == 512) ? kUSBf512Dil : kUSMaxDil);
    static constexpr int XPLANE = XW_MAX * PH * 2;    // bytes per f16 plane
    static constexpr int HPLANE = BN * PH * 2;
    static constexpr int PL1 = XPLANE > HPLANE ? XPLANE : HPLANE;   // bytes per plane
    static constexpr int PLANES = NP * PL1;           // NP = 2 (hi, lo) or 3 (bf16x3: hi, lo, mid)
    // + per-row table: rs1 b1 a2 | rs2 b2 a0, + range-guard votes (16 B) and wave maxima (16 floats)
    static constexpr int TAB = PLANES, VOTE = PLANES + 6 * C * 4, VRED = VOTE + 16;
    static constexpr int LDS = VRED + 64;
    static constexpr int G8 = C / 8;                  // 8-channel groups per window row
    static constexpr int XT = (XW_MAX * G8 + NT - 1) / NT;
    static constexpr int R = RB > 1 ? RAVE_US_RC : RAVE_US_R;   // weight ring depth (K-steps)
    static constexpr int G8R = C / (8 * RB);          // 8-channel groups of one member's rows
    // K-groups: two waves per output tile take alternate K-steps (both phases)
    static constexpr int RED = NWT * MI * CB * 16 * 64 * 4;  // partial-sum hand-off (bytes)
    static_assert(C % 64 == 0 && (MI == 1 || MI == 2) && NW <= 16, "geometry");
    static_assert(RB == 1 || (KG == 1 && WGN == 1 && C % (32 * MI * RB) == 0), "cooperative geometry");
    static_assert(KG == 1 || (KG == 2 && S1 % 2 == 0 && S2 % 2 == 0 && RED <= PLANES), "K-groups");
};

// F32 (RAVE_PREC_F32_RING): the same kernel in exact fp32 -- one fp32 plane in
// the bytes of the (hi, lo) pair (row pitch PH floats), weight fragments of 8
// floats per lane in the split image's slots (rave_unit_ring_pack_weight),
// eight v_mfma_f32_32x32x2_f32 per 16-deep K-step (K-slot (s, half h) =
// channel 8h + s), no range guard, row scales 1.
//
// BF (RAVE_PREC_BF16X3, both forms: one workgroup per slab, and the cooperative
// groups at C = 256 / 512 whose exchanged act2(h) rows stay fp32 and are split by
// each member into its own planes): fp32 on the bf16 matrix cores.  Every
// operand v is split exactly as hi + mid + lo (bf16 each: 24 significand bits,
// the fp32 exponent range, so no row scales and no range guard); three planes
// (hi, lo, mid) in LDS and three weight fragments per K-step; six
// v_mfma_f32_32x32x16_bf16 per K-step take every cross product but mid*lo,
// lo*mid and lo*lo (each below 2^-25 of |a b|, under fp32's own rounding of a
// product), smallest first, into one fp32 accumulator.
//
// Range guard, RB == 1 (GUARD = false first): the body runs with no guard code
// at all; an operand past the f16 range became inf in its hi half, so it shows
// as a non-finite output sum.  Only when some wave of the workgroup holds one
// (one vote per workgroup, before any store) does the workgroup run the body
// again with GUARD = true: the window and the seam vote, and a block past
// kSplitLimit is re-staged as v * 2^-s (rare: values past 2^15, or a genuine
// inf / NaN input, which then passes through as in fp32).  The cooperative form
// (RB > 1) runs guarded only (its members cannot repeat a hand-off alone).
// Returns false when the unguarded pass found a non-finite sum (its stores are
// then rewritten by the guarded pass).
template <int C, int WGN, int MI, int KG, int CB, bool SNAKE, int AR, int RB, bool GUARD>
__device__ __forceinline__ bool unit_split_body(const USArgs& a) {
    constexpr bool F32 = AR == 1, BF = AR == 2;      // arithmetic: 0 split16, 1 fp32, 2 bf16x3
    constexpr int NPW = BF ? 3 : 2;                  // operand planes / weight fragments per K-step
    using G = USGeo<C, WGN, MI, KG, CB, RB, NPW>;
    // cooperative form with one workgroup per CU (its LDS rules out a second):
    // the hand-off reads the exchange by sc1 loads instead of an agent acquire
    // (RAVE_COOP_SC1=0 keeps the acquire: A/B).  What this rests on is the
    // guide's measured form (MI355X_MICROARCH.md, Valid forms, Consumer bullet
    // (1)-(4), hand-off table row 1), every condition of which holds here:
    // every byte of the exchange is stored sc1 (the seam's publish) and read
    // only by sc1 buffer loads (stage_rows); each storing wave drains with
    // vmcnt(0) before the workgroup barrier behind which ONE lane adds to the
    // group's counter; ONE wave polls it with sc1 loads and the others load
    // behind the barrier it then joins; hipMalloc'd workspace; one workgroup per
    // CU (the predicate's LDS test).  Row 1 does not need the members on one
    // XCD: the XCD-local dealing in us_launch (blocks b, b + 8, ... of a group)
    // is for speed (the exchange stays in one L2) and for residency, not for
    // visibility.  Forms with two workgroups per CU (split16 C = 256) keep the
    // agent acquire, so both paths stay covered by the cooperative tests.
    constexpr bool SC1X = RB > 1 && RAVE_COOP_SC1 != 0 && 2 * G::LDS > 160 * 1024;
    static_assert(!SC1X || 2 * G::LDS > 160 * 1024, "sc1 hand-off: one workgroup per CU only");
    constexpr bool GV = GUARD && AR == 0 && RAVE_SPLIT_GUARD != 0;   // votes inside the body
    static_assert(RB == 1 || GUARD || AR != 0, "the cooperative split16 form runs guarded");
    constexpr int NT = G::NT, PH = G::PH, G8 = G::G8, XT = G::XT, R = G::R;
    constexpr int S1 = G::S1, ST = G::ST, CG = C / 16;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    _Float16* ph = reinterpret_cast<_Float16*>(lds);
    _Float16* pl = reinterpret_cast<_Float16*>(lds + G::PL1);
    _Float16* pm = reinterpret_cast<_Float16*>(lds + 2 * G::PL1);   // BF: the mid plane
    float* pf = reinterpret_cast<float*>(lds);                 // F32: the fp32 plane
    float* tab = reinterpret_cast<float*>(lds + G::TAB);      // [6][C]
    unsigned char* vote = reinterpret_cast<unsigned char*>(lds + G::VOTE);
    float* vred = reinterpret_cast<float*>(lds + G::VRED);

    US_AT(0, 0);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kg = wave / G::NWT;                    // K-group
    const int twave = wave - kg * G::NWT;
    const int wm = twave % G::WGM, wn = twave / G::WGM;
    const int hh = lane >> 5, l32 = lane & 31;
    int lg, rb = 0;
    if constexpr (RB == 1) {
        lg = __builtin_amdgcn_readfirstlane(xcd_major(blockIdx.x, gridDim.x));
    } else {
        // block b -> XCD slot b & 7; along that XCD's blocks (b >> 3) the members
        // of one group are consecutive; groups XCD-major (gridDim = 8k RB)
        const int q = blockIdx.x >> 3;
        rb = q % RB;
        lg = (blockIdx.x & 7) * (int)(gridDim.x / (8 * RB)) + q / RB;
        if (lg >= a.ngroups) return true;        // padding group (all its members leave)
    }
    const int b = lg / a.ntiles;
    const int n0 = (lg - b * a.ntiles) * G::BN;
    const float slope = a.act == RAVE_ACT_LEAKY ? a.slope : 1.0f;
    const int XW = a.XW;
    const int ntask = XW * G8;
    const int t0 = n0 - a.pad_l;

    const auto xrs = us_rsrc(a.x + (int64_t)b * a.x_sb, a.x_bytes);
    const auto wrs = us_rsrc(a.w, a.w_bytes);
    int sh0 = 0, sh2 = 0;                            // range-guard shifts of the two GEMMs' B operands

    // ------------------------------------------------------------ weight ring
    // this wave's m-blocks MI*wm .. MI*wm+MI-1; fragment (mb, s, plane) at ((mb*ST + s)*2 + plane) KB
    // (ring slot = this wave's local step t % R; s = the global K-step, t*KG + kg)
    us_h8 ring[R][MI][NPW];
    const int wmg = wm + rb * G::WGM;                // this wave's row-block index in the unit
    const unsigned abase = (unsigned)((MI * wmg) * ST * NPW) * 1024u + (unsigned)lane * 16u;
    auto load_a = [&](int slot, int s) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int p = 0; p < NPW; ++p)
                ring[slot][i][p] = __builtin_bit_cast(us_h8, __builtin_amdgcn_raw_buffer_load_b128(
                    wrs, s < ST ? abase + (unsigned)(((i * ST + s) * NPW + p) * 1024) : kUSOOB, 0, 0));
    };
    // (the 16-byte window path issues the ring's first fill after its window
    // loads, so the window's wait does not include the weights)
    auto prefetch_ring = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < R; ++t) load_a(t, t * KG + kg);
    };
    if (!a.xv) prefetch_ring();

    // ------------------------------------------------------------ per-row table -> LDS
    // every load in flight at once (a rolled loop waits out one round trip per
    // pass); issued here, stored after the window loads are issued
    // (C is a multiple of 64: the segment k = i / C and the range test are
    // wave-uniform, so the source pointer is a scalar and no load sits under an
    // exec mask -- a masked load made the compiler drain every load at the merge)
    constexpr int NTAB = (6 * C + NT - 1) / NT;
    float tabv[NTAB];
#pragma unroll
    for (int r = 0; r < NTAB; ++r) {
        const int i = tid + r * NT;
        const int k = __builtin_amdgcn_readfirstlane(i / C), m = i - k * C;
        const float* src = k == 0 ? a.rs1 : k == 1 ? a.b1 : k == 2 ? a.a2 : k == 3 ? a.rs2 : k == 4 ? a.b2 : a.a0;
        const bool has = k < 6 && ((k == 1 || k == 4) ? a.bias_bytes > 0 : (k == 2 || k == 5) ? SNAKE : true);
        tabv[r] = has ? src[m] : 0.f;
    }
    auto store_tab = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < NTAB; ++r)
            if (__builtin_amdgcn_readfirstlane(tid + r * NT) < 6 * C) tab[tid + r * NT] = tabv[r];
    };

    // ------------------------------------------------------------ prologue: act0(x) window
    // (xs: the range guard's power-of-two scale; returns max |act0(x) xs| of the
    // thread's values)
    auto stage_window = [&](float xs) __attribute__((always_inline)) {
        float cmax = 0.f;
        float rx[XT][8];
#pragma unroll
        for (int i = 0; i < XT; ++i) {
            const int e = tid + i * NT;
            const int g = (int)(((unsigned)e * a.xw_magic) >> 24);
            const int w = e - g * XW;
            const int t = min(max(t0 + w, 0), a.XL - 1);
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                const int c = min(g * 8 + v, C - 1);
                rx[i][v] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                    xrs, (unsigned)(c * a.x_sc + t) * 4u, 0, 0));
            }
        }
#pragma unroll
        for (int i = 0; i < XT; ++i) {
            const int e = tid + i * NT;
            const int g = (int)(((unsigned)e * a.xw_magic) >> 24);
            const int w = e - g * XW;
            const bool ok = (e < ntask) && (t0 + w >= 0) && (t0 + w < a.XL);
            us_f32x8 v8;
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                const float al = SNAKE ? a.a0[min(g * 8 + v, C - 1)] : 0.f;   // L1-hot
                v8[v] = ok ? us_act<SNAKE>(rx[i][v], slope, al) * xs : 0.f;
            }
            if constexpr (F32) {
                if (e < ntask) {
                    *reinterpret_cast<us_f32x4*>(pf + w * PH + g * 8) = us_f32x4{v8[0], v8[1], v8[2], v8[3]};
                    *reinterpret_cast<us_f32x4*>(pf + w * PH + g * 8 + 4) = us_f32x4{v8[4], v8[5], v8[6], v8[7]};
                }
            } else if constexpr (BF) {
                us_b8 hi, mid, lo;
                bf3_split(v8, hi, mid, lo);
                if (e < ntask) {
                    *reinterpret_cast<us_b8*>(ph + w * PH + g * 8) = hi;
                    *reinterpret_cast<us_b8*>(pl + w * PH + g * 8) = lo;
                    *reinterpret_cast<us_b8*>(pm + w * PH + g * 8) = mid;
                }
            } else {
                cmax = fmaxf(cmax, absmax8(v8));
                const us_h8 hi = __builtin_convertvector(v8, us_h8);
                const us_h8 lo = __builtin_convertvector((v8 - __builtin_convertvector(hi, us_f32x8)) * 2048.0f, us_h8);
                if (e < ntask) {
                    *reinterpret_cast<us_h8*>(ph + w * PH + g * 8) = hi;
                    *reinterpret_cast<us_h8*>(pl + w * PH + g * 8) = lo;
                }
            }
        }
        return cmax;
    };
    // 16-byte form (rows of whole 4-sample pieces, a.xv): task (8-channel group g,
    // 4-sample block k), k fastest along the lanes (coalesced rows); 8 b128
    // loads per task, every load of the window in flight at once, then four
    // transposed 8-channel plane rows per task.  Blocks are wholly inside or
    // wholly outside [0, XL) (XL % 4 == 0, 4-aligned block starts).
    auto stage_window_v = [&]() __attribute__((always_inline)) {
        constexpr int NBM = (G::XW_MAX + 3) / 4 + 1, XTV = (G8 * NBM + NT - 1) / NT;
        const int ta = t0 & ~3;
        const int nb = (t0 + XW - ta + 3) >> 2;
        const int ntv = G8 * nb;
        float cmax = 0.f;
        us_f32x4 rx[XTV][8];
#pragma unroll
        for (int i = 0; i < XTV; ++i) {
            const int e = tid + i * NT;
            const int g = (int)(((unsigned)e * a.nb_magic) >> 24);
            const int kb = e - g * nb;
            const int t = ta + 4 * kb;
            const bool ok = (e < ntv) && t >= 0 && t < a.XL;
#pragma unroll
            for (int v = 0; v < 8; ++v) {
#ifdef RAVE_EXP_NOWIN
                // timing-only A/B variant (wrong results, never shipped): no window
                // loads -- bounds what hiding the prologue's loads could buy
                rx[i][v] = us_f32x4{0.01f * v, 0.02f * i, ok ? 0.5f : 0.f, 0.25f};
#else
                rx[i][v] = __builtin_bit_cast(us_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                    xrs, ok ? (unsigned)((g * 8 + v) * a.x_sc + t) * 4u : kUSOOB, 0, 0));
#endif
            }
        }
        prefetch_ring();
        if constexpr (SNAKE) {
            store_tab();
            __syncthreads();                         // the per-row table (Snake alphas) is in LDS
        }
        if (RB == 1) US_AT(6, -1);
#pragma unroll
        for (int i = 0; i < XTV; ++i) {
            const int e = tid + i * NT;
            const int g = (int)(((unsigned)e * a.nb_magic) >> 24);
            const int kb = e - g * nb;
            if (e < ntv) {
                float al[8];
#pragma unroll
                for (int v = 0; v < 8; ++v) al[v] = SNAKE ? tab[5 * C + g * 8 + v] : 0.f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int w = ta + 4 * kb + q - t0;
                    us_f32x8 v8;
#pragma unroll
                    for (int v = 0; v < 8; ++v) v8[v] = us_act<SNAKE>(rx[i][v][q], slope, al[v]);
                    if (w < 0 || w >= XW) continue;
                    if constexpr (F32) {
                        *reinterpret_cast<us_f32x4*>(pf + w * PH + g * 8) = us_f32x4{v8[0], v8[1], v8[2], v8[3]};
                        *reinterpret_cast<us_f32x4*>(pf + w * PH + g * 8 + 4) = us_f32x4{v8[4], v8[5], v8[6], v8[7]};
                    } else if constexpr (BF) {
                        us_b8 hi, mid, lo;
                        bf3_split(v8, hi, mid, lo);
                        *reinterpret_cast<us_b8*>(ph + w * PH + g * 8) = hi;
                        *reinterpret_cast<us_b8*>(pl + w * PH + g * 8) = lo;
                        *reinterpret_cast<us_b8*>(pm + w * PH + g * 8) = mid;
                    } else {
                        cmax = fmaxf(cmax, absmax8(v8));
                        const us_h8 hi = __builtin_convertvector(v8, us_h8);
                        const us_h8 lo = __builtin_convertvector((v8 - __builtin_convertvector(hi, us_f32x8)) * 2048.0f, us_h8);
                        *reinterpret_cast<us_h8*>(ph + w * PH + g * 8) = hi;
                        *reinterpret_cast<us_h8*>(pl + w * PH + g * 8) = lo;
                    }
                }
            }
        }
        if constexpr (!SNAKE) store_tab();           // (published by the barrier after the staging)
        return cmax;
    };
    // range guard: when a wave saw |act0(x)| >= 2^15 the window is staged again
    // as act0(x) * 2^-sh0 by a rolled loop (small code, few registers: rare)
    {
        float cmax;
        if (a.xv) {
            cmax = stage_window_v();
        } else {
            store_tab();
            cmax = stage_window(1.0f);
        }
        if constexpr (GV) vote_cast(vote, wave, cmax);
        __syncthreads();
        if (GV && __builtin_expect(vote_any<G::NW>(vote), 0)) {
            sh0 = __builtin_amdgcn_readfirstlane(split_shift(block_max<G::NW>(cmax, vred)));
            const float xs = ldexpf(1.0f, -sh0);
#pragma nounroll
            for (int e = tid; e < ntask; e += NT) {
                const int g = (int)(((unsigned)e * a.xw_magic) >> 24);
                const int w = e - g * XW;
                const bool ok = (t0 + w >= 0) && (t0 + w < a.XL);
                const int t = min(max(t0 + w, 0), a.XL - 1);
                us_f32x8 v8;
#pragma unroll
                for (int v = 0; v < 8; ++v) {
                    const int c = min(g * 8 + v, C - 1);
                    const float xv = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                        xrs, (unsigned)(c * a.x_sc + t) * 4u, 0, 0));
                    v8[v] = ok ? us_act<SNAKE>(xv, slope, SNAKE ? a.a0[c] : 0.f) * xs : 0.f;
                }
                const us_h8 hi = __builtin_convertvector(v8, us_h8);
                const us_h8 lo = __builtin_convertvector((v8 - __builtin_convertvector(hi, us_f32x8)) * 2048.0f, us_h8);
                *reinterpret_cast<us_h8*>(ph + w * PH + g * 8) = hi;
                *reinterpret_cast<us_h8*>(pl + w * PH + g * 8) = lo;
            }
            __syncthreads();
        }
    }
    US_AT(1, 1);

    // ------------------------------------------------------------ K loop (both phases)
    // DA (cooperative form, one wave per SIMD): alternate K-steps accumulate into
    // two chains, so consecutive MFMAs do not wait on each other's result
    constexpr bool DA = RB > 1;
    us_f32x16 acc[MI][CB], accb[MI][CB];
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < CB; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = accb[i][j][r] = 0.f;
    };
    auto fold_acc = [&]() __attribute__((always_inline)) {
        if constexpr (DA) {
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < CB; ++j) acc[i][j] += accb[i][j];
        }
    };
    zero_acc();

    // B fragments: column wn*64 + j*32 + l32, 8 channels at 8*hh
    const int col0 = wn * 32 * CB + l32;
    struct BFr {
        us_h8 h[CB], l[CB], m[CB];
    };
    auto read_b = [&](int s, BFr& f) __attribute__((always_inline)) {
        int row, ch;
        if (s < S1) {
            const int tap = s / CG;
            row = col0 + tap * a.d;
            ch = (s - tap * CG) * 16;
        } else {
            row = col0;
            ch = (s - S1) * 16;
        }
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            const int off = (row + j * 32) * PH + ch + 8 * hh;
            if constexpr (F32) {   // 8 floats: channels 8hh..8hh+7 of the step's 16
                f.h[j] = *reinterpret_cast<const us_h8*>(pf + off);
                f.l[j] = *reinterpret_cast<const us_h8*>(pf + off + 4);
            } else {
                f.h[j] = *reinterpret_cast<const us_h8*>(ph + off);
                f.l[j] = *reinterpret_cast<const us_h8*>(pl + off);
                if constexpr (BF) f.m[j] = *reinterpret_cast<const us_h8*>(pm + off);
            }
        }
    };
    // execution order of the K-steps.  Cooperative form: phase 2 starts with the
    // member's own channel block (its planes are ready before the hand-off) and
    // wraps round; the weight ring follows the same order.
    auto smap = [&](int t) __attribute__((always_inline)) {
        if (RB == 1 || t < S1 || t >= ST) return t;   // (past ST: the ring's tail reads nothing)
        int u = t - S1 + rb * (CG / RB);
        if (u >= CG) u -= CG;
        return S1 + u;
    };
    auto step = [&](int t, int s, const BFr& f, us_f32x16 (&acc)[MI][CB]) __attribute__((always_inline)) {
        us_h8 ah[MI], al[MI], a2[MI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            ah[i] = ring[t % R][i][0];
            al[i] = ring[t % R][i][1];
            a2[i] = ah[i] * (_Float16)2048.0f;
        }
        if constexpr (BF) {
            us_b8 wh[MI], wl[MI], wmd[MI];
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                wh[i] = __builtin_bit_cast(us_b8, ring[t % R][i][0]);
                wl[i] = __builtin_bit_cast(us_b8, ring[t % R][i][1]);
                wmd[i] = __builtin_bit_cast(us_b8, ring[t % R][i][2]);
            }
            load_a(t % R, RB > 1 ? smap(t + R) : s + R * KG);   // refill the slot (runs on into W2)
            // smallest products first: lo*hi, hi*lo, mid*mid, mid*hi, hi*mid, hi*hi
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < CB; ++j) {
                    const us_b8 xh = __builtin_bit_cast(us_b8, f.h[j]), xl = __builtin_bit_cast(us_b8, f.l[j]),
                                xm = __builtin_bit_cast(us_b8, f.m[j]);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl[i], xh, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh[i], xl, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wmd[i], xm, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wmd[i], xh, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh[i], xm, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh[i], xh, acc[i][j], 0, 0, 0);
                }
            return;
        }
        load_a(t % R, RB > 1 ? smap(t + R) : s + R * KG);   // refill the slot (runs on into W2)
        if constexpr (F32) {
#pragma unroll
            for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int i = 0; i < MI; ++i)
#pragma unroll
                        for (int j = 0; j < CB; ++j) {
                            const us_f32x4 wv = __builtin_bit_cast(us_f32x4, hf ? al[i] : ah[i]);
                            const us_f32x4 xv = __builtin_bit_cast(us_f32x4, hf ? f.l[j] : f.h[j]);
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[e], xv[e], acc[i][j], 0, 0, 0);
                        }
            return;
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < CB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2[i], f.h[j], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < CB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], f.l[j], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < CB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], f.h[j], acc[i][j], 0, 0, 0);
    };

    // per-lane rows of the accumulators: m = 32 MI wm + 32i + 8g + 4hh + e
    const int mrow0 = 32 * MI * wmg + 4 * hh;
    // own K-steps [t0, t1) of this wave's group: global step t*KG + GG
    auto kloop = [&](auto gtag, auto t0tag, auto t1tag) __attribute__((always_inline)) {
        constexpr int GG = decltype(gtag)::value;
        constexpr int T0 = decltype(t0tag)::value, T1 = decltype(t1tag)::value;
        BFr f[2];
        auto sidx = [&](int t) __attribute__((always_inline)) { return RB > 1 ? smap(t) : t * KG + GG; };
        read_b(sidx(T0), f[0]);
#pragma unroll
        for (int t = T0; t < T1; ++t) {
            if (t + 1 < T1) read_b(sidx(t + 1), f[(t + 1 - T0) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            if (DA && ((t - T0) & 1)) step(t, sidx(t), f[(t - T0) & 1], accb);
            else step(t, sidx(t), f[(t - T0) & 1], acc);
        }
    };
    // group 1 hands its partial sums to group 0 through LDS (over the dead planes)
    float* red = reinterpret_cast<float*>(lds);
    auto combine = [&]() __attribute__((always_inline)) {
        if constexpr (KG == 2) {
            __syncthreads();                         // planes dead
            float* mine = red + twave * (MI * CB * 16 * 64);
            if (kg == 1) {
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < CB; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) mine[((i * CB + j) * 16 + r) * 64 + lane] = acc[i][j][r];
            }
            __syncthreads();
            if (kg == 0) {
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < CB; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) acc[i][j][r] += mine[((i * CB + j) * 16 + r) * 64 + lane];
            }
        }
    };
    if (KG == 1 || kg == 0) kloop(IC<0>{}, IC<0>{}, IC<S1 / KG>{});
    else kloop(IC<1>{}, IC<0>{}, IC<S1 / KG>{});
    fold_acc();
    combine();
    __syncthreads();                                 // window (and hand-off area) dead
    US_AT(2, 2);

    // ------------------------------------------------------------ seam: h = act2(h*rs1 + b1) -> planes
    // (phase 1 ran on act0(x) 2^-sh0: its scale 2^sh0 rides on rs1; xs = the
    // range guard's scale of h; returns max |h xs| of the thread's values)
    const float f0 = ldexpf(1.0f, sh0);
    // cooperative form: this group's exchange slot (act2(h) as [BN columns][C] fp32)
    const auto xcrs = us_rsrc(a.xch, RB > 1 ? a.xch_bytes : 0);
    const unsigned xslot = (unsigned)lg * (unsigned)(G::BN * C);
    auto seam = [&](float xs, auto pubtag) __attribute__((always_inline)) {
        constexpr bool publish = decltype(pubtag)::value != 0 && RB > 1;
        float cmax = 0.f;
        if (KG == 1 || kg == 0) {
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int m = mrow0 + 32 * i + 8 * g;
                    const us_f32x4 rs = *reinterpret_cast<const us_f32x4*>(tab + m) * f0;
                    const us_f32x4 bb = *reinterpret_cast<const us_f32x4*>(tab + C + m);
                    us_f32x4 al = {0.f, 0.f, 0.f, 0.f};
                    if constexpr (SNAKE) al = *reinterpret_cast<const us_f32x4*>(tab + 2 * C + m);
#pragma unroll
                    for (int j = 0; j < CB; ++j) {
                        us_f32x4 v;
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            v[e] = us_act<SNAKE>(acc[i][j][4 * g + e] * rs[e] + bb[e], slope, al[e]) * xs;
                        if constexpr (publish)   // write-through (sc1): read by the other members
                            __builtin_amdgcn_raw_buffer_store_b128(
                                __builtin_bit_cast(us_u32x4, v), xcrs,
                                (xslot + (unsigned)((col0 + 32 * j) * C + m)) * 4u, 0, 16);
                        if constexpr (F32) {
                            *reinterpret_cast<us_f32x4*>(pf + (col0 + 32 * j) * PH + m) = v;
                            continue;
                        }
                        if constexpr (BF) {
                            us_b4 hi, mid, lo;
                            bf3_split(v, hi, mid, lo);
                            *reinterpret_cast<us_b4*>(ph + (col0 + 32 * j) * PH + m) = hi;
                            *reinterpret_cast<us_b4*>(pl + (col0 + 32 * j) * PH + m) = lo;
                            *reinterpret_cast<us_b4*>(pm + (col0 + 32 * j) * PH + m) = mid;
                            continue;
                        }
#pragma unroll
                        for (int e = 0; e < 4; ++e) cmax = fmaxf(cmax, fabsf(v[e]));
                        const us_h4 hv = __builtin_convertvector(v, us_h4);
                        const us_h4 lv = __builtin_convertvector((v - __builtin_convertvector(hv, us_f32x4)) * 2048.0f, us_h4);
                        *reinterpret_cast<us_h4*>(ph + (col0 + 32 * j) * PH + m) = hv;
                        *reinterpret_cast<us_h4*>(pl + (col0 + 32 * j) * PH + m) = lv;
                    }
                }
        }
        return cmax;
    };
    bool gave_up = false;                        // cooperative seam: a member never arrived
    if constexpr (RB == 1) {                     // range guard of h (rare path: h * 2^-sh2)
        const float cmax = seam(1.0f, IC<0>{});
        if constexpr (GV) vote_cast(vote, wave, cmax);
        __syncthreads();
        if (GV && __builtin_expect(vote_any<G::NW>(vote), 0)) {
            sh2 = __builtin_amdgcn_readfirstlane(split_shift(block_max<G::NW>(cmax, vred)));
            (void)seam(ldexpf(1.0f, -sh2), IC<0>{});
            __syncthreads();
        }
    } else {
        // publish own rows (and own planes, optimistically unscaled), then the
        // workgroup's max |h|; every storing wave drains; one lane signals
        const float cmax = seam(1.0f, IC<1>{});
        const float mx = block_max<G::NW>(cmax, vred);
        unsigned* arrive = a.flags + a.flag_stride * lg;
        if (tid == 0)
            __hip_atomic_store(reinterpret_cast<unsigned*>(a.xmax) + lg * RB + rb, __builtin_bit_cast(unsigned, mx),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // phase 2 over the member's own rows while the others finish publishing
        constexpr int OWN = S1 + CG / RB;
        zero_acc();
        US_AT(3, 3);
        kloop(IC<0>{}, IC<S1>{}, IC<OWN>{});
        US_AT(-1, 4);
        if (wave == 0) {
            unsigned spins = 0;
            bool ok = true;
            for (;;) {
                const unsigned n = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (n >= (unsigned)RB) break;
                if (++spins > a.spin_limit) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (a.force_giveup) ok = false;
            // one workgroup per CU (SC1X): the exchanged bytes are read by sc1 loads
            // below, which replace the agent acquire (MI355X_MICROARCH.md, hand-off
            // table row 1: sc1 stores drained before the counter add, an sc1 poll,
            // sc1 loads behind the barrier this wave joins); else the acquire
            if constexpr (!SC1X) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (lane == 0) {
                vote[0] = ok ? 0 : 1;
                if (!ok) {
                    __hip_atomic_store(a.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (a.status) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
        __syncthreads();
        US_AT(6, 5);
        gave_up = __builtin_amdgcn_readfirstlane(vote[0]) != 0;
        // group-wide range guard: the members' maxima (vector sc1 loads, not the scalar path)
        float gmax = 0.f;
#pragma unroll
        for (int r = 0; r < RB; ++r)
            gmax = fmaxf(gmax, __builtin_bit_cast(float, __hip_atomic_load(reinterpret_cast<unsigned*>(a.xmax) + lg * RB + r,
                                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
        if constexpr (AR == 0) sh2 = __builtin_amdgcn_readfirstlane((RAVE_SPLIT_GUARD && gmax >= kSplitLimit) ? split_shift(gmax) : 0);
        // stage the other members' rows (all rows, scaled, on the rare guarded path)
        auto stage_rows = [&](auto alltag, float xs) __attribute__((always_inline)) {
            constexpr bool all = decltype(alltag)::value != 0;
            constexpr int NG = all ? C / 8 : C / 8 - G::G8R;           // 8-channel groups per column
            constexpr int NTK = (G::BN * NG + NT - 1) / NT;
            us_f32x4 v0[NTK], v1[NTK];
#pragma unroll
            for (int i = 0; i < NTK; ++i) {
                const int e = min(tid + i * NT, G::BN * NG - 1);
                const int w = e / NG;
                int g = e - w * NG;
                if (!all && g >= rb * G::G8R) g += G::G8R;
                if constexpr (SC1X) {
                    const unsigned off = (xslot + (unsigned)(w * C + g * 8)) * 4u;
                    v0[i] = __builtin_bit_cast(us_f32x4, __builtin_amdgcn_raw_buffer_load_b128(xcrs, off, 0, 16));
                    v1[i] = __builtin_bit_cast(us_f32x4, __builtin_amdgcn_raw_buffer_load_b128(xcrs, off + 16u, 0, 16));
                } else {
                    const float* src = a.xch + xslot + w * C + g * 8;
                    v0[i] = *reinterpret_cast<const us_f32x4*>(src);
                    v1[i] = *reinterpret_cast<const us_f32x4*>(src + 4);
                }
            }
#pragma unroll
            for (int i = 0; i < NTK; ++i) {
                const int e = tid + i * NT;
                if (e >= G::BN * NG) break;
                const int w = e / NG;
                int g = e - w * NG;
                if (!all && g >= rb * G::G8R) g += G::G8R;
                if constexpr (F32) {
                    *reinterpret_cast<us_f32x4*>(pf + w * PH + g * 8) = v0[i];
                    *reinterpret_cast<us_f32x4*>(pf + w * PH + g * 8 + 4) = v1[i];
                } else if constexpr (BF) {
                    const us_f32x8 v8 = us_f32x8{v0[i][0], v0[i][1], v0[i][2], v0[i][3],
                                                 v1[i][0], v1[i][1], v1[i][2], v1[i][3]};
                    us_b8 hi, mid, lo;
                    bf3_split(v8, hi, mid, lo);
                    *reinterpret_cast<us_b8*>(ph + w * PH + g * 8) = hi;
                    *reinterpret_cast<us_b8*>(pl + w * PH + g * 8) = lo;
                    *reinterpret_cast<us_b8*>(pm + w * PH + g * 8) = mid;
                } else {
                    const us_f32x8 v8 = us_f32x8{v0[i][0], v0[i][1], v0[i][2], v0[i][3],
                                                 v1[i][0], v1[i][1], v1[i][2], v1[i][3]} * xs;
                    const us_h8 hi = __builtin_convertvector(v8, us_h8);
                    const us_h8 lo = __builtin_convertvector((v8 - __builtin_convertvector(hi, us_f32x8)) * 2048.0f, us_h8);
                    *reinterpret_cast<us_h8*>(ph + w * PH + g * 8) = hi;
                    *reinterpret_cast<us_h8*>(pl + w * PH + g * 8) = lo;
                }
            }
        };
        auto depart = [&]() __attribute__((always_inline)) {
            // the last member to leave re-arms the group's counters
            if (tid == 0) {
                const unsigned prev = __hip_atomic_fetch_add(arrive + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (prev == (unsigned)RB - 1) {
                    __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(arrive + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        };
        if (__builtin_expect(sh2 != 0, 0)) {
            // rare: h past the f16 range somewhere in the group -- every row again
            // as h 2^-sh2, and the own block's K-steps again (ring refilled in order)
            stage_rows(IC<1>{}, ldexpf(1.0f, -sh2));
            __syncthreads();
            zero_acc();
#pragma unroll
            for (int t = S1; t < S1 + R; ++t) load_a(t % R, smap(t));
            kloop(IC<0>{}, IC<S1>{}, IC<OWN>{});
        } else {
            stage_rows(IC<0>{}, 1.0f);
            __syncthreads();
        }
        US_AT(-1, 6);
        depart();
        kloop(IC<0>{}, IC<OWN>{}, IC<ST>{});
    }
    if constexpr (RB == 1) {
        zero_acc();
        US_AT(3, 3);
        if (KG == 1 || kg == 0) kloop(IC<0>{}, IC<S1 / KG>{}, IC<ST / KG>{});
        else kloop(IC<1>{}, IC<S1 / KG>{}, IC<ST / KG>{});
    }
    fold_acc();
    combine();
    // unguarded pass: any non-finite output sum of a live column -> run again
    // guarded.  The flag is taken here; the workgroup vote follows the epilogue's
    // stores (KG == 1: the second pass rewrites them; a barrier there costs no
    // wave anything), or comes here (KG == 2: the partner waves leave below)
    constexpr bool CHECK = !GUARD && AR == 0 && RAVE_SPLIT_GUARD != 0;
    bool bad = false;
    if constexpr (CHECK) {
        if (KG == 1 || kg == 0) {
#pragma unroll
            for (int j = 0; j < CB; ++j) {
                const bool nok = n0 + col0 + 32 * j < a.T;
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int r = 0; r < 16; ++r) bad |= nok && !__builtin_isfinite(acc[i][j][r]);
            }
        }
    }
    auto vote_rerun = [&]() __attribute__((always_inline)) {
        vote_cast_any(vote, wave, bad);
        __syncthreads();
        if (__builtin_expect(vote_any<G::NW>(vote), 0)) {
            __syncthreads();                         // every wave read the vote
            return true;
        }
        return false;
    };
    if constexpr (CHECK && KG == 2) {
        if (vote_rerun()) return false;
    }
    if (KG == 2 && kg == 1) return true;             // (no barrier follows)

    US_AT(4, -1);
    // ------------------------------------------------------------ epilogue: y*rs2 + b2 + x
    // every residual load issued before the first store (one exposed latency)
    {
        const float f2 = ldexpf(1.0f, sh2);
        const auto yrs = us_rsrc(a.y + (int64_t)b * a.y_sb, a.y_bytes);
        float res[MI][CB][16];
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            const int n = n0 + col0 + 32 * j;
            const bool nok = n < a.T;
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = mrow0 + 32 * i + 8 * (r >> 2) + (r & 3);
                    res[i][j][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                        xrs, nok ? (unsigned)(m * a.x_sc + n + a.rsh) * 4u : kUSOOB, 0, 0));
                }
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int m = mrow0 + 32 * i + 8 * g;
                const us_f32x4 rs = *reinterpret_cast<const us_f32x4*>(tab + 3 * C + m) * f2;
                const us_f32x4 bb = *reinterpret_cast<const us_f32x4*>(tab + 4 * C + m);
#pragma unroll
                for (int j = 0; j < CB; ++j) {
                    const int n = n0 + col0 + 32 * j;
                    const bool nok = n < a.T;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        __builtin_amdgcn_raw_buffer_store_b32(
                            __builtin_bit_cast(unsigned, gave_up ? __builtin_nanf("")
                                                                 : acc[i][j][4 * g + e] * rs[e] + bb[e] + res[i][j][4 * g + e]),
                            yrs, nok ? (unsigned)((m + e) * a.y_sc + n) * 4u : kUSOOB, 0, RAVE_YAUX);
                }
            }
    }
    US_AT(5, -1);
    if constexpr (CHECK && KG == 1) {
        if (vote_rerun()) return false;
    }
    return true;
}

template <int C, int WGN, int MI, int KG, int CB, bool SNAKE, int RB>
__global__ __launch_bounds__(64 * (C / (32 * MI * RB)) * WGN * KG) void unit_split_kernel(USArgs a) {
    if constexpr (RB > 1 || RAVE_SPLIT_GUARD == 0) {
        (void)unit_split_body<C, WGN, MI, KG, CB, SNAKE, 0, RB, true>(a);
    } else {
        if (!unit_split_body<C, WGN, MI, KG, CB, SNAKE, 0, RB, false>(a))
            (void)unit_split_body<C, WGN, MI, KG, CB, SNAKE, 0, RB, true>(a);
    }
}
template <int C, int WGN, int MI, int KG, int CB, bool SNAKE, int RB>
__global__ __launch_bounds__(64 * (C / (32 * MI * RB)) * WGN * KG) void unit_ring_f32_kernel(USArgs a) {
    (void)unit_split_body<C, WGN, MI, KG, CB, SNAKE, 1, RB, false>(a);
}
template <int C, int WGN, int MI, int KG, int CB, bool SNAKE, int RB>
__global__ __launch_bounds__(64 * (C / (32 * MI * RB)) * WGN * KG) void unit_bf3_kernel(USArgs a) {
    (void)unit_split_body<C, WGN, MI, KG, CB, SNAKE, 2, RB, false>(a);
}

// cooperative launches of this process that can run at once: its hardware
// queues (GPU_MAX_HW_QUEUES; HIP's default 4)
static int coop_max_queues() {
    static const int q = [] {
        const char* e = std::getenv("GPU_MAX_HW_QUEUES");
        const int v = e ? std::atoi(e) : 0;
        return v > 0 ? v : 4;
    }();
    return q;
}

// ar: 0 split16, 1 exact fp32 (ring), 2 bf16x3
template <int C, int WGN, int MI, int KG, int CB, int RB = 1>
static int us_launch(USArgs k, int B, bool snake, int ar, hipStream_t st) {
    using G = USGeo<C, WGN, MI, KG, CB, RB>;
    using G3 = USGeo<C, WGN, MI, KG, CB, RB, 3>;
    const bool f32 = ar == 1;
    if (k.XW > (ar == 2 ? G3::XW_MAX : G::XW_MAX)) {
        set_error(ar == 2 && C == 512 ? "residual_unit(bf16x3): C = 512 supports dilations <= 4"
                                      : "residual_unit(split16): dilation too large");
        return RAVE_ERR_UNSUPPORTED;
    }
    k.ntiles = ceil_div(k.T, G::BN);
    void (*kern)(USArgs) = nullptr;
    int lds = G::LDS;
    if (ar == 2) {
        // three operand planes: built where they fit the CU's LDS
        if constexpr (G3::LDS <= 160 * 1024) {
            kern = snake ? unit_bf3_kernel<C, WGN, MI, KG, CB, true, RB> : unit_bf3_kernel<C, WGN, MI, KG, CB, false, RB>;
            lds = G3::LDS;
        } else {
            set_error("residual_unit(bf16x3): this width does not fit the CU's LDS as three planes");
            return RAVE_ERR_UNSUPPORTED;
        }
    } else {
        kern = f32 ? (snake ? unit_ring_f32_kernel<C, WGN, MI, KG, CB, true, RB> : unit_ring_f32_kernel<C, WGN, MI, KG, CB, false, RB>)
                   : (snake ? unit_split_kernel<C, WGN, MI, KG, CB, true, RB> : unit_split_kernel<C, WGN, MI, KG, CB, false, RB>);
    }
    static bool attr[6] = {false, false, false, false, false, false};
    if (lds > 65536 && !attr[2 * ar + snake]) {
        RAVE_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        attr[2 * ar + snake] = true;
    }
    int grid = k.ntiles * B;
    if constexpr (RB > 1) {
        // Forward progress needs a whole group resident on one XCD at once.  A
        // launch's workgroups reach an XCD in order and a group's members are
        // consecutive there, so at any moment a launch holds at most ONE partial
        // group per XCD (RB - 1 slots).  With Q cooperative launches of this
        // process in flight together (at most its hardware queues,
        // GPU_MAX_HW_QUEUES, 4 by default: engines on several streams, bench's
        // pipelined leg), the partial groups hold at most Q (RB - 1) of the XCD's
        // workgroup slots; if the XCD has room for RB more, some group is whole,
        // finishes and frees slots, and so on.  Kernels of other kinds only
        // delay (they finish unconditionally).  So the cooperative form runs
        // only where slots per XCD >= Q (RB - 1) + RB; else the caller runs the
        // one-workgroup form.  (Other processes sharing the GPU are not counted.)
        // Assumptions, stated: each hardware queue runs one kernel at a time
        // toward this bound (HIP sets the AQL barrier bit on every dispatch of a
        // stream), and the Q launches may be DIFFERENT cooperative kernels with
        // different footprints (C = 256 RB = 2 beside C = 512 RB = 4, split16 /
        // bf16x3 / fp32): a foreign partial group is charged a whole CU per member
        // (the most one workgroup can hold) with the largest group size of any
        // instantiation, kCoopMaxRB -- the second condition below.  Both hold on
        // MI355X by a wide margin (C = 512: 32 >= 16 slots and 32 >= 16 CUs).
        static int fits[6] = {-1, -1, -1, -1, -1, -1};
        int& f = fits[2 * ar + snake];
        if (f < 0) {
            int per_cu = 0, dev = 0, cus = 0;
            RAVE_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern),
                                                                        G::NT, lds));
            RAVE_CHECK_HIP(hipGetDevice(&dev));
            RAVE_CHECK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            const int64_t q = coop_max_queues();
            f = ((int64_t)per_cu * (cus / kXcds) >= q * (RB - 1) + RB &&
                 (int64_t)(cus / kXcds) >= q * (kCoopMaxRB - 1) + RB) ? 1 : 0;
        }
        if (!f) return kCoopNoFit;
        k.ngroups = grid;
        grid = ceil_div(grid, 8) * 8 * RB;          // whole groups per XCD slot
    }
    launch(kern, dim3(grid), dim3(G::NT), (uint32_t)lds, st, k);
    return launch_status(ar == 2 ? "unit_bf3_kernel" : f32 ? "unit_ring_f32_kernel" : "unit_split_kernel");
}

static bool us_supported(int C) { return C == 64 || C == 128 || C == 256 || C == 512; }

// Power-of-two row exponent: max |w * 2^e| in [8, 16) (e = 0 for an all-zero row).
static int us_row_exponent(double amax) {
    if (!(amax > 0.0)) return 0;
    int e = (int)std::floor(std::log2(16.0 / amax));
    while (std::ldexp(amax, e) >= 16.0) --e;
    while (std::ldexp(amax, e) < 8.0) ++e;
    return e;
}


}  // namespace rave

using namespace rave;

// packed: fragments [C/32 m-blocks][S1+S2 K-steps][hi, lo][64 lanes][8 halves], then
// rs1[C], rs2[C] (floats).  Sizes in floats.
extern "C" int64_t rave_unit_split_packed_size(int C) {
    if (!us_supported(C)) return -1;
    const int ST = 4 * C / 16;
    return (int64_t)(C / 32) * ST * 2 * 256 + 2 * C;
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

// mode: 0 split16 (hi, lo f16, row scales), 1 exact fp32, 2 bf16x3 (hi, lo, mid)
static int unit_pack(const float* w1, const float* w2, int C, float* packed, int mode) {
    const bool f32 = mode != 0;                      // (no row scales)
    const int NPW = mode == 2 ? 3 : 2;
    RAVE_CHECK_ARG(w1 && w2 && packed, "unit_split_pack_weight: null pointer");
    if (!us_supported(C)) {
        set_error("unit_split_pack_weight: split16 fused residual unit supports C in {64, 128, 256, 512}");
        return RAVE_ERR_UNSUPPORTED;
    }
    const int S1 = 3 * C / 16, ST = 4 * C / 16, CG = C / 16;
    std::vector<int> e1(C), e2(C);
    for (int m = 0; m < C; ++m) {
        double a1 = 0.0, a2 = 0.0;
        for (int k = 0; k < 3 * C; ++k) a1 = std::max(a1, (double)std::fabs(w1[(int64_t)m * 3 * C + k]));
        for (int k = 0; k < C; ++k) a2 = std::max(a2, (double)std::fabs(w2[(int64_t)m * C + k]));
        e1[m] = f32 ? 0 : us_row_exponent(a1);
        e2[m] = f32 ? 0 : us_row_exponent(a2);
    }
    _Float16* out = reinterpret_cast<_Float16*>(packed);
    uint16_t* bout = reinterpret_cast<uint16_t*>(packed);
    for (int mb = 0; mb < C / 32; ++mb)
        for (int s = 0; s < ST; ++s) {
            uint16_t* bp = bout + ((int64_t)(mb * ST + s) * 3) * 512;   // bf16x3: hi, lo, mid
            _Float16* hi = out + ((int64_t)(mb * ST + s) * 2) * 512;
            _Float16* lo = hi + 512;
            float* f32s = packed + ((int64_t)(mb * ST + s) * 2) * 256;   // fp32: floats 0-3 slot 0, 4-7 slot 1
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 8; ++e) {
                    const int m = mb * 32 + (l & 31);
                    const int kk = 8 * (l >> 5) + e;
                    float v;
                    if (s < S1) {
                        const int tap = s / CG, ci = (s % CG) * 16 + kk;
                        v = std::ldexp(w1[((int64_t)m * C + ci) * 3 + tap], e1[m]);
                    } else {
                        const int ci = (s - S1) * 16 + kk;
                        v = std::ldexp(w2[(int64_t)m * C + ci], e2[m]);
                    }
                    if (mode == 2) {
                        const uint16_t h = bf16_bits(v);
                        const float r = v - bf16_value(h);
                        const uint16_t md = bf16_bits(r);
                        bp[l * 8 + e] = h;
                        bp[1024 + l * 8 + e] = md;
                        bp[512 + l * 8 + e] = bf16_bits(r - bf16_value(md));
                        continue;
                    }
                    if (f32) {
                        f32s[(e >> 2) * 256 + l * 4 + (e & 3)] = v;
                        continue;
                    }
                    const _Float16 vh = (_Float16)v;
                    hi[l * 8 + e] = vh;
                    lo[l * 8 + e] = (_Float16)((v - (float)vh) * 2048.0f);
                }
        }
    float* rs = packed + (int64_t)(C / 32) * ST * NPW * 256;
    for (int m = 0; m < C; ++m) {
        rs[m] = f32 ? 1.0f : (float)std::ldexp(1.0, -(e1[m] + 11));
        rs[C + m] = f32 ? 1.0f : (float)std::ldexp(1.0, -(e2[m] + 11));
    }
    return RAVE_OK;
}

extern "C" int rave_unit_split_pack_weight(const float* w1, const float* w2, int C, float* packed) {
    return unit_pack(w1, w2, C, packed, 0);
}

extern "C" int rave_unit_ring_pack_weight(const float* w1, const float* w2, int C, float* packed) {
    return unit_pack(w1, w2, C, packed, 1);
}

// bf16x3: fragments [C/32][S1+S2][hi, lo, mid][64 lanes][8 bf16], then rs1, rs2 (= 1)
extern "C" int64_t rave_unit_bf3_packed_size(int C) {
    if (!us_supported(C)) return -1;
    const int ST = 4 * C / 16;
    return (int64_t)(C / 32) * ST * 3 * 256 + 2 * C;
}

extern "C" int rave_unit_bf3_pack_weight(const float* w1, const float* w2, int C, float* packed) {
    return unit_pack(w1, w2, C, packed, 2);
}

#ifdef RAVE_STAMPS
extern "C" int rave_diag_unit_stamps(void* p) {
    RAVE_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_us_stamps), &p, sizeof(p)));
    return RAVE_OK;
}
#endif

namespace rave {
// debug overrides of the cooperative hand-off (rave_debug_coop)
static std::atomic<unsigned> g_coop_spin{kUSSpinLimit};
static std::atomic<int> g_coop_force{0};
// Cooperative form (header comment): C = 256 and 512, groups of C/128 workgroups
// over 32-column slabs.  RAVE_UNIT_COOP=0 keeps one workgroup per slab (A/B).
static bool coop_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("RAVE_UNIT_COOP");
        return !(e && e[0] == '0');
    }();
    return on;
}
constexpr int kCoopBN = 32;
struct CoopLayout {
    int rb = 1, stride = 2;                               // counter words per group
    int64_t groups = 0, xmax = 0, xch = 0, floats = 0;   // offsets / sizes in floats
};
static CoopLayout coop_layout(const rave_unit_args& a) {
    CoopLayout L;
    const int C = a.channels;
    if ((C != 256 && C != 512) || !coop_enabled() || a.batch <= 0 || a.t_len <= 0) return L;
    if (a.precision != RAVE_PREC_SPLIT16 && a.precision != RAVE_PREC_F32_RING && a.precision != RAVE_PREC_BF16X3)
        return L;
    const int64_t ng = (int64_t)ceil_div(a.t_len, kCoopBN) * a.batch;
    const int64_t ngp = ceil_div64(ng, 8) * 8;
    // counters live in the split-K ticket words (zero at rest, as the conv
    // kernels leave theirs); the reserved last word is the give-up word
    if (2 * ngp > RAVE_SPLITK_STATUS_WORD) return L;
    // a group's counters on a 128-byte line of their own where the words allow
    while (L.stride < 32 && 2 * L.stride * ngp <= RAVE_SPLITK_STATUS_WORD) L.stride *= 2;
    // group size: C / 128, or the wide group (coop_rb = 4 at C = 256: twice the CUs
    // stream the slab's weights -- short inputs, where few slabs leave CUs idle)
    const int rb = a.coop_rb == 4 && C == 256 ? 4 : C / 128;
    if (a.coop_rb != 0 && a.coop_rb != rb) return L;      // (refused by residual_unit_split)
    L.groups = ng;
    L.xmax = RAVE_SPLITK_TICKETS;
    L.xch = L.xmax + ceil_div64(ngp * rb, 64) * 64;
    L.floats = L.xch + ngp * kCoopBN * C;
    if (ngp * kCoopBN * C * 4 >= (1ll << 31)) return CoopLayout{};
    L.rb = rb;
    return L;
}

int residual_unit_split(const rave_unit_args& a, void* stream) {
    const int C = a.channels;
    if (!us_supported(C)) {
        set_error("residual_unit(split16): fused unit supports C in {64, 128, 256, 512}");
        return RAVE_ERR_UNSUPPORTED;
    }
    if (a.coop_rb != 0 && !((C == 256 && (a.coop_rb == 2 || a.coop_rb == 4)) || (C == 512 && a.coop_rb == 4))) {
        set_error("residual_unit: coop_rb must be 0, or 2 / 4 at C = 256, 4 at C = 512");
        return RAVE_ERR_ARG;
    }
    USArgs k{};
    k.x = a.x; k.y = a.y; k.w = a.weight;
    const int ar = a.precision == RAVE_PREC_BF16X3 ? 2 : a.precision == RAVE_PREC_F32_RING ? 1 : 0;
    const int64_t frag = (int64_t)(C / 32) * (4 * C / 16) * (ar == 2 ? 3 : 2) * 256;
    k.rs1 = a.weight + frag; k.rs2 = a.weight + frag + C;
    k.b1 = a.bias1; k.b2 = a.bias2; k.a0 = a.alpha0; k.a2 = a.alpha2;
    k.x_sb = a.x_sb; k.x_sc = a.x_sc; k.y_sb = a.y_sb; k.y_sc = a.y_sc;
    k.T = a.t_len; k.d = a.dilation; k.pad_l = a.pad_left;
    k.XL = a.x_len > 0 ? a.x_len : a.t_len;
    k.rsh = a.res_shift;
    k.act = a.act; k.slope = a.leaky_slope;
    const int64_t xb = ((int64_t)(C - 1) * a.x_sc + k.XL) * 4;
    const int64_t yb = ((int64_t)(C - 1) * a.y_sc + a.t_len) * 4;
    RAVE_CHECK_ARG(xb < (1ll << 31) && yb < (1ll << 31), "residual_unit: tensors beyond 2 GiB per item");
    k.x_bytes = (int)xb; k.y_bytes = (int)yb;
    k.w_bytes = (int)(frag * 4);
    k.bias_bytes = a.bias1 ? C * 4 : 0;
    const bool snake = a.act == RAVE_ACT_SNAKE;
    hipStream_t st = as_stream(stream);
    // one 32-row block per wave (MI = 1): C/32 waves along rows, 64 columns each
    // (measured against two row blocks per wave, other column counts and
    // K-groups: tools/layer_bench.py unit_64/128/256)
    auto go = [&](auto cc, auto wgn, auto mi, auto kgt, auto cb, auto rbt) {
        constexpr int CC = decltype(cc)::value, WGN = decltype(wgn)::value, MI = decltype(mi)::value,
                      KG = decltype(kgt)::value, CB = decltype(cb)::value, RB = decltype(rbt)::value;
        k.XW = USGeo<CC, WGN, MI, KG, CB, RB>::BN + 2 * a.dilation;
        k.xw_magic = (unsigned)(((1u << 24) + k.XW - 1) / k.XW);
        const int off = (4 - a.pad_left % 4) % 4;      // window start past its 4-aligned block start
        const int nb = (off + k.XW + 3) / 4;
        k.nb_magic = (unsigned)(((1u << 24) + nb - 1) / nb);
        return us_launch<CC, WGN, MI, KG, CB, RB>(k, a.batch, snake, ar, st);
    };
    k.xv = (k.XL % 4 == 0 && a.x_sc % 4 == 0 && a.x_sb % 4 == 0 &&
            reinterpret_cast<uintptr_t>(a.x) % 16 == 0 && std::getenv("RAVE_UNIT_XV") == nullptr) ? 1 : 0;
    // cooperative form when the caller passed its workspace
    const CoopLayout L = coop_layout(a);
    if (L.rb > 1 && a.workspace) {
        k.flag_stride = L.stride;
        k.flags = reinterpret_cast<unsigned*>(a.workspace);
        k.tmo = k.flags + RAVE_SPLITK_STATUS_WORD;
        k.status = a.status;
        k.spin_limit = g_coop_spin.load(std::memory_order_relaxed);
        k.force_giveup = g_coop_force.load(std::memory_order_relaxed);
        k.xmax = a.workspace + L.xmax;
        k.xch = a.workspace + L.xch;
        k.xch_bytes = (int)((L.floats - L.xch) * 4);
        const int rc = C == 512 ? go(IC<512>{}, IC<1>{}, IC<1>{}, IC<1>{}, IC<1>{}, IC<4>{})
                       : L.rb == 4 ? go(IC<256>{}, IC<1>{}, IC<1>{}, IC<1>{}, IC<1>{}, IC<4>{})
                                   : go(IC<256>{}, IC<1>{}, IC<1>{}, IC<1>{}, IC<1>{}, IC<2>{});
        if (rc != kCoopNoFit) return rc;
        // (a group does not fit one XCD: the one-workgroup form below)
    }
    // (K-groups, KG = 2, measured slower for every C: 13.3/11.6/19.5 -> 16.8/12.0/21.5 us)
    // (WGN, CB) per C, measured (tools/layer_bench.py unit_*): C=256 with one
    // column block per wave 19.6 -> 14.4 us; C=128 11.6 -> 11.3 us; wider waves
    // (CB 3-4, one column wave) measured slower for C=64 and C=128
#ifndef RAVE_U64_CB
#define RAVE_U64_CB 2
#endif
#ifndef RAVE_U64_WGN
#define RAVE_U64_WGN 2
#endif
#ifndef RAVE_U128_WGN
#define RAVE_U128_WGN 2
#endif
    // exact fp32 (RAVE_PREC_F32_RING): its own geometry knobs (A/B builds; the
    // defaults are the split form's)
#ifndef RAVE_F64_WGN
#define RAVE_F64_WGN RAVE_U64_WGN
#endif
#ifndef RAVE_F64_CB
#define RAVE_F64_CB RAVE_U64_CB
#endif
#ifndef RAVE_F64_MI
#define RAVE_F64_MI 1
#endif
#ifndef RAVE_F128_WGN
#define RAVE_F128_WGN RAVE_U128_WGN
#endif
#ifndef RAVE_F128_CB
#define RAVE_F128_CB 1
#endif
#ifndef RAVE_F128_MI
#define RAVE_F128_MI 1
#endif
#ifndef RAVE_F256_WGN
#define RAVE_F256_WGN 1
#endif
#ifndef RAVE_F256_CB
#define RAVE_F256_CB 1
#endif
    if (a.precision == RAVE_PREC_F32_RING) {
        if (C == 64) return go(IC<64>{}, IC<RAVE_F64_WGN>{}, IC<RAVE_F64_MI>{}, IC<1>{}, IC<RAVE_F64_CB>{}, IC<1>{});
        if (C == 128) return go(IC<128>{}, IC<RAVE_F128_WGN>{}, IC<RAVE_F128_MI>{}, IC<1>{}, IC<RAVE_F128_CB>{}, IC<1>{});
        if (C == 256) return go(IC<256>{}, IC<RAVE_F256_WGN>{}, IC<1>{}, IC<1>{}, IC<RAVE_F256_CB>{}, IC<1>{});
    }
    // bf16x3: its own geometry knobs (A/B builds; the defaults are the split form's)
// C = 64 (round 5): four 32-column waves per 32-row block (8 waves, 128 VGPRs: four
// waves per SIMD at two workgroups per CU) against two 64-column waves (two per
// SIMD): unit_64 17.5 -> 16.4 us (profiles/r05_aa)
#ifndef RAVE_B64_WGN
#define RAVE_B64_WGN 4
#endif
#ifndef RAVE_B64_CB
#define RAVE_B64_CB 1
#endif
#ifndef RAVE_B64_MI
#define RAVE_B64_MI 1
#endif
#ifndef RAVE_B128_WGN
#define RAVE_B128_WGN RAVE_U128_WGN
#endif
#ifndef RAVE_B128_CB
#define RAVE_B128_CB 1
#endif
#ifndef RAVE_B128_MI
#define RAVE_B128_MI 1
#endif
    if (ar == 2) {
        if (C == 64) return go(IC<64>{}, IC<RAVE_B64_WGN>{}, IC<RAVE_B64_MI>{}, IC<1>{}, IC<RAVE_B64_CB>{}, IC<1>{});
        if (C == 128) return go(IC<128>{}, IC<RAVE_B128_WGN>{}, IC<RAVE_B128_MI>{}, IC<1>{}, IC<RAVE_B128_CB>{}, IC<1>{});
    }
    if (C == 64) return go(IC<64>{}, IC<RAVE_U64_WGN>{}, IC<1>{}, IC<1>{}, IC<RAVE_U64_CB>{}, IC<1>{});
#ifndef RAVE_U128_KG
#define RAVE_U128_KG 1
#endif
#ifndef RAVE_U256_KG
#define RAVE_U256_KG 1
#endif
    if (C == 128) return go(IC<128>{}, IC<RAVE_U128_WGN>{}, IC<1>{}, IC<RAVE_U128_KG>{}, IC<1>{}, IC<1>{});
    if (C == 256) return go(IC<256>{}, IC<1>{}, IC<1>{}, IC<RAVE_U256_KG>{}, IC<1>{}, IC<1>{});
    return go(IC<512>{}, IC<1>{}, IC<1>{}, IC<1>{}, IC<1>{}, IC<1>{});
}

}  // namespace rave

extern "C" int rave_debug_coop(int64_t spin_limit, int force_giveup) {
    rave::g_coop_spin.store(spin_limit < 0 ? rave::kUSSpinLimit
                                           : (unsigned)std::min<int64_t>(spin_limit, 0xFFFFFFFFll),
                            std::memory_order_relaxed);
    rave::g_coop_force.store(force_giveup ? 1 : 0, std::memory_order_relaxed);
    return RAVE_OK;
}

extern "C" int64_t rave_unit_workspace(const rave_unit_args* a) {
    RAVE_CHECK_ARG(a, "unit_workspace: null pointer");
    return rave::coop_layout(*a).floats;
}
