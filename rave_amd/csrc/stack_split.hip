// Fused residual stack on the f16 matrix cores (split-f16 arithmetic, as
// unit_split.hip): RAVE_STACK_UNITS consecutive Residual(DilatedUnit)s of one
// width -- the residual stacks of EncoderV2 (rave/blocks.py:533-558) and
// GeneratorV2 (rave/blocks.py:647-664), each unit
//
//     y_u = y_{u-1} + conv1x1_u(act2_u(conv3_{d_u}(act0_u(y_{u-1})) + b1_u)) + b2_u
//
// (rave/blocks.py:32-46, 84-113) -- in one launch.
//
// A workgroup owns BN output columns of one batch item and computes every unit
// over an extended range of BN + 64 columns (one 32-column block of margin per
// side).  The input window is read from HBM once; between units the running
// sum y stays in registers (each wave keeps its own 32 rows x 32*CB columns for
// the whole stack) and act0(y) goes back into the LDS planes.  Margin columns
// go stale unit by unit (their windows reach past the staged rows), but the
// receptive field of the centre columns stays inside the margin as long as
// pad_2 + pad_3 <= 32 and (2 d_2 - pad_2) + (2 d_3 - pad_3) <= 32 (host check).
// Sequence-boundary zero padding: planes hold 0 at columns outside [0, T).
//
// bf16x3 form (rave_stack_args.precision = RAVE_PREC_BF16X3; round 5): fp32 on
// the bf16 matrix cores as unit_split.hip's BF body -- every operand split
// exactly into hi + mid + lo bf16 (three LDS planes, three weight fragments per
// K-step from rave_unit_bf3_pack_weight), six v_mfma_f32_32x32x16_bf16 per
// K-step into one fp32 accumulator, no row scales and no range guard.  Three
// planes of the split form's 32-row halo do not fit the CU's LDS at C = 64 with
// 8 centre blocks, so this form keeps kSSBfHalo rows per side: every unit's
// taps must stay inside it (pad_u <= kSSBfHalo and 2 d_u - pad_u <= kSSBfHalo;
// host check).  The halo rows only ever feed margin columns.
#include "common.h"

#include <algorithm>

namespace rave {

typedef _Float16 ss_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 ss_h4 __attribute__((ext_vector_type(4)));
typedef float ss_f32x8 __attribute__((ext_vector_type(8)));
typedef float ss_f32x4 __attribute__((ext_vector_type(4)));
typedef float ss_f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 ss_b8 __attribute__((ext_vector_type(8)));
typedef __bf16 ss_b4 __attribute__((ext_vector_type(4)));

// fp32 -> three bf16 parts with v == hi + mid + lo exactly (unit_split.hip)
template <typename FV, typename BV>
__device__ __forceinline__ void ss_bf3_split(const FV& v, BV& hi, BV& mid, BV& lo) {
    bf3_split_pk(v, hi, mid, lo);
}

constexpr int kSSUnits = RAVE_STACK_UNITS;

#ifdef RAVE_STAMPS
// diagnostic build only: 8 clock stamps per workgroup (tools/stack_bench.py --stamps):
// 0 start, 1 window staged, 2/3/4 after unit 0/1/2 (running sums in registers),
// 5 after the stores, 7 wall clock at the start
__device__ unsigned long long* g_ss_stamps = nullptr;
#define SS_STAMP(k)                                                                            \
    do {                                                                                       \
        if (threadIdx.x == 0 && g_ss_stamps) {                                                 \
            g_ss_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime();                  \
            if ((k) == 0) g_ss_stamps[blockIdx.x * 8 + 7] = __builtin_amdgcn_s_memrealtime();  \
        }                                                                                      \
    } while (0)
#else
#define SS_STAMP(k) \
    do {            \
    } while (0)
#endif
constexpr unsigned kSSOOB = 0xFFFFFFF0u;
constexpr int kSSBfHalo = kStackBf3Halo;
#ifndef RAVE_SS_BF_R
#define RAVE_SS_BF_R 2
#endif                          // bf16x3: plane rows beyond the extended range, per side

struct SSArgs {
    const float* x; float* y;
    const float* w[kSSUnits];
    const float* rs1[kSSUnits]; const float* rs2[kSSUnits];
    const float* b1[kSSUnits]; const float* b2[kSSUnits];
    const float* a0[kSSUnits]; const float* a2[kSSUnits];
    int64_t x_sb, x_sc, y_sb, y_sc;
    int T, ntiles, act, x_bytes, y_bytes, w_bytes, has_bias;
    int d[kSSUnits], pad[kSSUnits];
    float slope;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ss_rsrc(const void* p, int bytes) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint64_t u = ((uint64_t)hi << 32) | lo;
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0,
                                             __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

template <bool SNAKE>
__device__ __forceinline__ float ss_act(float v, float slope, float alpha) {
    if constexpr (SNAKE) {
        const float r = 1.0f / (alpha + 1e-9f);
        return v + r * sin_squared(alpha * v);
    } else {
        return fmaxf(v, v * slope);         // leaky ReLU for slope <= 1 (host check); slope 1 == none
    }
}

// C channels (C/32 waves along rows, one 32-row block each); NB centre blocks
// of 32 columns + 2 margin blocks, CB blocks per wave; NP operand planes (2:
// split16 hi / lo, 3: bf16x3 hi / lo / mid).  WX > 0 (round 5): WX column waves
// with CB or CB - 1 blocks each (the first QF take CB), so that the SIMDs, each
// holding two waves of different column waves, carry equal block counts (C = 64,
// NB = 8, CB = 3, WX = 4: 3 + 2 blocks per SIMD pair of waves, 8 waves).
template <int C, int NB, int CB, int NP = 2, int WX = 0> struct SSGeo {
    static constexpr int WGM = C / 32, NBX = NB + 2, WGN = WX > 0 ? WX : NBX / CB, NW = WGM * WGN, NT = 64 * NW;
    static constexpr int QF = WX > 0 ? NBX - WX * (CB - 1) : WGN;   // column waves with CB blocks
    static constexpr int BN = 32 * NB;
    static constexpr int OFF = NP == 3 ? kSSBfHalo : 32;   // plane row of extended column 0
    static constexpr int XR = NBX * 32 + 2 * OFF;      // plane rows: extended range + OFF each side
    static constexpr int PH = C + 8;                   // halves per row (conflict-free b128 reads)
    static constexpr int PLANE = XR * PH;              // halves per plane
    static constexpr int S1 = 3 * C / 16, S2 = C / 16, ST = S1 + S2, CG = C / 16;
    // weight ring depth (K-steps; divides ST).  bf16x3: 2 (three fragments per
    // K-step; 10 waves leave 168 VGPRs per lane, and a 4-deep ring spilled)
    static constexpr int R = NP == 3 ? RAVE_SS_BF_R : 4;
    static constexpr int G8 = C / 8;
    static constexpr int XT = (XR * G8 + NT - 1) / NT; // window staging tasks per thread
    static constexpr int TAB = kSSUnits * 6 * C;       // per unit: rs1 b1 a2 rs2 b2 a0
    // + range-guard votes (16 B) and wave maxima (16 floats)
    static constexpr int VOTE = NP * PLANE * 2 + TAB * 4, VRED = VOTE + 16;
    static constexpr int LDS = VRED + 64;
    static_assert((WX > 0 ? (QF > 0 && QF <= WX) : NBX % CB == 0) && ST % R == 0 && NT <= 1024, "geometry");
};

// Range guard in two passes, as unit_split.hip: GUARD = false runs no guard
// code; a non-finite centre sum (an operand past the f16 range became inf in its
// hi half) makes the workgroup run the stack again with GUARD = true, whose
// window / seams / between-unit planes vote and re-stage scaled.  Returns false
// when the unguarded pass found one (the guarded pass rewrites its stores).
// BF (bf16x3): one pass, no guard code at all (the operands keep the fp32
// exponent range).
template <int C, int NB, int CB, bool SNAKE, bool GUARD, bool BF = false, int WX = 0>
__device__ __forceinline__ bool stack_split_body(const SSArgs& a) {
    constexpr int NPW = BF ? 3 : 2;                    // operand planes / weight fragments per K-step
    using G = SSGeo<C, NB, CB, NPW, WX>;
    constexpr bool GV = GUARD && !BF && RAVE_SPLIT_GUARD != 0;
    constexpr int NT = G::NT, PH = G::PH, XR = G::XR, G8 = G::G8, XT = G::XT, R = G::R;
    constexpr int S1 = G::S1, ST = G::ST, CG = G::CG, OFF = G::OFF;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    _Float16* ph = reinterpret_cast<_Float16*>(lds);
    _Float16* pl = ph + G::PLANE;
    _Float16* pm = pl + G::PLANE;                      // BF: the mid plane
    float* tab = reinterpret_cast<float*>(lds + NPW * G::PLANE * 2);
    unsigned char* vote = reinterpret_cast<unsigned char*>(lds + G::VOTE);
    float* vred = reinterpret_cast<float*>(lds + G::VRED);

    const int tid = threadIdx.x;
    SS_STAMP(0);
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % G::WGM, wn = wave / G::WGM;
    const int hh = lane >> 5, l32 = lane & 31;
#ifdef RAVE_STACK_XCD_MAP
    const int lg = __builtin_amdgcn_readfirstlane(xcd_major(blockIdx.x, gridDim.x));
#else
    const int lg = blockIdx.x;      // measured: the stack runs ~1 us slower XCD-major
#endif
    const int b = lg / a.ntiles;
    const int n0 = (lg - b * a.ntiles) * G::BN;
    const int ext0 = n0 - 32;                       // absolute column of extended column 0
    const int r0 = ext0 - OFF;                      // absolute column of plane row 0
    const float slope = a.act == RAVE_ACT_LEAKY ? a.slope : 1.0f;
    const auto xrs = ss_rsrc(a.x + (int64_t)b * a.x_sb, a.x_bytes);

    // ------------------------------------------------------------ per-unit row tables -> LDS
    // (every load in flight at once: a rolled loop waits out one round trip per pass)
    {
        constexpr int NTB = (kSSUnits * 6 * C + NT - 1) / NT;
        float tv[NTB];
#pragma unroll
        for (int r = 0; r < NTB; ++r) {
            // (segments of C, a multiple of 64: u and k are wave-uniform -- no masked loads)
            const int i = tid + r * NT;
            const int u = __builtin_amdgcn_readfirstlane(i / (6 * C)), iu = i - u * 6 * C;
            const int k = __builtin_amdgcn_readfirstlane(iu / C), m = iu - k * C;
            const int uu = min(u, kSSUnits - 1);
            const float* src = k == 0 ? a.rs1[uu] : k == 1 ? a.b1[uu] : k == 2 ? a.a2[uu]
                             : k == 3 ? a.rs2[uu] : k == 4 ? a.b2[uu] : a.a0[uu];
            const bool has = u < kSSUnits && ((k == 1 || k == 4) ? a.has_bias != 0 : (k == 2 || k == 5) ? SNAKE : true);
            tv[r] = has ? src[m] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < NTB; ++r)
            if (__builtin_amdgcn_readfirstlane(tid + r * NT) < kSSUnits * 6 * C) tab[tid + r * NT] = tv[r];
    }

    // ------------------------------------------------------------ weight ring (crosses units)
    ss_h8 ring[R][NPW];
    const unsigned abase = (unsigned)(wm * ST * NPW) * 1024u + (unsigned)lane * 16u;
    auto wrs_of = [&](int u) __attribute__((always_inline)) {
        const float* w = u == 0 ? a.w[0] : u == 1 ? a.w[1] : a.w[2];
        return ss_rsrc(w, u < kSSUnits ? a.w_bytes : 0);
    };
    // step s of the current unit; s >= ST: step s - ST of the next unit
    auto load_a = [&](int slot, __amdgpu_buffer_rsrc_t cur, __amdgpu_buffer_rsrc_t nxt, int s)
        __attribute__((always_inline)) {
        const bool here = s < ST;
        const int ss = here ? s : s - ST;
#pragma unroll
        for (int p = 0; p < NPW; ++p)
            ring[slot][p] = __builtin_bit_cast(ss_h8, __builtin_amdgcn_raw_buffer_load_b128(
                here ? cur : nxt, abase + (unsigned)((ss * NPW + p) * 1024), 0, 0));
    };
    {
        const auto w0 = wrs_of(0), w1 = wrs_of(1);
#pragma unroll
        for (int s = 0; s < R; ++s) load_a(s, w0, w1, s);
    }
    __syncthreads();                                   // tables visible

    // ------------------------------------------------------------ unit 0 input window
    // (xs: range-guard scale; returns max |act0(x) xs| of the thread's values)
    auto stage_window = [&](float xs) __attribute__((always_inline)) {
        float cmax = 0.f;
        float rx[XT][8];
#pragma unroll
        for (int i = 0; i < XT; ++i) {
            const int e = tid + i * NT;
            const int g = e / XR, w = e - g * XR;
            const int t = min(max(r0 + w, 0), a.T - 1);
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
            const int g = e / XR, w = e - g * XR;
            const bool ok = (e < XR * G8) && (r0 + w >= 0) && (r0 + w < a.T);
            ss_f32x8 v8;
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                const float al = SNAKE ? tab[5 * C + min(g * 8 + v, C - 1)] : 0.f;
                v8[v] = ok ? ss_act<SNAKE>(rx[i][v], slope, al) * xs : 0.f;
            }
            if constexpr (BF) {
                ss_b8 hi, mid, lo;
                ss_bf3_split(v8, hi, mid, lo);
                if (e < XR * G8) {
                    *reinterpret_cast<ss_b8*>(ph + w * PH + g * 8) = hi;
                    *reinterpret_cast<ss_b8*>(pl + w * PH + g * 8) = lo;
                    *reinterpret_cast<ss_b8*>(pm + w * PH + g * 8) = mid;
                }
                continue;
            }
            cmax = fmaxf(cmax, absmax8(v8));
            const ss_h8 hi = __builtin_convertvector(v8, ss_h8);
            const ss_h8 lo = __builtin_convertvector((v8 - __builtin_convertvector(hi, ss_f32x8)) * 2048.0f, ss_h8);
            if (e < XR * G8) {
                *reinterpret_cast<ss_h8*>(ph + w * PH + g * 8) = hi;
                *reinterpret_cast<ss_h8*>(pl + w * PH + g * 8) = lo;
            }
        }
        return cmax;
    };
    // running sum y (fp32): lane column col0 + 32j, rows mrow0 + 8(r>>2) + (r&3)
    // this wave's column blocks: nbw of them from extended block blk0 (uniform
    // geometry: CB from wn * CB)
    constexpr bool VAR = G::QF != G::WGN;
    const int nbw = VAR ? (wn < G::QF ? CB : CB - 1) : CB;
    const int blk0 = VAR ? (wn < G::QF ? wn * CB : G::QF * CB + (wn - G::QF) * (CB - 1)) : wn * CB;
    const int col0 = blk0 * 32 + l32;                  // extended column of this lane
    const int mrow0 = 32 * wm + 4 * hh;
    float yv[CB][16];
    auto load_y = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            if (VAR && j >= nbw) break;
            const int t = ext0 + col0 + 32 * j;
            const bool ok = t >= 0 && t < a.T;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mrow0 + 8 * (r >> 2) + (r & 3);
                yv[j][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                    xrs, ok ? (unsigned)(m * a.x_sc + t) * 4u : kSSOOB, 0, 0));
            }
        }
    };
    // (bf16x3: after the window is staged -- its registers and the window's do
    // not fit together at 10 waves; y is not read before unit 0's phase 2)
    if constexpr (!BF) load_y();
    // unit 0's act0(x) window, under the range guard: one pass in the common
    // case, a second one as act0(x) * 2^-sh0 when a wave saw |act0(x)| >= 2^15
    int sh0 = 0;                                       // range-guard shift of the current unit's act0(y) planes
    {
        const float cmax = stage_window(1.0f);
        if constexpr (BF) load_y();
        if constexpr (GV) vote_cast(vote, wave, cmax);
        __syncthreads();
        if (GV && __builtin_expect(vote_any<G::NW>(vote), 0)) {      // rare: a rolled re-staging loop
            sh0 = __builtin_amdgcn_readfirstlane(split_shift(block_max<G::NW>(cmax, vred)));
            const float xs = ldexpf(1.0f, -sh0);
#pragma nounroll
            for (int e = tid; e < XR * G8; e += NT) {
                const int g = e / XR, w = e - g * XR;
                const bool ok = (r0 + w >= 0) && (r0 + w < a.T);
                const int t = min(max(r0 + w, 0), a.T - 1);
                ss_f32x8 v8;
#pragma unroll
                for (int v = 0; v < 8; ++v) {
                    const int c = min(g * 8 + v, C - 1);
                    const float xv = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                        xrs, (unsigned)(c * a.x_sc + t) * 4u, 0, 0));
                    v8[v] = ok ? ss_act<SNAKE>(xv, slope, SNAKE ? tab[5 * C + c] : 0.f) * xs : 0.f;
                }
                const ss_h8 hi = __builtin_convertvector(v8, ss_h8);
                const ss_h8 lo = __builtin_convertvector((v8 - __builtin_convertvector(hi, ss_f32x8)) * 2048.0f, ss_h8);
                *reinterpret_cast<ss_h8*>(ph + w * PH + g * 8) = hi;
                *reinterpret_cast<ss_h8*>(pl + w * PH + g * 8) = lo;
            }
            __syncthreads();
        }
    }

    SS_STAMP(1);
    struct BFr {
        ss_h8 h[CB], l[CB], m[BF ? CB : 1];
    };
    auto read_b = [&](int row, int ch, BFr& f) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            if (VAR && j >= nbw) break;
            const int off = (row + j * 32) * PH + ch + 8 * hh;
            f.h[j] = *reinterpret_cast<const ss_h8*>(ph + off);
            f.l[j] = *reinterpret_cast<const ss_h8*>(pl + off);
            if constexpr (BF) f.m[j] = *reinterpret_cast<const ss_h8*>(pm + off);
        }
    };
    ss_f32x16 acc[CB];
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    };
    zero_acc();
    // act(v) * xs -> (hi, lo) planes at extended column col0 + 32j (zero outside
    // [0, T) if mask); returns max |act(v) xs| of the thread's values
    auto write_planes = [&](const float (*v)[16], const float* al_tab, bool mask, float xs)
        __attribute__((always_inline)) {
        float cmax = 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int m = mrow0 + 8 * g;
            ss_f32x4 al = {0.f, 0.f, 0.f, 0.f};
            if constexpr (SNAKE) al = *reinterpret_cast<const ss_f32x4*>(al_tab + m);
#pragma unroll
            for (int j = 0; j < CB; ++j) {
                if (VAR && j >= nbw) break;
                const int t = ext0 + col0 + 32 * j;
                const bool ok = !mask || (t >= 0 && t < a.T);
                ss_f32x4 w4;
#pragma unroll
                for (int e = 0; e < 4; ++e) w4[e] = ok ? ss_act<SNAKE>(v[j][4 * g + e], slope, al[e]) * xs : 0.f;
                if constexpr (BF) {
                    ss_b4 hi, mid, lo;
                    ss_bf3_split(w4, hi, mid, lo);
                    *reinterpret_cast<ss_b4*>(ph + (OFF + col0 + 32 * j) * PH + m) = hi;
                    *reinterpret_cast<ss_b4*>(pl + (OFF + col0 + 32 * j) * PH + m) = lo;
                    *reinterpret_cast<ss_b4*>(pm + (OFF + col0 + 32 * j) * PH + m) = mid;
                    continue;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) cmax = fmaxf(cmax, fabsf(w4[e]));
                const ss_h4 hv = __builtin_convertvector(w4, ss_h4);
                const ss_h4 lv = __builtin_convertvector((w4 - __builtin_convertvector(hv, ss_f32x4)) * 2048.0f, ss_h4);
                *reinterpret_cast<ss_h4*>(ph + (OFF + col0 + 32 * j) * PH + m) = hv;
                *reinterpret_cast<ss_h4*>(pl + (OFF + col0 + 32 * j) * PH + m) = lv;
            }
        }
        return cmax;
    };
    // optimistic planes, then the range guard's vote; on overflow the planes are
    // rewritten as act(v) 2^-s and the shift s is returned (else 0)
    auto guarded_planes = [&](const float (*v)[16], const float* al_tab, bool mask)
        __attribute__((always_inline)) {
        const float cmax = write_planes(v, al_tab, mask, 1.0f);
        if constexpr (GV) vote_cast(vote, wave, cmax);
        __syncthreads();
        int sh = 0;
        if (GV && __builtin_expect(vote_any<G::NW>(vote), 0)) {
            sh = __builtin_amdgcn_readfirstlane(split_shift(block_max<G::NW>(cmax, vred)));
            (void)write_planes(v, al_tab, mask, ldexpf(1.0f, -sh));
            __syncthreads();
        }
        return sh;
    };

#pragma unroll 1
    for (int u = 0; u < kSSUnits; ++u) {
        const auto wcur = wrs_of(u), wnxt = wrs_of(u + 1);
        const float* tu = tab + u * 6 * C;
        const int du = u == 0 ? a.d[0] : u == 1 ? a.d[1] : a.d[2];
        const int pu = u == 0 ? a.pad[0] : u == 1 ? a.pad[1] : a.pad[2];
        auto step = [&](int s, const BFr& f) __attribute__((always_inline)) {
            const ss_h8 ah = ring[s % R][0], al = ring[s % R][1];
            if constexpr (BF) {
                const ss_b8 wh = __builtin_bit_cast(ss_b8, ah), wl = __builtin_bit_cast(ss_b8, al),
                            wmd = __builtin_bit_cast(ss_b8, ring[s % R][NPW - 1]);
                load_a(s % R, wcur, wnxt, s + R);        // refill (runs on into the next unit)
                // smallest products first: lo*hi, hi*lo, mid*mid, mid*hi, hi*mid, hi*hi
#pragma unroll
                for (int j = 0; j < CB; ++j) {
                    if (VAR && j >= nbw) break;
                    const ss_b8 xh = __builtin_bit_cast(ss_b8, f.h[j]), xl = __builtin_bit_cast(ss_b8, f.l[j]),
                                xm = __builtin_bit_cast(ss_b8, f.m[j]);
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wmd, xm, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wmd, xh, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xm, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh, acc[j], 0, 0, 0);
                }
                return;
            }
            const ss_h8 a2 = ah * (_Float16)2048.0f;
            load_a(s % R, wcur, wnxt, s + R);            // refill (runs on into the next unit)
#pragma unroll
            for (int j = 0; j < CB; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2, f.h[j], acc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < CB; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, f.l[j], acc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < CB; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, f.h[j], acc[j], 0, 0, 0);
        };
        // phase 1: h = W1 . window (taps at row shifts q*d - pad)
        {
            const int rowb = OFF - pu + col0;
            BFr f[2];
            read_b(rowb, 8 * 0, f[0]);
#pragma unroll
            for (int s = 0; s < S1; ++s) {
                if (s + 1 < S1) {
                    const int tap = (s + 1) / CG;
                    read_b(rowb + tap * du, ((s + 1) - tap * CG) * 16, f[(s + 1) & 1]);
                }
                __builtin_amdgcn_sched_barrier(0);
                step(s, f[s & 1]);
            }
        }
        __syncthreads();                               // window dead
        // seam: h = act2(h * rs1 * 2^sh0 + b1) -> planes (2^sh0: the range guard of act0(y))
        int sh2 = 0;
        {
            float hv[CB][16];
            const float f0 = ldexpf(1.0f, sh0);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int m = mrow0 + 8 * g;
                const ss_f32x4 rs = *reinterpret_cast<const ss_f32x4*>(tu + m) * f0;
                const ss_f32x4 bb = *reinterpret_cast<const ss_f32x4*>(tu + C + m);
#pragma unroll
                for (int j = 0; j < CB; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) hv[j][4 * g + e] = acc[j][4 * g + e] * rs[e] + bb[e];
            }
            sh2 = guarded_planes(hv, tu + 2 * C, false);
            zero_acc();
        }
        // phase 2: y += W2 . h
        {
            BFr f[2];
            read_b(OFF + col0, 0, f[0]);
#pragma unroll
            for (int s = S1; s < ST; ++s) {
                if (s + 1 < ST) read_b(OFF + col0, (s + 1 - S1) * 16, f[(s + 1 - S1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
                step(s, f[(s - S1) & 1]);
            }
        }
        const float f2 = ldexpf(1.0f, sh2);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int m = mrow0 + 8 * g;
            const ss_f32x4 rs = *reinterpret_cast<const ss_f32x4*>(tu + 3 * C + m) * f2;
            const ss_f32x4 bb = *reinterpret_cast<const ss_f32x4*>(tu + 4 * C + m);
#pragma unroll
            for (int j = 0; j < CB; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    yv[j][4 * g + e] = acc[j][4 * g + e] * rs[e] + bb[e] + yv[j][4 * g + e];
        }
        zero_acc();
        SS_STAMP(2 + u);
        if (u + 1 < kSSUnits) {
            __syncthreads();                           // h dead
            sh0 = guarded_planes(yv, tu + 6 * C + 5 * C, true);    // next unit's act0(y)
        }
    }

    // unguarded pass: a non-finite centre sum -> run again guarded (flag here,
    // workgroup vote after the stores, which the guarded pass rewrites)
    constexpr bool CHECK = !GUARD && !BF && RAVE_SPLIT_GUARD != 0;
    bool bad = false;
    if constexpr (CHECK) {
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            const int blk = blk0 + j;
            const bool ok = blk >= 1 && blk <= NB && ext0 + col0 + 32 * j < a.T;
#pragma unroll
            for (int r = 0; r < 16; ++r) bad |= ok && !__builtin_isfinite(yv[j][r]);
        }
    }
    // ------------------------------------------------------------ centre blocks -> y
    const auto yrs = ss_rsrc(a.y + (int64_t)b * a.y_sb, a.y_bytes);
#pragma unroll
    for (int j = 0; j < CB; ++j) {
        if (VAR && j >= nbw) break;
        const int blk = blk0 + j;                      // extended block: 1..NB are the centre
        const int t = ext0 + col0 + 32 * j;
        const bool ok = blk >= 1 && blk <= NB && t < a.T;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = mrow0 + 8 * (r >> 2) + (r & 3);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, yv[j][r]), yrs,
                                                  ok ? (unsigned)(m * a.y_sc + t) * 4u : kSSOOB, 0, RAVE_YAUX);
        }
    }
    SS_STAMP(5);
    if constexpr (CHECK) {
        vote_cast_any(vote, wave, bad);
        __syncthreads();
        if (__builtin_expect(vote_any<G::NW>(vote), 0)) {
            __syncthreads();                           // every wave read the vote
            return false;
        }
    }
    return true;
}

template <int C, int NB, int CB, bool SNAKE>
__global__ __launch_bounds__(64 * (C / 32) * ((NB + 2) / CB)) void stack_split_kernel(SSArgs a) {
    if (!stack_split_body<C, NB, CB, SNAKE, RAVE_SPLIT_GUARD == 0>(a)) (void)stack_split_body<C, NB, CB, SNAKE, true>(a);
}
template <int C, int NB, int CB, bool SNAKE, int WX>
__global__ __launch_bounds__((SSGeo<C, NB, CB, 3, WX>::NT)) void stack_bf3_kernel(SSArgs a) {
    (void)stack_split_body<C, NB, CB, SNAKE, false, true, WX>(a);
}

template <int C, int NB, int CB, bool BF = false, int WX = 0>
static int ss_launch(const SSArgs& k0, int B, bool snake, hipStream_t st) {
    using G = SSGeo<C, NB, CB, BF ? 3 : 2, WX>;
    static_assert(BF || WX == 0, "split16 stacks: uniform geometry");
    SSArgs k = k0;
    k.ntiles = ceil_div(k.T, G::BN);
    void (*kern)(SSArgs) = nullptr;
    if constexpr (BF) kern = snake ? stack_bf3_kernel<C, NB, CB, true, WX> : stack_bf3_kernel<C, NB, CB, false, WX>;
    else kern = snake ? stack_split_kernel<C, NB, CB, true> : stack_split_kernel<C, NB, CB, false>;
    static bool attr[2] = {false, false};
    if (G::LDS > 65536 && !attr[snake]) {
        RAVE_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr[snake] = true;
    }
    static_assert(G::LDS <= 160 * 1024, "LDS budget");
    launch(kern, dim3(k.ntiles * B), dim3(G::NT), (uint32_t)G::LDS, st, k);
    return launch_status(BF ? "stack_bf3_kernel" : "stack_split_kernel");
}

}  // namespace rave

using namespace rave;

extern "C" int rave_stack_supported(int channels) { return channels == 64 || channels == 128; }

#ifdef RAVE_STAMPS
extern "C" int rave_diag_stack_stamps(void* p) {
    RAVE_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_ss_stamps), &p, sizeof(p)));
    return RAVE_OK;
}
#endif

extern "C" int rave_residual_stack(const rave_stack_args* p, void* stream) {
    RAVE_CHECK_ARG(p, "residual_stack: null args");
    const int C = p->channels;
    if (!rave_stack_supported(C)) {
        set_error("residual_stack: C in {64, 128}");
        return RAVE_ERR_UNSUPPORTED;
    }
    RAVE_CHECK_ARG(p->x && p->y && p->batch > 0 && p->t_len > 0, "residual_stack: empty shape or null tensor");
    RAVE_CHECK_ARG(p->act != RAVE_ACT_LEAKY || p->leaky_slope <= 1.0f, "residual_stack: leaky slope above 1");
    RAVE_CHECK_ARG(p->act == RAVE_ACT_LEAKY || p->act == RAVE_ACT_SNAKE || p->act == RAVE_ACT_NONE,
                   "residual_stack: unknown activation");
    const bool snake = p->act == RAVE_ACT_SNAKE;
    const bool has_bias = p->bias1[0] != nullptr;
    RAVE_CHECK_ARG(p->precision == 0 || p->precision == RAVE_PREC_SPLIT16 || p->precision == RAVE_PREC_BF16X3,
                   "residual_stack: precision must be RAVE_PREC_SPLIT16 or RAVE_PREC_BF16X3");
    const bool bf = p->precision == RAVE_PREC_BF16X3;
    int reach_l = 0, reach_r = 0;
    for (int u = 0; u < kSSUnits; ++u) {
        const int d = p->dilation[u], pl = p->pad_left[u];
        RAVE_CHECK_ARG(p->weight[u], "residual_stack: null weight");
        RAVE_CHECK_ARG(d >= 1 && d <= 16 && pl >= 0 && pl <= 2 * d, "residual_stack: dilation / padding out of range");
        RAVE_CHECK_ARG((p->bias1[u] != nullptr) == has_bias && (p->bias2[u] != nullptr) == has_bias,
                       "residual_stack: biases on every unit or on none");
        RAVE_CHECK_ARG(!snake || (p->alpha0[u] && p->alpha2[u]), "residual_stack: snake needs alphas");
        if (u > 0) {
            reach_l += pl;
            reach_r += 2 * d - pl;
        }
        if (bf && (pl > kSSBfHalo || 2 * d - pl > kSSBfHalo)) {
            set_error("residual_stack(bf16x3): a unit's taps reach past the 24-row plane halo (run the units separately)");
            return RAVE_ERR_UNSUPPORTED;
        }
    }
    if (reach_l > kStackMargin || reach_r > kStackMargin) {
        set_error("residual_stack: units 2..3 reach past the 32-column margin (run the units separately)");
        return RAVE_ERR_UNSUPPORTED;
    }
    const int64_t xb = ((int64_t)(C - 1) * p->x_sc + p->t_len) * 4;
    const int64_t yb = ((int64_t)(C - 1) * p->y_sc + p->t_len) * 4;
    RAVE_CHECK_ARG(xb < (1ll << 31) && yb < (1ll << 31), "residual_stack: tensors beyond 2 GiB per item");
    SSArgs k{};
    k.x = p->x; k.y = p->y;
    // rave_unit_split_pack_weight / rave_unit_bf3_pack_weight (fragments, then rs1, rs2)
    const int64_t frag = (int64_t)(C / 32) * (4 * C / 16) * (bf ? 3 : 2) * 256;
    for (int u = 0; u < kSSUnits; ++u) {
        k.w[u] = p->weight[u];
        k.rs1[u] = p->weight[u] + frag;
        k.rs2[u] = p->weight[u] + frag + C;
        k.b1[u] = has_bias ? p->bias1[u] : p->weight[u];
        k.b2[u] = has_bias ? p->bias2[u] : p->weight[u];
        k.a0[u] = snake ? p->alpha0[u] : p->weight[u];
        k.a2[u] = snake ? p->alpha2[u] : p->weight[u];
        k.d[u] = p->dilation[u];
        k.pad[u] = p->pad_left[u];
    }
    k.x_sb = p->x_sb; k.x_sc = p->x_sc; k.y_sb = p->y_sb; k.y_sc = p->y_sc;
    k.T = p->t_len; k.act = p->act; k.slope = p->leaky_slope;
    k.x_bytes = (int)xb; k.y_bytes = (int)yb; k.w_bytes = (int)(frag * 4);
    k.has_bias = has_bias;
    hipStream_t st = as_stream(stream);
    // geometry measured with tools/stack_bench.py (v2 sizes, B = 16): C = 64 with
    // 8 centre blocks, 5 blocks per wave (2 column waves share each weight row
    // block): 40.0 us against 46.5 us for the three unit launches; C = 128 (2
    // centre blocks, 2 per wave) 43.6 against 43.1 -- the autotuner keeps the units
    // Round 2 (same-box A/Bs in the bench step, profiles/r02_xcd/ab_stack_geometry.txt):
    // C = 64 with two blocks per wave (10 waves: 5 column waves per 32-row block)
    // 38.2 -> 35.5 us against five blocks per wave (4 waves)
#ifndef RAVE_S64_NB
#define RAVE_S64_NB 8
#define RAVE_S64_CB 2
#endif
#ifndef RAVE_S128_NB
#define RAVE_S128_NB 2
#define RAVE_S128_CB 2
#endif
    // bf16x3 (three planes, 24-row halo): C = 64 keeps 8 centre blocks (146 KB of
    // LDS); C = 128 fits 2 (152 KB).  C = 64 (round 5): 8 waves, column waves of
    // 3, 3, 2, 2 blocks (RAVE_B64S_WX = 4; 0 = 10 waves of 2 blocks, A/B)
#ifndef RAVE_B64S_NB
#define RAVE_B64S_NB 8
#endif
#ifndef RAVE_B64S_WX
#define RAVE_B64S_WX 4
#endif
#ifndef RAVE_B64S_CB
#define RAVE_B64S_CB (RAVE_B64S_WX > 0 ? 3 : 2)
#endif
#ifndef RAVE_B128S_NB
#define RAVE_B128S_NB 2
#define RAVE_B128S_CB 2
#endif
    if (bf) {
        if (C == 64) return ss_launch<64, RAVE_B64S_NB, RAVE_B64S_CB, true, RAVE_B64S_WX>(k, p->batch, snake, st);
        return ss_launch<128, RAVE_B128S_NB, RAVE_B128S_CB, true>(k, p->batch, snake, st);
    }
    if (C == 64) return ss_launch<64, RAVE_S64_NB, RAVE_S64_CB>(k, p->batch, snake, st);
    return ss_launch<128, RAVE_S128_NB, RAVE_S128_CB>(k, p->batch, snake, st);
}
