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
#include "common.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace rave {

typedef _Float16 us_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 us_h4 __attribute__((ext_vector_type(4)));
typedef float us_f32x8 __attribute__((ext_vector_type(8)));
typedef float us_f32x4 __attribute__((ext_vector_type(4)));
typedef float us_f32x16 __attribute__((ext_vector_type(16)));

constexpr int kUSMaxDil = 16;
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
constexpr unsigned kUSOOB = 0xFFFFFFF0u;

struct USArgs {
    const float* x; float* y; const float* w; const float* rs1; const float* rs2;
    const float* b1; const float* b2; const float* a0; const float* a2;
    int64_t x_sb, x_sc, y_sb, y_sc;
    int T, d, pad_l, ntiles, XW;
    int x_bytes, y_bytes, w_bytes, bias_bytes;
    int act;
    float slope;
    unsigned xw_magic;
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
        return v > 0.f ? v : v * slope;     // slope 1 == no activation
    }
}

// C channels; WGN waves along time (each 64 columns); C/(32 MI) waves along
// rows (each MI 32-row blocks).
template <int C, int WGN, int MI, int KG = 1, int CB = 2> struct USGeo {
    static constexpr int WGM = C / (32 * MI), NWT = WGM * WGN, NW = NWT * KG, NT = 64 * NW;
    static constexpr int BN = 32 * CB * WGN;           // CB 32-column blocks per wave
    static constexpr int S1 = 3 * C / 16, S2 = C / 16, ST = S1 + S2;   // K-steps
    static constexpr int PH = C + 8;                  // halves per LDS row (conflict-free b128)
    static constexpr int XW_MAX = BN + 2 * kUSMaxDil;
    static constexpr int XPLANE = XW_MAX * PH * 2;    // bytes per f16 plane
    static constexpr int HPLANE = BN * PH * 2;
    static constexpr int PLANES = 2 * (XPLANE > HPLANE ? XPLANE : HPLANE);
    // + per-row table: rs1 b1 a2 | rs2 b2 a0, + range-guard votes (16 B) and wave maxima (16 floats)
    static constexpr int TAB = PLANES, VOTE = PLANES + 6 * C * 4, VRED = VOTE + 16;
    static constexpr int LDS = VRED + 64;
    static constexpr int G8 = C / 8;                  // 8-channel groups per window row
    static constexpr int XT = (XW_MAX * G8 + NT - 1) / NT;
    static constexpr int R = 3;                       // weight ring depth (K-steps)
    // K-groups: two waves per output tile take alternate K-steps (both phases)
    static constexpr int RED = NWT * MI * CB * 16 * 64 * 4;  // partial-sum hand-off (bytes)
    static_assert(C % 64 == 0 && (MI == 1 || MI == 2) && NW <= 16, "geometry");
    static_assert(KG == 1 || (KG == 2 && S1 % 2 == 0 && S2 % 2 == 0 && RED <= PLANES), "K-groups");
};

template <int C, int WGN, int MI, int KG, int CB, bool SNAKE>
__global__ __launch_bounds__(64 * (C / (32 * MI)) * WGN * KG) void unit_split_kernel(USArgs a) {
    using G = USGeo<C, WGN, MI, KG, CB>;
    constexpr int NT = G::NT, PH = G::PH, G8 = G::G8, XT = G::XT, R = G::R;
    constexpr int S1 = G::S1, ST = G::ST, CG = C / 16;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    _Float16* ph = reinterpret_cast<_Float16*>(lds);
    _Float16* pl = reinterpret_cast<_Float16*>(lds + G::PLANES / 2);
    float* tab = reinterpret_cast<float*>(lds + G::TAB);      // [6][C]
    unsigned char* vote = reinterpret_cast<unsigned char*>(lds + G::VOTE);
    float* vred = reinterpret_cast<float*>(lds + G::VRED);

    US_STAMP(0);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kg = wave / G::NWT;                    // K-group
    const int twave = wave - kg * G::NWT;
    const int wm = twave % G::WGM, wn = twave / G::WGM;
    const int hh = lane >> 5, l32 = lane & 31;
    const int lg = __builtin_amdgcn_readfirstlane(xcd_major(blockIdx.x, gridDim.x));
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
    us_h8 ring[R][MI][2];
    const unsigned abase = (unsigned)((MI * wm) * ST * 2) * 1024u + (unsigned)lane * 16u;
    auto load_a = [&](int slot, int s) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int p = 0; p < 2; ++p)
                ring[slot][i][p] = __builtin_bit_cast(us_h8, __builtin_amdgcn_raw_buffer_load_b128(
                    wrs, s < ST ? abase + (unsigned)(((i * ST + s) * 2 + p) * 1024) : kUSOOB, 0, 0));
    };
#pragma unroll
    for (int t = 0; t < R; ++t) load_a(t, t * KG + kg);

    // ------------------------------------------------------------ per-row table -> LDS
    for (int i = tid; i < 6 * C; i += NT) {
        const int k = i / C, m = i - k * C;
        const float* src = k == 0 ? a.rs1 : k == 1 ? a.b1 : k == 2 ? a.a2 : k == 3 ? a.rs2 : k == 4 ? a.b2 : a.a0;
        const bool has = (k == 1 || k == 4) ? a.bias_bytes > 0 : (k == 2 || k == 5) ? SNAKE : true;
        tab[i] = has ? src[m] : 0.f;
    }

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
            const int t = min(max(t0 + w, 0), a.T - 1);
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
            const bool ok = (e < ntask) && (t0 + w >= 0) && (t0 + w < a.T);
            us_f32x8 v8;
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                const float al = SNAKE ? a.a0[min(g * 8 + v, C - 1)] : 0.f;   // L1-hot
                v8[v] = ok ? us_act<SNAKE>(rx[i][v], slope, al) * xs : 0.f;
            }
            cmax = fmaxf(cmax, absmax8(v8));
            const us_h8 hi = __builtin_convertvector(v8, us_h8);
            const us_h8 lo = __builtin_convertvector((v8 - __builtin_convertvector(hi, us_f32x8)) * 2048.0f, us_h8);
            if (e < ntask) {
                *reinterpret_cast<us_h8*>(ph + w * PH + g * 8) = hi;
                *reinterpret_cast<us_h8*>(pl + w * PH + g * 8) = lo;
            }
        }
        return cmax;
    };
    // range guard: when a wave saw |act0(x)| >= 2^15 the window is staged again
    // as act0(x) * 2^-sh0 by a rolled loop (small code, few registers: rare)
    {
        const float cmax = stage_window(1.0f);
        vote_cast(vote, wave, cmax);
        __syncthreads();
        if (__builtin_expect(vote_any<G::NW>(vote), 0)) {
            sh0 = __builtin_amdgcn_readfirstlane(split_shift(block_max<G::NW>(cmax, vred)));
            const float xs = ldexpf(1.0f, -sh0);
#pragma nounroll
            for (int e = tid; e < ntask; e += NT) {
                const int g = (int)(((unsigned)e * a.xw_magic) >> 24);
                const int w = e - g * XW;
                const bool ok = (t0 + w >= 0) && (t0 + w < a.T);
                const int t = min(max(t0 + w, 0), a.T - 1);
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
    US_STAMP(1);

    // ------------------------------------------------------------ K loop (both phases)
    us_f32x16 acc[MI][CB];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // B fragments: column wn*64 + j*32 + l32, 8 channels at 8*hh
    const int col0 = wn * 32 * CB + l32;
    struct BF {
        us_h8 h[CB], l[CB];
    };
    auto read_b = [&](int s, BF& f) __attribute__((always_inline)) {
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
            f.h[j] = *reinterpret_cast<const us_h8*>(ph + off);
            f.l[j] = *reinterpret_cast<const us_h8*>(pl + off);
        }
    };
    auto step = [&](int t, int s, const BF& f) __attribute__((always_inline)) {
        us_h8 ah[MI], al[MI], a2[MI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            ah[i] = ring[t % R][i][0];
            al[i] = ring[t % R][i][1];
            a2[i] = ah[i] * (_Float16)2048.0f;
        }
        load_a(t % R, s + R * KG);                   // refill the slot (runs on into W2)
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
    const int mrow0 = 32 * MI * wm + 4 * hh;
    // own K-steps [t0, t1) of this wave's group: global step t*KG + GG
    auto kloop = [&](auto gtag, auto t0tag, auto t1tag) __attribute__((always_inline)) {
        constexpr int GG = decltype(gtag)::value;
        constexpr int T0 = decltype(t0tag)::value, T1 = decltype(t1tag)::value;
        BF f[2];
        read_b(T0 * KG + GG, f[0]);
#pragma unroll
        for (int t = T0; t < T1; ++t) {
            if (t + 1 < T1) read_b((t + 1) * KG + GG, f[(t + 1 - T0) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            step(t, t * KG + GG, f[(t - T0) & 1]);
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
    combine();
    __syncthreads();                                 // window (and hand-off area) dead
    US_STAMP(2);

    // ------------------------------------------------------------ seam: h = act2(h*rs1 + b1) -> planes
    // (phase 1 ran on act0(x) 2^-sh0: its scale 2^sh0 rides on rs1; xs = the
    // range guard's scale of h; returns max |h xs| of the thread's values)
    const float f0 = ldexpf(1.0f, sh0);
    auto seam = [&](float xs) __attribute__((always_inline)) {
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
    {                                            // range guard of h (rare path: h * 2^-sh2)
        const float cmax = seam(1.0f);
        vote_cast(vote, wave, cmax);
        __syncthreads();
        if (__builtin_expect(vote_any<G::NW>(vote), 0)) {
            sh2 = __builtin_amdgcn_readfirstlane(split_shift(block_max<G::NW>(cmax, vred)));
            (void)seam(ldexpf(1.0f, -sh2));
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    US_STAMP(3);

    if (KG == 1 || kg == 0) kloop(IC<0>{}, IC<S1 / KG>{}, IC<ST / KG>{});
    else kloop(IC<1>{}, IC<S1 / KG>{}, IC<ST / KG>{});
    combine();
    if (KG == 2 && kg == 1) return;                  // (no barrier follows)

    US_STAMP(4);
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
                        xrs, nok ? (unsigned)(m * a.x_sc + n) * 4u : kUSOOB, 0, 0));
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
                            __builtin_bit_cast(unsigned, acc[i][j][4 * g + e] * rs[e] + bb[e] + res[i][j][4 * g + e]),
                            yrs, nok ? (unsigned)((m + e) * a.y_sc + n) * 4u : kUSOOB, 0, RAVE_YAUX);
                }
            }
    }
    US_STAMP(5);
}

template <int C, int WGN, int MI, int KG, int CB>
static int us_launch(USArgs k, int B, bool snake, hipStream_t st) {
    using G = USGeo<C, WGN, MI, KG, CB>;
    if (k.XW > G::XW_MAX) {
        set_error("residual_unit(split16): dilation too large");
        return RAVE_ERR_UNSUPPORTED;
    }
    k.ntiles = ceil_div(k.T, G::BN);
    auto kern = snake ? unit_split_kernel<C, WGN, MI, KG, CB, true> : unit_split_kernel<C, WGN, MI, KG, CB, false>;
    static bool attr[2] = {false, false};
    if (G::LDS > 65536 && !attr[snake]) {
        RAVE_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr[snake] = true;
    }
    launch(kern, dim3(k.ntiles * B), dim3(G::NT), (uint32_t)G::LDS, st, k);
    return launch_status("unit_split_kernel");
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

extern "C" int rave_unit_split_pack_weight(const float* w1, const float* w2, int C, float* packed) {
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
        e1[m] = us_row_exponent(a1);
        e2[m] = us_row_exponent(a2);
    }
    _Float16* out = reinterpret_cast<_Float16*>(packed);
    for (int mb = 0; mb < C / 32; ++mb)
        for (int s = 0; s < ST; ++s) {
            _Float16* hi = out + ((int64_t)(mb * ST + s) * 2) * 512;
            _Float16* lo = hi + 512;
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
                    const _Float16 vh = (_Float16)v;
                    hi[l * 8 + e] = vh;
                    lo[l * 8 + e] = (_Float16)((v - (float)vh) * 2048.0f);
                }
        }
    float* rs = packed + (int64_t)(C / 32) * ST * 2 * 256;
    for (int m = 0; m < C; ++m) {
        rs[m] = (float)std::ldexp(1.0, -(e1[m] + 11));
        rs[C + m] = (float)std::ldexp(1.0, -(e2[m] + 11));
    }
    return RAVE_OK;
}

#ifdef RAVE_STAMPS
extern "C" int rave_diag_unit_stamps(void* p) {
    RAVE_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_us_stamps), &p, sizeof(p)));
    return RAVE_OK;
}
#endif

namespace rave {
int residual_unit_split(const rave_unit_args& a, void* stream) {
    const int C = a.channels;
    if (!us_supported(C)) {
        set_error("residual_unit(split16): fused unit supports C in {64, 128, 256, 512}");
        return RAVE_ERR_UNSUPPORTED;
    }
    USArgs k{};
    k.x = a.x; k.y = a.y; k.w = a.weight;
    const int64_t frag = (int64_t)(C / 32) * (4 * C / 16) * 2 * 256;
    k.rs1 = a.weight + frag; k.rs2 = a.weight + frag + C;
    k.b1 = a.bias1; k.b2 = a.bias2; k.a0 = a.alpha0; k.a2 = a.alpha2;
    k.x_sb = a.x_sb; k.x_sc = a.x_sc; k.y_sb = a.y_sb; k.y_sc = a.y_sc;
    k.T = a.t_len; k.d = a.dilation; k.pad_l = a.pad_left;
    k.act = a.act; k.slope = a.leaky_slope;
    const int64_t xb = ((int64_t)(C - 1) * a.x_sc + a.t_len) * 4;
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
    auto go = [&](auto cc, auto wgn, auto mi, auto kgt, auto cb) {
        constexpr int CC = decltype(cc)::value, WGN = decltype(wgn)::value, MI = decltype(mi)::value,
                      KG = decltype(kgt)::value, CB = decltype(cb)::value;
        k.XW = USGeo<CC, WGN, MI, KG, CB>::BN + 2 * a.dilation;
        k.xw_magic = (unsigned)(((1u << 24) + k.XW - 1) / k.XW);
        return us_launch<CC, WGN, MI, KG, CB>(k, a.batch, snake, st);
    };
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
    if (C == 64) return go(IC<64>{}, IC<RAVE_U64_WGN>{}, IC<1>{}, IC<1>{}, IC<RAVE_U64_CB>{});
#ifndef RAVE_U128_KG
#define RAVE_U128_KG 1
#endif
#ifndef RAVE_U256_KG
#define RAVE_U256_KG 1
#endif
    if (C == 128) return go(IC<128>{}, IC<RAVE_U128_WGN>{}, IC<1>{}, IC<RAVE_U128_KG>{}, IC<1>{});
    if (C == 256) return go(IC<256>{}, IC<1>{}, IC<1>{}, IC<RAVE_U256_KG>{}, IC<1>{});
    return go(IC<512>{}, IC<1>{}, IC<1>{}, IC<1>{}, IC<1>{});
}
}  // namespace rave
