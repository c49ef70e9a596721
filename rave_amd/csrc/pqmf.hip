// PQMF analysis / synthesis filterbank kernels (gfx950).
//
// analysis  = CachedPQMF.forward (rave/pqmf.py:269-273): conv1d(1 -> n_band,
//             k = 513, stride n_band, get_padding(513)) + reverse_half (:13-17);
//             only the first n_out_bands are produced (RAVE.encode feeds
//             x[:, :6] to the encoder, rave/model.py:613).
// synthesis = CachedPQMF.inverse (rave/pqmf.py:275-284): reverse_half ->
//             conv1d(n -> n, k = 33) * n -> flip(channels) -> interleave, with
//             GeneratorV2's `x * sigmoid(amp) (+ noise) -> tanh` epilogue
//             (rave/blocks.py:699-707) fused into the input staging (mode 1).
//
// Both are direct FIR kernels: one HBM pass over the audio/frames, the window
// staged in LDS in polyphase order (stride-n_band reads become consecutive),
// the filter taps read through the scalar cache (wave-uniform index) for the
// analysis and from a padded LDS image for the synthesis.
#include "common.h"

namespace rave {

typedef float pq_f32x4 __attribute__((ext_vector_type(4)));

#ifdef RAVE_STAMPS
// diagnostic build only: 8 clock stamps per workgroup (tools/pqmf_bench.py)
__device__ unsigned long long* g_pq_stamps = nullptr;
#define PQ_STAMP(k)                                                                               \
    do {                                                                                          \
        if (threadIdx.x == 0 && g_pq_stamps) {                                                    \
            const int wg_ = blockIdx.x + gridDim.x * blockIdx.y;                                  \
            g_pq_stamps[wg_ * 8 + (k)] = __builtin_amdgcn_s_memtime();                            \
            if ((k) == 0) g_pq_stamps[wg_ * 8 + 7] = __builtin_amdgcn_s_memrealtime();            \
        }                                                                                         \
    } while (0)
#else
#define PQ_STAMP(k) \
    do {            \
    } while (0)
#endif

// Both filters run as exact-fp32 MFMA GEMMs (v_mfma_f32_16x16x4_f32: a k-ordered
// fmaf chain, bitwise equal to f32 FMAs in k order).  A wave owns four blocks of
// 16 frames; A = filter rows (16), B = the window im2col read straight from LDS
// with padded, bank-conflict-free strides.
constexpr int kPqWaves = 4;
constexpr int kPqBlk = 2;                                    // 16-frame blocks per wave
constexpr int kPqFrames = kPqWaves * kPqBlk * 16;            // frames per workgroup (128)

// ---------------------------------------------------------------- analysis
// y[band][t] = rh * sum_{j < taps} h[band][j] x[16t + j - pad]  (band < NBO)
// Window frame f (16 samples) at LDS f*17 + r: lanes 16 frames apart hit 16
// different banks.  Filter rows (16, rows >= NBO zero) at stride kAnaHR.
constexpr int kAnaHR = 521;                                  // 516 taps + pad (mod 32 = 9)
constexpr int kAnaSteps = 129;                               // 513 taps -> 516
template <int NBO>
__global__ __launch_bounds__(64 * kPqWaves) void pqmf_analysis_kernel(rave_pqmf_analysis_args a, int wframes) {
    constexpr int ksteps = kAnaSteps;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* hs = smem;                                  // [16][kAnaHR]
    float* xs = smem + 16 * kAnaHR;                    // [wframes][17]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lg_ = __builtin_amdgcn_readfirstlane(
        xcd_major(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y));
    const int b = lg_ / gridDim.x;
    const int t0 = (lg_ - b * gridDim.x) * kPqFrames;
    const float* xb = a.x + (int64_t)b * a.x_sb;
    // filter rows >= NBO are zero; rows < NBO: taps, zero-padded to 4*ksteps.
    // All loads of a thread are issued before its first LDS store.
    constexpr int NT = 64 * kPqWaves;
    constexpr int HT = (NBO * kAnaHR + NT - 1) / NT;
    for (int i = tid; i < (16 - NBO) * kAnaHR; i += NT) hs[NBO * kAnaHR + i] = 0.f;
    {
        float hv[HT];
#pragma unroll
        for (int it = 0; it < HT; ++it) {
            const int i = tid + it * NT;
            const int k = (int)__umulhi((unsigned)i, 8243700u);        // i / 521 (i < 2^16)
            const int j = i - k * kAnaHR;
            // clamped address + value select (a conditional load makes hipcc
            // branch around it with a vmcnt(0) wait per element)
            const float v = a.hkf[(int64_t)min(k, NBO - 1) * a.taps + min(j, a.taps - 1)];
            hv[it] = (i < NBO * kAnaHR && j < a.taps) ? v : 0.f;
        }
#pragma unroll
        for (int it = 0; it < HT; ++it) {
            const int i = tid + it * NT;
            if (i < NBO * kAnaHR) hs[i] = hv[it];
        }
    }
    const int s0 = t0 * 16 - a.pad_left;
    {
        constexpr int XT = ((kPqFrames + 136) * 16 + NT - 1) / NT;     // >= wframes * 16 / NT
        float xv[XT];
#pragma unroll
        for (int it = 0; it < XT; ++it) {
            const int i = tid + it * NT;
            const int t = s0 + i;
            const float v = xb[min(max(t, 0), a.t_in - 1)];
            xv[it] = (i < wframes * 16 && t >= 0 && t < a.t_in) ? v : 0.f;
        }
#pragma unroll
        for (int it = 0; it < XT; ++it) {
            const int i = tid + it * NT;
            if (i < wframes * 16) xs[(i >> 4) * 17 + (i & 15)] = xv[it];
        }
    }
    __syncthreads();
    const int kk = lane >> 4, col = lane & 15;
    const int fb = wave * kPqBlk * 16;                 // wave's first frame (local)
    pq_f32x4 acc[kPqBlk];
#pragma unroll
    for (int q = 0; q < kPqBlk; ++q) acc[q] = pq_f32x4{0.f, 0.f, 0.f, 0.f};
    const float* ha = hs + col * kAnaHR + kk;          // A: row = band (lane & 15), k = 4s + kk
    // tap j = 4s + kk -> window frame col + (4s >> 4), sample (4s & 15) + kk: all
    // LDS offsets compile-time immediates (fully unrolled)
    const float* xl = xs + (fb + col) * 17 + kk;
#pragma unroll
    for (int s = 0; s < ksteps; ++s) {
        const float av = ha[4 * s];
#pragma unroll
        for (int q = 0; q < kPqBlk; ++q)
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, xl[((4 * s) >> 4) * 17 + ((4 * s) & 15) + q * 16 * 17],
                                                          acc[q], 0, 0, 0);
    }
    // D: row = band 4*(lane>>4) + r, column = frame lane & 15
    float* yb = a.y + (int64_t)b * a.y_sb;
#pragma unroll
    for (int q = 0; q < kPqBlk; ++q) {
        const int t = t0 + fb + q * 16 + col;
        if (t >= a.t_out) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = 4 * kk + r;
            if (k < NBO) {
                float v = acc[q][r];
                if ((k & 1) && !(t & 1)) v = -v;       // reverse_half
                yb[(int64_t)k * a.y_sc + t] = v;
            }
        }
    }
}

// ---------------------------------------------------------------- synthesis
// c[m][t] = sum_{c, k} hki[m][c][k] in[c][t + k - pad];  y[16t + i] = 16 c[15 - i][t]
// K ordered (c, k): 16 x 33 = 528 = 132 MFMA steps.  in[] rows at stride XR
// (window + pad), filter rows at kSynHR.
constexpr int kSynHR = 537;                                  // 528 + pad (mod 32 = 25)
constexpr int kSynTaps = 33;
constexpr int kSynXW = kPqFrames + kSynTaps - 1;
constexpr int kSynXR = kSynXW + ((25 - kSynXW % 32) + 32) % 32;    // row stride = 25 mod 32
__global__ __launch_bounds__(64 * kPqWaves) void pqmf_synthesis_kernel(rave_pqmf_synthesis_args a,
                                                                       unsigned a_xw_magic) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int nb = 16, taps = kSynTaps, xr = kSynXR;
    constexpr int kdim = nb * taps, ksteps = kdim / 4;
    float* hs = smem;                        // [16][kSynHR]
    float* xs = smem + 16 * kSynHR;          // [16][xr]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lg_ = __builtin_amdgcn_readfirstlane(
        xcd_major(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y));
    const int b = lg_ / gridDim.x;
    const int n0 = (lg_ - b * gridDim.x) * kPqFrames;
    PQ_STAMP(0);
    // every load of a thread is issued before its first LDS store
    constexpr int NT = 64 * kPqWaves;
    {
        constexpr int HT = (16 * kSynHR + NT - 1) / NT;
        float hv[HT];
#pragma unroll
        for (int it = 0; it < HT; ++it) {
            const int i = tid + it * NT;
            const int m = (int)__umulhi((unsigned)i, 7998077u);        // i / 537 (i < 2^16)
            const int k = i - m * kSynHR;                               // K index = tap*16 + c
            const int kc = min(k, kdim - 1);
            const float v = a.hki[(int64_t)min(m, 15) * kdim + (kc & 15) * taps + (kc >> 4)];
            hv[it] = (i < 16 * kSynHR && k < kdim) ? v : 0.f;
        }
#pragma unroll
        for (int it = 0; it < HT; ++it) {
            const int i = tid + it * NT;
            if (i < 16 * kSynHR) hs[i] = hv[it];
        }
    }
    PQ_STAMP(1);
    const float* xb = a.x + (int64_t)b * a.x_sb;
    const float* nzb = a.noise ? a.noise + (int64_t)b * a.n_sb : nullptr;
    const int x_len = a.x_len > 0 ? a.x_len : a.t_in;
    constexpr int xw = kSynXW;
    {
        constexpr int XT = (16 * xw + NT - 1) / NT;
        float xv[XT], av[XT], nv[XT];
#pragma unroll
        for (int it = 0; it < XT; ++it) {
            const int i = tid + it * NT;
            const int c = (int)__umulhi((unsigned)i, a_xw_magic);
            const int w = i - c * xw;
            const int f = n0 - a.pad_left + w;
            const int cc = min(c, 15), ff = min(max(f, 0), max(x_len - 1, 0));
            xv[it] = xb[(int64_t)cc * a.x_sc + ff];                   // selects happen below
            av[it] = xb[(int64_t)(a.mode == 1 ? cc + 16 : cc) * a.x_sc + ff];
            nv[it] = nzb ? nzb[(int64_t)cc * a.n_sc + ff] : 0.f;     // uniform branch
        }
#pragma unroll
        for (int it = 0; it < XT; ++it) {
            const int i = tid + it * NT;
            const int c = (int)__umulhi((unsigned)i, a_xw_magic);
            const int w = i - c * xw;
            const int f = n0 - a.pad_left + w;
            const bool ok = i < 16 * xw && f >= 0 && f < x_len;
            float v = ok ? xv[it] : 0.f;
            if (a.mode != 0) {
                if (a.mode == 1) v = v * (1.0f / (1.0f + __expf(-av[it])));
                v = v + (ok ? nv[it] : 0.f);
                v = tanhf(v);
            }
            if ((c & 1) && !((a.frame0 + f) & 1)) v = -v;   // reverse_half
            if (i < 16 * xw) xs[c * xr + w] = ok ? v : 0.f;
        }
    }
    __syncthreads();
    PQ_STAMP(2);
    const int kk = lane >> 4, col = lane & 15;
    const int fb = wave * kPqBlk * 16;
    pq_f32x4 acc[kPqBlk];
#pragma unroll
    for (int q = 0; q < kPqBlk; ++q) acc[q] = pq_f32x4{0.f, 0.f, 0.f, 0.f};
    const float* ha = hs + col * kSynHR + kk;
    // K = (tap, c): step s covers channels 4(s%4)..+3 of tap s/4, lane kk one of
    // them; every LDS offset is a compile-time immediate (fully unrolled)
    const float* xl = xs + kk * xr + fb + col;
#pragma unroll
    for (int s = 0; s < ksteps; ++s) {
        const float av = ha[4 * s];
#pragma unroll
        for (int q = 0; q < kPqBlk; ++q)
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, xl[(4 * (s & 3)) * xr + (s >> 2) + q * 16], acc[q],
                                                          0, 0, 0);
    }
    PQ_STAMP(3);
    // D: row m = 4*(lane>>4) + r, column = frame: y[16t + 15 - m] = 16 * D, four
    // consecutive (descending) samples per lane -> one 16-byte store
    float* yb = a.y + (int64_t)b * a.y_sb;
#pragma unroll
    for (int q = 0; q < kPqBlk; ++q) {
        const int t = n0 + fb + q * 16 + col;
        if (t >= a.t_in) continue;
        const pq_f32x4 v = {16.f * acc[q][3], 16.f * acc[q][2], 16.f * acc[q][1], 16.f * acc[q][0]};
        *reinterpret_cast<pq_f32x4*>(yb + (int64_t)t * nb + 12 - 4 * kk) = v;
    }
    PQ_STAMP(4);
}

// ------------------------------------------------- split-f16 variants (RAVE_PREC_SPLIT16)
// The same two GEMMs on v_mfma_f32_16x16x32_f16 with conv_split.hip's
// arithmetic: every fp32 operand v is an f16 pair hi = f16(v), lo =
// f16((v - hi) 2^11); acc += (hi_h 2^11) hi_x + hi_h lo_x + lo_h hi_x (the lo*lo
// term and two roundings ~2^-22 relative); the filter is scaled by one power of
// two 2^e (max |h 2^e| in [8, 16), computed in-kernel) so its halves stay
// normal, and the epilogue multiplies by 2^-(e + 11) exactly.
// A wave owns kPsBlk blocks of 16 frames; a workgroup kPsWaves waves.
typedef _Float16 ps_h8 __attribute__((ext_vector_type(8)));
typedef float ps_f32x8 __attribute__((ext_vector_type(8)));
#ifndef RAVE_PS_WAVES
#define RAVE_PS_WAVES 4
#endif
constexpr int kPsWaves = RAVE_PS_WAVES;
#ifndef RAVE_PS_BLK
#define RAVE_PS_BLK 2                   // measured (profiles/r02_xcd/ab_pqmf_blk.txt): 2 beats 4 and 1
#endif
constexpr int kPsBlk = RAVE_PS_BLK;                         // 16-frame blocks per wave
constexpr int kPsFrames = kPsWaves * kPsBlk * 16;            // frames per workgroup (128)
// analysis: the same 128 frames per workgroup as 8 waves of one 16-frame block
// (12.9 -> 11.0 us against 4 waves of two, profiles/r02_xcd/ab_pqmf_waves.txt;
// synthesis keeps 4 x 2, which 8 x 1 slows)
#ifndef RAVE_PA_WAVES
#define RAVE_PA_WAVES 8
#endif
constexpr int kPaWaves = RAVE_PA_WAVES;
constexpr int kPaBlk = kPsFrames / (16 * kPaWaves);
constexpr int kPaFrames = kPaWaves * kPaBlk * 16;
static_assert(kPaFrames == kPsFrames && kPaBlk >= 1, "analysis geometry");
constexpr int kPsK = 17;                                     // 32-deep K-steps (<= 544 taps / K rows)
constexpr int kPsKP = 552;                                   // halves per filter row: 1104 B = 20 banks mod 64

// Power-of-two scales from the workgroup's maxima (wave max via LDS; `red`
// holds 2 W floats): the filter's 2^e with max |h 2^e| in [8, 16), and the
// signal's split-f16 range guard 2^-s (common.h split_shift: 1 unless the
// staged window reaches 2^15).
template <int W>
__device__ __forceinline__ float ps_scale(float amax, float xmax, float* red, float& xs) {
    amax = wave_max(amax);
    xmax = wave_max(xmax);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        red[wave] = amax;
        red[W + wave] = xmax;
    }
    __syncthreads();
    float m = red[0], mx = red[W];
#pragma unroll
    for (int w = 1; w < W; ++w) {
        m = fmaxf(m, red[w]);
        mx = fmaxf(mx, red[W + w]);
    }
    xs = ldexpf(1.f, -split_shift(mx));
    if (!(m > 0.f)) return 1.f;
    int e;
    (void)frexpf(m, &e);                  // m in [2^(e-1), 2^e)
    return ldexpf(1.f, 4 - e);            // m 2^(4-e) in [8, 16)
}

__device__ __forceinline__ void ps_split(float v, _Float16& hi, _Float16& lo) {
    hi = (_Float16)v;
    lo = (_Float16)((v - (float)hi) * 2048.0f);
}

// analysis: A = filter rows (band), k = tap j; B = window samples, frame f's
// K-run j..j+7 = samples 16 f + j .. +7 (flat f16 planes, 8 halves of pad every
// 128 samples: the 16 frames of a read land on 16 distinct bank quads)
__host__ __device__ constexpr int ps_xi(int i) { return i + 8 * (i >> 7); }
template <int NBO>
__global__ __launch_bounds__(64 * kPaWaves) void pqmf_analysis_split_kernel(rave_pqmf_analysis_args a, int wframes) {
    extern __shared__ __attribute__((aligned(16))) char ps_smem[];
    _Float16* fh = reinterpret_cast<_Float16*>(ps_smem);     // [16][kPsKP]
    _Float16* fl = fh + 16 * kPsKP;
    _Float16* xh = fl + 16 * kPsKP;                           // [ps_xi(wframes * 16)]
    const int WS = ps_xi(wframes * 16) + 8;
    _Float16* xl = xh + WS;
    float* red = reinterpret_cast<float*>(xl + WS);
    constexpr int NT = 64 * kPaWaves;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lg_ = __builtin_amdgcn_readfirstlane(
        xcd_major(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y));
    const int b = lg_ / gridDim.x;
    const int t0 = (lg_ - b * gridDim.x) * kPaFrames;
    const float* xb = a.x + (int64_t)b * a.x_sb;
    // filter: rows < NBO, taps < a.taps (all loads before the first LDS store)
    constexpr int KW = 32 * kPsK;                             // 544
    constexpr int HT = (NBO * KW + NT - 1) / NT;
    float hv[HT];
    float amax = 0.f;
#pragma unroll
    for (int it = 0; it < HT; ++it) {
        const int i = tid + it * NT;
        const int k = i / KW, j = i - k * KW;
        const float v = a.hkf[(int64_t)min(k, NBO - 1) * a.taps + min(j, a.taps - 1)];
        hv[it] = (i < NBO * KW && j < a.taps) ? v : 0.f;
        amax = fmaxf(amax, fabsf(hv[it]));
    }
    const int s0 = t0 * 16 - a.pad_left;
    constexpr int XT = ((kPaFrames + 40) * 16 + NT - 1) / NT;
    float xv[XT];
    float xmax = 0.f;
#pragma unroll
    for (int it = 0; it < XT; ++it) {
        const int i = tid + it * NT;
        const int t = s0 + i;
        const float v = xb[min(max(t, 0), a.t_in - 1)];
        xv[it] = (i < wframes * 16 && t >= 0 && t < a.t_in) ? v : 0.f;
        xmax = fmaxf(xmax, fabsf(xv[it]));
    }
    float xs;
    const float sc = ps_scale<kPaWaves>(amax, xmax, red, xs);
    for (int i = tid; i < (16 - NBO) * kPsKP; i += NT) {
        fh[NBO * kPsKP + i] = (_Float16)0.f;
        fl[NBO * kPsKP + i] = (_Float16)0.f;
    }
#pragma unroll
    for (int it = 0; it < HT; ++it) {
        const int i = tid + it * NT;
        if (i < NBO * KW) {
            const int k = i / KW, j = i - k * KW;
            ps_split(hv[it] * sc, fh[k * kPsKP + j], fl[k * kPsKP + j]);
        }
    }
#pragma unroll
    for (int it = 0; it < XT; ++it) {
        const int i = tid + it * NT;
        if (i < wframes * 16) ps_split(xv[it] * xs, xh[ps_xi(i)], xl[ps_xi(i)]);
    }
    __syncthreads();
    const int g = lane >> 4, col = lane & 15;
    const int fb = wave * kPaBlk * 16;
    pq_f32x4 acc[kPaBlk];
#pragma unroll
    for (int q = 0; q < kPaBlk; ++q) acc[q] = pq_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kPsK; ++s) {
        const int ka = col * kPsKP + 32 * s + 8 * g;
        const ps_h8 ah = *reinterpret_cast<const ps_h8*>(fh + ka);
        const ps_h8 al = *reinterpret_cast<const ps_h8*>(fl + ka);
        const ps_h8 a2 = ah * (_Float16)2048.0f;
#pragma unroll
        for (int q = 0; q < kPaBlk; ++q) {
            const int xi = ps_xi(16 * (fb + 16 * q + col) + 32 * s + 8 * g);
            const ps_h8 bh = *reinterpret_cast<const ps_h8*>(xh + xi);
            const ps_h8 bl = *reinterpret_cast<const ps_h8*>(xl + xi);
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, bh, acc[q], 0, 0, 0);
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc[q], 0, 0, 0);
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[q], 0, 0, 0);
        }
    }
    const float unscale = 1.0f / (sc * 2048.0f * xs);         // exact: powers of two
    float* yb = a.y + (int64_t)b * a.y_sb;
#pragma unroll
    for (int q = 0; q < kPaBlk; ++q) {
        const int t = t0 + fb + q * 16 + col;
        if (t >= a.t_out) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = 4 * g + r;
            if (k < NBO) {
                float v = acc[q][r] * unscale;
                if ((k & 1) && !(t & 1)) v = -v;              // reverse_half
                yb[(int64_t)k * a.y_sc + t] = v;
            }
        }
    }
}

// synthesis: A = hki rows m, k = tap * 16 + c (K 528 -> 544); B = the staged
// input channels-last, row w = frame + tap: a K-run (tap, 8 channels) is one
// 16-byte read; row stride 24 halves = 12 banks, conflict-free over 16 frames.
constexpr int kPsXW = kPsFrames + 34;                        // window rows (taps 0..33)
constexpr int kPsXP = 24;                                    // halves per window row
__global__ __launch_bounds__(64 * kPsWaves) void pqmf_synthesis_split_kernel(rave_pqmf_synthesis_args a,
                                                                             unsigned a_xw_magic) {
    extern __shared__ __attribute__((aligned(16))) char ps_smem[];
    _Float16* fh = reinterpret_cast<_Float16*>(ps_smem);     // [16][kPsKP]
    _Float16* fl = fh + 16 * kPsKP;
    _Float16* xh = fl + 16 * kPsKP;                           // [kPsXW][kPsXP]
    _Float16* xl = xh + kPsXW * kPsXP;
    float* red = reinterpret_cast<float*>(xl + kPsXW * kPsXP);
    constexpr int nb = 16, taps = kSynTaps, kdim = nb * taps;
    constexpr int NT = 64 * kPsWaves;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lg_ = __builtin_amdgcn_readfirstlane(
        xcd_major(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y));
    const int b = lg_ / gridDim.x;
    const int n0 = (lg_ - b * gridDim.x) * kPsFrames;
    constexpr int KW = 32 * kPsK;                             // 544
    constexpr int HT = (16 * KW + NT - 1) / NT;
    float hv[HT];
    float amax = 0.f;
#pragma unroll
    for (int it = 0; it < HT; ++it) {
        const int i = tid + it * NT;
        const int m = i / KW, k = i - m * KW;                 // K index = tap*16 + c
        const int kc = min(k, kdim - 1);
        const float v = a.hki[(int64_t)min(m, 15) * kdim + (kc & 15) * taps + (kc >> 4)];
        hv[it] = (i < 16 * KW && k < kdim) ? v : 0.f;
        amax = fmaxf(amax, fabsf(hv[it]));
    }
    const float* xb = a.x + (int64_t)b * a.x_sb;
    const float* nzb = a.noise ? a.noise + (int64_t)b * a.n_sb : nullptr;
    const int x_len = a.x_len > 0 ? a.x_len : a.t_in;
    constexpr int xw = kPsXW;
    constexpr int XT = (16 * xw + NT - 1) / NT;
    float xv[XT], av[XT], nv[XT];
#pragma unroll
    for (int it = 0; it < XT; ++it) {
        const int i = tid + it * NT;
        const int c = (int)__umulhi((unsigned)i, a_xw_magic);
        const int w = i - c * xw;
        const int f = n0 - a.pad_left + w;
        const int cc = min(c, 15), ff = min(max(f, 0), max(x_len - 1, 0));
        xv[it] = xb[(int64_t)cc * a.x_sc + ff];
        av[it] = xb[(int64_t)(a.mode == 1 ? cc + 16 : cc) * a.x_sc + ff];
        nv[it] = nzb ? nzb[(int64_t)cc * a.n_sc + ff] : 0.f;
    }
    float xmax = 0.f;
#pragma unroll
    for (int it = 0; it < XT; ++it) {
        const int i = tid + it * NT;
        const int c = (int)__umulhi((unsigned)i, a_xw_magic);
        const int w = i - c * xw;
        const int f = n0 - a.pad_left + w;
        const bool ok = i < 16 * xw && f >= 0 && f < x_len;
        float v = ok ? xv[it] : 0.f;
        if (a.mode != 0) {
            if (a.mode == 1) v = v * (1.0f / (1.0f + __expf(-av[it])));
            v = v + (ok ? nv[it] : 0.f);
            v = tanhf(v);
        }
        if ((c & 1) && !((a.frame0 + f) & 1)) v = -v;   // reverse_half
        xv[it] = ok ? v : 0.f;
        xmax = fmaxf(xmax, fabsf(xv[it]));
    }
    float xs;
    const float sc = ps_scale<kPsWaves>(amax, xmax, red, xs);
#pragma unroll
    for (int it = 0; it < HT; ++it) {
        const int i = tid + it * NT;
        if (i < 16 * KW) {
            const int m = i / KW, k = i - m * KW;
            ps_split(hv[it] * sc, fh[m * kPsKP + k], fl[m * kPsKP + k]);
        }
    }
#pragma unroll
    for (int it = 0; it < XT; ++it) {
        const int i = tid + it * NT;
        const int c = (int)__umulhi((unsigned)i, a_xw_magic);
        const int w = i - c * xw;
        if (i < 16 * xw) ps_split(xv[it] * xs, xh[w * kPsXP + c], xl[w * kPsXP + c]);
    }
    __syncthreads();
    const int g = lane >> 4, col = lane & 15;
    const int fb = wave * kPsBlk * 16;
    pq_f32x4 acc[kPsBlk];
#pragma unroll
    for (int q = 0; q < kPsBlk; ++q) acc[q] = pq_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kPsK; ++s) {
        // k = 32 s + 8 g + e: tap 2 s + (g >> 1), channels 8 (g & 1) + e
        const int ka = col * kPsKP + 32 * s + 8 * g;
        const ps_h8 ah = *reinterpret_cast<const ps_h8*>(fh + ka);
        const ps_h8 al = *reinterpret_cast<const ps_h8*>(fl + ka);
        const ps_h8 a2 = ah * (_Float16)2048.0f;
        const int tap = 2 * s + (g >> 1);
#pragma unroll
        for (int q = 0; q < kPsBlk; ++q) {
            const int xi = (fb + 16 * q + col + tap) * kPsXP + 8 * (g & 1);
            const ps_h8 bh = *reinterpret_cast<const ps_h8*>(xh + xi);
            const ps_h8 bl = *reinterpret_cast<const ps_h8*>(xl + xi);
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, bh, acc[q], 0, 0, 0);
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc[q], 0, 0, 0);
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[q], 0, 0, 0);
        }
    }
    const float o = 16.f / (sc * 2048.0f * xs);               // n_band x the exact unscale
    float* yb = a.y + (int64_t)b * a.y_sb;
#pragma unroll
    for (int q = 0; q < kPsBlk; ++q) {
        const int t = n0 + fb + q * 16 + col;
        if (t >= a.t_in) continue;
        const pq_f32x4 v = {o * acc[q][3], o * acc[q][2], o * acc[q][1], o * acc[q][0]};
        *reinterpret_cast<pq_f32x4*>(yb + (int64_t)t * nb + 12 - 4 * g) = v;
    }
}

#ifdef RAVE_STAMPS
extern "C" int rave_diag_pqmf_stamps(void* p) {
    RAVE_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_pq_stamps), &p, sizeof(p)));
    return RAVE_OK;
}
#endif

}  // namespace rave

using namespace rave;

extern "C" int rave_pqmf_analysis(const rave_pqmf_analysis_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y && p->hkf, "pqmf_analysis: null pointer");
    const rave_pqmf_analysis_args& a = *p;
    RAVE_CHECK_ARG(a.n_band == 16, "pqmf_analysis: kernel is built for 16 bands");
    RAVE_CHECK_ARG(a.n_out_bands == 6 || a.n_out_bands == 16,
                   "pqmf_analysis: n_out_bands must be 6 (RAVE.encode) or 16");
    RAVE_CHECK_ARG(a.taps > 0 && a.taps <= 1024, "pqmf_analysis: bad taps");
    RAVE_CHECK_ARG(a.batch > 0 && a.t_in > 0 && a.t_out > 0, "pqmf_analysis: empty shape");
    if ((a.taps + 3) / 4 != kAnaSteps) {
        set_error("pqmf_analysis: kernel is built for the 513-tap RAVE prototype");
        return RAVE_ERR_UNSUPPORTED;
    }
    RAVE_CHECK_ARG(a.precision == RAVE_PREC_F32 || a.precision == RAVE_PREC_SPLIT16,
                   "pqmf_analysis: precision must be RAVE_PREC_F32 or RAVE_PREC_SPLIT16");
    if (a.precision == RAVE_PREC_SPLIT16) {
        const int wframes = kPsFrames + (32 * kPsK + 15) / 16 + 1;
        const int ws = ps_xi(wframes * 16) + 8;
        const size_t lds = (size_t)(2 * 16 * kPsKP + 2 * ws) * 2 + 2 * kPaWaves * 4;
        dim3 grid(ceil_div(a.t_out, kPaFrames), a.batch);
        if (a.n_out_bands == 6)
            launch(pqmf_analysis_split_kernel<6>, grid, dim3(64 * kPaWaves), lds, as_stream(stream), a, wframes);
        else
            launch(pqmf_analysis_split_kernel<16>, grid, dim3(64 * kPaWaves), lds, as_stream(stream), a, wframes);
        return launch_status("pqmf_analysis_split_kernel");
    }
    const int wframes = kPqFrames + (4 * kAnaSteps + 15) / 16 + 1;
    const size_t lds = (size_t)(16 * kAnaHR + wframes * 17) * sizeof(float);
    dim3 grid(ceil_div(a.t_out, kPqFrames), a.batch);
    if (a.n_out_bands == 6)
        launch(pqmf_analysis_kernel<6>, grid, dim3(64 * kPqWaves), lds, as_stream(stream), a, wframes);
    else
        launch(pqmf_analysis_kernel<16>, grid, dim3(64 * kPqWaves), lds, as_stream(stream), a, wframes);
    return launch_status("pqmf_analysis_kernel");
}

extern "C" int rave_pqmf_synthesis(const rave_pqmf_synthesis_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y && p->hki, "pqmf_synthesis: null pointer");
    const rave_pqmf_synthesis_args& a = *p;
    RAVE_CHECK_ARG(a.n_band == 16, "pqmf_synthesis: kernel is built for 16 bands");
    RAVE_CHECK_ARG(a.taps > 0 && a.taps <= 64, "pqmf_synthesis: bad taps");
    RAVE_CHECK_ARG(a.batch > 0 && a.t_in > 0, "pqmf_synthesis: empty shape");
    RAVE_CHECK_ARG(a.mode >= 0 && a.mode <= 2, "pqmf_synthesis: mode must be 0, 1 or 2");
    if (a.taps != kSynTaps) {
        set_error("pqmf_synthesis: kernel is built for the 33-tap RAVE synthesis filter");
        return RAVE_ERR_UNSUPPORTED;
    }
    RAVE_CHECK_ARG(reinterpret_cast<uintptr_t>(a.y) % 16 == 0 && a.y_sb % 4 == 0,
                   "pqmf_synthesis: output must be 16-byte aligned");
    RAVE_CHECK_ARG(a.precision == RAVE_PREC_F32 || a.precision == RAVE_PREC_SPLIT16,
                   "pqmf_synthesis: precision must be RAVE_PREC_F32 or RAVE_PREC_SPLIT16");
    if (a.precision == RAVE_PREC_SPLIT16) {
        const size_t lds = (size_t)(2 * 16 * kPsKP + 2 * kPsXW * kPsXP) * 2 + 2 * kPsWaves * 4;
        dim3 grid(ceil_div(a.t_in, kPsFrames), a.batch);
        const unsigned xw_magic = (unsigned)((0x100000000ull + kPsXW - 1) / kPsXW);
        launch(pqmf_synthesis_split_kernel, grid, dim3(64 * kPsWaves), lds, as_stream(stream), a, xw_magic);
        return launch_status("pqmf_synthesis_split_kernel");
    }
    const int xw = kSynXW;
    const size_t lds = (size_t)(16 * kSynHR + 16 * kSynXR) * sizeof(float);
    dim3 grid(ceil_div(a.t_in, kPqFrames), a.batch);
    const unsigned xw_magic = (unsigned)((0x100000000ull + xw - 1) / xw);   // ceil(2^32 / xw)
    launch(pqmf_synthesis_kernel, grid, dim3(64 * kPqWaves), lds, as_stream(stream), a, xw_magic);
    return launch_status("pqmf_synthesis_kernel");
}
