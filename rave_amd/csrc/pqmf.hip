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
    const int t0 = blockIdx.x * kPqFrames;
    const int b = blockIdx.y;
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
    const int n0 = blockIdx.x * kPqFrames;
    const int b = blockIdx.y;
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
    const int xw = kSynXW;
    const size_t lds = (size_t)(16 * kSynHR + 16 * kSynXR) * sizeof(float);
    dim3 grid(ceil_div(a.t_in, kPqFrames), a.batch);
    const unsigned xw_magic = (unsigned)((0x100000000ull + xw - 1) / xw);   // ceil(2^32 / xw)
    launch(pqmf_synthesis_kernel, grid, dim3(64 * kPqWaves), lds, as_stream(stream), a, xw_magic);
    return launch_status("pqmf_synthesis_kernel");
}
