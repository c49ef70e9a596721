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

constexpr int kAnaT = 256;     // output frames per workgroup (one per thread)
constexpr int kSynT = 64;      // frames per workgroup

__global__ __launch_bounds__(256) void pqmf_analysis_kernel(rave_pqmf_analysis_args a, int xws) {
    extern __shared__ __attribute__((aligned(16))) float xs[];   // [n_band][xws]
    const int nb = a.n_band;
    const int t0 = blockIdx.x * kAnaT;
    const int b = blockIdx.y;
    const float* xb = a.x + (int64_t)b * a.x_sb;
    const int in0 = t0 * nb - a.pad_left;
    const int xw = (kAnaT - 1) * nb + a.taps;
    for (int i = threadIdx.x; i < xw; i += blockDim.x) {
        int t = in0 + i;
        float v = (t >= 0 && t < a.t_in) ? xb[t] : 0.f;
        xs[(i % nb) * xws + i / nb] = v;
    }
    __syncthreads();
    const int tl = threadIdx.x;
    const int t = t0 + tl;
    float acc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = 0.f;
    const int nbo = a.n_out_bands;
    for (int j0 = 0; j0 < a.taps; j0 += nb) {
        const int jn = min(nb, a.taps - j0);
        for (int p = 0; p < jn; ++p) {
            const float xv = xs[p * xws + tl + j0 / nb];
            const float* hcol = a.hkf + j0 + p;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (k < nbo) acc[k] = fmaf(hcol[(int64_t)k * a.taps], xv, acc[k]);
        }
    }
    if (t >= a.t_out) return;
    float* yb = a.y + (int64_t)b * a.y_sb;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (k < nbo) {
            float v = acc[k];
            if ((k & 1) && !(t & 1)) v = -v;   // reverse_half
            yb[(int64_t)k * a.y_sc + t] = v;
        }
    }
}

__global__ __launch_bounds__(256) void pqmf_synthesis_kernel(rave_pqmf_synthesis_args a, int hrow) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int nb = a.n_band;                 // 16
    const int taps = a.taps;                 // 33
    const int xw = kSynT + taps - 1;
    float* hs = smem;                        // [nb][hrow] (hrow = nb*taps + 1)
    float* xs = smem + nb * hrow;            // [nb][xw]
    const int n0 = blockIdx.x * kSynT;
    const int b = blockIdx.y;

    for (int i = threadIdx.x; i < nb * nb * taps; i += blockDim.x) {
        int m = i / (nb * taps);
        int r = i - m * nb * taps;
        hs[m * hrow + r] = a.hki[i];
    }
    const float* xb = a.x + (int64_t)b * a.x_sb;
    const float* nzb = a.noise ? a.noise + (int64_t)b * a.n_sb : nullptr;
    const int x_len = a.x_len > 0 ? a.x_len : a.t_in;
    for (int i = threadIdx.x; i < nb * xw; i += blockDim.x) {
        int c = i / xw;
        int w = i - c * xw;
        int f = n0 - a.pad_left + w;
        float v = 0.f;
        if (f >= 0 && f < x_len) {
            v = xb[(int64_t)c * a.x_sc + f];
            if (a.mode == 1) {
                float amp = xb[(int64_t)(c + nb) * a.x_sc + f];
                v = v * (1.0f / (1.0f + expf(-amp)));
                if (nzb) v = v + nzb[(int64_t)c * a.n_sc + f];
                v = tanhf(v);
            }
            if ((c & 1) && !((a.frame0 + f) & 1)) v = -v;   // reverse_half
        }
        xs[c * xw + w] = v;
    }
    __syncthreads();
    const int i = threadIdx.x & 15;          // output sample within a frame
    const int ng = threadIdx.x >> 4;         // 16 groups x 4 frames
    const int m = nb - 1 - i;                // channel flip
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const float* hm = hs + m * hrow;
    for (int c = 0; c < nb; ++c) {
        const float* xc = xs + c * xw + ng * 4;
        const float* hc = hm + c * taps;
        for (int k = 0; k < taps; ++k) {
            const float hv = hc[k];
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] = fmaf(hv, xc[q + k], acc[q]);
        }
    }
    float* yb = a.y + (int64_t)b * a.y_sb;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int n = n0 + ng * 4 + q;
        if (n < a.t_in) yb[(int64_t)n * nb + i] = acc[q] * (float)nb;
    }
}

}  // namespace rave

using namespace rave;

extern "C" int rave_pqmf_analysis(const rave_pqmf_analysis_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y && p->hkf, "pqmf_analysis: null pointer");
    const rave_pqmf_analysis_args& a = *p;
    RAVE_CHECK_ARG(a.n_band > 0 && a.n_band <= 16 && a.n_out_bands > 0 && a.n_out_bands <= a.n_band,
                   "pqmf_analysis: n_band must be in [1, 16]");
    RAVE_CHECK_ARG(a.taps > 0 && a.taps <= 2048, "pqmf_analysis: bad taps");
    RAVE_CHECK_ARG(a.batch > 0 && a.t_in > 0 && a.t_out > 0, "pqmf_analysis: empty shape");
    int xw = (kAnaT - 1) * a.n_band + a.taps;
    int xws = ceil_div(xw, a.n_band) + 1;
    size_t lds = (size_t)a.n_band * xws * sizeof(float);
    dim3 grid(ceil_div(a.t_out, kAnaT), a.batch);
    hipLaunchKernelGGL(pqmf_analysis_kernel, grid, dim3(256), lds, as_stream(stream), a, xws);
    return launch_status("pqmf_analysis_kernel");
}

extern "C" int rave_pqmf_synthesis(const rave_pqmf_synthesis_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y && p->hki, "pqmf_synthesis: null pointer");
    const rave_pqmf_synthesis_args& a = *p;
    RAVE_CHECK_ARG(a.n_band == 16, "pqmf_synthesis: kernel is built for 16 bands");
    RAVE_CHECK_ARG(a.taps > 0 && a.taps <= 64, "pqmf_synthesis: bad taps");
    RAVE_CHECK_ARG(a.batch > 0 && a.t_in > 0, "pqmf_synthesis: empty shape");
    RAVE_CHECK_ARG(a.mode == 0 || a.mode == 1, "pqmf_synthesis: mode must be 0 or 1");
    int hrow = a.n_band * a.taps + 1;
    size_t lds = (size_t)(a.n_band * hrow + a.n_band * (kSynT + a.taps - 1)) * sizeof(float);
    dim3 grid(ceil_div(a.t_in, kSynT), a.batch);
    hipLaunchKernelGGL(pqmf_synthesis_kernel, grid, dim3(256), lds, as_stream(stream), a, hrow);
    return launch_status("pqmf_synthesis_kernel");
}
