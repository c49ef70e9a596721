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

constexpr int kAnaT = 128;     // output frames per workgroup (one per thread)
constexpr int kSynT = 64;      // frames per workgroup
constexpr int kFrameStride = 20;   // LDS floats per 16-sample frame (16 + 4 pad: conflict-free b128)

// Analysis (16 bands): window stored frame-major [frame][20] so one ds_read_b128
// returns 4 consecutive taps of a thread's frame (lane stride 20 dwords keeps a
// 16-lane group on 64 distinct banks); the filter [band][taps rounded to 4] is
// read as wave-uniform float4 broadcasts.  NBO (bands produced) is compile-time
// so the accumulators stay in registers.
template <int NBO>
__global__ __launch_bounds__(kAnaT) void pqmf_analysis_kernel(rave_pqmf_analysis_args a, int taps4,
                                                              int wframes) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* hs = smem;                                  // [NBO][taps4]
    float* xs = smem + NBO * taps4;                    // [wframes][kFrameStride]
    const int t0 = blockIdx.x * kAnaT;
    const int b = blockIdx.y;
    const float* xb = a.x + (int64_t)b * a.x_sb;
    for (int i = threadIdx.x; i < NBO * taps4; i += kAnaT) {
        const int k = i / taps4, j = i - k * taps4;
        hs[i] = j < a.taps ? a.hkf[(int64_t)k * a.taps + j] : 0.f;
    }
    const int in0 = t0 * 16 - a.pad_left;
    for (int i = threadIdx.x; i < wframes * 16; i += kAnaT) {
        const int t = in0 + i;
        const float v = (t >= 0 && t < a.t_in) ? xb[t] : 0.f;
        xs[(i >> 4) * kFrameStride + (i & 15)] = v;
    }
    __syncthreads();
    const int tl = threadIdx.x;
    float acc[NBO];
#pragma unroll
    for (int k = 0; k < NBO; ++k) acc[k] = 0.f;
    for (int j = 0; j < taps4; j += 4) {
        const float4 xv = *reinterpret_cast<const float4*>(xs + (tl + (j >> 4)) * kFrameStride + (j & 15));
#pragma unroll
        for (int k = 0; k < NBO; ++k) {
            const float4 hv = *reinterpret_cast<const float4*>(hs + k * taps4 + j);
            acc[k] = fmaf(hv.x, xv.x, acc[k]);
            acc[k] = fmaf(hv.y, xv.y, acc[k]);
            acc[k] = fmaf(hv.z, xv.z, acc[k]);
            acc[k] = fmaf(hv.w, xv.w, acc[k]);
        }
    }
    const int t = t0 + tl;
    if (t >= a.t_out) return;
    float* yb = a.y + (int64_t)b * a.y_sb;
#pragma unroll
    for (int k = 0; k < NBO; ++k) {
        float v = acc[k];
        if ((k & 1) && !(t & 1)) v = -v;   // reverse_half
        yb[(int64_t)k * a.y_sc + t] = v;
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
            if (a.mode != 0) {
                if (a.mode == 1) {
                    float amp = xb[(int64_t)(c + nb) * a.x_sc + f];
                    v = v * (1.0f / (1.0f + expf(-amp)));
                }
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
    RAVE_CHECK_ARG(a.n_band == 16, "pqmf_analysis: kernel is built for 16 bands");
    RAVE_CHECK_ARG(a.n_out_bands == 6 || a.n_out_bands == 16,
                   "pqmf_analysis: n_out_bands must be 6 (RAVE.encode) or 16");
    RAVE_CHECK_ARG(a.taps > 0 && a.taps <= 1024, "pqmf_analysis: bad taps");
    RAVE_CHECK_ARG(a.batch > 0 && a.t_in > 0 && a.t_out > 0, "pqmf_analysis: empty shape");
    const int taps4 = (a.taps + 3) & ~3;
    const int wframes = kAnaT + taps4 / 16 + 1;
    size_t lds = (size_t)(a.n_out_bands * taps4 + wframes * kFrameStride) * sizeof(float);
    dim3 grid(ceil_div(a.t_out, kAnaT), a.batch);
    if (a.n_out_bands == 6)
        launch(pqmf_analysis_kernel<6>, grid, dim3(kAnaT), lds, as_stream(stream), a, taps4, wframes);
    else
        launch(pqmf_analysis_kernel<16>, grid, dim3(kAnaT), lds, as_stream(stream), a, taps4, wframes);
    return launch_status("pqmf_analysis_kernel");
}

extern "C" int rave_pqmf_synthesis(const rave_pqmf_synthesis_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y && p->hki, "pqmf_synthesis: null pointer");
    const rave_pqmf_synthesis_args& a = *p;
    RAVE_CHECK_ARG(a.n_band == 16, "pqmf_synthesis: kernel is built for 16 bands");
    RAVE_CHECK_ARG(a.taps > 0 && a.taps <= 64, "pqmf_synthesis: bad taps");
    RAVE_CHECK_ARG(a.batch > 0 && a.t_in > 0, "pqmf_synthesis: empty shape");
    RAVE_CHECK_ARG(a.mode >= 0 && a.mode <= 2, "pqmf_synthesis: mode must be 0, 1 or 2");
    int hrow = a.n_band * a.taps + 1;
    size_t lds = (size_t)(a.n_band * hrow + a.n_band * (kSynT + a.taps - 1)) * sizeof(float);
    dim3 grid(ceil_div(a.t_in, kSynT), a.batch);
    launch(pqmf_synthesis_kernel, grid, dim3(256), lds, as_stream(stream), a, hrow);
    return launch_status("pqmf_synthesis_kernel");
}
