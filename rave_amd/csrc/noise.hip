// NoiseGeneratorV2's filter stage (rave/blocks.py:281-291) after its conv
// stack: mod_sigmoid (rave/core.py:66-67) -> amp_to_impulse_response
// (rave/core.py:95-116) -> fft_convolve (rave/core.py:119-129) with the uniform
// noise, written band-major for the PQMF synthesis epilogue to add.
//
// The FFTs are tiny (irfft of noise_bands bins into fs = 2*(noise_bands-1)
// taps; a 2*target-point circular product whose kept half is a causal linear
// convolution), so each thread evaluates them directly for one
// (b, frame, band) cell: the impulse response in closed form from a cosine
// table in LDS, then the target-sample causal convolution in registers.
#include "common.h"

namespace rave {

constexpr int kNoiseThreads = 128;

template <int NB, int TARGET>
__global__ __launch_bounds__(kNoiseThreads) void noise_synth_kernel(rave_noise_args a) {
    constexpr int FS = 2 * (NB - 1);
    static_assert(TARGET >= FS, "amp_to_impulse_response pads to target_size >= fs");
    __shared__ float ctab[NB * FS];      // cos(2 pi k n / fs)
    __shared__ float win[FS];            // periodic Hann (torch.hann_window(fs))
    for (int i = threadIdx.x; i < NB * FS; i += kNoiseThreads) {
        const int k = i / FS, n = i - k * FS;
        ctab[i] = cospif((float)((2 * k * n) % (2 * FS)) / (float)FS);
    }
    for (int i = threadIdx.x; i < FS; i += kNoiseThreads)
        win[i] = 0.5f - 0.5f * cospif(2.0f * (float)i / (float)FS);
    __syncthreads();

    const int f = blockIdx.x * kNoiseThreads + threadIdx.x;
    const int j = blockIdx.y;
    const int b = blockIdx.z;
    if (f >= a.frames) return;

    // mod_sigmoid(x - 5) = 2 * sigmoid(x - 5)^2.3 + 1e-7
    float A[NB];
    const float* ap = a.amp + (int64_t)b * a.a_sb + (int64_t)(j * NB) * a.a_sc + f;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        const float s = 1.0f / (1.0f + expf(-(ap[(int64_t)k * a.a_sc] - 5.0f)));
        A[k] = 2.0f * powf(s, 2.3f) + 1e-7f;
    }
    // irfft (imaginary parts zero): ir[n] = (A0 + (-1)^n A_last + 2 sum_k A_k cos) / fs
    float ir[FS];
#pragma unroll
    for (int n = 0; n < FS; ++n) {
        float acc = 0.f;
#pragma unroll
        for (int k = 1; k < NB - 1; ++k) acc = fmaf(A[k], ctab[k * FS + n], acc);
        ir[n] = (A[0] + ((n & 1) ? -A[NB - 1] : A[NB - 1]) + 2.0f * acc) * (1.0f / FS);
    }
    // roll(fs/2) * hann, zero-pad to target, roll(-fs/2):
    //   h[n] = ir[n] * win[n + fs/2]                       n < fs/2
    //   h[n] = ir[n - target + fs] * win[n + fs/2 - target]  n >= target - fs/2
    float h[TARGET];
#pragma unroll
    for (int n = 0; n < TARGET; ++n) {
        if (n < FS / 2) h[n] = ir[n] * win[n + FS / 2];
        else if (n >= TARGET - FS / 2) h[n] = ir[n - TARGET + FS] * win[n + FS / 2 - TARGET];
        else h[n] = 0.f;
    }
    const float* up = a.u + (int64_t)b * a.u_sb + ((int64_t)f * a.n_band + j) * TARGET;
    float u[TARGET];
#pragma unroll
    for (int m = 0; m < TARGET; ++m) u[m] = up[m] * 2.0f - 1.0f;
    float* yp = a.y + (int64_t)b * a.y_sb + (int64_t)j * a.y_sc + (int64_t)f * TARGET;
#pragma unroll
    for (int i = 0; i < TARGET; ++i) {
        float acc = 0.f;
#pragma unroll
        for (int m = 0; m <= i; ++m) acc = fmaf(u[m], h[i - m], acc);
        yp[i] = acc;
    }
}

}  // namespace rave

using namespace rave;

extern "C" int rave_noise_synth(const rave_noise_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->amp && p->u && p->y, "noise_synth: null pointer");
    const rave_noise_args& a = *p;
    RAVE_CHECK_ARG(a.batch > 0 && a.frames > 0 && a.n_band > 0, "noise_synth: empty shape");
    RAVE_CHECK_ARG(a.target >= 2 * (a.noise_bands - 1), "noise_synth: target must be >= 2*(noise_bands-1)");
    dim3 grid(ceil_div(a.frames, kNoiseThreads), a.n_band, a.batch);
    if (a.noise_bands == 5 && a.target == 8)
        launch((noise_synth_kernel<5, 8>), grid, dim3(kNoiseThreads), 0, as_stream(stream), a);
    else if (a.noise_bands == 5 && a.target == 16)
        launch((noise_synth_kernel<5, 16>), grid, dim3(kNoiseThreads), 0, as_stream(stream), a);
    else if (a.noise_bands == 9 && a.target == 16)
        launch((noise_synth_kernel<9, 16>), grid, dim3(kNoiseThreads), 0, as_stream(stream), a);
    else {
        set_error("noise_synth: supported (noise_bands, target) are (5, 8), (5, 16), (9, 16)");
        return RAVE_ERR_UNSUPPORTED;
    }
    return launch_status("noise_synth_kernel");
}
