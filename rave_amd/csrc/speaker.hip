// Edge kernels of the encode->decode path: the Resampler's polyphase FIR
// (rave/resampler.py:9-66) and SpeakerRAVE's attentive statistics pooling
// head (rave/CombinedRave.py:301-328).  Every one of them is a streaming,
// HBM-bound VALU kernel (a few FLOP per byte): coalesced row loads, LDS
// staging of the FIR window and taps, wave64 shuffle reductions.  No MFMA --
// nothing here is a dense contraction (the speaker encoder's convolutions run
// on rave_conv1d / rave_residual_unit).
#include <algorithm>

#include "common.h"

namespace rave {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kFirOutputs = 1024;          // outputs per FIR workgroup (4 per lane)
constexpr int kFirLdsFloats = 16384;       // 64 KB of window + taps

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Sum of three values over the workgroup; every thread gets the totals.
__device__ __forceinline__ void block_sum3(float& a, float& b, float& c, float* red) {
    a = wave_sum(a);
    b = wave_sum(b);
    c = wave_sum(c);
    const int w = threadIdx.x >> 6;
    __syncthreads();                           // red may still be read by a previous call
    if ((threadIdx.x & 63) == 0) {
        red[w] = a;
        red[kWaves + w] = b;
        red[2 * kWaves + w] = c;
    }
    __syncthreads();
    a = b = c = 0.f;
#pragma unroll
    for (int i = 0; i < kWaves; ++i) {         // fixed order: bitwise reproducible
        a += red[i];
        b += red[kWaves + i];
        c += red[2 * kWaves + i];
    }
}

__device__ __forceinline__ float block_max(float v, float* red) {
    v = wave_max(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float m = red[0];
#pragma unroll
    for (int i = 1; i < kWaves; ++i) m = fmaxf(m, red[i]);
    return m;
}

__device__ __forceinline__ float act_read(float v, int act, float slope) {
    return (act == RAVE_ACT_LEAKY && v < 0.f) ? v * slope : v;
}

// ------------------------------------------------------------------ FIR
// One workgroup: `frames` consecutive output frames (all phases) of one row.
// The input window [t0*stride - pad_left, ...) and the taps are staged in LDS
// (zero outside [0, t_in)); lane o computes output (t0 + o / phases, o % phases),
// so the stores of a workgroup are one contiguous run of the interleaved row.
__global__ __launch_bounds__(kThreads) void fir_kernel(rave_fir_args a, int frames) {
    extern __shared__ float lds[];
    const int P = a.phases, K = a.taps, S = a.stride;
    const int b = blockIdx.y;
    const int t0 = blockIdx.x * frames;
    const int nf = min(frames, a.t_out - t0);
    const int win = (nf - 1) * S + K;
    float* h = lds;
    float* xw = lds + P * K;
    for (int i = threadIdx.x; i < P * K; i += kThreads) h[i] = a.h[i];
    const float* xr = a.x + (int64_t)b * a.x_sb;
    const int64_t base = (int64_t)t0 * S - a.pad_left;
    for (int i = threadIdx.x; i < win; i += kThreads) {
        const int64_t g = base + i;
        xw[i] = (g >= 0 && g < a.t_in) ? xr[g] : 0.f;
    }
    __syncthreads();
    float* yr = a.y + (int64_t)b * a.y_sb + (int64_t)t0 * P;
    for (int o = threadIdx.x; o < nf * P; o += kThreads) {
        const int t = o / P, p = o - t * P;
        const float* hp = h + p * K;
        const float* xp = xw + t * S;
        float acc = 0.f;
        for (int k = 0; k < K; ++k) acc = fmaf(hp[k], xp[k], acc);
        yr[o] = acc;
    }
}

// ------------------------------------------------------------------ row statistics
__global__ __launch_bounds__(kThreads) void row_stats_kernel(rave_row_stats_args a) {
    __shared__ float red[3 * kWaves];
    const int c = blockIdx.x, b = blockIdx.y;
    const float* xr = a.x + (int64_t)b * a.x_sb + (int64_t)c * a.x_sc;
    float s = 0.f, u0 = 0.f, u1 = 0.f;
    for (int t = threadIdx.x; t < a.t_len; t += kThreads) s += act_read(xr[t], a.act, a.leaky_slope);
    block_sum3(s, u0, u1, red);
    const float mean = s / (float)a.t_len;
    float q = 0.f;
    u0 = u1 = 0.f;
    for (int t = threadIdx.x; t < a.t_len; t += kThreads) {     // second pass: centred squares
        const float d = act_read(xr[t], a.act, a.leaky_slope) - mean;
        q = fmaf(d, d, q);
    }
    block_sum3(q, u0, u1, red);
    if (threadIdx.x == 0) {
        const float var = q / (float)(a.t_len - 1);            // unbiased, as torch.var
        float* yr = a.y + (int64_t)b * a.y_sb;
        yr[c] = mean;
        yr[a.channels + c] = sqrtf(fminf(fmaxf(var, a.var_min), a.var_max));
    }
}

// ------------------------------------------------------------------ attentive pooling
__global__ __launch_bounds__(kThreads) void attn_pool_kernel(rave_attn_pool_args a) {
    __shared__ float red[3 * kWaves];
    const int c = blockIdx.x, b = blockIdx.y;
    const float* xr = a.x + (int64_t)b * a.x_sb + (int64_t)c * a.x_sc;
    const float* lr = a.logits + (int64_t)b * a.l_sb + (int64_t)c * a.l_sc;
    float m = -INFINITY;
    for (int t = threadIdx.x; t < a.t_len; t += kThreads) m = fmaxf(m, lr[t]);
    m = block_max(m, red);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int t = threadIdx.x; t < a.t_len; t += kThreads) {
        const float e = __expf(lr[t] - m);
        const float v = act_read(xr[t], a.act, a.leaky_slope);
        s0 += e;
        s1 = fmaf(v, e, s1);
        s2 = fmaf(v * v, e, s2);
    }
    block_sum3(s0, s1, s2, red);
    if (threadIdx.x == 0) {
        const float inv = 1.f / s0;
        const float mu = s1 * inv;
        const float var = s2 * inv - mu * mu;
        float* yr = a.y + (int64_t)b * a.y_sb;
        yr[c] = mu;
        yr[a.channels + c] = sqrtf(fminf(fmaxf(var, a.var_min), a.var_max));
    }
}

// ------------------------------------------------------------------ linear
// One wave per output: lanes stride the input (coalesced weight row reads).
__global__ __launch_bounds__(kThreads) void linear_kernel(rave_linear_args a) {
    const int o = blockIdx.x * kWaves + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.y;
    if (o >= a.n_out) return;
    const float* w = a.w + (int64_t)o * a.n_in;
    const float* x = a.x + (int64_t)b * a.x_sb;
    float acc = 0.f;
    for (int i = lane; i < a.n_in; i += 64) acc = fmaf(w[i], x[i], acc);
    acc = wave_sum(acc);
    if (lane == 0) a.y[(int64_t)b * a.y_sb + o] = acc + (a.bias ? a.bias[o] : 0.f);
}

// ------------------------------------------------------------------ max pool
__global__ __launch_bounds__(kThreads) void maxpool_kernel(rave_maxpool_args a) {
    const int b = blockIdx.y;
    const int64_t total = (int64_t)a.channels * a.t_out;
    for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kThreads) {
        const int c = (int)(i / a.t_out);
        const int t = (int)(i - (int64_t)c * a.t_out);
        const float* xr = a.x + (int64_t)b * a.x_sb + (int64_t)c * a.x_sc + (int64_t)t * a.kernel;
        float m = xr[0];
        for (int j = 1; j < a.kernel; ++j) m = fmaxf(m, xr[j]);
        a.y[(int64_t)b * a.y_sb + (int64_t)c * a.y_sc + t] = m;
    }
}

}  // namespace
}  // namespace rave

using namespace rave;

extern "C" int rave_fir(const rave_fir_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y && p->h, "fir: null pointer");
    RAVE_CHECK_ARG(p->batch > 0 && p->t_in > 0 && p->t_out > 0 && p->phases > 0 && p->taps > 0 && p->stride > 0,
                   "fir: empty shape");
    RAVE_CHECK_ARG(p->pad_left >= 0, "fir: negative pad_left");
    RAVE_CHECK_ARG(p->taps <= 1024 && p->phases * p->taps <= 4096, "fir: too many taps");
    RAVE_CHECK_ARG(p->stride <= 64, "fir: stride above 64");
    RAVE_CHECK_ARG(p->y_sb >= (int64_t)p->t_out * p->phases, "fir: output rows overlap");
    int frames = std::max(1, kFirOutputs / p->phases);
    // window + taps must fit the LDS budget
    while (frames > 1 && (frames - 1) * p->stride + p->taps + p->phases * p->taps > kFirLdsFloats) frames /= 2;
    frames = std::min(frames, p->t_out);
    const size_t lds = sizeof(float) * ((size_t)(frames - 1) * p->stride + p->taps + (size_t)p->phases * p->taps);
    RAVE_CHECK_ARG(lds <= sizeof(float) * kFirLdsFloats, "fir: window does not fit LDS");
    launch(fir_kernel, dim3(ceil_div(p->t_out, frames), p->batch), dim3(kThreads), (uint32_t)lds,
           as_stream(stream), *p, frames);
    return launch_status("fir_kernel");
}

static bool act_ok(int act) { return act == RAVE_ACT_NONE || act == RAVE_ACT_LEAKY; }

extern "C" int rave_row_stats(const rave_row_stats_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y, "row_stats: null pointer");
    RAVE_CHECK_ARG(p->batch > 0 && p->channels > 0 && p->t_len > 0, "row_stats: empty shape");
    RAVE_CHECK_ARG(act_ok(p->act), "row_stats: act must be none or leaky");
    RAVE_CHECK_ARG(p->y_sb >= 2 * (int64_t)p->channels, "row_stats: output rows overlap");
    launch(row_stats_kernel, dim3(p->channels, p->batch), dim3(kThreads), 0, as_stream(stream), *p);
    return launch_status("row_stats_kernel");
}

extern "C" int rave_attn_pool(const rave_attn_pool_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->logits && p->y, "attn_pool: null pointer");
    RAVE_CHECK_ARG(p->batch > 0 && p->channels > 0 && p->t_len > 0, "attn_pool: empty shape");
    RAVE_CHECK_ARG(act_ok(p->act), "attn_pool: act must be none or leaky");
    RAVE_CHECK_ARG(p->y_sb >= 2 * (int64_t)p->channels, "attn_pool: output rows overlap");
    launch(attn_pool_kernel, dim3(p->channels, p->batch), dim3(kThreads), 0, as_stream(stream), *p);
    return launch_status("attn_pool_kernel");
}

extern "C" int rave_linear(const rave_linear_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->w && p->y, "linear: null pointer");
    RAVE_CHECK_ARG(p->batch > 0 && p->n_in > 0 && p->n_out > 0, "linear: empty shape");
    launch(linear_kernel, dim3(ceil_div(p->n_out, kWaves), p->batch), dim3(kThreads), 0, as_stream(stream), *p);
    return launch_status("linear_kernel");
}

extern "C" int rave_maxpool(const rave_maxpool_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y, "maxpool: null pointer");
    RAVE_CHECK_ARG(p->batch > 0 && p->channels > 0 && p->t_out > 0 && p->kernel > 0, "maxpool: empty shape");
    const int64_t total = (int64_t)p->channels * p->t_out;
    const int blocks = (int)std::min<int64_t>(ceil_div64(total, kThreads), 1024);
    launch(maxpool_kernel, dim3(blocks, p->batch), dim3(kThreads), 0, as_stream(stream), *p);
    return launch_status("maxpool_kernel");
}
