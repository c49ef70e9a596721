// AdaptiveInstanceNormalization, eval mode (rave/blocks.py:856-919): the
// nn~ style-transfer controls -- learn the target statistics (learn_y), learn
// the source statistics (learn_x), and transfer -- over the module's buffers
// kept resident on the device.
//
// One workgroup per (channel, batch) row: the row's mean and unbiased std are
// reduced in two passes (mean first, then squared deviations, as torch's
// x.std(-1) does), the running buffers are updated with the reference's
// incremental rule target += (source - target) / (num_updates + 1), and the
// transfer is applied with the reference's operation order.  The counter is
// bumped exactly once per call by the last workgroup to finish (ticket).
#include "common.h"

namespace rave {

constexpr int kAdaThreads = 256;

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kAdaThreads / 64; ++i) s += red[i];
    return s;
}

__global__ __launch_bounds__(kAdaThreads) void adain_kernel(rave_adain_args a) {
    __shared__ float red[kAdaThreads / 64];
    __shared__ float st[4];              // this row's mean_x, std_x, mean_y, std_y after the update
    const int c = blockIdx.x, b = blockIdx.y;
    const float* x = a.x + (int64_t)b * a.x_sb + (int64_t)c * a.x_sc;
    float* y = a.y + (int64_t)b * a.y_sb + (int64_t)c * a.y_sc;
    const int64_t plane = (int64_t)a.max_batch * a.channels;
    const int64_t row = (int64_t)(a.row0 + b) * a.channels + c;
    float* mean_x = a.stats + row;
    float* std_x = a.stats + plane + row;
    float* mean_y = a.stats + 2 * plane + row;
    float* std_y = a.stats + 3 * plane + row;
    float nx = a.counters[0], ny = a.counters[1];

    if (a.mode != 0) {
        float s = 0.f;
        for (int t = threadIdx.x; t < a.t_len; t += kAdaThreads) s += x[t];
        const float mean = block_sum(s, red) / (float)a.t_len;
        float ss = 0.f;
        for (int t = threadIdx.x; t < a.t_len; t += kAdaThreads) {
            const float d = x[t] - mean;
            ss = fmaf(d, d, ss);
        }
        const float sd = sqrtf(block_sum(ss, red) / (float)(a.t_len - 1));
        float* tm = a.mode == 1 ? mean_x : mean_y;
        float* ts = a.mode == 1 ? std_x : std_y;
        const float n = a.mode == 1 ? nx : ny;
        if (threadIdx.x == 0) {
            *tm = *tm + (mean - *tm) / (n + 1.0f);
            *ts = *ts + (sd - *ts) / (n + 1.0f);
        }
        if (a.mode == 1) nx += 1.0f;
    }
    const bool transfer = a.mode != 2 && nx != 0.f && ny != 0.f;
    if (threadIdx.x == 0) {   // same thread that updated: program order, broadcast through LDS
        st[0] = *mean_x; st[1] = *std_x; st[2] = *mean_y; st[3] = *std_y;
    }
    __syncthreads();
    if (transfer) {
        const float mx = st[0], sx = st[1] + 1e-5f, my = st[2], sy = st[3];
        for (int t = threadIdx.x; t < a.t_len; t += kAdaThreads) y[t] = (x[t] - mx) / sx * sy + my;
    } else if (y != x) {
        for (int t = threadIdx.x; t < a.t_len; t += kAdaThreads) y[t] = x[t];
    }
    if (a.mode != 0) {
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned total = gridDim.x * gridDim.y;
            if (atomicAdd(a.ticket, 1u) == total - 1) {
                a.counters[a.mode - 1] += 1.0f;
                atomicExch(a.ticket, 0u);
            }
        }
    }
}

}  // namespace rave

using namespace rave;

extern "C" int rave_adain(const rave_adain_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y && p->stats && p->counters, "adain: null pointer");
    const rave_adain_args& a = *p;
    RAVE_CHECK_ARG(a.batch > 0 && a.channels > 0 && a.t_len > 0, "adain: empty shape");
    RAVE_CHECK_ARG(a.mode >= 0 && a.mode <= 2, "adain: mode must be 0 (transfer), 1 (learn_x) or 2 (learn_y)");
    RAVE_CHECK_ARG(a.mode == 0 || a.ticket, "adain: learning modes need the ticket word");
    RAVE_CHECK_ARG(a.row0 >= 0 && a.row0 + a.batch <= a.max_batch,
                   "adain: batch exceeds the statistics buffers (cc.MAX_BATCH_SIZE rows)");
    launch(adain_kernel, dim3(a.channels, a.batch), dim3(kAdaThreads), 0, as_stream(stream), a);
    return launch_status("adain_kernel");
}
