// Small kernels of the path: speaker-channel fill (RAVE.encode concat,
// rave/model.py:618-620), streaming history shift (the cache update of
// cached_conv's CachedPadding1d), and residual vector quantization
// (rave/quantization.py:131-140, 239-249, 302-318).
#include "common.h"
#include "shift_batch.h"

#include <algorithm>
#include <cfloat>

namespace rave {

__global__ void fill_channels_kernel(rave_fill_args a) {
    const int64_t total = (int64_t)a.channels * a.t_len;
    const int b = blockIdx.y;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        int c = (int)(i / a.t_len);
        int t = (int)(i - (int64_t)c * a.t_len);
        a.y[(int64_t)b * a.y_sb + (int64_t)c * a.y_sc + t] = a.values[c];
    }
}

__global__ void copy_kernel(rave_copy_args a) {
    const int64_t total = (int64_t)a.channels * a.t_len;
    const int b = blockIdx.y;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        int c = (int)(i / a.t_len);
        int t = (int)(i - (int64_t)c * a.t_len);
        a.y[(int64_t)b * a.y_sb + (int64_t)c * a.y_sc + t] = a.x[(int64_t)b * a.x_sb + (int64_t)c * a.x_sc + t];
    }
}

// One thread per (b, c) row; ascending copy is safe because the destination
// [0, hist) never overtakes the source [t_new, t_new + hist) (t_new >= 1).
// Up to kShiftBatch history buffers per launch (a streaming plan shifts one
// buffer per conv input after every block; one launch instead of ~20).  One
// wave per (buffer, row): lanes move 64 consecutive columns per iteration in
// increasing order, so the in-place forward move never overwrites a column a
// later iteration still reads (t_new >= 1: reads run ahead of writes).
__global__ __launch_bounds__(256) void shift_history_kernel(ShiftBatch sb) {
    const rave_shift_args& a = sb.a[blockIdx.y];
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= a.batch * a.channels) return;
    const int lane = threadIdx.x & 63;
    const int b = row / a.channels, c = row - b * a.channels;
    float* r = a.buf + (int64_t)b * a.sb + (int64_t)c * a.sc;
    for (int i = lane; i < a.hist; i += 64) r[i] = r[a.t_new + i];
}

int shift_history_batch(const rave_shift_args* const* ops, int n, hipStream_t stream) {
    if (n < 1 || n > kShiftBatch) {
        set_error("shift_history: batch of " + std::to_string(n) + " buffers");
        return RAVE_ERR_ARG;
    }
    ShiftBatch sb{};
    int m = 0, max_rows = 0;
    for (int i = 0; i < n; ++i) {
        const rave_shift_args* p = ops[i];
        RAVE_CHECK_ARG(p && p->buf, "shift_history: null pointer");
        RAVE_CHECK_ARG(p->t_new >= 1 && p->hist >= 0 && p->batch >= 0 && p->channels >= 0,
                       "shift_history: bad sizes");
        if (p->hist == 0 || p->batch * p->channels == 0) continue;
        sb.a[m++] = *p;
        max_rows = std::max(max_rows, p->batch * p->channels);
    }
    if (m == 0) return RAVE_OK;
    launch(shift_history_kernel, dim3(ceil_div(max_rows, 4), m), dim3(256), 0, stream, sb);
    return launch_status("shift_history_kernel");
}

// ------------------------------------------------------------------ RVQ encode
// One workgroup per kFT frames, all quantizer layers in sequence (the residual
// never leaves LDS).  Each thread scores kCodes codebook rows against every
// frame of the tile: d = |e|^2 - 2 x.e (argmin == the reference's argmax of
// -(|x|^2 - 2 x.e + |e|^2)); ties resolve to the smallest index like
// torch.max.  The residual update r -= E[idx] is the reference's fp32 order.
constexpr int kFT = 8;
constexpr int kRvqThreads = 256;

template <int DIM>
__global__ __launch_bounds__(kRvqThreads) void rvq_encode_kernel(rave_rvq_args a, int n_frames) {
    __shared__ __attribute__((aligned(16))) float xs[kFT][DIM];
    __shared__ float best_d[kRvqThreads / 64][kFT];
    __shared__ int best_i[kRvqThreads / 64][kFT];
    __shared__ int sel[kFT];

    const int f0 = blockIdx.x * kFT;
    const int tid = threadIdx.x;
    // load the residual tile (frame f -> (b, t))
    for (int i = tid; i < kFT * DIM; i += kRvqThreads) {
        int f = i / DIM, d = i - f * DIM;
        int g = f0 + f;
        float v = 0.f;
        if (g < n_frames) {
            int b = g / a.t_len, t = g - b * a.t_len;
            v = a.z[(int64_t)b * a.z_sb + (int64_t)d * a.z_sc + t];
        }
        xs[f][d] = v;
    }
    __syncthreads();

    const int K = a.codebook_size;
    for (int q = 0; q < a.n_q; ++q) {
        const float* E = a.codebooks + (int64_t)q * K * DIM;
        float bd[kFT];
        int bi[kFT];
#pragma unroll
        for (int f = 0; f < kFT; ++f) { bd[f] = FLT_MAX; bi[f] = 0x7fffffff; }
        for (int k = tid; k < K; k += kRvqThreads) {
            const float4* e4 = reinterpret_cast<const float4*>(E + (int64_t)k * DIM);
            float dot[kFT];
#pragma unroll
            for (int f = 0; f < kFT; ++f) dot[f] = 0.f;
            float nrm = 0.f;
#pragma unroll 4
            for (int d4 = 0; d4 < DIM / 4; ++d4) {
                float4 e = e4[d4];
                nrm = fmaf(e.x, e.x, nrm); nrm = fmaf(e.y, e.y, nrm);
                nrm = fmaf(e.z, e.z, nrm); nrm = fmaf(e.w, e.w, nrm);
#pragma unroll
                for (int f = 0; f < kFT; ++f) {
                    float4 x = *reinterpret_cast<const float4*>(&xs[f][d4 * 4]);
                    dot[f] = fmaf(x.x, e.x, dot[f]); dot[f] = fmaf(x.y, e.y, dot[f]);
                    dot[f] = fmaf(x.z, e.z, dot[f]); dot[f] = fmaf(x.w, e.w, dot[f]);
                }
            }
#pragma unroll
            for (int f = 0; f < kFT; ++f) {
                float dv = nrm - 2.f * dot[f];
                if (dv < bd[f]) { bd[f] = dv; bi[f] = k; }   // k ascending per thread
            }
        }
        // wave reduction (min distance, then min index)
#pragma unroll
        for (int f = 0; f < kFT; ++f) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                float od = __shfl_xor(bd[f], off);
                int oi = __shfl_xor(bi[f], off);
                if (od < bd[f] || (od == bd[f] && oi < bi[f])) { bd[f] = od; bi[f] = oi; }
            }
        }
        const int w = tid >> 6;
        if ((tid & 63) == 0) {
#pragma unroll
            for (int f = 0; f < kFT; ++f) { best_d[w][f] = bd[f]; best_i[w][f] = bi[f]; }
        }
        __syncthreads();
        if (tid < kFT) {
            float d0 = best_d[0][tid];
            int i0 = best_i[0][tid];
            for (int ww = 1; ww < kRvqThreads / 64; ++ww) {
                float dd = best_d[ww][tid];
                int ii = best_i[ww][tid];
                if (dd < d0 || (dd == d0 && ii < i0)) { d0 = dd; i0 = ii; }
            }
            sel[tid] = i0;
            int g = f0 + tid;
            if (g < n_frames) {
                int b = g / a.t_len, t = g - b * a.t_len;
                a.idx[(int64_t)b * a.i_sb + (int64_t)q * a.i_sq + t] = (int64_t)i0;
            }
        }
        __syncthreads();
        for (int i = tid; i < kFT * DIM; i += kRvqThreads) {
            int f = i / DIM, d = i - f * DIM;
            xs[f][d] = xs[f][d] - E[(int64_t)sel[f] * DIM + d];
        }
        __syncthreads();
    }
}

__global__ void rvq_decode_kernel(rave_rvq_args a) {
    const int b = blockIdx.y;
    const int64_t total = (int64_t)a.dim * a.t_len;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        int d = (int)(i / a.t_len);
        int t = (int)(i - (int64_t)d * a.t_len);
        float acc = 0.f;   // quantized_out = 0.0; += layer.decode(...) in order
        for (int q = 0; q < a.n_q; ++q) {
            int64_t k = a.idx[(int64_t)b * a.i_sb + (int64_t)q * a.i_sq + t];
            k = k < 0 ? 0 : (k >= a.codebook_size ? a.codebook_size - 1 : k);  // DiscreteScriptedRAVE clamp
            acc = acc + a.codebooks[((int64_t)q * a.codebook_size + k) * a.dim + d];
        }
        a.y[(int64_t)b * a.y_sb + (int64_t)d * a.y_sc + t] = acc;
    }
}

}  // namespace rave

using namespace rave;

extern "C" int rave_fill_channels(const rave_fill_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->y && p->values, "fill_channels: null pointer");
    RAVE_CHECK_ARG(p->batch > 0 && p->channels > 0 && p->t_len > 0, "fill_channels: empty shape");
    int64_t total = (int64_t)p->channels * p->t_len;
    int blocks = (int)std::min<int64_t>(ceil_div64(total, 256), 1024);
    launch(fill_channels_kernel, dim3(blocks, p->batch), dim3(256), 0, as_stream(stream), *p);
    return launch_status("fill_channels_kernel");
}

extern "C" int rave_copy(const rave_copy_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y, "copy: null pointer");
    RAVE_CHECK_ARG(p->batch > 0 && p->channels > 0 && p->t_len > 0, "copy: empty shape");
    int64_t total = (int64_t)p->channels * p->t_len;
    int blocks = (int)std::min<int64_t>(ceil_div64(total, 256), 1024);
    launch(copy_kernel, dim3(blocks, p->batch), dim3(256), 0, as_stream(stream), *p);
    return launch_status("copy_kernel");
}

extern "C" int rave_shift_history(const rave_shift_args* p, void* stream) {
    return shift_history_batch(&p, 1, as_stream(stream));
}

extern "C" int rave_rvq_encode(const rave_rvq_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->z && p->idx && p->codebooks, "rvq_encode: null pointer");
    RAVE_CHECK_ARG(p->n_q > 0 && p->codebook_size > 0 && p->batch > 0 && p->t_len > 0,
                   "rvq_encode: empty shape");
    int n_frames = p->batch * p->t_len;
    dim3 grid(ceil_div(n_frames, kFT));
    switch (p->dim) {
        case 128: launch(rvq_encode_kernel<128>, grid, dim3(kRvqThreads), 0, as_stream(stream), *p, n_frames); break;
        case 64: launch(rvq_encode_kernel<64>, grid, dim3(kRvqThreads), 0, as_stream(stream), *p, n_frames); break;
        default: set_error("rvq_encode: dim must be 64 or 128"); return RAVE_ERR_UNSUPPORTED;
    }
    return launch_status("rvq_encode_kernel");
}

extern "C" int rave_rvq_decode(const rave_rvq_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->y && p->idx && p->codebooks, "rvq_decode: null pointer");
    RAVE_CHECK_ARG(p->n_q > 0 && p->dim > 0 && p->batch > 0 && p->t_len > 0, "rvq_decode: empty shape");
    int64_t total = (int64_t)p->dim * p->t_len;
    int blocks = (int)std::min<int64_t>(ceil_div64(total, 256), 1024);
    launch(rvq_decode_kernel, dim3(blocks, p->batch), dim3(256), 0, as_stream(stream), *p);
    return launch_status("rvq_decode_kernel");
}
