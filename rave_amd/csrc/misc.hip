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
// One launch per quantizer layer q over a (frame tiles x code splits) grid, so
// the chip fills at any batch (the layers are sequential; a frame's argmax
// spans every split).  Launch q, per frame tile:
//   1. (q >= 1) reduce layer q-1's per-split candidates -> idx[q-1] (split 0
//      stores it), and form r_q = r_{q-1} - E_{q-1}[idx] in LDS (the
//      reference's fp32 residual update; split 0 stores r_q for launch q+1);
//   2. score this split's kRvqCS codes against the tile: d = |e|^2 - 2 r.e
//      (argmin == the reference's argmax of -(|r|^2 - 2 r.e + |e|^2)), the
//      r.e dots as one 32x32 fp32 MFMA block per wave (K = DIM), |e|^2 on the
//      VALU; argmin per frame (ties -> smaller index, like torch.max) ->
//      best[q & 1][split][frame].
// A last launch (q = n_q) only does step 1.  Scratch (rave_rvq_workspace):
// resid[2][frames][DIM] | best_d[2][S][frames] | best_i[2][S][frames]; the
// double buffers make launch q's reads and writes disjoint.
constexpr int kRvqFT = 32;                   // frames per tile (MFMA columns)
constexpr int kRvqCS = 64;                   // codes per split (32 MFMA rows per wave)
constexpr int kRvqThreads = 128;
typedef float rvq_f32x16 __attribute__((ext_vector_type(16)));

struct RvqLayer {
    int q;            // layer scored by this launch (n_q: final reduction only)
    int n_frames;
    int splits;
};

__device__ inline int64_t rvq_zoff(const rave_rvq_args& a, int g, int d) {
    int b = g / a.t_len, t = g - b * a.t_len;
    return (int64_t)b * a.z_sb + (int64_t)d * a.z_sc + t;
}

template <int DIM>
__global__ __launch_bounds__(kRvqThreads) void rvq_encode_kernel(rave_rvq_args a, RvqLayer L) {
    __shared__ __attribute__((aligned(16))) float xs[kRvqFT][DIM + 4];   // +4: conflict-free b128 rows
    __shared__ __attribute__((aligned(16))) float es[kRvqCS][DIM + 4];
    __shared__ float nrm_s[kRvqCS];
    __shared__ float red_d[kRvqThreads / 64][kRvqFT];
    __shared__ int red_i[kRvqThreads / 64][kRvqFT];
    __shared__ int sel[kRvqFT];
    const int F = L.n_frames, S = L.splits, q = L.q;
    const int f0 = blockIdx.x * kRvqFT;
    const int split = blockIdx.y;
    const int tid = threadIdx.x;
    // this split's codewords (contiguous rows): coalesced loads issued first so
    // they overlap the index reduction and residual update below
    constexpr int EPER = kRvqCS * DIM / 4 / kRvqThreads;
    float4 ev4[EPER];
    if (q < a.n_q) {
        const float4* src = reinterpret_cast<const float4*>(
            a.codebooks + ((int64_t)q * a.codebook_size + (int64_t)split * kRvqCS) * DIM);
        const int rows = min(kRvqCS, a.codebook_size - split * kRvqCS);
#pragma unroll
        for (int u = 0; u < EPER; ++u) {
            int i = tid + u * kRvqThreads;               // float4 index in the block
            ev4[u] = (i / (DIM / 4) < rows) ? src[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    float* resid = a.work;
    float* best_d = a.work + (int64_t)2 * F * DIM;
    int* best_i = reinterpret_cast<int*>(best_d + (int64_t)2 * S * F);

    if (q >= 1) {
        // layer q-1's index per frame: the lexicographic min of (d, index) over
        // the splits (order-free, so equal to the first maximum of torch.max);
        // 8 lanes per frame, all candidate loads issued before the compares
        {
            constexpr int LPF = kRvqThreads / kRvqFT;          // lanes per frame
            const int f = tid / LPF, j = tid % LPF;
            const int g = f0 + f;
            const float* bd = best_d + (int64_t)((q - 1) & 1) * S * F;
            const int* bi = best_i + (int64_t)((q - 1) & 1) * S * F;
            float d0 = FLT_MAX;
            int i0 = 0x7fffffff;
            if (g < F) {
                for (int s0 = j; s0 < S; s0 += 8 * LPF) {
                    float dd[8];
                    int ii[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        int s = s0 + LPF * u;
                        dd[u] = s < S ? bd[(int64_t)s * F + g] : FLT_MAX;
                        ii[u] = s < S ? bi[(int64_t)s * F + g] : 0x7fffffff;
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (dd[u] < d0 || (dd[u] == d0 && ii[u] < i0)) { d0 = dd[u]; i0 = ii[u]; }
                }
            }
#pragma unroll
            for (int off = LPF / 2; off > 0; off >>= 1) {
                float od = __shfl_xor(d0, off);
                int oi = __shfl_xor(i0, off);
                if (od < d0 || (od == d0 && oi < i0)) { d0 = od; i0 = oi; }
            }
            if (j == 0) {
                if (g < F && split == 0) {
                    int b = g / a.t_len, t = g - b * a.t_len;
                    a.idx[(int64_t)b * a.i_sb + (int64_t)(q - 1) * a.i_sq + t] = (int64_t)i0;
                }
                sel[f] = g < F ? i0 : 0;
            }
        }
        if (q == a.n_q) return;              // final launch: indices only (grid y == 1)
        __syncthreads();
        const float* E = a.codebooks + (int64_t)(q - 1) * a.codebook_size * DIM;
        const float* rp = resid + (int64_t)((q - 1) & 1) * F * DIM;
        float* rn = resid + (int64_t)(q & 1) * F * DIM;
        constexpr int PER = kRvqFT * DIM / kRvqThreads;
        float rv[PER], ev[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {      // every load before any store
            int i = tid + u * kRvqThreads;
            int f = i / DIM, d = i - f * DIM;
            int g = f0 + f;
            rv[u] = 0.f;
            ev[u] = 0.f;
            if (g < F) {
                rv[u] = (q == 1) ? a.z[rvq_zoff(a, g, d)] : rp[(int64_t)g * DIM + d];
                ev[u] = E[(int64_t)sel[f] * DIM + d];
            }
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            int i = tid + u * kRvqThreads;
            int f = i / DIM, d = i - f * DIM;
            int g = f0 + f;
            float v = rv[u] - ev[u];
            if (g < F && split == 0 && q + 1 < a.n_q) rn[(int64_t)g * DIM + d] = v;
            xs[f][d] = (g < F) ? v : 0.f;
        }
    } else {
        constexpr int PER = kRvqFT * DIM / kRvqThreads;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            int i = tid + u * kRvqThreads;
            int f = i / DIM, d = i - f * DIM;
            int g = f0 + f;
            xs[f][d] = (g < F) ? a.z[rvq_zoff(a, g, d)] : 0.f;
        }
    }
#pragma unroll
    for (int u = 0; u < EPER; ++u) {
        int i = tid + u * kRvqThreads;
        int r = i / (DIM / 4), c4 = i - r * (DIM / 4);
        *reinterpret_cast<float4*>(&es[r][c4 * 4]) = ev4[u];
    }
    __syncthreads();

    // dots on the fp32 MFMA: wave w scores codes [32w, 32w+32) of the split (A =
    // codewords, rows) against the 32 frames (B = residuals, columns); lane half
    // h takes dimensions [h*DIM/2, (h+1)*DIM/2), so each lane streams one
    // contiguous row segment by 16-byte LDS reads
    const int lane = tid & 63, w = tid >> 6, l32 = lane & 31, h = lane >> 5;
    rvq_f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const float* ea = &es[w * 32 + l32][h * (DIM / 2)];
    const float* xb = &xs[l32][h * (DIM / 2)];
    float nrm = 0.f;                           // |e|^2 of this lane's half row, in order
#pragma unroll
    for (int s4 = 0; s4 < DIM / 8; ++s4) {
        const float4 e = *reinterpret_cast<const float4*>(ea + 4 * s4);
        const float4 x = *reinterpret_cast<const float4*>(xb + 4 * s4);
        nrm = fmaf(e.x, e.x, nrm); nrm = fmaf(e.y, e.y, nrm);
        nrm = fmaf(e.z, e.z, nrm); nrm = fmaf(e.w, e.w, nrm);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(e.x, x.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(e.y, x.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(e.z, x.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(e.w, x.w, acc, 0, 0, 0);
    }
    {
        const float other = __shfl_xor(nrm, 32);
        if (h == 0) nrm_s[w * 32 + l32] = nrm + other;     // low half + high half
    }
    __syncthreads();                           // nrm_s
    // d = |e|^2 - 2 r.e; per frame (column l32) the lexicographic min of
    // (d, code) -- order-free, so ties resolve to the smallest code
    float d0 = FLT_MAX;
    int i0 = 0x7fffffff;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = w * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;    // code within the split
        const int k = split * kRvqCS + m;
        if (k < a.codebook_size) {
            float dv = nrm_s[m] - 2.f * acc[r];
            if (dv < d0 || (dv == d0 && k < i0)) { d0 = dv; i0 = k; }
        }
    }
    {
        float od = __shfl_xor(d0, 32);
        int oi = __shfl_xor(i0, 32);
        if (od < d0 || (od == d0 && oi < i0)) { d0 = od; i0 = oi; }
    }
    if (h == 0) { red_d[w][l32] = d0; red_i[w][l32] = i0; }
    __syncthreads();
    if (tid < kRvqFT) {
        const int g = f0 + tid;
        float dd = red_d[0][tid];
        int ii = red_i[0][tid];
#pragma unroll
        for (int ww = 1; ww < kRvqThreads / 64; ++ww) {
            float od = red_d[ww][tid];
            int oi = red_i[ww][tid];
            if (od < dd || (od == dd && oi < ii)) { dd = od; ii = oi; }
        }
        if (g < F) {
            best_d[(int64_t)(q & 1) * S * F + (int64_t)split * F + g] = dd;
            best_i[(int64_t)(q & 1) * S * F + (int64_t)split * F + g] = ii;
        }
    }
}

static int rvq_splits(const rave_rvq_args* p) { return ceil_div(p->codebook_size, kRvqCS); }

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

// Counter-based uniform draw: a splitmix64 finaliser of (seed, index), top 24
// bits -> [0, 1).  Stateless, so any launch geometry gives the same values.
__global__ __launch_bounds__(256) void fill_uniform_kernel(float* y, int64_t n, uint64_t seed, float lo,
                                                           float scale) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        uint64_t z = seed + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        y[i] = lo + scale * ((float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f));
    }
}

}  // namespace rave

using namespace rave;

extern "C" int rave_fill_uniform(float* y, int64_t n, uint64_t seed, float lo, float hi, void* stream) {
    RAVE_CHECK_ARG(y && n >= 0, "fill_uniform: bad arguments");
    if (n == 0) return RAVE_OK;
    const int blocks = (int)std::min<int64_t>(ceil_div64(n, 256), 2048);
    launch(fill_uniform_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), y, n, seed, lo, hi - lo);
    return launch_status("fill_uniform_kernel");
}

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

extern "C" int64_t rave_rvq_workspace(const rave_rvq_args* p) {
    RAVE_CHECK_ARG(p && p->n_q > 0 && p->codebook_size > 0 && p->dim > 0 && p->batch >= 0 && p->t_len >= 0,
                   "rvq_workspace: bad shape");
    const int64_t F = (int64_t)p->batch * p->t_len;
    return 2 * F * p->dim + 4 * (int64_t)rvq_splits(p) * F;
}

extern "C" int rave_rvq_encode(const rave_rvq_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->z && p->idx && p->codebooks && p->work, "rvq_encode: null pointer");
    RAVE_CHECK_ARG(p->n_q > 0 && p->codebook_size > 0 && p->batch > 0 && p->t_len > 0,
                   "rvq_encode: empty shape");
    RAVE_CHECK_ARG((int64_t)p->batch * p->t_len <= (1 << 30), "rvq_encode: too many frames");
    const int F = p->batch * p->t_len;
    const int S = rvq_splits(p);
    auto kern = rvq_encode_kernel<128>;
    switch (p->dim) {
        case 128: kern = rvq_encode_kernel<128>; break;
        case 64: kern = rvq_encode_kernel<64>; break;
        default: set_error("rvq_encode: dim must be 64 or 128"); return RAVE_ERR_UNSUPPORTED;
    }
    const int tiles = ceil_div(F, kRvqFT);
    // the op's timing (rave_plan_profile) spans all launches: launch() records the
    // start event on the first and re-records the stop event on each
    for (int q = 0; q <= p->n_q; ++q) {
        launch(kern, dim3(tiles, q == p->n_q ? 1 : S), dim3(kRvqThreads), 0, as_stream(stream), *p,
               RvqLayer{q, F, S});
        int rc = launch_status("rvq_encode_kernel");
        if (rc != RAVE_OK) return rc;
    }
    return RAVE_OK;
}

extern "C" int rave_rvq_decode(const rave_rvq_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->y && p->idx && p->codebooks, "rvq_decode: null pointer");
    RAVE_CHECK_ARG(p->n_q > 0 && p->dim > 0 && p->batch > 0 && p->t_len > 0, "rvq_decode: empty shape");
    int64_t total = (int64_t)p->dim * p->t_len;
    int blocks = (int)std::min<int64_t>(ceil_div64(total, 256), 1024);
    launch(rvq_decode_kernel, dim3(blocks, p->batch), dim3(256), 0, as_stream(stream), *p);
    return launch_status("rvq_decode_kernel");
}
