// Pieces shared by the exact-fp32 (conv1d.hip) and split-f16 (conv_split.hip)
// implicit-GEMM conv kernels: the kernel argument block, buffer descriptors,
// the ConvTranspose row mapping, the epilogue store and the split-K reduce.
#pragma once
#include "common.h"

#include <algorithm>

namespace rave {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));   // native vector (HIP float4 is a struct)
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kSplitTickets = RAVE_SPLITK_TICKETS;   // int32 words ahead of the split-K slabs
constexpr int kSplitTicketsUsable = RAVE_SPLITK_STATUS_WORD;   // tiles with a ticket (the last word is reserved)
constexpr int kMaxDil = 16;       // largest dilation of a 3-tap conv the kernels stage

struct ConvKArgs {
    const float* x; const float* w; const float* bias; const float* alpha; const float* res;
    float* y; float* partial;
    int64_t x_sb, x_sc, y_sb, y_sc, r_sb, r_sc;
    int c_in, M, d, pad_l, t_in, U, B;
    int nchunks, Mpad, XW;
    unsigned xw_magic;            // ceil(2^24 / XW): e / XW == (e * magic) >> 24 for e < 2^13
    int x_bytes, w_bytes;         // buffer-descriptor extents (per batch item / whole packed weight)
    int y_bytes, r_bytes, bias_rows;
#ifdef RAVE_STAMPS
    unsigned long long* stamps;   // diagnostic build only: 8 per workgroup
#endif
    int S, cps;                   // splits, chunks per split
    int transposed, R, out_shift, t_y, act;
    int split_row, pad_g1, q0;    // ConvT phase groups: rows < split_row use pad_l, others pad_g1;
                                  // q0 = phases in group 0 (= R - out_shift)
    float slope;
    const float* rscale;          // split path: per-GEMM-row scale 2^-(e_m+11)
    int MB;                       // split path: 32-row blocks of the packed weight
    int vec_y, vec_p;             // split path: 16-byte epilogue stores allowed (y/res, slabs)
    unsigned rl_magic;            // split path: ceil(2^32 / raw window row length)
    int x_vec;                    // split path: 16-byte window DMA allowed
    int* tickets;                 // split path: per-tile arrival counters (zero between calls)
    int gx, gy;                   // split path: column / row tiles per batch item (1-D grid)
    int inlaunch;                 // split path: the last-arriving K-split sums the slabs
};

// Buffer descriptor from wave-uniform inputs (guide T8/T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* p, int bytes) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint64_t u = ((uint64_t)hi << 32) | lo;
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0,
                                             __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// --------------------------------------------------------------------- epilogue
// ConvT row m -> (output channel, phase).  Rows [0, split_row) hold phases
// [0, q0) of every channel (rows up to the 64-aligned group-1 start are
// padding: co >= c_out), rows [split_row, M) phases [q0, R).
__device__ __forceinline__ void convt_row(const ConvKArgs& a, int m, int& co, int& q) {
    const int p = a.R - a.q0;            // phases in row group 1 (0: no group 1)
    if (m < a.split_row) {
        co = m / a.q0;
        q = m - co * a.q0;
    } else if (p > 0) {
        const int mm = m - a.split_row;
        co = mm / p;
        q = a.q0 + (mm - co * p);
    } else {                             // padding row past a single group: never stored
        co = a.bias_rows;
        q = 0;
    }
}

__device__ __forceinline__ void store_out(const ConvKArgs& a, int b, int m, int n, float v) {
    if (a.transposed) {
        int co, q;
        convt_row(a, m, co, q);
        const int t = n * a.R + q;
        if (t >= a.t_y || co >= a.bias_rows) return;    // bias_rows = c_out
        if (a.bias) v += a.bias[co];
        a.y[(int64_t)b * a.y_sb + (int64_t)co * a.y_sc + t] = v;
    } else {
        if (a.bias) v += a.bias[m];
        if (a.res) v += a.res[(int64_t)b * a.r_sb + (int64_t)m * a.r_sc + n];
        a.y[(int64_t)b * a.y_sb + (int64_t)m * a.y_sc + n] = v;
    }
}

// Sum the split-K slabs in split order, then the normal epilogue (the slabs
// already carry the split path's row scale).  A template so each kernel TU
// instantiates its own copy.
template <int TAG>
__global__ __launch_bounds__(256) void conv1d_splitk_reduce_kernel(ConvKArgs a) {
    const int64_t per_b = (int64_t)a.M * a.U;
    const int64_t total = per_b * a.B;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        float v = 0.f;
        for (int s = 0; s < a.S; ++s) v += a.partial[(int64_t)s * total + i];
        const int b = (int)(i / per_b);
        const int64_t r = i - (int64_t)b * per_b;
        const int m = (int)(r / a.U);
        const int n = (int)(r - (int64_t)m * a.U);
        store_out(a, b, m, n, v);
    }
}

// First row of ConvT phase group 1: c_out*q0, rounded up to the 64-row tile
// so that no tile straddles the two window offsets (no group 1: all rows).
static inline int convt_group1_row(int c_out, int R, int q0) {
    const int g0 = c_out * q0;
    return q0 == R ? g0 : ceil_div(g0, 64) * 64;
}

struct LaunchCfg {
    int bm, bn, S;
    int sep = 0;          // gemv (bm == 0, bn = NMAX): the K-split slabs summed by a separate launch
    int inl = 0;          // fp32 MFMA tiles (bm > 0, config bit 9, round 6): summed in-launch instead
    int rows = 0;         // row-sliced skinny-N (tile 14, round 6): rows per workgroup (16 / 32), no K split
};

// Skinny-N fp32 family (conv_gemv.hip): weights spread over the chip, all
// output columns (U <= NMAX) per workgroup.  Launch-config tiles 8..13 of the
// exact-fp32 precision select it with NMAX = 4 << (tile - 8) (4 ... 128).
constexpr int kGemvMaxN = 128;
inline bool is_gemv_tile(int t) { return t >= 8 && t <= 13; }
inline int gemv_rows(int nmax) { return nmax <= 32 ? 256 : nmax == 64 ? 128 : 64; }   // rows per workgroup
inline int gemv_nmax(int t) { return 4 << (t - 8); }
bool gemv_fits(int taps, int U, int d, bool transposed, int cps, int nmax);
int conv1d_gemv(ConvKArgs k, int taps, int nmax, int sep, hipStream_t st);
// Row-sliced skinny-N form (conv_gemv.hip, round 6): config tile 14 (bit 9 = 32
// rows per workgroup, else 16) or 15 (8 rows), one K split; NMAX the smallest
// of 4..32 holding U
constexpr int kRowsTile = 14, kRowsTile8 = 15, kRowsMaxN = 32;
bool gemv_rows_fits(int taps, int U, int d, bool transposed, int nchunks, int nmax);
int conv1d_gemv_rows(ConvKArgs k, int taps, int nmax, int rt, hipStream_t st);
inline int rows_nmax(int U) { int n = 4; while (n < U) n *= 2; return n; }

// rave_conv1d_args.config: 0 = heuristic, else 1 + tile + 16 (S - 1) + 512 sep
// (tile: index into the precision's tile table; S: K-splits; sep: split-K
// combine in a separate reduce launch instead of in-launch)
struct ConfigCode {
    int tile, S, sep;
};
static inline bool decode_config(int cfg, ConfigCode& c) {
    if (cfg <= 0) return false;
    const int v = cfg - 1;
    c.tile = v & 15;
    c.S = ((v >> 4) & 31) + 1;
    c.sep = (v >> 9) & 1;
    return (v >> 10) == 0;
}
static inline int encode_config(int tile, int S, int sep) { return 1 + tile + 16 * (S - 1) + 512 * sep; }
// K-split counts the autotuner tries (an S whose chunks per split equal a smaller S's is skipped)
constexpr int kSplitCands[] = {1, 2, 3, 4, 6, 8, 12, 16};
static inline bool split_count_distinct(int S, int nchunks) {
    return S <= nchunks && ceil_div(nchunks, ceil_div(nchunks, S)) == S;
}

static inline double pad_waste(int M, int U, int bm, int bn) {
    return double(ceil_div(M, bm) * bm) * double(ceil_div(U, bn) * bn) / (double(M) * double(U));
}

static inline int family_stride(int taps) {
    switch (taps) {
        case 4: return 2;
        case 8: return 4;
        default: return 1;
    }
}

static inline bool family_supported(int taps) {
    return taps == 1 || taps == 2 || taps == 3 || taps == 4 || taps == 7 || taps == 8;
}

// Fill ConvKArgs from the public args (everything but the packed-weight
// geometry, which depends on the precision); returns status and the tap count.
static inline int prepare_common(const rave_conv1d_args& a, ConvKArgs& k, int& taps) {
    RAVE_CHECK_ARG(a.x && a.y && a.weight, "conv1d: null tensor");
    RAVE_CHECK_ARG(a.batch > 0 && a.t_in > 0 && a.t_out > 0 && a.c_in > 0 && a.c_out > 0,
                   "conv1d: empty shape");
    RAVE_CHECK_ARG(a.act != RAVE_ACT_SNAKE || a.alpha, "conv1d: snake needs alpha");
    RAVE_CHECK_ARG(a.pad_left >= 0 && a.pad_right >= 0, "conv1d: negative padding");
    k = ConvKArgs{};
    k.x = a.x; k.w = a.weight; k.bias = a.bias; k.alpha = a.alpha; k.res = a.residual; k.y = a.y;
    k.x_sb = a.x_sb; k.x_sc = a.x_sc; k.y_sb = a.y_sb; k.y_sc = a.y_sc; k.r_sb = a.r_sb; k.r_sc = a.r_sc;
    k.c_in = a.c_in; k.B = a.batch;
    k.act = a.act; k.slope = a.leaky_slope;
    k.pad_l = a.pad_left; k.t_in = a.t_in; k.t_y = a.t_out;
    if (a.transposed) {
        RAVE_CHECK_ARG(a.kernel == 2 * a.stride && a.stride % 2 == 0,
                       "conv1d: transposed needs kernel == 2*stride, even stride");
        RAVE_CHECK_ARG(a.residual == nullptr, "conv1d: residual unsupported on transposed conv");
        RAVE_CHECK_ARG(a.out_shift == 0 || a.out_shift == a.stride / 2,
                       "conv1d: transposed out_shift must be 0 (cached) or stride/2 (padding r//2)");
        RAVE_CHECK_ARG(a.pad_left == 0 || a.pad_left == 1, "conv1d: transposed pad_left = history columns (0/1)");
        k.transposed = 1; k.R = a.stride; k.out_shift = a.out_shift;
        taps = 2; k.d = 1;
        k.q0 = a.stride - a.out_shift;               // phases whose taps are (u-1, u)
        k.split_row = convt_group1_row(a.c_out, a.stride, k.q0);
        k.M = k.split_row + a.c_out * (a.stride - k.q0);
        k.pad_l = 1 - a.pad_left;                    // group 0 window starts at u-1
        k.pad_g1 = -a.pad_left;                      // group 1 window starts at u
        k.U = a.t_in - a.pad_left;
        RAVE_CHECK_ARG(k.U > 0, "conv1d: empty transposed input");
        RAVE_CHECK_ARG((int64_t)k.U * k.R == a.t_out, "conv1d: transposed t_out must be (t_in - pad_left) * stride");
    } else {
        taps = a.kernel;
        if (!family_supported(taps) || family_stride(taps) != a.stride) {
            set_error("conv1d: unsupported (kernel, stride) pair; supported: k1/k3/k7 s1, k4 s2, k8 s4");
            return RAVE_ERR_UNSUPPORTED;
        }
        RAVE_CHECK_ARG(a.dilation == 1 || taps == 3, "conv1d: dilation only on 3-tap convs");
        RAVE_CHECK_ARG(a.dilation >= 1 && a.dilation <= kMaxDil, "conv1d: dilation out of range");
        k.transposed = 0; k.R = 1; k.out_shift = 0;
        k.split_row = 1 << 30; k.pad_g1 = a.pad_left; k.q0 = 1;
        k.d = a.dilation;
        k.M = a.c_out;
        int span = (a.kernel - 1) * a.dilation + 1;
        int expect = (a.t_in + a.pad_left + a.pad_right - span) / a.stride + 1;
        RAVE_CHECK_ARG(expect == a.t_out, "conv1d: t_out does not match the conv arithmetic");
        k.U = a.t_out;
    }
    {
        const int64_t xb = ((int64_t)(a.c_in - 1) * a.x_sc + a.t_in) * 4;
        RAVE_CHECK_ARG(xb < (1ll << 31) && a.x_sc >= 0,
                       "conv1d: tensors beyond 2 GiB per batch item need 64-bit offsets");
        k.x_bytes = (int)xb;
        const int y_rows = a.c_out;
        const int64_t yb = ((int64_t)(y_rows - 1) * a.y_sc + a.t_out) * 4;
        const int64_t rb = a.residual ? ((int64_t)(a.c_out - 1) * a.r_sc + a.t_out) * 4 : 0;
        RAVE_CHECK_ARG(yb < (1ll << 31) && rb < (1ll << 31), "conv1d: output beyond 2 GiB per batch item");
        k.y_bytes = (int)yb;
        k.r_bytes = (int)rb;
        k.bias_rows = a.c_out;
    }
    return RAVE_OK;
}

// RAVE_PREC_SPLIT16 path (conv_split.hip)
int conv1d_split(const rave_conv1d_args& a, void* stream);
int64_t conv1d_split_workspace(const rave_conv1d_args& a);
int conv1d_split_configs(const rave_conv1d_args& a, int32_t* cfgs, int max_cfgs);

}  // namespace rave
