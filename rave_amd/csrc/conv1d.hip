// Implicit-GEMM Conv1d / ConvTranspose1d on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces cached_conv's Conv1d/ConvTranspose1d forward (F.pad + F.conv1d /
// F.conv_transpose1d; third-party cached-conv>=2.5.0, non-cached mode) at every
// call site of rave/blocks.py (DilatedUnit :96-106, EncoderV2 :533-584,
// GeneratorV2 :631-677, NoiseGeneratorV2 :257-266), fused with the activation
// module that precedes each conv (LeakyReLU(.2) / Snake) and the Residual add
// (rave/blocks.py:44-46).
//
// GEMM view: Y[m, n] = sum_kk W[m, kk] * X[kk, n] with kk = (ci, tap).
//  * The K dimension is walked in chunks of CI_T input channels x all taps.
//  * For each chunk the workgroup stages (a) the weight tile [BK][BM] (packed on
//    the host so every row is BM contiguous floats) and (b) the input window of
//    the dilated receptive field: CI_T rows x ((BN-1)*s + (k-1)*d + 1) columns,
//    read once from HBM (coalesced along time), activation applied, stored in
//    polyphase order (phase = column mod stride) so the strided B-fragment
//    reads of one tap are consecutive in LDS (conflict-free ds_read_b32).
//  * Each tap's B operand is a shifted view of the same LDS window: the halo is
//    fetched once, not k times.
//  * 4 waves per workgroup (2x2); each wave owns (BM/2)x(BN/2) of 32x32 MFMA
//    tiles; exact fp32 (the MFMA is a k-ordered fmaf chain).
//  * Global loads of chunk c+1 are issued into registers before the MFMAs of
//    chunk c (register-staged software pipeline).
//
// ConvTranspose1d(C, C', 2r, stride r) runs in polyphase form: the r output
// phases of input position u are rows m = co*r + q of a 2-tap conv over the
// input; the epilogue interleaves them to t = u*r + q - out_shift.
#include "common.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace rave {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));   // native vector (HIP float4 is a struct: memcpy -> scratch)

constexpr int kThreads = 256;
constexpr int kMaxBK = 64;        // taps * CI_T per chunk
constexpr int kXMax = 5120;       // floats of the staged input window per chunk
constexpr int kXRegs = kXMax / kThreads;   // 20
constexpr int kXSlack = kXMax + 1536;     // floats reserved for Xs (covers unconditional stores)

struct ConvKArgs {
    const float* x; const float* w; const float* bias; const float* alpha; const float* res;
    float* y;
    int64_t x_sb, x_sc, y_sb, y_sc, r_sb, r_sc;
    int c_in, M, taps, s, log2s, d, pad_l, t_in, U;
    int ci_t, nchunks, Mpad, XW, XWs, XR;
    int transposed, R, out_shift, t_y, act;
    float slope;
};

// --------------------------------------------------------------------- host helpers
static int ilog2(int v) { int l = 0; while ((1 << l) < v) ++l; return l; }

// Window length (columns) of the staged input for a BN-column output tile.
static int window_len(int bn, int s, int taps, int d) { return (bn - 1) * s + (taps - 1) * d + 1; }

static int row_stride(int bn, int s, int taps, int d) {
    int xw = window_len(bn, s, taps, d);
    int xws = ceil_div(xw, s);
    return xws * s;
}

int chunk_channels(int c_in, int taps, int s, int d) {
    // largest even CI_T (prefer divisors of c_in) with taps*CI_T <= 64 and the
    // staged window (at BN = 128) within kXMax floats
    int xr = row_stride(128, s, taps, d);
    int best = 0, best_div = 0;
    int cmax = std::min(kMaxBK / taps, kXMax / xr);
    int cin_even = (c_in + 1) & ~1;
    for (int c = 2; c <= cmax && c <= cin_even; c += 2) {
        best = c;
        if (cin_even % c == 0) best_div = c;
    }
    if (best == 0) return 0;
    // a divisor within 2x of the max is better than padding the last chunk
    if (best_div * 2 >= best) return best_div;
    return best;
}

// --------------------------------------------------------------------- kernel
template <int BM, int BN>
__global__ __launch_bounds__(kThreads) void conv1d_mfma_kernel(ConvKArgs a) {
    constexpr int WM = BM / 2, WN = BN / 2;
    constexpr int TM = WM / 32, TN = WN / 32;
    constexpr int NA4 = kMaxBK * BM / 4 / kThreads;   // float4 staging regs for A

    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int BK = a.ci_t * a.taps;
    float* As = smem;                 // [BK][BM] (kMaxBK rows reserved)
    float* Xs = smem + kMaxBK * BM;   // [CI_T][XR] polyphase (kXSlack floats reserved)

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm0 = (wave >> 1) * WM;
    const int wn0 = (wave & 1) * WN;
    const int h = lane >> 5;
    const int l32 = lane & 31;

    const int n0 = blockIdx.x * BN;
    const int m0 = blockIdx.y * BM;
    const int b = blockIdx.z;
    const int in0 = n0 * a.s - a.pad_l;

    const float* xb = a.x + (int64_t)b * a.x_sb;

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int a_elems4 = BK * BM / 4;
    const int x_elems = a.ci_t * a.XW;

    f32x4 ra[NA4];
    float rx[kXRegs];

    auto load_chunk = [&](int c) __attribute__((always_inline)) {
        const f32x4* wsrc = reinterpret_cast<const f32x4*>(a.w + (int64_t)c * BK * a.Mpad + m0);
        // Every load is unconditional from a clamped, valid address; validity is
        // a select afterwards.  (A load under a per-element branch makes hipcc
        // wait vmcnt(0) per element and spill the staging array to scratch.)
#pragma unroll
        for (int i = 0; i < NA4; ++i) {
            int e = min(tid + i * kThreads, a_elems4 - 1);
            int row = e / (BM / 4);
            int col4 = e - row * (BM / 4);
            ra[i] = wsrc[(int64_t)row * (a.Mpad / 4) + col4];
        }
        const int ci0 = c * a.ci_t;
        int ci = tid / a.XW;
        int w = tid - ci * a.XW;
#pragma unroll
        for (int i = 0; i < kXRegs; ++i) {
            int e = tid + i * kThreads;
            int cg = ci0 + ci;
            int t = in0 + w;
            bool ok = (e < x_elems) && (cg < a.c_in) && (t >= 0) && (t < a.t_in);
            int cgc = min(cg, a.c_in - 1);
            int tc = min(max(t, 0), a.t_in - 1);
            float v = xb[(int64_t)cgc * a.x_sc + tc];
            rx[i] = ok ? v : 0.f;
            w += kThreads;   // XW >= 64, so at most four wraps per step
            if (w >= a.XW) { w -= a.XW; ++ci; }
            if (w >= a.XW) { w -= a.XW; ++ci; }
            if (w >= a.XW) { w -= a.XW; ++ci; }
            if (w >= a.XW) { w -= a.XW; ++ci; }
        }
    };

    auto store_chunk = [&](int c) __attribute__((always_inline)) {
        // Unconditional stores: rows past the chunk land in LDS slack (As has
        // kMaxBK rows, Xs kXSlack floats), so no per-element branches.
#pragma unroll
        for (int i = 0; i < NA4; ++i) {
            int e = tid + i * kThreads;
            int row = e / (BM / 4);
            int col4 = e - row * (BM / 4);
            *reinterpret_cast<f32x4*>(As + row * BM + col4 * 4) = ra[i];
        }
        const int ci0 = c * a.ci_t;
        int ci = tid / a.XW;
        int w = tid - ci * a.XW;
#pragma unroll
        for (int i = 0; i < kXRegs; ++i) {
            {
                int cg = min(ci0 + ci, a.c_in - 1);
                float al = (a.act == RAVE_ACT_SNAKE) ? a.alpha[cg] : 0.f;
                float v = apply_act(rx[i], a.act, a.slope, al);
                int ph = w & (a.s - 1);
                int wq = w >> a.log2s;
                Xs[ci * a.XR + ph * a.XWs + wq] = v;
            }
            w += kThreads;   // XW >= 64, so at most four wraps per step
            if (w >= a.XW) { w -= a.XW; ++ci; }
            if (w >= a.XW) { w -= a.XW; ++ci; }
            if (w >= a.XW) { w -= a.XW; ++ci; }
            if (w >= a.XW) { w -= a.XW; ++ci; }
        }
    };

    load_chunk(0);
    for (int c = 0; c < a.nchunks; ++c) {
        __syncthreads();
        store_chunk(c);
        __syncthreads();
        load_chunk(min(c + 1, a.nchunks - 1));   // unconditional (redundant reload on the last chunk)

        const int half = a.ci_t >> 1;
        for (int j = 0; j < a.taps; ++j) {
            const float* Aj = As + (j * a.ci_t + h) * BM + wm0 + l32;
            int p = (wn0 + l32) * a.s + j * a.d;
            const float* Xj = Xs + h * a.XR + (p & (a.s - 1)) * a.XWs + (p >> a.log2s);
#pragma unroll 2
            for (int c2 = 0; c2 < half; ++c2) {
                float av[TM], bv[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) av[i] = Aj[c2 * 2 * BM + i * 32];
#pragma unroll
                for (int i = 0; i < TN; ++i) bv[i] = Xj[c2 * 2 * a.XR + i * 32];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int jj = 0; jj < TN; ++jj)
                        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[jj], acc[i][jj], 0, 0, 0);
            }
        }
    }

    // ---------------------------------------------------------------- epilogue
    float* yb = a.y + (int64_t)b * a.y_sb;
    const float* rb = a.res ? a.res + (int64_t)b * a.r_sb : nullptr;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) {
            const int n = n0 + wn0 + jj * 32 + l32;
            if (n >= a.U) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m >= a.M) continue;
                float v = acc[i][jj][r];
                if (a.transposed) {
                    const int co = m / a.R;
                    const int q = m - co * a.R;
                    const int t = n * a.R + q - a.out_shift;
                    if (t < 0 || t >= a.t_y) continue;
                    if (a.bias) v += a.bias[co];
                    yb[(int64_t)co * a.y_sc + t] = v;
                } else {
                    if (a.bias) v += a.bias[m];
                    if (rb) v += rb[(int64_t)m * a.r_sc + n];
                    yb[(int64_t)m * a.y_sc + n] = v;
                }
            }
        }
    }
}

// --------------------------------------------------------------------- launch
struct TileCfg { int bm, bn; };

static TileCfg pick_tile(int M, int U, int B) {
    const TileCfg cands[4] = {{128, 128}, {64, 128}, {128, 64}, {64, 64}};
    for (const auto& c : cands) {
        int64_t wg = (int64_t)ceil_div(M, c.bm) * ceil_div(U, c.bn) * B;
        double waste = double(ceil_div(M, c.bm) * c.bm) * double(ceil_div(U, c.bn) * c.bn) /
                       (double(M) * double(U));
        if (wg >= 512 && waste <= 1.15) return c;
    }
    // not enough work for two workgroups per CU: smallest tile
    return cands[3];
}

template <int BM, int BN>
static int launch_tile(ConvKArgs k, int B, hipStream_t st) {
    k.XW = window_len(BN, k.s, k.taps, k.d);
    k.XWs = ceil_div(k.XW, k.s);
    k.XR = k.XWs * k.s;
    if (k.ci_t * k.XW > kXMax || k.ci_t * k.XR > kXMax + 64 * 4) {
        set_error("conv1d: staged window exceeds LDS budget");
        return RAVE_ERR_UNSUPPORTED;
    }
    size_t lds = (size_t)(kMaxBK * BM + kXSlack) * sizeof(float);
    dim3 grid(ceil_div(k.U, BN), ceil_div(k.M, BM), B);
    hipLaunchKernelGGL((conv1d_mfma_kernel<BM, BN>), grid, dim3(kThreads), lds, st, k);
    return launch_status("conv1d_mfma_kernel");
}

}  // namespace rave

using namespace rave;

extern "C" int rave_conv1d_chunk(int c_in, int kernel, int stride, int dilation, int transposed) {
    int taps = transposed ? 2 : kernel;
    int s = transposed ? 1 : stride;
    int d = transposed ? 1 : dilation;
    return chunk_channels(c_in, taps, s, d);
}

extern "C" int64_t rave_conv1d_packed_size(int c_in, int c_out, int kernel, int stride, int dilation,
                                           int transposed) {
    int ci_t = rave_conv1d_chunk(c_in, kernel, stride, dilation, transposed);
    if (ci_t <= 0) return -1;
    int taps = transposed ? 2 : kernel;
    int M = transposed ? c_out * stride : c_out;
    int64_t Mpad = (int64_t)ceil_div(M, 128) * 128;
    int64_t nchunks = ceil_div(c_in, ci_t);
    return nchunks * ci_t * taps * Mpad;
}

extern "C" int rave_conv1d_pack_weight(const float* w, int c_in, int c_out, int kernel, int stride,
                                       int dilation, int transposed, float* packed) {
    RAVE_CHECK_ARG(w && packed, "pack_weight: null pointer");
    RAVE_CHECK_ARG(c_in > 0 && c_out > 0 && kernel > 0 && stride > 0 && dilation > 0,
                   "pack_weight: bad shape");
    RAVE_CHECK_ARG(!transposed || kernel == 2 * stride, "pack_weight: transposed needs kernel == 2*stride");
    int ci_t = rave_conv1d_chunk(c_in, kernel, stride, dilation, transposed);
    RAVE_CHECK_ARG(ci_t > 0, "pack_weight: unsupported layer shape");
    int taps = transposed ? 2 : kernel;
    int R = transposed ? stride : 1;
    int M = c_out * R;
    int64_t Mpad = (int64_t)ceil_div(M, 128) * 128;
    int nchunks = ceil_div(c_in, ci_t);
    int BK = ci_t * taps;
    std::memset(packed, 0, sizeof(float) * (size_t)nchunks * BK * Mpad);
    for (int c = 0; c < nchunks; ++c)
        for (int j = 0; j < taps; ++j)
            for (int cl = 0; cl < ci_t; ++cl) {
                int ci = c * ci_t + cl;
                if (ci >= c_in) continue;
                float* row = packed + ((int64_t)c * BK + j * ci_t + cl) * Mpad;
                for (int m = 0; m < M; ++m) {
                    float v;
                    if (transposed) {
                        int co = m / R, q = m % R;
                        // tap 0 multiplies x[u-1] -> kernel index q + r; tap 1 x[u] -> q
                        int kidx = (j == 0) ? q + R : q;
                        v = w[((int64_t)ci * c_out + co) * kernel + kidx];
                    } else {
                        v = w[((int64_t)m * c_in + ci) * kernel + j];
                    }
                    row[m] = v;
                }
            }
    return RAVE_OK;
}

extern "C" int rave_conv1d(const rave_conv1d_args* p, void* stream) {
    RAVE_CHECK_ARG(p, "conv1d: null args");
    const rave_conv1d_args& a = *p;
    RAVE_CHECK_ARG(a.x && a.y && a.weight, "conv1d: null tensor");
    RAVE_CHECK_ARG(a.batch > 0 && a.t_in > 0 && a.t_out > 0 && a.c_in > 0 && a.c_out > 0,
                   "conv1d: empty shape");
    RAVE_CHECK_ARG(a.act != RAVE_ACT_SNAKE || a.alpha, "conv1d: snake needs alpha");
    RAVE_CHECK_ARG(a.pad_left >= 0 && a.pad_right >= 0, "conv1d: negative padding");
    ConvKArgs k{};
    k.x = a.x; k.w = a.weight; k.bias = a.bias; k.alpha = a.alpha; k.res = a.residual; k.y = a.y;
    k.x_sb = a.x_sb; k.x_sc = a.x_sc; k.y_sb = a.y_sb; k.y_sc = a.y_sc; k.r_sb = a.r_sb; k.r_sc = a.r_sc;
    k.c_in = a.c_in;
    k.act = a.act; k.slope = a.leaky_slope;
    k.pad_l = a.pad_left; k.t_in = a.t_in; k.t_y = a.t_out;
    if (a.transposed) {
        RAVE_CHECK_ARG(a.kernel == 2 * a.stride, "conv1d: transposed needs kernel == 2*stride");
        RAVE_CHECK_ARG(a.residual == nullptr, "conv1d: residual unsupported on transposed conv");
        k.transposed = 1; k.R = a.stride; k.out_shift = a.out_shift;
        k.taps = 2; k.s = 1; k.log2s = 0; k.d = 1;
        k.M = a.c_out * a.stride;
        k.U = a.t_in + a.pad_left + a.pad_right - 1;
        RAVE_CHECK_ARG(k.U > 0, "conv1d: empty transposed output");
        RAVE_CHECK_ARG((int64_t)(k.U - 1) * k.R + (k.R - 1) - k.out_shift >= (int64_t)a.t_out - 1,
                       "conv1d: transposed t_out exceeds computed range");
    } else {
        RAVE_CHECK_ARG((a.stride & (a.stride - 1)) == 0, "conv1d: stride must be a power of two");
        k.transposed = 0; k.R = 1; k.out_shift = 0;
        k.taps = a.kernel; k.s = a.stride; k.log2s = ilog2(a.stride); k.d = a.dilation;
        k.M = a.c_out;
        int span = (a.kernel - 1) * a.dilation + 1;
        int expect = (a.t_in + a.pad_left + a.pad_right - span) / a.stride + 1;
        RAVE_CHECK_ARG(expect == a.t_out, "conv1d: t_out does not match the conv arithmetic");
        k.U = a.t_out;
    }
    k.ci_t = rave_conv1d_chunk(a.c_in, a.kernel, a.stride, a.dilation, a.transposed);
    RAVE_CHECK_ARG(k.ci_t > 0, "conv1d: unsupported layer shape");
    k.nchunks = ceil_div(a.c_in, k.ci_t);
    k.Mpad = ceil_div(k.M, 128) * 128;

    hipStream_t st = as_stream(stream);
    TileCfg t = pick_tile(k.M, k.U, a.batch);
    if (t.bm == 128 && t.bn == 128) return launch_tile<128, 128>(k, a.batch, st);
    if (t.bm == 64 && t.bn == 128) return launch_tile<64, 128>(k, a.batch, st);
    if (t.bm == 128 && t.bn == 64) return launch_tile<128, 64>(k, a.batch, st);
    return launch_tile<64, 64>(k, a.batch, st);
}
