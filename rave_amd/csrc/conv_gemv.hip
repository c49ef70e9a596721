// Skinny-N convolution ("GEMV" family) in exact fp32 on the VALU: the cached
// streaming convs at batch 1 (BASELINE configs[2], cached_conv's
// CachedConv1d / CachedConvTranspose1d at every call site of rave/blocks.py:
// DilatedUnit :96-106, EncoderV2 :533-584, GeneratorV2 :631-677) produce 2-32
// output frames per call while reading the layer's whole weight matrix.  The
// column-tiled MFMA kernels give such a layer a handful of workgroups, each
// streaming a large share of the weights through one CU.  Here the weight
// matrix is spread over the whole chip instead:
//
//   Y[m, n] = sum_kk W[m, kk] act(X)[kk, n] (+ bias, + residual)   n < U <= NMAX
//
//   * grid = (256-row tiles) x (K splits) x batch; a workgroup reads its rows'
//     share of W exactly once, straight from the exact-fp32 packed image of
//     conv1d.hip ([chunk][tap][channel][Mpad]: each K-row is Mpad contiguous
//     floats), one 16-byte load per lane per K-row (lane = 4 consecutive rows,
//     a wave covers 256 rows: fully coalesced);
//   * the split's input window (its channels x the U output columns' reach) is
//     staged once in LDS with the activation applied; every lane reads the
//     same x values (LDS broadcast) and keeps 4 x NMAX fp32 accumulators
//     (packed v_pk_fma_f32 over column pairs);
//   * the 4 waves take interleaved channels of every chunk and are summed
//     through LDS in wave order; K splits over workgroups write fp32 slabs that
//     the last-arriving split sums in split order (or a separate reduce launch)
//     -- fixed orders, bitwise reproducible, no float atomics.
// ConvTranspose1d runs in conv1d.hip's polyphase form (rows m = (co, phase q),
// 2 taps, phase group 1 one input column later).
#include "conv_shared.h"

namespace rave {

typedef float g_f32x2 __attribute__((ext_vector_type(2)));
typedef float g_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kGemvStage = 12288;                  // staged window floats per workgroup (48 KiB)
// in-launch split-K combine by sc1 stores / loads instead of an agent release /
// acquire pair (round 6; 0 = the fence form, for A/B builds)
#ifndef RAVE_GEMV_SC1
#define RAVE_GEMV_SC1 1
#endif
constexpr bool kGemvSc1 = RAVE_GEMV_SC1 != 0;
// dynamic LDS of an sc1 in-launch grid: more than half the CU's 160 KB, so no
// second workgroup of the launch shares the CU (the measured form's condition)
constexpr size_t kGemvOnePerCu = 80 * 1024 + 256;

// (channels per packed chunk, stride) of conv1d.hip's exact-fp32 families
template <int KT> struct GFam;
template <> struct GFam<1> { static constexpr int CIT = 32, ST = 1; };
template <> struct GFam<2> { static constexpr int CIT = 32, ST = 1; };
template <> struct GFam<3> { static constexpr int CIT = 16, ST = 1; };
template <> struct GFam<4> { static constexpr int CIT = 16, ST = 2; };
template <> struct GFam<7> { static constexpr int CIT = 8, ST = 1; };
template <> struct GFam<8> { static constexpr int CIT = 8, ST = 4; };

// window columns a split stages: every output column's reach, plus one column
// for ConvT phase group 1 (its taps start one input column later)
__host__ __device__ inline int gemv_xw(int KT, int ST, int U, int d, bool transposed) {
    return (U - 1) * ST + (KT - 1) * d + 1 + (transposed ? 1 : 0);
}

// GR<NMAX>: rows per lane (4 x NMAX accumulators at most 128 floats), rows
// per workgroup, threads per output row in the epilogue and columns per thread
template <int NMAX> struct GR {
    static constexpr int R = NMAX <= 32 ? 4 : NMAX == 64 ? 2 : 1;
    static constexpr int BM = 64 * R, TPR = 256 / BM, NC = NMAX / TPR;
};

template <int KT, int NMAX, bool SNAKE>
__global__ __launch_bounds__(256) void conv1d_gemv_kernel(ConvKArgs a) {
    constexpr int CIT = GFam<KT>::CIT, ST = GFam<KT>::ST, NP = NMAX / 2;
    constexpr int R = GR<NMAX>::R, BM = GR<NMAX>::BM, NC = GR<NMAX>::NC;
    constexpr unsigned kOOB = 0xFFFFFFF0u;
    extern __shared__ __attribute__((aligned(16))) float gsm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int MT = ceil_div(a.M, BM);
    // splits of one row tile on consecutive blocks of one XCD (blocks b, b+8, ...)
    int lg = blockIdx.x;
    if ((gridDim.x & 7) == 0) lg = (lg & 7) * (gridDim.x >> 3) + (lg >> 3);
    lg = __builtin_amdgcn_readfirstlane(lg);
    const int split = lg % a.S;
    const int tile = lg / a.S;                       // b * MT + mt (ticket index)
    const int mt = tile % MT, b = tile / MT;
    const int m0 = mt * BM;
    const int c_begin = split * a.cps, c_end = min(a.nchunks, c_begin + a.cps);
    const int nch = (c_end - c_begin) * CIT;         // staged channels
    const int U = a.U, XW = a.XW;
    const int t0 = -a.pad_l;                         // input time of window column 0
    const float slope = a.act == RAVE_ACT_LEAKY ? a.slope : 1.0f;

    // ---------------------------------------------------------------- window
    // (WB loads in flight per thread before any is used: a load-then-use loop
    // waits out one memory round trip per element)
    constexpr int WB = 8;
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(a.x + (int64_t)b * a.x_sb, a.x_bytes);
    for (int e0 = tid; e0 < nch * XW; e0 += 256 * WB) {
        float rv[WB];
#pragma unroll
        for (int i = 0; i < WB; ++i) {
            const int e = e0 + i * 256;
            const int cl = e / XW, w = e - cl * XW;
            const int ci = c_begin * CIT + cl, t = t0 + w;
            const bool ok = e < nch * XW && ci < a.c_in && t >= 0 && t < a.t_in;
            rv[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                xrs, ok ? (unsigned)(ci * a.x_sc + t) * 4u : kOOB, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < WB; ++i) {
            const int e = e0 + i * 256;
            if (e >= nch * XW) break;
            const int cl = e / XW, w = e - cl * XW;
            const int ci = c_begin * CIT + cl, t = t0 + w;
            const bool ok = ci < a.c_in && t >= 0 && t < a.t_in;
            float v = rv[i];
            if constexpr (SNAKE) {
                const float al = a.alpha[min(ci, a.c_in - 1)];
                v = v + (1.0f / (al + 1e-9f)) * sin_squared(al * v);
            } else {
                v = v > 0.f ? v : v * slope;
            }
            gsm[cl * XW + w] = ok ? v : 0.f;
        }
    }
    __syncthreads();

    // ---------------------------------------------------------------- K loop
    // lane: rows m0 + R lane .. + R-1; ConvT rows of phase group 1 read one column later
    const int mrow = m0 + R * lane;
    const int goff = (a.transposed && mrow >= a.split_row) ? 1 : 0;
    const bool rows_ok = mrow < a.Mpad;
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(a.w, a.w_bytes);
    g_f32x2 acc[R][NP];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int p = 0; p < NP; ++p) acc[r][p] = g_f32x2{0.f, 0.f};
    // this wave's K-rows: every (chunk, tap) and channels wave, wave + 4, ... of
    // the chunk, walked in batches of QB whose weight loads are all in flight
    // before the first FMA (a load-then-use loop is one round trip per K-row)
    constexpr int QC = CIT / 4, PER_C = KT * QC, QB = NMAX <= 8 ? 16 : 8;
    const int nq = (c_end - c_begin) * PER_C;
    for (int q0 = 0; q0 < nq; q0 += QB) {
        float wv[QB][R];
        int xo[QB];
#pragma unroll
        for (int i = 0; i < QB; ++i) {
            const int q = q0 + i;
            const int cc = q / PER_C, rem = q - cc * PER_C;
            const int j = rem / QC, cl = wave + 4 * (rem - j * QC);
            const unsigned kk = (unsigned)(((c_begin + cc) * KT + j) * CIT + cl);
            const bool ok = q < nq && rows_ok;
            const unsigned off = ok ? (kk * (unsigned)a.Mpad + (unsigned)mrow) * 4u : kOOB;
            if constexpr (R == 4) {
                const g_f32x4 w4 = __builtin_bit_cast(g_f32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, off, 0, 0));
#pragma unroll
                for (int r = 0; r < 4; ++r) wv[i][r] = w4[r];
            } else if constexpr (R == 2) {
                const g_f32x2 w2 = __builtin_bit_cast(g_f32x2, __builtin_amdgcn_raw_buffer_load_b64(wrs, off, 0, 0));
                wv[i][0] = w2[0];
                wv[i][1] = w2[1];
            } else {
                wv[i][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wrs, off, 0, 0));
            }
            xo[i] = q < nq ? (cc * CIT + cl) * XW + goff + j * a.d : 0;   // (past nq: zero weights)
        }
#pragma unroll
        for (int i = 0; i < QB; ++i) {
            const float* xr = gsm + xo[i];
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                const g_f32x2 xv = {xr[(2 * p) * ST], xr[(2 * p + 1) * ST]};
#pragma unroll
                for (int r = 0; r < R; ++r)
                    acc[r][p] = __builtin_elementwise_fma(g_f32x2{wv[i][r], wv[i][r]}, xv, acc[r][p]);
            }
        }
    }
    __syncthreads();                                  // window dead: the reduction area

    // ---------------------------------------------------------------- wave sum (fixed order)
    float* red = gsm;                                 // [wave][row 0..BM-1][NMAX]
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int p = 0; p < NP; ++p)
            *reinterpret_cast<g_f32x2*>(red + ((wave * BM + R * lane + r) * NMAX + 2 * p)) = acc[r][p];
    __syncthreads();
    // from here on a thread owns row m0 + tid % BM, columns [n0, n0 + NC)
    const int rl = tid % BM, n0 = (tid / BM) * NC;
    const int m = m0 + rl;
    float v[NC];
#pragma unroll
    for (int n = 0; n < NC; ++n) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) s += red[(w * BM + rl) * NMAX + n0 + n];
        v[n] = s;
    }

    // ---------------------------------------------------------------- K splits
    if (a.S > 1) {
        const int64_t total = (int64_t)a.B * a.M * U;
        float* slab = a.partial + (int64_t)split * total + ((int64_t)b * a.M + m) * U;
        // in-launch (sc1 form): the slab is stored write-through and read back only
        // by sc1 loads, so neither the agent release nor the acquire is needed
        const __amdgpu_buffer_rsrc_t srs = make_rsrc(a.partial, 0x7FFFFFF0);
        if (m < a.M)
#pragma unroll
            for (int n = 0; n < NC; ++n) {
                if (n0 + n >= U) continue;
                if (kGemvSc1 && a.inlaunch) {
                    const int64_t off = (int64_t)split * total + ((int64_t)b * a.M + m) * U + n0 + n;
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[n]), srs, (unsigned)(off * 4), 0,
                                                          16);
                } else {
                    slab[n0 + n] = v[n];
                }
            }
        if (!a.inlaunch) return;                      // a separate reduce launch sums the slabs
        // in-launch combine: draw the row tile's ticket; the split drawing S - 1
        // sums every slab in split order (bitwise the separate reduce).  Form
        // (kGemvSc1, the launch keeps one workgroup per CU): MI355X_MICROARCH.md's
        // hand-off table row 1 -- every slab byte stored sc1, every storing wave
        // drained before the barrier behind which ONE lane adds to the tile's
        // unsharded counter, the last adder told by the value its add returned,
        // its other waves loading behind the barrier, every load of the slabs sc1.
        // Else an agent release before the add and an acquire after it.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every thread's slab stores performed
        __syncthreads();
        __shared__ int last_s;
        if (tid == 0) {
            if constexpr (!kGemvSc1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const int prev = __hip_atomic_fetch_add(a.tickets + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = prev == a.S - 1;
            if (last) {
                __hip_atomic_store(a.tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if constexpr (!kGemvSc1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
            last_s = last;
        }
        __syncthreads();
        if (!last_s) return;
        if (m >= a.M) return;
#pragma unroll
        for (int n = 0; n < NC; ++n) v[n] = 0.f;
        // slabs summed in split order; SB splits' loads in flight at once
        constexpr int SB = NC <= 8 ? 8 : 4;
        const __amdgpu_buffer_rsrc_t prs = make_rsrc(a.partial, 0x7FFFFFF0);
        for (int s0 = 0; s0 < a.S; s0 += SB) {
            float t[SB][NC];
#pragma unroll
            for (int i = 0; i < SB; ++i)
#pragma unroll
                for (int n = 0; n < NC; ++n) {
                    const int64_t off = (int64_t)(s0 + i) * total + ((int64_t)b * a.M + m) * U + n0 + n;
                    t[i][n] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                        prs, (s0 + i < a.S && n0 + n < U) ? (unsigned)(off * 4) : kOOB, 0, kGemvSc1 ? 16 : 0));
                }
#pragma unroll
            for (int i = 0; i < SB; ++i)
                if (s0 + i < a.S)
#pragma unroll
                    for (int n = 0; n < NC; ++n) v[n] += t[i][n];
        }
    }
    if (m >= a.M) return;
#pragma unroll
    for (int n = 0; n < NC; ++n)
        if (n0 + n < U) store_out(a, b, m, n0 + n, v[n]);
}

// ---------------------------------------------------------------- row-sliced form
// Skinny-N conv with no K split (round 6): the C3 stream plans pay 4-5 us per
// launch whatever its work, and a K-split conv is two launches (or an in-launch
// combine of about the same cost).  Here a workgroup owns RT = 8, 16 or 32 output
// rows over the WHOLE K, so a conv is one launch with M / RT workgroups per
// batch item and nothing to combine:
//   * lane = kl * ML + ml: ML = RT / 4 lanes along the rows (4 consecutive rows
//     each, one 16-byte load per K-row: a wave instruction reads KL = 64 / ML
//     K-rows x RT * 4 contiguous bytes), KL lanes along K; the 4 waves take
//     interleaved K-row groups;
//   * the input window of every channel is staged once in LDS, activation
//     applied (as conv1d_gemv_kernel);
//   * each lane keeps 4 x NMAX fp32 sums; the KL lanes of one row group are
//     summed by a fixed xor-shuffle tree, the 4 waves through LDS in wave
//     order: deterministic, no atomics, no slabs.
constexpr int kRowsStage = 24576;                  // staged window floats (96 KiB)
#ifndef RAVE_ROWS_XCD
#define RAVE_ROWS_XCD 1                            // 0: plain block order (A/B builds)
#endif
// the wave-sum area after the window (+ slack: lanes read NMAX columns per row)
__host__ __device__ inline int rows_red_off(int window, int slack) { return ((window + 3) & ~3) + slack + 16; }

template <int KT, int NMAX, int RT, bool SNAKE>
__global__ __launch_bounds__(256) void conv1d_gemv_rows_kernel(ConvKArgs a) {
    constexpr int CIT = GFam<KT>::CIT, ST = GFam<KT>::ST;
    constexpr int ML = RT / 4, KL = 64 / ML, KRW = KT * CIT, QB = NMAX <= 8 ? 16 : 8;
    constexpr unsigned kOOB = 0xFFFFFFF0u;
    extern __shared__ __attribute__((aligned(16))) float gsm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ml = lane % ML, kl = lane / ML;
    const int MT = ceil_div(a.M, RT);
    // neighbouring row tiles (which read the same 128-byte weight lines at RT < 32)
    // on one XCD: blocks are dealt round-robin over the 8 XCDs (common.h xcd_major)
    const int tile = __builtin_amdgcn_readfirstlane(RAVE_ROWS_XCD ? xcd_major((int)blockIdx.x, (int)gridDim.x)
                                                                   : (int)blockIdx.x);
    const int mt = tile % MT, b = tile / MT;
    const int m0 = mt * RT;
    const int nch = a.nchunks * CIT;                 // staged channels (all of K)
    const int U = a.U, XW = a.XW;
    const int t0 = -a.pad_l;
    const float slope = a.act == RAVE_ACT_LEAKY ? a.slope : 1.0f;

    // K-row kr of the packed image ([chunk][tap][channel][Mpad]) = (chunk, tap j,
    // channel cl): x of column n at window (chunk * CIT + cl, goff + j d + n ST)
    const int mrow = m0 + 4 * ml;
    const int goff = (a.transposed && m0 >= a.split_row) ? 1 : 0;   // (RT | 64: no straddle)
    const bool rows_ok = mrow < a.Mpad;
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(a.w, a.w_bytes);
    const int nq = a.nchunks * KRW;
    constexpr int KS = 4 * KL;                       // K-rows per workgroup step
    // one batch: QB K-rows' weights (16 B per lane each) and window offsets
    auto load_batch = [&](int k0, f32x4* wv, int* xo) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < QB; ++i) {
            const int kr = k0 + i * KS;
            const bool ok = kr < nq && rows_ok;
            const unsigned off = ok ? ((unsigned)kr * (unsigned)a.Mpad + (unsigned)mrow) * 4u : kOOB;
            wv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, off, 0, 0));
            const int c = kr / KRW, rem = kr - c * KRW, j = rem / CIT, cl = rem - j * CIT;
            xo[i] = kr < nq ? (c * CIT + cl) * XW + goff + j * a.d : 0;   // (past nq: zero weights)
        }
    };
    // the first batch's weights are in flight while the window is staged (they
    // do not depend on it); each later batch is loaded under the previous one's FMAs
    const int kfirst = wave * KL + kl;
    f32x4 wv[QB];
    int xo[QB];
    load_batch(kfirst, wv, xo);

    // ---------------------------------------------------------------- window
    constexpr int WB = 8;
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(a.x + (int64_t)b * a.x_sb, a.x_bytes);
    for (int e0 = tid; e0 < nch * XW; e0 += 256 * WB) {
        float rv[WB];
#pragma unroll
        for (int i = 0; i < WB; ++i) {
            const int e = e0 + i * 256;
            const int ci = e / XW, w = e - ci * XW, t = t0 + w;
            const bool ok = e < nch * XW && ci < a.c_in && t >= 0 && t < a.t_in;
            rv[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                xrs, ok ? (unsigned)(ci * a.x_sc + t) * 4u : kOOB, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < WB; ++i) {
            const int e = e0 + i * 256;
            if (e >= nch * XW) break;
            const int ci = e / XW, w = e - ci * XW, t = t0 + w;
            const bool ok = ci < a.c_in && t >= 0 && t < a.t_in;
            float v = rv[i];
            if constexpr (SNAKE) {
                const float al = a.alpha[min(ci, a.c_in - 1)];
                v = v + (1.0f / (al + 1e-9f)) * sin_squared(al * v);
            } else {
                v = v > 0.f ? v : v * slope;
            }
            gsm[e] = ok ? v : 0.f;
        }
    }
    __syncthreads();

    // ---------------------------------------------------------------- K loop
    float acc[4][NMAX];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int n = 0; n < NMAX; ++n) acc[r][n] = 0.f;
    // (the batch loop runs per wave: its K-rows start at wave * KL, wave-uniform)
    for (int kw = wave * KL; kw < nq; kw += KS * QB) {
        f32x4 wn[QB];
        int xn[QB];
        if (kw + KS * QB < nq) load_batch(kw + KS * QB + kl, wn, xn);
#pragma unroll
        for (int i = 0; i < QB; ++i) {
            const float* xr = gsm + xo[i];
#pragma unroll
            for (int n = 0; n < NMAX; ++n) {
                const float xv = xr[n * ST];
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[r][n] = fmaf(wv[i][r], xv, acc[r][n]);
            }
        }
        if (kw + KS * QB < nq) {
#pragma unroll
            for (int i = 0; i < QB; ++i) {
                wv[i] = wn[i];
                xo[i] = xn[i];
            }
        }
    }

    // ---------------------------------------------------------------- sums (fixed order)
#pragma unroll
    for (int off = ML; off < 64; off *= 2)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int n = 0; n < NMAX; ++n) acc[r][n] += __shfl_xor(acc[r][n], off);
    float* red = gsm + rows_red_off(nch * XW, NMAX * ST);   // [wave][RT rows][NMAX]
    if (kl == 0)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int n = 0; n < NMAX; ++n) red[(wave * RT + 4 * ml + r) * NMAX + n] = acc[r][n];
    __syncthreads();
    for (int e = tid; e < RT * NMAX; e += 256) {
        const int row = e / NMAX, n = e - row * NMAX;
        const float v = ((red[row * NMAX + n] + red[(RT + row) * NMAX + n]) + red[(2 * RT + row) * NMAX + n]) +
                        red[(3 * RT + row) * NMAX + n];
        const int m = m0 + row;
        if (n < U && m < a.M) store_out(a, b, m, n, v);
    }
}

template <int KT, int NMAX, int RT>
static int rows_go(ConvKArgs k, hipStream_t st) {
    const int grid = ceil_div(k.M, RT) * k.B;
    const size_t lds = (size_t)(rows_red_off(k.nchunks * GFam<KT>::CIT * k.XW, NMAX * GFam<KT>::ST) + 4 * RT * NMAX) * 4;
    auto kern = k.act == RAVE_ACT_SNAKE ? conv1d_gemv_rows_kernel<KT, NMAX, RT, true>
                                        : conv1d_gemv_rows_kernel<KT, NMAX, RT, false>;
    static bool done[2] = {false, false};
    bool& d = done[k.act == RAVE_ACT_SNAKE];
    if (!d) {
        RAVE_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
        d = true;
    }
    launch(kern, dim3(grid), dim3(256), (uint32_t)lds, st, k);
    return launch_status("conv1d_gemv_rows_kernel");
}

template <int KT, int RT>
static int rows_family(const ConvKArgs& k, int nmax, hipStream_t st) {
    switch (nmax) {
        case 4: return rows_go<KT, 4, RT>(k, st);
        case 8: return rows_go<KT, 8, RT>(k, st);
        case 16: return rows_go<KT, 16, RT>(k, st);
        default: return rows_go<KT, 32, RT>(k, st);
    }
}

bool gemv_rows_fits(int taps, int U, int d, bool transposed, int nchunks, int nmax) {
    if (U > nmax || nmax > kRowsMaxN) return false;
    const int cit = taps == 1 || taps == 2 ? 32 : taps == 3 || taps == 4 ? 16 : 8;
    const int st = taps == 4 ? 2 : taps == 8 ? 4 : 1;
    return (int64_t)nchunks * cit * gemv_xw(taps, st, U, d, transposed) <= kRowsStage;
}

int conv1d_gemv_rows(ConvKArgs k, int taps, int nmax, int rt, hipStream_t st) {
    const int stv = taps == 4 ? 2 : taps == 8 ? 4 : 1;
    k.XW = gemv_xw(taps, stv, k.U, k.d, k.transposed != 0);
    if (!gemv_rows_fits(taps, k.U, k.d, k.transposed != 0, k.nchunks, nmax) || (rt != 8 && rt != 16 && rt != 32) ||
        (k.transposed && k.split_row < k.M && k.split_row % rt != 0)) {
        set_error("conv1d(gemv rows): window exceeds the staging area, or too many columns");
        return RAVE_ERR_UNSUPPORTED;
    }
    k.S = 1;
    switch (taps * 64 + rt) {
        case 1 * 64 + 8: return rows_family<1, 8>(k, nmax, st);
        case 2 * 64 + 8: return rows_family<2, 8>(k, nmax, st);
        case 3 * 64 + 8: return rows_family<3, 8>(k, nmax, st);
        case 4 * 64 + 8: return rows_family<4, 8>(k, nmax, st);
        case 7 * 64 + 8: return rows_family<7, 8>(k, nmax, st);
        case 8 * 64 + 8: return rows_family<8, 8>(k, nmax, st);
        case 1 * 64 + 16: return rows_family<1, 16>(k, nmax, st);
        case 1 * 64 + 32: return rows_family<1, 32>(k, nmax, st);
        case 2 * 64 + 16: return rows_family<2, 16>(k, nmax, st);
        case 2 * 64 + 32: return rows_family<2, 32>(k, nmax, st);
        case 3 * 64 + 16: return rows_family<3, 16>(k, nmax, st);
        case 3 * 64 + 32: return rows_family<3, 32>(k, nmax, st);
        case 4 * 64 + 16: return rows_family<4, 16>(k, nmax, st);
        case 4 * 64 + 32: return rows_family<4, 32>(k, nmax, st);
        case 7 * 64 + 16: return rows_family<7, 16>(k, nmax, st);
        case 7 * 64 + 32: return rows_family<7, 32>(k, nmax, st);
        case 8 * 64 + 16: return rows_family<8, 16>(k, nmax, st);
        case 8 * 64 + 32: return rows_family<8, 32>(k, nmax, st);
        default: set_error("conv1d(gemv rows): unsupported kernel size"); return RAVE_ERR_UNSUPPORTED;
    }
}

template <int KT, int NMAX>
static int gemv_go(ConvKArgs k, hipStream_t st) {
    const int MT = ceil_div(k.M, GR<NMAX>::BM);
    const int grid = MT * k.S * k.B;
    // (+ slack: lanes read all NMAX columns of a window row, the ones past U unused)
    size_t lds = (size_t)std::max(ceil_div(k.cps * GFam<KT>::CIT * k.XW, 4) * 4 + NMAX * GFam<KT>::ST + 16,
                                  4 * GR<NMAX>::BM * NMAX) * 4;
    if (kGemvSc1 && k.inlaunch) lds = std::max(lds, kGemvOnePerCu);
    if (lds > 150 * 1024) {
        set_error("conv1d(gemv): staging exceeds the LDS budget");
        return RAVE_ERR_UNSUPPORTED;
    }
    auto kern = k.act == RAVE_ACT_SNAKE ? conv1d_gemv_kernel<KT, NMAX, true> : conv1d_gemv_kernel<KT, NMAX, false>;
    if (lds > 64 * 1024) {
        static bool done[2] = {false, false};
        bool& d = done[k.act == RAVE_ACT_SNAKE];
        if (!d) {
            RAVE_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
            d = true;
        }
    }
    launch(kern, dim3(grid), dim3(256), (uint32_t)lds, st, k);
    return launch_status("conv1d_gemv_kernel");
}

template <int KT>
static int gemv_family(const ConvKArgs& k, int nmax, hipStream_t st) {
    switch (nmax) {
        case 4: return gemv_go<KT, 4>(k, st);
        case 8: return gemv_go<KT, 8>(k, st);
        case 16: return gemv_go<KT, 16>(k, st);
        case 32: return gemv_go<KT, 32>(k, st);
        case 64: return gemv_go<KT, 64>(k, st);
        default: return gemv_go<KT, 128>(k, st);
    }
}

bool gemv_fits(int taps, int U, int d, bool transposed, int cps, int nmax) {
    if (U > nmax || nmax > kGemvMaxN) return false;
    const int cit = taps == 1 || taps == 2 ? 32 : taps == 3 || taps == 4 ? 16 : 8;
    const int st = taps == 4 ? 2 : taps == 8 ? 4 : 1;
    return (int64_t)cps * cit * gemv_xw(taps, st, U, d, transposed) <= kGemvStage;
}

int conv1d_gemv(ConvKArgs k, int taps, int nmax, int sep, hipStream_t st) {
    const int cit = taps == 1 || taps == 2 ? 32 : taps == 3 || taps == 4 ? 16 : 8;
    const int stv = taps == 4 ? 2 : taps == 8 ? 4 : 1;
    (void)cit;
    k.XW = gemv_xw(taps, stv, k.U, k.d, k.transposed != 0);
    if (!gemv_fits(taps, k.U, k.d, k.transposed != 0, k.cps, nmax)) {
        set_error("conv1d(gemv): window of one K split exceeds the staging area, or too many columns");
        return RAVE_ERR_UNSUPPORTED;
    }
    const int rows = gemv_rows(nmax);                                 // GR<NMAX>::BM
    const int tiles = ceil_div(k.M, rows) * k.B;
    k.inlaunch = (k.S > 1 && !sep && k.partial && tiles <= kSplitTicketsUsable) ? 1 : 0;
    RAVE_CHECK_ARG(k.S <= 1 || k.partial, "conv1d(gemv): K splits need the workspace");
    int rc;
    switch (taps) {
        case 1: rc = gemv_family<1>(k, nmax, st); break;
        case 2: rc = gemv_family<2>(k, nmax, st); break;
        case 3: rc = gemv_family<3>(k, nmax, st); break;
        case 4: rc = gemv_family<4>(k, nmax, st); break;
        case 7: rc = gemv_family<7>(k, nmax, st); break;
        case 8: rc = gemv_family<8>(k, nmax, st); break;
        default: set_error("conv1d(gemv): unsupported kernel size"); return RAVE_ERR_UNSUPPORTED;
    }
    if (rc != RAVE_OK || k.S <= 1 || k.inlaunch) return rc;
    const int64_t total = (int64_t)k.B * k.M * k.U;
    const int blocks = (int)std::min<int64_t>(ceil_div64(total, 256), 4096);
    launch(conv1d_splitk_reduce_kernel<1>, dim3(blocks), dim3(256), 0, st, k);
    return launch_status("conv1d_splitk_reduce_kernel");
}

}  // namespace rave
