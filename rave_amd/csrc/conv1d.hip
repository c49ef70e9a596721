// Implicit-GEMM Conv1d / ConvTranspose1d on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces cached_conv's Conv1d/ConvTranspose1d forward (F.pad + F.conv1d /
// F.conv_transpose1d; third-party cached-conv>=2.5.0, non-cached mode) at every
// call site of rave/blocks.py (DilatedUnit :96-106, EncoderV2 :533-584,
// GeneratorV2 :631-677, NoiseGeneratorV2 :257-266), fused with the activation
// module that precedes each conv (LeakyReLU(.2) / Snake) and the Residual add
// (rave/blocks.py:44-46).
//
// GEMM view: Y[m, n] = sum_kk W[m, kk] * X[kk, n] with kk = (tap, ci).
//  * K is walked in chunks of CIT input channels x all KT taps (compile-time
//    per layer family, so the MFMA loop over a chunk is fully unrolled and the
//    LDS fragment reads use immediate offsets).
//  * Per chunk the workgroup stages (a) the weight tile [BK][BM] (host-packed:
//    each row is BM contiguous floats) and (b) the input window of the dilated
//    receptive field, CIT rows x ((BN-1)*ST + (KT-1)*d + 1) columns, read once
//    from HBM coalesced along time, activation applied, stored in polyphase
//    order (phase = column mod stride) so a tap's strided B-fragment reads are
//    consecutive in LDS.  Every tap reads a shifted view of that one window:
//    the dilated halo is fetched once, not KT times.
//  * 4 waves (2x2), each (BM/2)x(BN/2) of 32x32 MFMA tiles; exact fp32 (the
//    MFMA is a k-ordered fmaf chain).  Global loads of chunk c+1 are issued
//    into registers before the MFMAs of chunk c.
//  * Split-K over grid.z for tall-K / short-N layers: each split writes an fp32
//    partial slab, a second kernel sums the slabs in fixed order (bitwise
//    deterministic, no atomics) and applies bias / residual / interleave.
//
// ConvTranspose1d(C, C', 2r, stride r) runs in polyphase form: the r output
// phases of input position u are rows m = co*r + q of a 2-tap conv over the
// input; the epilogue interleaves them to t = u*r + q - out_shift.
#include "conv_shared.h"

#include <cstring>

namespace rave {

// Layer families: (taps, stride, chunk channels).  Every RAVE conv is one of
// these: k=1 (1x1), k=2 (ConvTranspose polyphase), k=3 (dilated / io),
// k=4 s=2 (down r=2, noise), k=7 (io), k=8 s=4 (down r=4).
template <int KT> struct Family;
template <> struct Family<1> { static constexpr int ST = 1, CIT = 32, DMAX = 1; };
template <> struct Family<2> { static constexpr int ST = 1, CIT = 32, DMAX = 1; };
template <> struct Family<3> { static constexpr int ST = 1, CIT = 16, DMAX = kMaxDil; };
template <> struct Family<4> { static constexpr int ST = 2, CIT = 16, DMAX = 1; };
template <> struct Family<7> { static constexpr int ST = 1, CIT = 8, DMAX = 1; };
template <> struct Family<8> { static constexpr int ST = 4, CIT = 8, DMAX = 1; };

template <int KT, int BN> struct Geo {
    static constexpr int ST = Family<KT>::ST, CIT = Family<KT>::CIT;
    static constexpr int BK = KT * CIT;
    static constexpr int XW_MAX = (BN - 1) * ST + (KT - 1) * Family<KT>::DMAX + 1;
    static constexpr int XWS = (XW_MAX + ST - 1) / ST;       // per-phase row length
    static constexpr int XR = XWS * ST;                        // LDS row stride (floats)
    static constexpr int XREGS = (CIT * XW_MAX + kThreads - 1) / kThreads;
    // rows reachable by the unconditional staging stores (the window is at
    // least XW_MIN columns, dilation 1)
    static constexpr int XW_MIN = (BN - 1) * ST + (KT - 1) + 1;
    static constexpr int XS_FLOATS = ((XREGS * kThreads - 1) / XW_MIN + 1) * XR;
};

// --------------------------------------------------------------------- kernel
// WG = 4 waves.  Each wave owns a 64x64 output tile (2x2 MFMA 32x32 tiles, four
// independent accumulator chains: 256 MFMA cycles per K-step hide the LDS
// fragment latency).  The WG tile is (BM/64) x (BN/64) wave tiles; the
// KS = 4 / (#wave tiles) wave groups split the K-steps of every chunk and are
// summed through LDS at the end.  LDS is double-buffered: chunk c+1 is staged
// into the other buffer while chunk c is multiplied (one barrier per chunk).
template <int BM, int BN, int KT, bool SNAKE>
__global__ __launch_bounds__(kThreads) void conv1d_mfma_kernel(ConvKArgs a) {
    using G = Geo<KT, BN>;
    constexpr int ST = G::ST, CIT = G::CIT, BK = G::BK, XR = G::XR, XWS = G::XWS;
    constexpr int WGM = BM / 64, WGN = BN / 64, NWT = WGM * WGN, KS = 4 / NWT;
    static_assert(NWT * KS == 4, "tile must hold 1, 2 or 4 wave tiles");
    constexpr int A4 = BK * BM / 4;                        // float4s of one weight chunk
    constexpr int NA4 = (A4 + kThreads - 1) / kThreads;
    constexpr int AROWS = NA4 * kThreads * 4 / BM;         // >= BK (slack rows)
    constexpr int XREGS = G::XREGS;
    constexpr int BUF = AROWS * BM + G::XS_FLOATS;         // floats per LDS buffer
    constexpr int HALF = CIT / 2;
    constexpr int NSTEP = KT * HALF;

    extern __shared__ __attribute__((aligned(16))) float smem[];

    const int tid = threadIdx.x;
#ifdef RAVE_STAMPS
    const int wg_lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    auto stamp = [&](int k) {
        if (tid == 0) {
            a.stamps[wg_lin * 8 + k] = __builtin_amdgcn_s_memtime();
            if (k == 0) a.stamps[wg_lin * 8 + 7] = __builtin_amdgcn_s_memrealtime();
        }
    };
    stamp(0);
#endif
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform (scalar branches)
    const int wt = wave % NWT;          // wave tile
    const int kg = wave / NWT;          // K group
    const int wm0 = (wt / WGN) * 64;
    const int wn0 = (wt % WGN) * 64;
    const int h = lane >> 5;
    const int l32 = lane & 31;

    // XCD-major order over the (column tile, row tile, batch x split) grid:
    // every XCD runs a contiguous run of batch items (common.h xcd_major)
    const int gxy = gridDim.x * gridDim.y;
    const int lg = __builtin_amdgcn_readfirstlane(
        xcd_major(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), gxy * gridDim.z));
    const int bz = __builtin_amdgcn_readfirstlane(lg / gxy);
    const int bxy = lg - bz * gxy;
    const int by = __builtin_amdgcn_readfirstlane(bxy / gridDim.x);
    const int n0 = (bxy - by * gridDim.x) * BN;
    const int m0 = by * BM;
    const int b = __builtin_amdgcn_readfirstlane(bz / a.S);
    const int split = __builtin_amdgcn_readfirstlane(bz - b * a.S);
    const int c_begin = split * a.cps;
    const int c_end = min(a.nchunks, c_begin + a.cps);
    const int in0 = n0 * ST - ((m0 < a.split_row) ? a.pad_l : a.pad_g1);   // ConvT phase groups
    const int XW = a.XW;
    const int x_elems = CIT * XW;
    // buffer descriptors: 32-bit voffsets instead of 64-bit addresses per load
    // (inputs readfirstlane'd so the compiler can PROVE the descriptor uniform;
    // otherwise every buffer op becomes a waterfall loop)
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(a.x + (int64_t)b * a.x_sb, a.x_bytes);
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(a.w, a.w_bytes);
    const float slope = a.act == RAVE_ACT_LEAKY ? a.slope : 1.0f;   // none: v * 1

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    f32x4 ra[NA4];
    float rx[XREGS];

    // Global -> registers.  Unconditional loads from clamped valid addresses,
    // validity as a select (a load under a per-element branch makes hipcc wait
    // vmcnt(0) per element); e / XW by a magic multiply, no branches.
    auto load_chunk = [&](int c) __attribute__((always_inline)) {
        const unsigned wbase = (unsigned)(((unsigned)c * BK * a.Mpad + m0) * 4u);
#pragma unroll
        for (int i = 0; i < NA4; ++i) {
            const int e = min(tid + i * kThreads, A4 - 1);
            const int row = e / (BM / 4);
            const int col4 = e - row * (BM / 4);
            ra[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                wrs, wbase + (unsigned)(row * a.Mpad + col4 * 4) * 4u, 0, 0));
        }
        const int ci0 = c * CIT;
#pragma unroll
        for (int i = 0; i < XREGS; ++i) {
            const int e = tid + i * kThreads;
            const int ci = (int)(((unsigned)e * a.xw_magic) >> 24);
            const int w = e - ci * XW;
            const int cg = ci0 + ci;
            const int t = in0 + w;
            const bool ok = (e < x_elems) && (cg < a.c_in) && (t >= 0) && (t < a.t_in);
            const int cgc = min(cg, a.c_in - 1);
            const int tc = min(max(t, 0), a.t_in - 1);
            const float v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                xrs, (unsigned)(cgc * a.x_sc + tc) * 4u, 0, 0));
            rx[i] = ok ? v : 0.f;
        }
    };

    // Registers -> LDS buffer, activation applied once per staged element.
    // Stores are unconditional: entries past the chunk land in buffer slack.
    auto store_chunk = [&](int c, float* buf) __attribute__((always_inline)) {
        float* As = buf;
        float* Xs = buf + AROWS * BM;
#pragma unroll
        for (int i = 0; i < NA4; ++i) {
            const int e = tid + i * kThreads;
            const int row = e / (BM / 4);
            const int col4 = e - row * (BM / 4);
            *reinterpret_cast<f32x4*>(As + row * BM + col4 * 4) = ra[i];
        }
        const int ci0 = c * CIT;
#pragma unroll
        for (int i = 0; i < XREGS; ++i) {
            const int e = tid + i * kThreads;
            const int ci = (int)(((unsigned)e * a.xw_magic) >> 24);
            const int w = e - ci * XW;
            float v = rx[i];
            if constexpr (SNAKE) {
                const float al = a.alpha[min(ci0 + ci, a.c_in - 1)];
                v = v + (1.0f / (al + 1e-9f)) * sin_squared(al * v);
            } else {
                v = v > 0.f ? v : v * slope;
            }
            Xs[ci * XR + (w % ST) * XWS + w / ST] = v;
        }
    };

    // per-lane LDS offsets of the B fragments of each tap (row h of the pair)
    int xoff[KT];
#pragma unroll
    for (int j = 0; j < KT; ++j) {
        const int p = (wn0 + l32) * ST + j * a.d;
        xoff[j] = h * XR + (p % ST) * XWS + p / ST;
    }
    const int aoff = h * BM + wm0 + l32;

    load_chunk(c_begin);
    store_chunk(c_begin, smem);
    if (c_begin + 1 < c_end) load_chunk(c_begin + 1);
    __syncthreads();
#ifdef RAVE_STAMPS
    stamp(1);
#endif

    for (int c = c_begin; c < c_end; ++c) {
        const int cur = (c - c_begin) & 1;
        float* bcur = smem + cur * BUF;
        if (c + 1 < c_end) {
            store_chunk(c + 1, smem + (cur ^ 1) * BUF);   // overlaps the MFMAs below
            if (c + 2 < c_end) load_chunk(c + 2);
        }
        const float* As = bcur;
        const float* Xs = bcur + AROWS * BM;
#pragma unroll
        for (int st = 0; st < NSTEP; ++st) {
            if constexpr (KS > 1) {
                if (st % KS != kg) continue;        // K-steps of this wave's group
            }
            const int j = st / HALF, c2 = st - (st / HALF) * HALF;
            float fa[2], fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[i] = As[aoff + (j * CIT + 2 * c2) * BM + i * 32];
#pragma unroll
            for (int i = 0; i < 2; ++i) fb[i] = Xs[xoff[j] + c2 * 2 * XR + i * 32];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int jj = 0; jj < 2; ++jj)
                    acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[jj], acc[i][jj], 0, 0, 0);
        }
        __syncthreads();
    }

    // ---------------------------------------------------------------- epilogue
    // With KS > 1 every wave parks its partial 64x64 tile in LDS and then
    // finishes the 32x32 sub-tiles q with q % KS == kg (sum over K groups in
    // group order).  Stores/loads are branch-free buffer ops: invalid elements
    // (tile edges, transposed interleave) get offset 0xFFFFFFFF, which the range
    // check drops (stores) or reads as 0 (loads).
    constexpr unsigned kOOB = 0xFFFFFFFFu;
#ifdef RAVE_STAMPS
    stamp(2);
#endif
    float* red = smem;   // staging buffers are dead after the last barrier
    if constexpr (KS > 1) {
        float* dst = red + (kg * NWT + wt) * 4096;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[(q * 16 + r) * 64 + lane] = acc[q >> 1][q & 1][r];
        __syncthreads();
    }
    const bool partial = a.S > 1;
    // in-launch split-K combine (round 6): the slabs are stored write-through and
    // the split drawing the tile's last ticket sums them in split order with sc1
    // loads (bitwise the separate reduce launch; the form of conv_gemv.hip)
    const bool inl = partial && a.inlaunch;
    const bool fin = !partial || inl;                // this workgroup may finish the tile
    const int ntl = gxy * a.B;                       // output tiles (in-launch slab layout)
    const __amdgpu_buffer_rsrc_t irs = make_rsrc(
        inl ? a.partial + ((int64_t)split * ntl + (b * gxy + bxy)) * (BM * BN) : a.y, inl ? BM * BN * 4 : 0);
    const __amdgpu_buffer_rsrc_t prs = make_rsrc(
        partial ? a.partial + ((int64_t)split * a.B + b) * (int64_t)a.M * a.U : a.y,
        partial ? a.M * a.U * 4 : 0);
    const __amdgpu_buffer_rsrc_t yrs = make_rsrc(a.y + (int64_t)b * a.y_sb, fin ? a.y_bytes : 0);
    const __amdgpu_buffer_rsrc_t brs = make_rsrc(a.bias ? a.bias : a.y, (a.bias && fin) ? a.bias_rows * 4 : 0);
    const __amdgpu_buffer_rsrc_t rrs = make_rsrc(
        a.res ? a.res + (int64_t)b * a.r_sb : a.y, (a.res && fin) ? a.r_bytes : 0);
    // bias, residual, ConvT interleave and the output store of sub-tile q
    auto finish = [&](int q, const float* v) __attribute__((always_inline)) {
        const int i = q >> 1, jj = q & 1;
        const int n = n0 + wn0 + jj * 32 + l32;
        float bv[16], rv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            int brow = m;
            if (a.transposed) {
                int qq;
                convt_row(a, m, brow, qq);
            }
            bv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(brs, (unsigned)brow * 4u, 0, 0));
            const unsigned roff = (m < a.M && n < a.U) ? (unsigned)(m * a.r_sc + n) * 4u : kOOB;
            rv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rrs, roff, 0, 0));
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            unsigned off;
            if (a.transposed) {
                int co, q;
                convt_row(a, m, co, q);
                const int t = n * a.R + q;
                off = (co < a.bias_rows && n < a.U && t < a.t_y) ? (unsigned)(co * a.y_sc + t) * 4u : kOOB;
            } else {
                off = (m < a.M && n < a.U) ? (unsigned)(m * a.y_sc + n) * 4u : kOOB;
            }
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[r] + bv[r] + rv[r]),
                                                  yrs, off, 0, 0);
        }
    };
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if constexpr (KS > 1) {
            if (q % KS != kg) continue;            // uniform
        }
        const int i = q >> 1, jj = q & 1;
        const int n = n0 + wn0 + jj * 32 + l32;
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if constexpr (KS > 1) {
                float sum = 0.f;
#pragma unroll
                for (int g = 0; g < KS; ++g) sum += red[((g * NWT + wt) * 4096) + (q * 16 + r) * 64 + lane];
                v[r] = sum;
            } else {
                v[r] = acc[i][jj][r];
            }
        }
        if (inl) {
            // the in-launch slab is private to the combine: lane-major 16-byte
            // pieces [split][tile][wave tile][q][r / 4][lane] (whole-wave
            // write-through stores, and the last arriver's loads, are 16 B)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(u32x4_t, f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]}), irs,
                    (unsigned)((((wt * 4 + q) * 4 + g) * 64 + lane) * 16), 0, 16);
            continue;
        }
        if (partial) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const unsigned off = (m < a.M && n < a.U) ? (unsigned)(m * a.U + n) * 4u : kOOB;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[r]), prs, off, 0, 0);
            }
            continue;
        }
        finish(q, v);
    }
    if (inl) {
        // MI355X_MICROARCH.md hand-off table row 1 (the launch keeps one workgroup
        // per CU): every slab byte stored sc1 and drained by its wave before the
        // barrier behind which one lane adds to the tile's unsharded ticket; the
        // last adder, told by the value its add returned, reads every slab sc1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        __shared__ int last_s;
        const int tile = b * gxy + bxy;
        if (tid == 0) {
            const int prev = __hip_atomic_fetch_add(a.tickets + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = prev == a.S - 1;
            if (last) __hip_atomic_store(a.tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last_s = last;
        }
        __syncthreads();
        if (!last_s) return;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if constexpr (KS > 1) {
                if (q % KS != kg) continue;
            }
            f32x4 v4[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) v4[g] = f32x4{0.f, 0.f, 0.f, 0.f};
            // splits in order; SB splits' loads in flight per round trip
            constexpr int SB = 4;
            for (int sp0 = 0; sp0 < a.S; sp0 += SB) {
                f32x4 t[SB][4];
#pragma unroll
                for (int u = 0; u < SB; ++u) {
                    const int sp = min(sp0 + u, a.S - 1);
                    const __amdgpu_buffer_rsrc_t srs = make_rsrc(a.partial + ((int64_t)sp * ntl + tile) * (BM * BN),
                                                                 BM * BN * 4);
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        t[u][g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                            srs, (unsigned)((((wt * 4 + q) * 4 + g) * 64 + lane) * 16), 0, 16));
                }
#pragma unroll
                for (int u = 0; u < SB; ++u)
                    if (sp0 + u < a.S)
#pragma unroll
                        for (int g = 0; g < 4; ++g) v4[g] += t[u][g];
            }
            float v[16];
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e) v[4 * g + e] = v4[g][e];
            finish(q, v);
        }
    }
#ifdef RAVE_STAMPS
    stamp(3);
#endif
}

// Launch of one layer family.  The kernel instantiations are spread over
// separate translation units (the Makefile compiles this file once per family
// with -DRAVE_F32_KT, and once without it for the host side) so the build runs
// in parallel.
template <int KT>
int f32_launch_family(ConvKArgs k, const LaunchCfg& c, hipStream_t st);

#ifdef RAVE_F32_KT
template <int BM, int BN, int KT>
static int launch_k(ConvKArgs k, hipStream_t st) {
    using G = Geo<KT, BN>;
    constexpr int A4 = G::BK * BM / 4;
    constexpr int NA4 = (A4 + kThreads - 1) / kThreads;
    constexpr int AROWS = NA4 * kThreads * 4 / BM;
    constexpr int BUF = AROWS * BM + G::XS_FLOATS;
    constexpr int NWT = (BM / 64) * (BN / 64);
    constexpr int RED = (NWT < 4) ? 4 * 64 * 64 : 0;        // K-group reduction area
    if (k.XW > G::XW_MAX) {
        set_error("conv1d: dilation too large for the staged window");
        return RAVE_ERR_UNSUPPORTED;
    }
    size_t lds = (size_t)std::max(2 * BUF, RED) * sizeof(float);
    static_assert((size_t)std::max(2 * BUF, RED) * sizeof(float) <= 150 * 1024, "LDS budget");
    // an in-launch combine keeps one workgroup per CU (the sc1 hand-off's measured form)
    if (k.inlaunch) lds = std::max(lds, (size_t)(80 * 1024 + 256));
    dim3 grid(ceil_div(k.U, BN), ceil_div(k.M, BM), k.B * k.S);
    auto kern = (k.act == RAVE_ACT_SNAKE) ? conv1d_mfma_kernel<BM, BN, KT, true>
                                           : conv1d_mfma_kernel<BM, BN, KT, false>;
    if (lds > 64 * 1024) {
        // opt in to more than 64 KiB of dynamic LDS (once per instantiation)
        static bool done[2] = {false, false};
        bool& d = done[k.act == RAVE_ACT_SNAKE];
        if (!d) {
            RAVE_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
            d = true;
        }
    }
    launch(kern, grid, dim3(kThreads), lds, st, k);
    return launch_status("conv1d_mfma_kernel");
}

template <int KT>
int f32_launch_family(ConvKArgs k, const LaunchCfg& c, hipStream_t st) {
    k.XW = (c.bn - 1) * Family<KT>::ST + (KT - 1) * k.d + 1;
    k.xw_magic = (unsigned)(((1u << 24) + k.XW - 1) / k.XW);
    if (c.bm == 128 && c.bn == 128) return launch_k<128, 128, KT>(k, st);
    if (c.bm == 64 && c.bn == 256) return launch_k<64, 256, KT>(k, st);
    if (c.bm == 128 && c.bn == 64) return launch_k<128, 64, KT>(k, st);
    if (c.bm == 64 && c.bn == 128) return launch_k<64, 128, KT>(k, st);
    return launch_k<64, 64, KT>(k, st);
}

template int f32_launch_family<RAVE_F32_KT>(ConvKArgs, const LaunchCfg&, hipStream_t);

}  // namespace rave
#else   // ------------------------------------------------------- host side

// --------------------------------------------------------------------- host side
static int family_cit(int taps) {
    switch (taps) {
        case 1: return Family<1>::CIT;
        case 2: return Family<2>::CIT;
        case 3: return Family<3>::CIT;
        case 4: return Family<4>::CIT;
        case 7: return Family<7>::CIT;
        case 8: return Family<8>::CIT;
        default: return 0;
    }
}

// Tile + split-K choice.  Prefer the largest tile (fewest K-groups) that gives
// >= 2 workgroups per CU with little padding; otherwise the least-padding tile
// with K split across workgroups until ~2 workgroups per CU.
constexpr int kF32Tiles[5][2] = {{128, 128}, {64, 256}, {128, 64}, {64, 128}, {64, 64}};

static LaunchCfg choose(int M, int U, int B, int nchunks, int split_row = 1 << 30) {
    const auto& all = kF32Tiles;
    int cand[5][2], nc = 0;
    for (auto& c : all)   // a tile may not straddle the ConvT phase-group boundary
        if (split_row >= M || split_row % c[0] == 0) { cand[nc][0] = c[0]; cand[nc][1] = c[1]; ++nc; }
    for (int ci = 0; ci < nc; ++ci) {
        const int* c = cand[ci];
        int64_t wg = (int64_t)ceil_div(M, c[0]) * ceil_div(U, c[1]) * B;
        if (wg >= 512 && pad_waste(M, U, c[0], c[1]) <= 1.12) return {c[0], c[1], 1};
    }
    LaunchCfg best{64, 64, 1};
    double bw = 1e30;
    for (int ci = 0; ci < nc; ++ci) {
        const int* c = cand[ci];
        double score = pad_waste(M, U, c[0], c[1]) * (c[0] * c[1] == 4096 ? 1.06 : 1.0);
        if (score < bw) { bw = score; best = {c[0], c[1], 1}; }
    }
    int64_t wg = (int64_t)ceil_div(M, best.bm) * ceil_div(U, best.bn) * B;
    int S = (int)std::min<int64_t>(16, ceil_div64(512, wg));
    S = std::min(S, std::max(1, nchunks / 2));
    best.S = std::max(1, S);
    return best;
}

// exact-fp32 layout: chunks of family_cit channels, rows padded to 128
static int prepare(const rave_conv1d_args& a, ConvKArgs& k, int& taps) {
    int rc = prepare_common(a, k, taps);
    if (rc != RAVE_OK) return rc;
    if (family_cit(taps) == 0) {
        set_error("conv1d: unsupported kernel size");
        return RAVE_ERR_UNSUPPORTED;
    }
    k.nchunks = ceil_div(a.c_in, family_cit(taps));
    k.Mpad = ceil_div(k.M, 128) * 128;
    const int64_t wb = (int64_t)k.nchunks * family_cit(taps) * taps * k.Mpad * 4;
    RAVE_CHECK_ARG(wb < (1ll << 31), "conv1d: packed weight beyond 2 GiB");
    k.w_bytes = (int)wb;
    return RAVE_OK;
}

}  // namespace rave

using namespace rave;

extern "C" int rave_conv1d_chunk(int c_in, int kernel, int stride, int dilation, int transposed) {
    (void)c_in; (void)dilation;
    if (transposed) return kernel == 2 * stride ? family_cit(2) : 0;
    if (family_cit(kernel) == 0 || family_stride(kernel) != stride) return 0;
    return family_cit(kernel);
}

extern "C" int64_t rave_conv1d_packed_size(int c_in, int c_out, int kernel, int stride, int dilation,
                                           int transposed) {
    int ci_t = rave_conv1d_chunk(c_in, kernel, stride, dilation, transposed);
    if (ci_t <= 0) return -1;
    int taps = transposed ? 2 : kernel;
    // transposed: the larger of the two row layouts (out_shift 0 / stride/2)
    int M = transposed ? std::max(c_out * stride, convt_group1_row(c_out, stride, stride - stride / 2) +
                                                      c_out * (stride / 2))
                       : c_out;
    int64_t Mpad = (int64_t)ceil_div(M, 128) * 128;
    int64_t nchunks = ceil_div(c_in, ci_t);
    return nchunks * ci_t * taps * Mpad;
}

extern "C" int rave_conv1d_pack_weight(const float* w, int c_in, int c_out, int kernel, int stride,
                                       int dilation, int transposed, int out_shift, float* packed) {
    RAVE_CHECK_ARG(w && packed, "pack_weight: null pointer");
    RAVE_CHECK_ARG(c_in > 0 && c_out > 0 && kernel > 0 && stride > 0 && dilation > 0,
                   "pack_weight: bad shape");
    int ci_t = rave_conv1d_chunk(c_in, kernel, stride, dilation, transposed);
    if (ci_t <= 0) {
        set_error("pack_weight: unsupported layer shape");
        return RAVE_ERR_UNSUPPORTED;
    }
    RAVE_CHECK_ARG(!transposed || out_shift == 0 || out_shift == stride / 2,
                   "pack_weight: transposed out_shift must be 0 or stride/2");
    int taps = transposed ? 2 : kernel;
    int R = transposed ? stride : 1;
    int q0 = R - (transposed ? out_shift : 0);       // ConvT phases in row group 0
    int split_row = transposed ? convt_group1_row(c_out, R, q0) : 1 << 30;
    int M = transposed ? split_row + c_out * (R - q0) : c_out;
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
                        // output t = u*R + q; with P = out_shift:
                        //   q <  R-P : y = W[q+P+R] x[u-1] + W[q+P] x[u]     (taps u-1, u)
                        //   q >= R-P : y = W[q+P]   x[u]   + W[q+P-R] x[u+1] (taps u, u+1)
                        int co, q;
                        if (m < split_row) { co = m / q0; q = m % q0; }
                        else { int p = R - q0; co = (m - split_row) / p; q = q0 + (m - split_row) % p; }
                        if (co >= c_out) { row[m] = 0.f; continue; }   // group-0 padding rows
                        int kidx;
                        if (q < q0) kidx = (j == 0) ? q + out_shift + R : q + out_shift;
                        else kidx = (j == 0) ? q + out_shift : q + out_shift - R;
                        v = w[((int64_t)ci * c_out + co) * kernel + kidx];
                    } else {
                        v = w[((int64_t)m * c_in + ci) * kernel + j];
                    }
                    row[m] = v;
                }
            }
    return RAVE_OK;
}

static bool f32_tile_ok(int ti, int M, int split_row) {
    return ti >= 0 && ti < 5 && (split_row >= M || split_row % kF32Tiles[ti][0] == 0);
}

// The launch configuration: args.config when set (validated), else the heuristic.
// the in-launch combine of an fp32 MFMA tile: one ticket per output tile
static bool f32_inl_ok(const ConvKArgs& k, int tile, int S) {
    if (tile < 0 || tile >= 5) return false;
    const int64_t tiles = (int64_t)ceil_div(k.M, kF32Tiles[tile][0]) * ceil_div(k.U, kF32Tiles[tile][1]) * k.B;
    return S > 1 && tiles <= kSplitTicketsUsable;
}

static int resolve(const rave_conv1d_args& a, const ConvKArgs& k, int taps, LaunchCfg& c) {
    if (a.config == 0) {
        c = choose(k.M, k.U, k.B, k.nchunks, k.split_row);
        return RAVE_OK;
    }
    ConfigCode cc;
    const bool dec = decode_config(a.config, cc);
    if (dec && (cc.tile == kRowsTile || cc.tile == kRowsTile8)) {   // row-sliced skinny-N (one launch, no K split)
        RAVE_CHECK_ARG(cc.S == 1 && k.U <= kRowsMaxN && (cc.tile == kRowsTile || !cc.sep) &&
                           gemv_rows_fits(taps, k.U, k.d, k.transposed != 0, k.nchunks, rows_nmax(k.U)),
                       "conv1d: gemv rows config not valid for these args (see rave_conv1d_configs)");
        c = {0, rows_nmax(k.U), 1};
        c.rows = cc.tile == kRowsTile8 ? 8 : cc.sep ? 32 : 16;
        return RAVE_OK;
    }
    if (dec && is_gemv_tile(cc.tile)) {   // the skinny-N family (conv_gemv.hip)
        RAVE_CHECK_ARG(split_count_distinct(cc.S, k.nchunks) && (cc.S > 1 || !cc.sep) &&
                           gemv_fits(taps, k.U, k.d, k.transposed != 0, ceil_div(k.nchunks, cc.S),
                                     gemv_nmax(cc.tile)),
                       "conv1d: gemv config not valid for these args (see rave_conv1d_configs)");
        c = {0, gemv_nmax(cc.tile), cc.S};
        c.sep = cc.sep;
        return RAVE_OK;
    }
    // bit 9 on an fp32 MFMA tile: the K splits combined in-launch (its meaning for
    // the gemv tiles is the opposite; both spellings predate the other's)
    RAVE_CHECK_ARG(dec && (cc.sep == 0 || (cc.S > 1 && f32_inl_ok(k, cc.tile, cc.S))) &&
                       f32_tile_ok(cc.tile, k.M, k.split_row) && split_count_distinct(cc.S, k.nchunks),
                   "conv1d: config not valid for these args (see rave_conv1d_configs)");
    c = {kF32Tiles[cc.tile][0], kF32Tiles[cc.tile][1], cc.S};
    c.inl = cc.sep;
    return RAVE_OK;
}

// K-split counts of the gemv family (more than the MFMA tiles': its row tiles are few)
constexpr int kGemvSplits[] = {1, 2, 4, 8, 16, 32};

extern "C" int rave_conv1d_configs(const rave_conv1d_args* p, int32_t* cfgs, int max_cfgs) {
    RAVE_CHECK_ARG(p && max_cfgs >= 0, "conv1d_configs: null args");
    if (p->precision == RAVE_PREC_SPLIT16 || p->precision == RAVE_PREC_F32_RING || p->precision == RAVE_PREC_BF16X3)
        return conv1d_split_configs(*p, cfgs, max_cfgs);
    RAVE_CHECK_ARG(p->precision == RAVE_PREC_F32, "conv1d_configs: unknown precision");
    ConvKArgs k;
    int taps;
    int rc = prepare(*p, k, taps);
    if (rc != RAVE_OK) return rc;
    int n = 0;
    for (int ti = 0; ti < 5; ++ti) {
        if (!f32_tile_ok(ti, k.M, k.split_row)) continue;
        const int64_t wg = (int64_t)ceil_div(k.M, kF32Tiles[ti][0]) * ceil_div(k.U, kF32Tiles[ti][1]) * k.B;
        for (int S : kSplitCands) {
            if (!split_count_distinct(S, k.nchunks)) continue;
            if (S > 1 && (wg * S > 8192 || wg >= 1024)) continue;      // enough workgroups unsplit
            if (n < max_cfgs && cfgs) cfgs[n] = encode_config(ti, S, 0);
            ++n;
            if (f32_inl_ok(k, ti, S)) {                                 // combined in-launch
                if (n < max_cfgs && cfgs) cfgs[n] = encode_config(ti, S, 1);
                ++n;
            }
        }
    }
    // skinny-N (gemv) configurations: the smallest column width holding U
    if (k.U <= kGemvMaxN) {
        int nmax = 4, tile = 8;
        while (nmax < k.U) nmax *= 2, ++tile;
        const int64_t tiles = (int64_t)ceil_div(k.M, gemv_rows(nmax)) * k.B;
        for (int S : kGemvSplits) {
            if (!split_count_distinct(S, k.nchunks) || tiles * S > 2048 ||
                !gemv_fits(taps, k.U, k.d, k.transposed != 0, ceil_div(k.nchunks, S), nmax))
                continue;
            if (S == 1 || tiles <= kSplitTicketsUsable) {
                if (n < max_cfgs && cfgs) cfgs[n] = encode_config(tile, S, 0);
                ++n;
            }
            if (S > 1) {
                if (n < max_cfgs && cfgs) cfgs[n] = encode_config(tile, S, 1);
                ++n;
            }
        }
    }
    // the row-sliced skinny-N form: 8, 16 and 32 rows per workgroup, no K split
    if (k.U <= kRowsMaxN && gemv_rows_fits(taps, k.U, k.d, k.transposed != 0, k.nchunks, rows_nmax(k.U)))
        for (int v = 0; v < 3; ++v) {
            const int rt = v == 0 ? 8 : v == 1 ? 16 : 32;
            if (k.transposed && k.split_row < k.M && k.split_row % rt != 0) continue;
            if (n < max_cfgs && cfgs) cfgs[n] = v == 0 ? encode_config(kRowsTile8, 1, 0) : encode_config(kRowsTile, 1, v - 1);
            ++n;
        }
    return n;
}

extern "C" int64_t rave_conv1d_workspace(const rave_conv1d_args* p) {
    if (!p) return -1;
    if (p->precision == RAVE_PREC_SPLIT16 || p->precision == RAVE_PREC_F32_RING || p->precision == RAVE_PREC_BF16X3) return conv1d_split_workspace(*p);
    if (p->precision != RAVE_PREC_F32) return -1;
    ConvKArgs k;
    int taps;
    if (prepare(*p, k, taps) != RAVE_OK) return -1;
    LaunchCfg c;
    if (resolve(*p, k, taps, c) != RAVE_OK) return -1;
    if (c.S <= 1) return 0;
    if (c.inl && c.bm > 0)   // the in-launch combine's private slabs: one whole tile per split and tile
        return kSplitTickets + (int64_t)c.S * ceil_div(k.M, c.bm) * ceil_div(k.U, c.bn) * k.B * c.bm * c.bn;
    return kSplitTickets + (int64_t)c.S * k.B * (int64_t)k.M * k.U;   // same layout as the split path
}

extern "C" int rave_conv1d(const rave_conv1d_args* p, void* stream) {
    RAVE_CHECK_ARG(p, "conv1d: null args");
    if (p->precision == RAVE_PREC_SPLIT16 || p->precision == RAVE_PREC_F32_RING || p->precision == RAVE_PREC_BF16X3) return conv1d_split(*p, stream);
    RAVE_CHECK_ARG(p->precision == RAVE_PREC_F32, "conv1d: unknown precision");
    ConvKArgs k;
    int taps;
    int rc = prepare(*p, k, taps);
    if (rc != RAVE_OK) return rc;
    LaunchCfg c;
    rc = resolve(*p, k, taps, c);
    if (rc != RAVE_OK) return rc;
    if (c.S > 1 && p->partial == nullptr) c.S = 1;   // no workspace given: single pass
    k.cps = ceil_div(k.nchunks, c.S);
    k.S = ceil_div(k.nchunks, k.cps);                 // no empty splits
    k.partial = p->partial ? p->partial + kSplitTickets : nullptr;   // slabs after the counters
    if (c.rows) return conv1d_gemv_rows(k, taps, c.bn, c.rows, as_stream(stream));
    if (c.bm == 0) {                                  // skinny-N family (tickets ahead of the slabs)
        k.tickets = reinterpret_cast<int*>(p->partial);
        if (!gemv_fits(taps, k.U, k.d, k.transposed != 0, k.cps, c.bn)) {
            set_error("conv1d(gemv): one K split's window exceeds the staging area (give the workspace)");
            return RAVE_ERR_UNSUPPORTED;
        }
        return conv1d_gemv(k, taps, c.bn, c.sep, as_stream(stream));
    }
#ifdef RAVE_STAMPS
    k.stamps = p->stamps;
#endif
    k.tickets = reinterpret_cast<int*>(p->partial);
    k.inlaunch = (k.S > 1 && c.inl && k.partial &&
                  (int64_t)ceil_div(k.M, c.bm) * ceil_div(k.U, c.bn) * k.B <= kSplitTicketsUsable) ? 1 : 0;
    hipStream_t st = as_stream(stream);
    switch (taps) {
        case 1: rc = f32_launch_family<1>(k, c, st); break;
        case 2: rc = f32_launch_family<2>(k, c, st); break;
        case 3: rc = f32_launch_family<3>(k, c, st); break;
        case 4: rc = f32_launch_family<4>(k, c, st); break;
        case 7: rc = f32_launch_family<7>(k, c, st); break;
        case 8: rc = f32_launch_family<8>(k, c, st); break;
        default: set_error("conv1d: unsupported kernel size"); return RAVE_ERR_UNSUPPORTED;
    }
    if (rc != RAVE_OK || k.S <= 1 || k.inlaunch) return rc;
    int64_t total = (int64_t)k.B * k.M * k.U;
    int blocks = (int)std::min<int64_t>(ceil_div64(total, 256), 4096);
    launch(conv1d_splitk_reduce_kernel<0>, dim3(blocks), dim3(256), 0, st, k);
    return launch_status("conv1d_splitk_reduce_kernel");
}
#endif  // RAVE_F32_KT
